// K1: polar -> Cartesian scatter with intensity threshold, per-file stride and gain fusion.
// Replaces load_radar_csv (PointCloudWork/4_temporal_object_tracker.py:200-232) + build_frame's
// concatenation (:312-352), and radar_pipeline sweep_to_point_cloud (core/transforms.py:37-79).
//
// Layout: echo [file][row][bin] (u8 — 1 B per echo sample, the radar's native 8-bit values — or
// f32), rows of 1024 bins.  One wave owns one row: with u8 echo a row is exactly one 16-B-per-lane
// coalesced load (1 KiB per wave instruction); f32 rows take four.  Kept elements are ranked in
// row-major order with a wave prefix sum over per-lane counts; the file rank comes from the
// row prefix written by the count pass (two reads of the echo, no atomics, deterministic).
//
// Arithmetic (each op rounded to float32, no contraction — the reference is separate numpy ufuncs):
//   step = scale[row] / (float)bins ; r = step * (float)bin ; x = r * cos_t[row] ; y = r * sin_t[row]
// cos_t / sin_t are inputs: numpy's float32 SIMD cos/sin are not correctly rounded, so the host
// evaluates them exactly as the reference does (4096 values per sweep geometry).
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "common.h"

#pragma clang fp contract(off)

namespace rpt {
namespace {

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;

template <class T>
__device__ __forceinline__ float to_f(T v) {
  return (float)v;
}

// Elements per lane per iteration: 16 u8 (one uint4) or 4 f32 (one float4).
template <class T>
struct Vec;
template <>
struct Vec<uint8_t> {
  static constexpr int N = 16;
  using L = uint4;
  __device__ static void unpack(const L& v, float (&o)[16]) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 16; ++k) o[k] = (float)((w[k >> 2] >> (8 * (k & 3))) & 0xffu);
  }
};
template <>
struct Vec<float> {
  static constexpr int N = 4;
  using L = float4;
  __device__ static void unpack(const L& v, float (&o)[4]) {
    o[0] = v.x;
    o[1] = v.y;
    o[2] = v.z;
    o[3] = v.w;
  }
};

__device__ __forceinline__ int wave_excl_scan(int v, int* total) {
  const int lane = threadIdx.x & 63;
  int incl = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(incl, off, 64);
    if (lane >= off) incl += o;
  }
  *total = __shfl(incl, 63, 64);
  return incl - v;
}

// Inclusive wave prefix sum with DPP (6 VALU ops, no LDS): row_shr 1/2/4/8 within 16-lane rows,
// then row_bcast:15 / row_bcast:31 carry the row totals (GFX9-family DPP, available on gfx950).
__device__ __forceinline__ int wave_incl_scan_dpp(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}

// Row pass: count kept elements per row.  VEC path needs bins % (64*N) == 0 and aligned rows.
template <class T, bool VEC>
__global__ __launch_bounds__(kBlock) void k_row_count(const T* __restrict__ echo,
                                                     int64_t n_rows, int bins, float thr,
                                                     int32_t* __restrict__ row_count) {
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / 64;
  const int64_t n_waves = (int64_t)gridDim.x * kWavesPerBlock;
  for (int64_t row = wave0; row < n_rows; row += n_waves) {
    const T* rp = echo + row * bins;
    int c = 0;
    if (VEC) {
      constexpr int N = Vec<T>::N;
      using L = typename Vec<T>::L;
      for (int b0 = lane * N; b0 < bins; b0 += 64 * N) {
        const L v = *reinterpret_cast<const L*>(rp + b0);
        float f[N];
        Vec<T>::unpack(v, f);
#pragma unroll
        for (int k = 0; k < N; ++k) c += (f[k] > thr) ? 1 : 0;
      }
    } else {
      for (int b = lane; b < bins; b += 64) c += (to_f(rp[b]) > thr) ? 1 : 0;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if (lane == 0) row_count[row] = c;
  }
}

// file_offsets[f] = sum over earlier files of ceil(kept / stride); kept from row_prefix.
__global__ void k_file_counts(const int64_t* __restrict__ row_prefix, int64_t n_files, int rows,
                              int stride, int64_t* __restrict__ file_out) {
  for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < n_files;
       f += (int64_t)gridDim.x * blockDim.x) {
    const int64_t kept = row_prefix[(f + 1) * rows] - row_prefix[f * rows];
    file_out[f] = (kept + stride - 1) / stride;
  }
}

struct RowGeo {
  const float* scale;   // per row (scale mode) or nullptr
  const float* ranges;  // [row][bin] (ranges mode) or nullptr
  const float* cos_t;
  const float* sin_t;
};

// Row pass 2: write the kept elements whose in-file rank is a multiple of stride.  Each lane ranks
// its kept elements, the emitted ones (bin, value) are staged in the wave's LDS slice in output
// order, and the wave then writes them with full-width coalesced stores (a row emits only
// ~kept/stride points, so storing from the ranking lanes directly would issue ~5 x 16 mostly
// masked store instructions per row).
template <class T, bool VEC>
__global__ __launch_bounds__(kBlock) void k_row_write(
    const T* __restrict__ echo, int64_t n_rows, int rows, int bins, float thr, int stride,
    RowGeo geo, const int32_t* __restrict__ gain, const int64_t* __restrict__ row_prefix,
    const int64_t* __restrict__ file_offsets, int files_per_frame, float* __restrict__ x,
    float* __restrict__ y, float* __restrict__ val, int32_t* __restrict__ gain_out,
    int32_t* __restrict__ pf_out) {
  constexpr int CH = VEC ? 64 * Vec<T>::N : 64;  // bins per chunk
  __shared__ uint16_t s_bin[kWavesPerBlock][CH];
  __shared__ float s_val[kWavesPerBlock][CH];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x / 64;
  const int64_t wave0 = (int64_t)blockIdx.x * kWavesPerBlock + wv;
  const int64_t n_waves = (int64_t)gridDim.x * kWavesPerBlock;
  const float fb = (float)bins;
  const uint32_t ustride = (uint32_t)stride;
  for (int64_t row = wave0; row < n_rows; row += n_waves) {
    const int64_t f = (int64_t)((uint32_t)row / (uint32_t)rows);  // n_rows < 2^32 (host check)
    const T* rp = echo + row * bins;
    // in-file rank of this row's first kept element (< rows*bins, fits 32 bits)
    uint32_t rank = (uint32_t)(row_prefix[row] - row_prefix[f * rows]);
    const int64_t out0 = file_offsets[f];
    const float step = geo.scale ? geo.scale[row] / fb : 0.f;
    const float ct = geo.cos_t[row], st = geo.sin_t[row];
    const int32_t g = gain ? gain[f] : 0;
    const int32_t fr = (int32_t)((uint32_t)f / (uint32_t)files_per_frame);
    for (int base = 0; base < bins; base += CH) {
      int tot;
      if (VEC) {
        constexpr int N = Vec<T>::N;
        using L = typename Vec<T>::L;
        const int b0 = base + lane * N;
        const L v = *reinterpret_cast<const L*>(rp + b0);
        float fv[N];
        Vec<T>::unpack(v, fv);
        int c = 0;
#pragma unroll
        for (int k = 0; k < N; ++k) c += (fv[k] > thr) ? 1 : 0;
        const uint32_t r = rank + (uint32_t)wave_excl_scan(c, &tot);
        if (c) {
          // emitted = kept elements with in-file rank % stride == 0: one 32-bit division per
          // lane, then a countdown; slot = output index - the chunk's first output index
          const uint32_t q = r / ustride, rem = r - q * ustride;
          uint32_t skip = rem ? ustride - rem : 0u;
          int slot = (int)(q + (rem ? 1u : 0u) - (rank + ustride - 1u) / ustride);
#pragma unroll
          for (int k = 0; k < N; ++k) {
            if (fv[k] > thr) {
              if (skip == 0u) {
                s_bin[wv][slot] = (uint16_t)(b0 + k - base);
                s_val[wv][slot] = fv[k];
                ++slot;
                skip = ustride - 1u;
              } else {
                --skip;
              }
            }
          }
        }
      } else {
        const int b = base + lane;
        const float v = (b < bins) ? to_f(rp[b]) : 0.f;
        const bool keep = (b < bins) && (v > thr);
        const uint64_t m = __ballot(keep);
        tot = __popcll(m);
        if (keep) {
          const uint32_t r = rank + (uint32_t)rank_in_mask(m);
          const uint32_t q = r / ustride;
          if (r - q * ustride == 0u) {
            const int slot = (int)(q - (rank + ustride - 1u) / ustride);
            s_bin[wv][slot] = (uint16_t)lane;
            s_val[wv][slot] = v;
          }
        }
      }
      const uint32_t first = (rank + ustride - 1u) / ustride;
      const int n_emit = (int)((rank + (uint32_t)tot + ustride - 1u) / ustride - first);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      for (int l = lane; l < n_emit; l += 64) {
        const int b = base + (int)s_bin[wv][l];
        const int64_t o = out0 + first + l;
        const float rr = geo.ranges ? geo.ranges[row * bins + b] : step * (float)b;
        x[o] = rr * ct;
        y[o] = rr * st;
        val[o] = s_val[wv][l];
        if (gain_out) gain_out[o] = g;
        if (pf_out) pf_out[o] = fr;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      rank += (uint32_t)tot;
    }
  }
}

// ---- u8 fast path (the radar's native sample type), bins == 1024: one 16-B load per lane per
// row.  For integer samples v in [0, 255], (float)v > thr  <=>  v > T with T = floor(thr) clamped
// to [-1, 255] (NaN -> 255: nothing kept), evaluated on 4 bytes at once (SWAR, exact per byte,
// no carries across bytes), K = (HI ? 255 - T : 127 - T) * 0x01010101:
//   T <= 127 : hi bit of ((x & 0x7f..) + K) | x
//   T >= 128 : hi bit of ((x & 0x7f..) + K) & x
template <bool HI>
__device__ __forceinline__ uint32_t keep_bits(uint32_t x, uint32_t K) {
  const uint32_t lo = x & 0x7f7f7f7fu;
  return (HI ? ((lo + K) & x) : ((lo + K) | x)) & 0x80808080u;
}
// The 16 per-byte keep bits of a lane (bytes 0x80 or 0 in m0..m3) -> a 16-bit mask, sample k ->
// bit k: two dot4 products per 8 samples (weights 1..8 and 16..128 on the 0x80 bytes) instead of
// a multiply-gather per dword.
__device__ __forceinline__ uint32_t mask16(uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3) {
  const uint32_t lo = __builtin_amdgcn_udot4(
      m0, 0x08040201u, __builtin_amdgcn_udot4(m1, 0x80402010u, 0u, false), false);
  const uint32_t hi = __builtin_amdgcn_udot4(
      m2, 0x08040201u, __builtin_amdgcn_udot4(m3, 0x80402010u, 0u, false), false);
  return (lo | (hi << 8)) >> 7;
}

// Position of the n-th (0-based) set bit of a 16-bit mask, n < popcount: binary search on
// popcounts of the low half, quarter, ... (v_cndmask selects, no branches).
__device__ __forceinline__ int nth_bit16(uint32_t m, uint32_t n) {
  int p = 0;
  uint32_t c = __popc(m & 0xffu);
  if (n >= c) { n -= c; p = 8; }
  c = __popc((m >> p) & 0xfu);
  if (n >= c) { n -= c; p += 4; }
  c = __popc((m >> p) & 0x3u);
  if (n >= c) { n -= c; p += 2; }
  c = (m >> p) & 1u;
  if (n >= c) p += 1;
  return p;
}

// Rows are handled in groups of kGroupRows consecutive rows of one file (the last group of a file
// may be short): a wave issues the group's loads together (4 KiB in flight) before ranking any of
// them.  The count pass writes one kept count per GROUP; the write pass walks the group's rows in
// order and carries the in-file rank across them, so no per-row reduction or prefix is needed.
constexpr int kGroupRows = 4;  // k_group_write_u8 selects the rows' geometry among 4
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct GroupMap {
  uint32_t gpf;   // groups per file = ceil(rows / kGroupRows)
  int rows;
};
// file, first row of the group in the stack and its row count (all wave-uniform)
__device__ __forceinline__ void group_rows(const GroupMap& gm, uint32_t grp, uint32_t* f,
                                           int64_t* row0, int* nr) {
  const uint32_t ff = grp / gm.gpf;
  const int r0 = (int)(grp - ff * gm.gpf) * kGroupRows;
  *f = ff;
  *row0 = (int64_t)ff * gm.rows + r0;
  *nr = min(kGroupRows, gm.rows - r0);
}

// Kept samples of a group by in-group rank.  A wave leaves its group's per-row inclusive lane
// counts, keep masks and sample bytes in its LDS slice; the kept sample of in-group rank i is then
// found by any lane: row from the row bases (scalar compares), lane by a 6-step binary search of
// the row's inclusive counts, bit by nth_bit16 of that lane's mask.  Work goes to the OUTPUT slots
// (consecutive lanes, full-width stores) instead of walking each input lane's mask bits, so a
// dense lane no longer holds its whole wave in a divergent loop.
struct GroupLds {  // 5 KiB per wave: 8 waves per SIMD fit the LDS (u16 counts and masks)
  uint16_t incl[kGroupRows][64];  // <= 1024
  uint16_t mask[kGroupRows][64];
  uint32_t bytes[kGroupRows][256];  // the group's 4 KiB of samples
};

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// xy bounds of the written points, folded into the K1 write kernels (the land grid's edges need
// them; a separate pass re-read x and y: ~0.1 ms at 1000 frames).  Floats as order-preserving
// u32 (-0 below +0), as k_bounds_xy: {min x, max x, min y, max y}; each block leaves one
// partial, k_bounds_parts reduces them.
__device__ __forceinline__ uint32_t f2ord(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
struct XyBounds {
  uint32_t v[4] = {0xffffffffu, 0u, 0xffffffffu, 0u};
  __device__ void add(float x, float y) {
    const uint32_t a = f2ord(x), b = f2ord(y);
    v[0] = min(v[0], a);
    v[1] = max(v[1], a);
    v[2] = min(v[2], b);
    v[3] = max(v[3], b);
  }
  // whole block (every thread calls it once, after its last add): partial of block blockIdx.x.
  // scratch: 4 LDS words per wave at scratch + 4 * wstride * wave, free for the caller by now
  // (a kernel's own LDS, so the reduction does not add to its LDS size and cost occupancy)
  __device__ void store_block(uint32_t* __restrict__ part, uint32_t* scratch, int wstride) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      v[0] = min(v[0], (uint32_t)__shfl_xor((int)v[0], off));
      v[1] = max(v[1], (uint32_t)__shfl_xor((int)v[1], off));
      v[2] = min(v[2], (uint32_t)__shfl_xor((int)v[2], off));
      v[3] = max(v[3], (uint32_t)__shfl_xor((int)v[3], off));
    }
    if ((threadIdx.x & 63) == 0)
      for (int k = 0; k < 4; ++k) scratch[4 * wstride * (threadIdx.x / 64) + k] = v[k];
    __syncthreads();
    if (threadIdx.x < 4) {
      const int k = threadIdx.x;
      uint32_t r = scratch[k];
      for (int w = 1; w < kWavesPerBlock; ++w) {
        const uint32_t o = scratch[4 * wstride * w + k];
        r = (k & 1) ? max(r, o) : min(r, o);
      }
      part[4 * blockIdx.x + k] = r;
    }
  }
};
__global__ __launch_bounds__(kBlock) void k_bounds_parts(const uint32_t* __restrict__ part, int nb,
                                                        uint32_t* __restrict__ out) {
  XyBounds b;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) {
    b.v[0] = min(b.v[0], part[4 * i + 0]);
    b.v[1] = max(b.v[1], part[4 * i + 1]);
    b.v[2] = min(b.v[2], part[4 * i + 2]);
    b.v[3] = max(b.v[3], part[4 * i + 3]);
  }
  __shared__ uint32_t sm[4 * kWavesPerBlock];
  b.store_block(out - 4 * blockIdx.x, sm, 1);  // one block: out[0..3]
}

__device__ __forceinline__ void group_to_lds(GroupLds& L, int lane, const uint32_t (&m)[kGroupRows],
                                             const int (&incl)[kGroupRows],
                                             const uint4 (&vv)[kGroupRows]) {
#pragma unroll
  for (int k = 0; k < kGroupRows; ++k) {
    L.incl[k][lane] = (uint16_t)incl[k];
    L.mask[k][lane] = (uint16_t)m[k];
    *reinterpret_cast<uint4*>(&L.bytes[k][lane * 4]) = vv[k];
  }
  wave_lds_sync();
}

// (row << 18) | (bin << 8) | sample of the kept sample of in-group rank i (i < rb[kGroupRows];
// rb[k] = kept samples of the rows before row k)
__device__ __forceinline__ uint32_t kept_entry(const GroupLds& L,
                                               const uint32_t (&rb)[kGroupRows + 1], uint32_t i) {
  const int k = (i >= rb[1]) + (i >= rb[2]) + (i >= rb[3]);
  const int ir = (int)(i - rb[k]);
  const uint16_t* inc = L.incl[k];
  int lo = 0;  // lanes whose inclusive count is <= ir
#pragma unroll
  for (int step = 32; step > 0; step >>= 1)
    if (inc[lo + step - 1] <= ir) lo += step;
  const uint32_t msk = L.mask[k][lo];
  const int j = ir - ((int)inc[lo] - __popc(msk));
  const int bit = nth_bit16(msk, (uint32_t)j);
  const int bin = lo * 16 + bit;
  const uint32_t w = L.bytes[k][bin >> 2];
  return ((uint32_t)k << 18) | ((uint32_t)bin << 8) | __builtin_amdgcn_ubfe(w, 8u * (bin & 3), 8u);
}

// Staged kept samples (nullable): when a group keeps at most kStageSlots samples the count pass
// also stores them in in-group rank order, as kept_entry() words, in the group's slot of
// kStageSlots words; the write pass then reads those instead of the group's 4 KiB of echo (one
// read of the echo for the whole K1).  A group that keeps more (dense sweeps) is read from the
// echo again by the write pass.
constexpr int kStageSlots = 512;  // (256: +39 us K1 at 1000 frames, profiles/r6/ab_stage512/)
// Slot position of in-group kept rank i in a staged group of `total` entries.  With stride 4 (the
// reference's POINT_STRIDE) the ranks of each residue mod 4 are contiguous and the four residues
// packed back to back in [0, total): the write pass reads every 4th rank from one residue, i.e.
// consecutive entries, instead of one entry in four from every line of the slot, while the count
// pass still fills one contiguous region per group (a fixed 64-entry stride per residue left four
// partly written lines per sparse group: +9 % on the count pass).
__device__ __forceinline__ uint32_t phase_base(uint32_t ph, uint32_t total) {
  uint32_t b = 0u;
#pragma unroll
  for (uint32_t j = 0u; j < 3u; ++j) b += (j < ph) ? ((total + 3u - j) >> 2) : 0u;
  return b;
}
__device__ __forceinline__ uint32_t stage_pos(uint32_t i, uint32_t total, bool ph4) {
  return ph4 ? phase_base(i & 3u, total) + (i >> 2) : i;
}
// the same with the group's residue bases computed once (wave-uniform: scalar registers)
struct StageBases {
  uint32_t b1, b2, b3;
  __device__ explicit StageBases(uint32_t total)
      : b1((total + 3u) >> 2), b2(b1 + ((total + 2u) >> 2)), b3(b2 + ((total + 1u) >> 2)) {}
  __device__ uint32_t pos(uint32_t i) const {
    const uint32_t r = i & 3u;
    return (r == 0u ? 0u : (r == 1u ? b1 : (r == 2u ? b2 : b3))) + (i >> 2);
  }
};

template <bool HI, bool STAGE>
__global__ __launch_bounds__(kBlock) void k_group_count_u8(const uint8_t* __restrict__ echo,
                                                          uint32_t n_groups, GroupMap gm,
                                                          uint32_t K,
                                                          int32_t* __restrict__ group_count,
                                                          uint32_t* __restrict__ entries,
                                                          int ph4) {
  const int lane = threadIdx.x & 63;
  const uint32_t wave0 = __builtin_amdgcn_readfirstlane(blockIdx.x * kWavesPerBlock +
                                                        threadIdx.x / 64);
  const uint32_t n_waves = gridDim.x * kWavesPerBlock;
  // the group's (file, group-in-file) stepped incrementally: one division per wave, not one per
  // group (a 32-bit division by a runtime value is a few dozen scalar instructions)
  const uint32_t dq = n_waves / gm.gpf, dr = n_waves - dq * gm.gpf;
  uint32_t gf = wave0 / gm.gpf, gr = wave0 - gf * gm.gpf;
  for (uint32_t g0 = wave0; g0 < n_groups; g0 += n_waves) {
    const uint32_t grp = g0;
    const uint32_t f = gf;
    const int r0 = (int)gr * kGroupRows;
    const int64_t row0 = (int64_t)f * gm.rows + r0;
    const int nr = min(kGroupRows, gm.rows - r0);
    gf += dq;
    gr += dr;
    if (gr >= gm.gpf) {
      gr -= gm.gpf;
      ++gf;
    }
    uint4 v[kGroupRows];
#pragma unroll
    for (int k = 0; k < kGroupRows; ++k) {
      // streamed once: non-temporal loads keep the echo out of L2's reuse set
      const u32x4 q = (k < nr) ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(
                                     echo + (row0 + k) * 1024 + lane * 16))
                               : u32x4{0u, 0u, 0u, 0u};
      v[k] = make_uint4(q.x, q.y, q.z, q.w);
    }
    if constexpr (STAGE) {
      uint32_t m[kGroupRows];
      int incl[kGroupRows];
#pragma unroll
      for (int k = 0; k < kGroupRows; ++k)
        m[k] = (k < nr) ? mask16(keep_bits<HI>(v[k].x, K), keep_bits<HI>(v[k].y, K),
                                 keep_bits<HI>(v[k].z, K), keep_bits<HI>(v[k].w, K))
                        : 0u;  // a zero sample is kept when T = -1: rows past nr keep nothing
      // two rows per scan: a row's inclusive lane count is <= 1024, so the low and high halves
      // of one 32-bit DPP scan never carry into each other (the pass is half VALU-bound: PMC)
      static_assert(kGroupRows == 4, "rows are scanned in pairs");
      uint32_t rb[kGroupRows + 1];
      rb[0] = 0;
#pragma unroll
      for (int k = 0; k < kGroupRows; k += 2) {
        const int pair = wave_incl_scan_dpp(__popc(m[k]) | (__popc(m[k + 1]) << 16));
        incl[k] = pair & 0xffff;
        incl[k + 1] = (int)((uint32_t)pair >> 16);
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane(pair, 63);
        rb[k + 1] = rb[k] + (tot & 0xffffu);
        rb[k + 2] = rb[k + 1] + (tot >> 16);
      }
      const uint32_t total = rb[kGroupRows];
      if (total != 0u && total <= (uint32_t)kStageSlots) {  // wave-uniform
        uint32_t* e = entries + (int64_t)grp * kStageSlots;
        __shared__ GroupLds s_lds[kWavesPerBlock];
        GroupLds& L = s_lds[threadIdx.x / 64];
        group_to_lds(L, lane, m, incl, v);
        const StageBases sb(total);
        for (uint32_t i = (uint32_t)lane; i < total; i += 64u)
          e[ph4 ? sb.pos(i) : i] = kept_entry(L, rb, i);
        wave_lds_sync();  // the slice is rewritten by the next group
      }
      if (lane == 0) group_count[grp] = (int32_t)total;
      continue;
    } else {
      uint32_t c = 0;
#pragma unroll
      for (int k = 0; k < kGroupRows; ++k) {
        if (k >= nr) break;  // a zero sample is kept when T = -1
        c += __popc(keep_bits<HI>(v[k].x, K)) + __popc(keep_bits<HI>(v[k].y, K)) +
             __popc(keep_bits<HI>(v[k].z, K)) + __popc(keep_bits<HI>(v[k].w, K));
      }
      int s = (int)c;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
      if (lane == 0) group_count[grp] = s;
    }
  }
}

// file_offsets input: per file ceil(kept / stride) from the group prefix
__global__ void k_file_counts_groups(const int64_t* __restrict__ gprefix, int64_t n_files,
                                     uint32_t gpf, int stride, int64_t* __restrict__ file_out) {
  for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < n_files;
       f += (int64_t)gridDim.x * blockDim.x) {
    const int64_t kept = gprefix[(f + 1) * gpf] - gprefix[f * gpf];
    file_out[f] = (kept + stride - 1) / stride;
  }
}

// Write pass: the kept samples whose in-file rank is a multiple of stride.  The group's emitted
// outputs [first, last) (in-file indices: ceil(rank / stride) ...) go to consecutive lanes; output
// o is the kept sample of in-group rank o * stride - rank, found with kept_entry() from the
// group's LDS slice (or, STAGED, read from the count pass's slot when the group was staged:
// no echo read at all).  Outputs at or beyond cap are dropped: a speculative launch (sized by an
// earlier run) is repeated by the caller when the count says it did not fit.
// LIST: the groups are the first *list_n entries of list (the unstaged groups of the expand
// write below), not 0 .. n_groups-1.
template <bool HI, bool STAGED, bool LIST = false>
__global__ __launch_bounds__(kBlock, 8) void k_group_write_u8(
    const uint8_t* __restrict__ echo, uint32_t n_groups, GroupMap gm, uint32_t K, int stride,
    const float* __restrict__ scale, const float* __restrict__ cos_t,
    const float* __restrict__ sin_t, const int32_t* __restrict__ gain,
    const int64_t* __restrict__ gprefix, const int64_t* __restrict__ file_offsets,
    int files_per_frame, float* __restrict__ x, float* __restrict__ y, float* __restrict__ val,
    int32_t* __restrict__ gain_out, int32_t* __restrict__ pf_out, int64_t cap,
    const uint32_t* __restrict__ entries, const uint32_t* __restrict__ list = nullptr,
    const uint32_t* __restrict__ list_n = nullptr, uint32_t* __restrict__ bpart = nullptr) {
  // bpart (nullable, kernel-uniform): this block's xy-bounds partial (XyBounds)
  __shared__ GroupLds s_lds[kWavesPerBlock];
  XyBounds xb;
  const int lane = threadIdx.x & 63;
  GroupLds& L = s_lds[threadIdx.x / 64];
  const uint32_t wave0 = blockIdx.x * kWavesPerBlock + threadIdx.x / 64;
  const uint32_t n_waves = gridDim.x * kWavesPerBlock;
  const uint32_t us = (uint32_t)stride;
  const bool pow2 = (us & (us - 1u)) == 0u;
  const uint32_t sh = (uint32_t)__builtin_ctz(us);
  const float inv_bins = 1.0f / 1024.0f;  // exact: step = scale / 1024 == scale * 2^-10
  const uint32_t n_items = LIST ? *list_n : n_groups;
  for (uint32_t g0 = wave0; g0 < n_items; g0 += n_waves) {
    const uint32_t grp = __builtin_amdgcn_readfirstlane(LIST ? list[g0] : g0);
    uint32_t f;
    int64_t row0;
    int nr;
    group_rows(gm, grp, &f, &row0, &nr);
    // the group's rows' geometry, loaded by lanes 0..3 together with the prefix reads (one
    // dependent load level less per output: ent -> row -> geometry becomes a lane shuffle)
    float g_sc = 0.f, g_c = 0.f, g_s = 0.f;
    if (lane < nr) {
      g_sc = scale[row0 + lane];
      g_c = cos_t[row0 + lane];
      g_s = sin_t[row0 + lane];
    }
    float r_sc[kGroupRows], r_c[kGroupRows], r_s[kGroupRows];  // wave-uniform (readlane)
#pragma unroll
    for (int k = 0; k < kGroupRows; ++k) {
      r_sc[k] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, g_sc), k));
      r_c[k] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, g_c), k));
      r_s[k] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, g_s), k));
    }
    // in-file rank of the group's first kept sample (< rows * 1024 < 2^32), its kept count, the
    // group's emitted outputs [first, last) and the file's output base
    const int64_t gp0 = gprefix[grp];
    const uint32_t rank = (uint32_t)(gp0 - gprefix[(int64_t)f * gm.gpf]);
    const uint32_t total = (uint32_t)(gprefix[grp + 1] - gp0);
    const uint32_t first = pow2 ? ((rank + us - 1u) >> sh) : (rank + us - 1u) / us;
    const uint32_t last = pow2 ? ((rank + total + us - 1u) >> sh) : (rank + total + us - 1u) / us;
    if (last == first) continue;  // wave-uniform: nothing emitted
    const int64_t out0 = file_offsets[f];
    const int32_t g = gain ? gain[f] : 0;
    const int32_t fr = (int32_t)(f / (uint32_t)files_per_frame);
    const bool staged = STAGED && total <= (uint32_t)kStageSlots;
    uint32_t rb[kGroupRows + 1];
    if (!staged) {
      uint4 vv[kGroupRows];
#pragma unroll
      for (int k = 0; k < kGroupRows; ++k)
        vv[k] = (k < nr) ? *reinterpret_cast<const uint4*>(echo + (row0 + k) * 1024 + lane * 16)
                         : make_uint4(0u, 0u, 0u, 0u);
      uint32_t m[kGroupRows];
      int incl[kGroupRows];
#pragma unroll
      for (int k = 0; k < kGroupRows; ++k) {
        m[k] = (k < nr) ? mask16(keep_bits<HI>(vv[k].x, K), keep_bits<HI>(vv[k].y, K),
                                 keep_bits<HI>(vv[k].z, K), keep_bits<HI>(vv[k].w, K))
                        : 0u;
        incl[k] = wave_incl_scan_dpp(__popc(m[k]));
      }
      rb[0] = 0;
#pragma unroll
      for (int k = 0; k < kGroupRows; ++k)
        rb[k + 1] = rb[k] + (uint32_t)__builtin_amdgcn_readlane(incl[k], 63);
      group_to_lds(L, lane, m, incl, vv);
    }
    const uint32_t* e = entries + (int64_t)grp * kStageSlots;
    for (uint32_t o = first + (uint32_t)lane; o < last; o += 64u) {
      const int64_t oo = out0 + o;
      if (oo >= cap) break;
      const uint32_t i = o * us - rank;  // in-group kept rank
      const uint32_t ent = staged ? e[stage_pos(i, total, us == 4u)] : kept_entry(L, rb, i);
      const int rk = (int)(ent >> 18);
      const float sc = rk == 0 ? r_sc[0] : (rk == 1 ? r_sc[1] : (rk == 2 ? r_sc[2] : r_sc[3]));
      const float cc = rk == 0 ? r_c[0] : (rk == 1 ? r_c[1] : (rk == 2 ? r_c[2] : r_c[3]));
      const float ss = rk == 0 ? r_s[0] : (rk == 1 ? r_s[1] : (rk == 2 ? r_s[2] : r_s[3]));
      const float rr = sc * inv_bins * (float)((ent >> 8) & 1023u);
      const float px = rr * cc, py = rr * ss;
      x[oo] = px;
      y[oo] = py;
      if (bpart) xb.add(px, py);
      val[oo] = (float)(ent & 0xffu);
      if (gain_out) gain_out[oo] = g;
      if (pf_out) pf_out[oo] = fr;
    }
    if (!staged) wave_lds_sync();  // the slice is rewritten by the next group
  }
  // (every wave is past its last group: each one's own LDS slice is free)
  if (bpart)
    xb.store_block(bpart, reinterpret_cast<uint32_t*>(&s_lds[0]),
                   (int)(sizeof(GroupLds) / sizeof(uint32_t) / 4));
}

// ---- expand write: output slots to threads (staged groups)
// The wave-per-group write above walks 3 M groups of ~16 outputs each with a dependent
// prefix -> entry -> store chain per group; its time is that chain times the groups per wave
// slot.  Here the outputs themselves are spread over the threads: per group one 64-bit word
//   bits 0..39  gs    = global index of the group's first emitted output
//   bits 40..62 phase = in-group kept rank of that output (first * stride - rank < stride)
//   bit 63      the group emits outputs but kept > kStageSlots samples (not staged): its
//               outputs are written by k_group_write_u8<.., LIST> over the list of such groups
// and a block walks a contiguous range of 1024-output tiles, finding each output's group by a
// binary search of an LDS window of those words (gs is non-decreasing in the group index).
constexpr int kGsBits = 40;
constexpr uint64_t kGsMask = (1ull << kGsBits) - 1ull;
constexpr uint64_t kUnstaged = 1ull << 63;
constexpr int kTileOut = 1024;  // outputs per block tile, 4 per thread (8: 86 VGPRs, slower)
constexpr int kOutPerThread = kTileOut / kBlock;
static_assert(kOutPerThread % 4 == 0, "k_expand_write stores a thread's outputs as 16-B vectors");
constexpr int kWin = 1024;  // groups in the LDS window

__global__ __launch_bounds__(kBlock) void k_group_starts(const int64_t* __restrict__ gprefix,
                                                        const int64_t* __restrict__ file_offsets,
                                                        uint32_t n_groups, uint32_t gpf,
                                                        uint32_t stride,
                                                        uint64_t* __restrict__ gword,
                                                        uint32_t* __restrict__ list,
                                                        uint32_t* __restrict__ list_n) {
  // the unstaged groups collect in a block LDS list over the whole grid-stride loop and go out
  // with ONE global atomic per block (one per block iteration was ~12 k same-address atomics per
  // 1000-frame stack, serialised in L2); a block whose list fills appends the rest directly
  constexpr uint32_t kCap = 2048;
  __shared__ uint32_t s_list[kCap];
  __shared__ uint32_t s_n, s_base;
  if (threadIdx.x == 0) s_n = 0u;
  __syncthreads();
  // power-of-two strides (the reference's 4) by shifts instead of 64-bit divisions
  const bool pow2 = (stride & (stride - 1u)) == 0u;
  const uint32_t sh = (uint32_t)__builtin_ctz(stride);
  for (uint32_t b0 = blockIdx.x * kBlock; b0 < n_groups; b0 += gridDim.x * kBlock) {
    const uint32_t g = b0 + threadIdx.x;
    if (g < n_groups) {
      const uint32_t f = g / gpf;
      const int64_t p0 = gprefix[g];
      const uint64_t rank = (uint64_t)(p0 - gprefix[(int64_t)f * gpf]);
      const uint64_t total = (uint64_t)(gprefix[g + 1] - p0);
      const uint64_t first = pow2 ? ((rank + stride - 1u) >> sh) : (rank + stride - 1u) / stride;
      const uint64_t last =
          pow2 ? ((rank + total + stride - 1u) >> sh) : (rank + total + stride - 1u) / stride;
      const uint64_t gs = (uint64_t)file_offsets[f] + first;
      // slot position of the first emitted output's entry: its in-group rank, or with stride 4
      // (residues packed, stage_pos) the base of its residue
      const uint64_t ph = first * stride - rank;
      const uint64_t phase = stride == 4u ? (uint64_t)phase_base((uint32_t)ph, (uint32_t)total)
                                          : ph;
      const bool un = last > first && total > (uint64_t)kStageSlots;
      gword[g] = gs | (phase << kGsBits) | (un ? kUnstaged : 0ull);
      if (un) {
        const uint32_t slot = atomicAdd(&s_n, 1u);
        if (slot < kCap)
          s_list[slot] = g;
        else
          list[atomicAdd(list_n, 1u)] = g;
      }
    }
  }
  __syncthreads();
  const uint32_t m = min(s_n, kCap);
  if (threadIdx.x == 0 && m) s_base = atomicAdd(list_n, m);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < m; i += kBlock) list[s_base + i] = s_list[i];
}

// largest g in [lo, hi) with gs(g) <= O, given gs(lo) <= O: one wave, 64-ary search
__device__ uint32_t wave_find_group(const uint64_t* __restrict__ gword, uint32_t lo, uint32_t hi,
                                    uint64_t O) {
  const uint32_t lane = threadIdx.x & 63u;
  while (hi - lo > 1u) {
    const uint32_t step = (hi - lo + 63u) / 64u;
    const uint32_t idx = lo + lane * step;
    const bool le = idx < hi && (gword[idx] & kGsMask) <= O;  // a prefix of the lanes
    const uint64_t m = __ballot(le);
    const uint32_t top = 63u - (uint32_t)__clzll((long long)m);
    lo = __builtin_amdgcn_readfirstlane(lo + top * step);
    hi = min(hi, lo + step);
  }
  return lo;
}

// same, one thread (the rare outputs beyond the LDS window)
__device__ uint32_t thread_find_group(const uint64_t* __restrict__ gword, uint32_t lo,
                                      uint32_t hi, uint64_t O) {
  while (hi - lo > 1u) {
    const uint32_t mid = lo + (hi - lo) / 2u;
    if ((gword[mid] & kGsMask) <= O)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

// largest j < wn with s_win[j].gs <= O (s_win[0].gs <= O)
__device__ __forceinline__ uint32_t lds_find(const uint64_t* s_win, uint32_t wn, uint64_t O) {
  uint32_t lo = 0u;
#pragma unroll
  for (uint32_t step = kWin / 2; step > 0u; step >>= 1)
    if (lo + step < wn && (s_win[lo + step] & kGsMask) <= O) lo += step;
  return lo;
}

// VEC: every output array is 16-B aligned (float4 / int4 stores of a thread's 4 outputs)
template <bool VEC>
__global__ __launch_bounds__(kBlock) void k_expand_write(
    const uint64_t* __restrict__ gword, uint32_t n_groups, GroupMap gm, uint32_t stride,
    const float* __restrict__ scale, const float* __restrict__ cos_t,
    const float* __restrict__ sin_t, const int32_t* __restrict__ gain,
    const int64_t* __restrict__ total_out, int files_per_frame, float* __restrict__ x,
    float* __restrict__ y, float* __restrict__ val, int32_t* __restrict__ gain_out,
    int32_t* __restrict__ pf_out, int64_t cap, const uint32_t* __restrict__ entries,
    uint32_t* __restrict__ bpart = nullptr) {
  // bpart (nullable): this block's xy-bounds partial of the outputs it writes (XyBounds)
  __shared__ uint64_t s_win[kWin];
  __shared__ uint32_t s_glo;
  const int64_t total = min(*total_out, cap);
  const int64_t n_tiles = (total + kTileOut - 1) / kTileOut;
  const int64_t t0 = n_tiles * blockIdx.x / gridDim.x;
  const int64_t t1 = n_tiles * (blockIdx.x + 1) / gridDim.x;
  if (t0 >= t1) {  // block-uniform
    if (bpart && threadIdx.x < 4)  // (no outputs: the identity)
      bpart[4 * blockIdx.x + threadIdx.x] = (threadIdx.x & 1) ? 0u : 0xffffffffu;
    return;
  }
  if (threadIdx.x < 64) {
    const uint32_t g = wave_find_group(gword, 0u, n_groups, (uint64_t)t0 * kTileOut);
    if (threadIdx.x == 0) s_glo = g;
  }
  __syncthreads();
  // the window of the next tile is loaded into registers while this tile's entries, geometry and
  // stores are in flight (its first group is known once phase A has searched this window)
  constexpr int kWinPer = kWin / kBlock;
  uint64_t wv[kWinPer];
  auto load_win = [&](uint32_t glo_) {
    const uint32_t wn_ = min((uint32_t)kWin, n_groups - glo_);
#pragma unroll
    for (int q = 0; q < kWinPer; ++q) {
      const uint32_t j = threadIdx.x + q * kBlock;
      wv[q] = j < wn_ ? gword[glo_ + j] : ~0ull;
    }
  };
  auto store_win = [&]() {
#pragma unroll
    for (int q = 0; q < kWinPer; ++q) s_win[threadIdx.x + q * kBlock] = wv[q];
  };
  uint32_t glo = s_glo;
  XyBounds xb;
  load_win(glo);
  store_win();
  __syncthreads();
  const float inv_bins = 1.0f / 1024.0f;  // exact: step = scale / 1024 == scale * 2^-10
  for (int64_t t = t0; t < t1; ++t) {
    const uint32_t wn = min((uint32_t)kWin, n_groups - glo);
    const bool truncated = glo + wn < n_groups;
    const uint64_t O0 = (uint64_t)t * kTileOut;
    // phase A: this thread's kOutPerThread consecutive outputs: the first one's group by the LDS
    // search, the others by stepping over group starts (empty groups share their successor's)
    auto word = [&](uint32_t g) -> uint64_t {
      return (g - glo < wn) ? s_win[g - glo] : gword[g];
    };
    auto next_gs = [&](uint32_t g) -> uint64_t {
      return g + 1u < n_groups ? (word(g + 1u) & kGsMask) : ~0ull;
    };
    const uint64_t Ob = O0 + (uint64_t)threadIdx.x * kOutPerThread;
    uint32_t grp[kOutPerThread], idx[kOutPerThread];
    bool ok[kOutPerThread];
    if ((int64_t)Ob < total) {
      const uint32_t j = lds_find(s_win, wn, Ob);
      uint32_t g = (j == wn - 1u && truncated) ? thread_find_group(gword, glo + j, n_groups, Ob)
                                               : glo + j;
      uint64_t w = word(g), nx = next_gs(g);
#pragma unroll
      for (int k = 0; k < kOutPerThread; ++k) {
        const uint64_t O = Ob + k;
        const bool in = (int64_t)O < total;
        while (in && O >= nx) {
          ++g;
          w = word(g);
          nx = next_gs(g);
        }
        ok[k] = in && !(w & kUnstaged);
        grp[k] = g;
        // the entry's slot position, mod 2^32 like the 64-bit form (only staged groups use it:
        // idx < kStageSlots): consecutive outputs are consecutive entries with stride 4
        const uint32_t d = (uint32_t)O - (uint32_t)w;
        idx[k] = (stride == 4u ? d : d * stride) + (uint32_t)((w & ~kUnstaged) >> kGsBits);
      }
    } else {
#pragma unroll
      for (int k = 0; k < kOutPerThread; ++k) {
        ok[k] = false;
        grp[k] = glo;
        idx[k] = 0u;
      }
    }
    // the next tile's first group (thread 0), before the window is rewritten
    if (threadIdx.x == 0 && t + 1 < t1) {
      const uint64_t On = O0 + kTileOut;
      const uint32_t j = lds_find(s_win, wn, On);
      s_glo = (j == wn - 1u && truncated) ? thread_find_group(gword, glo + j, n_groups, On)
                                          : glo + j;
    }
    __syncthreads();  // every search of this window done; s_glo of the next tile visible
    if (t + 1 < t1) {
      glo = s_glo;
      load_win(glo);
    }
    // phase B: the staged entries, then the rows' geometry, then the stores
    uint32_t ent[kOutPerThread];
    // every load unconditional (a slot that writes nothing reads entry 0 / its group's first
    // row) and masked by selects: conditional loads would each end in a full vmcnt wait
#pragma unroll
    for (int k = 0; k < kOutPerThread; ++k) {
      const uint32_t e = entries[ok[k] ? (int64_t)grp[k] * kStageSlots + idx[k] : 0];
      ent[k] = ok[k] ? e : 0u;
    }
    float sc[kOutPerThread], cc[kOutPerThread], ss[kOutPerThread];
    uint32_t fl[kOutPerThread], pfl[kOutPerThread];
    // one division per thread: its outputs' groups are grp[0] or a few after it (steps over
    // file / frame boundaries instead of dividing again)
    const uint32_t f0 = grp[0] / gm.gpf, r0 = grp[0] - f0 * gm.gpf;
    const uint32_t fpf = (uint32_t)files_per_frame, p0 = f0 / fpf, q0 = f0 - p0 * fpf;
#pragma unroll
    for (int k = 0; k < kOutPerThread; ++k) {
      uint32_t f = f0, r = r0 + (grp[k] - grp[0]);
      while (r >= gm.gpf) {
        r -= gm.gpf;
        ++f;
      }
      uint32_t pf = p0, q = q0 + (f - f0);
      while (q >= fpf) {
        q -= fpf;
        ++pf;
      }
      fl[k] = f;
      pfl[k] = pf;
      const int64_t row = (int64_t)f * gm.rows + (int64_t)r * kGroupRows + (ent[k] >> 18);
      sc[k] = scale[row];
      cc[k] = cos_t[row];
      ss[k] = sin_t[row];
    }
    float ox[kOutPerThread], oy[kOutPerThread], ov[kOutPerThread];
    int32_t og[kOutPerThread], op[kOutPerThread];
    bool all_ok = true;
#pragma unroll
    for (int k = 0; k < kOutPerThread; ++k) {
      const float rr = sc[k] * inv_bins * (float)((ent[k] >> 8) & 1023u);
      ox[k] = rr * cc[k];
      oy[k] = rr * ss[k];
      ov[k] = (float)(ent[k] & 0xffu);
      og[k] = gain ? gain[fl[k]] : 0;
      op[k] = (int32_t)pfl[k];
      all_ok = all_ok && ok[k];
      if (bpart && ok[k]) xb.add(ox[k], oy[k]);
    }
    if (VEC && all_ok) {  // 16-B stores (the common case)
#pragma unroll
      for (int h = 0; h < kOutPerThread; h += 4) {
        const uint64_t o = Ob + h;
        *reinterpret_cast<float4*>(x + o) = make_float4(ox[h], ox[h + 1], ox[h + 2], ox[h + 3]);
        *reinterpret_cast<float4*>(y + o) = make_float4(oy[h], oy[h + 1], oy[h + 2], oy[h + 3]);
        *reinterpret_cast<float4*>(val + o) = make_float4(ov[h], ov[h + 1], ov[h + 2], ov[h + 3]);
        if (gain_out)
          *reinterpret_cast<int4*>(gain_out + o) = make_int4(og[h], og[h + 1], og[h + 2], og[h + 3]);
        if (pf_out)
          *reinterpret_cast<int4*>(pf_out + o) = make_int4(op[h], op[h + 1], op[h + 2], op[h + 3]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < kOutPerThread; ++k) {
        if (!ok[k]) continue;
        const uint64_t oo = Ob + k;
        x[oo] = ox[k];
        y[oo] = oy[k];
        val[oo] = ov[k];
        if (gain_out) gain_out[oo] = og[k];
        if (pf_out) pf_out[oo] = op[k];
      }
    }
    if (t + 1 < t1) store_win();
    __syncthreads();  // the next tile's window
  }
  if (bpart) xb.store_block(bpart, reinterpret_cast<uint32_t*>(s_win), 1);  // (window done)
}

// integer threshold of u8 samples (see keep_bits)
inline int u8_threshold(float thr) {
  if (!(thr == thr)) return 255;
  const double f = std::floor((double)thr);
  return f < -1.0 ? -1 : (f > 255.0 ? 255 : (int)f);
}

template <class T>
constexpr bool is_u8() { return false; }
template <>
constexpr bool is_u8<uint8_t>() { return true; }

// The grouped u8 kernels take u8 sweeps of exactly 1024 bins with 16-B aligned rows; row_prefix
// then holds the per-GROUP exclusive prefix (n_files * ceil(rows / 4) + 1 values), otherwise the
// per-row one.  Count and write decide the same way from the same arguments.
template <class T>
bool grouped_u8(const T* echo, int bins) {
  return is_u8<T>() && bins == 1024 && (uintptr_t)echo % 16 == 0;
}

inline uint32_t u8_k(int T) {
  return (uint32_t)(T <= 127 ? 127 - T : 255 - T) * 0x01010101u;
}

// k_expand_write: a persistent grid (8 blocks per CU of the 256; each walks a contiguous tile
// range).  RPT_K1_EXPAND=0 keeps the wave-per-group write for A/B runs.
constexpr int kExpandBlocks = 2048;
constexpr int kListBlocks = 2048;  // blocks of the unstaged groups' write (at most)
inline bool expand_write_enabled() {
  static const bool on = [] {
    const char* e = ab_env("RPT_K1_EXPAND");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}

template <class T>
int32_t count_impl(const T* echo, int64_t n_files, int rows, int bins, float thr, int stride,
                   int64_t* row_prefix, int64_t* file_offsets, int64_t* total_host,
                   hipStream_t st, uint32_t* entries = nullptr) {
  const int64_t n_rows = n_files * rows;
  if ((int64_t)rows * bins >= (int64_t(1) << 32) || n_rows >= (int64_t(1) << 32)) {
    set_error("rpt_polar_count: rows*bins and n_files*rows must be < 2^32");
    return RPT_ENOTSUP;
  }
  const bool grouped = grouped_u8(echo, bins);
  const GroupMap gm{(uint32_t)((rows + kGroupRows - 1) / kGroupRows), rows};
  const int64_t n_units = grouped ? n_files * (int64_t)gm.gpf : n_rows;
  Scratch& sc = scratch(st);
  Budget b;
  b.add<int32_t>(n_units);
  b.add<int64_t>(n_files);
  RPT_TRY(sc.reserve(b.bytes, st));
  int32_t* rc = sc.carve_n<int32_t>(n_units);
  int64_t* fo = sc.carve_n<int64_t>(n_files);
  const bool vec = (bins % (64 * Vec<T>::N) == 0) && ((uintptr_t)echo % 16 == 0);
  const int grid = grid_for(n_units, kWavesPerBlock, 16384);
  if (grouped) {
    const int T8 = u8_threshold(thr);
    const auto* e8 = reinterpret_cast<const uint8_t*>(echo);
#define RPT_K1C(HI, S)                                                                    \
  hipLaunchKernelGGL((k_group_count_u8<HI, S>), dim3(grid), dim3(kBlock), 0, st, e8,        \
                     (uint32_t)n_units, gm, u8_k(T8), rc, entries, stride == 4 ? 1 : 0)
    if (entries) {
      if (T8 <= 127)
        RPT_K1C(false, true);
      else
        RPT_K1C(true, true);
    } else if (T8 <= 127) {
      RPT_K1C(false, false);
    } else {
      RPT_K1C(true, false);
    }
#undef RPT_K1C
  } else if (vec) {
    hipLaunchKernelGGL((k_row_count<T, true>), dim3(grid), dim3(kBlock), 0, st, echo, n_rows,
                       bins, thr, rc);
  } else {
    hipLaunchKernelGGL((k_row_count<T, false>), dim3(grid), dim3(kBlock), 0, st, echo, n_rows,
                       bins, thr, rc);
  }
  RPT_CHECK_LAUNCH();
  RPT_TRY(exclusive_scan_total_i32_to_i64(rc, row_prefix, n_units, st));
  if (grouped)
    hipLaunchKernelGGL(k_file_counts_groups, dim3(grid_for(n_files, 256, 1024)), dim3(256), 0, st,
                       row_prefix, n_files, gm.gpf, stride, fo);
  else
    hipLaunchKernelGGL(k_file_counts, dim3(grid_for(n_files, 256, 1024)), dim3(256), 0, st,
                       row_prefix, n_files, rows, stride, fo);
  RPT_CHECK_LAUNCH();
  RPT_TRY(exclusive_scan_total_i64(fo, file_offsets, n_files, st));
  if (total_host) {
    RPT_HIP(hipMemcpyAsync(total_host, file_offsets + n_files, sizeof(int64_t),
                           hipMemcpyDeviceToHost, st));
    RPT_TRY(wait_stream(st));
  }
  return RPT_OK;
}

template <class T>
int32_t write_impl(const T* echo, int64_t n_files, int rows, int bins, float thr, int stride,
                   RowGeo geo, const int32_t* gain, const int64_t* row_prefix,
                   const int64_t* file_offsets, int fpf, float* x, float* y, float* v,
                   int32_t* gout, int32_t* pf, hipStream_t st, int64_t cap = INT64_MAX,
                   const uint32_t* entries = nullptr, uint32_t* bnd = nullptr,
                   bool* bnd_done = nullptr) {
  // bnd (nullable; polar_bounds_words() words): on the expand-write path the written points' xy
  // bounds land in bnd[0..3] (ordered u32, as k_bounds_xy) and *bnd_done is set
  if (bnd_done) *bnd_done = false;
  const int64_t n_rows = n_files * rows;
  if ((int64_t)rows * bins >= (int64_t(1) << 32) || n_rows >= (int64_t(1) << 32) || stride < 1 ||
      fpf < 1) {
    set_error("rpt_polar_write: rows*bins and n_files*rows must be < 2^32, stride/fpf >= 1");
    return RPT_ENOTSUP;
  }
  const bool vec = (bins % (64 * Vec<T>::N) == 0) && ((uintptr_t)echo % 16 == 0);
  if (grouped_u8(echo, bins) && geo.scale) {
    const GroupMap gm{(uint32_t)((rows + kGroupRows - 1) / kGroupRows), rows};
    const int64_t n_groups = n_files * (int64_t)gm.gpf;
    const int grid = grid_for(n_groups, kWavesPerBlock, 16384);
    const int T8 = u8_threshold(thr);
    const auto* e8 = reinterpret_cast<const uint8_t*>(echo);
    if (entries && expand_write_enabled() && stride < (1 << 23) &&
        n_files * (int64_t)rows * 1024 < (int64_t(1) << kGsBits)) {
      // staged entries: outputs to threads (k_expand_write); the few unstaged groups listed by
      // k_group_starts are written by the wave-per-group kernel
      Scratch& sc = scratch(st);
      Budget b;
      b.add<uint64_t>(n_groups);
      b.add<uint32_t>(n_groups);
      RPT_TRY(sc.reserve(b.bytes, st));
      uint64_t* gword = sc.carve_n<uint64_t>(n_groups);
      uint32_t* list = sc.carve_n<uint32_t>(n_groups);
      uint32_t* list_n = nullptr;
      RPT_TRY(zero_n(st, 1, &list_n));
      hipLaunchKernelGGL(k_group_starts, dim3(grid_for(n_groups, kBlock, 4096)), dim3(kBlock), 0,
                         st, row_prefix, file_offsets, (uint32_t)n_groups, gm.gpf,
                         (uint32_t)stride, gword, list, list_n);
      RPT_CHECK_LAUNCH();
      auto al16 = [](const void* q) { return ((uintptr_t)q & 15u) == 0; };
      const bool vec4 = al16(x) && al16(y) && al16(v) && (!gout || al16(gout)) && (!pf || al16(pf));
      if (vec4)
        hipLaunchKernelGGL(k_expand_write<true>, dim3(kExpandBlocks), dim3(kBlock), 0, st, gword,
                           (uint32_t)n_groups, gm, (uint32_t)stride, geo.scale, geo.cos_t,
                           geo.sin_t, gain, file_offsets + n_files, fpf, x, y, v, gout, pf, cap,
                           entries, bnd ? bnd + 4 : nullptr);
      else
        hipLaunchKernelGGL(k_expand_write<false>, dim3(kExpandBlocks), dim3(kBlock), 0, st,
                           gword, (uint32_t)n_groups, gm, (uint32_t)stride, geo.scale, geo.cos_t,
                           geo.sin_t, gain, file_offsets + n_files, fpf, x, y, v, gout, pf, cap,
                           entries, bnd ? bnd + 4 : nullptr);
      RPT_CHECK_LAUNCH();
      const int lgrid = std::min(grid, kListBlocks);
#define RPT_K1L(HI)                                                                            \
  hipLaunchKernelGGL((k_group_write_u8<HI, false, true>), dim3(lgrid), dim3(kBlock), 0, st, e8, \
                     (uint32_t)n_groups, gm, u8_k(T8), stride, geo.scale, geo.cos_t, geo.sin_t,  \
                     gain, row_prefix, file_offsets, fpf, x, y, v, gout, pf, cap, entries, list, \
                     list_n, bnd ? bnd + 4 + 4 * kExpandBlocks : nullptr)
      if (T8 <= 127)
        RPT_K1L(false);
      else
        RPT_K1L(true);
#undef RPT_K1L
      if (bnd) {
        hipLaunchKernelGGL(k_bounds_parts, dim3(1), dim3(kBlock), 0, st, bnd + 4,
                           kExpandBlocks + lgrid, bnd);
        if (bnd_done) *bnd_done = true;
      }
      RPT_CHECK_LAUNCH();
      return RPT_OK;
    }
#define RPT_K1W(HI, M)                                                                       \
  hipLaunchKernelGGL((k_group_write_u8<HI, M>), dim3(grid), dim3(kBlock), 0, st, e8,          \
                     (uint32_t)n_groups, gm, u8_k(T8), stride, geo.scale, geo.cos_t, geo.sin_t, \
                     gain, row_prefix, file_offsets, fpf, x, y, v, gout, pf, cap, entries)
    if (entries) {
      if (T8 <= 127)
        RPT_K1W(false, true);
      else
        RPT_K1W(true, true);
    } else if (T8 <= 127) {
      RPT_K1W(false, false);
    } else {
      RPT_K1W(true, false);
    }
#undef RPT_K1W
  } else if (cap != INT64_MAX) {
    set_error("rpt_polar_write: a capacity-bounded write needs u8 sweeps of 1024 bins");
    return RPT_ENOTSUP;
  } else if (grouped_u8(echo, bins)) {
    set_error("rpt_polar_write: u8 sweeps take per-row scale geometry");
    return RPT_ENOTSUP;
  } else if (vec) {
    const int grid = grid_for(n_rows, kWavesPerBlock, 16384);
    hipLaunchKernelGGL((k_row_write<T, true>), dim3(grid), dim3(kBlock), 0, st, echo, n_rows,
                       rows, bins, thr, stride, geo, gain, row_prefix, file_offsets, fpf, x, y,
                       v, gout, pf);
  } else {
    const int grid = grid_for(n_rows, kWavesPerBlock, 16384);
    hipLaunchKernelGGL((k_row_write<T, false>), dim3(grid), dim3(kBlock), 0, st, echo, n_rows,
                       rows, bins, thr, stride, geo, gain, row_prefix, file_offsets, fpf, x, y,
                       v, gout, pf);
  }
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

__global__ void k_frame_times(const int32_t* __restrict__ pf, int64_t n,
                              const int64_t* __restrict__ ids, float* __restrict__ t,
                              const int64_t* __restrict__ n_dev) {
  if (n_dev) n = *n_dev;  // count on the device (at most the host n the grid was sized for)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t f = pf[i];
    t[i] = (float)(ids ? ids[f] : (int64_t)f);
  }
}

__global__ void k_polar_dense(const float* __restrict__ cos_t, const float* __restrict__ sin_t,
                              const float* __restrict__ ranges, int64_t rows, int64_t bins,
                              float* __restrict__ x, float* __restrict__ y) {
  const int64_t n = rows * bins;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / bins;
    const float rr = ranges[i];
    x[i] = rr * cos_t[r];
    y[i] = rr * sin_t[r];
  }
}

// ---------------------------------------------------------------- colour -> time
// clustering.py:39-46: diffs f32, dist2 = ((d0*d0) + d1*d1) + d2*d2, first argmin.
__global__ void k_colors(const uint8_t* __restrict__ colors, int64_t n,
                         const float* __restrict__ pal, int n_pal, float* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float r = colors[3 * i], g = colors[3 * i + 1], b = colors[3 * i + 2];
    int best = 0;
    float bd = 0.f;
    for (int k = 0; k < n_pal; ++k) {
      const float d0 = r - pal[3 * k], d1 = g - pal[3 * k + 1], d2 = b - pal[3 * k + 2];
      float d = d0 * d0;
      d = d + d1 * d1;
      d = d + d2 * d2;
      // np.argmin: first minimum; a NaN wins immediately (cannot occur for u8 colours)
      if (k == 0 || d < bd) {
        bd = d;
        best = k;
      }
    }
    out[i] = (float)best;
  }
}

// ---------------------------------------------------------------- synthetic echo
// Bit-identical restatement: rpt/synth.py::numpy_echo.
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

constexpr int kMaxTargets = 256;

// One block per (frame, gain, row); threads sweep the bins.
__global__ __launch_bounds__(kBlock) void k_synth(rpt_synth_params p, int64_t frame0,
                                                 int64_t n_frames, const float* __restrict__ cos_t,
                                                 const float* __restrict__ sin_t,
                                                 const uint32_t* __restrict__ clutter_thresh,
                                                 const float* __restrict__ targets,
                                                 const int32_t* __restrict__ trows,
                                                 const int32_t* __restrict__ tbins,
                                                 uint8_t* __restrict__ echo) {
  __shared__ int hits[kMaxTargets];
  __shared__ int n_hits;
  const int64_t n_rows_total = n_frames * p.n_gains * p.rows;
  for (int64_t rr = blockIdx.x; rr < n_rows_total; rr += gridDim.x) {
    const int row = (int)(rr % p.rows);
    const int64_t fg = rr / p.rows;
    const int gi = (int)(fg % p.n_gains);
    const int64_t fl = fg / p.n_gains;  // local frame
    const int64_t fa = frame0 + fl;      // absolute frame (hash input)
    __syncthreads();
    if (threadIdx.x == 0) n_hits = 0;
    __syncthreads();
    for (int k = threadIdx.x; k < p.n_targets; k += blockDim.x) {
      const int32_t* tr = trows + (fl * p.n_targets + k) * 2;
      if (row >= tr[0] && row <= tr[1]) hits[atomicAdd(&n_hits, 1)] = k;
    }
    __syncthreads();
    const int nh = n_hits;
    // deterministic target order: insertion sort of the (few) hits
    if (threadIdx.x == 0) {
      for (int a = 1; a < nh; ++a) {
        const int v = hits[a];
        int b = a - 1;
        while (b >= 0 && hits[b] > v) {
          hits[b + 1] = hits[b];
          --b;
        }
        hits[b + 1] = v;
      }
    }
    __syncthreads();
    const float step = p.scale / (float)p.bins;
    const float ct = cos_t[row], st = sin_t[row];
    const bool land_row = row >= p.land_row0 && row < p.land_row1;
    uint8_t* out = echo + rr * p.bins;
    for (int b = threadIdx.x; b < p.bins; b += blockDim.x) {
      const uint64_t idx = (((uint64_t)(fa * p.n_gains + gi) * (uint64_t)p.rows + row) *
                            (uint64_t)p.bins) + (uint64_t)b;
      const uint64_t h = splitmix64(p.seed ^ (idx * 0xD1B54A32D192ED03ull));
      uint32_t v = 0;
      if ((uint32_t)(h >> 32) < clutter_thresh[gi * p.bins + b]) v = 11u + (uint32_t)((h >> 16) & 0xffffu) % 29u;
      if (land_row && b >= p.land_bin0 && (uint32_t)(h & 0xffu) < p.land_fill_u8)
        v = 150u + (uint32_t)((h >> 8) & 0xffu) % 106u;
      if (nh) {
        const float r = step * (float)b;
        const float xx = r * ct, yy = r * st;
        for (int q = 0; q < nh; ++q) {
          const int k = hits[q];
          const int32_t* tb = tbins + (fl * p.n_targets + k) * 2;
          if (b < tb[0] || b > tb[1]) continue;
          const float* tg = targets + (fl * p.n_targets + k) * 4;
          const float dx = xx - tg[0], dy = yy - tg[1];
          float d2 = dx * dx;
          d2 = d2 + dy * dy;
          if (d2 <= tg[2]) {
            if ((uint32_t)((h >> 40) & 0xffu) < p.target_fill_u8)
              v = 60u + (uint32_t)((h >> 48) & 0xffu) % 40u;
            break;
          }
        }
      }
      out[b] = (uint8_t)v;
    }
  }
}

}  // namespace

// ---------------------------------------------------------------- C-ABI bodies
// words of the staged kept entries of rpt_polar_count / _write (u8 sweeps of 1024 bins; else 0)
int64_t polar_stage_words(int64_t n_files, int32_t rows) {
  return n_files * (int64_t)((rows + kGroupRows - 1) / kGroupRows) * kStageSlots;
}

int32_t polar_count(const void* echo, int32_t dt, int64_t n_files, int32_t rows, int32_t bins,
                    float thr, int32_t stride, int64_t* row_prefix, int64_t* file_offsets,
                    int64_t* total_host, hipStream_t st, uint32_t* entries) {
  if (!echo || n_files < 0 || rows <= 0 || bins <= 0 || stride < 1 || !row_prefix ||
      !file_offsets) {
    set_error("rpt_polar_count: bad arguments");
    return RPT_EINVAL;
  }
  if (n_files == 0) {
    RPT_HIP(hipMemsetAsync(file_offsets, 0, sizeof(int64_t), st));
    RPT_HIP(hipMemsetAsync(row_prefix, 0, sizeof(int64_t), st));
    if (total_host) *total_host = 0;
    return RPT_OK;
  }
  if (dt == RPT_ECHO_U8)
    return count_impl<uint8_t>((const uint8_t*)echo, n_files, rows, bins, thr, stride,
                               row_prefix, file_offsets, total_host, st,
                               grouped_u8((const uint8_t*)echo, bins) ? entries : nullptr);
  if (dt == RPT_ECHO_F32)
    return count_impl<float>((const float*)echo, n_files, rows, bins, thr, stride, row_prefix,
                             file_offsets, total_host, st);
  set_error("rpt_polar_count: unknown echo dtype %d", dt);
  return RPT_EINVAL;
}

int32_t polar_write(const void* echo, int32_t dt, int64_t n_files, int32_t rows, int32_t bins,
                    const float* scale, const float* cos_t, const float* sin_t,
                    const int32_t* gain, float thr, int32_t stride, const int64_t* row_prefix,
                    const int64_t* file_offsets, int32_t fpf, float* x, float* y, float* v,
                    int32_t* gout, int32_t* pf, hipStream_t st, const uint32_t* entries,
                    uint32_t* bnd, bool* bnd_done) {
  if (bnd_done) *bnd_done = false;
  if (n_files == 0) return RPT_OK;
  if (fpf < 1) {
    set_error("rpt_polar_write: files_per_frame must be >= 1");
    return RPT_EINVAL;
  }
  if (!echo || !scale || !cos_t || !sin_t || !row_prefix || !file_offsets || !x || !y || !v ||
      stride < 1) {
    set_error("rpt_polar_write: bad arguments");
    return RPT_EINVAL;
  }
  RowGeo geo{scale, nullptr, cos_t, sin_t};
  if (dt == RPT_ECHO_U8)
    return write_impl<uint8_t>((const uint8_t*)echo, n_files, rows, bins, thr, stride, geo, gain,
                               row_prefix, file_offsets, fpf, x, y, v, gout, pf, st, INT64_MAX,
                               grouped_u8((const uint8_t*)echo, bins) ? entries : nullptr, bnd,
                               bnd_done);
  if (dt == RPT_ECHO_F32)
    return write_impl<float>((const float*)echo, n_files, rows, bins, thr, stride, geo, gain,
                             row_prefix, file_offsets, fpf, x, y, v, gout, pf, st);
  set_error("rpt_polar_write: unknown echo dtype %d", dt);
  return RPT_EINVAL;
}

// rpt_polar_write into outputs of capacity cap (u8 sweeps of 1024 bins): points at or beyond
// cap are dropped; the caller compares the count with cap and writes again when it overflowed.
int32_t polar_write_cap(const uint8_t* echo, int64_t n_files, int32_t rows, float thr,
                        int32_t stride, const float* scale, const float* cos_t,
                        const float* sin_t, const int32_t* gain, const int64_t* row_prefix,
                        const int64_t* file_offsets, int32_t fpf, float* x, float* y, float* v,
                        int32_t* gout, int32_t* pf, int64_t cap, hipStream_t st,
                        const uint32_t* entries, uint32_t* bnd, bool* bnd_done) {
  if (bnd_done) *bnd_done = false;
  if (!grouped_u8(echo, 1024)) {
    set_error("polar_write_cap: u8 sweeps of 1024 bins with 16-B aligned rows only");
    return RPT_ENOTSUP;
  }
  RowGeo geo{scale, nullptr, cos_t, sin_t};
  return write_impl<uint8_t>(echo, n_files, rows, 1024, thr, stride, geo, gain, row_prefix,
                             file_offsets, fpf, x, y, v, gout, pf, st, cap, entries, bnd,
                             bnd_done);
}

// words of the bnd buffer of polar_write / polar_write_cap: 4 + the blocks' partials
int64_t polar_bounds_words() { return 4 + 4 * (int64_t)(kExpandBlocks + kListBlocks); }

int32_t sweep_to_points(const float* inten, const float* ranges, const float* cos_t,
                        const float* sin_t, int32_t rows, int32_t bins, float thr,
                        int32_t stride, float* x, float* y, float* z, int64_t capacity,
                        int64_t* n_out_host, hipStream_t st) {
  if (!inten || !ranges || !cos_t || !sin_t || rows <= 0 || bins <= 0 || stride < 1 ||
      !n_out_host) {
    set_error("rpt_sweep_to_points: bad arguments");
    return RPT_EINVAL;
  }
  // the count pass uses the pool; keep its outputs in a second reservation-free region
  int64_t* rp = nullptr;
  int64_t* fo = nullptr;
  RPT_HIP(hipMallocAsync((void**)&rp, sizeof(int64_t) * ((int64_t)rows + 1), st));
  RPT_HIP(hipMallocAsync((void**)&fo, sizeof(int64_t) * 2, st));
  int64_t total = 0;
  int32_t s = count_impl<float>(inten, 1, rows, bins, thr, stride, rp, fo, &total, st);
  if (s == RPT_OK) {
    if (total > capacity) {
      set_error("rpt_sweep_to_points: %lld points exceed capacity %lld", (long long)total,
                (long long)capacity);
      s = RPT_EINVAL;
    } else {
      RowGeo geo{nullptr, ranges, cos_t, sin_t};
      s = write_impl<float>(inten, 1, rows, bins, thr, stride, geo, nullptr, rp, fo, 1, x, y, z,
                            nullptr, nullptr, st);
    }
  }
  (void)hipFreeAsync(rp, st);
  (void)hipFreeAsync(fo, st);
  *n_out_host = total;
  return s;
}

int32_t frame_times(const int32_t* pf, int64_t n, const int64_t* ids, float* t, hipStream_t st) {
  if (n == 0) return RPT_OK;
  hipLaunchKernelGGL(k_frame_times, dim3(grid_for(n, 256, 8192)), dim3(256), 0, st, pf, n, ids, t,
                     (const int64_t*)nullptr);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

// n_dev: the count on the device, <= n_max
int32_t frame_times_dev(const int32_t* pf, int64_t n_max, const int64_t* n_dev, float* t,
                        hipStream_t st) {
  if (n_max == 0) return RPT_OK;
  hipLaunchKernelGGL(k_frame_times, dim3(grid_for(n_max, 256, 8192)), dim3(256), 0, st, pf,
                     n_max, (const int64_t*)nullptr, t, n_dev);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

int32_t polar_to_cartesian(const float* cos_t, const float* sin_t, const float* ranges,
                           int64_t rows, int64_t bins, float* x, float* y, hipStream_t st) {
  if (rows * bins == 0) return RPT_OK;
  hipLaunchKernelGGL(k_polar_dense, dim3(grid_for(rows * bins, 256, 8192)), dim3(256), 0, st,
                     cos_t, sin_t, ranges, rows, bins, x, y);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

int32_t infer_time_from_colors(const uint8_t* colors, int64_t n, const float* pal, int32_t n_pal,
                               float* out, hipStream_t st) {
  if (n == 0) return RPT_OK;
  if (n_pal <= 0) {
    set_error("attempt to get argmin of an empty sequence");
    return RPT_EINVAL;
  }
  hipLaunchKernelGGL(k_colors, dim3(grid_for(n, 256, 8192)), dim3(256), 0, st, colors, n, pal,
                     n_pal, out);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

int32_t synth_echo(const rpt_synth_params* p, int64_t frame0, int64_t n_frames,
                   const float* cos_t, const float* sin_t, const uint32_t* clutter_thresh,
                   const float* targets, const int32_t* trows, const int32_t* tbins,
                   uint8_t* echo, hipStream_t st) {
  if (!p || p->n_targets > kMaxTargets || p->rows <= 0 || p->bins <= 0 || p->n_gains <= 0) {
    set_error("rpt_synth_echo: bad parameters (n_targets <= %d)", kMaxTargets);
    return RPT_EINVAL;
  }
  const int64_t blocks = n_frames * p->n_gains * p->rows;
  if (blocks == 0) return RPT_OK;
  hipLaunchKernelGGL(k_synth, dim3((unsigned)std::min<int64_t>(blocks, 65536)), dim3(kBlock), 0,
                     st, *p, frame0, n_frames, cos_t, sin_t, clutter_thresh, targets, trows,
                     tbins, echo);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

}  // namespace rpt
