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
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
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

// ---- u8 fast path (the radar's native sample type).  For integer samples v in [0, 255],
// (float)v > thr  <=>  v > T  with T = floor(thr) clamped to [-1, 255] (NaN -> 255: nothing kept),
// evaluated on 4 bytes at once (SWAR, exact per byte, no carries across bytes):
//   T <= 127 : hi bit of ((x & 0x7f..) + (127 - T) * 0x01..) | x
//   T >= 128 : hi bit of ((x & 0x7f..) + (255 - T) * 0x01..) & x
__device__ __forceinline__ uint32_t gt_mask(uint32_t x, int T) {
  if (T < 0) return 0x80808080u;
  if (T >= 255) return 0u;
  const uint32_t lo = x & 0x7f7f7f7fu;
  if (T <= 127) return ((lo + (uint32_t)(127 - T) * 0x01010101u) | x) & 0x80808080u;
  return ((lo + (uint32_t)(255 - T) * 0x01010101u) & x) & 0x80808080u;
}
// the 4 per-byte hi bits of a mask -> 4-bit nibble (byte k -> bit k)
__device__ __forceinline__ uint32_t nib(uint32_t m) { return ((m >> 7) * 0x10204080u) >> 28; }

// Rows per wave iteration: their loads are issued together (4 KiB in flight per wave) before any
// row is reduced, instead of one dependent 1-KiB load per iteration.
constexpr int kRowsPerIter = 4;

__global__ __launch_bounds__(kBlock) void k_row_count_u8(const uint8_t* __restrict__ echo,
                                                        int64_t n_rows, int bins, int T,
                                                        int32_t* __restrict__ row_count) {
  const int lane = threadIdx.x & 63;
  const int64_t wave0 = (int64_t)blockIdx.x * kWavesPerBlock + threadIdx.x / 64;
  const int64_t n_waves = (int64_t)gridDim.x * kWavesPerBlock;
  const int64_t n_groups = (n_rows + kRowsPerIter - 1) / kRowsPerIter;
  for (int64_t grp = wave0; grp < n_groups; grp += n_waves) {
    const int64_t row0 = grp * kRowsPerIter;
    int c[kRowsPerIter];
#pragma unroll
    for (int k = 0; k < kRowsPerIter; ++k) c[k] = 0;
    for (int b0 = lane * 16; b0 < bins; b0 += 64 * 16) {
      uint4 v[kRowsPerIter];
#pragma unroll
      for (int k = 0; k < kRowsPerIter; ++k)
        v[k] = (row0 + k < n_rows) ? *reinterpret_cast<const uint4*>(echo + (row0 + k) * bins + b0)
                                   : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
      for (int k = 0; k < kRowsPerIter; ++k)
        c[k] += __popc(gt_mask(v[k].x, T)) + __popc(gt_mask(v[k].y, T)) +
                __popc(gt_mask(v[k].z, T)) + __popc(gt_mask(v[k].w, T));
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
#pragma unroll
      for (int k = 0; k < kRowsPerIter; ++k) c[k] += __shfl_xor(c[k], off);
    if (lane < kRowsPerIter) {
      int cv = c[0];
#pragma unroll
      for (int k = 1; k < kRowsPerIter; ++k) cv = (lane == k) ? c[k] : cv;
      if (row0 + lane < n_rows) row_count[row0 + lane] = cv;
    }
  }
}

// Emission of one u8 row of 1024 bins whose first kept element has in-file rank `rank`: the kept
// elements whose rank is a multiple of stride go to out0 + (their in-file emitted index).  Each
// lane ranks its kept elements (m* = per-byte keep masks of its 16 samples, c their count, incl
// the wave-inclusive count), the emitted (bin, sample) pairs are staged in the wave's LDS slice
// in output order and written with full-width stores.  Outputs at or beyond cap are dropped and
// flagged in *overflow (single-pass K1 writes into a capacity guessed from the last run).
__device__ __forceinline__ void emit_row_u8(const uint4 v, uint32_t m0, uint32_t m1, uint32_t m2,
                                            uint32_t m3, int c, int incl, int tot, uint32_t rank,
                                            int64_t out0, int64_t cap, float step,
                                            const float* __restrict__ ranges, float ct, float st,
                                            int32_t g, int32_t fr, uint32_t ustride, bool pow2,
                                            uint32_t sh, uint32_t* __restrict__ stage, int lane,
                                            float* __restrict__ x, float* __restrict__ y,
                                            float* __restrict__ val, int32_t* __restrict__ gain_out,
                                            int32_t* __restrict__ pf_out,
                                            uint32_t* __restrict__ overflow) {
  const uint32_t r = rank + (uint32_t)(incl - c);
  const uint32_t first = pow2 ? ((rank + ustride - 1u) >> sh) : (rank + ustride - 1u) / ustride;
  if (c) {
    uint32_t m = nib(m0) | (nib(m1) << 4) | (nib(m2) << 8) | (nib(m3) << 12);
    const uint32_t q = pow2 ? (r >> sh) : r / ustride;
    const uint32_t rem = r - q * ustride;
    int slot = (int)(q + (rem ? 1u : 0u) - first);
    // drop the kept elements before the first emitted rank, then emit every stride-th
    for (uint32_t t = rem ? ustride - rem : 0u; t > 0u && m; --t) m &= m - 1u;
    while (m) {
      const int k = __builtin_ctz(m);
      const uint32_t w = (k < 4) ? v.x : (k < 8) ? v.y : (k < 12) ? v.z : v.w;
      const uint32_t sample = __builtin_amdgcn_ubfe(w, (uint32_t)(8 * (k & 3)), 8u);
      stage[slot++] = ((uint32_t)(lane * 16 + k) << 8) | sample;
      for (uint32_t t = 0; t < ustride && m; ++t) m &= m - 1u;
    }
  }
  const int n_emit = (int)((pow2 ? ((rank + (uint32_t)tot + ustride - 1u) >> sh)
                                 : (rank + (uint32_t)tot + ustride - 1u) / ustride) -
                           first);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  for (int l = lane; l < n_emit; l += 64) {
    const uint32_t e = stage[l];
    const int b = (int)(e >> 8);
    const int64_t o = out0 + first + l;
    if (o >= cap) {
      if (overflow) atomicOr(overflow, 1u);
      continue;
    }
    const float rr = ranges ? ranges[b] : step * (float)b;
    x[o] = rr * ct;
    y[o] = rr * st;
    val[o] = (float)(e & 0xffu);
    if (gain_out) gain_out[o] = g;
    if (pf_out) pf_out[o] = fr;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Single-pass K1 for u8 sweeps of 1024 bins (rows % 64 == 0): the count and write passes fused
// with a decoupled look-back.  A block takes tiles of 64 rows (16 per wave, held in registers) in
// ticket order (one same-address atomic per 64 KiB: they serialise in L2); it publishes the
// tile's kept count, looks back over the earlier tiles of the same file for its in-file rank
// (status granules {flag:2 | value:62}, agent-scope relaxed atomics: the data is the flag), takes
// the file's output base from a second look-back over the files' emitted counts (fstat, published
// by each file's last group), and emits.  Every wait is on a smaller ticket, so all waits end;
// every spin is still bounded (a timeout sets *overflow and the host falls back to the two
// passes).  file_off[f] receives the exclusive per-file output offsets (file_off[n_files] = N).
constexpr uint64_t kK1Agg = 1ull << 62, kK1Inc = 2ull << 62, kK1Val = (1ull << 62) - 1;

// Exclusive prefix of item `self` over items [first, self) of a status array of granules
// {flag:2 | value:62} (aggregate or inclusive), one wave, 64 predecessors per round: the
// aggregates back to the nearest inclusive.  Bounded spin; a timeout sets *err.
__device__ __forceinline__ int64_t lookback(const uint64_t* __restrict__ status, int64_t self,
                                            int64_t first, int lane, uint32_t* __restrict__ err) {
  int64_t prefix = 0;
  uint32_t spins = 0;
  for (int64_t j = self - 1; j >= first;) {
    const int64_t idx = j - lane;
    const uint64_t st = (idx >= first) ? __hip_atomic_load(status + idx, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT)
                                       : kK1Inc;  // before the range: an inclusive zero
    const uint64_t incm = __ballot((st >> 62) == 2u);
    const uint64_t zero = __ballot((st >> 62) == 0u);
    const int fi = incm ? __ffsll((unsigned long long)incm) - 1 : 64;
    const uint64_t upto = (fi >= 63) ? ~0ull : ((2ull << fi) - 1ull);
    if (zero & upto) {
      if (++spins > (1u << 22)) {
        if (lane == 0) atomicOr(err, 2u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    int64_t part = (lane <= fi && idx >= first) ? (int64_t)(st & kK1Val) : 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off);
    prefix += part;
    if (fi < 64) break;
    j -= 64;
  }
  return prefix;
}
constexpr int kScanRowsPerWave = 16;                               // rows held in registers
constexpr int kScanTileRows = kScanRowsPerWave * kWavesPerBlock;  // 64 rows per ticket
__global__ __launch_bounds__(kBlock) void k_polar_scan_u8(
    const uint8_t* __restrict__ echo, int64_t n_rows, int rows, int T, int stride, RowGeo geo,
    const int32_t* __restrict__ gain, int files_per_frame, float* __restrict__ x,
    float* __restrict__ y, float* __restrict__ val, int32_t* __restrict__ gain_out,
    int32_t* __restrict__ pf_out, int64_t cap, uint64_t* __restrict__ status,
    uint64_t* __restrict__ fstat, int64_t* __restrict__ file_off, uint32_t* __restrict__ ticket,
    uint32_t* __restrict__ overflow) {
  constexpr int CH = 64 * 16;
  __shared__ uint32_t s_stage[kWavesPerBlock][CH];  // (bin << 8) | sample
  __shared__ int64_t s_wtot[kWavesPerBlock];
  __shared__ int64_t s_prefix, s_base;
  __shared__ uint32_t s_tile;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x / 64;
  const float fb = (float)CH;
  const uint32_t ustride = (uint32_t)stride;
  const bool pow2 = (ustride & (ustride - 1u)) == 0u;
  const uint32_t sh = (uint32_t)__builtin_ctz(ustride);
  const int64_t tpf = rows / kScanTileRows;  // tiles per file
  const int64_t n_tiles = n_rows / kScanTileRows;
  while (true) {
    if (threadIdx.x == 0) s_tile = atomicAdd(ticket, 1u);
    __syncthreads();
    const int64_t tile = s_tile;
    if (tile >= n_tiles) break;  // uniform over the block
    const int64_t f = tile / tpf;
    const int64_t ti = tile - f * tpf;
    const int64_t row0 = tile * kScanTileRows + wv * kScanRowsPerWave;
    uint4 vv[kScanRowsPerWave];
#pragma unroll
    for (int k = 0; k < kScanRowsPerWave; ++k)
      vv[k] = *reinterpret_cast<const uint4*>(echo + (row0 + k) * CH + lane * 16);
    int tt[kScanRowsPerWave];
    int wtot = 0;
#pragma unroll
    for (int k = 0; k < kScanRowsPerWave; ++k) {
      const int c = __popc(gt_mask(vv[k].x, T)) + __popc(gt_mask(vv[k].y, T)) +
                    __popc(gt_mask(vv[k].z, T)) + __popc(gt_mask(vv[k].w, T));
      tt[k] = c;
      wtot += c;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) wtot += __shfl_xor(wtot, off);
    if (lane == 0) s_wtot[wv] = wtot;
    __syncthreads();
    if (wv == 0) {
      int64_t total = 0;
#pragma unroll
      for (int w = 0; w < kWavesPerBlock; ++w) total += s_wtot[w];
      // the tile's count, then its in-file prefix from the earlier tiles of the file
      if (lane == 0)
        __hip_atomic_store(status + tile, (ti == 0 ? kK1Inc : kK1Agg) | (uint64_t)total,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int64_t prefix = lookback(status, tile, f * tpf, lane, overflow);
      if (lane == 0 && ti > 0)
        __hip_atomic_store(status + tile, kK1Inc | (uint64_t)(prefix + total), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      // the file's output base: a second look-back, over the files (fstat: the file's emitted
      // count as soon as its last tile knows it, then its inclusive base + count)
      const int64_t fcount = (prefix + total + stride - 1) / stride;
      if (ti == tpf - 1 && lane == 0)
        __hip_atomic_store(fstat + f, (f == 0 ? kK1Inc : kK1Agg) | (uint64_t)fcount,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int64_t base = lookback(fstat, f, 0, lane, overflow);
      if (ti == tpf - 1 && lane == 0) {
        if (f > 0)
          __hip_atomic_store(fstat + f, kK1Inc | (uint64_t)(base + fcount), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        file_off[f + 1] = base + fcount;
        if (f == 0) file_off[0] = 0;
      }
      if (lane == 0) {
        s_prefix = prefix;
        s_base = base;
      }
    }
    __syncthreads();
    // emission, row by row (ranks continue over the block's waves in row order)
    uint32_t rank = (uint32_t)s_prefix;
    for (int w = 0; w < wv; ++w) rank += (uint32_t)s_wtot[w];
    const int64_t base = s_base;
    const int32_t g = gain ? gain[f] : 0;
    const int32_t fr = (int32_t)((uint32_t)f / (uint32_t)files_per_frame);
#pragma unroll
    for (int k = 0; k < kScanRowsPerWave; ++k) {
      const int64_t row = row0 + k;
      const uint32_t m0 = gt_mask(vv[k].x, T), m1 = gt_mask(vv[k].y, T),
                     m2 = gt_mask(vv[k].z, T), m3 = gt_mask(vv[k].w, T);
      const int incl = wave_incl_scan_dpp(tt[k]);
      const int tot = __builtin_amdgcn_readlane(incl, 63);
      const float step = geo.scale[row] / fb;
      emit_row_u8(vv[k], m0, m1, m2, m3, tt[k], incl, tot, rank, base, cap, step, nullptr,
                  geo.cos_t[row], geo.sin_t[row], g, fr, ustride, pow2, sh, s_stage[wv], lane, x,
                  y, val, gain_out, pf_out, overflow);
      rank += (uint32_t)tot;
    }
    __syncthreads();  // s_tile / s_wtot reuse
  }
}

// Same contract as k_row_write (LDS-staged emission), u8 samples, bins == 1024 (one chunk per
// row): kRowsPerIter rows' samples are loaded before the first is ranked.
__global__ __launch_bounds__(kBlock) void k_row_write_u8(
    const uint8_t* __restrict__ echo, int64_t n_rows, int rows, int bins, int T, int stride,
    RowGeo geo, const int32_t* __restrict__ gain, const int64_t* __restrict__ row_prefix,
    const int64_t* __restrict__ file_offsets, int files_per_frame, float* __restrict__ x,
    float* __restrict__ y, float* __restrict__ val, int32_t* __restrict__ gain_out,
    int32_t* __restrict__ pf_out) {
  constexpr int CH = 64 * 16;
  __shared__ uint32_t s_stage[kWavesPerBlock][CH];  // (bin << 8) | sample
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x / 64;
  const int64_t wave0 = (int64_t)blockIdx.x * kWavesPerBlock + wv;
  const int64_t n_waves = (int64_t)gridDim.x * kWavesPerBlock;
  const float fb = (float)bins;
  const uint32_t ustride = (uint32_t)stride;
  const int64_t n_groups = (n_rows + kRowsPerIter - 1) / kRowsPerIter;
  const bool pow2 = (ustride & (ustride - 1u)) == 0u;
  const uint32_t sh = (uint32_t)__builtin_ctz(ustride);
  for (int64_t grp = wave0; grp < n_groups; grp += n_waves) {
    // wave-uniform: lets the per-row metadata below use scalar loads / SALU
    const int64_t row0 = (int64_t)__builtin_amdgcn_readfirstlane((int)grp) * kRowsPerIter;
    uint4 vv[kRowsPerIter];
#pragma unroll
    for (int k = 0; k < kRowsPerIter; ++k)
      vv[k] = (row0 + k < n_rows)
                  ? *reinterpret_cast<const uint4*>(echo + (row0 + k) * CH + lane * 16)
                  : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
    for (int kk = 0; kk < kRowsPerIter; ++kk) {
      const int64_t row = row0 + kk;
      if (row >= n_rows) break;
      const uint4 v = vv[kk];
      const int64_t f = (int64_t)((uint32_t)row / (uint32_t)rows);
      uint32_t rank = (uint32_t)(row_prefix[row] - row_prefix[f * rows]);
      const int64_t out0 = file_offsets[f];
      const float step = geo.scale ? geo.scale[row] / fb : 0.f;
      const float ct = geo.cos_t[row], st = geo.sin_t[row];
      const int32_t g = gain ? gain[f] : 0;
      const int32_t fr = (int32_t)((uint32_t)f / (uint32_t)files_per_frame);
      const uint32_t m0 = gt_mask(v.x, T), m1 = gt_mask(v.y, T), m2 = gt_mask(v.z, T),
                     m3 = gt_mask(v.w, T);
      const int c = __popc(m0) + __popc(m1) + __popc(m2) + __popc(m3);
      const int incl = wave_incl_scan_dpp(c);
      const int tot = __builtin_amdgcn_readlane(incl, 63);
      const float rs = geo.ranges ? 0.f : step;
      emit_row_u8(v, m0, m1, m2, m3, c, incl, tot, rank, out0, INT64_MAX, rs,
                  geo.ranges ? geo.ranges + row * bins : nullptr, ct, st, g, fr, ustride, pow2,
                  sh, s_stage[wv], lane, x, y, val, gain_out, pf_out, nullptr);
    }
  }
}

// integer threshold of u8 samples (see gt_mask)
inline int u8_threshold(float thr) {
  if (!(thr == thr)) return 255;
  const double f = std::floor((double)thr);
  return f < -1.0 ? -1 : (f > 255.0 ? 255 : (int)f);
}

template <class T>
constexpr bool is_u8() { return false; }
template <>
constexpr bool is_u8<uint8_t>() { return true; }

template <class T>
int32_t count_impl(const T* echo, int64_t n_files, int rows, int bins, float thr, int stride,
                   int64_t* row_prefix, int64_t* file_offsets, int64_t* total_host,
                   hipStream_t st) {
  const int64_t n_rows = n_files * rows;
  Scratch& sc = scratch();
  Budget b;
  b.add<int32_t>(n_rows + 1);
  b.add<int64_t>(n_files + 1);
  RPT_TRY(sc.reserve(b.bytes, st));
  int32_t* rc = sc.carve_n<int32_t>(n_rows + 1);
  int64_t* fo = sc.carve_n<int64_t>(n_files + 1);
  const bool vec = (bins % (64 * Vec<T>::N) == 0) && ((uintptr_t)echo % 16 == 0);
  const int grid = grid_for(n_rows, kWavesPerBlock, 16384);
  if (vec && is_u8<T>())
    hipLaunchKernelGGL(k_row_count_u8, dim3(grid), dim3(kBlock), 0, st,
                       reinterpret_cast<const uint8_t*>(echo), n_rows, bins, u8_threshold(thr),
                       rc);
  else if (vec)
    hipLaunchKernelGGL((k_row_count<T, true>), dim3(grid), dim3(kBlock), 0, st, echo, n_rows,
                       bins, thr, rc);
  else
    hipLaunchKernelGGL((k_row_count<T, false>), dim3(grid), dim3(kBlock), 0, st, echo, n_rows,
                       bins, thr, rc);
  RPT_CHECK_LAUNCH();
  RPT_TRY(exclusive_scan_total_i32_to_i64(rc, row_prefix, n_rows, st));
  hipLaunchKernelGGL(k_file_counts, dim3(grid_for(n_files, 256, 1024)), dim3(256), 0, st,
                     row_prefix, n_files, rows, stride, fo);
  RPT_CHECK_LAUNCH();
  RPT_TRY(exclusive_scan_total_i64(fo, file_offsets, n_files, st));
  if (total_host) {
    RPT_HIP(hipMemcpyAsync(total_host, file_offsets + n_files, sizeof(int64_t),
                           hipMemcpyDeviceToHost, st));
    RPT_HIP(hipStreamSynchronize(st));
  }
  return RPT_OK;
}

template <class T>
int32_t write_impl(const T* echo, int64_t n_files, int rows, int bins, float thr, int stride,
                   RowGeo geo, const int32_t* gain, const int64_t* row_prefix,
                   const int64_t* file_offsets, int fpf, float* x, float* y, float* v,
                   int32_t* gout, int32_t* pf, hipStream_t st) {
  const int64_t n_rows = n_files * rows;
  if ((int64_t)rows * bins >= (int64_t(1) << 32) || n_rows >= (int64_t(1) << 32) || stride < 1 ||
      fpf < 1) {
    set_error("rpt_polar_write: rows*bins and n_files*rows must be < 2^32, stride/fpf >= 1");
    return RPT_ENOTSUP;
  }
  const bool vec = (bins % (64 * Vec<T>::N) == 0) && ((uintptr_t)echo % 16 == 0);
  const int grid = grid_for(n_rows, kWavesPerBlock, 16384);
  if (vec && is_u8<T>() && bins == 64 * 16)
    hipLaunchKernelGGL(k_row_write_u8, dim3(grid), dim3(kBlock), 0, st,
                       reinterpret_cast<const uint8_t*>(echo), n_rows, rows, bins,
                       u8_threshold(thr), stride, geo, gain, row_prefix, file_offsets, fpf, x, y,
                       v, gout, pf);
  else if (vec)
    hipLaunchKernelGGL((k_row_write<T, true>), dim3(grid), dim3(kBlock), 0, st, echo, n_rows,
                       rows, bins, thr, stride, geo, gain, row_prefix, file_offsets, fpf, x, y,
                       v, gout, pf);
  else
    hipLaunchKernelGGL((k_row_write<T, false>), dim3(grid), dim3(kBlock), 0, st, echo, n_rows,
                       rows, bins, thr, stride, geo, gain, row_prefix, file_offsets, fpf, x, y,
                       v, gout, pf);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

__global__ void k_frame_times(const int32_t* __restrict__ pf, int64_t n,
                              const int64_t* __restrict__ ids, float* __restrict__ t) {
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
// Single-pass K1 (see k_polar_scan_u8).  Returns RPT_EINVAL when the shape does not qualify;
// *status_host: 0 ok, bit 0 = more than cap points (outputs incomplete), bit 1 = spin timeout.
int32_t polar_scan_u8(const uint8_t* echo, int64_t n_files, int32_t rows, int32_t bins, float thr,
                      int32_t stride, const float* scale, const float* cos_t, const float* sin_t,
                      const int32_t* gain, int32_t fpf, float* x, float* y, float* v,
                      int32_t* gout, int32_t* pf, int64_t cap, int64_t* file_off,
                      uint64_t* work, size_t work_words, hipStream_t st) {
  const int64_t n_rows = n_files * rows;
  if (bins != 64 * 16 || rows % kScanTileRows || n_files < 1 || stride < 1 || fpf < 1 ||
      (uintptr_t)echo % 16 || (int64_t)rows * bins >= (int64_t(1) << 32) ||
      n_rows >= (int64_t(1) << 31)) {
    set_error("polar_scan_u8: shape not supported");
    return RPT_EINVAL;
  }
  const int64_t n_groups = n_rows / kScanTileRows;  // tiles
  const size_t need = (size_t)n_groups + (size_t)n_files + 1 + 2;
  if (!work || work_words < need) {
    set_error("polar_scan_u8: work buffer too small");
    return RPT_EINVAL;
  }
  RPT_HIP(hipMemsetAsync(work, 0, need * sizeof(uint64_t), st));
  uint64_t* status = work;
  uint64_t* fstat = work + n_groups;
  uint32_t* ticket = reinterpret_cast<uint32_t*>(work + n_groups + n_files + 1);
  uint32_t* overflow = ticket + 2;
  RowGeo geo{scale, nullptr, cos_t, sin_t};
  int dev = 0, n_cu = 0;
  RPT_HIP(hipGetDevice(&dev));
  RPT_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  const int grid = (int)std::min<int64_t>((int64_t)std::max(n_cu, 1) * 4, n_groups);
  hipLaunchKernelGGL(k_polar_scan_u8, dim3(grid), dim3(kBlock), 0, st, echo, n_rows, rows,
                     u8_threshold(thr), stride, geo, gain, fpf, x, y, v, gout, pf, cap, status,
                     fstat, file_off, ticket, overflow);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

int32_t polar_count(const void* echo, int32_t dt, int64_t n_files, int32_t rows, int32_t bins,
                    float thr, int32_t stride, int64_t* row_prefix, int64_t* file_offsets,
                    int64_t* total_host, hipStream_t st) {
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
                               row_prefix, file_offsets, total_host, st);
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
                    int32_t* gout, int32_t* pf, hipStream_t st) {
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
                               row_prefix, file_offsets, fpf, x, y, v, gout, pf, st);
  if (dt == RPT_ECHO_F32)
    return write_impl<float>((const float*)echo, n_files, rows, bins, thr, stride, geo, gain,
                             row_prefix, file_offsets, fpf, x, y, v, gout, pf, st);
  set_error("rpt_polar_write: unknown echo dtype %d", dt);
  return RPT_EINVAL;
}

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
  hipLaunchKernelGGL(k_frame_times, dim3(grid_for(n, 256, 8192)), dim3(256), 0, st, pf, n, ids, t);
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
