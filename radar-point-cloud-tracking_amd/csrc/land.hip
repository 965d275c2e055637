// K2/K3: land (persistent background) filter.  Replaces build_occupancy_grid, identify_land_cells
// and filter_land_from_frame (PointCloudWork/4_temporal_object_tracker.py:359-436).
//
// Grid semantics are numpy's: edges are the float64 np.arange(min, max + res, res) the host
// builds from the float32 bounds (rpt_bounds_xy); a point's cell is
// clip(searchsorted(edges, v, 'right') - 1, 0, n_edges - 2) — an exact binary search over the
// edge array staged in LDS, so no floating-point re-derivation of the edges can disagree.
// Counts are int32 atomics (order-free); intensity sums are float64 atomics, exact for the
// integer echo values of the radar path (sums < 2^53), like np.add.at's sequential order.
#include <climits>
#include <cstdlib>
#include <cstring>

#include <algorithm>

#include "common.h"

#pragma clang fp contract(off)

namespace rpt {
namespace {

constexpr int kBlock = 256;
constexpr int kMaxEdges = 4096;  // LDS stage; larger grids fall back to global-memory search

__device__ __forceinline__ uint32_t f2ord(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__global__ __launch_bounds__(kBlock) void k_bounds_xy(const float* __restrict__ x,
                                                     const float* __restrict__ y, int64_t n,
                                                     uint32_t* __restrict__ out) {
  uint32_t mnx = 0xffffffffu, mxx = 0u, mny = 0xffffffffu, mxy = 0u;
  // kBU points per thread per round, loaded together from clamped indices (a repeated valid
  // point leaves minima and maxima unchanged)
  constexpr int kBU = 4;
  for (int64_t b0 = (int64_t)blockIdx.x * blockDim.x * kBU; b0 < n;
       b0 += (int64_t)gridDim.x * blockDim.x * kBU) {
    float xs[kBU], ys[kBU];
#pragma unroll
    for (int u = 0; u < kBU; ++u) {
      const int64_t i = min(b0 + (int64_t)u * blockDim.x + threadIdx.x, n - 1);
      xs[u] = x[i];
      ys[u] = y[i];
    }
#pragma unroll
    for (int u = 0; u < kBU; ++u) {
      const uint32_t a = f2ord(xs[u]), b = f2ord(ys[u]);
      mnx = min(mnx, a);
      mxx = max(mxx, a);
      mny = min(mny, b);
      mxy = max(mxy, b);
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mnx = min(mnx, (uint32_t)__shfl_xor((int)mnx, off));
    mxx = max(mxx, (uint32_t)__shfl_xor((int)mxx, off));
    mny = min(mny, (uint32_t)__shfl_xor((int)mny, off));
    mxy = max(mxy, (uint32_t)__shfl_xor((int)mxy, off));
  }
  __shared__ uint32_t sm[kBlock / 64][4];
  if ((threadIdx.x & 63) == 0) {
    sm[threadIdx.x / 64][0] = mnx;
    sm[threadIdx.x / 64][1] = mxx;
    sm[threadIdx.x / 64][2] = mny;
    sm[threadIdx.x / 64][3] = mxy;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kBlock / 64; ++w) {
      mnx = min(mnx, sm[w][0]);
      mxx = max(mxx, sm[w][1]);
      mny = min(mny, sm[w][2]);
      mxy = max(mxy, sm[w][3]);
    }
    // per-block partial; k_bounds_xy_final reduces them (no same-address atomics)
    out[4 * blockIdx.x + 0] = mnx;
    out[4 * blockIdx.x + 1] = mxx;
    out[4 * blockIdx.x + 2] = mny;
    out[4 * blockIdx.x + 3] = mxy;
  }
}

__global__ __launch_bounds__(kBlock) void k_bounds_xy_final(const uint32_t* __restrict__ part,
                                                           int nb, uint32_t* __restrict__ out) {
  uint32_t v[4] = {0xffffffffu, 0u, 0xffffffffu, 0u};
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    v[0] = min(v[0], part[4 * b + 0]);
    v[1] = max(v[1], part[4 * b + 1]);
    v[2] = min(v[2], part[4 * b + 2]);
    v[3] = max(v[3], part[4 * b + 3]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    v[0] = min(v[0], (uint32_t)__shfl_xor((int)v[0], off));
    v[1] = max(v[1], (uint32_t)__shfl_xor((int)v[1], off));
    v[2] = min(v[2], (uint32_t)__shfl_xor((int)v[2], off));
    v[3] = max(v[3], (uint32_t)__shfl_xor((int)v[3], off));
  }
  __shared__ uint32_t sm[kBlock / 64][4];
  if ((threadIdx.x & 63) == 0)
    for (int k = 0; k < 4; ++k) sm[threadIdx.x / 64][k] = v[k];
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kBlock / 64; ++w) {
      v[0] = min(v[0], sm[w][0]);
      v[1] = max(v[1], sm[w][1]);
      v[2] = min(v[2], sm[w][2]);
      v[3] = max(v[3], sm[w][3]);
    }
    for (int k = 0; k < 4; ++k) out[k] = v[k];
  }
}


// number of edges <= v  (np.searchsorted(edges, v, side='right'))
__device__ __forceinline__ int count_le(const double* e, int ne, double v) {
  int lo = 0, hi = ne;
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if (e[m] <= v)
      lo = m + 1;
    else
      hi = m;
  }
  return lo;
}

__device__ __forceinline__ int clip_idx(int c, int hi) { return c < 0 ? 0 : (c > hi ? hi : c); }

// count_le for the np.arange edges of the land grid (ascending, e[i] ~ e[0] + i*d): start at the
// arithmetic guess and step to the exact count with true edge comparisons, so the result is the
// binary search's for any ascending edges (NaN -> 0, like count_le) in ~2 loads instead of ~7
// dependent ones.
__device__ __forceinline__ int count_le_arith(const double* e, int ne, double v, double inv_d) {
  const double gd = floor((v - e[0]) * inv_d) + 1.0;
  int g = (gd >= 0.0) ? (gd < (double)ne ? (int)gd : ne) : 0;
  if (!(v == v)) return 0;
  while (g < ne && e[g] <= v) ++g;
  while (g > 0 && e[g - 1] > v) --g;
  return g;
}

// Stage both edge arrays in LDS when they fit.
struct Edges {
  const double* xe;
  const double* ye;
  int nxe, nye;
};
__device__ __forceinline__ Edges stage_edges(const double* xe, int nxe, const double* ye, int nye,
                                             double* lds) {
  Edges E{xe, ye, nxe, nye};
  if (nxe + nye <= kMaxEdges) {
    for (int i = threadIdx.x; i < nxe; i += blockDim.x) lds[i] = xe[i];
    for (int i = threadIdx.x; i < nye; i += blockDim.x) lds[nxe + i] = ye[i];
    __syncthreads();
    E.xe = lds;
    E.ye = lds + nxe;
  }
  return E;
}

// LDS-privatised form: int32 counts + f64 sums of the whole grid per block (fits when
// cells * 12 B + edges <= ~150 KiB), flushed with one atomic per non-empty cell.  One 1024-thread
// block per CU: the per-block cost (zeroing and flushing ~10k cells) is paid 256 times, not once
// per 256-thread block of a larger grid, and 16 waves per CU hide the LDS atomics' latency.
constexpr int kLdsGridCells = 10240;
constexpr int kGridBlock = 1024;
__global__ __launch_bounds__(kGridBlock) void k_land_grid_lds(const float* __restrict__ x,
                                                         const float* __restrict__ y,
                                                         const float* __restrict__ val, int64_t n,
                                                         const double* __restrict__ xe, int nxe,
                                                         const double* __restrict__ ye, int nye,
                                                         int32_t* __restrict__ cnt,
                                                         double* __restrict__ tot,
                                                         int32_t* __restrict__ cell_out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* lds_e = reinterpret_cast<double*>(smem);                    // nxe + nye edges
  const int ne = nxe + nye;
  const int ne_al = (ne + 1) & ~1;
  double* lds_t = lds_e + ne_al;                                       // cells f64 sums
  const int ny = nye - 1;
  const int cells = (nxe - 1) * ny;
  int32_t* lds_c = reinterpret_cast<int32_t*>(lds_t + cells);          // cells counts
  for (int i = threadIdx.x; i < nxe; i += blockDim.x) lds_e[i] = xe[i];
  for (int i = threadIdx.x; i < nye; i += blockDim.x) lds_e[nxe + i] = ye[i];
  for (int c = threadIdx.x; c < cells; c += blockDim.x) {
    lds_t[c] = 0.0;
    lds_c[c] = 0;
  }
  __syncthreads();
  const double* ex = lds_e;
  const double* ey = lds_e + nxe;
  const double idx_ = 1.0 / (ex[1] - ex[0]), idy_ = 1.0 / (ey[1] - ey[0]);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int ix = clip_idx(count_le_arith(ex, nxe, (double)x[i], idx_) - 1, nxe - 2);
    const int iy = clip_idx(count_le_arith(ey, nye, (double)y[i], idy_) - 1, nye - 2);
    const int c = ix * ny + iy;
    if (cell_out) cell_out[i] = c;
    atomicAdd(lds_c + c, 1);
    atomicAdd(lds_t + c, (double)val[i]);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < cells; c += blockDim.x) {
    const int k = lds_c[c];
    if (k) {
      atomicAdd(cnt + c, k);
      atomicAdd(tot + c, lds_t[c]);
    }
  }
}

// Same, for intensities that are integers in [0, 255] (u8 echo samples): one packed u64 LDS
// atomic per point, count << 40 | sum (a block's per-cell count < 2^24 and sum < 2^40, checked by
// the caller), instead of an int32 and a float64 atomic.  Integer sums below 2^53 are exact in any
// order, so the float64 grid equals the unpacked kernel's.
constexpr int kPackShift = 40;
__global__ __launch_bounds__(kGridBlock) void k_land_grid_lds_u8(
    const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ val,
    int64_t n, const double* __restrict__ xe, int nxe, const double* __restrict__ ye, int nye,
    int32_t* __restrict__ cnt, double* __restrict__ tot, int32_t* __restrict__ cell_out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  double* lds_e = reinterpret_cast<double*>(smem);  // nxe + nye edges
  const int ne = nxe + nye;
  const int ne_al = (ne + 1) & ~1;
  unsigned long long* lds_p = reinterpret_cast<unsigned long long*>(lds_e + ne_al);
  const int ny = nye - 1;
  const int cells = (nxe - 1) * ny;
  for (int i = threadIdx.x; i < nxe; i += blockDim.x) lds_e[i] = xe[i];
  for (int i = threadIdx.x; i < nye; i += blockDim.x) lds_e[nxe + i] = ye[i];
  for (int c = threadIdx.x; c < cells; c += blockDim.x) lds_p[c] = 0ull;
  __syncthreads();
  const double* ex = lds_e;
  const double* ey = lds_e + nxe;
  const double idx_ = 1.0 / (ex[1] - ex[0]), idy_ = 1.0 / (ey[1] - ey[0]);
  // one 1024-thread block per CU: kU points per thread per round, loads issued together (16
  // waves alone keep too few bytes in flight)
  constexpr int kU = 8;
  const int64_t chunk = (int64_t)kGridBlock * kU;
  for (int64_t b0 = (int64_t)blockIdx.x * chunk; b0 < n; b0 += (int64_t)gridDim.x * chunk) {
    float px[kU], py[kU], pv[kU];
#pragma unroll
    for (int k = 0; k < kU; ++k) {
      const int64_t i = min(b0 + (int64_t)k * kGridBlock + threadIdx.x, n - 1);  // branch-free
      px[k] = x[i];
      py[k] = y[i];
      pv[k] = val[i];
    }
#pragma unroll
    for (int k = 0; k < kU; ++k) {
      const int64_t i = b0 + (int64_t)k * kGridBlock + threadIdx.x;
      if (i >= n) break;
      const int ix = clip_idx(count_le_arith(ex, nxe, (double)px[k], idx_) - 1, nxe - 2);
      const int iy = clip_idx(count_le_arith(ey, nye, (double)py[k], idy_) - 1, nye - 2);
      const int c = ix * ny + iy;
      if (cell_out) cell_out[i] = c;
      atomicAdd(lds_p + c, (1ull << kPackShift) | (unsigned long long)(uint32_t)pv[k]);
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < cells; c += blockDim.x) {
    const unsigned long long v = lds_p[c];
    if (v) {
      atomicAdd(cnt + c, (int32_t)(v >> kPackShift));
      atomicAdd(tot + c, (double)(v & ((1ull << kPackShift) - 1ull)));
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_land_grid(const float* __restrict__ x,
                                                     const float* __restrict__ y,
                                                     const float* __restrict__ val, int64_t n,
                                                     const double* __restrict__ xe, int nxe,
                                                     const double* __restrict__ ye, int nye,
                                                     int32_t* __restrict__ cnt,
                                                     double* __restrict__ tot,
                                                     int32_t* __restrict__ cell_out) {
  __shared__ double lds[kMaxEdges];
  const Edges E = stage_edges(xe, nxe, ye, nye, lds);
  const int ny = nye - 1;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int ix = clip_idx(count_le(E.xe, nxe, (double)x[i]) - 1, nxe - 2);
    const int iy = clip_idx(count_le(E.ye, nye, (double)y[i]) - 1, nye - 2);
    const int64_t c = (int64_t)ix * ny + iy;
    if (cell_out) cell_out[i] = (int32_t)c;
    atomicAdd(cnt + c, 1);
    atomicAdd(tot + c, (double)val[i]);
  }
}

// identify_land_cells :400-408, all float64
__global__ void k_land_mask(const int32_t* __restrict__ cnt, const double* __restrict__ tot,
                            int64_t cells, double nf, double pthr, double ithr,
                            uint8_t* __restrict__ land, int32_t* __restrict__ n_land) {
  int local = 0;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < cells;
       c += (int64_t)gridDim.x * blockDim.x) {
    const int32_t k = cnt[c];
    const double pers = (double)k / nf;
    const double avg = (k > 0) ? tot[c] / (double)k : 0.0;
    const bool is_land = (pers >= pthr) && (avg >= ithr);
    land[c] = is_land ? 1 : 0;
    local += is_land ? 1 : 0;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) local += __shfl_xor(local, off);
  if ((threadIdx.x & 63) == 0 && local) atomicAdd(n_land, local);
}

__global__ __launch_bounds__(kBlock) void k_land_keep(const float* __restrict__ x,
                                                     const float* __restrict__ y, int64_t n,
                                                     const double* __restrict__ xe, int nxe,
                                                     const double* __restrict__ ye, int nye,
                                                     const uint8_t* __restrict__ land,
                                                     int32_t* __restrict__ keep) {
  __shared__ double lds[kMaxEdges];
  const Edges E = stage_edges(xe, nxe, ye, nye, lds);
  const int ny = nye - 1;
  const double idx_ = 1.0 / (E.xe[1] - E.xe[0]), idy_ = 1.0 / (E.ye[1] - E.ye[0]);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int ix = clip_idx(count_le_arith(E.xe, nxe, (double)x[i], idx_) - 1, nxe - 2);
    const int iy = clip_idx(count_le_arith(E.ye, nye, (double)y[i], idy_) - 1, nye - 2);
    keep[i] = land[(int64_t)ix * ny + iy] ? 0 : 1;
  }
}

// keep flags from the cells the grid pass stored (no edge search)
__global__ __launch_bounds__(kBlock) void k_land_keep_cells(const int32_t* __restrict__ cell,
                                                           int64_t n,
                                                           const uint8_t* __restrict__ land,
                                                           int32_t* __restrict__ keep) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    keep[i] = land[cell[i]] ? 0 : 1;
}

__global__ __launch_bounds__(kBlock) void k_land_scatter(
    const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ v,
    const int32_t* __restrict__ g, const int32_t* __restrict__ pf, int64_t n,
    const int32_t* __restrict__ keep, const int32_t* __restrict__ pos, float* __restrict__ xo,
    float* __restrict__ yo, float* __restrict__ vo, int32_t* __restrict__ go,
    int32_t* __restrict__ pfo) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (!keep[i]) continue;
    const int64_t o = pos[i];
    xo[o] = x[i];
    yo[o] = y[i];
    vo[o] = v[i];
    if (go) go[o] = g[i];
    if (pfo) pfo[o] = pf[i];
  }
}

__global__ void k_new_offsets(const int32_t* __restrict__ pos, const int64_t* __restrict__ off,
                              int n_frames, int64_t* __restrict__ out) {
  for (int f = blockIdx.x * blockDim.x + threadIdx.x; f <= n_frames; f += gridDim.x * blockDim.x)
    out[f] = pos[off[f]];
}


// ---- fused compaction of the stack driver (filter_land_from_frame, :426-436, over the stack) --
// Tiles of kCompTile points; item k of thread t is point tile*kCompTile + k*kCompBlock + t, so
// loads and (kept-order) stores are coalesced.  Pass 1 counts each tile's kept points (cell not
// land) from the cells the grid pass stored; after a scan of the tile counts, pass 2 recomputes
// the flags, ranks them (ballots + a 64-entry scan of the per-(item, wave) counts) and writes the
// kept points in order with their times (float32 frame slots, :460-467) and a per-tile partial of
// the ST-DBSCAN bounds -- the keep / position arrays, their full-length scan, the frame-time
// pass and the bounds pass of the separate kernels are gone.
constexpr int kCompBlock = 256, kCompItems = 16, kCompTile = kCompBlock * kCompItems;

struct BoundsPart {
  uint32_t mnx, mxx, mny, mxy;
  int32_t mnf, mxf, flags, pad;  // flags: 1 non-finite x/y, 2 frame slots descend
};

__device__ __forceinline__ bool kept_at(const int32_t* __restrict__ cell,
                                        const uint8_t* __restrict__ land, int64_t i, int64_t n) {
  return i < n && !land[cell[i]];
}

__global__ __launch_bounds__(kCompBlock) void k_land_tile_counts(const int32_t* __restrict__ cell,
                                                                int64_t n,
                                                                const uint8_t* __restrict__ land,
                                                                int32_t* __restrict__ tile_cnt) {
  const int64_t i0 = (int64_t)blockIdx.x * kCompTile + threadIdx.x;
  int32_t cl[kCompItems];
#pragma unroll
  for (int k = 0; k < kCompItems; ++k) {
    const int64_t i = i0 + (int64_t)k * kCompBlock;
    cl[k] = (i < n) ? cell[i] : -1;
  }
  uint32_t lnd[kCompItems];  // branch-free: the flags' loads in flight together (>= 1 cell)
#pragma unroll
  for (int k = 0; k < kCompItems; ++k) lnd[k] = land[cl[k] >= 0 ? cl[k] : 0];
  int c = 0;
#pragma unroll
  for (int k = 0; k < kCompItems; ++k) c += (cl[k] >= 0 && !lnd[k]) ? 1 : 0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
  __shared__ int ws[kCompBlock / 64];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x / 64] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
#pragma unroll
    for (int w = 0; w < kCompBlock / 64; ++w) t += ws[w];
    tile_cnt[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(kCompBlock) void k_land_compact(
    const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ v,
    const int32_t* __restrict__ g, const int32_t* __restrict__ pf, int64_t n,
    const int32_t* __restrict__ cell, const uint8_t* __restrict__ land,
    const int32_t* __restrict__ tile_base, float* __restrict__ xo, float* __restrict__ yo,
    float* __restrict__ vo, int32_t* __restrict__ go, int32_t* __restrict__ pfo,
    float* __restrict__ to, BoundsPart* __restrict__ part, int64_t t_base) {
  constexpr int NW = kCompBlock / 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x / 64;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int64_t i0 = (int64_t)blockIdx.x * kCompTile + threadIdx.x;
  int32_t cl[kCompItems];
#pragma unroll
  for (int k = 0; k < kCompItems; ++k) {
    const int64_t i = i0 + (int64_t)k * kCompBlock;
    cl[k] = (i < n) ? cell[i] : -1;
  }
  // every load below is branch-free (clamped index, result masked) so a thread's loads of a batch
  // are in flight together: conditional loads each ended in a full vmcnt wait
  uint32_t lnd[kCompItems];
#pragma unroll
  for (int k = 0; k < kCompItems; ++k) lnd[k] = land[cl[k] >= 0 ? cl[k] : 0];  // >= 1 cell
  uint32_t km = 0;
#pragma unroll
  for (int k = 0; k < kCompItems; ++k) km |= (cl[k] >= 0 && !lnd[k]) ? (1u << k) : 0u;
  __shared__ int cw[kCompItems * NW];  // per (item k, wave) counts, then their exclusive scan
#pragma unroll
  for (int k = 0; k < kCompItems; ++k) {
    const uint64_t bk = __ballot((km >> k) & 1u);
    if (lane == 0) cw[k * NW + w] = __popcll(bk);
  }
  __syncthreads();
  static_assert(kCompItems * NW == 64, "one wave scans the per-(item, wave) counts");
  if (w == 0) {
    const int c = cw[lane];
    int incl = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int o = __shfl_up(incl, off, 64);
      if (lane >= off) incl += o;
    }
    cw[lane] = incl - c;
  }
  __syncthreads();
  const int64_t tb = tile_base[blockIdx.x];
  uint32_t mnx = 0xffffffffu, mxx = 0u, mny = 0xffffffffu, mxy = 0u;
  int mnf = INT_MAX, mxf = INT_MIN, flags = 0;
  constexpr int kB = 4;  // items per batch of loads
#pragma unroll
  for (int k0 = 0; k0 < kCompItems; k0 += kB) {
    int fb[kB], fp[kB], gb[kB];
    float xb[kB], yb[kB], vb[kB];
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      const int64_t i = min(i0 + (int64_t)(k0 + u) * kCompBlock, n - 1);
      fb[u] = pf[i];
      fp[u] = pf[i > 0 ? i - 1 : 0];
      xb[u] = x[i];
      yb[u] = y[i];
      vb[u] = v[i];
      gb[u] = go ? g[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < kB; ++u) {
    const int k = k0 + u;
    const int64_t i = i0 + (int64_t)k * kCompBlock;
    const bool kp = (km >> k) & 1u;
    const uint64_t bk = __ballot(kp);
    if (i < n) {
      const int f = fb[u];
      // input order; the kept points descend only if the input does
      if (i > 0 && f < fp[u]) flags |= 2;
      if (kp) {
        const int64_t o = tb + cw[k * NW + w] + __popcll(bk & lt);
        const float px = xb[u], py = yb[u];
        xo[o] = px;
        yo[o] = py;
        vo[o] = vb[u];
        if (go) go[o] = gb[u];
        pfo[o] = f;
        to[o] = (float)(t_base + (int64_t)f);  // (t_base: the shard driver's first frame)
        if (!isfinite(px) || !isfinite(py)) flags |= 1;
        const uint32_t a = f2ord(px), b = f2ord(py);
        mnx = min(mnx, a);
        mxx = max(mxx, a);
        mny = min(mny, b);
        mxy = max(mxy, b);
        mnf = min(mnf, f);
        mxf = max(mxf, f);
      }
    }
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mnx = min(mnx, (uint32_t)__shfl_xor((int)mnx, off));
    mxx = max(mxx, (uint32_t)__shfl_xor((int)mxx, off));
    mny = min(mny, (uint32_t)__shfl_xor((int)mny, off));
    mxy = max(mxy, (uint32_t)__shfl_xor((int)mxy, off));
    mnf = min(mnf, __shfl_xor(mnf, off));
    mxf = max(mxf, __shfl_xor(mxf, off));
    flags |= __shfl_xor(flags, off);
  }
  __shared__ BoundsPart wp[NW];
  if (lane == 0) wp[w] = BoundsPart{mnx, mxx, mny, mxy, mnf, mxf, flags, 0};
  __syncthreads();
  if (threadIdx.x == 0) {
    BoundsPart r = wp[0];
    for (int q = 1; q < NW; ++q) {
      r.mnx = min(r.mnx, wp[q].mnx);
      r.mxx = max(r.mxx, wp[q].mxx);
      r.mny = min(r.mny, wp[q].mny);
      r.mxy = max(r.mxy, wp[q].mxy);
      r.mnf = min(r.mnf, wp[q].mnf);
      r.mxf = max(r.mxf, wp[q].mxf);
      r.flags |= wp[q].flags;
    }
    part[blockIdx.x] = r;
  }
}

// new_off[f] = first kept point of frame slot >= f (the kept frame slots ascend), new_off[F] =
// kept count: one binary search per frame slot
// new_off[f] = first kept point of frame >= f: ONE WAVE per frame, a 64-ary search (64 probes
// per round: ~5 dependent rounds over 45 M points instead of a thread's 26-step binary search)
__global__ void k_land_new_off(const int32_t* __restrict__ n_kept_dev,
                               const int32_t* __restrict__ pfo, int n_frames,
                               int64_t* __restrict__ new_off) {
  const int lane = threadIdx.x & 63;
  const int f = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  if (f > n_frames) return;  // (wave-uniform)
  const int64_t nk = *n_kept_dev;
  int64_t lo = 0, hi = nk;  // the answer lies in [lo, hi]
  while (lo < hi) {
    const int64_t step = (hi - lo + 63) / 64;
    const int64_t idx = lo + (int64_t)lane * step;
    const bool below = idx < hi && pfo[idx < hi ? idx : lo] < f;  // a prefix of the lanes
    const int c = __popcll(__ballot(below));
    if (c == 0) {
      hi = lo;
    } else {
      const int64_t nlo = lo + (int64_t)(c - 1) * step + 1;
      hi = min(hi, lo + (int64_t)c * step);
      lo = nlo;
    }
  }
  if (lane == 0) new_off[f] = (f == n_frames) ? nk : lo;
}

// the tiles' partials -> Bounds (what k_bounds<2> gives for the kept points with t = frame
// slot: z = 0, every t finite and integral below 2^24)
// (one 1024-thread block, four partials per thread per round with their loads issued together:
// the 12 k tile partials of a 1000-frame stack were 49 dependent rounds for 256 threads)
constexpr int kFinBlock = 1024;
__global__ __launch_bounds__(kFinBlock) void k_land_compact_final(
    const BoundsPart* __restrict__ part, int nt, const int32_t* __restrict__ n_kept_dev,
    Bounds* __restrict__ out, int64_t t_base) {
  const int64_t nk = *n_kept_dev;
  uint32_t mnx = 0xffffffffu, mxx = 0u, mny = 0xffffffffu, mxy = 0u;
  int mnf = INT_MAX, mxf = INT_MIN, flags = 0;
  for (int b0 = threadIdx.x; b0 < nt; b0 += 4 * blockDim.x) {
    BoundsPart q[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) q[u] = part[min(b0 + u * (int)blockDim.x, nt - 1)];  // repeats
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const BoundsPart& p = q[u];
      mnx = min(mnx, p.mnx);
      mxx = max(mxx, p.mxx);
      mny = min(mny, p.mny);
      mxy = max(mxy, p.mxy);
      mnf = min(mnf, p.mnf);
      mxf = max(mxf, p.mxf);
      flags |= p.flags;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mnx = min(mnx, (uint32_t)__shfl_xor((int)mnx, off));
    mxx = max(mxx, (uint32_t)__shfl_xor((int)mxx, off));
    mny = min(mny, (uint32_t)__shfl_xor((int)mny, off));
    mxy = max(mxy, (uint32_t)__shfl_xor((int)mxy, off));
    mnf = min(mnf, __shfl_xor(mnf, off));
    mxf = max(mxf, __shfl_xor(mxf, off));
    flags |= __shfl_xor(flags, off);
  }
  __shared__ BoundsPart wp[kFinBlock / 64];
  if ((threadIdx.x & 63) == 0) wp[threadIdx.x / 64] = BoundsPart{mnx, mxx, mny, mxy, mnf, mxf, flags, 0};
  __syncthreads();
  if (threadIdx.x == 0) {
    BoundsPart r = wp[0];
    for (int q = 1; q < kFinBlock / 64; ++q) {
      r.mnx = min(r.mnx, wp[q].mnx);
      r.mxx = max(r.mxx, wp[q].mxx);
      r.mny = min(r.mny, wp[q].mny);
      r.mxy = max(r.mxy, wp[q].mxy);
      r.mnf = min(r.mnf, wp[q].mnf);
      r.mxf = max(r.mxf, wp[q].mxf);
      r.flags |= wp[q].flags;
    }
    Bounds b;
    const uint32_t z = f2ord(0.f);
    const bool any = nk > 0;
    b.mn[0] = r.mnx;
    b.mx[0] = r.mxx;
    b.mn[1] = r.mny;
    b.mx[1] = r.mxy;
    b.mn[2] = any ? z : 0xffffffffu;
    b.mx[2] = any ? z : 0u;
    const int64_t t0 = t_base + r.mnf, t1 = t_base + r.mxf;
    b.mn[3] = any ? f2ord((float)t0) : 0xffffffffu;
    b.mx[3] = any ? f2ord((float)t1) : 0u;
    b.nonfinite_xyz = (r.flags & 1) ? 1 : 0;
    b.nonintegral_t = (any && (t1 >= 16777216 || t0 <= -16777216)) ? 1 : 0;
    b.n_finite_t = (int32_t)nk;
    b.t_descends = (r.flags & 2) ? 1 : 0;
    *out = b;
  }
}

}  // namespace

int32_t bounds_xy(const float* x, const float* y, int64_t n, float* out4, hipStream_t st) {
  if (n <= 0) {
    set_error("zero-size array to reduction operation minimum which has no identity");
    return RPT_EEMPTY;
  }
  const int nb = grid_for(n, kBlock, 1024);
  Scratch& sc = scratch(st);
  Budget bud;
  bud.add<uint32_t>(4);
  bud.add<uint32_t>(4 * (int64_t)nb);
  RPT_TRY(sc.reserve(bud.bytes, st));
  uint32_t* d = sc.carve_n<uint32_t>(4);
  uint32_t* part = sc.carve_n<uint32_t>(4 * (int64_t)nb);
  hipLaunchKernelGGL(k_bounds_xy, dim3(nb), dim3(kBlock), 0, st, x, y, n, part);
  hipLaunchKernelGGL(k_bounds_xy_final, dim3(1), dim3(kBlock), 0, st, part, nb, d);
  RPT_CHECK_LAUNCH();
  uint32_t h[4];
  RPT_HIP(hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, st));
  RPT_TRY(wait_stream(st));
  for (int k = 0; k < 4; ++k) {
    const uint32_t u = h[k];
    const uint32_t v = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
    std::memcpy(out4 + k, &v, 4);
  }
  return RPT_OK;
}

// RPT_LAND_U8=0: the int32 + float64 atomics kernel also for u8 points (A/B)
static bool land_u8_enabled() {
  static const bool on = [] {
    const char* e = ab_env("RPT_LAND_U8");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}

// the grid's counts and sums (and a caller's 64-bit counter) zeroed in ONE launch: two fills
// and a third for the counter each cost a launch right after the host-synchronous bounds
// readback, when the GPU idles on the host issuing them
__global__ void k_zero_land(int32_t* __restrict__ cnt, double* __restrict__ tot, int64_t cells,
                            int64_t* __restrict__ extra) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cells;
       i += (int64_t)gridDim.x * blockDim.x) {
    cnt[i] = 0;
    tot[i] = 0.0;
  }
  if (extra && blockIdx.x == 0 && threadIdx.x == 0) *extra = 0;
}

// cell_out (nullable, [n], int32 cells < 2^31): each point's grid cell, for land_filter_cells
// u8_vals: every val is an integer in [0, 255] (points of a u8 echo; packed-atomic kernel)
// zero_also (nullable): a 64-bit device counter zeroed with the grid
int32_t land_grid_cells(const float* x, const float* y, const float* val, int64_t n,
                        const double* xe, int32_t nxe, const double* ye, int32_t nye,
                        int32_t* cnt, double* tot, int32_t* cell_out, hipStream_t st,
                        int32_t u8_vals, int64_t* zero_also) {
  if (nxe < 2 || nye < 2) {
    set_error("rpt_land_grid: need at least two edges per axis");
    return RPT_EINVAL;
  }
  const int64_t cells = (int64_t)(nxe - 1) * (nye - 1);
  if (cell_out && cells >= (int64_t(1) << 31)) cell_out = nullptr;
  hipLaunchKernelGGL(k_zero_land, dim3(grid_for(cells, 256, 1024)), dim3(256), 0, st, cnt, tot,
                     cells, zero_also);
  RPT_CHECK_LAUNCH();
  if (n == 0) return RPT_OK;
  const int64_t ne_al = ((int64_t)nxe + nye + 1) & ~int64_t(1);
  const size_t lds = (size_t)ne_al * 8 + (size_t)cells * 12;
  const size_t lds_u8 = (size_t)ne_al * 8 + (size_t)cells * 8;
  int dev = 0, n_cu = 0;
  RPT_HIP(hipGetDevice(&dev));
  RPT_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  const int gb = grid_for(n, kGridBlock, std::max(n_cu, 1));
  if (u8_vals && lds_u8 <= 150 * 1024 && (n + gb - 1) / gb < (int64_t(1) << 24) &&
      land_u8_enabled()) {
    RPT_HIP(hipFuncSetAttribute((const void*)k_land_grid_lds_u8,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_u8));
    hipLaunchKernelGGL(k_land_grid_lds_u8, dim3(gb), dim3(kGridBlock), lds_u8, st, x, y, val, n,
                       xe, nxe, ye, nye, cnt, tot, cell_out);
  } else if (cells <= kLdsGridCells && lds <= 150 * 1024) {
    RPT_HIP(hipFuncSetAttribute((const void*)k_land_grid_lds,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    hipLaunchKernelGGL(k_land_grid_lds, dim3(gb),
                       dim3(kGridBlock), lds, st, x, y, val, n, xe, nxe, ye, nye, cnt, tot,
                       cell_out);
  } else {
    hipLaunchKernelGGL(k_land_grid, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, st, x, y,
                       val, n, xe, nxe, ye, nye, cnt, tot, cell_out);
  }
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

int32_t land_grid(const float* x, const float* y, const float* val, int64_t n, const double* xe,
                  int32_t nxe, const double* ye, int32_t nye, int32_t* cnt, double* tot,
                  hipStream_t st) {
  return land_grid_cells(x, y, val, n, xe, nxe, ye, nye, cnt, tot, nullptr, st, 0, nullptr);
}

// n_land_dev: int32 land-cell counter on the device, zeroed by the caller (no readback)
int32_t land_mask_dev(const int32_t* cnt, const double* tot, int64_t cells, int64_t num_frames,
                      double pthr, double ithr, uint8_t* land, int32_t* n_land_dev,
                      hipStream_t st) {
  const double nf = (double)(num_frames > 1 ? num_frames : 1);
  if (cells > 0) {
    hipLaunchKernelGGL(k_land_mask, dim3(grid_for(cells, 256, 1024)), dim3(256), 0, st, cnt, tot,
                       cells, nf, pthr, ithr, land, n_land_dev);
    RPT_CHECK_LAUNCH();
  }
  return RPT_OK;
}

int32_t land_mask(const int32_t* cnt, const double* tot, int64_t cells, int64_t num_frames,
                  double pthr, double ithr, uint8_t* land, int64_t* n_land_host,
                  hipStream_t st) {
  int32_t* d = nullptr;
  RPT_TRY(zero_n(st, 1, &d));
  const double nf = (double)(num_frames > 1 ? num_frames : 1);
  if (cells > 0) {
    hipLaunchKernelGGL(k_land_mask, dim3(grid_for(cells, 256, 1024)), dim3(256), 0, st, cnt, tot,
                       cells, nf, pthr, ithr, land, d);
    RPT_CHECK_LAUNCH();
  }
  if (n_land_host) {
    int32_t h = 0;
    RPT_HIP(hipMemcpyAsync(&h, d, sizeof h, hipMemcpyDeviceToHost, st));
    RPT_TRY(wait_stream(st));
    *n_land_host = h;
  }
  return RPT_OK;
}

// cell (nullable): the per-point cells from land_grid_cells over the same points and edges
int32_t land_filter_cells(const float* x, const float* y, const float* v, const int32_t* g,
                          const int32_t* pf, int64_t n, const int64_t* frame_off,
                          int32_t n_frames, const double* xe, int32_t nxe, const double* ye,
                          int32_t nye, const uint8_t* land, const int32_t* cell, float* xo,
                          float* yo, float* vo, int32_t* go, int32_t* pfo, int64_t* new_off,
                          int64_t* n_kept_host, hipStream_t st) {
  Scratch& sc = scratch(st);
  if (n >= (int64_t(1) << 31) - 1) {
    set_error("rpt_land_filter: n exceeds the int32 index space");
    return RPT_ENOTSUP;
  }
  Budget b;
  b.add<int32_t>(n + 1);
  b.add<int32_t>(n + 1);
  RPT_TRY(sc.reserve(b.bytes, st));
  int32_t* keep = sc.carve_n<int32_t>(n + 1);
  int32_t* pos = sc.carve_n<int32_t>(n + 1);  // int32 kept positions (n < 2^31)
  if (n > 0 && cell) {
    hipLaunchKernelGGL(k_land_keep_cells, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, st,
                       cell, n, land, keep);
    RPT_CHECK_LAUNCH();
  } else if (n > 0) {
    hipLaunchKernelGGL(k_land_keep, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, st, x, y,
                       n, xe, nxe, ye, nye, land, keep);
    RPT_CHECK_LAUNCH();
  }
  RPT_TRY(exclusive_scan_total_i32(keep, pos, n, st));
  if (n > 0) {
    hipLaunchKernelGGL(k_land_scatter, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, st, x,
                       y, v, g, pf, n, keep, pos, xo, yo, vo, go, pfo);
    RPT_CHECK_LAUNCH();
  }
  if (new_off && frame_off) {
    hipLaunchKernelGGL(k_new_offsets, dim3(grid_for(n_frames + 1, 256, 64)), dim3(256), 0, st,
                       pos, frame_off, n_frames, new_off);
    RPT_CHECK_LAUNCH();
  }
  if (n_kept_host) {
    int32_t k = 0;
    RPT_HIP(hipMemcpyAsync(&k, pos + n, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    RPT_TRY(wait_stream(st));
    *n_kept_host = k;
  }
  return RPT_OK;
}

// The stack driver's land compaction (see k_land_compact): kept points of [0, n) -- cells from
// land_grid_cells, land flags from land_mask_dev -- into xo / yo / vo / go (nullable) / pfo and
// their times to (float32 frame slot), new_off[n_frames + 1] (device: first kept point per
// frame slot, kept count last) and the kept points' ST-DBSCAN bounds (*bounds_out, device).
// pf must be non-decreasing (the stack's frame-major order).  No synchronisation.
int32_t land_compact_dev(const float* x, const float* y, const float* v, const int32_t* g,
                         const int32_t* pf, int64_t n, const int32_t* cell, const uint8_t* land,
                         int32_t n_frames, float* xo, float* yo, float* vo, int32_t* go,
                         int32_t* pfo, float* to, int64_t* new_off, Bounds* bounds_out,
                         hipStream_t st, int64_t t_base) {
  if (n < 0 || n >= (int64_t(1) << 31) - 1 || n_frames < 0) {
    set_error("land_compact_dev: bad sizes");
    return RPT_EINVAL;
  }
  const int64_t nt = std::max<int64_t>((n + kCompTile - 1) / kCompTile, 1);
  Scratch& sc = scratch(st);
  Budget bud;
  bud.add<int32_t>(nt + 1);
  bud.add<int32_t>(nt + 1);
  bud.add<BoundsPart>(nt);
  RPT_TRY(sc.reserve(bud.bytes, st));
  int32_t* cnt = sc.carve_n<int32_t>(nt + 1);
  int32_t* base = sc.carve_n<int32_t>(nt + 1);
  BoundsPart* part = sc.carve_n<BoundsPart>(nt);
  hipLaunchKernelGGL(k_land_tile_counts, dim3((unsigned)nt), dim3(kCompBlock), 0, st, cell, n,
                     land, cnt);
  RPT_CHECK_LAUNCH();
  RPT_TRY(exclusive_scan_total_i32(cnt, base, nt, st));
  hipLaunchKernelGGL(k_land_compact, dim3((unsigned)nt), dim3(kCompBlock), 0, st, x, y, v, g, pf,
                     n, cell, land, base, xo, yo, vo, go, pfo, to, part, t_base);
  hipLaunchKernelGGL(k_land_new_off, dim3((n_frames + 1 + 3) / 4), dim3(256), 0, st, base + nt,
                     pfo, n_frames, new_off);
  hipLaunchKernelGGL(k_land_compact_final, dim3(1), dim3(kFinBlock), 0, st, part, (int)nt,
                     base + nt, bounds_out, t_base);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

int32_t land_filter(const float* x, const float* y, const float* v, const int32_t* g,
                    const int32_t* pf, int64_t n, const int64_t* frame_off, int32_t n_frames,
                    const double* xe, int32_t nxe, const double* ye, int32_t nye,
                    const uint8_t* land, float* xo, float* yo, float* vo, int32_t* go,
                    int32_t* pfo, int64_t* new_off, int64_t* n_kept_host, hipStream_t st) {
  return land_filter_cells(x, y, v, g, pf, n, frame_off, n_frames, xe, nxe, ye, nye, land,
                           nullptr, xo, yo, vo, go, pfo, new_off, n_kept_host, st);
}

}  // namespace rpt
