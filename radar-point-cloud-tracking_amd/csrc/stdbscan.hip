// ST-DBSCAN on gfx950: uniform space x time grid, exact neighbour predicate, deterministic
// union-find labelling.  Replaces the BallTree + Python BFS of
//   PointCloudWork/3_stdbscan_point_clouds.py:101-136,
//   radar_pipeline/processors/clustering.py:49-115 and
//   PointCloudWork/4_temporal_object_tracker.py:466-506.
//
// Semantics reproduced bit-exactly:
//   nbr(i,j)  <=>  d2(i,j) <= eps^2  (float64: ((xi-xj)^2 + (yi-yj)^2 [+ (zi-zj)^2]), each op
//                  rounded, no FMA — sklearn's euclidean rdist on float64 copies of the f32 input)
//             and  |t_j - t_i| <= eps_t  (float32 arithmetic; eps_t rounded to float32 — the
//                  reference compares np.float32 values with a Python float under NEP 50)
//   core(i)   <=>  |{ j : nbr(i,j) }| >= min_samples   (the count includes i itself)
//   clusters  =    connected components of the core-core graph, numbered in ascending order of
//                  each component's minimum core-point index (the order the BFS starts them)
//   border    =    non-core point with a core neighbour: minimum adjacent cluster id
//   noise     =    -1
//
// Pipeline (K4..K8 of SURVEY.md §8a):
//   k_bounds      min/max per dimension and time, "times integral" flag        (1 sync)
//   k_keys        cell key per point: ((slab*nz + cz)*ny + cy)*nx + cx
//   radix sort    stable, so every cell lists its points in index order
//   k_gather      sorted float4 {x, y, z|t, t} + original index
//   k_cell_count  -> exclusive scan -> cell_start[C+1]
//   k_cell_box    per occupied cell: bounding box in space and time, "mutual" flag
//                 (box diagonal within eps and time span within eps_t: every pair adjacent)
//   k_core        neighbour count with early exit at min_samples; whole-cell accept/reject
//   k_cell_min_pair  the minimum-original-index core point of each cell (star init)
//   k_union       core-core union-find (min-index hooking); one edge per mutual cell suffices
//   k_compress    root of every point
//   k_cmin        minimum original index per component
//   k_ismin/scan  cluster id = rank of the component minimum among all minima
//   k_label       core: own id; non-core: min id over adjacent core points, else -1
//
// Cell side is 0.7 eps in 2-D and eps/2 in 3-D (x (1+2^-20)): at least eps/2, so every neighbour
// lies within +-2 cells, and small enough that a full cell's diagonal (0.99 eps in 2-D,
// eps*sqrt(3)/2 in 3-D) stays within eps, so dense cells can be "mutual" (decided from their
// actual boxes, k_cell_box).
#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "common.h"

#pragma clang fp contract(off)

namespace rpt {

namespace {

constexpr int kBlock = 256;

// ---------------------------------------------------------------- order-preserving f32 <-> u32
__device__ __forceinline__ uint32_t f2ord(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
inline float ord2f(uint32_t u) {  // host side
  uint32_t v = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
  float f;
  std::memcpy(&f, &v, 4);
  return f;
}

// ---------------------------------------------------------------- cross-lane reductions by DPP
// __shfl_xor compiles to a ds_bpermute round trip through LDS, each one waited for; DPP moves
// are VALU.  Within an aligned row of 16 lanes, step k of row_reduce makes every lane of the
// aligned 2^k-lane group hold the group's result: lane i reads i^1, i^2 (quad permutes), then
// 7-i of its eight (row_half_mirror), then 15-i of its row (row_mirror).  Every lane of a group
// must be active.
template <int Ctl>
__device__ __forceinline__ int dpp_mov(int v) {
  return __builtin_amdgcn_update_dpp(0, v, Ctl, 0xF, 0xF, false);
}
template <int Ctl>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(dpp_mov<Ctl>(__float_as_int(v)));
}
template <int Ctl>
__device__ __forceinline__ uint64_t dpp_mov(uint64_t v) {
  const uint32_t lo = (uint32_t)dpp_mov<Ctl>((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)dpp_mov<Ctl>((int)(uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
template <int G, class T, class F>
__device__ __forceinline__ T row_reduce(T v, F op) {
  static_assert(G == 2 || G == 4 || G == 8 || G == 16, "groups within a row");
#ifdef RPT_DEBUG_DPP
  // (debug builds, -DRPT_DEBUG_DPP) the DPP moves read 0 from an inactive lane: a min would
  // return 0 and a sum drop terms, so every lane of this lane's aligned G-lane group must be
  // active -- all callers keep their loops group-uniform
  {
    const uint64_t act = __ballot(1);
    const int g0 = (int)(threadIdx.x & 63) & ~(G - 1);
    const uint64_t need = (G == 64 ? ~0ull : ((1ull << G) - 1)) << g0;
    if ((act & need) != need) __builtin_trap();
  }
#endif
  v = op(v, dpp_mov<0xB1>(v));                 // quad_perm [1,0,3,2]
  if (G >= 4) v = op(v, dpp_mov<0x4E>(v));     // quad_perm [2,3,0,1]
  if (G >= 8) v = op(v, dpp_mov<0x141>(v));    // row_half_mirror
  if (G >= 16) v = op(v, dpp_mov<0x140>(v));   // row_mirror
  return v;
}
struct OpMin {  // floats: fminf (the ignore-NaN minimum the shuffle form used)
  template <class T>
  __device__ T operator()(T a, T b) const { return b < a ? b : a; }
  __device__ float operator()(float a, float b) const { return fminf(a, b); }
};
struct OpMax {
  template <class T>
  __device__ T operator()(T a, T b) const { return a < b ? b : a; }
  __device__ float operator()(float a, float b) const { return fmaxf(a, b); }
};
struct OpAdd {
  template <class T>
  __device__ T operator()(T a, T b) const { return a + b; }
};
struct OpOr {
  template <class T>
  __device__ T operator()(T a, T b) const { return a | b; }
};


template <int D>
__global__ __launch_bounds__(kBlock) void k_bounds(const float* __restrict__ x,
                                                  const float* __restrict__ y,
                                                  const float* __restrict__ z, int64_t stride,
                                                  const float* __restrict__ t, int64_t n,
                                                  Bounds* __restrict__ out,
                                                  const int64_t* __restrict__ n_dev = nullptr) {
  if (n_dev) n = *n_dev;  // count on the device (at most the host n the grid was sized for)
  uint32_t mn[4] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
  uint32_t mx[4] = {0u, 0u, 0u, 0u};
  int nonfin = 0, nonint = 0, nfin = 0, desc = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v[4];
    v[0] = x[i * stride];
    v[1] = y[i * stride];
    v[2] = (D == 3) ? z[i * stride] : 0.f;
    v[3] = t[i];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (!isfinite(v[k])) nonfin = 1;
      uint32_t o = f2ord(v[k]);
      mn[k] = min(mn[k], o);
      mx[k] = max(mx[k], o);
    }
    if (isfinite(v[3])) {
      ++nfin;
      uint32_t o = f2ord(v[3]);
      mn[3] = min(mn[3], o);
      mx[3] = max(mx[3], o);
      if (v[3] != floorf(v[3]) || fabsf(v[3]) >= 16777216.f) nonint = 1;
    }
    if (i > 0 && !(t[i - 1] <= v[3])) desc = 1;  // NaN counts as out of order
  }
  // wave reduce, then one partial per block
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      mn[k] = min(mn[k], (uint32_t)__shfl_xor((int)mn[k], off));
      mx[k] = max(mx[k], (uint32_t)__shfl_xor((int)mx[k], off));
    }
    nonfin |= __shfl_xor(nonfin, off);
    nonint |= __shfl_xor(nonint, off);
    nfin += __shfl_xor(nfin, off);
    desc |= __shfl_xor(desc, off);
  }
  __shared__ uint32_t smn[kBlock / 64][4], smx[kBlock / 64][4];
  __shared__ int sfl[kBlock / 64][4];
  const int w = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) {
    for (int k = 0; k < 4; ++k) {
      smn[w][k] = mn[k];
      smx[w][k] = mx[k];
    }
    sfl[w][0] = nonfin;
    sfl[w][1] = nonint;
    sfl[w][2] = nfin;
    sfl[w][3] = desc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int v = 1; v < kBlock / 64; ++v) {
      for (int k = 0; k < 4; ++k) {
        mn[k] = min(mn[k], smn[v][k]);
        mx[k] = max(mx[k], smx[v][k]);
      }
      nonfin |= sfl[v][0];
      nonint |= sfl[v][1];
      nfin += sfl[v][2];
      desc |= sfl[v][3];
    }
    // per-block partial, reduced by k_bounds_final (no same-address atomics)
    Bounds& o = out[blockIdx.x];
    for (int k = 0; k < 4; ++k) {
      o.mn[k] = mn[k];
      o.mx[k] = mx[k];
    }
    o.nonfinite_xyz = nonfin;
    o.nonintegral_t = nonint;
    o.n_finite_t = nfin;
    o.t_descends = desc;
  }
}

__global__ __launch_bounds__(kBlock) void k_bounds_final(const Bounds* __restrict__ part, int nb,
                                                        Bounds* __restrict__ out) {
  uint32_t mn[4] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
  uint32_t mx[4] = {0u, 0u, 0u, 0u};
  int nonfin = 0, nonint = 0, nfin = 0, desc = 0;
  for (int b = threadIdx.x; b < nb; b += blockDim.x) {
    const Bounds& p = part[b];
    for (int k = 0; k < 4; ++k) {
      mn[k] = min(mn[k], p.mn[k]);
      mx[k] = max(mx[k], p.mx[k]);
    }
    nonfin |= p.nonfinite_xyz;
    nonint |= p.nonintegral_t;
    nfin += p.n_finite_t;
    desc |= p.t_descends;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      mn[k] = min(mn[k], (uint32_t)__shfl_xor((int)mn[k], off));
      mx[k] = max(mx[k], (uint32_t)__shfl_xor((int)mx[k], off));
    }
    nonfin |= __shfl_xor(nonfin, off);
    nonint |= __shfl_xor(nonint, off);
    nfin += __shfl_xor(nfin, off);
    desc |= __shfl_xor(desc, off);
  }
  __shared__ Bounds sb[kBlock / 64];
  const int w = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) {
    for (int k = 0; k < 4; ++k) {
      sb[w].mn[k] = mn[k];
      sb[w].mx[k] = mx[k];
    }
    sb[w].nonfinite_xyz = nonfin;
    sb[w].nonintegral_t = nonint;
    sb[w].n_finite_t = nfin;
    sb[w].t_descends = desc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int v = 1; v < kBlock / 64; ++v) {
      for (int k = 0; k < 4; ++k) {
        mn[k] = min(mn[k], sb[v].mn[k]);
        mx[k] = max(mx[k], sb[v].mx[k]);
      }
      nonfin |= sb[v].nonfinite_xyz;
      nonint |= sb[v].nonintegral_t;
      nfin += sb[v].n_finite_t;
      desc |= sb[v].t_descends;
    }
    for (int k = 0; k < 4; ++k) {
      out->mn[k] = mn[k];
      out->mx[k] = mx[k];
    }
    out->nonfinite_xyz = nonfin;
    out->nonintegral_t = nonint;
    out->n_finite_t = nfin;
    out->t_descends = desc;
  }
}

// ---------------------------------------------------------------- grid geometry
// n / d for 0 <= n < 2^31 by one 32 x 32 -> 64-bit multiply and a shift (Granlund-Montgomery):
// m = ceil(2^(31+k) / d) with 2^(k-1) < d <= 2^k, so m < 2^32 and the rounding error n * (m / 2^(31+k)
// - 1 / d) < 2^-k <= 1 / d never reaches the next integer.  The cell-key decodes of the latency-
// bound window kernels divided by runtime grid sizes (a few dozen VALU instructions each).
struct FastDiv {
  uint32_t m;
  int s;
  void init(uint32_t d) {
    int k = 0;
    while ((uint64_t(1) << k) < d) ++k;
    s = 31 + k;
    m = (uint32_t)(((uint64_t(1) << s) + d - 1) / d);
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    return (uint32_t)(((uint64_t)n * m) >> s);
  }
};

struct Geom {
  double ox, oy, oz, ot;  // origins (minima)
  double cs;              // spatial cell side
  double ct;              // time slab width
  double inv_cs, inv_ct;  // their float64 reciprocals (cell_of)
  int nx, ny, nz, nt;
  int64_t cells;          // nx*ny*nz*nt (an extra "isolated" cell C holds non-finite t)
  double eps2;            // eps_space^2 (float64)
  float epst;             // float32(eps_time)
  int min_samples;
  // float32 box-bound screen (classify_cells<D, true>): a float32 squared box distance <= e2lo
  // (> e2hi) is <= (>) eps2 in the float64 bound too (margins 1e-5 >> the float32 rounding);
  // e2lo = -1 / e2hi = inf disable it (eps2 outside [1e-20, 1e30])
  float e2lo, e2hi;
  // integral times (slabs hold whole time values): every neighbour of a point or cell in slab s
  // lies in slabs [s - rt, s + rt] (DbscanState::slab_reach), so the scan windows take exactly
  // those; -1: non-integral times, windows from the time range with one slab of slack each side
  int rt;
  // 1: every time is an integer and a slab is ONE time value (ct == 1), so any two points whose
  // slabs lie within rt <= floor(eps_t) of each other pass the time test: the window kernels, whose
  // candidates all come from such windows, skip the time bounds of their box classifications
  int tfree;
  FastDiv fnx, fny, fnz, fslab;  // by nx, ny, nz and nx * ny * nz (a key's slab)
  // cell key (< 2^31) -> x, y, z, slab
  __device__ __forceinline__ void split(uint32_t k, int& x, int& y, int& z, int& s) const {
    const uint32_t r = fnx.div(k);
    x = (int)(k - r * (uint32_t)nx);
    const uint32_t r2 = fny.div(r);
    y = (int)(r - r2 * (uint32_t)ny);
    if (nz == 1) {
      z = 0;
      s = (int)r2;
    } else {
      const uint32_t r3 = fnz.div(r2);
      z = (int)(r2 - r3 * (uint32_t)nz);
      s = (int)r3;
    }
  }
  __device__ __forceinline__ int slab_of_key(int64_t k) const { return (int)fslab.div((uint32_t)k); }
};

// cell index floor((v - o) / side) as a multiply by the host's float64 reciprocal (a float64
// divide per coordinate dominated the grid build); every kernel assigns cells through this one
// function, so assignments stay consistent, and the 2^-20 margin on the side keeps every
// neighbour within +-2 cells whatever the last-bit rounding
__device__ __forceinline__ int cell_of(double v, double o, double inv, int n) {
  double q = floor((v - o) * inv);
  int c = (q < 0.0) ? 0 : (q >= (double)n ? n - 1 : (int)q);
  return c;
}
__device__ __forceinline__ int slab_of(float t, const Geom& g) {
  return cell_of((double)t, g.ot, g.inv_ct, g.nt);
}

template <int D>
__global__ __launch_bounds__(kBlock) void k_keys(const float* __restrict__ x,
                                                const float* __restrict__ y,
                                                const float* __restrict__ z, int64_t stride,
                                                const float* __restrict__ t, int64_t n, Geom g,
                                                uint32_t* __restrict__ keys,
                                                uint32_t* __restrict__ vals) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float ti = t[i];
    uint32_t key;
    if (!isfinite(ti)) {
      key = (uint32_t)g.cells;  // isolated: matches nothing, not even itself
    } else {
      const int cx = cell_of((double)x[i * stride], g.ox, g.inv_cs, g.nx);
      const int cy = cell_of((double)y[i * stride], g.oy, g.inv_cs, g.ny);
      const int cz = (D == 3) ? cell_of((double)z[i * stride], g.oz, g.inv_cs, g.nz) : 0;
      const int s = slab_of(ti, g);
      key = (uint32_t)((((int64_t)s * g.nz + cz) * g.ny + cy) * g.nx + cx);
    }
    keys[i] = key;
    vals[i] = (uint32_t)i;
  }
}

template <int D>
__global__ __launch_bounds__(kBlock) void k_gather(const float* __restrict__ x,
                                                  const float* __restrict__ y,
                                                  const float* __restrict__ z, int64_t stride,
                                                  const float* __restrict__ t, int64_t n,
                                                  const uint32_t* __restrict__ skeys,
                                                  const uint32_t* __restrict__ svals,
                                                  float4* __restrict__ pts,
                                                  int32_t* __restrict__ sorig,
                                                  int32_t* __restrict__ skey,
                                                  int32_t* __restrict__ spos) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n;
       s += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = svals[s];
    float4 p;
    p.x = x[i * stride];
    p.y = y[i * stride];
    p.w = t[i];
    p.z = (D == 3) ? z[i * stride] : p.w;
    pts[s] = p;
    sorig[s] = (int32_t)i;
    if (spos) spos[i] = (int32_t)s;
    skey[s] = (int32_t)skeys[s];
  }
}

// Cell occupancy from the sorted keys (no atomics on hot cells): a run's head subtracts its start
// and its tail adds its end, so cell_count[c] = run length (two uncontended atomics per occupied
// cell); head flags (scanned later) give the occupied-cell list in ascending key order.
__global__ __launch_bounds__(kBlock) void k_cell_runs(const int32_t* __restrict__ skey, int64_t n,
                                                     int32_t* __restrict__ cell_count,
                                                     int32_t* __restrict__ head) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n;
       s += (int64_t)gridDim.x * blockDim.x) {
    const int32_t k = skey[s];
    const bool h = (s == 0) || skey[s - 1] != k;
    const bool t = (s == n - 1) || skey[s + 1] != k;
    if (h && t) {
      cell_count[k] = 1;
    } else {
      if (h) atomicAdd(cell_count + k, -(int32_t)s);
      if (t) atomicAdd(cell_count + k, (int32_t)(s + 1));
    }
    head[s] = h ? 1 : 0;
  }
}

// pos = exclusive scan of the head flags: cell of every run head -> occ[pos]
// (+ the occupancy bitmap: one bit per cell, small enough to stay in L2, so window scans skip
// empty candidate cells without reading their records)
__global__ __launch_bounds__(kBlock) void k_occ_list(const int32_t* __restrict__ skey, int64_t n,
                                                    const int32_t* __restrict__ pos,
                                                    int32_t* __restrict__ occ,
                                                    uint32_t* __restrict__ occ_bits) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n;
       s += (int64_t)gridDim.x * blockDim.x)
    if (pos[s + 1] != pos[s]) {
      const int32_t c = skey[s];
      occ[pos[s]] = c;
      atomicOr(occ_bits + (c >> 5), 1u << (c & 31));
    }
}

// ---- K4 for time-ordered 2-D input (the stack path: points come frame-major from K1 / the land
// filter, and a slab is a frame): the cell sort is a counting sort of each slab's points by their
// (y, x) cell, one 1024-thread block per slab with the slab's cell histogram in LDS.  It replaces
// keys + three radix passes + the gather + the cell-count pass: two reads of x / y (/ t) and one
// scattered write of the sorted records per point, and the dense cell_start rows come out of the
// histogram scan directly.  Order inside a cell is arrival order: nothing downstream depends on
// it (roots are minimum ORIGINAL indices, counts and minima are order-free).
constexpr int kBucketBlock = 1024;
constexpr int kBucketCells = 16384;  // max per-slab cells for the LDS histogram (<= 64 KiB)
constexpr int kBucketU = 4;          // points per thread per round (loads in flight together)
constexpr int64_t kChunkPts = 16384;  // points per slab-bucket block when a slab is split
// RPT_SLAB_CHUNKS=k: k blocks per slab (1 = the single-block k_slab_bucket; A/B)
static int slab_chunks_override() {
  static const int v = [] {
    const char* e = ab_env("RPT_SLAB_CHUNKS");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

// A/B switch with three values: 0 off, 1 the default rule, 2 forced on (the parity tests of the
// A/B build run a path on inputs its default rule would not take it for)
static int ab_mode(const char* name) {
  const char* e = ab_env(name);
  const int v = e ? std::atoi(e) : 1;
  return (v == 0 || v == 2) ? v : 1;
}
// RPT_CELL_BOX_MIXED=0: 16 lanes for every cell's box (k_cell_box); 2: k_cell_box_mixed always
static int cell_box_mixed() {
  static const int v = ab_mode("RPT_CELL_BOX_MIXED");
  return v;
}
// RPT_UNION_SNAP=0: no root snapshot before the listed union pass; 2: also on dense slabs
static int union_snapshot() {
  static const int v = ab_mode("RPT_UNION_SNAP");
  return v;
}

// RPT_LABEL_ORIG=0: core labels scattered from sorted order (k_label_core); 2: the inverse
// permutation and original-order labels at every density
static int label_core_orig() {
  static const int v = ab_mode("RPT_LABEL_ORIG");
  return v;
}

// RPT_CHUNK_SCAN=1: the one-block-per-slab k_slab_chunk_scan (A/B)
static bool chunk_scan_legacy() {
  static const bool v = [] {
    const char* e = ab_env("RPT_CHUNK_SCAN");
    return e && std::atoi(e) == 1;
  }();
  return v;
}

// occ_base[s] = the first occupied-list position of slab s (the flags' exclusive scan at the
// slab's first cell), occ_base[nt] = the occupied count
__global__ void k_slab_occ_base(const int32_t* __restrict__ pos, int P, int64_t nt,
                                int32_t* __restrict__ occ_base) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= nt;
       s += (int64_t)gridDim.x * blockDim.x)
    occ_base[s] = pos[s * P];
}

// cell_start[cells] = n (the scan's total) -> the isolated cell (empty) ends there too
__global__ void k_cell_start_end(int32_t* __restrict__ cell_start, int64_t cells) {
  if (threadIdx.x == 0) cell_start[cells + 1] = cell_start[cells];
}

// slab_lo[s] = first point of slab s (points ordered by slab), slab_lo[nt] = n: ONE WAVE per
// slab, a 64-ary search (64 probes per round: ~5 dependent rounds over 50 M points instead of a
// thread's 26-step binary search).  Also clears zero[0, zwords) (the occupancy bits the slab
// bucket sets next: one launch instead of a memset and this).
__global__ void k_slab_lo(const float* __restrict__ t, int64_t n, Geom g,
                          int32_t* __restrict__ slab_lo, uint32_t* __restrict__ zero,
                          int64_t zwords) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < zwords;
       i += (int64_t)gridDim.x * blockDim.x)
    zero[i] = 0u;
  const int lane = threadIdx.x & 63;
  const int64_t wpb = blockDim.x / 64;
  for (int64_t s = (int64_t)blockIdx.x * wpb + threadIdx.x / 64; s <= g.nt;
       s += (int64_t)gridDim.x * wpb) {
    int64_t lo = 0, hi = n;  // the first point of slab >= s lies in [lo, hi]
    while (lo < hi) {
      const int64_t step = (hi - lo + 63) / 64;
      const int64_t idx = lo + (int64_t)lane * step;
      const bool below = idx < hi && slab_of(t[idx < hi ? idx : lo], g) < s;  // a lane prefix
      const int c = __popcll(__ballot(below));
      if (c == 0) {
        hi = lo;
      } else {
        const int64_t nlo = lo + (int64_t)(c - 1) * step + 1;
        hi = min(hi, lo + (int64_t)c * step);
        lo = nlo;
      }
    }
    if (lane == 0) slab_lo[s] = (int32_t)(s == g.nt ? n : lo);
  }
}

__global__ __launch_bounds__(kBucketBlock) void k_slab_bucket(
    const float* __restrict__ x, const float* __restrict__ y, int64_t stride,
    const float* __restrict__ t, Geom g, const int32_t* __restrict__ slab_lo,
    float4* __restrict__ pts, int32_t* __restrict__ sorig, int32_t* __restrict__ skey,
    int32_t* __restrict__ spos, int32_t* __restrict__ cell_start, int32_t* __restrict__ occ_tmp,
    int32_t* __restrict__ slab_occ, uint32_t* __restrict__ occ_bits,
    unsigned long long* __restrict__ cmin_all = nullptr) {
  // the slab's nx * ny cell counts, sized at launch (a 463-m sweep at cells of 5.6 m: 27 KiB, so
  // several slabs share a CU instead of one 64-KiB histogram each)
  // cmin_all (nullable; the fused K5): every occupied cell's (min original, sorted) pair over all
  // its points -- the smallest index per cell by an LDS atomicMin per run in the count pass (a
  // run's head lane holds its smallest index), written by that point at its scatter
  extern __shared__ int32_t hist[];
  __shared__ int32_t wsum[kBucketBlock / 64], wocc[kBucketBlock / 64];
  const int s = blockIdx.x;
  const int P = g.nx * g.ny;
  int32_t* mn = hist + P;  // (cmin_all only: the launch sizes 2P words)
  const int lo = slab_lo[s], hi = slab_lo[s + 1];
  for (int c = threadIdx.x; c < P; c += kBucketBlock) {
    hist[c] = 0;
    if (cmin_all) mn[c] = INT_MAX;
  }
  __syncthreads();
  // consecutive points (along a ray) often share a cell: a run of equal cells in a wave takes
  // ONE LDS atomic (by its head lane) instead of one per point
  const int ln = threadIdx.x & 63;
  auto runs = [&](int c, bool v, int& rank, int& len, int& head) {
    const int up = __shfl_up(c, 1, 64), dn = __shfl_down(c, 1, 64);
    const uint64_t hm = __ballot(v && (ln == 0 || up != c));
    const uint64_t lm = __ballot(v && (ln == 63 || dn != c));
    const uint64_t below = (ln == 63) ? ~0ull : ((2ull << ln) - 1ull);
    head = 63 - __builtin_clzll((hm & below) | 1ull);  // hm has a bit at or below ln when v
    const int last = ln + __builtin_ctzll((lm >> ln) | (1ull << (63 - ln)));
    rank = ln - head;
    len = last - head + 1;
  };
  // kBucketU points per thread per round, their loads issued together
  auto cell_xy = [&](float px, float py) {
    return cell_of((double)py, g.oy, g.inv_cs, g.ny) * g.nx +
           cell_of((double)px, g.ox, g.inv_cs, g.nx);
  };
  for (int i0 = lo; i0 < hi; i0 += kBucketBlock * kBucketU) {
    // loads from clamped indices (the slab is not empty here): a conditional load would be a
    // branch ending in a full vmcnt wait, one round trip per point instead of per round
    float px[kBucketU], py[kBucketU];
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) {
      const int i = min(i0 + u * kBucketBlock + (int)threadIdx.x, hi - 1);
      px[u] = x[(int64_t)i * stride];
      py[u] = y[(int64_t)i * stride];
    }
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) {
      const int i = i0 + u * kBucketBlock + threadIdx.x;
      const bool v = i < hi;
      const int c = v ? cell_xy(px[u], py[u]) : -1;
      int rank, len, head;
      runs(c, v, rank, len, head);
      if (v && rank == 0) {
        atomicAdd(&hist[c], len);
        if (cmin_all) atomicMin(&mn[c], i);
      }
    }
  }
  __syncthreads();
  // exclusive scan of hist[0, P): each thread a contiguous run, then the block's run sums
  const int per = (P + kBucketBlock - 1) / kBucketBlock;
  const int c0 = threadIdx.x * per, c1 = min(c0 + per, P);
  int run = 0, orun = 0;
  for (int c = c0; c < c1; ++c) {
    const int h = hist[c];
    run += h;
    orun += (h > 0) ? 1 : 0;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x / 64;
  int incl = run, oincl = orun;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(incl, off, 64);
    const int oo = __shfl_up(oincl, off, 64);
    if (lane >= off) {
      incl += o;
      oincl += oo;
    }
  }
  if (lane == 63) {
    wsum[w] = incl;
    wocc[w] = oincl;
  }
  __syncthreads();
  int before = 0, obefore = 0, otot = 0;
  for (int v = 0; v < kBucketBlock / 64; ++v) {
    if (v < w) {
      before += wsum[v];
      obefore += wocc[v];
    }
    otot += wocc[v];
  }
  int acc = before + incl - run;
  // the slab's occupied cells, ascending, at the front of its point range (a slab has no more
  // occupied cells than points), and their occupancy bits (one atomicOr per word of this run)
  int oacc = lo + obefore + oincl - orun;
  uint32_t word = 0xffffffffu, mask = 0u;
  for (int c = c0; c < c1; ++c) {
    const int h = hist[c];
    hist[c] = acc;
    cell_start[(int64_t)s * P + c] = lo + acc;
    acc += h;
    if (h > 0) {
      const int64_t key = (int64_t)s * P + c;
      occ_tmp[oacc++] = (int32_t)key;
      const uint32_t wd = (uint32_t)(key >> 5);
      if (wd != word) {
        if (mask) atomicOr(occ_bits + word, mask);
        word = wd;
        mask = 0u;
      }
      mask |= 1u << (key & 31);
    }
  }
  if (mask) atomicOr(occ_bits + word, mask);
  if (threadIdx.x == 0) slab_occ[s] = otot;
  __syncthreads();
  for (int i0 = lo; i0 < hi; i0 += kBucketBlock * kBucketU) {
    float px[kBucketU], py[kBucketU], pt[kBucketU];
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) {
      const int i = min(i0 + u * kBucketBlock + (int)threadIdx.x, hi - 1);  // branch-free
      px[u] = x[(int64_t)i * stride];
      py[u] = y[(int64_t)i * stride];
      pt[u] = t[i];
    }
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) {
      const int i = i0 + u * kBucketBlock + threadIdx.x;
      const bool v = i < hi;
      const int c = v ? cell_xy(px[u], py[u]) : -1;
      int rank, len, head;
      runs(c, v, rank, len, head);
      int base = (v && rank == 0) ? atomicAdd(&hist[c], len) : 0;
      base = __shfl(base, head, 64);
      if (v) {
        const int dst = lo + base + rank;
        pts[dst] = make_float4(px[u], py[u], pt[u], pt[u]);
        sorig[dst] = i;
        if (spos) spos[i] = dst;  // (kernel-uniform; coalesced: i runs over the lanes)
        skey[dst] = s * P + c;
        if (cmin_all && mn[c] == i)
          cmin_all[(int64_t)s * P + c] = ((unsigned long long)(uint32_t)i << 32) | (uint32_t)dst;
      }
    }
  }
  if (s == g.nt - 1 && threadIdx.x == 0) {  // the isolated cell (empty here) and the end
    cell_start[g.cells] = hi;
    cell_start[g.cells + 1] = hi;
  }
}

// Several blocks per slab (dense slabs: one block per slab leaves most CUs idle and serialises
// hundreds of thousands of points per block).  Chunk ch of slab s is its points
// [lo + ch*len/CH, lo + (ch+1)*len/CH).  hist: [nt][CH][P] per-chunk cell counts, turned by
// k_slab_chunk_scan into per-chunk write cursors; the scan also writes cell_start, the slab's
// occupied cells + bits and its occupied count exactly like k_slab_bucket.
__device__ __forceinline__ void slab_chunk(const int32_t* __restrict__ slab_lo, int s, int ch,
                                           int CH, int& lo, int& hi) {
  const int a = slab_lo[s], b = slab_lo[s + 1];
  const int64_t len = (int64_t)(b - a);
  lo = a + (int)(len * ch / CH);
  hi = a + (int)(len * (ch + 1) / CH);
}

__global__ __launch_bounds__(kBucketBlock) void k_slab_chunk_hist(
    const float* __restrict__ x, const float* __restrict__ y, int64_t stride, Geom g,
    const int32_t* __restrict__ slab_lo, int CH, int32_t* __restrict__ hist_g) {
  extern __shared__ int32_t hist[];
  const int s = blockIdx.x / CH, ch = blockIdx.x - s * CH;
  const int P = g.nx * g.ny;
  int lo, hi;
  slab_chunk(slab_lo, s, ch, CH, lo, hi);
  for (int c = threadIdx.x; c < P; c += kBucketBlock) hist[c] = 0;
  __syncthreads();
  for (int i0 = lo; i0 < hi; i0 += kBucketBlock * kBucketU) {
    float px[kBucketU], py[kBucketU];
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) {
      const int i = min(i0 + u * kBucketBlock + (int)threadIdx.x, hi - 1);  // branch-free
      px[u] = x[(int64_t)i * stride];
      py[u] = y[(int64_t)i * stride];
    }
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) {
      const int i = i0 + u * kBucketBlock + threadIdx.x;
      if (i < hi)
        atomicAdd(&hist[cell_of((double)py[u], g.oy, g.inv_cs, g.ny) * g.nx +
                        cell_of((double)px[u], g.ox, g.inv_cs, g.nx)], 1);
    }
  }
  __syncthreads();
  int32_t* out = hist_g + (int64_t)blockIdx.x * P;
  for (int c = threadIdx.x; c < P; c += kBucketBlock) out[c] = hist[c];
}

__global__ __launch_bounds__(kBucketBlock) void k_slab_chunk_scan(
    Geom g, const int32_t* __restrict__ slab_lo, int CH, int32_t* __restrict__ hist_g,
    int32_t* __restrict__ cell_start, int32_t* __restrict__ occ_tmp,
    int32_t* __restrict__ slab_occ, uint32_t* __restrict__ occ_bits) {
  __shared__ int32_t wsum[kBucketBlock / 64], wocc[kBucketBlock / 64];
  const int s = blockIdx.x;
  const int P = g.nx * g.ny;
  const int lo = slab_lo[s], hi = slab_lo[s + 1];
  int32_t* hs = hist_g + (int64_t)s * CH * P;
  const int per = (P + kBucketBlock - 1) / kBucketBlock;
  const int c0 = threadIdx.x * per, c1 = min(c0 + per, P);
  int run = 0, orun = 0;
  for (int c = c0; c < c1; ++c) {
    int h = 0;
    for (int ch = 0; ch < CH; ++ch) h += hs[(int64_t)ch * P + c];
    run += h;
    orun += (h > 0) ? 1 : 0;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x / 64;
  int incl = run, oincl = orun;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(incl, off, 64);
    const int oo = __shfl_up(oincl, off, 64);
    if (lane >= off) {
      incl += o;
      oincl += oo;
    }
  }
  if (lane == 63) {
    wsum[w] = incl;
    wocc[w] = oincl;
  }
  __syncthreads();
  int before = 0, obefore = 0, otot = 0;
  for (int v = 0; v < kBucketBlock / 64; ++v) {
    if (v < w) {
      before += wsum[v];
      obefore += wocc[v];
    }
    otot += wocc[v];
  }
  int acc = before + incl - run;
  int oacc = lo + obefore + oincl - orun;
  uint32_t word = 0xffffffffu, mask = 0u;
  for (int c = c0; c < c1; ++c) {
    cell_start[(int64_t)s * P + c] = lo + acc;
    int h = 0;
    for (int ch = 0; ch < CH; ++ch) {  // per-chunk cursors (slab-local), chunk order
      const int k = hs[(int64_t)ch * P + c];
      hs[(int64_t)ch * P + c] = acc + h;
      h += k;
    }
    acc += h;
    if (h > 0) {
      const int64_t key = (int64_t)s * P + c;
      occ_tmp[oacc++] = (int32_t)key;
      const uint32_t wd = (uint32_t)(key >> 5);
      if (wd != word) {
        if (mask) atomicOr(occ_bits + word, mask);
        word = wd;
        mask = 0u;
      }
      mask |= 1u << (key & 31);
    }
  }
  if (mask) atomicOr(occ_bits + word, mask);
  if (threadIdx.x == 0) slab_occ[s] = otot;
  if (s == g.nt - 1 && threadIdx.x == 0) {  // the isolated cell (empty here) and the end
    cell_start[g.cells] = hi;
    cell_start[g.cells + 1] = hi;
  }
}

// The same outputs as k_slab_chunk_scan from fully parallel, coalesced passes over every
// (slab, cell) -- one block per slab walking its cells in per-thread runs left most CUs idle
// and read the [chunk][cell] histograms with a lane stride (2.2 GB per dense 125-frame share):
//   k_chunk_totals   cell_start[key] = the cell's count over the slab's chunks
//   (in-place exclusive scan of cell_start: the points are slab-major, so the global prefix IS
//    every cell's first point)
//   k_chunk_cursors  per-chunk slab-local write cursors, occupancy words (one ballot per 64
//                    keys), occupied flags
//   (exclusive scan of the flags) -> k_occ_write: the ascending occupied list and its count.
__global__ void k_chunk_totals(const int32_t* __restrict__ hist_g, int64_t cells, int P, int CH,
                               int32_t* __restrict__ cell_start) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < cells;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = k / P;
    const int32_t* h = hist_g + s * (int64_t)CH * P + (k - s * P);
    int t = 0;
    for (int ch = 0; ch < CH; ++ch) t += h[(int64_t)ch * P];
    cell_start[k] = t;
  }
}

__global__ void k_chunk_cursors(int32_t* __restrict__ hist_g, int64_t cells, int P, int CH,
                                const int32_t* __restrict__ cell_start,
                                const int32_t* __restrict__ slab_lo,
                                uint32_t* __restrict__ occ_bits, int32_t* __restrict__ occf) {
  // whole waves over 64 consecutive keys (the grid stride is a multiple of 64): the wave's
  // ballot of occupied cells is two whole occupancy words
  const int lane = threadIdx.x & 63;
  for (int64_t k0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) & ~(int64_t)63; k0 < cells;
       k0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = k0 + lane;
    bool o = false;
    if (k < cells) {
      const int64_t s = k / P;
      int32_t* h = hist_g + s * (int64_t)CH * P + (k - s * P);
      int acc = cell_start[k] - slab_lo[s];
      const int first = acc;
      for (int ch = 0; ch < CH; ++ch) {
        const int v = h[(int64_t)ch * P];
        h[(int64_t)ch * P] = acc;
        acc += v;
      }
      o = acc > first;
      occf[k] = o ? 1 : 0;
    }
    const uint64_t m = __ballot(o);
    if (lane == 0) occ_bits[k0 >> 5] = (uint32_t)m;
    if (lane == 32) occ_bits[(k0 >> 5) + 1] = (uint32_t)(m >> 32);
  }
}

__global__ void k_occ_write(const int32_t* __restrict__ occf, const int32_t* __restrict__ pos,
                            int64_t cells, int32_t* __restrict__ occ) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < cells;
       k += (int64_t)gridDim.x * blockDim.x)
    if (occf[k]) occ[pos[k]] = (int32_t)k;
}

__global__ __launch_bounds__(kBucketBlock) void k_slab_chunk_scatter(
    const float* __restrict__ x, const float* __restrict__ y, int64_t stride,
    const float* __restrict__ t, Geom g, const int32_t* __restrict__ slab_lo, int CH,
    const int32_t* __restrict__ hist_g, float4* __restrict__ pts, int32_t* __restrict__ sorig,
    int32_t* __restrict__ skey, int32_t* __restrict__ spos) {
  extern __shared__ int32_t cur[];
  const int s = blockIdx.x / CH, ch = blockIdx.x - s * CH;
  const int P = g.nx * g.ny;
  int lo, hi;
  slab_chunk(slab_lo, s, ch, CH, lo, hi);
  const int base = slab_lo[s];
  const int32_t* hc = hist_g + (int64_t)blockIdx.x * P;
  for (int c = threadIdx.x; c < P; c += kBucketBlock) cur[c] = hc[c];
  __syncthreads();
  for (int i0 = lo; i0 < hi; i0 += kBucketBlock * kBucketU) {
    float px[kBucketU], py[kBucketU], pt[kBucketU];
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) {
      const int i = min(i0 + u * kBucketBlock + (int)threadIdx.x, hi - 1);  // branch-free
      px[u] = x[(int64_t)i * stride];
      py[u] = y[(int64_t)i * stride];
      pt[u] = t[i];
    }
#pragma unroll
    for (int u = 0; u < kBucketU; ++u) {
      const int i = i0 + u * kBucketBlock + threadIdx.x;
      if (i < hi) {
        const int c = cell_of((double)py[u], g.oy, g.inv_cs, g.ny) * g.nx +
                      cell_of((double)px[u], g.ox, g.inv_cs, g.nx);
        const int dst = base + atomicAdd(&cur[c], 1);
        pts[dst] = make_float4(px[u], py[u], pt[u], pt[u]);
        sorig[dst] = i;
        if (spos) spos[i] = dst;  // (kernel-uniform; coalesced: i runs over the lanes)
        skey[dst] = s * P + c;
      }
    }
  }
}

// the slabs' occupied-cell runs (k_slab_bucket, at each slab's point offset) -> the ascending list
__global__ __launch_bounds__(kBlock) void k_occ_gather(const int32_t* __restrict__ occ_tmp,
                                                      const int32_t* __restrict__ slab_lo,
                                                      const int32_t* __restrict__ occ_base,
                                                      int32_t* __restrict__ occ) {
  const int s = blockIdx.x;
  const int b = occ_base[s], m = occ_base[s + 1] - b, lo = slab_lo[s];
  for (int j = threadIdx.x; j < m; j += blockDim.x) occ[b + j] = occ_tmp[lo + j];
}

__device__ __forceinline__ bool occupied(const uint32_t* __restrict__ bits, int64_t c) {
  return (bits[c >> 5] >> (c & 31)) & 1u;
}

// grids of the persistent wave-per-item kernels (item counts live on the device)
// A/B build: RPT_WAVE_GRID_CAP caps the wave-per-item kernels' grids (fewer resident waves
// leave room for other stacks' kernels on the same CUs)
static int wave_grid_cap() {
  static const int cap = [] {
    const char* e = ab_env("RPT_WAVE_GRID_CAP");
    const int v = e ? std::atoi(e) : 0;
    return v >= 8 ? v : 4096;
  }();
  return cap;
}
inline int wave_grid(int64_t max_items) {  // a multiple of 8 blocks (XCD-aware ranges)
  const int g = grid_for(max_items, kBlock / 64, wave_grid_cap());
  return (g + 7) & ~7;
}
constexpr int kDefaultUfFlags = 2;
inline int tile_grid(int64_t n) { return grid_for(n, kBlock * 16, 2048); }

__device__ __forceinline__ float wave_minf(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fminf(v, __shfl_xor(v, off));
  return v;
}
__device__ __forceinline__ float wave_maxf(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
  return v;
}
// whole-wave sum (every lane active): rows by DPP, then the four row sums read as scalars
__device__ __forceinline__ int wave_sum(int v) {
  v = row_reduce<16>(v, OpAdd{});
  return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) +
         __builtin_amdgcn_readlane(v, 32) + __builtin_amdgcn_readlane(v, 48);
}
__device__ __forceinline__ int wave_excl_sum(int v, int* total) {
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
__device__ __forceinline__ int64_t wave_min64(int64_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const int64_t o = __shfl_xor(v, off);
    v = o < v ? o : v;
  }
  return v;
}

// Per occupied cell, its point range and bounding box in ONE record (32 B in 2-D, 48 B in 3-D), so
// a candidate cell of a window scan costs one load; empty cells are zero (b == e).
template <int D>
struct CellRec;
template <>
struct alignas(16) CellRec<2> {
  int b, e;
  float x0, x1, y0, y1, t0, t1;
};
template <>
struct alignas(16) CellRec<3> {
  int b, e;
  float x0, x1, y0, y1, z0, z1, t0, t1;
  int pad0, pad1;
};
template <int D>
__device__ __forceinline__ float4 rec_boxA(const CellRec<D>& r) {
  return make_float4(r.x0, r.x1, r.y0, r.y1);
}
__device__ __forceinline__ float4 rec_boxB(const CellRec<2>& r) {
  return make_float4(r.t0, r.t1, r.t0, r.t1);
}
__device__ __forceinline__ float4 rec_boxB(const CellRec<3>& r) {
  return make_float4(r.z0, r.z1, r.t0, r.t1);
}

// Per-cell records (point range and bounding box in space and time; the only copy of the boxes:
// the per-point union reads them from the records too), kCbLanes lanes per occupied cell, four
// cells per wave.  A wave waits for its densest cell (a few hundred points at the standard
// density, thousands in the dense stacks), so lanes per cell set the rate: same-box A/B
// (tools/kab2.sh, 1000 standard / 125 dense frames) 4 lanes 434 / 403 us, 8 lanes 353 / 347,
// 16 lanes 347 / 321, 32 lanes 453 / 387.  mutual[c] = 1 when every pair of points in the cell
// passes the neighbour test (computed conservatively from the box with the same rounding as the
// pair test).
constexpr int kCbLanes = 16;
template <int D>
__global__ __launch_bounds__(kBlock) void k_cell_box(const float4* __restrict__ pts,
                                                    const int32_t* __restrict__ cell_start,
                                                    const int32_t* __restrict__ occ,
                                                    const int32_t* __restrict__ n_occ, Geom g,
                                                    uint8_t* __restrict__ mutual,
                                                    CellRec<D>* __restrict__ crec,
                                                    unsigned long long* __restrict__ cmin =
                                                        nullptr,
                                                    const int32_t* __restrict__ sorig = nullptr) {
  // sorig (kernel-uniform): cmin[c] = the (min original, sorted) pair over ALL the cell's points
  // (the fused K5 keeps it for all-core cells), read alongside the points; otherwise none (~0)
  constexpr int L = kCbLanes;
  const int j = threadIdx.x & (L - 1);
  const int64_t no = *n_occ;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t - j < no * L;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = t / L;
    const bool act = q < no;
    int c = 0, b = 0, e = 0;
    if (act) {
      c = occ[q];
      b = cell_start[c];
      e = cell_start[c + 1];
    }
    float x0 = FLT_MAX, x1 = -FLT_MAX, y0 = FLT_MAX, y1 = -FLT_MAX;
    float z0 = FLT_MAX, z1 = -FLT_MAX, t0 = FLT_MAX, t1 = -FLT_MAX;
    uint64_t mn = ~0ull;
    // 8 loads in flight per lane: a dense cell (hundreds of points) is otherwise a chain of
    // dependent load round trips on its lanes
    constexpr int kU = 8;
    for (int s0 = b + j; s0 < e; s0 += L * kU) {
      float4 pp[kU];
      uint32_t so[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int s2 = s0 + L * u;
        const int sc = (s2 < e) ? s2 : s0;  // duplicates of a cell point leave the box as is
        pp[u] = pts[sc];
        if (sorig) so[u] = (uint32_t)sorig[sc];
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const float4 p = pp[u];
        x0 = fminf(x0, p.x); x1 = fmaxf(x1, p.x);
        y0 = fminf(y0, p.y); y1 = fmaxf(y1, p.y);
        z0 = fminf(z0, p.z); z1 = fmaxf(z1, p.z);
        t0 = fminf(t0, p.w); t1 = fmaxf(t1, p.w);
        if (sorig) {
          const int s2 = s0 + L * u;
          const uint64_t v = ((uint64_t)so[u] << 32) | (uint32_t)((s2 < e) ? s2 : s0);
          mn = v < mn ? v : mn;
        }
      }
    }
    // (the cell loop is uniform over the aligned 16-lane group: all its lanes are active)
    if (sorig) mn = row_reduce<L>(mn, OpMin{});
    x0 = row_reduce<L>(x0, OpMin{}); x1 = row_reduce<L>(x1, OpMax{});
    y0 = row_reduce<L>(y0, OpMin{}); y1 = row_reduce<L>(y1, OpMax{});
    z0 = row_reduce<L>(z0, OpMin{}); z1 = row_reduce<L>(z1, OpMax{});
    t0 = row_reduce<L>(t0, OpMin{}); t1 = row_reduce<L>(t1, OpMax{});
    if (D != 3) {
      z0 = t0;  // 2-D: pts[].z carries t (unused by the 2-D tests)
      z1 = t1;
    }
    if (act && j == 0) {
      CellRec<D> r{};
      r.b = b;
      r.e = e;
      r.x0 = x0;
      r.x1 = x1;
      r.y0 = y0;
      r.y1 = y1;
      if constexpr (D == 3) {
        r.z0 = z0;
        r.z1 = z1;
      }
      r.t0 = t0;
      r.t1 = t1;
      crec[c] = r;
      const double dx = (double)x1 - (double)x0;
      const double dy = (double)y1 - (double)y0;
      double d2 = dx * dx + dy * dy;
      if (D == 3) {
        const double dz = (double)z1 - (double)z0;
        d2 = d2 + dz * dz;
      }
      const float dt = t1 - t0;
      mutual[c] = (d2 <= g.eps2 && dt <= g.epst) ? 1 : 0;
      if (cmin) cmin[c] = sorig ? mn : ~0ull;  // the core pass's per-cell minima
    }
  }
}

// The same records with the small cells one LANE each: a wave takes 64 consecutive occupied
// cells, every lane the box of its own cell when it holds at most kCbSmall points (its points
// loaded together, branch-free), then the wave's other cells four at a time at kCbLanes lanes
// each.  Clutter singletons (most of the occupied cells at the standard density) no longer take
// a 16-lane group each.
constexpr int kCbSmall = 4;
template <int D>
__device__ __forceinline__ void cell_box_store(int c, int b, int e, float x0, float x1, float y0,
                                               float y1, float z0, float z1, float t0, float t1,
                                               uint64_t mn, bool has_mn, const Geom& g,
                                               uint8_t* __restrict__ mutual,
                                               CellRec<D>* __restrict__ crec,
                                               unsigned long long* __restrict__ cmin) {
  CellRec<D> r{};
  r.b = b;
  r.e = e;
  r.x0 = x0;
  r.x1 = x1;
  r.y0 = y0;
  r.y1 = y1;
  if constexpr (D == 3) {
    r.z0 = z0;
    r.z1 = z1;
  }
  r.t0 = t0;
  r.t1 = t1;
  crec[c] = r;
  const double dx = (double)x1 - (double)x0;
  const double dy = (double)y1 - (double)y0;
  double d2 = dx * dx + dy * dy;
  if (D == 3) {
    const double dz = (double)z1 - (double)z0;
    d2 = d2 + dz * dz;
  }
  const float dt = t1 - t0;
  mutual[c] = (d2 <= g.eps2 && dt <= g.epst) ? 1 : 0;
  if (cmin) cmin[c] = has_mn ? mn : ~0ull;  // the core pass's per-cell minima
}

template <int D>
__global__ __launch_bounds__(kBlock) void k_cell_box_mixed(const float4* __restrict__ pts,
                                                          const int32_t* __restrict__ cell_start,
                                                          const int32_t* __restrict__ occ,
                                                          const int32_t* __restrict__ n_occ,
                                                          Geom g, uint8_t* __restrict__ mutual,
                                                          CellRec<D>* __restrict__ crec,
                                                          unsigned long long* __restrict__ cmin =
                                                              nullptr,
                                                          const int32_t* __restrict__ sorig =
                                                              nullptr) {
  constexpr int L = kCbLanes;
  const int lane = threadIdx.x & 63;
  const int grp = lane / L, j = lane & (L - 1);
  const int64_t no = *n_occ;
  if (no == 0) return;
  const int64_t wpb = kBlock / 64;
  for (int64_t q0 = ((int64_t)blockIdx.x * wpb + threadIdx.x / 64) * 64; q0 < no;
       q0 += (int64_t)gridDim.x * wpb * 64) {
    const int64_t q = q0 + lane;
    const bool act = q < no;
    const int c = occ[act ? q : no - 1];
    const int b = cell_start[c], e = cell_start[c + 1];
    const bool small = act && e - b <= kCbSmall;
    {  // this lane's cell when small (every lane loads: branch-free)
      float4 pp[kCbSmall];
      uint32_t so[kCbSmall];
#pragma unroll
      for (int u = 0; u < kCbSmall; ++u) {
        const int sc = (b + u < e) ? b + u : b;  // duplicates of a cell point leave the box as is
        pp[u] = pts[sc];
        if (sorig) so[u] = (uint32_t)sorig[sc];
      }
      float x0 = FLT_MAX, x1 = -FLT_MAX, y0 = FLT_MAX, y1 = -FLT_MAX;
      float z0 = FLT_MAX, z1 = -FLT_MAX, t0 = FLT_MAX, t1 = -FLT_MAX;
      uint64_t mn = ~0ull;
#pragma unroll
      for (int u = 0; u < kCbSmall; ++u) {
        const float4 p = pp[u];
        x0 = fminf(x0, p.x); x1 = fmaxf(x1, p.x);
        y0 = fminf(y0, p.y); y1 = fmaxf(y1, p.y);
        z0 = fminf(z0, p.z); z1 = fmaxf(z1, p.z);
        t0 = fminf(t0, p.w); t1 = fmaxf(t1, p.w);
        if (sorig) {
          const uint64_t v = ((uint64_t)so[u] << 32) | (uint32_t)((b + u < e) ? b + u : b);
          mn = v < mn ? v : mn;
        }
      }
      if (D != 3) {
        z0 = t0;  // 2-D: pts[].z carries t
        z1 = t1;
      }
      if (small)
        cell_box_store<D>(c, b, e, x0, x1, y0, y1, z0, z1, t0, t1, mn, sorig != nullptr, g,
                          mutual, crec, cmin);
    }
    // the wave's other cells, four at a time (group grp takes the grp-th of them)
    uint64_t big = __ballot(act && !small);
    while (big) {  // (wave-uniform)
      int pick = -1;
#pragma unroll
      for (int k = 0; k < 64 / L; ++k) {
        const int lk = big ? __ffsll((unsigned long long)big) - 1 : -1;
        if (grp == k) pick = lk;
        if (big) big &= big - 1;
      }
      // (every lane takes part in the shuffles: a conditional one would read inactive lanes)
      const int src = pick < 0 ? 0 : pick;
      const int cc = __shfl(c, src), bb = __shfl(b, src), es = __shfl(e, src);
      const int ee = pick < 0 ? bb : es;
      float x0 = FLT_MAX, x1 = -FLT_MAX, y0 = FLT_MAX, y1 = -FLT_MAX;
      float z0 = FLT_MAX, z1 = -FLT_MAX, t0 = FLT_MAX, t1 = -FLT_MAX;
      uint64_t mn = ~0ull;
      constexpr int kU = 8;  // loads in flight per lane (as k_cell_box)
      for (int s0 = bb + j; s0 < ee; s0 += L * kU) {
        float4 pp[kU];
        uint32_t so[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const int s2 = s0 + L * u;
          const int sc = (s2 < ee) ? s2 : s0;
          pp[u] = pts[sc];
          if (sorig) so[u] = (uint32_t)sorig[sc];
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
          const float4 p = pp[u];
          x0 = fminf(x0, p.x); x1 = fmaxf(x1, p.x);
          y0 = fminf(y0, p.y); y1 = fmaxf(y1, p.y);
          z0 = fminf(z0, p.z); z1 = fmaxf(z1, p.z);
          t0 = fminf(t0, p.w); t1 = fmaxf(t1, p.w);
          if (sorig) {
            const int s2 = s0 + L * u;
            const uint64_t v = ((uint64_t)so[u] << 32) | (uint32_t)((s2 < ee) ? s2 : s0);
            mn = v < mn ? v : mn;
          }
        }
      }
      if (sorig) mn = row_reduce<L>(mn, OpMin{});
      x0 = row_reduce<L>(x0, OpMin{}); x1 = row_reduce<L>(x1, OpMax{});
      y0 = row_reduce<L>(y0, OpMin{}); y1 = row_reduce<L>(y1, OpMax{});
      z0 = row_reduce<L>(z0, OpMin{}); z1 = row_reduce<L>(z1, OpMax{});
      t0 = row_reduce<L>(t0, OpMin{}); t1 = row_reduce<L>(t1, OpMax{});
      if (D != 3) {
        z0 = t0;
        z1 = t1;
      }
      if (pick >= 0 && j == 0)
        cell_box_store<D>(cc, bb, ee, x0, x1, y0, y1, z0, z1, t0, t1, mn, sorig != nullptr, g,
                          mutual, crec, cmin);
    }
  }
}

// Actual time range per slab from its occupied cells' records (slabs are the slowest key
// dimension: a slab's cells are a contiguous range of the ascending occupied-cell list, found
// through the head-flag scan at the slab's first point).  One block per slab.
template <int D>
__global__ __launch_bounds__(kBlock) void k_slab_range(const CellRec<D>* __restrict__ crec,
                                                      const int32_t* __restrict__ occ,
                                                      const int32_t* __restrict__ hpos,
                                                      const int32_t* __restrict__ cell_start,
                                                      int64_t cells_per_slab, int nt,
                                                      float2* __restrict__ slab_t,
                                                      const int32_t* __restrict__ occ_base) {
  const int s = blockIdx.x;
  if (s >= nt) return;
  const int q0 = occ_base ? occ_base[s] : hpos[cell_start[(int64_t)s * cells_per_slab]];
  const int q1 = occ_base ? occ_base[s + 1] : hpos[cell_start[(int64_t)(s + 1) * cells_per_slab]];
  float lo = FLT_MAX, hi = -FLT_MAX;
  for (int q = q0 + threadIdx.x; q < q1; q += blockDim.x) {
    const CellRec<D> r = crec[occ[q]];
    lo = fminf(lo, r.t0);
    hi = fmaxf(hi, r.t1);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    lo = fminf(lo, __shfl_xor(lo, off));
    hi = fmaxf(hi, __shfl_xor(hi, off));
  }
  __shared__ float slo[kBlock / 64], shi[kBlock / 64];
  if ((threadIdx.x & 63) == 0) {
    slo[threadIdx.x / 64] = lo;
    shi[threadIdx.x / 64] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kBlock / 64; ++w) {
      lo = fminf(lo, slo[w]);
      hi = fmaxf(hi, shi[w]);
    }
    // empty slab: lo > hi, never matches
    slab_t[s] = make_float2(lo, hi);
  }
}

// ---------------------------------------------------------------- neighbour predicates

// Exact pair test (see file header): the float64 squared distance against eps^2.  A float32
// screen decides first (Geom::e2lo / e2hi, the classify_cells screen): the float32 distance is
// within a few 2^-24 of the float64 one (relative), far inside the 1e-5 margins, so only pairs
// within 1e-5 of eps reach the float64 test -- the float64 ops (half rate, plus conversions) were
// most of the VALU of the pair-testing kernels.
template <int D>
__device__ __forceinline__ bool adjacent(const float4& a, const float4& b, const Geom& g) {
  const float dt = fabsf(a.w - b.w);
  const float fx = a.x - b.x, fy = a.y - b.y;
  float f2 = fx * fx + fy * fy;
  if (D == 3) {
    const float fz = a.z - b.z;
    f2 = f2 + fz * fz;
  }
  bool near = !(f2 <= g.e2lo) && !(f2 > g.e2hi);  // (NaN: near, the float64 test decides)
  bool in = f2 <= g.e2lo;
  if (near) {
    const double dx = (double)a.x - (double)b.x;
    const double dy = (double)a.y - (double)b.y;
    double d2 = dx * dx + dy * dy;
    if (D == 3) {
      const double dz = (double)a.z - (double)b.z;
      d2 = d2 + dz * dz;
    }
    in = d2 <= g.eps2;
  }
  return in && (dt <= g.epst);
}

// |p - [lo, hi]| lower bound and the farthest-end distance, float64, each rounded like the pair
// test (monotone), so classification never contradicts the pair test.
__device__ __forceinline__ void span_dist(float p, float lo, float hi, double& dmin,
                                          double& dmax) {
  const double dp = (double)p;
  dmin = (p < lo) ? ((double)lo - dp) : ((p > hi) ? (dp - (double)hi) : 0.0);
  dmax = fmax(fabs(dp - (double)lo), fabs(dp - (double)hi));
}

// 0: no point of the cell can be adjacent; 1: every point is adjacent; 2: test pairs.
template <int D>
__device__ __forceinline__ int classify(const float4& p, const float4& A, const float4& B,
                                        const Geom& g) {
  // time (float32, same rounding as the pair test)
  const float tlo = B.z, thi = B.w;
  const float tmin = (p.w < tlo) ? (tlo - p.w) : ((p.w > thi) ? (p.w - thi) : 0.f);
  if (!(tmin <= g.epst)) return 0;
  const float tmax = fmaxf(fabsf(p.w - tlo), fabsf(p.w - thi));
  {
    // float32 screen of the spatial bounds (as adjacent / classify_cells): float64 only when a
    // bound lies within 1e-5 of eps^2
    auto fgap = [](float v, float lo, float hi) { return fmaxf(fmaxf(lo - v, v - hi), 0.f); };
    auto fspan = [](float v, float lo, float hi) { return fmaxf(fabsf(v - lo), fabsf(v - hi)); };
    const float gx = fgap(p.x, A.x, A.y), gy = fgap(p.y, A.z, A.w);
    const float sx = fspan(p.x, A.x, A.y), sy = fspan(p.y, A.z, A.w);
    float fmn = gx * gx + gy * gy, fmx = sx * sx + sy * sy;
    if (D == 3) {
      const float gz = fgap(p.z, B.x, B.y), sz = fspan(p.z, B.x, B.y);
      fmn = fmn + gz * gz;
      fmx = fmx + sz * sz;
    }
    if (fmn > g.e2hi) return 0;
    if (fmx <= g.e2lo) return (tmax <= g.epst) ? 1 : 2;
    if (fmn <= g.e2lo && fmx > g.e2hi) return 2;
  }
  double mnx, mxx, mny, mxy;
  span_dist(p.x, A.x, A.y, mnx, mxx);
  span_dist(p.y, A.z, A.w, mny, mxy);
  double dmin = mnx * mnx + mny * mny;
  double dmax = mxx * mxx + mxy * mxy;
  if (D == 3) {
    double mnz, mxz;
    span_dist(p.z, B.x, B.y, mnz, mxz);
    dmin = dmin + mnz * mnz;
    dmax = dmax + mxz * mxz;
  }
  if (!(dmin <= g.eps2)) return 0;
  return (dmax <= g.eps2 && tmax <= g.epst) ? 1 : 2;
}

// Candidate-cell enumeration shared by the three scan kernels.  Calls f(cell, begin, end, cls)
// for every non-empty cell that may hold a neighbour of point p (own cell included); f returns
// true to stop the enumeration.
template <int D, class F>
__device__ __forceinline__ void for_each_cell(const float4& p, int32_t key, const Geom& g,
                                              const int32_t* __restrict__ cell_start,
                                              const CellRec<D>* __restrict__ crec,
                                              const float2* __restrict__ slab_t, F&& f) {
  int cx, cy, cz, cs;
  g.split((uint32_t)key, cx, cy, cz, cs);
  // conservative slab window (+-1 slack), culled by each slab's actual time range
  const double tp = (double)p.w, et = (double)g.epst;
  int s0 = (int)fmax(floor((tp - et - g.ot) * g.inv_ct) - 1.0, 0.0);
  int s1 = (int)fmin(floor((tp + et - g.ot) * g.inv_ct) + 1.0, (double)(g.nt - 1));
  const int x0 = max(cx - 2, 0), x1 = min(cx + 2, g.nx - 1);
  const int y0 = max(cy - 2, 0), y1 = min(cy + 2, g.ny - 1);
  const int z0 = (D == 3) ? max(cz - 2, 0) : 0, z1 = (D == 3) ? min(cz + 2, g.nz - 1) : 0;
  (void)cs;
  for (int s = s0; s <= s1; ++s) {
    const float2 sr = slab_t[s];
    if (sr.x > sr.y) continue;  // empty slab
    const float smin = (p.w < sr.x) ? (sr.x - p.w) : ((p.w > sr.y) ? (p.w - sr.y) : 0.f);
    if (!(smin <= g.epst)) continue;
    for (int zz = z0; zz <= z1; ++zz) {
      for (int yy = y0; yy <= y1; ++yy) {
        const int64_t row = (((int64_t)s * g.nz + zz) * g.ny + yy) * g.nx;
        int b = cell_start[row + x0];
        for (int xx = x0; xx <= x1; ++xx) {
          const int e = cell_start[row + xx + 1];
          if (e > b) {
            const int64_t c = row + xx;
            const CellRec<D> cr = crec[c];
            const int cls = classify<D>(p, rec_boxA<D>(cr), rec_boxB(cr), g);
            if (cls != 0 && f(c, b, e, cls)) return;
          }
          b = e;
        }
      }
    }
  }
}

__device__ __forceinline__ int32_t rep_id(const int64_t* __restrict__ reps, int64_t nr, int64_t v) {
  int64_t lo = 0, hi = nr;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (reps[m] < v) lo = m + 1; else hi = m;
  }
  return (lo < nr && reps[lo] == v) ? (int32_t)lo : -2;  // -2: representative missing (bug)
}

// ---------------------------------------------------------------- block-aggregated append
// Every thread of the block evaluates pred(s) for kItems sorted indices of one 256*kItems tile;
// the indices with pred true are appended to list with ONE global atomic per tile (thousands of
// same-address atomics per launch otherwise serialise in L2).  Order inside a tile is
// thread-major; consumers do not depend on the order.
constexpr int kItems = 16;
struct AppendIndex {
  __device__ int32_t operator()(int64_t s) const { return (int32_t)s; }
};
// Same, with this thread's predicate bits already known (bit k <-> index tile0 + k*kBlock + tid).
template <class V = AppendIndex>
__device__ __forceinline__ void block_append_bits(int64_t tile0, uint32_t bits,
                                                  int32_t* __restrict__ list,
                                                  int32_t* __restrict__ counter, V value = V{});

template <class P, class V = AppendIndex>
__device__ __forceinline__ void block_append(int64_t tile0, int64_t n, P&& pred,
                                             int32_t* __restrict__ list,
                                             int32_t* __restrict__ counter, V value = V{}) {
  uint32_t bits = 0;
#pragma unroll
  for (int k = 0; k < kItems; ++k) {
    const int64_t s = tile0 + (int64_t)k * kBlock + threadIdx.x;
    if (s < n && pred(s)) bits |= 1u << k;
  }
  block_append_bits(tile0, bits, list, counter, value);
}

template <class V>
__device__ __forceinline__ void block_append_bits(int64_t tile0, uint32_t bits,
                                                  int32_t* __restrict__ list,
                                                  int32_t* __restrict__ counter, V value) {
  __shared__ int s_wsum[kBlock / 64];
  __shared__ int s_base;
  const int c = __popc(bits);
  // block exclusive scan of c
  const int lane = threadIdx.x & 63, w = threadIdx.x / 64;
  int incl = c;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(incl, off, 64);
    if (lane >= off) incl += o;
  }
  if (lane == 63) s_wsum[w] = incl;
  __syncthreads();
  int before = 0, total = 0;
#pragma unroll
  for (int v = 0; v < kBlock / 64; ++v) {
    const int t = s_wsum[v];
    before += (v < w) ? t : 0;
    total += t;
  }
  if (threadIdx.x == 0) s_base = total ? atomicAdd(counter, total) : 0;
  __syncthreads();
  int o = s_base + before + incl - c;
  while (bits) {
    const int k = __ffs(bits) - 1;
    bits &= bits - 1;
    list[o++] = value(tile0 + (int64_t)k * kBlock + threadIdx.x);
  }
  __syncthreads();  // s_wsum / s_base reuse by the next tile
}

// ---------------------------------------------------------------- candidate windows
// The cells that may hold a neighbour: +-2 cells in space (fixed 5-wide extents so candidate
// decoding divides by constants; out-of-grid candidates are skipped) over the slabs whose actual
// time range comes within eps_t of [tlo, thi] (the +-1-slab slack window is shrunk up front with
// the per-slab time ranges).
struct Window {
  int s0, x0, y0, z0;
  int nS;
  int total;
};

__device__ __forceinline__ bool slab_in_reach(const float2* __restrict__ slab_t, int s, float tlo,
                                              float thi, float epst) {
  const float2 sr = slab_t[s];
  if (sr.x > sr.y) return false;  // empty slab
  const float gap = (tlo > sr.y) ? (tlo - sr.y) : ((thi < sr.x) ? (sr.x - thi) : 0.f);
  return gap <= epst;
}

template <int D, bool SHRINK = true>
__device__ __forceinline__ Window make_window(int cx, int cy, int cz, float tlo, float thi,
                                              const Geom& g, const float2* __restrict__ slab_t,
                                              int s_min = 0) {
  constexpr int PER = (D == 3) ? 125 : 25;
  Window w;
  const double et = (double)g.epst;
  int s0, s1;
  if (g.rt >= 0) {  // integral times: the slabs of tlo / thi (exact) +- rt
    s0 = max(slab_of(tlo, g) - g.rt, s_min);
    s1 = min(slab_of(thi, g) + g.rt, g.nt - 1);
  } else {
    s0 = (int)fmax(floor(((double)tlo - et - g.ot) * g.inv_ct) - 1.0, (double)s_min);
    s1 = (int)fmin(floor(((double)thi + et - g.ot) * g.inv_ct) + 1.0, (double)(g.nt - 1));
  }
  // shrink to the slabs in reach: one lane per slab (independent loads), ballot (callers are
  // whole waves with uniform arguments)
  const int lane = threadIdx.x & 63;
  int lo = -1, hi = -1;
  if (!SHRINK) {  // callers that classify every candidate's time range themselves
    lo = s0;
    hi = s1;
  }
  for (int c = s0; SHRINK && c <= s1; c += 64) {
    const bool ok = (c + lane <= s1) && slab_in_reach(slab_t, c + lane, tlo, thi, g.epst);
    const uint64_t m = __ballot(ok);
    if (m) {
      if (lo < 0) lo = c + __ffsll((unsigned long long)m) - 1;
      hi = c + 63 - __clzll((long long)m);
    }
  }
  if (lo < 0) {
    s0 = 0;
    s1 = -1;
  } else {
    s0 = lo;
    s1 = hi;
  }
  w.s0 = s0;
  w.nS = max(s1 - s0 + 1, 0);
  w.x0 = cx - 2;
  w.y0 = cy - 2;
  w.z0 = (D == 3) ? cz - 2 : 0;
  w.total = w.nS * PER;
  return w;
}

template <int D>
__device__ __forceinline__ void decode_key(int64_t key, const Geom& g, int& cx, int& cy, int& cz) {
  // keys of real cells are < 2^30 (cmax): 32-bit divisions, not the 64-bit ones' call sequence
  int cs;
  g.split((uint32_t)key, cx, cy, cz, cs);
  if (D != 3) cz = 0;
}

// q-th cell of the window; -1 when outside the grid or its slab holds nothing within reach
template <int D>
__device__ __forceinline__ int64_t window_cell(const Window& w, int q, const Geom& g,
                                               const float2* __restrict__ slab_t, float tlo,
                                               float thi) {
  constexpr int PER = (D == 3) ? 125 : 25;
  const int ss = q / PER;
  int r = q - ss * PER;
  int zz = 0;
  if (D == 3) {
    zz = r / 25;
    r -= zz * 25;
  }
  const int yy = r / 5, xx = r - yy * 5;
  const int x = w.x0 + xx, y = w.y0 + yy, z = w.z0 + zz;
  if (x < 0 || x >= g.nx || y < 0 || y >= g.ny || (D == 3 && (z < 0 || z >= g.nz))) return -1;
  // slabs between the first and last in reach are in reach unless empty (then so are their
  // cells); the cell box's own time range is checked by classify
  const int sl = w.s0 + ss;
  return (((int64_t)sl * g.nz + z) * g.ny + y) * g.nx + x;
}

__device__ __forceinline__ float4 shfl_f4(const float4& v, int l) {
  return make_float4(__shfl(v.x, l), __shfl(v.y, l), __shfl(v.z, l), __shfl(v.w, l));
}

// Box-box classification of two cells with the pair test's rounding (monotone bounds):
// 0 no pair can be adjacent, 1 every pair is adjacent, 2 undecided.
// SCREEN: float32 bounds first, float64 only near the threshold (Geom::e2lo / e2hi) -- faster
// in the K5 cell pass; the union kernels measured slower with it (their loops schedule worse).
template <int D, bool SCREEN = false>
__device__ __forceinline__ int classify_cells(const float4& A1, const float4& B1,
                                              const float4& A2, const float4& B2,
                                              const Geom& g) {
  // interval gap: max(b0 - a1, a0 - b1, 0) (one v_max3; equal to the branchy form, since a
  // float32 difference has the sign of the exact one)
  auto gap = [](float a0, float a1, float b0, float b1) -> float {
    return fmaxf(fmaxf(b0 - a1, a0 - b1), 0.f);
  };
  auto gapd = [](float a0, float a1, float b0, float b1) -> double {
    return (b0 > a1) ? ((double)b0 - (double)a1) : ((a0 > b1) ? ((double)a0 - (double)b1) : 0.0);
  };
  float tm = 0.f;  // (tfree: every pair of the window is within eps_t)
  if (!g.tfree) {  // kernel-uniform
    const float tg = gap(A2.z, A2.w, B2.z, B2.w);
    if (!(tg <= g.epst)) return 0;
    tm = fmaxf(fabsf(B2.w - A2.z), fabsf(A2.w - B2.z));
  }
  if (D == 2 && SCREEN) {
    const float fx = gap(A1.x, A1.y, B1.x, B1.y), fy = gap(A1.z, A1.w, B1.z, B1.w);
    const float fmn = fx * fx + fy * fy;
    const float ux = fmaxf(fabsf(B1.y - A1.x), fabsf(A1.y - B1.x));
    const float uy = fmaxf(fabsf(B1.w - A1.z), fabsf(A1.w - B1.z));
    const float fmx = ux * ux + uy * uy;
    if (fmn > g.e2hi) return 0;
    if (fmx <= g.e2lo) return (tm <= g.epst) ? 1 : 2;
    if (fmn <= g.e2lo && fmx > g.e2hi) return 2;
  }
  const double gx = gapd(A1.x, A1.y, B1.x, B1.y), gy = gapd(A1.z, A1.w, B1.z, B1.w);
  double dmin = gx * gx + gy * gy;
  const double mx = fmax(fabs((double)B1.y - (double)A1.x), fabs((double)A1.y - (double)B1.x));
  const double my = fmax(fabs((double)B1.w - (double)A1.z), fabs((double)A1.w - (double)B1.z));
  double dmax = mx * mx + my * my;
  if (D == 3) {
    const double gz = gapd(A2.x, A2.y, B2.x, B2.y);
    dmin = dmin + gz * gz;
    const double mz = fmax(fabs((double)B2.y - (double)A2.x), fabs((double)A2.y - (double)B2.x));
    dmax = dmax + mz * mz;
  }
  if (!(dmin <= g.eps2)) return 0;
  return (dmax <= g.eps2 && tm <= g.epst) ? 1 : 2;
}

// Tuning flags of the union kernels (RPT_UF_FLAGS in the A/B build): bit 0 = finds inside the
// union kernels do not path-halve (agent-scope stores drop the line from the XCD's L2; k_compress
// compresses afterwards); bit 1 = XCD-aware item ranges (blockIdx % 8 = XCD under round-robin
// placement: each XCD unions a contiguous range of cells, so its L2 keeps their parents).
// XcdRange is also the item split of the K5 / K7 queue kernels.
struct XcdRange {
  int64_t first, step, end;
};
__device__ __forceinline__ XcdRange xcd_items(int64_t n_items, bool remap) {
  const int64_t wpb = kBlock / 64, wave = threadIdx.x / 64;
  if (!remap || (gridDim.x & 7)) {
    return XcdRange{(int64_t)blockIdx.x * wpb + wave, (int64_t)gridDim.x * wpb, n_items};
  }
  const int64_t x = blockIdx.x & 7, lb = blockIdx.x >> 3, nbx = gridDim.x >> 3;
  const int64_t lo = n_items * x / 8, hi = n_items * (x + 1) / 8;
  return XcdRange{lo + lb * wpb + wave, nbx * wpb, hi};
}

// ---------------------------------------------------------------- K5: core flags
constexpr int kR = 4;  // candidate cells per lane per super-round of the window scans
static_assert(kR >= 2, "the union passes' candidate masks cover two 64-position rounds");
// k_union_cells: the top bit of a cell's candidate mask = "not recorded, enumerate the window"
constexpr uint32_t kPmaskFull = 0x80000000u;
// RPT_CELL_ROOTS=0: k_ccmin walks every core point's parent chain (A/B)
static bool cell_roots_enabled() {
  static const bool on = [] {
    const char* e = ab_env("RPT_CELL_ROOTS");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}

// Level 1, one thread per occupied cell: a mutual cell (every pair adjacent) holding >=
// min_samples points is all core — the bulk of a radar stack.  Every other cell is queued for
// level 2 (the queue holds cell keys).  cflag (int32 per cell): 1 all core, 0 none, 2 decided
// per point (level 4).
__global__ __launch_bounds__(kBlock) void k_core_cell_fast(const int32_t* __restrict__ occ,
                                                          const int32_t* __restrict__ n_occ,
                                                          Geom g,
                                                          const int32_t* __restrict__ cell_start,
                                                          const uint8_t* __restrict__ mutual,
                                                          int32_t* __restrict__ cflag,
                                                          int32_t* __restrict__ queue,
                                                          int32_t* __restrict__ n_queue) {
  const int need = g.min_samples;
  const int64_t no = *n_occ;
  for (int64_t tile = (int64_t)blockIdx.x * kBlock * kItems; tile < no;
       tile += (int64_t)gridDim.x * kBlock * kItems) {
    block_append(
        tile, no,
        [&](int64_t q) -> bool {
          const int32_t c = occ[q];
          if ((int64_t)c >= g.cells || need <= 0) {  // non-finite time: no neighbours at all
            cflag[c] = (need <= 0) ? 1 : 0;
            return false;
          }
          if (mutual[c] && cell_start[c + 1] - cell_start[c] >= need) {
            cflag[c] = 1;
            return false;
          }
          return true;
        },
        queue, n_queue, [&](int64_t q) -> int32_t { return occ[q]; });
  }
}

// Level 2, one wave per queued cell A: lanes classify A's candidate cells against A's box
// (classify_cells: the pair test's rounding, monotone bounds).  Cells adjacent to every point of
// A give a count shared by all of A's points (a lower bound, self included); cells that may hold
// a neighbour give an upper bound.  Most sparse cells are decided here (flag 1 or 0) without
// touching a point; the rest get flag 2.
template <int D>
__global__ __launch_bounds__(kBlock) void k_core_cell_window(Geom g,
                                                            const int32_t* __restrict__ occ,
                                                            const CellRec<D>* __restrict__ crec,
                                                            const uint32_t* __restrict__ occ_bits,
                                                            const float2* __restrict__ slab_t,
                                                            const int32_t* __restrict__ queue,
                                                            const int32_t* __restrict__ n_queue,
                                                            int32_t* __restrict__ cflag) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (int64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
  const int64_t nw = (int64_t)gridDim.x * (kBlock / 64);
  const int64_t nq = *n_queue;
  const int need = g.min_samples;
  for (int64_t q = w0; q < nq; q += nw) {
    const int32_t ca = queue[q];
    const CellRec<D> ra = crec[ca];
    const float4 A1 = rec_boxA<D>(ra), A2 = rec_boxB(ra);
    int cx, cy, cz;
    decode_key<D>(ca, g, cx, cy, cz);
    const Window w = make_window<D, true>(cx, cy, cz, A2.z, A2.w, g, slab_t);
    int lo = 0, hi = 0;
    for (int base = 0; base < w.total && lo < need; base += 64 * kR) {
      int64_t c[kR];
      uint32_t wb[kR];
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        const int qq = base + r * 64 + lane;
        c[r] = (qq < w.total) ? window_cell<D>(w, qq, g, slab_t, A2.z, A2.w) : -1;
      }
#pragma unroll
      for (int r = 0; r < kR; ++r) wb[r] = (c[r] >= 0) ? occ_bits[c[r] >> 5] : 0u;
      int l = 0, h = 0;
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        if (c[r] >= 0 && ((wb[r] >> (c[r] & 31)) & 1u)) {
          const CellRec<D> cr = crec[c[r]];
          const int cls = classify_cells<D>(A1, rec_boxA<D>(cr), A2, rec_boxB(cr), g);
          l += (cls == 1) ? cr.e - cr.b : 0;
          h += (cls != 0) ? cr.e - cr.b : 0;
        }
      }
      lo += wave_sum(l);
      hi += wave_sum(h);
    }
    // an early exit leaves hi partial, but lo >= need already decides
    if (lane == 0) cflag[ca] = (lo >= need) ? 1 : ((hi < need) ? 0 : 2);
  }
}

// core flags v of the points [b, e) of one cell, by `lanes` lanes (j = this lane's index): bytes at
// the unaligned ends, dwords inside (cells list their points contiguously in sorted order)
__device__ __forceinline__ void write_cell_flags(uint8_t* __restrict__ core, int b, int e, int j,
                                                 int lanes, uint8_t v) {
  const int wb = (b + 3) & ~3, we = e & ~3;
  if (wb >= we) {
    for (int s = b + j; s < e; s += lanes) core[s] = v;
    return;
  }
  for (int s = b + j; s < wb; s += lanes) core[s] = v;
  const uint32_t vv = v ? 0x01010101u : 0u;
  for (int w = wb + 4 * j; w < we; w += 4 * lanes) *reinterpret_cast<uint32_t*>(core + w) = vv;
  for (int s = we + j; s < e; s += lanes) core[s] = v;
}

// Row of mask position k (0..4, own row first: dy = 0, -1, +1, -2, +2) as dy + 2, branch-free
// (3-bit fields of one constant): 2, 1, 3, 0, 4.
__device__ __forceinline__ int cw_row(int k) {
  return (int)__builtin_amdgcn_ubfe(16586u, (uint32_t)(3 * k), 3u);
}

// The FUSED epilogue of k_core_cells_oct (whole wave, wave-uniform control): lanes 8k hold cell k
// of the wave (act, key, point range [b, e), flag 0 / 1 / 2).  The cells' (min original, sorted)
// pairs over ALL their points come from k_cell_box (allmin): an all-core cell keeps it, every other
// cell is reset to none here (the undecided cells' core points are folded in by k_core_slow).
// The queued points go to the block's LDS queue (an LDS atomic per wave; one global atomic per
// BLOCK when the block flushes it at its end -- a global same-address atomic per wave serialised
// ~100 k of them at 1000 frames: +0.8 ms); a wave whose points no longer fit reserves globally.
constexpr int kCwQueue = 2048;
struct CwQueue {
  int32_t item[kCwQueue];
  int32_t key[kCwQueue];  // the queued point's cell key (k_core_slow skips its skey read)
  int n;      // reserved (may pass kCwQueue)
  int fail;   // first reservation that did not fit
  int base;
};
__device__ __forceinline__ void cells_fill_epilogue(const Geom& g, bool act, int32_t ca,
                                                    int32_t qk, int b, int e, int flag,
                                                    uint8_t* __restrict__ core,
                                                    unsigned long long* __restrict__ cmin,
                                                    int32_t* __restrict__ slow,
                                                    int32_t* __restrict__ slowk,
                                                    int32_t* __restrict__ n_slow, CwQueue& lq) {
  const int lane = threadIdx.x & 63;
  if (act && (lane & 7) == 0 && flag != 1 && (int64_t)ca < g.cells) cmin[ca] = ~0ull;
  // active cells are a prefix of the eight (occupied-list positions below the range end)
  const int na = __popcll(__ballot(act && (lane & 7) == 0));
  if (na == 0) return;
  int gb[8], gf[8], gc[8];
  int E = 0, nu = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    gb[k] = __builtin_amdgcn_readlane(b, 8 * k);
    gc[k] = __builtin_amdgcn_readlane(qk, 8 * k);  // the queue's per-point cell word
    const int ek = __builtin_amdgcn_readlane(e, 8 * k);
    gf[k] = __builtin_amdgcn_readlane(flag, 8 * k);
    if (k < na) {
      E = ek;
      nu += (gf[k] == 2) ? ek - gb[k] : 0;
    }
  }
  const int B = gb[0];
  int ub = 0;
  int32_t* qdst = lq.item;
  int32_t* kdst = lq.key;
  if (nu > 0) {  // the undecided cells' points: one queue reservation per wave
    if (lane == 0) {
      ub = atomicAdd(&lq.n, nu);
      if (ub + nu > kCwQueue) {
        atomicMin(&lq.fail, ub);
        ub = -1 - atomicAdd(n_slow, nu);
      }
    }
    ub = __shfl(ub, 0);
    if (ub < 0) {
      qdst = slow;
      kdst = slowk;
      ub = -1 - ub;
    }
  }
  const uint64_t below = (1ull << lane) - 1ull;
  for (int s0 = B; s0 < E; s0 += 64) {
    const int s = s0 + lane;
    const bool in = s < E;
    int fl = gf[0], c = gc[0];
#pragma unroll
    for (int k = 1; k < 8; ++k) {
      const bool sel = k < na && s >= gb[k];
      fl = sel ? gf[k] : fl;
      c = sel ? gc[k] : c;
    }
    const bool u = in && fl == 2;
    const uint64_t um = nu > 0 ? __ballot(u) : 0ull;
    if (u) {
      const int o = ub + __popcll(um & below);
      qdst[o] = s;
      kdst[o] = c;
    }
    ub += __popcll(um);
    if (in) core[s] = (fl == 1) ? 1 : 0;
  }
}

// 2-D grids whose slab window is at most 7 slabs (R <= 3): K5 levels 1-3 in one kernel, EIGHT
// lanes per occupied cell.  A mutual cell with >= min_samples points is all core (the bulk);
// otherwise lane j < 2R+1 owns slab cs - R + j of the cell's window.  The window comes from the
// cell's slab alone (R = ceil(eps_t / slab) + 1 slabs each side, pruned with the slabs' actual
// time ranges), so a lane loads its slab's range and the occupancy words of its 5 rows together
// with the cell's record, then the records of its (few) occupied candidates; eight cells per wave
// keep many short dependency chains in flight.  cflag as k_core_cell_fast / _window (level 3
// turns it into point flags).
//
// FUSED (the default pipeline): the level-3 fill folded in.  A wave's eight cells are consecutive
// occupied cells, so their points are ONE contiguous range of the sorted order (the cells between
// consecutive occupied keys are empty); after the decisions the whole wave walks that range 64
// points at a time: the point flags (byte stores, 64 consecutive bytes per instruction) and the
// undecided cells' points appended to the level-4 queue (one atomic per wave).  The all-core
// cells' (min original, sorted) pairs are k_cell_box's (allmin).  No per-point loads at all.
// Sum over each aligned group of eight lanes, every lane of the group getting it (row_reduce:
// DPP, no LDS round trips).  Every lane of a group must be active (the cell kernels' branches
// are group-uniform).
__device__ __forceinline__ int sum8(int v) { return row_reduce<8>(v, OpAdd{}); }

constexpr int kCwMaxR = 3;
constexpr int kCwBatch = 4;  // candidate records per lane in flight together (k_core_cells_oct)
// MASK (with FUSED, windows of W = 2R + 1 <= 5 slabs): every undecided cell hands its decisions
// to k_core_slow_masked -- its whole-accept count lo (clo[q], q = its occupied-list position) and
// the 128-bit mask of its candidates that box classification left partial (pmask[q]; window
// position 5 P + dx, P = the (slab, row) pair j + 8 i of lane j's slot i) -- and queues its points
// with q instead of the cell key.
template <bool FUSED = false, bool MASK = false>
// 5 waves/SIMD (<= 96 VGPRs; the fused epilogue and its LDS queue would take 99: 4 waves)
__global__ __launch_bounds__(kBlock, 5) void k_core_cells_oct(Geom g, int R,
                                                          const int32_t* __restrict__ occ,
                                                          const int32_t* __restrict__ n_occ,
                                                          const CellRec<2>* __restrict__ crec,
                                                          const uint8_t* __restrict__ mutual,
                                                          const uint32_t* __restrict__ occ_bits,
                                                          const float2* __restrict__ slab_t,
                                                          int32_t* __restrict__ cflag,
                                                          int32_t* __restrict__ zero_counter,
                                                          uint8_t* __restrict__ core,
                                                          unsigned long long* __restrict__ cmin =
                                                              nullptr,
                                                          int32_t* __restrict__ slow = nullptr,
                                                          int32_t* __restrict__ slowk = nullptr,
                                                          int32_t* __restrict__ n_slow = nullptr,
                                                          uint4* __restrict__ pmask = nullptr,
                                                          int32_t* __restrict__ clo = nullptr) {
  static_assert(!MASK || FUSED, "the masks feed the fused pipeline's slow pass");
  // legacy pipeline: the level-4 queue counter, zeroed here instead of by a memset launch
  // (k_core_fill, the next kernel on the stream, is its first user)
  if (!FUSED && zero_counter && blockIdx.x == 0 && threadIdx.x == 0) *zero_counter = 0;
  __shared__ CwQueue lq;
  // per lane its five (slab, row) slots' keys of column dx = 0, written once per cell and read
  // per candidate (recomputing them took ~20 VALU per candidate, three 32-bit multiplies among
  // them; five more registers spilled)
  __shared__ int32_t s_k0[5][kBlock];
  if (FUSED) {
    if (threadIdx.x == 0) {
      lq.n = 0;
      lq.fail = kCwQueue;
    }
    __syncthreads();
  }
  const int64_t no = *n_occ;
  const int need = g.min_samples;
  const int j = threadIdx.x & 7;
  // XCD-aware cell ranges (grid a multiple of 8): blocks sharing an XCD take one contiguous
  // eighth of the (slab-major) occupied cells, so the neighbouring slabs' records they read stay
  // in that XCD's L2 instead of being fetched by all eight
  const int64_t cpb = blockDim.x / 8;
  const int64_t xg = blockIdx.x & 7, nbx = gridDim.x >> 3;
  const int64_t qlo = no * xg / 8, qhi = no * (xg + 1) / 8;
  for (int64_t q0 = qlo + (int64_t)(blockIdx.x >> 3) * cpb; q0 < qhi; q0 += nbx * cpb) {
    const int64_t q = q0 + threadIdx.x / 8;
    const bool act = q < qhi;
    const int32_t ca = act ? occ[q] : 0;
    int flag = 0, b = 0, e = 0;
    if (act && (int64_t)ca >= g.cells) {  // non-finite time: no neighbours at all
      flag = (need <= 0) ? 1 : 0;
      const CellRec<2> ri = crec[ca];
      b = ri.b;
      e = ri.e;
    } else if (act) {
      int cx, cy, cz, cs;
      g.split((uint32_t)ca, cx, cy, cz, cs);
      // window of W = 2R + 1 slabs; lane j < W tests the time reach of slab cs - R + j
      const int W = 2 * R + 1;
      const int sl = cs + j - R;
      const bool sv = j < W && sl >= 0 && sl < g.nt;
      const CellRec<2> ra = crec[ca];
      const uint8_t mu = mutual[ca];
      b = ra.b;
      e = ra.e;
      const float2 own = slab_t[cs];
      float2 sr = make_float2(1.f, 0.f);
      // The window's 5 W (slab, row) pairs are spread over ALL eight lanes of the cell: pair
      // p = k W + si (row rank k: dy = 0, -1, +1, -2, +2, own row first; slab index si) is slot
      // p / 8 of lane p % 8.  (A lane per slab left 8 - W lanes idle through the candidate loop
      // -- 3 of 8 at the usual W = 5 -- and the busiest slab set the loop's trip count.)
      uint32_t m5[5];  // slot i: occupied columns dx = 0..4 of its row (x = cx - 2 + dx)
      int psi[5];      // slot i: slab index
      const uint32_t mg = (65535u + (uint32_t)W) / (uint32_t)W;  // p / W = (p * mg) >> 16
      {
        // branch-free: an invalid slot reads a valid word and masks it off, so all eleven loads
        // of every lane are in flight together (a conditional load is a branch ending in a full
        // vmcnt wait)
        const int slc = sv ? sl : cs;
        const float2 srv = slab_t[slc];
        sr = sv ? srv : sr;
        const int lo_x = cx - 2 < 0 ? 2 - cx : 0;
        const int hi_x = cx + 2 - (g.nx - 1);
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          const int p = j + 8 * i;
          const int k = min((int)(((uint32_t)p * mg) >> 16), 4);
          const int si = p - k * W;
          const int s2 = cs + si - R;
          const int y = cy + cw_row(k) - 2;
          const bool v = p < 5 * W && s2 >= 0 && s2 < g.nt && y >= 0 && y < g.ny;
          // (int32 keys: cells < 2^30)
          const int k0 = ((v ? s2 : cs) * g.ny + (v ? y : cy)) * g.nx + (cx - 2);
          s_k0[i][threadIdx.x] = k0;  // column dx = 0 of slot i (the lane's own LDS words)
          const int kk = k0 < 0 ? 0 : k0;
          const int w = kk >> 5;
          const uint32_t lo_w = occ_bits[w], hi_w = occ_bits[w + 1];
          uint32_t m = (k0 < 0) ? ((lo_w << (-k0)) & 31u)
                                : (__builtin_amdgcn_alignbit(hi_w, lo_w, (uint32_t)(kk & 31)) & 31u);
          m &= ~((1u << lo_x) - 1u);
          if (hi_x > 0) m &= (31u >> hi_x);
          m5[i] = v ? m : 0u;
          psi[i] = v ? si : 0;
        }
      }
      const float gap =
          (own.x > sr.y) ? (own.x - sr.y) : ((sr.x > own.y) ? (sr.x - own.y) : 0.f);
      const bool reach = sv && sr.x <= sr.y && gap <= g.epst;  // slab j is in reach
      // the cell's reach bits (slab index -> bit), from its eight lanes (group-uniform branch)
      const uint32_t rbits =
          (uint32_t)(__ballot(reach) >> (threadIdx.x & 56)) & 0xffu;
      // the lane's occupied candidates as one 25-bit mask, slot-major (bits 5i .. 5i + 4 = slot
      // i's columns): rows nearest first
      uint32_t m25 = 0;
#pragma unroll
      for (int i = 0; i < 5; ++i) m25 |= (((rbits >> psi[i]) & 1u) ? m5[i] : 0u) << (5 * i);
      if (need <= 0 || (mu && e - b >= need)) {
        flag = 1;
      } else {
        int lo = 0, hi = 0;
        const float4 A1 = rec_boxA<2>(ra), A2 = rec_boxB(ra);
        // taken kCwBatch at a time with all their record loads in flight together: a sparse
        // cell's few candidates cost ONE round trip instead of one per row; the eight lanes stop
        // as soon as the adjacent-to-every-point count reaches min_samples (dense cells: after
        // the own row's batch)
        bool decided = false;
        uint32_t pm25 = 0;  // (MASK) the lane's candidates left partial, bits as m25's
        while (true) {
          int rem = m25 ? 1 : 0;
          rem = sum8(rem);
          if (rem == 0) break;  // (uniform over the cell's eight lanes)
          CellRec<2> cr[kCwBatch];
          bool has[kCwBatch];
          const uint32_t mb = m25;  // (MASK) the batch takes the lowest set bits of mb
#pragma unroll
          for (int i = 0; i < kCwBatch; ++i) {
            // branch-free record loads (a lane without a candidate re-reads its own cell's)
            has[i] = m25 != 0;
            const int p = __builtin_ctz(m25 | (1u << 31));
            m25 &= m25 - 1;
            const int sl5 = (p * 13) >> 6;  // slot p / 5 (p < 32)
            const int key = s_k0[sl5][threadIdx.x] + (p - 5 * sl5);
            cr[i] = crec[has[i] ? key : ca];
          }
          uint32_t pf = 0;  // (MASK) batch entries left partial
#pragma unroll
          for (int i = 0; i < kCwBatch; ++i) {
            if (!has[i]) continue;
            const int cls =
                classify_cells<2, true>(A1, rec_boxA<2>(cr[i]), A2, rec_boxB(cr[i]), g);
            lo += (cls == 1) ? cr[i].e - cr[i].b : 0;
            hi += (cls != 0) ? cr[i].e - cr[i].b : 0;
            if (MASK) pf |= (cls == 2) ? (1u << i) : 0u;
          }
          if (MASK) {
            uint32_t tk = mb & ~m25;  // entry i = the i-th lowest bit taken
#pragma unroll
            for (int i = 0; i < kCwBatch; ++i) {
              pm25 |= ((pf >> i) & 1u) ? (tk & (0u - tk)) : 0u;
              tk &= tk - 1;
            }
          }
          int ls = lo;
          ls = sum8(ls);
          if (ls >= need) {
            decided = true;
            break;
          }
        }
        if (decided) {
          flag = 1;
        } else {
          lo = sum8(lo);
          hi = sum8(hi);
          flag = (lo >= need) ? 1 : ((hi < need) ? 0 : 2);
          if (MASK && flag == 2) {  // (group-uniform) hand the decisions to the slow pass
            // slot i of lane j = pair P = j + 8 i; its five columns go to window positions
            // 5 P .. 5 P + 4 (P < 5 W <= 25: slot 4 and most of slot 3 are never valid)
            uint64_t mlo = 0, mhi = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const uint64_t ch = (pm25 >> (5 * i)) & 31u;
              const int pos = 5 * (j + 8 * i);
              if (pos < 64) {
                mlo |= ch << pos;
                if (pos > 59) mhi |= ch >> (64 - pos);
              } else if (pos < 128) {
                mhi |= ch << (pos - 64);
              }
            }
            mlo = row_reduce<8>(mlo, OpOr{});
            mhi = row_reduce<8>(mhi, OpOr{});
            if (j == 0) {
              pmask[q] = make_uint4((uint32_t)mlo, (uint32_t)(mlo >> 32), (uint32_t)mhi,
                                    (uint32_t)(mhi >> 32));
              clo[q] = lo;
            }
          }
        }
      }
    }
    if constexpr (!FUSED) {
      if (act && j == 0) cflag[ca] = flag;
      // decided cells write their points' flags here (the undecided ones are k_core_slow_cells')
      if (core && act && flag != 2) write_cell_flags(core, b, e, j, 8, (uint8_t)flag);
    } else {
      // (MASK: the queue carries the cell's occupied-list position instead of its key)
      cells_fill_epilogue(g, act, ca, MASK ? (int32_t)q : ca, b, e, flag, core, cmin, slow, slowk,
                          n_slow, lq);
    }
  }
  if constexpr (FUSED) {  // flush the block's queue (the cell loop is block-uniform)
    __syncthreads();
    const int m = min(lq.n, lq.fail);
    if (threadIdx.x == 0) lq.base = m > 0 ? atomicAdd(n_slow, m) : 0;
    __syncthreads();
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
      slow[lq.base + i] = lq.item[i];
      slowk[lq.base + i] = lq.key[i];
    }
  }
}

// Level 3, one thread per point: the cell's decision; points of undecided cells are queued for
// level 4 (block-aggregated append; QUEUE = false: the undecided cells are left to
// k_core_slow_cells).
// cmin (nullable, ~0 for the occupied cells): the union's per-cell (min original, sorted) pair
// of the core points (k_cell_min_pair folded in): all-core cells here, by a segmented wave
// minimum over the sorted points; the undecided cells' core points in k_core_slow.
template <bool QUEUE>
__global__ __launch_bounds__(kBlock) void k_core_fill(const int32_t* __restrict__ skey, int64_t n,
                                                     const int32_t* __restrict__ cflag,
                                                     uint8_t* __restrict__ core,
                                                     int32_t* __restrict__ slow,
                                                     int32_t* __restrict__ n_slow,
                                                     const int32_t* __restrict__ sorig = nullptr,
                                                     unsigned long long* __restrict__ cmin =
                                                         nullptr,
                                                     int64_t cells = 0) {
  const int lane = threadIdx.x & 63;
  for (int64_t tile = (int64_t)blockIdx.x * kBlock * kItems; tile < n;
       tile += (int64_t)gridDim.x * kBlock * kItems) {
    // all keys, then all cell flags, in flight together (two rounds of memory latency per tile,
    // not two per item)
    // branch-free (clamped indices, results masked): each level's loads in flight together
    int32_t key[kItems];
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int64_t s = tile + (int64_t)k * kBlock + threadIdx.x;
      const int32_t kv = skey[min(s, n - 1)];
      key[k] = (s < n) ? kv : -1;
    }
    int f[kItems];
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int32_t fv = cflag[key[k] >= 0 ? key[k] : 0];
      f[k] = (key[k] >= 0) ? fv : 0;
    }
    uint32_t bits = 0;
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int64_t s = tile + (int64_t)k * kBlock + threadIdx.x;
      if (s < n) core[s] = (f[k] == 1) ? 1 : 0;
      bits |= (f[k] == 2) ? (1u << k) : 0u;
    }
    if (cmin) {  // kernel-uniform
      uint32_t so[kItems];
#pragma unroll
      for (int k = 0; k < kItems; ++k) {
        const int64_t s = tile + (int64_t)k * kBlock + threadIdx.x;
        so[k] = (f[k] == 1 && s < n) ? (uint32_t)sorig[s] : 0u;
      }
#pragma unroll
      for (int k = 0; k < kItems; ++k) {
        const int64_t s = tile + (int64_t)k * kBlock + threadIdx.x;
        const int kk = key[k];
        // sorted keys: a run of equal keys is one cell; dist = lanes since this lane's run head
        const int prevk = __shfl_up(kk, 1, 64), next = __shfl_down(kk, 1, 64);
        const uint64_t hm = __ballot(lane == 0 || prevk != kk);
        const uint64_t upto = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
        const int dist = lane - (63 - __builtin_clzll(hm & upto));
        const bool in = f[k] == 1 && kk >= 0 && (int64_t)kk < cells;
        const bool tail = (lane == 63 || next != kk) && kk >= 0;
        if (n < (int64_t(1) << 26)) {  // kernel-uniform: (original << 6 | lane) fits 32 bits
          uint32_t v = in ? ((so[k] << 6) | (uint32_t)lane) : ~0u;
#pragma unroll
          for (int off = 1; off < 64; off <<= 1) {
            const uint32_t o = (uint32_t)__shfl_up((int)v, off, 64);
            if (off <= dist) v = min(v, o);
          }
          if (tail && v != ~0u)
            atomicMin(cmin + kk, ((unsigned long long)(v >> 6) << 32) |
                                     (uint32_t)(s - lane + (int)(v & 63u)));
        } else {
          uint64_t v = in ? (((uint64_t)so[k] << 32) | (uint32_t)s) : ~0ull;
#pragma unroll
          for (int off = 1; off < 64; off <<= 1) {
            const uint32_t olo = (uint32_t)__shfl_up((int)(uint32_t)v, off, 64);
            const uint32_t ohi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), off, 64);
            if (off <= dist) v = min(v, ((uint64_t)ohi << 32) | olo);
          }
          if (tail && v != ~0ull) atomicMin(cmin + kk, (unsigned long long)v);
        }
      }
    }
    if (QUEUE) block_append_bits(tile, bits, slow, n_slow);
  }
}

// Level 4, one wave per queued point: lanes classify up to 64 candidate cells at a time against
// the cells' boxes (whole-cell accept adds the cell's count), then every undecided cell's points
// are tested 64 at a time; the wave stops as soon as min_samples neighbours are seen.
template <int D, int KR = kR>
// KR: candidate positions per lane per super-round (2 when the exact integral-time window of
// (2 rt + 1) x 25 positions fits 128: the other two rounds only masked positions off)
// 8 waves/SIMD (64 VGPRs, one spill; 72 gave 7): -3 % on the latency-bound queue pass
__global__ __launch_bounds__(kBlock, 8) void k_core_slow(const float4* __restrict__ pts,
                                                     const int32_t* __restrict__ skey, Geom g,
                                                     const CellRec<D>* __restrict__ crec,
                                                     const uint32_t* __restrict__ occ_bits,
                                                     const float2* __restrict__ slab_t,
                                                     const int32_t* __restrict__ slow,
                                                     const int32_t* __restrict__ n_slow,
                                                     uint8_t* __restrict__ core,
                                                     const int32_t* __restrict__ sorig = nullptr,
                                                     unsigned long long* __restrict__ cmin =
                                                         nullptr,
                                                     const int32_t* __restrict__ slowk = nullptr) {
  const int lane = threadIdx.x & 63;
  const int need = g.min_samples;
  // XCD-aware ranges of the (cell-ordered) queue: neighbouring points' windows share an L2
  const XcdRange xr = xcd_items(*n_slow, true);
  for (int64_t q = xr.first; q < xr.end; q += xr.step) {
    const int s = slow[q];
    // slowk (the fused cell pass): the key comes with the queue entry, and with integral times
    // the window is the key's slab +- rt, so the occupancy loads do not wait for the point
    const int32_t key = slowk ? slowk[q] : skey[s];
    const float4 p = pts[s];
    int cx, cy, cz;
    decode_key<D>(key, g, cx, cy, cz);
    Window w;
    if (slowk && g.rt >= 0) {  // slab_of(p.w) is the key's slab (same cell_of)
      const int cs = g.slab_of_key(key);
      w.s0 = max(cs - g.rt, 0);
      w.nS = max(min(cs + g.rt, g.nt - 1) - w.s0 + 1, 0);
      w.x0 = cx - 2;
      w.y0 = cy - 2;
      w.z0 = (D == 3) ? cz - 2 : 0;
      w.total = w.nS * ((D == 3) ? 125 : 25);
    } else {
      w = make_window<D, false>(cx, cy, cz, p.w, p.w, g, slab_t);
    }
    int cnt = 0;
    // super-rounds of KR candidates per lane: every lane's bitmap words, then records, are
    // loaded together (one dependent level each for up to 64*KR candidates)
    for (int base = 0; base < w.total && cnt < need; base += 64 * KR) {
      int64_t c[KR];
      uint32_t wb[KR];
#pragma unroll
      for (int r = 0; r < KR; ++r) {
        const int qq = base + r * 64 + lane;
        c[r] = (qq < w.total) ? window_cell<D>(w, qq, g, slab_t, p.w, p.w) : -1;
      }
#pragma unroll
      for (int r = 0; r < KR; ++r) wb[r] = (c[r] >= 0) ? occ_bits[c[r] >> 5] : 0u;
      int b[KR], e[KR], cls[KR];
#pragma unroll
      for (int r = 0; r < KR; ++r) {
        b[r] = e[r] = cls[r] = 0;
        if (c[r] >= 0 && ((wb[r] >> (c[r] & 31)) & 1u)) {
          const CellRec<D> cr = crec[c[r]];
          b[r] = cr.b;
          e[r] = cr.e;
          cls[r] = classify<D>(p, rec_boxA<D>(cr), rec_boxB(cr), g);
        }
      }
      // whole-cell accepts (lower bound) and every cell that may hold a neighbour (upper bound,
      // with the super-rounds still to come): a point whose upper bound stays below min_samples
      // is decided without a pair test
      int add = 0, may = 0;
#pragma unroll
      for (int r = 0; r < KR; ++r) {
        add += (cls[r] == 1) ? e[r] - b[r] : 0;
        may += (cls[r] == 2) ? e[r] - b[r] : 0;
      }
      cnt += wave_sum(add);
      const bool last = base + 64 * KR >= w.total;
      if (last && cnt + wave_sum(may) < need) break;
#pragma unroll
      for (int r = 0; r < KR; ++r) {
        uint64_t pm = __ballot(cls[r] == 2);
        while (pm && cnt < need) {
          const int l = __ffsll((unsigned long long)pm) - 1;
          pm &= pm - 1;
          const int bb = __shfl(b[r], l), ee = __shfl(e[r], l);
          for (int j0 = bb; j0 < ee && cnt < need; j0 += 64) {
            const int j = j0 + lane;
            const bool a = (j < ee) && adjacent<D>(p, pts[j], g);
            cnt += __popcll(__ballot(a));
          }
        }
      }
    }
    if (lane == 0) {
      core[s] = (cnt >= need) ? 1 : 0;
      if (cmin && cnt >= need && (int64_t)key < g.cells)
        atomicMin(cmin + key, ((unsigned long long)(uint32_t)sorig[s] << 32) | (uint32_t)s);
    }
  }
}

// Level 4 fed by the fused cell pass's decisions (k_core_cells_oct<true, true>; 2-D, W = 2R + 1
// <= 5): one wave per queued point, whose cell's candidates are already split into whole accepts
// (their count lo, exact for every point of the cell), rejects (no neighbour of any point of the
// cell) and the partial ones (pmask).  So the point starts at cnt = lo and classifies ONLY the
// partial candidates (lane l takes window positions l and l + 64 of the mask): no occupancy
// words, no record loads or box tests of the decided candidates -- then the pair tests of the
// candidates still partial for the point itself, early exit at min_samples, as k_core_slow.
__device__ __forceinline__ int mask_pos_key(int pos, const Geom& g, int R, int W, uint32_t mg,
                                            int cx, int cy, int cs) {
  const int P = pos / 5, dx = pos - 5 * P;
  const int k = min((int)(((uint32_t)P * mg) >> 16), 4);  // P / W
  const int si = P - k * W;
  const int s2 = cs + si - R;
  const int y = cy + cw_row(k) - 2;
  return (s2 * g.ny + y) * g.nx + (cx - 2 + dx);
}
__global__ __launch_bounds__(kBlock, 8) void k_core_slow_masked(
    const float4* __restrict__ pts, Geom g, int R, const CellRec<2>* __restrict__ crec,
    const int32_t* __restrict__ occ, const int32_t* __restrict__ slow,
    const int32_t* __restrict__ slowq, const int32_t* __restrict__ n_slow,
    const uint4* __restrict__ pmask, const int32_t* __restrict__ clo, uint8_t* __restrict__ core,
    const int32_t* __restrict__ sorig, unsigned long long* __restrict__ cmin) {
  const int lane = threadIdx.x & 63;
  const int need = g.min_samples;
  const int W = 2 * R + 1;
  const uint32_t mg = (65535u + (uint32_t)W) / (uint32_t)W;
  const XcdRange xr = xcd_items(*n_slow, true);
  for (int64_t q = xr.first; q < xr.end; q += xr.step) {
    const int s = slow[q];
    const int32_t cq = slowq[q];
    // all independent of each other: one round of memory latency
    const float4 p = pts[s];
    const int32_t key = occ[cq];
    const uint4 m = pmask[cq];
    int cnt = clo[cq];
    int cx, cy, cz, cs;
    g.split((uint32_t)key, cx, cy, cz, cs);
    const uint32_t w0 = lane < 32 ? m.x : m.y;  // positions lane, lane + 64
    const uint32_t w1 = lane < 32 ? m.z : m.w;
    const bool h0 = (w0 >> (lane & 31)) & 1u, h1 = (w1 >> (lane & 31)) & 1u;
    const int k0 = h0 ? mask_pos_key(lane, g, R, W, mg, cx, cy, cs) : key;
    const int k1 = h1 ? mask_pos_key(lane + 64, g, R, W, mg, cx, cy, cs) : key;
    const CellRec<2> c0 = crec[k0], c1 = crec[k1];  // (branch-free: the own record otherwise)
    const int cl0 = h0 ? classify<2>(p, rec_boxA<2>(c0), rec_boxB(c0), g) : 0;
    const int cl1 = h1 ? classify<2>(p, rec_boxA<2>(c1), rec_boxB(c1), g) : 0;
    int add = (cl0 == 1 ? c0.e - c0.b : 0) + (cl1 == 1 ? c1.e - c1.b : 0);
    int may = (cl0 == 2 ? c0.e - c0.b : 0) + (cl1 == 2 ? c1.e - c1.b : 0);
    cnt += wave_sum(add);
    if (cnt < need && cnt + wave_sum(may) >= need) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int cl = r ? cl1 : cl0;
        const int bq = r ? c1.b : c0.b, eq = r ? c1.e : c0.e;
        uint64_t pm = __ballot(cl == 2);
        while (pm && cnt < need) {
          const int l = __ffsll((unsigned long long)pm) - 1;
          pm &= pm - 1;
          const int bb = __shfl(bq, l), ee = __shfl(eq, l);
          for (int j0 = bb; j0 < ee && cnt < need; j0 += 64) {
            const int jj = j0 + lane;
            const bool a = (jj < ee) && adjacent<2>(p, pts[jj], g);
            cnt += __popcll(__ballot(a));
          }
        }
      }
    }
    if (lane == 0) {
      core[s] = (cnt >= need) ? 1 : 0;
      if (cmin && cnt >= need)
        atomicMin(cmin + key, ((unsigned long long)(uint32_t)sorig[s] << 32) | (uint32_t)s);
    }
  }
}

// Per cell the smallest (original index << 32 | sorted index) over its core points (segmented
// wave minimum over the sorted points, one atomicMin per run): the core point with the smallest
// ORIGINAL index is the cell's representative, which keeps every union-find root its component's
// minimum original index whatever the order inside the cell (the slab-bucket K4 does not keep
// index order), and the star initialisation reads it directly.
__global__ __launch_bounds__(kBlock) void k_cell_min_pair(const int32_t* __restrict__ skey,
                                                         const uint8_t* __restrict__ core,
                                                         const int32_t* __restrict__ sorig,
                                                         int64_t n, int64_t cells,
                                                         unsigned long long* __restrict__ cmin) {
  const int lane = threadIdx.x & 63;
  for (int64_t s0 = (int64_t)blockIdx.x * blockDim.x; s0 < n;
       s0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = s0 + threadIdx.x;
    const int key = (s < n) ? skey[s] : -1;
    uint64_t v = (s < n && core[s] && (int64_t)key < cells)
                     ? (((uint64_t)(uint32_t)sorig[s] << 32) | (uint32_t)s)
                     : ~0ull;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {  // sorted keys: equal at distance off = same run
      const uint32_t olo = (uint32_t)__shfl_up((int)(uint32_t)v, off, 64);
      const uint32_t ohi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), off, 64);
      const int ok = __shfl_up(key, off, 64);
      if (lane >= off && ok == key) v = min(v, ((uint64_t)ohi << 32) | olo);
    }
    const int next = __shfl_down(key, 1, 64);
    if ((lane == 63 || next != key) && key >= 0 && v != ~0ull)
      atomicMin(cmin + key, (unsigned long long)v);
  }
}

// rep = -1 and the (min original, sorted) pair = all-ones for the occupied cells only: every
// reader of rep / the pairs looks at occupied cells (occ list, occupancy bits or non-empty
// cell_start ranges), so the dense C-cell grid needs no clear.
__global__ __launch_bounds__(kBlock) void k_init_occ_cells(const int32_t* __restrict__ occ,
                                                          const int32_t* __restrict__ n_occ,
                                                          int64_t cells,
                                                          int32_t* __restrict__ rep,
                                                          unsigned long long* __restrict__ cmin,
                                                          int32_t* __restrict__ zero_counter =
                                                              nullptr,
                                                          int32_t* __restrict__ zero_counter2 =
                                                              nullptr) {
  // the union passes' cell-list counters, zeroed here (their first user is two launches later)
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (zero_counter) *zero_counter = 0;
    if (zero_counter2) *zero_counter2 = 0;
  }
  const int64_t m = *n_occ;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < m;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int32_t c = occ[q];
    if ((int64_t)c < cells) {
      rep[c] = -1;
      if (cmin) cmin[c] = ~0ull;
    }
  }
}

// Star initialisation from k_cell_min_pair: core points of a mutual cell under the cell's
// representative, other points roots; the representative records itself in rep.
// kPU points per thread per tile, every load branch-free (clamped indices, results masked by
// selects) so each tile costs two rounds of memory latency: keys + flags, then the cells' minima.
constexpr int kPU = 8;
__global__ __launch_bounds__(kBlock) void k_parent_init_pair(
    int32_t* __restrict__ parent, int64_t n, const uint8_t* __restrict__ core,
    const int32_t* __restrict__ skey, const uint8_t* __restrict__ mutual,
    const unsigned long long* __restrict__ cmin, int64_t cells, int32_t* __restrict__ rep) {
  for (int64_t tile = (int64_t)blockIdx.x * kBlock * kPU; tile < n;
       tile += (int64_t)gridDim.x * kBlock * kPU) {
    int32_t k[kPU];
    uint32_t c[kPU];
#pragma unroll
    for (int u = 0; u < kPU; ++u) {
      const int64_t s = min(tile + (int64_t)u * kBlock + threadIdx.x, n - 1);
      k[u] = skey[s];
      c[u] = core[s];
    }
    bool q[kPU];
    unsigned long long m[kPU];
    uint32_t mu[kPU];
#pragma unroll
    for (int u = 0; u < kPU; ++u) {
      q[u] = c[u] != 0u && k[u] >= 0 && (int64_t)k[u] < cells;
      const int32_t kk = q[u] ? k[u] : 0;  // cells >= 1 whenever n >= 1
      m[u] = cmin[kk];
      mu[u] = mutual[kk];
    }
#pragma unroll
    for (int u = 0; u < kPU; ++u) {
      const int64_t s = tile + (int64_t)u * kBlock + threadIdx.x;
      if (s < n) {
        const int32_t r = (int32_t)(uint32_t)m[u];
        if (q[u] && r == (int32_t)s) rep[k[u]] = r;
        parent[s] = (q[u] && mu[u]) ? r : (int32_t)s;
      }
    }
  }
}

// ---------------------------------------------------------------- union-find
__device__ __forceinline__ int uf_load(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void uf_store(int32_t* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Path-halving find.  Parents only ever decrease, so a stale read is an older ancestor and
// every returned root was a true ancestor at some point (connectivity is never overstated).
__device__ __forceinline__ int uf_find(int32_t* parent, int x, bool halve = true) {
  while (true) {
    const int p = uf_load(parent + x);
    if (p == x) return x;
    const int gp = uf_load(parent + p);
    if (gp == p) return p;
    if (halve) uf_store(parent + x, gp);
    x = gp;
  }
}
__device__ __forceinline__ void uf_unite(int32_t* parent, const int32_t* __restrict__ sorig,
                                         int a, int b, bool halve = true) {
  while (true) {
    a = uf_find(parent, a, halve);
    b = uf_find(parent, b, halve);
    if (a == b) return;
    if (sorig[a] < sorig[b]) {
      const int tmp = a;
      a = b;
      b = tmp;
    }
    const int old = atomicCAS(parent + a, a, b);
    if (old == a) return;
    a = old;
  }
}

// K6a: mutual-cell x mutual-cell unions, one wave per occupied cell A, lanes over the candidate
// cells B > A of its window (each unordered pair once).
// PARTIAL = false: only pairs the boxes prove fully adjacent (cheap, no search).  A wave takes 64
//                  occupied cells at a time: their headers (cell, rep, mutual) in one coalesced
//                  round, then the mutual cells with core points one after another (half the
//                  occupied cells of a radar stack are noise cells, each a wave's dependent load
//                  chain otherwise).  With pmask: each cell's undecided candidates are recorded,
//                  and the cells that have any are listed in plist (one atomic per 64 cells).
// PARTIAL = true : undecided pairs whose roots still differ after the first pass (a kernel
//                  boundary later, so most such pairs are already connected), searched for one
//                  adjacent core pair: B's core points that can reach A's box, each tested
//                  against A's points 64 at a time.  With plist: only the listed cells.
template <int D, bool PARTIAL>
__global__ __launch_bounds__(kBlock) void k_union_cells(const float4* __restrict__ pts, Geom g,
                                                       const int32_t* __restrict__ cell_start,
                                                       const int32_t* __restrict__ occ,
                                                       const int32_t* __restrict__ n_occ,
                                                       const CellRec<D>* __restrict__ crec,
                                                       const uint32_t* __restrict__ occ_bits,
                                                       const float2* __restrict__ slab_t,
                                                       const uint8_t* __restrict__ core,
                                                       const int32_t* __restrict__ rep,
                                                       const uint8_t* __restrict__ mutual,
                                                       const int32_t* __restrict__ sorig,
                                                       int32_t* __restrict__ parent,
                                                       int uf_flags,
                                                       uint4* __restrict__ pmask = nullptr,
                                                       int32_t* __restrict__ plist = nullptr,
                                                       int32_t* __restrict__ pcount = nullptr) {
  const int lane = threadIdx.x & 63;
  const bool halve = !(uf_flags & 1);
  const int64_t no = *n_occ;
  const bool from_list = PARTIAL && plist;
  const int64_t items = from_list ? (int64_t)*pcount : (no + 63) / 64;
  const XcdRange xr = xcd_items(items, (uf_flags & 2) != 0);
  for (int64_t it = xr.first; it < xr.end; it += xr.step) {
    int ql = -1, cal = INT_MAX, ral = -1;
    uint8_t mal = 0;
    if (from_list) {
      if (lane == 0) ql = plist[it];
    } else if (it * 64 + lane < no) {
      ql = (int)(it * 64 + lane);
    }
    if (ql >= 0) cal = occ[ql];
    if ((int64_t)cal < g.cells) {  // (not the isolated, non-finite time cell)
      ral = rep[cal];
      mal = mutual[cal];
    }
    uint64_t todo = __ballot(ral >= 0 && mal);
    uint64_t lmask = 0;  // !PARTIAL: cells of this chunk with undecided candidates (plist)
    while (todo) {
      const int lq = __ffsll((unsigned long long)todo) - 1;
      todo &= todo - 1;
      const int64_t q = __shfl(ql, lq);
      const int ca = __shfl(cal, lq);
      const int ra = __shfl(ral, lq);
      const CellRec<D> ra_rec = crec[ca];
      const int ba = ra_rec.b, ea = ra_rec.e;  // core points anywhere in [b, e): scans start at b
      const float4 A1 = rec_boxA<D>(ra_rec), A2 = rec_boxB(ra_rec);
      int cx, cy, cz;
      decode_key<D>(ca, g, cx, cy, cz);
      // only cells B > A: slabs from A's own on (slabs are the slowest key dimension); the boxes'
      // time ranges are checked by classify_cells, so the slab window is not shrunk first
      const int sa = g.slab_of_key(ca);
      const Window w = make_window<D, false>(cx, cy, cz, A2.z, A2.w, g, slab_t, sa);
      // PARTIAL with the first pass's mask of this cell's undecided candidates (window positions
      // < 127): only those are visited, no enumeration or classification of the window again
      uint4 pm = make_uint4(0u, 0u, 0u, kPmaskFull);
      if (PARTIAL && pmask) pm = pmask[q];
      const bool listed = PARTIAL && !(pm.w & kPmaskFull);
      for (int base = 0; base < w.total; base += 64 * kR) {
        int64_t cb[kR];
        uint32_t wb[kR];
        int rb[kR], cls[kR], ebv[kR], bbv[kR];
        if (listed) {
#pragma unroll
          for (int k = 0; k < kR; ++k) {
            rb[k] = -1;
            cls[k] = 0;
            ebv[k] = 0;
            bbv[k] = 0;
            const uint32_t word = k == 0 ? (lane < 32 ? pm.x : pm.y) : (lane < 32 ? pm.z : pm.w);
            if (k < 2 && ((word >> (lane & 31)) & 1u)) {
              const int64_t c = window_cell<D>(w, k * 64 + lane, g, slab_t, A2.z, A2.w);
              const CellRec<D> cr = crec[c];
              rb[k] = rep[c];
              ebv[k] = cr.e;
              bbv[k] = cr.b;
              cls[k] = 2;
            }
          }
        } else {
#pragma unroll
        for (int k = 0; k < kR; ++k) {
          const int qq = base + k * 64 + lane;
          cb[k] = (qq < w.total) ? window_cell<D>(w, qq, g, slab_t, A2.z, A2.w) : -1;
          if (cb[k] <= (int64_t)ca) cb[k] = -1;
        }
#pragma unroll
        for (int k = 0; k < kR; ++k) wb[k] = (cb[k] >= 0) ? occ_bits[cb[k] >> 5] : 0u;
#pragma unroll
        for (int k = 0; k < kR; ++k) {
          rb[k] = -1;
          cls[k] = 0;
          ebv[k] = 0;
          bbv[k] = 0;
          if (cb[k] >= 0 && ((wb[k] >> (cb[k] & 31)) & 1u)) {
            const CellRec<D> cr = crec[cb[k]];
            const int r = rep[cb[k]];
            const uint8_t m = mutual[cb[k]];
            ebv[k] = cr.e;
            bbv[k] = cr.b;
            if (r >= 0 && m) {
              rb[k] = r;
              cls[k] = classify_cells<D>(A1, rec_boxA<D>(cr), A2, rec_boxB(cr), g);
            }
          }
        }
        }
        if (!PARTIAL) {
          if (pmask && base == 0) {  // the undecided candidates for the second pass
            const uint64_t m0 = __ballot(cls[0] == 2), m1 = __ballot(cls[1] == 2);
            if (lane == 0)
              pmask[q] = (w.total < 128)
                             ? make_uint4((uint32_t)m0, (uint32_t)(m0 >> 32), (uint32_t)m1,
                                          (uint32_t)(m1 >> 32) & ~kPmaskFull)
                             : make_uint4(0u, 0u, 0u, kPmaskFull);
            if (w.total >= 128 || (m0 | m1)) lmask |= 1ull << lq;
          }
          // neighbours' roots in parallel, then ONE unite per distinct root (dense regions give
          // a dozen box-certain neighbours that mostly share a root already)
          const int rA = uf_find(parent, ra, halve);
#pragma unroll
          for (int k = 0; k < kR; ++k) {
            const int rt = (cls[k] == 1) ? uf_find(parent, rb[k], halve) : -1;
            bool pend = rt >= 0 && rt != rA;
            bool mine = false;
            uint64_t pm = __ballot(pend);
            while (pm) {
              const int l = __ffsll((unsigned long long)pm) - 1;
              const int v = __shfl(rt, l);
              mine = mine || (lane == l);
              pend = pend && (rt != v);
              pm = __ballot(pend);
            }
            if (mine) uf_unite(parent, sorig, rA, rt, halve);
          }
          continue;
        }
#pragma unroll
        for (int k = 0; k < kR; ++k) {
          // (candidates of one root need one adjacent pair: dropped after a hit, as in
          // k_union_listed)
          const int rbr = (cls[k] == 2) ? uf_find(parent, rb[k], halve) : -1;
          const bool cand = (cls[k] == 2) && uf_find(parent, ra, halve) != rbr;
          uint64_t pm = __ballot(cand);
          while (pm) {
            const int l = __ffsll((unsigned long long)pm) - 1;
            pm &= pm - 1;
            const int rbl = __shfl(rb[k], l);
            const int ebl = __shfl(ebv[k], l);
            const int bbl = __shfl(bbv[k], l);
            bool hit = false;
            for (int jb0 = bbl; jb0 < ebl && !hit; jb0 += 64) {
              const int jb = jb0 + lane;
              float4 pb = make_float4(0.f, 0.f, 0.f, 0.f);
              bool cb_ok = false;
              if (jb < ebl && core[jb]) {
                pb = pts[jb];
                cb_ok = classify<D>(pb, A1, A2, g) != 0;
              }
              uint64_t bm = __ballot(cb_ok);
              while (bm && !hit) {
                const int lb = __ffsll((unsigned long long)bm) - 1;
                bm &= bm - 1;
                const float4 pq = shfl_f4(pb, lb);
                for (int ja0 = ba; ja0 < ea && !hit; ja0 += 64) {
                  const int ja = ja0 + lane;
                  const bool adj = (ja < ea) && core[ja] && adjacent<D>(pq, pts[ja], g);
                  hit = __ballot(adj) != 0;
                }
              }
            }
            if (hit) {
              if (lane == 0) uf_unite(parent, sorig, ra, rbl, halve);
              const int rr = __shfl(rbr, l);
              pm &= ~__ballot(rbr == rr);
            }
          }
        }
      }
    }
    if (!PARTIAL && plist && lmask) {
      int base = 0;
      if (lane == 0) base = atomicAdd(pcount, __popcll(lmask));
      base = __shfl(base, 0);
      if ((lmask >> lane) & 1ull) plist[base + __popcll(lmask & ((1ull << lane) - 1ull))] = ql;
    }
  }
}

// A block's LDS list of ints, appended to a global list (count at *gcount) by ONE global atomic
// issued by the block's last wave to finish (no block barrier: the other waves leave at once):
// a same-address global atomic per wave iteration serialised, ~4 ns each (k_union_cells_pair's
// undecided-cell list, 10 k of them at 125 frames: 147 -> 123 us at 16 cells per wave, 278 -> 130
// at 4).  A wave whose entries no longer fit appends them itself.
template <int Cap>
struct BlockList {
  int32_t buf[Cap];
  int n, valid;
  __device__ void init() {  // (one thread, before a block barrier)
    n = 0;
    valid = 0;
  }
  // the lanes of m append v (wave-uniform call)
  __device__ void push(uint64_t m, int v, int lane, int32_t* glist, int32_t* gcount) {
    if (!m) return;
    const int c = __popcll(m);
    int base = 0;
    if (lane == 0) base = atomicAdd(&n, c);
    base = __shfl(base, 0);
    const bool fits = base + c <= Cap;  // (wave-uniform; n only grows, so the fits are a prefix)
    if (fits) {
      if (lane == 0) atomicMax(&valid, base + c);
    } else {
      if (lane == 0) base = atomicAdd(gcount, c);
      base = __shfl(base, 0);
    }
    if ((m >> lane) & 1ull) {
      const int at = base + __popcll(m & ((1ull << lane) - 1ull));
      if (fits)
        buf[at] = v;
      else
        glist[at] = v;
    }
  }
  __device__ void flush(int lane, int32_t* glist, int32_t* gcount) {  // (the block's last wave)
    const int cnt = valid;
    int base = 0;
    if (lane == 0 && cnt) base = atomicAdd(gcount, cnt);
    base = __shfl(base, 0);
    for (int k = lane; k < cnt; k += 64) glist[base + k] = buf[k];
  }
};
// true in the block's last wave to reach it (the LDS lists are complete then)
__device__ __forceinline__ bool block_last_wave(int* done, int lane) {
  __threadfence_block();
  int last = 0;
  if (lane == 0) last = atomicAdd(done, 1) == (int)(blockDim.x / 64) - 1;
  last = __shfl(last, 0);
  if (last) __threadfence_block();
  return last != 0;
}
// K6a (2-D, box-certain pass) with TWO cells per wave: each half-wave takes one mutual cell with
// core points of the 64-cell chunk, lanes over its candidate cells B > A (window positions
// k * 32 + lane, k < kR: the exact-slab windows of integral times hold 75 positions), so two
// cells' dependent load chains (record -> occupancy -> candidate records -> roots) are in flight
// per wave instead of one.  Same unions, undecided-candidate masks (position p -> bit p of the
// 128-bit pmask, as k_union_listed reads them) and plist as k_union_cells<2, false>.
// 6 waves/SIMD (77 VGPRs, no spill; the unconstrained build took 81 and 5)
__global__ __launch_bounds__(kBlock, 6) void k_union_cells_pair(
    const float4* __restrict__ pts, Geom g, const int32_t* __restrict__ occ,
    const int32_t* __restrict__ n_occ, const CellRec<2>* __restrict__ crec,
    const uint32_t* __restrict__ occ_bits, const float2* __restrict__ slab_t,
    const int32_t* __restrict__ rep, const uint8_t* __restrict__ mutual,
    const int32_t* __restrict__ sorig, int32_t* __restrict__ parent, int uf_flags,
    uint4* __restrict__ pmask, int32_t* __restrict__ plist, int32_t* __restrict__ pcount,
    int cpw, int32_t* __restrict__ nm_list, int32_t* __restrict__ nm_count) {
  // nm_list (nullable): the non-mutual cells with core points (k_union_nm's list)
  constexpr int W = 32;
  const int lane = threadIdx.x & 63;
  const int hl = lane & (W - 1), h0 = lane - hl;
  auto hbal = [&](bool v) -> uint32_t { return (uint32_t)(__ballot(v) >> h0); };
  const bool halve = !(uf_flags & 1);
  const int64_t no = *n_occ;
  // cpw (<= 64) occupied cells per wave iteration: 64 on large stacks (one header load per lane),
  // fewer on small ones, whose waves would otherwise each walk dozens of cells in turn while most
  // of the GPU idles
  const int64_t items = (no + cpw - 1) / cpw;
  const XcdRange xr = xcd_items(items, (uf_flags & 2) != 0);
  __shared__ BlockList<1024> s_pl;  // plist entries (4 KiB)
  __shared__ BlockList<256> s_nm;   // nm_list entries
  __shared__ int s_done;
  if (threadIdx.x == 0) {
    s_pl.init();
    s_nm.init();
    s_done = 0;
  }
  __syncthreads();
  for (int64_t it = xr.first; it < xr.end; it += xr.step) {
    int ql = -1, cal = INT_MAX, ral = -1;
    uint8_t mal = 0;
    if (lane < cpw && it * cpw + lane < no) ql = (int)(it * cpw + lane);
    if (ql >= 0) cal = occ[ql];
    if ((int64_t)cal < g.cells) {  // (not the isolated, non-finite time cell)
      ral = rep[cal];
      mal = mutual[cal];
    }
    if (nm_list) s_nm.push(__ballot(ral >= 0 && !mal), cal, lane, nm_list, nm_count);
    // every todo cell's record loaded here, with the chunk's headers (one dependent level), and
    // handed to its half by shuffles: the pair loop starts at the window's occupancy loads
    CellRec<2> rl{};
    if (ral >= 0 && mal) rl = crec[cal];
    uint64_t todo = __ballot(ral >= 0 && mal);
    uint64_t lmask = 0;  // cells of this chunk with undecided candidates (plist)
    while (todo) {  // (wave-uniform) two cells at a time, one per half
      const int l0 = __ffsll((unsigned long long)todo) - 1;
      todo &= todo - 1;
      const int l1 = todo ? __ffsll((unsigned long long)todo) - 1 : -1;
      if (l1 >= 0) todo &= todo - 1;
      const int lq = h0 ? l1 : l0;  // this half's cell (-1: the upper half idles)
      const int lsrc = lq < 0 ? 0 : lq;
      const int64_t q = __shfl(ql, lsrc);
      const int ca = __shfl(cal, lsrc);
      const int ra = __shfl(ral, lsrc);
      bool any_und = false;
      CellRec<2> ra_rec;  // (every lane takes part in the shuffles)
      ra_rec.b = __shfl(rl.b, lsrc);
      ra_rec.e = __shfl(rl.e, lsrc);
      ra_rec.x0 = __shfl(rl.x0, lsrc);
      ra_rec.x1 = __shfl(rl.x1, lsrc);
      ra_rec.y0 = __shfl(rl.y0, lsrc);
      ra_rec.y1 = __shfl(rl.y1, lsrc);
      ra_rec.t0 = __shfl(rl.t0, lsrc);
      ra_rec.t1 = __shfl(rl.t1, lsrc);
      if (lq >= 0) {  // (half-uniform)
        const float4 A1 = rec_boxA<2>(ra_rec), A2 = rec_boxB(ra_rec);
        int cx, cy, cz;
        decode_key<2>(ca, g, cx, cy, cz);
        const int sa = g.slab_of_key(ca);
        const Window w = make_window<2, false>(cx, cy, cz, A2.z, A2.w, g, slab_t, sa);
        for (int base = 0; base < w.total; base += W * kR) {
          int64_t cb[kR];
          uint32_t wb[kR];
          int rb[kR], cls[kR];
#pragma unroll
          for (int k = 0; k < kR; ++k) {
            const int qq = base + k * W + hl;
            cb[k] = (qq < w.total) ? window_cell<2>(w, qq, g, slab_t, A2.z, A2.w) : -1;
            if (cb[k] <= (int64_t)ca) cb[k] = -1;
          }
#pragma unroll
          for (int k = 0; k < kR; ++k) wb[k] = (cb[k] >= 0) ? occ_bits[cb[k] >> 5] : 0u;
#pragma unroll
          for (int k = 0; k < kR; ++k) {
            rb[k] = -1;
            cls[k] = 0;
            if (cb[k] >= 0 && ((wb[k] >> (cb[k] & 31)) & 1u)) {
              const CellRec<2> cr = crec[cb[k]];
              const int r = rep[cb[k]];
              const uint8_t m = mutual[cb[k]];
              if (r >= 0 && m) {
                rb[k] = r;
                cls[k] = classify_cells<2>(A1, rec_boxA<2>(cr), A2, rec_boxB(cr), g);
              }
            }
          }
          if (pmask && base == 0) {  // the undecided candidates for the second pass
            uint32_t wd[kR];
#pragma unroll
            for (int k = 0; k < kR; ++k) wd[k] = hbal(cls[k] == 2);
            static_assert(kR == 4, "the 128-bit pmask holds 4 x 32 window positions");
            if (hl == 0)
              pmask[q] = (w.total < 128)
                             ? make_uint4(wd[0], wd[1], wd[2], wd[3] & ~kPmaskFull)
                             : make_uint4(0u, 0u, 0u, kPmaskFull);
            any_und = w.total >= 128 || (wd[0] | wd[1] | wd[2] | wd[3]) != 0u;
          }
          // neighbours' roots in parallel, then ONE unite per distinct root
          const int rA = uf_find(parent, ra, halve);
#pragma unroll
          for (int k = 0; k < kR; ++k) {
            const int rt = (cls[k] == 1) ? uf_find(parent, rb[k], halve) : -1;
            bool pend = rt >= 0 && rt != rA;
            bool mine = false;
            uint32_t pm = hbal(pend);
            while (pm) {  // (half-uniform)
              const int l = h0 + __ffs(pm) - 1;
              const int v = __shfl(rt, l);
              mine = mine || (lane == l);
              pend = pend && (rt != v);
              pm = hbal(pend);
            }
            if (mine) uf_unite(parent, sorig, rA, rt, halve);
          }
        }
      }
      // cells with undecided candidates -> plist (lane 0 / 32 hold each half's flag)
      const bool u0 = __shfl((int)any_und, 0) != 0, u1 = __shfl((int)any_und, 32) != 0;
      if (u0) lmask |= 1ull << l0;
      if (u1 && l1 >= 0) lmask |= 1ull << l1;
    }
    if (plist) s_pl.push(lmask, ql, lane, plist, pcount);
  }
  if ((plist || nm_list) && block_last_wave(&s_done, lane)) {  // the block's lists -> global
    if (plist) s_pl.flush(lane, plist, pcount);
    if (nm_list) s_nm.flush(lane, nm_list, nm_count);
  }
}

// Root snapshot after the box-certain pass: croot[c] = root of rep[c] per occupied cell with core
// points (-1 otherwise).  Unions only merge, so equal snapshot roots stay connected: the listed
// pass then settles a candidate with ONE load instead of two parent-chain walks -- 99.5 % of the
// undecided candidates share A's root by then (1000 frames: 4.0 M candidates, 19 k roots
// different; configs[4] share: 33.7 M, 282 k).
__global__ __launch_bounds__(kBlock) void k_cell_root_snapshot(const int32_t* __restrict__ occ,
                                                              const int32_t* __restrict__ n_occ,
                                                              const int32_t* __restrict__ rep,
                                                              int32_t* __restrict__ parent,
                                                              int64_t cells, int uf_flags,
                                                              int32_t* __restrict__ croot) {
  const bool halve = !(uf_flags & 1);
  const int64_t no = *n_occ;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < no;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int c = occ[q];
    if ((int64_t)c >= cells) continue;  // (the isolated, non-finite time cell)
    const int r = rep[c];
    croot[c] = r >= 0 ? uf_find(parent, r, halve) : -1;
  }
}

// K6b over the first pass's cell list (2-D): one wave per listed cell, lane l over window
// positions l and l + 64 of its pmask (a window of >= 128 positions is walked 64 positions at a
// time instead, classifying again), then k_union_cells<D, true>'s search for each undecided
// pair whose roots still differ.  Without the kR-wide enumeration the kernel holds far fewer
// registers than k_union_cells<2, true> (twice the waves per SIMD: the pass is a chain of
// dependent loads per cell).
__global__ __launch_bounds__(kBlock) void k_union_listed(const float4* __restrict__ pts, Geom g,
                                                        const int32_t* __restrict__ occ,
                                                        const CellRec<2>* __restrict__ crec,
                                                        const uint32_t* __restrict__ occ_bits,
                                                        const float2* __restrict__ slab_t,
                                                        const uint8_t* __restrict__ core,
                                                        const int32_t* __restrict__ rep,
                                                        const uint8_t* __restrict__ mutual,
                                                        const int32_t* __restrict__ sorig,
                                                        int32_t* __restrict__ parent, int uf_flags,
                                                        const uint4* __restrict__ pmask,
                                                        const int32_t* __restrict__ plist,
                                                        const int32_t* __restrict__ pcount,
                                                        const int32_t* __restrict__ croot,
                                                        int32_t* __restrict__ lstat = nullptr) {
  // lstat (A/B build, RPT_STATS): undecided candidates, candidates whose roots differed, searches,
  // hits
  const int lane = threadIdx.x & 63;
  const bool halve = !(uf_flags & 1);
  const XcdRange xr = xcd_items(*pcount, false);
  if (xr.first >= xr.end) return;
  // software-pipelined headers (as k_cell_box): the next cell's key and mask and the one after's
  // list entry load while this cell is settled; branch-free from clamped list positions
  auto list_at = [&](int64_t ii) { return plist[ii < xr.end ? ii : xr.end - 1]; };
  int ca = occ[list_at(xr.first)];
  uint4 pm = pmask[list_at(xr.first)];
  int qn = list_at(xr.first + xr.step);
  for (int64_t i = xr.first; i < xr.end; i += xr.step) {
    const int ra = rep[ca];
    const int sra = croot ? croot[ca] : -1;  // A's snapshot root (kernel-uniform)
    const CellRec<2> ra_rec = crec[ca];
    const int can = occ[qn];
    const uint4 pmn = pmask[qn];
    const int qnn = list_at(i + 2 * xr.step);
    const int ba = ra_rec.b, ea = ra_rec.e;
    const float4 A1 = rec_boxA<2>(ra_rec), A2 = rec_boxB(ra_rec);
    int cx, cy, cz;
    decode_key<2>(ca, g, cx, cy, cz);
    const int sa = g.slab_of_key(ca);
    const Window w = make_window<2, false>(cx, cy, cz, A2.z, A2.w, g, slab_t, sa);
    // the undecided candidate of this lane (rb >= 0) -> one adjacent core pair unites A and B
    // Candidates sharing a root (e.g. one cell column over the slab window, united whole by the
    // first pass) need ONE adjacent pair between them: once a search unites A with a root, the
    // remaining candidates of that root are connected too and are dropped without a search.
    auto settle = [&](int rb, int bb, int eb) {
      const int rbr = rb >= 0 ? uf_find(parent, rb, halve) : -1;
      const bool cand = rb >= 0 && uf_find(parent, ra, halve) != rbr;
      uint64_t cm = __ballot(cand);
#ifdef RPT_AB
      if (lstat) {
        const int nb = __popcll(__ballot(rb >= 0));
        if (lane == 0) {
          atomicAdd(&lstat[0], nb);
          atomicAdd(&lstat[1], __popcll(cm));
        }
      }
#endif
      while (cm) {
        const int l = __ffsll((unsigned long long)cm) - 1;
        cm &= cm - 1;
        const int rbl = __shfl(rb, l);
        const int ebl = __shfl(eb, l);
        const int bbl = __shfl(bb, l);
        // other waves may have connected A and this candidate since the roots were read
        if (uf_find(parent, ra, halve) == uf_find(parent, rbl, halve)) continue;
#ifdef RPT_AB
        if (lstat && lane == 0) atomicAdd(&lstat[2], 1);
#endif
        bool hit = false;
        for (int jb0 = bbl; jb0 < ebl && !hit; jb0 += 64) {
          const int jb = jb0 + lane;
          float4 pb = make_float4(0.f, 0.f, 0.f, 0.f);
          bool cb_ok = false;
          if (jb < ebl && core[jb]) {
            pb = pts[jb];
            cb_ok = classify<2>(pb, A1, A2, g) != 0;
          }
          // this chunk's B core points that can reach A's box (bm) against A's core points 64
          // at a time: each lane loads ONE A point per chunk and tests it against every such B
          // point (shuffles, no loads), so an A chunk costs one round trip for all of them (B
          // point by B point, a pair with no adjacent points walked |B| x |A|/64 round trips)
          const uint64_t bm = __ballot(cb_ok);
          for (int ja0 = ba; bm && ja0 < ea && !hit; ja0 += 64) {
            const int ja = ja0 + lane;
            const bool va = (ja < ea) && core[ja];
            const float4 pa = va ? pts[ja] : make_float4(0.f, 0.f, 0.f, 0.f);
            bool adj = false;
            uint64_t rest = bm;
            while (rest) {  // (wave-uniform)
              const int lb = __ffsll((unsigned long long)rest) - 1;
              rest &= rest - 1;
              const float4 pq = shfl_f4(pb, lb);
              adj = adj || (va && adjacent<2>(pq, pa, g));
            }
            hit = __ballot(adj) != 0;
          }
        }
        if (hit) {
#ifdef RPT_AB
          if (lstat && lane == 0) atomicAdd(&lstat[3], 1);
#endif
          if (lane == 0) uf_unite(parent, sorig, ra, rbl, halve);
          const int rr = __shfl(rbr, l);
          cm &= ~__ballot(rbr == rr);
        }
      }
    };
    if (!(pm.w & kPmaskFull)) {
      int rb[2], ebv[2], bbv[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        rb[k] = -1;
        ebv[k] = bbv[k] = 0;
        const uint32_t word = k == 0 ? (lane < 32 ? pm.x : pm.y) : (lane < 32 ? pm.z : pm.w);
        if ((word >> (lane & 31)) & 1u) {
          const int64_t c = window_cell<2>(w, k * 64 + lane, g, slab_t, A2.z, A2.w);
          if (!croot || croot[c] != sra) {  // (else connected already: no record, no walk)
            const CellRec<2> cr = crec[c];
            rb[k] = rep[c];
            ebv[k] = cr.e;
            bbv[k] = cr.b;
          }
        }
      }
      settle(rb[0], bbv[0], ebv[0]);
      settle(rb[1], bbv[1], ebv[1]);
    } else {
      for (int base = 0; base < w.total; base += 64) {
        const int qq = base + lane;
        int64_t c = (qq < w.total) ? window_cell<2>(w, qq, g, slab_t, A2.z, A2.w) : -1;
        if (c <= (int64_t)ca || !((occ_bits[c >> 5] >> (c & 31)) & 1u)) c = -1;
        int rb = -1, bb = 0, eb = 0;
        if (c >= 0) {
          const CellRec<2> cr = crec[c];
          const int r = rep[c];
          if (r >= 0 && mutual[c] &&
              classify_cells<2>(A1, rec_boxA<2>(cr), A2, rec_boxB(cr), g) == 2) {
            rb = r;
            bb = cr.b;
            eb = cr.e;
          }
        }
        settle(rb, bb, eb);
      }
    }
    ca = can;
    pm = pmn;
    qn = qnn;
  }
}

// one core point's unions (k_union, k_union_nm)
template <int D>
__device__ __forceinline__ void union_point(int si, int32_t key, const float4* __restrict__ pts,
                                            Geom g, const int32_t* __restrict__ cell_start,
                                            const CellRec<D>* __restrict__ crec,
                                            const float2* __restrict__ slab_t,
                                            const uint8_t* __restrict__ core,
                                            const int32_t* __restrict__ rep,
                                            const uint8_t* __restrict__ mutual,
                                            const int32_t* __restrict__ sorig,
                                            int32_t* __restrict__ parent) {
  const float4 p = pts[si];
  for_each_cell<D>(p, key, g, cell_start, crec, slab_t,
                   [&](int64_t c, int b, int e, int cls) -> bool {
                     const int r = rep[c];
                     if (r < 0) return false;
                     if (mutual[c]) {
                       if (cls == 1) {
                         uf_unite(parent, sorig, si, r);
                         return false;
                       }
                       if (uf_find(parent, si) == uf_find(parent, r)) return false;
                       for (int j = b; j < e; ++j) {
                         if (core[j] && adjacent<D>(p, pts[j], g)) {
                           uf_unite(parent, sorig, si, j);
                           break;
                         }
                       }
                     } else {
                       for (int j = max(b, si + 1); j < e; ++j) {
                         if (core[j] && (cls == 1 || adjacent<D>(p, pts[j], g)))
                           uf_unite(parent, sorig, si, j);
                       }
                     }
                     return false;
                   });
}

// K6: core-core union.  Edge (s, j) with j in cell c:
//   * c mutual: all of c's core points are pairwise adjacent, hence one component; one edge
//     from s into c (to rep[c] when the whole cell is adjacent, else to the first adjacent core
//     point) spans every edge from s into c.
//   * c not mutual: every adjacent core j > s (the edge from the smaller end covers the pair;
//     when cell(s) is mutual the larger end's first-hit edge covers it too).
template <int D>
__global__ __launch_bounds__(kBlock) void k_union(const float4* __restrict__ pts,
                                                 const int32_t* __restrict__ skey, int64_t n,
                                                 Geom g, const int32_t* __restrict__ cell_start,
                                                 const CellRec<D>* __restrict__ crec,
                                                 const float2* __restrict__ slab_t,
                                                 const uint8_t* __restrict__ core,
                                                 const int32_t* __restrict__ rep,
                                                 const uint8_t* __restrict__ mutual,
                                                 const int32_t* __restrict__ sorig,
                                                 int32_t* __restrict__ parent) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n || !core[s]) return;
  const int32_t key = skey[s];
  if ((int64_t)key >= g.cells) return;
  if (mutual[key]) return;  // handled by the star init + k_union_cells
  union_point<D>((int)s, key, pts, g, cell_start, crec, slab_t, core, rep, mutual, sorig, parent);
}

// K6c (2-D pair path): k_union's unions for the core points of the NON-mutual cells with core
// points, listed by the box-certain pass -- one wave per listed cell, lanes over its points.
// With one-frame slabs every 2-D cell is mutual (box diagonal below eps, time span 0), so the
// bench stacks list none, where k_union read every point's flag for nothing (123 us at 1000
// frames).
template <int D>
__global__ __launch_bounds__(kBlock) void k_union_nm(const float4* __restrict__ pts, Geom g,
                                                    const int32_t* __restrict__ cell_start,
                                                    const CellRec<D>* __restrict__ crec,
                                                    const float2* __restrict__ slab_t,
                                                    const uint8_t* __restrict__ core,
                                                    const int32_t* __restrict__ rep,
                                                    const uint8_t* __restrict__ mutual,
                                                    const int32_t* __restrict__ sorig,
                                                    int32_t* __restrict__ parent,
                                                    const int32_t* __restrict__ nm_list,
                                                    const int32_t* __restrict__ nm_count) {
  const int lane = threadIdx.x & 63;
  const XcdRange xr = xcd_items(*nm_count, false);
  for (int64_t i = xr.first; i < xr.end; i += xr.step) {
    const int32_t key = nm_list[i];
    const int b = crec[key].b, e = crec[key].e;
    for (int s = b + lane; s < e; s += 64)
      if (core[s])
        union_point<D>(s, key, pts, g, cell_start, crec, slab_t, core, rep, mutual, sorig,
                       parent);
  }
}

__global__ __launch_bounds__(kBlock) void k_fill_i32(int32_t* p, int64_t n, int32_t v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

// Cluster id of a component minimum m = its rank among the minima: one bit per original index
// (set by k_ccmin) and an exclusive scan of the words' popcounts (total = cluster count at
// pref[words]): n/32 words to clear and scan instead of an n-length flag array.
struct MinRank {
  const uint32_t* bits;
  const int32_t* pref;
  __device__ __forceinline__ int32_t operator[](int32_t m) const {
    const uint32_t w = bits[m >> 5];
    return pref[m >> 5] + __popc(w & ((1u << (m & 31)) - 1u));
  }
};

__global__ void k_word_popc(const uint32_t* __restrict__ bits, int64_t words,
                            int32_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < words;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = __popc(bits[i]);
}

// ccmin[s] = component-min original index for core points, -1 otherwise; flags the minima and
// queues the non-core points for k_label.
// Root of every occupied mutual cell's core points (its representative's root): the core points
// of a mutual cell all hang under the representative (star init), so k_ccmin takes their root
// from here -- one cached per-cell read instead of a parent chain per point.
__global__ __launch_bounds__(kBlock) void k_cell_roots(int32_t* parent,
                                                      const int32_t* __restrict__ occ,
                                                      const int32_t* __restrict__ n_occ,
                                                      int64_t cells,
                                                      const uint8_t* __restrict__ mutual,
                                                      const int32_t* __restrict__ rep,
                                                      int32_t* __restrict__ cell_root,
                                                      int32_t* __restrict__ zero = nullptr,
                                                      uint32_t* __restrict__ zwords = nullptr,
                                                      int64_t nzw = 0,
                                                      int32_t* __restrict__ cmin_fill = nullptr) {
  // zero (nullable): a counter of the next kernel, cleared here instead of by a memset launch;
  // likewise the label pass's minimum bits (zwords, nzw words) and its per-cell smallest keys
  // (cmin_fill: every cell INT_MAX) -- both first written by k_ccmin / k_ccmin_global next
  if (zero && blockIdx.x == 0 && threadIdx.x == 0) *zero = 0;
  {
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t ts = (int64_t)gridDim.x * blockDim.x;
    if (zwords)
      for (int64_t i = t0; i < nzw; i += ts) zwords[i] = 0u;
    if (cmin_fill)
      for (int64_t i = t0; i < cells; i += ts) cmin_fill[i] = INT_MAX;
  }
  const int64_t m = *n_occ;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < m;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int32_t c = occ[q];
    if ((int64_t)c >= cells) continue;
    const int r = mutual[c] ? rep[c] : -1;
    cell_root[c] = (r >= 0) ? uf_find(parent, r) : -1;  // -1: walk each point's own chain
  }
}

// cell_root (nullable): k_cell_roots' output (-1: not a mutual cell with core points), read for
// core points through skey.
// cell_key (nullable, pre-filled with INT_MAX): per cell the smallest component key among its
// core points, by a segmented wave minimum over the sorted points (k_cell_min_key fused in).
// The kItems points of a thread go through the dependent loads level by level (keys + flags,
// cell roots, component minima), each level's loads in flight together; the atomics come last.
__global__ __launch_bounds__(kBlock) void k_ccmin(int32_t* parent,
                                                 const uint8_t* __restrict__ core, int64_t n,
                                                 const int32_t* __restrict__ sorig,
                                                 int32_t* __restrict__ ccmin,
                                                 uint32_t* __restrict__ min_bits,
                                                 int32_t* __restrict__ nc_list,
                                                 int32_t* __restrict__ nc_count,
                                                 const int32_t* __restrict__ skey = nullptr,
                                                 const uint8_t* __restrict__ mutual = nullptr,
                                                 const int32_t* __restrict__ cell_root = nullptr,
                                                 int64_t cells = 0,
                                                 int32_t* __restrict__ cell_key = nullptr) {
  const int lane = threadIdx.x & 63;
  (void)mutual;
  for (int64_t tile = (int64_t)blockIdx.x * kBlock * kItems; tile < n;
       tile += (int64_t)gridDim.x * kBlock * kItems) {
    int32_t key[kItems], x[kItems];
    uint32_t cbits = 0, inb = 0;
#pragma unroll
    // levels 1, 2 and 4 load branch-free (clamped indices, results masked), so each level's
    // loads are in flight together; only the parent-chain walk (points outside mutual cells)
    // stays conditional
    for (int k = 0; k < kItems; ++k) {
      const int64_t s = tile + (int64_t)k * kBlock + threadIdx.x;
      const int64_t sc = min(s, n - 1);
      const int32_t kv = skey ? skey[sc] : -1;  // kernel-uniform pointer test
      const uint8_t cv = core[sc];
      const bool in = s < n;
      key[k] = in ? kv : -1;
      inb |= in ? (1u << k) : 0u;
      cbits |= (in && cv) ? (1u << k) : 0u;
    }
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      x[k] = -1;
      if (cell_root) {  // kernel-uniform
        const bool q = ((cbits >> k) & 1u) && key[k] >= 0 && (int64_t)key[k] < cells;
        const int32_t r = cell_root[q ? key[k] : 0];  // cells >= 1
        x[k] = q ? r : -1;
      }
    }
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int s = (int)(tile + (int64_t)k * kBlock + threadIdx.x);
      if (((cbits >> k) & 1u) && x[k] < 0) x[k] = uf_find(parent, s);
    }
    int m[kItems];
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const bool c = (cbits >> k) & 1u;
      const int32_t v = sorig[c ? x[k] : 0];
      m[k] = c ? v : -1;
    }
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int64_t s = tile + (int64_t)k * kBlock + threadIdx.x;
      if ((inb >> k) & 1u) ccmin[s] = m[k];
      if (((cbits >> k) & 1u) && x[k] == (int)s) atomicOr(min_bits + (m[k] >> 5), 1u << (m[k] & 31));
    }
    if (cell_key) {  // kernel-uniform: every lane of the wave takes part
#pragma unroll
      for (int k = 0; k < kItems; ++k) {
        int v = (m[k] >= 0 && (int64_t)key[k] < cells) ? m[k] : INT_MAX;
        const int kk = key[k];
        // sorted keys: a run of equal keys is one cell; dist = lanes since this lane's run head
        const int prevk = __shfl_up(kk, 1, 64), next = __shfl_down(kk, 1, 64);
        const uint64_t hm = __ballot(lane == 0 || prevk != kk);
        const uint64_t upto = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
        const int dist = lane - (63 - __builtin_clzll(hm & upto));
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const int ov = __shfl_up(v, off, 64);
          if (off <= dist) v = min(v, ov);
        }
        if ((lane == 63 || next != kk) && kk >= 0 && v != INT_MAX) atomicMin(cell_key + kk, v);
      }
    }
    block_append_bits(tile, inb & ~cbits, nc_list, nc_count);
  }
}

// queue of the non-core points (phased / global labelling)
__global__ __launch_bounds__(kBlock) void k_nc_list(const uint8_t* __restrict__ core, int64_t n,
                                                   int32_t* __restrict__ nc_list,
                                                   int32_t* __restrict__ nc_count) {
  for (int64_t tile = (int64_t)blockIdx.x * kBlock * kItems; tile < n;
       tile += (int64_t)gridDim.x * kBlock * kItems)
    block_append(
        tile, n, [&](int64_t s) -> bool { return !core[s]; }, nc_list, nc_count);
}

// K7/K8 (core points): label = id of the component minimum
__global__ __launch_bounds__(kBlock) void k_label_core(const int32_t* __restrict__ ccmin,
                                                      int64_t n,
                                                      const int32_t* __restrict__ sorig,
                                                      MinRank cid,
                                                      int32_t* __restrict__ labels) {
  // kPU points per thread per tile, loads branch-free (clamped, masked): two memory rounds per
  // tile (ccmin + sorig, then the rank words) instead of two per point.  XCD-contiguous tiles
  // (grid a multiple of 8): the blocks of one XCD take one eighth of the sorted points, i.e. a
  // run of whole frames, so the labels they scatter (original order, within those frames) fill
  // their lines in that XCD's L2 instead of eight L2s writing partial lines of the same frames
  const int64_t T = (n + (int64_t)kBlock * kPU - 1) / ((int64_t)kBlock * kPU);
  const bool xm = (gridDim.x & 7) == 0;
  const int64_t xg = blockIdx.x & 7, nbx = gridDim.x >> 3;
  const int64_t t_lo = xm ? T * xg / 8 : blockIdx.x, t_hi = xm ? T * (xg + 1) / 8 : T;
  const int64_t t_step = xm ? nbx : gridDim.x;
  for (int64_t ti = t_lo + (xm ? (int64_t)(blockIdx.x >> 3) : 0); ti < t_hi; ti += t_step) {
    const int64_t tile = ti * kBlock * kPU;
    int32_t own[kPU], so[kPU];
#pragma unroll
    for (int u = 0; u < kPU; ++u) {
      const int64_t s = min(tile + (int64_t)u * kBlock + threadIdx.x, n - 1);
      own[u] = ccmin[s];
      so[u] = sorig[s];
    }
    uint32_t w[kPU];
    int32_t pr[kPU];
#pragma unroll
    for (int u = 0; u < kPU; ++u) {
      const int32_t m = own[u] >= 0 ? own[u] : 0;
      w[u] = cid.bits[m >> 5];
      pr[u] = cid.pref[m >> 5];
    }
#pragma unroll
    for (int u = 0; u < kPU; ++u) {
      const int64_t s = tile + (int64_t)u * kBlock + threadIdx.x;
      if (s < n && own[u] >= 0)
        labels[so[u]] = pr[u] + __popc(w[u] & ((1u << (own[u] & 31)) - 1u));
    }
  }
}

// The same in ORIGINAL order through the grid build's inverse permutation spos: the labels are
// written in whole lines and the component keys gathered (a frame's keys stay in L2) instead of
// 4-byte label writes scattered over each frame, whose partly written lines L2 evicts (dense
// share: 1.23 GB written for 0.25 GB of labels).  Non-core points are left to k_label.
__global__ __launch_bounds__(kBlock) void k_label_core_orig(const int32_t* __restrict__ ccmin,
                                                           int64_t n,
                                                           const int32_t* __restrict__ spos,
                                                           MinRank cid,
                                                           int32_t* __restrict__ labels) {
  const int64_t T = (n + (int64_t)kBlock * kPU - 1) / ((int64_t)kBlock * kPU);
  const bool xm = (gridDim.x & 7) == 0;  // XCD-contiguous tiles (runs of whole frames)
  const int64_t xg = blockIdx.x & 7, nbx = gridDim.x >> 3;
  const int64_t t_lo = xm ? T * xg / 8 : blockIdx.x, t_hi = xm ? T * (xg + 1) / 8 : T;
  const int64_t t_step = xm ? nbx : gridDim.x;
  for (int64_t ti = t_lo + (xm ? (int64_t)(blockIdx.x >> 3) : 0); ti < t_hi; ti += t_step) {
    const int64_t tile = ti * kBlock * kPU;
    int32_t sp[kPU], own[kPU];
#pragma unroll
    for (int u = 0; u < kPU; ++u)  // branch-free (clamped); streamed once
      sp[u] = __builtin_nontemporal_load(spos + min(tile + (int64_t)u * kBlock + threadIdx.x,
                                                     n - 1));
#pragma unroll
    for (int u = 0; u < kPU; ++u) own[u] = ccmin[sp[u]];
    uint32_t w[kPU];
    int32_t pr[kPU];
#pragma unroll
    for (int u = 0; u < kPU; ++u) {
      const int32_t m = own[u] >= 0 ? own[u] : 0;
      w[u] = cid.bits[m >> 5];
      pr[u] = cid.pref[m >> 5];
    }
#pragma unroll
    for (int u = 0; u < kPU; ++u) {
      const int64_t i = tile + (int64_t)u * kBlock + threadIdx.x;
      if (i < n && own[u] >= 0)
        labels[i] = pr[u] + __popc(w[u] & ((1u << (own[u] & 31)) - 1u));
    }
  }
}

// K7/K8 (non-core points, queued): the smallest component key over adjacent core points, else
// none.  One wave per point, one lane per candidate cell of its window.  A cell whose box is
// wholly adjacent contributes its smallest key (cell_key) with no point read; the others are
// resolved in increasing cell_key order and only while that key can still beat the best so far:
// a mutual cell (one component) needs one adjacent core point, any other cell the smallest key
// among its adjacent core points.
// GLOBAL = false: key = ccmin (component-min original index, local run), label = cid[key];
// GLOBAL = true : key = slab (the core point's final label: labels are ranks of the sorted global
//                 representatives, so the smallest label is the smallest representative).
template <int D, bool GLOBAL, int W = 64>
// 6 waves/SIMD (80 VGPRs, no spill; with two candidate points per lane per round 7 spilled 8)
// W = 32: two points per wave, one per half (the same candidate loads per point, twice the
// points in flight: the pass is a chain of dependent loads per point, not bandwidth)
__global__ __launch_bounds__(kBlock, 6) void k_label(const float4* __restrict__ pts,
                                                 const int32_t* __restrict__ skey, Geom g,
                                                 const CellRec<D>* __restrict__ crec,
                                                 const uint32_t* __restrict__ occ_bits,
                                                 const float2* __restrict__ slab_t,
                                                 const int32_t* __restrict__ key_of,
                                                 const int32_t* __restrict__ cell_key,
                                                 const uint8_t* __restrict__ mutual,
                                                 const int32_t* __restrict__ sorig,
                                                 MinRank cid,
                                                 const int32_t* __restrict__ nc_list,
                                                 const int32_t* __restrict__ nc_count,
                                                 int32_t* __restrict__ labels,
                                                 int32_t* __restrict__ kstat = nullptr) {
  // kstat (A/B build, RPT_STATS): queued points, points with a core cell in their window, points
  // that searched a partly reachable cell, points labelled
  static_assert(W == 32 || W == 64, "a point per wave or per half-wave");
  constexpr int P = 64 / W;  // points per wave
  const int lane = threadIdx.x & 63;
  const int hl = lane & (W - 1);      // lane within the point's group
  const int h0 = lane - hl;           // the group's first lane
  const int shift = (W == 64) ? 0 : h0;
  // the group's bits of a wave ballot
  auto gbal = [&](bool v) -> uint64_t {
    const uint64_t b = __ballot(v);
    return (W == 64) ? b : ((b >> shift) & 0xffffffffull);
  };
  auto gmin = [&](int v) -> int {  // rows by DPP, then the 16 (and 32) lane steps
    v = row_reduce<16>(v, OpMin{});
    v = min(v, __shfl_xor(v, 16));
    if (W == 64) v = min(v, __shfl_xor(v, 32));
    return v;
  };
  const int64_t nc = *nc_count;
  // XCD-aware ranges of the (cell-ordered) queue: neighbouring points' windows share an L2
  const XcdRange xr = xcd_items((nc + P - 1) / P, true);
  for (int64_t qp = xr.first; qp < xr.end; qp += xr.step) {
    const int64_t q = qp * P + (lane / W);
    if (q >= nc) continue;  // (group-uniform)
    const int s = nc_list[q];
    const int32_t key = skey[s];
    int best = INT_MAX;
#ifdef RPT_AB
    bool st_core = false, st_search = false;
#endif
    if ((int64_t)key < g.cells) {
      const float4 p = pts[s];
      int cx, cy, cz;
      decode_key<D>(key, g, cx, cy, cz);
      const Window w = make_window<D, false>(cx, cy, cz, p.w, p.w, g, slab_t);
      // super-rounds of kR candidates per lane, loads of one kind issued together: the cells'
      // smallest keys (empty cells hold INT_MAX, so no occupancy lookup), then the records of
      // the cells with core points -- two dependent rounds per super-round
      for (int base = 0; base < w.total; base += W * kR) {
        int64_t c[kR];
        int ck[kR], cb[kR], ce[kR], cls[kR], mu[kR];
#pragma unroll
        for (int k = 0; k < kR; ++k) {
          const int qq = base + k * W + hl;
          c[k] = (qq < w.total) ? window_cell<D>(w, qq, g, slab_t, p.w, p.w) : -1;
        }
#pragma unroll
        for (int k = 0; k < kR; ++k) ck[k] = (c[k] >= 0) ? cell_key[c[k]] : INT_MAX;
        int v = INT_MAX;
#pragma unroll
        for (int k = 0; k < kR; ++k) {
          cb[k] = ce[k] = cls[k] = mu[k] = 0;
          if (ck[k] != INT_MAX) {
            const CellRec<D> cr = crec[c[k]];
            cb[k] = cr.b;
            ce[k] = cr.e;
            mu[k] = mutual[c[k]];
            cls[k] = classify<D>(p, rec_boxA<D>(cr), rec_boxB(cr), g);
            if (cls[k] == 1) v = min(v, ck[k]);
          }
        }
        best = min(best, gmin(v));
#ifdef RPT_AB
        {
          bool anyc = false;
#pragma unroll
          for (int k = 0; k < kR; ++k) anyc = anyc || ck[k] != INT_MAX;
          st_core = st_core || gbal(anyc) != 0;
        }
#endif
        // the partially reachable cells, smallest key first, while a key can still win
        uint32_t pend = 0;
#pragma unroll
        for (int k = 0; k < kR; ++k) pend |= (cls[k] == 2) ? (1u << k) : 0u;
        while (true) {
          int mine = INT_MAX, mk = -1;
#pragma unroll
          for (int k = 0; k < kR; ++k)
            if (((pend >> k) & 1u) && ck[k] < best && ck[k] < mine) {
              mine = ck[k];
              mk = k;
            }
          const int mm = gmin(mine);
          if (mm == INT_MAX) break;
#ifdef RPT_AB
          st_search = true;
#endif
          const uint64_t at = gbal(mine == mm);
          const int l = h0 + __ffsll((unsigned long long)at) - 1;
          const int kl = __shfl(mk, l);
          int bsel = 0, esel = 0, msel = 0;
#pragma unroll
          for (int k = 0; k < kR; ++k)
            if (k == kl) {
              bsel = cb[k];
              esel = ce[k];
              msel = mu[k];
            }
          if (lane == l) pend &= ~(1u << kl);
          const int bl = __shfl(bsel, l), el = __shfl(esel, l);
          // two points per lane per round (their loads issued together): a dense cell costs
          // half the dependent round trips
          if (__shfl(msel, l)) {  // one component: a single adjacent core point decides
            bool hit = false;
            for (int j0 = bl; j0 < el && !hit; j0 += 2 * W) {
              const int j = j0 + hl, j2 = j + W;
              const bool v1 = j < el, v2 = j2 < el;
              const int k1 = v1 ? key_of[j] : -1, k2 = v2 ? key_of[j2] : -1;
              const float4 p1 = v1 ? pts[j] : p, p2 = v2 ? pts[j2] : p;
              hit = gbal((k1 >= 0 && adjacent<D>(p, p1, g)) ||
                         (k2 >= 0 && adjacent<D>(p, p2, g))) != 0;
            }
            if (hit) best = mm;
          } else {
            int lb = INT_MAX;
            for (int j0 = bl; j0 < el; j0 += 2 * W) {
              const int j = j0 + hl, j2 = j + W;
              const bool v1 = j < el, v2 = j2 < el;
              const int m1 = v1 ? key_of[j] : -1, m2 = v2 ? key_of[j2] : -1;
              const float4 p1 = v1 ? pts[j] : p, p2 = v2 ? pts[j2] : p;
              if (m1 >= 0 && m1 < best && m1 < lb && adjacent<D>(p, p1, g)) lb = m1;
              if (m2 >= 0 && m2 < best && m2 < lb && adjacent<D>(p, p2, g)) lb = m2;
            }
            best = min(best, gmin(lb));
          }
        }
      }
    }
    if (hl == 0) {
      int32_t out = -1;
      if (best != INT_MAX) out = GLOBAL ? best : cid[best];
      labels[sorig[s]] = out;
#ifdef RPT_AB
      if (kstat) {
        atomicAdd(&kstat[0], 1);
        if (st_core) atomicAdd(&kstat[1], 1);
        if (st_search) atomicAdd(&kstat[2], 1);
        if (best != INT_MAX) atomicAdd(&kstat[3], 1);
      }
#endif
    }
  }
}

#ifdef RPT_AB
#include "stdbscan_ab.inc"
#endif

// Degenerate parameters (negative/NaN eps): nobody has a neighbour, not even itself.
__global__ __launch_bounds__(kBlock) void k_isolated_labels(int32_t* labels, int64_t n,
                                                           int singletons) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    labels[i] = singletons ? (int32_t)i : -1;
}

// Non-finite-time points are isolated; with min_samples <= 0 they are singleton clusters and
// flagged as their own component minimum (handled by k_ccmin via parent = self).

// ---------------------------------------------------------------- phased state (multi-GPU)
__global__ void k_core_to_orig(const uint8_t* __restrict__ core, const int32_t* __restrict__ sorig,
                               int64_t n, uint8_t* __restrict__ out) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n;
       s += (int64_t)gridDim.x * blockDim.x)
    out[sorig[s]] = core[s];
}
__global__ void k_core_from_orig(const uint8_t* __restrict__ in, const int32_t* __restrict__ sorig,
                                 int64_t n, uint8_t* __restrict__ core) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n;
       s += (int64_t)gridDim.x * blockDim.x)
    core[s] = in[sorig[s]] ? 1 : 0;
}
// comp[orig] = minimum original index of the point's core component, -1 for non-core; a core
// point of a mutual cell takes its cell's root (k_cell_roots: one load instead of a parent-chain
// walk per point)
__global__ void k_comp_out(int32_t* parent, const uint8_t* __restrict__ core,
                           const int32_t* __restrict__ sorig, int64_t n,
                           int32_t* __restrict__ comp, const int32_t* __restrict__ skey,
                           const int32_t* __restrict__ cell_root, int64_t cells) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n;
       s += (int64_t)gridDim.x * blockDim.x) {
    int32_t out = -1;
    if (core[s]) {
      const int32_t key = skey[s];
      const int32_t cr = ((int64_t)key < cells) ? cell_root[key] : -1;  // -1: not mutual
      out = sorig[cr >= 0 ? cr : uf_find(parent, (int)s)];
    }
    comp[sorig[s]] = out;
  }
}
// k_comp_out for the original indices outside [lo_end, hi_begin) only (the frame-sharded
// driver needs the component ids of its halo points and of its own edge points, not of the
// window's interior): every sorted point is read (one coalesced index load), only the edge
// points pay a root lookup and a scattered store
__global__ void k_comp_out_edges(int32_t* parent, const uint8_t* __restrict__ core,
                                 const int32_t* __restrict__ sorig, int64_t n,
                                 int32_t* __restrict__ comp, const int32_t* __restrict__ skey,
                                 const int32_t* __restrict__ cell_root, int64_t cells,
                                 int64_t lo_end, int64_t hi_begin) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n;
       s += (int64_t)gridDim.x * blockDim.x) {
    const int32_t i = sorig[s];
    if (i >= lo_end && i < hi_begin) continue;
    int32_t out = -1;
    if (core[s]) {
      const int32_t key = skey[s];
      const int32_t cr = (cell_root && (int64_t)key < cells) ? cell_root[key] : -1;
      out = sorig[cr >= 0 ? cr : uf_find(parent, (int)s)];
    }
    comp[i] = out;
  }
}
// Global labelling, core points: ccmin[s] = component-min original index; each component's
// label = rank of its global representative (rep[min], from the equivalence merge) among the
// sorted representatives -- one binary search per component, at its root; non-core queued.
__global__ __launch_bounds__(kBlock) void k_ccmin_global(int32_t* parent,
                                                        const uint8_t* __restrict__ core,
                                                        int64_t n,
                                                        const int32_t* __restrict__ sorig,
                                                        const int64_t* __restrict__ rep,
                                                        const int64_t* __restrict__ reps,
                                                        int64_t nr, int32_t* __restrict__ ccmin,
                                                        int32_t* __restrict__ gl,
                                                        int32_t* __restrict__ nc_list,
                                                        int32_t* __restrict__ nc_count,
                                                        const int32_t* __restrict__ skey = nullptr,
                                                        const uint8_t* __restrict__ mutual = nullptr,
                                                        const int32_t* __restrict__ cell_root = nullptr,
                                                        int64_t cells = 0,
                                                        const int64_t* __restrict__ nr_dev = nullptr) {
  if (nr_dev) nr = *nr_dev;  // the representative count stays on the device (shard driver)
  // level by level as in k_ccmin (keys + flags, cell roots, originals: branch-free loads, each
  // level's loads in flight together); only the parent-chain walk stays conditional
  for (int64_t tile = (int64_t)blockIdx.x * kBlock * kItems; tile < n;
       tile += (int64_t)gridDim.x * kBlock * kItems) {
    int32_t key[kItems], x[kItems];
    uint32_t cbits = 0, nbits = 0;
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int64_t s = tile + (int64_t)k * kBlock + threadIdx.x;
      const int64_t sc = min(s, n - 1);
      const int32_t kv = cell_root ? skey[sc] : -1;  // kernel-uniform pointer test
      const uint8_t cv = core[sc];
      const bool in = s < n;
      key[k] = in ? kv : -1;
      cbits |= (in && cv) ? (1u << k) : 0u;
      nbits |= (in && !cv) ? (1u << k) : 0u;  // non-core: queued for k_label
    }
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      x[k] = -1;
      if (cell_root) {  // core points of a mutual cell: their cell's root (k_cell_roots)
        const bool q = ((cbits >> k) & 1u) && key[k] >= 0 && (int64_t)key[k] < cells;
        const int32_t kk = q ? key[k] : 0;  // cells >= 1
        const uint8_t mu = mutual[kk];
        const int32_t cr = cell_root[kk];
        x[k] = (q && mu) ? cr : -1;
      }
    }
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int s = (int)(tile + (int64_t)k * kBlock + threadIdx.x);
      if (((cbits >> k) & 1u) && x[k] < 0) x[k] = uf_find(parent, s);
    }
    int m[kItems];
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const bool c = (cbits >> k) & 1u;
      const int32_t v = sorig[c ? x[k] : 0];
      m[k] = c ? v : -1;
    }
#pragma unroll
    for (int k = 0; k < kItems; ++k) {
      const int64_t s = tile + (int64_t)k * kBlock + threadIdx.x;
      if ((cbits >> k) & 1u) {
        ccmin[s] = m[k];
        if (x[k] == (int)s) gl[m[k]] = rep_id(reps, nr, rep[m[k]]);
      }
    }
    block_append_bits(tile, nbits, nc_list, nc_count);
  }
}
// The core labels in original order through the grid build's inverse permutation (spos, the
// slab buffer before k_label_global_core reuses it): whole-line label writes (k_label_core_orig)
__global__ __launch_bounds__(kBlock) void k_label_global_orig(const uint8_t* __restrict__ core,
                                                             const int32_t* __restrict__ ccmin,
                                                             const int32_t* __restrict__ gl,
                                                             const int32_t* __restrict__ spos,
                                                             int64_t n,
                                                             int32_t* __restrict__ labels) {
  const int64_t T = (n + (int64_t)kBlock * kPU - 1) / ((int64_t)kBlock * kPU);
  for (int64_t ti = blockIdx.x; ti < T; ti += gridDim.x) {
    const int64_t tile = ti * kBlock * kPU;
    int32_t sp[kPU], m[kPU];
    uint8_t c[kPU];
#pragma unroll
    for (int u = 0; u < kPU; ++u)  // branch-free (clamped)
      sp[u] = __builtin_nontemporal_load(spos + min(tile + (int64_t)u * kBlock + threadIdx.x,
                                                     n - 1));
#pragma unroll
    for (int u = 0; u < kPU; ++u) {
      c[u] = core[sp[u]];
      m[u] = ccmin[sp[u]];
    }
#pragma unroll
    for (int u = 0; u < kPU; ++u) {
      const int64_t i = tile + (int64_t)u * kBlock + threadIdx.x;
      if (i < n && c[u]) labels[i] = gl[m[u]];
    }
  }
}

// slab[s] = final label of core point s (-1 for non-core); core labels written out
// The core points' final labels (slab[s] = label, -1 for non-core) and, k_cell_min_key folded in,
// per cell the smallest label of its core points (cell_key pre-filled with INT_MAX): a segmented
// wave minimum over the sorted points, one atomic per cell run of a wave.
__global__ __launch_bounds__(kBlock) void k_label_global_core(const uint8_t* __restrict__ core,
                                                             const int32_t* __restrict__ ccmin,
                                                             const int32_t* __restrict__ gl,
                                                             const int32_t* __restrict__ sorig,
                                                             int64_t n,
                                                             int32_t* __restrict__ slab,
                                                             int32_t* __restrict__ labels,
                                                             const int32_t* __restrict__ skey,
                                                             int64_t cells,
                                                             int32_t* __restrict__ cell_key) {
  const int lane = threadIdx.x & 63;
  for (int64_t s0 = (int64_t)blockIdx.x * blockDim.x; s0 < n;
       s0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = s0 + threadIdx.x;
    int32_t l = -1, key = -1;
    if (s < n) {
      key = skey[s];
      if (core[s]) {
        l = gl[ccmin[s]];
        if (labels) labels[sorig[s]] = l;  // (kernel-uniform; null: k_label_global_orig's)
      }
      slab[s] = l;
    }
    int v = (l >= 0 && (int64_t)key < cells) ? l : INT_MAX;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int ov = __shfl_up(v, off, 64);
      const int ok = __shfl_up(key, off, 64);
      if (lane >= off && ok == key) v = min(v, ov);
    }
    const int next = __shfl_down(key, 1, 64);
    if ((lane == 63 || next != key) && key >= 0 && v != INT_MAX) atomicMin(cell_key + key, v);
  }
}

// ---------------------------------------------------------------- denoise variant (O8)
// PointCloudWorkF/stdbscan_denoising_pipeline.py:264-369.  A point is core when it has
// >= min_samples space-time neighbours (itself included, as K5) AND those neighbours span
// >= min_frames distinct int32(t) frames (:308-315); clusters are expanded with a FIFO queue that
// never re-queues a visited point (:346-363).  The component structure is K6's; only the core
// condition and the border rule differ (see k_label_fifo).
//
// Frames, cell level (every finite t integral: a slab is one frame): a cell whose column (same
// x, y) holds, in >= min_frames - 1 other slabs, a cell every point of which is a neighbour of
// every point of this cell (box test) has all its core points frame-complete.
__global__ __launch_bounds__(kBlock) void k_frames_cells(Geom g, int R,
                                                        const int32_t* __restrict__ occ,
                                                        const int32_t* __restrict__ n_occ,
                                                        const CellRec<2>* __restrict__ crec,
                                                        const uint32_t* __restrict__ occ_bits,
                                                        int min_frames,
                                                        uint8_t* __restrict__ fok) {
  const int64_t no = *n_occ;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < no;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int32_t ca = occ[q];
    if ((int64_t)ca >= g.cells) continue;  // non-finite time: settled per point
    int cx, cy, cz_, cs;
    g.split((uint32_t)ca, cx, cy, cz_, cs);
    const CellRec<2> ra = crec[ca];
    const float4 A1 = rec_boxA<2>(ra), B1 = rec_boxB(ra);
    int frames = 1;  // the cell's own
    const int s0 = max(cs - R, 0), s1 = min(cs + R, g.nt - 1);
    for (int sl = s0; sl <= s1 && frames < min_frames; ++sl) {
      if (sl == cs) continue;
      const int64_t c = ((int64_t)sl * g.ny + cy) * g.nx + cx;
      if (!((occ_bits[c >> 5] >> (c & 31)) & 1u)) continue;
      const CellRec<2> rc = crec[c];
      // (box A of both cells, then box B of both: classify_cells' argument order)
      frames += (classify_cells<2>(A1, rec_boxA<2>(rc), B1, rec_boxB(rc), g) == 1) ? 1 : 0;
    }
    fok[ca] = frames >= min_frames ? 1 : 0;
  }
}

// Queue of the core points whose frame count is still open; points of the isolated cell
// (non-finite t: no neighbour, 0 frames) are settled here.
__global__ __launch_bounds__(kBlock) void k_frames_queue(const int32_t* __restrict__ skey,
                                                        int64_t n, int64_t cells,
                                                        const uint8_t* __restrict__ fok,
                                                        int min_frames, int refine,
                                                        uint8_t* __restrict__ core,
                                                        int32_t* __restrict__ list,
                                                        int32_t* __restrict__ count) {
  for (int64_t tile = (int64_t)blockIdx.x * kBlock * kItems; tile < n;
       tile += (int64_t)gridDim.x * kBlock * kItems)
    block_append(
        tile, n,
        [&](int64_t s) -> bool {
          if (!core[s]) return false;
          const int32_t key = skey[s];
          if ((int64_t)key >= cells) {
            core[s] = (min_frames <= 0) ? 1 : 0;
            return false;
          }
          return refine && !(fok && fok[key]);
        },
        list, count);
}

// Frame count of one queued core point per wave: the int32(t) offsets (within +-31 of its own:
// |dt| <= eps_t <= 30, checked by the host) of its neighbours as a 64-bit set, scanned cell by
// cell until min_frames distinct frames are seen.
template <int D>
__global__ __launch_bounds__(kBlock) void k_frames_points(const float4* __restrict__ pts,
                                                         const int32_t* __restrict__ skey, Geom g,
                                                         const CellRec<D>* __restrict__ crec,
                                                         const uint32_t* __restrict__ occ_bits,
                                                         const float2* __restrict__ slab_t,
                                                         int integral, int min_frames,
                                                         const int32_t* __restrict__ list,
                                                         const int32_t* __restrict__ count,
                                                         uint8_t* __restrict__ core) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (int64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
  const int64_t nw = (int64_t)gridDim.x * (kBlock / 64);
  const int64_t nq = *count;
  for (int64_t q = w0; q < nq; q += nw) {
    const int s = list[q];
    const float4 p = pts[s];
    const int own = (int)p.w;  // numpy astype(int32): truncation toward zero
    int cx, cy, cz;
    decode_key<D>(skey[s], g, cx, cy, cz);
    const Window w = make_window<D, false>(cx, cy, cz, p.w, p.w, g, slab_t);
    uint64_t seen = 0;
    for (int base = 0; base < w.total && __popcll(seen) < min_frames; base += 64) {
      const int qq = base + lane;
      const int64_t c = (qq < w.total) ? window_cell<D>(w, qq, g, slab_t, p.w, p.w) : -1;
      int b = 0, e = 0, cls = 0;
      if (c >= 0 && ((occ_bits[c >> 5] >> (c & 31)) & 1u)) {
        const CellRec<D> cr = crec[c];
        b = cr.b;
        e = cr.e;
        cls = classify<D>(p, rec_boxA<D>(cr), rec_boxB(cr), g);
      }
      uint64_t pm = __ballot(cls != 0);
      while (pm && __popcll(seen) < min_frames) {
        const int l = __ffsll((unsigned long long)pm) - 1;
        pm &= pm - 1;
        const int bb = __shfl(b, l), cl = __shfl(cls, l);
        // a whole-cell hit in frame-id data is one frame: its first point says which
        const int ee = (cl == 1 && integral) ? bb + 1 : __shfl(e, l);
        for (int j0 = bb; j0 < ee && __popcll(seen) < min_frames; j0 += 64) {
          const int j = j0 + lane;
          uint64_t bit = 0;
          if (j < ee) {
            const float4 pj = pts[j];
            if (cl == 1 || adjacent<D>(p, pj, g))  // |t| >= 2^31 (saturating casts): clamped
              bit = 1ull << min(max((int)pj.w - own + 32, 0), 63);
          }
#pragma unroll
          for (int off = 32; off > 0; off >>= 1)
            bit |= (uint64_t)__shfl_xor((unsigned long long)bit, off);
          seen |= bit;
        }
      }
    }
    if (lane == 0) core[s] = (__popcll(seen) >= min_frames) ? 1 : 0;
  }
}

// numpy float32 -> int32 astype on x86-64: truncation; NaN / out of range -> INT32_MIN
__device__ __forceinline__ int32_t np_i32(float v) {
  if (!(v == v) || v >= 2147483648.f || v < -2147483648.f) return INT32_MIN;
  return (int32_t)v;
}

// The same frame count for any eps_t (k_frames_points' 64-bit offset set needs |dt| <= 30): the
// distinct int32(t) frames seen so far are a list spread over the wave, kFramesPerLane per lane
// (lane k holds entries k, k + 64, ...), appended one new frame at a time, so at most
// min_frames <= 64 * kFramesPerLane entries ever exist (the host checks the bound).
constexpr int kFramesPerLane = 4;
template <int D>
__global__ __launch_bounds__(kBlock) void k_frames_points_list(
    const float4* __restrict__ pts, const int32_t* __restrict__ skey, Geom g,
    const CellRec<D>* __restrict__ crec, const uint32_t* __restrict__ occ_bits,
    const float2* __restrict__ slab_t, int integral, int min_frames,
    const int32_t* __restrict__ list, const int32_t* __restrict__ count,
    uint8_t* __restrict__ core) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (int64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
  const int64_t nw = (int64_t)gridDim.x * (kBlock / 64);
  const int64_t nq = *count;
  for (int64_t q = w0; q < nq; q += nw) {
    const int s = list[q];
    const float4 p = pts[s];
    int cx, cy, cz;
    decode_key<D>(skey[s], g, cx, cy, cz);
    const Window w = make_window<D, false>(cx, cy, cz, p.w, p.w, g, slab_t);
    int32_t fr[kFramesPerLane];
#pragma unroll
    for (int k = 0; k < kFramesPerLane; ++k) fr[k] = 0;
    int nseen = 0;
    // v (this lane's candidate frame, valid when has): add it unless already listed
    auto add = [&](bool has, int32_t v) {
      bool fresh = has;
      // membership: compare against every listed entry (broadcast one register row at a time;
      // nseen is wave-uniform, so every lane runs every shuffle)
#pragma unroll
      for (int r = 0; r < kFramesPerLane; ++r) {
        if (r * 64 >= nseen) break;
        const int lim = min(nseen - r * 64, 64);
        for (int k = 0; k < lim; ++k) {
          const int32_t e = __shfl(fr[r], k);
          if (e == v) fresh = false;
        }
      }
      // append the distinct fresh values, lowest lane first
      uint64_t m = __ballot(fresh);
      while (m && nseen < min_frames) {
        const int l = __ffsll((unsigned long long)m) - 1;
        const int32_t nv = __shfl(v, l);
        const int r = nseen / 64, k = nseen % 64;
#pragma unroll
        for (int rr = 0; rr < kFramesPerLane; ++rr)
          if (rr == r && lane == k) fr[rr] = nv;
        ++nseen;
        if (fresh && v == nv) fresh = false;
        m = __ballot(fresh);
      }
    };
    for (int base = 0; base < w.total && nseen < min_frames; base += 64) {
      const int qq = base + lane;
      const int64_t c = (qq < w.total) ? window_cell<D>(w, qq, g, slab_t, p.w, p.w) : -1;
      int b = 0, e = 0, cls = 0;
      if (c >= 0 && ((occ_bits[c >> 5] >> (c & 31)) & 1u)) {
        const CellRec<D> cr = crec[c];
        b = cr.b;
        e = cr.e;
        cls = classify<D>(p, rec_boxA<D>(cr), rec_boxB(cr), g);
      }
      uint64_t pm = __ballot(cls != 0);
      while (pm && nseen < min_frames) {
        const int l = __ffsll((unsigned long long)pm) - 1;
        pm &= pm - 1;
        const int bb = __shfl(b, l), cl = __shfl(cls, l);
        // a whole-cell hit in frame-id data is one frame: its first point says which
        const int ee = (cl == 1 && integral) ? bb + 1 : __shfl(e, l);
        for (int j0 = bb; j0 < ee && nseen < min_frames; j0 += 64) {
          const int j = j0 + lane;
          bool has = false;
          int32_t v = 0;
          if (j < ee) {
            const float4 pj = pts[j];
            if (cl == 1 || adjacent<D>(p, pj, g)) {
              has = true;
              v = np_i32(pj.w);
            }
          }
          add(has, v);
        }
      }
    }
    if (lane == 0) core[s] = (nseen >= min_frames) ? 1 : 0;
  }
}

// spos[orig] = sorted position (when the grid build did not write it)
__global__ void k_inverse_perm(const int32_t* __restrict__ sorig, int64_t n,
                               int32_t* __restrict__ spos) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n;
       s += (int64_t)gridDim.x * blockDim.x)
    spos[sorig[s]] = (int32_t)s;
}

// Border labels of the FIFO expansion (:340-367).  Clusters are drained one after another in
// seed order, the seed being the component's minimum core index m (what ccmin holds).  A non-core
// point p (original index P) is popped by cluster m -- and keeps the first such label -- iff it is
// adjacent to a core point of m and either P > m (still unvisited when m's cores expand) or p is a
// neighbour of the seed itself (the seed's neighbour list is queued whole, visited or not, :343).
// Every qualifying m < P beats every m > P, so the first kind is a plain minimum and the second is
// resolved smallest-first with one seed test per distinct m.  One wave per non-core point.
template <int D>
__global__ __launch_bounds__(kBlock) void k_label_fifo(const float4* __restrict__ pts,
                                                      const int32_t* __restrict__ skey, Geom g,
                                                      const CellRec<D>* __restrict__ crec,
                                                      const uint32_t* __restrict__ occ_bits,
                                                      const float2* __restrict__ slab_t,
                                                      const int32_t* __restrict__ ccmin,
                                                      const int32_t* __restrict__ rep,
                                                      const int32_t* __restrict__ sorig,
                                                      const int32_t* __restrict__ spos,
                                                      MinRank cid,
                                                      const int32_t* __restrict__ nc_list,
                                                      const int32_t* __restrict__ nc_count,
                                                      int32_t* __restrict__ labels) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (int64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
  const int64_t nw = (int64_t)gridDim.x * (kBlock / 64);
  const int64_t nq = *nc_count;
  for (int64_t q = w0; q < nq; q += nw) {
    const int s = nc_list[q];
    const int P = sorig[s];
    const int32_t key = skey[s];
    int best_lt = INT_MAX, best_gt = INT_MAX;
    if ((int64_t)key < g.cells) {
      const float4 p = pts[s];
      int cx, cy, cz;
      decode_key<D>(key, g, cx, cy, cz);
      const Window w = make_window<D, false>(cx, cy, cz, p.w, p.w, g, slab_t);
      for (int base = 0; base < w.total; base += 64) {
        const int qq = base + lane;
        const int64_t c = (qq < w.total) ? window_cell<D>(w, qq, g, slab_t, p.w, p.w) : -1;
        int b = 0, e = 0, cls = 0;
        if (c >= 0 && ((occ_bits[c >> 5] >> (c & 31)) & 1u) && rep[c] >= 0) {
          const CellRec<D> cr = crec[c];
          b = cr.b;
          e = cr.e;
          cls = classify<D>(p, rec_boxA<D>(cr), rec_boxB(cr), g);
        }
        uint64_t pm = __ballot(cls != 0);
        while (pm) {
          const int l = __ffsll((unsigned long long)pm) - 1;
          pm &= pm - 1;
          const int bb = __shfl(b, l), ee = __shfl(e, l), cl = __shfl(cls, l);
          for (int j0 = bb; j0 < ee; j0 += 64) {
            const int j = j0 + lane;
            int m = -1;
            if (j < ee) {
              m = ccmin[j];
              if (m >= 0 && cl != 1 && !adjacent<D>(p, pts[j], g)) m = -1;
            }
            int lt = (m >= 0 && m < P) ? m : INT_MAX;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) lt = min(lt, __shfl_xor(lt, off));
            best_lt = min(best_lt, lt);
            if (best_lt != INT_MAX) continue;  // a smaller qualifying cluster is known
            // m > P: the smallest not yet rejected whose seed is a neighbour of p
            int cand = (m > P && m < best_gt) ? m : INT_MAX;
            while (true) {
              int mm = cand;
#pragma unroll
              for (int off = 32; off > 0; off >>= 1) mm = min(mm, __shfl_xor(mm, off));
              if (mm == INT_MAX) break;
              if (adjacent<D>(p, pts[spos[mm]], g)) {
                best_gt = mm;
                break;
              }
              if (cand == mm) cand = INT_MAX;
            }
          }
        }
      }
    }
    if (lane == 0) {
      const int best = (best_lt != INT_MAX) ? best_lt : best_gt;
      labels[P] = (best != INT_MAX) ? cid[best] : -1;
    }
  }
}

struct Timer {
  bool on = false;
  hipStream_t st{};
  hipEvent_t ev[8]{};
  int k = 0;
  void start(bool enable, hipStream_t s) {
    on = enable;
    st = s;
    k = 0;
    if (!on) return;
    for (auto& e : ev)
      if (!e) (void)hipEventCreate(&e);
    (void)hipEventRecord(ev[k++], st);
  }
  void mark() {
    if (on && k < 8) (void)hipEventRecord(ev[k++], st);
  }
  double ms(int i) {
    float t = 0;
    (void)hipEventElapsedTime(&t, ev[i], ev[i + 1]);
    return t;
  }
  ~Timer() {
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
  }
};

}  // namespace

// One ST-DBSCAN problem on one device, split in phases so that a frame-sharded multi-GPU run
// can exchange halo core flags and component ids between them.  Owns its device memory.
struct DbscanState {
  Scratch arena;
  int dim = 2;
  int64_t n = 0;
  bool degenerate = false;  // negative/NaN eps: no pair passes, not even (i, i)
  int32_t min_samples = 0;
  Geom g{};
  int64_t C = 0, nt = 0;
  float4* pts = nullptr;
  int32_t *sorig = nullptr, *skey = nullptr, *cell_start = nullptr, *rep = nullptr;
  uint8_t *mutual = nullptr, *core = nullptr;
  float2* slab_t = nullptr;
  int32_t *parent = nullptr, *ccmin = nullptr, *cid = nullptr, *nc_list = nullptr;
  int32_t *occ = nullptr, *hpos = nullptr;  // occupied cells (ascending), head-flag scan
  const int32_t* n_occ_dev = nullptr;        // the occupied-cell count (hpos[n] or the slab scan's)
  uint64_t* cell_min_pair = nullptr;         // per cell (min core original index, its sorted index)
  bool cmin_ready = false;  // cell_min_pair filled by the core pass for the current core flags
  void* crec = nullptr;                      // CellRec<dim>[C + 1]
  uint32_t* occ_bits = nullptr;              // 1 bit per cell
  uint4* pmask = nullptr;  // union passes' undecided-candidate masks per occupied cell (aliases
                           // the grid build's radix key buffers, dead after the build)
  int union_list = -1;     // RPT_UNION_LIST=0: the second union pass enumerates every window
  int union_pair = -1;     // RPT_UNION_PAIR=0: one cell per wave in the box-certain union pass
  int union_nm = -1;       // RPT_UNION_NM=0: k_union over every point (not the listed cells')
  // occupied cells per wave iteration of k_union_cells_pair: 64 on large stacks (one header load
  // per lane), 16 on small ones (RPT_UNION_CPW in the A/B build)
  int union_cpw() const {
    const char* e = ab_env("RPT_UNION_CPW");
    const int v = e ? std::atoi(e) : 0;
    if (v >= 1 && v <= 64) return v;
    return n > (int64_t(1) << 24) ? 64 : 16;
  }
  int uf_compress = -1;    // RPT_UF_COMPRESS=1: a compression pass closes the union stage
  uint32_t* min_bits = nullptr;  // component minima, 1 bit per original index (MinRank)
  int32_t* min_pref = nullptr;   // exclusive popcount prefix of min_bits' words (+ total)
  int64_t min_words() const { return n / 32 + 1; }
  int32_t* n_clusters_ptr() const { return min_pref + min_words(); }
  int32_t cluster_ids(hipStream_t st, int32_t* cell_key, int32_t* zero = nullptr);
  int32_t* cell_root = nullptr;  // per cell: root of a mutual cell's core points (k_cell_roots)
  int uf_flags = -1;                         // see XcdRange; -1 = read RPT_UF_FLAGS once
  int k5_legacy = -1;                        // 1: round-1 K5 (fill + point queue); RPT_K5_MODE
  int k5_fill = 0;
  int k5_fused = -1;                         // 0: separate level-3 fill pass; RPT_K5_FUSED
  bool bucket_allmin = false;  // this build's cell minima came from k_slab_bucket
  void k5_env() {
    if (k5_legacy < 0) {  // RPT_K5_MODE: 0 round-1 queue pipeline, 1 cells write point flags,
                          // 2 cells + point-flag fill (no queue); both 1/2 end in k_core_slow_cells
      // default 0: the folded variants measured no faster on the 100- and 1000-frame stacks
      // (profiles/r2/ab_k5_k1.md): the per-point flag writes moved into the cell kernel by 8 lanes
      // per cell cost what the fill pass cost, and the cell-wise slow pass balances worse than the
      // point queue
      const char* e = ab_env("RPT_K5_MODE");
      k5_legacy = e ? std::atoi(e) : 0;
      k5_legacy = (k5_legacy == 0) ? 1 : 0;
      k5_fill = (e && std::atoi(e) == 2) ? 1 : 0;
    }
    if (k5_tiles < 0) {  // RPT_K5_TILES=1: the LDS-tile pass (k_core_tiles; measured slower)
      const char* e = ab_env("RPT_K5_TILES");
      k5_tiles = (e && std::atoi(e) == 1) ? 1 : 0;
    }
    if (k5_fused < 0) {  // RPT_K5_FUSED=0: the separate level-3 fill pass (A/B)
      const char* e = ab_env("RPT_K5_FUSED");
      k5_fused = (e && std::atoi(e) == 0) ? 0 : 1;
    }
  }
  // the default K5 pipeline: the cell pass writes the point flags and the queue itself, with the
  // all-core cells' minima from k_cell_box (decided at build time, before k_cell_box runs)
  int k5_mask_ = -1;  // 0: the slow pass re-classifies every window (k_core_slow); RPT_K5_MASK
  bool k5_mask() {
    if (k5_mask_ < 0) {
      const char* e = ab_env("RPT_K5_MASK");
      k5_mask_ = (e && std::atoi(e) == 0) ? 0 : 1;
    }
    return k5_mask_ == 1;
  }
  bool k5_fused_path() {
    k5_env();
    return oct_ok() && k5_legacy && k5_fused && !k5_tiles;
  }
  int k5_tiles = -1;                         // 1: K5 by LDS tiles (k_core_tiles); RPT_K5_TILES
  int k7_tiles = -1;                         // 1: K7 by LDS tiles (k_label_tiles); RPT_K7_TILES
  int32_t* rowq = nullptr;    // first occupied-list index of every (slab, row) + total (tiles)
  int32_t* rowcnt = nullptr;  // occupied cells per (slab, row)
  bool rowq_ok = false;       // rowq built for this grid (the core pass's tile path)
  int tile_by = 0, tile_nbands = 0, tile_R = 0;
  // the label pass on the core pass's tiles (rowq built, RPT_K7_TILES not 0)
  bool use_label_tiles() {
    if (k7_tiles < 0) {  // RPT_K7_TILES=1 (measured slower than k_label, see k_core_tiles)
      const char* e = ab_env("RPT_K7_TILES");
      k7_tiles = (e && std::atoi(e) == 1) ? 1 : 0;
    }
    return k7_tiles && rowq_ok && dim == 2 && g.nz == 1;
  }
  unsigned tile_grid_blocks() const {  // the tiles + the isolated cell's, a multiple of 8
    return (unsigned)((((int64_t)g.nt * tile_nbands + 1) + 7) & ~(int64_t)7);
  }
  // slabs each side a cell's points can reach: eps_t / slab width, +1 for the slab's extent;
  // integral times with integral slab widths: a slab holds whole time values, so ceil(floor(eps_t)
  // / width) slabs each side hold every time within eps_t
  double slab_reach() const {
    return integral_t ? std::ceil(std::floor((double)g.epst) / g.ct)
                      : std::ceil((double)g.epst / g.ct) + 1.0;
  }
  // the eight-lanes-per-cell K5 / K6 kernels (2-D, at most kCwMaxR slabs each side)
  bool oct_ok() const { return dim == 2 && g.nz == 1 && slab_reach() <= (double)kCwMaxR; }
  int k7_w = -1;  // lanes per non-core point in k_label (32: two points per wave); RPT_K7_W
  int label_w() {
    if (k7_w < 0) {
      const char* e = ab_env("RPT_K7_W");
      k7_w = (e && std::atoi(e) == 64) ? 64 : 32;
    }
    return k7_w;
  }
  int bucket_mode = -1;                      // RPT_K4_BUCKET (default 1): slab-bucket K4
  template <int D>
  const CellRec<D>* rec() const {
    return static_cast<const CellRec<D>*>(crec);
  }
  // per original point: its sorted position (the grid build's inverse permutation, read by the
  // label passes, when spos_on); the global path then reuses it for the sorted points' final
  // core labels
  int32_t* slab = nullptr;
  bool spos_on = false;
  bool dense_slabs = false;  // more than 8 kChunkPts points per slab on average (bucket path)
  int32_t* cell_min = nullptr;  // per cell: smallest component key (label pass)
  uint8_t* fok = nullptr;    // per cell: frame condition met by every core point (denoise)
  bool integral_t = false;   // every finite t integral (slab = one frame id)
  int64_t* stmp = nullptr;
  Timer tm;

  template <int D>
  int32_t build_t(const float* x, const float* y, const float* z, int64_t stride, const float* t,
                  double eps_space, double eps_time, hipStream_t st);
  const void* given_bounds = nullptr;  // host Bounds computed by the caller (stdbscan_bounds_dev)
  int32_t build(const float* x, const float* y, const float* z, int64_t stride, const float* t,
                int64_t n_, double eps_space, double eps_time, int32_t ms, bool timing,
                hipStream_t st);
  int32_t core_pass(hipStream_t st);
  int32_t union_pass(hipStream_t st);
  int32_t labels_local(int32_t* labels, rpt_stdbscan_stats* stats, hipStream_t st);
  // deferred mode: labels_local leaves the cluster count on the device (cid[n]) and the timing
  // events unread; fill_stats completes the stats once the caller has synchronised the stream
  bool defer = false;
  int32_t fill_stats(int32_t n_clusters, rpt_stdbscan_stats* stats);
  int32_t labels_global(const int64_t* rep_orig, const int64_t* reps, int64_t nr,
                        int32_t* labels, hipStream_t st, const int64_t* nr_dev = nullptr);
  // denoise variant: the min_frames core condition, then the FIFO border labels
  int32_t frames_pass(int32_t min_frames, hipStream_t st);
  int32_t labels_fifo(int32_t* labels, rpt_stdbscan_stats* stats, hipStream_t st);
};

template <int D>
int32_t DbscanState::build_t(const float* x, const float* y, const float* z, int64_t stride,
                             const float* t, double eps_space, double eps_time, hipStream_t st) {
  const int gb = grid_for(n, kBlock, 2048);
  // ---- bounds (one small sync); the arena is re-reserved below, so copy results out first
  const int nbb = grid_for(n, kBlock, 1024);
  {
    Budget bb;
    bb.add<Bounds>(1);
    bb.add<Bounds>(nbb);
    RPT_TRY(arena.reserve(bb.bytes, st));
  }
  Bounds* d_b = arena.carve_n<Bounds>(1);
  Bounds* d_part = arena.carve_n<Bounds>(nbb);
  Bounds hb;
  if (given_bounds) {  // the caller read them back with its own results
    std::memcpy(&hb, given_bounds, sizeof(Bounds));
  } else {
    hipLaunchKernelGGL(k_bounds<D>, dim3(nbb), dim3(kBlock), 0, st, x, y, z, stride, t, n,
                       d_part, (const int64_t*)nullptr);
    hipLaunchKernelGGL(k_bounds_final, dim3(1), dim3(kBlock), 0, st, d_part, nbb, d_b);
    RPT_CHECK_LAUNCH();
    RPT_HIP(hipMemcpyAsync(&hb, d_b, sizeof(Bounds), hipMemcpyDeviceToHost, st));
    RPT_TRY(wait_stream(st));
  }
  tm.mark();
  if (hb.nonfinite_xyz) {
    set_error("Input contains NaN or infinity in coordinates");
    return RPT_ENONFINITE;
  }
  const float epst = (float)eps_time;
  g = Geom{};
  g.eps2 = eps_space * eps_space;
  g.epst = epst;
  static const bool screen_on = [] {
    const char* e = ab_env("RPT_F32_SCREEN");
    return !(e && e[0] == '0');
  }();
  const bool screen = screen_on && g.eps2 >= 1e-20 && g.eps2 <= 1e30;
  g.e2lo = screen ? (float)(g.eps2 * (1.0 - 1e-5)) : -1.0f;
  g.e2hi = screen ? (float)(g.eps2 * (1.0 + 1e-5)) : INFINITY;
  g.min_samples = min_samples;
  double lo[4], hi[4];
  for (int k = 0; k < 4; ++k) {
    lo[k] = (double)ord2f(hb.mn[k]);
    hi[k] = (double)ord2f(hb.mx[k]);
  }
  if (hb.n_finite_t == 0) lo[3] = hi[3] = 0.0;
  integral_t = !hb.nonintegral_t;
  const double margin = 1.0 + 1.0 / 1048576.0;  // 2^-20
  // cell side: >= eps/2 keeps every neighbour within +-2 cells; in 2-D up to eps/sqrt(2) keeps a
  // full cell's diagonal within eps (mutual cells possible), and larger cells hold more points,
  // so more of them are decided whole: 0.7 eps in 2-D (1000-frame stack 12.86 -> 12.41 ms, the
  // dense share's K5 0.66 -> 0.84 of roofline, same box); RPT_CELL_SIDE overrides (0.5 - 0.7)
  static const double side_f = [] {
    const char* e = ab_env("RPT_CELL_SIDE");
    const double v = e ? std::atof(e) : 0.0;
    return (v >= 0.5 && v <= 0.7) ? v : 0.7;
  }();
  const double sf = (D == 2) ? side_f : 0.5;
  double cs = (eps_space > 0.0 ? eps_space * sf : 1.0) * margin;
  double ct = !hb.nonintegral_t ? 1.0 : (epst > 0.f ? (double)epst : 1.0) * margin;
  const int64_t cmax = std::min<int64_t>(std::max<int64_t>(int64_t(1) << 22, 4 * n),
                                         int64_t(1) << 30);
  auto dims = [&](double ext, double side) -> int64_t {
    const double q = floor(ext / side) + 1.0;
    return q > 1e9 ? (int64_t)1e9 : (int64_t)q;
  };
  int64_t nx = 1, ny = 1, nz = 1;
  for (int it = 0; it < 200; ++it) {
    nx = dims(hi[0] - lo[0], cs);
    ny = dims(hi[1] - lo[1], cs);
    nz = (D == 3) ? dims(hi[2] - lo[2], cs) : 1;
    nt = dims(hi[3] - lo[3], ct);
    if ((double)nx * ny * nz * nt <= (double)cmax) break;
    if ((double)nt > (double)nx * ny * nz)
      ct *= 2.0;
    else
      cs *= 2.0;
  }
  g.ox = lo[0];
  g.oy = lo[1];
  g.oz = lo[2];
  g.ot = lo[3];
  g.cs = cs;
  g.ct = ct;
  g.inv_cs = 1.0 / cs;
  g.inv_ct = 1.0 / ct;
  g.nx = (int)nx;
  g.ny = (int)ny;
  g.nz = (int)nz;
  g.nt = (int)nt;
  g.cells = nx * ny * nz * nt;
  g.fnx.init((uint32_t)nx);
  g.fny.init((uint32_t)ny);
  g.fnz.init((uint32_t)nz);
  g.fslab.init((uint32_t)(nx * ny * nz));
  {
    const double r = slab_reach();  // (infinite for an infinite eps_time: generic windows)
    g.rt = (integral_t && r < 1e9) ? (int)std::min(r, (double)nt) : -1;
    g.tfree = (g.rt >= 0 && ct == 1.0 && (double)g.rt <= std::floor((double)epst)) ? 1 : 0;
  }
  C = g.cells;
  const int64_t C1 = C + 1;  // + the isolated cell (non-finite t)
  Budget bud;
  bud.add<Bounds>(1);
  for (int k = 0; k < 4; ++k) bud.add<uint32_t>(n);  // keys, vals, alt
  bud.add<int64_t>(radix_tmp_elems(n));
  bud.add<float4>(n);
  bud.add<int32_t>(n);       // sorig
  bud.add<int32_t>(n);       // skey
  bud.add<int32_t>(C1 + 1);  // cell_start
  bud.add<int64_t>(scan_tmp_elems(C1 + 1) + scan_tmp_elems(n + 1));
  bud.add<uint8_t>(C1);
  bud.add<int32_t>(C1);  // rep
  bud.add<float2>(nt);
  bud.add<uint8_t>(n);      // core
  bud.add<int32_t>(n);      // parent
  bud.add<int32_t>(n);      // ccmin
  bud.add<int32_t>(n + 1);  // cid
  bud.add<int32_t>(n + 1);  // non-core list (+count)
  bud.add<int32_t>(n);      // slab (global finalize; denoise: orig -> sorted)
  bud.add<uint8_t>(C1);     // fok (denoise)
  bud.add<int32_t>(C1);     // cell_min
  bud.add<int32_t>(C1);     // cell_root
  bud.add<uint64_t>(C1);    // cell_min_pair (union star initialisation)
  bud.add<uint32_t>(n / 32 + 1);  // min_bits
  bud.add<int32_t>(n / 32 + 2);   // min_pref
  bud.add<int32_t>(n + 1);  // occ
  bud.add<int32_t>(n + 1);  // hpos
  bud.add<CellRec<D>>(C1);  // crec
  bud.add<uint32_t>(C1 / 32 + 2);  // occupancy bits
  bud.add<int32_t>(nt + 1);        // slab_lo (slab-bucket path)
  bud.add<int32_t>(nt + 1);        // slab_occ (slab-bucket path)
  bud.add<int32_t>(nt + 1);        // occ_base (slab-bucket path)
  bud.add<int32_t>((size_t)(ny * nz * nt) + 1);  // rowq (LDS-tile passes)
  bud.add<int32_t>((size_t)(ny * nz * nt) + 1);  // row counts
  RPT_TRY(arena.reserve(bud.bytes, st));
  (void)arena.carve_n<Bounds>(1);
  uint32_t* keys = arena.carve_n<uint32_t>(n);
  uint32_t* vals = arena.carve_n<uint32_t>(n);
  uint32_t* keys_alt = arena.carve_n<uint32_t>(n);
  uint32_t* vals_alt = arena.carve_n<uint32_t>(n);
  pmask = reinterpret_cast<uint4*>(keys);  // 4 x n u32, contiguous: room for n_occ <= n masks
  int64_t* rtmp = arena.carve_n<int64_t>(radix_tmp_elems(n));
  pts = arena.carve_n<float4>(n);
  sorig = arena.carve_n<int32_t>(n);
  skey = arena.carve_n<int32_t>(n);
  cell_start = arena.carve_n<int32_t>(C1 + 1);
  stmp = arena.carve_n<int64_t>(scan_tmp_elems(C1 + 1) + scan_tmp_elems(n + 1));
  mutual = arena.carve_n<uint8_t>(C1);
  rep = arena.carve_n<int32_t>(C1);
  slab_t = arena.carve_n<float2>(nt);
  core = arena.carve_n<uint8_t>(n);
  parent = arena.carve_n<int32_t>(n);
  ccmin = arena.carve_n<int32_t>(n);
  cid = arena.carve_n<int32_t>(n + 1);
  nc_list = arena.carve_n<int32_t>(n + 1);
  slab = arena.carve_n<int32_t>(n);
  fok = arena.carve_n<uint8_t>(C1);
  cell_min = arena.carve_n<int32_t>(C1);
  cell_root = arena.carve_n<int32_t>(C1);
  cell_min_pair = arena.carve_n<uint64_t>(C1);
  min_bits = arena.carve_n<uint32_t>(n / 32 + 1);
  min_pref = arena.carve_n<int32_t>(n / 32 + 2);
  occ = arena.carve_n<int32_t>(n + 1);
  hpos = arena.carve_n<int32_t>(n + 1);
  CellRec<D>* cr = arena.carve_n<CellRec<D>>(C1);
  crec = cr;
  occ_bits = arena.carve_n<uint32_t>(C1 / 32 + 2);  // +1: two-word window reads
  int32_t* slab_lo = arena.carve_n<int32_t>(nt + 1);
  int32_t* slab_occ = arena.carve_n<int32_t>(nt + 1);
  int32_t* occ_base = arena.carve_n<int32_t>(nt + 1);
  rowq = arena.carve_n<int32_t>((size_t)(ny * nz * nt) + 1);
  rowcnt = arena.carve_n<int32_t>((size_t)(ny * nz * nt) + 1);
  rowq_ok = false;
  if (!slab_lo || !rowcnt) {
    set_error("internal: scratch carve overflow");
    return RPT_ENOMEM;
  }
  if (bucket_mode < 0) {
    const char* e = ab_env("RPT_K4_BUCKET");
    bucket_mode = (e && std::atoi(e) == 0) ? 0 : 1;
  }
  // time-ordered finite 2-D points with a slab's cells fitting LDS: per-slab counting sort
  bucket_allmin = false;
  const bool bucket = bucket_mode && D == 2 && hb.n_finite_t == n && !hb.t_descends &&
                      (int64_t)nx * ny <= kBucketCells && nt < (int64_t(1) << 31);
  if (bucket) {
    hipLaunchKernelGGL(k_slab_lo, dim3(grid_for(64 * (nt + 1), kBlock, 4096)), dim3(kBlock), 0,
                       st, t, n, g, slab_lo, occ_bits, (int64_t)(C1 / 32 + 2));
    // the slabs write their occupied cells (ascending) into hpos at their point offsets, the
    // occupancy bits and their counts; one scan over the slabs and a gather give the list
    const size_t hist_bytes = sizeof(int32_t) * (size_t)nx * ny;
    // blocks per slab (measured, same box): dense slabs (> 128 k points) split into ~kChunkPts
    // point chunks (configs[4] share: grid 2.93 -> 2.04 ms); short stacks split until ~512 blocks
    // fill the GPU (125 frames: 0.193 -> 0.177 ms); 1000 standard slabs stay one block each
    // (three chunks measured 1.10 -> 1.25 ms).  The chunk histograms live in the radix key
    // buffers (4 n words, dead on this path).
    const int64_t avg = n / std::max<int64_t>(nt, 1);
    // dense slabs: the label passes' scattered core-label writes cost more than the inverse
    // permutation written here (configs[4] share: 676 -> 253 us for +57 in the scatter; at
    // standard density the scattered writes stay in L2 and the extra store costs +68 us)
    dense_slabs = avg > 8 * kChunkPts;
    spos_on = label_core_orig() == 2 || (label_core_orig() == 1 && dense_slabs);
    int32_t* spos_w = spos_on ? slab : nullptr;
    int64_t ch = avg > 8 * kChunkPts ? (avg + kChunkPts - 1) / kChunkPts : 1;
    ch = std::max<int64_t>(ch, (512 + nt - 1) / std::max<int64_t>(nt, 1));
    int CH = (int)std::min<int64_t>(ch, 64);
    while (CH > 1 && (int64_t)nt * CH * nx * ny > 4 * n) --CH;
    if (slab_chunks_override() > 0) CH = slab_chunks_override();
    const bool coalesced_scan = CH >= 8 && (int64_t)nt * CH * nx * ny <= 4 * n &&
                                !chunk_scan_legacy();
    if (CH > 1 && (int64_t)nt * CH * nx * ny <= 4 * n) {
      int32_t* hist_g = reinterpret_cast<int32_t*>(keys);
      // the coalesced passes pay for their extra launches only with many chunks per slab (dense
      // slabs: configs[4] share 357 -> 115 us); a few chunks per slab (short standard stacks,
      // split to fill the GPU) keep the one-block-per-slab scan (125 frames: 38 vs 53 us)
      RPT_HIP(hipFuncSetAttribute((const void*)k_slab_chunk_hist,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)hist_bytes));
      RPT_HIP(hipFuncSetAttribute((const void*)k_slab_chunk_scatter,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)hist_bytes));
      hipLaunchKernelGGL(k_slab_chunk_hist, dim3((unsigned)(nt * CH)), dim3(kBucketBlock),
                         hist_bytes, st, x, y, stride, g, slab_lo, CH, hist_g);
      if (!coalesced_scan) {
        hipLaunchKernelGGL(k_slab_chunk_scan, dim3((unsigned)nt), dim3(kBucketBlock), 0, st, g,
                           slab_lo, CH, hist_g, cell_start, hpos, slab_occ, occ_bits);
      } else {
        // cell_start, cursors, occupancy from coalesced passes; the flags and their positions in
        // cell_min / cell_root (C1 words each, first written after the grid build)
        const int64_t cells = (int64_t)nt * nx * ny;
        const int P = (int)(nx * ny);
        const int gc = grid_for(cells, kBlock, 8192);
        hipLaunchKernelGGL(k_chunk_totals, dim3(gc), dim3(kBlock), 0, st, hist_g, cells, P, CH,
                           cell_start);
        RPT_TRY(exclusive_scan_total_i32(cell_start, cell_start, cells, st));
        hipLaunchKernelGGL(k_chunk_cursors, dim3(gc), dim3(kBlock), 0, st, hist_g, cells, P, CH,
                           cell_start, slab_lo, occ_bits, cell_min);
        RPT_TRY(exclusive_scan_total_i32(cell_min, cell_root, cells, st));
        hipLaunchKernelGGL(k_occ_write, dim3(gc), dim3(kBlock), 0, st, cell_min, cell_root,
                           cells, occ);
        hipLaunchKernelGGL(k_cell_start_end, dim3(1), dim3(64), 0, st, cell_start, cells);
        hipLaunchKernelGGL(k_slab_occ_base, dim3(grid_for(nt + 1, kBlock, 1024)), dim3(kBlock), 0,
                           st, cell_root, P, nt, occ_base);
        RPT_CHECK_LAUNCH();
      }
      hipLaunchKernelGGL(k_slab_chunk_scatter, dim3((unsigned)(nt * CH)), dim3(kBucketBlock),
                         hist_bytes, st, x, y, stride, t, g, slab_lo, CH, hist_g, pts, sorig,
                         skey, spos_w);
    } else {
      // the fused K5's all-core cell minima from the counting sort when both LDS arrays fit 64 KiB
      bucket_allmin = k5_fused_path() && 2 * hist_bytes <= 65536 &&
                      ab_mode("RPT_BUCKET_ALLMIN") != 0;  // (=0: from k_cell_box; A/B)
      const size_t lds = bucket_allmin ? 2 * hist_bytes : hist_bytes;
      RPT_HIP(hipFuncSetAttribute((const void*)k_slab_bucket,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
#ifdef RPT_AB
      if (ab_env("RPT_STATS")) {  // A/B diagnostics: blocks per CU the runtime admits
        int nb = -1;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_slab_bucket, kBucketBlock, lds);
        std::fprintf(stderr, "[rpt stats] slab_bucket lds=%zu nx=%d ny=%d blocks_per_cu=%d\n", lds,
                     (int)nx, (int)ny, nb);
      }
#endif
      hipLaunchKernelGGL(k_slab_bucket, dim3((unsigned)nt), dim3(kBucketBlock), lds, st, x, y,
                         stride, t, g, slab_lo, pts, sorig, skey, spos_w, cell_start, hpos,
                         slab_occ,
                         occ_bits,
                         bucket_allmin ? reinterpret_cast<unsigned long long*>(cell_min_pair)
                                       : nullptr);
    }
    RPT_CHECK_LAUNCH();
    if (coalesced_scan) {
      n_occ_dev = occ_base + nt;  // the occupied list is written already
    } else {
      RPT_TRY(exclusive_scan_total_i32(slab_occ, occ_base, nt, st));
      hipLaunchKernelGGL(k_occ_gather, dim3((unsigned)nt), dim3(kBlock), 0, st, hpos, slab_lo,
                         occ_base, occ);
      RPT_CHECK_LAUNCH();
      n_occ_dev = occ_base + nt;
    }
  } else {
    hipLaunchKernelGGL(k_keys<D>, dim3(gb), dim3(kBlock), 0, st, x, y, z, stride, t, n, g, keys,
                       vals);
    RPT_CHECK_LAUNCH();
    int bits = 1;
    while ((int64_t(1) << bits) <= C1) ++bits;
    uint32_t *sk, *sv;
    RPT_TRY(radix_sort_pairs(keys, vals, keys_alt, vals_alt, n, bits, rtmp, &sk, &sv, st));
    dense_slabs = false;
    spos_on = label_core_orig() == 2;
    hipLaunchKernelGGL(k_gather<D>, dim3(gb), dim3(kBlock), 0, st, x, y, z, stride, t, n, sk, sv,
                       pts, sorig, skey, spos_on ? slab : nullptr);
    RPT_HIP(hipMemsetAsync(cell_start, 0, sizeof(int32_t) * C1, st));
    hipLaunchKernelGGL(k_cell_runs, dim3(gb), dim3(kBlock), 0, st, skey, n, cell_start, hpos);
    RPT_CHECK_LAUNCH();
    RPT_TRY(exclusive_scan_total_i32(cell_start, cell_start, C1, st));
    RPT_TRY(exclusive_scan_total_i32(hpos, hpos, n, st));
    RPT_HIP(hipMemsetAsync(occ_bits, 0, sizeof(uint32_t) * (C1 / 32 + 2), st));
    hipLaunchKernelGGL(k_occ_list, dim3(gb), dim3(kBlock), 0, st, skey, n, hpos, occ, occ_bits);
    RPT_CHECK_LAUNCH();
    n_occ_dev = hpos + n;
  }
  {
    auto* cmin_w = bucket_allmin ? nullptr : reinterpret_cast<unsigned long long*>(cell_min_pair);
    const int32_t* so_w = (k5_fused_path() && !bucket_allmin) ? (const int32_t*)sorig : nullptr;
    // small cells one lane each on large standard-density stacks (1000 frames: 346 -> 273 us);
    // the 125-frame share has too few 64-cell waves to fill the GPU (48 -> 60 us) and dense
    // slabs' cells are large (324 -> 402 us): 16 lanes for every cell there
    // (RPT_CELL_BOX_MIXED=0 in the A/B build: always)
    if (cell_box_mixed() == 2 ||
        (cell_box_mixed() == 1 && !dense_slabs && n > (int64_t(1) << 24)))
      hipLaunchKernelGGL(k_cell_box_mixed<D>, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock), 0, st,
                         pts, cell_start, occ, n_occ_dev, g, mutual, cr, cmin_w, so_w);
    else
      hipLaunchKernelGGL(k_cell_box<D>, dim3(grid_for(kCbLanes * n, kBlock, 8192)), dim3(kBlock),
                         0, st, pts, cell_start, occ, n_occ_dev, g, mutual, cr, cmin_w, so_w);
  }
  RPT_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_slab_range<D>, dim3((unsigned)nt), dim3(kBlock), 0, st, cr, occ, hpos,
                     cell_start, (int64_t)(C / nt), (int)nt, slab_t, bucket ? occ_base : nullptr);
  RPT_CHECK_LAUNCH();
  tm.mark();
  return RPT_OK;
}

int32_t DbscanState::build(const float* x, const float* y, const float* z, int64_t stride,
                           const float* t, int64_t n_, double eps_space, double eps_time,
                           int32_t ms, bool timing, hipStream_t st) {
  n = n_;
  dim = z ? 3 : 2;
  min_samples = ms;
  tm.start(timing, st);
  degenerate = !(eps_space >= 0.0) || !((float)eps_time >= 0.0f);
  if (degenerate) return RPT_OK;
  return dim == 2 ? build_t<2>(x, y, z, stride, t, eps_space, eps_time, st)
                  : build_t<3>(x, y, z, stride, t, eps_space, eps_time, st);
}

int32_t DbscanState::core_pass(hipStream_t st) {
  cmin_ready = false;
  if (degenerate) return RPT_OK;
  // cflag lives in rep (int32 per cell, rebuilt by union_pass); the cell queue in ccmin and the
  // point queue in nc_list (both rebuilt later), counters in cid[n] / nc_list[n]
  int32_t* cflag = rep;
  int32_t* cq = ccmin;
  int32_t* n_cq = cid + n;
  int32_t* slow = nc_list;
  int32_t* n_slow = nc_list + n;
  const int32_t* n_occ = n_occ_dev;
  k5_env();
  const double rs = slab_reach();
  const bool oct = oct_ok();
#ifdef RPT_AB  // A/B-only forms (stdbscan_ab.inc)
  if (oct && k5_tiles) {
    // LDS tiles: band height BY with the map (W slabs x BY + 4 rows x nx) and the undecided list
    // (BY x nx own cells) within their LDS arrays; rowq (kept for the label pass's tiles)
    const int R = (int)rs, W = 2 * R + 1;
    const int by = std::min({8, kTileMap / (W * g.nx) - 4, kTileUnd / g.nx});
    const int64_t nrows = (int64_t)g.nt * g.ny;
    if (by >= 1) {
      hipLaunchKernelGGL(k_row_occ, dim3(grid_for(nrows, kBlock, 4096)), dim3(kBlock), 0, st,
                         occ_bits, nrows, g.nx, rowcnt);
      RPT_CHECK_LAUNCH();
      RPT_TRY(exclusive_scan_total_i32(rowcnt, rowq, nrows, st));
      rowq_ok = true;
      const int nbands = (g.ny + by - 1) / by;
      tile_by = by;
      tile_nbands = nbands;
      tile_R = R;
      const int64_t ntiles = (int64_t)g.nt * nbands;
      const unsigned grid = (unsigned)(((ntiles + 1) + 7) & ~(int64_t)7);
      hipLaunchKernelGGL(k_core_tiles, dim3(grid), dim3(kTileBlock), 0, st, g, R, by, nbands,
                         ntiles, occ, n_occ, rowq, rec<2>(), mutual, occ_bits, slab_t, pts, core);
      RPT_CHECK_LAUNCH();
      tm.mark();
      return RPT_OK;
    }
  }
  if (!k5_legacy) {
    // cells decide (and write their points' flags) in one pass; the undecided cells' points are
    // settled by k_core_slow_cells, which walks the occupied cells itself (no queue, no fill)
    if (oct) {
      hipLaunchKernelGGL(k_core_cells_oct<false>, dim3((grid_for(8 * n, kBlock, 8192) + 7) & ~7), dim3(kBlock), 0,
                         st, g, (int)rs, occ, n_occ, rec<2>(), mutual, occ_bits, slab_t, cflag,
                         (int32_t*)nullptr, k5_fill ? (uint8_t*)nullptr : core);
      if (k5_fill)
        hipLaunchKernelGGL(k_core_fill<false>, dim3(tile_grid(n)), dim3(kBlock), 0, st, skey, n,
                           cflag, core, slow, n_slow);
    } else {
      RPT_TRY(zero_n(st, 1, &n_cq));
      hipLaunchKernelGGL(k_core_cell_fast, dim3(tile_grid(n)), dim3(kBlock), 0, st, occ, n_occ,
                         g, cell_start, mutual, cflag, cq, n_cq);
      if (dim == 2)
        hipLaunchKernelGGL(k_core_cell_window<2>, dim3(wave_grid(n)), dim3(kBlock), 0, st, g,
                           occ, rec<2>(), occ_bits, slab_t, cq, n_cq, cflag);
      else
        hipLaunchKernelGGL(k_core_cell_window<3>, dim3(wave_grid(n)), dim3(kBlock), 0, st, g,
                           occ, rec<3>(), occ_bits, slab_t, cq, n_cq, cflag);
      hipLaunchKernelGGL(k_core_fill<false>, dim3(tile_grid(n)), dim3(kBlock), 0, st, skey, n,
                         cflag, core, slow, n_slow);
    }
    const int gs = wave_grid(n);
    if (dim == 2)
      hipLaunchKernelGGL(k_core_slow_cells<2>, dim3(gs), dim3(kBlock), 0, st, pts, g, rec<2>(),
                         occ_bits, slab_t, occ, n_occ, cflag, core);
    else
      hipLaunchKernelGGL(k_core_slow_cells<3>, dim3(gs), dim3(kBlock), 0, st, pts, g, rec<3>(),
                         occ_bits, slab_t, occ, n_occ, cflag, core);
    RPT_CHECK_LAUNCH();
    tm.mark();
    return RPT_OK;
  }
#endif
  // oct: the union's per-cell minima (cell_min_pair) come out of the fill and slow passes
  auto* cm = oct ? reinterpret_cast<unsigned long long*>(cell_min_pair) : nullptr;
  if (k5_fused_path()) {
    RPT_TRY(zero_n(st, 1, &n_slow));
    // the cell pass's decisions handed to the slow pass when its window's 5 W (slab, row) pairs
    // x 5 columns fit a 128-bit mask (W <= 5; pmask / clo per occupied cell in the dead radix
    // buffers / cid, both rebuilt later)
    const bool masked = (int)rs <= 2 && k5_mask();
    uint4* k5m = reinterpret_cast<uint4*>(pmask);
    if (masked) {
      hipLaunchKernelGGL((k_core_cells_oct<true, true>),
                         dim3((grid_for(8 * n, kBlock, 8192) + 7) & ~7), dim3(kBlock), 0, st, g,
                         (int)rs, occ, n_occ, rec<2>(), mutual, occ_bits, slab_t,
                         (int32_t*)nullptr, (int32_t*)nullptr, core, cm, slow, cq, n_slow, k5m,
                         cid);
      hipLaunchKernelGGL(k_core_slow_masked, dim3(wave_grid(n)), dim3(kBlock), 0, st, pts, g,
                         (int)rs, rec<2>(), occ, slow, cq, n_slow, k5m, cid, core, sorig, cm);
    } else {
      hipLaunchKernelGGL(k_core_cells_oct<true>, dim3((grid_for(8 * n, kBlock, 8192) + 7) & ~7),
                         dim3(kBlock), 0, st, g, (int)rs, occ, n_occ, rec<2>(), mutual, occ_bits,
                         slab_t, (int32_t*)nullptr, (int32_t*)nullptr, core, cm, slow, cq,
                         n_slow);
    }
    if (masked) {
    } else if (g.rt >= 0 && (2 * g.rt + 1) * 25 <= 128)
      hipLaunchKernelGGL((k_core_slow<2, 2>), dim3(wave_grid(n)), dim3(kBlock), 0, st, pts, skey,
                         g, rec<2>(), occ_bits, slab_t, slow, n_slow, core, sorig, cm, cq);
    else
      hipLaunchKernelGGL(k_core_slow<2>, dim3(wave_grid(n)), dim3(kBlock), 0, st, pts, skey, g,
                         rec<2>(), occ_bits, slab_t, slow, n_slow, core, sorig, cm, cq);
    RPT_CHECK_LAUNCH();
    cmin_ready = true;
#ifdef RPT_AB
    if (ab_env("RPT_STATS")) {  // A/B diagnostics: K5's slow queue and its cells (syncs)
      int32_t h = 0;
      (void)hipMemcpyAsync(&h, n_slow, 4, hipMemcpyDeviceToHost, st);
      (void)hipStreamSynchronize(st);
      std::vector<int32_t> keys((size_t)std::max(h, 0));
      if (h > 0) (void)hipMemcpy(keys.data(), cq, sizeof(int32_t) * (size_t)h, hipMemcpyDeviceToHost);
      std::sort(keys.begin(), keys.end());
      int64_t distinct = 0, max_run = 0, run = 0;
      for (size_t i = 0; i < keys.size(); ++i) {
        run = (i > 0 && keys[i] == keys[i - 1]) ? run + 1 : 1;
        if (run == 1) ++distinct;
        max_run = std::max(max_run, run);
      }
      std::fprintf(stderr, "[rpt stats] n=%lld k5_slow_queue=%d cells=%lld max_per_cell=%lld\n",
                   (long long)n, h, (long long)distinct, (long long)max_run);
    }
#endif
    tm.mark();
    return RPT_OK;
  }
  if (oct) {
    hipLaunchKernelGGL(k_core_cells_oct<false>, dim3((grid_for(8 * n, kBlock, 8192) + 7) & ~7), dim3(kBlock), 0,
                       st, g, (int)rs, occ, n_occ, rec<2>(), mutual, occ_bits, slab_t, cflag,
                       n_slow, (uint8_t*)nullptr);
  } else {
    RPT_TRY(zero_n(st, 1, &n_slow));
    RPT_TRY(zero_n(st, 1, &n_cq));
    hipLaunchKernelGGL(k_core_cell_fast, dim3(tile_grid(n)), dim3(kBlock), 0, st, occ, n_occ, g,
                       cell_start, mutual, cflag, cq, n_cq);
    if (dim == 2)
      hipLaunchKernelGGL(k_core_cell_window<2>, dim3(wave_grid(n)), dim3(kBlock), 0, st, g, occ,
                         rec<2>(), occ_bits, slab_t, cq, n_cq, cflag);
    else
      hipLaunchKernelGGL(k_core_cell_window<3>, dim3(wave_grid(n)), dim3(kBlock), 0, st, g, occ,
                         rec<3>(), occ_bits, slab_t, cq, n_cq, cflag);
  }
  hipLaunchKernelGGL(k_core_fill<true>, dim3(tile_grid(n)), dim3(kBlock), 0, st, skey, n, cflag,
                     core, slow, n_slow, sorig, cm, C);
  if (dim == 2)
    hipLaunchKernelGGL(k_core_slow<2>, dim3(wave_grid(n)), dim3(kBlock), 0, st, pts, skey, g,
                       rec<2>(), occ_bits, slab_t, slow, n_slow, core, sorig, cm);
  else
    hipLaunchKernelGGL(k_core_slow<3>, dim3(wave_grid(n)), dim3(kBlock), 0, st, pts, skey, g,
                       rec<3>(), occ_bits, slab_t, slow, n_slow, core);
  RPT_CHECK_LAUNCH();
  cmin_ready = cm != nullptr;
  tm.mark();
  return RPT_OK;
}

int32_t DbscanState::union_pass(hipStream_t st) {
  if (degenerate) return RPT_OK;
  if (uf_flags < 0) {
    const char* e = ab_env("RPT_UF_FLAGS");
    uf_flags = e ? (std::atoi(e) & 3) : kDefaultUfFlags;
  }
  const int gb = grid_for(n, kBlock, 2048);
  const int gc = grid_for(C, kBlock, 8192);
  const int gw = wave_grid(n);
  const unsigned gp = (unsigned)((n + kBlock - 1) / kBlock);
  const int32_t* n_occ = n_occ_dev;
  (void)gc;
  // per-cell (min original index, sorted index) of the core points, one u64 per cell
  auto* cmin = reinterpret_cast<unsigned long long*>(cell_min_pair);
  if (union_list < 0) {
    const char* e = ab_env("RPT_UNION_LIST");
    union_list = (e && std::atoi(e) == 0) ? 0 : 1;
  }
  if (union_pair < 0) {
    const char* e = ab_env("RPT_UNION_PAIR");
    union_pair = (e && std::atoi(e) == 0) ? 0 : 1;
  }
  // 2-D: the first union pass lists its cells with undecided candidates in nc_list (free until
  // the label pass), their count at nc_list[n] (zeroed by k_init_occ_cells)
  const bool listing = union_list && dim == 2;
  int32_t* plist = listing ? nc_list : nullptr;
  int32_t* pcount = listing ? nc_list + n : nullptr;
  // 2-D pair path: the non-mutual cells with core points listed by the first pass in cid (free
  // until the label pass), their count at cid[n]; k_union_nm then takes only their points
  // (RPT_UNION_NM=0 in the A/B build: k_union over every point)
  if (union_nm < 0) {
    const char* e = ab_env("RPT_UNION_NM");
    union_nm = (e && std::atoi(e) == 0) ? 0 : 1;
  }
  const bool nm = dim == 2 && union_pair && union_nm;
  int32_t* nm_list = nm ? cid : nullptr;
  int32_t* nm_count = nm ? cid + n : nullptr;
  // the per-cell minima: from the core pass (cmin_ready) or from the final core flags here
  hipLaunchKernelGGL(k_init_occ_cells, dim3(gb), dim3(kBlock), 0, st, occ, n_occ, C, rep,
                     cmin_ready ? nullptr : cmin, pcount, nm_count);
  if (!cmin_ready)
    hipLaunchKernelGGL(k_cell_min_pair, dim3(gb), dim3(kBlock), 0, st, skey, core, sorig, n, C,
                       cmin);
  hipLaunchKernelGGL(k_parent_init_pair, dim3(grid_for(n, kBlock * kPU, 2048)), dim3(kBlock), 0,
                     st, parent, n, core, skey, mutual, cmin, C, rep);
  int32_t* lstat_dev = nullptr;  // (A/B diagnostics)
  if (dim == 2) {
    uint4* pm = listing ? pmask : nullptr;
    if (union_pair)  // two cells per wave (RPT_UNION_PAIR=0 in the A/B build: one)
      hipLaunchKernelGGL(k_union_cells_pair, dim3(gw), dim3(kBlock), 0, st, pts, g, occ, n_occ,
                         rec<2>(), occ_bits, slab_t, rep, mutual, sorig, parent, uf_flags, pm,
                         plist, pcount, union_cpw(), nm_list, nm_count);
    else
      hipLaunchKernelGGL((k_union_cells<2, false>), dim3(gw), dim3(kBlock), 0, st, pts, g,
                         cell_start, occ, n_occ, rec<2>(), occ_bits, slab_t, core, rep, mutual,
                         sorig, parent, uf_flags, pm, plist, pcount);
#ifdef RPT_AB
    if (listing && ab_env("RPT_STATS")) {  // (A/B diagnostics: a leaked 16 B per process)
      static int32_t* buf = nullptr;
      if (!buf) (void)hipMalloc(&buf, 16);
      lstat_dev = buf;
      (void)hipMemsetAsync(lstat_dev, 0, 16, st);
    }
#endif
    if (listing) {
      // the snapshot in cell_root (free until the label stage's k_cell_roots); not on dense
      // slabs, where it measured slower (configs[4] share: +38 us snapshot, listed 867 -> 916 us;
      // 1000 standard frames: listed 348 -> 202 us for +28)
      const bool snap = union_snapshot() == 2 || (union_snapshot() == 1 && !dense_slabs);
      if (snap)
        hipLaunchKernelGGL(k_cell_root_snapshot, dim3(grid_for(n, kBlock, 4096)), dim3(kBlock),
                           0, st, occ, n_occ, rep, parent, g.cells, uf_flags, cell_root);
      hipLaunchKernelGGL(k_union_listed, dim3(gw), dim3(kBlock), 0, st, pts, g, occ, rec<2>(),
                         occ_bits, slab_t, core, rep, mutual, sorig, parent, uf_flags, pm, plist,
                         pcount, snap ? (const int32_t*)cell_root : nullptr, lstat_dev);
    }
    else
      hipLaunchKernelGGL((k_union_cells<2, true>), dim3(gw), dim3(kBlock), 0, st, pts, g,
                         cell_start, occ, n_occ, rec<2>(), occ_bits, slab_t, core, rep, mutual,
                         sorig, parent, uf_flags, pm, plist, pcount);
    if (nm)
      hipLaunchKernelGGL(k_union_nm<2>, dim3(gw), dim3(kBlock), 0, st, pts, g, cell_start,
                         rec<2>(), slab_t, core, rep, mutual, sorig, parent, nm_list, nm_count);
    else
      hipLaunchKernelGGL(k_union<2>, dim3(gp), dim3(kBlock), 0, st, pts, skey, n, g, cell_start,
                         rec<2>(), slab_t, core, rep, mutual, sorig, parent);
  } else {
    hipLaunchKernelGGL((k_union_cells<3, false>), dim3(gw), dim3(kBlock), 0, st, pts, g,
                       cell_start, occ, n_occ, rec<3>(), occ_bits, slab_t, core, rep, mutual, sorig,
                       parent, uf_flags);
    hipLaunchKernelGGL((k_union_cells<3, true>), dim3(gw), dim3(kBlock), 0, st, pts, g,
                       cell_start, occ, n_occ, rec<3>(), occ_bits, slab_t, core, rep, mutual, sorig,
                       parent, uf_flags);
    hipLaunchKernelGGL(k_union<3>, dim3(gp), dim3(kBlock), 0, st, pts, skey, n, g, cell_start,
                       rec<3>(), slab_t, core, rep, mutual, sorig, parent);
  }
  RPT_CHECK_LAUNCH();
  // every later reader walks to the root with path halving (k_ccmin, k_comp_out, ...), so a
  // separate compression pass only moves that work; RPT_UF_COMPRESS=1 keeps it (A/B)
  if (uf_compress < 0) {
    const char* e = ab_env("RPT_UF_COMPRESS");
    uf_compress = (e && std::atoi(e) == 1) ? 1 : 0;
  }
#ifdef RPT_AB
  if (uf_compress)
    hipLaunchKernelGGL(k_compress, dim3(gb), dim3(kBlock), 0, st, parent, core, n, sorig,
                       (int32_t*)nullptr);
  if (ab_env("RPT_STATS")) {  // A/B diagnostics: the queue and list sizes of this run (syncs)
    int32_t h[2] = {0, 0}, ls[4] = {0, 0, 0, 0};
    (void)hipMemcpyAsync(&h[0], n_occ_dev, 4, hipMemcpyDeviceToHost, st);
    if (listing) (void)hipMemcpyAsync(&h[1], pcount, 4, hipMemcpyDeviceToHost, st);
    if (lstat_dev) (void)hipMemcpyAsync(ls, lstat_dev, 16, hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
    std::fprintf(stderr,
                 "[rpt stats] n=%lld occupied=%d listed_cells=%d listed: undecided=%d "
                 "roots_differ=%d searches=%d hits=%d\n",
                 (long long)n, h[0], h[1], ls[0], ls[1], ls[2], ls[3]);
  }
#endif
  RPT_CHECK_LAUNCH();
  tm.mark();
  return RPT_OK;
}

// component minima (k_ccmin; also queues the non-core points) -> MinRank prefix and cluster count
// cell_key (nullable, pre-filled with INT_MAX): also the per-cell smallest component key
int32_t DbscanState::cluster_ids(hipStream_t st, int32_t* cell_key, int32_t* zero) {
  const int64_t W = min_words();
  // per-cell roots of the mutual cells (read by k_ccmin for their core points); zero (nullable):
  // k_ccmin's non-core queue counter, cleared by k_cell_roots, which also clears the minimum
  // bits and fills cell_key (nullable) with INT_MAX (one launch instead of three)
  const bool cr = cell_roots_enabled();
  if (cr) {
    hipLaunchKernelGGL(k_cell_roots, dim3(grid_for(n, kBlock, 2048)), dim3(kBlock), 0, st, parent,
                       occ, n_occ_dev, C, mutual, rep, cell_root, zero, min_bits, W, cell_key);
  } else {
    RPT_HIP(hipMemsetAsync(min_bits, 0, sizeof(uint32_t) * W, st));
    if (zero) RPT_HIP(hipMemsetAsync(zero, 0, sizeof(int32_t), st));
    if (cell_key)
      hipLaunchKernelGGL(k_fill_i32, dim3(grid_for(C, kBlock, 8192)), dim3(kBlock), 0, st,
                         cell_key, C, INT_MAX);
  }
  hipLaunchKernelGGL(k_ccmin, dim3(tile_grid(n)), dim3(kBlock), 0, st, parent, core, n, sorig,
                     ccmin, min_bits, nc_list, nc_list + n, skey, mutual,
                     cr ? (const int32_t*)cell_root : nullptr, C, cell_key);
  hipLaunchKernelGGL(k_word_popc, dim3(grid_for(W, kBlock, 2048)), dim3(kBlock), 0, st, min_bits,
                     W, min_pref);
  RPT_CHECK_LAUNCH();
  return exclusive_scan_total_i32(min_pref, min_pref, W, st);
}

int32_t DbscanState::labels_local(int32_t* labels, rpt_stdbscan_stats* stats, hipStream_t st) {
  const int gb = grid_for(n, kBlock, 2048);
  if (degenerate) {
    hipLaunchKernelGGL(k_isolated_labels, dim3(gb), dim3(kBlock), 0, st, labels, n,
                       min_samples <= 0 ? 1 : 0);
    RPT_CHECK_LAUNCH();
    if (stats) {
      stats->n_points = n;
      stats->n_core = min_samples <= 0 ? n : 0;
      stats->n_clusters = min_samples <= 0 ? (int32_t)n : 0;
    }
    return RPT_OK;
  }
  int32_t* nc_count = nc_list + n;
  // also the per-cell smallest keys (k_cell_min_key fused; cell_min filled with INT_MAX by
  // cluster_ids' first kernel) and nc_count cleared
  RPT_TRY(cluster_ids(st, cell_min, nc_count));
  const MinRank mr{min_bits, min_pref};
  if (spos_on)
    hipLaunchKernelGGL(k_label_core_orig, dim3((grid_for(n, kBlock * kPU, 2048) + 7) & ~7),
                       dim3(kBlock), 0, st, ccmin, n, slab, mr, labels);
  else
    hipLaunchKernelGGL(k_label_core, dim3((grid_for(n, kBlock * kPU, 2048) + 7) & ~7),
                       dim3(kBlock), 0, st, ccmin, n, sorig, mr, labels);
  int32_t* kstat = nullptr;  // (A/B diagnostics)
#ifdef RPT_AB
  if (ab_env("RPT_STATS")) {  // (a leaked 16 B per process)
    static int32_t* buf = nullptr;
    if (!buf) (void)hipMalloc(&buf, 16);
    kstat = buf;
    (void)hipMemsetAsync(kstat, 0, 16, st);
  }
#endif
#ifdef RPT_AB
  if (use_label_tiles())
    hipLaunchKernelGGL((k_label_tiles<false>), dim3(tile_grid_blocks()), dim3(kTileBlock), 0, st,
                       g, tile_R, tile_by, tile_nbands, (int64_t)g.nt * tile_nbands, occ,
                       n_occ_dev, rowq, rec<2>(), mutual, occ_bits, slab_t, pts, ccmin, cell_min,
                       sorig, mr, min_samples, labels);
  else if (dim == 2 && label_w() == 64)
    hipLaunchKernelGGL((k_label<2, false, 64>), dim3(wave_grid(n)), dim3(kBlock), 0, st, pts,
                       skey, g, rec<2>(), occ_bits, slab_t, ccmin, cell_min, mutual, sorig, mr,
                       nc_list, nc_count, labels);
  else
#endif
  if (dim == 2)
    hipLaunchKernelGGL((k_label<2, false, 32>),
                       dim3(wave_grid(n)), dim3(kBlock), 0, st, pts, skey, g,
                       rec<2>(), occ_bits, slab_t, ccmin, cell_min, mutual, sorig, mr, nc_list,
                       nc_count, labels, kstat);
  else
    hipLaunchKernelGGL((k_label<3, false, 64>),
                       dim3(wave_grid(n)), dim3(kBlock), 0, st, pts, skey, g,
                       rec<3>(), occ_bits, slab_t, ccmin, cell_min, mutual, sorig, mr, nc_list,
                       nc_count, labels);
  RPT_CHECK_LAUNCH();
#ifdef RPT_AB
  if (kstat) {
    int32_t ks[4] = {0, 0, 0, 0};
    (void)hipMemcpyAsync(ks, kstat, 16, hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
    std::fprintf(stderr,
                 "[rpt stats] n=%lld label: queued=%d core_in_window=%d searched=%d labelled=%d\n",
                 (long long)n, ks[0], ks[1], ks[2], ks[3]);
  }
#endif
  tm.mark();
  if (stats && defer) return RPT_OK;  // fill_stats after the caller's sync
  if (stats) {
    int32_t ncl = 0;
    RPT_HIP(hipMemcpyAsync(&ncl, n_clusters_ptr(), sizeof(int32_t), hipMemcpyDeviceToHost, st));
    RPT_TRY(wait_stream(st));
    RPT_TRY(fill_stats(ncl, stats));
  }
  return RPT_OK;
}

int32_t DbscanState::fill_stats(int32_t ncl, rpt_stdbscan_stats* stats) {
  {
    stats->n_points = n;
    stats->n_clusters = ncl;
    stats->n_core = -1;
    stats->grid_dims[0] = g.nx;
    stats->grid_dims[1] = g.ny;
    stats->grid_dims[2] = g.nz;
    stats->grid_dims[3] = g.nt;
    stats->grid_cells = C;
    if (tm.on && tm.k >= 6) {
      RPT_HIP(hipEventSynchronize(tm.ev[tm.k - 1]));
      stats->ms_bounds = tm.ms(0);
      stats->ms_grid = tm.ms(1);
      stats->ms_core = tm.ms(2);
      stats->ms_union = tm.ms(3);
      stats->ms_label = tm.ms(4);
    }
  }
  return RPT_OK;
}

int32_t DbscanState::labels_global(const int64_t* rep_orig, const int64_t* reps, int64_t nr,
                                   int32_t* labels, hipStream_t st, const int64_t* nr_dev) {
  if (degenerate) {
    set_error("rpt_dbscan_labels_global: degenerate parameters are handled by rpt_stdbscan");
    return RPT_ENOTSUP;
  }
  const int gb = grid_for(n, kBlock, 2048);
  int32_t* nc_count = nc_list + n;
  const bool cr = cell_roots_enabled();
  if (cr) {  // (also clears nc_count for k_ccmin_global and fills cell_min with INT_MAX)
    hipLaunchKernelGGL(k_cell_roots, dim3(grid_for(n, kBlock, 2048)), dim3(kBlock), 0, st, parent,
                       occ, n_occ_dev, C, mutual, rep, cell_root, nc_count, (uint32_t*)nullptr,
                       (int64_t)0, cell_min);
  } else {
    RPT_HIP(hipMemsetAsync(nc_count, 0, sizeof(int32_t), st));
    hipLaunchKernelGGL(k_fill_i32, dim3(grid_for(C, kBlock, 8192)), dim3(kBlock), 0, st, cell_min,
                       C, INT_MAX);
  }
  hipLaunchKernelGGL(k_ccmin_global, dim3(tile_grid(n)), dim3(kBlock), 0, st, parent, core, n,
                     sorig, rep_orig, reps, nr, ccmin, cid, nc_list, nc_count, skey, mutual,
                     cr ? (const int32_t*)cell_root : nullptr, C, nr_dev);
  // the core labels in original order (before slab's inverse permutation is overwritten), then
  // per sorted point the final core labels with the per-cell smallest label folded in
  // (k_cell_min_key's pass)
  const bool orig = spos_on;
  if (orig)
    hipLaunchKernelGGL(k_label_global_orig, dim3(grid_for(n, kBlock * kPU, 2048)), dim3(kBlock), 0,
                       st, core, ccmin, cid, slab, n, labels);
  hipLaunchKernelGGL(k_label_global_core, dim3(gb), dim3(kBlock), 0, st, core, ccmin, cid, sorig,
                     n, slab, orig ? nullptr : labels, skey, C, cell_min);
  // slab now holds the sorted points' core labels, no longer the inverse permutation: a second
  // call on this state (the shard driver's redo of a step whose pairs / results overflowed, a
  // host merge, the K9 radix fallback) takes the sorted-order path
  spos_on = false;
#ifdef RPT_AB
  if (use_label_tiles())
    hipLaunchKernelGGL((k_label_tiles<true>), dim3(tile_grid_blocks()), dim3(kTileBlock), 0, st,
                       g, tile_R, tile_by, tile_nbands, (int64_t)g.nt * tile_nbands, occ,
                       n_occ_dev, rowq, rec<2>(), mutual, occ_bits, slab_t, pts, slab, cell_min,
                       sorig, MinRank{nullptr, nullptr}, min_samples, labels);
  else if (dim == 2 && label_w() == 64)
    hipLaunchKernelGGL((k_label<2, true, 64>), dim3(wave_grid(n)), dim3(kBlock), 0, st, pts,
                       skey, g, rec<2>(), occ_bits, slab_t, slab, cell_min, mutual, sorig,
                       MinRank{nullptr, nullptr}, nc_list, nc_count, labels);
  else
#endif
  if (dim == 2)
    hipLaunchKernelGGL((k_label<2, true, 32>),
                       dim3(wave_grid(n)), dim3(kBlock), 0, st, pts, skey, g,
                       rec<2>(), occ_bits, slab_t, slab, cell_min, mutual, sorig,
                       MinRank{nullptr, nullptr}, nc_list, nc_count, labels);
  else
    hipLaunchKernelGGL((k_label<3, true, 64>),
                       dim3(wave_grid(n)), dim3(kBlock), 0, st, pts, skey, g,
                       rec<3>(), occ_bits, slab_t, slab, cell_min, mutual, sorig,
                       MinRank{nullptr, nullptr}, nc_list, nc_count, labels);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

int32_t DbscanState::frames_pass(int32_t min_frames, hipStream_t st) {
  if (degenerate || min_frames < 1) return RPT_OK;  // <= 0: every core point qualifies
  cmin_ready = false;  // core points may be demoted below
  const bool refine = min_frames >= 2;
  int32_t* list = nc_list;  // free until labels_fifo rebuilds it
  int32_t* count = nc_list + n;
  const int32_t* n_occ = n_occ_dev;
  const bool cells = refine && integral_t && dim == 2 && g.nz == 1;
  // a whole-cell hit is one frame only when a slab is one frame: the cell cap can widen the slabs
  // (ct = 2, 4, ... for long runs of frames over a small region), then every point is read
  const int one_frame_cells = (integral_t && g.ct == 1.0) ? 1 : 0;
  if (cells) {
    const int R = (int)std::min<double>(std::floor((double)g.epst / g.ct), 64.0);
    hipLaunchKernelGGL(k_frames_cells, dim3(grid_for(n, kBlock, 8192)), dim3(kBlock), 0, st, g, R,
                       occ, n_occ, rec<2>(), occ_bits, min_frames, fok);
  }
  RPT_TRY(zero_n(st, 1, &count));
  hipLaunchKernelGGL(k_frames_queue, dim3(tile_grid(n)), dim3(kBlock), 0, st, skey, n, C,
                     cells ? (const uint8_t*)fok : (const uint8_t*)nullptr, (int)min_frames,
                     refine ? 1 : 0, core, list, count);
  if (refine) {
    // offsets of int32(t) within +-31 of the point's own frame fit the 64-bit set (|dt| <=
    // eps_t <= 30); larger windows list the distinct frames instead
    const bool small = (double)g.epst <= 30.0;
    if (dim == 2 && small)
      hipLaunchKernelGGL(k_frames_points<2>, dim3(wave_grid(n)), dim3(kBlock), 0, st, pts, skey, g,
                         rec<2>(), occ_bits, slab_t, one_frame_cells, (int)min_frames, list,
                         count, core);
    else if (small)
      hipLaunchKernelGGL(k_frames_points<3>, dim3(wave_grid(n)), dim3(kBlock), 0, st, pts, skey, g,
                         rec<3>(), occ_bits, slab_t, one_frame_cells, (int)min_frames, list,
                         count, core);
    else if (dim == 2)
      hipLaunchKernelGGL(k_frames_points_list<2>, dim3(wave_grid(n)), dim3(kBlock), 0, st, pts,
                         skey, g, rec<2>(), occ_bits, slab_t, one_frame_cells,
                         (int)min_frames, list, count, core);
    else
      hipLaunchKernelGGL(k_frames_points_list<3>, dim3(wave_grid(n)), dim3(kBlock), 0, st, pts,
                         skey, g, rec<3>(), occ_bits, slab_t, one_frame_cells,
                         (int)min_frames, list, count, core);
  }
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

int32_t DbscanState::labels_fifo(int32_t* labels, rpt_stdbscan_stats* stats, hipStream_t st) {
  int32_t* nc_count = nc_list + n;  // k_ccmin's non-core queue counter, cleared by cluster_ids
  int32_t* spos = slab;
  RPT_TRY(cluster_ids(st, nullptr, nc_count));
  if (!spos_on)  // (else the grid build's)
    hipLaunchKernelGGL(k_inverse_perm, dim3(grid_for(n, kBlock, 2048)), dim3(kBlock), 0, st,
                       sorig, n, spos);
  const MinRank mr{min_bits, min_pref};
  hipLaunchKernelGGL(k_label_core_orig, dim3((grid_for(n, kBlock * kPU, 2048) + 7) & ~7),
                     dim3(kBlock), 0, st, ccmin, n, spos, mr, labels);
  if (dim == 2)
    hipLaunchKernelGGL((k_label_fifo<2>), dim3(wave_grid(n)), dim3(kBlock), 0, st, pts, skey, g,
                       rec<2>(), occ_bits, slab_t, ccmin, rep, sorig, spos, mr, nc_list,
                       nc_count, labels);
  else
    hipLaunchKernelGGL((k_label_fifo<3>), dim3(wave_grid(n)), dim3(kBlock), 0, st, pts, skey, g,
                       rec<3>(), occ_bits, slab_t, ccmin, rep, sorig, spos, mr, nc_list,
                       nc_count, labels);
  RPT_CHECK_LAUNCH();
  tm.mark();
  int32_t ncl = 0;
  RPT_HIP(hipMemcpyAsync(&ncl, n_clusters_ptr(), sizeof(int32_t), hipMemcpyDeviceToHost, st));
  RPT_TRY(wait_stream(st));
  if (stats) RPT_TRY(fill_stats(ncl, stats));
  return RPT_OK;
}

static int32_t check_args(const float* x, const float* y, const float* z, int64_t stride,
                          const float* t, int64_t n, int dim) {
  if (n <= 0) {
    set_error("Found array with 0 sample(s) (shape=(0, %d)) while a minimum of 1 is required.",
              dim);
    return RPT_EEMPTY;
  }
  if (n >= (int64_t(1) << 31) - 2) {
    set_error("rpt_stdbscan: n=%lld exceeds the int32 index space", (long long)n);
    return RPT_ENOTSUP;
  }
  if (!x || !y || !t || (dim == 3 && !z) || stride < 1) {
    set_error("rpt_stdbscan: null pointer or bad stride");
    return RPT_EINVAL;
  }
  return RPT_OK;
}

static std::mutex g_state_mu;
// per (device, stream), for the fused single-call path
static std::vector<std::pair<std::pair<int, hipStream_t>, DbscanState*>> g_states;

int32_t stdbscan(const float* x, const float* y, const float* z, int64_t stride, const float* t,
                 int64_t n, double eps_space, double eps_time, int32_t min_samples,
                 int32_t* labels, rpt_stdbscan_stats* stats, hipStream_t st, int dim) {
  RPT_TRY(check_args(x, y, z, stride, t, n, dim));
  if (!labels) {
    set_error("rpt_stdbscan: null labels");
    return RPT_EINVAL;
  }
  int dev = 0;
  RPT_HIP(hipGetDevice(&dev));
  DbscanState* S;
  {
    std::lock_guard<std::mutex> lk(g_state_mu);
    S = nullptr;
    for (auto& e : g_states)
      if (e.first.first == dev && e.first.second == st) S = e.second;
    if (!S) {
      S = new DbscanState();
      g_states.push_back({{dev, st}, S});
    }
  }
  RPT_TRY(S->build(x, y, z, stride, t, n, eps_space, eps_time, min_samples,
                   stats && stats->timing, st));
  RPT_TRY(S->core_pass(st));
  RPT_TRY(S->union_pass(st));
  return S->labels_local(labels, stats, st);
}

// Denoise variant (PointCloudWorkF/stdbscan_denoising_pipeline.py:264-369), 2-D.
int32_t stdbscan_denoise(const float* x, const float* y, const float* t, int64_t n,
                         double eps_space, double eps_time, int32_t min_samples,
                         int32_t min_frames, int32_t* labels, rpt_stdbscan_stats* stats,
                         hipStream_t st) {
  if (n == 0) {  // the reference returns an empty label array (:286-287), no error
    if (stats) *stats = rpt_stdbscan_stats{};
    return RPT_OK;
  }
  RPT_TRY(check_args(x, y, nullptr, 1, t, n, 2));
  if (!labels) {
    set_error("rpt_stdbscan_denoise: null labels");
    return RPT_EINVAL;
  }
  if (min_frames > 64 * kFramesPerLane && !((float)eps_time <= 30.0f) &&
      (float)eps_time == (float)eps_time) {
    set_error("rpt_stdbscan_denoise: min_frames > %d with eps_time > 30 is not supported",
              64 * kFramesPerLane);
    return RPT_ENOTSUP;
  }
  int dev = 0;
  RPT_HIP(hipGetDevice(&dev));
  DbscanState* S;
  {
    std::lock_guard<std::mutex> lk(g_state_mu);
    S = nullptr;
    for (auto& e : g_states)
      if (e.first.first == dev && e.first.second == st) S = e.second;
    if (!S) {
      S = new DbscanState();
      g_states.push_back({{dev, st}, S});
    }
  }
  RPT_TRY(S->build(x, y, nullptr, 1, t, n, eps_space, eps_time, min_samples,
                   stats && stats->timing, st));
  if (S->degenerate) {
    // no pair passes (not even (i, i)): core iff 0 >= min_samples and 0 >= min_frames, each its
    // own cluster in index order
    const bool single = min_samples <= 0 && min_frames <= 0;
    hipLaunchKernelGGL(k_isolated_labels, dim3(grid_for(n, kBlock, 2048)), dim3(kBlock), 0, st,
                       labels, n, single ? 1 : 0);
    RPT_CHECK_LAUNCH();
    if (stats) {
      stats->n_points = n;
      stats->n_core = single ? n : 0;
      stats->n_clusters = single ? (int32_t)n : 0;
    }
    return wait_stream(st);
  }
  RPT_TRY(S->core_pass(st));
  RPT_TRY(S->frames_pass(min_frames, st));
  RPT_TRY(S->union_pass(st));
  return S->labels_fifo(labels, stats, st);
}

// The fused path without its readbacks (the native stack driver): the cluster count stays on the
// device at *n_clusters_dev (nullptr when the parameters are degenerate: stats is then complete)
// and stdbscan_fill_stats completes stats after the caller has synchronised the stream.
// Bounds of the 2-D points [0, *n_dev) (n_dev on the device, <= n_max) into out_dev
// (stdbscan_bounds_bytes(), device): what stdbscan_deferred's build would compute, for a caller
// that reads them back together with its own results.
size_t stdbscan_bounds_bytes() { return sizeof(Bounds); }
int32_t stdbscan_bounds_dev(const float* x, const float* y, const float* t, int64_t n_max,
                            const int64_t* n_dev, void* out_dev, void* part_dev,
                            hipStream_t st) {
  const int nbb = grid_for(std::max<int64_t>(n_max, 1), kBlock, 1024);
  hipLaunchKernelGGL(k_bounds<2>, dim3(nbb), dim3(kBlock), 0, st, x, y, (const float*)nullptr,
                     (int64_t)1, t, n_max, static_cast<Bounds*>(part_dev), n_dev);
  hipLaunchKernelGGL(k_bounds_final, dim3(1), dim3(kBlock), 0, st,
                     static_cast<const Bounds*>(part_dev), nbb, static_cast<Bounds*>(out_dev));
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}
int32_t stdbscan_bounds_final_dev(const void* part_dev, int nb, void* out_dev, hipStream_t st) {
  hipLaunchKernelGGL(k_bounds_final, dim3(1), dim3(kBlock), 0, st,
                     static_cast<const Bounds*>(part_dev), nb, static_cast<Bounds*>(out_dev));
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}
// the partials of a bounds pass of kBoundsBlock-thread blocks (k_bounds here, k_window in the
// shard driver) over at most n_max points: one per block of grid_for(n_max, kBoundsBlock, 1024)
static_assert(kBlock == kBoundsBlock, "k_bounds is launched with kBlock threads per block");
size_t stdbscan_bounds_part_bytes(int64_t n_max) {
  return sizeof(Bounds) * (size_t)grid_for(std::max<int64_t>(n_max, 1), kBoundsBlock, 1024);
}

int32_t stdbscan_deferred(const float* x, const float* y, const float* z, int64_t stride,
                          const float* t, int64_t n, double eps_space, double eps_time,
                          int32_t min_samples, int32_t* labels, rpt_stdbscan_stats* stats,
                          hipStream_t st, int dim, const int32_t** n_clusters_dev,
                          void** state, const void* host_bounds) {
  RPT_TRY(check_args(x, y, z, stride, t, n, dim));
  if (!labels || !stats || !n_clusters_dev || !state) {
    set_error("stdbscan_deferred: null argument");
    return RPT_EINVAL;
  }
  int dev = 0;
  RPT_HIP(hipGetDevice(&dev));
  DbscanState* S;
  {
    std::lock_guard<std::mutex> lk(g_state_mu);
    S = nullptr;
    for (auto& e : g_states)
      if (e.first.first == dev && e.first.second == st) S = e.second;
    if (!S) {
      S = new DbscanState();
      g_states.push_back({{dev, st}, S});
    }
  }
  S->given_bounds = host_bounds;
  const int32_t sb = S->build(x, y, z, stride, t, n, eps_space, eps_time, min_samples,
                              stats->timing != 0, st);
  S->given_bounds = nullptr;
  RPT_TRY(sb);
  RPT_TRY(S->core_pass(st));
  RPT_TRY(S->union_pass(st));
  S->defer = !S->degenerate;
  const int32_t s_ = S->labels_local(labels, stats, st);
  *n_clusters_dev = S->defer ? S->n_clusters_ptr() : nullptr;
  *state = S;
  return s_;
}

// core flags (original order) of the state's last run: the stack driver's K5 result, for tests
int32_t stdbscan_core_flags(void* state, int64_t n, uint8_t* out, hipStream_t st) {
  DbscanState* S = static_cast<DbscanState*>(state);
  if (!S || S->degenerate || S->n != n || !S->core || !S->sorig) {
    set_error("rpt_stack_core_flags: no core flags for this run");
    return RPT_EINVAL;
  }
  hipLaunchKernelGGL(k_core_to_orig, dim3(grid_for(n, kBlock, 2048)), dim3(kBlock), 0, st,
                     S->core, S->sorig, n, out);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

int32_t stdbscan_fill_stats(void* state, int32_t n_clusters, rpt_stdbscan_stats* stats) {
  DbscanState* S = static_cast<DbscanState*>(state);
  S->defer = false;
  return S->fill_stats(n_clusters, stats);
}

// ---- phased C-ABI bodies
DbscanState* dbscan_create() { return new DbscanState(); }
void dbscan_destroy(DbscanState* s) {
  if (s) {
    s->arena.release();
    delete s;
  }
}
int32_t dbscan_build(DbscanState* S, const float* x, const float* y, const float* z,
                     int64_t stride, const float* t, int64_t n, double eps_space,
                     double eps_time, int32_t ms, hipStream_t st) {
  RPT_TRY(check_args(x, y, z, stride, t, n, z ? 3 : 2));
  RPT_TRY(S->build(x, y, z, stride, t, n, eps_space, eps_time, ms, false, st));
  if (S->degenerate) {
    set_error("rpt_dbscan_build: negative or NaN eps (use rpt_stdbscan)");
    return RPT_ENOTSUP;
  }
  return RPT_OK;
}
int32_t dbscan_core(DbscanState* S, uint8_t* core_out, hipStream_t st) {
  RPT_TRY(S->core_pass(st));
  if (core_out) {
    hipLaunchKernelGGL(k_core_to_orig, dim3(grid_for(S->n, kBlock, 2048)), dim3(kBlock), 0, st,
                       S->core, S->sorig, S->n, core_out);
    RPT_CHECK_LAUNCH();
  }
  return RPT_OK;
}
int32_t dbscan_set_core(DbscanState* S, const uint8_t* core_in, hipStream_t st) {
  S->cmin_ready = false;
  hipLaunchKernelGGL(k_core_from_orig, dim3(grid_for(S->n, kBlock, 2048)), dim3(kBlock), 0, st,
                     core_in, S->sorig, S->n, S->core);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}
int32_t dbscan_components(DbscanState* S, int32_t* comp_out, hipStream_t st) {
  RPT_TRY(S->union_pass(st));
  if (S->degenerate || S->n == 0) {  // (no cell structure: every core point walks its chain)
    hipLaunchKernelGGL(k_comp_out, dim3(grid_for(S->n, kBlock, 2048)), dim3(kBlock), 0, st,
                       S->parent, S->core, S->sorig, S->n, comp_out, S->skey,
                       (const int32_t*)nullptr, (int64_t)0);
  } else {
    hipLaunchKernelGGL(k_cell_roots, dim3(grid_for(S->n, kBlock, 2048)), dim3(kBlock), 0, st,
                       S->parent, S->occ, S->n_occ_dev, S->C, S->mutual, S->rep, S->cell_root,
                       (int32_t*)nullptr);
    hipLaunchKernelGGL(k_comp_out, dim3(grid_for(S->n, kBlock, 2048)), dim3(kBlock), 0, st,
                       S->parent, S->core, S->sorig, S->n, comp_out, S->skey,
                       (const int32_t*)S->cell_root, S->C);
  }
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}
// the component ids (as dbscan_components) of the original indices outside [lo_end, hi_begin)
int32_t dbscan_components_edges(DbscanState* S, int32_t* comp_out, int64_t lo_end,
                                int64_t hi_begin, hipStream_t st) {
  if (lo_end >= hi_begin) return dbscan_components(S, comp_out, st);
  RPT_TRY(S->union_pass(st));
  if (S->n == 0) return RPT_OK;
  const bool cells = !S->degenerate;
  if (cells)
    hipLaunchKernelGGL(k_cell_roots, dim3(grid_for(S->n, kBlock, 2048)), dim3(kBlock), 0, st,
                       S->parent, S->occ, S->n_occ_dev, S->C, S->mutual, S->rep, S->cell_root,
                       (int32_t*)nullptr);
  hipLaunchKernelGGL(k_comp_out_edges, dim3(grid_for(S->n, kBlock, 2048)), dim3(kBlock), 0, st,
                     S->parent, S->core, S->sorig, S->n, comp_out, S->skey,
                     cells ? (const int32_t*)S->cell_root : nullptr, cells ? S->C : (int64_t)0,
                     lo_end, hi_begin);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}
// the union-find state for the shard driver's per-root passes: a core point s is its
// component's root iff parent[s] == s (the component's minimum original index is sorig[s])
void dbscan_uf_arrays(const DbscanState* S, const uint8_t** core, const int32_t** parent,
                      const int32_t** sorig, int64_t* n) {
  *core = S->core;
  *parent = S->parent;
  *sorig = S->sorig;
  *n = S->n;
}
int32_t dbscan_labels_global(DbscanState* S, const int64_t* rep, const int64_t* reps, int64_t nr,
                             int32_t* labels, hipStream_t st) {
  return S->labels_global(rep, reps, nr, labels, st);
}
// the frame-sharded driver's forms: grid bounds read back by the caller with its own results
// (host_bounds: a Bounds), the representative count on the device
int32_t dbscan_build_given(DbscanState* S, const float* x, const float* y, const float* t,
                           int64_t n, double eps_space, double eps_time, int32_t ms,
                           const void* host_bounds, hipStream_t st) {
  RPT_TRY(check_args(x, y, nullptr, 1, t, n, 2));
  S->given_bounds = host_bounds;
  const int32_t s_ = S->build(x, y, nullptr, 1, t, n, eps_space, eps_time, ms, false, st);
  S->given_bounds = nullptr;
  RPT_TRY(s_);
  if (S->degenerate) {
    set_error("rpt_shard: negative or NaN eps");
    return RPT_ENOTSUP;
  }
  return RPT_OK;
}
int32_t dbscan_labels_global_dev(DbscanState* S, const int64_t* rep, const int64_t* reps,
                                 const int64_t* nr_dev, int32_t* labels, hipStream_t st) {
  return S->labels_global(rep, reps, 0, labels, st, nr_dev);
}
// device u8 core flags in the state's sorted order -> original order (out) without a pass
// the shard driver's edge forms of dbscan_core / dbscan_set_core: core flags of the original
// indices [a0, a1) -> out_a and [b0, b1) -> out_b (its own edge frames, for the neighbours), and
// the halo points' flags from their owners (original indices [0, a1) <- in_a, [b0, n) <- in_b):
// one coalesced index read per sorted point instead of full-length scattered conversions both
// ways around the halo update
__global__ void k_core_to_orig_ranges(const uint8_t* __restrict__ core,
                                      const int32_t* __restrict__ sorig, int64_t n, int64_t a0,
                                      int64_t a1, uint8_t* __restrict__ out_a, int64_t b0,
                                      int64_t b1, uint8_t* __restrict__ out_b) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n;
       s += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = sorig[s];
    if (out_a && i >= a0 && i < a1) out_a[i - a0] = core[s];
    if (out_b && i >= b0 && i < b1) out_b[i - b0] = core[s];
  }
}
__global__ void k_core_from_orig_ranges(const uint8_t* __restrict__ in_a, int64_t a1,
                                        const uint8_t* __restrict__ in_b, int64_t b0,
                                        const int32_t* __restrict__ sorig, int64_t n,
                                        uint8_t* __restrict__ core) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n;
       s += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = sorig[s];
    if (in_a && i < a1) core[s] = in_a[i];
    if (in_b && i >= b0) core[s] = in_b[i - b0];
  }
}
int32_t dbscan_core_edges(DbscanState* S, int64_t a0, int64_t a1, uint8_t* out_a, int64_t b0,
                          int64_t b1, uint8_t* out_b, hipStream_t st) {
  if (S->n <= 0 || (!(out_a && a1 > a0) && !(out_b && b1 > b0))) return RPT_OK;
  hipLaunchKernelGGL(k_core_to_orig_ranges, dim3(grid_for(S->n, kBlock, 2048)), dim3(kBlock), 0,
                     st, S->core, S->sorig, S->n, a0, a1, a1 > a0 ? out_a : nullptr, b0, b1,
                     b1 > b0 ? out_b : nullptr);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}
int32_t dbscan_set_core_edges(DbscanState* S, const uint8_t* in_a, int64_t a1,
                              const uint8_t* in_b, int64_t b0, hipStream_t st) {
  const bool a = in_a && a1 > 0, b = in_b && b0 < S->n;
  if (S->n <= 0 || (!a && !b)) return RPT_OK;
  S->cmin_ready = false;  // core flags change: the core pass's cell minima no longer hold
  hipLaunchKernelGGL(k_core_from_orig_ranges, dim3(grid_for(S->n, kBlock, 2048)), dim3(kBlock), 0,
                     st, a ? in_a : nullptr, a1, b ? in_b : nullptr, b0, S->sorig, S->n, S->core);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}
int32_t dbscan_core_orig(DbscanState* S, uint8_t* out, hipStream_t st) {
  hipLaunchKernelGGL(k_core_to_orig, dim3(grid_for(S->n, kBlock, 2048)), dim3(kBlock), 0, st,
                     S->core, S->sorig, S->n, out);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

}  // namespace rpt
