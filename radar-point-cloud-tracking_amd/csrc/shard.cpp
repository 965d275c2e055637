// Frame-sharded multi-GPU driver: one rank's phases of ONE global stack whose
// contiguous frame ranges are spread over ranks (4_temporal_object_tracker.py:466-506 clusters the
// whole stack at once; the result here is identical to rpt_stack_run over the whole stack).
//
// The caller (rpt/dist.py: torch.distributed over RCCL, or gloo) runs the collectives between the
// phases on buffers it owns.  Only three points of a step wait on the host:
//
//   polar   K1 + xy bounds + the K1 counts of the edge frames          (readback 1)
//     [all_gather info]                                                (host: land edges, caps)
//   land    land grid over the global edges
//     [all_reduce grid]                                                (device)
//   halo    land mask + compaction, the own edge frames packed for the neighbours
//     [P2P x/y/t, capacity = the neighbour's K1 edge count]            (device)
//   window  [prev halo | own | next halo] assembled, bounds            (readback 2)
//           grid build (host-sized) + core flags, own edge flags packed
//     [P2P core flags]                                                 (device)
//   link    halo flags from their owners, components, own edge component ids packed
//     [P2P component ids]                                              (device)
//   pairs   distinct (my id, owner's id) pairs of the halo points
//     [all_gather pairs, capacity]                                     (device)
//   finish  equivalence merge on the device (every rank the same), representatives, labels,
//           K9 of the own points, everything rank 0 needs packed
//     [all_gather packed results, capacity]                            (readback 3)
//
// Point ids are (rank << 40) | own index, so no rank needs another rank's point count to number
// its points, and id order is the global point order (frames are in rank order).  Labels are
// numbered per rank (dense over the representatives its window sees, in id order) and mapped to
// the global numbering on rank 0, which has every rank's representative table: the numbering
// preserves order, so every "smallest adjacent cluster" decision is the global one.
#include "shard_pack.h"
#include "stack_impl.h"

namespace rpt {
int32_t dbscan_build_given(DbscanState* S, const float* x, const float* y, const float* t,
                           int64_t n, double eps_space, double eps_time, int32_t ms,
                           const void* host_bounds, hipStream_t st);
int32_t dbscan_labels_global_dev(DbscanState* S, const int64_t* rep, const int64_t* reps,
                                 const int64_t* nr_dev, int32_t* labels, hipStream_t st);
int32_t dbscan_core_orig(DbscanState* S, uint8_t* out, hipStream_t st);
int32_t dbscan_components_edges(DbscanState* S, int32_t* comp_out, int64_t lo_end,
                                int64_t hi_begin, hipStream_t st);
void dbscan_uf_arrays(const DbscanState* S, const uint8_t** core, const int32_t** parent,
                      const int32_t** sorig, int64_t* n);
int32_t dbscan_core_edges(DbscanState* S, int64_t a0, int64_t a1, uint8_t* out_a, int64_t b0,
                          int64_t b1, uint8_t* out_b, hipStream_t st);
int32_t dbscan_set_core_edges(DbscanState* S, const uint8_t* in_a, int64_t a1,
                              const uint8_t* in_b, int64_t b0, hipStream_t st);

namespace {

constexpr int kHaloHdr = 4;                       // int32 header words of a halo buffer
constexpr int kMergeMax = 8192;                   // ids merged in LDS by one workgroup

// window index -> global point id: [prev halo | own | next halo]
struct WinIds {
  int32_t rank;
  int64_t n_prev, n_own, k_prev_total;
  __device__ __host__ int64_t gid(int64_t c) const {
    if (c < n_prev) return ((int64_t)(rank - 1) << kGidShift) | (k_prev_total - n_prev + c);
    if (c < n_prev + n_own) return ((int64_t)rank << kGidShift) | (c - n_prev);
    return ((int64_t)(rank + 1) << kGidShift) | (c - n_prev - n_own);
  }
};

struct WinMeta {  // device, one per step: read back with the window bounds
  int64_t n_prev, n_own, n_next, k_prev_total, n_head, n_tail, n_window, pad;
};

// ordered-u32 min/max of x and y over [0, *n_dev) (n_dev on the device, grid sized for n_max)
__global__ void k_xy_bounds_part(const float* __restrict__ x, const float* __restrict__ y,
                                 int64_t n_max, const int64_t* __restrict__ n_dev,
                                 uint32_t* __restrict__ part) {
  const int64_t n = n_dev ? min(*n_dev, n_max) : n_max;  // speculative: never past n_max
  uint32_t mnx = 0xffffffffu, mxx = 0u, mny = 0xffffffffu, mxy = 0u;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t ux = __float_as_uint(x[i]), uy = __float_as_uint(y[i]);
    ux = (ux & 0x80000000u) ? ~ux : (ux | 0x80000000u);
    uy = (uy & 0x80000000u) ? ~uy : (uy | 0x80000000u);
    mnx = min(mnx, ux);
    mxx = max(mxx, ux);
    mny = min(mny, uy);
    mxy = max(mxy, uy);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mnx = min(mnx, (uint32_t)__shfl_xor((int)mnx, off));
    mxx = max(mxx, (uint32_t)__shfl_xor((int)mxx, off));
    mny = min(mny, (uint32_t)__shfl_xor((int)mny, off));
    mxy = max(mxy, (uint32_t)__shfl_xor((int)mxy, off));
  }
  // one set of atomics per block (per-wave atomics on 4 words serialise: ~0.4 ms at 2k blocks)
  __shared__ uint32_t red[4][4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = mnx;
    red[1][w] = mxx;
    red[2][w] = mny;
    red[3][w] = mxy;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k) {
      mnx = min(mnx, red[0][k]);
      mxx = max(mxx, red[1][k]);
      mny = min(mny, red[2][k]);
      mxy = max(mxy, red[3][k]);
    }
    atomicMin(part + 0, mnx);
    atomicMax(part + 1, mxx);
    atomicMin(part + 2, mny);
    atomicMax(part + 3, mxy);
  }
}

__global__ void k_init_bounds(uint32_t* part) {
  if (threadIdx.x == 0) {
    part[0] = 0xffffffffu;
    part[1] = 0u;
    part[2] = 0xffffffffu;
    part[3] = 0u;
  }
}

inline float ord_to_f(uint32_t u) {
  const uint32_t v = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
  float f;
  std::memcpy(&f, &v, 4);
  return f;
}

// land grid [counts | sums] in float64 for the all-reduce (integer-valued: exact in any order)
__global__ void k_cnt_to_f64(const int32_t* __restrict__ cnt, int64_t cells,
                             double* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cells;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (double)cnt[i];
}
__global__ void k_f64_to_cnt(const double* __restrict__ in, int64_t cells,
                             int32_t* __restrict__ cnt, int64_t* __restrict__ zero) {
  // zero: the land mask's cell counter, cleared here instead of by a memset launch
  if (blockIdx.x == 0 && threadIdx.x == 0) *zero = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cells;
       i += (int64_t)gridDim.x * blockDim.x)
    cnt[i] = (int32_t)in[i];
}

// The own edge frames for the neighbours: {count, own kept total (lo, hi), 0} then x, y and
// t = frame0 + slot (float32 bits) at fixed offsets of the buffer's capacity (the K1 count of
// those frames, which the land filter can only shrink).
__global__ void k_halo_pack(const float* __restrict__ x, const float* __restrict__ y,
                            const int32_t* __restrict__ pf, const int64_t* __restrict__ off,
                            int32_t F, int32_t hf, int64_t frame0, int32_t* __restrict__ sp,
                            int64_t cap_p, int32_t* __restrict__ sn, int64_t cap_n) {
  const int64_t K = off[F];
  const int64_t nh = min(off[hf], cap_p);
  const int64_t t0 = off[F - hf];
  const int64_t nt = min(K - t0, cap_n);
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  if (i0 == 0) {
    if (sp) {
      sp[0] = (int32_t)nh;
      sp[1] = (int32_t)(uint32_t)(uint64_t)K;
      sp[2] = (int32_t)(uint32_t)((uint64_t)K >> 32);
      sp[3] = 0;
    }
    if (sn) {
      sn[0] = (int32_t)nt;
      sn[1] = (int32_t)(uint32_t)(uint64_t)K;
      sn[2] = (int32_t)(uint32_t)((uint64_t)K >> 32);
      sn[3] = 0;
    }
  }
  if (sp)
    for (int64_t i = i0; i < nh; i += step) {
      sp[kHaloHdr + i] = __float_as_int(x[i]);
      sp[kHaloHdr + cap_p + i] = __float_as_int(y[i]);
      sp[kHaloHdr + 2 * cap_p + i] = __float_as_int((float)(frame0 + (int64_t)pf[i]));
    }
  if (sn)
    for (int64_t i = i0; i < nt; i += step) {
      const int64_t j = t0 + i;
      sn[kHaloHdr + i] = __float_as_int(x[j]);
      sn[kHaloHdr + cap_n + i] = __float_as_int(y[j]);
      sn[kHaloHdr + 2 * cap_n + i] = __float_as_int((float)(frame0 + (int64_t)pf[j]));
    }
}

__device__ __forceinline__ int64_t halo_total(const int32_t* h) {
  return (int64_t)(((uint64_t)(uint32_t)h[2] << 32) | (uint64_t)(uint32_t)h[1]);
}

// [prev halo | own | next halo] as x / y / t, the window's counts, and per block the partial of
// the window's ST-DBSCAN bounds (k_bounds' semantics, reduced by stdbscan_bounds_final_dev: no
// separate bounds pass over the window)
__global__ __launch_bounds__(kBoundsBlock) void k_window(
    const int32_t* __restrict__ rp, int64_t cap_rp, const int32_t* __restrict__ rn,
    int64_t cap_rn, const float* __restrict__ x, const float* __restrict__ y,
    const int32_t* __restrict__ pf, const int64_t* __restrict__ off, int32_t F, int32_t hf,
    int64_t frame0, float* __restrict__ X, float* __restrict__ Y, float* __restrict__ T,
    WinMeta* __restrict__ meta, Bounds* __restrict__ part) {
  const int64_t np = rp ? (int64_t)rp[0] : 0;
  const int64_t nn = rn ? (int64_t)rn[0] : 0;
  const int64_t K = off[F];
  const int64_t total = np + K + nn;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i0 == 0) {
    WinMeta m;
    m.n_prev = np;
    m.n_own = K;
    m.n_next = nn;
    m.k_prev_total = rp ? halo_total(rp) : 0;
    m.n_head = off[hf];
    m.n_tail = K - off[F - hf];
    m.n_window = total;
    m.pad = 0;
    *meta = m;
  }
  auto time_of = [&](int64_t i) -> float {
    if (i < np) return __int_as_float(rp[kHaloHdr + 2 * cap_rp + i]);
    if (i < np + K) return (float)(frame0 + (int64_t)pf[i - np]);
    return __int_as_float(rn[kHaloHdr + 2 * cap_rn + (i - np - K)]);
  };
  BoundsAcc acc;
  for (int64_t i = i0; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    float a, b, c;
    if (i < np) {
      a = __int_as_float(rp[kHaloHdr + i]);
      b = __int_as_float(rp[kHaloHdr + cap_rp + i]);
      c = __int_as_float(rp[kHaloHdr + 2 * cap_rp + i]);
    } else if (i < np + K) {
      const int64_t j = i - np;
      a = x[j];
      b = y[j];
      c = (float)(frame0 + (int64_t)pf[j]);
    } else {
      const int64_t j = i - np - K;
      a = __int_as_float(rn[kHaloHdr + j]);
      b = __int_as_float(rn[kHaloHdr + cap_rn + j]);
      c = __int_as_float(rn[kHaloHdr + 2 * cap_rn + j]);
    }
    X[i] = a;
    Y[i] = b;
    T[i] = c;
    acc.add(a, b, c, i > 0 ? time_of(i - 1) : 0.f, i > 0);
  }
  acc.block_store(part);
}

// the bounds of no point (the identity of k_bounds_final's reduction)
__global__ void k_empty_bounds(Bounds* __restrict__ out) {
  if (threadIdx.x == 0) {
    Bounds b;
    for (int k = 0; k < 4; ++k) {
      b.mn[k] = 0xffffffffu;
      b.mx[k] = 0u;
    }
    b.nonfinite_xyz = b.nonintegral_t = b.n_finite_t = b.t_descends = 0;
    *out = b;
  }
}

// The direct window (the land compaction already wrote the own points at own_off): the halo
// points placed around them -- prev halo at [own_off - np, own_off), next halo at
// [own_off + K, own_off + K + nn) -- the window's counts, and per block the partial of the halo
// points' bounds (k_window's semantics: every point's time against its window predecessor's);
// partial nb is the own points' bounds from the compaction, with the prev halo -> own junction
// folded in, so k_bounds_final over nb + 1 partials gives the window's bounds.
__global__ __launch_bounds__(kBoundsBlock) void k_window_halo(
    const int32_t* __restrict__ rp, int64_t cap_rp, const int32_t* __restrict__ rn,
    int64_t cap_rn, const int64_t* __restrict__ off, int32_t F, int32_t hf, int64_t own_off,
    float* __restrict__ X, float* __restrict__ Y, float* __restrict__ T,
    WinMeta* __restrict__ meta, Bounds* __restrict__ part, int nb,
    const Bounds* __restrict__ own_bnd) {
  const int64_t np = rp ? (int64_t)rp[0] : 0;
  const int64_t nn = rn ? (int64_t)rn[0] : 0;
  const int64_t K = off[F];
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i0 == 0) {
    WinMeta m;
    m.n_prev = np;
    m.n_own = K;
    m.n_next = nn;
    m.k_prev_total = rp ? halo_total(rp) : 0;
    m.n_head = off[hf];
    m.n_tail = K - off[F - hf];
    m.n_window = np + K + nn;
    m.pad = 0;
    *meta = m;
    Bounds o = *own_bnd;
    if (np > 0 && K > 0 && !(__int_as_float(rp[kHaloHdr + 2 * cap_rp + np - 1]) <= T[own_off]))
      o.t_descends = 1;  // (NaN counts as out of order, as in BoundsAcc)
    part[nb] = o;
  }
  BoundsAcc acc;
  for (int64_t h = i0; h < np + nn; h += (int64_t)gridDim.x * blockDim.x) {
    float a, b, c, tp;
    bool hp;
    if (h < np) {
      a = __int_as_float(rp[kHaloHdr + h]);
      b = __int_as_float(rp[kHaloHdr + cap_rp + h]);
      c = __int_as_float(rp[kHaloHdr + 2 * cap_rp + h]);
      const int64_t i = own_off - np + h;
      X[i] = a;
      Y[i] = b;
      T[i] = c;
      hp = h > 0;
      tp = hp ? __int_as_float(rp[kHaloHdr + 2 * cap_rp + h - 1]) : 0.f;
    } else {
      const int64_t j = h - np;
      a = __int_as_float(rn[kHaloHdr + j]);
      b = __int_as_float(rn[kHaloHdr + cap_rn + j]);
      c = __int_as_float(rn[kHaloHdr + 2 * cap_rn + j]);
      const int64_t i = own_off + K + j;
      X[i] = a;
      Y[i] = b;
      T[i] = c;
      // predecessor: the next halo's previous point, else the last own point, else the last
      // prev halo point
      hp = j > 0 || K > 0 || np > 0;
      tp = j > 0 ? __int_as_float(rn[kHaloHdr + 2 * cap_rn + j - 1])
                 : (K > 0 ? T[own_off + K - 1]
                          : (np > 0 ? __int_as_float(rp[kHaloHdr + 2 * cap_rp + np - 1]) : 0.f));
    }
    acc.add(a, b, c, tp, hp);
  }
  acc.block_store(part);
}

// own edge points' global component ids for the neighbours (-1: not core)
__global__ void k_comp_send(const int32_t* __restrict__ comp, WinIds w, int64_t n_head,
                            int64_t n_tail, int64_t* __restrict__ cp, int64_t* __restrict__ cn) {
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  if (cp)
    for (int64_t i = i0; i < n_head; i += step) {
      const int32_t c = comp[w.n_prev + i];
      cp[i] = c >= 0 ? w.gid(c) : -1;
    }
  if (cn)
    for (int64_t i = i0; i < n_tail; i += step) {
      const int32_t c = comp[w.n_prev + w.n_own - n_tail + i];
      cn[i] = c >= 0 ? w.gid(c) : -1;
    }
}

// equivalence pairs (my id of a halo point's component, its owner's), both core, distinct; a
// pair equal to the previous point's is skipped (runs of one component along the halo) and, while
// the pair fits a 64-bit key -- my component's window index (31 bits) and the owner's id as
// (rank - my rank + 2, own index < 2^30) -- every repeat of a pair (device hash set, 2x the halo
// size, so a probe always ends); any rest is merged all the same.  out[0] = the full count (may
// exceed cap: only cap pairs are stored, the caller grows cap and redoes the step).
__global__ void k_pairs(const int32_t* __restrict__ comp, int64_t c0, WinIds w,
                        const int64_t* __restrict__ owner, int64_t n, int64_t cap,
                        unsigned long long* __restrict__ count,
                        unsigned long long* __restrict__ set, uint64_t set_mask,
                        int64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t c = comp[c0 + i];
    const int64_t b = owner[i];
    if (c < 0 || b < 0) continue;
    const int64_t a = w.gid(c);
    if (a == b) continue;
    if (i > 0 && comp[c0 + i - 1] == c && owner[i - 1] == b) continue;
    const int64_t rd = (b >> kGidShift) - w.rank + 2;
    const int64_t bi = b & ((int64_t(1) << kGidShift) - 1);
    if (set && rd >= 0 && rd < 8 && bi < (int64_t(1) << 30)) {
      const unsigned long long key = ((unsigned long long)(uint32_t)c << 33) |
                                     ((unsigned long long)rd << 30) | (unsigned long long)bi;
      uint64_t slot = (key * 0x9E3779B97F4A7C15ull) >> 20;
      bool dup = false;
      for (;; ++slot) {
        slot &= set_mask;
        const unsigned long long prev = atomicCAS(&set[slot], ~0ull, key);
        if (prev == ~0ull) break;
        if (prev == key) {
          dup = true;
          break;
        }
      }
      if (dup) continue;
    }
    const int64_t lo = a < b ? a : b, hi = a < b ? b : a;
    const unsigned long long k = atomicAdd(count, 1ull);
    if ((int64_t)k < cap) {
      out[1 + 2 * k] = lo;
      out[2 + 2 * k] = hi;
    }
  }
}

// the pair count and the distinct-pair set (all ones = empty) of rpt_shard_pairs, in one launch
__global__ void k_pairs_init(unsigned long long* __restrict__ count,
                             unsigned long long* __restrict__ set, uint64_t size) {
  const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i0 == 0) *count = 0ull;
  for (uint64_t i = i0; i < size; i += (uint64_t)gridDim.x * blockDim.x) set[i] = ~0ull;
}

__global__ void k_store_count(const unsigned long long* __restrict__ count,
                              int64_t* __restrict__ out) {
  if (threadIdx.x == 0) out[0] = (int64_t)*count;
}

// Union of every rank's equivalence pairs (the all-gathered rows [count | 2*count ids], rows of
// row_words int64): ONE workgroup, ids in LDS -- bitonic sort, distinct ids, min-hooking
// union-find -- so every rank derives the same (keys sorted, vals = class minimum).  meta[0] = the
// number of ids, or -1 when more than merge_max (<= kMergeMax) would be merged (the caller merges
// on the host; rpt_shard_set_merge_limit lowers merge_max so tests reach that path);
// meta[1] = 1 when some row holds more pairs than its capacity (the step is redone).
__global__ __launch_bounds__(1024) void k_merge_pairs(const int64_t* __restrict__ g, int world,
                                                      int64_t row_words, int merge_max,
                                                      int64_t* __restrict__ keys,
                                                      int64_t* __restrict__ vals,
                                                      int64_t* __restrict__ meta) {
  __shared__ int64_t ids[kMergeMax];
  __shared__ int32_t par[kMergeMax];
  __shared__ int32_t s_total, s_ovf, s_changed, s_m;
  __shared__ int32_t s_wsum[16];
  const int tid = threadIdx.x;
  const int64_t cap = (row_words - 1) / 2;
  if (tid == 0) {
    int64_t tot = 0;
    int ovf = 0;
    for (int q = 0; q < world; ++q) {
      const int64_t c = g[(int64_t)q * row_words];
      ovf |= c > cap ? 1 : 0;
      tot += c < cap ? c : cap;
    }
    s_total = 2 * tot > merge_max ? -1 : (int32_t)tot;
    s_ovf = ovf;
  }
  __syncthreads();
  const int total = s_total;
  if (total < 0) {
    if (tid == 0) {
      meta[0] = -1;
      meta[1] = s_ovf;
    }
    return;
  }
  const int nid = 2 * total;
  int n2 = 2;
  while (n2 < nid) n2 <<= 1;
  // load the ids row by row (rows are few: the owning row by a linear walk)
  for (int i = tid; i < n2; i += 1024) {
    int64_t v = INT64_MAX;
    if (i < nid) {
      int p = i >> 1, q = 0;
      for (;; ++q) {
        const int64_t c = g[(int64_t)q * row_words];
        const int cc = (int)(c < cap ? c : cap);
        if (p < cc) break;
        p -= cc;
      }
      v = g[(int64_t)q * row_words + 1 + 2 * p + (i & 1)];
    }
    ids[i] = v;
  }
  __syncthreads();
  for (int k = 2; k <= n2; k <<= 1)
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < n2; i += 1024) {
        const int l = i ^ j;
        if (l > i) {
          const int64_t a = ids[i], b = ids[l];
          const bool up = (i & k) == 0;
          if ((a > b) == up) {
            ids[i] = b;
            ids[l] = a;
          }
        }
      }
      __syncthreads();
    }
  // distinct ids: a block scan of the run heads, then the survivors move down (in place: a
  // survivor's new position never exceeds its old one, and all reads finish before the writes)
  constexpr int kPer = kMergeMax / 1024;
  int64_t mine[kPer];
  int head[kPer];
  int cnt = 0;
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int i = tid * kPer + u;
    mine[u] = i < nid ? ids[i] : INT64_MAX;
    head[u] = (i < nid && (i == 0 || ids[i - 1] != mine[u])) ? 1 : 0;
    cnt += head[u];
  }
  // block exclusive scan of cnt
  int incl = cnt;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int v = __shfl_up(incl, off);
    if ((tid & 63) >= off) incl += v;
  }
  if ((tid & 63) == 63) s_wsum[tid >> 6] = incl;
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int w = 0; w < 16; ++w) {
      const int v = s_wsum[w];
      s_wsum[w] = run;
      run += v;
    }
    s_m = run;
  }
  __syncthreads();
  int pos = s_wsum[tid >> 6] + incl - cnt;
#pragma unroll
  for (int u = 0; u < kPer; ++u)
    if (head[u]) ids[pos++] = mine[u];
  __syncthreads();
  const int m = s_m;
  for (int i = tid; i < m; i += 1024) par[i] = i;
  // the pairs as index pairs (each thread keeps its own)
  constexpr int kPairsPer = kMergeMax / 2 / 1024;
  int ia[kPairsPer], ib[kPairsPer];
  auto find_id = [&](int64_t v) {
    int lo = 0, hi = m;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (ids[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
  };
#pragma unroll
  for (int u = 0; u < kPairsPer; ++u) {
    const int p = tid + u * 1024;
    ia[u] = -1;
    ib[u] = -1;
    if (p < total) {
      int pp = p, q = 0;
      for (;; ++q) {
        const int64_t c = g[(int64_t)q * row_words];
        const int cc = (int)(c < cap ? c : cap);
        if (pp < cc) break;
        pp -= cc;
      }
      ia[u] = find_id(g[(int64_t)q * row_words + 1 + 2 * pp]);
      ib[u] = find_id(g[(int64_t)q * row_words + 2 + 2 * pp]);
    }
  }
  __syncthreads();
  auto root = [&](int a) {
    while (true) {
      const int p = __hip_atomic_load(&par[a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (p == a) return a;
      a = p;
    }
  };
  for (int it = 0; it < 4 * kMergeMax; ++it) {
    __syncthreads();  // every thread has read the last round's s_changed
    if (tid == 0) s_changed = 0;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kPairsPer; ++u) {
      if (ia[u] < 0) continue;
      const int ra = root(ia[u]), rb = root(ib[u]);
      if (ra != rb) {
        atomicMin(&par[ra > rb ? ra : rb], ra < rb ? ra : rb);
        s_changed = 1;
      }
    }
    __syncthreads();
    for (int i = tid; i < m; i += 1024) par[i] = root(i);  // compress (values only decrease)
    __syncthreads();
    const int ch = s_changed;
    if (!ch) break;
  }
  __syncthreads();
  for (int i = tid; i < m; i += 1024) {
    keys[i] = ids[i];
    vals[i] = ids[root(i)];  // the class root is its smallest index = smallest id
  }
  if (tid == 0) {
    meta[0] = m;
    meta[1] = s_ovf;
  }
}

__device__ __forceinline__ int64_t lookup(const int64_t* __restrict__ keys,
                                          const int64_t* __restrict__ vals, int64_t m, int64_t v) {
  int64_t lo = 0, hi = m;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (keys[mid] < v) lo = mid + 1; else hi = mid;
  }
  return (lo < m && keys[lo] == v) ? vals[lo] : v;
}

// Flags of the representative list, one bit per entry k < keys_cap + n: the merge table's class
// minima below the window (external representatives) here -- a wave per 64 entries writes their
// two words and popcounts, which also clears the window part of both -- and the window points
// that are their own representative by k_root_reps after it.  The list's order comes from a
// scan over the (keys_cap + n) / 32 word counts.
__global__ void k_reps_keys(int64_t n, WinIds w, const int64_t* __restrict__ keys,
                            const int64_t* __restrict__ vals, const int64_t* __restrict__ meta,
                            int64_t keys_cap, uint32_t* __restrict__ bits,
                            int32_t* __restrict__ wcnt) {
  const int64_t m = meta[0] > 0 ? meta[0] : 0;
  const int64_t wstart = w.gid(0);
  const int lane = threadIdx.x & 63;
  const int64_t total = keys_cap + n;
  for (int64_t c0 = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * 64; c0 < total;
       c0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = c0 + lane;
    const bool f = k < keys_cap && k < m && keys[k] == vals[k] && keys[k] < wstart;
    const uint64_t b = __ballot(f);
    if (lane < 2) {
      const uint32_t word = (uint32_t)(b >> (32 * lane));
      bits[(c0 >> 5) + lane] = word;
      wcnt[(c0 >> 5) + lane] = __popc(word);
    }
  }
}

// Per ROOT of the window's core components (a core point s with parent[s] == s; its window
// index i = sorig[s] is the component's id, its minimum original index): rep[i] = the global
// representative (the merge table's class minimum of gid(i), else gid(i) itself) -- the only
// entries of rep the global label pass reads -- and, when the root is its own representative,
// its list flag (after k_reps_keys).  Components are few: the atomics are rare.  Replaces a
// representative per window point (which needed every point's component id).
__global__ void k_root_reps(const uint8_t* __restrict__ core, const int32_t* __restrict__ parent,
                            const int32_t* __restrict__ sorig, int64_t n, WinIds w,
                            const int64_t* __restrict__ keys, const int64_t* __restrict__ vals,
                            const int64_t* __restrict__ meta, int64_t keys_cap,
                            int64_t* __restrict__ rep, uint32_t* __restrict__ bits,
                            int32_t* __restrict__ wcnt) {
  const int64_t m = meta[0] > 0 ? meta[0] : 0;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n;
       s += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t c = core[s];  // (both loads issued together)
    const int32_t p = parent[s];
    if (!c || p != (int32_t)s) continue;
    const int32_t i = sorig[s];
    const int64_t g = w.gid(i);
    const int64_t r = lookup(keys, vals, m, g);
    rep[i] = r;
    if (r == g) {
      const int64_t k = keys_cap + i;
      atomicOr(&bits[k >> 5], 1u << (k & 31));
      atomicAdd(&wcnt[k >> 5], 1);
    }
  }
}

__global__ void k_reps_write(const uint32_t* __restrict__ bits, const int64_t* __restrict__ wpre,
                             int64_t keys_cap, int64_t n, WinIds w,
                             const int64_t* __restrict__ keys, int64_t* __restrict__ reps) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < keys_cap + n;
       k += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t word = bits[k >> 5];
    const uint32_t bit = 1u << (k & 31);
    if (word & bit)
      reps[wpre[k >> 5] + __popc(word & (bit - 1u))] = k < keys_cap ? keys[k] : w.gid(k - keys_cap);
  }
}

// built[f] = frame f holds a K1 point (file offsets of F frames x G files)
// Everything rank 0 needs from this rank, at fixed offsets of a buffer of cap int64 words:
//   [magic, S, n_reps, flags, words, F, frame0, kept] [built F] [first noise F]
//   [count S] [first S] [frame << 32 | label S] [cx | cy << 32 S] [mi S] [reps n_reps]
// flags: 1 this rank's pairs exceeded their capacity, 2 the merge ran on too many ids (host
// merge), 4 the buffer is too small (words holds the size needed).  S = -1: a frame held more
// labels than K9's frame sort takes (redo on the radix path).
__global__ void k_shard_pack(const int32_t* __restrict__ n_seg_dev, const int64_t* __restrict__ nr,
                             const int64_t* __restrict__ mmeta, const int64_t* __restrict__ pairs,
                             int64_t pair_cap, SegPack a, const int64_t* __restrict__ reps,
                             const int64_t* __restrict__ file_off, int32_t G, int32_t F,
                             int64_t frame0, int64_t kept, int64_t* __restrict__ out,
                             int64_t cap) {
  const int64_t S = n_seg_dev ? (int64_t)*n_seg_dev : 0;
  const int64_t R = *nr;
  const int64_t Sp = S > 0 ? S : 0;
  const int64_t words = kHdr + 2 * (int64_t)F + 5 * Sp + R;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  if (i0 == 0) {
    int64_t fl = 0;
    if (pairs && pairs[0] > pair_cap) fl |= 1;
    if (mmeta && (mmeta[1] != 0)) fl |= 1;
    if (mmeta && mmeta[0] < 0) fl |= 2;
    if (words > cap) fl |= 4;
    out[0] = kPackMagic;
    out[1] = S;
    out[2] = R;
    out[3] = fl;
    out[4] = words;
    out[5] = F;
    out[6] = frame0;
    out[7] = kept;
  }
  if (words > cap) return;
  int64_t* built = out + kHdr;
  int64_t* noise = built + F;
  int64_t* cnt = noise + F;
  int64_t* first = cnt + Sp;
  int64_t* fl = first + Sp;
  int64_t* cxy = fl + Sp;
  int64_t* mi = cxy + Sp;
  int64_t* rp = mi + Sp;
  for (int64_t f = i0; f < F; f += step) {
    built[f] = file_off[(int64_t)(f + 1) * G] > file_off[(int64_t)f * G] ? 1 : 0;
    noise[f] = a.noise[f];
  }
  for (int64_t s = i0; s < Sp; s += step) {
    cnt[s] = a.count[s];
    first[s] = a.first[s];
    fl[s] = ((int64_t)a.frame[s] << 32) | (int64_t)(uint32_t)a.label[s];
    cxy[s] = (int64_t)(((uint64_t)__float_as_uint(a.cy[s]) << 32) |
                       (uint64_t)__float_as_uint(a.cx[s]));
    mi[s] = (int64_t)(uint64_t)__float_as_uint(a.mi[s]);
  }
  for (int64_t r = i0; r < R; r += step) rp[r] = reps[r];
}

__global__ void k_map_labels(const int32_t* __restrict__ lab, int64_t n,
                             const int32_t* __restrict__ map, int64_t nr,
                             int32_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t l = lab[i];
    out[i] = (l >= 0 && l < nr) ? map[l] : -1;
  }
}

}  // namespace
}  // namespace rpt

using namespace rpt;

struct rpt_shard {
  rpt_stack st;                  // K1 / land buffers of the stack driver
  rpt::DbscanState* db = nullptr;
  DevBuf<uint32_t> bnd;          // xy bounds (ordered u32)
  DevBuf<float> X, Y, T;         // the window
  // core flags of the window in original order: filled on demand by rpt_shard_points (checks)
  mutable DevBuf<uint8_t> core;
  DevBuf<int32_t> comp, labels, flag;
  DevBuf<int64_t> rep, reps, keys, vals, pos, cnt64, meta;
  DevBuf<unsigned long long> pset;  // distinct-pair hash set
  DevBuf<char> wbnd;             // window meta + bounds (+ partials)
  rpt_stack_params p{};
  int64_t n_points = 0, frame0 = 0;
  int32_t F = 0, G = 0, hf = 0, rank = 0;
  rpt_shard_info info{};
  int64_t n_window = 0, k_prev_total = 0;
  // direct window (land filter on): the compaction wrote the own kept points' x / y / t into
  // X / Y / T at own_off (= the prev halo's capacity); the window then starts at win_base =
  // own_off - n_prev.  Otherwise the window is assembled from the K1 points at 0.
  bool direct = false;
  int64_t own_off = 0, own_cap_next = 0, win_base = 0;
  bool land = false;
  bool k9_radix = false;
  int32_t merge_max = kMergeMax;  // ids the device merge takes (rpt_shard_set_merge_limit)
  hipEvent_t ev[2] = {};         // around the core-flag pass (params.timing)
  bool ev_ok = false, core_timed = false;
  ~rpt_shard() {
    if (ev_ok)
      for (auto& e : ev) (void)hipEventDestroy(e);
    if (db) rpt::dbscan_destroy(db);
    bnd.release();
    X.release();
    Y.release();
    T.release();
    core.release();
    comp.release();
    labels.release();
    flag.release();
    rep.release();
    reps.release();
    keys.release();
    vals.release();
    pos.release();
    cnt64.release();
    meta.release();
    pset.release();
    wbnd.release();
  }
  WinIds ids() const {
    return WinIds{rank, info.n_prev, info.n_kept, k_prev_total};
  }
  // the own kept points' x / y (after the land filter, if any)
  const float* own_x() const { return direct ? X.p + own_off : (st.land_applied ? st.x2.p : st.x.p); }
  const float* own_y() const { return direct ? Y.p + own_off : (st.land_applied ? st.y2.p : st.y.p); }
};

extern "C" {

rpt_shard* rpt_shard_create(void) {
  rpt_shard* h = new rpt_shard();
  h->db = dbscan_create();
  return h;
}

void rpt_shard_destroy(rpt_shard* h) { delete h; }

int32_t rpt_shard_polar(rpt_shard* h, const rpt_stack_params* p, const void* echo,
                        const float* scale, const float* cos_t, const float* sin_t,
                        const int32_t* gain, rpt_shard_info* info, void* stream) {
  clear_error();
  if (!h || !p || !info || !echo || !scale || !cos_t || !sin_t || p->n_frames < 0 ||
      p->files_per_frame < 1 || p->rows <= 0 || p->bins <= 0 || p->stride < 1) {
    set_error("rpt_shard_polar: bad arguments");
    return RPT_EINVAL;
  }
  const hipStream_t st = as_stream(stream);
  RPT_TRY(zero_pool_arm(st));  // the step's counters (this call and the step's later ones)
  rpt_stack& S = h->st;
  h->p = *p;
  S.had_gain = gain != nullptr;  // per-point gains only with a gain table
  const int32_t F = p->n_frames, G = p->files_per_frame;
  h->F = F;
  h->G = G;
  // halo depth: floor(eps_time) frames (a neighbour is at most that many frames away)
  const double et = p->eps_time;
  h->hf = (std::isfinite(et) && et >= 0.0) ? (int32_t)std::min<double>(std::floor(et), F) : 0;
  const int64_t n_files = (int64_t)F * G;
  RPT_TRY(S.file_off.ensure((size_t)n_files + 1, st));
  RPT_TRY(S.row_prefix.ensure((size_t)n_files * p->rows + 1, st));
  RPT_TRY(h->bnd.ensure((size_t)std::max<int64_t>(8, polar_bounds_words()), st));
  const size_t down_bytes = sizeof(int64_t) * (size_t)(n_files + 2) + 16;
  RPT_TRY(S.down.ensure(down_bytes, st));
  const bool grouped = p->echo_dtype == RPT_ECHO_U8 && p->bins == 1024 &&
                       (uintptr_t)echo % 16 == 0;
  if (S.k1_staged < 0) {
    const char* e = ab_env("RPT_K1_STAGE");
    S.k1_staged = (e && std::atoi(e) == 0) ? 0 : 1;
  }
  uint32_t* mk = nullptr;  // staged kept samples, as in rpt_stack_run
  if (grouped && S.k1_staged) {
    RPT_TRY(S.k1_stage.ensure((size_t)polar_stage_words(n_files, p->rows), st));
    mk = S.k1_stage.p;
  }
  RPT_TRY(polar_count(echo, p->echo_dtype, n_files, p->rows, p->bins, p->threshold, p->stride,
                      S.row_prefix.p, S.file_off.p, nullptr, st, mk));
  int64_t spec_cap = -1;
  const int64_t* n_dev = S.file_off.p + n_files;
  if (grouped && S.x.p && S.y.p && S.v.p && S.g.p && S.pf.p) {
    // the write and the bounds are queued with the previous run's capacity; both are redone
    // below when the count exceeds it
    spec_cap = (int64_t)std::min({S.x.cap, S.y.cap, S.v.cap, S.g.cap, S.pf.cap});
    // (the expand write leaves the bounds in h->bnd itself; otherwise a bounds pass)
    bool fused = false;
    RPT_TRY(polar_write_cap((const uint8_t*)echo, n_files, p->rows, p->threshold, p->stride,
                            scale, cos_t, sin_t, gain, S.row_prefix.p, S.file_off.p, G, S.x.p,
                            S.y.p, S.v.p, gain ? S.g.p : nullptr, S.pf.p, spec_cap, st, mk,
                            mk ? h->bnd.p : nullptr, &fused));
    if (!fused) {
      hipLaunchKernelGGL(k_init_bounds, dim3(1), dim3(64), 0, st, h->bnd.p);
      hipLaunchKernelGGL(k_xy_bounds_part,
                         dim3(grid_for(std::max<int64_t>(spec_cap, 1), 256, 512)), dim3(256), 0,
                         st, S.x.p, S.y.p, spec_cap, n_dev, h->bnd.p);
    }
    RPT_CHECK_LAUNCH();
  }
  // one readback: file offsets (their last entry is the count) and the bounds
  int64_t* hfo = reinterpret_cast<int64_t*>(S.down.p);
  RPT_HIP(hipMemcpyAsync(hfo, S.file_off.p, sizeof(int64_t) * (n_files + 1),
                         hipMemcpyDeviceToHost, st));
  uint32_t* hb = reinterpret_cast<uint32_t*>(hfo + n_files + 1);
  if (spec_cap >= 0)
    RPT_HIP(hipMemcpyAsync(hb, h->bnd.p, 16, hipMemcpyDeviceToHost, st));
  RPT_TRY(wait_stream(st));
  const int64_t N = hfo[n_files];
  if (N > spec_cap) {
    const size_t cap = (size_t)std::max<int64_t>(N, 1);
    RPT_TRY(S.x.ensure(cap, st));
    RPT_TRY(S.y.ensure(cap, st));
    RPT_TRY(S.v.ensure(cap, st));
    RPT_TRY(S.g.ensure(cap, st));
    RPT_TRY(S.pf.ensure(cap, st));
    bool fused = false;
    RPT_TRY(polar_write(echo, p->echo_dtype, n_files, p->rows, p->bins, scale, cos_t, sin_t, gain,
                        p->threshold, p->stride, S.row_prefix.p, S.file_off.p, G, S.x.p, S.y.p,
                        S.v.p, gain ? S.g.p : nullptr, S.pf.p, st, mk, mk ? h->bnd.p : nullptr,
                        &fused));
    if (!fused) {
      hipLaunchKernelGGL(k_init_bounds, dim3(1), dim3(64), 0, st, h->bnd.p);
      hipLaunchKernelGGL(k_xy_bounds_part, dim3(grid_for(std::max<int64_t>(N, 1), 256, 512)),
                         dim3(256), 0, st, S.x.p, S.y.p, N, (const int64_t*)nullptr, h->bnd.p);
    }
    RPT_CHECK_LAUNCH();
    RPT_HIP(hipMemcpyAsync(hb, h->bnd.p, 16, hipMemcpyDeviceToHost, st));
    RPT_TRY(wait_stream(st));
  }
  S.fo_k1.resize((size_t)F + 1);
  for (int32_t f = 0; f <= F; ++f) S.fo_k1[(size_t)f] = hfo[(size_t)f * G];
  int32_t built = 0;
  for (int32_t f = 0; f < F; ++f) built += S.fo_k1[(size_t)f + 1] > S.fo_k1[(size_t)f];
  h->n_points = N;
  h->info = rpt_shard_info{};
  rpt_shard_info& I = h->info;
  I.n_points = N;
  I.n_built = built;
  I.halo_frames = h->hf;
  if (N > 0) {
    I.bounds[0] = ord_to_f(hb[0]);
    I.bounds[1] = ord_to_f(hb[1]);
    I.bounds[2] = ord_to_f(hb[2]);
    I.bounds[3] = ord_to_f(hb[3]);
  } else {
    I.bounds[0] = I.bounds[2] = INFINITY;
    I.bounds[1] = I.bounds[3] = -INFINITY;
  }
  I.n_head_k1 = S.fo_k1[(size_t)h->hf];
  I.n_tail_k1 = N - S.fo_k1[(size_t)(F - h->hf)];
  I.n_kept = N;
  *info = I;
  return RPT_OK;
}

int64_t rpt_shard_land_cells(const float* gbounds, double resolution) {
  if (!gbounds) return 0;
  const int64_t nx = (int64_t)arange_edges(gbounds[0], gbounds[1], resolution).size();
  const int64_t ny = (int64_t)arange_edges(gbounds[2], gbounds[3], resolution).size();
  return (nx >= 2 && ny >= 2) ? (nx - 1) * (ny - 1) : 0;
}

int32_t rpt_shard_land_grid(rpt_shard* h, const float* gbounds, double* grid, int64_t cells,
                            void* stream) {
  clear_error();
  if (!h || !gbounds || !grid) {
    set_error("rpt_shard_land_grid: bad arguments");
    return RPT_EINVAL;
  }
  const hipStream_t st = as_stream(stream);
  rpt_stack& S = h->st;
  const std::vector<double> xe = arange_edges(gbounds[0], gbounds[1], h->p.land_resolution);
  const std::vector<double> ye = arange_edges(gbounds[2], gbounds[3], h->p.land_resolution);
  const int32_t nxe = (int32_t)xe.size(), nye = (int32_t)ye.size();
  if (nxe < 2 || nye < 2 || (int64_t)(nxe - 1) * (nye - 1) != cells) {
    set_error("rpt_shard_land_grid: grid of %lld cells does not match the bounds",
              (long long)cells);
    return RPT_EINVAL;
  }
  const size_t n_up = (size_t)(nxe + nye);
  RPT_TRY(S.edges.ensure(n_up, st));
  RPT_TRY(S.up.ensure(sizeof(double) * n_up, st));  // its last upload completed: syncs since
  double* he = reinterpret_cast<double*>(S.up.p);
  std::memcpy(he, xe.data(), sizeof(double) * nxe);
  std::memcpy(he + nxe, ye.data(), sizeof(double) * nye);
  RPT_HIP(hipMemcpyAsync(S.edges.p, he, sizeof(double) * n_up, hipMemcpyHostToDevice, st));
  const size_t cap = (size_t)std::max<int64_t>(h->n_points, 1);
  RPT_TRY(S.land_cnt.ensure((size_t)cells, st));
  RPT_TRY(S.land_cell.ensure(cap, st));
  RPT_TRY(land_grid_cells(S.x.p, S.y.p, S.v.p, h->n_points, S.edges.p, nxe, S.edges.p + nxe,
                          nye, S.land_cnt.p, grid + cells, S.land_cell.p, st,
                          h->p.echo_dtype == RPT_ECHO_U8 ? 1 : 0));
  hipLaunchKernelGGL(k_cnt_to_f64, dim3(grid_for(cells, 256, 1024)), dim3(256), 0, st,
                     S.land_cnt.p, cells, grid);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

int32_t rpt_shard_halo(rpt_shard* h, const double* grid, int64_t cells, int32_t n_built_global,
                       int32_t rank, int64_t frame0, int32_t* send_prev, int32_t* send_next,
                       int64_t recv_cap_prev, int64_t recv_cap_next, void* stream) {
  clear_error();
  if (!h || rank < 0 || recv_cap_prev < 0 || recv_cap_next < 0) {
    set_error("rpt_shard_halo: bad arguments");
    return RPT_EINVAL;
  }
  const hipStream_t st = as_stream(stream);
  rpt_stack& S = h->st;
  const int32_t F = h->F;
  const int64_t N = h->n_points;
  h->rank = rank;
  h->frame0 = frame0;
  RPT_TRY(S.new_off.ensure((size_t)F + 2, st));
  RPT_TRY(S.scal.ensure(4, st));
  h->land = grid != nullptr && cells > 0;
  if (h->land) {
    RPT_TRY(S.land_cnt.ensure((size_t)cells, st));
    RPT_TRY(S.land_mask.ensure((size_t)cells, st));
    hipLaunchKernelGGL(k_f64_to_cnt, dim3(grid_for(cells, 256, 1024)), dim3(256), 0, st, grid,
                       cells, S.land_cnt.p, reinterpret_cast<int64_t*>(S.scal.p));
    RPT_CHECK_LAUNCH();
    RPT_TRY(land_mask_dev(S.land_cnt.p, grid + cells, cells, n_built_global, h->p.land_persistence,
                          h->p.land_min_intensity, S.land_mask.p,
                          reinterpret_cast<int32_t*>(S.scal.p), st));
    const size_t cap = (size_t)std::max<int64_t>(N, 1);
    RPT_TRY(S.v2.ensure(cap, st));
    RPT_TRY(S.g2.ensure(cap, st));
    RPT_TRY(S.pf2.ensure(cap, st));
    RPT_TRY(S.bnd.ensure(2 * sizeof(Bounds), st));
    // the window's arrays: [prev halo capacity | own (<= N) | next halo capacity]; the fused
    // compaction (kept points in order, new frame offsets and the own points' ST-DBSCAN bounds
    // on the device) writes x / y / t (= frame0 + frame slot) straight into the own part, so the
    // window phase only places the halo points around them
    const int64_t wcap = std::max<int64_t>(recv_cap_prev + N + recv_cap_next, 1);
    RPT_TRY(h->X.ensure((size_t)wcap, st));
    RPT_TRY(h->Y.ensure((size_t)wcap, st));
    RPT_TRY(h->T.ensure((size_t)wcap, st));
    h->direct = true;
    h->own_off = recv_cap_prev;
    h->own_cap_next = recv_cap_next;
    if (N > 0)
      RPT_TRY(land_compact_dev(S.x.p, S.y.p, S.v.p, S.had_gain ? S.g.p : nullptr, S.pf.p, N,
                               S.land_cell.p, S.land_mask.p, F, h->X.p + h->own_off,
                               h->Y.p + h->own_off, S.v2.p, S.had_gain ? S.g2.p : nullptr,
                               S.pf2.p, h->T.p + h->own_off, S.new_off.p,
                               reinterpret_cast<Bounds*>(S.bnd.p), st, frame0));
    else {
      RPT_HIP(hipMemsetAsync(S.new_off.p, 0, sizeof(int64_t) * (F + 1), st));
      hipLaunchKernelGGL(k_empty_bounds, dim3(1), dim3(64), 0, st,
                         reinterpret_cast<Bounds*>(S.bnd.p));
      RPT_CHECK_LAUNCH();
    }
  } else {
    h->direct = false;
    h->own_off = 0;
    RPT_HIP(hipMemsetAsync(S.scal.p, 0, sizeof(int64_t), st));  // (read back with the window)
    // no land filter: the kept points are the K1 points, offsets from the host copy
    RPT_TRY(S.up.ensure(sizeof(int64_t) * (size_t)(F + 1), st));
    std::memcpy(S.up.p, S.fo_k1.data(), sizeof(int64_t) * (F + 1));
    RPT_HIP(hipMemcpyAsync(S.new_off.p, S.up.p, sizeof(int64_t) * (F + 1), hipMemcpyHostToDevice,
                           st));
  }
  S.land_applied = h->land;
  const float* cx = h->own_x();
  const float* cy = h->own_y();
  const int32_t* cpf = h->land ? S.pf2.p : S.pf.p;
  if (send_prev || send_next) {
    const int64_t m = std::max(h->info.n_head_k1, h->info.n_tail_k1);
    hipLaunchKernelGGL(k_halo_pack, dim3(grid_for(std::max<int64_t>(m, 1), 256, 1024)), dim3(256),
                       0, st, cx, cy, cpf, S.new_off.p, F, h->hf, frame0, send_prev,
                       h->info.n_head_k1, send_next, h->info.n_tail_k1);
    RPT_CHECK_LAUNCH();
  }
  return RPT_OK;
}

int32_t rpt_shard_window(rpt_shard* h, const int32_t* recv_prev, int64_t cap_prev,
                         const int32_t* recv_next, int64_t cap_next, uint8_t* flags_prev,
                         uint8_t* flags_next, rpt_shard_info* info, void* stream) {
  clear_error();
  if (!h || !info || cap_prev < 0 || cap_next < 0 || (cap_prev > 0 && !recv_prev) ||
      (cap_next > 0 && !recv_next)) {
    set_error("rpt_shard_window: bad arguments");
    return RPT_EINVAL;
  }
  const hipStream_t st = as_stream(stream);
  rpt_stack& S = h->st;
  const int32_t F = h->F;
  const int64_t N = h->n_points;
  if (h->direct && (cap_prev != h->own_off || cap_next != h->own_cap_next)) {
    set_error("rpt_shard_window: halo capacities %lld / %lld differ from rpt_shard_halo's "
              "%lld / %lld", (long long)cap_prev, (long long)cap_next, (long long)h->own_off,
              (long long)h->own_cap_next);
    return RPT_EINVAL;
  }
  const int64_t wcap = std::max<int64_t>(cap_prev + N + cap_next, 1);
  if (!h->direct) {
    RPT_TRY(h->X.ensure((size_t)wcap, st));
    RPT_TRY(h->Y.ensure((size_t)wcap, st));
    RPT_TRY(h->T.ensure((size_t)wcap, st));
  }
  const size_t bb = stdbscan_bounds_bytes();
  const size_t part = stdbscan_bounds_part_bytes(wcap);
  RPT_TRY(h->wbnd.ensure(sizeof(WinMeta) + bb + part + sizeof(Bounds) + 256, st));
  WinMeta* meta = reinterpret_cast<WinMeta*>(h->wbnd.p);
  char* bnd = h->wbnd.p + sizeof(WinMeta);
  char* bpart = bnd + align_up(bb, 16);
  if (h->direct) {
    // (halo partials: at most grid_for(cap_prev + cap_next) <= grid_for(wcap), + the own one)
    const int nbh = grid_for(std::max<int64_t>(cap_prev + cap_next, 1), kBoundsBlock, 1024);
    hipLaunchKernelGGL(k_window_halo, dim3(nbh), dim3(kBoundsBlock), 0, st,
                       cap_prev > 0 ? recv_prev : nullptr, cap_prev,
                       cap_next > 0 ? recv_next : nullptr, cap_next, S.new_off.p, F, h->hf,
                       h->own_off, h->X.p, h->Y.p, h->T.p, meta,
                       reinterpret_cast<Bounds*>(bpart), nbh,
                       reinterpret_cast<const Bounds*>(S.bnd.p));
    RPT_CHECK_LAUNCH();
    RPT_TRY(stdbscan_bounds_final_dev(bpart, nbh + 1, bnd, st));
  } else {
    const float* cx = h->own_x();
    const float* cy = h->own_y();
    const int32_t* cpf = h->land ? S.pf2.p : S.pf.p;
    // (the partials' count is the bounds pass's grid: stdbscan_bounds_part_bytes)
    const int nbw = grid_for(wcap, kBoundsBlock, 1024);
    hipLaunchKernelGGL(k_window, dim3(nbw), dim3(kBoundsBlock), 0, st,
                       cap_prev > 0 ? recv_prev : nullptr, cap_prev,
                       cap_next > 0 ? recv_next : nullptr, cap_next, cx, cy, cpf, S.new_off.p, F,
                       h->hf, h->frame0, h->X.p, h->Y.p, h->T.p, meta,
                       reinterpret_cast<Bounds*>(bpart));
    RPT_CHECK_LAUNCH();
    RPT_TRY(stdbscan_bounds_final_dev(bpart, nbw, bnd, st));
  }
  // ONE readback: window counts, grid bounds, land-cell count, the kept frame offsets
  PackList pl;
  pl.add(meta, sizeof(WinMeta));
  pl.add(bnd, align_up(bb, 8));
  pl.add(S.scal.p, sizeof(int64_t));
  pl.add(S.new_off.p, sizeof(int64_t) * (F + 1));
  RPT_TRY(S.pack_d.ensure((size_t)pl.off[pl.k], st));
  RPT_TRY(S.down.ensure(sizeof(uint32_t) * (size_t)pl.off[pl.k], st));
  RPT_TRY(pack_arrays(pl, S.pack_d.p, st));
  RPT_HIP(hipMemcpyAsync(S.down.p, S.pack_d.p, sizeof(uint32_t) * (size_t)pl.off[pl.k],
                         hipMemcpyDeviceToHost, st));
  RPT_TRY(wait_stream(st));
  WinMeta hm;
  std::memcpy(&hm, S.down.p, sizeof(WinMeta));
  std::vector<char> hb(bb);
  std::memcpy(hb.data(), S.down.p + 4 * pl.off[1], bb);
  int64_t land_cells = 0;
  std::memcpy(&land_cells, S.down.p + 4 * pl.off[2], sizeof(int64_t));
  const int64_t* hoff = reinterpret_cast<const int64_t*>(S.down.p + 4 * pl.off[3]);
  S.fo_in.assign(hoff, hoff + F + 1);
  rpt_shard_info& I = h->info;
  I.n_kept = hm.n_own;
  I.n_head = hm.n_head;
  I.n_tail = hm.n_tail;
  I.n_prev = hm.n_prev;
  I.n_next = hm.n_next;
  I.n_land_cells = h->land ? land_cells : 0;
  h->k_prev_total = hm.k_prev_total;
  h->n_window = hm.n_window;
  S.n_frames = F;
  S.n_in = hm.n_own;
  *info = I;
  const int64_t n = hm.n_window;
  h->win_base = h->direct ? h->own_off - hm.n_prev : 0;
  if (n <= 0) return RPT_OK;
  // grid build sized on the host from the bounds just read, then K5
  const int64_t wb = h->win_base;
  RPT_TRY(dbscan_build_given(h->db, h->X.p + wb, h->Y.p + wb, h->T.p + wb, n, h->p.eps_space,
                             h->p.eps_time, h->p.min_samples, hb.data(), st));
  if (h->p.timing) {
    if (!h->ev_ok) {
      RPT_HIP(hipEventCreate(&h->ev[0]));
      RPT_HIP(hipEventCreate(&h->ev[1]));
      h->ev_ok = true;
    }
    RPT_HIP(hipEventRecord(h->ev[0], st));
  }
  RPT_TRY(dbscan_core(h->db, nullptr, st));  // (flags stay in sorted order)
  if (h->p.timing) RPT_HIP(hipEventRecord(h->ev[1], st));
  h->core_timed = h->p.timing != 0;
  // the own edge points' flags for the neighbours (their halo), straight into the send buffers
  RPT_TRY(dbscan_core_edges(h->db, hm.n_prev, hm.n_prev + hm.n_head, flags_prev,
                            hm.n_prev + hm.n_own - hm.n_tail, hm.n_prev + hm.n_own, flags_next,
                            st));
  return RPT_OK;
}

double rpt_shard_core_ms(rpt_shard* h) {
  if (!h || !h->core_timed) return -1.0;
  float ms = 0.f;
  if (hipEventSynchronize(h->ev[1]) != hipSuccess ||
      hipEventElapsedTime(&ms, h->ev[0], h->ev[1]) != hipSuccess)
    return -1.0;
  return ms;
}

int32_t rpt_shard_link(rpt_shard* h, const uint8_t* flags_prev, const uint8_t* flags_next,
                       int64_t* comp_prev, int64_t* comp_next, void* stream) {
  clear_error();
  if (!h || (h->info.n_prev > 0 && !flags_prev) || (h->info.n_next > 0 && !flags_next)) {
    set_error("rpt_shard_link: bad arguments");
    return RPT_EINVAL;
  }
  const hipStream_t st = as_stream(stream);
  const int64_t n = h->n_window;
  if (n <= 0) return RPT_OK;
  const rpt_shard_info& I = h->info;
  // halo points take their owners' flags (the owners see all their neighbours)
  RPT_TRY(h->comp.ensure((size_t)n, st));
  RPT_TRY(dbscan_set_core_edges(h->db, I.n_prev > 0 ? flags_prev : nullptr, I.n_prev,
                                I.n_next > 0 ? flags_next : nullptr, I.n_prev + I.n_kept, st));
  // component ids only where they are read: the halo points (k_pairs) and the own edge points
  // sent to the neighbours (k_comp_send); the labels take each root's representative directly
  // (k_root_reps)
  const int64_t lo_end = I.n_prev + (comp_prev ? I.n_head : 0);
  const int64_t hi_begin = I.n_prev + I.n_kept - (comp_next ? I.n_tail : 0);
  RPT_TRY(dbscan_components_edges(h->db, h->comp.p, lo_end, hi_begin, st));
  if ((comp_prev && I.n_head > 0) || (comp_next && I.n_tail > 0)) {
    hipLaunchKernelGGL(k_comp_send,
                       dim3(grid_for(std::max<int64_t>(std::max(I.n_head, I.n_tail), 1), 256, 1024)),
                       dim3(256), 0, st, h->comp.p, h->ids(), I.n_head, I.n_tail, comp_prev,
                       comp_next);
    RPT_CHECK_LAUNCH();
  }
  return RPT_OK;
}

int32_t rpt_shard_pairs(rpt_shard* h, const int64_t* owner_prev, const int64_t* owner_next,
                        int64_t* pairs, int64_t cap, void* stream) {
  clear_error();
  const rpt_shard_info& I = h ? h->info : rpt_shard_info{};
  if (!h || !pairs || cap < 0 || (I.n_prev > 0 && !owner_prev) ||
      (I.n_next > 0 && !owner_next)) {
    set_error("rpt_shard_pairs: bad arguments");
    return RPT_EINVAL;
  }
  const hipStream_t st = as_stream(stream);
  RPT_TRY(h->cnt64.ensure(2, st));
  auto* cnt = reinterpret_cast<unsigned long long*>(h->cnt64.p);
  uint64_t tsize = 64;
  while (tsize < (uint64_t)(2 * (I.n_prev + I.n_next))) tsize <<= 1;
  RPT_TRY(h->pset.ensure((size_t)tsize, st));
  hipLaunchKernelGGL(k_pairs_init, dim3(grid_for((int64_t)tsize, 256, 1024)), dim3(256), 0, st,
                     cnt, h->pset.p, tsize);
  const WinIds w = h->ids();
  if (I.n_prev > 0 && h->n_window > 0)
    hipLaunchKernelGGL(k_pairs, dim3(grid_for(I.n_prev, 256, 1024)), dim3(256), 0, st, h->comp.p,
                       (int64_t)0, w, owner_prev, I.n_prev, cap, cnt, h->pset.p, tsize - 1,
                       pairs);
  if (I.n_next > 0 && h->n_window > 0)
    hipLaunchKernelGGL(k_pairs, dim3(grid_for(I.n_next, 256, 1024)), dim3(256), 0, st, h->comp.p,
                       I.n_prev + I.n_kept, w, owner_next, I.n_next, cap, cnt, h->pset.p,
                       tsize - 1, pairs);
  hipLaunchKernelGGL(k_store_count, dim3(1), dim3(64), 0, st, cnt, pairs);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

int32_t rpt_shard_finish(rpt_shard* h, const int64_t* gathered_pairs, int32_t world,
                         int64_t row_words, const int64_t* own_pairs, const int64_t* keys_host,
                         const int64_t* vals_host, int64_t n_keys, int32_t force_radix,
                         int64_t* out, int64_t out_cap, void* stream) {
  clear_error();
  if (!h || !out || out_cap < kHdr || world < 1 || (gathered_pairs && row_words < 1) ||
      (!gathered_pairs && n_keys > 0 && (!keys_host || !vals_host))) {
    set_error("rpt_shard_finish: bad arguments");
    return RPT_EINVAL;
  }
  const hipStream_t st = as_stream(stream);
  rpt_stack& S = h->st;
  const int64_t n = h->n_window, K = h->info.n_kept;
  const int32_t F = h->F;
  if (force_radix) h->k9_radix = true;
  // ---- equivalence table (keys sorted, vals = class minimum), identical on every rank
  const int64_t keys_cap = gathered_pairs ? (int64_t)kMergeMax : std::max<int64_t>(n_keys, 1);
  RPT_TRY(h->keys.ensure((size_t)keys_cap, st));
  RPT_TRY(h->vals.ensure((size_t)keys_cap, st));
  RPT_TRY(h->meta.ensure(4, st));
  if (gathered_pairs) {
    hipLaunchKernelGGL(k_merge_pairs, dim3(1), dim3(1024), 0, st, gathered_pairs, world,
                       row_words, (int)h->merge_max, h->keys.p, h->vals.p, h->meta.p);
    RPT_CHECK_LAUNCH();
  } else {
    RPT_TRY(S.up.ensure(sizeof(int64_t) * (size_t)(2 * n_keys + 2), st));
    int64_t* hu = reinterpret_cast<int64_t*>(S.up.p);
    hu[0] = n_keys;
    hu[1] = 0;
    if (n_keys > 0) {
      std::memcpy(hu + 2, keys_host, sizeof(int64_t) * n_keys);
      std::memcpy(hu + 2 + n_keys, vals_host, sizeof(int64_t) * n_keys);
      RPT_HIP(hipMemcpyAsync(h->keys.p, hu + 2, sizeof(int64_t) * n_keys, hipMemcpyHostToDevice,
                             st));
      RPT_HIP(hipMemcpyAsync(h->vals.p, hu + 2 + n_keys, sizeof(int64_t) * n_keys,
                             hipMemcpyHostToDevice, st));
    }
    RPT_HIP(hipMemcpyAsync(h->meta.p, hu, 2 * sizeof(int64_t), hipMemcpyHostToDevice, st));
    // the upload buffer is reused only after the next readback (a sync) of this handle
  }
  // ---- representatives: rep per window point, the sorted list of those the window sees
  const WinIds w = h->ids();
  RPT_TRY(h->rep.ensure((size_t)std::max<int64_t>(n, 1), st));
  const size_t lw = (size_t)(2 * ((keys_cap + n + 63) / 64));  // list words (k_reps)
  RPT_TRY(h->flag.ensure(std::max((size_t)(keys_cap + n + 1), 2 * lw), st));
  RPT_TRY(h->pos.ensure(std::max((size_t)(keys_cap + n + 1), lw + 1), st));
  RPT_TRY(h->reps.ensure((size_t)(keys_cap + n + 1), st));
  // list entries as bits: nw words (a multiple of two), their popcounts after them in flag
  const int64_t nw = 2 * ((keys_cap + n + 63) / 64);
  uint32_t* rbits = reinterpret_cast<uint32_t*>(h->flag.p);
  int32_t* rcnt = h->flag.p + nw;
  if (n > 0) {
    hipLaunchKernelGGL(k_reps_keys, dim3(grid_for(keys_cap + n, 256, 4096)), dim3(256), 0, st, n,
                       w, h->keys.p, h->vals.p, h->meta.p, keys_cap, rbits, rcnt);
    const uint8_t* dcore;
    const int32_t *dpar, *dsorig;
    int64_t dn = 0;
    dbscan_uf_arrays(h->db, &dcore, &dpar, &dsorig, &dn);
    hipLaunchKernelGGL(k_root_reps, dim3(grid_for(dn, 256, 4096)), dim3(256), 0, st, dcore, dpar,
                       dsorig, dn, w, h->keys.p, h->vals.p, h->meta.p, keys_cap, h->rep.p, rbits,
                       rcnt);
    RPT_CHECK_LAUNCH();
    RPT_TRY(exclusive_scan_total_i32_to_i64(rcnt, h->pos.p, nw, st));
    hipLaunchKernelGGL(k_reps_write, dim3(grid_for(keys_cap + n, 256, 4096)), dim3(256), 0, st,
                       rbits, h->pos.p, keys_cap, n, w, h->keys.p, h->reps.p);
    RPT_CHECK_LAUNCH();
  } else {
    RPT_HIP(hipMemsetAsync(h->pos.p + nw, 0, sizeof(int64_t), st));
  }
  const int64_t* nr_dev = h->pos.p + nw;
  // ---- labels of the window (local numbering), K9 of the own points
  RPT_TRY(h->labels.ensure((size_t)std::max<int64_t>(n, 1), st));
  if (n > 0) RPT_TRY(dbscan_labels_global_dev(h->db, h->rep.p, h->reps.p, nr_dev, h->labels.p, st));
  const bool l = S.land_applied;
  const float* x = h->own_x();
  const float* y = h->own_y();
  const float* v = l ? S.v2.p : S.v.p;
  const int32_t* pf = l ? S.pf2.p : S.pf.p;
  const size_t cap2 = (size_t)std::max<int64_t>(K, 1);
  RPT_TRY(S.seg_frame.ensure(cap2, st));
  RPT_TRY(S.seg_label.ensure(cap2, st));
  RPT_TRY(S.seg_count.ensure(cap2, st));
  RPT_TRY(S.seg_first.ensure(cap2, st));
  RPT_TRY(S.seg_cx.ensure(cap2, st));
  RPT_TRY(S.seg_cy.ensure(cap2, st));
  RPT_TRY(S.seg_mi.ensure(cap2, st));
  RPT_TRY(S.first_noise.ensure((size_t)std::max(F, 1), st));
  const int32_t* nseg_dev = nullptr;
  if (K > 0) {
    // label bits only matter on the radix path; the labels are below keys_cap + n
    const int bits = radix_bits_for(keys_cap + n);
    RPT_TRY(cluster_summaries_dev(h->labels.p + h->info.n_prev, x, y, v, pf, K, F, bits,
                                  K, S.seg_frame.p,
                                  S.seg_label.p, S.seg_count.p, S.seg_first.p, S.seg_cx.p,
                                  S.seg_cy.p, S.seg_mi.p, S.first_noise.p, &nseg_dev,
                                  h->k9_radix, nullptr, st));
  } else if (F > 0) {  // no own point: every frame without noise
    RPT_HIP(hipMemsetAsync(S.first_noise.p, 0xFF, sizeof(int64_t) * F, st));
  }
  SegPack sp{S.seg_count.p, S.seg_first.p, S.first_noise.p, S.seg_frame.p,
             S.seg_label.p, S.seg_cx.p,    S.seg_cy.p,      S.seg_mi.p};
  const int64_t pair_cap = row_words > 0 ? (row_words - 1) / 2 : 0;
  hipLaunchKernelGGL(k_shard_pack, dim3(grid_for(std::max<int64_t>(K, F) + 1, 256, 512)),
                     dim3(256), 0, st, nseg_dev, nr_dev, h->meta.p,
                     own_pairs, pair_cap, sp, h->reps.p, S.file_off.p, h->G, F, h->frame0, K,
                     out, out_cap);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

int32_t rpt_shard_labels(const rpt_shard* h, const int32_t* local_to_global, int64_t n_reps,
                         int32_t* out, void* stream) {
  clear_error();
  if (!h || !out || n_reps < 0 || (n_reps > 0 && !local_to_global)) {
    set_error("rpt_shard_labels: bad arguments");
    return RPT_EINVAL;
  }
  const int64_t K = h->info.n_kept;
  if (K == 0) return RPT_OK;
  if (!h->labels.p || h->labels.cap < (size_t)(h->info.n_prev + K)) {
    set_error("rpt_shard_labels: no labels (rpt_shard_finish first)");
    return RPT_EINVAL;
  }
  hipLaunchKernelGGL(k_map_labels, dim3(grid_for(K, 256, 4096)), dim3(256), 0, as_stream(stream),
                     h->labels.p + h->info.n_prev, K, local_to_global, n_reps, out);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

}  // extern "C"

// (rank 0's host stage and the equivalence merge: shard_host.cpp)

extern "C" {

int32_t rpt_shard_set_merge_limit(rpt_shard* h, int32_t max_ids) {
  clear_error();
  if (!h || max_ids < 0) {
    set_error("rpt_shard_set_merge_limit: bad arguments");
    return RPT_EINVAL;
  }
  h->merge_max = std::min<int32_t>(max_ids, kMergeMax);
  return RPT_OK;
}

int32_t rpt_shard_points(const rpt_shard* h, float* x, float* y, float* intensity,
                         int32_t* point_frame, uint8_t* core, void* stream) {
  clear_error();
  if (!h) {
    set_error("rpt_shard_points: bad arguments");
    return RPT_EINVAL;
  }
  const int64_t K = h->info.n_kept;
  if (K == 0) return RPT_OK;
  const rpt_stack& S = h->st;
  if (core && h->n_window < h->info.n_prev + K) {
    set_error("rpt_shard_points: no core flags (rpt_shard_window first)");
    return RPT_EINVAL;
  }
  const hipStream_t st = as_stream(stream);
  if (core) {  // the window's final core flags in original order (checks only)
    RPT_TRY(h->core.ensure((size_t)h->n_window, st));
    RPT_TRY(dbscan_core_orig(h->db, h->core.p, st));
  }
  const bool l = S.land_applied;
  auto cp = [&](void* dst, const void* src, size_t bytes) -> int32_t {
    if (dst) RPT_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st));
    return RPT_OK;
  };
  RPT_TRY(cp(x, h->own_x(), sizeof(float) * (size_t)K));
  RPT_TRY(cp(y, h->own_y(), sizeof(float) * (size_t)K));
  RPT_TRY(cp(intensity, l ? S.v2.p : S.v.p, sizeof(float) * (size_t)K));
  RPT_TRY(cp(point_frame, l ? S.pf2.p : S.pf.p, sizeof(int32_t) * (size_t)K));
  RPT_TRY(cp(core, h->core.p + h->info.n_prev, (size_t)K));
  return RPT_OK;
}

int32_t rpt_shard_frame_offsets(const rpt_shard* h, int32_t which, int64_t* out) {
  if (!h) return RPT_EINVAL;
  return rpt_stack_frame_offsets(&h->st, which, out);
}

}  // extern "C"
