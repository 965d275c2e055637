// K9: per-(frame, label) cluster summaries.  Replaces the per-frame Cluster extraction of
// PointCloudWork/4_temporal_object_tracker.py:508-536 (Cluster :143-158).
//
// Reduction orders are numpy's, reproduced exactly:
//   centroid       = np.mean(pts (k,2) float32, axis=0): sequential float32 sum in point order
//                    starting from the first point, then one float32 division by k;
//   mean_intensity = np.mean(I (k,) float32): np.add.reduce over 8192-element buffer chunks,
//                    each chunk summed pairwise (numpy pairwise_sum: 8 accumulators up to 128
//                    elements, halving split above), chunks accumulated sequentially, then a
//                    float32 division by k.
// Segments: a stable per-frame counting sort (one 8-wave block per frame, labels hashed to LDS
// slots; up to kFsMaxKeys labels per frame) or, beyond that, a stable radix sort of (label+1,
// index) keeps each label's points in index order, so every (frame, label) run is contiguous and
// ordered; segments come frame-major (hash order inside a frame) from the counting sort,
// label-major from the radix sort (consumers bucket them by frame, tracker.cpp order_clusters).
// Runs of up to kLaneChainMax points: one lane per run (k_runs_lane: 64 runs' order-preserving
// float32 chains per add instruction); a longer run takes one wave for its x and y chains (lanes 0
// and 1, fed from LDS, so it costs ~k dependent adds of ~4.4 cycles, not k memory latencies) and
// one for its intensity.
// Radix path: noise (key 0) sorts first in index order, so each frame's first noise point is the
// head of its frame within the noise run (no atomics).
#include <climits>
#include <cstdlib>

#include <algorithm>

#include "common.h"

#pragma clang fp contract(off)

namespace rpt {
namespace {

constexpr int kBlock = 256;

__global__ void k_sum_keys(const int32_t* __restrict__ labels, int64_t n,
                           uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    keys[i] = (uint32_t)(labels[i] + 1);  // noise (-1) -> 0, sorts first
    vals[i] = (uint32_t)i;
  }
}

// head[p] = 1 where a (label, frame) run starts among clustered points; for the noise run, the
// first noise point of each frame is recorded.
__global__ void k_heads(const uint32_t* __restrict__ sk, const uint32_t* __restrict__ sv,
                        const int32_t* __restrict__ pf, int64_t n, int32_t* __restrict__ head,
                        int64_t* __restrict__ first_noise) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t k = sk[p], i = sv[p];
    const int32_t f = pf[i];
    const bool h = (p == 0) || k != sk[p - 1] || f != pf[sv[p - 1]];
    head[p] = (k != 0u && h) ? 1 : 0;
    if (k == 0u && h && first_noise) first_noise[f] = (int64_t)i;
  }
}

__global__ void k_seg_starts(const int32_t* __restrict__ head, const int32_t* __restrict__ pos,
                             int64_t n, int64_t* __restrict__ seg_start) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * blockDim.x)
    if (head[p]) seg_start[pos[p]] = p;
}

// numpy pairwise_sum over a[b .. b+len) (float32), iterative form of the recursion.  Only
// reached when intensities are not small non-negative integers (see k_summarize).
__device__ float pairwise_f32(const float* __restrict__ a, int64_t b, int64_t len) {
  int64_t sb[40], sl[40];
  int st[40];
  float vs[40];
  int sp = 0, vp = 0;
  sb[0] = b;
  sl[0] = len;
  st[0] = 0;
  sp = 1;
  while (sp > 0) {
    const int64_t bb = sb[sp - 1], ll = sl[sp - 1];
    if (ll < 8) {
      float r = 0.f;  // numpy: res = 0.; res += a[i]
      for (int64_t i = 0; i < ll; ++i) r = r + a[bb + i];
      --sp;
      vs[vp++] = r;
    } else if (ll <= 128) {
      float r[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) r[k] = a[bb + k];
      int64_t i = 8;
      for (; i < ll - (ll % 8); i += 8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = r[k] + a[bb + i + k];
      }
      float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
      for (; i < ll; ++i) res = res + a[bb + i];
      --sp;
      vs[vp++] = res;
    } else {
      int64_t n2 = ll / 2;
      n2 -= n2 % 8;
      if (st[sp - 1] == 0) {
        st[sp - 1] = 1;
        sb[sp] = bb;  // left half first
        sl[sp] = n2;
        st[sp] = 0;
        ++sp;
      } else if (st[sp - 1] == 1) {
        st[sp - 1] = 2;
        sb[sp] = bb + n2;
        sl[sp] = ll - n2;
        st[sp] = 0;
        ++sp;
      } else {
        const float right = vs[--vp];
        const float left = vs[--vp];
        --sp;
        vs[vp++] = left + right;
      }
    }
  }
  return vs[0];
}

// points of every run gathered contiguously (coalesced writes, one gather read per point)
__global__ void k_gather_runs(const uint32_t* __restrict__ sv, int64_t n,
                              const float* __restrict__ x, const float* __restrict__ y,
                              const float* __restrict__ inten, float* __restrict__ gx,
                              float* __restrict__ gy, float* __restrict__ gi) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t i = sv[p];
    gx[p] = x[i];
    gy[p] = y[i];
    gi[p] = inten[i];
  }
}

// Order-preserving float32 sums of gx[b..e) and gy[b..e) (np.add.reduce from the first element),
// computed by ONE wave: lanes stage 1,024-element chunks of both in the wave's LDS slice (the next
// chunks' loads in flight meanwhile) and the chains run in lane 0 (x) and lane 1 (y) of the same
// instructions, each lane consuming 16-byte LDS reads of its own half issued a batch ahead: one
// dependent v_add_f32 (~4.4 cycles on gfx950, tools/microbench/chain.hip) per element advances
// both chains, so a run costs one SIMD's issue slots once, not twice (a packed x/y add would be
// no faster: 8.5 cycles).  Lane 0 returns the x sum, lane 1 the y sum (other lanes repeat them).
constexpr int kSeqChunk = 1024;
__device__ __forceinline__ float seq_sum(const float* __restrict__ gx,
                                         const float* __restrict__ gy, int b, int e, int lane,
                                         float* __restrict__ sbuf) {
  constexpr int kPre = kSeqChunk / 64, kChunk = kSeqChunk, V = 8;
  float pre[kPre], prey[kPre];
  auto load_chunk = [&](int c0) {
#pragma unroll
    for (int t = 0; t < kPre; ++t) {
      const int idx = c0 + t * 64 + lane;
      pre[t] = (idx < e) ? gx[idx] : 0.f;
      prey[t] = (idx < e) ? gy[idx] : 0.f;
    }
  };
  float* __restrict__ sb = sbuf + (lane & 1) * kChunk;  // this lane's chain: x or y
  float acc = 0.f;
  load_chunk(b);
  for (int c0 = b; c0 < e; c0 += kChunk) {
#pragma unroll
    for (int t = 0; t < kPre; ++t) {
      sbuf[t * 64 + lane] = pre[t];
      sbuf[kChunk + t * 64 + lane] = prey[t];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (c0 + kChunk < e) load_chunk(c0 + kChunk);
    const int m = (e - c0 < kChunk) ? (e - c0) : kChunk;
    int i = 0;
    if (c0 == b) {  // start from the first element, then reach a 4-aligned position
      acc = sb[0];
      for (i = 1; i < 4 && i < m; ++i) acc = acc + sb[i];
    }
    const float4* sb4 = reinterpret_cast<const float4*>(sb);
    if (i == 0 && m == kChunk) {
      // a whole chunk (the bulk of a long run): two 32-element register windows in ping-pong,
      // each filled by ONE burst of 8 LDS reads issued a window ahead of its adds (bursts, not
      // four reads between every 16 adds: 1.70 -> 1.56 ms on the dense share's 490 k-point
      // chains, tools/microbench/chain_lds.hip, where 64-element windows measure the same; the
      // dependent add alone, register operands, costs 5.0 cycles there and this feed 7.6)
      constexpr int kW = 8, kNw = kChunk / (4 * kW);
      float4 wa[kW], wb[kW];
#pragma unroll
      for (int u = 0; u < kW; ++u) wa[u] = sb4[u];
#pragma unroll
      for (int w = 0; w < kNw; w += 2) {
#pragma unroll
        for (int u = 0; u < kW; ++u) wb[u] = sb4[(w + 1) * kW + u];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < kW; ++u) {
          acc = acc + wa[u].x;
          acc = acc + wa[u].y;
          acc = acc + wa[u].z;
          acc = acc + wa[u].w;
        }
        if (w + 2 < kNw) {
#pragma unroll
          for (int u = 0; u < kW; ++u) wa[u] = sb4[(w + 2) * kW + u];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < kW; ++u) {
          acc = acc + wb[u].x;
          acc = acc + wb[u].y;
          acc = acc + wb[u].z;
          acc = acc + wb[u].w;
        }
      }
      i = kChunk;
    } else if (i + 8 * V <= m) {
      // ping-pong register batches: the next 4V elements are read from LDS while the chain
      // consumes the current ones (no register copies between batches)
      float4 pa[V], pb[V];
#pragma unroll
      for (int u = 0; u < V; ++u) pa[u] = sb4[i / 4 + u];
      while (true) {
#pragma unroll
        for (int u = 0; u < V; ++u) pb[u] = sb4[i / 4 + V + u];
        __builtin_amdgcn_sched_barrier(0);  // keep the next batch's reads ahead of the chain
#pragma unroll
        for (int u = 0; u < V; ++u) {
          acc = acc + pa[u].x;
          acc = acc + pa[u].y;
          acc = acc + pa[u].z;
          acc = acc + pa[u].w;
        }
        i += 4 * V;
        if (i + 8 * V > m) {
#pragma unroll
          for (int u = 0; u < V; ++u) {
            acc = acc + pb[u].x;
            acc = acc + pb[u].y;
            acc = acc + pb[u].z;
            acc = acc + pb[u].w;
          }
          i += 4 * V;
          break;
        }
#pragma unroll
        for (int u = 0; u < V; ++u) pa[u] = sb4[i / 4 + V + u];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < V; ++u) {
          acc = acc + pb[u].x;
          acc = acc + pb[u].y;
          acc = acc + pb[u].z;
          acc = acc + pb[u].w;
        }
        i += 4 * V;
        if (i + 8 * V > m) {
#pragma unroll
          for (int u = 0; u < V; ++u) {
            acc = acc + pa[u].x;
            acc = acc + pa[u].y;
            acc = acc + pa[u].z;
            acc = acc + pa[u].w;
          }
          i += 4 * V;
          break;
        }
      }
    }
    for (; i < m; ++i) acc = acc + sb[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  return acc;
}

// Mean intensity of g[b..e) by one wave: when every intensity is a non-negative integer and the
// total stays below 2^24, every summation order is exact (integer lane sums), which equals
// numpy's pairwise result; otherwise numpy's chunked pairwise sum is evaluated by lane 0.
// 32 loads per lane in flight per round.
__device__ __forceinline__ float mean_intensity(const float* __restrict__ gi, int b, int e,
                                                int lane) {
  constexpr int kU = 32;
  uint64_t isum = 0;
  bool small_int = true;
  for (int c0 = b; c0 < e; c0 += 64 * kU) {
    float v[kU];
#pragma unroll
    for (int t = 0; t < kU; ++t) {
      const int idx = c0 + t * 64 + lane;
      v[t] = idx < e ? gi[idx] : 0.f;
    }
#pragma unroll
    for (int t = 0; t < kU; ++t) {
      small_int = small_int && (v[t] >= 0.f && v[t] == floorf(v[t]) && v[t] < 16777216.f);
      isum += (uint32_t)v[t];
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) isum += __shfl_xor(isum, off);
  const bool all_int = __all(small_int);
  const int k = e - b;
  const float fk = (float)k;
  if (all_int && isum < 16777216u) return (float)isum / fk;
  float tot = 0.f;
  if (lane == 0)
    for (int64_t c = 0; c < k; c += 8192) {
      const int64_t len = (k - c < 8192) ? (k - c) : 8192;
      tot = tot + pairwise_f32(gi, b + c, len);
    }
  return tot / fk;
}

// Runs of at most kLaneChainMax points are summarised one LANE per run (k_runs_lane below);
// longer runs take a wave for both chains (seq_sum: a wave-wide chain issues one or two useful
// adds per wave instruction, and thousands of short runs made K9 VALU-issue and latency bound).
// A lane streams ~32 points per memory round trip, a wave's chain ~1,000 per 4 us: the lane form
// wins only for short runs (3,072 made the 125-frame stack's K9 slower: 143 us of lane chains).
constexpr int kLaneChainMax = 128;

// META: run [b, e) of segment su (o_count holds the lengths: runs are not adjacent, noise slots
// sit between frames); otherwise runs tile [0, n).
template <bool META>
__device__ __forceinline__ void run_bounds(const int64_t* __restrict__ seg_start,
                                           const int64_t* __restrict__ o_count, int64_t n_seg,
                                           int64_t n, int64_t su, int& b, int& e) {
  b = (int)seg_start[su];
  e = META ? (int)(b + o_count[su]) : (int)((su + 1 < n_seg) ? seg_start[su + 1] : n);
}

// One lane per run: lane l of wave w summarises run 64 w + l -- the x and y chains
// (sequentially from the first point, np.mean axis 0) and the intensity sum (exact integer sum,
// see mean_intensity; numpy's pairwise sum by the lane otherwise) in one pass over 16-B loads,
// kLq float4s of each column per block, all in flight together: 64 runs' chains advance per add
// instruction, and the loads in flight per lane bound it (a radar stack's runs are a few points
// each, plus one long run per frame).  Runs longer than kLaneChainMax are listed for k_summarize
// (long_list / *n_long, zeroed beforehand) instead.  Every lane takes part in the wave-level
// steps; lanes without a run of their own walk an empty range.
constexpr int kLq = 8;  // float4 loads per column per block (32 points)
template <bool META>
__global__ __launch_bounds__(kBlock, 2) void k_runs_lane(
    const uint32_t* __restrict__ sk, const uint32_t* __restrict__ sv,
    const int64_t* __restrict__ seg_start, const int32_t* __restrict__ n_seg_dev, int64_t n,
    const float* __restrict__ gx, const float* __restrict__ gy, const float* __restrict__ gi,
    const int32_t* __restrict__ pf, int32_t* __restrict__ o_frame, int32_t* __restrict__ o_label,
    int64_t* __restrict__ o_count, int64_t* __restrict__ o_first, float* __restrict__ o_cx,
    float* __restrict__ o_cy, float* __restrict__ o_mi, int32_t* __restrict__ long_list,
    int32_t* __restrict__ n_long) {
  const int64_t n_seg = *n_seg_dev;
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (int64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
  const int64_t nw = (int64_t)gridDim.x * (kBlock / 64);
  const int64_t groups = (n_seg + 63) / 64;
  for (int64_t w = w0; w < groups; w += nw) {  // (wave-uniform)
    const int64_t su = w * 64 + lane;
    const bool valid = su < n_seg;
    int b = 0, e = 0;
    if (valid) run_bounds<META>(seg_start, o_count, n_seg, n, su, b, e);
    const bool lng = valid && e - b > kLaneChainMax;
    const uint64_t lm = __ballot(lng);
    if (lm) {
      int base = 0;
      if (lane == 0) base = atomicAdd(n_long, __popcll(lm));
      base = __shfl(base, 0);
      if (lng) long_list[base + __popcll(lm & ((1ull << lane) - 1ull))] = (int32_t)su;
    }
    const bool mine = valid && !lng;
    if (!mine) b = e = 0;
    float ax = 0.f, ay = 0.f;
    uint64_t isum = 0;
    bool small_int = true;
    auto ivisit = [&](float v, bool on) {
      const bool ok = v >= 0.f && v == floorf(v) && v < 16777216.f;
      small_int = small_int && (ok || !on);
      isum += on ? (uint64_t)(uint32_t)v : 0ull;
    };
    int i = b;
    if (i < e) {
      ax = gx[i];
      ay = gy[i];
      ivisit(gi[i], true);
      ++i;
    }
    for (; i < e && (i & 3); ++i) {
      ax = ax + gx[i];
      ay = ay + gy[i];
      ivisit(gi[i], true);
    }
    // whole float4s [i, i + 4 nq) in blocks of kLq per column; the block loop runs to the wave's
    // largest block count with branch-free loads (a lane past its own blocks re-reads a valid
    // block, the longest lane's if it has none) and selects instead of branches around the adds
    const int nq = (e - i) >> 2;
    const int nblk = nq / kLq;
    int nbmax = nblk;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) nbmax = max(nbmax, __shfl_xor(nbmax, off));
    if (nbmax > 0) {
      const int lmax = __ffsll((unsigned long long)__ballot(nblk == nbmax)) - 1;
      const int i0 = nblk > 0 ? i : __shfl(i, lmax);
      const int last = nblk > 0 ? nblk - 1 : 0;
      const float4* __restrict__ px = reinterpret_cast<const float4*>(gx + i0);
      const float4* __restrict__ py = reinterpret_cast<const float4*>(gy + i0);
      const float4* __restrict__ pi = reinterpret_cast<const float4*>(gi + i0);
      for (int k = 0; k < nbmax; ++k) {
        const int kk = min(k, last);
        float4 qx[kLq], qy[kLq], qi[kLq];
#pragma unroll
        for (int u = 0; u < kLq; ++u) {
          qx[u] = px[kk * kLq + u];
          qy[u] = py[kk * kLq + u];
          qi[u] = pi[kk * kLq + u];
        }
        const bool on = k < nblk;
#pragma unroll
        for (int u = 0; u < kLq; ++u) {
          float tx = ax + qx[u].x, ty = ay + qy[u].x;
          tx = tx + qx[u].y;
          ty = ty + qy[u].y;
          tx = tx + qx[u].z;
          ty = ty + qy[u].z;
          tx = tx + qx[u].w;
          ty = ty + qy[u].w;
          ax = on ? tx : ax;
          ay = on ? ty : ay;
          ivisit(qi[u].x, on);
          ivisit(qi[u].y, on);
          ivisit(qi[u].z, on);
          ivisit(qi[u].w, on);
        }
      }
    }
    for (int q = nblk * kLq; q < nq; ++q) {
      const float4 vx = reinterpret_cast<const float4*>(gx + i)[q];
      const float4 vy = reinterpret_cast<const float4*>(gy + i)[q];
      const float4 vi = reinterpret_cast<const float4*>(gi + i)[q];
      ax = ax + vx.x;
      ax = ax + vx.y;
      ax = ax + vx.z;
      ax = ax + vx.w;
      ay = ay + vy.x;
      ay = ay + vy.y;
      ay = ay + vy.z;
      ay = ay + vy.w;
      ivisit(vi.x, true);
      ivisit(vi.y, true);
      ivisit(vi.z, true);
      ivisit(vi.w, true);
    }
    for (i += 4 * nq; i < e; ++i) {
      ax = ax + gx[i];
      ay = ay + gy[i];
      ivisit(gi[i], true);
    }
    if (mine) {
      const int k = e - b;
      const float fk = (float)k;
      o_cx[su] = ax / fk;
      o_cy[su] = ay / fk;
      float mi;
      if (small_int && isum < 16777216u) {
        mi = (float)isum / fk;
      } else {  // numpy's pairwise sum (k <= kLaneChainMax < 8192: one buffer chunk)
        float tot = 0.f;
        tot = tot + pairwise_f32(gi, b, k);
        mi = tot / fk;
      }
      o_mi[su] = mi;
      if (!META) {
        const uint32_t i0 = sv[b];
        o_frame[su] = pf[i0];
        o_label[su] = (int32_t)sk[b] - 1;
        o_count[su] = k;
        o_first[su] = i0;
      }
    }
  }
}

// The runs longer than kLaneChainMax (k_runs_lane's list): two waves each, one for the mean
// intensity (lane-parallel) and one for the x and y chains (np.mean axis 0, sequential float32 in
// index order; seq_sum) -- pure dependent-add chains, so no other work sits in their instruction
// stream.  META: the frame sort already wrote frame/label/count/first; otherwise the metadata
// comes from the sorted keys (written by the intensity wave).
template <bool META>
// 2 waves/SIMD (up to 256 VGPRs: the x and y prefetch registers and the chain's two register
// windows; 4 waves spilled 17; a long run's waves are few, occupancy does not bound them)
__global__ __launch_bounds__(kBlock, 2) void k_summarize(
    const uint32_t* __restrict__ sk, const uint32_t* __restrict__ sv,
    const int64_t* __restrict__ seg_start, const int32_t* __restrict__ n_seg_dev, int64_t n,
    const float* __restrict__ gx, const float* __restrict__ gy, const float* __restrict__ gi,
    const int32_t* __restrict__ pf, int32_t* __restrict__ o_frame, int32_t* __restrict__ o_label,
    int64_t* __restrict__ o_count, int64_t* __restrict__ o_first, float* __restrict__ o_cx,
    float* __restrict__ o_cy, float* __restrict__ o_mi, const int32_t* __restrict__ long_list,
    const int32_t* __restrict__ n_long_dev) {
  __shared__ float s_buf[kBlock / 64][2 * kSeqChunk];
  const int64_t n_seg = *n_seg_dev;  // the segment count stays on the device (no readback)
  const int64_t n_long = *n_long_dev;
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (int64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
  const int64_t nw = (int64_t)gridDim.x * (kBlock / 64);
  for (int64_t w = w0; w < 2 * n_long; w += nw) {
    const int su = __builtin_amdgcn_readfirstlane(long_list[w >> 1]);
    const int comp = __builtin_amdgcn_readfirstlane((int)(w & 1));
    int b, e;
    run_bounds<META>(seg_start, o_count, n_seg, n, su, b, e);
    b = __builtin_amdgcn_readfirstlane(b);
    e = __builtin_amdgcn_readfirstlane(e);
    const int k = e - b;
    const float fk = (float)k;
    if (comp == 1) {
      const float mi = mean_intensity(gi, b, e, lane);
      if (lane == 0) {
        o_mi[su] = mi;
        if (!META) {
          const uint32_t i0 = sv[b];
          o_frame[su] = pf[i0];
          o_label[su] = (int32_t)sk[b] - 1;
          o_count[su] = k;
          o_first[su] = i0;
        }
      }
      continue;
    }
    const float sum = seq_sum(gx, gy, b, e, lane, s_buf[threadIdx.x / 64]);
    if (lane < 2) (lane ? o_cy : o_cx)[su] = sum / fk;
  }
}

// pandas groupby(...).mean() of float32 columns (pandas/_libs/groupby.pyx group_mean, pandas
// 2.x): per group, in row order, a float32 Kahan-compensated sum (y = v - c; t = s + y;
// c = (t - s) - y; c = 0 if NaN; s = t), then s / (float)count.  One wave per run: lanes stage
// chunks in LDS, lane 0 runs the dependent chain.
__device__ __forceinline__ float kahan_mean(const float* __restrict__ g, int b, int e, int lane,
                                            float* __restrict__ sb) {
  constexpr int kPre = 16, kChunk = 64 * kPre;
  float s = 0.f, c = 0.f;
  for (int c0 = b; c0 < e; c0 += kChunk) {
#pragma unroll
    for (int t = 0; t < kPre; ++t) {
      const int idx = c0 + t * 64 + lane;
      sb[t * 64 + lane] = (idx < e) ? g[idx] : 0.f;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int m = (e - c0 < kChunk) ? (e - c0) : kChunk;
    if (lane == 0)
      for (int i = 0; i < m; ++i) {
        const float y = sb[i] - c;
        const float t = s + y;
        c = (t - s) - y;
        if (c != c) c = 0.f;
        s = t;
      }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  return s / (float)(e - b);
}

// head[p] = 1 where a label run starts among clustered points (noise, key 0, excluded)
__global__ void k_label_heads(const uint32_t* __restrict__ sk, int64_t n,
                              int32_t* __restrict__ head) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t k = sk[p];
    head[p] = (k != 0u && (p == 0 || k != sk[p - 1])) ? 1 : 0;
  }
}

// Three waves per label run: x, y, intensity group means; outputs indexed by label.
__global__ __launch_bounds__(kBlock) void k_label_means(
    const uint32_t* __restrict__ sk, const int64_t* __restrict__ seg_start,
    const int32_t* __restrict__ n_seg_dev, int64_t n, const float* __restrict__ gx,
    const float* __restrict__ gy, const float* __restrict__ gi, int64_t n_labels,
    int64_t* __restrict__ o_count, float* __restrict__ o_x, float* __restrict__ o_y,
    float* __restrict__ o_v) {
  __shared__ float s_buf[kBlock / 64][1024];
  const int64_t n_seg = *n_seg_dev;
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (int64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
  const int64_t nw = (int64_t)gridDim.x * (kBlock / 64);
  for (int64_t w = w0; w < 3 * n_seg; w += nw) {
    const int su = __builtin_amdgcn_readfirstlane((int)(w / 3));
    const int comp = __builtin_amdgcn_readfirstlane((int)(w - (int64_t)su * 3));
    const int b = __builtin_amdgcn_readfirstlane((int)seg_start[su]);
    const int e = __builtin_amdgcn_readfirstlane(
        (int)((su + 1 < n_seg) ? seg_start[su + 1] : n));
    const int64_t lab = (int64_t)sk[b] - 1;
    const float m = kahan_mean(comp == 0 ? gx : (comp == 1 ? gy : gi), b, e, lane,
                               s_buf[threadIdx.x / 64]);
    if (lane == 0 && lab < n_labels) {
      if (comp == 0) {
        o_x[lab] = m;
        o_count[lab] = e - b;
      } else if (comp == 1) {
        o_y[lab] = m;
      } else {
        o_v[lab] = m;
      }
    }
  }
}

// ---- per-frame counting sort (point_frame non-decreasing) ----------------------------------
// One 16-wave block per frame (8 waves: the frame's chunk chain per wave set the time at 125 frames).  Each wave owns a contiguous part of the frame's points; the frame's
// clustered labels get LDS hash slots (at most kFsMaxKeys distinct labels per frame, else the
// frame reports an overflow and the caller redoes K9 on the radix path), counted per (wave, slot),
// scanned into frame-local offsets and per-wave cursors, and the points scattered stably — a
// (frame, label) run is then contiguous and in index order, as the radix path gives.  Noise is
// not scattered; each frame's first noise point is the first one of its lowest wave.
constexpr int kFsWaves = 16, kFsSlots = 1024, kFsMaxKeys = kFsSlots / 2;
constexpr int kFsSpt = kFsSlots / (kFsWaves * 64);  // scan slots per thread
static_assert(kFsSpt >= 1 && kFsSpt * kFsWaves * 64 == kFsSlots, "frame sort slot split");

struct FsLds {
  int keys[kFsSlots];               // label + 1 per slot, or -1
  uint32_t cnt[kFsWaves][kFsSlots]; // per-wave counts, then per-wave cursors
  int off[kFsSlots];                // run start (frame-local) per slot
  uint32_t wsum[2][kFsWaves];
  int fnoise[kFsWaves];
  int nkeys, overflow;
};

__device__ __forceinline__ uint32_t fs_hash(int v) {
  return ((uint32_t)v * 2654435761u) >> (32 - 10);
}

__device__ int fs_insert(FsLds& L, int v) {
  uint32_t s = fs_hash(v);
  for (int probe = 0; probe < kFsSlots; ++probe) {
    const int k = __atomic_load_n(&L.keys[s], __ATOMIC_RELAXED);
    if (k == v) return (int)s;
    if (k == -1) {
      const int old = atomicCAS(&L.keys[s], -1, v);
      if (old == -1) {
        if (atomicAdd(&L.nkeys, 1) >= kFsMaxKeys) L.overflow = 1;
        return (int)s;
      }
      if (old == v) return (int)s;
    }
    s = (s + 1) & (kFsSlots - 1);
  }
  L.overflow = 1;
  return -1;
}

__device__ __forceinline__ int fs_find_keys(const int* keys, int v) {
  uint32_t s = fs_hash(v);
  for (int probe = 0; probe < kFsSlots; ++probe) {
    const int k = keys[s];
    if (k == v) return (int)s;
    if (k == -1) return -1;
    s = (s + 1) & (kFsSlots - 1);
  }
  return -1;
}
__device__ __forceinline__ int fs_find(const FsLds& L, int v) { return fs_find_keys(L.keys, v); }

// Lanes with equal keys in this 64-point step: the lowest such lane (leader), the lane's rank
// among them and their number.  One ballot per distinct key, scalar loop.
__device__ __forceinline__ void wave_group(int v, bool valid, int lane, int& leader, int& rank,
                                           int& cnt) {
  uint64_t rem = __ballot(valid);
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  leader = -1;
  rank = 0;
  cnt = 0;
  while (rem) {
    const int l = __builtin_ctzll(rem);
    const int u = __builtin_amdgcn_readlane(v, l);
    const bool mine = valid && v == u;
    const uint64_t m = __ballot(mine);
    if (mine) {
      leader = l;
      rank = __popcll(m & lt);
      cnt = __popcll(m);
    }
    rem &= ~m;
  }
}

// first index with a[i] >= key in the non-decreasing a[0, n), by the WHOLE wave (uniform
// arguments, every lane active; the result is uniform): a 64-ary search, 64 probes per round, ~5
// dependent rounds over a 50 M-point stack where a thread's binary search took 26 -- the frame
// sort blocks began with two such searches each
__device__ __forceinline__ int64_t lower_bound_i32(const int32_t* __restrict__ a, int64_t n,
                                                   int32_t key) {
  const int lane = threadIdx.x & 63;
  int64_t lo = 0, hi = n;  // the answer lies in [lo, hi]
  while (lo < hi) {
    const int64_t step = (hi - lo + 63) / 64;
    const int64_t idx = lo + (int64_t)lane * step;
    const bool below = idx < hi && a[idx < hi ? idx : lo] < key;  // a prefix of the lanes
    const int c = __popcll(__ballot(below));
    if (c == 0) {
      hi = lo;
    } else {
      const int64_t nlo = lo + (int64_t)(c - 1) * step + 1;
      hi = min(hi, lo + (int64_t)c * step);
      lo = nlo;
    }
  }
  return lo;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x, int lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t o = __shfl_up(x, off);
    if (lane >= off) x += o;
  }
  return x;
}

// Per segment q of the frame the frame-local lists at [lo + q] get the run's start position,
// length and label; tmp_first[start] gets the run's first point index.
__global__ __launch_bounds__(kFsWaves * 64) void k_frame_sort(
    const int32_t* __restrict__ labels, const int32_t* __restrict__ pf, int64_t n,
    const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ inten,
    float* __restrict__ gx, float* __restrict__ gy, float* __restrict__ gi,
    int32_t* __restrict__ fstart, int32_t* __restrict__ tmp_start, int32_t* __restrict__ tmp_len,
    int32_t* __restrict__ tmp_label, int32_t* __restrict__ tmp_first,
    int32_t* __restrict__ nseg_f, int64_t* __restrict__ first_noise,
    int32_t* __restrict__ overflow) {
  __shared__ FsLds L;
  const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lo = __builtin_amdgcn_readfirstlane((int)lower_bound_i32(pf, n, f));
  const int hi = __builtin_amdgcn_readfirstlane((int)lower_bound_i32(pf, n, f + 1));
  for (int s = tid; s < kFsSlots; s += kFsWaves * 64) {
    L.keys[s] = -1;
#pragma unroll
    for (int q = 0; q < kFsWaves; ++q) L.cnt[q][s] = 0u;
  }
  if (tid == 0) {
    L.nkeys = 0;
    L.overflow = 0;
    fstart[f] = lo;
  }
  __syncthreads();
  // this wave's chunks of 64 points
  const int nch = (hi - lo + 63) / 64, cpw = (nch + kFsWaves - 1) / kFsWaves;
  const int cb0 = w * cpw, cb1 = min(nch, cb0 + cpw);
  // pass 1: counts per (wave, slot), one LDS update per distinct label per step (its leader)
  int wfn = INT_MAX;
  constexpr int U1 = 8;
  for (int cb = cb0; cb < cb1; cb += U1) {
    int lab[U1];
#pragma unroll
    for (int u = 0; u < U1; ++u) {
      const int i = lo + (cb + u) * 64 + lane;
      lab[u] = (cb + u < cb1 && i < hi) ? labels[i] : -2;
    }
#pragma unroll
    for (int u = 0; u < U1; ++u) {
      const int v = lab[u] + 1;
      if (wfn == INT_MAX) {
        const uint64_t m0 = __ballot(v == 0);
        if (m0) wfn = lo + (cb + u) * 64 + __builtin_ctzll(m0);
      }
      const bool valid = v >= 1;
      int leader, rank, cm;
      wave_group(v, valid, lane, leader, rank, cm);
      if (valid && lane == leader) {
        const int s = fs_insert(L, v);
        if (s >= 0) L.cnt[w][s] += (uint32_t)cm;
      }
    }
  }
  if (lane == 0) L.fnoise[w] = wfn;
  __syncthreads();
  if (L.overflow) {
    if (tid == 0) {
      nseg_f[f] = 0;
      atomicExch(overflow, 1);
    }
    return;
  }
  if (tid == 0 && first_noise) {
    int m = INT_MAX;
#pragma unroll
    for (int q = 0; q < kFsWaves; ++q) m = min(m, L.fnoise[q]);
    if (m != INT_MAX) first_noise[f] = m;
  }
  // scan: kFsSpt consecutive slots per thread; run offsets and segment slots in slot order
  uint32_t tt[kFsSpt];
  uint32_t a = 0u, pcount = 0u;
#pragma unroll
  for (int j = 0; j < kFsSpt; ++j) {
    const int sj = kFsSpt * tid + j;
    uint32_t t = 0u;
#pragma unroll
    for (int q = 0; q < kFsWaves; ++q) t += L.cnt[q][sj];
    tt[j] = t;
    a += t;
    pcount += (t != 0u);
  }
  const uint32_t ia = wave_incl_scan(a, lane), ip = wave_incl_scan(pcount, lane);
  if (lane == 63) {
    L.wsum[0][w] = ia;
    L.wsum[1][w] = ip;
  }
  __syncthreads();
  uint32_t pa = 0, pp = 0, ta = 0, tp = 0;
#pragma unroll
  for (int q = 0; q < kFsWaves; ++q) {
    if (q < w) {
      pa += L.wsum[0][q];
      pp += L.wsum[1][q];
    }
    ta += L.wsum[0][q];
    tp += L.wsum[1][q];
  }
  const uint32_t eo = pa + ia - a, eq = pp + ip - pcount;
  auto emit = [&](int s, uint32_t t, uint32_t o, uint32_t q) {
    if (t == 0u) return;
    L.off[s] = (int)o;
    tmp_start[lo + q] = lo + (int)o;
    tmp_len[lo + q] = (int)t;
    tmp_label[lo + q] = L.keys[s] - 1;
    uint32_t run = o;
#pragma unroll
    for (int r = 0; r < kFsWaves; ++r) {
      const uint32_t c = L.cnt[r][s];
      L.cnt[r][s] = run;
      run += c;
    }
  };
  {
    uint32_t o = eo, q = eq;
#pragma unroll
    for (int j = 0; j < kFsSpt; ++j) {
      emit(kFsSpt * tid + j, tt[j], o, q);
      o += tt[j];
      q += (tt[j] != 0u);
    }
  }
  if (tid == 0) nseg_f[f] = (int)tp;
  (void)ta;
  __syncthreads();
  // pass 2: stable scatter through the per-wave cursors
  constexpr int U2 = 4;
  for (int cb = cb0; cb < cb1; cb += U2) {
    int lab[U2];
    float px[U2], py[U2], pv[U2];
#pragma unroll
    for (int u = 0; u < U2; ++u) {
      const int i = lo + (cb + u) * 64 + lane;
      const bool in = cb + u < cb1 && i < hi;
      lab[u] = in ? labels[i] : -2;
      px[u] = in ? x[i] : 0.f;
      py[u] = in ? y[i] : 0.f;
      pv[u] = in ? inten[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U2; ++u) {
      const int i = lo + (cb + u) * 64 + lane;
      const int v = lab[u] + 1;
      const bool valid = v >= 1;
      int leader, rank, cm;
      wave_group(v, valid, lane, leader, rank, cm);
      int base = 0;
      if (valid && lane == leader) {
        const int s = fs_find(L, v);
        base = (int)L.cnt[w][s];
        L.cnt[w][s] = (uint32_t)(base + cm);
        if (base == L.off[s]) tmp_first[lo + base] = i;
      }
      base = __shfl(base, leader < 0 ? lane : leader);
      if (valid) {
        const int p = lo + base + rank;
        gx[p] = px[u];
        gy[p] = py[u];
        gi[p] = pv[u];
      }
    }
  }
}

// ---- the per-frame counting sort with C blocks per frame (frames of hundreds of thousands of
// points: one block per frame left most CUs idle for the whole sort -- the dense share's 125
// frames on 256 CUs).  Chunk c of frame f is its points [lo + len*c/C, lo + len*(c+1)/C), each
// chunk's waves own contiguous parts of it exactly as k_frame_sort's waves own the frame's:
//   k_fsc_count   per chunk: k_frame_sort's pass 1; its labels (slot order) with their per-wave
//                 counts -> the chunk's entry list, and its first noise point
//   k_fsc_merge   per frame: the chunks' labels in one LDS hash, the run offsets and segment
//                 lists exactly as k_frame_sort, then per chunk IN ORDER each entry's base =
//                 its run's start + the counts of the earlier chunks (stable across chunks)
//   k_fsc_scatter per chunk: per-wave cursors from the bases and the per-wave counts, then
//                 k_frame_sort's pass 2.
constexpr int kFsCap = kFsMaxKeys;  // entries per chunk list (more labels: overflow -> radix)

__device__ __forceinline__ void fsc_chunk(const int32_t* __restrict__ pf, int64_t n, int C,
                                          int b, int& f, int& lo, int& clo, int& chi) {
  f = b / C;
  const int c = b - f * C;
  lo = __builtin_amdgcn_readfirstlane((int)lower_bound_i32(pf, n, f));
  const int hi = __builtin_amdgcn_readfirstlane((int)lower_bound_i32(pf, n, f + 1));
  const int64_t len = hi - lo;
  clo = lo + (int)(len * c / C);
  chi = lo + (int)(len * (c + 1) / C);
}

__global__ __launch_bounds__(kFsWaves * 64) void k_fsc_count(
    const int32_t* __restrict__ labels, const int32_t* __restrict__ pf, int64_t n, int C,
    int32_t* __restrict__ ent_key, uint32_t* __restrict__ ent_cnt, int32_t* __restrict__ nent,
    int32_t* __restrict__ fnoise_c, int32_t* __restrict__ overflow) {
  __shared__ FsLds L;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int f, lo, clo, chi;
  fsc_chunk(pf, n, C, blockIdx.x, f, lo, clo, chi);
  for (int s = tid; s < kFsSlots; s += kFsWaves * 64) {
    L.keys[s] = -1;
#pragma unroll
    for (int q = 0; q < kFsWaves; ++q) L.cnt[q][s] = 0u;
  }
  if (tid == 0) {
    L.nkeys = 0;
    L.overflow = 0;
  }
  __syncthreads();
  const int nch = (chi - clo + 63) / 64, cpw = (nch + kFsWaves - 1) / kFsWaves;
  const int cb0 = w * cpw, cb1 = min(nch, cb0 + cpw);
  int wfn = INT_MAX;
  constexpr int U1 = 8;
  for (int cb = cb0; cb < cb1; cb += U1) {
    int lab[U1];
#pragma unroll
    for (int u = 0; u < U1; ++u) {
      const int i = clo + (cb + u) * 64 + lane;
      lab[u] = (cb + u < cb1 && i < chi) ? labels[i] : -2;
    }
#pragma unroll
    for (int u = 0; u < U1; ++u) {
      const int v = lab[u] + 1;
      if (wfn == INT_MAX) {
        const uint64_t m0 = __ballot(v == 0);
        if (m0) wfn = clo + (cb + u) * 64 + __builtin_ctzll(m0);
      }
      const bool valid = v >= 1;
      int leader, rank, cm;
      wave_group(v, valid, lane, leader, rank, cm);
      if (valid && lane == leader) {
        const int s = fs_insert(L, v);
        if (s >= 0) L.cnt[w][s] += (uint32_t)cm;
      }
    }
  }
  if (lane == 0) L.fnoise[w] = wfn;
  __syncthreads();
  if (L.overflow) {
    if (tid == 0) {
      nent[blockIdx.x] = 0;
      atomicExch(overflow, 1);
    }
    return;
  }
  if (tid == 0) {
    int m = INT_MAX;
#pragma unroll
    for (int q = 0; q < kFsWaves; ++q) m = min(m, L.fnoise[q]);
    fnoise_c[blockIdx.x] = m;
  }
  // the occupied slots in slot order -> entries 0 .. K-1
  uint32_t pcount = 0u;
#pragma unroll
  for (int j = 0; j < kFsSpt; ++j) pcount += (L.keys[kFsSpt * tid + j] != -1) ? 1u : 0u;
  const uint32_t ip = wave_incl_scan(pcount, lane);
  if (lane == 63) L.wsum[1][w] = ip;
  __syncthreads();
  uint32_t pp = 0, tp = 0;
#pragma unroll
  for (int q = 0; q < kFsWaves; ++q) {
    if (q < w) pp += L.wsum[1][q];
    tp += L.wsum[1][q];
  }
  uint32_t k = pp + ip - pcount;
  const int64_t e0 = (int64_t)blockIdx.x * kFsCap;
#pragma unroll
  for (int j = 0; j < kFsSpt; ++j) {
    const int sj = kFsSpt * tid + j;
    if (L.keys[sj] != -1) {
      ent_key[e0 + k] = L.keys[sj];
#pragma unroll
      for (int q = 0; q < kFsWaves; ++q) ent_cnt[(e0 + k) * kFsWaves + q] = L.cnt[q][sj];
      ++k;
    }
  }
  if (tid == 0) nent[blockIdx.x] = (int32_t)tp;
}

struct FscLds {
  int keys[kFsSlots];
  uint32_t tot[kFsSlots];
  int off[kFsSlots];
  uint32_t run[kFsSlots];
  uint32_t wsum[2][kFsWaves];
  int nkeys, overflow;
};

__device__ int fsc_insert(FscLds& L, int v) {
  uint32_t s = fs_hash(v);
  for (int probe = 0; probe < kFsSlots; ++probe) {
    const int k = __atomic_load_n(&L.keys[s], __ATOMIC_RELAXED);
    if (k == v) return (int)s;
    if (k == -1) {
      const int old = atomicCAS(&L.keys[s], -1, v);
      if (old == -1) {
        if (atomicAdd(&L.nkeys, 1) >= kFsMaxKeys) L.overflow = 1;
        return (int)s;
      }
      if (old == v) return (int)s;
    }
    s = (s + 1) & (kFsSlots - 1);
  }
  L.overflow = 1;
  return -1;
}

__global__ __launch_bounds__(kFsWaves * 64) void k_fsc_merge(
    const int32_t* __restrict__ pf, int64_t n, int C, const int32_t* __restrict__ ent_key,
    const uint32_t* __restrict__ ent_cnt, const int32_t* __restrict__ nent,
    const int32_t* __restrict__ fnoise_c, int32_t* __restrict__ ent_base,
    int32_t* __restrict__ ent_run, int32_t* __restrict__ fstart,
    int32_t* __restrict__ tmp_start, int32_t* __restrict__ tmp_len,
    int32_t* __restrict__ tmp_label, int32_t* __restrict__ nseg_f,
    int64_t* __restrict__ first_noise, int32_t* __restrict__ overflow) {
  __shared__ FscLds L;
  const int f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lo = __builtin_amdgcn_readfirstlane((int)lower_bound_i32(pf, n, f));
  for (int s = tid; s < kFsSlots; s += kFsWaves * 64) {
    L.keys[s] = -1;
    L.tot[s] = 0u;
  }
  if (tid == 0) {
    L.nkeys = 0;
    L.overflow = 0;
    fstart[f] = lo;
  }
  __syncthreads();
  if (*overflow) {  // a chunk overflowed: K9 is redone on the radix path
    if (tid == 0) nseg_f[f] = 0;
    return;
  }
  auto entry_total = [&](int64_t e) {
    uint32_t t = 0u;
#pragma unroll
    for (int q = 0; q < kFsWaves; ++q) t += ent_cnt[e * kFsWaves + q];
    return t;
  };
  for (int c = 0; c < C; ++c) {
    const int b = f * C + c, m = nent[b];
    for (int k = tid; k < m; k += kFsWaves * 64) {
      const int64_t e = (int64_t)b * kFsCap + k;
      const int s = fsc_insert(L, ent_key[e]);
      if (s >= 0) atomicAdd(&L.tot[s], entry_total(e));
    }
  }
  __syncthreads();
  if (L.overflow) {
    if (tid == 0) {
      nseg_f[f] = 0;
      atomicExch(overflow, 1);
    }
    return;
  }
  if (tid == 0 && first_noise) {
    int m = INT_MAX;
    for (int c = 0; c < C; ++c) m = min(m, fnoise_c[f * C + c]);
    if (m != INT_MAX) first_noise[f] = m;
  }
  // run offsets and the frame's segment list, in slot order (as k_frame_sort)
  uint32_t tt[kFsSpt];
  uint32_t a = 0u, pcount = 0u;
#pragma unroll
  for (int j = 0; j < kFsSpt; ++j) {
    const uint32_t t = L.tot[kFsSpt * tid + j];
    tt[j] = t;
    a += t;
    pcount += (t != 0u);
  }
  const uint32_t ia = wave_incl_scan(a, lane), ip = wave_incl_scan(pcount, lane);
  if (lane == 63) {
    L.wsum[0][w] = ia;
    L.wsum[1][w] = ip;
  }
  __syncthreads();
  uint32_t pa = 0, pp = 0, tp = 0;
#pragma unroll
  for (int q = 0; q < kFsWaves; ++q) {
    if (q < w) {
      pa += L.wsum[0][q];
      pp += L.wsum[1][q];
    }
    tp += L.wsum[1][q];
  }
  {
    uint32_t o = pa + ia - a, q = pp + ip - pcount;
#pragma unroll
    for (int j = 0; j < kFsSpt; ++j) {
      const int sj = kFsSpt * tid + j;
      if (tt[j] != 0u) {
        L.off[sj] = (int)o;
        L.run[sj] = o;
        tmp_start[lo + q] = lo + (int)o;
        tmp_len[lo + q] = (int)tt[j];
        tmp_label[lo + q] = L.keys[sj] - 1;
      }
      o += tt[j];
      q += (tt[j] != 0u);
    }
  }
  if (tid == 0) nseg_f[f] = (int)tp;
  __syncthreads();
  // each chunk's entry base: its run's start plus the earlier chunks' counts of the label (a
  // chunk's entries hold distinct labels, so its threads never share a slot)
  for (int c = 0; c < C; ++c) {
    const int b = f * C + c, m = nent[b];
    for (int k = tid; k < m; k += kFsWaves * 64) {
      const int64_t e = (int64_t)b * kFsCap + k;
      const int s = fs_find_keys(L.keys, ent_key[e]);
      ent_base[e] = (int)L.run[s];
      ent_run[e] = L.off[s];
      L.run[s] += entry_total(e);
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(kFsWaves * 64) void k_fsc_scatter(
    const int32_t* __restrict__ labels, const int32_t* __restrict__ pf, int64_t n, int C,
    const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ inten,
    float* __restrict__ gx, float* __restrict__ gy, float* __restrict__ gi,
    int32_t* __restrict__ tmp_first, const int32_t* __restrict__ ent_key,
    const uint32_t* __restrict__ ent_cnt, const int32_t* __restrict__ nent,
    const int32_t* __restrict__ ent_base, const int32_t* __restrict__ ent_run,
    const int32_t* __restrict__ overflow) {
  __shared__ FsLds L;
  if (*overflow) return;  // (block-uniform)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int f, lo, clo, chi;
  fsc_chunk(pf, n, C, blockIdx.x, f, lo, clo, chi);
  for (int s = tid; s < kFsSlots; s += kFsWaves * 64) L.keys[s] = -1;
  if (tid == 0) {
    L.nkeys = 0;
    L.overflow = 0;
  }
  __syncthreads();
  const int m = nent[blockIdx.x];
  for (int k = tid; k < m; k += kFsWaves * 64) {
    const int64_t e = (int64_t)blockIdx.x * kFsCap + k;
    const int s = fs_insert(L, ent_key[e]);
    uint32_t run = (uint32_t)ent_base[e];
#pragma unroll
    for (int q = 0; q < kFsWaves; ++q) {
      L.cnt[q][s] = run;
      run += ent_cnt[e * kFsWaves + q];
    }
    L.off[s] = ent_run[e];
  }
  __syncthreads();
  const int nch = (chi - clo + 63) / 64, cpw = (nch + kFsWaves - 1) / kFsWaves;
  const int cb0 = w * cpw, cb1 = min(nch, cb0 + cpw);
  constexpr int U2 = 4;
  for (int cb = cb0; cb < cb1; cb += U2) {
    int lab[U2];
    float px[U2], py[U2], pv[U2];
#pragma unroll
    for (int u = 0; u < U2; ++u) {
      const int i = clo + (cb + u) * 64 + lane;
      const bool in = cb + u < cb1 && i < chi;
      lab[u] = in ? labels[i] : -2;
      px[u] = in ? x[i] : 0.f;
      py[u] = in ? y[i] : 0.f;
      pv[u] = in ? inten[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U2; ++u) {
      const int i = clo + (cb + u) * 64 + lane;
      const int v = lab[u] + 1;
      const bool valid = v >= 1;
      int leader, rank, cm;
      wave_group(v, valid, lane, leader, rank, cm);
      int base = 0;
      if (valid && lane == leader) {
        const int s = fs_find(L, v);
        base = (int)L.cnt[w][s];
        L.cnt[w][s] = (uint32_t)(base + cm);
        if (base == L.off[s]) tmp_first[lo + base] = i;
      }
      base = __shfl(base, leader < 0 ? lane : leader);
      if (valid) {
        const int p = lo + base + rank;
        gx[p] = px[u];
        gy[p] = py[u];
        gi[p] = pv[u];
      }
    }
  }
}

__global__ void k_seg_total_fix(const int32_t* __restrict__ overflow, int32_t* __restrict__ total) {
  if (threadIdx.x == 0 && *overflow) *total = -1;
}

// Frame-local segment lists -> the global frame-major list (one wave per frame).
__global__ void k_seg_compact(int32_t F, const int32_t* __restrict__ fstart,
                              const int32_t* __restrict__ nseg_f, const int32_t* __restrict__ base,
                              const int32_t* __restrict__ tmp_start,
                              const int32_t* __restrict__ tmp_len,
                              const int32_t* __restrict__ tmp_label,
                              const int32_t* __restrict__ tmp_first, int32_t* __restrict__ o_frame,
                              int32_t* __restrict__ o_label, int64_t* __restrict__ o_count,
                              int64_t* __restrict__ o_first, int64_t* __restrict__ seg_start) {
  const int lane = threadIdx.x & 63;
  const int w0 = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const int nw = gridDim.x * (blockDim.x / 64);
  for (int f = w0; f < F; f += nw) {
    const int lo = fstart[f], m = nseg_f[f], b = base[f];
    for (int q = lane; q < m; q += 64) {
      const int s = tmp_start[lo + q];
      o_frame[b + q] = f;
      o_label[b + q] = tmp_label[lo + q];
      o_count[b + q] = tmp_len[lo + q];
      o_first[b + q] = tmp_first[s];
      seg_start[b + q] = s;
    }
  }
}

// p[0, n) = v; zero2 (nullable): two counters of the next kernel cleared (no memset launch)
__global__ void k_fill_i64(int64_t* p, int64_t n, int64_t v, int32_t* zero2 = nullptr) {
  if (zero2 && blockIdx.x == 0 && threadIdx.x < 2) zero2[threadIdx.x] = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

}  // namespace

// k_summarize's grid: two waves per long run, the count known only on the device (loops)
static int long_grid(int64_t s_hint) {
  return grid_for(2 * std::min<int64_t>(s_hint, 8192), kBlock / 64, 4096);
}

// bits: radix bits of the label keys (label + 1 < 2^bits); s_hint: expected segment count (sizes
// the summarize grid, which loops over the device count); *n_seg_dev: the count, on the device.
static int32_t summaries_impl(const int32_t* labels, const float* x, const float* y,
                              const float* inten, const int32_t* pf, int64_t n, int32_t n_frames,
                              int bits, int64_t s_hint, int32_t* o_frame, int32_t* o_label,
                              int64_t* o_count, int64_t* o_first, float* o_cx, float* o_cy,
                              float* o_mi, int64_t* frame_first_noise,
                              const int32_t** n_seg_dev, bool force_radix, bool* radix_used,
                              hipStream_t st) {
  if (n >= (int64_t(1) << 31) - 1) {
    set_error("rpt_cluster_summaries: n exceeds the int32 index space");
    return RPT_ENOTSUP;
  }
  Scratch& sc = scratch(st);
  // frame_first_noise = -1 (the frame-sort path clears its counters in the same launch)
  auto fill_noise = [&](int32_t* zero2) -> int32_t {
    if (n_frames > 0 && frame_first_noise) {
      hipLaunchKernelGGL(k_fill_i64, dim3(grid_for(n_frames, 256, 64)), dim3(256), 0, st,
                         frame_first_noise, (int64_t)n_frames, (int64_t)-1, zero2);
    } else if (zero2) {
      RPT_HIP(hipMemsetAsync(zero2, 0, 2 * sizeof(int32_t), st));
    }
    return RPT_OK;
  };
  const int64_t sh = std::max<int64_t>(1, std::min<int64_t>(s_hint, n));
  // per-frame counting sort unless forced off (RPT_K9_RADIX=1, or a redo after a frame held more
  // than kFsMaxKeys labels) or frames are huge (one 8-wave block per frame)
  static const bool env_radix = [] {
    const char* e = ab_env("RPT_K9_RADIX");
    return e && e[0] == '1';
  }();
  const bool frame_sort = !force_radix && !env_radix && n_frames > 0 && n > 0 &&
                          n / n_frames <= (int64_t(1) << 20);
  if (radix_used) *radix_used = !frame_sort;
  if (frame_sort) {
    // blocks per frame: one up to 64 k points per frame on average, else ~64 k points each (at
    // most 16): the dense share's 490 k-point frames take 8
    const int64_t ppf = n / std::max<int32_t>(n_frames, 1);
    const int C = (int)std::min<int64_t>(16, std::max<int64_t>(1, (ppf + 65535) / 65536));
    const int64_t NC = (int64_t)n_frames * C;
    Budget b;
    for (int k = 0; k < 3; ++k) b.add<float>(n + 1);
    for (int k = 0; k < 4; ++k) b.add<int32_t>(n + 1);
    b.add<int64_t>(n + 1);
    for (int k = 0; k < 3; ++k) b.add<int32_t>((int64_t)n_frames + 1);
    b.add<int32_t>(2);
    if (C > 1) {
      b.add<int32_t>(NC * kFsCap);
      b.add<uint32_t>(NC * kFsCap * kFsWaves);
      b.add<int32_t>(NC * kFsCap);
      b.add<int32_t>(NC * kFsCap);
      b.add<int32_t>(NC);
      b.add<int32_t>(NC);
    }
    RPT_TRY(sc.reserve(b.bytes, st));
    float* gx = sc.carve_n<float>(n + 1);
    float* gy = sc.carve_n<float>(n + 1);
    float* gi = sc.carve_n<float>(n + 1);
    int32_t* tstart = sc.carve_n<int32_t>(n + 1);
    int32_t* tlen = sc.carve_n<int32_t>(n + 1);
    int32_t* tlabel = sc.carve_n<int32_t>(n + 1);
    int32_t* tfirst = sc.carve_n<int32_t>(n + 1);
    int64_t* seg_start = sc.carve_n<int64_t>(n + 1);
    int32_t* fstart = sc.carve_n<int32_t>((int64_t)n_frames + 1);
    int32_t* nseg_f = sc.carve_n<int32_t>((int64_t)n_frames + 1);
    int32_t* base = sc.carve_n<int32_t>((int64_t)n_frames + 1);
    int32_t* ovf = sc.carve_n<int32_t>(2);  // [overflow flag, long-run count]
    int32_t *ent_key = nullptr, *nent = nullptr, *fnoise_c = nullptr, *ent_base = nullptr,
            *ent_run = nullptr;
    uint32_t* ent_cnt = nullptr;
    if (C > 1) {
      ent_key = sc.carve_n<int32_t>(NC * kFsCap);
      ent_cnt = sc.carve_n<uint32_t>(NC * kFsCap * kFsWaves);
      ent_base = sc.carve_n<int32_t>(NC * kFsCap);
      ent_run = sc.carve_n<int32_t>(NC * kFsCap);
      nent = sc.carve_n<int32_t>(NC);
      fnoise_c = sc.carve_n<int32_t>(NC);
    }
    RPT_TRY(fill_noise(ovf));
    if (C == 1) {
      hipLaunchKernelGGL(k_frame_sort, dim3(n_frames), dim3(kFsWaves * 64), 0, st, labels, pf, n,
                         x, y, inten, gx, gy, gi, fstart, tstart, tlen, tlabel, tfirst, nseg_f,
                         frame_first_noise, ovf);
    } else {
      hipLaunchKernelGGL(k_fsc_count, dim3((unsigned)NC), dim3(kFsWaves * 64), 0, st, labels, pf,
                         n, C, ent_key, ent_cnt, nent, fnoise_c, ovf);
      hipLaunchKernelGGL(k_fsc_merge, dim3(n_frames), dim3(kFsWaves * 64), 0, st, pf, n, C,
                         ent_key, ent_cnt, nent, fnoise_c, ent_base, ent_run, fstart, tstart,
                         tlen, tlabel, nseg_f, frame_first_noise, ovf);
      hipLaunchKernelGGL(k_fsc_scatter, dim3((unsigned)NC), dim3(kFsWaves * 64), 0, st, labels,
                         pf, n, C, x, y, inten, gx, gy, gi, tfirst, ent_key, ent_cnt, nent,
                         ent_base, ent_run, ovf);
    }
    RPT_CHECK_LAUNCH();
    RPT_TRY(exclusive_scan_total_i32(nseg_f, base, n_frames, st));
    hipLaunchKernelGGL(k_seg_compact, dim3(grid_for(n_frames, 4, 1024)), dim3(256), 0, st,
                       n_frames, fstart, nseg_f, base, tstart, tlen, tlabel, tfirst, o_frame,
                       o_label, o_count, o_first, seg_start);
    hipLaunchKernelGGL(k_seg_total_fix, dim3(1), dim3(64), 0, st, ovf, base + n_frames);
    // short runs one lane each; the long ones listed (in tlen, dead after the compaction) for
    // k_summarize's waves
    hipLaunchKernelGGL(k_runs_lane<true>, dim3(grid_for((sh + 63) / 64, kBlock / 64, 4096)),
                       dim3(kBlock), 0, st, nullptr, nullptr, seg_start, base + n_frames, n, gx,
                       gy, gi, pf, o_frame, o_label, o_count, o_first, o_cx, o_cy, o_mi, tlen,
                       ovf + 1);
    hipLaunchKernelGGL(k_summarize<true>, dim3(long_grid(sh)), dim3(kBlock), 0, st, nullptr,
                       nullptr, seg_start, base + n_frames, n, gx, gy, gi, pf, o_frame, o_label,
                       o_count, o_first, o_cx, o_cy, o_mi, tlen, ovf + 1);
    RPT_CHECK_LAUNCH();
    *n_seg_dev = base + n_frames;
    return RPT_OK;
  }
  RPT_TRY(fill_noise(nullptr));
  Budget b;
  for (int k = 0; k < 4; ++k) b.add<uint32_t>(n + 1);
  b.add<int64_t>(radix_tmp_elems(n));
  b.add<int32_t>(n + 1);
  b.add<int32_t>(n + 1);
  b.add<int64_t>(n + 1);
  for (int k = 0; k < 3; ++k) b.add<float>(n + 1);
  b.add<int32_t>(1);
  RPT_TRY(sc.reserve(b.bytes, st));
  uint32_t* keys = sc.carve_n<uint32_t>(n + 1);
  uint32_t* vals = sc.carve_n<uint32_t>(n + 1);
  uint32_t* ka = sc.carve_n<uint32_t>(n + 1);
  uint32_t* va = sc.carve_n<uint32_t>(n + 1);
  int64_t* rtmp = sc.carve_n<int64_t>(radix_tmp_elems(n));
  int32_t* head = sc.carve_n<int32_t>(n + 1);
  int32_t* pos = sc.carve_n<int32_t>(n + 1);  // int32: n < 2^31 (checked above)
  int64_t* seg_start = sc.carve_n<int64_t>(n + 1);
  float* gx = sc.carve_n<float>(n + 1);
  float* gy = sc.carve_n<float>(n + 1);
  float* gi = sc.carve_n<float>(n + 1);
  int32_t* n_long = sc.carve_n<int32_t>(1);
  if (n == 0) {
    RPT_HIP(hipMemsetAsync(pos, 0, sizeof(int32_t), st));
    *n_seg_dev = pos;
    RPT_CHECK_LAUNCH();
    return RPT_OK;
  }
  const int g = grid_for(n, kBlock, 8192);
  hipLaunchKernelGGL(k_sum_keys, dim3(g), dim3(kBlock), 0, st, labels, n, keys, vals);
  RPT_CHECK_LAUNCH();
  uint32_t *sk, *sv;
  RPT_TRY(radix_sort_pairs(keys, vals, ka, va, n, bits, rtmp, &sk, &sv, st));
  hipLaunchKernelGGL(k_heads, dim3(g), dim3(kBlock), 0, st, sk, sv, pf, n, head,
                     frame_first_noise);
  RPT_TRY(exclusive_scan_total_i32(head, pos, n, st));
  hipLaunchKernelGGL(k_seg_starts, dim3(g), dim3(kBlock), 0, st, head, pos, n, seg_start);
  hipLaunchKernelGGL(k_gather_runs, dim3(g), dim3(kBlock), 0, st, sv, n, x, y, inten, gx, gy, gi);
  // short runs one lane each; the long ones listed (in head, dead after k_seg_starts)
  RPT_HIP(hipMemsetAsync(n_long, 0, sizeof(int32_t), st));
  hipLaunchKernelGGL(k_runs_lane<false>, dim3(grid_for((sh + 63) / 64, kBlock / 64, 4096)),
                     dim3(kBlock), 0, st, sk, sv, seg_start, pos + n, n, gx, gy, gi, pf, o_frame,
                     o_label, o_count, o_first, o_cx, o_cy, o_mi, head, n_long);
  hipLaunchKernelGGL(k_summarize<false>, dim3(long_grid(sh)), dim3(kBlock), 0, st, sk, sv,
                     seg_start, pos + n, n, gx, gy, gi, pf, o_frame, o_label, o_count, o_first,
                     o_cx, o_cy, o_mi, head, n_long);
  RPT_CHECK_LAUNCH();
  *n_seg_dev = pos + n;
  return RPT_OK;
}

static int radix_bits_for(int64_t n_clusters) {
  int bits = 1;
  while ((int64_t(1) << bits) <= n_clusters) ++bits;
  return bits;
}

int32_t cluster_summaries(const int32_t* labels, const float* x, const float* y,
                          const float* inten, const int32_t* pf, int64_t n, int32_t n_frames,
                          int32_t n_clusters, int32_t* o_frame, int32_t* o_label,
                          int64_t* o_count, int64_t* o_first, float* o_cx, float* o_cy,
                          float* o_mi, int64_t* frame_first_noise, int64_t* n_seg_host,
                          hipStream_t st) {
  if (n < 0 || n_frames < 0 || n_clusters < 0 || !n_seg_host) {
    set_error("rpt_cluster_summaries: bad arguments");
    return RPT_EINVAL;
  }
  // the summarize grid is sized for one wave per run component once the count is known; a
  // frame with more than kFsMaxKeys labels sends K9 to the radix path
  const int32_t* nd = nullptr;
  int32_t n_seg = 0;
  for (int pass = 0; pass < 2; ++pass) {
    RPT_TRY(summaries_impl(labels, x, y, inten, pf, n, n_frames, radix_bits_for(n_clusters),
                           (int64_t)n_clusters * std::max(n_frames, 1) + 1, o_frame, o_label,
                           o_count, o_first, o_cx, o_cy, o_mi, frame_first_noise, &nd, pass == 1,
                           nullptr, st));
    RPT_HIP(hipMemcpyAsync(&n_seg, nd, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    RPT_TRY(wait_stream(st));
    if (n_seg >= 0) break;
  }
  *n_seg_host = n_seg;
  return RPT_OK;
}

// No readback: the caller passes the radix bits and a segment-count estimate, and reads the
// count (*n_seg_dev) with its other results after one sync.  A count of -1 means a frame held
// more labels than the frame sort takes: redo with force_radix.  *radix_used tells whether the
// label bits mattered (radix path) — the frame sort takes any labels.
int32_t cluster_summaries_dev(const int32_t* labels, const float* x, const float* y,
                              const float* inten, const int32_t* pf, int64_t n, int32_t n_frames,
                              int bits, int64_t s_hint, int32_t* o_frame, int32_t* o_label,
                              int64_t* o_count, int64_t* o_first, float* o_cx, float* o_cy,
                              float* o_mi, int64_t* frame_first_noise,
                              const int32_t** n_seg_dev, bool force_radix, bool* radix_used,
                              hipStream_t st) {
  if (n < 0 || n_frames < 0 || bits < 1 || bits > 32 || !n_seg_dev) {
    set_error("cluster_summaries_dev: bad arguments");
    return RPT_EINVAL;
  }
  return summaries_impl(labels, x, y, inten, pf, n, n_frames, bits, s_hint, o_frame, o_label,
                        o_count, o_first, o_cx, o_cy, o_mi, frame_first_noise, n_seg_dev,
                        force_radix, radix_used, st);
}

// Per-label pandas group means (count, x, y, intensity) of labels in [0, n_labels); labels
// without points keep count 0.  Synchronises once.
int32_t label_means(const int32_t* labels, const float* x, const float* y, const float* inten,
                    int64_t n, int64_t n_labels, int64_t* o_count, float* o_x, float* o_y,
                    float* o_v, hipStream_t st) {
  if (n < 0 || n_labels < 0 || (n > 0 && (!labels || !x || !y || !inten)) ||
      (n_labels > 0 && (!o_count || !o_x || !o_y || !o_v))) {
    set_error("rpt_label_means: bad arguments");
    return RPT_EINVAL;
  }
  if (n >= (int64_t(1) << 31) - 1 || n_labels >= (int64_t(1) << 31) - 1) {
    set_error("rpt_label_means: n exceeds the int32 index space");
    return RPT_ENOTSUP;
  }
  if (n_labels > 0) {
    RPT_HIP(hipMemsetAsync(o_count, 0, sizeof(int64_t) * (size_t)n_labels, st));
    RPT_HIP(hipMemsetAsync(o_x, 0, sizeof(float) * (size_t)n_labels, st));
    RPT_HIP(hipMemsetAsync(o_y, 0, sizeof(float) * (size_t)n_labels, st));
    RPT_HIP(hipMemsetAsync(o_v, 0, sizeof(float) * (size_t)n_labels, st));
  }
  if (n == 0) return wait_stream(st);
  Scratch& sc = scratch(st);
  Budget b;
  for (int k = 0; k < 4; ++k) b.add<uint32_t>(n + 1);
  b.add<int64_t>(radix_tmp_elems(n));
  b.add<int32_t>(n + 1);
  b.add<int32_t>(n + 1);
  b.add<int64_t>(n + 1);
  for (int k = 0; k < 3; ++k) b.add<float>(n + 1);
  b.add<int32_t>(1);
  RPT_TRY(sc.reserve(b.bytes, st));
  uint32_t* keys = sc.carve_n<uint32_t>(n + 1);
  uint32_t* vals = sc.carve_n<uint32_t>(n + 1);
  uint32_t* ka = sc.carve_n<uint32_t>(n + 1);
  uint32_t* va = sc.carve_n<uint32_t>(n + 1);
  int64_t* rtmp = sc.carve_n<int64_t>(radix_tmp_elems(n));
  int32_t* head = sc.carve_n<int32_t>(n + 1);
  int32_t* pos = sc.carve_n<int32_t>(n + 1);
  int64_t* seg_start = sc.carve_n<int64_t>(n + 1);
  float* gx = sc.carve_n<float>(n + 1);
  float* gy = sc.carve_n<float>(n + 1);
  float* gi = sc.carve_n<float>(n + 1);
  const int g = grid_for(n, kBlock, 8192);
  hipLaunchKernelGGL(k_sum_keys, dim3(g), dim3(kBlock), 0, st, labels, n, keys, vals);
  RPT_CHECK_LAUNCH();
  int bits = 1;
  while ((int64_t(1) << bits) <= n_labels + 1) ++bits;
  uint32_t *sk, *sv;
  RPT_TRY(radix_sort_pairs(keys, vals, ka, va, n, bits, rtmp, &sk, &sv, st));
  hipLaunchKernelGGL(k_label_heads, dim3(g), dim3(kBlock), 0, st, sk, n, head);
  RPT_TRY(exclusive_scan_total_i32(head, pos, n, st));
  hipLaunchKernelGGL(k_seg_starts, dim3(g), dim3(kBlock), 0, st, head, pos, n, seg_start);
  hipLaunchKernelGGL(k_gather_runs, dim3(g), dim3(kBlock), 0, st, sv, n, x, y, inten, gx, gy, gi);
  hipLaunchKernelGGL(k_label_means, dim3(grid_for(3 * (n_labels + 1), kBlock / 64, 16384)),
                     dim3(kBlock), 0, st, sk, seg_start, pos + n, n, gx, gy, gi, n_labels,
                     o_count, o_x, o_y, o_v);
  RPT_CHECK_LAUNCH();
  return wait_stream(st);
}

}  // namespace rpt
