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
// Segments: a stable radix sort of (label+1, index) keeps each label's points in index order, so
// every (label, frame) run is contiguous and ordered.  One wave per run: lanes load 64 points at a
// time (coalesced), the order-preserving float32 chain reads them back lane by lane from
// registers (v_readlane), so a run of k points costs ~k dependent adds, not k memory latencies.
// Noise (key 0) sorts first in index order, so each frame's first noise point is the head of its
// frame within the noise run (no atomics).
#include <climits>

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

__global__ void k_seg_starts(const int32_t* __restrict__ head, const int64_t* __restrict__ pos,
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

__device__ __forceinline__ float lane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// One wave per (frame, label) run: sequential float32 sums in index order (np.mean axis 0).
// Mean intensity: when every intensity is a non-negative integer and the total stays below 2^24,
// every summation order is exact (integer lane sums), which equals numpy's pairwise result;
// otherwise numpy's chunked pairwise sum is evaluated by lane 0.
__global__ __launch_bounds__(kBlock) void k_summarize(
    const uint32_t* __restrict__ sk, const uint32_t* __restrict__ sv,
    const int64_t* __restrict__ seg_start, int64_t n_seg, int64_t n,
    const float* __restrict__ gx, const float* __restrict__ gy, const float* __restrict__ gi,
    const int32_t* __restrict__ pf, int32_t* __restrict__ o_frame, int32_t* __restrict__ o_label,
    int64_t* __restrict__ o_count, int64_t* __restrict__ o_first, float* __restrict__ o_cx,
    float* __restrict__ o_cy, float* __restrict__ o_mi) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (int64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
  const int64_t nw = (int64_t)gridDim.x * (kBlock / 64);
  for (int64_t s = w0; s < n_seg; s += nw) {
    const int64_t b = seg_start[s];
    const int64_t e = (s + 1 < n_seg) ? seg_start[s + 1] : n;
    const int64_t k = e - b;
    float sx = gx[b], sy = gy[b];  // numpy's reduction starts from the first row
    bool small_int = true;
    int64_t isum = 0;
    for (int64_t j0 = b; j0 < e; j0 += 64) {
      const int64_t j = j0 + lane;
      const bool in = j < e;
      const float vx = in ? gx[j] : 0.f, vy = in ? gy[j] : 0.f, vi = in ? gi[j] : 0.f;
      small_int = small_int && (!in || (vi >= 0.f && vi == floorf(vi) && vi < 16777216.f));
      isum += in ? (int64_t)vi : 0;
      const int first = (j0 == b) ? 1 : 0;
      const int m = (int)((e - j0 < 64) ? (e - j0) : 64);
      if (m == 64 && !first) {
#pragma unroll
        for (int l = 0; l < 64; ++l) {
          sx = sx + lane_f(vx, l);
          sy = sy + lane_f(vy, l);
        }
      } else {
        for (int l = first; l < m; ++l) {
          sx = sx + lane_f(vx, l);
          sy = sy + lane_f(vy, l);
        }
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) isum += __shfl_xor(isum, off);
    const bool all_int = __all(small_int);
    if (lane == 0) {
      const float fk = (float)k;
      float mi;
      if (all_int && isum < 16777216) {
        mi = (float)isum / fk;
      } else {
        float tot = 0.f;
        for (int64_t c = 0; c < k; c += 8192) {
          const int64_t len = (k - c < 8192) ? (k - c) : 8192;
          tot = tot + pairwise_f32(gi, b + c, len);
        }
        mi = tot / fk;
      }
      const uint32_t i0 = sv[b];
      o_frame[s] = pf[i0];
      o_label[s] = (int32_t)sk[b] - 1;
      o_count[s] = k;
      o_first[s] = i0;
      o_cx[s] = sx / fk;
      o_cy[s] = sy / fk;
      o_mi[s] = mi;
    }
  }
}

__global__ void k_fill_i64(int64_t* p, int64_t n, int64_t v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

}  // namespace

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
  if (n >= (int64_t(1) << 32) - 1) {
    set_error("rpt_cluster_summaries: n exceeds the u32 index space");
    return RPT_ENOTSUP;
  }
  Scratch& sc = scratch();
  Budget b;
  for (int k = 0; k < 4; ++k) b.add<uint32_t>(n + 1);
  b.add<int64_t>(radix_tmp_elems(n));
  b.add<int32_t>(n + 1);
  b.add<int64_t>(n + 1);
  b.add<int64_t>(n + 1);
  b.add<int64_t>(scan_tmp_elems(n + 1));
  for (int k = 0; k < 3; ++k) b.add<float>(n + 1);
  RPT_TRY(sc.reserve(b.bytes, st));
  uint32_t* keys = sc.carve_n<uint32_t>(n + 1);
  uint32_t* vals = sc.carve_n<uint32_t>(n + 1);
  uint32_t* ka = sc.carve_n<uint32_t>(n + 1);
  uint32_t* va = sc.carve_n<uint32_t>(n + 1);
  int64_t* rtmp = sc.carve_n<int64_t>(radix_tmp_elems(n));
  int32_t* head = sc.carve_n<int32_t>(n + 1);
  int64_t* pos = sc.carve_n<int64_t>(n + 1);
  int64_t* seg_start = sc.carve_n<int64_t>(n + 1);
  int64_t* tmp = sc.carve_n<int64_t>(scan_tmp_elems(n + 1));
  float* gx = sc.carve_n<float>(n + 1);
  float* gy = sc.carve_n<float>(n + 1);
  float* gi = sc.carve_n<float>(n + 1);
  if (n_frames > 0 && frame_first_noise)
    hipLaunchKernelGGL(k_fill_i64, dim3(grid_for(n_frames, 256, 64)), dim3(256), 0, st,
                       frame_first_noise, (int64_t)n_frames, (int64_t)-1);
  if (n == 0) {
    *n_seg_host = 0;
    RPT_CHECK_LAUNCH();
    return RPT_OK;
  }
  const int g = grid_for(n, kBlock, 8192);
  hipLaunchKernelGGL(k_sum_keys, dim3(g), dim3(kBlock), 0, st, labels, n, keys, vals);
  RPT_CHECK_LAUNCH();
  int bits = 1;
  while ((int64_t(1) << bits) <= (int64_t)n_clusters) ++bits;
  uint32_t *sk, *sv;
  RPT_TRY(radix_sort_pairs(keys, vals, ka, va, n, bits, rtmp, &sk, &sv, st));
  hipLaunchKernelGGL(k_heads, dim3(g), dim3(kBlock), 0, st, sk, sv, pf, n, head,
                     frame_first_noise);
  RPT_HIP(hipMemsetAsync(head + n, 0, sizeof(int32_t), st));
  RPT_TRY(exclusive_scan_i32_to_i64(head, pos, n + 1, tmp, st));
  hipLaunchKernelGGL(k_seg_starts, dim3(g), dim3(kBlock), 0, st, head, pos, n, seg_start);
  RPT_CHECK_LAUNCH();
  int64_t n_seg = 0;
  RPT_HIP(hipMemcpyAsync(&n_seg, pos + n, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  RPT_HIP(hipStreamSynchronize(st));
  if (n_seg > 0) {
    hipLaunchKernelGGL(k_gather_runs, dim3(g), dim3(kBlock), 0, st, sv, n, x, y, inten, gx, gy,
                       gi);
    hipLaunchKernelGGL(k_summarize, dim3(grid_for(n_seg, kBlock / 64, 16384)), dim3(kBlock), 0,
                       st, sk, sv, seg_start, n_seg, n, gx, gy, gi, pf, o_frame, o_label, o_count,
                       o_first, o_cx, o_cy, o_mi);
    RPT_CHECK_LAUNCH();
  }
  *n_seg_host = n_seg;
  return RPT_OK;
}

}  // namespace rpt
