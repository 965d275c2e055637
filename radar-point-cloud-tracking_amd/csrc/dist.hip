// Small device steps of the frame-sharded multi-GPU merge: map each local
// component (its min local original index, shifted to the global point numbering) to its
// global representative, and list the representatives a rank owns.
#include "common.h"

namespace rpt {
namespace {

__global__ void k_remap(const int32_t* __restrict__ comp, int64_t n, int64_t base,
                        const int64_t* __restrict__ keys, const int64_t* __restrict__ vals,
                        int64_t nk, int64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t c = comp[i];
    if (c < 0) {
      out[i] = -1;
      continue;
    }
    const int64_t g = base + c;
    int64_t lo = 0, hi = nk;
    while (lo < hi) {
      const int64_t m = (lo + hi) >> 1;
      if (keys[m] < g) lo = m + 1; else hi = m;
    }
    out[i] = (lo < nk && keys[lo] == g) ? vals[lo] : g;
  }
}

__global__ void k_root_flags(const int64_t* __restrict__ rep, int64_t base, int64_t lo,
                             int64_t m, int32_t* __restrict__ flag) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m;
       k += (int64_t)gridDim.x * blockDim.x)
    flag[k] = rep[lo + k] == base + lo + k;
}

__global__ void k_root_write(const int32_t* __restrict__ flag, const int64_t* __restrict__ pos,
                             int64_t base, int64_t lo, int64_t m, int64_t* __restrict__ out) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m;
       k += (int64_t)gridDim.x * blockDim.x)
    if (flag[k]) out[pos[k]] = base + lo + k;
}

}  // namespace

int32_t remap_components(const int32_t* comp, int64_t n, int64_t base, const int64_t* keys,
                         const int64_t* vals, int64_t nk, int64_t* out, hipStream_t st) {
  if (n == 0) return RPT_OK;
  hipLaunchKernelGGL(k_remap, dim3(grid_for(n, 256, 4096)), dim3(256), 0, st, comp, n, base, keys,
                     vals, nk, out);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

int32_t select_roots(const int64_t* rep, int64_t base, int64_t lo, int64_t hi, int64_t* out,
                     int64_t* count_host, hipStream_t st) {
  const int64_t m = hi - lo;
  if (m <= 0 || !count_host) {
    if (count_host) *count_host = 0;
    return RPT_OK;
  }
  Scratch& sc = scratch(st);
  Budget b;
  b.add<int32_t>(m + 1);
  b.add<int64_t>(m + 1);
  RPT_TRY(sc.reserve(b.bytes, st));
  int32_t* flag = sc.carve_n<int32_t>(m + 1);
  int64_t* pos = sc.carve_n<int64_t>(m + 1);
  hipLaunchKernelGGL(k_root_flags, dim3(grid_for(m, 256, 4096)), dim3(256), 0, st, rep, base, lo,
                     m, flag);
  RPT_CHECK_LAUNCH();
  RPT_TRY(exclusive_scan_total_i32_to_i64(flag, pos, m, st));
  hipLaunchKernelGGL(k_root_write, dim3(grid_for(m, 256, 4096)), dim3(256), 0, st, flag, pos,
                     base, lo, m, out);
  RPT_CHECK_LAUNCH();
  RPT_HIP(hipMemcpyAsync(count_host, pos + m, sizeof(int64_t), hipMemcpyDeviceToHost, st));
  RPT_TRY(wait_stream(st));
  return RPT_OK;
}

}  // namespace rpt
