// extern "C" surface of librpt.so (declared in include/rpt.h).  Thin: argument checks,
// error-code translation, dispatch into the rpt:: implementations.
#include <hip/hip_runtime.h>

#include <cstring>

#include "common.h"

namespace rpt {
const char* last_error_cstr();
void release_scratch_current();
int32_t stdbscan(const float* x, const float* y, const float* z, int64_t stride, const float* t,
                 int64_t n, double eps_space, double eps_time, int32_t min_samples,
                 int32_t* labels, rpt_stdbscan_stats* stats, hipStream_t st, int dim);
}  // namespace rpt

extern "C" {

int32_t rpt_version(void) { return 100; }  // 0.1.0

const char* rpt_last_error(void) { return rpt::last_error_cstr(); }

int32_t rpt_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int32_t rpt_set_device(int32_t device) {
  RPT_HIP(hipSetDevice(device));
  return RPT_OK;
}

void rpt_release_scratch(void) { rpt::release_scratch_current(); }

int32_t rpt_stdbscan(const float* x, const float* y, const float* z, int64_t stride,
                     const float* times, int64_t n, double eps_space, double eps_time,
                     int32_t min_samples, int32_t* labels, rpt_stdbscan_stats* stats,
                     void* stream) {
  rpt::clear_error();
  const int dim = z ? 3 : 2;
  return rpt::stdbscan(x, y, z, stride, times, n, eps_space, eps_time, min_samples, labels,
                       stats, rpt::as_stream(stream), dim);
}

}  // extern "C"
