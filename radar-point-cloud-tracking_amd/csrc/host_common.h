// Host-only part of librpt's shared helpers: the error plumbing and small utilities used by the
// host translation units that never touch HIP (csv.cpp, tracker.cpp, shard_host.cpp,
// errors.cpp).  Kept free of <hip/hip_runtime.h> so those units also build with a plain host
// compiler -- tools/asan/Makefile compiles them with -fsanitize=address,undefined.
#pragma once

#include <cstddef>
#include <cstdint>

#include "../../include/rpt.h"

namespace rpt {

// ---- error plumbing (thread-local last error, no exceptions across the ABI) -----------
void set_error(const char* fmt, ...);
void clear_error();
const char* last_error_cstr();

#define RPT_TRY(expr)              \
  do {                             \
    int32_t s__ = (expr);          \
    if (s__ != RPT_OK) return s__; \
  } while (0)

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

int32_t order_clusters(int32_t n_frames, int64_t n_seg, const int32_t* seg_frame,
                       const int32_t* seg_label, const int64_t* seg_first,
                       const int64_t* frame_first_noise, int64_t* frame_off, int64_t* order);

}  // namespace rpt
