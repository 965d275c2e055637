// Shared host/device helpers for librpt (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "host_common.h"

namespace rpt {

#define RPT_HIP(expr)                                                               \
  do {                                                                              \
    hipError_t e__ = (expr);                                                        \
    if (e__ != hipSuccess) {                                                        \
      ::rpt::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e__),      \
                       __FILE__, __LINE__);                                         \
      return RPT_EHIP;                                                              \
    }                                                                               \
  } while (0)

#define RPT_CHECK_LAUNCH() RPT_HIP(hipGetLastError())

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// A/B switches (RPT_* environment variables selecting a replaced kernel form for same-box
// measurements) exist only in the A/B build (-DRPT_AB, tools/ab_*.sh): the shipped librpt.so
// ignores the environment and always runs the default forms the parity suite covers.
inline const char* ab_env(const char* name) {
#ifdef RPT_AB
  return std::getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

// Waits for the work queued on st so far by polling an event (readback latency; prims.hip).
int32_t wait_stream(hipStream_t st);  // also reports device faults (check_device_faults)
int32_t check_device_faults();
unsigned int* device_fault_word();  // mapped pinned fault word for bounded device spins

// ---- scratch pool ------------------------------------------------------------------------
// A bump arena per (device, stream) that grows on demand.  Calls reserve() once with their total
// need (so no hipMalloc happens mid-call), then carve() 256-byte aligned slices.
class Scratch {
 public:
  int32_t reserve(size_t bytes, hipStream_t stream);
  void* carve(size_t bytes);
  template <class T>
  T* carve_n(size_t n) { return static_cast<T*>(carve(n * sizeof(T))); }
  void reset() { off_ = 0; }
  void release();
  size_t capacity() const { return cap_; }

 private:
  char* base_ = nullptr;
  size_t cap_ = 0;
  size_t off_ = 0;
};
Scratch& scratch(hipStream_t st);  // for the current device and this stream

// ---- pre-zeroed device words ---------------------------------------------------------------
// Counters a call needs zeroed (atomic cursors, list lengths).  A driver that runs many calls on
// one stream arms the stream's pool once per run -- one memset for all of them -- and
// zero_words() then hands out zeroed words of the pool without a launch of its own; unarmed, or
// once the armed pool is used up, zero_words() clears the words it hands out with a memset (the
// standalone entry points).  Words are handed out in 64-byte slots, ring-wise per stream: a word
// stays valid for the work queued on the stream before the ring comes round (kZeroSlots takes).
constexpr int kZeroSlots = 256;
int32_t zero_pool_arm(hipStream_t st);
int32_t zero_words(hipStream_t st, size_t words, void** out);
template <class T>
int32_t zero_n(hipStream_t st, size_t n, T** out) {
  void* p = nullptr;
  const int32_t r = zero_words(st, (n * sizeof(T) + 3) / 4, &p);
  *out = static_cast<T*>(p);
  return r;
}

// Byte budget helper: sum of aligned array sizes.
struct Budget {
  size_t bytes = 0;
  template <class T>
  void add(size_t n) { bytes += align_up(n * sizeof(T), 256); }
};

// ---- device utilities --------------------------------------------------------------------
constexpr int kWave = 64;

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// number of active lanes below this one with their bit set in `mask`
__device__ __forceinline__ int rank_in_mask(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                   __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}

inline int grid_for(int64_t n, int block, int cap = 65535 * 8) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// ---- primitives implemented in prims.hip --------------------------------------------------
// Exclusive scan of int64 values (in/out may alias).  tmp needs scan_tmp_elems(n) int64s.
size_t scan_tmp_elems(int64_t n);
int32_t exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, int64_t* tmp,
                           hipStream_t stream);
// Same for int32 input -> int64 output.
int32_t exclusive_scan_i32_to_i64(const int32_t* in, int64_t* out, int64_t n, int64_t* tmp,
                                  hipStream_t stream);

// int32 -> int32 (values must fit; in == out allowed).
int32_t exclusive_scan_i32(const int32_t* in, int32_t* out, int64_t n, int64_t* tmp,
                           hipStream_t stream);

// out[0..n] = exclusive scan of in[0..n) plus the grand total at out[n] (out has n+1 entries;
// in == out allowed): no sentinel element to clear.  Totals must stay below 2^46.
int32_t exclusive_scan_total_i64(const int64_t* in, int64_t* out, int64_t n, hipStream_t stream);
int32_t exclusive_scan_total_i32_to_i64(const int32_t* in, int64_t* out, int64_t n,
                                        hipStream_t stream);
int32_t exclusive_scan_total_i32(const int32_t* in, int32_t* out, int64_t n, hipStream_t stream);

// Back-to-back copy of up to kPackMax device arrays (sizes in 4-byte words) into dst.
constexpr int kPackMax = 10;
// Point-set bounds of the ST-DBSCAN grid build (k_bounds in stdbscan.hip; also produced by the
// fused land compaction, land.hip): ordered-u32 (sign-flipped float bits) minima / maxima.
struct Bounds {
  uint32_t mn[4];   // ordered-u32 minima of x, y, z, t (t over finite values only)
  uint32_t mx[4];
  int32_t nonfinite_xyz;  // any NaN/inf coordinate
  int32_t nonintegral_t;  // any finite t with t != floor(t) or |t| >= 2^24
  int32_t n_finite_t;
  int32_t t_descends;     // some t[i] < t[i-1]: the points are not in time order
};

// Device accumulator of a Bounds partial with k_bounds' semantics (stdbscan.hip), for kernels
// that produce the ST-DBSCAN bounds of points they write anyway (the shard window).  add() per
// point (t_prev: the previous point's t in the set's order, has_prev false for the first point),
// then block_store() by EVERY thread of a block of kBoundsBlock threads: one partial per block,
// reduced by stdbscan_bounds_final_dev.
constexpr int kBoundsBlock = 256;
struct BoundsAcc {
  uint32_t mn[4] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
  uint32_t mx[4] = {0u, 0u, 0u, 0u};
  int nonfin = 0, nonint = 0, nfin = 0, desc = 0;
  __device__ static uint32_t ord(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  }
  __device__ void add(float x, float y, float t, float t_prev, bool has_prev) {
    const float v[3] = {x, y, 0.f};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (!isfinite(v[k])) nonfin = 1;
      const uint32_t o = ord(v[k]);
      mn[k] = min(mn[k], o);
      mx[k] = max(mx[k], o);
    }
    if (isfinite(t)) {
      ++nfin;
      const uint32_t o = ord(t);
      mn[3] = min(mn[3], o);
      mx[3] = max(mx[3], o);
      if (t != floorf(t) || fabsf(t) >= 16777216.f) nonint = 1;
    }
    if (has_prev && !(t_prev <= t)) desc = 1;  // NaN counts as out of order
  }
  __device__ void block_store(Bounds* __restrict__ out) {
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
    __shared__ Bounds sb[kBoundsBlock / 64];
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
      Bounds o = sb[0];
      for (int v = 1; v < kBoundsBlock / 64; ++v) {
        for (int k = 0; k < 4; ++k) {
          o.mn[k] = min(o.mn[k], sb[v].mn[k]);
          o.mx[k] = max(o.mx[k], sb[v].mx[k]);
        }
        o.nonfinite_xyz |= sb[v].nonfinite_xyz;
        o.nonintegral_t |= sb[v].nonintegral_t;
        o.n_finite_t += sb[v].n_finite_t;
        o.t_descends |= sb[v].t_descends;
      }
      out[blockIdx.x] = o;
    }
  }
};
// the partials of nb blocks -> out (one launch, k_bounds_final)
int32_t stdbscan_bounds_final_dev(const void* part_dev, int nb, void* out_dev, hipStream_t st);

struct PackList {
  const uint32_t* src[kPackMax];
  int64_t off[kPackMax + 1];  // word offsets in dst, off[0] = 0
  int k = 0;
  void add(const void* p, size_t bytes) {
    if (k == 0) off[0] = 0;
    src[k] = static_cast<const uint32_t*>(p);
    off[k + 1] = off[k] + (int64_t)(bytes / 4);
    ++k;
  }
};
int32_t pack_arrays(const PackList& l, uint32_t* dst, hipStream_t st);

// Stable LSD radix sort of (key,u32 value) pairs on the low `bits` bits of key.
// Buffers: keys/vals in, keys_alt/vals_alt ping-pong; the result ends in whichever buffer the
// returned pointer pair names (out_keys/out_vals).  tmp needs radix_tmp_elems(n) int64s.
size_t radix_tmp_elems(int64_t n);
int32_t radix_sort_pairs(uint32_t* keys, uint32_t* vals, uint32_t* keys_alt, uint32_t* vals_alt,
                         int64_t n, int bits, int64_t* tmp, uint32_t** out_keys,
                         uint32_t** out_vals, hipStream_t stream);

}  // namespace rpt
