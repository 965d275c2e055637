// Device-wide primitives used by the ST-DBSCAN grid build and the cluster summaries:
//  * exclusive scan — single pass with decoupled look-back (one launch, no memset),
//  * stable LSD radix sort of (u32 key, u32 value) pairs, 8-bit digits, wave-granular
//    histograms so that a pass needs no block-level barriers inside the scatter loop.
// Plus the per-(device, stream) scratch pools.
#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstring>
#include <mutex>

#include "common.h"

namespace rpt {

// (the error plumbing lives in errors.cpp)

// ------------------------------------------------------------------ readback wait
// The path's size readbacks are tiny and the GPU idles until the host has launched the next
// stage, so the wait polls an event (for up to 200 us, then it blocks) instead of blocking in
// hipStreamSynchronize right away.  One cached event per (thread, device).
//
// Device-side faults that must not pass silently (today: a look-back scan whose predecessor tile
// never published within its spin bound, i.e. a wrong prefix) set a word in mapped pinned host
// memory; every readback wait checks and clears it and fails the call with RPT_EHIP.
static unsigned int* g_fault_host = nullptr;
static unsigned int* g_fault_dev = nullptr;
static std::mutex g_fault_mu;

unsigned int* device_fault_word() {
  std::lock_guard<std::mutex> lk(g_fault_mu);
  if (!g_fault_dev) {
    void* h = nullptr;
    if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      return nullptr;
    std::memset(h, 0, 64);
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
      (void)hipHostFree(h);
      return nullptr;
    }
    g_fault_host = static_cast<unsigned int*>(h);
    g_fault_dev = static_cast<unsigned int*>(d);
  }
  return g_fault_dev;
}

int32_t check_device_faults() {
  if (!g_fault_host) return RPT_OK;
  const unsigned int f = __atomic_exchange_n(g_fault_host, 0u, __ATOMIC_ACQ_REL);
  if (f & 1u) {
    set_error("exclusive scan: a look-back predecessor never published (prefix sums invalid)");
    return RPT_EHIP;
  }
  return RPT_OK;
}

int32_t wait_stream(hipStream_t st) {
  static thread_local std::vector<hipEvent_t> evs;
  int dev = 0;
  RPT_HIP(hipGetDevice(&dev));
  if ((int)evs.size() <= dev) evs.resize(dev + 1, nullptr);
  if (!evs[dev]) RPT_HIP(hipEventCreateWithFlags(&evs[dev], hipEventDisableTiming));
  RPT_HIP(hipEventRecord(evs[dev], st));
  // poll for up to ~200 us (the readbacks of the path), then block instead of burning a core
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipEventQuery(evs[dev]);
    if (e == hipSuccess) return check_device_faults();
    if (e != hipErrorNotReady) RPT_HIP(e);
    if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) break;
  }
  RPT_HIP(hipEventSynchronize(evs[dev]));
  return check_device_faults();
}

// ------------------------------------------------------------------ scratch pool
int32_t Scratch::reserve(size_t bytes, hipStream_t stream) {
  off_ = 0;
  if (bytes <= cap_) return RPT_OK;
  if (base_) {
    RPT_HIP(hipStreamSynchronize(stream));
    RPT_HIP(hipDeviceSynchronize());
    RPT_HIP(hipFree(base_));
    base_ = nullptr;
    cap_ = 0;
  }
  size_t want = align_up(bytes + bytes / 4 + (1u << 20), 1u << 20);
  hipError_t e = hipMalloc(&base_, want);
  if (e != hipSuccess) {
    base_ = nullptr;
    set_error("scratch hipMalloc(%zu bytes) failed: %s", want, hipGetErrorString(e));
    return RPT_ENOMEM;
  }
  cap_ = want;
  return RPT_OK;
}

void* Scratch::carve(size_t bytes) {
  size_t a = align_up(bytes, 256);
  if (off_ + a > cap_) return nullptr;  // callers reserve() first; a null here is a bug
  void* p = base_ + off_;
  off_ += a;
  return p;
}

void Scratch::release() {
  if (base_) (void)hipFree(base_);
  base_ = nullptr;
  cap_ = off_ = 0;
}

// One arena per (device, stream): work on different streams (concurrent stacks) never shares it.
static std::mutex g_scratch_mu;
static std::vector<std::pair<std::pair<int, hipStream_t>, Scratch*>> g_scratch;

Scratch& scratch(hipStream_t st) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_scratch_mu);
  for (auto& e : g_scratch)
    if (e.first.first == dev && e.first.second == st) return *e.second;
  g_scratch.push_back({{dev, st}, new Scratch()});
  return *g_scratch.back().second;
}

// ------------------------------------------------------------------ pre-zeroed words
namespace {
struct ZeroPool {
  std::mutex mu;
  uint32_t* base = nullptr;  // kZeroSlots slots of 16 words
  int64_t next = 0;          // slots handed out since the pool was created (ring position)
  int64_t armed_end = -1;    // slots up to this ring position are zero from the last arm()
};
constexpr int kZeroSlotWords = 16;
std::mutex g_zero_mu;
std::vector<std::pair<std::pair<int, hipStream_t>, ZeroPool*>> g_zero;

int32_t zero_pool(hipStream_t st, ZeroPool** out) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  ZeroPool* z = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_zero_mu);
    for (auto& e : g_zero)
      if (e.first.first == dev && e.first.second == st) z = e.second;
    if (!z) {
      z = new ZeroPool();
      g_zero.push_back({{dev, st}, z});
    }
  }
  if (!z->base) {
    hipError_t e = hipMalloc(&z->base, sizeof(uint32_t) * kZeroSlots * kZeroSlotWords);
    if (e != hipSuccess) {
      z->base = nullptr;
      set_error("zero pool hipMalloc failed: %s", hipGetErrorString(e));
      return RPT_ENOMEM;
    }
  }
  *out = z;
  return RPT_OK;
}
}  // namespace

int32_t zero_pool_arm(hipStream_t st) {
  ZeroPool* z = nullptr;
  RPT_TRY(zero_pool(st, &z));
  std::lock_guard<std::mutex> lk(z->mu);
  // one memset of the whole ring; the next kZeroSlots takes need none
  RPT_HIP(hipMemsetAsync(z->base, 0, sizeof(uint32_t) * kZeroSlots * kZeroSlotWords, st));
  z->next = (z->next + kZeroSlots - 1) / kZeroSlots * kZeroSlots;  // start of a ring round
  z->armed_end = z->next + kZeroSlots;
  return RPT_OK;
}

int32_t zero_words(hipStream_t st, size_t words, void** out) {
  ZeroPool* z = nullptr;
  RPT_TRY(zero_pool(st, &z));
  const int64_t slots = (int64_t)((words + kZeroSlotWords - 1) / kZeroSlotWords);
  if (slots < 1 || slots > kZeroSlots / 4) {
    set_error("zero_words: %zu words", words);
    return RPT_EINVAL;
  }
  std::lock_guard<std::mutex> lk(z->mu);
  int64_t at = z->next;
  if (at % kZeroSlots + slots > kZeroSlots) at = (at / kZeroSlots + 1) * kZeroSlots;  // no wrap
  z->next = at + slots;
  uint32_t* p = z->base + (at % kZeroSlots) * kZeroSlotWords;
  if (at + slots > z->armed_end)  // not covered by the last arm(): clear with a memset
    RPT_HIP(hipMemsetAsync(p, 0, sizeof(uint32_t) * slots * kZeroSlotWords, st));
  *out = p;
  return RPT_OK;
}

void release_scan_states(int dev);  // below, with the scan

void release_scratch_current() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  {
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    for (auto& e : g_scratch)
      if (e.first.first == dev) e.second->release();
  }
  {
    std::lock_guard<std::mutex> lk(g_zero_mu);
    for (auto& e : g_zero)
      if (e.first.first == dev && e.second->base) {
        std::lock_guard<std::mutex> lz(e.second->mu);
        (void)hipFree(e.second->base);
        e.second->base = nullptr;
        e.second->armed_end = -1;
      }
  }
  release_scan_states(dev);
}

// ------------------------------------------------------------------ exclusive scan
constexpr int kScanBlock = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanBlock * kScanItems;  // 2048

// Block-wide exclusive scan of one int64 per thread; returns the exclusive prefix and
// writes the block total to *total.
__device__ __forceinline__ int64_t block_exclusive_scan(int64_t v, int64_t* total) {
  __shared__ int64_t wsum[kScanBlock / kWave];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  int64_t incl = v;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    int64_t o = __shfl_up(incl, off, kWave);
    if (lane >= off) incl += o;
  }
  if (lane == kWave - 1) wsum[wid] = incl;
  __syncthreads();
  int64_t wprefix = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kScanBlock / kWave; ++w) {
    int64_t s = wsum[w];
    if (w < wid) wprefix += s;
    tot += s;
  }
  __syncthreads();  // wsum may be reused by the caller's next call
  *total = tot;
  return wprefix + incl - v;
}

// One-block scan of up to kScanTile outputs (same n_in / n_out contract as k_scan_lb).
template <class T, class U>
__global__ __launch_bounds__(kScanBlock) void k_scan_small(const T* __restrict__ in, int64_t n_in,
                                                          int64_t n_out, U* __restrict__ out) {
  const int64_t base = (int64_t)threadIdx.x * kScanItems;
  int64_t vals[kScanItems];
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    int64_t i = base + k;
    vals[k] = (i < n_in) ? (int64_t)in[i] : 0;
    s += vals[k];
  }
  int64_t tot;
  int64_t run = block_exclusive_scan(s, &tot);
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    int64_t i = base + k;
    if (i < n_out) out[i] = (U)run;
    run += vals[k];
  }
}

// Single-pass form (decoupled look-back): tiles of kLbItems x B items are taken in ticket order;
// a tile publishes its aggregate, then its inclusive prefix once its predecessors' are known.
// The status words are 64-bit granules {flag:2 | epoch:16 | value:46} written and read with
// agent-scope relaxed atomics: the data IS the flag (MI355X guide §6 Guideline 16, R2), so no
// fences.  Values are non-negative counts whose running total is < 2^46.
//
// No memset per scan: the status array and the ticket live in a persistent per-(device, stream)
// ScanState.  Every launch gets a fresh epoch, and a granule of another epoch reads as "not
// published" (the array is zeroed once per 65535 launches, before an epoch is reused); the block
// that draws the last ticket resets the counter for the next launch on the stream.  Every spin is
// bounded.
constexpr int kLbItems = 16;
constexpr int kLbBig = 1024;  // block size of the large-n kernel: 16384 items per ticket
constexpr uint64_t kLbAgg = 1ull << 62, kLbInc = 2ull << 62, kLbVal = (1ull << 46) - 1;
constexpr int kLbEpochShift = 46;

template <int B>
__device__ __forceinline__ int64_t block_excl_scan_b(int64_t v, int64_t* total) {
  constexpr int NW = B / kWave;
  __shared__ int64_t wsum[NW];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  int64_t incl = v;
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    int64_t o = __shfl_up(incl, off, kWave);
    if (lane >= off) incl += o;
  }
  if (lane == kWave - 1) wsum[wid] = incl;
  __syncthreads();
  // every wave scans the NW wave totals in its first lanes
  int64_t w = lane < NW ? wsum[lane] : 0;
#pragma unroll
  for (int off = 1; off < NW; off <<= 1) {
    int64_t o = __shfl_up(w, off, kWave);
    if (lane >= off) w += o;
  }
  *total = __shfl(w, NW - 1, kWave);
  const int64_t wprefix = wid ? __shfl(w, wid > 0 ? wid - 1 : 0, kWave) : 0;
  return wprefix + incl - v;
}

// 16 consecutive items of a thread, in registers, in their input type (16 or 32 VGPRs: full
// occupancy, so a whole 8M-item scan is resident in one round).  VEC: 16-B vector accesses (the
// thread's items are 64 B of int32 or 128 B of int64, so a wave's k-th vector access covers every
// k-th 16-B piece of 4 / 8 KiB: the pieces of a line meet in L2 and HBM sees each line once) — no
// LDS staging.
template <class T, bool VEC>
__device__ __forceinline__ void load16(const T* __restrict__ in, int64_t i0, int64_t n_in,
                                       T (&v)[kLbItems]) {
  if (VEC && i0 + kLbItems <= n_in) {
    if constexpr (sizeof(T) == 4) {
      const int4* p = reinterpret_cast<const int4*>(in + i0);
#pragma unroll
      for (int q = 0; q < kLbItems / 4; ++q) {
        const int4 w = p[q];
        v[4 * q] = w.x;
        v[4 * q + 1] = w.y;
        v[4 * q + 2] = w.z;
        v[4 * q + 3] = w.w;
      }
    } else {
      const longlong2* p = reinterpret_cast<const longlong2*>(in + i0);
#pragma unroll
      for (int q = 0; q < kLbItems / 2; ++q) {
        const longlong2 w = p[q];
        v[2 * q] = w.x;
        v[2 * q + 1] = w.y;
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < kLbItems; ++k) v[k] = (i0 + k < n_in) ? in[i0 + k] : T(0);
  }
}

// out[i0 + k] = run + sum of v[0..k), computed while storing
template <class T, class U, bool VEC>
__device__ __forceinline__ void store16(U* __restrict__ out, int64_t i0, int64_t n_out,
                                        const T (&v)[kLbItems], int64_t run) {
  if (VEC && i0 + kLbItems <= n_out) {
    if constexpr (sizeof(U) == 4) {
      int4* p = reinterpret_cast<int4*>(out + i0);
#pragma unroll
      for (int q = 0; q < kLbItems / 4; ++q) {
        int4 w;
        w.x = (int)run;
        run += v[4 * q];
        w.y = (int)run;
        run += v[4 * q + 1];
        w.z = (int)run;
        run += v[4 * q + 2];
        w.w = (int)run;
        run += v[4 * q + 3];
        p[q] = w;
      }
    } else {
      longlong2* p = reinterpret_cast<longlong2*>(out + i0);
#pragma unroll
      for (int q = 0; q < kLbItems / 2; ++q) {
        longlong2 w;
        w.x = run;
        run += v[2 * q];
        w.y = run;
        run += v[2 * q + 1];
        p[q] = w;
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < kLbItems; ++k) {
      if (i0 + k < n_out) out[i0 + k] = (U)run;
      run += v[k];
    }
  }
}

// out[i] = sum of in[0..i) for i < n_out, with in[i] read as 0 for i >= n_in (n_out <= n_in + 1:
// n_out = n_in + 1 writes the grand total at out[n_in]).  in == out is allowed (a thread reads
// its own 16 items before it writes them, and no other thread touches them).
// (B = 1024: 8 waves per SIMD, i.e. two blocks per CU, 512 tiles = 8M items resident at once)
template <class T, class U, int B, bool VEC>
__global__ __launch_bounds__(B, B >= 1024 ? 8 : 2) void k_scan_lb(const T* __restrict__ in, int64_t n_in,
                                               U* __restrict__ out, int64_t n_out,
                                               uint64_t* __restrict__ status,
                                               unsigned long long* __restrict__ ticket,
                                               uint64_t epoch, uint32_t nt,
                                               unsigned int* __restrict__ fault) {
  constexpr int kTile = B * kLbItems;
  __shared__ uint32_t s_tile;
  __shared__ int64_t s_prefix;
  if (threadIdx.x == 0) {
    const uint32_t t = (uint32_t)atomicAdd(ticket, 1ull);
    // the last ticket of this launch: nobody draws again before the next launch on the stream
    if (t == nt - 1u)
      __hip_atomic_store(ticket, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_tile = t;
  }
  __syncthreads();
  const int64_t tile = s_tile;
  const int64_t i0 = tile * kTile + (int64_t)threadIdx.x * kLbItems;
  T v[kLbItems];
  load16<T, VEC>(in, i0, n_in, v);
  int64_t sum = 0;
#pragma unroll
  for (int k = 0; k < kLbItems; ++k) sum += (int64_t)v[k];
  int64_t tot;
  const int64_t excl = block_excl_scan_b<B>(sum, &tot);
  const uint64_t tag = epoch << kLbEpochShift;
  if (threadIdx.x < kWave) {
    const int lane = threadIdx.x;
    if (lane == 0)
      __hip_atomic_store(status + tile, (tile == 0 ? kLbInc : kLbAgg) | tag | (uint64_t)tot,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int64_t prefix = 0;
    int64_t j = tile - 1;  // nearest predecessor not yet accounted for
    uint32_t spins = 0;
    while (j >= 0) {
      const int64_t idx = j - lane;
      uint64_t st = (idx >= 0) ? __hip_atomic_load(status + idx, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT)
                               : (kLbInc | tag);  // before tile 0: an inclusive zero
      if (((st >> kLbEpochShift) & 0xffffu) != epoch) st = 0;  // another launch's granule
      const uint64_t inc = __ballot((st >> 62) == 2u);
      const uint64_t zero = __ballot((st >> 62) == 0u);
      const int first_inc = inc ? __ffsll((unsigned long long)inc) - 1 : kWave;
      const uint64_t upto = (first_inc >= kWave - 1) ? ~0ull : ((2ull << first_inc) - 1ull);
      if (zero & upto) {  // a predecessor before the nearest inclusive one is not published yet
        if (++spins > (1u << 24)) {  // bounded: a lost tile gives a wrong sum, not a hang --
          if (lane == 0 && fault)    // reported at the next readback wait (check_device_faults)
            __hip_atomic_store(fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      int64_t part = (lane <= first_inc && idx >= 0) ? (int64_t)(st & kLbVal) : 0;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) part += __shfl_xor(part, off);
      prefix += part;
      if (first_inc < kWave) break;
      j -= kWave;
    }
    if (lane == 0) {
      if (tile > 0)
        __hip_atomic_store(status + tile, kLbInc | tag | (uint64_t)(prefix + tot),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_prefix = prefix;
    }
  }
  __syncthreads();
  store16<T, U, VEC>(out, i0, n_out, v, s_prefix + excl);
}

size_t scan_tmp_elems(int64_t n) {
  (void)n;
  return 64;  // the look-back state is persistent (ScanState); kept for the callers' budgets
}

namespace {
struct ScanState {
  uint64_t* status = nullptr;  // [cap] granules, then the ticket word
  size_t cap = 0;
  uint32_t epoch = 0;
};
std::mutex g_scan_mu;
std::vector<std::pair<std::pair<int, hipStream_t>, ScanState*>> g_scan_states;

// The look-back state of (current device, stream) with room for nt tiles, and this launch's epoch.
int32_t scan_state(hipStream_t st, int64_t nt, ScanState** out, uint32_t* epoch) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  ScanState* s = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_scan_mu);
    for (auto& e : g_scan_states)
      if (e.first.first == dev && e.first.second == st) s = e.second;
    if (!s) {
      s = new ScanState();
      g_scan_states.push_back({{dev, st}, s});
    }
  }
  if ((size_t)nt > s->cap) {
    if (s->status) {
      RPT_HIP(hipStreamSynchronize(st));  // earlier scans on this stream still read it
      RPT_HIP(hipFree(s->status));
      s->status = nullptr;
      s->cap = 0;
    }
    const size_t want = std::max<size_t>((size_t)nt + (size_t)nt / 2, 4096);
    hipError_t e = hipMalloc(&s->status, sizeof(uint64_t) * (want + 1));
    if (e != hipSuccess) {
      s->status = nullptr;
      set_error("scan state hipMalloc failed: %s", hipGetErrorString(e));
      return RPT_ENOMEM;
    }
    RPT_HIP(hipMemsetAsync(s->status, 0, sizeof(uint64_t) * (want + 1), st));
    s->cap = want;
    s->epoch = 0;
  }
  if (++s->epoch > 0xffffu) {  // an epoch is about to be reused: clear every granule first
    RPT_HIP(hipMemsetAsync(s->status, 0, sizeof(uint64_t) * s->cap, st));
    s->epoch = 1;
  }
  *out = s;
  *epoch = s->epoch;
  return RPT_OK;
}
}  // namespace

// rpt_release_scratch: the look-back states of the device too (re-created, zeroed, on next use)
void release_scan_states(int dev) {
  std::lock_guard<std::mutex> lk(g_scan_mu);
  for (auto& e : g_scan_states)
    if (e.first.first == dev && e.second->status) {
      (void)hipFree(e.second->status);
      e.second->status = nullptr;
      e.second->cap = 0;
      e.second->epoch = 0;
    }
}

template <class T, class U>
static int32_t scan_impl(const T* in, int64_t n_in, U* out, int64_t n_out, hipStream_t stream) {
  if (n_out <= 0) return RPT_OK;
  const int64_t nb = (n_out + kScanTile - 1) / kScanTile;
  if (nb == 1) {
    hipLaunchKernelGGL((k_scan_small<T, U>), dim3(1), dim3(kScanBlock), 0, stream, in, n_in,
                       n_out, out);
    RPT_CHECK_LAUNCH();
    return RPT_OK;
  }
  // 1024-thread tiles for large aligned scans (fewer tickets); unaligned ones take the 256-thread
  // kernel, whose scalar path fits its registers
  const bool vec = (uintptr_t)in % 16 == 0 && (uintptr_t)out % 16 == 0;
  const bool big = vec && n_out > (int64_t)kScanBlock * kLbItems * 16;
  const int64_t tile = (big ? kLbBig : kScanBlock) * (int64_t)kLbItems;
  const int64_t nt = (n_out + tile - 1) / tile;
  if (nt >= (int64_t(1) << 31)) {
    set_error("exclusive scan: too many tiles");
    return RPT_ENOTSUP;
  }
  ScanState* s = nullptr;
  uint32_t epoch = 0;
  RPT_TRY(scan_state(stream, nt, &s, &epoch));
  auto* ticket = reinterpret_cast<unsigned long long*>(s->status + s->cap);
  unsigned int* fault = device_fault_word();
  const uint64_t ep = epoch;
  const unsigned grid = (unsigned)nt;
  if (big)
    hipLaunchKernelGGL((k_scan_lb<T, U, kLbBig, true>), dim3(grid), dim3(kLbBig), 0, stream, in,
                       n_in, out, n_out, s->status, ticket, ep, (uint32_t)nt, fault);
  else if (vec)
    hipLaunchKernelGGL((k_scan_lb<T, U, kScanBlock, true>), dim3(grid), dim3(kScanBlock), 0,
                       stream, in, n_in, out, n_out, s->status, ticket, ep, (uint32_t)nt, fault);
  else
    hipLaunchKernelGGL((k_scan_lb<T, U, kScanBlock, false>), dim3(grid), dim3(kScanBlock), 0,
                       stream, in, n_in, out, n_out, s->status, ticket, ep, (uint32_t)nt, fault);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

int32_t exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, int64_t* tmp,
                           hipStream_t stream) {
  (void)tmp;
  return scan_impl<int64_t, int64_t>(in, n, out, n, stream);
}
int32_t exclusive_scan_i32_to_i64(const int32_t* in, int64_t* out, int64_t n, int64_t* tmp,
                                  hipStream_t stream) {
  (void)tmp;
  return scan_impl<int32_t, int64_t>(in, n, out, n, stream);
}
int32_t exclusive_scan_i32(const int32_t* in, int32_t* out, int64_t n, int64_t* tmp,
                           hipStream_t stream) {
  (void)tmp;
  return scan_impl<int32_t, int32_t>(in, n, out, n, stream);
}
int32_t exclusive_scan_total_i64(const int64_t* in, int64_t* out, int64_t n, hipStream_t stream) {
  return scan_impl<int64_t, int64_t>(in, n, out, n + 1, stream);
}
int32_t exclusive_scan_total_i32_to_i64(const int32_t* in, int64_t* out, int64_t n,
                                        hipStream_t stream) {
  return scan_impl<int32_t, int64_t>(in, n, out, n + 1, stream);
}
int32_t exclusive_scan_total_i32(const int32_t* in, int32_t* out, int64_t n, hipStream_t stream) {
  return scan_impl<int32_t, int32_t>(in, n, out, n + 1, stream);
}

// ------------------------------------------------------------------ packed readback
// Copies up to kPackMax device arrays (4-byte multiples) back to back into dst, so that a
// readback is one DMA instead of one per array (each D2H costs ~10 us of issue on the stream).
__global__ void k_pack(PackList l, uint32_t* __restrict__ dst) {
  const int64_t total = l.off[l.k];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    int s = 0;
    while (s + 1 < l.k && i >= l.off[s + 1]) ++s;
    dst[i] = l.src[s][i - l.off[s]];
  }
}

int32_t pack_arrays(const PackList& l, uint32_t* dst, hipStream_t st) {
  if (l.k <= 0 || l.off[l.k] == 0) return RPT_OK;
  hipLaunchKernelGGL(k_pack, dim3(grid_for(l.off[l.k], 256, 2048)), dim3(256), 0, st, l, dst);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

// ------------------------------------------------------------------ radix sort
// Stable LSD radix sort with digits of up to 12 bits, so the ST-DBSCAN cell keys (≤ 24 bits)
// take two passes and the K9 label keys (≤ 12 bits) one.  A block owns a tile of 4 waves x 1024
// items (16 rows of 64 per wave).  Per pass: (1) per-tile digit counts (LDS atomics) written
// digit-major as int32, (2) one exclusive scan over them = each tile's first output slot per
// digit, (3) the scatter: the tile's items are re-counted per wave in LDS to give each wave its
// start per digit (waves in order), then each wave ranks its rows of 64 items by ballots over the
// digit bits and writes them.  Order inside a tile is wave, row, lane: stable.
constexpr int kSortBlock = 256;
constexpr int kSortRows = 16;                  // items per lane
constexpr int kSortWaveItems = kWave * kSortRows;  // 1024 items per wave
constexpr int kSortWavesPerBlock = kSortBlock / kWave;
constexpr int kSortTile = kSortWaveItems * kSortWavesPerBlock;  // 4096 items per block
constexpr int kSortMaxBits = 12;

// hist[d * n_tiles + tile] = number of items of the tile whose digit is d.
template <int R>
__global__ __launch_bounds__(kSortBlock) void k_radix_hist(const uint32_t* __restrict__ keys,
                                                          int64_t n, int shift, int64_t n_tiles,
                                                          int32_t* __restrict__ hist) {
  constexpr int D = 1 << R;
  __shared__ int cnt[kSortWavesPerBlock][D];  // one sub-histogram per wave: 4x less contention
  const int wl = threadIdx.x / kWave;
  for (int d = threadIdx.x; d < D * kSortWavesPerBlock; d += kSortBlock) (&cnt[0][0])[d] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kSortTile;
#pragma unroll 4
  for (int r = 0; r < kSortTile / kSortBlock; ++r) {
    const int64_t i = base + (int64_t)r * kSortBlock + threadIdx.x;
    if (i < n) atomicAdd(&cnt[wl][(keys[i] >> shift) & (uint32_t)(D - 1)], 1);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += kSortBlock) {
    int c = 0;
#pragma unroll
    for (int w = 0; w < kSortWavesPerBlock; ++w) c += cnt[w][d];
    hist[(int64_t)d * n_tiles + blockIdx.x] = c;
  }
}

template <int R>
__global__ __launch_bounds__(kSortBlock) void k_radix_scatter(
    const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals, int64_t n, int shift,
    int64_t n_tiles, const int32_t* __restrict__ offs, uint32_t* __restrict__ keys_out,
    uint32_t* __restrict__ vals_out) {
  constexpr int D = 1 << R;
  __shared__ int32_t run[kSortWavesPerBlock][D];
  const int lane = threadIdx.x & (kWave - 1);
  const int wl = threadIdx.x / kWave;
  for (int d = lane; d < D; d += kWave) run[wl][d] = 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const int64_t base = (int64_t)blockIdx.x * kSortTile + (int64_t)wl * kSortWaveItems;
  uint32_t k[kSortRows], v[kSortRows];
#pragma unroll
  for (int r = 0; r < kSortRows; ++r) {
    const int64_t i = base + (int64_t)r * kWave + lane;
    k[r] = i < n ? keys[i] : 0u;
    v[r] = i < n ? vals[i] : 0u;
  }
#pragma unroll
  for (int r = 0; r < kSortRows; ++r) {
    const int64_t i = base + (int64_t)r * kWave + lane;
    if (i < n) atomicAdd(&run[wl][(k[r] >> shift) & (uint32_t)(D - 1)], 1);
  }
  __syncthreads();
  // counts -> each wave's first slot per digit: the tile's slot plus the earlier waves' counts
  for (int d = threadIdx.x; d < D; d += kSortBlock) {
    int32_t pos = offs[(int64_t)d * n_tiles + blockIdx.x];
#pragma unroll
    for (int w = 0; w < kSortWavesPerBlock; ++w) {
      const int32_t c = run[w][d];
      run[w][d] = pos;
      pos += c;
    }
  }
  __syncthreads();
#pragma unroll 1
  for (int r = 0; r < kSortRows; ++r) {
    const int64_t i = base + (int64_t)r * kWave + lane;
    const bool valid = i < n;
    const uint32_t d = (k[r] >> shift) & (uint32_t)(D - 1);
    uint64_t mask = __ballot(valid);
#pragma unroll
    for (int b = 0; b < R; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t bb = __ballot(valid && bit);
      mask &= bit ? bb : ~bb;
    }
    const int rank = rank_in_mask(mask);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int32_t pos = run[wl][d] + rank;
    if (valid) {
      keys_out[pos] = k[r];
      vals_out[pos] = v[r];
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (valid && rank == 0) run[wl][d] += __popcll(mask);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

size_t radix_tmp_elems(int64_t n) {
  const int64_t n_tiles = (n + kSortTile - 1) / kSortTile;
  const int64_t h = ((int64_t)1 << kSortMaxBits) * n_tiles;  // int32 entries
  return (size_t)(h + 1) / 2 + 64;
}

template <int R>
static int32_t radix_pass(const uint32_t* ks, const uint32_t* vs, uint32_t* kd, uint32_t* vd,
                          int64_t n, int shift, int32_t* hist, hipStream_t st) {
  const int64_t n_tiles = (n + kSortTile - 1) / kSortTile;
  const int64_t h = ((int64_t)1 << R) * n_tiles;
  hipLaunchKernelGGL(k_radix_hist<R>, dim3((unsigned)n_tiles), dim3(kSortBlock), 0, st, ks, n,
                     shift, n_tiles, hist);
  RPT_CHECK_LAUNCH();
  RPT_TRY(exclusive_scan_i32(hist, hist, h, nullptr, st));
  hipLaunchKernelGGL(k_radix_scatter<R>, dim3((unsigned)n_tiles), dim3(kSortBlock), 0, st, ks, vs,
                     n, shift, n_tiles, (const int32_t*)hist, kd, vd);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

int32_t radix_sort_pairs(uint32_t* keys, uint32_t* vals, uint32_t* keys_alt, uint32_t* vals_alt,
                         int64_t n, int bits, int64_t* tmp, uint32_t** out_keys,
                         uint32_t** out_vals, hipStream_t st) {
  *out_keys = keys;
  *out_vals = vals;
  if (n <= 1 || bits <= 0) return RPT_OK;
  if (n >= (int64_t(1) << 31) || bits > 32) {
    set_error("radix sort: n must be < 2^31 and bits <= 32");
    return RPT_ENOTSUP;
  }
  // one pass up to kSortMaxBits bits (K9 label keys); wider keys (grid cells) in 8-bit digits,
  // where the ballot ranking and the digit-major histogram stay cheapest per bit (measured:
  // 2 x 11-12 bits cost more than 3 x 8 for the 22-bit cell keys)
  const int passes = bits <= kSortMaxBits ? 1 : (bits + 7) / 8;
  const int r0 = (bits + passes - 1) / passes;
  int32_t* hist = reinterpret_cast<int32_t*>(tmp);
  uint32_t *ks = keys, *vs = vals, *kd = keys_alt, *vd = vals_alt;
  for (int p = 0, shift = 0; p < passes; ++p) {
    const int r = std::min(r0, bits - shift);
    int32_t s = RPT_OK;
    switch (r) {
      case 1: case 2: case 3: case 4: case 5: case 6: s = radix_pass<6>(ks, vs, kd, vd, n, shift, hist, st); break;
      case 7: case 8: s = radix_pass<8>(ks, vs, kd, vd, n, shift, hist, st); break;
      case 9: case 10: s = radix_pass<10>(ks, vs, kd, vd, n, shift, hist, st); break;
      default: s = radix_pass<12>(ks, vs, kd, vd, n, shift, hist, st); break;
    }
    if (s != RPT_OK) return s;
    shift += r;
    std::swap(ks, kd);
    std::swap(vs, vd);
  }
  *out_keys = ks;
  *out_vals = vs;
  return RPT_OK;
}

}  // namespace rpt
