// The host stage's building blocks shared by the stack driver's fused order + track
// (tracker.cpp: rpt_order_and_track) and rank 0's shard host stage (shard_host.cpp): segments
// bucketed by frame, each frame's reference cluster order computed by frame range, and a
// producer thread that orders frames ahead of the (sequential) tracker consuming them.
// Host-only (tools/asan/Makefile builds it with -fsanitize=address,undefined).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace rpt {

// Segments bucketed by frame: cnt[f] .. cnt[f + 1] index byf, the segment ids of frame f in
// segment order.
struct FrameBuckets {
  std::vector<int64_t> cnt, byf;
  // frame_off (nullable) receives cnt; RPT_EINVAL for a segment frame outside [0, n_frames)
  int32_t build(int32_t n_frames, int64_t n_seg, const int32_t* seg_frame, int64_t* frame_off);
  // order_out[cnt[f] + q] = (q-th segment of frame f in the reference order) + add, for the
  // frames [f_lo, f_hi) (4_temporal_object_tracker.py:519-522)
  void order(int32_t f_lo, int32_t f_hi, const int32_t* seg_label, const int64_t* seg_first,
             const int64_t* frame_first_noise, int64_t* order_out, int64_t add) const;
};

// A producer (one thread) publishes how many leading frames are ready; the consumer waits for
// a frame before reading its outputs.  Producer writes happen-before the consumer's reads of
// a published frame (release/acquire on done_).  A producer that throws publishes every frame
// and sets failed().
class OrderAhead {
 public:
  // runs producer(*this) on a new thread (threaded) or inline before returning
  void start(std::function<void(OrderAhead&)> producer, bool threaded);
  void publish(int64_t frames_done);
  void wait_for(int64_t frame);  // until frames [0, frame] are published
  void join();
  bool failed() const { return failed_.load(std::memory_order_acquire); }
  ~OrderAhead() { join(); }

 private:
  std::atomic<int64_t> done_{-1};
  std::atomic<bool> failed_{false};
  std::mutex mu_;
  std::condition_variable cv_;
  std::thread th_;
};

}  // namespace rpt
