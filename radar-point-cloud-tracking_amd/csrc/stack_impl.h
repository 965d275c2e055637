// Internals shared by the native stack driver (stack.cpp) and the frame-sharded driver
// (shard.cpp): grow-only device / pinned buffers, the library stages they call, and the stack
// handle (whose K1 / land / K9 buffers the shard handle reuses).
#pragma once
#include <algorithm>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "common.h"

namespace rpt {
int32_t polar_count(const void* echo, int32_t dt, int64_t n_files, int32_t rows, int32_t bins,
                    float thr, int32_t stride, int64_t* row_prefix, int64_t* file_offsets,
                    int64_t* total_host, hipStream_t st, uint32_t* entries);
int32_t polar_write_cap(const uint8_t* echo, int64_t n_files, int32_t rows, float thr,
                        int32_t stride, const float* scale, const float* cos_t,
                        const float* sin_t, const int32_t* gain, const int64_t* row_prefix,
                        const int64_t* file_offsets, int32_t fpf, float* x, float* y, float* v,
                        int32_t* gout, int32_t* pf, int64_t cap, hipStream_t st,
                        const uint32_t* entries, uint32_t* bnd = nullptr,
                        bool* bnd_done = nullptr);
int32_t polar_write(const void* echo, int32_t dt, int64_t n_files, int32_t rows, int32_t bins,
                    const float* scale, const float* cos_t, const float* sin_t,
                    const int32_t* gain, float thr, int32_t stride, const int64_t* row_prefix,
                    const int64_t* file_offsets, int32_t files_per_frame, float* x, float* y,
                    float* v, int32_t* gout, int32_t* pf, hipStream_t st, const uint32_t* entries,
                    uint32_t* bnd = nullptr, bool* bnd_done = nullptr);
// words of polar_write's bnd buffer; the bounds it leaves in bnd[0..3] read back as floats
int64_t polar_bounds_words();
int64_t polar_stage_words(int64_t n_files, int32_t rows);
int32_t frame_times(const int32_t* pf, int64_t n, const int64_t* ids, float* t, hipStream_t st);
int32_t bounds_xy(const float* x, const float* y, int64_t n, float* out4, hipStream_t st);
int32_t land_grid_cells(const float* x, const float* y, const float* val, int64_t n,
                        const double* xe, int32_t nxe, const double* ye, int32_t nye,
                        int32_t* cnt, double* tot, int32_t* cell_out, hipStream_t st,
                        int32_t u8_vals, int64_t* zero_also = nullptr);
int32_t land_mask(const int32_t* cnt, const double* tot, int64_t cells, int64_t num_frames,
                  double pthr, double ithr, uint8_t* land, int64_t* n_land_host,
                  hipStream_t st);
int32_t land_mask_dev(const int32_t* cnt, const double* tot, int64_t cells, int64_t num_frames,
                      double pthr, double ithr, uint8_t* land, int32_t* n_land_dev,
                      hipStream_t st);
int32_t land_compact_dev(const float* x, const float* y, const float* v, const int32_t* g,
                         const int32_t* pf, int64_t n, const int32_t* cell, const uint8_t* land,
                         int32_t n_frames, float* xo, float* yo, float* vo, int32_t* go,
                         int32_t* pfo, float* to, int64_t* new_off, Bounds* bounds_out,
                         hipStream_t st, int64_t t_base = 0);
int32_t stdbscan(const float* x, const float* y, const float* z, int64_t stride, const float* t,
                 int64_t n, double eps_space, double eps_time, int32_t min_samples,
                 int32_t* labels, rpt_stdbscan_stats* stats, hipStream_t st, int dim);
int32_t stdbscan_deferred(const float* x, const float* y, const float* z, int64_t stride,
                          const float* t, int64_t n, double eps_space, double eps_time,
                          int32_t min_samples, int32_t* labels, rpt_stdbscan_stats* stats,
                          hipStream_t st, int dim, const int32_t** n_clusters_dev,
                          void** state, const void* host_bounds);
size_t stdbscan_bounds_bytes();
size_t stdbscan_bounds_part_bytes(int64_t n_max);
int32_t stdbscan_bounds_dev(const float* x, const float* y, const float* t, int64_t n_max,
                            const int64_t* n_dev, void* out_dev, void* part_dev, hipStream_t st);
int32_t frame_times_dev(const int32_t* pf, int64_t n_max, const int64_t* n_dev, float* t,
                        hipStream_t st);
int32_t stdbscan_fill_stats(void* state, int32_t n_clusters, rpt_stdbscan_stats* stats);
int32_t stdbscan_core_flags(void* state, int64_t n, uint8_t* out, hipStream_t st);
int32_t cluster_summaries_dev(const int32_t* labels, const float* x, const float* y,
                              const float* inten, const int32_t* pf, int64_t n, int32_t n_frames,
                              int bits, int64_t s_hint, int32_t* o_frame, int32_t* o_label,
                              int64_t* o_count, int64_t* o_first, float* o_cx, float* o_cy,
                              float* o_mi, int64_t* frame_first_noise,
                              const int32_t** n_seg_dev, bool force_radix, bool* radix_used,
                              hipStream_t st);
int32_t cluster_summaries(const int32_t* labels, const float* x, const float* y,
                          const float* inten, const int32_t* pf, int64_t n, int32_t n_frames,
                          int32_t n_clusters, int32_t* o_frame, int32_t* o_label,
                          int64_t* o_count, int64_t* o_first, float* o_cx, float* o_cy,
                          float* o_mi, int64_t* frame_first_noise, int64_t* n_seg_host,
                          hipStream_t st);

int32_t remap_components(const int32_t* comp, int64_t n, int64_t base, const int64_t* keys,
                         const int64_t* vals, int64_t nk, int64_t* out, hipStream_t st);
int32_t select_roots(const int64_t* rep, int64_t base, int64_t lo, int64_t hi, int64_t* out,
                     int64_t* count_host, hipStream_t st);
struct DbscanState;
DbscanState* dbscan_create();
void dbscan_destroy(DbscanState* s);
int32_t dbscan_build(DbscanState* S, const float* x, const float* y, const float* z,
                     int64_t stride, const float* t, int64_t n, double eps_space,
                     double eps_time, int32_t ms, hipStream_t st);
int32_t dbscan_core(DbscanState* S, uint8_t* core_out, hipStream_t st);
int32_t dbscan_set_core(DbscanState* S, const uint8_t* core_in, hipStream_t st);
int32_t dbscan_components(DbscanState* S, int32_t* comp_out, hipStream_t st);
int32_t dbscan_labels_global(DbscanState* S, const int64_t* rep, const int64_t* reps, int64_t nr,
                             int32_t* labels, hipStream_t st);


std::vector<double> arange_edges(float lo, float hi, double res);

struct SegPack {
  const int64_t* count;
  const int64_t* first;
  const int64_t* noise;
  const int32_t* frame;
  const int32_t* label;
  const float* cx;
  const float* cy;
  const float* mi;
};
inline size_t seg_pack_bytes(int64_t sc, int32_t F) {
  return 16 + (size_t)sc * (8 + 8 + 4 + 4 + 4 + 4 + 4) + (size_t)F * 8;
}

inline int radix_bits_for(int64_t v) {
  int bits = 1;
  while ((int64_t(1) << bits) <= v) ++bits;
  return bits;
}

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;
  // grows only between syncs of the owning stream (callers synchronise before growing)
  int32_t ensure(size_t n, hipStream_t st) {
    if (n <= cap && p) return RPT_OK;
    if (p) {
      RPT_HIP(hipStreamSynchronize(st));
      RPT_HIP(hipFree(p));
      p = nullptr;
      cap = 0;
    }
    const size_t want = std::max<size_t>(n + n / 8 + 64, 256);
    if (hipMalloc((void**)&p, want * sizeof(T)) != hipSuccess) {
      p = nullptr;
      set_error("rpt_stack: hipMalloc of %zu bytes failed", want * sizeof(T));
      return RPT_ENOMEM;
    }
    cap = want;
    return RPT_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct PinnedBuf {
  char* p = nullptr;
  size_t cap = 0;
  int32_t ensure(size_t bytes, hipStream_t st) {
    if (bytes <= cap && p) return RPT_OK;
    if (p) {
      RPT_HIP(hipStreamSynchronize(st));
      RPT_HIP(hipHostFree(p));
      p = nullptr;
      cap = 0;
    }
    const size_t want = align_up(bytes + bytes / 8 + 4096, 4096);
    if (hipHostMalloc((void**)&p, want, hipHostMallocDefault) != hipSuccess) {
      p = nullptr;
      set_error("rpt_stack: hipHostMalloc of %zu bytes failed", want);
      return RPT_ENOMEM;
    }
    cap = want;
    return RPT_OK;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};


}  // namespace rpt

using rpt::DevBuf;
using rpt::PinnedBuf;
// K1 turns of several stack handles (lanes): each run's K1 (count + write, HBM-bound) is
// enqueued only after the previous run's, and its stream waits on the device for that one to end,
// so the lanes' K1 passes never share the HBM and always overlap other lanes' latency-bound
// stages.  Turns go in arrival order (a run takes the next ticket when it reaches K1): a waiting
// run only waits for runs already inside their K1 enqueue, so no cycle can form.
struct rpt_k1_gate {
  static constexpr int kRing = 16;
  std::mutex mu;
  std::condition_variable cv;
  int64_t issued = 0, next = 0;  // tickets handed out / the ticket whose turn it is
  hipEvent_t ev[kRing] = {};     // ev[t % kRing]: recorded after ticket t's K1
  ~rpt_k1_gate() {
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
  }
};

struct rpt_stack {
  DevBuf<uint32_t> pack_d;  // packed readback staging
  rpt_k1_gate* k1_gate = nullptr;  // (not owned) rpt_stack_set_k1_gate
  DevBuf<int64_t> row_prefix, file_off, new_off, first_noise, seg_count, seg_first, scal;
  DevBuf<float> x, y, v, x2, y2, v2, t, seg_cx, seg_cy, seg_mi;
  DevBuf<int32_t> g, pf, g2, pf2, labels, land_cnt, land_cell, seg_frame, seg_label;
  DevBuf<double> land_tot, edges;
  DevBuf<uint8_t> land_mask;
  DevBuf<uint32_t> k1_stage;           // K1 staged kept samples (count pass -> write pass)
  DevBuf<uint32_t> k1_bnd;             // K1 write's xy bounds + block partials
  int k1_staged = -1;                  // RPT_K1_STAGE (default on), read once
  DevBuf<uint8_t> bnd;                 // ST-DBSCAN bounds (+ partials) of the kept points
  std::vector<char> dbscan_bounds;     // their host copy, from the land readback
  PinnedBuf up, down;  // host staging: uploads (edges, offsets), readbacks
  std::vector<int64_t> fo_k1, fo_in;
  std::vector<int32_t> h_frame, h_label;
  std::vector<int64_t> h_count, h_first, h_noise;
  std::vector<float> h_cx, h_cy, h_mi;
  bool land_applied = false;
  int32_t n_frames = 0;
  int64_t n_in = 0;
  hipEvent_t ev[5] = {};
  bool ev_ok = false;
  hipEvent_t ev_rb = nullptr;  // readback marker of the speculative K1 write
  int sum_bits = 12;           // radix bits of the K9 label keys, from the previous run
  bool k9_radix = false;       // a frame held more labels than K9's frame sort takes
  int64_t seg_hint = 0;        // segment-count estimate from the previous run

  ~rpt_stack() {
    DevBuf<int64_t>* i64[] = {&row_prefix, &file_off, &new_off, &first_noise, &seg_count,
                              &seg_first, &scal};
    for (auto* b : i64) b->release();
    DevBuf<float>* f32[] = {&x, &y, &v, &x2, &y2, &v2, &t, &seg_cx, &seg_cy, &seg_mi};
    for (auto* b : f32) b->release();
    DevBuf<int32_t>* i32[] = {&g,        &pf,       &g2,        &pf2,      &labels,
                              &land_cnt, &land_cell, &seg_frame, &seg_label};
    for (auto* b : i32) b->release();
    land_tot.release();
    edges.release();
    pack_d.release();
    bnd.release();
    land_mask.release();
    k1_stage.release();
    k1_bnd.release();
    up.release();
    down.release();
    if (ev_ok)
      for (auto& e : ev) (void)hipEventDestroy(e);
    if (ev_rb) (void)hipEventDestroy(ev_rb);
  }

  bool had_gain = false;  // the last run wrote per-point gains (gain table given)
  void* db_state = nullptr;      // the last run's ST-DBSCAN state (per device and stream) ...
  hipStream_t db_stream = nullptr;  // ... and its stream (rpt_stack_core_flags)
  int32_t run(const rpt_stack_params& p, const void* echo, const float* scale,
              const float* cos_t, const float* sin_t, const int32_t* gain, rpt_stack_result* out,
              hipStream_t st);
};

