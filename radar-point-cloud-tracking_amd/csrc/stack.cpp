// Native driver of the single-device stack path: the compute stages of run_pipeline
// (PointCloudWork/4_temporal_object_tracker.py:941-991) over a stack of sweeps already in HBM,
//
//   K1 polar scatter + fusion -> land filter (> 10 built frames, :954) -> ST-DBSCAN over the
//   stack -> per-(frame, label) summaries,
//
// in ONE library call.  The data-dependent sizes (points per file, land-filter bounds and kept
// count, grid bounds, segment count) still need host readbacks, but each is a pinned-memory copy
// and a stream sync inside C++ instead of a Python round trip per stage, and the results come
// back in one packed copy.  Buffers are owned by the handle and grow only.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
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
                        const uint32_t* entries);
int32_t polar_write(const void* echo, int32_t dt, int64_t n_files, int32_t rows, int32_t bins,
                    const float* scale, const float* cos_t, const float* sin_t,
                    const int32_t* gain, float thr, int32_t stride, const int64_t* row_prefix,
                    const int64_t* file_offsets, int32_t files_per_frame, float* x, float* y,
                    float* v, int32_t* gout, int32_t* pf, hipStream_t st, const uint32_t* entries);
int64_t polar_stage_words(int64_t n_files, int32_t rows);
int32_t frame_times(const int32_t* pf, int64_t n, const int64_t* ids, float* t, hipStream_t st);
int32_t bounds_xy(const float* x, const float* y, int64_t n, float* out4, hipStream_t st);
int32_t land_grid_cells(const float* x, const float* y, const float* val, int64_t n,
                        const double* xe, int32_t nxe, const double* ye, int32_t nye,
                        int32_t* cnt, double* tot, int32_t* cell_out, hipStream_t st,
                        int32_t u8_vals);
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
                         hipStream_t st);
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

// np.arange(lo, hi + res, res) for float32 lo/hi (numpy 2.x, NEP 50 weak Python floats): the
// stop and the length are float32 arithmetic, element 1 is float32(lo + res), the rest are
// float64 start + i * (e1 - e0).  Checked against numpy in tests/test_host_native.py.
std::vector<double> arange_edges(float lo, float hi, double res) {
  const float rf = (float)res;
  const float stop = hi + rf;
  const float q = (stop - lo) / rf;
  const double len_d = std::ceil((double)q);
  const int64_t len = (len_d > 0.0) ? (int64_t)len_d : 0;
  std::vector<double> e((size_t)len);
  if (len == 0) return e;
  e[0] = (double)lo;
  if (len == 1) return e;
  e[1] = (double)(float)(lo + rf);
  const double d = e[1] - e[0];
  for (int64_t i = 2; i < len; ++i) e[(size_t)i] = e[0] + (double)i * d;
  return e;
}

namespace {

// The run's results in one readback without knowing the segment count on the host: header
// {S, n_clusters} then arrays at offsets fixed by the capacity sc (entries >= S are not written).
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
__global__ void k_pack_segs(const int32_t* __restrict__ n_seg, const int32_t* __restrict__ ncl,
                            SegPack a, int64_t sc, int32_t F, char* __restrict__ out) {
  const int64_t S = *n_seg;
  const int64_t m = S < sc ? S : sc;
  int64_t* hdr = reinterpret_cast<int64_t*>(out);
  int64_t* count = hdr + 2;
  int64_t* first = count + sc;
  int64_t* noise = first + sc;
  int32_t* frame = reinterpret_cast<int32_t*>(noise + F);
  int32_t* label = frame + sc;
  float* cx = reinterpret_cast<float*>(label + sc);
  float* cy = cx + sc;
  float* mi = cy + sc;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i0 == 0) {
    hdr[0] = S;
    hdr[1] = ncl ? (int64_t)*ncl : -1;
  }
  for (int64_t i = i0; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    count[i] = a.count[i];
    first[i] = a.first[i];
    frame[i] = a.frame[i];
    label[i] = a.label[i];
    cx[i] = a.cx[i];
    cy[i] = a.cy[i];
    mi[i] = a.mi[i];
  }
  for (int64_t i = i0; i < F; i += (int64_t)gridDim.x * blockDim.x) noise[i] = a.noise[i];
}

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

}  // namespace
}  // namespace rpt

using namespace rpt;

struct rpt_stack {
  DevBuf<uint32_t> pack_d;  // packed readback staging
  DevBuf<int64_t> row_prefix, file_off, new_off, first_noise, seg_count, seg_first, scal;
  DevBuf<float> x, y, v, x2, y2, v2, t, seg_cx, seg_cy, seg_mi;
  DevBuf<int32_t> g, pf, g2, pf2, labels, land_cnt, land_cell, seg_frame, seg_label;
  DevBuf<double> land_tot, edges;
  DevBuf<uint8_t> land_mask;
  DevBuf<uint32_t> k1_stage;           // K1 staged kept samples (count pass -> write pass)
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

int32_t rpt_stack::run(const rpt_stack_params& p, const void* echo, const float* scale,
                       const float* cos_t, const float* sin_t, const int32_t* gain,
                       rpt_stack_result* out, hipStream_t st) {
  const int32_t F = p.n_frames, G = p.files_per_frame;
  if (F < 0 || G < 1 || p.rows <= 0 || p.bins <= 0 || p.stride < 1 || !echo || !scale ||
      !cos_t || !sin_t) {
    set_error("rpt_stack_run: bad arguments");
    return RPT_EINVAL;
  }
  const int64_t n_files = (int64_t)F * G;
  n_frames = F;
  land_applied = false;
  had_gain = gain != nullptr;
  db_state = nullptr;
  const bool timing = p.timing != 0;
  if (timing && !ev_ok) {
    for (auto& e : ev) RPT_HIP(hipEventCreate(&e));
    ev_ok = true;
  }
  if (timing) RPT_HIP(hipEventRecord(ev[0], st));
  rpt_stack_result r{};

  // ---- K1: count -> per-file offsets (one readback sizes the outputs) -> write
  RPT_TRY(file_off.ensure((size_t)n_files + 1, st));
  RPT_TRY(down.ensure(sizeof(int64_t) * (size_t)(n_files + 2 * F + 8), st));
  int64_t* hfo = reinterpret_cast<int64_t*>(down.p);
  RPT_TRY(row_prefix.ensure((size_t)n_files * p.rows + 1, st));
  // u8 sweeps of 1024 bins: the count pass stages the kept samples of every group that keeps at
  // most 128 of them (the sparse radar case) and the write pass reads those instead of the echo,
  // so K1 reads the echo once (RPT_K1_STAGE=0: two full reads)
  const bool grouped = p.echo_dtype == RPT_ECHO_U8 && p.bins == 1024 &&
                       (uintptr_t)echo % 16 == 0;
  if (k1_staged < 0) {
    const char* e = ab_env("RPT_K1_STAGE");
    k1_staged = (e && std::atoi(e) == 0) ? 0 : 1;
  }
  uint32_t* mk = nullptr;
  if (grouped && k1_staged) {
    RPT_TRY(k1_stage.ensure((size_t)polar_stage_words(n_files, p.rows), st));
    mk = k1_stage.p;
  }
  RPT_TRY(polar_count(echo, p.echo_dtype, n_files, p.rows, p.bins, p.threshold, p.stride,
                      row_prefix.p, file_off.p, nullptr, st, mk));
  RPT_HIP(hipMemcpyAsync(hfo, file_off.p, sizeof(int64_t) * (n_files + 1), hipMemcpyDeviceToHost,
                         st));
  // u8 sweeps of 1024 bins, outputs sized by an earlier run: the write is queued right behind
  // the readback (capacity-bounded) instead of after the host has seen the count; when the
  // count exceeds the capacity the buffers grow and the write runs again
  int64_t spec_cap = -1;
  if (grouped && x.p && y.p && v.p && g.p && pf.p) {
    spec_cap = (int64_t)std::min({x.cap, y.cap, v.cap, g.cap, pf.cap});
    if (!ev_rb) RPT_HIP(hipEventCreateWithFlags(&ev_rb, hipEventDisableTiming));
    RPT_HIP(hipEventRecord(ev_rb, st));
    RPT_TRY(polar_write_cap((const uint8_t*)echo, n_files, p.rows, p.threshold, p.stride, scale,
                            cos_t, sin_t, gain, row_prefix.p, file_off.p, G, x.p, y.p, v.p,
                            gain ? g.p : nullptr, pf.p, spec_cap, st, mk));
    RPT_HIP(hipEventSynchronize(ev_rb));  // the readback only; the write keeps running
  } else {
    RPT_TRY(wait_stream(st));
  }
  const int64_t N = hfo[n_files];
  fo_k1.resize((size_t)F + 1);
  for (int32_t f = 0; f <= F; ++f) fo_k1[(size_t)f] = hfo[(size_t)f * G];
  r.n_points = N;
  int32_t n_built = 0;
  for (int32_t f = 0; f < F; ++f) n_built += (fo_k1[(size_t)f + 1] > fo_k1[(size_t)f]) ? 1 : 0;
  r.n_built = n_built;
  const size_t cap = (size_t)std::max<int64_t>(N, 1);
  if (N > spec_cap) {
    RPT_TRY(x.ensure(cap, st));
    RPT_TRY(y.ensure(cap, st));
    RPT_TRY(v.ensure(cap, st));
    RPT_TRY(g.ensure(cap, st));
    RPT_TRY(pf.ensure(cap, st));
    RPT_TRY(polar_write(echo, p.echo_dtype, n_files, p.rows, p.bins, scale, cos_t, sin_t, gain,
                        p.threshold, p.stride, row_prefix.p, file_off.p, G, x.p, y.p, v.p,
                        gain ? g.p : nullptr, pf.p, st, mk));
  }
  if (timing) RPT_HIP(hipEventRecord(ev[1], st));
  if (N == 0) {
    // no frame built: st_dbscan(frames) stacks nothing and returns {} (:463-464) -- no error,
    // no clusters, the tracker sees no frame
    RPT_TRY(wait_stream(st));
    fo_in = fo_k1;
    n_in = 0;
    h_count.clear();
    h_first.clear();
    h_frame.clear();
    h_label.clear();
    h_cx.clear();
    h_cy.clear();
    h_mi.clear();
    h_noise.assign((size_t)F, -1);
    seg_hint = 0;
    if (out) *out = r;
    return RPT_OK;
  }

  // ---- land filter (global grid over the stack, :954 gate: more than 10 built frames)
  float* cx = x.p;
  float* cy = y.p;
  float* cv = v.p;
  int32_t* cpf = pf.p;
  int64_t n_in_ = N;
  fo_in = fo_k1;
  r.n_land_cells = 0;
  if (p.land_filter && n_built > 10 && N > 0) {
    float b4[4];
    RPT_TRY(bounds_xy(x.p, y.p, N, b4, st));  // synchronises
    const std::vector<double> xe = arange_edges(b4[0], b4[1], p.land_resolution);
    const std::vector<double> ye = arange_edges(b4[2], b4[3], p.land_resolution);
    const int32_t nxe = (int32_t)xe.size(), nye = (int32_t)ye.size();
    if (nxe < 2 || nye < 2) {
      set_error("rpt_stack_run: degenerate land grid");
      return RPT_EINVAL;
    }
    const int64_t cells = (int64_t)(nxe - 1) * (nye - 1);
    // edges and the K1 frame offsets in ONE upload: [x edges | y edges | offsets (int64)]
    const size_t n_up = (size_t)(nxe + nye) + (size_t)F + 1;
    RPT_TRY(edges.ensure(n_up, st));
    RPT_TRY(up.ensure(sizeof(double) * n_up, st));
    double* he = reinterpret_cast<double*>(up.p);
    std::memcpy(he, xe.data(), sizeof(double) * nxe);
    std::memcpy(he + nxe, ye.data(), sizeof(double) * nye);
    int64_t* hf = reinterpret_cast<int64_t*>(he + nxe + nye);
    std::memcpy(hf, fo_k1.data(), sizeof(int64_t) * (F + 1));
    RPT_HIP(hipMemcpyAsync(edges.p, he, sizeof(double) * n_up, hipMemcpyHostToDevice, st));
    const int64_t* fo_dev = reinterpret_cast<const int64_t*>(edges.p + nxe + nye);
    RPT_TRY(land_cnt.ensure((size_t)cells, st));
    RPT_TRY(land_tot.ensure((size_t)cells, st));
    RPT_TRY(land_mask.ensure((size_t)cells, st));
    RPT_TRY(land_cell.ensure(cap, st));
    RPT_TRY(land_grid_cells(x.p, y.p, v.p, N, edges.p, nxe, edges.p + nxe, nye, land_cnt.p,
                            land_tot.p, land_cell.p, st, p.echo_dtype == RPT_ECHO_U8 ? 1 : 0));
    // the land-cell count accumulates (int32) into the low half of a zeroed int64 slot
    RPT_TRY(scal.ensure(4, st));
    RPT_HIP(hipMemsetAsync(scal.p, 0, sizeof(int64_t), st));
    RPT_TRY(land_mask_dev(land_cnt.p, land_tot.p, cells, n_built, p.land_persistence,
                          p.land_min_intensity, land_mask.p, reinterpret_cast<int32_t*>(scal.p),
                          st));
    RPT_TRY(x2.ensure(cap, st));
    RPT_TRY(y2.ensure(cap, st));
    RPT_TRY(v2.ensure(cap, st));
    RPT_TRY(g2.ensure(cap, st));
    RPT_TRY(pf2.ensure(cap, st));
    RPT_TRY(new_off.ensure((size_t)F + 1, st));
    // one fused compaction: the kept points in order, their frame times and their ST-DBSCAN
    // bounds (the kept count new_off[F] stays on the device), read back with the offsets and the
    // land-cell count: ONE round trip
    (void)fo_dev;
    RPT_TRY(t.ensure(cap, st));
    const size_t bnd_bytes = stdbscan_bounds_bytes();
    RPT_TRY(bnd.ensure(2 * bnd_bytes, st));
    RPT_TRY(land_compact_dev(x.p, y.p, v.p, gain ? g.p : nullptr, pf.p, N, land_cell.p,
                             land_mask.p, F, x2.p, y2.p, v2.p, gain ? g2.p : nullptr, pf2.p, t.p,
                             new_off.p, reinterpret_cast<Bounds*>(bnd.p), st));
    int64_t* hn = reinterpret_cast<int64_t*>(down.p);
    PackList pl;
    pl.add(new_off.p, sizeof(int64_t) * (F + 1));
    pl.add(scal.p, sizeof(int64_t));
    pl.add(bnd.p, bnd_bytes);
    RPT_TRY(pack_d.ensure((size_t)pl.off[pl.k], st));
    RPT_TRY(pack_arrays(pl, pack_d.p, st));
    RPT_HIP(hipMemcpyAsync(hn, pack_d.p, sizeof(uint32_t) * (size_t)pl.off[pl.k],
                           hipMemcpyDeviceToHost, st));
    RPT_TRY(wait_stream(st));
    fo_in.assign(hn, hn + F + 1);
    n_in_ = hn[F];
    r.n_land_cells = hn[F + 1];
    dbscan_bounds.assign(reinterpret_cast<const char*>(hn + F + 2),
                         reinterpret_cast<const char*>(hn + F + 2) + bnd_bytes);
    cx = x2.p;
    cy = y2.p;
    cv = v2.p;
    cpf = pf2.p;
    land_applied = true;
  }
  if (timing) RPT_HIP(hipEventRecord(ev[2], st));
  n_in = n_in_;
  r.n_clustered = n_in_;
  if (n_in_ == 0) {
    set_error("Found array with 0 sample(s) (shape=(0, 2)) while a minimum of 1 is required.");
    return RPT_EEMPTY;
  }

  // ---- ST-DBSCAN over the stack (times = frame slot as float32, :460-467)
  const size_t cap2 = (size_t)n_in_;
  RPT_TRY(labels.ensure(cap2, st));
  if (!land_applied) {  // with the land filter, the times and bounds came with its readback
    RPT_TRY(t.ensure(cap2, st));
    RPT_TRY(frame_times(cpf, n_in_, nullptr, t.p, st));
  }
  // ST-DBSCAN and K9 without readbacks in between: the cluster count and the segment count stay
  // on the device and come back with the results in ONE readback; the K9 sort runs with the
  // previous run's label bits and the summarize grid with its segment count, and both are
  // redone (rare) when the counts show they did not fit
  rpt_stdbscan_stats sts{};
  sts.timing = p.timing;
  const int32_t* ncl_dev = nullptr;
  void* dstate = nullptr;
  RPT_TRY(stdbscan_deferred(cx, cy, nullptr, 1, t.p, n_in_, p.eps_space, p.eps_time,
                            p.min_samples, labels.p, &sts, st, 2, &ncl_dev, &dstate,
                            land_applied ? dbscan_bounds.data() : nullptr));
  db_state = dstate;
  db_stream = st;
  if (timing) RPT_HIP(hipEventRecord(ev[3], st));

  // ---- K9 summaries (per-(frame, label) segments)
  RPT_TRY(seg_frame.ensure(cap2, st));
  RPT_TRY(seg_label.ensure(cap2, st));
  RPT_TRY(seg_count.ensure(cap2, st));
  RPT_TRY(seg_first.ensure(cap2, st));
  RPT_TRY(seg_cx.ensure(cap2, st));
  RPT_TRY(seg_cy.ensure(cap2, st));
  RPT_TRY(seg_mi.ensure(cap2, st));
  RPT_TRY(first_noise.ensure((size_t)std::max(F, 1), st));
  const int bits = ncl_dev ? sum_bits : radix_bits_for(sts.n_clusters);
  const int64_t sc = std::min<int64_t>(
      std::max<int64_t>(seg_hint > 0 ? seg_hint + seg_hint / 4 + 64 : 4096, 1), n_in_);
  const int32_t* nseg_dev = nullptr;
  bool radix_used = false;
  RPT_TRY(cluster_summaries_dev(labels.p, cx, cy, cv, cpf, n_in_, F, bits, sc, seg_frame.p,
                                seg_label.p, seg_count.p, seg_first.p, seg_cx.p, seg_cy.p,
                                seg_mi.p, first_noise.p, &nseg_dev, k9_radix, &radix_used, st));
  SegPack sp{seg_count.p, seg_first.p, first_noise.p, seg_frame.p,
             seg_label.p, seg_cx.p,    seg_cy.p,      seg_mi.p};
  size_t bytes = seg_pack_bytes(sc, F);
  RPT_TRY(pack_d.ensure(bytes / 4 + 1, st));
  RPT_TRY(down.ensure(bytes, st));
  hipLaunchKernelGGL(k_pack_segs, dim3(grid_for(std::max<int64_t>(sc, F), 256, 256)), dim3(256),
                     0, st, nseg_dev, ncl_dev, sp, sc, F, reinterpret_cast<char*>(pack_d.p));
  RPT_CHECK_LAUNCH();
  RPT_HIP(hipMemcpyAsync(down.p, pack_d.p, bytes, hipMemcpyDeviceToHost, st));
  if (timing) RPT_HIP(hipEventRecord(ev[4], st));
  RPT_TRY(wait_stream(st));
  int64_t S = reinterpret_cast<const int64_t*>(down.p)[0];
  const int64_t ncl = ncl_dev ? reinterpret_cast<const int64_t*>(down.p)[1] : sts.n_clusters;
  if (ncl_dev) RPT_TRY(stdbscan_fill_stats(dstate, (int32_t)ncl, &sts));
  int64_t sc_used = sc;
  // K9 again when the frame sort met a frame with too many labels (S = -1: the radix path, from
  // now on) or the radix path's label keys needed more bits; then the readback repeats until it
  // holds every segment (a redo changes the count)
  const bool bits_short = radix_used && (int64_t(1) << bits) <= ncl;
  if (S < 0 || bits_short || S > sc) {
    const bool rerun = S < 0 || bits_short;
    if (S < 0) k9_radix = true;
    if (rerun)
      RPT_TRY(cluster_summaries_dev(labels.p, cx, cy, cv, cpf, n_in_, F, radix_bits_for(ncl),
                                    std::max<int64_t>(S, sc), seg_frame.p, seg_label.p,
                                    seg_count.p, seg_first.p, seg_cx.p, seg_cy.p, seg_mi.p,
                                    first_noise.p, &nseg_dev, k9_radix, nullptr, st));
    sc_used = rerun ? sc : std::max<int64_t>(S, 1);
    for (int pass = 0; pass < 2; ++pass) {
      bytes = seg_pack_bytes(sc_used, F);
      RPT_TRY(pack_d.ensure(bytes / 4 + 1, st));
      RPT_TRY(down.ensure(bytes, st));
      hipLaunchKernelGGL(k_pack_segs, dim3(grid_for(std::max<int64_t>(sc_used, F), 256, 256)),
                         dim3(256), 0, st, nseg_dev, ncl_dev, sp, sc_used, F,
                         reinterpret_cast<char*>(pack_d.p));
      RPT_CHECK_LAUNCH();
      RPT_HIP(hipMemcpyAsync(down.p, pack_d.p, bytes, hipMemcpyDeviceToHost, st));
      RPT_TRY(wait_stream(st));
      S = reinterpret_cast<const int64_t*>(down.p)[0];
      if (S <= sc_used) break;
      sc_used = S;
    }
  }
  // next run's guesses: one pass of up to 12 bits when the count allows, with headroom
  const int exact = radix_bits_for(ncl);
  sum_bits = std::max(exact, std::min(radix_bits_for(2 * ncl + 64), std::max(exact, 12)));
  seg_hint = S;
  r.n_clusters = (int32_t)ncl;
  r.dbscan = sts;
  r.n_segments = S;
  const char* h = down.p + 16;
  const int64_t* hcount = reinterpret_cast<const int64_t*>(h);
  const int64_t* hfirst = hcount + sc_used;
  const int64_t* hnoise = hfirst + sc_used;
  const int32_t* hframe = reinterpret_cast<const int32_t*>(hnoise + F);
  const int32_t* hlabel = hframe + sc_used;
  const float* hcx = reinterpret_cast<const float*>(hlabel + sc_used);
  const float* hcy = hcx + sc_used;
  const float* hmi = hcy + sc_used;
  h_count.assign(hcount, hcount + S);
  h_first.assign(hfirst, hfirst + S);
  h_noise.assign(hnoise, hnoise + F);
  h_frame.assign(hframe, hframe + S);
  h_label.assign(hlabel, hlabel + S);
  h_cx.assign(hcx, hcx + S);
  h_cy.assign(hcy, hcy + S);
  h_mi.assign(hmi, hmi + S);
  if (timing) {
    float ms[4];
    for (int k = 0; k < 4; ++k) RPT_HIP(hipEventElapsedTime(&ms[k], ev[k], ev[k + 1]));
    r.ms_polar = ms[0];
    r.ms_land = ms[1];
    r.ms_stdbscan = ms[2];
    r.ms_summaries = ms[3];
  }
  if (out) *out = r;
  return RPT_OK;
}

extern "C" {

int32_t rpt_arange_edges(float lo, float hi, double res, double* out, int32_t cap) {
  const std::vector<double> e = arange_edges(lo, hi, res);
  if (out) std::copy(e.begin(), e.begin() + std::min<size_t>(e.size(), (size_t)std::max(cap, 0)), out);
  return (int32_t)e.size();
}

rpt_stack* rpt_stack_create(void) { return new rpt_stack(); }

void rpt_stack_destroy(rpt_stack* h) { delete h; }

int32_t rpt_stack_run(rpt_stack* h, const rpt_stack_params* p, const void* echo,
                      const float* scale, const float* cos_t, const float* sin_t,
                      const int32_t* gain, rpt_stack_result* out, void* stream) {
  clear_error();
  if (!h || !p) {
    set_error("rpt_stack_run: null handle or params");
    return RPT_EINVAL;
  }
  return h->run(*p, echo, scale, cos_t, sin_t, gain, out, as_stream(stream));
}

int32_t rpt_stack_frame_offsets(const rpt_stack* h, int32_t which, int64_t* out) {
  if (!h || !out || (which != 0 && which != 1)) return RPT_EINVAL;
  const auto& v = which == 0 ? h->fo_k1 : h->fo_in;
  std::copy(v.begin(), v.end(), out);
  return RPT_OK;
}

int32_t rpt_stack_segments(const rpt_stack* h, int32_t* frame, int32_t* label, int64_t* count,
                           int64_t* first, float* cx, float* cy, float* mean_i,
                           int64_t* frame_first_noise) {
  if (!h) return RPT_EINVAL;
  auto cp = [](const auto& v, auto* dst) {
    if (dst) std::copy(v.begin(), v.end(), dst);
  };
  cp(h->h_frame, frame);
  cp(h->h_label, label);
  cp(h->h_count, count);
  cp(h->h_first, first);
  cp(h->h_cx, cx);
  cp(h->h_cy, cy);
  cp(h->h_mi, mean_i);
  cp(h->h_noise, frame_first_noise);
  return RPT_OK;
}

int32_t rpt_stack_points(const rpt_stack* h, float* x, float* y, float* intensity,
                         int32_t* gain, int32_t* point_frame, int32_t* labels, void* stream) {
  clear_error();
  if (!h) return RPT_EINVAL;
  const hipStream_t st = as_stream(stream);
  const size_t n = (size_t)h->n_in;
  auto cp = [&](void* dst, const void* src, size_t es) -> int32_t {
    if (dst && src && n) RPT_HIP(hipMemcpyAsync(dst, src, n * es, hipMemcpyDeviceToDevice, st));
    return RPT_OK;
  };
  if (gain && !h->had_gain) {
    set_error("rpt_stack_points: the last rpt_stack_run had no gain table, so no per-point gains");
    return RPT_EINVAL;
  }
  const bool l = h->land_applied;
  RPT_TRY(cp(x, l ? h->x2.p : h->x.p, 4));
  RPT_TRY(cp(y, l ? h->y2.p : h->y.p, 4));
  RPT_TRY(cp(intensity, l ? h->v2.p : h->v.p, 4));
  RPT_TRY(cp(gain, l ? h->g2.p : h->g.p, 4));
  RPT_TRY(cp(point_frame, l ? h->pf2.p : h->pf.p, 4));
  RPT_TRY(cp(labels, h->labels.p, 4));
  return RPT_OK;
}

int32_t rpt_stack_core_flags(const rpt_stack* h, uint8_t* core, void* stream) {
  clear_error();
  if (!h || !core) return RPT_EINVAL;
  if (!h->db_state || h->n_in <= 0) {
    set_error("rpt_stack_core_flags: the last rpt_stack_run clustered no points");
    return RPT_EINVAL;
  }
  if (as_stream(stream) != h->db_stream) {
    set_error("rpt_stack_core_flags: call on the stream of the last rpt_stack_run");
    return RPT_EINVAL;
  }
  return stdbscan_core_flags(h->db_state, h->n_in, core, as_stream(stream));
}

}  // extern "C"

// =====================================================================================
// Frame-sharded multi-GPU driver: the per-rank phases of one global stack split
// over ranks.  The caller (rpt/dist.py, torch.distributed over RCCL) runs the collectives between
// the phases on device tensors it owns; every phase here is a few kernels plus at most one packed
// readback, so a rank's step costs the single-GPU driver's kernels plus ~10 small syncs.
namespace rpt {
namespace {

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

// own kept points -> the caller's x / y / t arrays, t = float32(frame0 + slot) (the global frame
// id of the stack, :460-467)
__global__ void k_pack_xyt(const float* __restrict__ x, const float* __restrict__ y,
                           const int32_t* __restrict__ pf, int64_t n, int64_t frame0,
                           float* __restrict__ xo, float* __restrict__ yo, float* __restrict__ to) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    xo[i] = x[i];
    yo[i] = y[i];
    to[i] = (float)(frame0 + (int64_t)pf[i]);
  }
}

// land grid [counts | sums] in float64 for the all-reduce (integer-valued: exact in any order)
__global__ void k_cnt_to_f64(const int32_t* __restrict__ cnt, int64_t cells,
                             double* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cells;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (double)cnt[i];
}
__global__ void k_f64_to_cnt(const double* __restrict__ in, int64_t cells,
                             int32_t* __restrict__ cnt) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cells;
       i += (int64_t)gridDim.x * blockDim.x)
    cnt[i] = (int32_t)in[i];
}

// global component ids: base + local component-min index, -1 for non-core
__global__ void k_comp_global(const int32_t* __restrict__ comp, int64_t n, int64_t base,
                              int64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = comp[i] >= 0 ? base + comp[i] : -1;
}

// equivalence pairs (my view of a halo point's component, its owner's view), both core, distinct;
// a pair equal to the previous point's is skipped (runs of one component along the halo) and,
// while ids fit 32 bits, every repeat of a pair (device hash set); the host dedupes any rest.  out[0] = count, pairs from out[1].
__global__ void k_pairs(const int64_t* __restrict__ mine, const int64_t* __restrict__ owner,
                        int64_t n, int64_t cap, unsigned long long* __restrict__ count,
                        unsigned long long* __restrict__ set, uint64_t set_mask,
                        int64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t a = mine[i], b = owner[i];
    if (a < 0 || b < 0 || a == b) continue;
    if (i > 0 && mine[i - 1] == a && owner[i - 1] == b) continue;
    const int64_t lo = a < b ? a : b, hi = a < b ? b : a;
    if (set && hi < (int64_t(1) << 32)) {
      // distinct pairs only: open-addressing set of (lo, hi) packed in 64 bits (2x the halo
      // size, so a probe always ends); the first inserter of a pair emits it
      const unsigned long long key = ((unsigned long long)lo << 32) | (unsigned long long)hi;
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
    const unsigned long long k = atomicAdd(count, 1ull);
    if ((int64_t)k < cap) {
      out[1 + 2 * k] = lo;
      out[2 + 2 * k] = hi;
    }
  }
}

__global__ void k_store_count(const unsigned long long* __restrict__ count, int64_t cap,
                              int64_t* __restrict__ out) {
  if (threadIdx.x == 0) out[0] = (int64_t)(*count < (unsigned long long)cap ? *count : cap);
}

}  // namespace
}  // namespace rpt

struct rpt_shard {
  rpt_stack st;                  // K1 / land buffers and the segment readback of the stack driver
  rpt::DbscanState* db = nullptr;
  rpt::DevBuf<uint32_t> bnd;     // xy bounds (ordered u32)
  rpt::DevBuf<int32_t> comp;     // local component ids of [prev | own | next]
  rpt::DevBuf<int64_t> rep, keys, vals, cnt64;
  rpt::DevBuf<unsigned long long> pset;  // distinct-pair hash set of rpt_shard_pairs
  rpt::DevBuf<int32_t> labels;
  rpt::DevBuf<uint8_t> scratch8;
  std::vector<double> xe, ye;
  rpt_stack_params p{};
  int64_t n_points = 0, n_kept = 0, n_total = 0, n_prev = 0;
  int32_t F = 0;
  bool land = false;
  hipEvent_t ev[2] = {};         // around the core-flag pass (params.timing)
  bool ev_ok = false, core_timed = false;
  ~rpt_shard() {
    if (ev_ok)
      for (auto& e : ev) (void)hipEventDestroy(e);
    if (db) rpt::dbscan_destroy(db);
    bnd.release();
    comp.release();
    rep.release();
    keys.release();
    vals.release();
    cnt64.release();
    labels.release();
    scratch8.release();
  }
};

using namespace rpt;

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
  rpt_stack& S = h->st;
  h->p = *p;
  S.had_gain = gain != nullptr;  // per-point gains only with a gain table
  const int32_t F = p->n_frames, G = p->files_per_frame;
  h->F = F;
  const int64_t n_files = (int64_t)F * G;
  RPT_TRY(S.file_off.ensure((size_t)n_files + 1, st));
  RPT_TRY(S.row_prefix.ensure((size_t)n_files * p->rows + 1, st));
  RPT_TRY(h->bnd.ensure(8, st));
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
    RPT_TRY(polar_write_cap((const uint8_t*)echo, n_files, p->rows, p->threshold, p->stride,
                            scale, cos_t, sin_t, gain, S.row_prefix.p, S.file_off.p, G, S.x.p,
                            S.y.p, S.v.p, gain ? S.g.p : nullptr, S.pf.p, spec_cap, st, mk));
    hipLaunchKernelGGL(k_init_bounds, dim3(1), dim3(64), 0, st, h->bnd.p);
    hipLaunchKernelGGL(k_xy_bounds_part, dim3(grid_for(std::max<int64_t>(spec_cap, 1), 256, 512)),
                       dim3(256), 0, st, S.x.p, S.y.p, spec_cap, n_dev, h->bnd.p);
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
    RPT_TRY(polar_write(echo, p->echo_dtype, n_files, p->rows, p->bins, scale, cos_t, sin_t, gain,
                        p->threshold, p->stride, S.row_prefix.p, S.file_off.p, G, S.x.p, S.y.p,
                        S.v.p, gain ? S.g.p : nullptr, S.pf.p, st, mk));
    hipLaunchKernelGGL(k_init_bounds, dim3(1), dim3(64), 0, st, h->bnd.p);
    hipLaunchKernelGGL(k_xy_bounds_part, dim3(grid_for(std::max<int64_t>(N, 1), 256, 512)),
                       dim3(256), 0, st, S.x.p, S.y.p, N, (const int64_t*)nullptr, h->bnd.p);
    RPT_CHECK_LAUNCH();
    RPT_HIP(hipMemcpyAsync(hb, h->bnd.p, 16, hipMemcpyDeviceToHost, st));
    RPT_TRY(wait_stream(st));
  }
  S.fo_k1.resize((size_t)F + 1);
  for (int32_t f = 0; f <= F; ++f) S.fo_k1[(size_t)f] = hfo[(size_t)f * G];
  int32_t built = 0;
  for (int32_t f = 0; f < F; ++f) built += S.fo_k1[(size_t)f + 1] > S.fo_k1[(size_t)f];
  h->n_points = N;
  *info = rpt_shard_info{};
  info->n_points = N;
  info->n_built = built;
  if (N > 0) {
    info->bounds[0] = ord_to_f(hb[0]);
    info->bounds[1] = ord_to_f(hb[1]);
    info->bounds[2] = ord_to_f(hb[2]);
    info->bounds[3] = ord_to_f(hb[3]);
  } else {
    info->bounds[0] = info->bounds[2] = INFINITY;
    info->bounds[1] = info->bounds[3] = -INFINITY;
  }
  info->n_kept = N;
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
  h->xe = arange_edges(gbounds[0], gbounds[1], h->p.land_resolution);
  h->ye = arange_edges(gbounds[2], gbounds[3], h->p.land_resolution);
  const int32_t nxe = (int32_t)h->xe.size(), nye = (int32_t)h->ye.size();
  if (nxe < 2 || nye < 2 || (int64_t)(nxe - 1) * (nye - 1) != cells) {
    set_error("rpt_shard_land_grid: grid of %lld cells does not match the bounds",
              (long long)cells);
    return RPT_EINVAL;
  }
  const int32_t F = h->F;
  const size_t n_up = (size_t)(nxe + nye) + (size_t)F + 1;
  RPT_TRY(S.edges.ensure(n_up, st));
  RPT_TRY(S.up.ensure(sizeof(double) * n_up, st));  // its last upload completed: syncs since
  double* he = reinterpret_cast<double*>(S.up.p);
  std::memcpy(he, h->xe.data(), sizeof(double) * nxe);
  std::memcpy(he + nxe, h->ye.data(), sizeof(double) * nye);
  std::memcpy(reinterpret_cast<int64_t*>(he + nxe + nye), S.fo_k1.data(),
              sizeof(int64_t) * (F + 1));
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

int32_t rpt_shard_land_apply(rpt_shard* h, const double* grid, int64_t cells,
                             int32_t n_built_global, int32_t halo_frames, int64_t frame0,
                             float* x_out, float* y_out, float* t_out, rpt_shard_info* info,
                             void* stream) {
  clear_error();
  if (!h || !info || (h->n_points > 0 && (!x_out || !y_out || !t_out)) || halo_frames < 0) {
    set_error("rpt_shard_land_apply: bad arguments");
    return RPT_EINVAL;
  }
  const hipStream_t st = as_stream(stream);
  rpt_stack& S = h->st;
  const int32_t F = h->F;
  const int64_t N = h->n_points;
  const int32_t hf = std::min(halo_frames, F);
  RPT_TRY(S.new_off.ensure((size_t)F + 2, st));
  RPT_TRY(S.scal.ensure(4, st));
  h->land = grid != nullptr && cells > 0 && N >= 0;
  const float* cx = S.x.p;
  const float* cy = S.y.p;
  const int32_t* cpf = S.pf.p;
  int64_t* hn = reinterpret_cast<int64_t*>(S.down.p);
  RPT_TRY(S.down.ensure(sizeof(int64_t) * (size_t)(F + 4), st));
  hn = reinterpret_cast<int64_t*>(S.down.p);
  if (h->land) {
    RPT_TRY(S.land_cnt.ensure((size_t)cells, st));
    RPT_TRY(S.land_mask.ensure((size_t)cells, st));
    hipLaunchKernelGGL(k_f64_to_cnt, dim3(grid_for(cells, 256, 1024)), dim3(256), 0, st, grid,
                       cells, S.land_cnt.p);
    RPT_CHECK_LAUNCH();
    RPT_HIP(hipMemsetAsync(S.scal.p, 0, sizeof(int64_t), st));
    RPT_TRY(land_mask_dev(S.land_cnt.p, grid + cells, cells, n_built_global, h->p.land_persistence,
                          h->p.land_min_intensity, S.land_mask.p,
                          reinterpret_cast<int32_t*>(S.scal.p), st));
    const size_t cap = (size_t)std::max<int64_t>(N, 1);
    RPT_TRY(S.x2.ensure(cap, st));
    RPT_TRY(S.y2.ensure(cap, st));
    RPT_TRY(S.v2.ensure(cap, st));
    RPT_TRY(S.g2.ensure(cap, st));
    RPT_TRY(S.pf2.ensure(cap, st));
    if (N > 0) {  // the fused compaction (kept points in order, new frame offsets)
      RPT_TRY(S.t.ensure(cap, st));
      RPT_TRY(S.bnd.ensure(2 * sizeof(Bounds), st));
      RPT_TRY(land_compact_dev(S.x.p, S.y.p, S.v.p, S.had_gain ? S.g.p : nullptr, S.pf.p, N,
                               S.land_cell.p, S.land_mask.p, F, S.x2.p, S.y2.p, S.v2.p,
                               S.had_gain ? S.g2.p : nullptr, S.pf2.p, S.t.p,
                               S.new_off.p, reinterpret_cast<Bounds*>(S.bnd.p), st));
    } else
      RPT_HIP(hipMemsetAsync(S.new_off.p, 0, sizeof(int64_t) * (F + 1), st));
    RPT_HIP(hipMemcpyAsync(hn, S.new_off.p, sizeof(int64_t) * (F + 1), hipMemcpyDeviceToHost,
                           st));
    RPT_HIP(hipMemcpyAsync(hn + F + 1, S.scal.p, sizeof(int64_t), hipMemcpyDeviceToHost, st));
    RPT_TRY(wait_stream(st));
    S.fo_in.assign(hn, hn + F + 1);
    info->n_land_cells = hn[F + 1];
    cx = S.x2.p;
    cy = S.y2.p;
    cpf = S.pf2.p;
  } else {
    S.fo_in = S.fo_k1;
    info->n_land_cells = 0;
  }
  S.land_applied = h->land;
  const int64_t K = S.fo_in[(size_t)F];
  h->n_kept = K;
  if (K > 0) {
    hipLaunchKernelGGL(k_pack_xyt, dim3(grid_for(K, 256, 4096)), dim3(256), 0, st, cx, cy, cpf,
                       K, frame0, x_out, y_out, t_out);
    RPT_CHECK_LAUNCH();
  }
  info->n_points = N;
  info->n_kept = K;
  info->n_head = S.fo_in[(size_t)hf];
  info->n_tail = K - S.fo_in[(size_t)(F - hf)];
  return RPT_OK;
}

int32_t rpt_shard_core(rpt_shard* h, const float* x, const float* y, const float* t, int64_t n,
                       uint8_t* core, void* stream) {
  clear_error();
  if (!h || !x || !y || !t || !core || n <= 0) {
    set_error("rpt_shard_core: bad arguments (n must be > 0)");
    return RPT_EINVAL;
  }
  const hipStream_t st = as_stream(stream);
  h->n_total = n;
  RPT_TRY(dbscan_build(h->db, x, y, nullptr, 1, t, n, h->p.eps_space, h->p.eps_time,
                       h->p.min_samples, st));
  if (h->p.timing) {
    if (!h->ev_ok) {
      RPT_HIP(hipEventCreate(&h->ev[0]));
      RPT_HIP(hipEventCreate(&h->ev[1]));
      h->ev_ok = true;
    }
    RPT_HIP(hipEventRecord(h->ev[0], st));
  }
  RPT_TRY(dbscan_core(h->db, core, st));
  if (h->p.timing) RPT_HIP(hipEventRecord(h->ev[1], st));
  h->core_timed = h->p.timing != 0;
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

int32_t rpt_shard_components(rpt_shard* h, const uint8_t* core, int64_t base, int64_t* comp,
                             void* stream) {
  clear_error();
  if (!h || !core || !comp) {
    set_error("rpt_shard_components: bad arguments");
    return RPT_EINVAL;
  }
  const hipStream_t st = as_stream(stream);
  const int64_t n = h->n_total;
  RPT_TRY(h->comp.ensure((size_t)n, st));
  RPT_TRY(dbscan_set_core(h->db, core, st));
  RPT_TRY(dbscan_components(h->db, h->comp.p, st));
  hipLaunchKernelGGL(k_comp_global, dim3(grid_for(n, 256, 4096)), dim3(256), 0, st, h->comp.p,
                     n, base, comp);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

int32_t rpt_shard_pairs(rpt_shard* h, const int64_t* comp, int64_t n_prev,
                        const int64_t* owner_prev, int64_t n_next, const int64_t* owner_next,
                        int64_t* pairs, int64_t cap, void* stream) {
  clear_error();
  if (!h || !comp || !pairs || cap < 0 || (n_prev > 0 && !owner_prev) ||
      (n_next > 0 && !owner_next)) {
    set_error("rpt_shard_pairs: bad arguments");
    return RPT_EINVAL;
  }
  const hipStream_t st = as_stream(stream);
  RPT_TRY(h->cnt64.ensure(2, st));
  RPT_HIP(hipMemsetAsync(h->cnt64.p, 0, sizeof(int64_t), st));
  auto* cnt = reinterpret_cast<unsigned long long*>(h->cnt64.p);
  uint64_t tsize = 64;
  while (tsize < (uint64_t)(2 * (n_prev + n_next))) tsize <<= 1;
  RPT_TRY(h->pset.ensure((size_t)tsize, st));
  RPT_HIP(hipMemsetAsync(h->pset.p, 0xFF, tsize * sizeof(unsigned long long), st));
  if (n_prev > 0)
    hipLaunchKernelGGL(k_pairs, dim3(grid_for(n_prev, 256, 1024)), dim3(256), 0, st, comp,
                       owner_prev, n_prev, cap, cnt, h->pset.p, tsize - 1, pairs);
  if (n_next > 0)
    hipLaunchKernelGGL(k_pairs, dim3(grid_for(n_next, 256, 1024)), dim3(256), 0, st,
                       comp + (h->n_total - n_next), owner_next, n_next, cap, cnt, h->pset.p,
                       tsize - 1, pairs);
  hipLaunchKernelGGL(k_store_count, dim3(1), dim3(64), 0, st, cnt, cap, pairs);
  RPT_CHECK_LAUNCH();
  return RPT_OK;
}

int32_t rpt_shard_roots(rpt_shard* h, const int64_t* keys, const int64_t* vals, int64_t n_keys,
                        int64_t base, int64_t n_prev, int64_t n_own, int64_t* roots,
                        int64_t* n_roots, void* stream) {
  clear_error();
  if (!h || !roots || !n_roots || n_keys < 0 || (n_keys > 0 && (!keys || !vals))) {
    set_error("rpt_shard_roots: bad arguments");
    return RPT_EINVAL;
  }
  const hipStream_t st = as_stream(stream);
  const int64_t n = h->n_total;
  h->n_prev = n_prev;
  RPT_TRY(h->rep.ensure((size_t)n, st));
  RPT_TRY(h->keys.ensure((size_t)std::max<int64_t>(2 * n_keys, 1), st));
  rpt_stack& S = h->st;
  if (n_keys > 0) {
    RPT_TRY(S.up.ensure(sizeof(int64_t) * 2 * (size_t)n_keys, st));  // idle: syncs since
    int64_t* hu = reinterpret_cast<int64_t*>(S.up.p);
    std::memcpy(hu, keys, sizeof(int64_t) * n_keys);
    std::memcpy(hu + n_keys, vals, sizeof(int64_t) * n_keys);
    RPT_HIP(hipMemcpyAsync(h->keys.p, hu, sizeof(int64_t) * 2 * n_keys, hipMemcpyHostToDevice,
                           st));
  }
  RPT_TRY(remap_components(h->comp.p, n, base, h->keys.p, h->keys.p + n_keys, n_keys, h->rep.p,
                           st));
  return select_roots(h->rep.p, base, n_prev, n_prev + n_own, roots, n_roots, st);
}

int32_t rpt_shard_finish(rpt_shard* h, const int64_t* reps_sorted, int64_t n_reps,
                         int64_t* n_segments, void* stream) {
  clear_error();
  if (!h || !n_segments || (n_reps > 0 && !reps_sorted)) {
    set_error("rpt_shard_finish: bad arguments");
    return RPT_EINVAL;
  }
  const hipStream_t st = as_stream(stream);
  rpt_stack& S = h->st;
  const int64_t n = h->n_total, K = h->n_kept;
  const int32_t F = h->F;
  RPT_TRY(h->labels.ensure((size_t)std::max<int64_t>(n, 1), st));
  RPT_TRY(dbscan_labels_global(h->db, h->rep.p, reps_sorted, n_reps, h->labels.p, st));
  const int32_t* lab = h->labels.p + h->n_prev;
  const bool l = S.land_applied;
  const float* x = l ? S.x2.p : S.x.p;
  const float* y = l ? S.y2.p : S.y.p;
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
  int bits = 1;
  while ((int64_t(1) << bits) <= n_reps) ++bits;
  int64_t Sg = 0;
  if (K > 0) {
    const int32_t* nseg_dev = nullptr;
    auto k9 = [&]() {
      return cluster_summaries_dev(lab, x, y, v, pf, K, F, bits, K, S.seg_frame.p, S.seg_label.p,
                                   S.seg_count.p, S.seg_first.p, S.seg_cx.p, S.seg_cy.p,
                                   S.seg_mi.p, S.first_noise.p, &nseg_dev, S.k9_radix, nullptr,
                                   st);
    };
    RPT_TRY(k9());
    SegPack sp{S.seg_count.p, S.seg_first.p, S.first_noise.p, S.seg_frame.p,
               S.seg_label.p, S.seg_cx.p,    S.seg_cy.p,      S.seg_mi.p};
    // readback sized by the previous run's segment count (+ headroom); again when it overflows,
    // and after a redo on the radix path when a frame held too many labels (count -1)
    int64_t sc = std::min<int64_t>(std::max<int64_t>(S.seg_hint > 0 ? S.seg_hint + S.seg_hint / 4 + 64
                                                                   : 4096, 1), K);
    for (int pass = 0; pass < 3; ++pass) {
      const size_t bytes = seg_pack_bytes(sc, F);
      RPT_TRY(S.pack_d.ensure(bytes / 4 + 1, st));
      RPT_TRY(S.down.ensure(bytes, st));
      hipLaunchKernelGGL(k_pack_segs, dim3(grid_for(std::max<int64_t>(sc, F), 256, 256)),
                         dim3(256), 0, st, nseg_dev, (const int32_t*)nullptr, sp, sc, F,
                         reinterpret_cast<char*>(S.pack_d.p));
      RPT_CHECK_LAUNCH();
      RPT_HIP(hipMemcpyAsync(S.down.p, S.pack_d.p, bytes, hipMemcpyDeviceToHost, st));
      RPT_TRY(wait_stream(st));
      Sg = reinterpret_cast<const int64_t*>(S.down.p)[0];
      if (Sg < 0 && !S.k9_radix) {
        S.k9_radix = true;
        RPT_TRY(k9());
        continue;
      }
      if (Sg <= sc) break;
      sc = Sg;
    }
    S.seg_hint = Sg;
    const char* hp = S.down.p + 16;
    const int64_t* hcount = reinterpret_cast<const int64_t*>(hp);
    const int64_t* hfirst = hcount + sc;
    const int64_t* hnoise = hfirst + sc;
    const int32_t* hframe = reinterpret_cast<const int32_t*>(hnoise + F);
    const int32_t* hlabel = hframe + sc;
    const float* hcx = reinterpret_cast<const float*>(hlabel + sc);
    const float* hcy = hcx + sc;
    const float* hmi = hcy + sc;
    S.h_count.assign(hcount, hcount + Sg);
    S.h_first.assign(hfirst, hfirst + Sg);
    S.h_noise.assign(hnoise, hnoise + F);
    S.h_frame.assign(hframe, hframe + Sg);
    S.h_label.assign(hlabel, hlabel + Sg);
    S.h_cx.assign(hcx, hcx + Sg);
    S.h_cy.assign(hcy, hcy + Sg);
    S.h_mi.assign(hmi, hmi + Sg);
  } else {
    S.h_count.clear();
    S.h_first.clear();
    S.h_frame.clear();
    S.h_label.clear();
    S.h_cx.clear();
    S.h_cy.clear();
    S.h_mi.clear();
    S.h_noise.assign((size_t)F, -1);
  }
  S.n_frames = F;
  S.n_in = K;
  *n_segments = Sg;
  return RPT_OK;
}

int32_t rpt_shard_segments(const rpt_shard* h, int32_t* frame, int32_t* label, int64_t* count,
                           int64_t* first, float* cx, float* cy, float* mean_i,
                           int64_t* frame_first_noise) {
  if (!h) return RPT_EINVAL;
  return rpt_stack_segments(&h->st, frame, label, count, first, cx, cy, mean_i,
                            frame_first_noise);
}

int32_t rpt_shard_labels(const rpt_shard* h, int32_t* out, void* stream) {
  clear_error();
  if (!h || !out) {
    set_error("rpt_shard_labels: bad arguments");
    return RPT_EINVAL;
  }
  if (h->n_kept == 0) return RPT_OK;
  if (!h->labels.p || h->labels.cap < (size_t)(h->n_prev + h->n_kept)) {
    set_error("rpt_shard_labels: no labels (rpt_shard_finish first)");
    return RPT_EINVAL;
  }
  RPT_HIP(hipMemcpyAsync(out, h->labels.p + h->n_prev, sizeof(int32_t) * (size_t)h->n_kept,
                         hipMemcpyDeviceToDevice, as_stream(stream)));
  return RPT_OK;
}

int32_t rpt_shard_frame_offsets(const rpt_shard* h, int32_t which, int64_t* out) {
  if (!h) return RPT_EINVAL;
  return rpt_stack_frame_offsets(&h->st, which, out);
}

/* host: union of equivalence pairs (a, b) -> sorted distinct ids with their class minimum */
int64_t rpt_merge_equivalences(const int64_t* pairs, int64_t n_pairs, int64_t* keys_out,
                               int64_t* reps_out, int64_t cap) {
  std::vector<int64_t> ids;
  ids.reserve((size_t)(2 * std::max<int64_t>(n_pairs, 0)));
  for (int64_t i = 0; i < 2 * n_pairs; ++i) ids.push_back(pairs[i]);
  std::sort(ids.begin(), ids.end());
  ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
  const int64_t m = (int64_t)ids.size();
  std::vector<int64_t> par((size_t)m);
  for (int64_t i = 0; i < m; ++i) par[(size_t)i] = i;
  auto find = [&](int64_t a) {
    while (par[(size_t)a] != a) {
      par[(size_t)a] = par[(size_t)par[(size_t)a]];
      a = par[(size_t)a];
    }
    return a;
  };
  auto idx = [&](int64_t v) {
    return (int64_t)(std::lower_bound(ids.begin(), ids.end(), v) - ids.begin());
  };
  for (int64_t i = 0; i < n_pairs; ++i) {
    int64_t a = find(idx(pairs[2 * i])), b = find(idx(pairs[2 * i + 1]));
    if (a == b) continue;
    if (a > b) std::swap(a, b);
    par[(size_t)b] = a;  // ids are sorted: the smaller index is the smaller id
  }
  if (keys_out && reps_out)
    for (int64_t i = 0; i < std::min(m, cap); ++i) {
      keys_out[i] = ids[(size_t)i];
      reps_out[i] = ids[(size_t)find(i)];
    }
  return m;
}

}  // extern "C"
