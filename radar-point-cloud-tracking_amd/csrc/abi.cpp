// extern "C" surface of librpt.so (declared in include/rpt.h).  Thin: argument checks,
// error-code translation, dispatch into the rpt:: implementations.
#include <hip/hip_runtime.h>

#include <cstring>

#include "common.h"

namespace rpt {
void release_scratch_current();
int32_t label_means(const int32_t* labels, const float* x, const float* y, const float* inten,
                    int64_t n, int64_t n_labels, int64_t* o_count, float* o_x, float* o_y,
                    float* o_v, hipStream_t st);
int32_t stdbscan_denoise(const float* x, const float* y, const float* t, int64_t n,
                         double eps_space, double eps_time, int32_t min_samples,
                         int32_t min_frames, int32_t* labels, rpt_stdbscan_stats* stats,
                         hipStream_t st);
int32_t stdbscan(const float* x, const float* y, const float* z, int64_t stride, const float* t,
                 int64_t n, double eps_space, double eps_time, int32_t min_samples,
                 int32_t* labels, rpt_stdbscan_stats* stats, hipStream_t st, int dim);
int32_t polar_count(const void* echo, int32_t dt, int64_t n_files, int32_t rows, int32_t bins,
                    float thr, int32_t stride, int64_t* row_prefix, int64_t* file_offsets,
                    int64_t* total_host, hipStream_t st, uint32_t* entries);
int32_t polar_write(const void* echo, int32_t dt, int64_t n_files, int32_t rows, int32_t bins,
                    const float* scale, const float* cos_t, const float* sin_t,
                    const int32_t* gain, float thr, int32_t stride, const int64_t* row_prefix,
                    const int64_t* file_offsets, int32_t files_per_frame, float* x, float* y,
                    float* v, int32_t* gout, int32_t* pf, hipStream_t st, const uint32_t* entries,
                    uint32_t* bnd = nullptr, bool* bnd_done = nullptr);
int64_t polar_stage_words(int64_t n_files, int32_t rows);
int32_t frame_times(const int32_t* pf, int64_t n, const int64_t* ids, float* t, hipStream_t st);
int32_t sweep_to_points(const float* inten, const float* ranges, const float* cos_t,
                        const float* sin_t, int32_t rows, int32_t bins, float thr,
                        int32_t stride, float* x, float* y, float* z, int64_t capacity,
                        int64_t* n_out_host, hipStream_t st);
int32_t polar_to_cartesian(const float* cos_t, const float* sin_t, const float* ranges,
                           int64_t rows, int64_t bins, float* x, float* y, hipStream_t st);
int32_t infer_time_from_colors(const uint8_t* colors, int64_t n, const float* pal, int32_t n_pal,
                               float* out, hipStream_t st);
int32_t synth_echo(const rpt_synth_params* p, int64_t frame0, int64_t n_frames,
                   const float* cos_t, const float* sin_t, const uint32_t* clutter_thresh,
                   const float* targets, const int32_t* trows, const int32_t* tbins,
                   uint8_t* echo, hipStream_t st);
int32_t bounds_xy(const float* x, const float* y, int64_t n, float* out4, hipStream_t st);
int32_t land_grid(const float* x, const float* y, const float* val, int64_t n, const double* xe,
                  int32_t nxe, const double* ye, int32_t nye, int32_t* cnt, double* tot,
                  hipStream_t st);
int32_t land_mask(const int32_t* cnt, const double* tot, int64_t cells, int64_t num_frames,
                  double pthr, double ithr, uint8_t* land, int64_t* n_land_host,
                  hipStream_t st);
int32_t land_filter(const float* x, const float* y, const float* v, const int32_t* g,
                    const int32_t* pf, int64_t n, const int64_t* frame_off, int32_t n_frames,
                    const double* xe, int32_t nxe, const double* ye, int32_t nye,
                    const uint8_t* land, float* xo, float* yo, float* vo, int32_t* go,
                    int32_t* pfo, int64_t* new_off, int64_t* n_kept_host, hipStream_t st);
int32_t cluster_summaries(const int32_t* labels, const float* x, const float* y,
                          const float* inten, const int32_t* pf, int64_t n, int32_t n_frames,
                          int32_t n_clusters, int32_t* o_frame, int32_t* o_label,
                          int64_t* o_count, int64_t* o_first, float* o_cx, float* o_cy,
                          float* o_mi, int64_t* frame_first_noise, int64_t* n_seg_host,
                          hipStream_t st);
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
int32_t remap_components(const int32_t* comp, int64_t n, int64_t base, const int64_t* keys,
                         const int64_t* vals, int64_t nk, int64_t* out, hipStream_t st);
int32_t select_roots(const int64_t* rep, int64_t base, int64_t lo, int64_t hi, int64_t* out,
                     int64_t* count_host, hipStream_t st);
}  // namespace rpt

struct rpt_dbscan {
  rpt::DbscanState* s;
};

extern "C" {

rpt_dbscan* rpt_dbscan_create(void) { return new rpt_dbscan{rpt::dbscan_create()}; }

void rpt_dbscan_destroy(rpt_dbscan* h) {
  if (!h) return;
  rpt::dbscan_destroy(h->s);
  delete h;
}

int32_t rpt_dbscan_build(rpt_dbscan* h, const float* x, const float* y, const float* z,
                         int64_t stride, const float* times, int64_t n, double eps_space,
                         double eps_time, int32_t min_samples, void* stream) {
  rpt::clear_error();
  return rpt::dbscan_build(h->s, x, y, z, stride, times, n, eps_space, eps_time, min_samples,
                           rpt::as_stream(stream));
}

int32_t rpt_dbscan_core(rpt_dbscan* h, uint8_t* core_out, void* stream) {
  rpt::clear_error();
  return rpt::dbscan_core(h->s, core_out, rpt::as_stream(stream));
}

int32_t rpt_dbscan_set_core(rpt_dbscan* h, const uint8_t* core_in, void* stream) {
  rpt::clear_error();
  return rpt::dbscan_set_core(h->s, core_in, rpt::as_stream(stream));
}

int32_t rpt_dbscan_components(rpt_dbscan* h, int32_t* comp_out, void* stream) {
  rpt::clear_error();
  return rpt::dbscan_components(h->s, comp_out, rpt::as_stream(stream));
}

int32_t rpt_dbscan_labels_global(rpt_dbscan* h, const int64_t* rep, const int64_t* reps_sorted,
                                 int64_t n_reps, int32_t* labels, void* stream) {
  rpt::clear_error();
  return rpt::dbscan_labels_global(h->s, rep, reps_sorted, n_reps, labels,
                                   rpt::as_stream(stream));
}

int32_t rpt_remap_components(const int32_t* comp, int64_t n, int64_t base, const int64_t* keys,
                             const int64_t* vals, int64_t n_keys, int64_t* rep_out,
                             void* stream) {
  rpt::clear_error();
  return rpt::remap_components(comp, n, base, keys, vals, n_keys, rep_out,
                               rpt::as_stream(stream));
}

int32_t rpt_select_roots(const int64_t* rep, int64_t base, int64_t lo, int64_t hi, int64_t* out,
                         int64_t* count_host, void* stream) {
  rpt::clear_error();
  return rpt::select_roots(rep, base, lo, hi, out, count_host, rpt::as_stream(stream));
}




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

int32_t rpt_exclusive_scan(const void* in, int32_t in_dtype, int64_t n, void* out,
                           int32_t out_dtype, int32_t with_total, void* stream) {
  rpt::clear_error();
  if (n < 0 || (n > 0 && (!in || !out))) {
    rpt::set_error("rpt_exclusive_scan: bad arguments");
    return RPT_EINVAL;
  }
  const hipStream_t st = rpt::as_stream(stream);
  const auto* i32 = static_cast<const int32_t*>(in);
  if (in_dtype == RPT_I32 && out_dtype == RPT_I32)
    return with_total ? rpt::exclusive_scan_total_i32(i32, static_cast<int32_t*>(out), n, st)
                      : rpt::exclusive_scan_i32(i32, static_cast<int32_t*>(out), n, nullptr, st);
  if (in_dtype == RPT_I32 && out_dtype == RPT_I64)
    return with_total
               ? rpt::exclusive_scan_total_i32_to_i64(i32, static_cast<int64_t*>(out), n, st)
               : rpt::exclusive_scan_i32_to_i64(i32, static_cast<int64_t*>(out), n, nullptr, st);
  if (in_dtype == RPT_I64 && out_dtype == RPT_I64) {
    const auto* i64 = static_cast<const int64_t*>(in);
    return with_total ? rpt::exclusive_scan_total_i64(i64, static_cast<int64_t*>(out), n, st)
                      : rpt::exclusive_scan_i64(i64, static_cast<int64_t*>(out), n, nullptr, st);
  }
  rpt::set_error("rpt_exclusive_scan: dtypes must be i32->i32, i32->i64 or i64->i64");
  return RPT_ENOTSUP;
}

int32_t rpt_stdbscan(const float* x, const float* y, const float* z, int64_t stride,
                     const float* times, int64_t n, double eps_space, double eps_time,
                     int32_t min_samples, int32_t* labels, rpt_stdbscan_stats* stats,
                     void* stream) {
  rpt::clear_error();
  const int dim = z ? 3 : 2;
  return rpt::stdbscan(x, y, z, stride, times, n, eps_space, eps_time, min_samples, labels,
                       stats, rpt::as_stream(stream), dim);
}

int32_t rpt_label_means(const int32_t* labels, const float* x, const float* y,
                        const float* intensity, int64_t n, int64_t n_labels, int64_t* count,
                        float* mean_x, float* mean_y, float* mean_intensity, void* stream) {
  rpt::clear_error();
  return rpt::label_means(labels, x, y, intensity, n, n_labels, count, mean_x, mean_y,
                          mean_intensity, rpt::as_stream(stream));
}

int32_t rpt_stdbscan_denoise(const float* x, const float* y, const float* times, int64_t n,
                             double eps_space, double eps_time, int32_t min_samples,
                             int32_t min_frames, int32_t* labels, rpt_stdbscan_stats* stats,
                             void* stream) {
  rpt::clear_error();
  if (n < 0) {
    rpt::set_error("rpt_stdbscan_denoise: n < 0");
    return RPT_EINVAL;
  }
  return rpt::stdbscan_denoise(x, y, times, n, eps_space, eps_time, min_samples, min_frames,
                               labels, stats, rpt::as_stream(stream));
}

int32_t rpt_polar_count(const void* echo, int32_t echo_dtype, int64_t n_files, int32_t rows,
                        int32_t bins, float threshold, int32_t stride, int64_t* row_prefix,
                        int64_t* file_offsets, int64_t* total_host, void* stream) {
  rpt::clear_error();
  return rpt::polar_count(echo, echo_dtype, n_files, rows, bins, threshold, stride, row_prefix,
                          file_offsets, total_host, rpt::as_stream(stream), nullptr);
}

int64_t rpt_polar_stage_words(int64_t n_files, int32_t rows) {
  return (n_files > 0 && rows > 0) ? rpt::polar_stage_words(n_files, rows) : 0;
}

int32_t rpt_polar_count_staged(const void* echo, int32_t echo_dtype, int64_t n_files,
                               int32_t rows, int32_t bins, float threshold, int32_t stride,
                               int64_t* row_prefix, int64_t* file_offsets, int64_t* total_host,
                               uint32_t* entries, void* stream) {
  rpt::clear_error();
  return rpt::polar_count(echo, echo_dtype, n_files, rows, bins, threshold, stride, row_prefix,
                          file_offsets, total_host, rpt::as_stream(stream), entries);
}

int32_t rpt_polar_write(const void* echo, int32_t echo_dtype, int64_t n_files, int32_t rows,
                        int32_t bins, const float* scale, const float* cos_t, const float* sin_t,
                        const int32_t* gain, float threshold, int32_t stride,
                        const int64_t* row_prefix, const int64_t* file_offsets,
                        int32_t files_per_frame, float* x, float* y, float* intensity,
                        int32_t* gain_out, int32_t* point_frame_out, void* stream) {
  rpt::clear_error();
  return rpt::polar_write(echo, echo_dtype, n_files, rows, bins, scale, cos_t, sin_t, gain,
                          threshold, stride, row_prefix, file_offsets, files_per_frame, x, y,
                          intensity, gain_out, point_frame_out, rpt::as_stream(stream), nullptr);
}

int32_t rpt_polar_write_staged(const void* echo, int32_t echo_dtype, int64_t n_files,
                               int32_t rows, int32_t bins, const float* scale, const float* cos_t,
                               const float* sin_t, const int32_t* gain, float threshold,
                               int32_t stride, const int64_t* row_prefix,
                               const int64_t* file_offsets, int32_t files_per_frame, float* x,
                               float* y, float* intensity, int32_t* gain_out,
                               int32_t* point_frame_out, const uint32_t* entries,
                               void* stream) {
  rpt::clear_error();
  return rpt::polar_write(echo, echo_dtype, n_files, rows, bins, scale, cos_t, sin_t, gain,
                          threshold, stride, row_prefix, file_offsets, files_per_frame, x, y,
                          intensity, gain_out, point_frame_out, rpt::as_stream(stream),
                          entries);
}

int32_t rpt_frame_times(const int32_t* point_frame, int64_t n, const int64_t* frame_ids,
                        float* times_out, void* stream) {
  rpt::clear_error();
  return rpt::frame_times(point_frame, n, frame_ids, times_out, rpt::as_stream(stream));
}

int32_t rpt_sweep_to_points(const float* intensities, const float* ranges, const float* cos_t,
                            const float* sin_t, int32_t rows, int32_t bins, float threshold,
                            int32_t stride, float* x, float* y, float* z, int64_t capacity,
                            int64_t* n_out_host, void* stream) {
  rpt::clear_error();
  return rpt::sweep_to_points(intensities, ranges, cos_t, sin_t, rows, bins, threshold, stride,
                              x, y, z, capacity, n_out_host, rpt::as_stream(stream));
}

int32_t rpt_polar_to_cartesian(const float* cos_t, const float* sin_t, const float* ranges,
                               int64_t rows, int64_t bins, float* x, float* y, void* stream) {
  rpt::clear_error();
  return rpt::polar_to_cartesian(cos_t, sin_t, ranges, rows, bins, x, y,
                                 rpt::as_stream(stream));
}

int32_t rpt_bounds_xy(const float* x, const float* y, int64_t n, float* out4_host,
                      void* stream) {
  rpt::clear_error();
  return rpt::bounds_xy(x, y, n, out4_host, rpt::as_stream(stream));
}

int32_t rpt_land_grid(const float* x, const float* y, const float* intensity, int64_t n,
                      const double* x_edges, int32_t nxe, const double* y_edges, int32_t nye,
                      int32_t* count_grid, double* intensity_grid, void* stream) {
  rpt::clear_error();
  return rpt::land_grid(x, y, intensity, n, x_edges, nxe, y_edges, nye, count_grid,
                        intensity_grid, rpt::as_stream(stream));
}

int32_t rpt_land_mask(const int32_t* count_grid, const double* intensity_grid, int64_t cells,
                      int64_t num_frames, double persistence_threshold, double min_intensity,
                      uint8_t* land_mask, int64_t* land_cells_host, void* stream) {
  rpt::clear_error();
  return rpt::land_mask(count_grid, intensity_grid, cells, num_frames, persistence_threshold,
                        min_intensity, land_mask, land_cells_host, rpt::as_stream(stream));
}

int32_t rpt_land_filter(const float* x, const float* y, const float* intensity,
                        const int32_t* gain, const int32_t* point_frame, int64_t n,
                        const int64_t* frame_offsets, int32_t n_frames, const double* x_edges,
                        int32_t nxe, const double* y_edges, int32_t nye,
                        const uint8_t* land_mask, float* x_out, float* y_out,
                        float* intensity_out, int32_t* gain_out, int32_t* point_frame_out,
                        int64_t* new_frame_offsets, int64_t* n_kept_host, void* stream) {
  rpt::clear_error();
  if (n >= (int64_t(1) << 31) - 1) {  // int32 kept positions
    rpt::set_error("rpt_land_filter: n=%lld exceeds the int32 index space", (long long)n);
    return RPT_ENOTSUP;
  }
  return rpt::land_filter(x, y, intensity, gain, point_frame, n, frame_offsets, n_frames,
                          x_edges, nxe, y_edges, nye, land_mask, x_out, y_out, intensity_out,
                          gain_out, point_frame_out, new_frame_offsets, n_kept_host,
                          rpt::as_stream(stream));
}

int32_t rpt_infer_time_from_colors(const uint8_t* colors, int64_t n, const float* palette,
                                   int32_t n_pal, float* times_out, void* stream) {
  rpt::clear_error();
  return rpt::infer_time_from_colors(colors, n, palette, n_pal, times_out,
                                     rpt::as_stream(stream));
}

int32_t rpt_cluster_summaries(const int32_t* labels, const float* x, const float* y,
                              const float* intensity, const int32_t* point_frame, int64_t n,
                              int32_t n_frames, int32_t n_clusters, int32_t* seg_frame,
                              int32_t* seg_label, int64_t* seg_count, int64_t* seg_first,
                              float* seg_cx, float* seg_cy, float* seg_mean_i,
                              int64_t* frame_first_noise, int64_t* n_segments_host,
                              void* stream) {
  rpt::clear_error();
  if (n >= (int64_t(1) << 31) - 1) {  // int32 segment positions
    rpt::set_error("rpt_cluster_summaries: n=%lld exceeds the int32 index space", (long long)n);
    return RPT_ENOTSUP;
  }
  return rpt::cluster_summaries(labels, x, y, intensity, point_frame, n, n_frames, n_clusters,
                                seg_frame, seg_label, seg_count, seg_first, seg_cx, seg_cy,
                                seg_mean_i, frame_first_noise, n_segments_host,
                                rpt::as_stream(stream));
}

int32_t rpt_synth_echo(const rpt_synth_params* p, int64_t frame0, int64_t n_frames,
                       const float* cos_t, const float* sin_t, const uint32_t* clutter_thresh,
                       const float* targets, const int32_t* target_rows,
                       const int32_t* target_bins, uint8_t* echo, void* stream) {
  rpt::clear_error();
  return rpt::synth_echo(p, frame0, n_frames, cos_t, sin_t, clutter_thresh, targets,
                         target_rows, target_bins, echo, rpt::as_stream(stream));
}

}  // extern "C"
