/*
 * rpt.h — C-ABI of librpt.so, the MI355X-native (gfx950) ST-DBSCAN + tracking engine.
 *
 * Every entry point takes plain pointers, sizes and a hipStream_t passed as void*.
 * Device pointers are marked (dev), host pointers (host). All device work is
 * enqueued on `stream`; calls that must return a size to the host synchronise that
 * stream and say so. Status codes are RPT_* below; the message of the last failure on
 * the calling thread is rpt_last_error(). No C++ exception crosses this boundary.
 *
 * Reference interface each entry replaces (paths relative to the reference repo root):
 *   rpt_polar_count/rpt_polar_write   load_radar_csv  PointCloudWork/4_temporal_object_tracker.py:184-232
 *                                     + concatenation build_frame :312-352
 *                                     (package form radar_pipeline/core/transforms.py:37-79)
 *   rpt_polar_to_cartesian           radar_pipeline/core/transforms.py:13-34
 *   rpt_bounds_xy / rpt_land_grid /  build_occupancy_grid :359-391, identify_land_cells :394-410,
 *   rpt_land_mask / rpt_land_filter  filter_land_from_frame :413-436
 *   rpt_stdbscan                     st_dbscan  PointCloudWork/3_stdbscan_point_clouds.py:101-136,
 *                                     radar_pipeline/processors/clustering.py:49-115,
 *                                     the labelling half of 4_temporal_object_tracker.py:443-506
 *   rpt_infer_time_from_colors       radar_pipeline/processors/clustering.py:17-46, 3_stdbscan...py:91-98
 *   rpt_cluster_summaries            per-frame Cluster extraction 4_temporal_object_tracker.py:508-536
 *   rpt_set_order                    CPython set(frame_labels) iteration order :519
 *   rpt_lsap                         scipy.optimize.linear_sum_assignment as called at :590
 *   rpt_tracker_*                    ObjectTracker :543-688 (+ TrackedObject :111-140)
 *   rpt_stack_*                      the compute stages of run_pipeline :941-991 (K1 .. K9) in one call
 *   rpt_shard_*                      the same stages over a frame range of a multi-GPU stack
 *   rpt_fuse_gains_max               fuse_gains_max PointCloudWork/5_gain_fusion_ply_builder.py:222-273
 *   rpt_csv_*                        pd.read_csv + fillna/to_numpy of load_radar_csv :189-211
 *   rpt_synth_echo                   (bench/test input generator; no reference counterpart)
 */
#ifndef RPT_H
#define RPT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RPT_OK 0
#define RPT_EINVAL 1      /* bad argument (maps to ValueError)                           */
#define RPT_ENOMEM 2      /* device allocation failed                                     */
#define RPT_EHIP 3        /* HIP runtime error, or a device-side fault reported at a readback */
#define RPT_EEMPTY 4      /* empty input where the reference raises (sklearn ValueError)  */
#define RPT_ENOTSUP 5     /* input outside what the device path implements                */
#define RPT_ENONFINITE 6  /* NaN/inf coordinates (sklearn check_array raises ValueError)  */

#define RPT_ECHO_F32 0
#define RPT_ECHO_U8 1

/* ---- library ---------------------------------------------------------------------- */
int32_t rpt_version(void);               /* major*10000 + minor*100 + patch            */
const char* rpt_last_error(void);        /* thread-local; "" when none                 */
int32_t rpt_device_count(void);          /* hipGetDeviceCount; 0 when no GPU           */
int32_t rpt_set_device(int32_t device);  /* hipSetDevice                               */
/* Frees the current device's scratch arenas and scan look-back states (every stream's; they are
 * re-created on next use).  The per-stream ST-DBSCAN working sets and rpt_stack / rpt_dbscan
 * handles are not touched.  Only valid while NO library call is in flight on this device, from
 * any thread: a scan launched concurrently would run on freed memory. */
void rpt_release_scratch(void);

/* Device exclusive prefix sum (the primitive under K1's offsets, the land compaction, the grid
 * build and the summaries): out[i] = sum of in[0..i) for i < n; with_total != 0 also writes the
 * grand total at out[n] (out then holds n+1 values).  in == out allowed for equal dtypes.
 * Single pass (decoupled look-back), no memset, stream-ordered.  Values are non-negative and
 * their total is below 2^46.  Dtypes: RPT_I32->RPT_I32, RPT_I32->RPT_I64, RPT_I64->RPT_I64. */
enum { RPT_I32 = 0, RPT_I64 = 1 };
int32_t rpt_exclusive_scan(const void* in, int32_t in_dtype, int64_t n, void* out,
                           int32_t out_dtype, int32_t with_total, void* stream);

/* ---- K1: polar -> Cartesian scatter ---------------------------------------------
 * A batch of sweeps ("files"), each echo[rows][bins] (f32 or u8), concatenated in file
 * order (= ascending gain inside a frame, as build_frame does).  Pass 1 counts kept
 * points (echo > threshold, strictly) and writes the exclusive per-file output offsets
 * file_offsets[n_files+1] (dev, int64): file f contributes ceil(kept_f / stride) points.
 * Pass 2 writes x, y, intensity (f32) and gain_out (i32, the file's gain) for every
 * kept element whose row-major rank inside its file is a multiple of `stride`.
 *   x = ((scale[row] / bins) * bin) * cos_t[row]   (f32, each op rounded, no FMA)
 * cos_t/sin_t are the per-row float32 np.cos/np.sin values of the reference (input). */
int32_t rpt_polar_count(const void* echo, int32_t echo_dtype, int64_t n_files, int32_t rows,
                        int32_t bins, float threshold, int32_t stride,
                        int64_t* row_prefix /*dev [n_files*rows+1], work data for
                                              rpt_polar_write: kept before each row, or before
                                              each group of 4 rows for u8 sweeps of 1024 bins*/,
                        int64_t* file_offsets /*dev [n_files+1]*/,
                        int64_t* total_host /*host, may be NULL: then no sync*/, void* stream);
int32_t rpt_polar_write(const void* echo, int32_t echo_dtype, int64_t n_files, int32_t rows,
                        int32_t bins, const float* scale /*dev [n_files*rows]*/,
                        const float* cos_t /*dev [n_files*rows]*/, const float* sin_t,
                        const int32_t* gain /*dev [n_files]*/, float threshold, int32_t stride,
                        const int64_t* row_prefix /*dev, from rpt_polar_count*/,
                        const int64_t* file_offsets /*dev*/, int32_t files_per_frame,
                        float* x, float* y, float* intensity, int32_t* gain_out /*nullable*/,
                        int32_t* point_frame_out /*nullable: file / files_per_frame*/,
                        void* stream);
/* Same two passes with the kept samples staged between them (u8 sweeps of 1024 bins with 16-B
 * aligned rows; other sweeps ignore the buffer): for every group of 4 rows that keeps at most 128
 * samples the count pass stores them as 32-bit (row, bin, sample) entries in the group's slot of
 * entries (dev, rpt_polar_stage_words(n_files, rows) words), and the write pass reads those
 * instead of the group's echo -- one read of the echo for sparse sweeps (what rpt_stack_run
 * does).  Same outputs as rpt_polar_count + rpt_polar_write. */
int64_t rpt_polar_stage_words(int64_t n_files, int32_t rows);
int32_t rpt_polar_count_staged(const void* echo, int32_t echo_dtype, int64_t n_files,
                               int32_t rows, int32_t bins, float threshold, int32_t stride,
                               int64_t* row_prefix, int64_t* file_offsets, int64_t* total_host,
                               uint32_t* entries /*dev*/, void* stream);
int32_t rpt_polar_write_staged(const void* echo, int32_t echo_dtype, int64_t n_files,
                               int32_t rows, int32_t bins, const float* scale, const float* cos_t,
                               const float* sin_t, const int32_t* gain, float threshold,
                               int32_t stride, const int64_t* row_prefix,
                               const int64_t* file_offsets, int32_t files_per_frame, float* x,
                               float* y, float* intensity, int32_t* gain_out,
                               int32_t* point_frame_out, const uint32_t* entries /*dev*/,
                               void* stream);
/* times_out[i] = (float)frame_ids[point_frame[i]] (frame_ids dev int64 per frame slot; NULL =
 * the slot itself): the float32 frame_ids stack of 4_temporal_object_tracker.py:460-467. */
int32_t rpt_frame_times(const int32_t* point_frame, int64_t n, const int64_t* frame_ids,
                        float* times_out, void* stream);
/* Generic form for radar_pipeline.sweep_to_point_cloud: ranges is a full [rows][bins] f32
 * matrix, intensities f32 [rows][bins]; one sweep.  Outputs x,y,z(=intensity). */
int32_t rpt_sweep_to_points(const float* intensities, const float* ranges, const float* cos_t,
                            const float* sin_t, int32_t rows, int32_t bins, float threshold,
                            int32_t stride, float* x, float* y, float* z, int64_t capacity,
                            int64_t* n_out_host /*sync*/, void* stream);
/* x = ranges * cos_t[:,None], y = ranges * sin_t[:,None]  (transforms.py:13-34) */
int32_t rpt_polar_to_cartesian(const float* cos_t, const float* sin_t, const float* ranges,
                               int64_t rows, int64_t bins, float* x, float* y, void* stream);

/* ---- K2/K3: land filter ------------------------------------------------------------ */
/* out4_host = {min x, max x, min y, max y} (float32, exact); synchronises. */
int32_t rpt_bounds_xy(const float* x, const float* y, int64_t n, float* out4_host, void* stream);
/* count_grid[(nxe-1)*(nye-1)] int32 and intensity_grid f64 are zeroed then accumulated
 * with numpy.digitize semantics against the given float64 edges (np.add.at). */
int32_t rpt_land_grid(const float* x, const float* y, const float* intensity, int64_t n,
                      const double* x_edges /*dev*/, int32_t nxe, const double* y_edges,
                      int32_t nye, int32_t* count_grid, double* intensity_grid, void* stream);
int32_t rpt_land_mask(const int32_t* count_grid, const double* intensity_grid, int64_t cells,
                      int64_t num_frames, double persistence_threshold, double min_intensity,
                      uint8_t* land_mask /*dev [cells]*/, int64_t* land_cells_host /*sync*/,
                      void* stream);
/* Stable compaction of the points NOT on land (n < 2^31 - 1, else RPT_ENOTSUP: int32 positions).  point_frame[n] (dev, i32) is the frame slot
 * of each point (non-decreasing), frame_offsets[n_frames+1] (dev, int64) the frame starts;
 * new_frame_offsets[n_frames+1] (dev) receives the starts of the kept points.
 * *n_kept_host (sync). */
int32_t rpt_land_filter(const float* x, const float* y, const float* intensity,
                        const int32_t* gain, const int32_t* point_frame, int64_t n,
                        const int64_t* frame_offsets, int32_t n_frames, const double* x_edges,
                        int32_t nxe, const double* y_edges, int32_t nye,
                        const uint8_t* land_mask, float* x_out, float* y_out,
                        float* intensity_out, int32_t* gain_out, int32_t* point_frame_out,
                        int64_t* new_frame_offsets, int64_t* n_kept_host, void* stream);

/* ---- K4-K8: ST-DBSCAN ------------------------------------------------------------------
 * coords: dim (2 or 3) float32 component pointers sharing `stride` (elements between
 * consecutive points: 1 for SoA, dim for an (N,dim) row-major array).  times float32.
 * Labels (dev, int32 [n]) are bit-identical to the reference BFS: cluster ids ascend with
 * each cluster's minimum core-point index, border points take the minimum adjacent id,
 * noise is -1.  Neighbour test: float64 d2 = sum_k (x_k,i - x_k,j)^2 (left to right,
 * each op rounded) <= eps_space^2, and float32 |t_i - t_j| <= float32(eps_time).
 * Synchronises once (grid bounds). */
typedef struct rpt_stdbscan_stats {
  int64_t n_points;
  int64_t n_core;
  int32_t n_clusters;
  int32_t grid_dims[4];   /* nx, ny, nz (1 for dim 2), nt */
  int64_t grid_cells;
  double ms_bounds, ms_grid, ms_core, ms_union, ms_label; /* filled when timing != 0 */
  int32_t timing;         /* in: 1 = record per-stage times with hipEvents             */
} rpt_stdbscan_stats;
int32_t rpt_stdbscan(const float* x, const float* y, const float* z, int64_t stride,
                     const float* times, int64_t n, double eps_space, double eps_time,
                     int32_t min_samples, int32_t* labels, rpt_stdbscan_stats* stats,
                     void* stream);
/* Denoise variant (replaces st_dbscan of PointCloudWorkF/stdbscan_denoising_pipeline.py:264-369;
 * 2-D, x / y / times dev float32 [n]): core = >= min_samples neighbours (itself included, same
 * test as rpt_stdbscan) spanning >= min_frames distinct int32(times) frames; clusters numbered by
 * their minimum core index; a non-core point takes the smallest cluster m adjacent to it through a
 * core point with (its index > m, or it is a neighbour of core point m) -- the FIFO expansion's
 * result, :340-367.  n == 0 is not an error (no labels written).  RPT_ENOTSUP when
 * eps_time > 30 with min_frames > 256 (the distinct-frame list of a wave).  Synchronises. */
/* pandas DataFrame.groupby(labels).mean() of float32 x / y / intensity columns (pandas 2.x
 * group_mean: float32 Kahan-compensated sum in row order, / (float)count), for labels in
 * [0, n_labels) (noise -1 and labels >= n_labels ignored): count (dev int64) and the three means
 * (dev float32), each [n_labels]; the cluster table of stdbscan_denoising_pipeline.py:997-1012.
 * Synchronises. */
int32_t rpt_label_means(const int32_t* labels, const float* x, const float* y,
                        const float* intensity, int64_t n, int64_t n_labels, int64_t* count,
                        float* mean_x, float* mean_y, float* mean_intensity, void* stream);
int32_t rpt_stdbscan_denoise(const float* x, const float* y, const float* times, int64_t n,
                             double eps_space, double eps_time, int32_t min_samples,
                             int32_t min_frames, int32_t* labels, rpt_stdbscan_stats* stats,
                             void* stream);

/* ---- phased ST-DBSCAN (frame-sharded multi-GPU) -------------------------------------
 * The fused rpt_stdbscan split into phases so ranks can exchange halo data between them:
 * build (bounds + grid, 1 sync) -> core (flags, optionally copied out in original order) ->
 * set_core (overwrite flags, e.g. halo points with their owner's) -> components (comp[i] = min
 * original index of i's core component, -1 for non-core) -> labels_global (ids from global
 * representatives).  The handle owns its device memory. */
typedef struct rpt_dbscan rpt_dbscan;
rpt_dbscan* rpt_dbscan_create(void);
void rpt_dbscan_destroy(rpt_dbscan* h);
int32_t rpt_dbscan_build(rpt_dbscan* h, const float* x, const float* y, const float* z,
                         int64_t stride, const float* times, int64_t n, double eps_space,
                         double eps_time, int32_t min_samples, void* stream);
int32_t rpt_dbscan_core(rpt_dbscan* h, uint8_t* core_out /*dev [n] or NULL*/, void* stream);
int32_t rpt_dbscan_set_core(rpt_dbscan* h, const uint8_t* core_in /*dev [n]*/, void* stream);
int32_t rpt_dbscan_components(rpt_dbscan* h, int32_t* comp_out /*dev [n]*/, void* stream);
/* rep[i] (dev int64 [n]): global representative of core point i (-1 otherwise); reps_sorted
 * (dev int64 [n_reps]) all representatives ascending; label = rank of the representative;
 * non-core points take the smallest adjacent representative (reference border rule). */
int32_t rpt_dbscan_labels_global(rpt_dbscan* h, const int64_t* rep, const int64_t* reps_sorted,
                                 int64_t n_reps, int32_t* labels, void* stream);
/* rep_out[i] = map(comp[i] + base) for comp[i] >= 0 (map = sorted keys -> vals, identity when
 * absent), -1 otherwise. */
int32_t rpt_remap_components(const int32_t* comp, int64_t n, int64_t base, const int64_t* keys,
                             const int64_t* vals, int64_t n_keys, int64_t* rep_out,
                             void* stream);
/* Global indices g = base + i, i in [lo, hi), with rep[i] == g, ascending; *count_host (sync). */
int32_t rpt_select_roots(const int64_t* rep, int64_t base, int64_t lo, int64_t hi,
                         int64_t* out /*dev, capacity hi-lo*/, int64_t* count_host,
                         void* stream);

/* nearest palette colour index (first minimum) as float32: colors u8 [n][3],
 * palette f32 [n_pal][3] in ascending-gain order. */
int32_t rpt_infer_time_from_colors(const uint8_t* colors, int64_t n, const float* palette,
                                   int32_t n_pal, float* times_out, void* stream);

/* ---- max-intensity gain fusion (5_gain_fusion_ply_builder.py fuse_gains_max :222-273) ------
 * Points x, y, intensity (dev, float32 [n], intensities > 0: the loader's threshold) on a
 * grid_resolution grid anchored at the float32 minima: per cell the maximum intensity; occupied
 * cells in np.where(valid.T) order (y-major, then x) as float64 cell centres
 * (x_min + ix * res) + res / 2 and float32 maxima.  Outputs (dev) need capacity n (one cell per
 * point at most).  *n_out_host: the cell count (sync).  n = 0 gives 0 cells. */
int32_t rpt_fuse_gains_max(const float* x, const float* y, const float* intensity, int64_t n,
                           double grid_resolution, double* out_x, double* out_y,
                           float* out_intensity, int64_t* n_out_host, void* stream);

/* ---- K9: per-(frame, label) cluster summaries ---------------------------------------
 * point_frame[n] (dev, i32, non-decreasing frame slot per point), labels[n] from
 * rpt_stdbscan.  Segment s = one (frame, label>=0) pair; the order of segments is unspecified
 * (frame-major when n_clusters < 8192 and frames average <= 2^18 points, label-major otherwise):
 * rpt_order_clusters buckets them.
 * centroid = sequential float32 sum in point order / count (np.mean axis 0);
 * mean intensity = numpy 1-D float32 mean (pairwise sums over 8192-element chunks).
 * frame_first_noise[n_frames] (dev, int64) = first point index of label -1 per frame, or -1.
 * *n_segments_host (sync).  Output arrays have capacity n.  n < 2^31 - 1 (int32 positions),
 * else RPT_ENOTSUP. */
int32_t rpt_cluster_summaries(const int32_t* labels, const float* x, const float* y,
                              const float* intensity, const int32_t* point_frame, int64_t n,
                              int32_t n_frames, int32_t n_clusters, int32_t* seg_frame,
                              int32_t* seg_label, int64_t* seg_count, int64_t* seg_first,
                              float* seg_cx, float* seg_cy, float* seg_mean_i,
                              int64_t* frame_first_noise, int64_t* n_segments_host,
                              void* stream);

/* ---- native stack driver (single device) -----------------------------------------------
 * The compute stages of run_pipeline (PointCloudWork/4_temporal_object_tracker.py:941-991) over
 * a stack of sweeps in device memory, in ONE call: K1 (rpt_polar_count/write over
 * n_frames*files_per_frame files, ascending gain inside a frame) -> land filter when enabled and
 * more than 10 frames are non-empty (:954; grid edges = np.arange(min, max + res, res) as numpy
 * evaluates it) -> rpt_stdbscan of (x, y) with times = frame slot -> rpt_cluster_summaries.
 * Equivalent to calling those entry points in sequence; the size readbacks they need happen
 * inside (pinned memory).  Synchronises `stream`.  No built frame at all gives an empty result
 * (st_dbscan(frames) returns {}, :463-464); built frames whose points the land filter removed
 * entirely return RPT_EEMPTY (BallTree on 0 samples: sklearn's ValueError).  The handle owns its device buffers (grow-only); results stay valid
 * until the next run on the handle. */
/* host: the land-grid edges np.arange(lo, hi + res, res) for float32 lo/hi, as numpy 2.x
 * evaluates it (float32 stop and length, float64 values); returns the length, writes up to cap */
int32_t rpt_arange_edges(float lo, float hi, double res, double* out, int32_t cap);
typedef struct rpt_stack rpt_stack;
typedef struct rpt_stack_params {
  int32_t n_frames, files_per_frame, rows, bins, echo_dtype;
  float threshold;              /* INTENSITY_THRESHOLD (strict >) */
  int32_t stride;               /* POINT_STRIDE */
  int32_t land_filter;          /* 0 = --no-land-filter */
  double land_resolution;       /* LAND_GRID_RESOLUTION 5.0 */
  double land_persistence;      /* LAND_PERSISTENCE_THRESHOLD 0.8 */
  double land_min_intensity;    /* LAND_MIN_INTENSITY 100 */
  double eps_space, eps_time;
  int32_t min_samples;
  int32_t timing;               /* 1 = per-stage hipEvent times in the result */
} rpt_stack_params;
typedef struct rpt_stack_result {
  int64_t n_points;             /* K1 points ("Total points", :950-951) */
  int64_t n_clustered;          /* points entering ST-DBSCAN */
  int64_t n_land_cells;
  int64_t n_segments;           /* (frame, label >= 0) pairs */
  int32_t n_built;              /* frames with at least one K1 point */
  int32_t n_clusters;
  double ms_polar, ms_land, ms_stdbscan, ms_summaries;  /* timing != 0 */
  rpt_stdbscan_stats dbscan;
} rpt_stack_result;
rpt_stack* rpt_stack_create(void);
void rpt_stack_destroy(rpt_stack* h);
/* K1 turns for several handles in flight on one GPU (one stream each): runs of handles that share
 * a gate enqueue their K1 (count + write) one at a time, in the order they reach it, each behind
 * the previous one on the device -- the HBM-bound K1 passes of concurrent stacks never coincide
 * and always overlap other stacks' latency-bound stages.  NULL detaches.  The gate must outlive
 * every run of the handles attached to it. */
typedef struct rpt_k1_gate rpt_k1_gate;
rpt_k1_gate* rpt_k1_gate_create(void);
void rpt_k1_gate_destroy(rpt_k1_gate* g);
int32_t rpt_stack_set_k1_gate(rpt_stack* h, rpt_k1_gate* g);
int32_t rpt_stack_run(rpt_stack* h, const rpt_stack_params* params, const void* echo /*dev*/,
                      const float* scale /*dev [files*rows]*/, const float* cos_t,
                      const float* sin_t, const int32_t* gain /*dev [files], nullable*/,
                      rpt_stack_result* result /*host*/, void* stream);
/* host [n_frames+1]: which 0 = K1 frame offsets, 1 = offsets of the clustered points */
int32_t rpt_stack_frame_offsets(const rpt_stack* h, int32_t which, int64_t* out);
/* host copies of the last run's segments (rpt_cluster_summaries layout; each nullable) and
 * frame_first_noise [n_frames] */
int32_t rpt_stack_segments(const rpt_stack* h, int32_t* frame, int32_t* label, int64_t* count,
                           int64_t* first, float* cx, float* cy, float* mean_i,
                           int64_t* frame_first_noise);
/* device copies (each nullable, [n_clustered]) of the clustered points and their labels; gain
 * only after a run given a gain table (RPT_EINVAL otherwise: without one the per-point gains
 * are not written -- 8 B per point less K1 and land traffic) */
int32_t rpt_stack_points(const rpt_stack* h, float* x, float* y, float* intensity,
                         int32_t* gain, int32_t* point_frame, int32_t* labels, void* stream);
/* core flags (dev u8 [n_clustered], 1 = core) of the last run's clustered points, in the order
 * of rpt_stack_points: K5's result, for full-size invariant checks.  Call on the stream of that
 * run, before another ST-DBSCAN runs on it (the flags live in that stream's ST-DBSCAN state). */
int32_t rpt_stack_core_flags(const rpt_stack* h, uint8_t* core, void* stream);
/* ---- frame-sharded multi-GPU driver ----------------------------------------
 * One rank's phases of ONE global stack whose contiguous frame ranges are spread over ranks
 * (replaces the whole-stack st_dbscan(frames) of 4_temporal_object_tracker.py:466-506 when the
 * stack is split over GPUs); the caller runs the collectives between phases (rpt/dist.py:
 * torch.distributed over RCCL / gloo) on buffers it owns.  Results equal rpt_stack_run over the
 * whole stack.  Per step (host waits marked *):
 *   polar* -> [all_gather info*] -> land_grid -> [all_reduce grid] -> halo ->
 *   [P2P x/y/t, capacities = the neighbours' n_head_k1 / n_tail_k1] -> window* ->
 *   [P2P core flags] -> link -> [P2P component ids] -> pairs -> [all_gather pairs] ->
 *   finish -> [all_gather packed results*] -> rpt_shard_host_stage on rank 0.
 * Point ids are (rank << 40) | own index; labels are numbered per rank and mapped to the global
 * numbering with the representative tables of the packed results. */
typedef struct rpt_shard rpt_shard;
typedef struct rpt_shard_info {
  int64_t n_points;        /* K1 points of this rank's frames */
  int32_t n_built;         /* of them, frames with at least one point */
  int32_t halo_frames;     /* hf = min(floor(eps_time), n_frames), 0 if eps_time is not >= 0 */
  float bounds[4];         /* min x, max x, min y, max y of the K1 points (+inf/-inf: none) */
  int64_t n_head_k1;       /* K1 points of the first hf frames (the prev rank's halo capacity) */
  int64_t n_tail_k1;       /* K1 points of the last hf frames (the next rank's halo capacity) */
  /* set by rpt_shard_window: */
  int64_t n_kept;          /* own points after the land filter */
  int64_t n_head, n_tail;  /* own kept points of the first / last hf frames */
  int64_t n_prev, n_next;  /* halo points received from rank - 1 / rank + 1 */
  int64_t n_land_cells;
} rpt_shard_info;
rpt_shard* rpt_shard_create(void);
void rpt_shard_destroy(rpt_shard* h);
/* K1 over the rank's frames (rpt_stack_params as for rpt_stack_run) + bounds; synchronises */
int32_t rpt_shard_polar(rpt_shard* h, const rpt_stack_params* params, const void* echo,
                        const float* scale, const float* cos_t, const float* sin_t,
                        const int32_t* gain, rpt_shard_info* info, void* stream);
/* land-grid cells for the GLOBAL bounds (host; (len(x edges)-1) * (len(y edges)-1), 0 if < 2) */
int64_t rpt_shard_land_cells(const float* global_bounds, double resolution);
/* this rank's land grid over the global edges into grid (dev float64 [2*cells]: counts | sums) */
int32_t rpt_shard_land_grid(rpt_shard* h, const float* global_bounds, double* grid, int64_t cells,
                            void* stream);
/* land mask from the all-reduced grid (NULL: no land filter) with the GLOBAL built-frame count,
 * compaction, and the own first / last hf frames packed for the neighbours: send_prev / send_next
 * (dev int32 [4 + 3 * n_head_k1] / [4 + 3 * n_tail_k1], nullable) = {count, own kept total lo,
 * hi, 0} then x, y, t (float32 bits; t = frame0 + frame slot) at offsets 4, 4 + cap, 4 + 2 cap.
 * recv_cap_prev / recv_cap_next: the capacities of the halo buffers this rank will receive (the
 * same values rpt_shard_window gets): with the land filter the compaction writes the kept points
 * straight into the window at that offset.  No sync. */
int32_t rpt_shard_halo(rpt_shard* h, const double* grid, int64_t cells, int32_t n_built_global,
                       int32_t rank, int64_t frame0, int32_t* send_prev, int32_t* send_next,
                       int64_t recv_cap_prev, int64_t recv_cap_next, void* stream);
/* the window [prev halo | own | next halo] from the received halo buffers (capacities as sent;
 * NULL / 0 at the ends of the rank chain), its grid build and K5 core flags; flags_prev /
 * flags_next (dev u8, capacity n_head_k1 / n_tail_k1) receive the own edge points' flags for the
 * neighbours; the window counts in info.  Synchronises once (counts + grid bounds). */
int32_t rpt_shard_window(rpt_shard* h, const int32_t* recv_prev, int64_t cap_prev,
                         const int32_t* recv_next, int64_t cap_next, uint8_t* flags_prev,
                         uint8_t* flags_next, rpt_shard_info* info, void* stream);
/* duration of the last core-flag pass (params.timing != 0; synchronises), -1 if not timed */
double rpt_shard_core_ms(rpt_shard* h);
/* halo flags from their owners (dev u8 [n_prev] / [n_next]), components; comp_prev / comp_next
 * (dev int64 [n_head] / [n_tail], nullable) receive the own edge points' component ids (-1: not
 * core).  No sync. */
int32_t rpt_shard_link(rpt_shard* h, const uint8_t* flags_prev, const uint8_t* flags_next,
                       int64_t* comp_prev, int64_t* comp_next, void* stream);
/* distinct equivalence pairs between the halo points' components and their owners' ids
 * (owner_prev / owner_next, dev int64 [n_prev] / [n_next]): pairs (dev int64 [1 + 2 cap]) =
 * the full pair count (may exceed cap), then (min, max) pairs.  No sync. */
int32_t rpt_shard_pairs(rpt_shard* h, const int64_t* owner_prev, const int64_t* owner_next,
                        int64_t* pairs, int64_t cap, void* stream);
/* host: union of equivalence pairs [n_pairs][2] -> sorted distinct ids (keys_out) and each
 * id's class minimum (reps_out), up to cap; returns the number of ids */
int64_t rpt_merge_equivalences(const int64_t* pairs, int64_t n_pairs, int64_t* keys_out,
                               int64_t* reps_out, int64_t cap);
/* equivalence merge of every rank's pairs (gathered_pairs: dev int64 [world][row_words], the
 * all_gather of rpt_shard_pairs' buffers; or NULL with the host merge keys_host / vals_host
 * [n_keys]), representatives, labels, K9 of the own points, and everything rank 0 needs packed
 * into out (dev int64 [out_cap]): [magic, S, n_reps, flags, words, F, frame0, kept] [built F]
 * [first noise F] [count S] [first S] [frame << 32 | local label S] [cx | cy << 32 S] [mi S]
 * [reps n_reps]; flags 1: some rank's pairs exceeded their capacity, 2: too many ids for the
 * device merge (merge on the host), 4: out_cap too small (words = the size needed); S = -1: a
 * frame held more labels than K9's frame sort takes (force_radix).  own_pairs: this rank's
 * rpt_shard_pairs buffer.  No sync. */
int32_t rpt_shard_finish(rpt_shard* h, const int64_t* gathered_pairs, int32_t world,
                         int64_t row_words, const int64_t* own_pairs, const int64_t* keys_host,
                         const int64_t* vals_host, int64_t n_keys, int32_t force_radix,
                         int64_t* out, int64_t out_cap, void* stream);
/* labels (dev int32 [n_kept]) of the own kept points of the last finish, through
 * local_to_global (dev int32 [n_reps], from rpt_shard_host_stage); no sync */
int32_t rpt_shard_labels(const rpt_shard* h, const int32_t* local_to_global, int64_t n_reps,
                         int32_t* out, void* stream);
int32_t rpt_shard_frame_offsets(const rpt_shard* h, int32_t which, int64_t* out);
/* ids the device equivalence merge of rpt_shard_finish takes (default and maximum 8192); a step
 * whose gathered pairs hold more is merged on the host (flag 2, rpt_merge_equivalences).  Lower
 * limits (0: always the host merge) exist so tests reach that path. */
int32_t rpt_shard_set_merge_limit(rpt_shard* h, int32_t max_ids);
/* device copies of the own kept points of the last step (each output nullable, dev [n_kept]):
 * x, y, intensity, frame slot, and (after rpt_shard_window) their K5 core flags -- for
 * full-size invariant checks, on the stream of that step, before the handle's next step */
int32_t rpt_shard_points(const rpt_shard* h, float* x, float* y, float* intensity,
                         int32_t* point_frame, uint8_t* core, void* stream);
/* host, over the all-gathered packed results (host int64 [world][row_words]): sizes[4] = total
 * segments, built frames, frames, clusters (distinct representatives) */
int32_t rpt_shard_gathered_sizes(const int64_t* gathered, int32_t world, int64_t row_words,
                                 int64_t* sizes);
struct rpt_tracker;
/* host: rank 0's stage -- the global label numbering (rank of each representative), every
 * segment (frame = global frame id), the built frame ids, per frame slot the reference cluster
 * order (frame_off [frames + 1], order [segments]: indices into the segments), and the tracker
 * (nullable) updated over the built frames; each output nullable (seg_frame NULL: only
 * local_to_global [n_reps of which_rank], the label map of one rank).  No device work. */
int32_t rpt_shard_host_stage(const int64_t* gathered, int32_t world, int64_t row_words,
                             struct rpt_tracker* trk, int32_t* seg_frame, int32_t* seg_label,
                             int64_t* seg_count, int64_t* seg_first, float* seg_cx,
                             float* seg_cy, float* seg_mi, int64_t* built_ids,
                             int64_t* frame_off, int64_t* order, int32_t* local_to_global,
                             int32_t which_rank);

/* ---- host: per-frame cluster order of the reference -----------------------------------
 * From the segments of rpt_cluster_summaries (copied to host) and frame_first_noise: for each
 * frame the segment indices in the order st_dbscan(frames) lists that frame's clusters
 * (CPython set iteration over the frame's labels inserted in first-occurrence order, -1
 * discarded).  frame_offsets_out[n_frames+1], order_out[n_segments]. */
int32_t rpt_order_clusters(int32_t n_frames, int64_t n_segments, const int32_t* seg_frame,
                           const int32_t* seg_label, const int64_t* seg_first,
                           const int64_t* frame_first_noise, int64_t* frame_offsets_out,
                           int64_t* order_out);

/* ---- host: cluster order + tracker of one stack in one call ------------------------------
 * rpt_order_clusters (frame_offsets_out, order_out as there) followed by rpt_tracker_update on
 * trk for each built slot (built_slots[n_built], strictly ascending, in [0, n_frames)) with the
 * slot's segments' seg_cx/seg_cy in that order and frame id frame_ids[slot] (NULL: the slot) --
 * the host stage of pipeline.py's order_and_track (4_temporal_object_tracker.py:519-522 then
 * :984-991).  Frames are ordered on a second thread ahead of the tracker.  trk NULL: only the
 * order.  Returns RPT_OK or an error code (the tracker's included). */
int32_t rpt_order_and_track(int32_t n_frames, int64_t n_segments, const int32_t* seg_frame,
                            const int32_t* seg_label, const int64_t* seg_first,
                            const int64_t* frame_first_noise, const float* seg_cx,
                            const float* seg_cy, int32_t n_built, const int64_t* built_slots,
                            const int64_t* frame_ids, struct rpt_tracker* trk,
                            int64_t* frame_offsets_out, int64_t* order_out);

/* ---- host: CPython set iteration order --------------------------------------------------
 * keys = the distinct labels of a frame in first-occurrence order (may include -1).
 * order_out receives the keys in the order `iter(set(keys))` yields them on CPython 3.10
 * (int hash = value, hash(-1) = -2), -1 removed (set.discard(-1)).  Returns count. */
int32_t rpt_set_order(const int32_t* keys, int32_t n, int32_t* order_out);

/* ---- host: rectangular linear sum assignment (scipy 1.15 shortest augmenting path) ----
 * cost row-major [nr][nc] float64; rows_out/cols_out receive min(nr,nc) pairs sorted by
 * row, identical to scipy.optimize.linear_sum_assignment including tie-breaking. */
int32_t rpt_lsap(const double* cost, int32_t nr, int32_t nc, int64_t* rows_out,
                 int64_t* cols_out);

/* ---- host: ObjectTracker --------------------------------------------------------------- */
typedef struct rpt_tracker rpt_tracker;
typedef struct rpt_tracker_params {
  double max_association_distance; /* 50.0 */
  int32_t max_missed_frames;        /* 10   */
  int32_t motion_history_frames;    /* 5    */
  double stationary_velocity_threshold; /* 1.0 */
} rpt_tracker_params;
typedef struct rpt_object_info {
  int64_t object_id;
  int32_t object_type;     /* 0 unknown, 1 buoy, 2 boat */
  int32_t n_positions;     /* == len(frames_seen) */
  int32_t n_velocities;
  int64_t last_seen_frame;
  double average_velocity; /* value of TrackedObject.average_velocity */
  int32_t average_velocity_is_f32; /* 1 when the reference returns np.float32 */
  int32_t color[3];
} rpt_object_info;
rpt_tracker* rpt_tracker_new(const rpt_tracker_params* params /*NULL = defaults*/);
void rpt_tracker_free(rpt_tracker* t);
/* One ObjectTracker.update(clusters, frame_id): clusters in list order. Returns the number
 * of objects after the update (len of the returned list). */
int32_t rpt_tracker_update(rpt_tracker* t, int64_t frame_id, int32_t k, const float* cx,
                           const float* cy, const int64_t* cluster_frame_id);
/* Batch driver: frames[i] has clusters [offsets[i], offsets[i+1]) already in reference
 * order; equivalent to calling rpt_tracker_update per frame. */
int32_t rpt_tracker_run(rpt_tracker* t, int32_t n_frames, const int64_t* frame_ids,
                        const int64_t* offsets, const float* cx, const float* cy);
int32_t rpt_tracker_num_objects(const rpt_tracker* t);
int32_t rpt_tracker_object_info(const rpt_tracker* t, int32_t idx, rpt_object_info* out);
/* positions (x,y f32) + frames_seen of object idx (dict order); velocities as f64 pairs
 * (exact widening of the f32 values; velocity 0 is the f64 zero).  Buffers sized from info. */
int32_t rpt_tracker_object_history(const rpt_tracker* t, int32_t idx, float* px, float* py,
                                   int64_t* frames, double* vx, double* vy);

/* ---- host: radar CSV ingest ---------------------------------------------------------------
 * The file half of load_radar_csv (PointCloudWork/4_temporal_object_tracker.py:189-211;
 * radar_pipeline/core/loaders.py:46-101): pd.read_csv(header=None, names=Status, Scale, Range,
 * Gain, Angle, Echo_0..Echo_{bins-1}, skiprows=1), echo fillna(0) -> float32, Scale/Angle ->
 * float32, parsed by n_threads host threads (<= 0: all cores), one file per task.
 * rpt_csv_count_rows: rows_out[i] = data rows of file i (blank lines skipped), -1 unreadable.
 * rpt_csv_parse_sweeps: file i -> echo + i*rows_cap*bins (u8 or f32 per echo_dtype), scale/angle
 * + i*rows_cap (float32; NaN where pandas reads NaN), gain_col[i] = the Gain value when every row
 * holds the same one, else NaN; rows past the
 * file's end are zero.  status_out[i]: 0 ok, 1 unreadable or more fields than names (read_csv
 * raises: the reference returns an empty sweep), 2 no data row (df.empty: empty sweep), 3 a value
 * that is not an integer in 0..255 with echo_dtype u8 (parse again as f32), 4 a non-numeric value
 * (the reference's to_numpy(float32) raises ValueError).
 * detail_out (nullable) [n_files][5]: {kind (0 none, 1 I/O error, 2 tokenizing error, 3
 * non-numeric value, 5 genfromtxt rows of < 5 fields), errno | expected fields | field index |
 * field count, physical line (1-based), fields seen, gain flags (bit 0 the first row's Gain is
 * NaN, bit 1 rows disagree -- NaN-aware like Series.unique())}: the parts of the exception
 * texts read_csv / to_numpy raise ("Error tokenizing data. C error: Expected E fields in line L,
 * saw S") and of int(df["Gain"].iloc[0]) / unique().
 * mode 0: read_csv as above.  mode 1: np.genfromtxt(delimiter=',', skip_header=1,
 * filling_values=0.0) first, read_csv when genfromtxt raises (rows of different field counts) --
 * the denoise loader (PointCloudWorkF/stdbscan_denoising_pipeline.py:97-119): '#' starts a
 * comment, empty or unreadable fields are 0.0, one data row is an empty sweep (status 2);
 * status 6: a field count other than 5 + bins (not supported). */
int32_t rpt_csv_count_rows(const char* const* paths, int32_t n_files, int64_t* rows_out,
                           int32_t n_threads);
int32_t rpt_csv_parse_sweeps(const char* const* paths, int32_t n_files, int32_t rows_cap,
                             int32_t bins, int32_t echo_dtype, void* echo /*host*/,
                             float* scale, float* angle, float* gain_col, int32_t* status_out,
                             int64_t* detail_out, int32_t mode, int32_t n_threads);

/* ---- synthetic input (bench / parity tests) -----------------------------------------
 * Deterministic u8 echo [n_frames][n_gains][rows][bins] from integer hashes; see
 * rpt/synth.py for the bit-identical numpy restatement.  Geometry tables come from host. */
typedef struct rpt_synth_params {
  uint64_t seed;
  int32_t rows, bins, n_gains, n_targets;
  float scale;                  /* Scale column (m) */
  uint32_t target_fill_u8;      /* target keep threshold on an 8-bit hash draw */
  uint32_t land_fill_u8;        /* land keep threshold */
  int32_t land_row0, land_row1, land_bin0; /* land sector [row0,row1) x [bin0, bins) */
} rpt_synth_params;
int32_t rpt_synth_echo(const rpt_synth_params* p, int64_t frame0, int64_t n_frames,
                       const float* cos_t /*dev [rows]*/, const float* sin_t,
                       const uint32_t* clutter_thresh /*dev [n_gains][bins]*/,
                       const float* targets /*dev [n_frames][n_targets][4]: tx,ty,r2,-*/,
                       const int32_t* target_rows /*dev [n_frames][n_targets][2] row lo/hi (incl) */,
                       const int32_t* target_bins /*dev [n_frames][n_targets][2] bin lo/hi (incl) */,
                       uint8_t* echo /*dev*/, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RPT_H */
