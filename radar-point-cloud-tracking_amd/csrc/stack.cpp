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
#include "stack_impl.h"

namespace rpt {

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

}  // namespace
}  // namespace rpt

using namespace rpt;

namespace {
// One run's K1 turn at a gate (nullable: no gate, no-op).  enter() waits for the turn and makes
// the stream wait for the previous K1; leave() records this K1's end and passes the turn (also
// on an error path, from the destructor, so no later run waits forever).
class K1Turn {
 public:
  K1Turn(rpt_k1_gate* g, hipStream_t st) : g_(g), st_(st) {}
  int32_t enter() {
    if (!g_) return RPT_OK;
    std::unique_lock<std::mutex> lk(g_->mu);
    t_ = g_->issued++;
    g_->cv.wait(lk, [&] { return g_->next == t_; });
    in_ = true;
    hipEvent_t& mine = g_->ev[t_ % rpt_k1_gate::kRing];
    if (!mine) RPT_HIP(hipEventCreateWithFlags(&mine, hipEventDisableTiming));
    if (t_ > 0) RPT_HIP(hipStreamWaitEvent(st_, g_->ev[(t_ - 1) % rpt_k1_gate::kRing], 0));
    return RPT_OK;
  }
  int32_t leave() {
    if (!g_ || !in_) return RPT_OK;
    in_ = false;
    std::lock_guard<std::mutex> lk(g_->mu);
    const hipError_t e = hipEventRecord(g_->ev[t_ % rpt_k1_gate::kRing], st_);
    g_->next = t_ + 1;
    g_->cv.notify_all();
    RPT_HIP(e);
    return RPT_OK;
  }
  ~K1Turn() { (void)leave(); }

 private:
  rpt_k1_gate* g_;
  hipStream_t st_;
  int64_t t_ = -1;
  bool in_ = false;
};
}  // namespace

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
  K1Turn k1turn(k1_gate, st);
  RPT_TRY(k1turn.enter());
  RPT_TRY(polar_count(echo, p.echo_dtype, n_files, p.rows, p.bins, p.threshold, p.stride,
                      row_prefix.p, file_off.p, nullptr, st, mk));
  RPT_HIP(hipMemcpyAsync(hfo, file_off.p, sizeof(int64_t) * (n_files + 1), hipMemcpyDeviceToHost,
                         st));
  // u8 sweeps of 1024 bins, outputs sized by an earlier run: the write is queued right behind
  // the readback (capacity-bounded) instead of after the host has seen the count; when the
  // count exceeds the capacity the buffers grow and the write runs again
  int64_t spec_cap = -1;
  // the write leaves the points' xy bounds (the land grid's edges) in k1_bnd when it takes the
  // expand path: no separate bounds pass over x and y
  bool k1_bounds = false;
  if (grouped && mk) RPT_TRY(k1_bnd.ensure((size_t)polar_bounds_words(), st));
  uint32_t* kb = (grouped && mk) ? k1_bnd.p : nullptr;
  if (grouped && x.p && y.p && v.p && g.p && pf.p) {
    spec_cap = (int64_t)std::min({x.cap, y.cap, v.cap, g.cap, pf.cap});
    if (!ev_rb) RPT_HIP(hipEventCreateWithFlags(&ev_rb, hipEventDisableTiming));
    RPT_HIP(hipEventRecord(ev_rb, st));
    RPT_TRY(polar_write_cap((const uint8_t*)echo, n_files, p.rows, p.threshold, p.stride, scale,
                            cos_t, sin_t, gain, row_prefix.p, file_off.p, G, x.p, y.p, v.p,
                            gain ? g.p : nullptr, pf.p, spec_cap, st, mk, kb, &k1_bounds));
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
                        gain ? g.p : nullptr, pf.p, st, mk, kb, &k1_bounds));
  }
  RPT_TRY(k1turn.leave());
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
    if (k1_bounds) {
      uint32_t hb[4];
      RPT_HIP(hipMemcpyAsync(hb, kb, sizeof hb, hipMemcpyDeviceToHost, st));
      RPT_TRY(wait_stream(st));
      for (int k = 0; k < 4; ++k) {
        const uint32_t u = hb[k];
        const uint32_t w = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
        std::memcpy(b4 + k, &w, 4);
      }
    } else {
      RPT_TRY(bounds_xy(x.p, y.p, N, b4, st));  // synchronises
    }
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
    // the land-cell count accumulates (int32) into the low half of an int64 slot, zeroed with
    // the grid
    RPT_TRY(scal.ensure(4, st));
    RPT_TRY(land_grid_cells(x.p, y.p, v.p, N, edges.p, nxe, edges.p + nxe, nye, land_cnt.p,
                            land_tot.p, land_cell.p, st, p.echo_dtype == RPT_ECHO_U8 ? 1 : 0,
                            reinterpret_cast<int64_t*>(scal.p)));
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

rpt_k1_gate* rpt_k1_gate_create(void) { return new rpt_k1_gate(); }

void rpt_k1_gate_destroy(rpt_k1_gate* g) { delete g; }

int32_t rpt_stack_set_k1_gate(rpt_stack* h, rpt_k1_gate* g) {
  if (!h) return RPT_EINVAL;
  h->k1_gate = g;
  return RPT_OK;
}

void rpt_stack_destroy(rpt_stack* h) { delete h; }

int32_t rpt_stack_run(rpt_stack* h, const rpt_stack_params* p, const void* echo,
                      const float* scale, const float* cos_t, const float* sin_t,
                      const int32_t* gain, rpt_stack_result* out, void* stream) {
  clear_error();
  if (!h || !p) {
    set_error("rpt_stack_run: null handle or params");
    return RPT_EINVAL;
  }
  // the run's counters from one clear of the stream's zero pool (common.h)
  RPT_TRY(zero_pool_arm(as_stream(stream)));
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

