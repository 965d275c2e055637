// Host-side sequential stage of the path: per-frame cluster order,
// Hungarian association and object state.  Replaces ObjectTracker / TrackedObject of
// PointCloudWork/4_temporal_object_tracker.py:111-140, 543-688 and the cluster ordering of
// :519-522, reproducing the reference's numerics exactly:
//
//  * cluster order in a frame = CPython 3.10 `set` iteration order of the frame's labels
//    inserted in first-occurrence order (np.int32 hash = value, hash(-1) = -2), -1 discarded;
//  * linear_sum_assignment = scipy 1.15 rectangular LSAP (shortest augmenting path, Crouse
//    2016) including its tie-breaking (remaining columns scanned in reverse order, a tie on the
//    minimum prefers an unassigned column) and the transpose for tall matrices;
//  * TrackedObject.predict_position: mean of the last 5 velocities — float64 while the initial
//    float64 zero velocity is in the window, float32 afterwards (numpy result-type promotion);
//    the cost is np.linalg.norm: float64 dot (OpenBLAS ddot: sqrt(fma(dy,dy,dx*dx))) or float32
//    dot (sdot: sqrtf(dx*dx + dy*dy), no FMA) — both measured against the reference in
//    tests/golden/g5_tracker.npz;
//  * velocities (c - last) / frames_elapsed in float32; average_velocity = mean of norms
//    (float64 mean when the window holds the float64 zero, float32 otherwise).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <numeric>
#include <system_error>
#include <vector>

#include <immintrin.h>

#include "host_common.h"
#include "host_stage.h"

#pragma STDC FP_CONTRACT OFF

namespace rpt {

// ------------------------------------------------------------------ CPython set emulation
namespace {

struct PySetEmu {
  struct Entry {
    int64_t hash;
    int32_t key;
    bool used;
  };
  std::vector<Entry> table;
  size_t mask = 7, fill = 0, used = 0;
  std::vector<Entry> spare;
  PySetEmu() : table(8, Entry{0, 0, false}) {}
  void reset() {
    table.assign(8, Entry{0, 0, false});
    mask = 7;
    fill = used = 0;
  }

  static int64_t hash_of(int32_t v) { return v == -1 ? -2 : (int64_t)v; }

  static void insert_clean(std::vector<Entry>& t, size_t mask, int32_t key, int64_t hash) {
    size_t perturb = (size_t)hash;
    size_t i = (size_t)hash & mask;
    while (true) {
      Entry* e = &t[i];
      if (!e->used) {
        *e = Entry{hash, key, true};
        return;
      }
      if (i + 9 <= mask) {
        for (int j = 0; j < 9; ++j) {
          ++e;
          if (!e->used) {
            *e = Entry{hash, key, true};
            return;
          }
        }
      }
      perturb >>= 5;
      i = (i * 5 + 1 + perturb) & mask;
    }
  }

  void resize(size_t minused) {
    size_t newsize = 8;
    while (newsize <= minused) newsize <<= 1;
    spare.assign(newsize, Entry{0, 0, false});
    for (const Entry& e : table)
      if (e.used) insert_clean(spare, newsize - 1, e.key, e.hash);
    table.swap(spare);
    mask = newsize - 1;
    fill = used;
  }

  // set_add_entry for a key known to be absent (distinct first-occurrence sequence)
  void add(int32_t key) {
    const int64_t hash = hash_of(key);
    size_t perturb = (size_t)hash;
    size_t i = (size_t)hash & mask;
    Entry* e = &table[i];
    while (true) {
      if (!e->used) break;
      if (e->hash == hash && e->key == key) return;
      if (i + 9 <= mask) {
        bool found = false;
        for (int j = 0; j < 9; ++j) {
          ++e;
          if (!e->used) {
            found = true;
            break;
          }
          if (e->hash == hash && e->key == key) return;
        }
        if (found) break;
      }
      perturb >>= 5;
      i = (i * 5 + 1 + perturb) & mask;
      e = &table[i];
    }
    *e = Entry{hash, key, true};
    ++fill;
    ++used;
    if (fill * 5 >= mask * 3) resize(used > 50000 ? used * 2 : used * 4);
  }
};

}  // namespace

int32_t set_order(const int32_t* keys, int32_t n, int32_t* out) {
  thread_local PySetEmu s;
  s.reset();
  for (int32_t i = 0; i < n; ++i) s.add(keys[i]);
  int32_t m = 0;
  for (const auto& e : s.table)
    if (e.used && e.key != -1) out[m++] = e.key;
  return m;
}

int32_t FrameBuckets::build(int32_t n_frames, int64_t n_seg, const int32_t* seg_frame,
                            int64_t* frame_off) {
  cnt.assign((size_t)n_frames + 1, 0);
  for (int64_t s = 0; s < n_seg; ++s) {
    if (seg_frame[s] < 0 || seg_frame[s] >= n_frames) {
      set_error("rpt_order_clusters: segment frame %d out of range", seg_frame[s]);
      return RPT_EINVAL;
    }
    ++cnt[(size_t)seg_frame[s] + 1];
  }
  for (int32_t f = 0; f < n_frames; ++f) cnt[(size_t)f + 1] += cnt[(size_t)f];
  if (frame_off)
    for (int32_t f = 0; f <= n_frames; ++f) frame_off[f] = cnt[(size_t)f];
  byf.resize((size_t)n_seg);
  std::vector<int64_t> cur(cnt.begin(), cnt.end() - 1);
  for (int64_t s = 0; s < n_seg; ++s) byf[(size_t)cur[(size_t)seg_frame[s]]++] = s;
  return RPT_OK;
}

// order[b + q] (+ add) for the frames [f_lo, f_hi) of the buckets; set_order's table is
// thread_local, so ranges may be ordered on any thread
void FrameBuckets::order(int32_t f_lo, int32_t f_hi, const int32_t* seg_label,
                         const int64_t* seg_first, const int64_t* frame_first_noise,
                         int64_t* order_out, int64_t add) const {
  std::vector<std::pair<int64_t, int32_t>> occ;  // (first index, label)
  std::vector<int32_t> keys, ord;
  std::vector<std::pair<int32_t, int64_t>> l2s;
  for (int32_t f = f_lo; f < f_hi; ++f) {
    const int64_t b = cnt[(size_t)f], e = cnt[(size_t)f + 1];
    occ.clear();
    for (int64_t q = b; q < e; ++q) occ.emplace_back(seg_first[byf[q]], seg_label[byf[q]]);
    if (frame_first_noise && frame_first_noise[f] >= 0) occ.emplace_back(frame_first_noise[f], -1);
    std::sort(occ.begin(), occ.end());
    keys.resize(occ.size());
    for (size_t q = 0; q < occ.size(); ++q) keys[q] = occ[q].second;
    ord.resize(occ.size());
    const int32_t m = set_order(keys.data(), (int32_t)keys.size(), ord.data());
    // label -> segment (labels are unique within a frame)
    l2s.clear();
    for (int64_t q = b; q < e; ++q) l2s.emplace_back(seg_label[byf[q]], byf[q]);
    std::sort(l2s.begin(), l2s.end());
    for (int32_t q = 0; q < m; ++q) {
      auto it = std::lower_bound(l2s.begin(), l2s.end(), std::make_pair(ord[q], int64_t(-1)));
      order_out[b + q] = it->second + add;
    }
  }
}

int32_t order_clusters(int32_t n_frames, int64_t n_seg, const int32_t* seg_frame,
                       const int32_t* seg_label, const int64_t* seg_first,
                       const int64_t* frame_first_noise, int64_t* frame_off, int64_t* order) {
  FrameBuckets fb;
  RPT_TRY(fb.build(n_frames, n_seg, seg_frame, frame_off));
  fb.order(0, n_frames, seg_label, seg_first, frame_first_noise, order, 0);
  return RPT_OK;
}

// ------------------------------------------------------------------ ordering ahead of a consumer
void OrderAhead::publish(int64_t frames_done) {
  std::lock_guard<std::mutex> g(mu_);
  done_.store(frames_done, std::memory_order_release);
  cv_.notify_all();
}

void OrderAhead::wait_for(int64_t frame) {
  if (done_.load(std::memory_order_acquire) > frame) return;
  for (int spin = 0; spin < 2000; ++spin) {  // chunks finish within microseconds
    if (done_.load(std::memory_order_acquire) > frame) return;
    std::this_thread::yield();
  }
  std::unique_lock<std::mutex> g(mu_);
  cv_.wait(g, [&] { return done_.load(std::memory_order_acquire) > frame; });
}

void OrderAhead::start(std::function<void(OrderAhead&)> producer, bool threaded) {
  done_.store(-1);
  failed_.store(false);
  auto body = [this, producer] {
    try {
      producer(*this);
    } catch (...) {
      failed_.store(true, std::memory_order_release);
      publish(INT64_MAX);
    }
  };
  if (threaded) {
    try {
      th_ = std::thread(body);
      return;
    } catch (const std::system_error&) {  // no thread: produce everything first
    }
  }
  body();
}

void OrderAhead::join() {
  if (th_.joinable()) th_.join();
}

// ------------------------------------------------------------------ scipy LSAP
// Rectangular LSAP exactly as scipy 1.15 (_lsap.c, Crouse 2016): shortest augmenting path per
// row, remaining columns scanned from a reversed list, ties on the minimum prefer an unassigned
// column, tall matrices solved transposed.  Scratch is kept across calls (one solver per tracker).
namespace {

bool host_has_avx2() {
  static const bool v = __builtin_cpu_supports("avx2");
  return v;
}

// r_j = ((0 + c_j) - u_i) - v_j for every column, path_j = i; returns min_j r_j
double first_scan_base(int64_t nc, const double* row, double ui, const double* vv, double* sp,
                       int64_t* pa, int64_t i) {
  double mn = std::numeric_limits<double>::infinity();
  for (int64_t j = 0; j < nc; ++j) {
    const double r = 0.0 + row[j] - ui - vv[j];
    sp[j] = r;
    pa[j] = i;
    mn = r < mn ? r : mn;
  }
  return mn;
}

__attribute__((target("avx2"))) double first_scan_avx2(int64_t nc, const double* row, double ui,
                                                       const double* vv, double* sp, int64_t* pa,
                                                       int64_t i) {
  const __m256d z = _mm256_setzero_pd(), uv = _mm256_set1_pd(ui);
  const __m256i iv = _mm256_set1_epi64x(i);
  __m256d m0 = _mm256_set1_pd(std::numeric_limits<double>::infinity()), m1 = m0;
  int64_t j = 0;
  for (; j + 8 <= nc; j += 8) {
    const __m256d r0 = _mm256_sub_pd(_mm256_sub_pd(_mm256_add_pd(z, _mm256_loadu_pd(row + j)), uv),
                                     _mm256_loadu_pd(vv + j));
    const __m256d r1 = _mm256_sub_pd(
        _mm256_sub_pd(_mm256_add_pd(z, _mm256_loadu_pd(row + j + 4)), uv),
        _mm256_loadu_pd(vv + j + 4));
    _mm256_storeu_pd(sp + j, r0);
    _mm256_storeu_pd(sp + j + 4, r1);
    _mm256_storeu_si256((__m256i*)(pa + j), iv);
    _mm256_storeu_si256((__m256i*)(pa + j + 4), iv);
    m0 = _mm256_min_pd(r0, m0);  // (r < m) ? r : m
    m1 = _mm256_min_pd(r1, m1);
  }
  m0 = _mm256_min_pd(m0, m1);
  __m128d lo = _mm_min_pd(_mm256_castpd256_pd128(m0), _mm256_extractf128_pd(m0, 1));
  double mn = _mm_cvtsd_f64(_mm_min_sd(lo, _mm_unpackhi_pd(lo, lo)));
  for (; j < nc; ++j) {
    const double r = 0.0 + row[j] - ui - vv[j];
    sp[j] = r;
    pa[j] = i;
    mn = r < mn ? r : mn;
  }
  return mn;
}

// bit j of bits = (sp[j] == mn)
void eq_bits_base(int64_t nc, const double* sp, double mn, uint64_t* bits) {
  for (int64_t j = 0; j < nc; ++j)
    if (sp[j] == mn) bits[j >> 6] |= 1ull << (j & 63);
}

__attribute__((target("avx2"))) void eq_bits_avx2(int64_t nc, const double* sp, double mn,
                                                  uint64_t* bits) {
  const __m256d m = _mm256_set1_pd(mn);
  for (int64_t w = 0; w * 64 < nc; ++w) {
    const int64_t e = std::min<int64_t>(nc, w * 64 + 64);
    uint64_t acc = 0;
    int64_t j = w * 64;
    for (; j + 4 <= e; j += 4)
      acc |= (uint64_t)_mm256_movemask_pd(_mm256_cmp_pd(_mm256_loadu_pd(sp + j), m, _CMP_EQ_OQ))
             << (j & 63);
    for (; j < e; ++j) acc |= (uint64_t)(sp[j] == mn) << (j & 63);
    bits[w] |= acc;
  }
}

inline double bits_all_ones() {
  const uint64_t u = ~0ull;
  double d;
  std::memcpy(&d, &u, 8);
  return d;
}

// One later Dijkstra scan over ALL columns, masked to the remaining ones (live[j] all-ones):
// r = ((mv + c_j) - u_i) - v_j, spc_j = min(spc_j, r) with path_j = i where it drops.  Returns
// the minimum of the remaining columns' new spc.
__attribute__((target("avx2"))) double rest_scan_masked_avx2(int64_t nc, const double* row,
                                                             double mv, double ui,
                                                             const double* vv,
                                                             const double* live, double* sp,
                                                             int64_t* pa, int64_t i) {
  const __m256d m = _mm256_set1_pd(mv), uv = _mm256_set1_pd(ui);
  const __m256d inf = _mm256_set1_pd(std::numeric_limits<double>::infinity());
  const __m256d iv = _mm256_castsi256_pd(_mm256_set1_epi64x(i));
  __m256d best = inf;
  int64_t j = 0;
  for (; j + 4 <= nc; j += 4) {
    const __m256d r = _mm256_sub_pd(_mm256_sub_pd(_mm256_add_pd(m, _mm256_loadu_pd(row + j)), uv),
                                    _mm256_loadu_pd(vv + j));
    const __m256d so = _mm256_loadu_pd(sp + j);
    const __m256d lv = _mm256_loadu_pd(live + j);
    const __m256d upd = _mm256_and_pd(_mm256_cmp_pd(r, so, _CMP_LT_OQ), lv);
    const __m256d sj = _mm256_blendv_pd(so, r, upd);
    _mm256_storeu_pd(sp + j, sj);
    const __m256d po = _mm256_loadu_pd(reinterpret_cast<const double*>(pa + j));
    _mm256_storeu_pd(reinterpret_cast<double*>(pa + j), _mm256_blendv_pd(po, iv, upd));
    best = _mm256_min_pd(_mm256_blendv_pd(inf, sj, lv), best);
  }
  __m128d lo = _mm_min_pd(_mm256_castpd256_pd128(best), _mm256_extractf128_pd(best, 1));
  double mn = _mm_cvtsd_f64(_mm_min_sd(lo, _mm_unpackhi_pd(lo, lo)));
  for (; j < nc; ++j) {
    uint64_t lb;
    std::memcpy(&lb, live + j, 8);
    if (!lb) continue;
    const double r = mv + row[j] - ui - vv[j];
    if (r < sp[j]) {
      sp[j] = r;
      pa[j] = i;
    }
    mn = sp[j] < mn ? sp[j] : mn;
  }
  return mn;
}

// bit j of bits = (sp[j] == mn) for the remaining columns
__attribute__((target("avx2"))) void eq_bits_live_avx2(int64_t nc, const double* sp, double mn,
                                                       const double* live, uint64_t* bits) {
  const __m256d m = _mm256_set1_pd(mn);
  for (int64_t w = 0; w * 64 < nc; ++w) {
    const int64_t e = std::min<int64_t>(nc, w * 64 + 64);
    uint64_t acc = 0;
    int64_t j = w * 64;
    for (; j + 4 <= e; j += 4)
      acc |= (uint64_t)_mm256_movemask_pd(_mm256_and_pd(
                 _mm256_cmp_pd(_mm256_loadu_pd(sp + j), m, _CMP_EQ_OQ), _mm256_loadu_pd(live + j)))
             << (j & 63);
    for (; j < e; ++j) {
      uint64_t lb;
      std::memcpy(&lb, live + j, 8);
      acc |= (uint64_t)(lb && sp[j] == mn) << (j & 63);
    }
    bits[w] |= acc;
  }
}

}  // namespace

struct Lsap {
  std::vector<double> u, v, spc, tmp, scan;
  std::vector<int64_t> path, col4row, row4col, remaining, idx, sr_list, sc_list, pos;
  std::vector<uint64_t> eqbits;
  std::vector<double> live;   // all-ones bit pattern: column still in rem (masked scans)

  // One shortest augmenting path from row i (scipy's augmenting_path).  The rows / columns it
  // visits are recorded in sr_list / sc_list (scipy's SR / SC flags) so that the dual updates
  // touch only those; spc is (re)initialised by the first scan, which visits every column.
  int64_t augmenting_path(int64_t nc, const double* cost, int64_t i, double* p_min) {
    double minVal = 0;
    int64_t num_remaining = nc;
    int64_t* rem = remaining.data();
    double* sp = spc.data();
    int64_t* pa = path.data();
    const int64_t* r4c = row4col.data();
    const double* vv = v.data();
    // rem (scipy's reversed list of remaining columns) is only materialised when the first scan
    // does not reach a sink; until then rem[it] = nc - 1 - it implicitly
    sr_list.clear();
    sc_list.clear();
    int64_t sink = -1;
    bool first = true;
    while (sink == -1) {
      int64_t index = -1;
      double lowest = std::numeric_limits<double>::infinity();
      const bool scan0 = first;
      sr_list.push_back(i);
      const double* row = cost + i * nc;
      const double ui = u[i];
      if (first) {
        // First scan: every spc[j] is inf (the test r < spc[j] always passes) and the scan order
        // is j = nc-1 .. 0, so it runs as contiguous (vectorised) loops.  The sequential rule
        // "strictly lower, or equal and the column unassigned" selects, among the columns at the
        // minimum, the last unassigned one in scan order after the first one, else the first:
        // with the order descending in j, that is the smallest unassigned j below the largest
        // minimum j, else the largest minimum j.  r is never -0.0 (0 + c - u - v), so a lane-wise
        // minimum is the sequential one.
        const double mn = (host_has_avx2() ? first_scan_avx2 : first_scan_base)(nc, row, ui, vv,
                                                                                 sp, pa, i);
        // columns at the minimum as a bit set (a handful of words: nc is the object count)
        eqbits.assign((size_t)((nc + 63) >> 6), 0);
        (host_has_avx2() ? eq_bits_avx2 : eq_bits_base)(nc, sp, mn, eqbits.data());
        int64_t jmax = -1;
        for (int64_t w = (int64_t)eqbits.size() - 1; w >= 0; --w)
          if (eqbits[w]) {
            jmax = w * 64 + 63 - __builtin_clzll(eqbits[w]);
            break;
          }
        int64_t jsel = jmax;
        for (int64_t w = 0; w * 64 < jmax && jsel == jmax; ++w) {
          uint64_t b = eqbits[w];
          while (b) {
            const int64_t j = w * 64 + __builtin_ctzll(b);
            if (j >= jmax) break;
            if (r4c[j] == -1) {
              jsel = j;
              break;
            }
            b &= b - 1;
          }
        }
        lowest = mn;
        index = (jmax < 0) ? -1 : nc - 1 - jsel;
        if (mn == std::numeric_limits<double>::infinity()) index = -1;
        first = false;
      } else if (host_has_avx2()) {
        // Later scans: the new spc values do not depend on the scan order, so they are computed
        // for all columns at once (contiguous, masked to the remaining ones: no gathers); the
        // sequential selection rule is then applied by rem position: among the remaining columns
        // at the minimum, the first in scan order, replaced by the last later one whose column
        // is unassigned.
        const double mn =
            rest_scan_masked_avx2(nc, row, minVal, ui, vv, live.data(), sp, pa, i);
        lowest = mn;
        index = -1;
        if (mn != std::numeric_limits<double>::infinity()) {
          eqbits.assign((size_t)((nc + 63) >> 6), 0);
          eq_bits_live_avx2(nc, sp, mn, live.data(), eqbits.data());
          int64_t p0 = std::numeric_limits<int64_t>::max();
          for (size_t w = 0; w < eqbits.size(); ++w)
            for (uint64_t bb = eqbits[w]; bb; bb &= bb - 1) {
              const int64_t pj = pos[(int64_t)w * 64 + __builtin_ctzll(bb)];
              p0 = pj < p0 ? pj : p0;
            }
          index = p0;
          int64_t best = -1;
          for (size_t w = 0; w < eqbits.size(); ++w)
            for (uint64_t bb = eqbits[w]; bb; bb &= bb - 1) {
              const int64_t j = (int64_t)w * 64 + __builtin_ctzll(bb);
              if (pos[j] > p0 && r4c[j] == -1 && pos[j] > best) best = pos[j];
            }
          if (best >= 0) index = best;
        }
      } else {
        for (int64_t it = 0; it < num_remaining; ++it) {
          const int64_t j = rem[it];
          const double r = minVal + row[j] - ui - vv[j];
          const bool upd = r < sp[j];
          pa[j] = upd ? i : pa[j];
          const double sj = upd ? r : sp[j];
          sp[j] = sj;
          const bool better = (sj < lowest) | ((sj == lowest) & (r4c[j] == -1));
          lowest = better ? sj : lowest;
          index = better ? it : index;
        }
      }
      minVal = lowest;
      if (minVal == std::numeric_limits<double>::infinity()) return -1;
      const int64_t j = scan0 ? nc - 1 - index : rem[index];
      if (r4c[j] == -1)
        sink = j;
      else
        i = r4c[j];
      sc_list.push_back(j);
      if (scan0 && sink == -1) {
        for (int64_t it = 0; it < nc; ++it) rem[it] = nc - it - 1;
        if (host_has_avx2()) {  // rem positions and the remaining-column mask of the masked scans
          live.assign((size_t)nc, -1.0);
          const double ones = bits_all_ones();
          for (int64_t c2 = 0; c2 < nc; ++c2) {
            pos[c2] = nc - 1 - c2;
            live[c2] = ones;
          }
        }
      }
      if (sink == -1) {
        if (host_has_avx2()) {
          live[j] = 0.0;
          pos[rem[num_remaining - 1]] = index;
          pos[j] = -1;
        }
        rem[index] = rem[--num_remaining];
      }
    }
    *p_min = minVal;
    return sink;
  }

  // finite_known: the caller guarantees no NaN / -inf entry (the tracker, from finite inputs)
  int32_t solve(const double* cost_in, int32_t nr_in, int32_t nc_in, int64_t* a, int64_t* b,
                bool finite_known = false) {
    int64_t nr = nr_in, nc = nc_in;
    if (nr == 0 || nc == 0) return RPT_OK;
    const bool transpose = nc < nr;
    const double* cost = cost_in;
    if (transpose) {
      tmp.resize(nr * nc);
      for (int64_t i = 0; i < nr; ++i)
        for (int64_t j = 0; j < nc; ++j) tmp[j * nr + i] = cost_in[i * nc + j];
      std::swap(nr, nc);
      cost = tmp.data();
    }
    bool bad = false;
    for (int64_t i = 0; i < (finite_known ? 0 : nr * nc); ++i)
      bad |= (cost[i] != cost[i]) | (cost[i] == -std::numeric_limits<double>::infinity());
    if (bad) {
      set_error("matrix contains invalid numeric entries");
      return RPT_EINVAL;
    }
    u.assign(nr, 0.0);
    v.assign(nc, 0.0);
    spc.resize(nc);
    path.assign(nc, -1);
    col4row.assign(nr, -1);
    row4col.assign(nc, -1);
    remaining.resize(nc);
    pos.resize(nc);
    live.resize(nc);
    for (int64_t cur = 0; cur < nr; ++cur) {
      double minVal;
      const int64_t sink = augmenting_path(nc, cost, cur, &minVal);
      if (sink < 0) {
        set_error("cost matrix is infeasible");
        return RPT_EINVAL;
      }
      // scipy updates u over i in SR (ascending i) and v over j in SC; each entry is updated
      // independently, so the visiting order does not change any value
      u[cur] += minVal;
      for (const int64_t i : sr_list)
        if (i != cur) u[i] += minVal - spc[col4row[i]];
      for (const int64_t j : sc_list) v[j] -= minVal - spc[j];
      int64_t j = sink;
      while (true) {
        const int64_t i = path[j];
        row4col[j] = i;
        std::swap(col4row[i], j);
        if (i == cur) break;
      }
    }
    if (transpose) {
      idx.resize(nr);
      std::iota(idx.begin(), idx.end(), 0);
      std::sort(idx.begin(), idx.end(),
                [&](int64_t p, int64_t q) { return col4row[p] < col4row[q]; });
      for (int64_t k = 0; k < nr; ++k) {
        a[k] = col4row[idx[k]];
        b[k] = idx[k];
      }
    } else {
      for (int64_t k = 0; k < nr; ++k) {
        a[k] = k;
        b[k] = col4row[k];
      }
    }
    return RPT_OK;
  }
};

int32_t lsap(const double* cost_in, int32_t nr_in, int32_t nc_in, int64_t* a, int64_t* b) {
  thread_local Lsap solver;
  return solver.solve(cost_in, nr_in, nc_in, a, b);
}

// ------------------------------------------------------------------ tracker
namespace {

enum { kUnknown = 0, kBuoy = 1, kBoat = 2 };

struct Vel {
  float x, y;
  bool f64_zero;  // the float64 [0, 0] every object starts with
  float nrm;      // f32_norm(x, y) (average_velocity's terms), computed once
};

struct Object {
  int64_t id;
  int type = kUnknown;
  std::vector<float> px, py;
  std::vector<int64_t> frames;
  int64_t last_seen;
  std::vector<Vel> vel;
  int color[3];
  // mean of the last motion_history_frames velocities, in the dtype numpy gives it (refreshed
  // whenever vel changes; the prediction itself depends on the frame gap)
  bool mean64;
  double m64x, m64y;
  float m32x, m32y;
};

inline float f32_norm(float x, float y) {  // np.linalg.norm float32: sdot without FMA
  const float xx = x * x;
  const float yy = y * y;
  return std::sqrt(xx + yy);
}
inline Vel make_vel(float x, float y) { return Vel{x, y, false, f32_norm(x, y)}; }
inline double f64_norm(double x, double y) {  // np.linalg.norm float64: ddot with FMA
  return std::sqrt(std::fma(y, y, x * x));
}

// Cost matrix of one frame, [k clusters][m objects]: per object the prediction in the dtype numpy
// uses (float64 while its velocity window holds the float64 zero, float32 after), cost =
// np.linalg.norm of the difference.  Every entry gets the float32 norm (8-wide), then the columns
// listed in c64 (float64 predictions p64x/p64y[q] of column c64[q]: young objects) are
// overwritten with the float64 norm, computed 4-wide into t64 first.  The
// float64 norm's fused multiply-add must be the hardware instruction for speed (libm's software
// fma gives the same, correctly rounded, result), hence one build for AVX2+FMA hosts, dispatched
// at run time, and a baseline build.
#define RPT_FILL_COSTS_BODY                                              \
  for (int32_t i = 0; i < k; ++i) {                                      \
    const float fx = cx[i], fy = cy[i];                                  \
    const double dxs = (double)fx, dys = (double)fy;                     \
    double* row = cost + (size_t)i * m;                                  \
    for (int32_t j = 0; j < m; ++j) {                                    \
      const float ex = fx - p32x[j], ey = fy - p32y[j];                  \
      const float exx = ex * ex, eyy = ey * ey;                          \
      row[j] = (double)__builtin_sqrtf(exx + eyy);                       \
    }                                                                    \
    for (int32_t q = 0; q < n64; ++q) {                                  \
      const double dx = dxs - p64x[q], dy = dys - p64y[q];               \
      t64[q] = __builtin_sqrt(__builtin_fma(dy, dy, dx * dx));           \
    }                                                                    \
    for (int32_t q = 0; q < n64; ++q) row[c64[q]] = t64[q];              \
  }

__attribute__((target("avx2,fma"))) void fill_costs_v3(
    int32_t k, int32_t m, const float* __restrict__ cx, const float* __restrict__ cy,
    int32_t n64, const int32_t* __restrict__ c64, const double* __restrict__ p64x,
    const double* __restrict__ p64y, const float* __restrict__ p32x,
    const float* __restrict__ p32y, double* __restrict__ t64, double* __restrict__ cost) {
  RPT_FILL_COSTS_BODY
}
void fill_costs_base(int32_t k, int32_t m, const float* __restrict__ cx,
                     const float* __restrict__ cy, int32_t n64, const int32_t* __restrict__ c64,
                     const double* __restrict__ p64x, const double* __restrict__ p64y,
                     const float* __restrict__ p32x, const float* __restrict__ p32y,
                     double* __restrict__ t64, double* __restrict__ cost) {
  RPT_FILL_COSTS_BODY
}
#undef RPT_FILL_COSTS_BODY

bool host_has_fma() {
  static const bool v = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
  return v;
}

}  // namespace

struct Tracker {
  rpt_tracker_params p;
  std::vector<Object> objs;  // insertion (= id) order, like the reference dict
  int64_t next_id = 1;
  int64_t current = 0;
  // scratch (kept across frames)
  std::vector<double> cost;
  std::vector<int64_t> ra, ca;
  std::vector<int> live;
  std::vector<char> assigned;
  std::vector<int32_t> c64;
  std::vector<double> p64x, p64y, t64;  // float64 predictions of the columns in c64
  std::vector<float> p32x, p32y;
  Lsap solver;

  static void color_of(int64_t oid, int* rgb) {  // _generate_color :666-688 (float64)
    const double hue = std::fmod((double)oid * 0.618033988749895, 1.0);
    const int h_i = (int)(hue * 6);
    const double f = hue * 6 - h_i;
    const double q = 1 - f;
    double r, g, b;
    switch (h_i) {
      case 0: r = 1; g = f; b = 0; break;
      case 1: r = q; g = 1; b = 0; break;
      case 2: r = 0; g = 1; b = f; break;
      case 3: r = 0; g = q; b = 1; break;
      case 4: r = f; g = 0; b = 1; break;
      default: r = 1; g = 0; b = q; break;
    }
    rgb[0] = (int)(r * 255);
    rgb[1] = (int)(g * 255);
    rgb[2] = (int)(b * 255);
  }

  void create(float cx, float cy, int64_t fid) {
    Object o;
    o.id = next_id;
    o.px.push_back(cx);
    o.py.push_back(cy);
    o.frames.push_back(fid);
    o.last_seen = fid;
    o.vel.push_back(Vel{0.f, 0.f, true, 0.f});
    refresh_mean(o);
    color_of(next_id, o.color);
    objs.push_back(std::move(o));
    ++next_id;
  }

  // average_velocity :127-133; returns value and whether numpy yields float32
  double avg_velocity(const Object& o, bool* is_f32) const {
    *is_f32 = false;
    if (o.vel.size() < 2) return 0.0;
    const size_t H = (size_t)p.motion_history_frames;
    const size_t b = o.vel.size() > H ? o.vel.size() - H : 0;
    bool has64 = false;
    for (size_t k = b; k < o.vel.size(); ++k) has64 |= o.vel[k].f64_zero;
    const size_t m = o.vel.size() - b;
    if (has64) {  // np.mean over float64 array (< 8 values: sequential from 0.)
      double s = 0.0;
      for (size_t k = b; k < o.vel.size(); ++k)
        s = s + (o.vel[k].f64_zero ? 0.0 : (double)o.vel[k].nrm);
      return s / (double)m;
    }
    float s = 0.f;
    for (size_t k = b; k < o.vel.size(); ++k) s = s + o.vel[k].nrm;
    *is_f32 = true;
    return (double)(s / (float)m);
  }

  // prediction of object o `ahead` frames on (:135-140), in the dtype numpy would use
  struct Pred {
    bool f64;
    double x, y;  // float64 prediction (f64) or the float32 value widened
  };
  void refresh_mean(Object& o) const {
    const size_t H = (size_t)p.motion_history_frames;
    const size_t b = o.vel.size() > H ? o.vel.size() - H : 0;
    const size_t m = o.vel.size() - b;
    bool has64 = false;
    for (size_t k = b; k < o.vel.size(); ++k) has64 |= o.vel[k].f64_zero;
    o.mean64 = has64;
    if (has64) {  // np.mean(axis=0) float64: first row then sequential adds, one division
      double sx = o.vel[b].f64_zero ? 0.0 : (double)o.vel[b].x;
      double sy = o.vel[b].f64_zero ? 0.0 : (double)o.vel[b].y;
      for (size_t k = b + 1; k < o.vel.size(); ++k) {
        sx = sx + (o.vel[k].f64_zero ? 0.0 : (double)o.vel[k].x);
        sy = sy + (o.vel[k].f64_zero ? 0.0 : (double)o.vel[k].y);
      }
      o.m64x = sx / (double)m;
      o.m64y = sy / (double)m;
      return;
    }
    float sx = o.vel[b].x, sy = o.vel[b].y;
    for (size_t k = b + 1; k < o.vel.size(); ++k) {
      sx = sx + o.vel[k].x;
      sy = sy + o.vel[k].y;
    }
    o.m32x = sx / (float)m;
    o.m32y = sy / (float)m;
  }

  Pred predict(const Object& o, int64_t ahead) const {
    const float lx = o.px.back(), ly = o.py.back();
    if (o.mean64)
      return Pred{true, (double)lx + o.m64x * (double)ahead, (double)ly + o.m64y * (double)ahead};
    const float px = lx + o.m32x * (float)ahead;
    const float py = ly + o.m32y * (float)ahead;
    return Pred{false, (double)px, (double)py};
  }
  void cleanup() {  // _cleanup_lost_objects: in place, order kept (dict deletion)
    size_t w = 0;
    for (size_t r = 0; r < objs.size(); ++r) {
      if (current - objs[r].last_seen > p.max_missed_frames) continue;
      if (w != r) objs[w] = std::move(objs[r]);
      ++w;
    }
    objs.erase(objs.begin() + w, objs.end());
  }

  int32_t update(int64_t fid, int32_t k, const float* cx, const float* cy, const int64_t* cfid) {
    current = fid;
    if (k == 0) {
      cleanup();
      return (int32_t)objs.size();
    }
    if (objs.empty()) {
      for (int32_t i = 0; i < k; ++i) create(cx[i], cy[i], cfid ? cfid[i] : fid);
      return (int32_t)objs.size();
    }
    live.clear();
    for (int q = 0; q < (int)objs.size(); ++q)
      if (fid - objs[q].last_seen <= p.max_missed_frames) live.push_back(q);
    if (live.empty()) {
      for (int32_t i = 0; i < k; ++i) create(cx[i], cy[i], cfid ? cfid[i] : fid);
      return (int32_t)objs.size();
    }
    const int32_t m = (int32_t)live.size();
    cost.resize((size_t)k * m);
    c64.clear();
    p64x.clear();
    p64y.clear();
    p32x.resize(m);
    p32y.resize(m);
    // every input finite: no cost entry can be NaN or -inf (a difference of finite floats is
    // finite or +-inf, its norm finite or +inf), so the solver's scan of the matrix is skipped
    bool finite = true;
    for (int32_t j = 0; j < m; ++j) {
      const Object& o = objs[live[j]];
      const Pred q = predict(o, fid - o.last_seen);  // depends on the object only
      if (q.f64) {
        c64.push_back(j);
        p64x.push_back(q.x);
        p64y.push_back(q.y);
      }
      p32x[j] = (float)q.x;
      p32y[j] = (float)q.y;
      finite = finite && std::isfinite(q.x) && std::isfinite(q.y);
    }
    for (int32_t i = 0; i < k; ++i) finite = finite && std::isfinite(cx[i]) && std::isfinite(cy[i]);
    t64.resize(c64.size());
    (host_has_fma() ? fill_costs_v3 : fill_costs_base)(k, m, cx, cy, (int32_t)c64.size(),
                                                         c64.data(), p64x.data(), p64y.data(),
                                                         p32x.data(), p32y.data(), t64.data(),
                                                         cost.data());
    const int32_t np_ = std::min(k, m);
    ra.resize(np_);
    ca.resize(np_);
    const int32_t ls = solver.solve(cost.data(), k, m, ra.data(), ca.data(), finite);
    if (ls != RPT_OK) return -ls;  // negative = error (counts are >= 0)
    assigned.assign(k, 0);
    for (int32_t q = 0; q < np_; ++q) {
      const int64_t i = ra[q], j = ca[q];
      if (cost[(size_t)i * m + j] <= p.max_association_distance) {
        Object& o = objs[live[j]];
        const int64_t fe = fid - o.last_seen;
        if (fe > 0) {
          const float fef = (float)fe;
          o.vel.push_back(make_vel((cx[i] - o.px.back()) / fef, (cy[i] - o.py.back()) / fef));
          refresh_mean(o);
        }
        o.px.push_back(cx[i]);
        o.py.push_back(cy[i]);
        o.frames.push_back(fid);
        o.last_seen = fid;
        if ((int)o.vel.size() < p.motion_history_frames) {
          o.type = kUnknown;
        } else {
          bool f32;
          const double av = avg_velocity(o, &f32);
          o.type = (av < p.stationary_velocity_threshold) ? kBuoy : kBoat;
        }
        assigned[i] = 1;
      }
    }
    for (int32_t i = 0; i < k; ++i)
      if (!assigned[i]) create(cx[i], cy[i], cfid ? cfid[i] : fid);
    cleanup();
    return (int32_t)objs.size();
  }
};

}  // namespace rpt

using rpt::Tracker;

extern "C" {

struct rpt_tracker {
  Tracker t;
};

int32_t rpt_set_order(const int32_t* keys, int32_t n, int32_t* order_out) {
  return rpt::set_order(keys, n, order_out);
}

int32_t rpt_order_clusters(int32_t n_frames, int64_t n_segments, const int32_t* seg_frame,
                           const int32_t* seg_label, const int64_t* seg_first,
                           const int64_t* frame_first_noise, int64_t* frame_offsets_out,
                           int64_t* order_out) {
  rpt::clear_error();
  return rpt::order_clusters(n_frames, n_segments, seg_frame, seg_label, seg_first,
                             frame_first_noise, frame_offsets_out, order_out);
}

int32_t rpt_order_and_track(int32_t n_frames, int64_t n_segments, const int32_t* seg_frame,
                            const int32_t* seg_label, const int64_t* seg_first,
                            const int64_t* frame_first_noise, const float* seg_cx,
                            const float* seg_cy, int32_t n_built, const int64_t* built_slots,
                            const int64_t* frame_ids, rpt_tracker* trk,
                            int64_t* frame_offsets_out, int64_t* order_out) {
  rpt::clear_error();
  if (n_frames < 0 || n_segments < 0 || n_built < 0 || !frame_offsets_out ||
      (n_segments > 0 && (!seg_frame || !seg_label || !seg_first || !order_out)) ||
      (trk && n_built > 0 && (!built_slots || (n_segments > 0 && (!seg_cx || !seg_cy))))) {
    rpt::set_error("rpt_order_and_track: bad arguments");
    return RPT_EINVAL;
  }
  if (trk)
    for (int32_t b = 0; b < n_built; ++b)
      if (built_slots[b] < 0 || built_slots[b] >= n_frames ||
          (b > 0 && built_slots[b] <= built_slots[b - 1])) {
        rpt::set_error("rpt_order_and_track: built slot %lld out of order or range",
                       (long long)built_slots[b]);
        return RPT_EINVAL;
      }
  rpt::FrameBuckets fb;
  RPT_TRY(fb.build(n_frames, n_segments, seg_frame, frame_offsets_out));
  if (!trk) {
    fb.order(0, n_frames, seg_label, seg_first, frame_first_noise, order_out, 0);
    return RPT_OK;
  }
  // frames ordered on a producer thread in chunks, ahead of the tracker (the sequential part:
  // ~4 us per frame against ~1.5 for the order), so the stage costs about the tracker alone
  constexpr int32_t kChunk = 32;
  rpt::OrderAhead ahead;
  ahead.start(
      [&](rpt::OrderAhead& a) {
        for (int32_t f = 0; f < n_frames; f += kChunk) {
          const int32_t hi = std::min(n_frames, f + kChunk);
          fb.order(f, hi, seg_label, seg_first, frame_first_noise, order_out, 0);
          a.publish(hi);
        }
      },
      n_built >= 2 * kChunk);
  std::vector<float> cx, cy;
  int32_t r = 0;
  for (int32_t b = 0; b < n_built && r >= 0; ++b) {
    const int64_t slot = built_slots[b];
    ahead.wait_for(slot);
    if (ahead.failed()) break;
    const int64_t lo = fb.cnt[(size_t)slot], hi = fb.cnt[(size_t)slot + 1];
    cx.resize((size_t)(hi - lo));
    cy.resize((size_t)(hi - lo));
    for (int64_t k = lo; k < hi; ++k) {
      cx[(size_t)(k - lo)] = seg_cx[order_out[k]];
      cy[(size_t)(k - lo)] = seg_cy[order_out[k]];
    }
    r = trk->t.update(frame_ids ? frame_ids[slot] : slot, (int32_t)(hi - lo), cx.data(),
                      cy.data(), nullptr);
  }
  ahead.join();
  if (ahead.failed()) {
    rpt::set_error("rpt_order_and_track: cluster order failed (out of memory)");
    return RPT_ENOMEM;
  }
  return r < 0 ? -r : RPT_OK;
}

int32_t rpt_lsap(const double* cost, int32_t nr, int32_t nc, int64_t* rows_out,
                 int64_t* cols_out) {
  rpt::clear_error();
  return rpt::lsap(cost, nr, nc, rows_out, cols_out);
}

rpt_tracker* rpt_tracker_new(const rpt_tracker_params* params) {
  auto* h = new rpt_tracker();
  if (params) {
    h->t.p = *params;
  } else {
    h->t.p.max_association_distance = 50.0;
    h->t.p.max_missed_frames = 10;
    h->t.p.motion_history_frames = 5;
    h->t.p.stationary_velocity_threshold = 1.0;
  }
  return h;
}

void rpt_tracker_free(rpt_tracker* t) { delete t; }

int32_t rpt_tracker_update(rpt_tracker* t, int64_t frame_id, int32_t k, const float* cx,
                           const float* cy, const int64_t* cluster_frame_id) {
  rpt::clear_error();
  return t->t.update(frame_id, k, cx, cy, cluster_frame_id);
}

int32_t rpt_tracker_run(rpt_tracker* t, int32_t n_frames, const int64_t* frame_ids,
                        const int64_t* offsets, const float* cx, const float* cy) {
  rpt::clear_error();
  int32_t r = 0;
  for (int32_t f = 0; f < n_frames; ++f) {
    const int64_t b = offsets[f];
    const int32_t k = (int32_t)(offsets[f + 1] - b);
    r = t->t.update(frame_ids[f], k, cx + b, cy + b, nullptr);
    if (r < 0) return r;
  }
  return r;
}

int32_t rpt_tracker_num_objects(const rpt_tracker* t) { return (int32_t)t->t.objs.size(); }

int32_t rpt_tracker_object_info(const rpt_tracker* t, int32_t idx, rpt_object_info* out) {
  if (idx < 0 || idx >= (int32_t)t->t.objs.size()) return RPT_EINVAL;
  const auto& o = t->t.objs[idx];
  out->object_id = o.id;
  out->object_type = o.type;
  out->n_positions = (int32_t)o.px.size();
  out->n_velocities = (int32_t)o.vel.size();
  out->last_seen_frame = o.last_seen;
  bool f32 = false;
  out->average_velocity = t->t.avg_velocity(o, &f32);
  out->average_velocity_is_f32 = f32 ? 1 : 0;
  for (int c = 0; c < 3; ++c) out->color[c] = o.color[c];
  return RPT_OK;
}

int32_t rpt_tracker_object_history(const rpt_tracker* t, int32_t idx, float* px, float* py,
                                   int64_t* frames, double* vx, double* vy) {
  if (idx < 0 || idx >= (int32_t)t->t.objs.size()) return RPT_EINVAL;
  const auto& o = t->t.objs[idx];
  for (size_t k = 0; k < o.px.size(); ++k) {
    if (px) px[k] = o.px[k];
    if (py) py[k] = o.py[k];
    if (frames) frames[k] = o.frames[k];
  }
  for (size_t k = 0; k < o.vel.size(); ++k) {
    if (vx) vx[k] = o.vel[k].f64_zero ? 0.0 : (double)o.vel[k].x;
    if (vy) vy[k] = o.vel[k].f64_zero ? 0.0 : (double)o.vel[k].y;
  }
  return RPT_OK;
}

}  // extern "C"
