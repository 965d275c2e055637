// Rank 0's host stage of the frame-sharded driver (shard.cpp) over the all-gathered packed
// per-rank results -- the global cluster numbering, every segment in global frame ids, the
// reference cluster order per frame (4_temporal_object_tracker.py:519-522) and the tracker over
// the built frames (:984-991), the parts unpacked and ordered on a producer thread ahead of the
// tracker -- and the host equivalence merge used when a step's gathered pairs
// exceed the device merge.  No device work: host-only, so tools/asan/Makefile also builds it with
// -fsanitize=address,undefined.
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "host_common.h"
#include "host_stage.h"
#include "shard_pack.h"

namespace rpt {
// ---- rank 0's host stage over the all-gathered packed results (no device work)
namespace {
struct Part {
  const int64_t* p;
  int64_t S, R, F, frame0, kept;
  const int64_t *built, *noise, *cnt, *first, *fl, *cxy, *mi, *reps;
};
int32_t parse_parts(const int64_t* g, int32_t world, int64_t row, std::vector<Part>& parts) {
  parts.clear();
  for (int32_t q = 0; q < world; ++q) {
    const int64_t* p = g + (int64_t)q * row;
    Part a{};
    a.p = p;
    if (p[0] != kPackMagic || p[1] < 0 || p[3] != 0 || p[4] > row) {
      set_error("rpt_shard host stage: rank %d's packed result is not complete (S %lld, flags "
                "%lld)", q, (long long)p[1], (long long)p[3]);
      return RPT_EINVAL;
    }
    a.S = p[1];
    a.R = p[2];
    a.F = p[5];
    a.frame0 = p[6];
    a.kept = p[7];
    a.built = p + kHdr;
    a.noise = a.built + a.F;
    a.cnt = a.noise + a.F;
    a.first = a.cnt + a.S;
    a.fl = a.first + a.S;
    a.cxy = a.fl + a.S;
    a.mi = a.cxy + a.S;
    a.reps = a.mi + a.S;
    parts.push_back(a);
  }
  return RPT_OK;
}
}  // namespace
}  // namespace rpt

using namespace rpt;

extern "C" {

/* sizes[4]: total segments, built frames, frames, global clusters */
int32_t rpt_shard_gathered_sizes(const int64_t* g, int32_t world, int64_t row_words,
                                 int64_t* sizes) {
  clear_error();
  if (!g || !sizes || world < 1 || row_words < kHdr) {
    set_error("rpt_shard_gathered_sizes: bad arguments");
    return RPT_EINVAL;
  }
  std::vector<Part> parts;
  RPT_TRY(parse_parts(g, world, row_words, parts));
  int64_t S = 0, B = 0, F = 0;
  std::vector<int64_t> all;
  for (const Part& a : parts) {
    S += a.S;
    F += a.F;
    for (int64_t f = 0; f < a.F; ++f) B += a.built[f] ? 1 : 0;
    all.insert(all.end(), a.reps, a.reps + a.R);
  }
  std::sort(all.begin(), all.end());
  sizes[0] = S;
  sizes[1] = B;
  sizes[2] = F;
  sizes[3] = (int64_t)(std::unique(all.begin(), all.end()) - all.begin());
  return RPT_OK;
}

int32_t rpt_shard_host_stage(const int64_t* g, int32_t world, int64_t row_words,
                             rpt_tracker* trk, int32_t* seg_frame, int32_t* seg_label,
                             int64_t* seg_count, int64_t* seg_first, float* seg_cx,
                             float* seg_cy, float* seg_mi, int64_t* built_ids,
                             int64_t* frame_off, int64_t* order, int32_t* local_to_global,
                             int32_t which_rank) {
  clear_error();
  if (!g || world < 1 || row_words < kHdr) {
    set_error("rpt_shard_host_stage: bad arguments");
    return RPT_EINVAL;
  }
  std::vector<Part> parts;
  RPT_TRY(parse_parts(g, world, row_words, parts));
  std::vector<int64_t> all;
  for (const Part& a : parts) all.insert(all.end(), a.reps, a.reps + a.R);
  std::sort(all.begin(), all.end());
  all.erase(std::unique(all.begin(), all.end()), all.end());
  auto glabel = [&](int64_t rep) {
    return (int32_t)(std::lower_bound(all.begin(), all.end(), rep) - all.begin());
  };
  if (local_to_global && which_rank >= 0 && which_rank < world) {
    const Part& a = parts[(size_t)which_rank];
    for (int64_t l = 0; l < a.R; ++l) local_to_global[l] = glabel(a.reps[l]);
  }
  if (!seg_frame) return RPT_OK;  // only the label map
  if (!seg_label || !seg_count || !seg_first || !seg_cx || !seg_cy || !seg_mi ||
      (trk && (!built_ids || !frame_off))) {
    set_error("rpt_shard_host_stage: bad arguments");
    return RPT_EINVAL;
  }
  // where each part's segments and frames go; the built frames (in order) from the headers
  std::vector<int64_t> s0s, fbases;
  int64_t s_tot = 0, f_tot = 0, nb = 0;
  for (const Part& a : parts) {
    s0s.push_back(s_tot);
    fbases.push_back(f_tot);
    for (int64_t f = 0; f < a.F; ++f) {
      if (a.built[f] && built_ids) built_ids[nb] = a.frame0 + f;
      nb += a.built[f] ? 1 : 0;
    }
    s_tot += a.S;
    f_tot += a.F;
  }
  if (frame_off) frame_off[0] = 0;
  std::vector<int64_t> own_order;
  if (!order) own_order.resize((size_t)std::max<int64_t>(s_tot, 1));
  int64_t* ord_out = order ? order : own_order.data();
  // producer: per part the segments in global numbering and frame ids, then the reference
  // cluster order of its frames in chunks, published as global frame slots
  constexpr int32_t kChunk = 32;
  int32_t perr = RPT_OK;
  std::string pmsg;
  OrderAhead ahead;
  ahead.start(
      [&](OrderAhead& ah) {
        std::vector<int32_t> lf, gl, map;
        FrameBuckets fb;
        for (size_t q = 0; q < parts.size(); ++q) {
          const Part& a = parts[q];
          const int64_t S = a.S, F = a.F, s0 = s0s[q], fbase = fbases[q];
          map.resize((size_t)a.R);
          for (int64_t l = 0; l < a.R; ++l) map[(size_t)l] = glabel(a.reps[l]);
          lf.resize((size_t)S);
          gl.resize((size_t)S);
          for (int64_t s = 0; s < S; ++s) {
            const int32_t fr = (int32_t)(a.fl[s] >> 32);
            const int32_t ll = (int32_t)(uint32_t)(a.fl[s] & 0xffffffff);
            lf[(size_t)s] = fr;
            gl[(size_t)s] = (ll >= 0 && ll < a.R) ? map[(size_t)ll] : -2;
            seg_frame[s0 + s] = (int32_t)(fr + a.frame0);
            seg_label[s0 + s] = gl[(size_t)s];
            seg_count[s0 + s] = a.cnt[s];
            seg_first[s0 + s] = a.first[s];
            const uint64_t b = (uint64_t)a.cxy[s];
            const uint32_t bx = (uint32_t)b, by = (uint32_t)(b >> 32),
                           bm = (uint32_t)(uint64_t)a.mi[s];
            std::memcpy(&seg_cx[s0 + s], &bx, 4);
            std::memcpy(&seg_cy[s0 + s], &by, 4);
            std::memcpy(&seg_mi[s0 + s], &bm, 4);
          }
          // the reference cluster order of each frame of the part (local frame slots, local
          // firsts), segment ids shifted to the global numbering
          const int32_t st = fb.build((int32_t)F, S, lf.data(), nullptr);
          if (st != RPT_OK) {
            perr = st;
            pmsg = last_error_cstr();
            ah.publish(INT64_MAX);
            return;
          }
          if (frame_off)
            for (int64_t f = 0; f < F; ++f) frame_off[fbase + f + 1] = fb.cnt[(size_t)f + 1] + s0;
          for (int64_t f = 0; f < F; f += kChunk) {
            const int64_t hi = std::min<int64_t>(F, f + kChunk);
            fb.order((int32_t)f, (int32_t)hi, gl.data(), a.first, a.noise, ord_out + s0, s0);
            ah.publish(fbase + hi);
          }
        }
        ah.publish(INT64_MAX);
      },
      trk != nullptr && f_tot >= 2 * kChunk);
  int32_t r = 0;
  if (trk) {
    // the tracker over the built frames in order, each frame's clusters in the reference order
    // (frame slots are global frame ids less rank 0's first frame), frame by frame as the
    // producer publishes them
    const int64_t f0 = parts.empty() ? 0 : parts[0].frame0;
    std::vector<float> cxs, cys;
    for (int64_t b = 0; b < nb && r >= 0; ++b) {
      const int64_t slot = built_ids[b] - f0;
      ahead.wait_for(slot);
      if (perr != RPT_OK || ahead.failed()) break;
      const int64_t lo = frame_off[slot], hi = frame_off[slot + 1];
      cxs.resize((size_t)(hi - lo));
      cys.resize((size_t)(hi - lo));
      for (int64_t k = lo; k < hi; ++k) {
        cxs[(size_t)(k - lo)] = seg_cx[ord_out[k]];
        cys[(size_t)(k - lo)] = seg_cy[ord_out[k]];
      }
      r = rpt_tracker_update(trk, built_ids[b], (int32_t)(hi - lo), cxs.data(), cys.data(),
                             nullptr);
    }
  }
  ahead.join();
  if (perr != RPT_OK) {
    set_error("%s", pmsg.c_str());
    return perr;
  }
  if (ahead.failed()) {
    set_error("rpt_shard_host_stage: host stage failed (out of memory)");
    return RPT_ENOMEM;
  }
  return r < 0 ? -r : RPT_OK;
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
