// Native radar-CSV ingest: the file half of load_radar_csv,
//
//   pd.read_csv(path, header=None, names=[Status, Scale, Range, Gain, Angle, Echo_0..1023],
//               skiprows=1, engine="c")                 PointCloudWork/4_temporal_object_tracker.py:189-198
//   echo = df.iloc[:, 5:].fillna(0).to_numpy(float32); Scale, Angle .to_numpy(float32)  :203-211
//
// parsed by a pool of host threads straight into the caller's (pinned) buffers laid out as the
// device stack wants them: echo [file][rows_cap][bins] (u8 when every value is an integer in
// 0..255 -- the radar's native samples, 1 byte per sample in HBM -- else float32), Scale and
// Angle float32 [file][rows_cap].  Rows past a file's end are zero (they keep no point).
//
// pandas semantics kept: the first physical line is skipped (skiprows=1), blank lines are
// skipped, k extra fields in the first data row become an implicit index (the data shift right
// by k), a later row with more fields than that is a tokenizing error (read_csv raises; the
// reference catches it and returns an empty sweep), missing trailing fields are NaN (echo
// fillna(0); Scale/Angle stay NaN), a file with no data row is `df.empty` (empty sweep).  Numbers
// are parsed to float64 as pandas' round-trip parser does (integers exactly, decimals correctly
// rounded) and then rounded to float32 like to_numpy(np.float32).  A non-numeric value makes
// pandas give an object column that to_numpy(np.float32) refuses: reported per file.
#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "common.h"

namespace rpt {
namespace {

bool read_file(const char* path, std::string& buf) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  buf.clear();
  if (std::fseek(f, 0, SEEK_END) == 0) {
    const long sz = std::ftell(f);
    if (sz > 0) buf.reserve((size_t)sz + 1);
    std::fseek(f, 0, SEEK_SET);
  }
  char tmp[1 << 16];
  size_t k;
  while ((k = std::fread(tmp, 1, sizeof tmp, f)) > 0) buf.append(tmp, k);
  const bool ok = !std::ferror(f);
  std::fclose(f);
  return ok;
}

inline bool is_blank_line(const char* a, const char* b) {
  for (const char* p = a; p < b; ++p)
    if (*p != ' ' && *p != '\t' && *p != '\r') return false;
  return true;
}

// Data lines after the first physical line: [begin, end) ranges without the newline.
void data_lines(const std::string& s, std::vector<std::pair<const char*, const char*>>& out) {
  out.clear();
  const char* p = s.data();
  const char* e = p + s.size();
  const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(e - p)));
  if (!nl) return;  // header only (or nothing)
  p = nl + 1;
  while (p < e) {
    const char* q = static_cast<const char*>(std::memchr(p, '\n', (size_t)(e - p)));
    const char* le = q ? q : e;
    const char* lt = le;
    if (lt > p && lt[-1] == '\r') --lt;
    if (lt > p && !is_blank_line(p, lt)) out.push_back({p, lt});
    p = q ? q + 1 : e;
  }
}

enum FieldKind { kNum = 0, kMissing = 1, kBad = 2 };

// One field [a, b): float64 value (pandas' C parser: surrounding spaces allowed, integers
// exact, decimals correctly rounded).
inline FieldKind parse_field(const char* a, const char* b, double* v) {
  while (a < b && (*a == ' ' || *a == '\t')) ++a;
  while (b > a && (b[-1] == ' ' || b[-1] == '\t')) --b;
  if (a == b) return kMissing;
  // fast path: [+-]digits (up to 15 digits: exact in float64)
  const char* p = a;
  bool neg = false;
  if (*p == '+' || *p == '-') {
    neg = *p == '-';
    ++p;
  }
  if (p < b && (b - p) <= 15) {
    int64_t acc = 0;
    const char* q = p;
    while (q < b && *q >= '0' && *q <= '9') acc = acc * 10 + (*q++ - '0');
    if (q == b) {
      *v = neg ? -(double)acc : (double)acc;
      return kNum;
    }
  }
  char tmp[128];
  const size_t len = (size_t)(b - a);
  if (len >= sizeof tmp) return kBad;
  std::memcpy(tmp, a, len);
  tmp[len] = 0;
  // pandas' NaN spellings read as missing
  static const char* const kNa[] = {"nan", "NaN", "NAN", "-nan", "-NaN", "NA", "N/A", "n/a",
                                    "null", "NULL", "<NA>", "#N/A", "-1.#IND", "1.#QNAN",
                                    "#NA", "#N/A N/A", "-1.#QNAN", "1.#IND", "None"};
  for (const char* na : kNa)
    if (std::strcmp(tmp, na) == 0) return kMissing;
  for (size_t k = 0; k < len; ++k)  // strtod's hex floats and nan(...) are not numbers to pandas
    if (tmp[k] == 'x' || tmp[k] == 'X' || tmp[k] == 'p' || tmp[k] == 'P' || tmp[k] == '(')
      return kBad;
  char* end = nullptr;
  errno = 0;
  const double d = std::strtod(tmp, &end);
  if (end != tmp + len) return kBad;
  *v = d;
  return kNum;
}

constexpr int kMeta = 5;  // Status, Scale, Range, Gain, Angle

// status: 0 ok, 1 unreadable / tokenizing error (empty sweep), 2 no data row (df.empty),
// 3 a value not representable in u8 (the caller re-parses as float32), 4 non-numeric value
int32_t parse_one(const char* path, int32_t rows_cap, int32_t bins, int32_t dt, void* echo_f,
                  float* scale_f, float* angle_f, float* gain_f, std::string& buf,
                  std::vector<std::pair<const char*, const char*>>& lines) {
  const size_t row_bytes = (size_t)bins * (dt == RPT_ECHO_U8 ? 1 : 4);
  auto zero_tail = [&](int64_t from) {
    if (from >= rows_cap) return;
    std::memset(static_cast<char*>(echo_f) + (size_t)from * row_bytes, 0,
                (size_t)(rows_cap - from) * row_bytes);
    for (int64_t r = from; r < rows_cap; ++r) scale_f[r] = angle_f[r] = 0.0f;
  };
  *gain_f = 0.0f;
  if (!read_file(path, buf)) {
    zero_tail(0);
    return 1;
  }
  data_lines(buf, lines);
  if (lines.empty()) {
    zero_tail(0);
    return 2;
  }
  const int64_t R = std::min<int64_t>((int64_t)lines.size(), rows_cap);
  const int n_fields = kMeta + bins;
  // pandas: when the FIRST data row has k fields more than the names, its first k columns become
  // the (implicit) index and every row's data starts at field k; a row with more than
  // names + k fields is a tokenizing error
  int skip = 0;
  {
    const char* p = lines[0].first;
    const char* e = lines[0].second;
    int64_t nf = 1;
    for (const char* q = p; (q = static_cast<const char*>(std::memchr(q, ',', (size_t)(e - q))));
         ++q)
      ++nf;
    if (nf > n_fields) skip = (int)(nf - n_fields);
  }
  for (int64_t r = 0; r < R; ++r) {
    const char* p = lines[(size_t)r].first;
    const char* e = lines[(size_t)r].second;
    uint8_t* e8 = static_cast<uint8_t*>(echo_f) + (size_t)r * bins;
    float* e32 = static_cast<float*>(echo_f) + (size_t)r * bins;
    int f = 0;
    float sc = NAN, an = NAN;
    for (;;) {
      const char* c = static_cast<const char*>(std::memchr(p, ',', (size_t)(e - p)));
      const char* fe = c ? c : e;
      if (f >= n_fields + skip) {
        zero_tail(0);
        return 1;  // "Expected 1029 fields ... saw more": read_csv raises
      }
      if (f < skip) {  // index columns
        ++f;
        if (!c) break;
        p = c + 1;
        continue;
      }
      double v = 0.0;
      const FieldKind k = parse_field(p, fe, &v);
      if (k == kBad) {
        zero_tail(0);
        return 4;
      }
      const int fc = f - skip;  // column among the names
      if (fc >= kMeta) {
        const double ev = (k == kNum) ? v : 0.0;  // fillna(0)
        if (dt == RPT_ECHO_U8) {
          if (!(ev >= 0.0 && ev <= 255.0 && ev == std::floor(ev))) {
            zero_tail(0);
            return 3;
          }
          e8[fc - kMeta] = (uint8_t)ev;
        } else {
          e32[fc - kMeta] = (float)ev;
        }
      } else if (fc == 1) {
        sc = (k == kNum) ? (float)v : NAN;
      } else if (fc == 4) {
        an = (k == kNum) ? (float)v : NAN;
      } else if (fc == 3) {  // Gain: the first value, NaN when rows disagree (unique() > 1)
        const float gv = (k == kNum) ? (float)v : NAN;
        if (r == 0)
          *gain_f = gv;
        else if (!(gv == *gain_f))
          *gain_f = NAN;
      }
      ++f;
      if (!c) break;
      p = c + 1;
    }
    for (int g = std::max(f - skip, kMeta); g < n_fields; ++g) {  // missing trailing fields
      if (dt == RPT_ECHO_U8)
        e8[g - kMeta] = 0;
      else
        e32[g - kMeta] = 0.0f;
    }
    scale_f[r] = sc;
    angle_f[r] = an;
  }
  zero_tail(R);
  return 0;
}

int resolve_threads(int32_t n_threads, int32_t n_files) {
  int t = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
  if (t < 1) t = 1;
  return std::min(t, std::max(n_files, 1));
}

}  // namespace
}  // namespace rpt

using namespace rpt;

extern "C" {

int32_t rpt_csv_count_rows(const char* const* paths, int32_t n_files, int64_t* rows_out,
                           int32_t n_threads) {
  clear_error();
  if (n_files < 0 || (n_files > 0 && (!paths || !rows_out))) {
    set_error("rpt_csv_count_rows: bad arguments");
    return RPT_EINVAL;
  }
  std::atomic<int32_t> next{0};
  auto work = [&]() {
    std::string buf;
    for (;;) {
      const int32_t i = next.fetch_add(1);
      if (i >= n_files) return;
      if (!read_file(paths[i], buf)) {
        rows_out[i] = -1;
        continue;
      }
      std::vector<std::pair<const char*, const char*>> lines;
      data_lines(buf, lines);
      rows_out[i] = (int64_t)lines.size();
    }
  };
  const int T = resolve_threads(n_threads, n_files);
  std::vector<std::thread> th;
  for (int k = 1; k < T; ++k) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  return RPT_OK;
}

int32_t rpt_csv_parse_sweeps(const char* const* paths, int32_t n_files, int32_t rows_cap,
                             int32_t bins, int32_t echo_dtype, void* echo, float* scale,
                             float* angle, float* gain_col, int32_t* status_out,
                             int32_t n_threads) {
  clear_error();
  if (n_files < 0 || rows_cap < 0 || bins <= 0 ||
      (echo_dtype != RPT_ECHO_U8 && echo_dtype != RPT_ECHO_F32) ||
      (n_files > 0 && (!paths || !echo || !scale || !angle || !gain_col || !status_out))) {
    set_error("rpt_csv_parse_sweeps: bad arguments");
    return RPT_EINVAL;
  }
  const size_t es = echo_dtype == RPT_ECHO_U8 ? 1 : 4;
  std::atomic<int32_t> next{0};
  auto work = [&]() {
    std::string buf;
    std::vector<std::pair<const char*, const char*>> lines;
    for (;;) {
      const int32_t i = next.fetch_add(1);
      if (i >= n_files) return;
      status_out[i] = parse_one(
          paths[i], rows_cap, bins, echo_dtype,
          static_cast<char*>(echo) + (size_t)i * (size_t)rows_cap * (size_t)bins * es,
          scale + (size_t)i * rows_cap, angle + (size_t)i * rows_cap, gain_col + i, buf, lines);
    }
  };
  const int T = resolve_threads(n_threads, n_files);
  std::vector<std::thread> th;
  for (int k = 1; k < T; ++k) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  return RPT_OK;
}

}  // extern "C"
