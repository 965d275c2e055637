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
#include <cctype>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "host_common.h"

namespace rpt {
namespace {

bool read_file(const char* path, std::string& buf, int* err = nullptr) {
  errno = 0;
  FILE* f = std::fopen(path, "rb");
  if (!f) {
    if (err) *err = errno;
    return false;
  }
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
  if (!ok && err) *err = errno ? errno : EIO;
  std::fclose(f);
  return ok;
}

inline bool is_blank_line(const char* a, const char* b) {
  for (const char* p = a; p < b; ++p)
    if (*p != ' ' && *p != '\t' && *p != '\r') return false;
  return true;
}

// Data lines after the first physical line: [begin, end) ranges without the newline, and (when
// asked) their 1-based physical line numbers.
void data_lines(const std::string& s, std::vector<std::pair<const char*, const char*>>& out,
                std::vector<int64_t>* lineno = nullptr) {
  out.clear();
  if (lineno) lineno->clear();
  const char* p = s.data();
  const char* e = p + s.size();
  const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(e - p)));
  if (!nl) return;  // header only (or nothing)
  p = nl + 1;
  int64_t ln = 2;
  while (p < e) {
    const char* q = static_cast<const char*>(std::memchr(p, '\n', (size_t)(e - p)));
    const char* le = q ? q : e;
    const char* lt = le;
    if (lt > p && lt[-1] == '\r') --lt;
    if (lt > p && !is_blank_line(p, lt)) {
      out.push_back({p, lt});
      if (lineno) lineno->push_back(ln);
    }
    p = q ? q + 1 : e;
    ++ln;
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

// Python float(str) on one field [a, b): surrounding whitespace, optional sign, decimal digits
// with single underscores between digits, optional fraction / exponent, or nan / inf /
// infinity in any case.  false = float() raises (genfromtxt then uses the filling value).
inline bool py_float(const char* a, const char* b, double* v) {
  auto ws = [](char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\v' || c == '\f'; };
  while (a < b && ws(*a)) ++a;
  while (b > a && ws(b[-1])) --b;
  if (a == b || b - a > 120) return false;
  char tmp[128];
  int n = 0;
  const char* p = a;
  if (*p == '+' || *p == '-') tmp[n++] = *p++;
  auto word = [&](const char* w) {
    const size_t L = std::strlen(w);
    if ((size_t)(b - p) != L) return false;
    for (size_t k = 0; k < L; ++k)
      if (std::tolower((unsigned char)p[k]) != w[k]) return false;
    return true;
  };
  if (word("nan") || word("inf") || word("infinity")) {
    *v = std::tolower((unsigned char)*p) == 'n' ? NAN : INFINITY;
    if (n && tmp[0] == '-') *v = -*v;
    return true;
  }
  // digits (with underscores between digits) [. digits] [e [sign] digits]
  auto digits = [&](bool& any) {
    any = false;
    bool prev_digit = false;
    while (p < b) {
      if (*p >= '0' && *p <= '9') {
        tmp[n++] = *p++;
        any = prev_digit = true;
      } else if (*p == '_' && prev_digit && p + 1 < b && p[1] >= '0' && p[1] <= '9') {
        ++p;
        prev_digit = false;
      } else {
        break;
      }
    }
  };
  bool int_part = false, frac_part = false;
  digits(int_part);
  if (p < b && *p == '.') {
    tmp[n++] = *p++;
    digits(frac_part);
  }
  if (!int_part && !frac_part) return false;
  if (p < b && (*p == 'e' || *p == 'E')) {
    tmp[n++] = *p++;
    if (p < b && (*p == '+' || *p == '-')) tmp[n++] = *p++;
    bool ex = false;
    digits(ex);
    if (!ex) return false;
  }
  if (p != b) return false;
  tmp[n] = 0;
  *v = std::strtod(tmp, nullptr);
  return true;
}

// np.genfromtxt(path, delimiter=',', skip_header=1, dtype=float32, filling_values=0.0), the first
// loader of PointCloudWorkF/stdbscan_denoising_pipeline.py:97-119: the first physical line is
// skipped, text from '#' on is a comment, blank lines are skipped, a field float() cannot read
// (empty, non-numeric) is 0.0, every row must have the first row's field count (else genfromtxt
// raises and the reference falls back to pandas: return -1).  One row gives a 1-D array and no
// column gives none: both the reference's "data.ndim != 2" empty sweep (return 2).  Field counts
// other than 5 + bins: return 6 (fewer than 5 make data[:, 4] raise in the reference, det[0] = 5).
int32_t parse_genfromtxt(const std::string& buf, int32_t rows_cap, int32_t bins, int32_t dt,
                         void* echo_f, float* scale_f, float* angle_f, int64_t* det,
                         std::vector<std::pair<const char*, const char*>>& lines) {
  lines.clear();
  const char* p = buf.data();
  const char* e = p + buf.size();
  const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(e - p)));
  p = nl ? nl + 1 : e;
  int64_t ncols = -1;
  while (p < e) {
    const char* q = static_cast<const char*>(std::memchr(p, '\n', (size_t)(e - p)));
    const char* le = q ? q : e;
    const char* hc = static_cast<const char*>(std::memchr(p, '#', (size_t)(le - p)));
    const char* lt = hc ? hc : le;
    if (!is_blank_line(p, lt)) {
      int64_t nf = 1;
      for (const char* c = p; (c = static_cast<const char*>(std::memchr(c, ',', (size_t)(lt - c)))); ++c)
        ++nf;
      if (ncols < 0) ncols = nf;
      if (nf != ncols) return -1;  // genfromtxt: "Line #k (got m columns instead of n)"
      lines.push_back({p, lt});
    }
    p = q ? q + 1 : e;
  }
  const int64_t R = (int64_t)lines.size();
  if (R <= 1 || ncols <= 1) return 2;
  if (ncols < kMeta) {
    det[0] = 5;
    det[1] = ncols;
    return 1;
  }
  if (ncols != kMeta + bins) {  // another bin count: the caller re-parses with ncols - 5 bins
    det[1] = ncols;
    return 6;
  }
  if (R > rows_cap) return 6;
  for (int64_t r = 0; r < R; ++r) {
    const char* a = lines[(size_t)r].first;
    const char* le = lines[(size_t)r].second;
    uint8_t* e8 = static_cast<uint8_t*>(echo_f) + (size_t)r * bins;
    float* e32 = static_cast<float*>(echo_f) + (size_t)r * bins;
    for (int64_t f = 0; f < ncols; ++f) {
      const char* c = static_cast<const char*>(std::memchr(a, ',', (size_t)(le - a)));
      const char* fe = c ? c : le;
      double v = 0.0;
      if (!py_float(a, fe, &v)) v = 0.0;  // filling_values
      if (f >= kMeta) {
        if (dt == RPT_ECHO_U8) {
          if (!(v >= 0.0 && v <= 255.0 && v == std::floor(v))) return 3;
          e8[f - kMeta] = (uint8_t)v;
        } else {
          e32[f - kMeta] = (float)v;
        }
      } else if (f == 1) {
        scale_f[r] = (float)v;
      } else if (f == 4) {
        angle_f[r] = (float)v;
      }
      a = c ? c + 1 : le;
    }
  }
  return 0;
}

// status: 0 ok, 1 unreadable / tokenizing error (empty sweep), 2 no data row (df.empty),
// 3 a value not representable in u8 (the caller re-parses as float32), 4 non-numeric value.
// det[5]: {kind (0 none, 1 I/O error, 2 tokenizing error, 3 non-numeric value, 5 genfromtxt
// rows of fewer than 5 fields), errno | expected fields | field index | field count,
// physical line, fields seen, gain flags (bit 0 first-row Gain NaN, bit 1 rows disagree)}
constexpr int kDetail = 5;
int32_t parse_one(const char* path, int32_t rows_cap, int32_t bins, int32_t dt, void* echo_f,
                  float* scale_f, float* angle_f, float* gain_f, std::string& buf,
                  std::vector<std::pair<const char*, const char*>>& lines,
                  std::vector<int64_t>& lineno, int64_t* det, int32_t mode) {
  const size_t row_bytes = (size_t)bins * (dt == RPT_ECHO_U8 ? 1 : 4);
  auto zero_tail = [&](int64_t from) {
    if (from >= rows_cap) return;
    std::memset(static_cast<char*>(echo_f) + (size_t)from * row_bytes, 0,
                (size_t)(rows_cap - from) * row_bytes);
    for (int64_t r = from; r < rows_cap; ++r) scale_f[r] = angle_f[r] = 0.0f;
  };
  *gain_f = 0.0f;
  for (int k = 0; k < kDetail; ++k) det[k] = 0;
  int err = 0;
  if (!read_file(path, buf, &err)) {
    det[0] = 1;
    det[1] = err;
    zero_tail(0);
    return 1;
  }
  if (mode == 1) {  // genfromtxt first; pandas when it raises (inconsistent field counts)
    const int32_t gs = parse_genfromtxt(buf, rows_cap, bins, dt, echo_f, scale_f, angle_f, det,
                                        lines);
    if (gs >= 0) {
      if (gs == 0) {
        zero_tail((int64_t)lines.size());
      } else {
        zero_tail(0);
        if (gs == 2) lines.clear();
      }
      return gs;
    }
  }
  data_lines(buf, lines, &lineno);
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
      if (f >= n_fields + skip) {  // "Expected 1029 fields in line L, saw S": read_csv raises
        int64_t saw = f + 1;
        for (const char* q = fe; q < e && (q = static_cast<const char*>(
                                               std::memchr(q, ',', (size_t)(e - q))));
             ++q)
          ++saw;
        det[0] = 2;
        det[1] = n_fields + skip;
        det[2] = lineno[(size_t)r];
        det[3] = saw;
        zero_tail(0);
        return 1;
      }
      if (f < skip) {  // index columns
        ++f;
        if (!c) break;
        p = c + 1;
        continue;
      }
      double v = 0.0;
      const FieldKind k = parse_field(p, fe, &v);
      // read_csv mode: the tracker never converts Status / Range (object columns are harmless
      // there) and reads Gain only through int(iloc[0]) / unique(): a text Gain counts as NaN
      const int fcol = f - skip;
      if (k == kBad && !(mode == 0 && (fcol == 0 || fcol == 2 || fcol == 3))) {
        // to_numpy(float32) of the object column(s): numpy converts column block by column
        // block, so the value it names is the first bad one of the LEFTMOST bad column
        int64_t bl = lineno[(size_t)r], bc = f;
        for (int64_t r2 = r + 1; r2 < (int64_t)lines.size() && bc > 0; ++r2) {
          const char* a2 = lines[(size_t)r2].first;
          const char* e2 = lines[(size_t)r2].second;
          for (int64_t f2 = 0; f2 < bc; ++f2) {
            const char* c2 = static_cast<const char*>(std::memchr(a2, ',', (size_t)(e2 - a2)));
            double v2;
            const int fc2 = (int)(f2 - skip);
            if (f2 >= skip && !(mode == 0 && (fc2 == 0 || fc2 == 2 || fc2 == 3)) &&
                parse_field(a2, c2 ? c2 : e2, &v2) == kBad) {
              bl = lineno[(size_t)r2];
              bc = f2;
              break;
            }
            if (!c2) break;
            a2 = c2 + 1;
          }
        }
        det[0] = 3;
        det[1] = bc;  // physical field index (implicit index columns included)
        det[2] = bl;
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
        if (r == 0) {
          *gain_f = gv;
          if (gv != gv) det[4] |= 1;
        } else if (!(gv == *gain_f) && !(gv != gv && (det[4] & 1))) {
          *gain_f = NAN;
          det[4] |= 2;
        }
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
                             int64_t* detail_out, int32_t mode, int32_t n_threads) {
  clear_error();
  if (n_files < 0 || rows_cap < 0 || bins <= 0 ||
      (echo_dtype != RPT_ECHO_U8 && echo_dtype != RPT_ECHO_F32) || mode < 0 || mode > 1 ||
      (n_files > 0 && (!paths || !echo || !scale || !angle || !gain_col || !status_out))) {
    set_error("rpt_csv_parse_sweeps: bad arguments");
    return RPT_EINVAL;
  }
  const size_t es = echo_dtype == RPT_ECHO_U8 ? 1 : 4;
  std::atomic<int32_t> next{0};
  auto work = [&]() {
    std::string buf;
    std::vector<std::pair<const char*, const char*>> lines;
    std::vector<int64_t> lineno;
    int64_t det_local[kDetail];
    for (;;) {
      const int32_t i = next.fetch_add(1);
      if (i >= n_files) return;
      status_out[i] = parse_one(
          paths[i], rows_cap, bins, echo_dtype,
          static_cast<char*>(echo) + (size_t)i * (size_t)rows_cap * (size_t)bins * es,
          scale + (size_t)i * rows_cap, angle + (size_t)i * rows_cap, gain_col + i, buf, lines,
          lineno, detail_out ? detail_out + (size_t)i * kDetail : det_local, mode);
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
