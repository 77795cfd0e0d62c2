// box_parse.cpp — multithreaded EMAN BOX parser with the exact acceptance rules of the
// reference's get_box_coords (reference repic/utils/common.py:71-114):
//
//   * text mode, universal newlines (\n, \r\n, \r); str.split() whitespace inside a line
//   * header: line 1 is skipped iff its first token is not a Python float (:79-80);
//     a line 1 with no token raises IndexError (caller: "skip micrograph")
//   * rows are zipped column-wise: the SHORTEST row must have exactly 5 tokens, else
//     ValueError (:81); extra tokens in longer rows are ignored
//   * x / y tokens that are not floats are dropped (:87-88); every weight must be a float
//     (ValueError otherwise, :89); len(x) != len(y) -> AssertionError (:96)
//   * coords = zip(x, y, w) (truncating); empty -> IndexError at coords[-1] (:112)
//   * sigmoid flag: min(weights) < 0 with NaN propagating like np.min (:92)
//
// Python float() grammar (sign, digits with single underscores between digits, optional
// fraction / exponent, inf / infinity / nan case-insensitively) is validated here and the
// value converted with the correctly-rounded strtod_l in the "C" locale (CPython's dtoa is
// also correctly rounded).  Files with any byte >= 0x80 are returned as FALLBACK so the
// host parses them with Python's own str/float semantics.
#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cfloat>
#include <cstring>
#include <cstdint>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>
#include <locale.h>
#include <string>
#include <thread>
#include <vector>

#include "../../include/repic_gc.h"

namespace {

struct FileResult {
  int status = RGC_PARSE_OK;
  bool sigmoid = false;
  std::vector<double> x, y, s;
};

inline bool is_space(unsigned char c) {
  return c == ' ' || c == '\t' || c == '\v' || c == '\f' || (c >= 0x1c && c <= 0x1f);
}
inline bool is_digit(unsigned char c) { return c >= '0' && c <= '9'; }

inline bool ieq(const char* p, size_t n, const char* lit) {
  const size_t m = std::strlen(lit);
  if (n != m) return false;
  for (size_t i = 0; i < n; ++i) {
    char c = p[i];
    if (c >= 'A' && c <= 'Z') c = (char)(c - 'A' + 'a');
    if (c != lit[i]) return false;
  }
  return true;
}

// digitpart ::= digit (["_"] digit)* ; returns digits consumed (0 if none), -1 if malformed
inline int digitpart(const char* p, size_t n, size_t& i) {
  int d = 0;
  while (i < n) {
    if (is_digit((unsigned char)p[i])) {
      ++d;
      ++i;
    } else if (p[i] == '_' && d > 0 && i + 1 < n && is_digit((unsigned char)p[i + 1])) {
      ++i;
    } else {
      break;
    }
  }
  return d;
}

locale_t c_locale() {
  static locale_t loc = newlocale(LC_ALL_MASK, "C", (locale_t)0);
  return loc;
}

// Exact powers of ten 10^0 .. 10^27 in x87 extended precision (5^27 < 2^64: every one is exact)
// fast_decimal reads the 64-bit significand of the quotient from the low 8 bytes of the long
// double: only valid for the x87 80-bit format (a 64-bit or IEEE-quad long double would misparse)
static_assert(LDBL_MANT_DIG == 64 && sizeof(long double) >= 10,
              "box_parse.cpp's fast decimal path needs x87 80-bit long double");
struct Pow10L {
  long double v[28];
  Pow10L() {
    long double t = 1.0L;
    for (int i = 0; i < 28; ++i, t *= 10.0L) v[i] = t;
  }
};
const Pow10L kPow10L;

// Fast path of Python float() for the tokens BOX files are made of: [sign] digits [. digits]
// with at most 19 significant digits and 27 fraction digits (no exponent, no underscores).
// m / 10^f is computed in x87 extended precision (64-bit significand: m and 10^f are exact, so
// the quotient is correctly rounded to 64 bits) and then rounded to double.  That double
// rounding equals the correctly rounded result unless the 64-bit quotient lies within one unit
// of a double rounding midpoint (its low 11 significand bits 0x3FF..0x401): those, and every
// other shape, return false and take the strtod path.
inline bool fast_decimal(const char* p, size_t n, double* out) {
  size_t i = 0;
  bool neg = false;
  if (i < n && (p[i] == '+' || p[i] == '-')) neg = p[i++] == '-';
  uint64_t m = 0;
  int digits = 0, frac = 0;
  bool any = false, dot = false;
  for (; i < n; ++i) {
    const unsigned char c = (unsigned char)p[i];
    if (c >= '0' && c <= '9') {
      any = true;
      if (digits > 0 || c != '0') {
        if (++digits > 19) return false;
      }
      m = m * 10 + (c - '0');
      if (dot && ++frac > 27) return false;
    } else if (c == '.' && !dot) {
      dot = true;
    } else {
      return false;   // exponent, underscore, letters: strtod path (or not a float at all)
    }
  }
  if (!any) return false;
  if (frac == 0 && m < (1ULL << 53)) {
    const double d = (double)m;
    *out = neg ? -d : d;
    return true;
  }
  const long double q = (long double)m / kPow10L.v[frac];
  if (frac > 0) {
    uint64_t sig;
    std::memcpy(&sig, &q, sizeof(sig));   // x87 extended: 64-bit significand in the low bytes
    const uint32_t low = (uint32_t)(sig & 0x7FF);
    if (low >= 0x3FF && low <= 0x401) return false;
  }
  const double d = (double)q;
  *out = neg ? -d : d;
  return true;
}

// Python float(token) for an ASCII token without whitespace.
bool py_float(const char* p, size_t n, double* out) {
  if (n == 0) return false;
  if (fast_decimal(p, n, out)) return true;
  size_t i = 0;
  bool neg = false;
  if (p[0] == '+' || p[0] == '-') {
    neg = p[0] == '-';
    i = 1;
  }
  const char* r = p + i;
  const size_t rn = n - i;
  if (ieq(r, rn, "inf") || ieq(r, rn, "infinity")) {
    *out = neg ? -INFINITY : INFINITY;
    return true;
  }
  if (ieq(r, rn, "nan")) {
    *out = neg ? -NAN : NAN;
    return true;
  }
  size_t j = i;
  const int di = digitpart(p, n, j);
  int df = 0;
  if (j < n && p[j] == '.') {
    ++j;
    df = digitpart(p, n, j);
  }
  if (di + df == 0) return false;
  if (j < n && (p[j] == 'e' || p[j] == 'E')) {
    ++j;
    if (j < n && (p[j] == '+' || p[j] == '-')) ++j;
    if (digitpart(p, n, j) == 0) return false;
  }
  if (j != n) return false;
  char buf[128];
  std::string big;
  char* dst = buf;
  if (n >= sizeof(buf)) {
    big.resize(n + 1);
    dst = &big[0];
  }
  size_t w = 0;
  for (size_t q = 0; q < n; ++q)
    if (p[q] != '_') dst[w++] = p[q];
  dst[w] = 0;
  *out = strtod_l(dst, nullptr, c_locale());
  return true;
}

struct Tok {
  const char* p;
  size_t n;
};

// Split one line into tokens; returns the token count, keeps the first 5.
inline int split5(const char* b, const char* e, Tok* t) {
  int cnt = 0;
  const char* q = b;
  while (q < e) {
    while (q < e && is_space((unsigned char)*q)) ++q;
    if (q >= e) break;
    const char* s = q;
    while (q < e && !is_space((unsigned char)*q)) ++q;
    if (cnt < 5) t[cnt] = Tok{s, (size_t)(q - s)};
    ++cnt;
  }
  return cnt;
}

struct Row {
  Tok x, y, w;
};

void parse_one(const char* path, FileResult& R) {
  const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    R.status = RGC_PARSE_OSERROR;
    return;
  }
  // one read of the whole file (sized by fstat; grown if the file is longer than reported)
  thread_local std::string data;
  struct stat stt;
  size_t cap = (::fstat(fd, &stt) == 0 && stt.st_size > 0) ? (size_t)stt.st_size + 1 : 1 << 16;
  data.resize(cap);
  size_t len = 0;
  bool err = false;
  for (;;) {
    if (len == data.size()) data.resize(2 * data.size());
    const ssize_t got = ::read(fd, &data[len], data.size() - len);
    if (got < 0) {
      if (errno == EINTR) continue;
      err = true;
      break;
    }
    if (got == 0) break;
    len += (size_t)got;
  }
  ::close(fd);
  if (err) {
    R.status = RGC_PARSE_OSERROR;
    return;
  }
  data.resize(len);
  {
    // any byte >= 0x80 (8 bytes per step)
    const char* q = data.data();
    const size_t nb = data.size();
    uint64_t acc = 0;
    size_t i = 0;
    for (; i + 8 <= nb; i += 8) {
      uint64_t w;
      std::memcpy(&w, q + i, 8);
      acc |= w;
    }
    for (; i < nb; ++i) acc |= (unsigned char)q[i];
    if (acc & 0x8080808080808080ULL) {
      R.status = RGC_PARSE_FALLBACK;
      return;
    }
  }
  const char* p = data.data();
  const char* end = p + data.size();
  // universal-newline line iterator (memchr for '\n' when the file has no '\r')
  const bool has_cr = std::memchr(p, '\r', data.size()) != nullptr;
  auto next_line = [&](const char*& cur, const char*& lb, const char*& le) -> bool {
    if (cur >= end) return false;
    lb = cur;
    const char* q;
    if (!has_cr) {
      q = static_cast<const char*>(std::memchr(cur, '\n', (size_t)(end - cur)));
      if (!q) q = end;
    } else {
      q = cur;
      while (q < end && *q != '\n' && *q != '\r') ++q;
    }
    le = q;
    if (q < end) {
      if (*q == '\r' && q + 1 < end && q[1] == '\n') q += 2;
      else q += 1;
    }
    cur = q;
    return true;
  };
  const char* cur = p;
  const char *lb, *le;
  Tok t[5];
  double v;
  // header check on line 1 (an empty file / blank first line -> IndexError)
  if (!next_line(cur, lb, le) || split5(lb, le, t) == 0) {
    R.status = RGC_PARSE_INDEX;
    return;
  }
  if (py_float(t[0].p, t[0].n, &v)) cur = p;  // f.seek(0)
  thread_local std::vector<Row> rows;
  rows.clear();
  int min_tok = 1 << 30;
  while (next_line(cur, lb, le)) {
    const int c = split5(lb, le, t);
    min_tok = std::min(min_tok, c);
    if (c >= 5) rows.push_back(Row{t[0], t[1], t[4]});
    else rows.push_back(Row{Tok{nullptr, 0}, Tok{nullptr, 0}, Tok{nullptr, 0}});
  }
  if (rows.empty() || min_tok != 5) {
    R.status = RGC_PARSE_VALUE;  // zip(*rows) does not unpack into 5 columns
    return;
  }
  std::vector<double> X, Y, W;
  X.reserve(rows.size());
  Y.reserve(rows.size());
  W.reserve(rows.size());
  for (const Row& r : rows) {
    if (py_float(r.x.p, r.x.n, &v)) X.push_back(v);
    if (py_float(r.y.p, r.y.n, &v)) Y.push_back(v);
  }
  bool any_nan = false;
  double mn = INFINITY;
  for (const Row& r : rows) {
    if (!py_float(r.w.p, r.w.n, &v)) {
      R.status = RGC_PARSE_VALUE;  // float(weight) raises
      return;
    }
    if (std::isnan(v)) any_nan = true;
    mn = std::min(mn, v);
    W.push_back(v);
  }
  R.sigmoid = !any_nan && mn < 0;
  if (X.size() != Y.size()) {
    R.status = RGC_PARSE_ASSERT;
    return;
  }
  const size_t nn = std::min(X.size(), W.size());
  if (nn == 0) {
    R.status = RGC_PARSE_INDEX;
    return;
  }
  X.resize(nn);
  Y.resize(nn);
  W.resize(nn);
  R.x.swap(X);
  R.y.swap(Y);
  R.s.swap(W);
}

}  // namespace

extern "C" {

int rgc_parse_files(const char* const* paths, int64_t n_files, int n_threads, rgc_parsed** out) {
  *out = nullptr;
  std::vector<FileResult> res((size_t)n_files);
  std::atomic<int64_t> next{0};
  auto worker = [&]() {
    for (;;) {
      const int64_t i = next.fetch_add(1);
      if (i >= n_files) break;
      parse_one(paths[i], res[(size_t)i]);
    }
  };
  if (n_threads < 1) n_threads = 1;
  n_threads = (int)std::min<int64_t>(n_threads, std::max<int64_t>(1, n_files));
  std::vector<std::thread> th;
  for (int t = 1; t < n_threads; ++t) th.emplace_back(worker);
  worker();
  for (auto& t : th) t.join();

  rgc_parsed* P = (rgc_parsed*)std::calloc(1, sizeof(rgc_parsed));
  P->n_files = n_files;
  P->status = (int32_t*)std::malloc(sizeof(int32_t) * (n_files + 1));
  P->off = (int64_t*)std::malloc(sizeof(int64_t) * (n_files + 1));
  P->sigmoid = (uint8_t*)std::malloc(n_files + 1);
  int64_t tot = 0;
  for (int64_t i = 0; i < n_files; ++i) {
    P->off[i] = tot;
    P->status[i] = res[i].status;
    P->sigmoid[i] = res[i].sigmoid ? 1 : 0;
    tot += (int64_t)res[i].x.size();
  }
  P->off[n_files] = tot;
  P->x = (double*)std::malloc(sizeof(double) * (tot + 1));
  P->y = (double*)std::malloc(sizeof(double) * (tot + 1));
  P->score = (double*)std::malloc(sizeof(double) * (tot + 1));
  for (int64_t i = 0; i < n_files; ++i) {
    const size_t nn = res[i].x.size();
    if (!nn) continue;
    std::memcpy(P->x + P->off[i], res[i].x.data(), nn * 8);
    std::memcpy(P->y + P->off[i], res[i].y.data(), nn * 8);
    std::memcpy(P->score + P->off[i], res[i].s.data(), nn * 8);
  }
  *out = P;
  return 0;
}

void rgc_parsed_free(rgc_parsed* P) {
  if (!P) return;
  std::free(P->status);
  std::free(P->off);
  std::free(P->sigmoid);
  std::free(P->x);
  std::free(P->y);
  std::free(P->score);
  std::free(P);
}

}  // extern "C"
