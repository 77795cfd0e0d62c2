// out_write.cpp — native writer of get_cliques' per-micrograph output files.
//
// Reference get_cliques.py:204-229: per micrograph
//   <base>_weight_vector.pickle          numpy float32 [C]
//   <base>_consensus_coords.pickle       list of C (x: float, y: float, id: int) tuples
//   <base>_consensus_confidences.pickle  numpy float32 [C]
//   <base>_constraint_matrix.pickle      scipy.sparse coo_matrix, int64 ones at
//                                        (rows int32, cols int32), shape (V, C)
//   <base>_runtime.tsv                   "seconds\tlargest CC\tnumber of CCs\n"
// all pickled with pickle.HIGHEST_PROTOCOL (5).  The pickles are emitted opcode by opcode in
// the layout CPython's C pickler gives these objects (the numpy _frombuffer reduction with an
// in-band BYTEARRAY8 buffer, the coo_matrix __dict__ state, memo numbering included), without
// the optional FRAME opcodes.  The module / class names come from the installed numpy and
// scipy (rgc_pickle_fmt), and repic_amd/writers.py only enables this writer after comparing its
// bytes with pickle.dumps of the same objects (frame stripped); the unchanged consumer
// (run_ilp.py:29-80) unpickles identical objects.  No GIL, no interpreter per file: threads
// write whole micrographs.
#include <cerrno>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fcntl.h>
#include <string>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

#include "../../include/repic_gc.h"

namespace {

struct Out {
  std::string b;
  int memo = 0;
  void op(uint8_t c) { b.push_back((char)c); }
  void memoize() { op(0x94); ++memo; }
  void u8(uint8_t v) { op(v); }
  void le(uint64_t v, int n) {
    for (int i = 0; i < n; ++i) op((uint8_t)(v >> (8 * i)));
  }
  void str(const char* s) {   // SHORT_BINUNICODE + MEMOIZE
    const size_t n = strlen(s);
    op(0x8c);
    op((uint8_t)n);
    b.append(s, n);
    memoize();
  }
  void get(int idx) {   // BINGET / LONG_BINGET
    if (idx < 256) { op('h'); op((uint8_t)idx); }
    else { op('j'); le((uint32_t)idx, 4); }
  }
  // save_long of CPython's C pickler (protocol >= 2)
  void integer(int64_t v) {
    if (v >= 0 && v <= 0xff) { op('K'); op((uint8_t)v); }
    else if (v >= 0 && v <= 0xffff) { op('M'); le((uint64_t)v, 2); }
    else if (v >= -0x80000000LL && v <= 0x7fffffffLL) { op('J'); le((uint32_t)(int32_t)v, 4); }
    else {
      // LONG1: little-endian two's complement, (bit_length >> 3) + 1 bytes
      const uint64_t mag = v < 0 ? (uint64_t)(-(v + 1)) : (uint64_t)v;
      int nbits = 0;
      for (uint64_t m = mag; m; m >>= 1) ++nbits;
      int nb = (nbits >> 3) + 1;
      op(0x8a);
      op((uint8_t)nb);
      le((uint64_t)v, nb);
    }
  }
  void binfloat(double d) {   // BINFLOAT: big-endian IEEE double
    uint64_t u;
    memcpy(&u, &d, 8);
    op('G');
    for (int i = 7; i >= 0; --i) op((uint8_t)(u >> (8 * i)));
  }
};

// memo slots of the objects an array pickle can refer back to
struct ArrMemo {
  int fb = -1;       // _frombuffer global
  int dcls = -1;     // numpy.dtype class
  int lt = -1;       // '<'
  int corder = -1;   // 'C'
};

// numpy array (1-D, little-endian, C order) as numpy's __reduce_ex__(5) pickles it:
// _frombuffer(bytearray, dtype(code), (n,), 'C').  dtype_memo: memo slot of an identical dtype
// object pickled earlier in the same stream (numpy dtypes are singletons), or -1.
void save_array(Out& o, const rgc_pickle_fmt& f, ArrMemo& am, const void* data, int64_t n,
                int esize, const char* code, int* dtype_memo) {
  if (am.fb < 0) {
    o.str(f.arr_mod);
    o.str(f.arr_fn);
    o.op(0x93);   // STACK_GLOBAL
    o.memoize();
    am.fb = o.memo - 1;
  } else {
    o.get(am.fb);
  }
  o.op('(');   // MARK
  o.op(0x96);  // BYTEARRAY8
  o.le((uint64_t)(n * esize), 8);
  o.b.append(reinterpret_cast<const char*>(data), (size_t)(n * esize));
  o.memoize();
  if (*dtype_memo >= 0) {
    o.get(*dtype_memo);
  } else {
    if (am.dcls < 0) {
      o.str(f.dtype_mod);
      o.str(f.dtype_cls);
      o.op(0x93);
      o.memoize();
      am.dcls = o.memo - 1;
    } else {
      o.get(am.dcls);
    }
    o.str(code);
    o.op(0x89);   // NEWFALSE
    o.op(0x88);   // NEWTRUE
    o.op(0x87);   // TUPLE3
    o.memoize();
    o.op('R');
    o.memoize();
    *dtype_memo = o.memo - 1;
    // dtype state (3, '<', None, None, None, -1, -1, 0)
    o.op('(');
    o.integer(3);
    if (am.lt < 0) {
      o.str("<");
      am.lt = o.memo - 1;
    } else {
      o.get(am.lt);
    }
    o.op('N'); o.op('N'); o.op('N');
    o.integer(-1);
    o.integer(-1);
    o.integer(0);
    o.op('t');
    o.memoize();
    o.op('b');    // BUILD
  }
  o.integer(n);
  o.op(0x85);   // TUPLE1
  o.memoize();
  if (am.corder < 0) {
    o.str("C");
    am.corder = o.memo - 1;
  } else {
    o.get(am.corder);
  }
  o.op('t');
  o.memoize();
  o.op('R');
  o.memoize();
}

void begin(Out& o) {
  o.b.clear();
  o.memo = 0;
  o.op(0x80);
  o.op(5);
}

void pickle_f32(Out& o, const rgc_pickle_fmt& f, const float* v, int64_t n) {
  begin(o);
  ArrMemo am;
  int dm = -1;
  save_array(o, f, am, v, n, 4, "f4", &dm);
  o.op('.');
}

void pickle_coords(Out& o, const double* x, const double* y, const int64_t* id, int64_t n) {
  begin(o);
  o.op(']');   // EMPTY_LIST
  o.memoize();
  auto item = [&](int64_t i) {
    o.binfloat(x[i]);
    o.binfloat(y[i]);
    o.integer(id[i]);
    o.op(0x87);
    o.memoize();
  };
  if (n == 1) {
    item(0);
    o.op('a');   // APPEND
  } else if (n > 1) {
    for (int64_t s = 0; s < n; s += 1000) {   // the pickler's batches of 1000
      o.op('(');
      for (int64_t i = s; i < std::min<int64_t>(n, s + 1000); ++i) item(i);
      o.op('e');   // APPENDS
    }
  }
  o.op('.');
}

// coo_matrix((int64 ones, (rows, cols)), shape=(V, C)) with cols = j repeated k times
void pickle_coo(Out& o, const rgc_pickle_fmt& f, const int32_t* rows, int64_t C, int k,
                int64_t V, std::vector<int32_t>& colbuf, std::vector<int64_t>& onebuf) {
  const int64_t nnz = C * k;
  colbuf.resize((size_t)nnz);
  onebuf.assign((size_t)nnz, 1);
  for (int64_t j = 0; j < C; ++j)
    for (int i = 0; i < k; ++i) colbuf[(size_t)(j * k + i)] = (int32_t)j;
  begin(o);
  o.str(f.coo_mod);
  o.str(f.coo_cls);
  o.op(0x93);
  o.memoize();
  o.op(')');    // EMPTY_TUPLE
  o.op(0x81);   // NEWOBJ
  o.memoize();
  o.op('}');    // EMPTY_DICT
  o.memoize();
  o.op('(');
  o.str("_shape");
  o.integer(V);
  o.integer(C);
  o.op(0x86);   // TUPLE2
  o.memoize();
  o.str("maxprint");
  o.integer(f.maxprint);
  o.str("coords");
  ArrMemo am;
  int d32 = -1, d64 = -1;
  save_array(o, f, am, rows, nnz, 4, "i4", &d32);
  save_array(o, f, am, colbuf.data(), nnz, 4, "i4", &d32);
  o.op(0x86);
  o.memoize();
  o.str("data");
  save_array(o, f, am, onebuf.data(), nnz, 8, "i8", &d64);
  o.str("has_canonical_format");
  o.op(0x89);
  o.op('u');    // SETITEMS
  o.op('b');    // BUILD
  o.op('.');
}

// str(float) of CPython (repr, 'r' format with ADD_DOT_0): shortest round-trip digits; fixed
// notation when -4 < decimal exponent <= 16, else d[.ddd]e+XX
std::string py_float(double v) {
  if (std::isnan(v)) return "nan";
  if (std::isinf(v)) return v > 0 ? "inf" : "-inf";
  char buf[64];
  auto r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::scientific);
  std::string s(buf, r.ptr);
  const size_t e = s.find('e');
  std::string mant = s.substr(0, e);
  const int ex = atoi(s.c_str() + e + 1);
  bool neg = false;
  if (!mant.empty() && mant[0] == '-') { neg = true; mant.erase(0, 1); }
  std::string dig;
  for (char ch : mant)
    if (ch != '.') dig.push_back(ch);
  const int decpt = ex + 1;   // value = 0.DIGITS x 10^decpt
  std::string out;
  if (decpt > -4 && decpt <= 16) {
    if (decpt <= 0) {
      out = "0." + std::string((size_t)(-decpt), '0') + dig;
    } else if ((int)dig.size() <= decpt) {
      out = dig + std::string((size_t)(decpt - (int)dig.size()), '0') + ".0";
    } else {
      out = dig.substr(0, (size_t)decpt) + "." + dig.substr((size_t)decpt);
    }
  } else {
    out = dig.substr(0, 1);
    if (dig.size() > 1) out += "." + dig.substr(1);
    char eb[16];
    snprintf(eb, sizeof(eb), "e%c%02d", ex < 0 ? '-' : '+', ex < 0 ? -ex : ex);
    out += eb;
  }
  return neg ? "-" + out : out;
}

int write_file(const std::string& path, const std::string& data) {
  const int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0666);
  if (fd < 0) return -errno;
  size_t off = 0;
  while (off < data.size()) {
    const ssize_t w = write(fd, data.data() + off, data.size() - off);
    if (w < 0) {
      if (errno == EINTR) continue;
      const int e = -errno;
      close(fd);
      return e;
    }
    off += (size_t)w;
  }
  return close(fd) == 0 ? 0 : -errno;
}

const char* const kLabels[4] = {"weight_vector", "consensus_coords", "consensus_confidences",
                                "constraint_matrix"};

// one micrograph's pickle `which` (0..3, kLabels order) into o
void pickle_one(Out& o, const rgc_pickle_fmt& f, const rgc_write_in& in, int m, int which,
                std::vector<int32_t>& colbuf, std::vector<int64_t>& onebuf) {
  const int64_t c0 = in.clique_off[m], C = in.clique_off[m + 1] - c0;
  switch (which) {
    case 0: pickle_f32(o, f, in.w + c0, C); break;
    case 1: pickle_coords(o, in.cx + c0, in.cy + c0, in.cid + c0, C); break;
    case 2: pickle_f32(o, f, in.conf + c0, C); break;
    default: pickle_coo(o, f, in.rows + c0 * in.k, C, in.k, in.n_vert[m], colbuf, onebuf);
  }
}

}  // namespace

extern "C" int rgc_pickle_bytes(const rgc_pickle_fmt* fmt, const rgc_write_in* in, int mg,
                                int which, uint8_t* buf, int64_t cap, int64_t* len) {
  if (!fmt || !in || mg < 0 || mg >= in->n_mg || which < 0 || which > 3) return -1;
  Out o;
  std::vector<int32_t> cb;
  std::vector<int64_t> ob;
  pickle_one(o, *fmt, *in, mg, which, cb, ob);
  *len = (int64_t)o.b.size();
  if (buf && cap >= *len) memcpy(buf, o.b.data(), o.b.size());
  return 0;
}

extern "C" int rgc_write_outputs(const rgc_pickle_fmt* fmt, const rgc_write_in* in, int n_threads,
                                 int64_t* failed_mg) {
  if (!fmt || !in || !in->out_dir) return -1;
  const int n = in->n_mg;
  if (failed_mg) *failed_mg = -1;
  const int nt = std::max(1, std::min(n_threads, n));
  std::vector<int> err((size_t)nt, 0);
  std::vector<int64_t> bad((size_t)nt, -1);
  const std::string dir = std::string(in->out_dir) + "/";
  auto work = [&](int t) {
    Out o;
    std::vector<int32_t> cb;
    std::vector<int64_t> ob;
    // contiguous ranges: the first failing micrograph of the lowest range is the first overall
    const int m0 = (int)((int64_t)n * t / nt), m1 = (int)((int64_t)n * (t + 1) / nt);
    for (int m = m0; m < m1; ++m) {
      const std::string base = dir + in->bases[m];
      int e = 0;
      for (int which = 0; which < 4 && !e; ++which) {
        pickle_one(o, *fmt, *in, m, which, cb, ob);
        e = write_file(base + "_" + kLabels[which] + ".pickle", o.b);
      }
      if (!e) {
        const std::string tsv = py_float(in->seconds[m]) + "\t" + std::to_string(in->cc_max[m]) +
                                "\t" + std::to_string(in->cc_cnt[m]) + "\n";
        e = write_file(base + "_runtime.tsv", tsv);
      }
      if (e) {
        err[(size_t)t] = e;
        bad[(size_t)t] = m;
        return;
      }
    }
  };
  if (nt == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back(work, t);
    for (auto& x : th) x.join();
  }
  for (int t = 0; t < nt; ++t)
    if (err[(size_t)t]) {
      if (failed_mg) *failed_mg = bad[(size_t)t];
      return err[(size_t)t];
    }
  return 0;
}

extern "C" int rgc_py_float_repr(double v, char* buf, int cap) {
  const std::string s = py_float(v);
  if ((int)s.size() + 1 > cap) return -1;
  memcpy(buf, s.c_str(), s.size() + 1);
  return (int)s.size();
}
