// rgc_fused.hip — the whole get_cliques hot path for one micrograph in ONE workgroup.
//
// Everything between reading a micrograph's boxes and writing its ILP structures stays in
// LDS: boxes (f32 or f64 x/y), one uniform grid per picker, the forward adjacency CSR (u16
// targets), union-find, the clique DFS and the vertex ranks.  Graph nodes are the boxes'
// SORTED POSITIONS (picker-major grid order, local index order inside a cell): stencil
// ranges then yield every forward list already sorted, and all per-node arrays are indexed
// by position; local (file-order) indices only enter where the reference orders by box id.  HBM sees
// the compulsory traffic only: 16 B/box of coordinates in, 8 B per clique member of scores
// in (gathered), and C*(4k + 12) bytes of clique outputs out.  No global scans, no
// mid-pipeline host syncs, no global atomics except one clique-range reservation per
// micrograph.  Micrographs whose boxes/edges do not fit the launch's LDS capacities are
// returned with status DEFER and run through the multi-kernel path (rgc_kernels.hip).
//
// Phases (barrier-separated), reference repic/commands/get_cliques.py:
//   P0 load x, y; bounding box
//   P1 grid + LDS counting sort by cell                       (pair loop structure :62-63)
//   P2 JI pairs: count -> scan -> fill, sort each list        (:40-46, :59-69, :138)
//   P3 union-find, CC stats, --get_cc target                  (:145-156)
//   P4 k-clique DFS count, mark vertices, reserve outputs    (:49-56, :160-161)
//   P5 vertex rank by (x, y, id) via x-major grid columns    (:164, :193)
//   P6 clique DFS fill + epilogue + COO rows                 (:169-202)
#pragma clang fp contract(off)

#include <type_traits>

#ifdef RGC_STAMPS
// Diagnostic build only: every workgroup barrier of this file (and of the rgc_device.h scans
// it inlines) adds the cycles each wave waits in it to that wave's counter, read and reset by
// STAMP at each phase end, so a phase's barrier-wait share (waves idle behind the slowest
// wave of the workgroup) separates from its other stalls.
#include <hip/hip_runtime.h>
namespace rgc {
__shared__ unsigned long long g_bwait[16];
__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__device__ __forceinline__ void timed_barrier() {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  raw_barrier();
  if ((threadIdx.x & 63) == 0) g_bwait[threadIdx.x >> 6] += __builtin_amdgcn_s_memtime() - t0;
}
}  // namespace rgc
#define __syncthreads() ::rgc::timed_barrier()
#endif

#include "rgc_device.h"
#include "rgc_kernels.h"

namespace rgc {

constexpr int MAXW = 16;            // reduction slots: up to 1024-thread workgroups
// Workgroup sizes compiled: 512 for every k; 768 / 1024 threads (12 / 16 waves) for k <= 5,
// launched when LDS allows few workgroups per CU but VGPRs allow more waves (rgc_abi.cpp);
// 256 threads for k <= 3 (fewer per-wave fixed costs per micrograph, fewer resident waves).
// boxes per thread kept in registers from P0 to P1: 2 (4 with 256-thread workgroups; 5 with
// 1024: C3's ~4.1k boxes all stay in registers, VGPRs to spare at 4 waves per SIMD; boxes past
// RB * NT are re-read from HBM in each of P0's and P1's passes)
constexpr int fused_rb(int nt) { return nt <= 256 ? 4 : nt >= 1024 ? 5 : 2; }

struct FusedHdr {
  // reduction scratch: the single-value reductions alias the 4-way one (every reduction
  // starts behind a barrier)
  union {
    struct {
      double redd[MAXW];
      int64_t red64[MAXW];
      uint64_t redu[MAXW];
      int redi[MAXW];
    };
    double red4[4][MAXW];
  };
  double minx, miny, cell, inv_cell, inv_celly;
  double xbs;       // P5 x-bucket scale: bucket(x) = min(trunc((x - minx) * xbs), n - 1)
  float inv_gy;
  int gx, gy, ncell, nkey;   // per-picker grid gx x gy; keys picker * ncell + cell; nkey = none
  int E, nodes, cc_cnt, cc_max, target, V, status;
  uint32_t ccur;    // P4 clique-queue cursor
  int tief[2];      // P6: some clique of the chunk needs the order pass (by chunk parity)
  int qslot;        // QG (K = 4): the workgroup's HBM level-tree slot (-1: none, LDS queue)
  int64_t C, base;
};

// cell budget (keys over all pickers' grids) of a size class: 4 n up to 2048 boxes; 2 n above,
// where LDS is the limit (one workgroup per CU) and larger cells only cost P2 candidates
__host__ __device__ inline int fused_cells(int nmax) { return nmax <= 2048 ? 4 * nmax : 2 * nmax; }

// wide: f64 coordinates in LDS; otherwise f32 (every coordinate of the micrograph is exactly
// representable as f32, checked in P0, so the f64 values are recovered exactly)
__host__ __device__ inline FusedLayout fused_layout(int nmax, int ecap, bool wide) {
  FusedLayout L;
  auto al = [](int v) { return (v + 15) & ~15; };
  int o = al((int)sizeof(FusedHdr));
  // live until the end of the kernel
  L.off_sxy = o; o += al((wide ? 16 : 8) * nmax);   // (x, y) in cell-sorted order
  L.off_cnt = o; o += al(4 * (nmax + 4));
  L.off_fwd = o; o += al(2 * (nmax + 4));     // u16 CSR offsets (E <= ecap <= 65535)
  L.off_pos = o; o += al(2 * nmax);           // local box index -> sorted position
  L.off_vrank = o; o += al(2 * nmax);
  L.off_dst = o; o += al(2 * ecap);
  // P1-P3 grid and union-find; the cell starts (dead after P2) become the clique buffer of
  // P4-P6, parent..scell (dead after P5) the f64 scores of P6
  L.off_union = o;
  L.off_cstart = o; o += al(2 * (fused_cells(nmax) + 8));   // u16 cell starts
  L.off_parent = o; o += al(2 * (nmax + 8));    // u16 union-find parents; P5 u16 bucket counts
  L.off_scell = o; o += al(2 * nmax);         // sorted position -> cell
  L.off_citems = o; o += al(2 * nmax);        // sorted position -> local box index
  L.off_flags = o; o += al(nmax);             // by local index: 1 graph node, 3 clique vertex
  L.off_smark = o;
  L.total = o;
  L.off_cbuf = L.off_cstart;
  return L;
}

int fused_lds_bytes(int nmax, int ecap, bool wide) { return fused_layout(nmax, ecap, wide).total; }

struct FShared {
  void* sxy;        // cell-sorted coordinates: double2 (wide) or float2
  uint16_t* cstart;
  uint32_t* cnt;
  uint16_t* fwd;
  uint16_t* parent;
  uint16_t* citems;
  uint16_t* pos;
  uint16_t* scell;
  uint16_t* vrank;
  uint8_t* flags;   // by local index: 0 no edge, 1 graph node, 3 clique vertex
  uint16_t* dst;
  uint16_t* split;  // P3-P4 (scell region): end of each box's first picker segment in dst
  uint16_t* cbuf;   // P4-P6 (cell starts): clique queue, or the current chunk of the re-walk
  double* vscore;   // P6 (parent..scell, dead after P5): score of each clique vertex by row
                    // rank, used when 8 V bytes fit there (vstaged); else scores are
                    // gathered from HBM
  bool vstaged;
};

template <bool W>
__device__ __forceinline__ double2 ld_xy(const FShared& S, int t) {
  if constexpr (W) {
    return reinterpret_cast<const double2*>(S.sxy)[t];
  } else {
    const float2 f = reinterpret_cast<const float2*>(S.sxy)[t];
    return make_double2((double)f.x, (double)f.y);
  }
}
template <bool W>
__device__ __forceinline__ void st_xy(const FShared& S, int t, double x, double y) {
  if constexpr (W) reinterpret_cast<double2*>(S.sxy)[t] = make_double2(x, y);
  else reinterpret_cast<float2*>(S.sxy)[t] = make_float2((float)x, (float)y);
}

template <int K>
struct FCtx {
  // copies of the kernel arguments (taking the address of the kernarg struct would move it
  // to scratch)
  double B, two_b2;
  float Bf, two_b2f;   // (float) copies, wave-uniform (SGPRs)
  int flags;
  gptr<const double> score;
  gptr<int32_t> rows;
  gptr<float> w;
  gptr<float> conf;
  gptr<int32_t> consensus;
  gptr<int32_t> members;
  gptr<uint8_t> order;
  FShared S;
  int pb[K + 1];     // picker bounds (local box indices)
  int pp[K + 1];     // picker bounds (sorted positions; pp[K] = first non-finite box)
  int m, b0, n;
  int64_t idb;       // global id of local box 0
  bool set_order;    // networkx iterates set(sorted(clique)) (2k < |G|)
  int64_t out;       // next clique index within the micrograph (fill)
  int64_t c0, c1;    // clique chunk being buffered in cbuf (fill)
  int64_t count;
  uint16_t* cq_ord;  // P4 queue: ordinal of each queued clique within its root's DFS
  uint32_t* ccur;    // P4 queue cursor (LDS)
  int cq_cap;        // P4 queue capacity (cliques)
  gptr<int32_t> tie_list;         // set-order ties for k_fused_ties
  gptr<unsigned long long> tie_count;
  int64_t tie_cap;
};

__device__ __forceinline__ uint32_t lds_ld(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t p16_ld(uint16_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void p16_st(uint16_t* p, uint32_t v) {
  __hip_atomic_store(p, (uint16_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// u16 parents (positions < 2^16), path halving
__device__ __forceinline__ uint32_t uf_find_lds(uint16_t* parent, uint32_t x) {
  for (;;) {
    const uint32_t p = p16_ld(parent + x);
    if (p == x) return x;
    const uint32_t gp = p16_ld(parent + p);
    if (gp != p) p16_st(parent + x, gp);
    x = gp;
  }
}
// lock-free union (link the larger root under the smaller): CAS on the 32-bit word holding
// the root's u16 entry (a concurrent store to the other half only makes the CAS retry)
__device__ __forceinline__ void uf_union_lds(uint16_t* parent, uint32_t a, uint32_t b) {
  for (;;) {
    a = uf_find_lds(parent, a);
    b = uf_find_lds(parent, b);
    if (a == b) return;
    if (a < b) { const uint32_t t = a; a = b; b = t; }
    uint32_t* wp = reinterpret_cast<uint32_t*>(parent) + (a >> 1);
    const int sh = 16 * (a & 1);
    const uint32_t w = lds_ld(wp);
    if (((w >> sh) & 0xFFFFu) != a) continue;   // a was linked meanwhile
    const uint32_t nw = (w & ~(0xFFFFu << sh)) | (b << sh);
    if (atomicCAS(wp, w, nw) == w) return;
  }
}

// u32 parents (the dead P2 count words, see P2's union): path halving by plain stores (any
// ancestor is a valid parent, and parents only ever decrease), linking by atomicMin of the
// larger root's word to the smaller root - no CAS retry loop, no false conflicts between two
// u16 halves of one word.  If the larger root was linked meanwhile (old != a), its old parent
// and b are joined in turn (hooking as in ECL-CC).
__device__ __forceinline__ uint32_t uf_find32(uint32_t* parent, uint32_t x) {
  for (;;) {
    const uint32_t p = lds_ld(parent + x);
    if (p == x) return x;
    const uint32_t gp = lds_ld(parent + p);
    if (gp != p) lds_st(parent + x, gp);
    x = gp;
  }
}
__device__ __forceinline__ void uf_union32(uint32_t* parent, uint32_t a, uint32_t b) {
  for (;;) {
    a = uf_find32(parent, a);
    b = uf_find32(parent, b);
    if (a == b) return;
    if (a < b) { const uint32_t t = a; a = b; b = t; }
    const uint32_t old = atomicMin(parent + a, b);
    if (old == a) return;
    a = old;
  }
}

template <int K>
__device__ __forceinline__ int picker_of(const int (&pb)[K + 1], int i) {
  int p = 0;
#pragma unroll
  for (int q = 1; q < K; ++q) p += (i >= pb[q]);
  return p;
}
// first box index after box i's picker.  Written as sums of differences, never as a select
// between array elements: the optimiser folds such selects into a dynamically indexed load,
// which would move the whole context struct to scratch.
template <int K>
__device__ __forceinline__ int picker_end(const int (&pb)[K + 1], int i) {
  int e = pb[1];
#pragma unroll
  for (int q = 1; q < K; ++q) e += (i >= pb[q]) ? (pb[q + 1] - pb[q]) : 0;
  return e;
}
// end (in box index) of the picker after box i's picker: targets of box i below it form the
// first segment of i's forward list
template <int K>
__device__ __forceinline__ int next_picker_end(const int (&pb)[K + 1], int i) {
  int e = pb[K < 2 ? K : 2];
#pragma unroll
  for (int q = 1; q < K; ++q) e += (i >= pb[q]) ? (q + 2 <= K ? pb[q + 2] - pb[q + 1] : 0) : 0;
  return e;
}
template <int K>
__device__ __forceinline__ int picker_begin(const int (&pb)[K + 1], int p) {
  int b = pb[0];
#pragma unroll
  for (int q = 1; q < K; ++q) b += (p >= q) ? (pb[q] - pb[q - 1]) : 0;
  return b;
}

__device__ __forceinline__ int lb16(const uint16_t* a, int lo, int hi, int v) {
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((int)a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ bool contains16(const uint16_t* a, int lo, int hi, int v) {
  const int p = lb16(a, lo, hi, v);
  return p < hi && (int)a[p] == v;
}

// wave-uniform copies (SGPRs) of values every lane reads from the LDS header
__device__ __forceinline__ int ufl(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ float uff(float v) {
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v)));
}
__device__ __forceinline__ double ufd(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xFFFFFFFF));
  const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ int64_t ufl64(int64_t v) {
  const int lo = __builtin_amdgcn_readfirstlane((int)(v & 0xFFFFFFFF));
  const int hi = __builtin_amdgcn_readfirstlane((int)(v >> 32));
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// the micrograph's grid geometry, uniform across the workgroup
struct GridU {
  double minx, miny, inv_cell, inv_celly;   // columns >= 1.08 B wide, rows >= 0.54 B tall
  float inv_cellf;                          // (float)inv_cell: P2's half-column test
  float inv_gy;
  int gx, gy, ncell, nkey;
};
__device__ __forceinline__ GridU grid_u(const FusedHdr& H) {
  GridU G;
  G.minx = ufd(H.minx); G.miny = ufd(H.miny); G.inv_cell = ufd(H.inv_cell);
  G.inv_celly = ufd(H.inv_celly); G.inv_cellf = uff((float)H.inv_cell);
  G.inv_gy = uff(H.inv_gy);
  G.gx = ufl(H.gx); G.gy = ufl(H.gy); G.ncell = ufl(H.ncell); G.nkey = ufl(H.nkey);
  return G;
}

// P1 sort key of a box of picker p: its cell in picker p's grid (x-major), or nkey when the
// box cannot have an edge (non-finite coordinates).  Monotone in x and y per picker.
// f32 layout (!W): on floats.  The column is floor of the very product P2's half-column test
// takes (f32 difference of the exact f32 values, times (float)inv_cell), and any consistent
// map with the cell sizes' slack keeps the stencil exact (see P1).
template <bool W>
__device__ __forceinline__ int box_key(const GridU& H, int p, double x, double y) {
  if (H.ncell == 0 || !isfinite(x) || !isfinite(y)) return H.nkey;
  int cx, cy;
  if constexpr (W) {
    cx = (int)fmin(floor((x - H.minx) * H.inv_cell), (double)(H.gx - 1));
    cy = (int)fmin(floor((y - H.miny) * H.inv_celly), (double)(H.gy - 1));
  } else {
    cx = min((int)floorf(((float)x - (float)H.minx) * H.inv_cellf), H.gx - 1);
    cy = min((int)floorf(((float)y - (float)H.miny) * (float)H.inv_celly), H.gy - 1);
  }
  return p * H.ncell + cx * H.gy + cy;
}

// graph insertion key of a clique vertex u (a position; tiny graphs only): first appearance
// of the node in the edge enumeration (picker pair, a index, b index, side) in local (file)
// order, get_cliques.py:33-34,135-143
template <int K>
__device__ __forceinline__ uint64_t ins_key(const FCtx<K>& c, int u) {
  const int pu = picker_of<K>(c.pp, u);
  const int bu = picker_begin<K>(c.pb, pu);
  const int lu = (int)c.S.citems[u] - bu;
  for (int a = 0; a < bu; ++a) {   // lower-picker boxes in file order
    const int ap = c.S.pos[a];
    if (contains16(c.S.dst, c.S.fwd[ap], c.S.fwd[ap + 1], u)) {
      const int qa = picker_of<K>(c.pb, a);
      return ((uint64_t)pair_index(qa, pu, K) << 49) |
             ((uint64_t)(a - picker_begin<K>(c.pb, qa)) << 25) | ((uint64_t)lu << 1) | 1ULL;
    }
  }
  // no incoming edge: its first outgoing edge = lowest target picker, smallest file index
  const int e0 = c.S.fwd[u], e1 = c.S.fwd[u + 1];
  const int d0 = c.S.dst[e0];
  const int pd = picker_of<K>(c.pp, d0);
  const int se = lb16(c.S.dst, e0, e1, picker_end<K>(c.pp, d0));
  int dmin = 1 << 30;
  for (int e = e0; e < se; ++e) dmin = min(dmin, (int)c.S.citems[c.S.dst[e]]);
  return ((uint64_t)pair_index(pu, pd, K) << 49) | ((uint64_t)lu << 25) |
         ((uint64_t)(dmin - picker_begin<K>(c.pb, pd)) << 1);
}

// ILP epilogue of one buffered clique (thread per clique): reference get_cliques.py:169-202.
// j = output index; mem = member positions in picker order.  Main pass: COO rows, weight,
// confidence, members and the consensus when one member has the largest weighted degree;
// returns true when the consensus needs the node-iteration order (a degree tie, or
// --multi_out), which fused_epilogue_order computes in a second, rarely-taken pass (its
// 64-bit hashing stays out of this pass's register budget).
// INTP (integer coordinates below 2^23, B <= 2896, f32 layout): every overlap B - |dx| and
// product is an integer below 2^24, exact in f32, so the overlaps, their median network and the
// f32 degree JIs (2 B^2 - I exact too) run on floats; the median overlaps are converted back
// to f64 exactly for the reference's divisions.  Same results, half the registers.
template <int K, bool W, bool INTP = false>
__device__ __forceinline__ bool fused_epilogue_main(const FCtx<K>& c, int64_t j,
                                                    const int (&mem)[K]) {
  constexpr int NE = K * (K - 1) / 2;
  using OT = typename std::conditional<INTP, float, double>::type;
  OT I[NE];       // overlaps of the member pairs (a < b) in reference op order
  int li[K];      // local (file-order) indices: id order
  {
    double s[K];
    OT xs[K], ys[K];
    int r[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
      if constexpr (INTP) {
        const float2 xy = reinterpret_cast<const float2*>(c.S.sxy)[mem[i]];
        xs[i] = xy.x;
        ys[i] = xy.y;
      } else {
        const double2 xy = ld_xy<W>(c.S, mem[i]);
        xs[i] = xy.x;
        ys[i] = xy.y;
      }
      li[i] = c.S.citems[mem[i]];
      r[i] = c.S.vrank[mem[i]];
    }
    if (c.S.vstaged) {
#pragma unroll
      for (int i = 0; i < K; ++i) s[i] = c.S.vscore[r[i]];
    } else {
#pragma unroll
      for (int i = 0; i < K; ++i) s[i] = c.score[c.b0 + li[i]];
    }
    cmpnet_apply<K, false>(r);   // ascending rows
#pragma unroll
    for (int i = 0; i < K; ++i) c.rows[j * K + i] = r[i];
    {
      int t = 0;
#pragma unroll
      for (int a = 0; a < K; ++a)
#pragma unroll
        for (int b = a + 1; b < K; ++b) {
          if constexpr (INTP) {
            I[t++] = fmaxf(c.Bf - fabsf(xs[a] - xs[b]), 0.0f) *
                     fmaxf(c.Bf - fabsf(ys[a] - ys[b]), 0.0f);
          } else {
            I[t++] = overlap(xs[a], ys[a], xs[b], ys[b], c.B);
          }
        }
    }
    // conf = f32(median score); w = f32(f64(conf) * median JI) where median JI = JI of the
    // median overlap (JI = I / (2 B^2 - I) is non-decreasing in I, so sorting by I sorts the
    // JIs): one or two reference divisions instead of one per pair
    const double cf = median_n<K>(s);
    OT Is[NE];
#pragma unroll
    for (int t = 0; t < NE; ++t) Is[t] = I[t];
    double med;
    if constexpr (INTP) {   // finite integers: no NaN
      mid_n<NE>(Is);
      if (NE & 1) {
        med = (double)Is[NE / 2];
        med = med / (c.two_b2 - med);
      } else {
        const double a = (double)Is[NE / 2 - 1], b = (double)Is[NE / 2];
        med = ((a / (c.two_b2 - a)) + (b / (c.two_b2 - b))) / 2.0;
      }
    } else if (NE & 1) {
      med = median_n<NE>(Is);   // sorted copy's middle element
      med = med / (c.two_b2 - med);
    } else {
      bool nan = false;
#pragma unroll
      for (int t = 0; t < NE; ++t) nan |= isnan(Is[t]);
      mid_n<NE>(Is);
      const double a = Is[NE / 2 - 1], b = Is[NE / 2];
      med = nan ? NAN : ((a / (c.two_b2 - a)) + (b / (c.two_b2 - b))) / 2.0;
    }
    const float conf32 = (float)cf;
    c.w[j] = (float)((double)conf32 * med);
    c.conf[j] = conf32;
  }
  if (c.flags & (2 | 32)) {
#pragma unroll
    for (int i = 0; i < K; ++i) c.members[j * K + i] = c.b0 + li[i];
  }
  if (c.flags & 2) return true;
  // weighted degrees from f32 JIs: f32 operands (2^-24 each) and v_rcp_f32 (1 ulp) give
  // < 4e-7 per JI <= 1, < 5.5e-6 per sum of <= 7 terms with its f32 additions; a maximum
  // clear by 3e-5 is the reference's, anything closer goes to the exact f64 pass (ties)
  float deg[K];
#pragma unroll
  for (int i = 0; i < K; ++i) deg[i] = 0.0f;
  {
    int t = 0;
#pragma unroll
    for (int a = 0; a < K; ++a)
#pragma unroll
      for (int b = a + 1; b < K; ++b) {
        float jf;
        if constexpr (INTP) jf = I[t] * __builtin_amdgcn_rcpf(c.two_b2f - I[t]);
        else jf = (float)I[t] * __builtin_amdgcn_rcpf((float)(c.two_b2 - I[t]));
        deg[a] += jf;
        deg[b] += jf;
        ++t;
      }
  }
  float d1 = deg[0], d2 = -INFINITY;
  int arg = 0;
#pragma unroll
  for (int i = 1; i < K; ++i) {
    const float d = deg[i];
    d2 = d > d1 ? d1 : fmaxf(d2, d);
    arg = d > d1 ? i : arg;
    d1 = fmaxf(d1, d);
  }
  if (!(d1 - d2 > 3e-5f)) return true;
  int cons = li[0];
#pragma unroll
  for (int i = 1; i < K; ++i) cons = (arg == i) ? li[i] : cons;
  c.consensus[j] = c.b0 + cons;
  return false;
}

// second pass for the cliques fused_epilogue_main deferred: networkx node-iteration order
// (CPython set order or graph insertion order), consensus among the tied maximal members,
// and the --multi_out member order
template <int K, bool W>
__device__ __forceinline__ void fused_epilogue_order(const FCtx<K>& c, int64_t j,
                                                     const int (&mem)[K]) {
  double ji[K][K], xs[K], ys[K];
  int li[K];
  uint64_t ins[K] = {};
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const double2 xy = ld_xy<W>(c.S, mem[i]);
    xs[i] = xy.x;
    ys[i] = xy.y;
    li[i] = c.S.citems[mem[i]];
  }
#pragma unroll
  for (int a = 0; a < K; ++a)
#pragma unroll
    for (int b = a + 1; b < K; ++b) ji[a][b] = jaccard(xs[a], ys[a], xs[b], ys[b], c.B, c.two_b2);
  if (!c.set_order) {
    for (int i = 0; i < K; ++i) ins[i] = ins_key<K>(c, mem[i]);
  }
  uint32_t top;
  int arg = epi_degree_max<K>(ji, &top);
  const bool tie = (top & (top - 1)) != 0;
  const bool multi = (c.flags & 2) != 0;
  if (tie || multi) {
    if (c.set_order) {
      // CPython set order (64-bit tuple hashing and set probing): appended for k_fused_ties,
      // which keeps that code out of this kernel's registers (ties: ~0.6 % of C2's cliques)
      const unsigned long long t = atomicAdd((unsigned long long*)c.tie_count, 1ull);
      if ((int64_t)t < c.tie_cap) {
        gptr<int32_t> e = c.tie_list + (int64_t)t * (4 + K);
        e[0] = (int32_t)(uint32_t)(uint64_t)j;
        e[1] = (int32_t)(uint32_t)((uint64_t)j >> 32);
        e[2] = c.m;
        e[3] = (int32_t)(top | (tie ? 0x10000u : 0u) | (multi ? 0x20000u : 0u));
#pragma unroll
        for (int i = 0; i < K; ++i) e[4 + i] = c.b0 + li[i];
      }
      if (tie) return;   // consensus by k_fused_ties
    } else {
      const uint32_t ord = node_order_ins<K>(ins);
      if (tie) arg = epi_tie_arg<K>(top, ord);
      if (multi) {
#pragma unroll
        for (int i = 0; i < K; ++i) c.order[j * K + i] = (uint8_t)((ord >> (4 * i)) & 15);
      }
    }
  }
  int cons = li[0];
#pragma unroll
  for (int i = 1; i < K; ++i) cons = (arg == i) ? li[i] : cons;
  c.consensus[j] = c.b0 + cons;
}

// Static-recursion DFS: level D picks the picker-D member among the forward neighbours of
// the picker-(D-1) member that are also forward neighbours of every earlier member.
template <int K, int D, bool FILL>
struct FLevel {
  __device__ __forceinline__ static void run(FCtx<K>& c, int (&mem)[K]) {
    // the picker-D neighbours of mem[D-1] (a picker D-1 box) are the first segment of its
    // forward list: [fwd, split) from P3, or by binary search in the P6 re-walk (split's
    // LDS is reused by then)
    const int prev = mem[D - 1];
    const int lo = c.S.fwd[prev];
    int hi;
    if (FILL) hi = lb16(c.S.dst, lo, c.S.fwd[prev + 1], c.pp[D + 1]);
    else hi = c.S.split[prev];
    for (int e = lo; e < hi; ++e) {
      const int h = c.S.dst[e];
      bool ok = true;
#pragma unroll
      for (int q = 0; q < D - 1; ++q) {
        if (!contains16(c.S.dst, c.S.fwd[mem[q]], c.S.fwd[mem[q] + 1], h)) { ok = false; break; }
      }
      if (!ok) continue;
      mem[D] = h;
      FLevel<K, D + 1, FILL>::run(c, mem);
    }
  }
};
template <int K, bool FILL>
struct FLevel<K, K, FILL> {
  __device__ __forceinline__ static void run(FCtx<K>& c, int (&mem)[K]) {
    if (FILL) {
      const int64_t j = c.out++;
      if (j >= c.c0 && j < c.c1) {
        uint16_t* dstb = c.S.cbuf + (j - c.c0) * K;
#pragma unroll
        for (int i = 0; i < K; ++i) dstb[i] = (uint16_t)mem[i];
        c.cq_ord[j - c.c0] = 0;
      }
    } else {
      // queue the clique (members + ordinal within the root's DFS) while the queue has room;
      // its output index is known once the per-root counts are scanned
      const uint32_t o = (uint32_t)c.count++;
      const uint32_t slot = atomicAdd(c.ccur, 1u);
      if (slot < (uint32_t)c.cq_cap) {
#pragma unroll
        for (int i = 0; i < K; ++i) c.S.cbuf[slot * K + i] = (uint16_t)mem[i];
        c.cq_ord[slot] = (uint16_t)o;
      }
#pragma unroll
      for (int i = 0; i < K; ++i) {
        c.S.flags[mem[i]] = 3;
      }
    }
  }
};

// ----------------------------------------------------------------------------- P4 (BFS)
// Level-synchronous k-clique enumeration (get_cliques.py:49-56 restated for a k-partite
// graph).  Level D holds every D-member prefix (one member per picker 0..D-1, pairwise
// adjacent) in lexicographic order as a tree entry (index of its parent prefix << 16 | last
// member); level 1 is implicit (the picker-0 roots).  Expanding a level: count + 32-bit mask
// of the valid extensions per entry (candidates = first forward segment of the last member,
// kept if every earlier member's list contains them), workgroup scan, write pass.  Level K
// holds the cliques (lexicographic = per-root DFS order), followed by one zeroed flag word
// per clique; the last expansion marks the members.  All levels live in the queue region
// q[0, qbytes); the temps of the level being expanded sit at its top.  Every prefix is one
// thread's work, so a root's subtree no longer serialises on one lane.
template <int K>
struct BfsOut {
  int64_t C;        // cliques, or -1: a level did not fit (caller falls back to the DFS)
  int lvl[K + 1];   // byte offset in q of each level's entries (2..K)
  float fit;        // capacity / demand: of the level that overflowed (C = -1, < 1), else the
                    // smallest over the levels (>= 1)
};
__device__ __forceinline__ float bfs_fit(int64_t need, int64_t have) {
  return need > 0 ? (float)max(have, (int64_t)0) / (float)need : 1.0f;
}

// REWALK (P6 re-run of a root chunk): the split array and the union-find parents are dead by
// then, so first segments come from a binary search for the next picker's first position and
// a root is valid iff it was marked as a clique vertex in P4 (it has a clique, which lies in
// the --get_cc target component); vertices are already marked.
// WE (wide entries, K <= 4, the HBM level-tree slot of the QG launches): an entry holds its
// prefix's members themselves (four u16 in 8 bytes) instead of (parent index, last member), so
// reading a prefix is one load instead of a chain of D - 1 dependent ones (L2 latency each).
template <bool WE>
constexpr int bfs_es() { return WE ? 8 : 4; }
__device__ __forceinline__ uint2 we_pack(const int (&mm)[4], int d, int h) {
  int t[4] = {mm[0], mm[1], mm[2], mm[3]};
  t[d] = h;
  return make_uint2((uint32_t)t[0] | ((uint32_t)t[1] << 16), (uint32_t)t[2] | ((uint32_t)t[3] << 16));
}
template <int K, int D, int NT, bool WE = false>
struct BfsLevel {
  // prefix members of entry e of level D (D members, compile-time indices only)
  __device__ __forceinline__ static void unpack(const uint2 v, int (&mm)[K]) {
    const int t[4] = {(int)(v.x & 0xFFFF), (int)(v.x >> 16), (int)(v.y & 0xFFFF), (int)(v.y >> 16)};
#pragma unroll
    for (int d = 0; d < D && d < 4; ++d) mm[d] = t[d];
  }
  __device__ __forceinline__ static void prefix(const char* q, const int (&lvl)[K + 1],
                                                uint32_t e, int (&mm)[K]) {
    if constexpr (WE) {
      unpack(reinterpret_cast<const uint2*>(q + lvl[D])[e], mm);
      return;
    }
    uint32_t ent = reinterpret_cast<const uint32_t*>(q + lvl[D])[e];
    mm[D - 1] = (int)(ent & 0xFFFF);
    uint32_t cur = ent >> 16;
#pragma unroll
    for (int d = D - 1; d >= 2; --d) {
      ent = reinterpret_cast<const uint32_t*>(q + lvl[d])[cur];
      mm[d - 1] = (int)(ent & 0xFFFF);
      cur = ent >> 16;
    }
    mm[0] = (int)cur;
  }

  template <bool REWALK>
  __device__ __forceinline__ static int seg_end(const FShared& S, const int (&pp)[K + 1], int m) {
    if (REWALK) return lb16(S.dst, S.fwd[m], S.fwd[m + 1], pp[D + 1]);
    return S.split[m];
  }

  template <bool REWALK, typename EP>
  __device__ __forceinline__ static BfsOut<K> run(const FShared& S, FusedHdr& H, char* q,
                                                  int qbytes, BfsOut<K>& out, int64_t nD, int tid,
                                                  const int (&pp)[K + 1], const EP& ep) {
    int (&lvl)[K + 1] = out.lvl;
    constexpr int ES = bfs_es<WE>();
    // temps of this level at the top of q
    const int tb = (qbytes - 8 * (int)(nD + 1)) & ~7;
    if (K >= 4) {   // (K = 3 runs one attempt: no chunk sizing)
      const float f = fminf(bfs_fit(nD, 65535), bfs_fit((8 + ES) * nD, qbytes - lvl[D] - 8));
      out.fit = fminf(out.fit, f);
    }
    if (nD > 65535 || tb < lvl[D] + ES * (int)nD) {
      out.C = -1;
      out.fit = fminf(out.fit, 0.999f);
      return out;
    }
    uint32_t* MK = reinterpret_cast<uint32_t*>(q + tb);
    uint32_t* CN = MK + nD;
    for (int e = tid; e < nD; e += NT) {
      int mm[K];
      prefix(q, lvl, (uint32_t)e, mm);
      const int m = mm[D - 1];
      const int lo = S.fwd[m], hi = seg_end<REWALK>(S, pp, m);
      uint32_t mask = 0, cnt = 0;
      // an extension h (picker D) must be adjacent to every earlier member: the graph's edges
      // are exactly the pairs of different pickers with JI > 0.3, so instead of a binary
      // search of h in each member's sorted list (three dependent LDS loads each), P2's own
      // test on the two boxes' coordinates decides it (ep.edge: the same function on the same
      // LDS values, so the same answer); the members' coordinates stay in registers
      typename EP::CT mc[K > 2 ? K - 2 : 1];
#pragma unroll
      for (int d = 0; d < D - 1; ++d) mc[d] = ep.pt(S, mm[d]);
      for (int t = lo; t < hi; ++t) {
        const int h = S.dst[t];
        const typename EP::CT ch = ep.pt(S, h);
        bool ok = true;
#pragma unroll
        for (int d = 0; d < D - 1; ++d) ok &= ep.edge(mc[d], ch);
        cnt += ok ? 1u : 0u;
        mask |= (ok && t - lo < 32) ? (1u << (t - lo)) : 0u;
      }
      MK[e] = mask;
      CN[e] = cnt;
    }
    __syncthreads();
    // (32-bit scan: nD <= 65535 entries of at most n <= 4608 extensions each, < 2^31)
    const int64_t nN = ufl(block_scan_dpp32<NT>(CN, (int)nD, H.redi));
    constexpr bool last = D + 1 == K;
    const int nb = ufl((lvl[D] + ES * (int)nD + 7) & ~7);   // next level starts here
    if (K >= 4) {
      const float f = fminf(bfs_fit(nN, 65535), bfs_fit(nN * (last ? ES + 2 : ES), tb - nb));
      out.fit = fminf(out.fit, f);
    }
    if (nN > 65535 || nN * (last ? ES + 2 : ES) > tb - nb) {
      out.C = -1;
      out.fit = fminf(out.fit, 0.999f);
      return out;
    }
    for (int e = tid; e < nD; e += NT) {
      int mm[K];
      prefix(q, lvl, (uint32_t)e, mm);
      const int m = mm[D - 1];
      const int lo = S.fwd[m], hi = seg_end<REWALK>(S, pp, m);
      const uint32_t mask = MK[e];
      uint32_t o = CN[e];
      for (int t = lo; t < hi; ++t) {
        const int h = S.dst[t];
        bool ok;
        if (t - lo < 32) {
          ok = (mask >> (t - lo)) & 1u;
        } else {
          const typename EP::CT ch = ep.pt(S, h);
          ok = true;
#pragma unroll
          for (int d = 0; d < D - 1; ++d) ok &= ep.edge(ep.pt(S, mm[d]), ch);
        }
        if (!ok) continue;
        if constexpr (WE) {
          int m4[4] = {0, 0, 0, 0};
#pragma unroll
          for (int d = 0; d < D && d < 4; ++d) m4[d] = mm[d];
          reinterpret_cast<uint2*>(q + nb)[o] = we_pack(m4, D < 4 ? D : 3, h);
        } else {
          reinterpret_cast<uint32_t*>(q + nb)[o] = ((uint32_t)e << 16) | (uint32_t)h;
        }
        if (last) {
          if (!REWALK) {
#pragma unroll
            for (int d = 0; d < K - 1; ++d) S.flags[mm[d]] = 3;
            S.flags[h] = 3;
          }
          reinterpret_cast<uint16_t*>(q + nb + ES * (int)nN)[o] = 0;
        }
        ++o;
      }
    }
    __syncthreads();
    lvl[D + 1] = nb;
    if constexpr (D + 1 < K) {
      return BfsLevel<K, D + 1, NT, WE>::template run<REWALK>(S, H, q, qbytes, out, nN, tid, pp, ep);
    } else {
      out.C = nN;
      return out;
    }
  }
};

// Cliques of the roots [r0, r1) (picker-0 positions).  Returns C = -1 when a level does not
// fit the queue region; the caller then retries with fewer roots (root chunks, P4) and falls
// back to the per-root DFS only when a single root does not fit.
template <int K, bool REWALK, int NT, bool WE = false, typename EP>
__device__ __forceinline__ BfsOut<K> bfs_cliques(const FShared& S, FusedHdr& H, char* q,
                                                 int qbytes, int r0, int r1, bool get_cc,
                                                 uint32_t target, int tid,
                                                 const int (&pp)[K + 1], const EP& ep) {
  BfsOut<K> out;
  out.C = -1;
  out.fit = 4.0f;
#pragma unroll
  for (int d = 0; d <= K; ++d) out.lvl[d] = 0;
  const int nr = r1 - r0;
  auto root_ok = [&](int r) {
    if (REWALK) return S.flags[r] == 3;
    return S.fwd[r] < S.fwd[r + 1] && (!get_cc || S.parent[r] == target);
  };
  auto seg_end = [&](int r) {
    if (REWALK) return lb16(S.dst, S.fwd[r], S.fwd[r + 1], pp[2]);
    return (int)S.split[r];
  };
  // level 1 -> 2: every root's first segment (picker-1 neighbours), no checks needed
  uint32_t* cnt = S.cnt;
  for (int i = tid; i < nr; i += NT) {
    const int r = r0 + i;
    cnt[i] = root_ok(r) ? (uint32_t)(seg_end(r) - S.fwd[r]) : 0u;
  }
  __syncthreads();
  const int64_t n2 = ufl(block_scan_dpp32<NT>(cnt, nr, H.redi));   // (< n^2 < 2^31)
  constexpr bool last = K == 2;
  constexpr int ES = bfs_es<WE>();
  if (K >= 4) out.fit = fminf(bfs_fit(n2, 65535), bfs_fit(n2 * (last ? ES + 2 : ES), qbytes));
  if (n2 > 65535 || n2 * (last ? ES + 2 : ES) > qbytes) {
    out.fit = fminf(out.fit, 0.999f);
    return out;
  }
  for (int i = tid; i < nr; i += NT) {
    const int r = r0 + i;
    if (!root_ok(r)) continue;
    uint32_t o = cnt[i];
    const int se = seg_end(r);
    for (int t = S.fwd[r]; t < se; ++t, ++o) {
      const int h = S.dst[t];
      if constexpr (WE) reinterpret_cast<uint2*>(q)[o] = make_uint2((uint32_t)r | ((uint32_t)h << 16), 0u);
      else reinterpret_cast<uint32_t*>(q)[o] = ((uint32_t)r << 16) | (uint32_t)h;
      if (last) {
        if (!REWALK) {
          S.flags[r] = 3;
          S.flags[h] = 3;
        }
        reinterpret_cast<uint16_t*>(q + ES * (int)n2)[o] = 0;
      }
    }
  }
  __syncthreads();
  out.lvl[2] = 0;
  if constexpr (K > 2) {
    return BfsLevel<K, 2, NT, WE>::template run<REWALK>(S, H, q, qbytes, out, n2, tid, pp, ep);
  } else {
    out.C = n2;
    return out;
  }
}

// P2: boxes with up to FILL_FAST forward edges have their targets kept by the count (the
// last two in cnt, the first of three in the CC-size slot, zero until P3); the fill writes
// them without walking the stencil again
constexpr int FILL_FAST = 2;

// Candidates of a box: the 2x3 cell stencil at its cell in the grid of every HIGHER picker
// (forward edges only): columns cx, cx + 1 from cx = its column - 1 or its column (by the
// half of the column the box lies in), rows y0..y1, i.e. up to 2 (K - 1 - p) ranges of
// sorted positions.
struct Stencil {
  int p, cx, y0, y1;   // p = K: no candidates
  double2 a;
};

template <int K, bool W>
__device__ __forceinline__ void stencil_setup(Stencil& st, int ts, const FShared& S,
                                              const GridU& H) {
  const int key = S.scell[ts];
  st.a = ld_xy<W>(S, ts);
  st.p = K;
  st.cx = 0;
  st.y0 = 0;
  st.y1 = -1;
  if (key >= H.nkey) return;
  const int gy = H.gy, nc = H.ncell;
  // key / ncell and cell / gy through float reciprocals, corrected to the exact quotients
  int p = 0;
#pragma unroll
  for (int q = 1; q < K; ++q) p += (key >= q * nc) ? 1 : 0;
  const int cell = key - p * nc;
  int cx = (int)((float)cell * H.inv_gy);
  cx += ((cx + 1) * gy <= cell) ? 1 : 0;
  cx -= (cx * gy > cell) ? 1 : 0;
  const int cy = cell - cx * gy;
  // half-column test in f32 (0.0014 columns of slack, see P1): left half -> columns cx-1, cx
  const float u = (float)(st.a.x - H.minx) * H.inv_cellf;   // = box_key's product on !W
  st.p = p;
  st.cx = cx - ((u - (float)cx) < 0.5f ? 1 : 0);
  st.y0 = max(cy - 1, 0);
  st.y1 = min(cy + 1, gy - 1);
}

// column range [lo, hi) of the stencil in picker q's grid, column st.cx + d (d = 0, 1)
__device__ __forceinline__ void stencil_range(const Stencil& st, const FShared& S,
                                              const GridU& H, int q, int d, int& lo, int& hi) {
  const int col = st.cx + d;
  lo = hi = 0;
  if (col < 0 || col >= H.gx) return;
  const int cb = q * H.ncell + col * H.gy;
  lo = S.cstart[cb + st.y0];
  hi = S.cstart[cb + st.y1 + 1];
}

// v_min_f64 / v_max_f64 without the sNaN canonicalisation fmin/fmax carry: grid candidates
// have finite coordinates (non-finite boxes are never in a grid cell), where they equal
// np.min / np.max
__device__ __forceinline__ double min_f64(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double max_f64(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// JI > 0.3 (get_cliques.py:40-46, 64-65): branch-free overlap; the reference quotient is
// evaluated only inside the ambiguity band [i_lo, i_hi] (rare, divergent)
__device__ __forceinline__ bool edge_test(double2 a, double2 b, double B, double two_b2,
                                          double i_lo, double i_hi) {
  double xo = (min_f64(a.x, b.x) + B) - max_f64(a.x, b.x);
  double yo = (min_f64(a.y, b.y) + B) - max_f64(a.y, b.y);
  xo = max_f64(xo, 0.0);
  yo = max_f64(yo, 0.0);
  const double inter = xo * yo;
  bool e = inter > i_hi;
  if (!e && inter >= i_lo) e = inter / (two_b2 - inter) > 0.3;   // reference quotient
  return e;
}

// P2's edge decision on two boxes' LDS coordinates (lower picker first), for P4's adjacency
// tests: the integer test of pairs_count_int on the f32 layout, edge_test on the f64 layout
template <bool W>
struct EdgeP {
  using CT = typename std::conditional<W, double2, float2>::type;
  float Bf, Tf;
  double B, two_b2, ilo, ihi;
  __device__ __forceinline__ CT pt(const FShared& S, int p) const {
    return reinterpret_cast<const CT*>(S.sxy)[p];
  }
  __device__ __forceinline__ bool edge(CT a, CT b) const {
    if constexpr (W) {
      return edge_test(a, b, B, two_b2, ilo, ihi);
    } else {
      const float xo = fmaxf(Bf - fabsf(a.x - b.x), 0.0f);
      const float yo = fmaxf(Bf - fabsf(a.y - b.y), 0.0f);
      return xo * yo > Tf;
    }
  }
};

// P2 count for the box at sorted position ts (thread per box): JI test against every stencil
// candidate of a higher picker; returns the edge count and, for the fill, either the targets
// themselves (at most 2 edges: first << 16 | second, ascending) or the bitmask of edge
// candidates (candidates 0..31 in stencil order; later candidates are re-tested by the fill).
template <int K, bool W>
__device__ __forceinline__ int pairs_count(const Stencil& st, const FShared& S, const GridU& H,
                                           double B, double two_b2, double i_lo, double i_hi,
                                           uint32_t* mask_out, uint32_t* first_out) {
  uint32_t mask = 0, pk = 0, first = 0;
  int cnt = 0, kk = 0;
  // f32 layout: reject in f32 first.  An edge needs both overlaps > (6/13) B, i.e. |dx| and
  // |dy| < (7/13) B = 0.5385 B; the f32 difference of two exact f32 values is within 2^-24 of
  // the true one, so |dx| >= 0.54 B (as computed) can never be an edge.
  const float rej = 0.54f * (float)B;
  const float ax = (float)st.a.x, ay = (float)st.a.y;
  for (int q = st.p + 1; q < K; ++q) {
#pragma unroll
    for (int d = 0; d <= 1; ++d) {
      int lo, hi;
      stencil_range(st, S, H, q, d, lo, hi);
      for (int t = lo; t < hi; ++t, ++kk) {
        bool e;
        if constexpr (W) {
          e = edge_test(st.a, ld_xy<W>(S, t), B, two_b2, i_lo, i_hi);
        } else {
          const float2 bf = reinterpret_cast<const float2*>(S.sxy)[t];
          e = false;
          if (fabsf(ax - bf.x) < rej && fabsf(ay - bf.y) < rej)
            e = edge_test(st.a, make_double2((double)bf.x, (double)bf.y), B, two_b2, i_lo,
                          i_hi);
        }
        if (e) {
          first = cnt == 0 ? (uint32_t)t : first;
          ++cnt;
          mask |= (kk < 32) ? (1u << kk) : 0u;
          pk = (pk << 16) | (uint32_t)t;
        }
      }
    }
  }
  *mask_out = cnt <= FILL_FAST ? pk : mask;
  *first_out = first;
  return cnt;
}

// P2 count on integer coordinates (f32 layout, see P2): exact f32 overlaps, I > floor(6B^2/13)
template <int K>
__device__ __forceinline__ int pairs_count_int(const Stencil& st, const FShared& S,
                                               const GridU& H, float Bf, float Tf,
                                               uint32_t* mask_out, uint32_t* first_out) {
  uint32_t mask = 0, pk = 0, first = 0;
  int cnt = 0, kk = 0;
  const float ax = (float)st.a.x, ay = (float)st.a.y;
  for (int q = st.p + 1; q < K; ++q) {
#pragma unroll
    for (int d = 0; d <= 1; ++d) {
      int lo, hi;
      stencil_range(st, S, H, q, d, lo, hi);
      for (int t = lo; t < hi; ++t, ++kk) {
        const float2 bf = reinterpret_cast<const float2*>(S.sxy)[t];
        const float xo = fmaxf(Bf - fabsf(ax - bf.x), 0.0f);
        const float yo = fmaxf(Bf - fabsf(ay - bf.y), 0.0f);
        if (xo * yo > Tf) {
          first = cnt == 0 ? (uint32_t)t : first;
          ++cnt;
          mask |= (kk < 32) ? (1u << kk) : 0u;
          pk = (pk << 16) | (uint32_t)t;
        }
      }
    }
  }
  *mask_out = cnt <= FILL_FAST ? pk : mask;
  *first_out = first;
  return cnt;
}

// P2 fill: write the box's forward targets (positions) at d[0..cnt) from the count's bitmask
// (re-testing candidates past the 32nd).  Grids are visited in picker order and each grid's
// column ranges in key order, so the list comes out sorted.
template <int K, bool W>
__device__ __forceinline__ void pairs_fill(const Stencil& st, const FShared& S, const GridU& H,
                                           uint32_t mask, uint16_t* d, int cnt, double B,
                                           double two_b2, double i_lo, double i_hi) {
  int c = 0, kk = 0;
  for (int q = st.p + 1; q < K; ++q) {
#pragma unroll
    for (int dd = 0; dd <= 1; ++dd) {
      int lo, hi;
      stencil_range(st, S, H, q, dd, lo, hi);
      const int len = hi - lo;
      if (kk + len <= 32) {
        uint32_t bits = kk < 32 ? (mask >> kk) : 0u;
        bits &= len >= 32 ? ~0u : ((1u << len) - 1u);
        while (bits) {
          const int b = __builtin_ctz(bits);
          bits &= bits - 1;
          d[c++] = (uint16_t)(lo + b);
        }
      } else {
        for (int t = lo; t < hi; ++t) {
          const int idx = kk + (t - lo);
          const bool e = idx < 32 ? ((mask >> idx) & 1u) != 0
                                  : edge_test(st.a, ld_xy<W>(S, t), B, two_b2, i_lo, i_hi);
          if (e) d[c++] = (uint16_t)t;
        }
      }
      kk += len;
    }
  }
}

// per-micrograph results of workgroup thread 0; finished micrographs add their edges to the
// batch total (deferred ones are counted by the pass that finishes them)
__device__ __forceinline__ void put_stats(const FusedArgs& A, int m, int status, int64_t edges,
                                          int nodes, int cc_cnt, int cc_max, int V, int64_t base,
                                          int64_t C) {
  A.o.status[m] = status;
  A.o.cc_max[m] = cc_max;
  A.o.cc_cnt[m] = cc_cnt;
  A.o.n_nodes[m] = nodes;
  A.o.n_vert[m] = V;
  A.o.n_edges[m] = edges;
  A.o.clique_base[m] = base;
  A.o.clique_cnt[m] = C;
  // a micrograph that needs another pass is counted, so a run's totals alone tell the host
  // (lazy stats); the edges of finished ones are summed after the launch (k_fused_ties).
  // DEFER_WIDE ones are also counted on cursor[5]; with a device-side f64 pass to follow
  // (wide_list) they go to its list and are not a deferral for the host
  if (status == RGC_ST_DEFER_WIDE) {
    const unsigned long long q = atomicAdd(A.cursor + 5, 1ull);
    if (A.wide_list) {
      A.wide_list[q] = m;
      return;
    }
  }
  if (!(status == 0 || status == RGC_ST_NO_CLIQUES || status == RGC_ST_NO_EDGES))
    atomicAdd(A.cursor + 4, 1ull);
}

// Waves per SIMD the register allocator targets.  K = 3 fits 64 VGPRs (4 small spills) for 8
// waves per SIMD = 4 workgroups per CU, which the f32-coordinate LDS layout also allows; larger
// K keep the compiler's choice (their VGPRs, not LDS, bound the occupancy).
constexpr int fused_waves_per_eu(int k, int nt) {
  return nt == 1024 ? 4 : (nt == 768 ? 6 : (nt == 256 ? 4 : (nt == 384 ? 6 : (k <= 3 ? 8 : 1))));
}

// HBM level-tree slots (QG launches): claim a free bit of the slot bitmap (one thread), or -1
// after a bounded search (then the workgroup keeps the LDS queue).  There are twice as many
// slots as workgroups of such a launch can be resident, so the search normally succeeds on
// its first pass; every claimed slot is released by its workgroup before it ends.
__device__ int qg_claim(const FusedArgs& A) {
  const int nw = A.qg_nslots >> 5;
  const int w0 = (int)(blockIdx.x % (unsigned)max(nw, 1));
  for (int pass = 0; pass < 4; ++pass) {
    for (int i = 0; i < nw; ++i) {
      const int wd = (w0 + i) % nw;
      uint32_t v = __hip_atomic_load(A.qg_slots + wd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int t = 0; t < 32 && v != 0xFFFFFFFFu; ++t) {
        const int b = __builtin_ctz(~v);
        const uint32_t old = atomicOr(A.qg_slots + wd, 1u << b);
        if (!(old & (1u << b))) return wd * 32 + b;
        v = old | (1u << b);
      }
    }
  }
  return -1;
}

template <int K, bool W, int NT, bool QG>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(fused_waves_per_eu(K, NT))))
void k_fused(FusedArgs A) {
  constexpr int FWG = NT;   // threads of this instance
  constexpr int FNW = NT / 64;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  FusedHdr& H = *reinterpret_cast<FusedHdr*>(smem);
  const FusedLayout L = fused_layout(A.nmax, A.ecap, W);
  FShared S;
  S.sxy = smem + L.off_sxy;
  S.cstart = reinterpret_cast<uint16_t*>(smem + L.off_cstart);
  S.cnt = reinterpret_cast<uint32_t*>(smem + L.off_cnt);
  S.fwd = reinterpret_cast<uint16_t*>(smem + L.off_fwd);
  S.split = reinterpret_cast<uint16_t*>(smem + L.off_scell);
  S.vscore = reinterpret_cast<double*>(smem + L.off_parent);
  S.vstaged = false;
  S.parent = reinterpret_cast<uint16_t*>(smem + L.off_parent);
  S.citems = reinterpret_cast<uint16_t*>(smem + L.off_citems);
  S.pos = reinterpret_cast<uint16_t*>(smem + L.off_pos);
  S.scell = reinterpret_cast<uint16_t*>(smem + L.off_scell);
  S.vrank = reinterpret_cast<uint16_t*>(smem + L.off_vrank);
  S.flags = reinterpret_cast<uint8_t*>(smem + L.off_flags);
  S.dst = reinterpret_cast<uint16_t*>(smem + L.off_dst);
  S.cbuf = reinterpret_cast<uint16_t*>(smem + L.off_cbuf);
  const int tid = threadIdx.x;
  // (device-side f64 pass: the list's length is known on the device only)
  if (A.mg_count && blockIdx.x >= *A.mg_count) return;
  const int m = A.mg_list ? A.mg_list[blockIdx.x] : (int)blockIdx.x;
  if (blockIdx.x == 0 && tid < 16 && A.cursor_clear) A.cursor_clear[tid] = 0;   // next run's
#ifdef RGC_STAMPS
  // diagnostic build only: per-phase s_memtime stamps of thread 0 (never in the product .so)
#define STAMP(i)                                                                            \
  do {                                                                                      \
    if ((tid & 63) == 0) {                                                                  \
      A.stamps[(int64_t)blockIdx.x * STAMP_SLOTS + 16 + 16 * (i) + (tid >> 6)] =              \
          (i) == 0 ? 0ull : g_bwait[tid >> 6];                                              \
      g_bwait[tid >> 6] = 0;                                                                \
    }                                                                                       \
    raw_barrier();                                                                          \
    if (tid == 0) A.stamps[(int64_t)blockIdx.x * STAMP_SLOTS + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#endif
#ifdef RGC_STOP_AFTER
  // ablation build only: stop after phase RGC_STOP_AFTER (outputs incomplete)
#define STOP_AFTER(ph)                            \
  do {                                            \
    if ((ph) == RGC_STOP_AFTER) {                 \
      if (tid == 0) put_stats(A, m, 0, 0, 0, 0, 0, 0, 0, 0); \
      return;                                     \
    }                                             \
  } while (0)
#else
#define STOP_AFTER(ph) \
  do {                 \
  } while (0)
#endif
  STAMP(0);
#ifdef RGC_STAMPS
  // workgroup timeline (s_memrealtime, 100 MHz, chip-wide): start in the low half of slot 13
  const uint32_t rt0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
#endif
  FCtx<K> c;
  c.B = sdetach(A.B); c.two_b2 = sdetach(A.two_b2); c.flags = sdetach(A.flags);
  c.score = gdetach(A.score);
  c.Bf = uff((float)A.B);
  c.two_b2f = uff((float)A.two_b2);
  c.rows = gdetach(A.rows); c.w = gdetach(A.w); c.conf = gdetach(A.conf);
  c.consensus = gdetach(A.consensus);
  c.members = gdetach(A.members); c.order = gdetach(A.order);
  c.tie_list = gdetach(A.tie_list); c.tie_count = gdetach(A.cursor) + CUR_TIES;
  c.tie_cap = sdetach(A.tie_cap);
  const gptr<const double> ax = gdetach(A.x);
  const gptr<const double> ay = gdetach(A.y);
  c.S = S;
  c.m = m;
  c.b0 = A.box_off[m * K];
  c.n = A.box_off[m * K + K] - c.b0;
#pragma unroll
  for (int i = 0; i <= K; ++i) c.pb[i] = A.box_off[m * K + i] - c.b0;
  c.idb = A.id_base[m];
  const int n = c.n, b0 = c.b0;

  // ---- P0: load coordinates (the first RB boxes of each thread stay in registers for P1),
  // bounding box (one combined workgroup reduction)
  constexpr int RB = fused_rb(NT);
  double rx[RB], ry[RB];
#pragma unroll
  for (int j = 0; j < RB; ++j) {
    const int i = tid + j * FWG;
    rx[j] = i < n ? ax[b0 + i] : 0.0;
    ry[j] = i < n ? ay[b0 + i] : 0.0;
  }
  // fn(i, x, y) for every box of this thread
  auto each_box = [&](auto&& fn) {
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const int i = tid + j * FWG;
      if (i < n) fn(i, rx[j], ry[j]);
    }
    for (int i = tid + RB * FWG; i < n; i += FWG) fn(i, ax[b0 + i], ay[b0 + i]);
  };
  // bounding box on floats for the f32 layout (exact there; a micrograph with inexact
  // coordinates is deferred to the f64 layout, where it is computed in f64)
  using BT = typename std::conditional<W, double, float>::type;
  BT bmnx = INFINITY, bmny = INFINITY, bmxx = -INFINITY, bmxy = -INFINITY;
  // The f32 layout is the INTEGER layout: every finite coordinate an integer below 2^23 and
  // an integer box size 1 <= B <= 2896, so P2's overlaps and P6's overlap products are exact
  // floats (INTP); any other micrograph is deferred to the f64 ("wide") layout, whose kernel
  // carries the f64 arithmetic.  (Real picker BOX files hold integer pixel coordinates.)
  bool inexact = !W && !(A.B >= 1.0 && A.B <= 2896.0 && A.B == floor(A.B));
  each_box([&](int, double xv, double yv) {
    if (isfinite(xv) && isfinite(yv)) {
      bmnx = fmin(bmnx, (BT)xv); bmxx = fmax(bmxx, (BT)xv);
      bmny = fmin(bmny, (BT)yv); bmxy = fmax(bmxy, (BT)yv);
      if (!W)
        inexact |= xv != rint(xv) || yv != rint(yv) || fabs(xv) >= 0x1p23 || fabs(yv) >= 0x1p23;
    }
  });
  if (inexact) bmnx = -INFINITY;   // (impossible otherwise) carried through the min reduction
  // P1's packed bucket counters (the whole cell-start region of the size class), union-find
  // parents, node flags and P2's packed CC-size counters are set up here, so the bounding-box
  // barrier orders them too
  {
    uint32_t* cw = reinterpret_cast<uint32_t*>(S.cstart);
    const int ncw = (fused_cells(A.nmax) + 8) / 2;
    for (int q = tid; q < ncw; q += FWG) cw[q] = 0;
    for (int i = tid; i < n; i += FWG) {
      S.parent[i] = i;
      S.flags[i] = 0;
    }
    uint32_t* ccsz = reinterpret_cast<uint32_t*>(S.vrank);
    for (int q = tid; q < (n + 1) / 2; q += FWG) ccsz[q] = 0;
  }
  {
    BT bv[4] = {bmnx, bmny, -bmxx, -bmxy};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if constexpr (W) bv[r] = wave_incl_scan(bv[r], [](BT a, BT b) { return fmin(a, b); });
      else bv[r] = wave_incl_min_f32(bv[r]);
    }
    if ((tid & 63) == 63)
#pragma unroll
      for (int r = 0; r < 4; ++r) H.red4[r][tid >> 6] = (double)bv[r];
  }
  STOP_AFTER(0);
  STAMP(1);
  // ---- P1: one grid per picker (x-major cells, K * gx * gy <= 4 nmax + 4 cells in all) and
  // an LDS counting sort of the boxes by (picker, cell).  JI > 0.3 implies I > (6/13) B^2 and
  // so |dx|, |dy| < (7/13) B = 0.5385 B: with cells >= 1.08 B wide and >= 0.54 B tall every
  // edge partner lies in the box's own column or the neighbouring column on the side of the
  // box's half of its column (its x is within 0.4986 columns), three rows around its row: a
  // 2x3 stencil, i.e. two contiguous position ranges per grid.  Per-picker grids let a box
  // visit the boxes of higher pickers only.
  // Wave 0 alone reduces the per-wave bounding boxes and plans the grid (wave-uniform work:
  // done by every wave it cost ~8x its VALU); the other waves read the plan from the header
  // after one barrier.  Planned in f32 with hardware reciprocals: exactness is not needed,
  // only cells >= 1.08 B x 0.54 B (0.28 % above what an edge needs, far above f32 rounding;
  // the half-column test has 0.0014 columns of slack), K gx gy within the budget (checked on
  // the integers used), and one inv_cell / inv_celly used by every key.
  __syncthreads();
  if (tid < 64) {
    double v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[r] = H.red4[r][0];
#pragma unroll
      for (int w = 1; w < FNW; ++w) v[r] = fmin(v[r], H.red4[r][w]);
    }
    const double mnx = v[0], mny = v[1], mxx = -v[2], mxy = -v[3];
    double cl = A.B, icl = 0.0, icly = 0.0;
    int gx = 0, gy = 0;
    if (mnx <= mxx && A.B > 0.0) {
      const double ex = mxx - mnx, ey = mxy - mny;
      if (!(ex < 0x1p40 && ey < 0x1p40)) {
        cl = INFINITY; gx = 1; gy = 1;
      } else {
        const int budget = (fused_cells(A.nmax) + 4) / K;
        const float fex = (float)ex, fey = (float)ey, rb = __builtin_amdgcn_rcpf((float)budget);
        // row height h, column width 2 h
        float fch = fmaxf((float)(0.54 * A.B) * 1.000001f,
                          fmaxf(__builtin_sqrtf(0.5f * fex * fey * rb),
                                fmaxf(0.5f * fex, fey) * rb));
        for (;;) {
          const float iry = __builtin_amdgcn_rcpf(fch);
          const int fx = (int)floorf(fex * (0.5f * iry)) + 1, fy = (int)floorf(fey * iry) + 1;
          if (fx <= budget && fy <= budget && fx * fy <= budget) {
            gx = fx; gy = fy;
            break;
          }
          fch *= 1.0625f;
        }
        cl = (double)fch;
        icly = (double)__builtin_amdgcn_rcpf(fch);
        icl = 0.5 * icly;
        // keys use icl / icly: columns must stay >= 1.08 B wide, rows >= 0.54 B tall
        if (icl * (1.08 * A.B) > 1.0) icl = 1.0 / (1.08 * A.B);
        if (icly * (0.54 * A.B) > 1.0) icly = 1.0 / (0.54 * A.B);
      }
    }
    if (tid == 0) {
      const double ex = mxx - mnx;
      H.minx = mnx; H.miny = mny; H.cell = cl; H.inv_cell = icl; H.inv_celly = icly;
      H.gx = gx; H.gy = gy;
      H.ncell = gx * gy; H.nkey = K * gx * gy;
      H.inv_gy = gy > 0 ? __builtin_amdgcn_rcpf((float)gy) : 0.0f;
      H.xbs = (mnx < mxx && ex < 0x1p60) ? (double)((float)n * __builtin_amdgcn_rcpf((float)ex))
                                         : 0.0;
      // -inf minimum: some coordinate is not an integer below 2^23 (P0), the host relaunches
      // the micrograph with the f64 layout
      H.status = (!W && mnx == -INFINITY) ? RGC_ST_DEFER_WIDE : 0;
      H.C = 0; H.base = 0; H.V = 0; H.target = -1; H.ccur = 0;
      H.tief[0] = H.tief[1] = 0;
      H.qslot = 0;
    }
  }
  __syncthreads();
  if (!W && H.status == RGC_ST_DEFER_WIDE) {
    if (tid == 0) put_stats(A, m, RGC_ST_DEFER_WIDE, 0, 0, 0, 0, 0, 0, 0);
    return;
  }
  const GridU G = grid_u(H);
  const int nk = G.nkey;
  // counting sort by key with packed u16 counters (two keys per LDS word, zeroed in P0).
  // Counts go to slot key + 1, so the exclusive scan leaves bucket q's start in slot q + 1;
  // the scatter's cursors advance it to bucket q's end = bucket q+1's start, which leaves
  // cstart[q] = start of bucket q for q = 0..nk+1 with no rebuild pass.  The key waits in
  // pos[i] between the passes.
  uint32_t* cw = reinterpret_cast<uint32_t*>(S.cstart);
  each_box([&](int i, double xv, double yv) {
    const int q = box_key<W>(G, picker_of<K>(c.pb, i), xv, yv) + 1;
    S.pos[i] = (uint16_t)q;
    atomicAdd(&cw[q >> 1], 1u << (16 * (q & 1)));
  });
  __syncthreads();
  block_scan_dpp32<FWG>(S.cstart, nk + 2, H.redi);
  // arrival order into fwd (free until P2), made deterministic by the placement pass
  uint16_t* arrival = S.fwd;
  each_box([&](int i, double, double) {
    const int q = S.pos[i];
    const int sh = 16 * (q & 1);
    const int t = (atomicAdd(&cw[q >> 1], 1u << sh) >> sh) & 0xFFFF;
    arrival[t] = (uint16_t)i;
  });
  __syncthreads();
  // placement: by local index inside each bucket (buckets hold a few boxes)
  each_box([&](int i, double xv, double yv) {
    const int q = S.pos[i];
    const int lo = S.cstart[q - 1], hi = S.cstart[q];
    int t = lo;
#pragma nounroll
    for (int u = lo; u < hi; ++u) t += (int)arrival[u] < i ? 1 : 0;
    S.scell[t] = (uint16_t)(q - 1);
    S.citems[t] = (uint16_t)i;
    S.pos[i] = (uint16_t)t;
    st_xy<W>(S, t, xv, yv);
  });
  __syncthreads();
  // picker bounds in position space: grid p occupies [pp[p], pp[p+1]); non-finite boxes follow
#pragma unroll
  for (int p = 0; p <= K; ++p) c.pp[p] = ufl(S.cstart[p * G.ncell]);

  STOP_AFTER(1);
  STAMP(2);
  // ---- P2: Jaccard pairs (forward edges to higher pickers): count (JI test, edge bitmask
  // per box) -> scan -> fill (bitmask replay, no atomics) + per-list sort.
  const double B = A.B, two_b2 = A.two_b2;
  // JI > 0.3  <=>  I > (6/13) B^2 exactly; decide without the division unless I lies within a
  // 2^-40 relative band of the threshold, where the reference's f64 quotient is evaluated.
  // Outside the band the quotient's two roundings (< 3e-16 relative) cannot cross 0.3 (the
  // band moves the quotient by >= 1.1e-12 relative), so the decision is the reference's.
  const double t_star = 0.6 * B * B / 1.3;
  const double i_lo = t_star * (1.0 - 0x1p-40), i_hi = t_star * (1.0 + 0x1p-40);
  // f32 layout = integer coordinates (|v| < 2^23) and an integer 1 <= B <= 2896: the overlaps B - |dx| and
  // their product (< 2^24) are exact in f32 and JI > 0.3 <=> I > floor(6 B^2 / 13) (at
  // I = 6 B^2 / 13 the reference's quotient rounds to 0.3 itself, not above it), so the count
  // pass decides every candidate with six f32 operations (edge_test_int)
  // (the f32 layout is integer-only: P0)
  const int ti = W ? 0 : (6 * (int)B * (int)B) / 13;
  const EdgeP<W> ep{(float)B, (float)ti, B, two_b2, i_lo, i_hi};   // (P4's adjacency tests)
  // thread per box (sorted position): lanes of a wave hold neighbouring boxes of one picker,
  // so their stencils overlap (similar trip counts, broadcast LDS reads), and the waves of
  // picker K-1 have nothing to do.  cnt[] (dead until P3) keeps
  // each box's targets (<= 2 edges) or edge bitmask for the fill.
  uint32_t* ccsz = reinterpret_cast<uint32_t*>(S.vrank);   // packed u16 CC sizes (P2-P3)
  // boustrophedon box order: odd rounds walk their FWG positions backwards, so a thread that
  // took a low-picker box (most grids to search) in one round takes a high-picker box (fewest)
  // in the next; K = 3, ~900 boxes: at most 6 instead of 9 column ranges per thread
  for (int r0 = 0, odd = 0; r0 < n; r0 += FWG, odd ^= 1) {
    const int ts = odd ? r0 + FWG - 1 - tid : r0 + tid;
    if (ts >= n) continue;
    Stencil st;
    stencil_setup<K, W>(st, ts, S, G);
    uint32_t mask, first;
    int ec;
    if constexpr (!W) ec = pairs_count_int<K>(st, S, G, (float)B, (float)ti, &mask, &first);
    else ec = pairs_count<K, W>(st, S, G, B, two_b2, i_lo, i_hi, &mask, &first);
    S.fwd[ts] = (uint16_t)ec;
    S.cnt[ts] = mask;
    if (FILL_FAST == 3 && ec == 3) S.vrank[ts] = (uint16_t)first;
  }
  __syncthreads();
  STAMP(3);   // count
  STOP_AFTER(21);
  
  // fwd[n] = E is written by the scan; the status is the same in every thread
  const int E = block_scan_dpp32<FWG>(S.fwd, n, H.redi);
  const int st2 = E == 0 ? RGC_ST_NO_EDGES : (E > A.ecap ? RGC_ST_DEFER : 0);
  if (tid == 0) {
    H.E = E;
    H.status = st2;
  }
  STAMP(4);   // scan
  STOP_AFTER(22);
  bool cc32 = false;   // the unions ran on u32 parents in cnt
  // QG launches: the workgroup's HBM level-tree slot (claimed here when the edge sources do not
  // fit dst's tail: they go to the slot, dead again by P4, which reuses it for the trees)
  int qslot = -1;
  uint16_t* esrc_g = nullptr;
  if constexpr (QG) {
    if (st2 == 0 && 2 * E > A.ecap && A.qg_base) {
      if (tid == 0) H.qslot = qg_claim(A);
      __syncthreads();
      qslot = ufl(H.qslot);
      if (qslot >= 0) esrc_g = reinterpret_cast<uint16_t*>(A.qg_base + (size_t)qslot * A.qg_bytes);
    }
  }
  if (st2 == 0) {
    // fill each list (already sorted: position order) and record each edge's source in dst's
    // unused tail when it has room; then union the edges one thread per edge (lock-free
    // union-find, balanced across lanes whatever the degrees).  Without room: union per box.
    const bool src_ok = 2 * E <= A.ecap || (QG && esrc_g != nullptr);
    uint16_t* esrc = S.dst + E;
    // (QG: esrc_g in HBM when dst's tail is short; separate loops keep esrc's LDS accesses
    // ds_* instructions instead of flat ones)
    const bool src_hbm = QG && esrc_g != nullptr;
    auto fill_walk = [&](int i, int base, int cnt) {
      Stencil st;
      stencil_setup<K, W>(st, i, S, G);
      pairs_fill<K, W>(st, S, G, S.cnt[i], S.dst + base, cnt, B, two_b2, i_lo, i_hi);
    };
    // with room for esrc the unions run after the fill on u32 parents in cnt (each box's
    // count word is dead once its own thread has read it): identity parents written here
    for (int r0 = 0, odd = 0; r0 < n; r0 += FWG, odd ^= 1) {   // same order as the count
      const int ts = odd ? r0 + FWG - 1 - tid : r0 + tid;
      if (ts >= n) continue;
      const int i = ts;
      const int base = S.fwd[i], cnt = (int)S.fwd[i + 1] - base;
      if (cnt > 0) {
        uint16_t* d = S.dst + base;
        if (cnt <= 2) {   // the count kept the targets themselves (ascending)
          const uint32_t cw0 = S.cnt[ts];
          d[0] = (uint16_t)(cnt == 2 ? cw0 >> 16 : cw0);
          if (cnt == 2) d[1] = (uint16_t)cw0;
        } else if (FILL_FAST == 3 && cnt == 3) {
          const uint32_t cw0 = S.cnt[ts];
          d[0] = S.vrank[ts];
          S.vrank[ts] = 0;   // (CC-size slot: zero for P3)
          d[1] = (uint16_t)(cw0 >> 16);
          d[2] = (uint16_t)cw0;
        } else {
          fill_walk(i, base, cnt);
        }
        S.flags[i] = 1;
        if (src_hbm) {
          for (int e = 0; e < cnt; ++e) esrc_g[base + e] = (uint16_t)i;
        } else if (src_ok) {
          for (int e = 0; e < cnt; ++e) esrc[base + e] = (uint16_t)i;
        } else {
          for (int e = 0; e < cnt; ++e) {
            S.flags[d[e]] = 1;
            uf_union_lds(S.parent, (uint32_t)i, (uint32_t)d[e]);
          }
        }
      }
      if (src_ok) S.cnt[ts] = (uint32_t)ts;
    }
    __syncthreads();
    STAMP(5);   // fill
    STOP_AFTER(23);
    if (src_hbm) {
      // sources from HBM (L2) in batches of 8 loads in flight per thread, then the unions
      constexpr int UB = 8;
      for (int e0 = tid; e0 < E; e0 += UB * FWG) {
        uint32_t sv[UB];
#pragma unroll
        for (int u = 0; u < UB; ++u) {
          const int e = e0 + u * FWG;
          sv[u] = e < E ? esrc_g[e] : 0u;
        }
#pragma unroll
        for (int u = 0; u < UB; ++u) {
          const int e = e0 + u * FWG;
          if (e >= E) break;
          const uint32_t h = S.dst[e];
          S.flags[h] = 1;
          uf_union32(S.cnt, sv[u], h);
        }
      }
      __syncthreads();
    } else if (src_ok) {
      for (int e = tid; e < E; e += FWG) {
        const uint32_t h = S.dst[e];
        S.flags[h] = 1;
        uf_union32(S.cnt, esrc[e], h);
      }
      __syncthreads();
    }
    cc32 = src_ok;
    if (A.eu) {
      // RGC_F_EDGES test hook: the edge list with the reference's f64 JI (get_cliques.py:40-46)
      if (tid == 0) H.base = (int64_t)atomicAdd(A.cursor + 2, (unsigned long long)E);
      __syncthreads();
      const int64_t eb = H.base;
      if (eb + E <= A.ecap_out) {
        for (int i = tid; i < n; i += FWG) {
          const double2 a = ld_xy<W>(S, i);
          for (int e = S.fwd[i]; e < (int)S.fwd[i + 1]; ++e) {
            const int h = S.dst[e];
            const double2 b = ld_xy<W>(S, h);
            A.eu[eb + e] = b0 + S.citems[i];
            A.ev[eb + e] = b0 + S.citems[h];
            A.eji[eb + e] = jaccard(a.x, a.y, b.x, b.y, B, two_b2);
          }
        }
      }
      __syncthreads();
      if (tid == 0) H.base = 0;
    }
  }
  if (st2 != 0) {
    if (tid == 0) put_stats(A, m, st2, E, 0, 0, 0, 0, 0, 0);
    return;
  }

  STOP_AFTER(2);
  
  // ---- P3: connected components: the unions ran in the P2 fill; compress, count sizes
  STAMP(6);   // union (one thread per edge)
  for (int i = tid; i < n; i += FWG) {
    if (!S.flags[i]) continue;
    const int e0 = S.fwd[i], e1 = S.fwd[i + 1];
    S.split[i] = (uint16_t)lb16(S.dst, e0, e1, next_picker_end<K>(c.pp, i));   // every node
    const uint32_t r = cc32 ? uf_find32(S.cnt, i) : uf_find_lds(S.parent, i);
    p16_st(S.parent + i, r);
    atomicAdd(&ccsz[r >> 1], 1u << (16 * (r & 1)));
  }
  __syncthreads();
  auto cc_size = [&](uint32_t r) { return (int)((ccsz[r >> 1] >> (16 * (r & 1))) & 0xFFFF); };
  int nodes, cc_max;
  {
    // nodes and roots packed in one 64-bit sum, the largest size in one max; every thread
    // reads the per-wave partials (no thread-0 section and second barrier)
    // nodes << 16 | roots (both <= n < 2^16) in one 32-bit sum
    int nr = 0;
    int mx = 0;
    for (int i = tid; i < n; i += FWG) {
      if (S.flags[i]) {
        nr += 1 << 16;
        if (S.parent[i] == (uint32_t)i) { nr += 1; mx = max(mx, cc_size(i)); }
      }
    }
    nr = wave_incl_add32(nr);
    mx = wave_incl_max32(mx);
    if ((tid & 63) == 63) { H.redi[tid >> 6] = nr; reinterpret_cast<int*>(H.redu)[tid >> 6] = mx; }
    __syncthreads();
    int t = 0;
    int m2 = 0;
#pragma unroll
    for (int w = 0; w < FNW; ++w) {
      t += H.redi[w];
      m2 = max(m2, reinterpret_cast<const int*>(H.redu)[w]);
    }
    nodes = t >> 16;
    cc_max = m2;
    if (tid == 0) { H.nodes = nodes; H.cc_cnt = t & 0xFFFF; H.cc_max = cc_max; }
  }
  // (no barrier: the P4 passes below start with their own before touching the reduction
  // slots, and no array read here is written before it)
  const bool get_cc = (A.flags & 1) != 0;
  int target = -1;
  if (get_cc) {
    // largest CC; ties -> the component whose first edge comes first in the enumeration
    uint64_t best = ~0ULL;
    for (int i = tid; i < n; i += FWG) {
      const int e0 = S.fwd[i], e1 = S.fwd[i + 1];
      if (e0 == e1) continue;
      const uint32_t r = S.parent[i];
      if (cc_size(r) != cc_max) continue;
      // the box's first edge in enumeration order: lowest target picker (the first segment
      // of the position-sorted list), smallest file index inside it
      const int pi = picker_of<K>(c.pp, i);
      const int h0 = S.dst[e0];
      const int ph = picker_of<K>(c.pp, h0);
      const int se = lb16(S.dst, e0, e1, picker_end<K>(c.pp, h0));
      int hmin = 1 << 30;
      for (int e = e0; e < se; ++e) hmin = min(hmin, (int)S.citems[S.dst[e]]);
      const uint64_t key = ((uint64_t)pair_index(pi, ph, K) << 48) |
                           ((uint64_t)(S.citems[i] - picker_begin<K>(c.pb, pi)) << 32) |
                           ((uint64_t)(hmin - picker_begin<K>(c.pb, ph)) << 16) | r;
      best = key < best ? key : best;
    }
    // redu is not aliased by red64/redi (only P0's red4 covers it): one barrier
    best = wave_incl_scan(best, [](uint64_t a, uint64_t b) { return a < b ? a : b; });
    if ((tid & 63) == 63) H.redu[tid >> 6] = best;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < FNW; ++w) best = H.redu[w] < best ? H.redu[w] : best;
    target = (int)(best & 0xFFFF);
    if (tid == 0) H.target = target;
  }

  STOP_AFTER(3);
  STAMP(7);   // CC stats
  // ---- P4: k-cliques (level-synchronous BFS into the queue region; per-root DFS counts as the
  // fallback when a level does not fit), vertex marking, output reservation
  c.set_order = 2 * K < nodes;
  const int n0 = c.pp[1];   // roots: picker-0 positions
  // queue region: after the E used entries of dst through the cell starts (contiguous: dst
  // immediately precedes the cell starts in the layout)
  const int qoff = (L.off_dst + 2 * H.E + 15) & ~15;
  const int qbytes_lds = L.off_parent - qoff;
  char* q = smem + qoff;
  int qbytes = qbytes_lds;
  if constexpr (QG) {
    // large micrographs: the level trees in an HBM slot (no root chunks to re-walk), the
    // LDS region when no slot is free (P2 may have claimed the slot already for esrc)
    if (qslot < 0) {
      if (tid == 0) H.qslot = A.qg_base ? qg_claim(A) : -1;
      __syncthreads();
      qslot = ufl(H.qslot);
    }
    if (qslot >= 0) {
      q = A.qg_base + (size_t)qslot * (size_t)A.qg_bytes;
      qbytes = A.qg_bytes;
    }
  }
  // wide level-tree entries (members, not parent chains) in the HBM slot
  const bool we = QG && K <= 4 && qslot >= 0;
  // Root chunks: all roots at once when the levels fit the queue region, else consecutive
  // root ranges (halved after a level overflows, doubled after a success).  Chunk i covers
  // roots [rs[i], rs[i+1]) and cliques [cs[i], cs[i+1]) of the micrograph's lexicographic
  // order; the table lives in cnt behind the n0 entries the level-2 counts use.  A chunk's
  // tree is rebuilt in P6 (BFS REWALK), except the last one, still in the queue region.
  uint32_t* const chtab = S.cnt + n0 + 1;
  // (K = 3 keeps one attempt: the rebuild in P6 would push it past its 64-VGPR budget, and
  // its level trees rarely overflow)
  const int maxch = K >= 4 ? min(64, (n + 3 - n0) / 2 - 1) : 1;
  BfsOut<K> bo;
  int nch = 0;
  int64_t C = 0;
  {
    int r0 = 0, len = n0;
    bool ok = maxch >= 1;
    if (tid == 0) { chtab[0] = 0; chtab[1] = 0; }
    while (ok && r0 < n0) {
      len = min(len, n0 - r0);
      if (QG && K <= 4 && qslot >= 0)
        bo = bfs_cliques<K, false, NT, QG && K <= 4>(S, H, q, qbytes, r0, r0 + len, get_cc,
                                                     (uint32_t)target, tid, c.pp, ep);
      else
        bo = bfs_cliques<K, false, NT>(S, H, q, qbytes, r0, r0 + len, get_cc, (uint32_t)target,
                                       tid, c.pp, ep);
      if (bo.C < 0) {
        // shrink to the estimated fit of the overflowing level (demand grows about linearly
        // with the roots), with a small margin; strictly smaller each time
        ok = K >= 4 && len > 1;
        len = max(1, min(len - 1, (int)((float)len * bo.fit * 0.95f)));
        continue;
      }
      if (nch == maxch) { ok = false; break; }
      C += bo.C;
      r0 += len;
      ++nch;
      if (tid == 0) { chtab[2 * nch] = (uint32_t)r0; chtab[2 * nch + 1] = (uint32_t)C; }
      // next chunk: as many roots as the tightest level of this one leaves room for
      len = max(len + 1, (int)((float)len * fminf(bo.fit, 2.0f) * 0.95f));
    }
    if (!ok) { nch = 0; C = 0; bo.C = -1; }
  }
  const bool bfs_ok = nch > 0;
  if (bfs_ok) {
    // cliques = level-K tree entries (members by walking parents); their flag words follow
    c.cq_cap = (int)max(bo.C, (int64_t)1);
    c.cq_ord = reinterpret_cast<uint16_t*>(q + bo.lvl[K] + (we ? 8 : 4) * (int)bo.C);
  } else {
    S.cbuf = reinterpret_cast<uint16_t*>(smem + qoff);   // (LDS even when QG)
    c.cq_cap = 0;   // the DFS only counts; P6 re-walks it chunk by chunk
    c.ccur = &H.ccur;
    for (int r = tid; r < n0; r += FWG) {
      uint32_t cntr = 0;
      if (S.fwd[r] < S.fwd[r + 1] && (!get_cc || S.parent[r] == (uint32_t)target)) {
        int mem[K];
        mem[0] = r;
        c.count = 0;
        FLevel<K, 1, false>::run(c, mem);
        cntr = (uint32_t)c.count;
      }
      S.cnt[r] = cntr;
    }
    __syncthreads();
    C = block_scan_dpp<FWG>(S.cnt, n0, H.red64);
    if (tid == 0) S.cnt[n0] = (uint32_t)C;
    c.cq_cap = qbytes_lds / (2 * K + 2);
    c.cq_ord = S.cbuf + (size_t)c.cq_cap * K;
  }
  c.S.cbuf = S.cbuf;
  STAMP(8);   // cliques
#ifdef RGC_STAMPS
  if (tid == 0) {   // diagnostic build: root chunks of the BFS (0 = DFS fallback) and cliques
    A.stamps[(int64_t)blockIdx.x * STAMP_SLOTS + 14] = (unsigned long long)nch;
    A.stamps[(int64_t)blockIdx.x * STAMP_SLOTS + 15] = (unsigned long long)C;
  }
#endif
  // the output reservation: one returning atomic on the batch cursor per micrograph.  Its
  // result is first needed by P6, so thread 0 only reads it at the end of P5: the round trip
  // (microseconds with every CU's workgroups on the one cursor word) overlaps P5
  unsigned long long resv = 0;
  if (tid == 0) {
    H.C = C;
    if (C == 0) {
      H.status = RGC_ST_NO_CLIQUES;
    } else if (C > 0x7fffffff) {
      H.status = RGC_ST_DEFER;   // P6 indexes a micrograph's cliques in 32 bits
    } else {
      // (a lane-varying zero offset keeps the atomic optimizer's wave-reduction expansion,
      // which consumes the result at once, off this single-lane atomic)
      int vz;
      asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
      resv = atomicAdd(A.cursor + vz, (unsigned long long)C);
    }
  }
  __syncthreads();

  STOP_AFTER(4);
  STAMP(9);   // scan + reserve
  // ---- P5: row index = rank of each clique vertex by (x, y, id).  Counting sort of the
  // vertices by a fine x bucket (n buckets over the x extent; monotone in x), then rank inside
  // the bucket.  The grid arrays of P1 are dead: parent holds the bucket counters, scell the
  // vertices (sorted positions) in bucket order.
  if (H.status == 0) {
    // bucket counts as packed u16 (two per LDS word; a bucket holds < 2^16 vertices) in the
    // dead union-find parents
    uint16_t* bcnt = S.parent;
    uint32_t* bw = reinterpret_cast<uint32_t*>(S.parent);
    uint16_t* blist = S.scell;
    // f32 layout: coordinates exact as floats, so bucket and (x, y) comparisons run on floats
    // (same order); the bucket map only has to be monotone in x and the same in every pass
    using CT = typename std::conditional<W, double, float>::type;
    using CT2 = typename std::conditional<W, double2, float2>::type;
    auto ld = [&](int t) -> CT2 { return reinterpret_cast<const CT2*>(S.sxy)[t]; };
    const CT minx = (CT)H.minx, xbs = (CT)H.xbs, nlast = (CT)(n - 1);
    auto xbucket = [&](CT xv) { return (int)fmin((xv - minx) * xbs, nlast); };
    for (int q = tid; q <= (n + 1) / 2; q += FWG) bw[q] = 0;
    __syncthreads();
    for (int t = tid; t < n; t += FWG) {
      if (S.flags[t] != 3) continue;
      const int q = xbucket(ld(t).x);
      const int sh = 16 * (q & 1);
      S.vrank[t] = (uint16_t)((atomicAdd(&bw[q >> 1], 1u << sh) >> sh) & 0xFFFFu);
    }
    __syncthreads();
    const int V = block_scan_dpp32<FWG>(bcnt, n, H.redi);
    if (tid == 0) { H.V = (int)V; bcnt[n] = (uint16_t)V; }
    for (int t = tid; t < n; t += FWG) {
      if (S.flags[t] != 3) continue;
      blist[bcnt[xbucket(ld(t).x)] + S.vrank[t]] = (uint16_t)t;
    }
    __syncthreads();
    // ranks over the dense bucket-ordered vertex list (every lane holds a vertex; the
    // position loop above skips the non-vertices)
    for (int u0 = tid; u0 < V; u0 += FWG) {
      const int t = blist[u0];
      const int vi = S.citems[t];
      const CT2 v = ld(t);
      const int b = xbucket(v.x);
      const int lo = bcnt[b], hi = bcnt[b + 1];
      uint32_t rk = lo;
      for (int u = lo; u < hi; ++u) {
        const int tu = blist[u];
        const CT2 w = ld(tu);
        const int ui = S.citems[tu];
        rk += (w.x < v.x) || (w.x == v.x && (w.y < v.y || (w.y == v.y && ui < vi)));
      }
      S.vrank[t] = (uint16_t)rk;
    }
    if (tid == 0) H.base = (int64_t)resv;   // (the reservation's round trip ends here)
    __syncthreads();
    // every thread reads the base; an output overflow skips P6 (the host regrows and re-runs)
    const bool overflow = H.base + H.C > A.cap;
    if (overflow && tid == 0) H.status = RGC_ST_OVERFLOW;

    STOP_AFTER(5);
    STAMP(10);  // rank
    if (!overflow) {
    // ---- P6: stage the clique vertices' scores in LDS, then the ILP epilogue + COO rows with
    // one thread per clique (coalesced output stores).  Cliques come from the P4 queue, whose
    // output index is (root's scanned offset + ordinal within the root): the same order as a
    // sequential root-by-root walk.  Micrographs whose cliques overflowed the queue re-walk
    // the DFS per chunk of <= cq_cap cliques.
    // scores of the clique vertices into LDS by row rank when they fit in parent..scell
    c.S.vstaged = 8 * H.V <= L.off_citems - L.off_parent;
    if (c.S.vstaged) {
      for (int t = tid; t < n; t += FWG)
        if (S.flags[t] == 3) c.S.vscore[S.vrank[t]] = c.score[b0 + S.citems[t]];
      __syncthreads();
    }

    STAMP(11);  // score staging
    // per chunk of queued cliques: main pass (thread per clique), then the order pass over
    // the cliques it flagged (bit 15 of the slot's ordinal word; the slot's output index is
    // kept in the low bits).  Micrographs whose cliques overflowed the queue re-walk the DFS
    // per chunk of <= cq_cap cliques into the same buffer.
    // chunk bounds and the output base are wave-uniform and 32-bit (C < 2^31, checked at the
    // reservation): they live in SGPRs instead of spilled 64-bit VGPR pairs
    const int Cm = ufl((int)H.C);
    const int cap = ufl(c.cq_cap);
    const int64_t obase = (int64_t)(((uint64_t)(uint32_t)ufl((int)(H.base >> 32)) << 32) |
                                    (uint32_t)ufl((int)H.base));
    // BFS: root chunk by chunk (the last one first: its tree is still in the queue region,
    // the others are rebuilt there); DFS fallback: chunks of <= cap cliques re-walked into cbuf
    const int nit = bfs_ok ? nch : (Cm + cap - 1) / cap;
    BfsOut<K> cur = bo;
    for (int ci = 0; ci < nit; ++ci) {
      int c0, c1;
      if (tid == 0) H.tief[(ci + 1) & 1] = 0;   // last read before the previous chunk's end
      if (bfs_ok) {
        const int ch = ci == 0 ? nch - 1 : ci - 1;
        c0 = ufl((int)chtab[2 * ch + 1]);
        c1 = ufl((int)chtab[2 * ch + 3]);
        if constexpr (K >= 4) {
          if (ci > 0)
            cur = we ? bfs_cliques<K, true, NT, QG && K <= 4>(S, H, q, qbytes, ufl((int)chtab[2 * ch]),
                                       ufl((int)chtab[2 * ch + 2]), get_cc, (uint32_t)target,
                                       tid, c.pp, ep)
                     : bfs_cliques<K, true, NT>(S, H, q, qbytes, ufl((int)chtab[2 * ch]),
                                       ufl((int)chtab[2 * ch + 2]), get_cc, (uint32_t)target,
                                       tid, c.pp, ep);
        }
        c.cq_ord = reinterpret_cast<uint16_t*>(q + cur.lvl[K] + (we ? 8 : 4) * (c1 - c0));
      } else {
        c0 = ci * cap;
        c1 = min(Cm, c0 + cap);
        c.c0 = c0;
        c.c1 = c1;
        for (int r = tid; r < n0; r += FWG) {
          const int64_t lo = S.cnt[r], hi = S.cnt[r + 1];
          if (lo == hi || hi <= c0 || lo >= c1) continue;
          int mem[K];
          mem[0] = r;
          c.out = lo;
          FLevel<K, 1, true>::run(c, mem);
        }
        __syncthreads();
      }
      // members of chunk slot sl: BFS tree walk or the re-walk buffer; the output index of
      // the slot; the order-pass flag of the slot
      auto clique_members = [&](int sl, int (&mem)[K]) -> int64_t {
        if (bfs_ok) {
          if (we) BfsLevel<K, K, NT, QG && K <= 4>::prefix(q, cur.lvl, (uint32_t)sl, mem);
          else BfsLevel<K, K, NT>::prefix(q, cur.lvl, (uint32_t)sl, mem);
        } else {
          const uint16_t* sb = S.cbuf + sl * K;
#pragma unroll
          for (int i = 0; i < K; ++i) mem[i] = sb[i];
        }
        return obase + (c0 + sl);
      };
      auto set_order_flag = [&](int sl) {
        c.cq_ord[sl] |= 0x8000;
      };
      auto order_flag = [&](int sl) -> bool {
        return (c.cq_ord[sl] & 0x8000) != 0;
      };
      bool any = false;
      auto epi = [&](int sl, int (&mem)[K]) {
        const int64_t jo = obase + (c0 + sl);
        bool order;
        if constexpr (!W) order = fused_epilogue_main<K, W, true>(c, jo, mem);
        else order = fused_epilogue_main<K, W, false>(c, jo, mem);
        if (order) {
          set_order_flag(sl);
          any = true;
        }
      };
      if constexpr (QG && K <= 4) {
        if (bfs_ok && we) {
          // wide entries in the HBM slot: the next clique's members are loaded before this
          // one's epilogue runs (an L2 round trip per clique otherwise sits on the chain)
          const uint2* ent = reinterpret_cast<const uint2*>(q + cur.lvl[K]);
          const int cnt = c1 - c0;
          uint2 nx = tid < cnt ? ent[tid] : make_uint2(0u, 0u);
          for (int sl = tid; sl < cnt; sl += FWG) {
            const uint2 v = nx;
            if (sl + FWG < cnt) nx = ent[sl + FWG];
            const int t[4] = {(int)(v.x & 0xFFFF), (int)(v.x >> 16), (int)(v.y & 0xFFFF),
                              (int)(v.y >> 16)};
            int mem[K];
#pragma unroll
            for (int i = 0; i < K; ++i) mem[i] = t[i];
            epi(sl, mem);
          }
        } else {
          for (int sl = tid; sl < c1 - c0; sl += FWG) {
            int mem[K];
            clique_members(sl, mem);
            epi(sl, mem);
          }
        }
      } else {
        for (int sl = tid; sl < c1 - c0; sl += FWG) {
          int mem[K];
          clique_members(sl, mem);
          epi(sl, mem);
        }
      }
      if (any) H.tief[ci & 1] = 1;
      __syncthreads();
      if (H.tief[ci & 1]) {
        for (int sl = tid; sl < c1 - c0; sl += FWG) {
          if (!order_flag(sl)) continue;
          int mem[K];
          const int64_t jo = clique_members(sl, mem);
          fused_epilogue_order<K, W>(c, jo, mem);
        }
      }
      __syncthreads();
    }
    }   // !overflow
  }
  STAMP(12);
#ifdef RGC_STAMPS
  if (tid == 0)
    A.stamps[(int64_t)blockIdx.x * STAMP_SLOTS + 13] =
        ((unsigned long long)(uint32_t)__builtin_amdgcn_s_memrealtime() << 32) | rt0;
#endif
  if constexpr (QG) {
    if (qslot >= 0) {   // every thread is done with the slot
      __syncthreads();
      if (tid == 0) {
        __threadfence();
        atomicAnd(A.qg_slots + (qslot >> 5), ~(1u << (qslot & 31)));
      }
    }
  }
  if (tid == 0)
    put_stats(A, m, H.status, H.E, H.nodes, H.cc_cnt, H.cc_max, H.V, H.base, H.C);
}

// Consensus on set-order ties and the --multi_out node order of the cliques the fused kernel
// appended (fused_epilogue_order): networkx iterates set(sorted(clique)) (get_cliques.py:182-183
// -> CPython set order of the (x, y, id) node keys, pyset.h), first tied member in that order.
// Grid-stride over the entries [from, cursor[CUR_TIES]).
template <int K>
__global__ __launch_bounds__(256) void k_fused_ties(FusedArgs A, int64_t from) {
  if (A.esum_n > 0 && blockIdx.x < 16) {
    // edges of the finished micrographs into cursor[1]: 16 workgroups, one atomic each
    __shared__ int64_t red[4];
    int64_t e = 0;
    for (int m = blockIdx.x * 256 + threadIdx.x; m < A.esum_n; m += 16 * 256) {
      const int st = A.o.status[m];
      if (st == 0 || st == RGC_ST_NO_CLIQUES || st == RGC_ST_NO_EDGES) e += A.o.n_edges[m];
    }
    e = block_sum64<256>(e, red);
    if (threadIdx.x == 0 && e) atomicAdd(A.cursor + 1, (unsigned long long)e);
  }
  const int64_t n = min((int64_t)__hip_atomic_load(A.cursor + CUR_TIES, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT), A.tie_cap);
  for (int64_t t = from + (int64_t)blockIdx.x * 256 + threadIdx.x; t < n;
       t += (int64_t)gridDim.x * 256) {
    const int32_t* e = A.tie_list + t * (4 + K);
    const int64_t j = (int64_t)(((uint64_t)(uint32_t)e[1] << 32) | (uint32_t)e[0]);
    const int m = e[2];
    const uint32_t fl = (uint32_t)e[3];
    const int64_t idb = A.id_base[m] - (int64_t)A.box_off[m * K];
    int mem[K];
    double xs[K], ys[K];
    int64_t ids[K];
    const uint64_t ins[K] = {};
#pragma unroll
    for (int i = 0; i < K; ++i) {
      mem[i] = e[4 + i];
      xs[i] = A.x[mem[i]];
      ys[i] = A.y[mem[i]];
      ids[i] = idb + mem[i];
    }
    const uint32_t ord = node_order<K>(mem, xs, ys, ids, true, ins);
    if (fl & 0x10000u) A.consensus[j] = mem[epi_tie_arg<K>(fl & 0xFFFFu, ord)];
    if (fl & 0x20000u) {
#pragma unroll
      for (int i = 0; i < K; ++i) A.order[j * K + i] = (uint8_t)((ord >> (4 * i)) & 15);
    }
  }
  if (A.host_stats) {
    // the per-micrograph stats to the host, every workgroup a slice (final: the fused launches
    // before this one wrote them; the kernel's end makes the writes visible to the host)
    const int64_t n16 = A.stats_bytes / 16;
    const uint4* src = reinterpret_cast<const uint4*>(A.stats_dev);
    uint4* dst = reinterpret_cast<uint4*>(A.host_stats);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256)
      dst[i] = src[i];
  }
}

int launch_fused_ties(hipStream_t stream, const FusedArgs& A, int64_t from) {
  if (!A.tie_list || A.tie_cap <= from) return 0;
  // (256 workgroups: 32 were 6 % slower on C4, whose steps hold thousands of tie entries)
  const dim3 g(256), b(256);
  switch (A.k) {
#define RGC_TIES_CASE(KK) \
  case KK: hipLaunchKernelGGL((k_fused_ties<KK>), g, b, 0, stream, A, from); break;
    RGC_TIES_CASE(2) RGC_TIES_CASE(3) RGC_TIES_CASE(4) RGC_TIES_CASE(5) RGC_TIES_CASE(6)
    RGC_TIES_CASE(7) RGC_TIES_CASE(8)
#undef RGC_TIES_CASE
    default:
      return -1;
  }
  return (int)hipGetLastError();
}

template <int K, bool W, int NT, bool QG = false>
static int launch_fused_t(hipStream_t stream, int n_blocks, int lds_bytes, const FusedArgs& A) {
  static std::atomic<uint64_t> attr_set{0};   // per device
#ifdef RGC_STAMPS
  constexpr int kStaticLds = 256;   // (diagnostic build: g_bwait is static LDS)
#else
  constexpr int kStaticLds = 0;
#endif
  const hipError_t e = set_dyn_lds_once(attr_set, reinterpret_cast<const void*>(&k_fused<K, W, NT, QG>),
                                        160 * 1024 - kStaticLds);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL((k_fused<K, W, NT, QG>), dim3(n_blocks), dim3(NT), lds_bytes, stream, A);
  return (int)hipGetLastError();
}

template <int K, bool W, int NT, bool QG = false>
static int fused_vgprs_t() {
  hipFuncAttributes at;
  if (hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&k_fused<K, W, NT, QG>)) != hipSuccess)
    return -1;
  return at.numRegs;
}

// workgroup sizes compiled for k (fused_nt_ok) and their dispatch
bool fused_nt_ok(int k, int nt) {
  if (k < 2 || k > 8) return false;
  return nt == 512 || ((nt == 768 || nt == 1024) && k <= 5) ||
         ((nt == 256 || nt == 384) && k <= 3);
}

template <int K, bool W>
static int fused_vgprs_k(int nt) {
  if constexpr (K <= 3) {
    if (nt == 256) return fused_vgprs_t<K, W, 256>();
    if (nt == 384) return fused_vgprs_t<K, W, 384>();
  }
  if constexpr (K <= 5) {
    if (nt == 768) return fused_vgprs_t<K, W, 768>();
    if (nt == 1024) return fused_vgprs_t<K, W, 1024, (K == 4)>();
  }
  return nt == 512 ? fused_vgprs_t<K, W, 512>() : -1;
}

template <int K, bool W>
static int launch_fused_k(hipStream_t stream, int n_blocks, int lds_bytes, const FusedArgs& A,
                          int nt) {
  if constexpr (K <= 3) {
    if (nt == 256) return launch_fused_t<K, W, 256>(stream, n_blocks, lds_bytes, A);
    if (nt == 384) return launch_fused_t<K, W, 384>(stream, n_blocks, lds_bytes, A);
  }
  if constexpr (K <= 5) {
    if (nt == 768) return launch_fused_t<K, W, 768>(stream, n_blocks, lds_bytes, A);
    // 1024 threads (LDS admits one workgroup per CU): K = 4 level trees in HBM slots (K = 5
    // keeps the LDS queue: the flat pointers would push it past 128 VGPRs into scratch)
    if (nt == 1024) return launch_fused_t<K, W, 1024, (K == 4)>(stream, n_blocks, lds_bytes, A);
  }
  return nt == 512 ? launch_fused_t<K, W, 512>(stream, n_blocks, lds_bytes, A) : -1;
}

int fused_vgprs(int k, bool wide, int nt) {
  if (!fused_nt_ok(k, nt)) return -1;
  switch (k) {
#define RGC_VG_CASE(KK) \
  case KK: return wide ? fused_vgprs_k<KK, true>(nt) : fused_vgprs_k<KK, false>(nt);
    RGC_VG_CASE(2) RGC_VG_CASE(3) RGC_VG_CASE(4) RGC_VG_CASE(5) RGC_VG_CASE(6) RGC_VG_CASE(7)
    RGC_VG_CASE(8)
#undef RGC_VG_CASE
    default:
      return -1;
  }
}

int launch_fused(hipStream_t stream, int n_blocks, int lds_bytes, const FusedArgs& A, bool wide,
                 int nt) {
  if (n_blocks <= 0) return 0;
  if (!fused_nt_ok(A.k, nt)) return -1;
  switch (A.k) {
#define RGC_FUSED_CASE(KK)                                                            \
  case KK:                                                                            \
    return wide ? launch_fused_k<KK, true>(stream, n_blocks, lds_bytes, A, nt)        \
                : launch_fused_k<KK, false>(stream, n_blocks, lds_bytes, A, nt);
    RGC_FUSED_CASE(2)
    RGC_FUSED_CASE(3)
    RGC_FUSED_CASE(4)
    RGC_FUSED_CASE(5)
    RGC_FUSED_CASE(6)
    RGC_FUSED_CASE(7)
    RGC_FUSED_CASE(8)
#undef RGC_FUSED_CASE
    default:
      return -1;
  }
  return 0;
}

}  // namespace rgc
