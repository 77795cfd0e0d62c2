// rgc_fused.hip — the whole get_cliques hot path for one micrograph in ONE workgroup.
//
// Everything between reading a micrograph's boxes and writing its ILP structures stays in
// LDS: boxes (f64 x/y), the uniform grid (x-major cells, side >= box_size), the forward
// adjacency CSR (u16 targets), union-find, the clique DFS and the vertex ranks.  HBM sees
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

#include "rgc_device.h"
#include "rgc_kernels.h"

namespace rgc {

struct FusedHdr {
  double redd[NW];
  int64_t red64[NW];
  uint64_t redu[NW];
  int redi[NW];
  double minx, miny, cell;
  int gx, gy, ncell;
  int E, nodes, cc_cnt, cc_max, target, V, status;
  int64_t C, base;
};

__host__ __device__ inline FusedLayout fused_layout(int nmax, int ecap) {
  FusedLayout L;
  auto al = [](int v) { return (v + 15) & ~15; };
  int o = al((int)sizeof(FusedHdr));
  L.off_xs = o; o += al(8 * nmax);
  L.off_ys = o; o += al(8 * nmax);
  L.off_cstart = o; o += al(4 * (nmax + 4));
  L.off_cnt = o; o += al(4 * (nmax + 4));
  L.off_fwd = o; o += al(4 * (nmax + 4));
  L.off_parent = o; o += al(4 * (nmax + 4));
  L.off_citems = o; o += al(2 * nmax);
  L.off_vrank = o; o += al(2 * nmax);
  L.off_flags = o; o += al(nmax);
  L.off_dst = o; o += al(2 * ecap);
  L.total = o;
  return L;
}

int fused_lds_bytes(int nmax, int ecap) { return fused_layout(nmax, ecap).total; }

struct FShared {
  double* xs;
  double* ys;
  uint32_t* cstart;
  uint32_t* cnt;
  uint32_t* fwd;
  uint32_t* parent;
  uint16_t* citems;
  uint16_t* vrank;
  uint8_t* flags;   // 0: no edge, 1: graph node, 3: clique vertex
  uint16_t* dst;
};

template <int K>
struct FCtx {
  const FusedArgs* A;
  FShared S;
  int pb[K + 1];     // picker bounds (local box indices)
  int m, b0, n;
  int64_t idb;       // global id of local box 0
  bool set_order;    // networkx iterates set(sorted(clique)) (2k < |G|)
  int64_t out;       // next output clique index (fill)
  int64_t count;
};

__device__ __forceinline__ uint32_t lds_ld(uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t uf_find_lds(uint32_t* parent, uint32_t x) {
  for (;;) {
    const uint32_t p = lds_ld(parent + x);
    if (p == x) return x;
    const uint32_t gp = lds_ld(parent + p);
    if (gp != p) lds_st(parent + x, gp);
    x = gp;
  }
}

template <int K>
__device__ __forceinline__ int picker_of(const int (&pb)[K + 1], int i) {
  int p = 0;
#pragma unroll
  for (int q = 1; q < K; ++q) p += (i >= pb[q]);
  return p;
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

__device__ __forceinline__ int cell_xm(const FusedHdr& H, double x, double y, int* cx, int* cy) {
  if (H.ncell == 0 || !isfinite(x) || !isfinite(y)) return H.ncell;
  *cx = (int)fmin(floor((x - H.minx) / H.cell), (double)(H.gx - 1));
  *cy = (int)fmin(floor((y - H.miny) / H.cell), (double)(H.gy - 1));
  return *cx * H.gy + *cy;
}

// graph insertion key of a clique vertex (tiny graphs only): first appearance of the node in
// the edge enumeration (picker pair, a index, b index, side), get_cliques.py:33-34,135-143
template <int K>
__device__ uint64_t ins_key(const FCtx<K>& c, int u) {
  const int pu = picker_of<K>(c.pb, u);
  const int lu = u - c.pb[pu];
  for (int a = 0; a < c.pb[pu]; ++a) {
    if (contains16(c.S.dst, c.S.fwd[a], c.S.fwd[a + 1], u)) {
      const int qa = picker_of<K>(c.pb, a);
      return ((uint64_t)pair_index(qa, pu, K) << 49) | ((uint64_t)(a - c.pb[qa]) << 25) |
             ((uint64_t)lu << 1) | 1ULL;
    }
  }
  const int d0 = c.S.dst[c.S.fwd[u]];
  const int pd = picker_of<K>(c.pb, d0);
  return ((uint64_t)pair_index(pu, pd, K) << 49) | ((uint64_t)lu << 25) |
         ((uint64_t)(d0 - c.pb[pd]) << 1);
}

template <int K>
__device__ void fused_emit(FCtx<K>& c, const int (&mem)[K]) {
  const FusedArgs& A = *c.A;
  const int64_t j = c.out++;
  double ji[K][K], s[K], xs[K], ys[K];
  int64_t ids[K];
  uint64_t ins[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    xs[i] = c.S.xs[mem[i]];
    ys[i] = c.S.ys[mem[i]];
    s[i] = A.score[c.b0 + mem[i]];
    ids[i] = c.idb + mem[i];
  }
#pragma unroll
  for (int a = 0; a < K; ++a)
#pragma unroll
    for (int b = a + 1; b < K; ++b) ji[a][b] = jaccard(xs[a], ys[a], xs[b], ys[b], A.B, A.two_b2);
  const bool multi = (A.flags & 2) != 0;
  if (!c.set_order) {
    for (int i = 0; i < K; ++i) ins[i] = ins_key<K>(c, mem[i]);
  }
  Epi<K> e;
  epilogue<K>(mem, ji, s, xs, ys, ids, c.set_order, ins, multi, e);
  int r[K];
#pragma unroll
  for (int i = 0; i < K; ++i) r[i] = c.S.vrank[mem[i]];
#pragma unroll
  for (int i = 0; i < K; ++i)
#pragma unroll
    for (int q = 0; q < K - 1 - i; ++q) {
      const int a = r[q], b = r[q + 1];
      r[q] = min(a, b);
      r[q + 1] = max(a, b);
    }
#pragma unroll
  for (int i = 0; i < K; ++i) A.rows[j * K + i] = r[i];
  A.w[j] = e.w;
  A.conf[j] = e.conf;
  A.consensus[j] = c.b0 + mem[e.arg];
  if (A.flags & (2 | 32)) {
#pragma unroll
    for (int i = 0; i < K; ++i) A.members[j * K + i] = c.b0 + mem[i];
  }
  if (multi) {
#pragma unroll
    for (int i = 0; i < K; ++i) A.order[j * K + i] = (uint8_t)e.ord[i];
  }
}

// Static-recursion DFS: level D picks the picker-D member among the forward neighbours of
// the picker-(D-1) member that are also forward neighbours of every earlier member.
template <int K, int D, bool FILL>
struct FLevel {
  __device__ static void run(FCtx<K>& c, int (&mem)[K]) {
    const int prev = mem[D - 1];
    const int l0 = c.S.fwd[prev], h0 = c.S.fwd[prev + 1];
    const int lo = lb16(c.S.dst, l0, h0, c.pb[D]);
    const int hi = lb16(c.S.dst, lo, h0, c.pb[D + 1]);
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
  __device__ static void run(FCtx<K>& c, int (&mem)[K]) {
    if (FILL) {
      fused_emit<K>(c, mem);
    } else {
      ++c.count;
#pragma unroll
      for (int i = 0; i < K; ++i) c.S.flags[mem[i]] = 3;
    }
  }
};

template <int K>
__global__ __launch_bounds__(WG) void k_fused(FusedArgs A) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  FusedHdr& H = *reinterpret_cast<FusedHdr*>(smem);
  const FusedLayout L = fused_layout(A.nmax, A.ecap);
  FShared S;
  S.xs = reinterpret_cast<double*>(smem + L.off_xs);
  S.ys = reinterpret_cast<double*>(smem + L.off_ys);
  S.cstart = reinterpret_cast<uint32_t*>(smem + L.off_cstart);
  S.cnt = reinterpret_cast<uint32_t*>(smem + L.off_cnt);
  S.fwd = reinterpret_cast<uint32_t*>(smem + L.off_fwd);
  S.parent = reinterpret_cast<uint32_t*>(smem + L.off_parent);
  S.citems = reinterpret_cast<uint16_t*>(smem + L.off_citems);
  S.vrank = reinterpret_cast<uint16_t*>(smem + L.off_vrank);
  S.flags = reinterpret_cast<uint8_t*>(smem + L.off_flags);
  S.dst = reinterpret_cast<uint16_t*>(smem + L.off_dst);
  const int tid = threadIdx.x;
  const int m = A.mg_list[blockIdx.x];
  FCtx<K> c;
  c.A = &A;
  c.S = S;
  c.m = m;
  c.b0 = A.box_off[m * K];
  c.n = A.box_off[m * K + K] - c.b0;
#pragma unroll
  for (int i = 0; i <= K; ++i) c.pb[i] = A.box_off[m * K + i] - c.b0;
  c.idb = A.id_base[m];
  const int n = c.n, b0 = c.b0;

  // ---- P0: load coordinates, bounding box
  double mnx = INFINITY, mny = INFINITY, mxx = -INFINITY, mxy = -INFINITY;
  for (int i = tid; i < n; i += WG) {
    const double xv = A.x[b0 + i], yv = A.y[b0 + i];
    S.xs[i] = xv;
    S.ys[i] = yv;
    if (isfinite(xv) && isfinite(yv)) {
      mnx = fmin(mnx, xv); mxx = fmax(mxx, xv);
      mny = fmin(mny, yv); mxy = fmax(mxy, yv);
    }
  }
  mnx = block_min(mnx, H.redd);
  mny = block_min(mny, H.redd);
  mxx = block_max(mxx, H.redd);
  mxy = block_max(mxy, H.redd);

  // ---- P1: grid (x-major cells, side >= box_size, at most n + 1 cells)
  if (tid == 0) {
    H.minx = mnx; H.miny = mny; H.cell = A.B; H.gx = 0; H.gy = 0; H.ncell = 0;
    H.status = 0; H.C = 0; H.base = 0; H.V = 0; H.target = -1;
    if (mnx <= mxx && A.B > 0.0) {
      const double ex = mxx - mnx, ey = mxy - mny;
      if (!(ex < 0x1p40 && ey < 0x1p40)) {
        H.cell = INFINITY; H.gx = 1; H.gy = 1;
      } else {
        double cl = A.B;
        for (;;) {
          const double fx = floor(ex / cl) + 1.0, fy = floor(ey / cl) + 1.0;
          if (fx * fy <= (double)(n + 1)) { H.gx = (int)fx; H.gy = (int)fy; break; }
          cl *= 2.0;
        }
        H.cell = cl;
      }
      H.ncell = H.gx * H.gy;
    }
  }
  __syncthreads();
  const int nc = H.ncell;
  for (int q = tid; q <= nc; q += WG) S.cnt[q] = 0;
  __syncthreads();
  for (int i = tid; i < n; i += WG) {
    int cx, cy;
    atomicAdd(&S.cnt[cell_xm(H, S.xs[i], S.ys[i], &cx, &cy)], 1u);
  }
  __syncthreads();
  for (int q = tid; q <= nc; q += WG) S.cstart[q] = S.cnt[q];
  __syncthreads();
  block_scan_array(S.cstart, nc + 1, H.red64);
  if (tid == 0) S.cstart[nc + 1] = n;
  for (int i = tid; i < n; i += WG) {
    int cx, cy;
    const int q = cell_xm(H, S.xs[i], S.ys[i], &cx, &cy);
    const uint32_t old = atomicSub(&S.cnt[q], 1u);
    S.citems[S.cstart[q] + old - 1] = (uint16_t)i;
  }
  __syncthreads();

  // ---- P2: Jaccard pairs (forward edges to higher pickers), count -> scan -> fill
  const double B = A.B, two_b2 = A.two_b2;
  for (int pass = 0; pass < 2; ++pass) {
    for (int i = tid; i < n; i += WG) {
      int cx = 0, cy = 0;
      const double xa = S.xs[i], ya = S.ys[i];
      const int q = cell_xm(H, xa, ya, &cx, &cy);
      int cntv = 0;
      const int base = pass ? (int)S.fwd[i] : 0;
      if (q < nc) {
        const int pe = c.pb[picker_of<K>(c.pb, i) + 1];
        const int y0 = max(cy - 1, 0), y1 = min(cy + 1, H.gy - 1);
        for (int col = max(cx - 1, 0); col <= min(cx + 1, H.gx - 1); ++col) {
          const int lo = S.cstart[col * H.gy + y0], hi = S.cstart[col * H.gy + y1 + 1];
          for (int t = lo; t < hi; ++t) {
            const int j = S.citems[t];
            if (j < pe) continue;
            double ji;
            if (is_edge(xa, ya, S.xs[j], S.ys[j], B, two_b2, &ji)) {
              if (pass) S.dst[base + cntv] = (uint16_t)j;
              ++cntv;
            }
          }
        }
      }
      if (!pass) {
        S.fwd[i] = cntv;
      } else {
        for (int a = base + 1; a < base + cntv; ++a) {
          const uint16_t key = S.dst[a];
          int b = a - 1;
          while (b >= base && S.dst[b] > key) { S.dst[b + 1] = S.dst[b]; --b; }
          S.dst[b + 1] = key;
        }
      }
    }
    __syncthreads();
    if (!pass) {
      const int64_t E = block_scan_array(S.fwd, n, H.red64);
      if (tid == 0) {
        S.fwd[n] = (uint32_t)E;
        H.E = (int)E;
        if (E == 0) H.status = RGC_ST_NO_EDGES;
        else if (E > A.ecap) H.status = RGC_ST_DEFER;
      }
      __syncthreads();
      if (H.status != 0) break;
    }
  }
  if (H.status != 0) {
    if (tid == 0) {
      MgStat st = {};
      st.n_edges = H.E;
      st.status = H.status;
      st.target = -1;
      A.st[m] = st;
    }
    return;
  }

  // ---- P3: connected components (union-find in LDS)
  for (int i = tid; i < n; i += WG) { S.parent[i] = i; S.flags[i] = 0; S.cnt[i] = 0; }
  __syncthreads();
  for (int i = tid; i < n; i += WG) {
    const int e0 = S.fwd[i], e1 = S.fwd[i + 1];
    if (e0 == e1) continue;
    S.flags[i] = 1;
    for (int e = e0; e < e1; ++e) {
      const uint32_t h = S.dst[e];
      S.flags[h] = 1;
      uint32_t a = i, b = h;
      for (;;) {
        a = uf_find_lds(S.parent, a);
        b = uf_find_lds(S.parent, b);
        if (a == b) break;
        if (a < b) { const uint32_t t = a; a = b; b = t; }
        if (atomicCAS(&S.parent[a], a, b) == a) break;
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < n; i += WG) {
    if (!S.flags[i]) continue;
    const uint32_t r = uf_find_lds(S.parent, i);
    lds_st(S.parent + i, r);
    atomicAdd(&S.cnt[r], 1u);
  }
  __syncthreads();
  {
    int64_t nodes = 0, roots = 0;
    int mx = 0;
    for (int i = tid; i < n; i += WG) {
      if (S.flags[i]) {
        ++nodes;
        if (S.parent[i] == (uint32_t)i) { ++roots; mx = max(mx, (int)S.cnt[i]); }
      }
    }
    nodes = block_sum64(nodes, H.red64);
    roots = block_sum64(roots, H.red64);
    mx = block_max_i(mx, H.redi);
    if (tid == 0) { H.nodes = (int)nodes; H.cc_cnt = (int)roots; H.cc_max = mx; }
  }
  const bool get_cc = (A.flags & 1) != 0;
  if (get_cc) {
    // largest CC; ties -> the component whose first edge comes first in the enumeration
    __syncthreads();
    uint64_t best = ~0ULL;
    for (int i = tid; i < n; i += WG) {
      const int e0 = S.fwd[i], e1 = S.fwd[i + 1];
      if (e0 == e1) continue;
      const uint32_t r = S.parent[i];
      if ((int)S.cnt[r] != H.cc_max) continue;
      const int pi = picker_of<K>(c.pb, i);
      const int h = S.dst[e0];   // lists are sorted: the first target is the smallest key
      const int ph = picker_of<K>(c.pb, h);
      const uint64_t key = ((uint64_t)pair_index(pi, ph, K) << 48) |
                           ((uint64_t)(i - c.pb[pi]) << 32) | ((uint64_t)(h - c.pb[ph]) << 16) | r;
      best = key < best ? key : best;
    }
    best = block_min_u64(best, H.redu);
    if (tid == 0) H.target = (int)(best & 0xFFFF);
  }
  __syncthreads();

  // ---- P4: clique count per picker-0 root, vertex marking, output reservation
  c.set_order = 2 * K < H.nodes;
  const int n0 = c.pb[1];
  const int target = H.target;
  for (int r = tid; r < n0; r += WG) {
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
  const int64_t C = block_scan_array(S.cnt, n0, H.red64);
  if (tid == 0) {
    S.cnt[n0] = (uint32_t)C;
    H.C = C;
    if (C == 0) {
      H.status = RGC_ST_NO_CLIQUES;
    } else {
      const unsigned long long base = atomicAdd(A.cursor, (unsigned long long)C);
      H.base = (int64_t)base;
      if ((int64_t)base + C > A.cap) H.status = RGC_ST_OVERFLOW;
    }
  }
  __syncthreads();

  // ---- P5: row index = rank of each clique vertex by (x, y, id): x-major grid columns
  if (H.status == 0) {
    const int gx = H.gx, gy = H.gy;
    uint32_t* colc = S.parent;
    for (int q = tid; q <= gx; q += WG) colc[q] = 0;
    __syncthreads();
    for (int v = tid; v < n; v += WG) {
      if (S.flags[v] != 3) continue;
      int cx, cy;
      cell_xm(H, S.xs[v], S.ys[v], &cx, &cy);
      atomicAdd(&colc[cx], 1u);
    }
    __syncthreads();
    const int64_t V = block_scan_array(colc, gx, H.red64);
    if (tid == 0) H.V = (int)V;
    for (int v = tid; v < n; v += WG) {
      if (S.flags[v] != 3) continue;
      int cx, cy;
      cell_xm(H, S.xs[v], S.ys[v], &cx, &cy);
      const double xv = S.xs[v], yv = S.ys[v];
      uint32_t rk = colc[cx];
      const int lo = S.cstart[cx * gy], hi = S.cstart[(cx + 1) * gy];
      for (int t = lo; t < hi; ++t) {
        const int u = S.citems[t];
        if (S.flags[u] != 3) continue;
        const double xu = S.xs[u], yu = S.ys[u];
        rk += (xu < xv) || (xu == xv && (yu < yv || (yu == yv && u < v)));
      }
      S.vrank[v] = (uint16_t)rk;
    }
    __syncthreads();

    // ---- P6: clique fill + ILP epilogue + COO rows
    for (int r = tid; r < n0; r += WG) {
      if (S.cnt[r + 1] == S.cnt[r]) continue;
      int mem[K];
      mem[0] = r;
      c.out = H.base + S.cnt[r];
      FLevel<K, 1, true>::run(c, mem);
    }
  }
  if (tid == 0) {
    MgStat st = {};
    st.n_edges = H.E;
    st.n_nodes = H.nodes;
    st.cc_cnt = H.cc_cnt;
    st.cc_max = H.cc_max;
    st.status = H.status;
    st.target = H.target;
    st.n_vert = H.V;
    st.clique_base = H.base;
    st.clique_cnt = H.C;
    A.st[m] = st;
  }
}

int launch_fused(hipStream_t stream, int n_blocks, int lds_bytes, const FusedArgs& A) {
  if (n_blocks <= 0) return 0;
  switch (A.k) {
#define RGC_FUSED_CASE(KK)                                                                    \
  case KK: {                                                                                  \
    static bool attr_set = false;                                                             \
    if (!attr_set) {                                                                          \
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_fused<KK>),                    \
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=     \
          hipSuccess)                                                                         \
        return -2;                                                                            \
      attr_set = true;                                                                        \
    }                                                                                         \
    hipLaunchKernelGGL(k_fused<KK>, dim3(n_blocks), dim3(WG), lds_bytes, stream, A);          \
    break;                                                                                    \
  }
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
