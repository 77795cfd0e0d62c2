// rgc_cliques.hip — k-clique enumeration and the ILP epilogue of the large-micrograph route.
//
// Reference repic/commands/get_cliques.py:49-56,160-161 (find_cliques, keep size k) and
// :164-202 (rows, confidence, weight, consensus).  The graph is k-partite (edges only join
// boxes of different pickers, :135-138), so the size-k cliques are exactly the
// one-box-per-picker k-tuples that are pairwise adjacent.  Every such tuple has one picker-0
// member, its "root"; the other k-1 members are forward neighbours of the root.
//
// One WAVEFRONT per root:
//   * lane i holds the i-th forward neighbour of the root (sorted by box index, so the
//     neighbours of picker p form one contiguous run of lanes);
//   * each lane merges its own forward list against the neighbourhood and keeps the result
//     as a 64-bit adjacency row in LDS; one ballot per picker gives the picker masks;
//   * the cliques of the root are then the picker-by-picker choices v1 in pm[1],
//     v2 in pm[2] & adj[v1], v3 in pm[3] & adj[v1] & adj[v2], ... : bitwise ANDs and ctz,
//     no list intersections; lane v1 walks the subtree of its own picker-1 choice and the
//     last level is a popcount.
// COUNT writes the clique count of every root and flags the clique vertices (for the row
// ranks); FILL recomputes the per-lane counts, scans them across the wave and writes the
// members at the root's scanned offset: lexicographic order, deterministic.  The ILP
// epilogue runs one THREAD per clique afterwards (balanced, coalesced output stores).
// Roots with more than RB_W forward neighbours go to the thread-per-root DFS in
// rgc_kernels.hip, which writes into the same arrays.
#pragma clang fp contract(off)

#include "rgc_device.h"
#include "rgc_kernels.h"

namespace rgc {

constexpr int CWG = 256;            // 4 wavefronts (roots) per workgroup
constexpr int CNW = CWG / 64;

__device__ __forceinline__ void wave_sync() {
  // LDS written by other lanes of this wavefront becomes visible (and is not reordered)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

struct RootInfo {
  int r;        // root box (sub-batch index)
  int d;        // forward neighbours
  int64_t lo;   // start of its forward list
  bool ok;      // enumerated by the wavefront kernels
};

// wavefront w -> the w-th picker-0 box of the sub-batch (micrograph by binary search)
__device__ __forceinline__ RootInfo root_info(const CliqueArgs& A, int w) {
  int lo = 0, hi = A.n_mg;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (A.p0off[mid] <= w) lo = mid; else hi = mid;
  }
  const int m = lo;
  RootInfo R;
  R.r = A.box_off[m * A.k] + (w - A.p0off[m]);
  R.lo = A.fwd_off[R.r];
  const int64_t d = A.fwd_off[R.r + 1] - R.lo;
  R.d = (int)d;
  const MgStat s = A.st[m];
  R.ok = d > 0 && d <= RB_W && s.status == 0 && (!(A.flags & 1) || A.parent[R.r] == s.target);
  return R;
}

// neighbourhood of the root in LDS: nb[i] = i-th forward neighbour, adj[i] = bitmask of the
// neighbourhood members adjacent to it (forward edges only: higher pickers); pm[p] = lanes
// holding picker-p boxes
template <int K>
__device__ __forceinline__ void neighbourhood(const CliqueArgs& A, const RootInfo& R, int lane,
                                              int32_t* nb, uint64_t* adj, uint64_t (&pm)[K]) {
  int u = -1, pk = -1;
  if (lane < R.d) {
    u = A.e_dst[R.lo + lane];
    pk = A.bpick[u];
    nb[lane] = u;
  }
  wave_sync();
  uint64_t mask = 0;
  if (lane < R.d) {
    // merge u's sorted forward list with the sorted neighbourhood (targets of u sort after u)
    int64_t e = A.fwd_off[u];
    const int64_t e1 = A.fwd_off[u + 1];
    int j = lane + 1;
    int v = j < R.d ? nb[j] : 0;
    while (e < e1 && j < R.d) {
      const int t = A.e_dst[e];
      if (t < v) {
        ++e;
      } else {
        if (t == v) { mask |= 1ull << j; ++e; }
        ++j;
        v = j < R.d ? nb[j] : 0;
      }
    }
  }
  adj[lane] = mask;
  pm[0] = 0;
#pragma unroll
  for (int p = 1; p < K; ++p) pm[p] = __ballot(pk == p);
  wave_sync();
}

// cliques below a prefix whose common-neighbour mask is M, choosing pickers D..K-1
template <int K, int D>
struct BCount {
  __device__ __forceinline__ static uint32_t run(const uint64_t* adj, const uint64_t (&pm)[K],
                                                 uint64_t M, uint64_t& used) {
    if constexpr (D == K - 1) {
      const uint64_t c = M & pm[D];
      used |= c;
      return (uint32_t)__popcll(c);
    } else {
      uint64_t c = M & pm[D];
      uint32_t tot = 0;
      while (c) {
        const int v = __builtin_ctzll(c);
        c &= c - 1;
        const uint32_t n = BCount<K, D + 1>::run(adj, pm, M & adj[v], used);
        if (n) {
          used |= 1ull << v;
          tot += n;
        }
      }
      return tot;
    }
  }
};

template <int K, int D>
struct BFill {
  __device__ __forceinline__ static void run(const uint64_t* adj, const int32_t* nb,
                                             const uint64_t (&pm)[K], uint64_t M, int (&mem)[K],
                                             int32_t* out, int64_t& j) {
    uint64_t c = M & pm[D];
    while (c) {
      const int v = __builtin_ctzll(c);
      c &= c - 1;
      mem[D] = nb[v];
      if constexpr (D == K - 1) {
#pragma unroll
        for (int i = 0; i < K; ++i) out[j * K + i] = mem[i];
        ++j;
      } else {
        BFill<K, D + 1>::run(adj, nb, pm, M & adj[v], mem, out, j);
      }
    }
  }
};

// cliques whose picker-1 member is this lane's neighbour (0 if it is not a picker-1 box)
template <int K>
__device__ __forceinline__ uint32_t lane_count(const uint64_t* adj, const uint64_t (&pm)[K],
                                               int lane, uint64_t& used) {
  if (!((pm[1] >> lane) & 1)) return 0;
  uint32_t n;
  if constexpr (K == 2) {
    n = 1;
  } else {
    n = BCount<K, 2>::run(adj, pm, adj[lane], used);
  }
  if (n) used |= 1ull << lane;
  return n;
}

__device__ __forceinline__ uint64_t wave_or(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
  return v;
}

template <int K>
__global__ __launch_bounds__(CWG) void k5b_count(CliqueArgs A) {
  __shared__ int32_t s_nb[CNW][RB_W];
  __shared__ uint64_t s_adj[CNW][RB_W];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int w = blockIdx.x * CNW + wv;
  if (w >= A.n_roots) return;
  const RootInfo R = root_info(A, w);
  if (!R.ok) return;   // wave-uniform; counts were zeroed
  int32_t* nb = s_nb[wv];
  uint64_t* adj = s_adj[wv];
  uint64_t pm[K];
  neighbourhood<K>(A, R, lane, nb, adj, pm);
  uint64_t used = 0;
  uint32_t cnt = lane_count<K>(adj, pm, lane, used);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  used = wave_or(used);
  if (lane == 0) {
    A.ccount[R.r] = (int32_t)cnt;
    if (cnt) A.in_clique[R.r] = 1;
  }
  if (lane < R.d && ((used >> lane) & 1)) A.in_clique[nb[lane]] = 1;
}

template <int K>
__global__ __launch_bounds__(CWG) void k5b_fill(CliqueArgs A) {
  __shared__ int32_t s_nb[CNW][RB_W];
  __shared__ uint64_t s_adj[CNW][RB_W];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int w = blockIdx.x * CNW + wv;
  if (w >= A.n_roots) return;
  const RootInfo R = root_info(A, w);
  if (!R.ok) return;
  int32_t* nb = s_nb[wv];
  uint64_t* adj = s_adj[wv];
  uint64_t pm[K];
  neighbourhood<K>(A, R, lane, nb, adj, pm);
  uint64_t used = 0;
  const uint32_t n = lane_count<K>(adj, pm, lane, used);
  // exclusive prefix of the lane counts (lane order = picker-1 member order)
  uint32_t inc = n;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (!n) return;
  int64_t j = A.clique_off[R.r] + (inc - n);
  int mem[K];
  mem[0] = R.r;
  mem[1] = nb[lane];
  if constexpr (K == 2) {
    A.members[j * K] = mem[0];
    A.members[j * K + 1] = mem[1];
  } else {
    BFill<K, 2>::run(adj, nb, pm, adj[lane], mem, A.members, j);
  }
}

// ILP epilogue, one thread per clique (get_cliques.py:164-202): COO rows (vertex ranks by
// (x, y, id), ascending), conf = f32(median score), w = f32(f64(conf) * median JI), and the
// consensus box (largest weighted degree, CPython set-order tie-break); --multi_out: the
// networkx node-iteration order of the members.  Same arithmetic as the fused kernel's
// epilogue (rgc_fused.hip fused_epilogue_main / _order).
template <int K>
__global__ __launch_bounds__(WG) void k5_epilogue(CliqueArgs A) {
  constexpr int NE = K * (K - 1) / 2;
  const int64_t j = (int64_t)blockIdx.x * WG + threadIdx.x;
  if (j >= A.C) return;
  int mem[K];
#pragma unroll
  for (int i = 0; i < K; ++i) mem[i] = A.members[j * K + i];
  double xs[K], ys[K], s[K];
  int r[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    xs[i] = A.x[mem[i]];
    ys[i] = A.y[mem[i]];
    s[i] = A.score[mem[i]];
    r[i] = A.vrow[mem[i]];
  }
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
  const double B = A.B, two_b2 = A.two_b2;
  double I[NE];   // member-pair overlaps (a < b), reference op order
  {
    int t = 0;
#pragma unroll
    for (int a = 0; a < K; ++a)
#pragma unroll
      for (int b = a + 1; b < K; ++b) I[t++] = overlap(xs[a], ys[a], xs[b], ys[b], B);
  }
  // conf = f32(median score); median JI = JI of the median overlap (JI is non-decreasing in
  // I and the f64 quotient keeps that order), so one or two reference divisions
  double sc[K];
#pragma unroll
  for (int i = 0; i < K; ++i) sc[i] = s[i];
  const float conf32 = (float)median_n<K>(sc);
  double med;
  {
    double Is[NE];
#pragma unroll
    for (int t = 0; t < NE; ++t) Is[t] = I[t];
    if (NE & 1) {
      med = median_n<NE>(Is);
      med = med / (two_b2 - med);
    } else {
      bool nan = false;
#pragma unroll
      for (int t = 0; t < NE; ++t) nan |= isnan(Is[t]);
      sort_n<NE>(Is);
      const double a = Is[NE / 2 - 1], b = Is[NE / 2];
      med = nan ? NAN : ((a / (two_b2 - a)) + (b / (two_b2 - b))) / 2.0;
    }
  }
  A.w[j] = (float)((double)conf32 * med);
  A.conf[j] = conf32;
  const bool multi = (A.flags & 2) != 0;
  int arg = 0;
  bool exact = multi;
  if (!multi) {
    // weighted degrees from f32 JIs (error < 2e-6 per sum): a clear maximum is the
    // reference's; anything within 1e-5 takes the exact f64 pass (ties included)
    float deg[K];
#pragma unroll
    for (int i = 0; i < K; ++i) deg[i] = 0.0f;
    int t = 0;
#pragma unroll
    for (int a = 0; a < K; ++a)
#pragma unroll
      for (int b = a + 1; b < K; ++b) {
        const float jf = (float)I[t] / (float)(two_b2 - I[t]);
        deg[a] += jf;
        deg[b] += jf;
        ++t;
      }
    float d1 = deg[0], d2 = -INFINITY;
#pragma unroll
    for (int i = 1; i < K; ++i) {
      const float d = deg[i];
      d2 = d > d1 ? d1 : fmaxf(d2, d);
      arg = d > d1 ? i : arg;
      d1 = fmaxf(d1, d);
    }
    exact = !(d1 - d2 > 1e-5f);
  }
  if (exact) {
    const int m = A.bmg[mem[0]];
    const int64_t idb = A.id_base[m] - (int64_t)A.box_off[m * A.k];
    double ji[K][K];
    int64_t ids[K];
    uint64_t ins[K] = {};
#pragma unroll
    for (int a = 0; a < K; ++a) {
      ids[a] = idb + mem[a];
#pragma unroll
      for (int b = a + 1; b < K; ++b) ji[a][b] = jaccard(xs[a], ys[a], xs[b], ys[b], B, two_b2);
    }
    const bool set_order = 2 * K < A.st[m].n_nodes;
    if (!set_order) {
#pragma unroll
      for (int i = 0; i < K; ++i) ins[i] = A.ins_key[mem[i]];
    }
    uint32_t top;
    arg = epi_degree_max<K>(ji, &top);
    const bool tie = (top & (top - 1)) != 0;
    if (tie || multi) {
      const uint32_t ord = node_order<K>(mem, xs, ys, ids, set_order, ins);
      if (tie) arg = epi_tie_arg<K>(top, ord);
      if (multi) {
#pragma unroll
        for (int i = 0; i < K; ++i) A.order[j * K + i] = (uint8_t)((ord >> (4 * i)) & 15);
      }
    }
  }
  int cons = mem[0];
#pragma unroll
  for (int i = 1; i < K; ++i) cons = (arg == i) ? mem[i] : cons;
  A.consensus[j] = cons;
}

template <int K>
static void launch_cliques_k(hipStream_t stream, int phase, int N, const CliqueArgs& A) {
  if (phase == 0 || phase == 1) {
    const int nb = (A.n_roots + CNW - 1) / CNW;
    if (nb > 0) {
      if (phase == 0) hipLaunchKernelGGL((k5b_count<K>), dim3(nb), dim3(CWG), 0, stream, A);
      else hipLaunchKernelGGL((k5b_fill<K>), dim3(nb), dim3(CWG), 0, stream, A);
    }
    launch_cliques_dfs(stream, phase == 1, N, A);
  } else {
    const int64_t nb = (A.C + WG - 1) / WG;
    if (nb > 0) hipLaunchKernelGGL((k5_epilogue<K>), dim3(nb), dim3(WG), 0, stream, A);
  }
}

int launch_cliques(hipStream_t stream, int phase, int N, const CliqueArgs& A) {
  switch (A.k) {
    case 2: launch_cliques_k<2>(stream, phase, N, A); break;
    case 3: launch_cliques_k<3>(stream, phase, N, A); break;
    case 4: launch_cliques_k<4>(stream, phase, N, A); break;
    case 5: launch_cliques_k<5>(stream, phase, N, A); break;
    case 6: launch_cliques_k<6>(stream, phase, N, A); break;
    case 7: launch_cliques_k<7>(stream, phase, N, A); break;
    case 8: launch_cliques_k<8>(stream, phase, N, A); break;
    default: return -1;
  }
  return 0;
}

}  // namespace rgc
