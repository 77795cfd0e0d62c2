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

constexpr int ECAP = 64;            // prefixes per level buffer (per wavefront)

// A prefix of a root's clique: members for pickers 1..D as neighbourhood lanes (6 bits each,
// picker q at bits 6(q-1)) and the mask of neighbourhood lanes adjacent to all of them.
struct Ent {
  uint64_t M;
  uint64_t P;
};

// per-wavefront LDS
template <int K>
struct WaveLds {
  int32_t nb[RB_W];           // neighbourhood (forward neighbours of the root), sorted
  uint64_t adj[RB_W];         // adj[i]: neighbourhood lanes adjacent to lane i (forward)
  uint64_t pm[K];             // pm[p]: neighbourhood lanes of picker p
  Ent buf[K - 1][ECAP];       // level D prefixes (D = 0..K-2; level 0 = the root alone)
  uint32_t sc[ECAP];          // fill: inclusive scan of the leaf counts of the leaf level
};

// neighbourhood of the root: nb, adj, pm
template <int K>
__device__ __forceinline__ void neighbourhood(const CliqueArgs& A, const RootInfo& R, int lane,
                                              WaveLds<K>& L) {
  int u = -1, pk = -1;
  if (lane < R.d) {
    u = A.e_dst[R.lo + lane];
    pk = A.bpick[u];
    L.nb[lane] = u;
  }
  wave_sync();
  uint64_t mask = 0;
  if (lane < R.d) {
    // merge u's sorted forward list with the sorted neighbourhood (targets of u sort after u)
    int64_t e = A.fwd_off[u];
    const int64_t e1 = A.fwd_off[u + 1];
    int j = lane + 1;
    int v = j < R.d ? L.nb[j] : 0;
    while (e < e1 && j < R.d) {
      const int t = A.e_dst[e];
      if (t < v) {
        ++e;
      } else {
        if (t == v) { mask |= 1ull << j; ++e; }
        ++j;
        v = j < R.d ? L.nb[j] : 0;
      }
    }
  }
  L.adj[lane] = mask;
#pragma unroll
  for (int p = 0; p < K; ++p) {
    const uint64_t b = __ballot(pk == p);
    if (lane == 0) L.pm[p] = b;
  }
  wave_sync();
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

__device__ __forceinline__ uint64_t wave_or(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
  return v;
}

// Expand level-D prefixes, from *cur on, into the (empty) level D+1 buffer until it is full.
// A child is kept only if it can still be completed (it has a candidate in picker D+2).
// Wave-cooperative: one prefix per lane, children placed by a wave scan; whole prefixes
// only, in order, so level D+1 stays lexicographic.  Returns the children written.
template <int K>
__device__ int expand(WaveLds<K>& L, int D, int& cur, int n_src, int lane) {
  const uint64_t pnext = L.pm[D + 1];
  const uint64_t pafter = D + 2 < K ? L.pm[D + 2] : ~0ull;
  Ent* src = L.buf[D];
  Ent* dst = L.buf[D + 1];
  int nd = 0;
  while (cur < n_src && nd < ECAP) {
    const int e = cur + lane;
    Ent x = {0, 0};
    uint32_t cnt = 0;
    if (e < n_src) {
      x = src[e];
      uint64_t c = x.M & pnext;
      while (c) {
        const int v = __builtin_ctzll(c);
        c &= c - 1;
        cnt += (x.M & L.adj[v] & pafter) ? 1u : 0u;
      }
    }
    const uint32_t inc = wave_incl_scan(cnt, lane);
    const bool ok = e < n_src && (int)inc <= ECAP - nd;
    const int nacc = __popcll(__ballot(ok));
    if (ok && cnt) {
      int o = nd + (int)(inc - cnt);
      uint64_t c = x.M & pnext;
      while (c) {
        const int v = __builtin_ctzll(c);
        c &= c - 1;
        const uint64_t m2 = x.M & L.adj[v];
        if (m2 & pafter) {
          Ent y;
          y.M = m2;
          y.P = x.P | ((uint64_t)v << (6 * D));
          dst[o++] = y;
        }
      }
    }
    if (nacc == 0) break;   // the next prefix's children do not fit: go deeper first
    nd += (int)__shfl(inc, nacc - 1, 64);
    cur += nacc;
  }
  wave_sync();
  return nd;
}

// All cliques of one root, lexicographic, by a depth-first walk over chunks of level-
// synchronous prefix buffers (each level <= ECAP prefixes).  COUNT: returns the number of
// cliques and ORs the clique-vertex lanes into *used.  FILL: writes the members of clique
// out0 + t (t = 0, 1, ...) to A.members.
template <int K, bool FILL>
__device__ uint32_t root_cliques(const CliqueArgs& A, const RootInfo& R, int lane, WaveLds<K>& L,
                                 uint64_t* used, int64_t out0) {
  const uint64_t plast = L.pm[K - 1];
  int n[K], cur[K];   // wave-uniform; constant-indexed through the unrolled switches below
  uint32_t total = 0;
  uint64_t usedl = 0;
  if (lane == 0) {
    Ent r0;
    r0.M = ~0ull;
    r0.P = 0;
    L.buf[0][0] = r0;
  }
  wave_sync();
#pragma unroll
  for (int q = 0; q < K; ++q) { n[q] = 0; cur[q] = 0; }
  n[0] = 1;
  int D = 0;
  for (;;) {
    if (D == K - 2) {
      // leaf level: the cliques of each prefix are its candidates in the last picker
      int nl = 0;
#pragma unroll
      for (int q = 0; q < K - 1; ++q) if (q == D) nl = n[q];
      const Ent* src = L.buf[K - 2];
      if constexpr (!FILL) {
        for (int e = lane; e < nl; e += 64) {
          const Ent x = src[e];
          const uint64_t c = x.M & plast;
          total += (uint32_t)__popcll(c);
          if (c) {
            usedl |= c;
#pragma unroll
            for (int q = 0; q < K - 2; ++q) usedl |= 1ull << ((x.P >> (6 * q)) & 63);
          }
        }
      } else {
        // one prefix per lane (nl <= ECAP = 64), then the leaves spread over the lanes
        uint64_t c = 0;
        if (lane < nl) c = src[lane].M & plast;
        const uint32_t cnt = (uint32_t)__popcll(c);
        const uint32_t inc = wave_incl_scan(cnt, lane);
        L.sc[lane] = inc;
        const uint32_t T = __shfl(inc, 63, 64);
        wave_sync();
        for (uint32_t t = lane; t < T; t += 64) {
          int lo = 0, hi = 63;   // first prefix with inclusive count > t
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (L.sc[mid] > t) hi = mid; else lo = mid + 1;
          }
          const Ent x = src[lo];
          uint64_t cc = x.M & plast;
          for (uint32_t r = t - (L.sc[lo] - (uint32_t)__popcll(cc)); r > 0; --r) cc &= cc - 1;
          const int v = __builtin_ctzll(cc);
          const int64_t j = out0 + total + t;
          A.members[j * K] = R.r;
#pragma unroll
          for (int q = 0; q < K - 2; ++q)
            A.members[j * K + 1 + q] = L.nb[(x.P >> (6 * q)) & 63];
          A.members[j * K + K - 1] = L.nb[v];
        }
        total += T;
        wave_sync();
      }
      if (D == 0) break;
      --D;
      continue;
    }
    int nD = 0, cD = 0;
#pragma unroll
    for (int q = 0; q < K - 1; ++q)
      if (q == D) { nD = n[q]; cD = cur[q]; }
    if (cD < nD) {
      const int nd = expand<K>(L, D, cD, nD, lane);
#pragma unroll
      for (int q = 0; q < K - 1; ++q) {
        if (q == D) cur[q] = cD;
        if (q == D + 1) { n[q] = nd; cur[q] = 0; }
      }
      ++D;
    } else {
      if (D == 0) break;
      --D;
    }
  }
  if constexpr (!FILL) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) total += __shfl_xor(total, o, 64);
    *used = wave_or(usedl);
  }
  return total;
}

template <int K>
__global__ __launch_bounds__(CWG) void k5b_count(CliqueArgs A) {
  __shared__ WaveLds<K> s_w[CNW];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int w = blockIdx.x * CNW + wv;
  if (w >= A.n_roots) return;
  const RootInfo R = root_info(A, w);
  if (!R.ok) return;   // wave-uniform; counts were zeroed
  WaveLds<K>& L = s_w[wv];
  neighbourhood<K>(A, R, lane, L);
  uint64_t used = 0;
  uint32_t cnt;
  if constexpr (K == 2) {
    used = L.pm[1];
    cnt = (uint32_t)__popcll(used);
  } else {
    cnt = root_cliques<K, false>(A, R, lane, L, &used, 0);
  }
  if (lane == 0) {
    A.ccount[R.r] = (int32_t)cnt;
    if (cnt) A.in_clique[R.r] = 1;
  }
  if (lane < R.d && ((used >> lane) & 1)) A.in_clique[L.nb[lane]] = 1;
}

template <int K>
__global__ __launch_bounds__(CWG) void k5b_fill(CliqueArgs A) {
  __shared__ WaveLds<K> s_w[CNW];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int w = blockIdx.x * CNW + wv;
  if (w >= A.n_roots) return;
  const RootInfo R = root_info(A, w);
  if (!R.ok) return;
  WaveLds<K>& L = s_w[wv];
  neighbourhood<K>(A, R, lane, L);
  const int64_t out0 = A.clique_off[R.r];
  if constexpr (K == 2) {
    const uint64_t c = L.pm[1];
    if ((c >> lane) & 1) {
      const int64_t j = out0 + __popcll(c & ((1ull << lane) - 1));
      A.members[j * 2] = R.r;
      A.members[j * 2 + 1] = L.nb[lane];
    }
  } else {
    uint64_t used;
    root_cliques<K, true>(A, R, lane, L, &used, out0);
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
