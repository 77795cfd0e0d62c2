// rgc_cliques.hip — k-clique enumeration and the ILP epilogue of the large-micrograph route.
//
// Reference repic/commands/get_cliques.py:49-56,160-161 (find_cliques, keep size k) and
// :164-202 (rows, confidence, weight, consensus).  The graph is k-partite (edges only join
// boxes of different pickers, :135-138), so the size-k cliques are exactly the
// one-box-per-picker k-tuples that are pairwise adjacent.  Every such tuple has one picker-0
// member, its "root"; the other k-1 members are forward neighbours of the root.
//
// 1. Neighbourhood bitmaps (k5n_build): a group of 16 lanes per root (four roots per
//    wavefront), lane l holding the root's forward neighbours l, l + 16, ... (sorted by box
//    index, so each picker is a contiguous run of neighbour indices).  The adjacency row of
//    neighbour i inside the neighbourhood (a 64-bit mask, forward edges only) goes to
//    adjg[fwd_off[root] + i] and the picker run starts to rbound[root].
// 2. Level-synchronous prefix expansion over the whole sub-batch (k5l<K, ...>): a level-D
//    prefix = (root, mask M of neighbourhood lanes adjacent to all chosen members, chosen
//    lanes P, 6 bits each); its children are the picker-(D+1) lanes v in M, with mask
//    M & adj[v].  One THREAD per prefix, count -> scan -> fill per level, so the work of a
//    root with 27k cliques (C5) is spread over the GPU instead of serialised on one lane or
//    wave.  A child is kept only when it can still be completed (it has a candidate in
//    picker D+2).  At the last level the cliques of a prefix are its candidate lanes in the
//    last picker: COUNT flags the clique vertices (row ranks), FILL writes members.  Items
//    stay in parent order, so cliques come out lexicographic (deterministic) and grouped by
//    root, hence by micrograph.
// 3. The ILP epilogue: one THREAD per clique (balanced, coalesced output stores).
// Micrographs with a root of more than RB_W forward neighbours run through the
// thread-per-root DFS of rgc_kernels.hip instead (their cliques follow the others).
#pragma clang fp contract(off)

#include "rgc_device.h"
#include "rgc_kernels.h"

#include <algorithm>
#include <climits>

namespace rgc {

__device__ __forceinline__ uint64_t mask_below(int n) { return n >= 64 ? ~0ull : ((1ull << n) - 1); }

// lanes of picker p (1..K-1) in a root's neighbourhood: byte p-1 of rbound = first lane of
// picker p, byte p = first lane after it (byte K-1 = d)
__device__ __forceinline__ uint64_t picker_lanes(uint64_t rb, int p) {
  const int s = (int)((rb >> (8 * (p - 1))) & 0xFF);
  const int e = (int)((rb >> (8 * p)) & 0xFF);
  return mask_below(e) & ~mask_below(s);
}

// valid clique root: picker-0 box with forward edges in a finished micrograph (and in the
// --get_cc target component)
__device__ __forceinline__ bool root_valid(const CliqueArgs& A, int g, int m) {
  if (A.bpick[g] != 0 || A.fwd_off[g] == A.fwd_off[g + 1]) return false;
  const MgStat s = A.st[m];
  return s.status == 0 && (!(A.flags & 1) || A.parent[g] == s.target);
}

// Thread per box: the root list (wavefront-free indexing of picker-0 boxes) and the route of
// each micrograph (DFS when a root has more than RB_W forward neighbours).
__global__ __launch_bounds__(WG) void k5_route(int N, CliqueArgs A) {
  const int g = blockIdx.x * WG + threadIdx.x;
  if (g >= N || A.bpick[g] != 0) return;
  const int m = A.bmg[g];
  A.root_box[A.p0off[m] + (g - A.box_off[m * A.k])] = g;
  if (root_valid(A, g, m) && A.fwd_off[g + 1] - A.fwd_off[g] > RB_W) A.dfs_mg[m] = 1;
}

// Neighbourhood bitmaps, NBG lanes per root; lane l holds neighbours l, l + NBG, ...
constexpr int NBG = 16;
constexpr int NBQ = RB_W / NBG;

__global__ __launch_bounds__(WG) void k5n_build(CliqueArgs A) {
  constexpr int NG = WG / NBG;
  __shared__ int32_t s_nb[NG][RB_W];
  const int grp = threadIdx.x / NBG, lane = threadIdx.x % NBG;
  const int w = blockIdx.x * NG + grp;   // one group per picker-0 box
  if (w >= A.n_roots) return;
  const int g = A.root_box[w];
  const int m = A.bmg[g];
  if (!root_valid(A, g, m) || A.dfs_mg[m]) return;
  const int64_t lo = A.fwd_off[g];
  const int d = (int)(A.fwd_off[g + 1] - lo);
  int32_t* nb = s_nb[grp];
  int u[NBQ], pk[NBQ];
#pragma unroll
  for (int q = 0; q < NBQ; ++q) {
    const int i = lane + q * NBG;
    u[q] = -1;
    pk[q] = A.k;
    if (i < d) {
      u[q] = A.e_dst[lo + i];
      pk[q] = A.bpick[u[q]];
      nb[i] = u[q];
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  const int last = nb[d - 1];
#pragma unroll
  for (int q = 0; q < NBQ; ++q) {
    const int i = lane + q * NBG;
    if (i >= d) break;
    // adjacency row: u's forward targets looked up in the sorted neighbourhood (only lanes
    // after u can match); four loads in flight per step
    uint64_t mask = 0;
    const int64_t e0 = A.fwd_off[u[q]], e1 = A.fwd_off[u[q] + 1];
    for (int64_t e = e0; e < e1; e += 4) {
      int t[4];
#pragma unroll
      for (int z = 0; z < 4; ++z) t[z] = e + z < e1 ? A.e_dst[e + z] : INT_MAX;
#pragma unroll
      for (int z = 0; z < 4; ++z) {
        if (t[z] > last) continue;
        int a = i + 1, b = d;   // first lane with nb >= t
        while (a < b) {
          const int mid = (a + b) >> 1;
          if (nb[mid] < t[z]) a = mid + 1; else b = mid;
        }
        if (a < d && nb[a] == t[z]) mask |= 1ull << a;
      }
      if (t[3] >= last) break;
    }
    A.adjg[lo + i] = mask;
  }
  // picker runs: lanes are sorted picker-major, so the first lane of picker p = #lanes below p
  const uint64_t gmask = ((1ull << NBG) - 1) << ((threadIdx.x & 63) / NBG * NBG);
  uint64_t rb = 0;
#pragma unroll
  for (int p = 1; p < MAX_K; ++p) {
    int s = 0;
#pragma unroll
    for (int q = 0; q < NBQ; ++q) s += __popcll(__ballot(pk[q] < p) & gmask);
    if (p < A.k) rb |= (uint64_t)s << (8 * (p - 1));
  }
  rb |= (uint64_t)d << (8 * (A.k - 1));
  if (lane == 0) {
    A.rbound[g] = rb;
    A.rflag[g] = 1;
  }
}

// One level of prefix expansion (thread per prefix).  FIRST: the prefixes are the roots
// themselves (thread per box, M = all lanes).  LEAF: the children are cliques.
template <int K, bool FIRST, bool LEAF, bool FILL>
__global__ __launch_bounds__(WG) void k5l(CliqueArgs A, LevelArgs L) {
  const int64_t i = (int64_t)blockIdx.x * WG + threadIdx.x;
  if constexpr (LEAF && !FILL && !FIRST) {
    // leaf count + clique-vertex marks.  A wave's prefixes come grouped by root (parent order),
    // and a root's prefixes share most of their members: the marks (members of every prefix
    // with a leaf, and its leaves, as lanes of the root's forward list) are OR-ed over each
    // run of equal roots in the wave (segmented DPP-free shuffle scan), and the run's last
    // lane stores each marked member once - instead of every prefix storing its K - 2 members
    // and all its leaves (C5: ~62 M cliques' worth of scattered byte stores per step).
    const int lane = threadIdx.x & 63;
    const bool valid = i < L.n_items;
    int r = -1 - lane;   // (invalid lanes: roots of their own, never joined)
    uint64_t bits = 0;
    int64_t lo = 0;
    if (valid) {
      r = L.in_root[i];
      const uint64_t P = L.in_P[i];
      const uint64_t c = L.in_M[i] & picker_lanes(A.rbound[r], L.D + 1);
      L.cnt[i] = __popcll(c);
      lo = A.fwd_off[r];
      if (c) {
        bits = c;
#pragma unroll
        for (int q = 0; q < K - 2; ++q) bits |= 1ull << ((P >> (6 * q)) & 63);
      }
    }
#pragma unroll
    for (int sft = 1; sft < 64; sft <<= 1) {
      const uint64_t ob = __shfl_up(bits, sft, 64);
      const int orr = __shfl_up(r, sft, 64);
      if (lane >= sft && orr == r) bits |= ob;
    }
    const int nr = __shfl_down(r, 1, 64);
    const bool tail = lane == 63 || nr != r;
    if (valid && tail && bits) {
      A.in_clique[r] = 1;
      while (bits) {
        const int v = __builtin_ctzll(bits);
        bits &= bits - 1;
        A.in_clique[A.e_dst[lo + v]] = 1;
      }
    }
    return;
  }
  if constexpr (FILL && !LEAF) {
    if (L.next_cnt) {   // (launch-uniform) the last fill: its children are the leaf prefixes
      // Each child's cliques are the lanes m2 & pa (never empty: a child is kept only when it
      // has one), so its leaf count goes to next_cnt and every member and leaf is a clique
      // vertex: the leaf count pass is not needed.  The marks are OR-ed per root over the
      // wave (its prefixes come grouped by root) and the run's last lane stores them, as the
      // leaf count pass did.
      const int lane = threadIdx.x & 63;
      int r = -1 - lane;   // (lanes without a prefix: roots of their own, never joined)
      uint64_t bits = 0;
      int64_t lo = 0;
      if (i < L.n_items && (!FIRST || A.rflag[(int)i])) {
        r = FIRST ? (int)i : L.in_root[i];
        const uint64_t M = FIRST ? ~0ull : L.in_M[i];
        const uint64_t P = FIRST ? 0ull : L.in_P[i];
        const int D = L.D;
        const uint64_t rb = A.rbound[r];
        lo = A.fwd_off[r];
        uint64_t c = M & picker_lanes(rb, D + 1);
        const uint64_t pa = picker_lanes(rb, D + 2);
        int64_t o = L.off[i];
        while (c) {
          const int v = __builtin_ctzll(c);
          c &= c - 1;
          const uint64_t m2 = M & A.adjg[lo + v];
          const uint64_t lv = m2 & pa;
          if (lv) {
            L.out_root[o] = r;
            L.out_M[o] = lv;   // (a leaf prefix's mask matters only in its leaf picker)
            L.out_P[o] = P | ((uint64_t)v << (6 * D));
            L.next_cnt[o] = __popcll(lv);
            bits |= lv | (1ull << v);
            ++o;
          }
        }
        if (bits)
#pragma unroll
          for (int q = 0; q < K - 3; ++q)
            if (q < D) bits |= 1ull << ((P >> (6 * q)) & 63);
      }
#pragma unroll
      for (int sft = 1; sft < 64; sft <<= 1) {
        const uint64_t ob = __shfl_up(bits, sft, 64);
        const int orr = __shfl_up(r, sft, 64);
        if (lane >= sft && orr == r) bits |= ob;
      }
      const int nr = __shfl_down(r, 1, 64);
      const bool tail = lane == 63 || nr != r;
      if (r >= 0 && tail && bits) {
        A.in_clique[r] = 1;
        while (bits) {
          const int v = __builtin_ctzll(bits);
          bits &= bits - 1;
          A.in_clique[A.e_dst[lo + v]] = 1;
        }
      }
      return;
    }
  }
  if (i >= L.n_items) return;
  int r;
  uint64_t M, P;
  if (FIRST) {
    r = (int)i;
    if (!A.rflag[r]) return;   // cnt stays 0 (zeroed)
    M = ~0ull;
    P = 0;
  } else {
    r = L.in_root[i];
    M = L.in_M[i];
    P = L.in_P[i];
  }
  const int D = L.D;   // members chosen so far (pickers 1..D)
  const uint64_t rb = A.rbound[r];
  const int64_t lo = A.fwd_off[r];
  uint64_t c = M & picker_lanes(rb, D + 1);
  if (LEAF) {
    if (!FILL) {
      L.cnt[i] = __popcll(c);
      if (c) {
        A.in_clique[r] = 1;
#pragma unroll
        for (int q = 0; q < K - 2; ++q) A.in_clique[A.e_dst[lo + ((P >> (6 * q)) & 63)]] = 1;
        while (c) {
          const int v = __builtin_ctzll(c);
          c &= c - 1;
          A.in_clique[A.e_dst[lo + v]] = 1;
        }
      }
    } else {
      if (!c) return;
      int mem[K];
      mem[0] = r;
#pragma unroll
      for (int q = 0; q < K - 2; ++q) mem[q + 1] = A.e_dst[lo + ((P >> (6 * q)) & 63)];
      int64_t j = L.off[i];
      while (c) {
        const int v = __builtin_ctzll(c);
        c &= c - 1;
        mem[K - 1] = A.e_dst[lo + v];
#pragma unroll
        for (int q = 0; q < K; ++q) A.members[j * K + q] = mem[q];
        ++j;
      }
    }
    return;
  }
  const uint64_t pa = picker_lanes(rb, D + 2);
  if (!FILL) {
    int n = 0;
    while (c) {
      const int v = __builtin_ctzll(c);
      c &= c - 1;
      n += (M & A.adjg[lo + v] & pa) ? 1 : 0;
    }
    L.cnt[i] = n;
  } else {
    int64_t o = L.off[i];
    while (c) {
      const int v = __builtin_ctzll(c);
      c &= c - 1;
      const uint64_t m2 = M & A.adjg[lo + v];
      if (m2 & pa) {
        L.out_root[o] = r;
        L.out_M[o] = m2;
        L.out_P[o] = P | ((uint64_t)v << (6 * D));
        ++o;
      }
    }
  }
}

// Leaf fill, wavefront-cooperative (k >= 3): a wave takes 64 leaf prefixes (one per lane)
// and writes their cliques as ONE contiguous range of the output (their scanned offsets are
// consecutive).  The prefixes' data goes to LDS; then lane l writes cliques l, l + 64, ... of
// the range: it finds its prefix by a binary search over the 64 local offsets and its leaf as
// the rank-th set bit of the prefix's candidate mask.  Consecutive lanes write consecutive
// cliques, so each member store covers whole cache lines (the thread-per-prefix fill wrote
// 64 scattered K-int runs per store: 2 GB of partial-line writes per C5 step).
template <int K>
__global__ __launch_bounds__(WG) void k5_leaf_fill(CliqueArgs A, LevelArgs L) {
  constexpr int NWV = WG / 64;
  __shared__ uint32_t s_ex[NWV][65];    // local exclusive offsets (+ total)
  __shared__ uint64_t s_c[NWV][64];     // candidate (leaf) masks
  __shared__ uint64_t s_p[NWV][64];     // chosen lanes of pickers 1..K-2
  __shared__ int64_t s_lo[NWV][64];     // root's forward-list start
  __shared__ int32_t s_r[NWV][64];      // root box
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t i0 = ((int64_t)blockIdx.x * WG) + wv * 64;
  if (i0 >= L.n_items) return;   // wave-uniform
  const int64_t i = i0 + lane;
  const int64_t iend = min(i0 + 64, L.n_items);
  const int64_t j0 = L.off[i0];
  uint64_t c = 0, P = 0;
  int64_t lo = 0;
  int r = 0;
  if (i < L.n_items) {
    r = L.in_root[i];
    P = L.in_P[i];
    const uint64_t rb = A.rbound[r];
    lo = A.fwd_off[r];
    c = L.in_M[i] & picker_lanes(rb, L.D + 1);
  }
  s_ex[wv][lane] = (uint32_t)((i < L.n_items ? L.off[i] : L.off[iend]) - j0);
  if (lane == 0) s_ex[wv][64] = (uint32_t)(L.off[iend] - j0);
  s_c[wv][lane] = c;
  s_p[wv][lane] = P;
  s_lo[wv][lane] = lo;
  s_r[wv][lane] = r;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  const int T = (int)s_ex[wv][64];
  for (int q = lane; q < T; q += 64) {
    // prefix s: the last local offset <= q (a prefix without cliques shares the next one's
    // offset and is never the last such)
    int a = 0, b = 63;
    while (a < b) {
      const int mid = (a + b + 1) >> 1;
      if (s_ex[wv][mid] <= (uint32_t)q) a = mid; else b = mid - 1;
    }
    uint64_t m = s_c[wv][a];
    for (int t = q - (int)s_ex[wv][a]; t > 0; --t) m &= m - 1;   // rank-th set bit
    const int v = __builtin_ctzll(m);
    const uint64_t pp = s_p[wv][a];
    const int64_t plo = s_lo[wv][a];
    int mem[K];
    mem[0] = s_r[wv][a];
#pragma unroll
    for (int t = 0; t < K - 2; ++t) mem[t + 1] = A.e_dst[plo + ((pp >> (6 * t)) & 63)];
    mem[K - 1] = A.e_dst[plo + v];
    int32_t* dst = A.members + (j0 + q) * K;
    if constexpr (K == 8) {
      reinterpret_cast<int4*>(dst)[0] = make_int4(mem[0], mem[1], mem[2], mem[3]);
      reinterpret_cast<int4*>(dst)[1] = make_int4(mem[4], mem[5], mem[6], mem[7]);
    } else if constexpr (K == 4) {
      reinterpret_cast<int4*>(dst)[0] = make_int4(mem[0], mem[1], mem[2], mem[3]);
    } else {
#pragma unroll
      for (int t = 0; t < K; ++t) dst[t] = mem[t];
    }
  }
}

// Per-micrograph clique range.  Level-route cliques [0, C1) are sorted by root (box index, so
// by micrograph): binary search for the micrograph's first and last picker-0 box.  DFS-route
// micrographs: their roots' scanned offsets after C1.
// (leaf_root / leaf_off: the leaf prefixes' roots, nondecreasing, and clique offsets, when the
// members were not written: the first clique of root g is leaf_off[lower_bound(leaf_root, g)])
__global__ __launch_bounds__(WG) void k5_ranges(CliqueArgs A, int64_t C1, int64_t* rlo,
                                               int64_t* rhi, const int32_t* leaf_root,
                                               const int64_t* leaf_off, int64_t n_leaf) {
  const int m = blockIdx.x * WG + threadIdx.x;
  if (m >= A.n_mg) return;
  const int g0 = A.box_off[m * A.k], g1 = A.box_off[m * A.k + 1];
  if (A.dfs_mg[m]) {
    rlo[m] = C1 + A.clique_off[g0];
    rhi[m] = C1 + A.clique_off[g1];
    return;
  }
  int64_t b[2];
  const int key[2] = {g0, g1};
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    if (leaf_root) {
      int64_t a = 0, z = n_leaf;
      while (a < z) {
        const int64_t mid = (a + z) >> 1;
        if (leaf_root[mid] < key[t]) a = mid + 1; else z = mid;
      }
      b[t] = leaf_off[a];
    } else {
      int64_t a = 0, z = C1;
      while (a < z) {
        const int64_t mid = (a + z) >> 1;
        if (A.members[mid * A.k] < key[t]) a = mid + 1; else z = mid;
      }
      b[t] = a;
    }
  }
  rlo[m] = b[0];
  rhi[m] = b[1];
}

// Weighted-degree consensus candidate and median JI of one clique from its member coordinates
// (get_cliques.py:169-190).  T = float only for integer coordinates below 2^23 and B <= 2896:
// every overlap B - |dx| (and their products, and 2 B^2 - I) is then an exact float.
template <int K, typename T>
__device__ __forceinline__ void epi_core(const T (&xs)[K], const T (&ys)[K], T B, double two_b2,
                                         bool multi, bool* exact, int* arg, double* med) {
  constexpr int NE = K * (K - 1) / 2;
  constexpr bool F = sizeof(T) == 4;
  T I[NE];   // member-pair overlaps (a < b), reference op order
  {
    int t = 0;
#pragma unroll
    for (int a = 0; a < K; ++a)
#pragma unroll
      for (int b = a + 1; b < K; ++b) {
        if constexpr (F)
          I[t++] = fmaxf(B - fabsf(xs[a] - xs[b]), 0.0f) * fmaxf(B - fabsf(ys[a] - ys[b]), 0.0f);
        else
          I[t++] = overlap(xs[a], ys[a], xs[b], ys[b], B);
      }
  }
  if (!multi) {
    // weighted degrees from f32 JIs: f32 operands (2^-24 each) and v_rcp_f32 (1 ulp) give
    // < 4e-7 per JI <= 1, < 5.5e-6 per sum of <= 7 terms with its f32 additions; a maximum
    // clear by 3e-5 is the reference's, anything closer takes the exact f64 pass (ties)
    float deg[K];
#pragma unroll
    for (int i = 0; i < K; ++i) deg[i] = 0.0f;
    int t = 0;
#pragma unroll
    for (int a = 0; a < K; ++a)
#pragma unroll
      for (int b = a + 1; b < K; ++b) {
        float jf;
        if constexpr (F) jf = I[t] * __builtin_amdgcn_rcpf((float)two_b2 - I[t]);
        else jf = (float)I[t] * __builtin_amdgcn_rcpf((float)(two_b2 - I[t]));
        deg[a] += jf;
        deg[b] += jf;
        ++t;
      }
    float d1 = deg[0], d2 = -INFINITY;
    int ag = 0;
#pragma unroll
    for (int i = 1; i < K; ++i) {
      const float d = deg[i];
      d2 = d > d1 ? d1 : fmaxf(d2, d);
      ag = d > d1 ? i : ag;
      d1 = fmaxf(d1, d);
    }
    *arg = ag;
    *exact = !(d1 - d2 > 3e-5f);
  }
  // median JI = JI of the median overlap (JI is non-decreasing in I and the f64 quotient
  // keeps that order): one or two reference divisions; I is partially sorted in place
  bool nan = false;
  if constexpr (!F) {
#pragma unroll
    for (int t = 0; t < NE; ++t) nan |= isnan(I[t]);
  }
  mid_n<NE>(I);
  if (NE & 1) {
    const double m = (double)I[NE / 2];
    *med = nan ? NAN : m / (two_b2 - m);
  } else {
    const double a = (double)I[NE / 2 - 1], b = (double)I[NE / 2];
    *med = nan ? NAN : ((a / (two_b2 - a)) + (b / (two_b2 - b))) / 2.0;
  }
}

// One 16-byte record per box for the epilogue's member gathers: the score, the row rank and,
// for integer coordinates in [-16384, 16383], both coordinates biased by 2^14 as u16s below
// 2^15 (0xffffffff otherwise: that clique takes the f64 path from A.x / A.y).  One 16-byte
// load per member and no per-clique integrality tests.
__global__ __launch_bounds__(WG) void k5_pack(int N, CliqueArgs A) {
  const int i = blockIdx.x * WG + threadIdx.x;
  if (i >= N) return;
  const double x = A.x[i], y = A.y[i];
  uint32_t xy = 0xffffffffu;
  if (x == rint(x) && y == rint(y) && x >= -16384.0 && x <= 16383.0 && y >= -16384.0 &&
      y <= 16383.0)
    xy = (uint32_t)((int)x + 16384) | ((uint32_t)((int)y + 16384) << 16);
  const uint64_t ry = (uint64_t)(uint32_t)A.vrow[i] | ((uint64_t)xy << 32);
  reinterpret_cast<double2*>(A.pk)[i] = make_double2(A.score[i], __longlong_as_double((long long)ry));
}

// Member gathers of one clique: COO rows (vertex ranks by (x, y, id), ascending) stored,
// conf = f32(median score), the packed coordinates for the overlap paths.
template <int K, typename MemF>
__device__ __forceinline__ void epi_gather_mem(const CliqueArgs& A, int64_t j, MemF&& mem,
                                               uint32_t (&xy)[K], float* conf32) {
  double s[K];
  int r[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const double2 p = reinterpret_cast<const double2*>(A.pk)[mem(i)];
    const uint64_t ry = (uint64_t)__double_as_longlong(p.y);
    s[i] = p.x;
    r[i] = (int)(uint32_t)ry;
    xy[i] = (uint32_t)(ry >> 32);
  }
  cmpnet_apply<K, false>(r);   // ascending rows
#pragma unroll
  for (int i = 0; i < K; ++i) A.rows[j * K + i] = r[i];
  *conf32 = (float)median_n<K>(s);   // conf = f32(median score)
}
template <int K>
__device__ __forceinline__ void epi_gather(const CliqueArgs& A, int64_t j, int (&mem)[K],
                                           uint32_t (&xy)[K], float* conf32) {
#pragma unroll
  for (int i = 0; i < K; ++i) mem[i] = A.members[j * K + i];
  epi_gather_mem<K>(A, j, [&](int i) { return mem[i]; }, xy, conf32);
}

// One clique's weighted-degree candidate and median JI: exact floats for integer coordinates
// (k5_pack) and integer B <= 2896 (as the fused epilogue's INTP path), f64 otherwise.
template <int K, typename MemF>
__device__ __forceinline__ void epi_single(const CliqueArgs& A, MemF&& mem,
                                           const uint32_t (&xy)[K], bool multi, bool* exact,
                                           int* arg, double* med) {
  const double B = A.B, two_b2 = A.two_b2;
  bool intok = B >= 1.0 && B <= 2896.0 && B == floor(B);
#pragma unroll
  for (int i = 0; i < K; ++i) intok = intok && xy[i] != 0xffffffffu;
  if (intok) {
    float xf[K], yf[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {   // 2^23 + u: exact, and differences stay float ops
      xf[i] = __uint_as_float(0x4b000000u | (xy[i] & 0xffffu));
      yf[i] = __uint_as_float(0x4b000000u | (xy[i] >> 16));
    }
    epi_core<K, float>(xf, yf, (float)B, two_b2, multi, exact, arg, med);
  } else {
    double xs[K], ys[K];
#pragma unroll
    for (int i = 0; i < K; ++i) { xs[i] = A.x[mem(i)]; ys[i] = A.y[mem(i)]; }
    epi_core<K, double>(xs, ys, B, two_b2, multi, exact, arg, med);
  }
}

// Two cliques at once for integer coordinates and integer B <= 255: every overlap
// max(B - |dx|, 0) * max(B - |dy|, 0) <= 65025 is an exact u16, so the overlaps and their
// median network run on packed u16 pairs (v_pk_sub/min/mul_lo_u16, v_pk_min/max_u16; the
// biased coordinates are below 2^15, so u16 differences never wrap past B).  Degrees and
// median JIs per clique exactly as epi_core's float path.
template <int K>
__device__ __forceinline__ void epi_pair(const uint32_t (&xy0)[K], const uint32_t (&xy1)[K],
                                         uint32_t b16, double two_b2, bool multi, bool* ex,
                                         int* arg, double* med) {
  constexpr int NE = K * (K - 1) / 2;
  u16x2 X[K], Y[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    X[i] = __builtin_bit_cast(u16x2, (xy0[i] & 0xffffu) | (xy1[i] << 16));
    Y[i] = __builtin_bit_cast(u16x2, (xy0[i] >> 16) | (xy1[i] & 0xffff0000u));
  }
  const u16x2 Bv = __builtin_bit_cast(u16x2, b16 | (b16 << 16));
  u16x2 I[NE];
  {
    int t = 0;
#pragma unroll
    for (int a = 0; a < K; ++a)
#pragma unroll
      for (int b = a + 1; b < K; ++b) {
        const u16x2 ox = __builtin_elementwise_sub_sat(
            Bv, __builtin_elementwise_min(X[a] - X[b], X[b] - X[a]));
        const u16x2 oy = __builtin_elementwise_sub_sat(
            Bv, __builtin_elementwise_min(Y[a] - Y[b], Y[b] - Y[a]));
        I[t++] = ox * oy;
      }
  }
  if (!multi) {
    const float c = (float)two_b2;
    float d0[K], d1[K];
#pragma unroll
    for (int i = 0; i < K; ++i) { d0[i] = 0.0f; d1[i] = 0.0f; }
    int t = 0;
#pragma unroll
    for (int a = 0; a < K; ++a)
#pragma unroll
      for (int b = a + 1; b < K; ++b) {
        const float i0 = (float)I[t].x, i1 = (float)I[t].y;
        const float j0 = i0 * __builtin_amdgcn_rcpf(c - i0);
        const float j1 = i1 * __builtin_amdgcn_rcpf(c - i1);
        d0[a] += j0; d0[b] += j0;
        d1[a] += j1; d1[b] += j1;
        ++t;
      }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      float m1 = q ? d1[0] : d0[0], m2 = -INFINITY;
      int ag = 0;
#pragma unroll
      for (int i = 1; i < K; ++i) {
        const float d = q ? d1[i] : d0[i];
        m2 = d > m1 ? m1 : fmaxf(m2, d);
        ag = d > m1 ? i : ag;
        m1 = fmaxf(m1, d);
      }
      arg[q] = ag;
      ex[q] = !(m1 - m2 > 3e-5f);   // epi_core's margin
    }
  }
  mid_n<NE>(I);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    if (NE & 1) {
      const double m = (double)(q ? I[NE / 2].y : I[NE / 2].x);
      med[q] = m / (two_b2 - m);
    } else {
      const double a = (double)(q ? I[NE / 2 - 1].y : I[NE / 2 - 1].x);
      const double b = (double)(q ? I[NE / 2].y : I[NE / 2].x);
      med[q] = ((a / (two_b2 - a)) + (b / (two_b2 - b))) / 2.0;
    }
  }
}

// spread the low 32 bits of v to the even bit positions of a 64-bit word
__device__ __forceinline__ uint64_t spread_even(uint64_t v) {
  v &= 0xffffffffull;
  v = (v | (v << 16)) & 0x0000ffff0000ffffull;
  v = (v | (v << 8)) & 0x00ff00ff00ff00ffull;
  v = (v | (v << 4)) & 0x0f0f0f0f0f0f0f0full;
  v = (v | (v << 2)) & 0x3333333333333333ull;
  v = (v | (v << 1)) & 0x5555555555555555ull;
  return v;
}

// ILP epilogue, two cliques per thread (get_cliques.py:164-202): COO rows, conf = f32(median
// score), w = f32(f64(conf) * median JI), and the consensus box (largest weighted degree,
// CPython set-order tie-break); --multi_out: the networkx node-iteration order of the members.
// Same arithmetic as the fused kernel's epilogue (rgc_fused.hip fused_epilogue_main / _order).
// Thread t takes cliques 2t and 2t + 1: the packed-u16 pair path when both qualify, one at a
// time otherwise.
// (4 waves per SIMD: the k = 8 instances spill 80 bytes per lane to fit 128 VGPRs and still
// run 2.0 % (C5) / 2.4 % (C5_256) faster than at 3 without spills; 5 and 6 waves spill
// 356 / 500 bytes and run 29 % / 46 % slower: profiles/r06al_*, r06am_*)
#ifndef RGC_EPI_WPE_N
#define RGC_EPI_WPE_N 4
#endif
#define RGC_EPI_WPE __attribute__((amdgpu_waves_per_eu(RGC_EPI_WPE_N)))
// The epilogue of cliques j0 and j1 (j1 only with ``two``) whose members are known: rows and
// conf (epi_gather_mem), then w and the consensus; cliques that need the exact f64 pass get
// their bit in exmask (zeroed before the launch; bit j & 63 of word j >> 6) and, with
// ``keep_members``, their members for that pass.
// (mem(h, i): member i of clique h = 0 / 1, read where it is used: a caller that derives the
// members from LDS does not hold 2 K of them in registers through the arithmetic)
template <int K, typename MemF>
__device__ __forceinline__ void epi_two(const CliqueArgs& A, int64_t j0, int64_t j1, bool two,
                                        MemF&& mem, bool keep_members) {
  auto mem0 = [&](int i) { return mem(0, i); };
  auto mem1 = [&](int i) { return mem(1, i); };
  uint32_t xy0[K], xy1[K];
  float cf0, cf1 = 0.0f;
  epi_gather_mem<K>(A, j0, mem0, xy0, &cf0);
  if (two) epi_gather_mem<K>(A, j1, mem1, xy1, &cf1);
  const double B = A.B;
  const bool multi = (A.flags & 2) != 0;
  bool ex[2] = {multi, multi};
  int arg[2] = {0, 0};
  double med[2] = {0.0, 0.0};
  bool pair = two && B >= 1.0 && B <= 255.0 && B == floor(B);
#pragma unroll
  for (int i = 0; i < K; ++i) pair = pair && xy0[i] != 0xffffffffu && xy1[i] != 0xffffffffu;
  if (pair) {
    epi_pair<K>(xy0, xy1, (uint32_t)B, A.two_b2, multi, ex, arg, med);
  } else {
    epi_single<K>(A, mem0, xy0, multi, &ex[0], &arg[0], &med[0]);
    if (two) epi_single<K>(A, mem1, xy1, multi, &ex[1], &arg[1], &med[1]);
  }
  A.w[j0] = (float)((double)cf0 * med[0]);
  A.conf[j0] = cf0;
  if (two) {
    A.w[j1] = (float)((double)cf1 * med[1]);
    A.conf[j1] = cf1;
  }
  // the cliques that need exact f64 degrees / node order (~3 % on C5): k5_ex_wtot /
  // k5_ex_write + k5_epi_exact, their 64-bit hashing and K x K JIs out of this kernel's
  // register budget.  One non-returning atomic OR per such clique into the zeroed words.
  if (ex[0]) {
    atomicOr(reinterpret_cast<unsigned long long*>(A.exmask) + (j0 >> 6), 1ull << (j0 & 63));
    if (keep_members)
#pragma unroll
      for (int i = 0; i < K; ++i) A.members[j0 * K + i] = mem0(i);
  } else {
    A.consensus[j0] = mem0(arg[0]);
  }
  if (two) {
    if (ex[1]) {
      atomicOr(reinterpret_cast<unsigned long long*>(A.exmask) + (j1 >> 6), 1ull << (j1 & 63));
      if (keep_members)
#pragma unroll
        for (int i = 0; i < K; ++i) A.members[j1 * K + i] = mem1(i);
    } else {
      A.consensus[j1] = mem1(arg[1]);
    }
  }
}

// Thread t takes cliques epi_lo + 2t and epi_lo + 2t + 1 (members from A.members).
template <int K>
__global__ __launch_bounds__(WG) RGC_EPI_WPE void k5_epilogue(CliqueArgs A) {
  const int64_t j0 = A.epi_lo + 2 * ((int64_t)blockIdx.x * WG + threadIdx.x);
  if (j0 >= A.C) return;
  const bool two = j0 + 1 < A.C;
  int mem0[K], mem1[K];
#pragma unroll
  for (int i = 0; i < K; ++i) mem0[i] = A.members[j0 * K + i];
  if (two)
#pragma unroll
    for (int i = 0; i < K; ++i) mem1[i] = A.members[(j0 + 1) * K + i];
  epi_two<K>(A, j0, j0 + 1, two, [&](int h, int i) {
    int v = mem0[0];
#pragma unroll
    for (int t = 0; t < K; ++t) v = i == t ? (h ? mem1[t] : mem0[t]) : v;
    return v;
  }, false);
}

// The level route's leaf level and the epilogue in one pass (k >= 3, outputs without
// members).  Wave w takes cliques [128 w, 128 w + 128) of the level route (the old epilogue's
// balance: two per lane); every leaf prefix holds 1..64 cliques (a prefix is kept only when it
// has a leaf), so those cliques come from at most 128 consecutive prefixes, starting at the one
// the leaf level's scan recorded for the wave (launch_scan's bucket output, no pass of its
// own).  The prefixes' forward-list starts and members are
// staged in LDS, and each staging lane writes, for every clique of its prefix in the wave's
// range, the prefix's slot and the leaf's lane in the root's forward list (walking the set
// bits of the leaf mask); lane l then reads the members of cliques l and l + 64 from there
// (two LDS bytes, the leaf's box from the root's forward list: no search) and runs the
// epilogue on them.  The members never go to HBM (except
// those of the ~3 % of cliques the exact pass takes): k5_leaf_fill wrote C K ints that
// k5_epilogue read back (4 GB of traffic per C5 step of 64 micrographs).
constexpr int LE_Q = LEAF_Q;   // cliques per wave

template <int K>
__global__ __launch_bounds__(WG) RGC_EPI_WPE void k5_leaf_epi(CliqueArgs A, LevelArgs L,
                                                           const int32_t* bucket, int64_t C1) {
  constexpr int NWV = WG / 64;
  constexpr int NM = K - 1;                  // staged members: the root and pickers 1..K-2
  __shared__ uint8_t s_slot[NWV][LE_Q];      // clique -> its prefix's staging slot
  __shared__ uint8_t s_lv[NWV][LE_Q];        // clique -> its leaf's lane in the root's list
  __shared__ int64_t s_lo[NWV][LE_Q];        // root's forward-list start
  __shared__ int32_t s_m[NWV][NM][LE_Q];     // the prefix's members (the same for its cliques)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t w = (int64_t)blockIdx.x * NWV + wv;
  const int64_t j0 = w * LE_Q;
  if (j0 >= C1) return;   // wave-uniform
  const int64_t a0 = bucket[w];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int t = lane + 64 * h;
    const int64_t i = a0 + t;
    if (i < L.n_items) {
      const int64_t oi = L.off[i] - j0;
      if (oi < LE_Q) {   // (prefixes past the wave's range stay unstaged)
        const int r = L.in_root[i];
        const uint64_t P = L.in_P[i];
        const int64_t lo = A.fwd_off[r];
        uint64_t c = L.in_M[i];   // (the last fill stored the leaf mask itself)
        s_lo[wv][t] = lo;
        s_m[wv][0][t] = r;
#pragma unroll
        for (int u = 0; u < K - 2; ++u) s_m[wv][u + 1][t] = A.e_dst[lo + ((P >> (6 * u)) & 63)];
        // the prefix's cliques in the wave's range: slot and leaf lane by clique (the
        // first prefix may start before the range)
        for (int q = (int)oi; c && q < LE_Q; ++q) {
          const int v = __builtin_ctzll(c);
          c &= c - 1;
          if (q >= 0) {
            s_slot[wv][q] = (uint8_t)t;
            s_lv[wv][q] = (uint8_t)v;
          }
        }
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  // clique q: its prefix's staging slot and its leaf box
  auto locate = [&](int q, int* slot, int* leaf) {
    const int a = s_slot[wv][q];
    *slot = a;
    *leaf = A.e_dst[s_lo[wv][a] + s_lv[wv][q]];
  };
  const int qa = lane, qb = lane + 64;
  if (j0 + qa >= C1) return;
  const bool two = j0 + qb < C1;
  int sa, la, sb = 0, lb = 0;
  locate(qa, &sa, &la);
  if (two) locate(qb, &sb, &lb);
  else { sb = sa; lb = la; }
  // members read from the staging where they are used (the slots and leaf boxes stay live, not
  // 2 K member ids: k = 8 spilled otherwise)
  epi_two<K>(A, j0 + qa, j0 + qb, two, [&](int h, int i) {
    return i == K - 1 ? (h ? lb : la) : s_m[wv][i][h ? sb : sa];
  }, true);
}

// The deferred cliques as a list: one wave per 64 ballot words (4096 cliques) ranks their set
// bits with a DPP scan of the word popcounts and reserves its slice of the list with one
// atomic (C / 4096 atomics per launch instead of one per epilogue wave).
// The exact list without a shared counter: per compaction wave (64 ballot words = 4096
// cliques) its count (k5_ex_wtot), a one-pass scan of the counts, then each wave writes its
// slice (k5_ex_write).  (k5_ex_compact's one atomic per wave on one word: 15k serialised
// returning atomics per C5 step, ~0.16 ms, replaced in round 5.)
__global__ __launch_bounds__(WG) void k5_ex_wtot(CliqueArgs A) {
  const int lane = threadIdx.x & 63;
  const int64_t nwords = (A.C + 63) >> 6;
  const int64_t wv = ((int64_t)blockIdx.x * WG + threadIdx.x) >> 6;
  const int64_t w0 = wv * 64;
  if (w0 >= nwords) return;   // wave-uniform
  const uint64_t word = w0 + lane < nwords ? A.exmask[w0 + lane] : 0ull;
  const int total = __shfl(wave_incl_add32(__popcll(word)), 63);
  if (lane == 0) A.exwtot[wv] = total;
}
__global__ __launch_bounds__(WG) void k5_ex_write(CliqueArgs A) {
  const int lane = threadIdx.x & 63;
  const int64_t nwords = (A.C + 63) >> 6;
  const int64_t wv = ((int64_t)blockIdx.x * WG + threadIdx.x) >> 6;
  const int64_t w0 = wv * 64;
  if (w0 >= nwords) return;   // wave-uniform
  const uint64_t word = w0 + lane < nwords ? A.exmask[w0 + lane] : 0ull;
  const int cnt = __popcll(word);
  const int incl = wave_incl_add32(cnt);
  int64_t o = A.exwoff[wv] + incl - cnt;
  for (uint64_t w = word; w; w &= w - 1) A.exlist[o++] = ((w0 + lane) << 6) + __builtin_ctzll(w);
}


// Consensus (and --multi_out node order) of the cliques k5_epilogue deferred: exact f64
// weighted degrees (get_cliques.py:182-183) and, on ties, the first tied member in networkx's
// node-iteration order (CPython set order of (x, y, id), or graph insertion order when
// 2k >= |G|).  Grid-stride over the deferred list.
// (k = 8: 159 VGPRs, 3 waves per SIMD; forced to 4 it spills 92 bytes and runs 1 % slower
// per C5 step: profiles/r06an_*)
template <int K>
__global__ __launch_bounds__(WG) void k5_epi_exact(CliqueArgs A) {
  const int64_t n = (int64_t)*A.excount;
  for (int64_t t = (int64_t)blockIdx.x * WG + threadIdx.x; t < n; t += (int64_t)gridDim.x * WG) {
    const int64_t j = A.exlist[t];
    int mem[K];
    double xs[K], ys[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
      mem[i] = A.members[j * K + i];
      xs[i] = A.x[mem[i]];
      ys[i] = A.y[mem[i]];
    }
    const int m = A.bmg[mem[0]];
    const int64_t idb = A.id_base[m] - (int64_t)A.box_off[m * A.k];
    double ji[K][K];
    int64_t ids[K];
    uint64_t ins[K] = {};
#pragma unroll
    for (int a = 0; a < K; ++a) {
      ids[a] = idb + mem[a];
#pragma unroll
      for (int b = a + 1; b < K; ++b) ji[a][b] = jaccard(xs[a], ys[a], xs[b], ys[b], A.B, A.two_b2);
    }
    const bool set_order = 2 * K < A.st[m].n_nodes;
    if (!set_order) {
#pragma unroll
      for (int i = 0; i < K; ++i) ins[i] = A.ins_key[mem[i]];
    }
    uint32_t top;
    int arg = epi_degree_max<K>(ji, &top);
    const bool tie = (top & (top - 1)) != 0;
    const bool multi = (A.flags & 2) != 0;
    if (tie || multi) {
      const uint32_t ord = node_order<K>(mem, xs, ys, ids, set_order, ins);
      if (tie) arg = epi_tie_arg<K>(top, ord);
      if (multi) {
#pragma unroll
        for (int i = 0; i < K; ++i) A.order[j * K + i] = (uint8_t)((ord >> (4 * i)) & 15);
      }
    }
    int cons = mem[0];
#pragma unroll
    for (int i = 1; i < K; ++i) cons = (arg == i) ? mem[i] : cons;
    A.consensus[j] = cons;
  }
}

template <int K>
static int launch_level_k(hipStream_t stream, bool first, bool leaf, bool fill, const CliqueArgs& A,
                          const LevelArgs& L) {
  const int64_t nb = (L.n_items + WG - 1) / WG;
  if (nb <= 0) return 0;
#define RGC_LVL(F, LF, FL) \
  hipLaunchKernelGGL((k5l<K, F, LF, FL>), dim3(nb), dim3(WG), 0, stream, A, L)
  if (first) {
    if (leaf) { if (fill) RGC_LVL(true, true, true); else RGC_LVL(true, true, false); }
    else { if (fill) RGC_LVL(true, false, true); else RGC_LVL(true, false, false); }
  } else {
    if (leaf) {
      if (fill) {
        if constexpr (K >= 3)   // wavefront-cooperative (coalesced member stores)
          hipLaunchKernelGGL((k5_leaf_fill<K>), dim3(nb), dim3(WG), 0, stream, A, L);
        else
          RGC_LVL(false, true, true);
      } else {
        RGC_LVL(false, true, false);
      }
    }
    else { if (fill) RGC_LVL(false, false, true); else RGC_LVL(false, false, false); }
  }
#undef RGC_LVL
  return 0;
}

int launch_clique_level(hipStream_t stream, bool first, bool leaf, bool fill, const CliqueArgs& A,
                        const LevelArgs& L) {
  switch (A.k) {
    case 2: return launch_level_k<2>(stream, first, leaf, fill, A, L);
    case 3: return launch_level_k<3>(stream, first, leaf, fill, A, L);
    case 4: return launch_level_k<4>(stream, first, leaf, fill, A, L);
    case 5: return launch_level_k<5>(stream, first, leaf, fill, A, L);
    case 6: return launch_level_k<6>(stream, first, leaf, fill, A, L);
    case 7: return launch_level_k<7>(stream, first, leaf, fill, A, L);
    case 8: return launch_level_k<8>(stream, first, leaf, fill, A, L);
    default: return -1;
  }
}

void launch_clique_setup(hipStream_t stream, int N, const CliqueArgs& A) {
  const int nb = (N + WG - 1) / WG;
  if (!nb) return;
  hipLaunchKernelGGL(k5_route, dim3(nb), dim3(WG), 0, stream, N, A);
  const int nr = A.n_roots;
  if (nr) hipLaunchKernelGGL(k5n_build, dim3((nr + WG / NBG - 1) / (WG / NBG)), dim3(WG), 0, stream, A);
}

#ifndef RGC_EXGRID
#define RGC_EXGRID 1024
#endif
static void ex_compact(hipStream_t stream, const CliqueArgs& A, int64_t nb) {
  const int64_t nwv = (((A.C + 63) >> 6) + 63) / 64;   // compaction waves
  hipLaunchKernelGGL(k5_ex_wtot, dim3((nb + 63) / 64), dim3(WG), 0, stream, A);
  launch_scan(stream, nwv, A.exwtot, A.exwoff, A.tiles, reinterpret_cast<int64_t*>(A.excount));
  hipLaunchKernelGGL(k5_ex_write, dim3((nb + 63) / 64), dim3(WG), 0, stream, A);
}

int launch_clique_epilogue(hipStream_t stream, bool exact_pass, const CliqueArgs& A) {
  const int64_t nb = (A.C + WG - 1) / WG;
  if (nb <= 0) return 0;
  const int64_t nbe = (A.C - A.epi_lo + WG - 1) / WG;   // k5_epilogue: [epi_lo, C)
  switch (A.k) {
#define RGC_EPI(KK)                                                                      \
  case KK:                                                                               \
    if (!exact_pass) {                                                                   \
      if (nbe > 0)                                                                       \
        hipLaunchKernelGGL((k5_epilogue<KK>), dim3((nbe + 1) / 2), dim3(WG), 0, stream, A); \
    } else {                                                                             \
      ex_compact(stream, A, nb);                                                         \
      hipLaunchKernelGGL((k5_epi_exact<KK>), dim3(std::min<int64_t>(nb, RGC_EXGRID)),      \
                         dim3(WG), 0, stream, A);                                        \
    }                                                                                    \
    break;
    RGC_EPI(2) RGC_EPI(3) RGC_EPI(4) RGC_EPI(5) RGC_EPI(6) RGC_EPI(7) RGC_EPI(8)
#undef RGC_EPI
    default: return -1;
  }
  return 0;
}

int launch_clique_leaf_epi(hipStream_t stream, const CliqueArgs& A, const LevelArgs& L,
                           int32_t* bucket, int64_t C1) {
  if (L.n_items <= 0 || C1 <= 0) return 0;
  const int64_t nw = (C1 + LE_Q - 1) / LE_Q, nbe = (nw + WG / 64 - 1) / (WG / 64);
  switch (A.k) {
#define RGC_LE(KK) \
  case KK:         \
    hipLaunchKernelGGL((k5_leaf_epi<KK>), dim3(nbe), dim3(WG), 0, stream, A, L, bucket, C1); \
    break;
    RGC_LE(3) RGC_LE(4) RGC_LE(5) RGC_LE(6) RGC_LE(7) RGC_LE(8)
#undef RGC_LE
    default: return -1;
  }
  return 0;
}

void launch_clique_pack(hipStream_t stream, int N, const CliqueArgs& A) {
  if (N > 0) hipLaunchKernelGGL(k5_pack, dim3((N + WG - 1) / WG), dim3(WG), 0, stream, N, A);
}

void launch_clique_ranges(hipStream_t stream, const CliqueArgs& A, int64_t C1, int64_t* rlo,
                          int64_t* rhi, const int32_t* leaf_root, const int64_t* leaf_off,
                          int64_t n_leaf) {
  if (A.n_mg > 0)
    hipLaunchKernelGGL(k5_ranges, dim3((A.n_mg + WG - 1) / WG), dim3(WG), 0, stream, A, C1, rlo,
                       rhi, leaf_root, leaf_off, n_leaf);
}

}  // namespace rgc
