// rgc_ilp.hip — exact max-weight set packing: the ILP of run_ilp.
//
// Reference repic/commands/run_ilp.py:50-63: per micrograph, binary x over the cliques
// (columns of the constraint matrix A), maximise w.x subject to A x <= 1 (every box in at most
// one chosen clique), solved there by Gurobi.  Two cliques conflict iff they share a box, and
// the problem splits into the connected components of that conflict graph (cliques of a box
// graph component, usually a handful).  Pipeline (all on the device, one batch of many
// micrographs; rows are global box ids, so micrographs never mix):
//   1. k_ilp_rep / k_ilp_union / k_ilp_root: lock-free union-find of the columns through
//      their rows (each row links its columns to the smallest one).
//   2. components numbered by a scan over roots, member lists filled, rows -> columns CSR.
//   3. k_ilp_small: one THREAD per component of 2..64 cliques; k_ilp_wave: one WAVEFRONT per
//      larger component (bitsets one 64-bit word per lane, up to 4096 cliques).  Both run the
//      same depth-first branch and bound over candidates sorted by weight (include the
//      heaviest remaining candidate first, then exclude it), pruning with the box-partition
//      bound: assign every candidate to one of its boxes (its a-th row); at most one
//      candidate per box can be chosen, so sum over boxes of the heaviest candidate is an
//      upper bound; the minimum over the k assignments is used.  Weights are f32 values
//      summed in f64 (exact), so "optimal" is exact.  A component that exceeds the node
//      limit keeps the best packing found and is reported as not proven optimal.
#include "rgc_kernels.h"
#include "../../include/repic_gc.h"

#include <climits>

namespace rgc {

constexpr int ILP_WG = 256;
constexpr uint8_t ST_IN_SEED = 1;        // (= ST_IN below: the pre-search packing)
constexpr int ILP_SMALL = 64;     // thread-per-component limit (one 64-bit mask)
constexpr int ILP_BIG = 4096;     // wave-per-component limit (64 lanes x 64 bits)
// the wave search stops at Gurobi's MIPGap (GAP_OK) only after this many nodes: a component
// whose search proves optimality sooner gets its exact optimum (status OPTIMAL), as an exact
// solver's choice, and only the hard ones take the 1e-4 early stop
constexpr int64_t ILP_GAP_NODES = 1 << 16;

__device__ __forceinline__ int32_t ilp_find(int32_t* p, int32_t x) {
  for (;;) {
    const int32_t q = __hip_atomic_load(p + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (q == x) return x;
    const int32_t g = __hip_atomic_load(p + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (g != q) __hip_atomic_store(p + x, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    x = g;
  }
}

__device__ __forceinline__ void ilp_union(int32_t* p, int32_t a, int32_t b) {
  for (;;) {
    a = ilp_find(p, a);
    b = ilp_find(p, b);
    if (a == b) return;
    if (a < b) { const int32_t t = a; a = b; b = t; }
    if (atomicCAS(p + a, a, b) == a) return;
  }
}

__global__ __launch_bounds__(ILP_WG) void k_ilp_init(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c < A.n_cols) {
    A.parent[c] = (int32_t)c;
    A.csize[c] = 0;
  }
  if (c < A.n_rows) {
    A.rep[c] = INT_MAX;
    A.rloc[c] = INT_MAX;
    A.rcnt[c] = 0;
    A.rcur[c] = 0;
  }
}

// 1. smallest column of every row
__global__ __launch_bounds__(ILP_WG) void k_ilp_rep(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c >= A.n_cols) return;
  for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e) atomicMin(A.rep + A.row_idx[e], (int)c);
}

__global__ __launch_bounds__(ILP_WG) void k_ilp_union(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c >= A.n_cols) return;
  for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e) {
    const int32_t r = A.rep[A.row_idx[e]];
    if (r != (int32_t)c) ilp_union(A.parent, (int32_t)c, r);
  }
}

// compress; root flags (for the component scan) and component sizes by root; rows -> column
// counts (the transpose's CSR)
__global__ __launch_bounds__(ILP_WG) void k_ilp_root(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c >= A.n_cols) return;
  const int32_t r = ilp_find(A.parent, (int32_t)c);
  A.parent[c] = r;
  A.is_root[c] = r == (int32_t)c ? 1 : 0;
  atomicAdd(A.csize + r, 1);
  for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e) atomicAdd(A.rcnt + A.row_idx[e], 1);
}

// component sizes in component order (comp id = scanned root index)
__global__ __launch_bounds__(ILP_WG) void k_ilp_csize(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c >= A.n_cols || !A.is_root[c]) return;
  A.comp_n[A.comp_id[c]] = A.csize[c];
}

// member lists (arbitrary order; the solvers sort them) and the rows -> columns lists
__global__ __launch_bounds__(ILP_WG) void k_ilp_fill(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c >= A.n_cols) return;
  const int64_t comp = A.comp_id[A.parent[c]];
  const int slot = atomicAdd(A.comp_cur + comp, 1);
  A.members[A.comp_off[comp] + slot] = (int32_t)c;
  for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e) {
    const int32_t r = A.row_idx[e];
    A.rcols[A.rptr[r] + atomicAdd(A.rcur + r, 1)] = (int32_t)c;
  }
}

// Local numbering of a component: members sorted by (weight desc, column asc), so the lowest
// set bit of a candidate set is its heaviest candidate.  Rank sort: member i's position is
// the number of members that come before it (lanes / threads share the O(n^2) count).
__device__ __forceinline__ bool ilp_before(const IlpArgs& A, int32_t d, int32_t c) {
  const double wd = A.w[d], wc = A.w[c];
  return wd > wc || (wd == wc && d < c);
}

// Local rows (boxes) of a component and each member's packed row info, in scratch:
// lr[i * (K + 1) + a] = local id of member i's a-th row (a < deg; padded with its last row),
// lr[i * (K + 1) + K] = its opener box: the row with the most columns (ties: first).  Local
// ids via the winner of an atomicMin over member slots (i * K + a) on the global row array
// rloc (rows belong to one component only), then a counter.  Steps are separated by the
// caller's barriers: step 0 claims, step 1 numbers the winners, step 2 writes lr.
template <bool SERIAL>
__device__ void ilp_rows_step(const IlpArgs& A, const int32_t* m, int n, int K, int step, int i0,
                              int di, int32_t* tmpid, uint16_t* lr, int* counter) {
  for (int i = i0; i < n; i += di) {
    const int32_t c = m[i];
    const int64_t e0 = A.col_ptr[c], e1 = A.col_ptr[c + 1];
    int best_deg = -1, best_row = 0;
    for (int a = 0; a < K; ++a) {
      const int64_t e = e0 + a < e1 ? e0 + a : e1 - 1;
      const int32_t r = A.row_idx[e];
      const int32_t slot = i * K + a;
      if (step == 0) {
        if (e0 + a < e1) atomicMin(A.rloc + r, slot);
      } else if (step == 1) {
        if (e0 + a < e1 && A.rloc[r] == slot) tmpid[slot] = SERIAL ? (*counter)++ : atomicAdd(counter, 1);
      } else {
        const int id = tmpid[A.rloc[r]];
        lr[i * (K + 1) + a] = (uint16_t)id;
        const int deg = (int)(A.rptr[r + 1] - A.rptr[r]);
        if (deg > best_deg) { best_deg = deg; best_row = id; }
      }
    }
    if (step == 2) lr[i * (K + 1) + K] = (uint16_t)best_row;
  }
}

// One thread per component of 2..64 cliques.  Scratch ((2 kmax + 8) 64-bit words per member
// at the component's offset): weights, adjacency masks, DFS stack, row info.  The bound is a
// greedy clique cover of the candidates by boxes: heaviest first, a candidate with one of its
// boxes already opened joins that box's group (it conflicts with every member), otherwise it
// opens its opener box and adds its weight.  At most one candidate per group can be chosen,
// so the sum of the openers' weights bounds the best packing of the candidates.
constexpr int ILP_SMALL_ROWWORDS = ILP_SMALL * 8 / 64;   // open-box bits per thread (K <= 8)

__global__ __launch_bounds__(ILP_WG) void k_ilp_small(IlpArgs A) {
  __shared__ uint64_t open_lds[ILP_WG][ILP_SMALL_ROWWORDS];
  const int64_t comp = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (comp >= A.n_comp) return;
  const int n = A.comp_n[comp];
  const int64_t off = A.comp_off[comp];
  int32_t* m = A.members + off;
  if (n == 1) {
    const int32_t c = m[0];
    A.x[c] = A.w[c] > 0.0 ? 1 : 0;
    A.exact[c] = 1;
    return;
  }
  if (n > ILP_SMALL) return;
  const int K = A.kmax;
  double* wl = reinterpret_cast<double*>(A.scratch + off * (2 * K + 8));   // n
  uint64_t* adj = reinterpret_cast<uint64_t*>(wl + n);                    // n
  uint64_t* stk = adj + n;                                                 // 3 n
  int32_t* tmpid = reinterpret_cast<int32_t*>(stk + 3 * n);                // K n
  uint16_t* lr = reinterpret_cast<uint16_t*>(tmpid + K * n);               // (K + 1) n
  int32_t* sorted = reinterpret_cast<int32_t*>(stk);                       // (before the DFS)
  // rank sort by (weight desc, column asc)
  for (int i = 0; i < n; ++i) {
    int r = 0;
    for (int q = 0; q < n; ++q) r += ilp_before(A, m[q], m[i]) ? 1 : 0;
    sorted[r] = m[i];
  }
  for (int i = 0; i < n; ++i) m[i] = sorted[i];
  for (int i = 0; i < n; ++i) {
    A.loc[m[i]] = i;
    wl[i] = A.w[m[i]];
  }
  int nrow = 0;
  for (int step = 0; step < 3; ++step) ilp_rows_step<true>(A, m, n, K, step, 0, 1, tmpid, lr, &nrow);
  for (int i = 0; i < n; ++i) {
    uint64_t a = 0;
    const int32_t c = m[i];
    for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e) {
      const int32_t r = A.row_idx[e];
      for (int64_t f = A.rptr[r]; f < A.rptr[r + 1]; ++f) a |= 1ull << A.loc[A.rcols[f]];
    }
    adj[i] = a & ~(1ull << i);
  }
  uint64_t* open = open_lds[threadIdx.x];
  const int ow = (nrow + 63) / 64;
  auto bound = [&](uint64_t P) {
    for (int q = 0; q < ow; ++q) open[q] = 0;
    double s = 0.0;
    while (P) {
      const int i = __builtin_ctzll(P);
      P &= P - 1;
      const uint16_t* li = lr + i * (K + 1);
      bool cov = false;
      for (int a = 0; a < K; ++a) cov |= (open[li[a] >> 6] >> (li[a] & 63)) & 1;
      if (!cov) {
        open[li[K] >> 6] |= 1ull << (li[K] & 63);
        s += wl[i];
      }
    }
    return s;
  };
  const uint64_t all = (n == 64) ? ~0ull : ((1ull << n) - 1);
  double best = -1.0, cur = 0.0;
  uint64_t best_set = 0, chosen = 0, P = all;
  int depth = 0;
  int64_t nodes = 0;
  bool exact = true;
  for (;;) {
    bool back = false;
    if (++nodes > A.node_limit) { exact = false; break; }
    if (P == 0) {
      if (cur > best) { best = cur; best_set = chosen; }
      back = true;
    } else if (cur + bound(P) <= best) {
      back = true;
    } else {
      // include the heaviest candidate j (lowest bit) first; its frame keeps P and cur
      const int j = __builtin_ctzll(P);
      stk[3 * depth] = P;
      stk[3 * depth + 1] = (uint64_t)__double_as_longlong(cur);
      stk[3 * depth + 2] = ((uint64_t)j << 1) | 1u;
      ++depth;
      P &= ~adj[j] & ~(1ull << j);
      cur += wl[j];
      chosen |= 1ull << j;
    }
    if (back) {
      // unwind to the nearest frame still on its include branch and take its exclude branch
      bool found = false;
      while (depth > 0) {
        const uint64_t fr = stk[3 * (depth - 1) + 2];
        const int j = (int)(fr >> 1);
        if (fr & 1u) {
          stk[3 * (depth - 1) + 2] = (uint64_t)j << 1;
          P = stk[3 * (depth - 1)] & ~(1ull << j);
          cur = __longlong_as_double((long long)stk[3 * (depth - 1) + 1]);
          chosen &= (1ull << j) - 1;   // earlier frames chose only members < j
          found = true;
          break;
        }
        --depth;
      }
      if (!found) break;
    }
  }
  for (int i = 0; i < n; ++i) {
    A.x[m[i]] = (best_set >> i) & 1 ? 1 : 0;
    A.exact[m[i]] = exact ? 1 : 0;
  }
}

// list of the components handled by the wave solver
__global__ __launch_bounds__(ILP_WG) void k_ilp_biglist(IlpArgs A) {
  const int64_t comp = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (comp >= A.n_comp) return;
  if (A.comp_n[comp] > ILP_SMALL) A.big[atomicAdd(A.n_big, 1u)] = (int32_t)comp;
}

constexpr int ILP_LRCAP = 16384;   // u16 row-info entries kept in LDS (wave solver)

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// One wavefront per component of 65..4096 cliques (persistent: waves take components from
// the list).  Lane l holds word l of every bitset; adjacency rows and the DFS stack in the
// wave's scratch; open boxes and (when they fit) the members' row info in LDS.  The greedy
// clique-cover bound runs 64 candidates at a time: candidates covered by boxes opened in
// earlier chunks drop out, then the lowest (heaviest) uncovered lane opens its box and the
// lanes holding that box drop out, until none is left - the sequential greedy's result.
__global__ __launch_bounds__(64) void k_ilp_wave(IlpArgs A, int n_big) {
  __shared__ uint64_t open[ILP_BIG * 8 / 64];
  __shared__ uint64_t mark[ILP_BIG * 8 / 64];   // rows of the candidates (Lagrangian bound)
  __shared__ uint16_t lrs[ILP_LRCAP];
  __shared__ int counter;
  const int lane = threadIdx.x;
  uint64_t* base = A.wscratch + (int64_t)blockIdx.x * A.wstride;
  for (int bi = blockIdx.x; bi < n_big; bi += gridDim.x) {
    const int64_t comp = A.big[bi];
    const int n = A.comp_n[comp];
    int32_t* m = A.members + A.comp_off[comp];
    if (n > ILP_BIG) {
      for (int i = lane; i < n; i += 64) { A.x[m[i]] = 0; A.exact[m[i]] = 0; }
      continue;
    }
    const int W = (n + 63) / 64;
    const int K = A.kmax;
    uint64_t* adj = base;                                         // n W
    uint64_t* stk = adj + (int64_t)n * W;                         // n (W + 2)
    double* wl = reinterpret_cast<double*>(stk + (int64_t)n * (W + 2));   // n
    int32_t* tmpid = reinterpret_cast<int32_t*>(wl + n);          // K n
    uint16_t* lrg = reinterpret_cast<uint16_t*>(tmpid + (int64_t)K * n);   // (K + 1) n
    // Lagrangian bound data (components with pre-B&B multipliers, cert == 3): multiplier of
    // each local row, max(0, reduced weight) of each member
    double* lamloc = reinterpret_cast<double*>(base + A.wlag_off);          // K n
    double* posw = lamloc + (int64_t)K * n;                                 // n
    int32_t* sorted = reinterpret_cast<int32_t*>(stk);
    for (int i = lane; i < n; i += 64) {
      int r = 0;
      for (int q = 0; q < n; ++q) r += ilp_before(A, m[q], m[i]) ? 1 : 0;
      sorted[r] = m[i];
    }
    wave_sync();
    for (int i = lane; i < n; i += 64) {
      m[i] = sorted[i];
      A.loc[sorted[i]] = i;
      wl[i] = A.w[sorted[i]];
    }
    if (lane == 0) counter = 0;
    wave_sync();
    for (int step = 0; step < 3; ++step) {
      ilp_rows_step<false>(A, m, n, K, step, lane, 64, tmpid, lrg, &counter);
      wave_sync();
    }
    const int nrow = counter;
    // adjacency rows: lane i builds row i's words
    for (int i = lane; i < n; i += 64) {
      uint64_t* row = adj + (int64_t)i * W;
      for (int q = 0; q < W; ++q) row[q] = 0;
      const int32_t c = m[i];
      for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e) {
        const int32_t r = A.row_idx[e];
        for (int64_t f = A.rptr[r]; f < A.rptr[r + 1]; ++f) {
          const int j = A.loc[A.rcols[f]];
          if (j != i) row[j >> 6] |= 1ull << (j & 63);
        }
      }
    }
    const bool lds_rows = n * (K + 1) <= ILP_LRCAP;
    if (lds_rows)
      for (int t = lane; t < n * (K + 1); t += 64) lrs[t] = lrg[t];
    const uint16_t* lr = lds_rows ? lrs : lrg;
    // Lagrangian relaxation of the box constraints with the component's multipliers lam >= 0
    // (projected subgradient before the search, rgc_ilp_solve): for any candidate set P,
    //   max packing of P <= sum over rows r of P of lam_r + sum over i in P of max(0, w_i - sum
    //   over i's rows of lam_r),
    // near the LP optimum when lam is, so it prunes where the greedy clique cover cannot (the
    // crowded C3 components' integrality gaps are 0.03-0.8 %).  Used as min(cover, lagrangian)
    const bool lag = A.cert != nullptr && A.lam != nullptr && A.cert[comp] == 3;
    if (lag) {
      for (int i = lane; i < n; i += 64) {
        const int32_t c = m[i];
        const int64_t e0 = A.col_ptr[c], e1 = A.col_ptr[c + 1];
        double rc = wl[i];
        for (int64_t e = e0; e < e1; ++e) {
          const double l = A.lam[A.row_idx[e]];
          rc -= l;
          lamloc[lr[i * (K + 1) + (int)(e - e0)]] = l;
        }
        posw[i] = rc > 0.0 ? rc : 0.0;
      }
    }
    wave_sync();
    const int ow = (nrow + 63) / 64;
    // the Lagrangian bound of candidate set P (all lanes get the wave's sum), padded by a
    // relative 1e-12 so its f64 rounding can never prune a better packing
    auto lag_bound = [&](uint64_t P) {
      for (int q = lane; q < ow; q += 64) mark[q] = 0;
      __builtin_amdgcn_wave_barrier();
      double s = 0.0;
      for (int q = 0; q < W; ++q) {
        const uint64_t word = __shfl(P, q, 64);
        if (!((word >> lane) & 1)) continue;
        const int i = q * 64 + lane;
        s += posw[i];
        const uint16_t* li = lr + i * (K + 1);
        for (int a = 0; a < K; ++a)
          atomicOr(reinterpret_cast<unsigned long long*>(mark) + (li[a] >> 6), 1ull << (li[a] & 63));
      }
      __builtin_amdgcn_wave_barrier();
      for (int q = lane; q < ow; q += 64) {
        uint64_t wd = mark[q];
        while (wd) {
          s += lamloc[q * 64 + __builtin_ctzll(wd)];
          wd &= wd - 1;
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      return s * (1.0 + 1e-12);
    };
    auto bound = [&](uint64_t P) {
      for (int q = lane; q < ow; q += 64) open[q] = 0;
      __builtin_amdgcn_wave_barrier();
      double s = 0.0;
      for (int q = 0; q < W; ++q) {
        const uint64_t word = __shfl(P, q, 64);
        if (word == 0) continue;
        const int i = q * 64 + lane;
        bool pend = (word >> lane) & 1;
        uint16_t rr[8];
        uint16_t o = 0;
        if (pend) {
          const uint16_t* li = lr + i * (K + 1);
          bool cov = false;
#pragma unroll
          for (int a = 0; a < 8; ++a) {
            rr[a] = a < K ? li[a] : li[0];
            cov |= (open[rr[a] >> 6] >> (rr[a] & 63)) & 1;
          }
          o = li[K];
          pend = !cov;
        }
        for (;;) {
          const uint64_t bal = __ballot(pend);
          if (bal == 0) break;
          const int f = __builtin_ctzll(bal);
          const int ob = __shfl((int)o, f, 64);
          s += wl[q * 64 + f];
          if (lane == f) {
            open[ob >> 6] |= 1ull << (ob & 63);
            pend = false;
          }
          if (pend) {
#pragma unroll
            for (int a = 0; a < 8; ++a) pend = pend && rr[a] != ob;
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
      return s;
    };
    // lane-sliced sets: P (candidates), chosen
    uint64_t P = 0, chosen = 0, best_set = 0;
    if (lane < W) P = (lane == W - 1 && (n & 63)) ? ((1ull << (n & 63)) - 1) : ~0ull;
    // the root's bound: the search stops once the incumbent is within Gurobi's MIPGap (1e-4,
    // relative; run_ilp.py:50-63 solves with default parameters) of it - status GAP_OK
    const double root_bound = lag ? fmin(bound(P), lag_bound(P)) : bound(P);
    double best = -1.0, cur = 0.0;
    // incumbent seeded with the pre-search packing (greedy + swaps, A.st of the cert-3
    // components): the search prunes against it from the first node and may stop at once
    if (lag && A.st) {
      uint64_t bs = 0;
      double v = 0.0;
      if (lane < W)
        for (int b = 0; b < 64; ++b) {
          const int i = lane * 64 + b;
          if (i >= n) break;
          if (A.st[m[i]] == ST_IN_SEED) {
            bs |= 1ull << b;
            v += wl[i];
          }
        }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      // (a hair below its value: a packing of equal weight met in the search's heaviest-first
      // order still replaces it, so ties resolve as without the seed)
      if (v > 0.0) {
        best = v * (1.0 - 1e-12);
        best_set = bs;
      }
    }
    int depth = 0;
    int64_t nodes = 0;
    uint8_t status = RGC_ILP_OPTIMAL;
    // node budget in work units: a node costs O(W) (bound passes over P's words), so
    // components above 1024 cliques get node_limit * 16 / W nodes.  The budget is the only
    // limit of the search (no clock): the result does not depend on the device's speed or load
    const int64_t node_cap = A.node_limit * 16 / (W > 16 ? W : 16);
    for (; status == RGC_ILP_OPTIMAL;) {
      bool back = false;
      if (++nodes > node_cap) { status = RGC_ILP_NODE_LIMIT; break; }
      // past ILP_GAP_NODES the MIPGap stop, checked every 1024 nodes
      if ((nodes & 1023) == 0) {
        if (nodes >= ILP_GAP_NODES && best > 0.0 && root_bound - best <= 1e-4 * best) {
          status = RGC_ILP_GAP_OK;
          break;
        }
      }
      const uint64_t nz = __ballot(P != 0);
      if (nz == 0) {
        if (cur > best) {
          best = cur;
          best_set = chosen;
          if (nodes >= ILP_GAP_NODES && root_bound - best <= 1e-4 * best && depth > 0) {
            status = RGC_ILP_GAP_OK;
            break;
          }
        }
        back = true;
      } else if ((lag && cur + lag_bound(P) <= best) || cur + bound(P) <= best) {
        back = true;
      } else {
        const int fl = __builtin_ctzll(nz);
        const uint64_t pw = __shfl(P, fl, 64);
        const int j = fl * 64 + __builtin_ctzll(pw);
        uint64_t* fr = stk + (int64_t)depth * (W + 2);
        if (lane < W) fr[lane] = P;
        if (lane == 0) {
          fr[W] = (uint64_t)__double_as_longlong(cur);
          fr[W + 1] = ((uint64_t)j << 1) | 1u;
        }
        ++depth;
        const uint64_t aw = lane < W ? adj[(int64_t)j * W + lane] : 0;
        P &= ~aw;
        if (lane == (j >> 6)) {
          P &= ~(1ull << (j & 63));
          chosen |= 1ull << (j & 63);
        }
        cur += wl[j];
      }
      if (back) {
        bool found = false;
        wave_sync();
        while (depth > 0) {
          uint64_t* fr = stk + (int64_t)(depth - 1) * (W + 2);
          const uint64_t f = fr[W + 1];
          const int j = (int)(f >> 1);
          if (f & 1u) {
            wave_sync();
            if (lane == 0) fr[W + 1] = (uint64_t)j << 1;
            P = lane < W ? fr[lane] : 0;
            cur = __longlong_as_double((long long)fr[W]);
            // candidates chosen below this frame are all > j (heavier ones come first)
            if (lane == (j >> 6)) {
              P &= ~(1ull << (j & 63));
              chosen &= (1ull << (j & 63)) - 1;
            } else if (lane > (j >> 6)) {
              chosen = 0;
            }
            found = true;
            break;
          }
          --depth;
        }
        if (!found) break;
      }
    }
    // x: lane l owns members 64 l .. 64 l + 63
    if (lane < W) {
      for (int b = 0; b < 64; ++b) {
        const int i = lane * 64 + b;
        if (i >= n) break;
        A.x[m[i]] = (best_set >> b) & 1 ? 1 : 0;
        A.exact[m[i]] = status;
      }
    }
    // GAP_OK: the certified gap at the component's first member (the certification below
    // leaves such components alone: only NODE_LIMIT ones are flagged)
    if (status == RGC_ILP_GAP_OK && A.gap && lane == 0) A.gap[m[0]] = fmax(root_bound - best, 0.0);
    wave_sync();
  }
}

// ----------------------------------------------------------------------------- certification
// Components the branch and bound did not prove optimal: more than ILP_BIG cliques (never
// searched) or node_limit hit.  Gurobi (run_ilp.py:50-63, default parameters) reports a model
// optimal once its bound is within MIPGap = 1e-4 (relative) of the incumbent, so these get:
//   * a primal packing: the B&B incumbent, or for unsearched components the greedy packing by
//     (weight desc, column asc) - computed in parallel rounds, a clique joins when it is the
//     heaviest undecided clique on every one of its boxes (same result as the sequential
//     greedy) - then improving swaps (add a clique, drop the chosen cliques on its boxes)
//     claimed per box by gain, rounds until none improves;
//   * a dual bound: the Lagrangian relaxation of the box constraints, L(lam) = sum_r lam_r +
//     sum_c max(0, w_c - sum_{r in c} lam_r) >= OPT for every lam >= 0, lowered by projected
//     subgradient steps (per component, Polyak step towards the primal);
//   * RGC_ILP_GAP_OK when lbest - primal <= 1e-4 primal, else the packing with status
//     NODE_LIMIT / HEURISTIC.
constexpr uint8_t ST_UND = 0, ST_IN = 1, ST_OUT = 2, ST_NONE = 3;
constexpr int CS = 10;  // doubles per component record: lsum g2 lbest mu primal step stall flag
                        // repacked-primal (spare)

// Per-component sums of f64 terms over many columns / rows (the Lagrangian value and the
// packing values, slots 0, 4 and 8 of the record) are accumulated in fixed point, 2^-32
// units in an int64, so the result does not depend on the order of the atomics: the whole
// solve is deterministic (two runs give the same x).  Terms of the dual bound round up and
// terms of a packing value round down, so certified gaps stay valid (the slack is 2^-32 per
// term: < 2e-4 absolute over a 705k-clique micrograph, 1.5e-7 of its objective).
constexpr double FX_ONE = 4294967296.0;
__device__ __forceinline__ void fx_add_up(double* slot, double v) {
  atomicAdd(reinterpret_cast<unsigned long long*>(slot), (unsigned long long)(long long)ceil(v * FX_ONE));
}
__device__ __forceinline__ void fx_add_dn(double* slot, double v) {
  atomicAdd(reinterpret_cast<unsigned long long*>(slot), (unsigned long long)(long long)floor(v * FX_ONE));
}
__device__ __forceinline__ long long fx_raw(const double* slot) {
  return *reinterpret_cast<const long long*>(slot);
}
__device__ __forceinline__ double fx_get(const double* slot) { return (double)fx_raw(slot) / FX_ONE; }

__device__ __forceinline__ int64_t ilp_comp(const IlpArgs& A, int64_t c) {
  return A.comp_id[A.parent[c]];
}
__device__ __forceinline__ int64_t ilp_row_comp(const IlpArgs& A, int64_t r) {
  return A.rptr[r + 1] > A.rptr[r] ? ilp_comp(A, A.rcols[A.rptr[r]]) : -1;
}

// per component: what the branch and bound left unproven
__global__ __launch_bounds__(ILP_WG) void k_cert_flag(IlpArgs A) {
  const int64_t comp = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (comp >= A.n_comp) return;
  const int n = A.comp_n[comp];
  uint8_t f = 0;
  const uint8_t ex = n > 1 ? A.exact[A.members[A.comp_off[comp]]] : 1;
  if (n > ILP_BIG) f = 2;
  else if (ex == 0) f = 1;
  A.cert[comp] = f;
  if (f) atomicAdd(A.count + 1, 1u);   // flagged components (the host skips the rest when 0)
  double* cs = A.cs + comp * CS;
  cs[0] = 0.0; cs[1] = 0.0; cs[2] = INFINITY; cs[3] = 2.0; cs[4] = 0.0; cs[5] = 0.0; cs[6] = 0.0;
  cs[7] = 0.0; cs[8] = 0.0; cs[9] = 0.0;
}

// before the wave search: components of 65..ILP_BIG cliques get multipliers for the search's
// Lagrangian bound (cert 3: greedy primal, swaps, subgradient, like the certification below)
__global__ __launch_bounds__(ILP_WG) void k_cert_flag_pre(IlpArgs A) {
  const int64_t comp = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (comp >= A.n_comp) return;
  const int n = A.comp_n[comp];
  const uint8_t f = (n > ILP_SMALL && n <= ILP_BIG) ? 3 : 0;
  A.cert[comp] = f;
  if (f) atomicAdd(A.count + 1, 1u);
  double* cs = A.cs + comp * CS;
  cs[0] = 0.0; cs[1] = 0.0; cs[2] = INFINITY; cs[3] = 2.0; cs[4] = 0.0; cs[5] = 0.0; cs[6] = 0.0;
  cs[7] = 0.0; cs[8] = 0.0; cs[9] = 0.0;
}
// after the pre-search subgradient: the best multipliers (kept in rmax) become lam
__global__ __launch_bounds__(ILP_WG) void k_lr_take_best(IlpArgs A) {
  const int64_t r = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (r >= A.n_rows) return;
  const int64_t comp = ilp_row_comp(A, r);
  if (comp < 0 || A.cert[comp] == 0) return;
  A.lam[r] = reinterpret_cast<const double*>(A.rmax)[r];
}

// per column: priority key and state; chosen columns of node-limit components own their rows
__global__ __launch_bounds__(ILP_WG) void k_cert_cols(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c >= A.n_cols) return;
  const uint8_t f = A.cert[ilp_comp(A, c)];
  const double w = A.w[c];
  A.key[c] = ((uint64_t)__float_as_uint((float)fmax(w, 0.0)) << 32) | (uint32_t)~(uint32_t)c;
  uint8_t st = ST_NONE;
  if (f == 2 || f == 3) st = w > 0.0 ? ST_UND : ST_OUT;
  else if (f == 1) st = A.x[c] ? ST_IN : ST_OUT;
  A.st[c] = st;
  if (st == ST_IN)
    for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e) A.owner[A.row_idx[e]] = (int32_t)c;
}

__global__ __launch_bounds__(ILP_WG) void k_cert_rows_init(IlpArgs A) {
  const int64_t r = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (r >= A.n_rows) return;
  A.owner[r] = -1;
  A.rmax[r] = 0;
  A.grad[r] = 0.0;
  A.lam[r] = 0.0;
}

// greedy round: claims, winners, losers (the heaviest undecided clique on each of its boxes
// joins; cliques on a taken box leave; the rest reset their boxes' claims)
__global__ __launch_bounds__(ILP_WG) void k_gr_claim(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c >= A.n_cols || A.st[c] != ST_UND) return;
  const unsigned long long k = A.key[c];
  for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e)
    atomicMax(reinterpret_cast<unsigned long long*>(A.rmax + A.row_idx[e]), k);
}
__global__ __launch_bounds__(ILP_WG) void k_gr_win(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c >= A.n_cols || A.st[c] != ST_UND) return;
  bool win = true;
  for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e) win &= A.rmax[A.row_idx[e]] == A.key[c];
  if (!win) return;
  A.st[c] = ST_IN;
  for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e) A.owner[A.row_idx[e]] = (int32_t)c;
}
__global__ __launch_bounds__(ILP_WG) void k_gr_lose(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c >= A.n_cols || A.st[c] != ST_UND) return;
  bool hit = false;
  for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e) hit |= A.owner[A.row_idx[e]] >= 0;
  if (hit) {
    A.st[c] = ST_OUT;
    return;
  }
  for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e) A.rmax[A.row_idx[e]] = 0;
  atomicAdd(A.count, 1u);
}

// swap round: an unchosen clique whose weight exceeds the chosen cliques on its boxes claims
// its boxes and those cliques' boxes by gain; winners (all claims held) swap in
__device__ __forceinline__ int swap_victims(const IlpArgs& A, int64_t c, int32_t (&v)[8]) {
  int nv = 0;
  for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e) {
    const int32_t o = A.owner[A.row_idx[e]];
    if (o < 0) continue;
    bool seen = false;
    for (int i = 0; i < nv; ++i) seen |= v[i] == o;
    if (!seen) v[nv++] = o;
  }
  return nv;
}
__device__ __forceinline__ bool swap_gain(const IlpArgs& A, int64_t c, uint64_t* key) {
  int32_t v[8];
  const int nv = swap_victims(A, c, v);
  double lost = 0.0;
  for (int i = 0; i < nv; ++i) lost += A.w[v[i]];
  const double gain = A.w[c] - lost;
  if (!(gain > 1e-12 * A.w[c])) return false;
  *key = ((uint64_t)__float_as_uint((float)gain) << 32) | (uint32_t)~(uint32_t)c;
  return true;
}
template <int STEP>
__global__ __launch_bounds__(ILP_WG) void k_ls(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c >= A.n_cols || A.st[c] != ST_OUT) return;
  uint64_t key;
  if (!swap_gain(A, c, &key)) return;
  int32_t v[8];
  const int nv = swap_victims(A, c, v);
  auto each_row = [&](auto&& fn) {
    for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e) fn(A.row_idx[e]);
    for (int i = 0; i < nv; ++i)
      for (int64_t e = A.col_ptr[v[i]]; e < A.col_ptr[v[i] + 1]; ++e) fn(A.row_idx[e]);
  };
  if (STEP == 0) {          // claim
    each_row([&](int32_t r) { atomicMax(reinterpret_cast<unsigned long long*>(A.rmax + r), key); });
  } else if (STEP == 1) {   // winners: drop the victims (their boxes freed), mark the winner
    bool win = true;
    each_row([&](int32_t r) { win &= A.rmax[r] == key; });
    if (!win) return;
    for (int i = 0; i < nv; ++i) {
      A.st[v[i]] = ST_OUT;
      for (int64_t e = A.col_ptr[v[i]]; e < A.col_ptr[v[i] + 1]; ++e) A.owner[A.row_idx[e]] = -1;
    }
    A.st[c] = 4;   // (swapping in: takes its boxes in the next step)
    atomicAdd(A.count, 1u);
  }
}
__global__ __launch_bounds__(ILP_WG) void k_ls_take(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c >= A.n_cols) return;
  if (A.st[c] == 4) {
    A.st[c] = ST_IN;
    for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e) A.owner[A.row_idx[e]] = (int32_t)c;
  }
}
__global__ __launch_bounds__(ILP_WG) void k_ls_clear(IlpArgs A) {
  const int64_t r = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (r < A.n_rows) A.rmax[r] = 0;
}

// primal value per component and the initial multipliers lam_r = max_{c on r} w_c / |c|
// (every reduced cost <= 0: L(lam0) = sum_r lam_r)
__global__ __launch_bounds__(ILP_WG) void k_lr_init(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c >= A.n_cols || A.st[c] == ST_NONE) return;
  const int64_t comp = ilp_comp(A, c);
  if (A.st[c] == ST_IN) fx_add_dn(A.cs + comp * CS + 4, A.w[c]);
  const double share = fmax(A.w[c], 0.0) / (double)(A.col_ptr[c + 1] - A.col_ptr[c]);
  for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e)
    atomicMax(reinterpret_cast<unsigned long long*>(A.lam + A.row_idx[e]),
              (unsigned long long)__double_as_longlong(share));   // (non-negative doubles)
}
// one subgradient iteration: reduced costs -> cover counts -> L, |g|^2 -> step -> lam
__global__ __launch_bounds__(ILP_WG) void k_lr_cols(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c >= A.n_cols || A.st[c] == ST_NONE) return;
  double rc = A.w[c];
  for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e) rc -= A.lam[A.row_idx[e]];
  if (!(rc > 0.0)) return;
  fx_add_up(A.cs + ilp_comp(A, c) * CS + 0, rc);
  for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e) atomicAdd(A.grad + A.row_idx[e], 1.0);
}
__global__ __launch_bounds__(ILP_WG) void k_lr_rows(IlpArgs A) {
  const int64_t r = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (r >= A.n_rows) return;
  const int64_t comp = ilp_row_comp(A, r);
  if (comp < 0 || A.cert[comp] == 0) return;
  double g = 1.0 - A.grad[r];           // d L / d lam_r
  if (A.lam[r] <= 0.0 && g > 0.0) g = 0.0;   // projected: lam stays at 0
  A.grad[r] = g;
  double* cs = A.cs + comp * CS;
  fx_add_up(cs + 0, A.lam[r]);
  atomicAdd(cs + 1, g * g);   // (integers: exact in any order)
}
__global__ __launch_bounds__(ILP_WG) void k_lr_step(IlpArgs A) {
  const int64_t comp = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (comp >= A.n_comp || A.cert[comp] == 0) return;
  double* cs = A.cs + comp * CS;
  const double L = fx_get(cs + 0), g2 = cs[1], P = fx_get(cs + 4);
  // cs[7]: 1 = this lam is the best so far (rows keep a copy), 2 = restart from that copy
  cs[7] = 0.0;
  if (!(L >= cs[2] - 1e-9 * fabs(cs[2]))) {   // (first iteration: cs[2] = inf)
    cs[2] = fmin(cs[2], L);
    cs[6] = 0.0;
    cs[7] = 1.0;
  } else {
    cs[6] += 1.0;
  }
  if (cs[6] >= 40.0) {          // no progress: shrink the step, restart from the best lam
    cs[3] *= 0.7;
    cs[6] = 0.0;
    cs[7] = 2.0;
  }
  cs[5] = g2 > 0.0 ? cs[3] * fmax(L - P, 0.0) / g2 : 0.0;
  cs[0] = 0.0;
  cs[1] = 0.0;
}
__global__ __launch_bounds__(ILP_WG) void k_lr_lam(IlpArgs A) {
  const int64_t r = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (r >= A.n_rows) return;
  const int64_t comp = ilp_row_comp(A, r);
  if (comp < 0 || A.cert[comp] == 0) return;
  const double* cs = A.cs + comp * CS;
  // the best lam lives in rmax (the claims are dead by now) as double bits
  double* best = reinterpret_cast<double*>(A.rmax);
  if (cs[7] == 1.0) best[r] = A.lam[r];
  if (cs[7] == 2.0) A.lam[r] = best[r];
  else A.lam[r] = fmax(0.0, A.lam[r] - cs[5] * A.grad[r]);
  A.grad[r] = 0.0;
}
// Lagrangian repack (certification): the LP of these models is nearly integral (a full C5
// micrograph: 229 fractional of 705,588 columns), and with multipliers near the LP duals the
// columns of positive reduced cost w_c - sum_r lam_r are nearly its support.  So the packing
// is rebuilt greedily by reduced cost (heaviest reduced cost first), improved by the same
// swaps, and kept per component when it beats the weight-greedy one.
__device__ __forceinline__ uint32_t sortable_f32(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
// rows of flagged components: lam = the best multipliers (rmax), claims and owners cleared
__global__ __launch_bounds__(ILP_WG) void k_rp_rows(IlpArgs A) {
  const int64_t r = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (r >= A.n_rows) return;
  const int64_t comp = ilp_row_comp(A, r);
  if (comp < 0 || A.cert[comp] == 0) return;
  A.lam[r] = reinterpret_cast<const double*>(A.rmax)[r];
  A.rmax[r] = 0;
  A.owner[r] = -1;
}
// columns: save the packing, key by reduced cost, undecided again
__global__ __launch_bounds__(ILP_WG) void k_rp_cols(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c >= A.n_cols || A.st[c] == ST_NONE) return;
  if (A.cert[ilp_comp(A, c)] == 0) return;
  A.st_save[c] = A.st[c];
  const double w = A.w[c];
  double rc = w;
  for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e) rc -= A.lam[A.row_idx[e]];
  A.key[c] = ((uint64_t)sortable_f32((float)rc) << 32) | (uint32_t)~(uint32_t)c;
  A.st[c] = w > 0.0 ? ST_UND : ST_OUT;
}
__global__ __launch_bounds__(ILP_WG) void k_rp_primal(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c >= A.n_cols || A.st[c] != ST_IN) return;
  const int64_t comp = ilp_comp(A, c);
  if (A.cert[comp] != 0) fx_add_dn(A.cs + comp * CS + 8, A.w[c]);
}
// keep the better packing per component (ties: the earlier one)
__global__ __launch_bounds__(ILP_WG) void k_rp_pick(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c >= A.n_cols || A.st[c] == ST_NONE) return;
  const int64_t comp = ilp_comp(A, c);
  if (A.cert[comp] == 0) return;
  const double* cs = A.cs + comp * CS;
  if (!(fx_raw(cs + 8) > fx_raw(cs + 4))) A.st[c] = A.st_save[c];
}
__global__ __launch_bounds__(ILP_WG) void k_rp_comps(IlpArgs A) {
  const int64_t comp = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (comp >= A.n_comp || A.cert[comp] == 0) return;
  double* cs = A.cs + comp * CS;
  if (fx_raw(cs + 8) > fx_raw(cs + 4)) cs[4] = cs[8];   // (fixed-point bits)
  cs[8] = 0.0;
}
// rows: the best multipliers back where the subgradient's restarts read them
__global__ __launch_bounds__(ILP_WG) void k_rp_best(IlpArgs A) {
  const int64_t r = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (r >= A.n_rows) return;
  const int64_t comp = ilp_row_comp(A, r);
  if (comp < 0 || A.cert[comp] == 0) return;
  reinterpret_cast<double*>(A.rmax)[r] = A.lam[r];
  A.owner[r] = -1;
}

// x and the component statuses
__global__ __launch_bounds__(ILP_WG) void k_cert_final(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c >= A.n_cols || A.st[c] == ST_NONE) return;
  const int64_t comp = ilp_comp(A, c);
  const double* cs = A.cs + comp * CS;
  A.x[c] = A.st[c] == ST_IN ? 1 : 0;
  const double P = fx_get(cs + 4), Lb = cs[2];
  const bool ok = Lb - P <= 1e-4 * fabs(P);
  A.exact[c] = ok ? RGC_ILP_GAP_OK : (A.cert[comp] == 2 ? RGC_ILP_HEURISTIC : RGC_ILP_NODE_LIMIT);
  // the component's absolute gap, once (at its first column), for micrograph-level MIPGap
  if (A.gap && c == A.members[A.comp_off[comp]]) A.gap[c] = fmax(Lb - P, 0.0);
}
// (before k_lr_init: the primal value is recounted from the final packing)
__global__ __launch_bounds__(ILP_WG) void k_cert_reset_primal(IlpArgs A) {
  const int64_t comp = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (comp < A.n_comp) A.cs[comp * CS + 4] = 0.0;
}

// ------------------------------------------------------------------ reduced-cost fixing
// After the certification, a flagged component has a packing P and multipliers lam (the best
// ones, in rmax) with dual bound L(lam) = sum_r lam_r + sum_c max(0, rc_c), rc_c = w_c -
// sum_{r in c} lam_r.  Fixing x_c = 1 in the Lagrangian gives: every packing that contains
// column c is worth at most L + min(0, rc_c).  So a column with rc_c <= P - L cannot be part
// of a packing better than P, and the component's optimum is max(P, optimum over the kept
// columns rc_c > P - L).  These models are nearly integral with few rows per component
// (dense clusters: 17-54 boxes, up to 79k cliques, in a crowded C5 micrograph), and the
// columns within the bound's gap of zero reduced cost are a few hundred: that restricted
// problem is small enough for the exact search (rgc_ilp_solve runs it as a second pass).
// L and P are recomputed here in fixed point (L rounded up, P down), so the kept set is a
// superset of what exact arithmetic would keep; the packing's own columns are always kept.
__global__ __launch_bounds__(ILP_WG) void k_fs_init(IlpArgs A) {
  const int64_t comp = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (comp >= A.n_comp) return;
  A.fs[2 * comp] = 0.0;
  A.fs[2 * comp + 1] = 0.0;
  A.fs_cnt[comp] = 0;
}
__global__ __launch_bounds__(ILP_WG) void k_fs_rows(IlpArgs A) {
  const int64_t r = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (r >= A.n_rows) return;
  const int64_t comp = ilp_row_comp(A, r);
  if (comp < 0 || A.cert[comp] == 0) return;
  fx_add_up(A.fs + 2 * comp, reinterpret_cast<const double*>(A.rmax)[r]);
}
__device__ __forceinline__ double fs_rc(const IlpArgs& A, int64_t c) {
  const double* lam = reinterpret_cast<const double*>(A.rmax);
  double rc = A.w[c];
  for (int64_t e = A.col_ptr[c]; e < A.col_ptr[c + 1]; ++e) rc -= lam[A.row_idx[e]];
  return rc;
}
__global__ __launch_bounds__(ILP_WG) void k_fs_cols(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c >= A.n_cols) return;
  const int64_t comp = ilp_comp(A, c);
  A.loc[c] = (int32_t)comp;   // (the solvers' local numbering is dead: the host maps columns)
  A.fs_keep[c] = 0;
  if (A.cert[comp] == 0) return;
  const double rc = fs_rc(A, c);
  if (rc > 0.0) fx_add_up(A.fs + 2 * comp, rc);
  if (A.st[c] == ST_IN) fx_add_dn(A.fs + 2 * comp + 1, A.w[c]);
}
__global__ __launch_bounds__(ILP_WG) void k_fs_keep(IlpArgs A) {
  const int64_t c = (int64_t)blockIdx.x * ILP_WG + threadIdx.x;
  if (c >= A.n_cols) return;
  const int64_t comp = A.loc[c];
  if (A.cert[comp] == 0) return;
  const double L = fx_get(A.fs + 2 * comp), P = fx_get(A.fs + 2 * comp + 1);
  // (a relative 1e-12 of slack for the f64 rounding of rc)
  const bool keep = A.st[c] == ST_IN || fs_rc(A, c) > P - L - 1e-12 * (1.0 + fabs(L));
  if (!keep) return;
  A.fs_keep[c] = 1;
  atomicAdd(A.fs_cnt + comp, 1u);
}

void launch_ilp_cert(hipStream_t stream, int phase, const IlpArgs& A) {
  const int64_t nbc = (A.n_cols + ILP_WG - 1) / ILP_WG;
  const int64_t nbr = (A.n_rows + ILP_WG - 1) / ILP_WG;
  const int64_t nbk = (A.n_comp + ILP_WG - 1) / ILP_WG;
  if (!nbc) return;
#define RGC_L(kern, nb) hipLaunchKernelGGL(kern, dim3(nb), dim3(ILP_WG), 0, stream, A)
  switch (phase) {
    case 0:
      RGC_L(k_cert_flag, nbk);
      if (nbr) RGC_L(k_cert_rows_init, nbr);
      RGC_L(k_cert_cols, nbc);
      break;
    case 1:
      RGC_L(k_gr_claim, nbc);
      RGC_L(k_gr_win, nbc);
      RGC_L(k_gr_lose, nbc);
      break;
    case 2:
      RGC_L((k_ls<0>), nbc);
      RGC_L((k_ls<1>), nbc);
      RGC_L(k_ls_take, nbc);
      if (nbr) RGC_L(k_ls_clear, nbr);
      break;
    case 3:
      RGC_L(k_cert_reset_primal, nbk);
      if (nbr) RGC_L(k_cert_rows_init, nbr);   // (owner no longer needed)
      RGC_L(k_lr_init, nbc);
      break;
    case 4:
      RGC_L(k_lr_cols, nbc);
      if (nbr) RGC_L(k_lr_rows, nbr);
      RGC_L(k_lr_step, nbk);
      if (nbr) RGC_L(k_lr_lam, nbr);
      break;
    case 5:
      RGC_L(k_cert_final, nbc);
      break;
    case 6:   // pre-search setup (cert 3) = phase 0 with k_cert_flag_pre
      RGC_L(k_cert_flag_pre, nbk);
      if (nbr) RGC_L(k_cert_rows_init, nbr);
      RGC_L(k_cert_cols, nbc);
      break;
    case 7:
      if (nbr) RGC_L(k_lr_take_best, nbr);
      break;
    case 8:   // Lagrangian repack: setup (then greedy rounds, swap rounds, phase 9)
      if (nbr) RGC_L(k_rp_rows, nbr);
      RGC_L(k_rp_cols, nbc);
      break;
    case 9:   // repack: value, pick per component, multipliers restored
      RGC_L(k_rp_primal, nbc);
      RGC_L(k_rp_pick, nbc);
      RGC_L(k_rp_comps, nbk);
      if (nbr) RGC_L(k_rp_best, nbr);
      break;
    case 10:  // reduced-cost fixing: dual bound and packing value, then the kept columns
      RGC_L(k_fs_init, nbk);
      if (nbr) RGC_L(k_fs_rows, nbr);
      RGC_L(k_fs_cols, nbc);
      RGC_L(k_fs_keep, nbc);
      break;
  }
#undef RGC_L
}

int ilp_small_max() { return ILP_SMALL; }
int ilp_big_max() { return ILP_BIG; }

void launch_ilp(hipStream_t stream, int phase, const IlpArgs& A, int n_big, int n_waves) {
  const int64_t nbc = (A.n_cols + ILP_WG - 1) / ILP_WG;
  const int64_t nbk = (A.n_comp + ILP_WG - 1) / ILP_WG;
  switch (phase) {
    case 0:
      if (A.n_cols > 0 || A.n_rows > 0) {
        const int64_t nbi = ((A.n_cols > A.n_rows ? A.n_cols : A.n_rows) + ILP_WG - 1) / ILP_WG;
        hipLaunchKernelGGL(k_ilp_init, dim3(nbi), dim3(ILP_WG), 0, stream, A);
      }
      if (nbc) {
        hipLaunchKernelGGL(k_ilp_rep, dim3(nbc), dim3(ILP_WG), 0, stream, A);
        hipLaunchKernelGGL(k_ilp_union, dim3(nbc), dim3(ILP_WG), 0, stream, A);
        hipLaunchKernelGGL(k_ilp_root, dim3(nbc), dim3(ILP_WG), 0, stream, A);
      }
      break;
    case 1:
      if (nbc) hipLaunchKernelGGL(k_ilp_csize, dim3(nbc), dim3(ILP_WG), 0, stream, A);
      break;
    case 2:
      if (nbc) hipLaunchKernelGGL(k_ilp_fill, dim3(nbc), dim3(ILP_WG), 0, stream, A);
      break;
    case 3:
      if (nbk) {
        hipLaunchKernelGGL(k_ilp_small, dim3(nbk), dim3(ILP_WG), 0, stream, A);
        hipLaunchKernelGGL(k_ilp_biglist, dim3(nbk), dim3(ILP_WG), 0, stream, A);
      }
      break;
    case 4:
      if (n_big > 0) hipLaunchKernelGGL(k_ilp_wave, dim3(n_waves), dim3(64), 0, stream, A, n_big);
      break;
  }
}

}  // namespace rgc
