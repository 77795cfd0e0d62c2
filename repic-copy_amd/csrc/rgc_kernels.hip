// rgc_kernels.hip — gfx950 kernels for the batched `get_cliques` hot path.
//
// One launch of each kernel covers a whole batch of micrographs (SoA/CSR layout in HBM,
// see DESIGN.md §3).  Reference functions replaced (reference repic/commands/get_cliques.py):
//   k1_bin            spatial grid (cell >= box_size) so the O(n_a*n_b) pair loop (:59-69)
//                     becomes a 3x3 cell stencil
//   k2_pairs<FILL>    calc_jaccard (:40-46) + |dx| <= B prefilter + JI > 0.3 (:64-65,:138),
//                     two-phase count -> scan -> fill; forward CSR sorted by target box
//   k4_*              nx.connected_components stats (:145-149), --get_cc (:151-156)
//   k5_cliques<K,..>  find_cliques (:49-56) for micrographs with a root of more than RB_W
//                     forward neighbours (the level kernels of rgc_cliques.hip take the
//                     rest; the ILP epilogue is k5_epilogue there)
//   k7_*              row index v.index() (:164,:193) as a per-micrograph rank by
//                     (x, y, id): x-bucket count -> scan -> scatter -> rank
//
// Floating point: every JI / degree / median operation keeps the reference's f64 operation
// order; contraction into FMA is forbidden (the pragma below + -ffp-contract=off).
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "rgc_device.h"
#include "rgc_kernels.h"

#include <algorithm>
#include <atomic>

namespace rgc {

// ----------------------------------------------------------------------------- K1 bin
// Per-picker grids (the fused kernel's P1 restated for whole-GPU kernels): every picker gets
// its own gx x gy grid of cells >= 1.08 B wide and >= 0.54 B tall over the micrograph's
// bounding box, keys picker * ncell + (cx * gy + cy) (x-major), the non-finite boxes in key
// nkey = K * ncell.  JI > 0.3 needs I > (6/13) B^2, i.e. |dx|, |dy| < (7/13) B = 0.5385 B, so
// an edge partner lies within 0.4986 columns: in the box's own column or the neighbouring
// one on the side of the box's half of its column, and within one row: a 2 x 3 stencil = two
// contiguous position ranges per higher picker's grid (forward edges only).  Keys and the
// half test use the same f64 product (x - minx) * inv_cell for every box, so the plan is
// consistent (0.0014 columns of slack against rounding).
__device__ __forceinline__ int bin_key(const MgGrid& G, int p, double x, double y) {
  if (G.ncell == 0 || !isfinite(x) || !isfinite(y)) return G.nkey;
  const int cx = (int)fmin(floor((x - G.minx) * G.inv_cell), (double)(G.gx - 1));
  const int cy = (int)fmin(floor((y - G.miny) * G.inv_celly), (double)(G.gy - 1));
  return p * G.ncell + cx * G.gy + cy;
}

// One workgroup per micrograph: bounding box, grid plan, integer-layout flag (every finite
// coordinate an integer below 2^23 and an integer 1 <= B <= 2896: P2's exact f32 test),
// LDS counting sort of the boxes by key.  cell_start[cell_off[m] + key] = first sorted
// position (local to the micrograph) of each key; entry nkey + 1 = n.
template <bool WIDE>
__global__ __launch_bounds__(1024) void k1_bin(int k, double B, const int32_t* __restrict__ box_off,
                                               const int32_t* __restrict__ cell_off,
                                               const double* __restrict__ x,
                                               const double* __restrict__ y, MgGrid* grid,
                                               int32_t* cell_start, double* sx, double* sy,
                                               int32_t* sbox, uint8_t* spick, int32_t* smg,
                                               int32_t* bmg, uint8_t* bpick) {
  constexpr int BT = 1024, BW = BT / 64;
  extern __shared__ __attribute__((aligned(16))) uint32_t cntw[];   // packed counters
  __shared__ double redd[BW];
  __shared__ int64_t red64[BW];
  __shared__ int32_t poff[MAX_K + 1];
  __shared__ int notint;
  __shared__ MgGrid G;
  const int m = blockIdx.x;
  const int b0 = box_off[m * k], b1 = box_off[m * k + k], n = b1 - b0;
  if ((int)threadIdx.x <= k) poff[threadIdx.x] = box_off[m * k + threadIdx.x] - b0;
  if (threadIdx.x == 0) notint = !(B >= 1.0 && B <= 2896.0 && B == floor(B));
  double mnx = INFINITY, mny = INFINITY, mxx = -INFINITY, mxy = -INFINITY;
  bool ni = false;
  for (int i = threadIdx.x; i < n; i += BT) {
    const double xv = x[b0 + i], yv = y[b0 + i];
    if (isfinite(xv) && isfinite(yv)) {
      mnx = fmin(mnx, xv); mxx = fmax(mxx, xv);
      mny = fmin(mny, yv); mxy = fmax(mxy, yv);
      ni |= xv != rint(xv) || yv != rint(yv) || fabs(xv) >= 0x1p23 || fabs(yv) >= 0x1p23;
    }
  }
  __syncthreads();
  if (ni) notint = 1;
  mnx = block_min<BT>(mnx, redd);
  mny = block_min<BT>(mny, redd);
  mxx = block_max<BT>(mxx, redd);
  mxy = block_max<BT>(mxy, redd);
  const int budget = bin_budget(n, WIDE);
  if (threadIdx.x == 0) {
    MgGrid g;
    g.minx = mnx; g.miny = mny; g.cell = INFINITY; g.inv_cell = 0.0; g.inv_celly = 0.0;
    g.gx = 0; g.gy = 0; g.ncell = 0; g.nkey = 0; g.flags = notint ? 0 : 1;
    if (mnx <= mxx && B > 0.0) {
      const double ex = mxx - mnx, ey = mxy - mny;
      if (!(ex < 0x1p40 && ey < 0x1p40)) {
        // beyond the exactness range of the stencil argument: one cell per picker, all pairs
        g.gx = 1; g.gy = 1;
      } else {
        // row height h, column width 2 h (>= 1.08 B x 0.54 B), k gx gy <= budget
        const int per = budget / k;
        double h = fmax(0.54 * B * (1.0 + 1e-9), fmax(sqrt(0.5 * ex * ey / per),
                                                     fmax(0.5 * ex, ey) / per));
        for (;;) {
          const double fx = floor(ex / (2.0 * h)) + 1.0, fy = floor(ey / h) + 1.0;
          if (fx * fy <= (double)per) { g.gx = (int)fx; g.gy = (int)fy; break; }
          h *= 1.0625;
        }
        g.cell = 2.0 * h;
        g.inv_cell = 1.0 / (2.0 * h);
        g.inv_celly = 1.0 / h;
        if (g.inv_cell * (1.08 * B) > 1.0) g.inv_cell = 1.0 / (1.08 * B);
        if (g.inv_celly * (0.54 * B) > 1.0) g.inv_celly = 1.0 / (0.54 * B);
      }
      g.ncell = g.gx * g.gy;
      g.nkey = k * g.ncell;
    }
    G = g;
    grid[m] = g;
  }
  __syncthreads();
  const int nk = G.nkey;   // keys 0..nk (nk: non-finite boxes)
  const int nwords = WIDE ? nk + 2 : (nk + 3) / 2;
  for (int c = threadIdx.x; c < nwords; c += BT) cntw[c] = 0;
  __syncthreads();
  auto picker = [&](int i) {
    int p = 0;
    for (int q = 1; q < k; ++q) p += i >= poff[q] ? 1 : 0;
    return p;
  };
  for (int i = threadIdx.x; i < n; i += BT) {
    const int q = bin_key(G, picker(i), x[b0 + i], y[b0 + i]);
    if (WIDE) atomicAdd(&cntw[q], 1u);
    else atomicAdd(&cntw[q >> 1], 1u << (16 * (q & 1)));
  }
  __syncthreads();
  // exclusive scan of the nk + 1 counters into cell starts (LDS and cell_start)
  auto cnt_at = [&](int c) -> uint32_t {
    return WIDE ? cntw[c] : (cntw[c >> 1] >> (16 * (c & 1))) & 0xFFFFu;
  };
  const int per = (nk + 1 + BT - 1) / BT;
  const int c0 = min((int)threadIdx.x * per, nk + 1), c1 = min(c0 + per, nk + 1);
  int64_t s = 0;
  for (int c = c0; c < c1; ++c) s += cnt_at(c);
  int64_t tot;
  int64_t pre = block_excl_scan<BT>(s, red64, &tot);
  int32_t* cs = cell_start + cell_off[m];
  for (int c = c0; c < c1; ++c) cs[c] = (int)pre, pre += cnt_at(c);
  if (threadIdx.x == 0) cs[nk + 1] = n;
  __syncthreads();   // every thread read its counters before they become cursors
  // cursors = cell starts, in the counters' representation (u16 pairs: n <= 65535, so a
  // cursor never carries into its neighbour)
  for (int c = threadIdx.x; c < nwords; c += BT) {
    if (WIDE) {
      cntw[c] = c <= nk ? (uint32_t)cs[c] : 0u;
    } else {
      const int c0w = 2 * c, c1w = 2 * c + 1;
      cntw[c] = (c0w <= nk ? (uint32_t)cs[c0w] : 0u) | ((c1w <= nk ? (uint32_t)cs[c1w] : 0u) << 16);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += BT) {
    const int g = b0 + i;
    const double xv = x[g], yv = y[g];
    const int p = picker(i);
    const int q = bin_key(G, p, xv, yv);
    int slot;
    if (WIDE) {
      slot = (int)atomicAdd(&cntw[q], 1u);
    } else {
      const int sh = 16 * (q & 1);
      slot = (int)((atomicAdd(&cntw[q >> 1], 1u << sh) >> sh) & 0xFFFFu);
    }
    const int pos = b0 + slot;
    sx[pos] = xv; sy[pos] = yv; sbox[pos] = g; spick[pos] = (uint8_t)p; smg[pos] = m;
    bmg[g] = m; bpick[g] = (uint8_t)p;
  }
}

// ----------------------------------------------------------------------------- K2 pairs
// One thread per box (sorted position, so neighbouring threads share stencil cells in L1/L2):
// the 2 x 3 stencil (see K1) in the grid of every HIGHER picker.  Integer micrographs decide
// JI > 0.3 exactly on f32 (overlaps B - |dx| and their product < 2^24 are exact: I >
// floor(6 B^2 / 13), the fused kernel's P2 test); others test I > (6/13) B^2 in f64 and
// evaluate the reference quotient (get_cliques.py:40-46) only inside a 2^-40 relative band of
// the threshold.  COUNT: forward-edge count per box.  FILL: write the targets (and, for the
// RGC_F_EDGES hook only, the reference JI) into the box's CSR slot, sorted by target box index
// (picker-major, file order) for the clique intersections.
template <bool FILL>
__global__ __launch_bounds__(WG) void k2_pairs(int N, int k, double B, double two_b2,
                                               const int32_t* __restrict__ box_off,
                                               const int32_t* __restrict__ cell_off,
                                               const MgGrid* __restrict__ grid,
                                               const int32_t* __restrict__ cell_start,
                                               const double* __restrict__ sx,
                                               const double* __restrict__ sy,
                                               const int32_t* __restrict__ sbox,
                                               const uint8_t* __restrict__ spick,
                                               const int32_t* __restrict__ smg, int32_t* fwd_cnt,
                                               const int64_t* __restrict__ fwd_off,
                                               int32_t* e_dst, double* e_ji) {
  const int t = blockIdx.x * WG + threadIdx.x;
  if (t >= N) return;
  const int m = smg[t];
  const MgGrid G = grid[m];
  const double xa = sx[t], ya = sy[t];
  const int p = spick[t];
  const int g = sbox[t];
  int cnt = 0;
  int64_t base = 0;
  if (FILL) base = fwd_off[g];
  // fill: each higher picker's targets (a segment of the sorted list: box indices are
  // picker-major) collect in registers, up to FILL_REGS of them, and are sorted there by a
  // compare-exchange network (an insertion sort through global memory costs a dependent L2
  // round trip per shift; C5's picker-0 boxes have ~7-20 targets over 7 pickers, one to three
  // per picker); a longer segment, and the RGC_F_EDGES dump with its JIs, go through e_dst
  constexpr int FILL_REGS = 8;
  const bool reg = FILL && e_ji == nullptr;
  const int key = bin_key(G, p, xa, ya);
  if (key < G.nkey && p + 1 < k) {
    const int cell = key - p * G.ncell;
    const int cx = cell / G.gy, cy = cell - (cell / G.gy) * G.gy;
    const double u = (xa - G.minx) * G.inv_cell;
    const int sc = cx - ((u - (double)cx) < 0.5 ? 1 : 0);   // stencil columns sc, sc + 1
    const int y0 = max(cy - 1, 0), y1 = min(cy + 1, G.gy - 1);
    const int b0 = box_off[m * k];
    const int32_t* cs = cell_start + cell_off[m];
    const bool intl = (G.flags & 1) != 0;
    const float Bf = (float)B, Tf = (float)((6 * (int64_t)B * (int64_t)B) / 13);
    const float axf = (float)xa, ayf = (float)ya;
    const double t_star = 0.6 * B * B / 1.3;
    const double i_lo = t_star * (1.0 - 0x1p-40), i_hi = t_star * (1.0 + 0x1p-40);
    for (int q = p + 1; q < k; ++q) {
      int rk[FILL_REGS];
#pragma unroll
      for (int i = 0; i < FILL_REGS; ++i) rk[i] = INT32_MAX;
      const int64_t sb = base + cnt;   // (fill) this picker's segment
      int cq = 0;
      for (int d = 0; d <= 1; ++d) {
        const int col = sc + d;
        if (col < 0 || col >= G.gx) continue;
        const int kb = q * G.ncell + col * G.gy;
        const int lo = b0 + cs[kb + y0], hi = b0 + cs[kb + y1 + 1];
        for (int v = lo; v < hi; ++v) {
          const double xb = sx[v], yb = sy[v];
          bool e;
          if (intl) {
            const float xo = fmaxf(Bf - fabsf(axf - (float)xb), 0.0f);
            const float yo = fmaxf(Bf - fabsf(ayf - (float)yb), 0.0f);
            e = xo * yo > Tf;
          } else {
            const double xo = fmax((fmin(xa, xb) + B) - fmax(xa, xb), 0.0);
            const double yo = fmax((fmin(ya, yb) + B) - fmax(ya, yb), 0.0);
            const double inter = xo * yo;
            e = inter > i_hi;
            if (!e && inter >= i_lo) e = inter / (two_b2 - inter) > 0.3;   // reference quotient
          }
          if (e) {
            if (FILL) {
              if (reg) {   // a register shift chain; more: spill in arrival order, write through
                if (cq == FILL_REGS) {
#pragma unroll
                  for (int i = 0; i < FILL_REGS; ++i) e_dst[sb + i] = rk[FILL_REGS - 1 - i];
                }
                if (cq < FILL_REGS) {
#pragma unroll
                  for (int i = FILL_REGS - 1; i > 0; --i) rk[i] = rk[i - 1];
                  rk[0] = sbox[v];
                } else {
                  e_dst[sb + cq] = sbox[v];
                }
              } else {
                e_dst[base + cnt] = sbox[v];
                if (e_ji) e_ji[base + cnt] = jaccard(xa, ya, xb, yb, B, two_b2);
              }
            }
            ++cnt;
            ++cq;
          }
        }
      }
      if (reg && cq > 0) {
        if (cq <= FILL_REGS) {
          cmpnet_apply<FILL_REGS, false>(rk);   // ascending; unused slots hold INT32_MAX
#pragma unroll
          for (int i = 0; i < FILL_REGS; ++i)
            if (i < cq) e_dst[sb + i] = rk[i];
        } else {
          for (int i = 1; i < cq; ++i) {   // (rare) insertion sort of the segment
            const int kd = e_dst[sb + i];
            int j = i - 1;
            while (j >= 0 && e_dst[sb + j] > kd) {
              e_dst[sb + j + 1] = e_dst[sb + j];
              --j;
            }
            e_dst[sb + j + 1] = kd;
          }
        }
      }
    }
  }
  if (!FILL) {
    fwd_cnt[g] = cnt;
  } else if (!reg) {
    // insertion sort by target box (each picker's segment arrives in cell order)
    for (int i = 1; i < cnt; ++i) {
      const int kd = e_dst[base + i];
      const double kj = e_ji[base + i];
      int j = i - 1;
      while (j >= 0 && e_dst[base + j] > kd) {
        e_dst[base + j + 1] = e_dst[base + j];
        e_ji[base + j + 1] = e_ji[base + j];
        --j;
      }
      e_dst[base + j + 1] = kd;
      e_ji[base + j + 1] = kj;
    }
  }
}

// ----------------------------------------------------------------------------- scan
// Exclusive scan of int32 counts into int64 offsets (out[n] = total) in a single pass
// (decoupled look-back), reading the counts once and writing the offsets once.  Tiles of
// ONE_TILE counts are claimed in order on a counter (a tile's predecessors are then already
// running or done, whatever the dispatch order); each tile publishes its aggregate, looks back
// over its predecessors' published states (one wave, 64 states per step) for the exclusive
// prefix, then publishes its inclusive prefix.  A tile state is one 64-bit word: flag (2 bits:
// 1 aggregate, 2 inclusive prefix), launch epoch (22 bits: states of earlier launches read as
// unpublished, so the array needs no clearing) and value (40 bits).  The launch's last claim
// zeroes the counter for the next launch.  Counter and states live in the caller's tile buffer:
// word 0 the counter (zero when the buffer is new), states from word 1.
constexpr int ONE_PER = 16;
constexpr int ONE_TILE = WG * ONE_PER;
constexpr uint64_t ST_AGG = 1ull << 62, ST_INC = 2ull << 62;
constexpr uint64_t ST_VAL = (1ull << 40) - 1;

__device__ __forceinline__ uint64_t ep_mask() { return ((1ull << 22) - 1) << 40; }
__device__ __forceinline__ uint64_t st_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_store(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(WG) void scan_onepass(int64_t n, const int32_t* __restrict__ in,
                                                   int64_t* __restrict__ out, int64_t* total,
                                                   uint64_t* buf, uint32_t epoch,
                                                   int32_t* bucket, int bq) {
  __shared__ int64_t red[NW];
  __shared__ int64_t s_pre;
  __shared__ uint32_t s_tile;
  uint32_t* ctr = reinterpret_cast<uint32_t*>(buf);
  uint64_t* state = buf + 1;
  const uint64_t ep = (uint64_t)epoch << 40;
  const int ntiles = (int)gridDim.x;
  if (threadIdx.x == 0) {
    int vz;
    asm volatile("v_mov_b32 %0, 0" : "=v"(vz));   // (keeps the atomic optimizer off it)
    const uint32_t t = atomicAdd(ctr + vz, 1u);
    if (t == (uint32_t)ntiles - 1u) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_tile = t;
  }
  __syncthreads();
  const int tile = (int)s_tile;
  const int64_t t0 = (int64_t)tile * ONE_TILE + (int64_t)threadIdx.x * ONE_PER;
  int32_t v[ONE_PER];
  const bool vec = ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) == 0;
  if (vec && t0 + ONE_PER <= n) {
    const int4* q = reinterpret_cast<const int4*>(in + t0);
#pragma unroll
    for (int i = 0; i < ONE_PER / 4; ++i) {
      const int4 w = q[i];
      v[4 * i] = w.x; v[4 * i + 1] = w.y; v[4 * i + 2] = w.z; v[4 * i + 3] = w.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < ONE_PER; ++i) v[i] = t0 + i < n ? in[t0 + i] : 0;
  }
  int64_t s = 0;
#pragma unroll
  for (int i = 0; i < ONE_PER; ++i) s += v[i];
  int64_t agg;
  int64_t pre = block_excl_scan(s, red, &agg);
  if (threadIdx.x < 64) {   // wave 0: publish, look back, publish the inclusive prefix
    const int lane = threadIdx.x;
    if (lane == 0) st_store(state + tile, (tile == 0 ? ST_INC : ST_AGG) | ep | (uint64_t)agg);
    int64_t excl = 0;
    int j = tile - 1;   // the highest predecessor not yet folded in
    bool done = j < 0;
    for (int guard = 0; !done && guard < (1 << 24); ++guard) {
      const int idx = j - lane;
      uint64_t w = idx >= 0 ? st_load(state + idx) : (ST_INC | ep);   // (before tile 0: 0)
      const bool ready = (w & ep_mask()) == ep && (w >> 62) != 0;
      if (__ballot(!ready)) continue;   // some state of this window is not published yet
      const uint64_t inc = __ballot((w >> 62) == 2);
      // lanes up to and including the first inclusive one (lowest lane = highest tile)
      const int first = inc ? __builtin_ctzll(inc) : 64;
      int64_t val = (lane <= first && idx >= 0) ? (int64_t)(w & ST_VAL) : 0;
      for (int o = 32; o > 0; o >>= 1) val += __shfl_xor(val, o, 64);
      excl += val;
      j -= 64;
      done = inc != 0 || j < 0;
    }
    if (lane == 0) {
      if (!done) {
        // look-back guard exhausted (a predecessor never published: a stale tile buffer):
        // no prefix is published, and the totals read -1 so the host's check of the total
        // fails instead of sizing allocations from a wrong prefix
        out[n] = -1;
        *total = -1;
      } else {
        if (tile > 0) st_store(state + tile, ST_INC | ep | (uint64_t)(excl + agg));
        if (tile == ntiles - 1) {
          out[n] = excl + agg;
          *total = excl + agg;
        }
      }
      s_pre = excl;
    }
  }
  __syncthreads();
  pre += s_pre;
  if (bucket) {
    // (optional) bucket[b] = the item whose range [out[i], out[i + 1]) holds position b * bq,
    // b = 0 .. total / bq: the leaf epilogue's first prefix per wave of bq cliques
    int64_t a = pre;
#pragma unroll
    for (int i = 0; i < ONE_PER; ++i) {
      const int64_t e = a + v[i];
      for (int64_t b = (a + bq - 1) / bq; b * bq < e; ++b) bucket[b] = (int32_t)(t0 + i);
      a = e;
    }
  }
  if (vec && t0 + ONE_PER <= n) {
#pragma unroll
    for (int i = 0; i < ONE_PER; i += 2) {
      const int64_t a = pre;
      pre += v[i];
      reinterpret_cast<longlong2*>(out + t0)[i / 2] = make_longlong2(a, pre);
      pre += v[i + 1];
    }
  } else {
#pragma unroll
    for (int i = 0; i < ONE_PER; ++i) {
      if (t0 + i < n) out[t0 + i] = pre;
      pre += v[i];
    }
  }
}

// Several memsets in one launch (the large route zeroes ~10 per-box arrays per run: one
// fill packet each cost ~5 us of mostly idle GPU).  blockIdx.y = segment; 16-byte stores over
// the aligned body, byte stores for the tail.
__global__ __launch_bounds__(WG) void k_fill_multi(FillSegs F) {
  const int sg = blockIdx.y;
  if (sg >= F.n) return;
  uint8_t* p = static_cast<uint8_t*>(F.p[sg]);
  const size_t bytes = F.bytes[sg];
  const uint32_t b = F.val[sg];
  const uint32_t w4 = b | (b << 8) | (b << 16) | (b << 24);
  const uint4 v = make_uint4(w4, w4, w4, w4);
  const size_t nv = bytes / 16;
  for (size_t i = (size_t)blockIdx.x * WG + threadIdx.x; i < nv; i += (size_t)gridDim.x * WG)
    reinterpret_cast<uint4*>(p)[i] = v;
  if (blockIdx.x == 0 && threadIdx.x < (bytes & 15)) p[nv * 16 + threadIdx.x] = (uint8_t)b;
}

void launch_fill_multi(hipStream_t stream, const FillSegs& F) {
  size_t mx = 0;
  for (int i = 0; i < F.n; ++i) mx = std::max(mx, F.bytes[i] / 16);
  const int gx = (int)std::min<size_t>(std::max<size_t>((mx + WG - 1) / WG, 1), 2048);
  if (F.n > 0) hipLaunchKernelGGL(k_fill_multi, dim3(gx, F.n), dim3(WG), 0, stream, F);
}

// ----------------------------------------------------------------------------- K4 CC
__device__ __forceinline__ int ld_par(int32_t* parent, int i) {
  return __hip_atomic_load(parent + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int uf_find(int32_t* parent, int x) {
  for (;;) {
    const int p = ld_par(parent, x);
    if (p == x) return x;
    const int gp = ld_par(parent, p);
    if (gp != p) __hip_atomic_store(parent + x, gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    x = gp;
  }
}

__global__ __launch_bounds__(WG) void k4_init(int N, int32_t* parent) {
  const int g = blockIdx.x * WG + threadIdx.x;
  if (g < N) parent[g] = g;
}

// Lock-free union-find over the forward edges (hook the larger root under the smaller).
__global__ __launch_bounds__(WG) void k4_union(int N, const int64_t* __restrict__ fwd_off,
                                               const int32_t* __restrict__ e_dst, int32_t* parent,
                                               uint8_t* has_edge) {
  const int g = blockIdx.x * WG + threadIdx.x;
  if (g >= N) return;
  const int64_t e0 = fwd_off[g], e1 = fwd_off[g + 1];
  if (e0 == e1) return;
  has_edge[g] = 1;
  for (int64_t e = e0; e < e1; ++e) {
    const int h = e_dst[e];
    has_edge[h] = 1;
    int a = g, b = h;
    for (;;) {
      a = uf_find(parent, a);
      b = uf_find(parent, b);
      if (a == b) break;
      if (a < b) { const int t = a; a = b; b = t; }
      int expect = a;
      if (__hip_atomic_compare_exchange_strong(parent + a, &expect, b, __ATOMIC_RELAXED,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        break;
    }
  }
}

// Same union-find, one 1024-thread workgroup per micrograph with its parents in LDS (int32
// per box, micrographs up to UF_LDS_MAX boxes): LDS hops instead of L2 round trips.  Writes the
// final root of every box (global index), so k4_compress finds it in one hop.
constexpr int UF_LDS_MAX = 39936;   // 156 KiB of int32 parents
__device__ __forceinline__ int uf_find_l(int32_t* P, int x) {
  for (;;) {
    const int p = __hip_atomic_load(P + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (p == x) return x;
    const int gp = __hip_atomic_load(P + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (gp != p) __hip_atomic_store(P + x, gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    x = gp;
  }
}
__global__ __launch_bounds__(1024) void k4_union_lds(int k, const int32_t* __restrict__ box_off,
                                                     const int64_t* __restrict__ fwd_off,
                                                     const int32_t* __restrict__ e_dst,
                                                     int32_t* parent, uint8_t* has_edge) {
  extern __shared__ int32_t P[];
  const int m = blockIdx.x;
  const int b0 = box_off[m * k], n = box_off[m * k + k] - b0;
  for (int i = threadIdx.x; i < n; i += 1024) P[i] = i;
  __syncthreads();
  // one workgroup per micrograph (C5: 64 of 256 CUs, ~27 boxes and ~270 unions per thread):
  // the global loads are the latency chain, so a box's targets are read UF_B at a time and
  // the next box's edge range is loaded before this box's unions
  constexpr int UF_B = 8;
  int64_t e0 = 0, e1 = 0;
  if (threadIdx.x < n) { e0 = fwd_off[b0 + threadIdx.x]; e1 = fwd_off[b0 + threadIdx.x + 1]; }
  for (int i = threadIdx.x; i < n; i += 1024) {
    const int64_t c0 = e0, c1 = e1;
    if (i + 1024 < n) { e0 = fwd_off[b0 + i + 1024]; e1 = fwd_off[b0 + i + 1025]; }
    if (c0 == c1) continue;
    has_edge[b0 + i] = 1;
    // ri: a root of box i's set as last seen (still a root unless another thread hooked it:
    // then the find below walks on from it), so each edge costs one find of its target
    int ri = uf_find_l(P, i);
    for (int64_t e = c0; e < c1; e += UF_B) {
      int hs[UF_B];
#pragma unroll
      for (int u = 0; u < UF_B; ++u) hs[u] = e + u < c1 ? e_dst[e + u] - b0 : -1;
#pragma unroll
      for (int u = 0; u < UF_B; ++u) {
        const int h = hs[u];
        if (h < 0) continue;
        has_edge[b0 + h] = 1;
        int b = h;
        for (;;) {
          ri = uf_find_l(P, ri);
          b = uf_find_l(P, b);
          if (ri == b) break;
          // hook the larger root under the smaller; i's root is the smaller one afterwards
          const int hi = ri > b ? ri : b, lo = ri > b ? b : ri;
          int expect = hi;
          if (__hip_atomic_compare_exchange_strong(P + hi, &expect, lo, __ATOMIC_RELAXED,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
            ri = lo;
            break;
          }
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += 1024) parent[b0 + i] = b0 + uf_find_l(P, i);
}

__global__ __launch_bounds__(WG) void k4_compress(int N, const uint8_t* __restrict__ has_edge,
                                                  int32_t* parent, int32_t* csize) {
  const int g = blockIdx.x * WG + threadIdx.x;
  if (g >= N || !has_edge[g]) return;
  const int r = uf_find(parent, g);
  __hip_atomic_store(parent + g, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the lanes in the first active lane's component add once (a dense micrograph's giant
  // component would otherwise queue one atomic per box on one address)
  const int rf = __builtin_amdgcn_readfirstlane(r);
  const uint64_t same = __ballot(r == rf);
  if (r != rf) atomicAdd(&csize[r], 1);
  else if (__lane_id() == __builtin_ctzll(same)) atomicAdd(&csize[r], (int)__popcll(same));
}

// Per-micrograph CC statistics (runtime.tsv columns 2-3) and NO_EDGES status.
__global__ __launch_bounds__(WG) void k4_stats(int k, const int32_t* __restrict__ box_off,
                                               const int64_t* __restrict__ fwd_off,
                                               const uint8_t* __restrict__ has_edge,
                                               const int32_t* __restrict__ parent,
                                               const int32_t* __restrict__ csize, MgStat* st) {
  __shared__ int64_t red[NW];
  __shared__ int redi[NW];
  const int m = blockIdx.x;
  const int b0 = box_off[m * k], b1 = box_off[m * k + k];
  int64_t nodes = 0, roots = 0;
  int mx = 0;
  // (one workgroup per micrograph: loads of four boxes in flight per thread)
#pragma unroll 4
  for (int g = b0 + threadIdx.x; g < b1; g += WG) {
    const bool he = has_edge[g];
    const bool root = parent[g] == g;
    nodes += he ? 1 : 0;
    if (he && root) { ++roots; mx = max(mx, csize[g]); }
  }
  nodes = block_sum64(nodes, red);
  roots = block_sum64(roots, red);
  mx = block_max_i(mx, redi);
  if (threadIdx.x == 0) {
    MgStat s;
    s.n_edges = fwd_off[b1] - fwd_off[b0];
    s.n_nodes = (int)nodes;
    s.cc_cnt = (int)roots;
    s.cc_max = mx;
    s.status = s.n_edges == 0 ? 1 : 0;
    s.target = -1;
    s.n_vert = 0;
    s.clique_base = 0;
    s.clique_cnt = 0;
    st[m] = s;
  }
}

__device__ __forceinline__ uint64_t ins_pack(int pair, int la, int lb, int side) {
  return ((uint64_t)pair << 49) | ((uint64_t)la << 25) | ((uint64_t)lb << 1) | (uint64_t)side;
}

// Graph node insertion order (networkx add_node order, get_cliques.py:33-34): a node's key
// is its first appearance in the edge enumeration (picker pair, a index, b index, side).
// Only needed where networkx iterates graph order: |G| <= 2k (FilterAtlas) or --get_cc.
__global__ __launch_bounds__(WG) void k4_ins_keys(int N, int k, int get_cc,
                                                  const int32_t* __restrict__ box_off,
                                                  const int32_t* __restrict__ bmg,
                                                  const uint8_t* __restrict__ bpick,
                                                  const int64_t* __restrict__ fwd_off,
                                                  const int32_t* __restrict__ e_dst,
                                                  const MgStat* __restrict__ st,
                                                  unsigned long long* ins_key) {
  const int g = blockIdx.x * WG + threadIdx.x;
  if (g >= N) return;
  const int64_t e0 = fwd_off[g], e1 = fwd_off[g + 1];
  if (e0 == e1) return;
  const int m = bmg[g];
  if (!get_cc && st[m].n_nodes > 2 * k) return;
  const int pa = bpick[g];
  const int la = g - box_off[m * k + pa];
  {
    const int h = e_dst[e0];
    const int ph = bpick[h];
    atomicMin(ins_key + g, ins_pack(pair_index(pa, ph, k), la, h - box_off[m * k + ph], 0));
  }
  for (int64_t e = e0; e < e1; ++e) {
    const int h = e_dst[e];
    const int ph = bpick[h];
    atomicMin(ins_key + h, ins_pack(pair_index(pa, ph, k), la, h - box_off[m * k + ph], 1));
  }
}

__global__ __launch_bounds__(WG) void k4_comp_min(int N, const uint8_t* __restrict__ has_edge,
                                                  const int32_t* __restrict__ parent,
                                                  const unsigned long long* __restrict__ ins_key,
                                                  unsigned long long* comp_min) {
  const int g = blockIdx.x * WG + threadIdx.x;
  if (g >= N || !has_edge[g]) return;
  atomicMin(comp_min + parent[g], ins_key[g]);
}

// --get_cc: largest CC, ties -> first discovered (smallest first-inserted node).
__global__ __launch_bounds__(WG) void k4_target(int k, const int32_t* __restrict__ box_off,
                                                const uint8_t* __restrict__ has_edge,
                                                const int32_t* __restrict__ parent,
                                                const int32_t* __restrict__ csize,
                                                const unsigned long long* __restrict__ comp_min,
                                                MgStat* st) {
  __shared__ unsigned long long best[WG];
  __shared__ int bestg[WG];
  const int m = blockIdx.x;
  const int b0 = box_off[m * k], b1 = box_off[m * k + k];
  const int cmax = st[m].cc_max;
  unsigned long long bk = ~0ULL;
  int bg = -1;
  for (int g = b0 + threadIdx.x; g < b1; g += WG) {
    if (has_edge[g] && parent[g] == g && csize[g] == cmax && comp_min[g] < bk) {
      bk = comp_min[g];
      bg = g;
    }
  }
  best[threadIdx.x] = bk;
  bestg[threadIdx.x] = bg;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < WG; ++i)
      if (best[i] < bk) { bk = best[i]; bg = bestg[i]; }
    st[m].target = bg;
  }
}

// ----------------------------------------------------------------------------- K5 fallback
// Micrographs with a root whose forward neighbourhood exceeds the bitmap width of the level
// kernels (rgc_cliques.hip, RB_W boxes) are enumerated here, one thread per root,
// depth-first over the global forward CSR (sorted-list membership by binary search).  COUNT:
// cliques per root and the clique-vertex flags; FILL: the members of each clique at the
// root's scanned offset after the level route's cliques (the ILP epilogue is the shared
// thread-per-clique kernel).  Lexicographic order, like the level kernels.
__device__ __forceinline__ int64_t lower_bound(const int32_t* a, int64_t lo, int64_t hi, int v) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

template <int K>
struct Walk {
  int mem[K];        // chosen box per picker
  int pb[K + 1];     // picker box bounds of this micrograph
  int64_t count;
  int64_t out;       // next output clique index (FILL)
};

template <int K, int D, bool FILL>
struct Level {
  __device__ static void run(const CliqueArgs& A, Walk<K>& W) {
    const int prev = W.mem[D - 1];
    int64_t lo = A.fwd_off[prev];
    const int64_t hi0 = A.fwd_off[prev + 1];
    lo = lower_bound(A.e_dst, lo, hi0, W.pb[D]);
    const int64_t hi = lower_bound(A.e_dst, lo, hi0, W.pb[D + 1]);
    for (int64_t e = lo; e < hi; ++e) {
      const int h = A.e_dst[e];
      bool ok = true;
#pragma unroll
      for (int q = 0; q < D - 1; ++q) {
        const int c = W.mem[q];
        const int64_t c0 = A.fwd_off[c], c1 = A.fwd_off[c + 1];
        const int64_t pos = lower_bound(A.e_dst, c0, c1, h);
        if (pos >= c1 || A.e_dst[pos] != h) { ok = false; break; }
      }
      if (!ok) continue;
      W.mem[D] = h;
      Level<K, D + 1, FILL>::run(A, W);
    }
  }
};
template <int K, bool FILL>
struct Level<K, K, FILL> {
  __device__ static void run(const CliqueArgs& A, Walk<K>& W) {
    if (FILL) {
      const int64_t j = W.out++;
#pragma unroll
      for (int i = 0; i < K; ++i) A.members[j * K + i] = W.mem[i];
    } else {
      ++W.count;
#pragma unroll
      for (int i = 0; i < K; ++i) A.in_clique[W.mem[i]] = 1;
    }
  }
};

template <int K, bool FILL>
__global__ __launch_bounds__(WG) void k5_cliques(int N, CliqueArgs A) {
  const int g = blockIdx.x * WG + threadIdx.x;
  if (g >= N) return;
  if (A.bpick[g] != 0) return;
  const int m = A.bmg[g];
  if (!A.dfs_mg[m]) return;   // the level kernels' micrograph
  if (A.fwd_off[g] == A.fwd_off[g + 1]) return;
  const MgStat s = A.st[m];
  if (s.status != 0) return;
  if ((A.flags & 1) && A.parent[g] != s.target) return;
  Walk<K> W;
  W.count = 0;
  W.out = FILL ? A.dfs_base + A.clique_off[g] : 0;
#pragma unroll
  for (int i = 0; i <= K; ++i) W.pb[i] = A.box_off[m * A.k + i];
  W.mem[0] = g;
  Level<K, 1, FILL>::run(A, W);
  if (!FILL) A.ccount[g] = (int32_t)W.count;
}

// ----------------------------------------------------------------------------- K7 rows
// Row index of each clique vertex = its rank by (x, y, id) among the micrograph's clique
// vertices (v = sorted(set(...)); v.index(val), get_cliques.py:164,193).  Thread-per-box
// kernels over the whole sub-batch (a micrograph of 27k boxes is not serialised on one
// workgroup): each micrograph owns n_m x-buckets (a monotone map of x over its bounding
// box, at box-index offsets, so the buckets of all micrographs form one array); count ->
// scan -> scatter; the rank is the bucket's start inside the micrograph plus the number of
// smaller vertices in the bucket.
__device__ __forceinline__ int rank_bucket(const MgGrid& G, int b0, int n, double x) {
  const double ext = (double)G.gx * G.cell;
  const double sc = ext > 0.0 && ext < INFINITY ? (double)n / ext : 0.0;
  const double f = (x - G.minx) * sc;
  return b0 + (int)fmin(fmax(f, 0.0), (double)(n - 1));
}

__global__ __launch_bounds__(WG) void k7_bucket(int N, int k, const int32_t* __restrict__ box_off,
                                                const int32_t* __restrict__ bmg,
                                                const MgGrid* __restrict__ grid,
                                                const double* __restrict__ x,
                                                const uint8_t* __restrict__ in_clique,
                                                int32_t* bcnt, int32_t* bslot, int32_t* bbk) {
  const int g = blockIdx.x * WG + threadIdx.x;
  if (g >= N || !in_clique[g]) return;
  const int m = bmg[g];
  const int b0 = box_off[m * k];
  const int bk = rank_bucket(grid[m], b0, box_off[m * k + k] - b0, x[g]);
  bslot[g] = atomicAdd(&bcnt[bk], 1);
  bbk[g] = bk;   // (the place passes start from the bucket, not the grid lookup chain)
}

template <bool RANK>
__global__ __launch_bounds__(WG) void k7_place(int N, int k, const int32_t* __restrict__ box_off,
                                               const int32_t* __restrict__ bmg,
                                               const double* __restrict__ x,
                                               const double* __restrict__ y,
                                               const uint8_t* __restrict__ in_clique,
                                               const int64_t* __restrict__ boff,
                                               const int32_t* __restrict__ bslot,
                                               const int32_t* __restrict__ bbk, int32_t* vsort,
                                               int32_t* vrow) {
  const int g = blockIdx.x * WG + threadIdx.x;
  if (g >= N || !in_clique[g]) return;
  const int bk = bbk[g];
  const int64_t lo = boff[bk];
  if (!RANK) {
    vsort[lo + bslot[g]] = g;
    return;
  }
  const int b0 = box_off[bmg[g] * k];
  const double gx = x[g];
  const int64_t hi = boff[bk + 1];
  const double gy = y[g];
  int r = (int)(lo - boff[b0]);
  for (int64_t q = lo; q < hi; ++q) {
    const int u = vsort[q];
    const double ux = x[u], uy = y[u];
    r += (ux < gx) || (ux == gx && (uy < gy || (uy == gy && u < g)));
  }
  vrow[g] = r;
}

__global__ __launch_bounds__(WG) void k7_nvert(int n_mg, int k, const int32_t* __restrict__ box_off,
                                               const int64_t* __restrict__ boff, MgStat* st) {
  const int m = blockIdx.x * WG + threadIdx.x;
  if (m >= n_mg) return;
  st[m].n_vert = (int)(boff[box_off[m * k + k]] - boff[box_off[m * k]]);
}

// ----------------------------------------------------------------------------- sub-batch
// Gather the boxes of deferred micrographs into a compact sub-batch for this path.
__global__ __launch_bounds__(WG) void k_gather(int k, const int32_t* __restrict__ sub_mg,
                                               const int32_t* __restrict__ box_off,
                                               const int32_t* __restrict__ sub_box_off,
                                               const double* __restrict__ x,
                                               const double* __restrict__ y,
                                               const double* __restrict__ s, double* ox,
                                               double* oy, double* os, int32_t* orig) {
  const int mp = blockIdx.x, m = sub_mg[mp];
  const int b0 = box_off[m * k], n = box_off[m * k + k] - b0, d0 = sub_box_off[mp * k];
  for (int i = threadIdx.x; i < n; i += WG) {
    ox[d0 + i] = x[b0 + i];
    oy[d0 + i] = y[b0 + i];
    os[d0 + i] = s[b0 + i];
    orig[d0 + i] = b0 + i;
  }
}

__global__ __launch_bounds__(WG) void k_remap(int64_t C, int k, const int32_t* __restrict__ orig,
                                              int32_t* consensus, int32_t* members) {
  const int64_t j = (int64_t)blockIdx.x * WG + threadIdx.x;
  if (j >= C) return;
  consensus[j] = orig[consensus[j]];
  if (members)   // (only when members are outputs: otherwise most were never written)
    for (int i = 0; i < k; ++i) members[j * k + i] = orig[members[j * k + i]];
}

// RGC_F_EDGES test hook: the sub-batch's edge list (u, v, JI) in batch box indices.
__global__ __launch_bounds__(WG) void k_dump_edges(int N, const int64_t* __restrict__ fwd_off,
                                                   const int32_t* __restrict__ e_dst,
                                                   const double* __restrict__ e_ji,
                                                   const int32_t* __restrict__ orig, int32_t* eu,
                                                   int32_t* ev, double* eji) {
  const int g = blockIdx.x * WG + threadIdx.x;
  if (g >= N) return;
  for (int64_t e = fwd_off[g]; e < fwd_off[g + 1]; ++e) {
    eu[e] = orig ? orig[g] : g;
    ev[e] = orig ? orig[e_dst[e]] : e_dst[e];
    eji[e] = e_ji[e];
  }
}

// ----------------------------------------------------------------------------- launchers
void launch_dump_edges(hipStream_t stream, int N, const int64_t* fwd_off, const int32_t* e_dst,
                       const double* e_ji, const int32_t* orig, int32_t* eu, int32_t* ev,
                       double* eji) {
  const int nb = (N + WG - 1) / WG;
  if (nb > 0)
    hipLaunchKernelGGL(k_dump_edges, dim3(nb), dim3(WG), 0, stream, N, fwd_off, e_dst, e_ji, orig,
                       eu, ev, eji);
}

void launch_gather(hipStream_t stream, int n_sub, int k, const int32_t* sub_mg,
                   const int32_t* box_off, const int32_t* sub_box_off, const double* x,
                   const double* y, const double* s, double* ox, double* oy, double* os,
                   int32_t* orig) {
  if (n_sub > 0)
    hipLaunchKernelGGL(k_gather, dim3(n_sub), dim3(WG), 0, stream, k, sub_mg, box_off,
                       sub_box_off, x, y, s, ox, oy, os, orig);
}

void launch_remap(hipStream_t stream, int64_t C, int k, const int32_t* orig, int32_t* consensus,
                  int32_t* members) {
  const int64_t nb = (C + WG - 1) / WG;
  if (nb > 0)
    hipLaunchKernelGGL(k_remap, dim3(nb), dim3(WG), 0, stream, C, k, orig, consensus, members);
}

#define RGC_LAUNCH(kern, grid, block, ...) \
  hipLaunchKernelGGL(kern, dim3(grid), dim3(block), 0, stream, __VA_ARGS__)

void launch_bin(hipStream_t stream, int n_mg, int k, double B, const int32_t* box_off,
                const int32_t* cell_off, const double* x, const double* y, MgGrid* grid,
                int32_t* cell_start, double* sx, double* sy, int32_t* sbox, uint8_t* spick,
                int32_t* smg, int32_t* bmg, uint8_t* bpick, bool wide, int max_n) {
  // (the caller passes wide = some micrograph of the batch has more than 65535 boxes, and
  // the batch's largest micrograph: the counters of its key budget set the dynamic LDS)
  if (n_mg <= 0) return;
  const int keys = bin_budget(max_n, wide) + 2;
  const int lds = (wide ? 4 * keys : 2 * (keys + 2)) + 16;
  if (wide) {
    static std::atomic<uint64_t> attr{0};
    (void)set_dyn_lds_once(attr, reinterpret_cast<const void*>(&k1_bin<true>), 132 * 1024);
    hipLaunchKernelGGL(k1_bin<true>, dim3(n_mg), dim3(1024), lds, stream, k, B, box_off,
                       cell_off, x, y, grid, cell_start, sx, sy, sbox, spick, smg, bmg, bpick);
  } else {
    static std::atomic<uint64_t> attr{0};
    (void)set_dyn_lds_once(attr, reinterpret_cast<const void*>(&k1_bin<false>), 132 * 1024);
    hipLaunchKernelGGL(k1_bin<false>, dim3(n_mg), dim3(1024), lds, stream, k, B, box_off,
                       cell_off, x, y, grid, cell_start, sx, sy, sbox, spick, smg, bmg, bpick);
  }
}

void launch_pairs(hipStream_t stream, bool fill, int N, int k, double B, double two_b2,
                  const int32_t* box_off, const int32_t* cell_off, const MgGrid* grid,
                  const int32_t* cell_start, const double* sx, const double* sy,
                  const int32_t* sbox, const uint8_t* spick, const int32_t* smg,
                  int32_t* fwd_cnt, const int64_t* fwd_off, int32_t* e_dst, double* e_ji) {
  const int nb = (N + WG - 1) / WG;
  if (nb == 0) return;
  if (fill)
    RGC_LAUNCH(k2_pairs<true>, nb, WG, N, k, B, two_b2, box_off, cell_off, grid, cell_start, sx,
               sy, sbox, spick, smg, fwd_cnt, fwd_off, e_dst, e_ji);
  else
    RGC_LAUNCH(k2_pairs<false>, nb, WG, N, k, B, two_b2, box_off, cell_off, grid, cell_start,
               sx, sy, sbox, spick, smg, fwd_cnt, fwd_off, e_dst, e_ji);
}

// tile buffer words: the one-pass scan's claim counter + one state per tile
int64_t scan_tiles_needed(int64_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE + 2; }

// (64-bit: the count never wraps, so an epoch value recurs exactly every 2^22 - 1 launches)
static std::atomic<uint64_t> g_scan_epochs{0};
uint64_t scan_epoch_count() { return g_scan_epochs.load(); }

void launch_scan(hipStream_t stream, int64_t n, const int32_t* in, int64_t* out,
                 int64_t* tile_buf, int64_t* total, int32_t* bucket, int bq) {
  // launch epochs are process-wide (any two launches sharing a tile buffer differ; an epoch
  // repeats after 2^22 - 1 launches, so the owner of a tile buffer zeroes it at least every
  // SCAN_EPOCH_REFRESH launches: scan_epoch_count)
  const uint32_t e = (uint32_t)(g_scan_epochs.fetch_add(1) % ((1u << 22) - 1)) + 1;
  const int64_t nt = std::max<int64_t>(1, (n + ONE_TILE - 1) / ONE_TILE);
  RGC_LAUNCH(scan_onepass, nt, WG, n, in, out, total, reinterpret_cast<uint64_t*>(tile_buf), e,
             bucket, bq);
}

void launch_cc(hipStream_t stream, int phase, int N, int n_mg, int k, int get_cc,
               const int32_t* box_off, const int32_t* bmg, const uint8_t* bpick,
               const int64_t* fwd_off, const int32_t* e_dst, int32_t* parent, uint8_t* has_edge,
               int32_t* csize, MgStat* st, unsigned long long* ins_key,
               unsigned long long* comp_min, int max_n) {
  const int nb = (N + WG - 1) / WG;
  switch (phase) {
    case 0: if (nb) RGC_LAUNCH(k4_init, nb, WG, N, parent); break;
    case 1:
      // LDS union-find needs the 160 KiB dynamic-LDS limit on this device; if it cannot be
      // set, the global-memory union-find runs instead
      static std::atomic<uint64_t> lds_attr{0};
      if (nb && max_n <= UF_LDS_MAX &&
          set_dyn_lds_once(lds_attr, reinterpret_cast<const void*>(&k4_union_lds), 160 * 1024) ==
              hipSuccess) {
        hipLaunchKernelGGL(k4_union_lds, dim3(n_mg), dim3(1024), (size_t)max_n * 4, stream, k,
                           box_off, fwd_off, e_dst, parent, has_edge);
      } else if (nb) {
        RGC_LAUNCH(k4_union, nb, WG, N, fwd_off, e_dst, parent, has_edge);
      }
      break;
    case 2: if (nb) RGC_LAUNCH(k4_compress, nb, WG, N, has_edge, parent, csize); break;
    case 3: RGC_LAUNCH(k4_stats, n_mg, WG, k, box_off, fwd_off, has_edge, parent, csize, st); break;
    case 4:
      if (nb) RGC_LAUNCH(k4_ins_keys, nb, WG, N, k, get_cc, box_off, bmg, bpick, fwd_off, e_dst,
                         st, ins_key);
      break;
    case 5: if (nb) RGC_LAUNCH(k4_comp_min, nb, WG, N, has_edge, parent, ins_key, comp_min); break;
    case 6: RGC_LAUNCH(k4_target, n_mg, WG, k, box_off, has_edge, parent, csize, comp_min, st); break;
  }
}

template <int K>
static void launch_dfs_k(hipStream_t stream, bool fill, int N, const CliqueArgs& A) {
  const int nb = (N + WG - 1) / WG;
  if (!nb) return;
  if (fill) RGC_LAUNCH((k5_cliques<K, true>), nb, WG, N, A);
  else RGC_LAUNCH((k5_cliques<K, false>), nb, WG, N, A);
}

int launch_cliques_dfs(hipStream_t stream, bool fill, int N, const CliqueArgs& A) {
  switch (A.k) {
    case 2: launch_dfs_k<2>(stream, fill, N, A); break;
    case 3: launch_dfs_k<3>(stream, fill, N, A); break;
    case 4: launch_dfs_k<4>(stream, fill, N, A); break;
    case 5: launch_dfs_k<5>(stream, fill, N, A); break;
    case 6: launch_dfs_k<6>(stream, fill, N, A); break;
    case 7: launch_dfs_k<7>(stream, fill, N, A); break;
    case 8: launch_dfs_k<8>(stream, fill, N, A); break;
    default: return -1;
  }
  return 0;
}

void launch_rank(hipStream_t stream, int N, int n_mg, int k, const int32_t* box_off,
                 const int32_t* bmg, const MgGrid* grid, const double* x, const double* y,
                 const uint8_t* in_clique, int32_t* bcnt, int32_t* bslot, int32_t* bbk,
                 int64_t* boff, int64_t* tile_buf, int64_t* total, int32_t* vsort, int32_t* vrow,
                 MgStat* st) {
  const int nb = (N + WG - 1) / WG;
  if (nb) RGC_LAUNCH(k7_bucket, nb, WG, N, k, box_off, bmg, grid, x, in_clique, bcnt, bslot, bbk);
  launch_scan(stream, N, bcnt, boff, tile_buf, total);
  if (nb) {
    RGC_LAUNCH(k7_place<false>, nb, WG, N, k, box_off, bmg, x, y, in_clique, boff, bslot, bbk,
               vsort, vrow);
    RGC_LAUNCH(k7_place<true>, nb, WG, N, k, box_off, bmg, x, y, in_clique, boff, bslot, bbk,
               vsort, vrow);
  }
  RGC_LAUNCH(k7_nvert, (n_mg + WG - 1) / WG, WG, n_mg, k, box_off, boff, st);
}

}  // namespace rgc

namespace {
template <int K>
int test_epilogue_k(const double* x, const double* y, const double* score, const int64_t* ids,
                    const double* ji, int set_order, const uint64_t* ins, int* arg, int8_t* ord,
                    float* w, float* conf) {
  int mem[K];
  double jj[K][K] = {}, s[K], xs[K], ys[K];
  int64_t id[K];
  uint64_t in[K];
  int64_t idmin = ids[0];
  for (int i = 1; i < K; ++i) idmin = ids[i] < idmin ? ids[i] : idmin;
  for (int i = 0; i < K; ++i) {
    mem[i] = (int)(ids[i] - idmin);   // any handle monotone in id
    s[i] = score[i]; xs[i] = x[i]; ys[i] = y[i]; id[i] = ids[i];
    in[i] = ins ? ins[i] : 0;
    for (int j = i + 1; j < K; ++j) jj[i][j] = ji[i * K + j];
  }
  rgc::Epi<K> e;
  rgc::epilogue<K>(mem, jj, s, xs, ys, id, set_order != 0, in, true, e);
  *arg = e.arg;
  for (int i = 0; i < K; ++i) ord[i] = e.ord[i];
  *w = e.w;
  *conf = e.conf;
  return 0;
}
}  // namespace

extern "C" int rgc_test_epilogue(int k, const double* x, const double* y, const double* score,
                                 const int64_t* ids, const double* ji, int set_order,
                                 const uint64_t* ins, int* arg, int8_t* ord, float* w,
                                 float* conf) {
  switch (k) {
#define RGC_TE(KK) \
  case KK: return test_epilogue_k<KK>(x, y, score, ids, ji, set_order, ins, arg, ord, w, conf);
    RGC_TE(2) RGC_TE(3) RGC_TE(4) RGC_TE(5) RGC_TE(6) RGC_TE(7) RGC_TE(8)
#undef RGC_TE
    default: return -1;
  }
}
