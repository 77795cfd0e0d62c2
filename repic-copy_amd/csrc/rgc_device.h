// rgc_device.h — device helpers shared by the multi-kernel and fused pipelines.
#pragma once
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "pyset.h"

namespace rgc {

constexpr int WG = 256;
constexpr int NW = WG / 64;

// A kernel argument as its own scalar value.  The kernel-argument lowering loads neighbouring
// FusedArgs fields with one s_load_dwordx16; kept live across the kernel, such a 16-SGPR tuple
// is spilled to VGPR lanes as a unit, and every later use of ONE of its fields reloaded all 16
// lanes (v_readlane: VALU issue slots) - 74 per clique in P6.  An s_mov through asm copies the
// field out of the tuple once (a new value the coalescer cannot fold back into the tuple), so
// a spill of it costs one or two lanes.  Pointers come back as global (address space 1)
// pointers, so their accesses stay global_load / global_store.
template <typename T>
using gptr = __attribute__((address_space(1))) T*;
#if defined(RGC_STAMPS)
template <typename T>
__device__ __forceinline__ gptr<T> gdetach(T* p) { return (gptr<T>)p; }
__device__ __forceinline__ double sdetach(double v) { return v; }
__device__ __forceinline__ int sdetach(int v) { return v; }
__device__ __forceinline__ int64_t sdetach(int64_t v) { return v; }
#else
template <typename T>
__device__ __forceinline__ gptr<T> gdetach(T* p) {
  uint64_t v = (uint64_t)p, r;
  asm volatile("s_mov_b64 %0, %1" : "=s"(r) : "s"(v));
  return (gptr<T>)(T*)r;
}
__device__ __forceinline__ double sdetach(double v) {
  double r;
  asm volatile("s_mov_b64 %0, %1" : "=s"(r) : "s"(v));
  return r;
}
__device__ __forceinline__ int sdetach(int v) {
  int r;
  asm volatile("s_mov_b32 %0, %1" : "=s"(r) : "s"(v));
  return r;
}
__device__ __forceinline__ int64_t sdetach(int64_t v) {
  int64_t r;
  asm volatile("s_mov_b64 %0, %1" : "=s"(r) : "s"(v));
  return r;
}
#endif


// ----------------------------------------------------------------------------- block reductions
template <int BS = WG>
__device__ __forceinline__ double block_min(double v, double* lds) {
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = lds[0];
  for (int i = 1; i < BS / 64; ++i) r = fmin(r, lds[i]);
  return r;
}
template <int BS = WG>
__device__ __forceinline__ double block_max(double v, double* lds) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = lds[0];
  for (int i = 1; i < BS / 64; ++i) r = fmax(r, lds[i]);
  return r;
}
template <int BS = WG>
__device__ __forceinline__ int64_t block_sum64(int64_t v, int64_t* lds) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  int64_t r = 0;
  for (int i = 0; i < BS / 64; ++i) r += lds[i];
  return r;
}
template <int BS = WG>
__device__ __forceinline__ int block_max_i(int v, int* lds) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  int r = lds[0];
  for (int i = 1; i < BS / 64; ++i) r = max(r, lds[i]);
  return r;
}
template <int BS = WG>
__device__ __forceinline__ uint64_t block_min_u64(uint64_t v, uint64_t* lds) {
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t t = __shfl_xor(v, o, 64);
    v = t < v ? t : v;
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t r = lds[0];
  for (int i = 1; i < BS / 64; ++i) r = lds[i] < r ? lds[i] : r;
  return r;
}

// ----------------------------------------------------------------------------- DPP wave scans
// gfx9 wave64 Hillis-Steele scan on DPP lane moves: row_shr:1/2/4/8 inside each 16-lane row,
// then row_bcast:15 (lane 15 of a row to the next row) and row_bcast:31 (lane 31 to rows 2-3).
// VALU only: no ds_bpermute round trips through the LDS crossbar.  64-bit values move as two
// 32-bit halves.
template <int CTRL, typename T>
__device__ __forceinline__ T dpp_mov(T v) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32- or 64-bit lanes");
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(
        T, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
  } else {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xf,
                                                               0xf, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL,
                                                               0xf, 0xf, false);
    return __builtin_bit_cast(T, ((uint64_t)hi << 32) | lo);
  }
}
// inclusive scan across the wave with an associative, commutative op (lane 63: the total)
template <typename T, typename Op>
__device__ __forceinline__ T wave_incl_scan(T v, Op op) {
  const int lane = threadIdx.x & 63, rl = lane & 15;
  T t;
  t = dpp_mov<0x111>(v); if (rl >= 1) v = op(t, v);
  t = dpp_mov<0x112>(v); if (rl >= 2) v = op(t, v);
  t = dpp_mov<0x114>(v); if (rl >= 4) v = op(t, v);
  t = dpp_mov<0x118>(v); if (rl >= 8) v = op(t, v);
  t = dpp_mov<0x142>(v); if (lane & 16) v = op(t, v);
  t = dpp_mov<0x143>(v); if (lane >= 32) v = op(t, v);
  return v;
}

// 32-bit inclusive add / max scans across the wave (lane 63: the total) with the DPP moves'
// bound_ctrl / row_mask: lanes without a source lane read 0, so every step is one move and
// one unconditional op (max: non-negative values only)
__device__ __forceinline__ int dpp_shr_add(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);   // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return v;
}
__device__ __forceinline__ int wave_incl_add32(int v) { return dpp_shr_add(v); }
__device__ __forceinline__ int wave_incl_max32(int v) {
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true));
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true));
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true));
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true));
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false));
  v = max(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false));
  return v;
}

// float minimum across the wave (lane 63: the result); lanes without a source lane read +inf.
// v_min_f32 through asm: no sNaN canonicalisation of the DPP operand (inputs are never NaN)
__device__ __forceinline__ float vmin_f32(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float wave_incl_min_f32(float v) {
  const int inf = 0x7f800000;
#define RGC_DPP_MIN(ctrl, rm, bc)                                                          \
  v = vmin_f32(v, __int_as_float(__builtin_amdgcn_update_dpp(inf, __float_as_int(v), ctrl, \
                                                             rm, 0xf, bc)))
  RGC_DPP_MIN(0x111, 0xf, false);
  RGC_DPP_MIN(0x112, 0xf, false);
  RGC_DPP_MIN(0x114, 0xf, false);
  RGC_DPP_MIN(0x118, 0xf, false);
  RGC_DPP_MIN(0x142, 0xa, false);
  RGC_DPP_MIN(0x143, 0xc, false);
#undef RGC_DPP_MIN
  return v;
}

// In-place exclusive scan of a[0..n) in LDS whose total fits 31 bits (u16 arrays: boxes,
// edges, vertices), a[n] = total, on 32-bit DPP wave scans; same barriers and contract as
// block_scan_dpp below (lds: BS / 64 ints).
template <int BS, typename A>
__device__ __forceinline__ int block_scan_dpp32(A* a, int n, int* lds) {
  // u16 arrays (4-byte aligned): each thread an even-length chunk read and written as u32
  // pairs (half the LDS operations); an odd tail element only in the last chunk
  constexpr bool PAIRS = sizeof(A) == 2;
  const int per0 = (n + BS - 1) / BS;
  const int per = PAIRS ? (per0 + 1) & ~1 : per0;
  const int c0 = min((int)threadIdx.x * per, n), c1 = min(c0 + per, n);
  uint32_t* a2 = reinterpret_cast<uint32_t*>(a);
  const int ce = PAIRS ? c0 + ((c1 - c0) & ~1) : c1;   // end of the pairs
  int s = 0;
  if constexpr (PAIRS) {
    for (int c = c0; c < ce; c += 2) {
      const uint32_t v = a2[c >> 1];
      s += (int)(v & 0xFFFFu) + (int)(v >> 16);
    }
    if (ce < c1) s += a[ce];
  } else {
    for (int c = c0; c < c1; ++c) s += a[c];
  }
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int inc = wave_incl_add32(s);
  if (l == 63) lds[w] = inc;
  __syncthreads();
  int pre = inc - s, tot = 0;
#pragma unroll
  for (int i = 0; i < BS / 64; ++i) {
    const int x = lds[i];
    pre += (i < w) ? x : 0;
    tot += x;
  }
  if constexpr (PAIRS) {
    for (int c = c0; c < ce; c += 2) {
      const uint32_t v = a2[c >> 1];
      const int p1 = pre + (int)(v & 0xFFFFu);
      a2[c >> 1] = ((uint32_t)pre & 0xFFFFu) | ((uint32_t)p1 << 16);
      pre = p1 + (int)(v >> 16);
    }
    if (ce < c1) a[ce] = (A)pre;
  } else {
    for (int c = c0; c < c1; ++c) {
      const int v = a[c];
      a[c] = (A)pre;
      pre += v;
    }
  }
  if (threadIdx.x == BS - 1) a[n] = (A)tot;
  __syncthreads();
  return tot;
}

// Exclusive scan of one value per thread across the workgroup on DPP wave scans.  ONE barrier:
// the caller guarantees a barrier between any earlier use of lds and this call.
template <int BS, typename T>
__device__ __forceinline__ T block_excl_scan_dpp(T v, T* lds, T* total) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const T inc = wave_incl_scan(v, [](T a, T b) { return a + b; });
  if (l == 63) lds[w] = inc;
  __syncthreads();
  T pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < BS / 64; ++i) {
    const T x = lds[i];
    pre += (i < w) ? x : (T)0;
    tot += x;
  }
  *total = tot;
  return pre + inc - v;
}

// In-place exclusive scan of a[0..n) in LDS (each thread a contiguous chunk), a[n] = total,
// ending with a barrier: two barriers in all, the caller guaranteeing one before (see above).
// A = uint16_t (totals < 2^16) or uint32_t.
template <int BS, typename A>
__device__ __forceinline__ int64_t block_scan_dpp(A* a, int n, int64_t* lds) {
  const int per = (n + BS - 1) / BS;
  const int c0 = min((int)threadIdx.x * per, n), c1 = min(c0 + per, n);
  int64_t s = 0;
  for (int c = c0; c < c1; ++c) s += a[c];
  int64_t tot;
  int64_t pre = block_excl_scan_dpp<BS>(s, lds, &tot);
  for (int c = c0; c < c1; ++c) {
    const A v = a[c];
    a[c] = (A)pre;
    pre += v;
  }
  if (threadIdx.x == BS - 1) a[n] = (A)tot;
  __syncthreads();
  return tot;
}

// Exclusive scan of one value per thread across the workgroup.
template <int BS = WG>
__device__ __forceinline__ int64_t block_excl_scan(int64_t v, int64_t* lds, int64_t* total) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t inc = v;
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t t = __shfl_up(inc, o, 64);
    if (l >= o) inc += t;
  }
  __syncthreads();
  if (l == 63) lds[w] = inc;
  __syncthreads();
  int64_t pre = 0, tot = 0;
  for (int i = 0; i < BS / 64; ++i) {
    if (i < w) pre += lds[i];
    tot += lds[i];
  }
  *total = tot;
  return pre + inc - v;
}

// In-place exclusive scan of a[0..n) (LDS, u32), each thread a contiguous chunk.
// Returns the total.  Ends with a barrier.
template <int BS = WG>
__device__ __forceinline__ int64_t block_scan_array(uint32_t* a, int n, int64_t* lds) {
  const int per = (n + BS - 1) / BS;
  const int c0 = min((int)threadIdx.x * per, n), c1 = min(c0 + per, n);
  int64_t s = 0;
  for (int c = c0; c < c1; ++c) s += a[c];
  int64_t tot;
  int64_t pre = block_excl_scan<BS>(s, lds, &tot);
  for (int c = c0; c < c1; ++c) {
    const uint32_t v = a[c];
    a[c] = (uint32_t)pre;
    pre += v;
  }
  __syncthreads();
  return tot;
}

// In-place exclusive scan of a[0..n) (LDS, u16 values whose total fits 16 bits).
template <int BS = WG>
__device__ __forceinline__ int64_t block_scan_u16(uint16_t* a, int n, int64_t* lds) {
  const int per = (n + BS - 1) / BS;
  const int c0 = min((int)threadIdx.x * per, n), c1 = min(c0 + per, n);
  int64_t s = 0;
  for (int c = c0; c < c1; ++c) s += a[c];
  int64_t tot;
  int64_t pre = block_excl_scan<BS>(s, lds, &tot);
  for (int c = c0; c < c1; ++c) {
    const uint16_t v = a[c];
    a[c] = (uint16_t)pre;
    pre += v;
  }
  __syncthreads();
  return tot;
}

// ----------------------------------------------------------------------------- arithmetic
// overlap area of two boxes, reference op order (get_cliques.py:42-44), no FMA.
__host__ __device__ __forceinline__ double overlap(double x, double y, double a, double b, double B) {
  const double xo = fmax((fmin(x, a) + B) - fmax(x, a), 0.0);
  const double yo = fmax((fmin(y, b) + B) - fmax(y, b), 0.0);
  return xo * yo;
}

// reference calc_jaccard (get_cliques.py:40-46), same f64 op order, no FMA.
__host__ __device__ __forceinline__ double jaccard(double x, double y, double a, double b, double B,
                                          double two_b2) {
  const double xo = fmax((fmin(x, a) + B) - fmax(x, a), 0.0);
  const double yo = fmax((fmin(y, b) + B) - fmax(y, b), 0.0);
  const double inter = xo * yo;
  return inter / (two_b2 - inter);
}

// JI > 0.3 test including the |dx| <= B prefilter (get_cliques.py:64-65)
__device__ __forceinline__ bool is_edge(double xa, double ya, double xb, double yb, double B,
                                        double two_b2, double* ji) {
  if (!(fabs(xa - xb) <= B)) return false;
  *ji = jaccard(xa, ya, xb, yb, B, two_b2);
  return *ji > 0.3;
}

// Compare-exchange networks on register arrays (fully unrolled: no scratch).  Batcher's
// odd-even merge sort on the next power of two, comparators that touch the padding (+inf
// slots above N, never moved) dropped; WANT_MID keeps only the comparators the middle
// element(s) depend on (backward liveness from outputs N/2, and N/2 - 1 for even N).  Any
// sorting network yields the same sorted values, so medians are the bubble network's: for
// k = 8 the 28 pair overlaps take 126 compare-exchanges instead of 378.
struct CmpNet {
  int n;
  unsigned char a[256], b[256];
};
template <int N, bool WANT_MID>
constexpr CmpNet make_cmpnet() {
  CmpNet all{}, net{};
  int P = 1;
  while (P < N) P <<= 1;
  for (int p = 1; p < P; p += p)
    for (int k = p; k > 0; k /= 2)
      for (int j = k % p; j + k < P; j += 2 * k)
        for (int i = 0; i < k; ++i)
          if (i + j + k < N && (i + j) / (2 * p) == (i + j + k) / (2 * p)) {
            all.a[all.n] = (unsigned char)(i + j);
            all.b[all.n] = (unsigned char)(i + j + k);
            ++all.n;
          }
  bool need[64] = {};
  for (int i = 0; i < N; ++i) need[i] = !WANT_MID || i == N / 2 || (N % 2 == 0 && i == N / 2 - 1);
  bool keep[256] = {};
  for (int c = all.n - 1; c >= 0; --c)
    if (need[all.a[c]] || need[all.b[c]]) {
      keep[c] = true;
      need[all.a[c]] = need[all.b[c]] = true;
    }
  for (int c = 0; c < all.n; ++c)
    if (keep[c]) {
      net.a[net.n] = all.a[c];
      net.b[net.n] = all.b[c];
      ++net.n;
    }
  return net;
}
template <int N, bool WANT_MID>
struct CmpNetOf {
  static constexpr CmpNet net = make_cmpnet<N, WANT_MID>();
};
// v_min_f64 / v_max_f64 (a total order with -0 < +0 on NaN-free values) and integer min/max
__host__ __device__ __forceinline__ double cmp_lo(double x, double y) { return fmin(x, y); }
__host__ __device__ __forceinline__ double cmp_hi(double x, double y) { return fmax(x, y); }
__host__ __device__ __forceinline__ float cmp_lo(float x, float y) { return fminf(x, y); }
__host__ __device__ __forceinline__ float cmp_hi(float x, float y) { return fmaxf(x, y); }
__host__ __device__ __forceinline__ int cmp_lo(int x, int y) { return x < y ? x : y; }
__host__ __device__ __forceinline__ int cmp_hi(int x, int y) { return x < y ? y : x; }
// two u16 lanes per register (v_pk_min_u16 / v_pk_max_u16): the large-route epilogue's
// clique pairs (rgc_cliques.hip k5_epilogue)
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 cmp_lo(u16x2 x, u16x2 y) { return __builtin_elementwise_min(x, y); }
__device__ __forceinline__ u16x2 cmp_hi(u16x2 x, u16x2 y) { return __builtin_elementwise_max(x, y); }
template <int N, bool WANT_MID, typename T>
__host__ __device__ __forceinline__ void cmpnet_apply(T (&v)[N]) {
  constexpr int n = CmpNetOf<N, WANT_MID>::net.n;
#pragma unroll
  for (int c = 0; c < n; ++c) {
    const int a = CmpNetOf<N, WANT_MID>::net.a[c], b = CmpNetOf<N, WANT_MID>::net.b[c];
    const T x = v[a], y = v[b];
    v[a] = cmp_lo(x, y);
    v[b] = cmp_hi(x, y);
  }
}

// full ascending sort (values only: NaN-free inputs)
template <int N>
__host__ __device__ __forceinline__ void sort_n(double (&v)[N]) {
  cmpnet_apply<N, false>(v);
}
// v[N / 2] (and v[N / 2 - 1] for even N) hold the sorted middle values afterwards
template <int N, typename T>
__host__ __device__ __forceinline__ void mid_n(T (&v)[N]) {
  cmpnet_apply<N, true>(v);
}

// numpy median (numpy/lib/_function_base_impl.py _median): middle value, or the mean of the
// two middle values ((a + b) / 2) for even n; NaN if any value is NaN.
template <int N>
__host__ __device__ __forceinline__ double median_n(double (&v)[N]) {
  bool nan = false;
#pragma unroll
  for (int i = 0; i < N; ++i) nan |= isnan(v[i]);
  if (nan) return NAN;
  mid_n<N>(v);
  if (N & 1) return v[N / 2];
  return (v[N / 2 - 1] + v[N / 2]) / 2.0;
}

__device__ __forceinline__ int pair_index(int j, int l, int k) {  // itertools.combinations
  return j * (2 * k - j - 1) / 2 + (l - j - 1);
}

// Result of the ILP epilogue of one clique (get_cliques.py:169-190).
template <int K>
struct Epi {
  float w, conf;
  int arg;        // picker index of the consensus member
  int8_t ord[K];  // networkx node-iteration order (picker indices)
};

// graph insertion order of a clique's members by their insertion keys (nibble r = member
// index of the r-th node; ties by member index)
template <int K>
__host__ __device__ __forceinline__ uint32_t node_order_ins(const uint64_t (&ins)[K]) {
  uint32_t ord = 0;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    int rk = 0;
#pragma unroll
    for (int q = 0; q < K; ++q) rk += (ins[q] < ins[i] || (ins[q] == ins[i] && q < i)) ? 1 : 0;
    ord |= (uint32_t)i << (4 * rk);
  }
  return ord;
}

// networkx node-iteration order of a clique (nibble r = member index of the r-th node): set
// order = CPython set(sorted(clique)) iteration (2k < |G|), else graph insertion order.
// Needed only on weighted-degree ties or for --multi_out.
template <int K>
__host__ __device__ __forceinline__ uint32_t node_order(const int (&mem)[K], const double (&xs)[K],
                                                     const double (&ys)[K],
                                                     const int64_t (&ids)[K], bool set_order,
                                                     const uint64_t (&ins)[K]) {
  // Sorting is done by ranks (rank_i = number of members ordered before member i), so no
  // private array is ever permuted or dynamically indexed.
  uint32_t inv = 0;   // nibble t = member index at sorted position t
  uint32_t ord = 0;
  if (set_order) {
    // insertion order = sorted (x, y, id); then CPython set iteration order
    uint64_t hs[K];
#pragma unroll
    for (int i = 0; i < K; ++i) {
      int rk = 0;
#pragma unroll
      for (int q = 0; q < K; ++q) {
        const bool lt = (xs[q] < xs[i]) ||
                        (xs[q] == xs[i] && (ys[q] < ys[i] || (ys[q] == ys[i] && mem[q] < mem[i])));
        rk += lt ? 1 : 0;
      }
      inv |= (uint32_t)i << (4 * rk);
    }
    // hashes in insertion (sorted) order: hs[t] = hash of the member at position t
#pragma unroll
    for (int t = 0; t < K; ++t) {
      const int i = (inv >> (4 * t)) & 15;
      double hx = xs[0], hy = ys[0];
      int64_t hid = ids[0];
#pragma unroll
      for (int q = 1; q < K; ++q) {
        const bool h = (i == q);
        hx = h ? xs[q] : hx;
        hy = h ? ys[q] : hy;
        hid = h ? ids[q] : hid;
      }
      hs[t] = pyset::hash_node(hx, hy, hid);
    }
    const uint32_t so = pyset::set_order_packed<K>(hs);
#pragma unroll
    for (int r = 0; r < K; ++r) {
      const int t = (so >> (4 * r)) & 15;
      ord |= ((inv >> (4 * t)) & 15) << (4 * r);
    }
  } else {
    ord = node_order_ins<K>(ins);
  }
  return ord;
}

// conf = f32(median(scores)), w = f32(f64(conf) * median(JIs)) (get_cliques.py:169-170,186-190)
template <int K>
__host__ __device__ __forceinline__ void epi_weights(const double (&ji)[K][K], const double (&s)[K],
                                                     float* w, float* conf) {
  double sc[K];
#pragma unroll
  for (int i = 0; i < K; ++i) sc[i] = s[i];
  const double cf = median_n<K>(sc);
  constexpr int NE = K * (K - 1) / 2;
  double ej[NE];
  {
    int t = 0;
#pragma unroll
    for (int a = 0; a < K; ++a)
#pragma unroll
      for (int b = a + 1; b < K; ++b) ej[t++] = ji[a][b];
  }
  const double med = median_n<NE>(ej);
  const float conf32 = (float)cf;
  *conf = conf32;
  *w = (float)((double)conf32 * med);
}

// weighted degrees: JIs to the other members summed in increasing picker order (networkx
// DegreeView over adjacency insertion order; naive left-to-right f64 sum, :182-183); returns
// the first maximal member and the bitmask of all maximal members
template <int K>
__host__ __device__ __forceinline__ int epi_degree_max(const double (&ji)[K][K], uint32_t* top) {
  double deg[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    double d = 0.0;
#pragma unroll
    for (int q = 0; q < K; ++q) {
      if (q == i) continue;
      d = d + (q < i ? ji[q][i] : ji[i][q]);
    }
    deg[i] = d;
  }
  double dmax = deg[0];
  int arg = 0;
#pragma unroll
  for (int i = 1; i < K; ++i)
    if (deg[i] > dmax) { dmax = deg[i]; arg = i; }
  uint32_t t = 0;
#pragma unroll
  for (int i = 0; i < K; ++i) t |= (deg[i] == dmax ? 1u : 0u) << i;
  *top = t;
  return arg;
}

// consensus among tied maximal members: the first of them in node-iteration order
template <int K>
__host__ __device__ __forceinline__ int epi_tie_arg(uint32_t top, uint32_t ord) {
  int arg = 0;
  bool found = false;
#pragma unroll
  for (int r = 0; r < K; ++r) {
    const int mi = (ord >> (4 * r)) & 15;
    if (!found && ((top >> mi) & 1u)) { arg = mi; found = true; }
  }
  return arg;
}

// mem[i]  : any box handle, only used to break (x, y) ties by id order (monotone in handle)
// ji[i][j]: JI of members i < j;  s[i]: scores;  xs/ys: coordinates;  ids: global box ids
// set_order: networkx iterates set(sorted(clique)) (2k < |G|) vs graph insertion order;
// ins[i]  : graph insertion key of member i (used only when !set_order)
// All private arrays are indexed with compile-time indices only (no scratch).
template <int K>
__host__ __device__ __forceinline__ void epilogue(const int (&mem)[K], const double (&ji)[K][K],
                                         const double (&s)[K], const double (&xs)[K],
                                         const double (&ys)[K], const int64_t (&ids)[K],
                                         bool set_order, const uint64_t (&ins)[K], bool need_order,
                                         Epi<K>& out) {
  epi_weights<K>(ji, s, &out.w, &out.conf);
  uint32_t top;
  int arg = epi_degree_max<K>(ji, &top);
  const bool tie = (top & (top - 1)) != 0;
  if (tie || need_order) {
    const uint32_t ord = node_order<K>(mem, xs, ys, ids, set_order, ins);
    if (tie) arg = epi_tie_arg<K>(top, ord);
#pragma unroll
    for (int i = 0; i < K; ++i) out.ord[i] = (int8_t)((ord >> (4 * i)) & 15);
  }
  out.arg = arg;
}

}  // namespace rgc
