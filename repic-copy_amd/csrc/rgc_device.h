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
// reference calc_jaccard (get_cliques.py:40-46), same f64 op order, no FMA.
__device__ __forceinline__ double jaccard(double x, double y, double a, double b, double B,
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

// numpy median (numpy/lib/_function_base_impl.py _median): middle value, or the mean of the
// two middle values ((a + b) / 2) for even n; NaN if any value is NaN.  Sorting network on a
// register array (fully unrolled: no scratch).
template <int N>
__device__ __forceinline__ double median_n(double (&v)[N]) {
  bool nan = false;
#pragma unroll
  for (int i = 0; i < N; ++i) nan |= isnan(v[i]);
  if (nan) return NAN;
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < N - 1 - i; ++j) {
      const double a = v[j], b = v[j + 1];
      v[j] = fmin(a, b);
      v[j + 1] = fmax(a, b);
    }
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

// mem[i]  : any box handle, only used to break (x, y) ties by id order (monotone in handle)
// ji[i][j]: JI of members i < j;  s[i]: scores;  xs/ys: coordinates;  ids: global box ids
// set_order: networkx iterates set(sorted(clique)) (2k < |G|) vs graph insertion order;
// ins[i]  : graph insertion key of member i (used only when !set_order)
template <int K>
__device__ __forceinline__ void epilogue(const int (&mem)[K], const double (&ji)[K][K],
                                         const double (&s)[K], const double (&xs)[K],
                                         const double (&ys)[K], const int64_t (&ids)[K],
                                         bool set_order, const uint64_t* ins, bool need_order,
                                         Epi<K>& out) {
  double sc[K];
#pragma unroll
  for (int i = 0; i < K; ++i) sc[i] = s[i];
  const double conf = median_n<K>(sc);
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
  const float conf32 = (float)conf;
  out.conf = conf32;
  out.w = (float)((double)conf32 * med);
  // weighted degree: JIs to the other members summed in increasing picker order
  // (networkx DegreeView over adjacency insertion order; naive left-to-right f64 sum)
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
  int nmax = 1, arg = 0;
#pragma unroll
  for (int i = 1; i < K; ++i) {
    if (deg[i] > dmax) { dmax = deg[i]; nmax = 1; arg = i; }
    else if (deg[i] == dmax) ++nmax;
  }
  if (nmax > 1 || need_order) {
    int8_t ord[K];
#pragma unroll
    for (int i = 0; i < K; ++i) ord[i] = (int8_t)i;
    if (set_order) {
      // insertion order = sorted (x, y, id); then CPython set iteration order
      int8_t srt[K];
#pragma unroll
      for (int i = 0; i < K; ++i) srt[i] = (int8_t)i;
      for (int i = 1; i < K; ++i) {
        const int8_t t = srt[i];
        int q = i - 1;
        while (q >= 0) {
          const int u = srt[q];
          const bool gt = (xs[u] > xs[t]) ||
                          (xs[u] == xs[t] && (ys[u] > ys[t] || (ys[u] == ys[t] && mem[u] > mem[t])));
          if (!gt) break;
          srt[q + 1] = srt[q];
          --q;
        }
        srt[q + 1] = t;
      }
      uint64_t hs[K];
      for (int i = 0; i < K; ++i) hs[i] = pyset::hash_node(xs[srt[i]], ys[srt[i]], ids[srt[i]]);
      int8_t so[K];
      pyset::set_order(hs, K, so);
      for (int i = 0; i < K; ++i) ord[i] = srt[so[i]];
    } else {
      for (int i = 1; i < K; ++i) {
        const int8_t t = ord[i];
        int q = i - 1;
        while (q >= 0 && ins[ord[q]] > ins[t]) { ord[q + 1] = ord[q]; --q; }
        ord[q + 1] = t;
      }
    }
    if (nmax > 1) {
      for (int i = 0; i < K; ++i)
        if (deg[ord[i]] == dmax) { arg = ord[i]; break; }
    }
#pragma unroll
    for (int i = 0; i < K; ++i) out.ord[i] = ord[i];
  }
  out.arg = arg;
}

}  // namespace rgc
