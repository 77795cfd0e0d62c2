// rgc_score.hip — particle-set scoring: the raster/reduce of score_detections.
//
// Reference repic/utils/score_detections.py:16-48 (get_segmentation_scores): every ground-
// truth and every picked box (above the confidence threshold) is painted into an int16
// (H x W) mask with numpy slice assignment; the scores are sum(pckr), sum(gt * pckr) and
// sum(gt).  Here the masks never exist in HBM: each workgroup owns one tile of the image
// (R rows x TW 64-pixel words, two 1-bit masks in LDS), paints the part of every box that
// falls into it with LDS atomic ORs, and reduces three popcounts into the pair's counters.
// The host normalises each box to its numpy slice bounds (Python slice.indices semantics:
// negative starts wrap, everything clamps to the mask), so a box is the pixel rectangle
// [r0, r1) x [c0, c1) with r0 < r1, c0 < c1.
#include "rgc_kernels.h"

namespace rgc {

constexpr int SC_WG = 256;
constexpr int SC_WORDS = 2048;   // 64-bit words per mask per tile (16 KB): 32 KB of LDS per WG

__device__ __forceinline__ void paint(uint64_t* m, int tr0, int tw0, int R, int TW, int4 b,
                                      int lane) {
  // overlap of box b with the tile, in tile-local rows and pixel columns
  const int pr0 = max(b.x, tr0), pr1 = min(b.y, tr0 + R);
  const int pc0 = max(b.z, tw0 * 64), pc1 = min(b.w, (tw0 + TW) * 64);
  if (pr0 >= pr1 || pc0 >= pc1) return;
  const int w0 = pc0 / 64, w1 = (pc1 - 1) / 64;   // inclusive word range
  const int nw = w1 - w0 + 1;
  const int items = (pr1 - pr0) * nw;
  for (int it = lane; it < items; it += 64) {
    const int r = pr0 + it / nw, w = w0 + it % nw;
    uint64_t bits = ~0ull;
    if (w == w0) bits &= ~0ull << (pc0 & 63);
    if (w == w1) bits &= ~0ull >> (63 - ((pc1 - 1) & 63));
    atomicOr(reinterpret_cast<unsigned long long*>(&m[(r - tr0) * TW + (w - tw0)]),
             (unsigned long long)bits);
  }
}

// One workgroup per (pair, tile).  Boxes of the pair are scanned in chunks of SC_WG: the ones
// touching the tile are compacted into LDS, then each wavefront paints whole boxes (lanes
// over the box's (row, word) items, so a 180 x 180 box is ~3 items per lane).
__global__ __launch_bounds__(SC_WG) void k_score_raster(ScoreArgs A) {
  __shared__ uint64_t m[2][SC_WORDS];
  __shared__ int list[SC_WG];
  __shared__ int nlist;
  __shared__ unsigned long long red[3][SC_WG / 64];
  const int t = blockIdx.x;
  const int p = A.tile_pair[t];
  const int tr0 = A.tile_r0[t], tw0 = A.tile_w0[t];
  const int R = A.R, TW = A.TW;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  for (int i = tid; i < 2 * SC_WORDS; i += SC_WG) (&m[0][0])[i] = 0;
  const int tc0 = tw0 * 64, tc1 = (tw0 + TW) * 64;
  for (int which = 0; which < 2; ++which) {
    const int64_t b0 = which ? A.pk_off[p] : A.gt_off[p];
    const int64_t b1 = which ? A.pk_off[p + 1] : A.gt_off[p + 1];
    for (int64_t c0 = b0; c0 < b1; c0 += SC_WG) {
      if (tid == 0) nlist = 0;
      __syncthreads();
      const int64_t i = c0 + tid;
      if (i < b1) {
        const int4 b = A.boxes[i];
        if (b.x < tr0 + R && b.y > tr0 && b.z < tc1 && b.w > tc0)
          list[atomicAdd(&nlist, 1)] = (int)(i - c0);
      }
      __syncthreads();
      const int n = nlist;
      for (int j = wv; j < n; j += SC_WG / 64) paint(m[which], tr0, tw0, R, TW, A.boxes[c0 + list[j]], lane);
      __syncthreads();
    }
  }
  unsigned long long g = 0, k = 0, tp = 0;
  for (int i = tid; i < R * TW; i += SC_WG) {
    const uint64_t a = m[0][i], b = m[1][i];
    g += __popcll(a);
    k += __popcll(b);
    tp += __popcll(a & b);
  }
  for (int o = 32; o > 0; o >>= 1) {
    g += __shfl_xor(g, o, 64);
    k += __shfl_xor(k, o, 64);
    tp += __shfl_xor(tp, o, 64);
  }
  if (lane == 0) { red[0][wv] = g; red[1][wv] = k; red[2][wv] = tp; }
  __syncthreads();
  if (tid < 3) {
    unsigned long long s = 0;
    for (int w = 0; w < SC_WG / 64; ++w) s += red[tid][w];
    if (s) atomicAdd(&A.counts[3 * p + tid], s);
  }
}

int score_tile_words() { return SC_WORDS; }

void launch_score_raster(hipStream_t stream, int n_tiles, const ScoreArgs& A) {
  if (n_tiles > 0)
    hipLaunchKernelGGL(k_score_raster, dim3(n_tiles), dim3(SC_WG), 0, stream, A);
}

}  // namespace rgc
