// Probe: do SALU, LDS and exec-mask instructions take issue slots from the VALU on gfx950?
// At 8 waves per SIMD (256-thread workgroups, 8 per CU), each variant's loop holds 32 VALU
// (v_add_u32, independent) plus a mix of other instructions; the SIMD cycles per loop
// iteration say whether they issue beside the VALU or in its place.
//   M0: 32 v_add                      M1: + 32 s_add (independent SGPR chains)
//   M2: + 16 divergent one-statement ifs (the compiler's exec-mask bookkeeping: s_and_saveexec,
//       s_or exec, branches)
//   M3: + 8 LDS reads (ds_read_b32, the compiler's waits)   M4: + 16 s_nop 0
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                              \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);      \
      return 1;                                                             \
    }                                                                       \
  } while (0)

constexpr int ITERS = 512;

#define V4(a, b, c, d, x)                                     \
  asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(x));    \
  asm volatile("v_add_u32 %0, %0, %1" : "+v"(b) : "v"(x));    \
  asm volatile("v_add_u32 %0, %0, %1" : "+v"(c) : "v"(x));    \
  asm volatile("v_add_u32 %0, %0, %1" : "+v"(d) : "v"(x));
#define S4(a, b, c, d, x)                                     \
  asm volatile("s_add_u32 %0, %0, %1" : "+s"(a) : "s"(x));    \
  asm volatile("s_add_u32 %0, %0, %1" : "+s"(b) : "s"(x));    \
  asm volatile("s_add_u32 %0, %0, %1" : "+s"(c) : "s"(x));    \
  asm volatile("s_add_u32 %0, %0, %1" : "+s"(d) : "s"(x));

template <int MODE>
__global__ __launch_bounds__(256) void k_mix(unsigned* out, unsigned long long* stamps) {
  __shared__ unsigned lds[256 * 8];
  for (int i = threadIdx.x; i < 256 * 8; i += 256) lds[i] = i;
  __syncthreads();
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  unsigned a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  unsigned s0 = blockIdx.x, s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3;
  const unsigned sx = __builtin_amdgcn_readfirstlane(blockIdx.x | 1);
  const unsigned x = blockIdx.x | 1;
  unsigned r0 = 0, r1 = 0;
  const unsigned* lp = lds + threadIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      V4(a0, a1, a2, a3, x)
      if (MODE == 1) { S4(s0, s1, s2, s3, sx) }
      if (MODE == 2) {   // compiler-generated divergence bookkeeping around two one-lane-set blocks
        if ((a0 & 1u) != 0u) r0 += x;
        if ((a1 & 2u) != 0u) r1 += x;
      }
      if (MODE == 3) r0 += lp[256 * ((it + g) & 7)];
      if (MODE == 4) asm volatile("s_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0");
      V4(a4, a5, a6, a7, x)
      if (MODE == 1) { S4(s0, s1, s2, s3, sx) }
      if (MODE == 2) {
        if ((a4 & 1u) != 0u) r0 += x;
        if ((a5 & 2u) != 0u) r1 += x;
      }
      if (MODE == 3) r1 += lp[256 * ((it + g + 3) & 7)];
      if (MODE == 4) asm volatile("s_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0");
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ s0 ^ s1 ^ s2 ^ s3 ^ r0 ^ r1;
  if (threadIdx.x == 0) stamps[blockIdx.x] = t1 - t0;
}

template <int MODE>
static int run(int cus, unsigned* out, unsigned long long* st, int wps, const char* name) {
  const int nb = cus * wps;   // 4 waves per block: wps waves per SIMD
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  float best = 1e9f;
  for (int rep = 0; rep < 4; ++rep) {
    CHK(hipEventRecord(e0));
    k_mix<MODE><<<nb, 256>>>(out, st);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    if (rep > 0 && ms < best) best = ms;
  }
  unsigned long long h[4096];
  CHK(hipMemcpy(h, st, (size_t)nb * 8, hipMemcpyDeviceToHost));
  double cyc = 0;
  for (int i = 0; i < nb; ++i) cyc += (double)h[i];
  cyc /= nb;
  // per SIMD: wps waves x ITERS iterations x 32 VALU
  printf("{\"mode\": \"%s\", \"waves_per_simd\": %d, \"wall_ms\": %.5f, \"loop_cycles_per_wave\": %.0f, "
         "\"simd_cycles_per_valu\": %.3f}\n",
         name, wps, best, cyc, cyc / ((double)wps * ITERS * 32));
  fflush(stdout);
  return 0;
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : -1;   // -1: every mode
  hipDeviceProp_t pr;
  CHK(hipGetDeviceProperties(&pr, 0));
  const int cus = pr.multiProcessorCount;
  unsigned* out = nullptr;
  unsigned long long* st = nullptr;
  CHK(hipMalloc(&out, (size_t)cus * 8 * 256 * 4));
  CHK(hipMalloc(&st, (size_t)cus * 8 * 8));
  for (int wps : {2, 8}) {
    if ((mode < 0 || mode == 0) && run<0>(cus, out, st, wps, "valu32")) return 1;
    if ((mode < 0 || mode == 1) && run<1>(cus, out, st, wps, "valu32+salu32")) return 1;
    if ((mode < 0 || mode == 2) && run<2>(cus, out, st, wps, "valu32+divergent_if16")) return 1;
    if ((mode < 0 || mode == 3) && run<3>(cus, out, st, wps, "valu32+ds_read8")) return 1;
    if ((mode < 0 || mode == 4) && run<4>(cus, out, st, wps, "valu32+s_nop32")) return 1;
  }
  return 0;
}
