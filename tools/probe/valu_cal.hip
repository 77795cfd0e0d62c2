// Probe: what SQ_ACTIVE_INST_VALU / SQ_INSTS_VALU mean in cycles on gfx950 (VERDICT r04 item 1:
// is a wave64 VALU instruction 4 or 2 SIMD cycles?).  A kernel of independent v_add_u32 (8
// accumulators per lane, asm volatile so nothing folds) runs at 1, 2, 4 and 8 waves per SIMD
// (256-thread workgroups, blocks = CUs x waves/SIMD); each launch reports its wall time and the
// in-kernel clock (s_memtime / s_memrealtime, median-free: one wave's stamps), so
//   cycles per instruction per SIMD = wall x clock / (instructions issued per SIMD).
// Run it under rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
// (tools/gpu_valu_cal.sh) and compare the counters to the known instruction counts.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHK(x)                                                                 \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);         \
      return 1;                                                                \
    }                                                                          \
  } while (0)

constexpr int ITERS = 4096;   // 8 v_add_u32 per iteration
constexpr int UNROLL = 8;

template <bool DEP>
__global__ __launch_bounds__(256) void k_valu(unsigned* out, unsigned long long* stamps) {
  unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  unsigned a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  const unsigned b = blockIdx.x | 1;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < ITERS / UNROLL; ++i) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      if (DEP) {   // one dependent chain: latency-bound
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(b));
      } else {
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a1) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a2) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a3) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a4) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a5) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a6) : "v"(b));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(a7) : "v"(b));
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (threadIdx.x == 0 && stamps) {
    stamps[2 * blockIdx.x] = t1 - t0;
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int main() {
  hipDeviceProp_t pr;
  CHK(hipGetDeviceProperties(&pr, 0));
  const int cus = pr.multiProcessorCount;
  const int maxb = cus * 8;
  unsigned* out = nullptr;
  unsigned long long* st = nullptr;
  CHK(hipMalloc(&out, (size_t)maxb * 256 * 4));
  CHK(hipMalloc(&st, (size_t)maxb * 16));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  std::vector<unsigned long long> h(2 * maxb);
  printf("{\"cus\": %d, \"iters\": %d, \"valu_per_wave_loop\": %d, \"runs\": [\n", cus, ITERS,
         ITERS);
  bool first = true;
  for (int dep = 0; dep < 2; ++dep) {
    for (int wps : {1, 2, 4, 8}) {
      const int nb = cus * wps;   // 4 waves per 256-thread block: wps waves per SIMD
      for (int rep = 0; rep < 3; ++rep) {   // warm-up, then two timed launches
        CHK(hipEventRecord(e0));
        if (dep)
          k_valu<true><<<nb, 256>>>(out, st);
        else
          k_valu<false><<<nb, 256>>>(out, st);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms = 0;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        CHK(hipMemcpy(h.data(), st, (size_t)nb * 16, hipMemcpyDeviceToHost));
        double cyc = 0, real = 0;
        for (int i = 0; i < nb; ++i) {
          cyc += h[2 * i];
          real += h[2 * i + 1];
        }
        cyc /= nb;
        real /= nb;
        const double ghz = cyc / (real * 10.0);   // s_memrealtime: 100 MHz
        const double insts_per_simd = (double)wps * ITERS;   // loop VALU per SIMD
        printf("%s {\"dep\": %d, \"waves_per_simd\": %d, \"rep\": %d, \"wall_ms\": %.5f, "
               "\"loop_cycles_per_wave\": %.0f, \"clock_ghz\": %.3f, "
               "\"loop_cycles_per_valu_per_simd\": %.4f}\n",
               first ? " " : ",", dep, wps, rep, ms, cyc, ghz, cyc / insts_per_simd);
        first = false;
      }
    }
  }
  printf("]}\n");
  CHK(hipFree(out));
  CHK(hipFree(st));
  return 0;
}
