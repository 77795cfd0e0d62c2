// Probe: workgroups per CU for a 512-thread kernel as the dynamic LDS size grows, from the
// HIP occupancy API and measured (a fixed-duration spin kernel: concurrency = WG time x WGs
// / wall time / CUs).  Reveals the LDS allocation granularity on this GPU.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(512) void k(int* p, long long spin) {
  extern __shared__ int s[];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < spin) __builtin_amdgcn_s_sleep(2);
  if (p) p[threadIdx.x] = s[511 - threadIdx.x];
}
int main() {
  hipFuncSetAttribute(reinterpret_cast<const void*>(&k), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  int prev = -1;
  for (int b = 2048; b <= 160 * 1024; b += 16) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k, 512, b) != hipSuccess) { printf("err at %d\n", b); return 1; }
    if (nb != prev) { printf("api: lds %6d -> %d WG/CU\n", b, nb); prev = nb; }
  }
  hipDeviceProp_t pr;
  hipGetDeviceProperties(&pr, 0);
  const int cus = pr.multiProcessorCount;
  const long long spin = 2000;   // s_memrealtime is 100 MHz: 20 us
  const int sizes[] = {32768, 40960, 40961, 41984, 53248, 53680, 53760, 53761, 53904, 54272, 54613, 81920, 81921};
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int b : sizes) {
    const int nblk = cus * 16;
    hipLaunchKernelGGL(k, dim3(nblk), dim3(512), b, 0, nullptr, spin);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(nblk), dim3(512), b, 0, nullptr, spin);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("measured: lds %6d  %.3f ms  -> %.2f WG/CU concurrent\n", b, ms, 16 * 0.020 / ms);
  }
  return 0;
}
