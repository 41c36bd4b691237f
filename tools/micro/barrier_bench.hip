// Micro-benchmark: cost of a workgroup barrier round on gfx950 (cycles per
// iteration, s_memtime), with and without an LDS write->read dependency.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void k(unsigned long long* out, int iters) {
  __shared__ double buf[2048];
  double acc = threadIdx.x;
  buf[threadIdx.x] = acc;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
    if (MODE == 1) {
      buf[(threadIdx.x + i) & 2047] = acc;
    }
    if (MODE == 2) {
      if (threadIdx.x == (i & 1023)) buf[i & 2047] = acc;
    }
    __syncthreads();
    if (MODE >= 1) acc += buf[(i * 7) & 2047];
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = (t1 - t0) / iters;
  if (acc == -1.0) out[1] = 1;
}

int main() {
  unsigned long long* d;
  hipMalloc(&d, 16);
  const int threads[] = {64, 256, 512, 1024};
  for (int m = 0; m < 3; m++)
    for (int t : threads) {
      unsigned long long h = 0;
      for (int rep = 0; rep < 2; rep++) {
        if (m == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(t), 0, 0, d, 1000);
        if (m == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(t), 0, 0, d, 1000);
        if (m == 2) hipLaunchKernelGGL(k<2>, dim3(1), dim3(t), 0, 0, d, 1000);
        hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
      }
      printf("mode %d threads %4d: %llu cycles/iter\n", m, t, h);
    }
  return 0;
}
