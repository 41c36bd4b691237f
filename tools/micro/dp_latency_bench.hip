// Micro-benchmark: latency (cycles) of dependent FP64 ops on gfx950, and of
// the correctly rounded sqrt / division sequences.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ void k(double* out, unsigned long long* cyc, double x0, int iters) {
  double a = x0 + threadIdx.x, b = 1.0000001;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i += 16) {
#pragma unroll
   for (int u = 0; u < 16; u++) {
    if (OP == 0) a = a + b;
    if (OP == 1) a = a * b;
    if (OP == 2) a = __builtin_fma(a, b, 1e-9);
    if (OP == 3) a = sqrt(a) + 1.0;
    if (OP == 4) a = 1.0 / a + 1.0;
    if (OP == 5) a = (float)a + 1.0f;
   }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) *cyc = (t1 - t0) / iters;
}

int main() {
  double* d;
  unsigned long long* c;
  (void)hipMalloc(&d, 1024 * 8);
  (void)hipMalloc(&c, 8);
  const char* names[] = {"add_f64", "mul_f64", "fma_f64", "sqrt_f64+add", "div_f64+add", "f32 cvt+add"};
  for (int op = 0; op < 6; op++) {
    unsigned long long h = 0;
    for (int rep = 0; rep < 2; rep++) {
      switch (op) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 0, 0, d, c, 1.5, 4096); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 0, 0, d, c, 1.5, 4096); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 0, 0, d, c, 1.5, 4096); break;
        case 3: hipLaunchKernelGGL(k<3>, dim3(1), dim3(64), 0, 0, d, c, 1.5, 4096); break;
        case 4: hipLaunchKernelGGL(k<4>, dim3(1), dim3(64), 0, 0, d, c, 1.5, 4096); break;
        case 5: hipLaunchKernelGGL(k<5>, dim3(1), dim3(64), 0, 0, d, c, 1.5, 4096); break;
      }
      (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    }
    printf("%-14s %llu cycles per dependent op (1 wave)\n", names[op], h);
  }
  return 0;
}
