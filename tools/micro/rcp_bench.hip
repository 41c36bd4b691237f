// Micro-benchmark: v_rcp_f64 on gfx950 -- dependent-chain latency (cycles) of the raw
// reciprocal and of the reciprocal with one / two Newton steps, and the accuracy of each
// against the correctly rounded 1/d over 4M random d (log-uniform in [1e-8, 1e8], both signs).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <vector>

template <int NR>
__device__ inline double rcp_n(double d) {
  double r = __builtin_amdgcn_rcp(d);
  if (NR >= 1) r = fma(r, fma(-d, r, 1.0), r);
  if (NR >= 2) r = fma(r, fma(-d, r, 1.0), r);
  return r;
}

template <int NR>
__global__ void k_lat(double* out, unsigned long long* cyc, double x0, int iters) {
  double a = x0 + threadIdx.x * 1e-3;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i += 16) {
#pragma unroll
    for (int u = 0; u < 16; u++) a = rcp_n<NR>(a);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) *cyc = (t1 - t0) / iters;
}

// issue rate: 8 independent FMA chains in one wave (cycles per v_fma_f64 / v_fma_f32)
template <typename T>
__global__ void k_thr(T* out, unsigned long long* cyc, int iters) {
  T a[8];
#pragma unroll
  for (int j = 0; j < 8; j++) a[j] = (T)(threadIdx.x + j);
  const T b = (T)1.0000001, c = (T)1e-9;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) a[j] = __builtin_fma(a[j], b, c);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  T s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s += a[j];
  out[threadIdx.x] = s;
  if (threadIdx.x == 0) *cyc = (t1 - t0) * 100 / ((unsigned long long)iters * 8);
}

template <int NR>
__global__ void k_acc(const double* d, double* r, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) r[i] = rcp_n<NR>(d[i]);
}

int main() {
  double* dout;
  unsigned long long* c;
  (void)hipMalloc(&dout, 1024 * 8);
  (void)hipMalloc(&c, 8);
  for (int nr = 0; nr < 3; nr++) {
    unsigned long long h = 0;
    for (int rep = 0; rep < 2; rep++) {
      if (nr == 0) hipLaunchKernelGGL(k_lat<0>, dim3(1), dim3(64), 0, 0, dout, c, 1.5, 4096);
      if (nr == 1) hipLaunchKernelGGL(k_lat<1>, dim3(1), dim3(64), 0, 0, dout, c, 1.5, 4096);
      if (nr == 2) hipLaunchKernelGGL(k_lat<2>, dim3(1), dim3(64), 0, 0, dout, c, 1.5, 4096);
      (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    }
    printf("{\"what\": \"latency\", \"newton_steps\": %d, \"cycles_per_dependent_rcp\": %llu}\n", nr, h);
  }
  {
    unsigned long long h = 0;
    float* fo;
    (void)hipMalloc(&fo, 1024 * 4);
    for (int rep = 0; rep < 2; rep++) {
      hipLaunchKernelGGL(k_thr<double>, dim3(1), dim3(64), 0, 0, dout, c, 4096);
      (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    }
    printf("{\"what\": \"issue\", \"op\": \"v_fma_f64\", \"cycles_x100_per_wave_instr\": %llu}\n", h);
    for (int rep = 0; rep < 2; rep++) {
      hipLaunchKernelGGL(k_thr<float>, dim3(1), dim3(64), 0, 0, fo, c, 4096);
      (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    }
    printf("{\"what\": \"issue\", \"op\": \"v_fma_f32\", \"cycles_x100_per_wave_instr\": %llu}\n", h);
  }
  const int n = 1 << 22;
  std::vector<double> hd(n), hr(n);
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < n; i++) {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    const double u = (double)(s >> 11) / 9007199254740992.0;  // [0, 1)
    hd[i] = std::pow(10.0, -8.0 + 16.0 * u) * ((s & 1) ? -1.0 : 1.0);
  }
  double *dd, *dr;
  (void)hipMalloc(&dd, n * 8);
  (void)hipMalloc(&dr, n * 8);
  (void)hipMemcpy(dd, hd.data(), n * 8, hipMemcpyHostToDevice);
  for (int nr = 0; nr < 3; nr++) {
    if (nr == 0) hipLaunchKernelGGL(k_acc<0>, dim3(n / 256), dim3(256), 0, 0, dd, dr, n);
    if (nr == 1) hipLaunchKernelGGL(k_acc<1>, dim3(n / 256), dim3(256), 0, 0, dd, dr, n);
    if (nr == 2) hipLaunchKernelGGL(k_acc<2>, dim3(n / 256), dim3(256), 0, 0, dd, dr, n);
    (void)hipMemcpy(hr.data(), dr, n * 8, hipMemcpyDeviceToHost);
    double maxrel = 0;
    long long exact = 0;
    for (int i = 0; i < n; i++) {
      const double ref = 1.0 / hd[i];
      const double rel = std::fabs(hr[i] - ref) / std::fabs(ref);
      maxrel = rel > maxrel ? rel : maxrel;
      exact += hr[i] == ref;
    }
    printf("{\"what\": \"accuracy\", \"newton_steps\": %d, \"max_rel_err\": %.3e, \"correctly_rounded_frac\": %.6f}\n", nr,
           maxrel, (double)exact / n);
  }
  return 0;
}
