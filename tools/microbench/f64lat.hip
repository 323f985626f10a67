// micro-benchmark: dependent / independent f64 add and mul latency and issue (diagnostics only)
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void dep_add(double *out, double a, double b, int n, unsigned long long *clk) {
  double x = a + threadIdx.x;
  unsigned long long t0 = clock64();
  for (int i = 0; i < n; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++) x = x + b;
  }
  unsigned long long t1 = clock64();
  out[threadIdx.x + blockIdx.x * blockDim.x] = x;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void dep_mul(double *out, double a, double b, int n, unsigned long long *clk) {
  double x = a + threadIdx.x;
  unsigned long long t0 = clock64();
  for (int i = 0; i < n; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++) x = x * b;
  }
  unsigned long long t1 = clock64();
  out[threadIdx.x + blockIdx.x * blockDim.x] = x;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void ind_add(double *out, double a, double b, int n, unsigned long long *clk) {
  double x[8];
  for (int k = 0; k < 8; k++) x[k] = a + threadIdx.x + k;
  unsigned long long t0 = clock64();
  for (int i = 0; i < n; i++) {
#pragma unroll
    for (int u = 0; u < 2; u++)
#pragma unroll
      for (int k = 0; k < 8; k++) x[k] = x[k] + b;
  }
  unsigned long long t1 = clock64();
  double s = 0;
  for (int k = 0; k < 8; k++) s += x[k];
  out[threadIdx.x + blockIdx.x * blockDim.x] = s;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void dep_lds(double *out, int n, unsigned long long *clk) {
  __shared__ double s[256];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  int idx = threadIdx.x;
  double x = 0;
  unsigned long long t0 = clock64();
  for (int i = 0; i < n * 16; i++) {
    x = s[idx];
    idx = ((int)x + 1) & 255;
  }
  unsigned long long t1 = clock64();
  out[threadIdx.x + blockIdx.x * blockDim.x] = x;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
int main() {
  double *out;
  unsigned long long *clk, h[1];
  hipMalloc(&out, 1 << 20);
  hipMalloc(&clk, 8 * 1024);
  const int n = 1000;
  for (int wv = 1; wv <= 16; wv *= 2) {
    // one block of wv waves (all on different SIMDs up to 4)
    hipLaunchKernelGGL(dep_add, dim3(1), dim3(64 * wv), 0, 0, out, 1.0, 1e-9, n, clk);
    hipDeviceSynchronize();
    hipMemcpy(h, clk, 8, hipMemcpyDeviceToHost);
    printf("waves %d dep add: %.2f clk/op\n", wv, (double)h[0] / (16.0 * n));
    hipLaunchKernelGGL(dep_mul, dim3(1), dim3(64 * wv), 0, 0, out, 1.0, 1.0000001, n, clk);
    hipDeviceSynchronize();
    hipMemcpy(h, clk, 8, hipMemcpyDeviceToHost);
    printf("waves %d dep mul: %.2f clk/op\n", wv, (double)h[0] / (16.0 * n));
    hipLaunchKernelGGL(ind_add, dim3(1), dim3(64 * wv), 0, 0, out, 1.0, 1e-9, n, clk);
    hipDeviceSynchronize();
    hipMemcpy(h, clk, 8, hipMemcpyDeviceToHost);
    printf("waves %d indep add (8 chains): %.2f clk/op\n", wv, (double)h[0] / (16.0 * n));
  }
  hipLaunchKernelGGL(dep_lds, dim3(1), dim3(64), 0, 0, out, n, clk);
  hipDeviceSynchronize();
  hipMemcpy(h, clk, 8, hipMemcpyDeviceToHost);
  printf("dep ds_read_b64 chain: %.2f clk/op\n", (double)h[0] / (16.0 * n));
  return 0;
}
