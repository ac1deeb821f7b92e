// Throughput of the FP64 instructions of the FP64 mulmod on gfx950:
// v_fma_f64 chains vs v_rndne_f64 chains vs the magic-number rint.
// hipcc --offload-arch=gfx950 -O3 scripts/ubench_rndne.hip -o scripts/ubench_rndne
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)
constexpr int ITERS = 4096, CH = 8;

__global__ void k_fma(double *o, double s)
{
  double x[CH];
  for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c * s;
  for (int i = 0; i < ITERS; i++)
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = __fma_rn(x[c], s, 0.5);
  double r = 0;
  for (int c = 0; c < CH; c++) r += x[c];
  o[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_rndne(double *o, double s)
{
  double x[CH];
  for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c * s;
  for (int i = 0; i < ITERS; i++)
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = rint(x[c] * s);  // mul + rndne
  double r = 0;
  for (int c = 0; c < CH; c++) r += x[c];
  o[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_magic(double *o, double s)
{
  double x[CH];
  for (int c = 0; c < CH; c++) x[c] = threadIdx.x + c * s;
  for (int i = 0; i < ITERS; i++)
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = __fma_rn(x[c], s, 0x1.8p52) - 0x1.8p52;  // fma + add
  double r = 0;
  for (int c = 0; c < CH; c++) r += x[c];
  o[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main()
{
  double *o;
  CK(hipMalloc(&o, 1 << 24));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int blocks = 256 * 8, th = 256;
  auto run = [&](const char *name, auto k, double per_iter_ops) {
    hipLaunchKernelGGL(k, dim3(blocks), dim3(th), 0, 0, o, 1.0000001);
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(th), 0, 0, o, 1.0000001);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double lane_ops = 5.0 * blocks * th * (double)ITERS * CH * per_iter_ops;
    printf("%-8s %8.3f ms  %.3e lane-instr/s\n", name, ms, lane_ops / (ms * 1e-3));
  };
  run("fma", k_fma, 1);
  run("mul+rnd", k_rndne, 2);
  run("fma+add", k_magic, 2);
  return 0;
}
