// Throughput of the basis-conversion term on gfx950: 128-bit integer MAC vs
// exact FP64 term (rint vs magic-number rounding), plus single-instruction
// rates (v_rndne_f64, v_mul_f64).  8 independent chains per thread.
// hipcc --offload-arch=gfx950 -O3 scripts/ubench_fbc.hip -o scripts/ubench_fbc
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#define IT 256
#define CH 8

__global__ void k_u128(uint64_t *io, const uint64_t *c, uint64_t q, uint64_t qn)
{
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t y[CH];
  for (int k = 0; k < CH; k++) y[k] = io[t * CH + k];
  for (int it = 0; it < IT; it++) {
    const uint64_t c0 = c[it & 63], c1 = c[(it + 1) & 63], c2 = c[(it + 2) & 63], c3 = c[(it + 3) & 63];
#pragma unroll
    for (int k = 0; k < CH; k++) {
      unsigned __int128 a = (unsigned __int128)y[k] * c0 + (unsigned __int128)(y[k] ^ 1) * c1 +
                            (unsigned __int128)(y[k] ^ 2) * c2 + (unsigned __int128)(y[k] ^ 3) * c3;
      const uint64_t lo = (uint64_t)a, hi = (uint64_t)(a >> 64);
      uint64_t r = hi + __umul64hi(lo * qn, q) + (lo != 0);
      y[k] = r >= q ? r - q : r;
    }
  }
  for (int k = 0; k < CH; k++) io[t * CH + k] = y[k];
}

template <int MODE>
__global__ void k_f64(double *io, const double *c, double q, double qinv)
{
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  double y[CH];
  for (int k = 0; k < CH; k++) y[k] = io[t * CH + k];
  const double M = 0x1.8p52;
  for (int it = 0; it < IT; it++) {
    double cw[4], cq[4];
    for (int i = 0; i < 4; i++) { cw[i] = c[2 * ((it + i) & 63)]; cq[i] = c[2 * ((it + i) & 63) + 1]; }
#pragma unroll
    for (int k = 0; k < CH; k++) {
      double s = 0;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const double yy = y[k] + i;
        const double h = yy * cw[i], l = __fma_rn(yy, cw[i], -h);
        const double qt = MODE == 0 ? rint(yy * cq[i]) : __fma_rn(yy, cq[i], M) - M;
        s += __fma_rn(-qt, q, h) + l;
      }
      y[k] = MODE == 0 ? __fma_rn(-rint(s * qinv), q, s) : __fma_rn(-(__fma_rn(s, qinv, M) - M), q, s);
    }
  }
  for (int k = 0; k < CH; k++) io[t * CH + k] = y[k];
}

__global__ void k_rndne(double *io)
{
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  double y[CH];
  for (int k = 0; k < CH; k++) y[k] = io[t * CH + k];
  for (int it = 0; it < IT * 8; it++)
#pragma unroll
    for (int k = 0; k < CH; k++) y[k] = rint(y[k] * 1.0000001);
  for (int k = 0; k < CH; k++) io[t * CH + k] = y[k];
}

__global__ void k_mul(double *io)
{
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  double y[CH];
  for (int k = 0; k < CH; k++) y[k] = io[t * CH + k];
  for (int it = 0; it < IT * 8; it++)
#pragma unroll
    for (int k = 0; k < CH; k++) y[k] = y[k] * 1.0000001 * 0.9999999;
  for (int k = 0; k < CH; k++) io[t * CH + k] = y[k];
}

int main()
{
  const size_t threads = 256 * 1024 * 4;
  void *io, *c;
  hipMalloc(&io, threads * CH * 8);
  hipMalloc(&c, 128 * 8);
  hipMemset(io, 0, threads * CH * 8);
  hipMemset(c, 0, 128 * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto run = [&](const char *name, auto launch, double ops_per_thread, const char *unit) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-16s %.3e %s\n", name, ops_per_thread * threads * 5 / (ms * 1e-3), unit);
  };
  dim3 g(threads / 256), bl(256);
  const double q = 1125899906842597.0;
  run("fbc_u128", [&] { hipLaunchKernelGGL(k_u128, g, bl, 0, 0, (uint64_t *)io, (uint64_t *)c, 1125899906842597ull, 12345ull); }, 4.0 * IT * CH, "terms/s");
  run("fbc_f64_rint", [&] { hipLaunchKernelGGL(k_f64<0>, g, bl, 0, 0, (double *)io, (double *)c, q, 1 / q); }, 4.0 * IT * CH, "terms/s");
  run("fbc_f64_magic", [&] { hipLaunchKernelGGL(k_f64<1>, g, bl, 0, 0, (double *)io, (double *)c, q, 1 / q); }, 4.0 * IT * CH, "terms/s");
  run("v_rndne_f64+mul", [&] { hipLaunchKernelGGL(k_rndne, g, bl, 0, 0, (double *)io); }, 2.0 * IT * 8 * CH, "op/s");
  run("v_mul_f64", [&] { hipLaunchKernelGGL(k_mul, g, bl, 0, 0, (double *)io); }, 2.0 * IT * 8 * CH, "op/s");
  return 0;
}
