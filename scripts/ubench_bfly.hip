// Butterfly microbenchmark: int64 lazy-Shoup CT butterflies vs exact FP64
// butterflies (q < 2^50), with an exactness check of the FP64 path.
// hipcc --offload-arch=gfx950 -O3 scripts/ubench_bfly.hip -o scripts/ubench_bfly
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned __int128 u128;
#define ITERS 64

__device__ __forceinline__ uint64_t mulhi64(uint64_t a, uint64_t b) { return __umul64hi(a, b); }

// 16-element register block, 4 CT stages (the NTT's round B), ITERS times
__global__ void bfly_int(uint64_t *io, const uint64_t *tw, uint64_t q)
{
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t x[16];
  for (int k = 0; k < 16; k++) x[k] = io[t * 16 + k];
  const uint64_t q2 = 2 * q;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int s = 0; s < 4; s++) {
      const int half = 8 >> s;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        if (k & half) continue;
        const int ti = (it * 15 + s * 4 + (k >> (4 - s))) & 63;
        const uint64_t w = tw[2 * ti], wp = tw[2 * ti + 1];
        uint64_t U = x[k] >= q2 ? x[k] - q2 : x[k];
        const uint64_t V = x[k + half] * w - mulhi64(x[k + half], wp) * q;
        x[k] = U + V;
        x[k + half] = U - V + q2;
      }
    }
  }
  for (int k = 0; k < 16; k++) {
    uint64_t v = x[k] % q;
    io[t * 16 + k] = v;
  }
}

__device__ __forceinline__ double mulmod_f64(double y, double w, double wq, double q)
{
  const double h = y * w;
  const double l = __fma_rn(y, w, -h);
  const double qt = rint(y * wq);
  const double r = __fma_rn(-qt, q, h);
  return r + l;
}
__device__ __forceinline__ double red_f64(double x, double q, double qinv)
{
  return __fma_rn(-rint(x * qinv), q, x);
}

__global__ void bfly_f64(uint64_t *io, const double *twd, double q, double qinv, uint64_t qi)
{
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  double x[16];
  for (int k = 0; k < 16; k++) x[k] = (double)io[t * 16 + k];
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int s = 0; s < 4; s++) {
      const int half = 8 >> s;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        if (k & half) continue;
        const int ti = (it * 15 + s * 4 + (k >> (4 - s))) & 63;
        const double w = twd[2 * ti], wq = twd[2 * ti + 1];
        const double X = red_f64(x[k], q, qinv);
        const double T = mulmod_f64(x[k + half], w, wq, q);
        x[k] = X + T;
        x[k + half] = X - T;
      }
    }
  }
  for (int k = 0; k < 16; k++) {
    double v = red_f64(x[k], q, qinv);
    v = v < 0 ? v + q : v;
    v = v >= q ? v - q : v;
    io[t * 16 + k] = (uint64_t)v;
  }
}

int main()
{
  const uint64_t qs[] = {1125899906826241ull, 1125899906629633ull, 562949953421231ull,    // < 2^50
                         2251799813554177ull, 2251799813685119ull, 2251799813160961ull};  // < 2^51 (odd, not nec. prime)
  const size_t nth = 256 * 4096, words = nth * 16;
  uint64_t *h = (uint64_t *)malloc(words * 8), *hi = (uint64_t *)malloc(words * 8), *hf = (uint64_t *)malloc(words * 8);
  uint64_t *d;
  uint64_t *dtw;
  double *dtd;
  hipMalloc(&d, words * 8);
  hipMalloc(&dtw, 128 * 8);
  hipMalloc(&dtd, 128 * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (uint64_t q : qs) {
    uint64_t tw[128];
    double td[128];
    uint64_t st = q * 2654435761ull;
    for (int i = 0; i < 64; i++) {
      st = st * 6364136223846793005ull + 1442695040888963407ull;
      const uint64_t w = (st >> 11) % q;
      tw[2 * i] = w;
      tw[2 * i + 1] = (uint64_t)(((u128)w << 64) / q);
      td[2 * i] = (double)w;
      td[2 * i + 1] = (double)w / (double)q;
    }
    for (size_t i = 0; i < words; i++) {
      st = st * 6364136223846793005ull + 1442695040888963407ull;
      h[i] = (st >> 7) % q;
    }
    hipMemcpy(dtw, tw, sizeof(tw), hipMemcpyHostToDevice);
    hipMemcpy(dtd, td, sizeof(td), hipMemcpyHostToDevice);
    float ms_i, ms_f;
    hipMemcpy(d, h, words * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(bfly_int, dim3(nth / 256), dim3(256), 0, 0, d, dtw, q);
    hipMemcpy(d, h, words * 8, hipMemcpyHostToDevice);
    hipEventRecord(a);
    hipLaunchKernelGGL(bfly_int, dim3(nth / 256), dim3(256), 0, 0, d, dtw, q);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms_i, a, b);
    hipMemcpy(hi, d, words * 8, hipMemcpyDeviceToHost);
    hipMemcpy(d, h, words * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(bfly_f64, dim3(nth / 256), dim3(256), 0, 0, d, dtd, (double)q, 1.0 / (double)q, q);
    hipMemcpy(d, h, words * 8, hipMemcpyHostToDevice);
    hipEventRecord(a);
    hipLaunchKernelGGL(bfly_f64, dim3(nth / 256), dim3(256), 0, 0, d, dtd, (double)q, 1.0 / (double)q, q);
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ms_f, a, b);
    hipMemcpy(hf, d, words * 8, hipMemcpyDeviceToHost);
    size_t bad = 0;
    for (size_t i = 0; i < words; i++)
      bad += hi[i] != hf[i];
    const double bfl = (double)nth * ITERS * 32;
    printf("q=%llu int %.3f ms (%.2e bfly/s)  f64 %.3f ms (%.2e bfly/s)  mismatches %zu / %zu\n",
           (unsigned long long)q, ms_i, bfl / ms_i * 1e3, ms_f, bfl / ms_f * 1e3, bad, words);
  }
  return 0;
}
