// Microbenchmark: issue rate of the 64-bit modular-multiply building blocks
// on gfx950 (v_mad_u64_u32 chains, Shoup, Barrett, Montgomery, FP64 FMA).
// Each thread runs IND independent chains of ITERS ops; prints ops/s/chip.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include "../hectr_amd/csrc/gpqhe_internal.h"

#define ITERS 4096
#define IND 8

template <int KIND>
__global__ void bench(uint64_t *out, uint64_t q, uint64_t w, uint64_t wp, ModConst mc, uint64_t qinv)
{
  uint64_t x[IND];
  for (int i = 0; i < IND; i++)
    x[i] = (threadIdx.x * 2654435761u + i * 977u + blockIdx.x) % q;
  double d[IND];
  for (int i = 0; i < IND; i++)
    d[i] = (double)x[i];
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < IND; i++) {
      if (KIND == 0)  // Shoup
        x[i] = mul_shoup(x[i], w, wp, q);
      else if (KIND == 1)  // Barrett var x var
        x[i] = mul_mod(x[i], x[(i + 1) % IND] | 1, mc);
      else if (KIND == 2) {  // Montgomery REDC of x * w
        const uint64_t lo = x[i] * w, hi = __umul64hi(x[i], w);
        const uint64_t m = lo * qinv;
        const uint64_t t = hi - __umul64hi(m, q);
        x[i] = (int64_t)t < 0 ? t + q : t;
      } else if (KIND == 3) {  // 32x32 -> 64 mad chain
        x[i] = (uint64_t)(uint32_t)x[i] * (uint32_t)w + x[i];  // v_mad_u64_u32
      } else if (KIND == 4) {  // fp64 fma
        d[i] = fma(d[i], 1.0000001, -0.5);
      } else if (KIND == 5) {  // lazy Shoup (no correction)
        x[i] = mul_shoup_lazy(x[i], w, wp, q);
      }
    }
  }
  uint64_t acc = 0;
  for (int i = 0; i < IND; i++)
    acc ^= x[i] ^ (uint64_t)d[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int KIND>
double run(uint64_t *out, uint64_t q, uint64_t w, uint64_t wp, ModConst mc, uint64_t qinv)
{
  const int blocks = 256 * 8, threads = 256;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(bench<KIND>, dim3(blocks), dim3(threads), 0, 0, out, q, w, wp, mc, qinv);
  hipEventRecord(a);
  for (int r = 0; r < 3; r++)
    hipLaunchKernelGGL(bench<KIND>, dim3(blocks), dim3(threads), 0, 0, out, q, w, wp, mc, qinv);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double ops = 3.0 * blocks * threads * (double)ITERS * IND;
  return ops / (ms * 1e-3);
}

void gpqhe_die(const char *fmt, ...) { abort(); }

int main()
{
  const uint64_t q = 0x0ffffffffffc0001ull;  // 60-bit-ish (not necessarily prime: rate test)
  ModConst mc;
  memset(&mc, 0, sizeof(mc));
  mc.q = q;
  mc.k = 64 - __builtin_clzll(q);
  mc.mu = (uint64_t)(((unsigned __int128)1 << (2 * mc.k)) / q);
  const uint64_t w = 0x0123456789abcdull % q;
  const uint64_t wp = (uint64_t)(((unsigned __int128)w << 64) / q);
  uint64_t qinv = 1;  // -q^-1 mod 2^64 via Newton
  for (int i = 0; i < 6; i++)
    qinv *= 2 - q * qinv;
  qinv = -qinv;
  uint64_t *out;
  hipMalloc(&out, 256 * 8 * 256 * 8);
  printf("shoup      %.3e modmul/s\n", run<0>(out, q, w, wp, mc, qinv));
  printf("shoup_lazy %.3e modmul/s\n", run<5>(out, q, w, wp, mc, qinv));
  printf("barrett    %.3e modmul/s\n", run<1>(out, q, w, wp, mc, qinv));
  printf("montgomery %.3e modmul/s\n", run<2>(out, q, w, wp, mc, qinv));
  printf("mad_u64    %.3e op/s\n", run<3>(out, q, w, wp, mc, qinv));
  printf("fp64 fma   %.3e op/s\n", run<4>(out, q, w, wp, mc, qinv));
  return 0;
}
