// Issue cost of the integer multiplies behind the 60-bit limbs (gfx950):
// v_mad_u64_u32 (32 x 32 + 64 -> 64), v_mul_lo_u32, v_mul_hi_u32, against
// v_fma_f64 and v_add_u32, 8 independent chains per lane.
// hipcc --offload-arch=gfx950 -O3 scripts/ubench_imad.hip -o scripts/ubench_imad
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define IT 4096

__global__ void k_mad64(uint64_t *o, uint32_t s)
{
  uint64_t a[8];
  uint32_t b = threadIdx.x * 2654435761u + s;
#pragma unroll
  for (int i = 0; i < 8; i++)
    a[i] = threadIdx.x + i;
  for (int it = 0; it < IT; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++)
      a[i] = (uint64_t)(uint32_t)a[i] * b + (a[i] >> 32);
  }
  uint64_t r = 0;
  for (int i = 0; i < 8; i++)
    r ^= a[i];
  o[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mullo(uint64_t *o, uint32_t s)
{
  uint32_t a[8];
  const uint32_t b = threadIdx.x * 2654435761u + s;
#pragma unroll
  for (int i = 0; i < 8; i++)
    a[i] = threadIdx.x + i;
  for (int it = 0; it < IT; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++)
      a[i] = a[i] * b;
  }
  uint64_t r = 0;
  for (int i = 0; i < 8; i++)
    r ^= a[i];
  o[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_mulhi(uint64_t *o, uint32_t s)
{
  uint32_t a[8];
  const uint32_t b = threadIdx.x * 2654435761u + s;
#pragma unroll
  for (int i = 0; i < 8; i++)
    a[i] = threadIdx.x + i + 0x80000000u;
  for (int it = 0; it < IT; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++)
      a[i] = __umulhi(a[i], b) | 0x80000000u;
  }
  uint64_t r = 0;
  for (int i = 0; i < 8; i++)
    r ^= a[i];
  o[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

__global__ void k_fma64(uint64_t *o, uint32_t s)
{
  double a[8];
  const double b = 1.0 + 1e-9 * (threadIdx.x + s);
#pragma unroll
  for (int i = 0; i < 8; i++)
    a[i] = threadIdx.x + i;
  for (int it = 0; it < IT; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++)
      a[i] = __fma_rn(a[i], b, 0.5);
  }
  double r = 0;
  for (int i = 0; i < 8; i++)
    r += a[i];
  o[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)r;
}

__global__ void k_add32(uint64_t *o, uint32_t s)
{
  uint32_t a[8];
  const uint32_t b = threadIdx.x * 2654435761u + s;
#pragma unroll
  for (int i = 0; i < 8; i++)
    a[i] = threadIdx.x + i;
  for (int it = 0; it < IT; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++)
      a[i] = (a[i] ^ b) + i;
  }
  uint64_t r = 0;
  for (int i = 0; i < 8; i++)
    r ^= a[i];
  o[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main()
{
  const int blocks = 256 * 8, threads = 256;
  uint64_t *o;
  (void)hipMalloc(&o, (size_t)blocks * threads * 8);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  struct K {
    const char *name;
    void (*f)(uint64_t *, uint32_t);
    int ops;  // counted instructions per inner step (the operation itself)
  } ks[] = {{"v_mad_u64_u32", k_mad64, 1}, {"v_mul_lo_u32", k_mullo, 1}, {"v_mul_hi_u32 (+or)", k_mulhi, 1},
            {"v_fma_f64", k_fma64, 1}, {"v_xor+v_add_u32", k_add32, 2}};
  for (auto &k : ks) {
    for (int rep = 0; rep < 2; rep++) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, o, 7u);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double waveinst = (double)blocks * threads / 64 * IT * 8 * k.ops;
      if (rep)
        printf("%-22s %.3f ms  %.1f G wave-instr/s  (%.2f cycles per wave-instr per SIMD at 2.4 GHz)\n", k.name, ms,
               waveinst / ms / 1e6, 1024 * 2.4e9 / (waveinst / ms * 1e3));
    }
  }
  return 0;
}
