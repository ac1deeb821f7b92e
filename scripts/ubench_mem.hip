// Memory-pattern microbenchmark for the NTT tile passes (gfx950).
// hipcc --offload-arch=gfx950 -O3 scripts/ubench_mem.hip -o scripts/ubench_mem
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

__global__ void copy8(uint64_t *o, const uint64_t *x, size_t n)
{
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * 256)
    o[i] = x[i] + 1;
}
__global__ void copy16(ulonglong2 *o, const ulonglong2 *x, size_t n2)
{
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  for (; i < n2; i += (size_t)gridDim.x * 256) {
    ulonglong2 v = x[i];
    v.x++; v.y++;
    o[i] = v;
  }
}
// column pass pattern: limb of n = 2^16 as 256 rows x 256; tile = 256 rows x 16 cols
// thread (c = t % 16, l = t / 16) touches rows l + 16 k, k < 16
__global__ void cols8(uint64_t *o, const uint64_t *x)
{
  const unsigned tile = blockIdx.x % 16, limb = blockIdx.x / 16;
  const uint64_t *xs = x + ((size_t)limb << 16) + tile * 16;
  uint64_t *os = o + ((size_t)limb << 16) + tile * 16;
  const int c = threadIdx.x % 16, l = threadIdx.x / 16;
  uint64_t r[16];
#pragma unroll
  for (int k = 0; k < 16; k++)
    r[k] = xs[(size_t)(l + 16 * k) * 256 + c];
#pragma unroll
  for (int k = 0; k < 16; k++)
    os[(size_t)(l + 16 * k) * 256 + c] = r[k] + 1;
}
// 16 B per lane variant of the column pattern: tile = 256 rows x 32 cols, 512 threads
// thread (c2 = t % 16 -> cols 2 c2, 2 c2 + 1; l = t / 16 (0..31)), rows l + 32 k, k < 8
__global__ void cols16(ulonglong2 *o, const ulonglong2 *x)
{
  const unsigned tile = blockIdx.x % 8, limb = blockIdx.x / 8;
  const ulonglong2 *xs = x + ((size_t)limb << 15) + tile * 16;
  ulonglong2 *os = o + ((size_t)limb << 15) + tile * 16;
  const int c = threadIdx.x % 16, l = threadIdx.x / 16;
  ulonglong2 r[8];
#pragma unroll
  for (int k = 0; k < 8; k++)
    r[k] = xs[(size_t)(l + 32 * k) * 128 + c];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    r[k].x++; r[k].y++;
    os[(size_t)(l + 32 * k) * 128 + c] = r[k];
  }
}
// row pass pattern: tile = 16 rows x 256; thread (l = t % 16, rr = t / 16), elements rr*256 + l + 16 k
__global__ void rows8(uint64_t *o, const uint64_t *x)
{
  const size_t base = (size_t)blockIdx.x * 4096;
  const int l = threadIdx.x % 16, rr = threadIdx.x / 16;
  uint64_t r[16];
#pragma unroll
  for (int k = 0; k < 16; k++)
    r[k] = x[base + rr * 256 + l + 16 * k];
#pragma unroll
  for (int k = 0; k < 16; k++)
    o[base + rr * 256 + l + 16 * k] = r[k] + 1;
}
// contiguous-block pattern with 8 B lanes (store side of the row pass)
__global__ void tile8(uint64_t *o, const uint64_t *x)
{
  const size_t base = (size_t)blockIdx.x * 4096;
  uint64_t r[16];
#pragma unroll
  for (int i = 0; i < 16; i++)
    r[i] = x[base + threadIdx.x + 256 * i];
#pragma unroll
  for (int i = 0; i < 16; i++)
    o[base + threadIdx.x + 256 * i] = r[i] + 1;
}
// ks_rows2 / ntt3_rows input pattern at N2 = 256: 2048-element tile, thread
// (row = t / 32, l = t % 32) reads words (row << 8) + l + 32 k, k < 8 (8 B lanes,
// 256 contiguous bytes per half wave)
__global__ void rows8w(uint64_t *o, const uint64_t *x)
{
  const size_t base = (size_t)blockIdx.x * 2048;
  const int row = threadIdx.x / 32, l = threadIdx.x % 32;
  uint64_t r[8];
#pragma unroll
  for (int k = 0; k < 8; k++)
    r[k] = x[base + (row << 8) + l + 32 * k];
#pragma unroll
  for (int k = 0; k < 8; k++)
    o[base + (row << 8) + l + 32 * k] = r[k] + 1;
}
__global__ void tile16(ulonglong2 *o, const ulonglong2 *x)
{
  const size_t base = (size_t)blockIdx.x * 2048;
  ulonglong2 r[8];
#pragma unroll
  for (int i = 0; i < 8; i++)
    r[i] = x[base + threadIdx.x + 256 * i];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r[i].x++; r[i].y++;
    o[base + threadIdx.x + 256 * i] = r[i];
  }
}

// Every kernel reads the 1 GiB buffer x once and writes the 1 GiB buffer o
// once per launch, so a rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE pass over this
// binary calibrates the counters per access pattern (scripts/fetch_calib.py).
int main()
{
  const size_t limbs = 2048, n = limbs << 16;  // 1 GiB per buffer
  uint64_t *x, *o;
  CK(hipMalloc(&x, n * 8));
  CK(hipMalloc(&o, n * 8));
  CK(hipMemset(x, 1, n * 8));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto run = [&](const char *name, auto launch) {
    launch();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int r = 0; r < 10; r++)
      launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    printf("%-8s %7.1f GB/s\n", name, 2.0 * n * 8 * 10 / (ms * 1e6));
  };
  run("copy8", [&] { hipLaunchKernelGGL(copy8, dim3(8192), dim3(256), 0, 0, o, x, n); });
  run("copy16", [&] { hipLaunchKernelGGL(copy16, dim3(8192), dim3(256), 0, 0, (ulonglong2 *)o, (const ulonglong2 *)x, n / 2); });
  run("tile8", [&] { hipLaunchKernelGGL(tile8, dim3(n / 4096), dim3(256), 0, 0, o, x); });
  run("tile16", [&] { hipLaunchKernelGGL(tile16, dim3(n / 4096), dim3(256), 0, 0, (ulonglong2 *)o, (const ulonglong2 *)x); });
  run("rows8w", [&] { hipLaunchKernelGGL(rows8w, dim3(n / 2048), dim3(256), 0, 0, o, x); });
  run("rows8", [&] { hipLaunchKernelGGL(rows8, dim3(n / 4096), dim3(256), 0, 0, o, x); });
  run("cols8", [&] { hipLaunchKernelGGL(cols8, dim3(limbs * 16), dim3(256), 0, 0, o, x); });
  run("cols16", [&] { hipLaunchKernelGGL(cols16, dim3(limbs * 8), dim3(512), 0, 0, (ulonglong2 *)o, (const ulonglong2 *)x); });
  return 0;
}
