// HBM read bandwidth by per-lane access shape (gfx950): does a thread that
// reads its own 64 contiguous bytes as four 16-byte loads (the split key
// switch's input pattern, lanes 64 B apart) stream as fast as 16-byte loads
// with consecutive lanes 16 B apart?
// hipcc --offload-arch=gfx950 -O3 scripts/ubench_lanes.hip -o scripts/ubench_lanes
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

// each 256-thread block reads one 16 KiB chunk per iteration (4 loads per lane)
template <int MODE>
__global__ void __launch_bounds__(256) rd(const ulonglong2 *__restrict__ in, size_t chunks, uint64_t *out)
{
  uint64_t acc = 0;
  const unsigned t = threadIdx.x;
  for (size_t c = blockIdx.x; c < chunks; c += gridDim.x) {
    const ulonglong2 *b = in + c * 1024;  // 16 KiB = 1024 x 16 B
    ulonglong2 v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (MODE == 0)
        v[j] = b[256 * j + t];  // consecutive lanes 16 B apart
      else if (MODE == 1)
        v[j] = b[4 * t + j];  // a lane's own 64 B, lanes 64 B apart
      else
        v[j] = b[(t & ~63) * 4 + 64 * j + (t & 63)];  // a wave's 4 KiB, lanes 16 B apart
    }
#pragma unroll
    for (int j = 0; j < 4; j++)
      acc += v[j].x ^ v[j].y;
  }
  if (acc == 0x12345)
    out[0] = acc;
}

// copy with the same shape on both sides (read one chunk, write it elsewhere)
template <int MODE>
__global__ void __launch_bounds__(256) cp(const ulonglong2 *__restrict__ in, ulonglong2 *__restrict__ o, size_t chunks)
{
  const unsigned t = threadIdx.x;
  for (size_t c = blockIdx.x; c < chunks; c += gridDim.x) {
    const ulonglong2 *b = in + c * 1024;
    ulonglong2 *d = o + c * 1024;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const size_t i = MODE == 0 ? 256 * j + t : MODE == 1 ? 4 * t + j : (t & ~63) * 4 + 64 * j + (t & 63);
      d[i] = b[i];
    }
  }
}

// keep-like mix: four input streams read per chunk (read shape R), one
// output stream written coalesced (lanes 16 B apart)
template <int R>
__global__ void __launch_bounds__(256) mix(const ulonglong2 *__restrict__ in, ulonglong2 *__restrict__ o, size_t chunks)
{
  const unsigned t = threadIdx.x;
  for (size_t c = blockIdx.x; c < chunks; c += gridDim.x) {
    ulonglong2 acc[4];
#pragma unroll
    for (int j = 0; j < 4; j++)
      acc[j] = make_ulonglong2(0, 0);
#pragma unroll
    for (int s = 0; s < 4; s++) {
      const ulonglong2 *b = in + ((size_t)s * chunks + c) * 1024;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const size_t i = R == 0 ? 256 * j + t : 4 * t + j;
        const ulonglong2 v = b[i];
        acc[j].x ^= v.x;
        acc[j].y += v.y;
      }
    }
    ulonglong2 *d = o + c * 1024;
#pragma unroll
    for (int j = 0; j < 4; j++)
      d[256 * j + t] = acc[j];
  }
}

int main()
{
  const size_t bytes = (size_t)2 << 30, chunks = bytes / 16384;
  ulonglong2 *a, *b;
  uint64_t *o;
  hipMalloc(&a, bytes);
  hipMalloc(&b, bytes);
  hipMalloc(&o, 64);
  hipMemset(a, 1, bytes);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char *names[3] = {"lanes 16 B apart (block)", "lane-own 64 B (4 x 16 B)", "lanes 16 B apart (wave 4 KiB)"};
  for (int grid : {2048, 8192}) {
    for (int m = 0; m < 3; m++) {
      for (int rep = 0; rep < 2; rep++) {
        hipEventRecord(e0);
        for (int i = 0; i < 5; i++) {
          if (m == 0) hipLaunchKernelGGL(rd<0>, dim3(grid), dim3(256), 0, 0, a, chunks, o);
          if (m == 1) hipLaunchKernelGGL(rd<1>, dim3(grid), dim3(256), 0, 0, a, chunks, o);
          if (m == 2) hipLaunchKernelGGL(rd<2>, dim3(grid), dim3(256), 0, 0, a, chunks, o);
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        float ms2;
        hipEventRecord(e0);
        for (int i = 0; i < 5; i++) {
          if (m == 0) hipLaunchKernelGGL(cp<0>, dim3(grid), dim3(256), 0, 0, a, b, chunks / 2);
          if (m == 1) hipLaunchKernelGGL(cp<1>, dim3(grid), dim3(256), 0, 0, a, b, chunks / 2);
          if (m == 2) hipLaunchKernelGGL(cp<2>, dim3(grid), dim3(256), 0, 0, a, b, chunks / 2);
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms2, e0, e1);
        if (rep)
          printf("grid %5d  %-32s read %.2f TB/s   copy %.2f TB/s (read + write)\n", grid, names[m],
                 5.0 * bytes / ms / 1e9, 5.0 * bytes / ms2 / 1e9);
      }
    }
  }
  // the mix: 4 reads + 1 write per 16 KiB chunk
  {
    const size_t mchunks = bytes / 16384 / 4;  // 4 input streams of mchunks chunks in a
    for (int r = 0; r < 2; r++) {
      for (int rep = 0; rep < 2; rep++) {
        hipEventRecord(e0);
        for (int i = 0; i < 5; i++) {
          if (r == 0) hipLaunchKernelGGL(mix<0>, dim3(8192), dim3(256), 0, 0, a, b, mchunks);
          else hipLaunchKernelGGL(mix<1>, dim3(8192), dim3(256), 0, 0, a, b, mchunks);
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (rep)
          printf("mix 4 reads (%s) + 1 coalesced write: %.2f TB/s\n", r ? "lane-own 64 B" : "lanes 16 B apart",
                 5.0 * (5.0 / 4.0) * bytes / ms / 1e9);
      }
    }
  }
  return 0;
}
