// Cross-stream dependency cost on MI355X (HIP events): the device time a
// hipStreamWaitEvent adds to a chain of small kernels when the event it
// waits on has long completed, and when it completes during the wait.
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_streams.hip -o scripts/ubench_streams
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <chrono>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__global__ void k_small(uint64_t *x, int iters)
{
  uint64_t v = x[threadIdx.x];
  for (int i = 0; i < iters; i++)
    v = v * 6364136223846793005ull + 1442695040888963407ull;
  x[threadIdx.x] = v;
}

int main(int argc, char **argv)
{
  uint64_t *a, *b;
  CK(hipMalloc(&a, 4096 * 8));
  CK(hipMalloc(&b, 4096 * 8));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t ev, t0, t1;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  const int N = 200, IT = argc > 1 ? atoi(argv[1]) : 2000;
  for (int mode = 0; mode < 4; mode++) {
    // mode 0: 10-kernel chain on s0 only
    // mode 1: + record on s1 (after one kernel there, long done) and wait on s0 mid-chain
    // mode 2: + a long kernel on s1 the chain waits for mid-chain
    // mode 3: record + wait on the same stream (s0) mid-chain
    float tot = 0;
    double host = 0;
    for (int r = 0; r < N; r++) {
      CK(hipDeviceSynchronize());
      if (mode == 1) {
        hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s1, b, 10);
        CK(hipEventRecord(ev, s1));
        CK(hipStreamSynchronize(s1));
      }
      auto h0 = std::chrono::steady_clock::now();
      CK(hipEventRecord(t0, s0));
      for (int k = 0; k < 10; k++) {
        if (k == 5 && mode == 2) {
          hipLaunchKernelGGL(k_small, dim3(1), dim3(64), 0, s1, b, IT);
          CK(hipEventRecord(ev, s1));
        }
        if (k == 5 && mode == 3)
          CK(hipEventRecord(ev, s0));
        if (k == 5 && mode >= 1)
          CK(hipStreamWaitEvent(s0, ev, 0));
        hipLaunchKernelGGL(k_small, dim3(8), dim3(64), 0, s0, a, IT);
      }
      CK(hipEventRecord(t1, s0));
      host += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count();
      CK(hipEventSynchronize(t1));
      float ms;
      CK(hipEventElapsedTime(&ms, t0, t1));
      if (r >= 10)
        tot += ms;
    }
    const char *nm[4] = {"chain of 10 on one stream", "+ wait on an event long done (other stream)",
                         "+ wait on a kernel of the other stream", "+ record and wait on the same stream"};
    printf("%-46s device %8.2f us  host %8.2f us per chain\n", nm[mode], 1000.0 * tot / (N - 10), host / N);
  }
  return 0;
}
