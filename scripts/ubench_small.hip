// Small-N (n = 4096) latency microbenchmark: where the ~9 us of a
// single-workgroup limb transform goes (config 4's device chain).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I hectr_amd/csrc scripts/ubench_small.hip -o scripts/ubench_small
// For each kernel kind: the mean time per launch of 200 back-to-back launches
// (HIP events) and, from s_memrealtime stamps (100 MHz) taken by every block
// at entry and exit, the in-kernel span (first entry to last exit) and the
// gap from one launch's last exit to the next launch's first entry.
#include "ntt_device.h"

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <chrono>
#include <algorithm>

void gpqhe_die(const char *fmt, ...)
{
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
  fputc('\n', stderr);
  exit(1);
}

constexpr int LOGN = 12, N = 1 << LOGN;

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ void st_begin(uint64_t *st)
{
  if (threadIdx.x == 0)
    st[2 * blockIdx.x] = now();
}
__device__ __forceinline__ void st_end(uint64_t *st)
{
  __syncthreads();
  if (threadIdx.x == 0)
    st[2 * blockIdx.x + 1] = now();
}

__global__ void __launch_bounds__(512) k_empty(uint64_t *, Tw2, double, uint64_t, uint64_t *st)
{
  st_begin(st);
  st_end(st);
}

__global__ void __launch_bounds__(512) k_copy(uint64_t *x, Tw2, double, uint64_t, uint64_t *st)
{
  st_begin(st);
  uint64_t *p = x + (size_t)blockIdx.x * N;
  uint64_t v[8];
#pragma unroll
  for (int k = 0; k < 8; k++)
    v[k] = p[threadIdx.x + k * 512];
#pragma unroll
  for (int k = 0; k < 8; k++)
    p[threadIdx.x + k * 512] = v[k] ^ 1;
  st_end(st);
}

// one LDS round trip + barrier per "round", no arithmetic (4 rounds)
__global__ void __launch_bounds__(512) k_lds4(uint64_t *x, Tw2, double, uint64_t, uint64_t *st)
{
  __shared__ uint64_t lds[N];
  st_begin(st);
  uint64_t *p = x + (size_t)blockIdx.x * N;
  uint64_t v[8];
#pragma unroll
  for (int k = 0; k < 8; k++)
    v[k] = p[threadIdx.x + k * 512];
#pragma unroll
  for (int r = 0; r < 3; r++) {
    const int d8 = N >> (3 * r + 3), pos0 = (threadIdx.x / d8) * 8 * d8 + threadIdx.x % d8;
#pragma unroll
    for (int k = 0; k < 8; k++)
      lds[pos0 + k * d8] = v[k];
    __syncthreads();
    const int e8 = N >> (3 * r + 6), pos1 = (threadIdx.x / e8) * 8 * e8 + threadIdx.x % e8;
#pragma unroll
    for (int k = 0; k < 8; k++)
      v[k] = lds[pos1 + k * e8] + 1;
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < 8; k++)
    p[threadIdx.x + k * 512] = v[k];
  st_end(st);
}

template <bool F64, bool INV, int REPS>
__global__ void __launch_bounds__(512) k_ntt(uint64_t *x, Tw2 tw, double qd, uint64_t q, uint64_t *st)
{
  __shared__ __attribute__((aligned(16))) uint64_t lds[N];
  st_begin(st);
  uint64_t *p = x + (size_t)blockIdx.x * N;
  auto run = [&](const auto &ar) {
    using A = std::decay_t<decltype(ar)>;
    for (int rep = 0; rep < REPS; rep++) {
      if (rep)
        __syncthreads();
      if constexpr (INV)
        small_inv<LOGN>(
            ar, lds, [&](int, int i) { return A::load(p[i]); }, [&](int, int i, typename A::V a) { p[i] = ar.canon(a); });
      else
        small_fwd<LOGN>(
            ar, lds, [&](int, int i) { return A::load(p[i]); }, [&](int, int i, typename A::V a) { p[i] = ar.canon(a); });
    }
  };
  if constexpr (F64)
    run(ArF64{qd, 1.0 / qd, tw.fwdd, tw.invd, qd < (double)(1ull << 50)});
  else
    run(ArInt{q, tw.fwd, tw.inv});
  st_end(st);
}

// kernel arguments of the size the small-N kernels pass (CoefArg: 2.6 KB)
struct BigArg {
  int64_t v[320];
  unsigned clog, row;
};
__global__ void __launch_bounds__(512) k_bigarg_lane(uint64_t *x, BigArg a, uint64_t *st)
{
  st_begin(st);
  uint64_t *p = x + (size_t)blockIdx.x * N;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int i = threadIdx.x + k * 512;
    p[i] = (i & 127) ? 0 : (uint64_t)a.v[(blockIdx.x * a.row + (i >> 7)) % 320];
  }
  st_end(st);
}
__global__ void __launch_bounds__(512) k_bigarg_uni(uint64_t *x, BigArg a, uint64_t *st)
{
  st_begin(st);
  uint64_t *p = x + (size_t)blockIdx.x * N;
#pragma unroll
  for (int k = 0; k < 8; k++)
    p[threadIdx.x + k * 512] = (uint64_t)a.v[blockIdx.x] + a.row;
  st_end(st);
}
__global__ void __launch_bounds__(512) k_smallarg(uint64_t *x, const int64_t *v, unsigned row, uint64_t *st)
{
  st_begin(st);
  uint64_t *p = x + (size_t)blockIdx.x * N;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int i = threadIdx.x + k * 512;
    p[i] = (i & 127) ? 0 : (uint64_t)v[(blockIdx.x * row + (i >> 7)) % 320];
  }
  st_end(st);
}

typedef void (*Kern)(uint64_t *, Tw2, double, uint64_t, uint64_t *);

int main()
{
  const uint64_t qf = (1ull << 49) - 0x1ffff, qi = (1ull << 59) - 0x3ffff;  // sizes only (timing)
  const int MAXB = 64, LAUNCH = 200, SEQ = 24;
  std::vector<uint64_t> h((size_t)MAXB * N), t2(2 * N), ti2(2 * N);
  std::vector<double> td(2 * N);
  srand(1);
  for (size_t i = 0; i < h.size(); i++)
    h[i] = (((uint64_t)rand() << 31) ^ rand()) % qf;
  for (int i = 0; i < N; i++) {
    const uint64_t w = (((uint64_t)rand() << 40) ^ ((uint64_t)rand() << 20) ^ rand()) % qi;
    t2[2 * i] = w;
    t2[2 * i + 1] = (uint64_t)(((unsigned __int128)w << 64) / qi);
    const double wd = (double)((((uint64_t)rand() << 31) ^ rand()) % qf);
    td[2 * i] = wd;
    td[2 * i + 1] = wd / (double)qf;
  }
  uint64_t *x, *tw, *st;
  double *twd;
  HIP_CHECK(hipMalloc(&x, h.size() * 8));
  HIP_CHECK(hipMalloc(&tw, t2.size() * 8));
  HIP_CHECK(hipMalloc(&twd, td.size() * 8));
  HIP_CHECK(hipMalloc(&st, (size_t)SEQ * MAXB * 2 * 8));
  HIP_CHECK(hipMemcpy(x, h.data(), h.size() * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(tw, t2.data(), t2.size() * 8, hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy(twd, td.data(), td.size() * 8, hipMemcpyHostToDevice));
  const Tw2 T{tw, tw, twd, twd};
  struct Case {
    const char *name;
    Kern k;
  } cases[] = {
      {"empty", k_empty},
      {"copy 8 words/thread", k_copy},
      {"4 LDS rounds, no arithmetic", k_lds4},
      {"fwd FP64 (q < 2^50)", k_ntt<true, false, 1>},
      {"inv FP64 (q < 2^50)", k_ntt<true, true, 1>},
      {"fwd int64 (59-bit)", k_ntt<false, false, 1>},
      {"inv int64 (59-bit)", k_ntt<false, true, 1>},
      {"fwd FP64 x4 in one launch", k_ntt<true, false, 4>},
      {"fwd int64 x4 in one launch", k_ntt<false, false, 4>},
  };
  hipEvent_t e0, e1;
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));
  for (int blocks : {1, 10, 64}) {
    printf("== %d blocks of 512 threads\n", blocks);
    printf("%-30s %10s %10s %10s %10s\n", "kernel", "us/launch", "span us", "gap us", "entry skew");
    for (auto &c : cases) {
      for (int i = 0; i < 20; i++)
        hipLaunchKernelGGL(c.k, dim3(blocks), dim3(512), 0, 0, x, T, (double)qf, qi, st);
      HIP_CHECK(hipEventRecord(e0, 0));
      for (int i = 0; i < LAUNCH; i++)
        hipLaunchKernelGGL(c.k, dim3(blocks), dim3(512), 0, 0, x, T, (double)qf, qi, st);
      HIP_CHECK(hipEventRecord(e1, 0));
      HIP_CHECK(hipEventSynchronize(e1));
      float ms;
      HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
      for (int i = 0; i < SEQ; i++)
        hipLaunchKernelGGL(c.k, dim3(blocks), dim3(512), 0, 0, x, T, (double)qf, qi, st + (size_t)i * MAXB * 2);
      HIP_CHECK(hipDeviceSynchronize());
      std::vector<uint64_t> s((size_t)SEQ * MAXB * 2);
      HIP_CHECK(hipMemcpy(s.data(), st, s.size() * 8, hipMemcpyDeviceToHost));
      double span = 0, gap = 0, skew = 0;
      int ng = 0;
      uint64_t prev_end = 0;
      for (int i = 4; i < SEQ; i++) {
        uint64_t b0 = ~0ull, b1 = 0, e = 0;
        for (int b = 0; b < blocks; b++) {
          const uint64_t *v = &s[((size_t)i * MAXB + b) * 2];
          b0 = v[0] < b0 ? v[0] : b0;
          b1 = v[0] > b1 ? v[0] : b1;
          e = v[1] > e ? v[1] : e;
        }
        span += (e - b0) * 0.01;
        skew += (b1 - b0) * 0.01;
        if (prev_end) {
          gap += ((double)b0 - (double)prev_end) * 0.01;
          ng++;
        }
        prev_end = e;
      }
      printf("%-30s %10.2f %10.2f %10.2f %10.2f\n", c.name, 1000.0 * ms / LAUNCH, span / (SEQ - 4), gap / ng,
             skew / (SEQ - 4));
    }
  }
  {
    // kernel-argument size: a 2.6 KB argument read per lane / uniformly, and
    // the same values through a pointer
    BigArg ba{};
    for (int i = 0; i < 320; i++)
      ba.v[i] = i;
    ba.row = 32;
    int64_t *dv;
    HIP_CHECK(hipMalloc(&dv, 320 * 8));
    HIP_CHECK(hipMemcpy(dv, ba.v, 320 * 8, hipMemcpyHostToDevice));
    printf("== kernel arguments, 10 blocks\n%-30s %10s %10s %10s\n", "kernel", "us/launch", "span us", "gap us");
    for (int kind = 0; kind < 3; kind++) {
      auto launch = [&](uint64_t *s_) {
        if (kind == 0)
          hipLaunchKernelGGL(k_bigarg_lane, dim3(10), dim3(512), 0, 0, x, ba, s_);
        else if (kind == 1)
          hipLaunchKernelGGL(k_bigarg_uni, dim3(10), dim3(512), 0, 0, x, ba, s_);
        else
          hipLaunchKernelGGL(k_smallarg, dim3(10), dim3(512), 0, 0, x, (const int64_t *)dv, 32u, s_);
      };
      for (int i = 0; i < 20; i++)
        launch(st);
      HIP_CHECK(hipEventRecord(e0, 0));
      for (int i = 0; i < LAUNCH; i++)
        launch(st);
      HIP_CHECK(hipEventRecord(e1, 0));
      HIP_CHECK(hipEventSynchronize(e1));
      float ms;
      HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
      for (int i = 0; i < SEQ; i++)
        launch(st + (size_t)i * MAXB * 2);
      HIP_CHECK(hipDeviceSynchronize());
      std::vector<uint64_t> s((size_t)SEQ * MAXB * 2);
      HIP_CHECK(hipMemcpy(s.data(), st, s.size() * 8, hipMemcpyDeviceToHost));
      double span = 0, gap = 0;
      uint64_t prev_end = 0;
      for (int i = 4; i < SEQ; i++) {
        uint64_t b0 = ~0ull, e = 0;
        for (int b = 0; b < 10; b++) {
          b0 = std::min(b0, s[((size_t)i * MAXB + b) * 2]);
          e = std::max(e, s[((size_t)i * MAXB + b) * 2 + 1]);
        }
        span += (e - b0) * 0.01;
        if (prev_end)
          gap += ((double)b0 - (double)prev_end) * 0.01;
        prev_end = e;
      }
      const char *nm[3] = {"2.6 KB arg, per-lane index", "2.6 KB arg, uniform index", "pointer arg"};
      printf("%-30s %10.2f %10.2f %10.2f\n", nm[kind], 1000.0 * ms / LAUNCH, span / (SEQ - 4), gap / (SEQ - 5));
    }
  }
  // the same kernels after the device has idled (host spin between launches,
  // as the control loop's host work between steps)
  for (int idle_us : {20, 50, 200}) {
    printf("== 10 blocks, launched after %d us of device idle\n", idle_us);
    printf("%-30s %10s %10s\n", "kernel", "event us", "span us");
    for (auto &c : cases) {
      double ev = 0, span = 0;
      const int R = 20;
      for (int r = 0; r < R; r++) {
        HIP_CHECK(hipDeviceSynchronize());
        const auto t0 = std::chrono::steady_clock::now();
        while (std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() < idle_us) {
        }
        HIP_CHECK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(c.k, dim3(10), dim3(512), 0, 0, x, T, (double)qf, qi, st);
        HIP_CHECK(hipEventRecord(e1, 0));
        HIP_CHECK(hipEventSynchronize(e1));
        float ms;
        HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
        std::vector<uint64_t> s(2 * 10);
        HIP_CHECK(hipMemcpy(s.data(), st, s.size() * 8, hipMemcpyDeviceToHost));
        uint64_t b0 = ~0ull, e = 0;
        for (int b = 0; b < 10; b++) {
          b0 = s[2 * b] < b0 ? s[2 * b] : b0;
          e = s[2 * b + 1] > e ? s[2 * b + 1] : e;
        }
        if (r >= 4) {
          ev += 1000.0 * ms;
          span += (e - b0) * 0.01;
        }
      }
      printf("%-30s %10.2f %10.2f\n", c.name, ev / (R - 4), span / (R - 4));
    }
  }
  return 0;
}
