/*
 * Minimal libpmu-compatible timing macros so the unchanged HECTR harness
 * compiles (reference src/ctr.c:22, tests/hectr.c:24 include "pmu.h";
 * usage: TEST_BEGIN(); TEST_DO("label"); ... TEST_DONE(); TEST_END();
 * e.g. src/ctr.c:528-533,570,597).  libpmu is an empty submodule in the
 * reference (.gitmodules:4-6); these macros only time wall-clock.
 */
#ifndef PMU_H
#define PMU_H
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

static inline double pmu_now_(void)
{
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

#define TEST_BEGIN() double pmu_t0_ = pmu_now_(); (void)pmu_t0_
#define TEST_DO(label) do { const char *pmu_label_ = (label); double pmu_t_ = pmu_now_();
#define TEST_DONE() fprintf(stderr, "[pmu] %-40s %10.3f ms\n", pmu_label_, 1e3 * (pmu_now_() - pmu_t_)); } while (0)
#define TEST_END() ((void)0)

#endif /* PMU_H */
