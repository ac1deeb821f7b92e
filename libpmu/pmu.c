/* libpmu.so for HECTR's `-lpmu` link (reference tests/Makefile:25); the
 * timing macros are header-only (pmu.h), so the library carries no code. */
#include "pmu.h"
int pmu_version(void) { return 1; }
