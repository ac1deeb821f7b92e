/*
 * Drop-in location when this repository is checked out as HECTR's GPQHE
 * submodule: HECTR includes "../GPQHE/src/gpqhe.h" (reference src/hectr.h:35,
 * src/ctr.c:23).  The ABI lives in include/gpqhe.h.
 */
#include "../include/gpqhe.h"
