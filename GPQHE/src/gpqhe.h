/*
 * Forwarding header at the include path HECTR expects:
 *   reference src/hectr.h:35 and src/ctr.c:23 `#include "../GPQHE/src/gpqhe.h"`.
 * The ABI itself lives in include/gpqhe.h.
 */
#include "../../include/gpqhe.h"
