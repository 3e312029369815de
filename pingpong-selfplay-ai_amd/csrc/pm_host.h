// Host-side helpers shared by the libpongmi translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pongmi.h"

int pm_fail(int code, const char* fmt, ...);

#define PM_REQUIRE(cond, code, ...)                        \
    do {                                                   \
        if (!(cond)) return pm_fail((code), __VA_ARGS__);  \
    } while (0)

#define PM_LAUNCHED(name)                                                                  \
    do {                                                                                   \
        hipError_t e_ = hipGetLastError();                                                 \
        if (e_ != hipSuccess) return pm_fail((int)e_, "%s: %s", name, hipGetErrorString(e_)); \
    } while (0)

static inline hipStream_t pm_stream(void* s) { return (hipStream_t)s; }
static inline unsigned pm_blocks(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

// ---------------------------------------------------------------- diagnostic stamps (PM_DIAG builds only)
// libpongmi_diag.so is built with -DPM_DIAG: thread 0 of block 0 records s_memrealtime (100 MHz)
// at named phase boundaries into pm_diag_buf; pm_diag_read copies them out. The product library
// compiles every stamp to nothing.
