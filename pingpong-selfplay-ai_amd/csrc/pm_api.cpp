// libpongmi host utilities: error reporting, ABI introspection, launch timing.
#include <stdarg.h>
#include <stdio.h>

#include "pm_host.h"

namespace {
thread_local char g_err[512] = "";
}

int pm_fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

extern "C" const char* pm_last_error(void) { return g_err; }

// ---------------------------------------------------------------- launch timing
namespace {
struct LaunchTimer {
    hipEvent_t ev[2] = {nullptr, nullptr};
    int device = -1;
    bool armed = false, pending = false;
};
LaunchTimer g_timer[PM_TIMER_N];
}  // namespace

bool pm_timer_take(int kernel, hipEvent_t* start, hipEvent_t* stop) {
    LaunchTimer& t = g_timer[kernel];
    if (!t.armed) return false;
    t.armed = false;
    t.pending = true;
    *start = t.ev[0];
    *stop = t.ev[1];
    return true;
}

extern "C" int pm_timer_arm(int32_t kernel) {
    PM_REQUIRE(kernel >= 0 && kernel < PM_TIMER_N, PM_E_ARG, "pm_timer_arm: no kernel %d", kernel);
    LaunchTimer& t = g_timer[kernel];
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return pm_fail((int)e, "pm_timer_arm: %s", hipGetErrorString(e));
    if (t.device != dev) {
        for (hipEvent_t& ev : t.ev) {
            if (ev) (void)hipEventDestroy(ev);
            ev = nullptr;
        }
        for (hipEvent_t& ev : t.ev)
            if ((e = hipEventCreate(&ev)) != hipSuccess)
                return pm_fail((int)e, "pm_timer_arm: hipEventCreate: %s", hipGetErrorString(e));
        t.device = dev;
    }
    t.armed = true;
    t.pending = false;
    return 0;
}

extern "C" int pm_timer_read(int32_t kernel, float* ms) {
    PM_REQUIRE(kernel >= 0 && kernel < PM_TIMER_N && ms, PM_E_ARG, "pm_timer_read: kernel %d", kernel);
    LaunchTimer& t = g_timer[kernel];
    PM_REQUIRE(t.pending, PM_E_ARG, "pm_timer_read: kernel %d was not launched since pm_timer_arm", kernel);
    hipError_t e = hipEventSynchronize(t.ev[1]);
    if (e == hipSuccess) e = hipEventElapsedTime(ms, t.ev[0], t.ev[1]);
    if (e != hipSuccess) return pm_fail((int)e, "pm_timer_read: %s", hipGetErrorString(e));
    t.pending = false;
    return 0;
}

extern "C" int pm_abi_version(void) { return PM_ABI_VERSION; }

extern "C" int32_t pm_sizeof(int32_t which) {
    switch (which) {
        case 0: return (int32_t)sizeof(pm_env_params);
        case 1: return (int32_t)sizeof(pm_env_state);
        case 2: return (int32_t)sizeof(pm_ctrl);
        case 3: return (int32_t)sizeof(pm_selfplay);
        case 4: return (int32_t)sizeof(pm_drqn);
        case 5: return (int32_t)sizeof(pm_drqn_stats);
        case 6: return (int32_t)sizeof(pm_rnn_ctrl);
        case 7: return (int32_t)sizeof(pm_rnn_selfplay);
        default: return -1;
    }
}

