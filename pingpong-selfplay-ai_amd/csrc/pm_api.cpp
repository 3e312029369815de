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
// Per kernel, a FIFO of kTimerSlots begin/end event pairs: pm_timer_arm queues one more launch to
// time, the launch takes the next slot, pm_timer_read returns the oldest timed launch's duration.
namespace {
constexpr int kTimerSlots = 64;
struct LaunchTimer {
    hipEvent_t ev[kTimerSlots][2] = {};
    int device = -1;
    int armed = 0, pending = 0, head = 0;  // head: the oldest pending slot
};
LaunchTimer g_timer[PM_TIMER_N];
}  // namespace

// The next armed slot of `kernel` for a launch on the current device. A launch on another device than
// the one the timer was armed on stays untimed (its events belong to that device), and the slot
// stays armed for the next launch there.
bool pm_timer_take(int kernel, hipEvent_t* start, hipEvent_t* stop) {
    LaunchTimer& t = g_timer[kernel];
    if (t.armed == 0) return false;
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev != t.device) return false;
    const int slot = (t.head + t.pending) % kTimerSlots;
    --t.armed;
    ++t.pending;
    *start = t.ev[slot][0];
    *stop = t.ev[slot][1];
    return true;
}

// A timed launch that failed to enqueue: its slot goes back to armed (its events were never
// recorded, so a pm_timer_read of it would fail and shift every later read by one).
void pm_timer_release(int kernel) {
    LaunchTimer& t = g_timer[kernel];
    if (t.pending > 0) {
        --t.pending;
        ++t.armed;
    }
}

extern "C" int pm_timer_arm(int32_t kernel) {
    PM_REQUIRE(kernel >= 0 && kernel < PM_TIMER_N, PM_E_ARG, "pm_timer_arm: no kernel %d", kernel);
    LaunchTimer& t = g_timer[kernel];
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return pm_fail((int)e, "pm_timer_arm: %s", hipGetErrorString(e));
    if (t.device != dev) {
        PM_REQUIRE(t.armed == 0 && t.pending == 0, PM_E_ARG, "pm_timer_arm: kernel %d has launches timed on "
                   "device %d", kernel, t.device);
        for (auto& pair : t.ev)
            for (hipEvent_t& ev : pair) {
                if (ev) (void)hipEventDestroy(ev);
                ev = nullptr;
            }
        for (auto& pair : t.ev)
            for (hipEvent_t& ev : pair)
                if ((e = hipEventCreate(&ev)) != hipSuccess)
                    return pm_fail((int)e, "pm_timer_arm: hipEventCreate: %s", hipGetErrorString(e));
        t.device = dev;
    }
    PM_REQUIRE(t.armed + t.pending < kTimerSlots, PM_E_ARG, "pm_timer_arm: kernel %d has %d launches armed or "
               "unread (at most %d)", kernel, t.armed + t.pending, kTimerSlots);
    ++t.armed;
    return 0;
}

extern "C" int pm_timer_read(int32_t kernel, float* ms) {
    PM_REQUIRE(kernel >= 0 && kernel < PM_TIMER_N && ms, PM_E_ARG, "pm_timer_read: kernel %d", kernel);
    LaunchTimer& t = g_timer[kernel];
    PM_REQUIRE(t.pending > 0, PM_E_ARG, "pm_timer_read: no timed launch of kernel %d to read", kernel);
    hipError_t e = hipEventSynchronize(t.ev[t.head][1]);
    if (e == hipSuccess) e = hipEventElapsedTime(ms, t.ev[t.head][0], t.ev[t.head][1]);
    if (e != hipSuccess) return pm_fail((int)e, "pm_timer_read: %s", hipGetErrorString(e));
    t.head = (t.head + 1) % kTimerSlots;
    --t.pending;
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
        case 8: return (int32_t)sizeof(pm_roll_replay);
        default: return -1;
    }
}

