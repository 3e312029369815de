// Host-side helpers shared by the libpongmi translation units.
#pragma once
#include <hip/hip_ext.h>
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

// K5 act over part of the grid (pm_rnn.hip): part PM_ACT_ALL / PM_ACT_B (modelB's side only) /
// PM_ACT_A (the opponents' side only); max_blocks > 0 caps the grid (blocks loop over the groups).
int pm_rnn_act_part(const float* w_opp, const int32_t* opp_id, int32_t n_opp, const float* w_B, const float* obsA,
                    const float* obsB, float* hA, float* cA, float* hB, float* cB, const uint8_t* reset, float epsilon,
                    const double* eps_dev, uint64_t seed, uint64_t counter, const uint64_t* counter_dev, int8_t* aA,
                    int8_t* aB, float* qA, float* qB, int32_t n, int32_t chunk0, int32_t chunk1,
                    const int32_t* opp_list, const int32_t* opp_cnt, int32_t part, int32_t max_blocks, void* stream,
                    const float* hA_in = nullptr, const float* cA_in = nullptr);

static inline unsigned pm_blocks(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

// Launch timing (pm_timer_arm / pm_timer_read, pm_api.cpp): an armed kernel's next launch goes
// through hipExtLaunchKernel with the timer's events; every other launch is a plain one.
bool pm_timer_take(int kernel, hipEvent_t* start, hipEvent_t* stop);
void pm_timer_release(int kernel);

template <typename F, typename... Args>
inline void pm_launch(int timer, F kernel, dim3 grid, dim3 block, hipStream_t st, Args... args) {
    hipEvent_t t0, t1;
    if (pm_timer_take(timer, &t0, &t1)) {
        // the error state is sticky per thread: clear whatever an earlier, unrelated call left, so the
        // peek below sees this launch's own result (the caller's PM_LAUNCHED still consumes it)
        (void)hipGetLastError();
        hipExtLaunchKernelGGL(kernel, grid, block, 0, st, t0, t1, 0, args...);
        if (hipPeekAtLastError() != hipSuccess) pm_timer_release(timer);  // never enqueued: not pending
    } else {
        hipLaunchKernelGGL(kernel, grid, block, 0, st, args...);
    }
}

// ---------------------------------------------------------------- diagnostic stamps (PM_DIAG builds only)
// libpongmi_diag.so is built with -DPM_DIAG: thread 0 of block 0 records s_memrealtime (100 MHz)
// at named phase boundaries into pm_diag_buf; pm_diag_read copies them out. The product library
// compiles every stamp to nothing.
