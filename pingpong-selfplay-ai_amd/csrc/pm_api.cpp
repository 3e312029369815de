// libpongmi host utilities: error reporting and ABI introspection.
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

