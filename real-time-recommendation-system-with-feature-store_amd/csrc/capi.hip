// ABI bookkeeping: version, status strings, last HIP error.
#include <stdio.h>

#include "rt_common.h"

namespace rt {
static thread_local char g_last_error[256] = "";

void set_last_error(const char* what, hipError_t e) {
    snprintf(g_last_error, sizeof(g_last_error), "%s: %s", what, hipGetErrorString(e));
}
}  // namespace rt

extern "C" int rt_abi_version(void) { return 1; }

extern "C" const char* rt_status_string(int status) {
    switch (status) {
        case RT_OK: return "ok";
        case RT_ERR_INVALID: return "invalid argument";
        case RT_ERR_UNSUPPORTED: return "unsupported shape/dtype";
        case RT_ERR_WORKSPACE: return "workspace too small";
        case RT_ERR_HIP: return "HIP runtime error";
        default: return "unknown status";
    }
}

extern "C" const char* rt_last_error(void) { return rt::g_last_error; }
