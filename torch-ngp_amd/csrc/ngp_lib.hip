// Library-wide entry points: ABI version and per-thread error message.
#include "ngp_common.h"
#include "ngp_error.h"

#include <cstdio>
#include <cstdarg>

static thread_local char g_last_error[512] = "";

int ngp_set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
    return code;
}

int ngp_check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        return ngp_set_error(NGP_ERR_HIP, "%s: HIP launch failed: %s", what, hipGetErrorString(e));
    }
    return NGP_OK;
}

extern "C" int ngp_abi_version(void) { return 1; }

extern "C" const char* ngp_last_error(void) { return g_last_error; }
