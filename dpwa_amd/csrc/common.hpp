// common.hpp -- error reporting shared by the translation units of libdpwa_hip.so.
#pragma once

#include <cstdarg>
#include <cstdio>

#include "../../include/dpwa_hip.h"

namespace dpwa {

// Records `msg` as the calling thread's last error and returns `code`.
int set_error(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

}  // namespace dpwa

// Returns DPWA_ERR_HIP with the failing call recorded when a HIP call fails.
#define HIP_TRY(expr)                                                                                  \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess)                                                                          \
            return set_error(DPWA_ERR_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #expr, hipGetErrorString(e_)); \
    } while (0)
