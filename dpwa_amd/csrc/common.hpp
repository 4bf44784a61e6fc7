// common.hpp -- error reporting shared by the translation units of libdpwa_hip.so.
#pragma once

#include <cstdarg>
#include <cstdio>

#include "../../include/dpwa_hip.h"

namespace dpwa {

// Records `msg` as the calling thread's last error and returns `code`.
int set_error(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

// roctx ranges (trace.cpp): on only when DPWA_ROCTX=1 was set when the library loaded.
extern const bool g_trace;
void trace_push(const char *name);
void trace_pop();

// A named range over the scope; off, one load and a not-taken branch.
class TraceRange {
public:
    explicit TraceRange(const char *name) : on_(g_trace)
    {
        if (on_) trace_push(name);
    }
    ~TraceRange()
    {
        if (on_) trace_pop();
    }
    TraceRange(const TraceRange &) = delete;
    TraceRange &operator=(const TraceRange &) = delete;

private:
    bool on_;
};

}  // namespace dpwa

// Returns DPWA_ERR_HIP with the failing call recorded when a HIP call fails.
#define HIP_TRY(expr)                                                                                  \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess)                                                                          \
            return set_error(DPWA_ERR_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #expr, hipGetErrorString(e_)); \
    } while (0)
