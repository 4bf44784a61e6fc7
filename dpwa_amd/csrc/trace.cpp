// trace.cpp -- roctx ranges on the gossip round (SURVEY §5 tracing; the reference's only tracing
// is LOGGER.debug at dpwa.py:119,152-153 and conn.py:242-243,296).  With DPWA_ROCTX=1 in the
// environment when the library loads, the ranges named in node.cpp / learner.cpp are pushed and
// popped through the ROCm profiler SDK's roctx library (opened with dlopen, so the library links
// no profiler), and `rocprofv3 --marker-trace` shows each round's host phases between its kernels.
// Off (the default), a range is one load and a not-taken branch: nothing else runs.
#include <dlfcn.h>

#include <cstdlib>
#include <cstring>
#include <initializer_list>

#include "common.hpp"

namespace dpwa {

namespace {

using PushFn = int (*)(const char *);
using PopFn = int (*)();

PushFn g_push = nullptr;
PopFn g_pop = nullptr;

bool open_roctx()
{
    const char *on = getenv("DPWA_ROCTX");
    if (!on || strcmp(on, "1") != 0) return false;
    for (const char *lib : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                            "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1"}) {
        void *h = dlopen(lib, RTLD_NOW | RTLD_LOCAL);
        if (!h) continue;
        g_push = reinterpret_cast<PushFn>(dlsym(h, "roctxRangePushA"));
        g_pop = reinterpret_cast<PopFn>(dlsym(h, "roctxRangePop"));
        if (g_push && g_pop) return true;
        g_push = nullptr;
        g_pop = nullptr;
    }
    return false;
}

}  // namespace

// Decided once, at load (static initialisation), before any thread can call in.
extern const bool g_trace = open_roctx();

void trace_push(const char *name) { g_push(name); }
void trace_pop() { g_pop(); }

}  // namespace dpwa

extern "C" int dpwa_trace_enabled(void) { return dpwa::g_trace ? 1 : 0; }

extern "C" int dpwa_trace_push(const char *name)
{
    if (dpwa::g_trace && name) dpwa::trace_push(name);
    return DPWA_OK;
}

extern "C" int dpwa_trace_pop(void)
{
    if (dpwa::g_trace) dpwa::trace_pop();
    return DPWA_OK;
}
