// common.hpp -- error reporting shared by the translation units of libdpwa_hip.so.
#pragma once

#include <cstdarg>
#include <cstdio>

#include "../../include/dpwa_hip.h"

namespace dpwa {

// Records `msg` as the calling thread's last error and returns `code`.
int set_error(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

}  // namespace dpwa
