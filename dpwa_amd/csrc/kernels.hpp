// kernels.hpp -- internal launch API of the HIP kernels (kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "common.hpp"

namespace dpwa {

// Size in bytes of one element of `dtype`, 0 if unknown.
inline size_t dtype_size(int32_t dtype)
{
    return dtype == DPWA_F32 ? 4 : dtype == DPWA_BF16 ? 2 : 0;
}

// Lerp over n elements; coefficients from `coef` (device) or, when coef is null, from (a, b).
hipError_t launch_lerp(int32_t dtype, void *param, const void *peer, int64_t n, const dpwa_coef *coef,
                       float a, float b, hipStream_t s);

// Factor + clock (one thread).  `status_mirror` (nullable) is a device-visible pinned host
// word that receives the status as well.
hipError_t launch_factor(const dpwa_interp &cfg, double *clock, const dpwa_header *peer, double loss,
                         const double *loss_dev, dpwa_coef *coef, int32_t *status_mirror, hipStream_t s);

// Snapshot publish: slot header {clock+1, loss, version, n, dtype} + payload copy of `nbytes`.
// `system_release` adds a system-scope release so that other devices (IPC peers) read the
// bytes from memory rather than from this device's L2.
hipError_t launch_publish(char *slot, const void *flat, int64_t nbytes, int64_t n, int32_t dtype,
                          double *clock, double loss, const double *loss_dev, uint64_t version,
                          bool system_release, hipStream_t s);

// Grid size used for streaming kernels over `vec_items` 16-byte items.
int stream_grid(int64_t vec_items, int per_thread);

}  // namespace dpwa
