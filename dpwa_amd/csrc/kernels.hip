// kernels.hip -- CDNA4 (gfx950) kernels of the pairwise-averaging hot path.
//
//  * lerp:    the averaging statement of dpwa/adapters/pytorch.py:68,
//             param = f32(f32(a*peer) + f32(b*param)), fused into ONE streaming pass over
//             the flat parameter buffer (the reference runs three ATen kernels and allocates
//             three temporaries per tensor).  Pure HBM streaming: 16-byte loads per lane,
//             several independent loads in flight per lane, grid-stride; no LDS, no MFMA
//             (0.25 flop/byte).  Separate roundings are required for bit parity with the
//             reference (an FMA changes up to ~30% of results near cancellation), so
//             contraction is switched off for this whole file.
//  * factor:  dpwa/dpwa.py:139-155 + dpwa/interpolation.py:13-33 in IEEE fp64, one thread,
//             writing the coefficients the lerp reads (no host round trip).
//  * publish: update_send's snapshot (dpwa.py:111-116, pytorch.py:49-53) -- clock += 1 on the
//             device and one copy of the flat buffer into a snapshot slot behind its header.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels.hpp"

namespace dpwa {

constexpr int kBlock = 256;      // 4 waves of 64
constexpr int kUnroll = 4;       // 16-byte items per lane per operand in flight
constexpr int kMaxGrid = 2048;   // 256 CUs x 8 resident blocks

int stream_grid(int64_t vec_items, int per_thread)
{
    int64_t per_block = (int64_t)kBlock * per_thread;
    int64_t g = (vec_items + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > kMaxGrid) g = kMaxGrid;
    return (int)g;
}

struct AB {
    float a, b;
};

// Coefficients: a device block written by the factor kernel (status != 0 -> no-op), or
// values passed by the host.  Uniform address -> scalar loads.
__device__ __forceinline__ bool load_coef(const dpwa_coef *coef, float ha, float hb, AB &ab)
{
    if (coef) {
        if (coef->status != DPWA_STATUS_OK) return false;
        ab.a = coef->a;
        ab.b = coef->b;
    } else {
        ab.a = ha;
        ab.b = hb;
    }
    return true;
}

__device__ __forceinline__ float lerp1(float a, float b, float peer, float param)
{
    float x = a * peer;     // f32(a*t)          pytorch.py:68 `factor * t`
    float y = b * param;    // f32(b*p)          pytorch.py:68 `(1 - factor) * param.data`
    return x + y;           // f32(x + y)        contraction is off for this file
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 lerp4(float a, float b, f32x4 q, f32x4 p)
{
    f32x4 x = a * q;
    f32x4 y = b * p;
    return x + y;
}

// ---------------------------------------------------------------- bf16 helpers
typedef float float2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// Two f32 -> packed bf16, round-to-nearest-even (v_cvt_pk_bf16_f32 on gfx950).
__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi)
{
    float2v v = {lo, hi};
    bf16x2v r = __builtin_convertvector(v, bf16x2v);
    return __builtin_bit_cast(uint32_t, r);
}

// bf16(bf16(a*q) + bf16(b*p)) for the two bf16 held in each 32-bit word (torch-eager form).
__device__ __forceinline__ uint32_t lerp_bf16x2(float a, float b, uint32_t q, uint32_t p)
{
    uint32_t x = pk_bf16(a * bf_lo(q), a * bf_hi(q));
    uint32_t y = pk_bf16(b * bf_lo(p), b * bf_hi(p));
    return pk_bf16(bf_lo(x) + bf_lo(y), bf_hi(x) + bf_hi(y));
}

__device__ __forceinline__ uint4 lerp_bf16x8(float a, float b, uint4 q, uint4 p)
{
    uint4 r;
    r.x = lerp_bf16x2(a, b, q.x, p.x);
    r.y = lerp_bf16x2(a, b, q.y, p.y);
    r.z = lerp_bf16x2(a, b, q.z, p.z);
    r.w = lerp_bf16x2(a, b, q.w, p.w);
    return r;
}

__device__ __forceinline__ uint16_t lerp_bf16x1(float a, float b, uint16_t q, uint16_t p)
{
    return (uint16_t)(lerp_bf16x2(a, b, (uint32_t)q, (uint32_t)p) & 0xffffu);
}

// ---------------------------------------------------------------- lerp kernels
// 16-byte vector path: both pointers 16-byte aligned.  Each lane keeps kUnroll
// param and kUnroll peer loads in flight; a wave instruction covers 1 KiB.
__global__ __launch_bounds__(kBlock) void k_lerp_f32(f32x4 *__restrict__ param,
                                                     const f32x4 *__restrict__ peer, int64_t n,
                                                     const dpwa_coef *__restrict__ coef, float ha, float hb)
{
    AB ab;
    if (!load_coef(coef, ha, hb, ab)) return;
    const int64_t n4 = n >> 2;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    for (; i + (kUnroll - 1) * stride < n4; i += kUnroll * stride) {
        f32x4 p[kUnroll], q[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            q[u] = peer[i + u * stride];
            p[u] = param[i + u * stride];
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) param[i + u * stride] = lerp4(ab.a, ab.b, q[u], p[u]);
    }
    for (; i < n4; i += stride) param[i] = lerp4(ab.a, ab.b, peer[i], param[i]);
    // ragged tail (n % 4 elements)
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        float *pf = reinterpret_cast<float *>(param);
        const float *qf = reinterpret_cast<const float *>(peer);
        const int64_t j = (n4 << 2) + threadIdx.x;
        pf[j] = lerp1(ab.a, ab.b, qf[j], pf[j]);
    }
}

__global__ __launch_bounds__(kBlock) void k_lerp_bf16(uint4 *__restrict__ param, const uint4 *__restrict__ peer,
                                                      int64_t n, const dpwa_coef *__restrict__ coef, float ha,
                                                      float hb)
{
    AB ab;
    if (!load_coef(coef, ha, hb, ab)) return;
    const int64_t n8 = n >> 3;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    for (; i + (kUnroll - 1) * stride < n8; i += kUnroll * stride) {
        uint4 p[kUnroll], q[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            q[u] = peer[i + u * stride];
            p[u] = param[i + u * stride];
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) param[i + u * stride] = lerp_bf16x8(ab.a, ab.b, q[u], p[u]);
    }
    for (; i < n8; i += stride) param[i] = lerp_bf16x8(ab.a, ab.b, peer[i], param[i]);
    if (blockIdx.x == 0 && threadIdx.x < (n & 7)) {
        uint16_t *ph = reinterpret_cast<uint16_t *>(param);
        const uint16_t *qh = reinterpret_cast<const uint16_t *>(peer);
        const int64_t j = (n8 << 3) + threadIdx.x;
        ph[j] = lerp_bf16x1(ab.a, ab.b, qh[j], ph[j]);
    }
}

// Element-wise path for pointers that are not 16-byte aligned (arbitrary views).
__global__ __launch_bounds__(kBlock) void k_lerp_f32_unaligned(float *__restrict__ param,
                                                               const float *__restrict__ peer, int64_t n,
                                                               const dpwa_coef *__restrict__ coef, float ha,
                                                               float hb)
{
    AB ab;
    if (!load_coef(coef, ha, hb, ab)) return;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        param[i] = lerp1(ab.a, ab.b, peer[i], param[i]);
}

__global__ __launch_bounds__(kBlock) void k_lerp_bf16_unaligned(uint16_t *__restrict__ param,
                                                                const uint16_t *__restrict__ peer, int64_t n,
                                                                const dpwa_coef *__restrict__ coef, float ha,
                                                                float hb)
{
    AB ab;
    if (!load_coef(coef, ha, hb, ab)) return;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride)
        param[i] = lerp_bf16x1(ab.a, ab.b, peer[i], param[i]);
}

static inline bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

hipError_t launch_lerp(int32_t dtype, void *param, const void *peer, int64_t n, const dpwa_coef *coef,
                       float a, float b, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    const bool vec = aligned16(param) && aligned16(peer);
    if (dtype == DPWA_F32) {
        if (vec) {
            int g = stream_grid(n >> 2, kUnroll);
            hipLaunchKernelGGL(k_lerp_f32, dim3(g), dim3(kBlock), 0, s, (f32x4 *)param, (const f32x4 *)peer, n,
                               coef, a, b);
        } else {
            int g = stream_grid(n, 1);
            hipLaunchKernelGGL(k_lerp_f32_unaligned, dim3(g), dim3(kBlock), 0, s, (float *)param,
                               (const float *)peer, n, coef, a, b);
        }
    } else if (dtype == DPWA_BF16) {
        if (vec) {
            int g = stream_grid(n >> 3, kUnroll);
            hipLaunchKernelGGL(k_lerp_bf16, dim3(g), dim3(kBlock), 0, s, (uint4 *)param, (const uint4 *)peer, n,
                               coef, a, b);
        } else {
            int g = stream_grid(n, 1);
            hipLaunchKernelGGL(k_lerp_bf16_unaligned, dim3(g), dim3(kBlock), 0, s, (uint16_t *)param,
                               (const uint16_t *)peer, n, coef, a, b);
        }
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ---------------------------------------------------------------- factor
// dpwa.py:139-155 in IEEE double with every operation separately rounded, exactly as
// CPython evaluates it.  Python raises ZeroDivisionError on x/0.0; here that is status 1,
// the clock is left unchanged and the lerp becomes a no-op.
__global__ void k_factor(dpwa_interp cfg, double *__restrict__ clock, const dpwa_header *__restrict__ peer,
                         double loss_h, const double *__restrict__ loss_d, dpwa_coef *__restrict__ coef,
                         int32_t *__restrict__ status_mirror)
{
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    const double loss = loss_d ? *loss_d : loss_h;
    const double c = *clock;
    const double pc = peer->clock;
    const double pl = peer->loss;
    int32_t status = DPWA_STATUS_OK;
    double f = 0.0;
    if (cfg.method == DPWA_INTERP_CONSTANT) {          // interpolation.py:13-15
        f = cfg.value;
    } else if (cfg.method == DPWA_INTERP_CLOCK) {      // interpolation.py:22-24
        const double den = c + pc;
        if (den == 0.0) status = DPWA_STATUS_ZERO_DIVISION;
        else f = pc / den;
    } else {                                           // interpolation.py:31-33
        const double den = loss + pl;
        if (den == 0.0) status = DPWA_STATUS_ZERO_DIVISION;
        else f = loss / den;
    }
    if (status == DPWA_STATUS_OK && loss < cfg.divergence_threshold) {   // dpwa.py:146-147
        if (cfg.divergence_threshold == 0.0) status = DPWA_STATUS_ZERO_DIVISION;
        else f = f * (loss / cfg.divergence_threshold);
    }
    dpwa_coef out;
    out.status = status;
    out.reserved = 0;
    if (status == DPWA_STATUS_OK) {
        const double nc = f * pc + (1.0 - f) * c;      // dpwa.py:150
        out.factor = f;
        out.new_clock = nc;
        out.a = (float)f;                              // torch: Python float -> fp32 scalar
        out.b = (float)(1.0 - f);                      // `1 - factor` in double, then fp32
        *clock = nc;                                   // dpwa.py:155
    } else {
        out.factor = 0.0;
        out.new_clock = c;
        out.a = 0.0f;
        out.b = 1.0f;
    }
    *coef = out;
    if (status_mirror && status != DPWA_STATUS_OK) *status_mirror = status;   // sticky pinned host word
}

hipError_t launch_factor(const dpwa_interp &cfg, double *clock, const dpwa_header *peer, double loss,
                         const double *loss_dev, dpwa_coef *coef, int32_t *status_mirror, hipStream_t s)
{
    hipLaunchKernelGGL(k_factor, dim3(1), dim3(64), 0, s, cfg, clock, peer, loss, loss_dev, coef, status_mirror);
    return hipGetLastError();
}

// ---------------------------------------------------------------- publish
template <bool VEC, bool SYS_RELEASE>
__global__ __launch_bounds__(kBlock) void k_publish(char *__restrict__ slot, const char *__restrict__ flat,
                                                    int64_t nbytes, int64_t n, int32_t dtype,
                                                    double *__restrict__ clock, double loss_h,
                                                    const double *__restrict__ loss_d, uint64_t version)
{
    char *payload = slot + sizeof(dpwa_header);
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (VEC) {
        const int64_t n16 = nbytes >> 4;
        const uint4 *src = reinterpret_cast<const uint4 *>(flat);
        uint4 *dst = reinterpret_cast<uint4 *>(payload);
        for (; i + (kUnroll - 1) * stride < n16; i += kUnroll * stride) {
            uint4 v[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) v[u] = src[i + u * stride];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) dst[i + u * stride] = v[u];
        }
        for (; i < n16; i += stride) dst[i] = src[i];
        if (blockIdx.x == 0 && threadIdx.x < (nbytes & 15)) {
            const int64_t j = (n16 << 4) + threadIdx.x;
            payload[j] = flat[j];
        }
    } else {
        for (; i < nbytes; i += stride) payload[i] = flat[i];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        dpwa_header *h = reinterpret_cast<dpwa_header *>(slot);
        const double c = *clock + 1.0;                 // dpwa.py:112  self.clock += 1
        *clock = c;
        h->clock = c;                                  // dpwa.py:115  state = {'clock', 'loss'}
        h->loss = loss_d ? *loss_d : loss_h;
        h->version = version;
        h->n = n;
        h->dtype = dtype;
    }
    if (SYS_RELEASE) {
        __syncthreads();
        if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope
    }
}

hipError_t launch_publish(char *slot, const void *flat, int64_t nbytes, int64_t n, int32_t dtype, double *clock,
                          double loss, const double *loss_dev, uint64_t version, bool system_release,
                          hipStream_t s)
{
    const bool vec = aligned16(flat);
    const int g = vec ? stream_grid(nbytes >> 4, kUnroll) : stream_grid(nbytes, 4);
    const char *src = (const char *)flat;
    if (vec && system_release)
        hipLaunchKernelGGL((k_publish<true, true>), dim3(g), dim3(kBlock), 0, s, slot, src, nbytes, n, dtype, clock,
                           loss, loss_dev, version);
    else if (vec)
        hipLaunchKernelGGL((k_publish<true, false>), dim3(g), dim3(kBlock), 0, s, slot, src, nbytes, n, dtype,
                           clock, loss, loss_dev, version);
    else if (system_release)
        hipLaunchKernelGGL((k_publish<false, true>), dim3(g), dim3(kBlock), 0, s, slot, src, nbytes, n, dtype,
                           clock, loss, loss_dev, version);
    else
        hipLaunchKernelGGL((k_publish<false, false>), dim3(g), dim3(kBlock), 0, s, slot, src, nbytes, n, dtype,
                           clock, loss, loss_dev, version);
    return hipGetLastError();
}

}  // namespace dpwa
