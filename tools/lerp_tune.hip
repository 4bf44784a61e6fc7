// lerp_tune.hip -- standalone variant sweep for the fused lerp (not part of the product).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -o tools/lerp_tune tools/lerp_tune.hip
// Run:   tools/lerp_tune [numel] [rounds]
// Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24); buffers rotate over
// > 1 GiB so every launch streams from HBM, not the 256 MiB Infinity Cache.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e = (x);                                                                   \
        if (e != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e));  \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 lerp4(float a, float b, f32x4 q, f32x4 p)
{
    f32x4 x = a * q;
    f32x4 y = b * p;
    return x + y;
}

template <typename T>
__device__ __forceinline__ T ld(const T *p, bool nt)
{
    return nt ? __builtin_nontemporal_load(p) : *p;
}
template <typename T>
__device__ __forceinline__ void st(T *p, T v, bool nt)
{
    if (nt) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// Grid-stride, U items per lane in flight (interleaved by grid stride).
template <int BLOCK, int U, bool NT_LD_Q, bool NT_LD_P, bool NT_ST>
__global__ __launch_bounds__(BLOCK) void k_gs(f32x4 *__restrict__ param, const f32x4 *__restrict__ peer,
                                              int64_t n4, float a, float b)
{
    const int64_t stride = (int64_t)gridDim.x * BLOCK;
    int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    for (; i + (U - 1) * stride < n4; i += U * stride) {
        f32x4 p[U], q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            q[u] = ld(peer + i + u * stride, NT_LD_Q);
            p[u] = ld(param + i + u * stride, NT_LD_P);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) st(param + i + u * stride, lerp4(a, b, q[u], p[u]), NT_ST);
    }
    for (; i < n4; i += stride) st(param + i, lerp4(a, b, ld(peer + i, NT_LD_Q), ld(param + i, NT_LD_P)), NT_ST);
}

// Block-contiguous tiles: block t owns items [t*BLOCK*U, (t+1)*BLOCK*U), lanes interleaved within.
template <int BLOCK, int U, bool NT>
__global__ __launch_bounds__(BLOCK) void k_tile(f32x4 *__restrict__ param, const f32x4 *__restrict__ peer,
                                                int64_t n4, float a, float b)
{
    const int64_t tiles = (n4 + (int64_t)BLOCK * U - 1) / ((int64_t)BLOCK * U);
    for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        const int64_t base = t * BLOCK * U + threadIdx.x;
        if (base + (U - 1) * BLOCK < n4) {
            f32x4 p[U], q[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                q[u] = ld(peer + base + u * BLOCK, NT);
                p[u] = ld(param + base + u * BLOCK, false);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) st(param + base + u * BLOCK, lerp4(a, b, q[u], p[u]), NT);
        } else {
            for (int u = 0; u < U; ++u) {
                int64_t i = base + u * BLOCK;
                if (i < n4) param[i] = lerp4(a, b, peer[i], param[i]);
            }
        }
    }
}

// Software-pipelined grid stride: the next item's loads are issued before this item's
// store, so the in-order vmcnt wait for them does not also wait for the store.
template <int BLOCK, bool NT_ST>
__global__ __launch_bounds__(BLOCK) void k_pipe(f32x4 *__restrict__ param, const f32x4 *__restrict__ peer,
                                                int64_t n4, float a, float b)
{
    const int64_t stride = (int64_t)gridDim.x * BLOCK;
    int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n4) return;
    f32x4 q = peer[i], p = param[i];
    for (;;) {
        const int64_t j = i + stride;
        f32x4 q2, p2;
        const bool more = j < n4;
        if (more) {
            q2 = peer[j];
            p2 = param[j];
        }
        st(param + i, lerp4(a, b, q, p), NT_ST);
        if (!more) break;
        q = q2;
        p = p2;
        i = j;
    }
}

// One item per lane, exact grid, optional second destination (publish fused into the lerp).
template <int BLOCK, bool DUAL, bool NT_ST>
__global__ __launch_bounds__(BLOCK) void k_one(f32x4 *__restrict__ param, const f32x4 *__restrict__ peer,
                                               f32x4 *__restrict__ snap, int64_t n4, float a, float b)
{
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n4) return;
    const f32x4 r = lerp4(a, b, peer[i], param[i]);
    st(param + i, r, NT_ST);
    if (DUAL) st(snap + i, r, NT_ST);
}

// One item per lane with a cache policy per operand (nt = streamed once, no reuse).
template <int BLOCK, bool NTQ, bool NTP, bool NTS>
__global__ __launch_bounds__(BLOCK) void k_one_nt(f32x4 *__restrict__ param, const f32x4 *__restrict__ peer,
                                                  int64_t n4, float a, float b)
{
    const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n4) return;
    const f32x4 q = ld(peer + i, NTQ);
    const f32x4 p = ld(param + i, NTP);
    st(param + i, lerp4(a, b, q, p), NTS);
}

// One item per lane, blockIdx remapped so that each XCD (blocks are dealt round-robin over
// the 8 XCDs) sweeps one contiguous eighth of the buffer.  Grid padded to a multiple of 8.
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_one_xcd(f32x4 *__restrict__ param, const f32x4 *__restrict__ peer,
                                                   int64_t n4, float a, float b)
{
    const uint32_t per = gridDim.x / 8;
    const uint32_t t = (blockIdx.x % 8) * per + blockIdx.x / 8;
    const int64_t i = (int64_t)t * BLOCK + threadIdx.x;
    if (i >= n4) return;
    param[i] = lerp4(a, b, peer[i], param[i]);
}

// Buffer loads/stores (range-checked, no branch) with explicit aux cache bits
// (gfx950: 1 = sc0, 2 = nt, 16 = sc1).  32-bit byte offsets: operands < 2 GiB.
typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));
template <int BLOCK, int AUXQ, int AUXP, int AUXS>
__global__ __launch_bounds__(BLOCK) void k_buf(float *__restrict__ param, const float *__restrict__ peer, int64_t n4,
                                               float a, float b)
{
    const int nbytes = (int)(n4 * 16);
    __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(param, 0, nbytes, 0x00020000);
    __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc((void *)peer, 0, nbytes, 0x00020000);
    const int off = (int)(((int64_t)blockIdx.x * BLOCK + threadIdx.x) * 16);
    const u32x4v q = __builtin_amdgcn_raw_buffer_load_b128(rq, off, 0, AUXQ);
    const u32x4v p = __builtin_amdgcn_raw_buffer_load_b128(rp, off, 0, AUXP);
    const f32x4 r = lerp4(a, b, __builtin_bit_cast(f32x4, q), __builtin_bit_cast(f32x4, p));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, r), rp, off, 0, AUXS);
}

// U items per lane, each block one contiguous BLOCK*16*U-byte span; all 2U loads issued
// before the first store (fewer, fatter workgroups than k_buf).
template <int BLOCK, int U, int AUXL, int AUXS>
__global__ __launch_bounds__(BLOCK) void k_bufu(float *__restrict__ param, const float *__restrict__ peer, int64_t n4,
                                                float a, float b)
{
    const int nbytes = (int)(n4 * 16);
    __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(param, 0, nbytes, 0x00020000);
    __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc((void *)peer, 0, nbytes, 0x00020000);
    const int base = (int)((int64_t)blockIdx.x * BLOCK * U * 16) + threadIdx.x * 16;
    u32x4v q[U], p[U];
#pragma unroll
    for (int u = 0; u < U; ++u) q[u] = __builtin_amdgcn_raw_buffer_load_b128(rq, base + u * BLOCK * 16, 0, AUXL);
#pragma unroll
    for (int u = 0; u < U; ++u) p[u] = __builtin_amdgcn_raw_buffer_load_b128(rp, base + u * BLOCK * 16, 0, AUXL);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const f32x4 r = lerp4(a, b, __builtin_bit_cast(f32x4, q[u]), __builtin_bit_cast(f32x4, p[u]));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, r), rp, base + u * BLOCK * 16, 0, AUXS);
    }
}

// Two items per lane, block-contiguous (512 items per 256-thread block): all four loads are
// issued before the first store.
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_two(f32x4 *__restrict__ param, const f32x4 *__restrict__ peer, int64_t n4,
                                               float a, float b)
{
    const int64_t i = (int64_t)blockIdx.x * (2 * BLOCK) + threadIdx.x;
    const int64_t j = i + BLOCK;
    if (j < n4) {
        const f32x4 q0 = peer[i], p0 = param[i], q1 = peer[j], p1 = param[j];
        param[i] = lerp4(a, b, q0, p0);
        param[j] = lerp4(a, b, q1, p1);
    } else if (i < n4) {
        param[i] = lerp4(a, b, peer[i], param[i]);
    }
}

// One-item-per-lane buffer copy (the publish shape) with a load cache policy.
template <int BLOCK, int AUXL, int AUXS>
__global__ __launch_bounds__(BLOCK) void k_copybuf(float *__restrict__ dst, const float *__restrict__ src, int64_t n4)
{
    const int nbytes = (int)(n4 * 16);
    __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(dst, 0, nbytes, 0x00020000);
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)src, 0, nbytes, 0x00020000);
    const int off = (int)(((int64_t)blockIdx.x * BLOCK + threadIdx.x) * 16);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, AUXL), rd, off, 0, AUXS);
}

// Copy (1R:1W) and read-only reduction, for calibration.
__global__ __launch_bounds__(256) void k_copy(f32x4 *__restrict__ dst, const f32x4 *__restrict__ src, int64_t n4)
{
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n4; i += 4 * stride) {
        f32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = src[i + u * stride];
#pragma unroll
        for (int u = 0; u < 4; ++u) dst[i + u * stride] = v[u];
    }
    for (; i < n4; i += stride) dst[i] = src[i];
}

struct Variant {
    std::string name;
    double bytes_factor;   // x numel*4
    std::function<void(float *, float *, int64_t, hipStream_t)> run;
};

static int grid_for(int64_t items, int per_block, int cap)
{
    int64_t g = (items + per_block - 1) / per_block;
    if (cap > 0 && g > cap) g = cap;
    return (int)std::max<int64_t>(g, 1);
}

template <int BLOCK, int U, bool A, bool B, bool C>
Variant gs(const char *name, int cap)
{
    return {name, 3.0, [cap](float *p, float *q, int64_t n, hipStream_t s) {
                int64_t n4 = n / 4;
                int g = grid_for(n4, BLOCK * U, cap);
                hipLaunchKernelGGL((k_gs<BLOCK, U, A, B, C>), dim3(g), dim3(BLOCK), 0, s, (f32x4 *)p, (const f32x4 *)q,
                                   n4, 0.5f, 0.5f);
            }};
}

template <int BLOCK, int U, bool NT>
Variant tile(const char *name, int cap)
{
    return {name, 3.0, [cap](float *p, float *q, int64_t n, hipStream_t s) {
                int64_t n4 = n / 4;
                int g = grid_for(n4, BLOCK * U, cap);
                hipLaunchKernelGGL((k_tile<BLOCK, U, NT>), dim3(g), dim3(BLOCK), 0, s, (f32x4 *)p, (const f32x4 *)q, n4,
                                   0.5f, 0.5f);
            }};
}

template <int BLOCK, bool NT>
Variant pipe(const char *name, int cap)
{
    return {name, 3.0, [cap](float *p, float *q, int64_t n, hipStream_t s) {
                int64_t n4 = n / 4;
                int g = grid_for(n4, BLOCK, cap);
                hipLaunchKernelGGL((k_pipe<BLOCK, NT>), dim3(g), dim3(BLOCK), 0, s, (f32x4 *)p, (const f32x4 *)q, n4,
                                   0.5f, 0.5f);
            }};
}

static float *g_snap = nullptr;

template <int BLOCK, bool DUAL, bool NT>
Variant one(const char *name)
{
    return {name, DUAL ? 4.0 : 3.0, [](float *p, float *q, int64_t n, hipStream_t s) {
                int64_t n4 = n / 4;
                int g = grid_for(n4, BLOCK, 0);
                hipLaunchKernelGGL((k_one<BLOCK, DUAL, NT>), dim3(g), dim3(BLOCK), 0, s, (f32x4 *)p, (const f32x4 *)q,
                                   (f32x4 *)g_snap, n4, 0.5f, 0.5f);
            }};
}

template <int BLOCK, bool NTQ, bool NTP, bool NTS>
Variant one_nt(const char *name)
{
    return {name, 3.0, [](float *p, float *q, int64_t n, hipStream_t s) {
                int64_t n4 = n / 4;
                hipLaunchKernelGGL((k_one_nt<BLOCK, NTQ, NTP, NTS>), dim3(grid_for(n4, BLOCK, 0)), dim3(BLOCK), 0, s,
                                   (f32x4 *)p, (const f32x4 *)q, n4, 0.5f, 0.5f);
            }};
}

template <int BLOCK>
Variant one_xcd(const char *name)
{
    return {name, 3.0, [](float *p, float *q, int64_t n, hipStream_t s) {
                int64_t n4 = n / 4;
                int g = (grid_for(n4, BLOCK, 0) + 7) / 8 * 8;
                hipLaunchKernelGGL((k_one_xcd<BLOCK>), dim3(g), dim3(BLOCK), 0, s, (f32x4 *)p, (const f32x4 *)q, n4,
                                   0.5f, 0.5f);
            }};
}

template <int BLOCK, int AQ, int AP, int AS>
Variant buf(const char *name)
{
    return {name, 3.0, [](float *p, float *q, int64_t n, hipStream_t s) {
                int64_t n4 = n / 4;
                hipLaunchKernelGGL((k_buf<BLOCK, AQ, AP, AS>), dim3(grid_for(n4, BLOCK, 0)), dim3(BLOCK), 0, s, p, q,
                                   n4, 0.5f, 0.5f);
            }};
}

template <int BLOCK, int U, int AL, int AS>
Variant bufu(const char *name)
{
    return {name, 3.0, [](float *p, float *q, int64_t n, hipStream_t s) {
                int64_t n4 = n / 4;
                hipLaunchKernelGGL((k_bufu<BLOCK, U, AL, AS>), dim3(grid_for(n4, BLOCK * U, 0)), dim3(BLOCK), 0, s, p,
                                   q, n4, 0.5f, 0.5f);
            }};
}

template <int BLOCK>
Variant two(const char *name)
{
    return {name, 3.0, [](float *p, float *q, int64_t n, hipStream_t s) {
                int64_t n4 = n / 4;
                hipLaunchKernelGGL((k_two<BLOCK>), dim3(grid_for(n4, 2 * BLOCK, 0)), dim3(BLOCK), 0, s, (f32x4 *)p,
                                   (const f32x4 *)q, n4, 0.5f, 0.5f);
            }};
}

template <int BLOCK, int AUXL, int AUXS>
Variant copybuf(const char *name)
{
    return {name, 2.0, [](float *p, float *q, int64_t n, hipStream_t s) {
                int64_t n4 = n / 4;
                hipLaunchKernelGGL((k_copybuf<BLOCK, AUXL, AUXS>), dim3(grid_for(n4, BLOCK, 0)), dim3(BLOCK), 0, s, p, q, n4);
            }};
}

int main(int argc, char **argv)
{
    int64_t n = argc > 1 ? atoll(argv[1]) : 11173962;
    int rounds = argc > 2 ? atoi(argv[2]) : 20;
    n = n / 4 * 4;
    const size_t bytes = (size_t)n * 4;
    // argv[3]: buffer pairs to rotate over (default: > 1.5 GB between reuses = cold;
    // 1 = the same pair every launch, Infinity-Cache warm like the in-loop kernel)
    int pairs = (int)std::max<size_t>(4, (size_t)(1.5e9 / (2 * bytes)) + 1);
    if (argc > 3) pairs = std::max(1, atoi(argv[3]));
    std::vector<float *> P(pairs), Q(pairs);
    for (int i = 0; i < pairs; ++i) {
        CHECK(hipMalloc(&P[i], bytes));
        CHECK(hipMalloc(&Q[i], bytes));
        std::vector<float> h((size_t)n);
        uint32_t x = 12345u + (uint32_t)i;
        for (auto &v : h) {   // random data (zero-filled operands can change the clock the chip holds)
            x = x * 1664525u + 1013904223u;
            v = (float)((int32_t)(x >> 8) - (1 << 23)) / (float)(1 << 23);
        }
        CHECK(hipMemcpy(P[i], h.data(), bytes, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(Q[i], h.data(), bytes, hipMemcpyHostToDevice));
    }
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    CHECK(hipMalloc(&g_snap, bytes));
    std::vector<Variant> vs = {
        buf<256, 2, 2, 16>("buf256 nt loads sc1 store (r01d product)"),
        buf<64, 2, 2, 16>("buf64 nt loads sc1 store (product)"),
        buf<64, 0, 0, 16>("buf64 plain loads sc1 store"),
        buf<64, 2, 0, 16>("buf64 nt peer, plain param, sc1 store"),
        buf<64, 2, 2, 2>("buf64 nt loads nt store"),
        buf<64, 2, 2, 17>("buf64 nt loads sc0+sc1 store"),
        buf<64, 2, 2, 0>("buf64 nt loads plain store"),
        buf<64, 18, 18, 16>("buf64 nt+sc1 loads sc1 store"),
        buf<128, 2, 2, 16>("buf128 nt loads sc1 store"),
        bufu<64, 2, 2, 16>("bufu64x2 nt loads sc1 store"),
        copybuf<256, 2, 16>("copybuf256 nt load sc1 store (x2 bytes)"),
        copybuf<64, 2, 16>("copybuf64 nt load sc1 store (x2 bytes)"),
        {"hipMemcpyAsync D2D (x2 bytes)", 2.0,
         [](float *p, float *q, int64_t n, hipStream_t s) { (void)hipMemcpyAsync(p, q, n * 4, hipMemcpyDeviceToDevice, s); }},
    };
    std::vector<std::vector<double>> us(vs.size());
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    int rot = 0;
    for (int r = 0; r < rounds + 2; ++r) {
        for (size_t v = 0; v < vs.size(); ++v) {
            const int reps = 8;
            CHECK(hipEventRecord(e0, s));
            for (int k = 0; k < reps; ++k) {
                vs[v].run(P[rot % pairs], Q[rot % pairs], n, s);
                rot++;
            }
            CHECK(hipEventRecord(e1, s));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2) us[v].push_back(1e3 * ms / reps);
        }
    }
    printf("numel %lld (%.1f MB per operand), %d rotating pairs, %d rounds x 8 launches\n", (long long)n, bytes / 1e6,
           pairs, rounds);
    for (size_t v = 0; v < vs.size(); ++v) {
        auto x = us[v];
        std::sort(x.begin(), x.end());
        double med = x[x.size() / 2], best = x[0];
        double gb = vs[v].bytes_factor * bytes;
        printf("%-34s median %8.2f us  %7.1f GB/s (%.1f%%)   best %7.1f GB/s\n", vs[v].name.c_str(), med, gb / med / 1e3,
               100.0 * gb / med / 1e3 / 8000.0, gb / best / 1e3);
    }
    return 0;
}
