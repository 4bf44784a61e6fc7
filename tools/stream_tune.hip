// stream_tune.hip -- per-launch cold timing of HBM streaming shapes (not part of the product).
//
// Characterises the chip's streaming ceilings by access mix (read-only, write-only, copy, the
// 2R:1W average, the 2R:2W write-through average) and tries work shapes for the averaging
// kernel.  Every launch is timed by its own dispatch begin/end events (hipExtLaunchKernelGGL),
// buffers rotate over > 1.5 GB so nothing is served from the 256 MiB Infinity Cache, and the
// variants are interleaved round by round (one process, same clocks).
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -o tools/stream_tune tools/stream_tune.hip
// Run:   tools/stream_tune [numel] [rounds]
#pragma clang fp contract(off)
#include <hip/hip_ext.h>
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
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int NT = 2, SC1 = 16;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, int64_t off, int64_t total, int span)
{
    const int64_t rem = total - off;
    const int num = rem <= 0 ? 0 : (rem < span ? (int)rem : span);
    return __builtin_amdgcn_make_buffer_rsrc((void *)((const char *)p + off), 0, num, 0x00020000);
}
template <int AUX>
__device__ __forceinline__ f32x4 ld(__amdgpu_buffer_rsrc_t r, int off)
{
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX));
}
template <int AUX>
__device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, int off, f32x4 v)
{
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, AUX);
}
__device__ __forceinline__ f32x4 lerp4(float a, float b, f32x4 q, f32x4 p)
{
    f32x4 x = a * q;
    f32x4 y = b * p;
    return x + y;
}

struct Args {
    float *param;
    const float *peer;
    float *snap;
    float *sink;
    int64_t bytes;   // per operand
};

// ---- ceilings --------------------------------------------------------------------------
template <int BLOCK, int U>
__global__ __launch_bounds__(BLOCK) void k_read(Args a)
{
    const int64_t span = (int64_t)BLOCK * 16 * U;
    const int64_t off = (int64_t)blockIdx.x * span;
    auto r = rsrc(a.peer, off, a.bytes, (int)span);
    f32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) acc += ld<NT>(r, threadIdx.x * 16 + u * BLOCK * 16);
    if (acc.x == 1234.5f) a.sink[threadIdx.x] = acc.y;   // keeps the loads
}
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_write(Args a)
{
    const int64_t span = (int64_t)BLOCK * 16;
    const int64_t off = (int64_t)blockIdx.x * span;
    st<SC1>(rsrc(a.param, off, a.bytes, (int)span), threadIdx.x * 16, f32x4{1, 2, 3, 4});
}
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_copy(Args a)
{
    const int64_t span = (int64_t)BLOCK * 16;
    const int64_t off = (int64_t)blockIdx.x * span;
    st<SC1>(rsrc(a.param, off, a.bytes, (int)span), threadIdx.x * 16, ld<NT>(rsrc(a.peer, off, a.bytes, (int)span), threadIdx.x * 16));
}

// ---- averaging shapes ------------------------------------------------------------------
// U items per lane, block span BLOCK*16*U, all loads first; DUAL also stores into snap.
template <int BLOCK, int U, bool DUAL, int AUXP = NT, int AUXS = SC1, int AUXN = AUXS>
__global__ __launch_bounds__(BLOCK) void k_avg(Args a)
{
    const int64_t span = (int64_t)BLOCK * 16 * U;
    const int64_t off = (int64_t)blockIdx.x * span;
    auto rq = rsrc(a.peer, off, a.bytes, (int)span);
    auto rp = rsrc(a.param, off, a.bytes, (int)span);
    f32x4 q[U], p[U];
#pragma unroll
    for (int u = 0; u < U; ++u) q[u] = ld<NT>(rq, threadIdx.x * 16 + u * BLOCK * 16);
#pragma unroll
    for (int u = 0; u < U; ++u) p[u] = ld<AUXP>(rp, threadIdx.x * 16 + u * BLOCK * 16);
    auto rs = rsrc(a.snap, off, a.bytes, (int)span);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const f32x4 r = lerp4(0.5f, 0.5f, q[u], p[u]);
        st<AUXS>(rp, threadIdx.x * 16 + u * BLOCK * 16, r);
        if (DUAL) st<AUXN>(rs, threadIdx.x * 16 + u * BLOCK * 16, r);
    }
}

// The resident (out-of-place) average: reads param and peer, stores ONLY into snap (2R:1W to a
// third buffer: the learner reads the published slot and writes the other one).
template <int BLOCK, int U, int AUXS = SC1>
__global__ __launch_bounds__(BLOCK) void k_oop(Args a)
{
    const int64_t span = (int64_t)BLOCK * 16 * U;
    const int64_t off = (int64_t)blockIdx.x * span;
    auto rq = rsrc(a.peer, off, a.bytes, (int)span);
    auto rp = rsrc(a.param, off, a.bytes, (int)span);
    f32x4 q[U], p[U];
#pragma unroll
    for (int u = 0; u < U; ++u) q[u] = ld<NT>(rq, threadIdx.x * 16 + u * BLOCK * 16);
#pragma unroll
    for (int u = 0; u < U; ++u) p[u] = ld<NT>(rp, threadIdx.x * 16 + u * BLOCK * 16);
    auto rs = rsrc(a.snap, off, a.bytes, (int)span);
#pragma unroll
    for (int u = 0; u < U; ++u) st<AUXS>(rs, threadIdx.x * 16 + u * BLOCK * 16, lerp4(0.5f, 0.5f, q[u], p[u]));
}

// Persistent grid, software-pipelined: the next span's loads are issued before this span's
// stores, so the in-order vmcnt wait for them never waits on a store.
template <int BLOCK, bool DUAL>
__global__ __launch_bounds__(BLOCK) void k_pipe(Args a)
{
    const int64_t span = (int64_t)BLOCK * 16;
    const int64_t nspan = (a.bytes + span - 1) / span;
    int64_t t = blockIdx.x;
    if (t >= nspan) return;
    f32x4 q = ld<NT>(rsrc(a.peer, t * span, a.bytes, (int)span), threadIdx.x * 16);
    f32x4 p = ld<NT>(rsrc(a.param, t * span, a.bytes, (int)span), threadIdx.x * 16);
    for (;;) {
        const int64_t nt = t + gridDim.x;
        f32x4 q2, p2;
        if (nt < nspan) {
            q2 = ld<NT>(rsrc(a.peer, nt * span, a.bytes, (int)span), threadIdx.x * 16);
            p2 = ld<NT>(rsrc(a.param, nt * span, a.bytes, (int)span), threadIdx.x * 16);
        }
        const f32x4 r = lerp4(0.5f, 0.5f, q, p);
        st<SC1>(rsrc(a.param, t * span, a.bytes, (int)span), threadIdx.x * 16, r);
        if (DUAL) st<SC1>(rsrc(a.snap, t * span, a.bytes, (int)span), threadIdx.x * 16, r);
        if (nt >= nspan) break;
        q = q2;
        p = p2;
        t = nt;
    }
}

// Two passes per launch over halves is not a shape; instead: one item per lane, but the
// workgroup order is reversed every other XCD slot (spreads concurrently open rows).
template <int BLOCK, bool DUAL>
__global__ __launch_bounds__(BLOCK) void k_avg_xcdslab(Args a)
{
    // each XCD (blockIdx % 8 under round-robin dispatch) sweeps its own contiguous eighth
    const int64_t span = (int64_t)BLOCK * 16;
    const uint32_t per = (gridDim.x + 7) / 8;
    const int64_t t = (int64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
    const int64_t off = t * span;
    auto rq = rsrc(a.peer, off, a.bytes, (int)span);
    auto rp = rsrc(a.param, off, a.bytes, (int)span);
    const f32x4 q = ld<NT>(rq, threadIdx.x * 16);
    const f32x4 p = ld<NT>(rp, threadIdx.x * 16);
    const f32x4 r = lerp4(0.5f, 0.5f, q, p);
    st<SC1>(rp, threadIdx.x * 16, r);
    if (DUAL) st<SC1>(rsrc(a.snap, off, a.bytes, (int)span), threadIdx.x * 16, r);
}

struct Variant {
    std::string name;
    double factor;       // bytes moved / operand bytes
    std::function<void(const Args &, hipStream_t, hipEvent_t, hipEvent_t)> run;
};

template <class K>
static void launch(K k, int grid, int block, const Args &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1)
{
    hipExtLaunchKernelGGL(k, dim3(grid), dim3(block), 0, s, e0, e1, 0, a);
}

static int grid_of(int64_t bytes, int64_t span) { return (int)((bytes + span - 1) / span); }

template <int B, int U, bool D, int AP = NT, int AS = SC1, int AN = AS>
static Variant avg(const char *name)
{
    return {name, D ? 4.0 : 3.0, [](const Args &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
                launch(k_avg<B, U, D, AP, AS, AN>, grid_of(a.bytes, (int64_t)B * 16 * U), B, a, s, e0, e1);
            }};
}

int main(int argc, char **argv)
{
    int64_t n = argc > 1 ? atoll(argv[1]) : 11173962;
    const int rounds = argc > 2 ? atoi(argv[2]) : 12;
    n = n / 4 * 4;
    const int64_t bytes = n * 4;
    const int sets = (int)std::max<int64_t>(3, (int64_t)(1.5e9 / (3.0 * bytes)) + 1);
    std::vector<Args> A(sets);
    for (int i = 0; i < sets; ++i) {
        float *p, *q, *sn;
        CHECK(hipMalloc(&p, bytes));
        CHECK(hipMalloc(&q, bytes));
        CHECK(hipMalloc(&sn, bytes));
        std::vector<float> h((size_t)n);
        uint32_t x = 777u + (uint32_t)i;
        for (auto &v : h) {
            x = x * 1664525u + 1013904223u;
            v = (float)((int32_t)(x >> 8) - (1 << 23)) / (float)(1 << 23);
        }
        CHECK(hipMemcpy(p, h.data(), bytes, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(q, h.data(), bytes, hipMemcpyHostToDevice));
        A[i] = Args{p, q, sn, nullptr, bytes};
    }
    float *sink;
    CHECK(hipMalloc(&sink, 4096));
    for (auto &a : A) a.sink = sink;
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<Variant> vs = {
        {"read-only  64x4 nt (1R)", 1.0, [](const Args &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
             launch(k_read<64, 4>, grid_of(a.bytes, 64 * 16 * 4), 64, a, s, e0, e1); }},
        {"read-only  64x1 nt (1R)", 1.0, [](const Args &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
             launch(k_read<64, 1>, grid_of(a.bytes, 64 * 16), 64, a, s, e0, e1); }},
        {"write-only 64 sc1 (1W)", 1.0, [](const Args &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
             launch(k_write<64>, grid_of(a.bytes, 64 * 16), 64, a, s, e0, e1); }},
        {"copy       64 (1R1W)", 2.0, [](const Args &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
             launch(k_copy<64>, grid_of(a.bytes, 64 * 16), 64, a, s, e0, e1); }},
        avg<64, 1, false>("avg  64x1 (product, 2R1W)"),
        avg<64, 2, false>("avg  64x2"),
        avg<64, 4, false>("avg  64x4"),
        avg<128, 1, false>("avg 128x1"),
        avg<256, 1, false>("avg 256x1"),
        avg<64, 1, false, NT, SC1 | NT>("avg  64x1 nt+sc1 store"),
        {"avg  pipe 64, 16 WG/CU", 3.0, [cus](const Args &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
             launch(k_pipe<64, false>, std::min(grid_of(a.bytes, 64 * 16), cus * 16), 64, a, s, e0, e1); }},
        {"avg  pipe 64, 32 WG/CU", 3.0, [cus](const Args &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
             launch(k_pipe<64, false>, std::min(grid_of(a.bytes, 64 * 16), cus * 32), 64, a, s, e0, e1); }},
        {"avg  xcd-slab 64", 3.0, [](const Args &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
             launch(k_avg_xcdslab<64, false>, (grid_of(a.bytes, 64 * 16) + 7) / 8 * 8, 64, a, s, e0, e1); }},
        {"oop  64x1 (resident, 2R1W')", 3.0, [](const Args &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
             launch(k_oop<64, 1>, grid_of(a.bytes, 64 * 16), 64, a, s, e0, e1); }},
        {"oop  64x2", 3.0, [](const Args &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
             launch(k_oop<64, 2>, grid_of(a.bytes, 64 * 16 * 2), 64, a, s, e0, e1); }},
        {"oop  64x4", 3.0, [](const Args &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
             launch(k_oop<64, 4>, grid_of(a.bytes, 64 * 16 * 4), 64, a, s, e0, e1); }},
        {"oop 128x1", 3.0, [](const Args &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
             launch(k_oop<128, 1>, grid_of(a.bytes, 128 * 16), 128, a, s, e0, e1); }},
        {"oop 256x1", 3.0, [](const Args &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
             launch(k_oop<256, 1>, grid_of(a.bytes, 256 * 16), 256, a, s, e0, e1); }},
        {"oop  64x1 nt+sc1 store", 3.0, [](const Args &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
             launch(k_oop<64, 1, SC1 | NT>, grid_of(a.bytes, 64 * 16), 64, a, s, e0, e1); }},
        // round 4: system-scope (sc0 sc1) stores, written through past the XCD L2, so the kernel's
        // end-of-launch L2 write-back finds nothing dirty
        {"oop  64x1 sc0+sc1 store", 3.0, [](const Args &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
             launch(k_oop<64, 1, SC1 | 1>, grid_of(a.bytes, 64 * 16), 64, a, s, e0, e1); }},
        {"oop  64x1 nt+sc0+sc1 store", 3.0, [](const Args &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
             launch(k_oop<64, 1, SC1 | 1 | NT>, grid_of(a.bytes, 64 * 16), 64, a, s, e0, e1); }},
        avg<64, 1, true>("dual 64x1 (product WT, 2R2W)"),
        avg<64, 2, true>("dual 64x2"),
        avg<64, 4, true>("dual 64x4"),
        avg<256, 1, true>("dual 256x1"),
        avg<64, 1, true, NT, SC1 | NT>("dual 64x1 nt+sc1 stores"),
        avg<64, 1, true, NT, SC1 | 1>("dual 64x1 sc0+sc1 stores"),
        avg<64, 1, true, NT, SC1 | NT, SC1>("dual 64x1 param nt+sc1, snap sc1 (policy 8)"),
        avg<64, 1, true, NT, SC1 | NT, SC1 | 1>("dual 64x1 param nt+sc1, snap sc0+sc1"),
        avg<64, 1, true, NT, SC1 | 1, SC1>("dual 64x1 param sc0+sc1, snap sc1"),
        avg<64, 1, false, NT, SC1 | 1>("avg  64x1 sc0+sc1 store (full)"),
        {"dual pipe 64, 16 WG/CU", 4.0, [cus](const Args &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
             launch(k_pipe<64, true>, std::min(grid_of(a.bytes, 64 * 16), cus * 16), 64, a, s, e0, e1); }},
        {"dual xcd-slab 64", 4.0, [](const Args &a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
             launch(k_avg_xcdslab<64, true>, (grid_of(a.bytes, 64 * 16) + 7) / 8 * 8, 64, a, s, e0, e1); }},
    };
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    const int reps = 6;
    std::vector<hipEvent_t> ev(2 * reps);
    for (auto &evt : ev) CHECK(hipEventCreate(&evt));
    std::vector<std::vector<double>> us(vs.size());
    int rot = 0;
    for (int r = 0; r < rounds + 1; ++r) {
        for (size_t v = 0; v < vs.size(); ++v) {
            for (int k = 0; k < reps; ++k) vs[v].run(A[rot++ % sets], s, ev[2 * k], ev[2 * k + 1]);
            CHECK(hipStreamSynchronize(s));
            if (r == 0) continue;
            for (int k = 0; k < reps; ++k) {
                float ms;
                CHECK(hipEventElapsedTime(&ms, ev[2 * k], ev[2 * k + 1]));
                us[v].push_back(1e3 * ms);
            }
        }
    }
    printf("numel %lld (%.1f MB per operand), %d rotating sets, %d rounds x %d launches, %d CUs\n", (long long)n,
           bytes / 1e6, sets, rounds, reps, cus);
    for (size_t v = 0; v < vs.size(); ++v) {
        auto x = us[v];
        std::sort(x.begin(), x.end());
        double mean = 0;
        for (double y : x) mean += y;
        mean /= x.size();
        const double gb = vs[v].factor * bytes;
        printf("%-32s mean %9.2f us  %7.1f GB/s (%5.1f%%)  median %9.2f  best %7.1f GB/s\n", vs[v].name.c_str(), mean,
               gb / mean / 1e3, 100.0 * gb / mean / 1e3 / 8000.0, x[x.size() / 2], gb / x[0] / 1e3);
    }
    return 0;
}
