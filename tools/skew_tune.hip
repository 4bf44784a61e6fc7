// skew_tune.hip -- does the relative placement of the averaging kernel's operands matter?
// (tuning experiment, not part of the product)
//
// The product's operands are the torch-owned parameter buffer, the peer snapshot and (write-
// through) the next snapshot slot, each at whatever address its allocator chose.  If the
// DRAM channel/bank of an address depended only on its low bits, operands that start at the
// same offset modulo the interleave would send every workgroup's 2-4 accesses to one bank in
// different rows.  This tool places the three operands of every rotating set inside one arena
// at chosen relative skews and times the product's shapes (2R1W average, 2R2W write-through
// average, one 16-B item per lane, 64-lane workgroups, nt loads, sc1 stores) per launch with
// dispatch events, cold (> 1.5 GB rotation), variants interleaved round by round.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/skew_tune tools/skew_tune.hip
// Run:   tools/skew_tune [numel] [rounds]
#pragma clang fp contract(off)
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

struct Args {
    float *param;
    const float *peer;
    float *snap;
    int64_t bytes;
};

// SNAP_FIRST: the write-through kernel stores the snapshot before the parameters.
template <bool DUAL, bool SNAP_FIRST = false>
__global__ __launch_bounds__(64) void k_avg(Args a)
{
    constexpr int span = 64 * 16;
    const int64_t off = (int64_t)blockIdx.x * span;
    auto rq = rsrc(a.peer, off, a.bytes, span);
    auto rp = rsrc(a.param, off, a.bytes, span);
    const f32x4 q = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rq, threadIdx.x * 16, 0, NT));
    const f32x4 p = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rp, threadIdx.x * 16, 0, NT));
    const f32x4 r = 0.5f * q + 0.5f * p;
    const u32x4 w = __builtin_bit_cast(u32x4, r);
    if (DUAL && SNAP_FIRST)
        __builtin_amdgcn_raw_buffer_store_b128(w, rsrc(a.snap, off, a.bytes, span), threadIdx.x * 16, 0, SC1);
    __builtin_amdgcn_raw_buffer_store_b128(w, rp, threadIdx.x * 16, 0, SC1);
    if (DUAL && !SNAP_FIRST)
        __builtin_amdgcn_raw_buffer_store_b128(w, rsrc(a.snap, off, a.bytes, span), threadIdx.x * 16, 0, SC1);
}

struct Layout {
    std::string name;
    int64_t skew_q, skew_s;   // peer and snapshot offsets relative to the parameters, beyond `bytes`
};

int main(int argc, char **argv)
{
    int64_t n = argc > 1 ? atoll(argv[1]) : 11173962;
    const int rounds = argc > 2 ? atoi(argv[2]) : 10;
    n = n / 4 * 4;
    const int64_t bytes = n * 4;
    const int64_t MB2 = 2 << 20;
    const int64_t stride = (bytes + 4 * MB2 + MB2 - 1) / MB2 * MB2;   // per operand, room for the skews
    const int sets = (int)std::max<int64_t>(3, (int64_t)(1.5e9 / (3.0 * bytes)) + 1);
    char *arena;
    CHECK(hipMalloc(&arena, (size_t)(3 * stride * sets + MB2)));
    std::vector<float> h((size_t)n);
    uint32_t x = 777u;
    for (auto &v : h) {
        x = x * 1664525u + 1013904223u;
        v = (float)((int32_t)(x >> 8) - (1 << 23)) / (float)(1 << 23);
    }
    const std::vector<Layout> layouts = {
        {"aligned (same offset mod 2 MiB)", 0, 0},
        {"peer +256 B, snap +256 B (slot header)", 256, 256},
        {"peer +4 KiB, snap +8 KiB", 4096, 8192},
        {"peer +64 KiB, snap +128 KiB", 65536, 131072},
        {"peer +1 MiB, snap +2 MiB+4 KiB", 1 << 20, (2 << 20) + 4096},
        {"peer +3 MiB+12 KiB, snap +1.5 MiB", (3 << 20) + 12288, 3 << 19},
    };
    // every layout gets its own pointer sets (same arena, same rotation order)
    auto args_of = [&](const Layout &l, int i) {
        char *base = arena + (int64_t)i * 3 * stride;
        return Args{(float *)base, (const float *)(base + stride + l.skew_q), (float *)(base + 2 * stride + l.skew_s),
                    bytes};
    };
    for (int i = 0; i < sets; ++i)
        for (const auto &l : layouts) {
            Args a = args_of(l, i);
            CHECK(hipMemcpy(a.param, h.data(), bytes, hipMemcpyHostToDevice));
            CHECK(hipMemcpy((void *)a.peer, h.data(), bytes, hipMemcpyHostToDevice));
        }
    const int grid = (int)((bytes + 1023) / 1024);
    struct V {
        std::string name;
        int layout;
        int kind;   // 0 avg, 1 dual, 2 dual snapshot-first
    };
    std::vector<V> vs;
    for (int k = 0; k < 3; ++k)
        for (int l = 0; l < (int)layouts.size(); ++l)
            vs.push_back({std::string(k == 0 ? "avg 2R1W  " : k == 1 ? "dual 2R2W " : "dual snap1st ") + layouts[l].name,
                          l, k});
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    const int reps = 6;
    std::vector<hipEvent_t> ev(2 * reps);
    for (auto &evt : ev) CHECK(hipEventCreate(&evt));
    std::vector<std::vector<double>> us(vs.size());
    int rot = 0;
    for (int r = 0; r < rounds + 1; ++r) {
        for (size_t v = 0; v < vs.size(); ++v) {
            for (int k = 0; k < reps; ++k) {
                const Args a = args_of(layouts[vs[v].layout], rot++ % sets);
                if (vs[v].kind == 0)
                    hipExtLaunchKernelGGL(k_avg<false>, dim3(grid), dim3(64), 0, s, ev[2 * k], ev[2 * k + 1], 0, a);
                else if (vs[v].kind == 1)
                    hipExtLaunchKernelGGL(k_avg<true>, dim3(grid), dim3(64), 0, s, ev[2 * k], ev[2 * k + 1], 0, a);
                else
                    hipExtLaunchKernelGGL((k_avg<true, true>), dim3(grid), dim3(64), 0, s, ev[2 * k], ev[2 * k + 1], 0,
                                          a);
            }
            CHECK(hipStreamSynchronize(s));
            if (r == 0) continue;
            for (int k = 0; k < reps; ++k) {
                float ms;
                CHECK(hipEventElapsedTime(&ms, ev[2 * k], ev[2 * k + 1]));
                us[v].push_back(1e3 * ms);
            }
        }
    }
    printf("numel %lld (%.1f MB per operand), %d rotating sets, %d rounds x %d launches\n", (long long)n, bytes / 1e6,
           sets, rounds, reps);
    for (size_t v = 0; v < vs.size(); ++v) {
        auto y = us[v];
        std::sort(y.begin(), y.end());
        double mean = 0;
        for (double t : y) mean += t;
        mean /= y.size();
        const double gb = (vs[v].kind == 0 ? 3.0 : 4.0) * bytes;
        printf("%-56s mean %8.2f us %7.1f GB/s (%5.1f%%)  median %8.2f  best %7.1f GB/s\n", vs[v].name.c_str(), mean,
               gb / mean / 1e3, 100.0 * gb / mean / 1e3 / 8000.0, y[y.size() / 2], gb / y[0] / 1e3);
    }
    return 0;
}
