// product_tune.hip -- the product averaging kernels (through libdpwa_hip.so's stateless C ABI)
// beside stand-alone streaming kernels of the same access mix, in ONE harness (not part of the
// product).  Separates what the product kernel costs beyond the bare stream (the fused fp64 factor's
// scalar loads, a large kernel-argument block) from what a measurement harness costs (allocator,
// buffer placement).  Every launch is timed by its own dispatch begin/end events, buffers rotate
// over > 1.5 GB, variants interleave round by round.
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -Iinclude -o tools/product_tune
//        tools/product_tune.hip -Ldpwa_amd -ldpwa_hip -Wl,-rpath,'$ORIGIN/../dpwa_amd'
// Run:   DPWA_LERP_POLICY=<p> tools/product_tune [numel] [rounds]
//        (TUNE_DUAL=1: the write-through rows only; TUNE_ONLY="name;name;...": those rows, in that order)
#pragma clang fp contract(off)
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "dpwa_hip.h"

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
constexpr int NT = 2, SC1 = 16, SC0 = 1;
constexpr int64_t kOff = DPWA_SLOT_PAYLOAD_OFFSET;

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

struct Set {
    float *param;        // n
    char *slot;          // [header | pad | n]  (the peer snapshot)
    char *snap;          // [header | pad | n]  (the destination slot)
    double *clock;       // [2]
    dpwa_coef *coef;
    float *other;        // n: a fourth buffer (the bare mix's distinct first destination)
};

struct Args {
    const float *param;
    const float *peer;
    float *snap;
    int64_t bytes;
    const double *clock;
    const double *hdr;   // the peer slot's header (clock, loss)
};

// the bare write-through stream: 2 reads, 2 writes -- the parameters in place (as the product
// stores them, `nt sc1`) and the next snapshot (`sc1`); DISTINCT: the first store goes to a fourth
// buffer instead (dpwa_stream_mix's shape); FACTOR: + the clock/header scalar loads
template <bool DISTINCT, bool FACTOR>
__global__ __launch_bounds__(64) void k_dual(Args a, float *other)
{
    const int64_t off = (int64_t)blockIdx.x * 1024;
    const __amdgpu_buffer_rsrc_t rp = rsrc(a.param, off, a.bytes, 1024);
    const f32x4 q = ld<NT>(rsrc(a.peer, off, a.bytes, 1024), threadIdx.x * 16);
    const f32x4 p = ld<NT>(rp, threadIdx.x * 16);
    float fa = 0.5f, fb = 0.5f;
    if (FACTOR) {
        const double c = *a.clock, pc = a.hdr[0];
        const double f = (c + pc) > -1.0 ? 0.5 : 0.25;
        fa = (float)f;
        fb = (float)(1.0 - f);
    }
    const f32x4 r = fa * q + fb * p;
    st<NT | SC1>(DISTINCT ? rsrc(other, off, a.bytes, 1024) : rp, threadIdx.x * 16, r);
    st<SC1>(rsrc(a.snap, off, a.bytes, 1024), threadIdx.x * 16, r);
}

// The same write-through stream with its two reads by LDS-DMA (`global_load_lds_dwordx4`, no VGPR
// destination; aux AUXL: 2 = nt): each wave DMAs its 1-KiB span of the peer snapshot and of the
// parameters into its own LDS, waits for them (vmcnt(0)), reads them back with ds_read_b128, and
// stores as k_dual.  WAVES one-wave spans per workgroup.  (the one load path
// the averaging kernel had not tried.)  A span that does not fit whole takes the buffer loads.
typedef __attribute__((address_space(3))) void *lds_ptr_t;
typedef __attribute__((address_space(1))) void *gbl_ptr_t;

template <int AUXL, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_dual_glds(Args a)
{
    __shared__ f32x4 lds[WAVES][2][64];
    const int w = WAVES == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform
    const int lane = threadIdx.x & 63;
    const int64_t off = ((int64_t)blockIdx.x * WAVES + w) * 1024;
    if (off >= a.bytes) return;
    f32x4 q, p;
    if (off + 1024 <= a.bytes) {
        __builtin_amdgcn_global_load_lds((gbl_ptr_t)((const char *)a.peer + off + lane * 16), (lds_ptr_t)&lds[w][0][0],
                                         16, 0, AUXL);
        __builtin_amdgcn_global_load_lds((gbl_ptr_t)((const char *)a.param + off + lane * 16),
                                         (lds_ptr_t)&lds[w][1][0], 16, 0, AUXL);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        q = lds[w][0][lane];
        p = lds[w][1][lane];
    } else {
        q = ld<NT>(rsrc(a.peer, off, a.bytes, 1024), lane * 16);
        p = ld<NT>(rsrc(a.param, off, a.bytes, 1024), lane * 16);
    }
    const f32x4 r = 0.5f * q + 0.5f * p;
    st<NT | SC1>(rsrc(a.param, off, a.bytes, 1024), lane * 16, r);
    st<SC1>(rsrc(a.snap, off, a.bytes, 1024), lane * 16, r);
}

// Control for k_dual_glds: the same multi-wave workgroups with the product's buffer loads into VGPRs.
template <int WAVES>
__global__ __launch_bounds__(64 * WAVES) void k_dual_wg(Args a)
{
    const int w = WAVES == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t off = ((int64_t)blockIdx.x * WAVES + w) * 1024;
    if (off >= a.bytes) return;
    const __amdgpu_buffer_rsrc_t rp = rsrc(a.param, off, a.bytes, 1024);
    const f32x4 q = ld<NT>(rsrc(a.peer, off, a.bytes, 1024), lane * 16);
    const f32x4 p = ld<NT>(rp, lane * 16);
    const f32x4 r = 0.5f * q + 0.5f * p;
    st<NT | SC1>(rp, lane * 16, r);
    st<SC1>(rsrc(a.snap, off, a.bytes, 1024), lane * 16, r);
}

struct BigArgs {         // the same plus padding to the product's kernel-argument size
    Args a;
    char pad[192];
};

// the bare resident stream: 2 reads, 1 write to a third buffer
template <int AUXS>
__global__ __launch_bounds__(64) void k_oop(Args a)
{
    const int64_t off = (int64_t)blockIdx.x * 1024;
    const f32x4 q = ld<NT>(rsrc(a.peer, off, a.bytes, 1024), threadIdx.x * 16);
    const f32x4 p = ld<NT>(rsrc(a.param, off, a.bytes, 1024), threadIdx.x * 16);
    st<AUXS>(rsrc(a.snap, off, a.bytes, 1024), threadIdx.x * 16, 0.5f * q + 0.5f * p);
}

// + every wave reads the clock and the peer header (scalar loads) and derives (a, b) from them
template <int AUXS>
__global__ __launch_bounds__(64) void k_oop_factor(Args a)
{
    const int64_t off = (int64_t)blockIdx.x * 1024;
    const f32x4 q = ld<NT>(rsrc(a.peer, off, a.bytes, 1024), threadIdx.x * 16);
    const f32x4 p = ld<NT>(rsrc(a.param, off, a.bytes, 1024), threadIdx.x * 16);
    const double c = *a.clock, pc = a.hdr[0];
    const double f = (c + pc) > -1.0 ? 0.5 : 0.25;     // uniform, depends on the loads
    const float fa = (float)f, fb = (float)(1.0 - f);
    st<AUXS>(rsrc(a.snap, off, a.bytes, 1024), threadIdx.x * 16, fa * q + fb * p);
}

// + a 232-byte kernel-argument block
template <int AUXS>
__global__ __launch_bounds__(64) void k_oop_bigarg(BigArgs b)
{
    const Args &a = b.a;
    const int64_t off = (int64_t)blockIdx.x * 1024;
    const f32x4 q = ld<NT>(rsrc(a.peer, off, a.bytes, 1024), threadIdx.x * 16);
    const f32x4 p = ld<NT>(rsrc(a.param, off, a.bytes, 1024), threadIdx.x * 16);
    st<AUXS>(rsrc(a.snap, off, a.bytes, 1024), threadIdx.x * 16, 0.5f * q + 0.5f * p);
}

struct Variant {
    std::string name;
    double factor;
    std::function<void(const Set &, hipStream_t, hipEvent_t, hipEvent_t)> run;
};

int main(int argc, char **argv)
{
    int64_t n = argc > 1 ? atoll(argv[1]) : 11173962;
    const int rounds = argc > 2 ? atoi(argv[2]) : 12;
    n = n / 4 * 4;
    const int64_t bytes = n * 4;
    const int sets = (int)std::max<int64_t>(3, (int64_t)(1.5e9 / (3.0 * bytes)) + 1);
    const bool dual_only = getenv("TUNE_DUAL") != nullptr;
    std::vector<Set> S(sets);
    for (int i = 0; i < sets; ++i) {
        Set &s = S[i];
        CHECK(hipMalloc(&s.param, bytes));
        CHECK(hipMalloc(&s.slot, kOff + bytes));
        CHECK(hipMalloc(&s.snap, kOff + bytes));
        CHECK(hipMalloc(&s.clock, 2 * sizeof(double)));
        CHECK(hipMalloc(&s.coef, sizeof(dpwa_coef)));
        CHECK(hipMalloc(&s.other, bytes));
        CHECK(hipMemset(s.slot, 0, kOff));
        CHECK(hipMemset(s.snap, 0, kOff));
        CHECK(hipMemset(s.clock, 0, 2 * sizeof(double)));
        std::vector<float> h((size_t)n);
        uint32_t x = 777u + (uint32_t)i;
        for (auto &v : h) {
            x = x * 1664525u + 1013904223u;
            v = (float)((int32_t)(x >> 8) - (1 << 23)) / (float)(1 << 23);
        }
        CHECK(hipMemcpy(s.param, h.data(), bytes, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(s.slot + kOff, h.data(), bytes, hipMemcpyHostToDevice));
    }
    static dpwa_interp cfg{DPWA_INTERP_CONSTANT, 0, 0.5, 0.0};
    const int grid = (int)((bytes + 1023) / 1024);
    auto args_of = [bytes](const Set &s) {
        return Args{s.param, (const float *)(s.slot + kOff), (float *)(s.snap + kOff), bytes, s.clock,
                    (const double *)s.slot};
    };
    std::vector<Variant> vs = {
        {"product resident (dpwa_average_many_resident x1)", 3.0,
         [n](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             dpwa_average_desc d{s.param, s.slot, n, s.clock, 1.0, s.coef, s.snap + kOff};
             if (dpwa_average_many_resident(DPWA_F32, &d, 1, &cfg, st, e0, e1)) { fprintf(stderr, "%s\n", dpwa_last_error()); exit(1); }
         }},
        {"product write-through single (dpwa_average)", 4.0,
         [n](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             if (dpwa_average(DPWA_F32, s.param, s.slot, n, &cfg, s.clock, 1.0, s.coef, s.snap + kOff, st, e0, e1)) {
                 fprintf(stderr, "%s\n", dpwa_last_error());
                 exit(1);
             }
         }},
        {"bare dual in place", 4.0, [&](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             hipExtLaunchKernelGGL((k_dual<false, false>), dim3(grid), dim3(64), 0, st, e0, e1, 0, args_of(s), s.other); }},
        {"bare dual distinct (4 buffers)", 4.0, [&](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             hipExtLaunchKernelGGL((k_dual<true, false>), dim3(grid), dim3(64), 0, st, e0, e1, 0, args_of(s), s.other); }},
        {"bare dual in place + factor loads", 4.0, [&](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             hipExtLaunchKernelGGL((k_dual<false, true>), dim3(grid), dim3(64), 0, st, e0, e1, 0, args_of(s), s.other); }},
        {"dpwa_stream_mix 2R:2W (4 buffers)", 4.0, [bytes](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             void *dst[2] = {s.other, s.snap + kOff};
             const void *src[2] = {s.slot + kOff, s.param};
             if (dpwa_stream_mix(dst, 2, src, 2, bytes, st, e0, e1)) { fprintf(stderr, "%s\n", dpwa_last_error()); exit(1); }
         }},
        {"dpwa_stream_mix 2R:2W in place", 4.0, [bytes](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             void *dst[2] = {s.param, s.snap + kOff};
             const void *src[2] = {s.slot + kOff, s.param};
             if (dpwa_stream_mix(dst, 2, src, 2, bytes, st, e0, e1)) { fprintf(stderr, "%s\n", dpwa_last_error()); exit(1); }
         }},
        {"glds dual in place (nt, 1 wave/WG)", 4.0, [&](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             hipExtLaunchKernelGGL((k_dual_glds<NT, 1>), dim3(grid), dim3(64), 0, st, e0, e1, 0, args_of(s)); }},
        {"glds dual in place (default policy, 1 wave/WG)", 4.0, [&](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             hipExtLaunchKernelGGL((k_dual_glds<0, 1>), dim3(grid), dim3(64), 0, st, e0, e1, 0, args_of(s)); }},
        {"glds dual in place (nt, 2 waves/WG)", 4.0, [&](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             hipExtLaunchKernelGGL((k_dual_glds<NT, 2>), dim3((grid + 1) / 2), dim3(128), 0, st, e0, e1, 0, args_of(s)); }},
        {"glds dual in place (nt, 4 waves/WG)", 4.0, [&](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             hipExtLaunchKernelGGL((k_dual_glds<NT, 4>), dim3((grid + 3) / 4), dim3(256), 0, st, e0, e1, 0, args_of(s)); }},
        {"glds dual in place (nt, 8 waves/WG)", 4.0, [&](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             hipExtLaunchKernelGGL((k_dual_glds<NT, 8>), dim3((grid + 7) / 8), dim3(512), 0, st, e0, e1, 0, args_of(s)); }},
        {"vgpr dual in place (nt, 4 waves/WG)", 4.0, [&](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             hipExtLaunchKernelGGL((k_dual_wg<4>), dim3((grid + 3) / 4), dim3(256), 0, st, e0, e1, 0, args_of(s)); }},
        {"vgpr dual in place (nt, 2 waves/WG)", 4.0, [&](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             hipExtLaunchKernelGGL((k_dual_wg<2>), dim3((grid + 1) / 2), dim3(128), 0, st, e0, e1, 0, args_of(s)); }},
        {"bare oop sc1", 3.0, [&](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             hipExtLaunchKernelGGL(k_oop<SC1>, dim3(grid), dim3(64), 0, st, e0, e1, 0, args_of(s)); }},
        {"bare oop sc0+sc1", 3.0, [&](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             hipExtLaunchKernelGGL(k_oop<SC1 | SC0>, dim3(grid), dim3(64), 0, st, e0, e1, 0, args_of(s)); }},
        {"oop+factor loads sc1", 3.0, [&](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             hipExtLaunchKernelGGL(k_oop_factor<SC1>, dim3(grid), dim3(64), 0, st, e0, e1, 0, args_of(s)); }},
        {"oop+factor loads sc0+sc1", 3.0, [&](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             hipExtLaunchKernelGGL(k_oop_factor<SC1 | SC0>, dim3(grid), dim3(64), 0, st, e0, e1, 0, args_of(s)); }},
        {"oop+232B kernargs sc1", 3.0, [&](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             BigArgs b{};
             b.a = args_of(s);
             hipExtLaunchKernelGGL(k_oop_bigarg<SC1>, dim3(grid), dim3(64), 0, st, e0, e1, 0, b); }},
        {"oop+232B kernargs sc0+sc1", 3.0, [&](const Set &s, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
             BigArgs b{};
             b.a = args_of(s);
             hipExtLaunchKernelGGL(k_oop_bigarg<SC1 | SC0>, dim3(grid), dim3(64), 0, st, e0, e1, 0, b); }},
    };
    if (dual_only) {   // TUNE_DUAL: the write-through rows only
        std::vector<Variant> keep;
        for (auto &v : vs)
            if (v.factor == 4.0) keep.push_back(v);
        vs.swap(keep);
    }
    if (const char *only = getenv("TUNE_ONLY")) {   // ';'-separated name substrings, run in that order
        std::vector<Variant> keep;
        std::string list(only);
        size_t pos = 0;
        while (pos <= list.size()) {
            const size_t end = std::min(list.find(';', pos), list.size());
            const std::string key = list.substr(pos, end - pos);
            for (auto &v : vs)
                if (!key.empty() && v.name.find(key) != std::string::npos) {
                    keep.push_back(v);
                    break;
                }
            pos = end + 1;
        }
        vs.swap(keep);
    }
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    const int reps = 6;
    std::vector<hipEvent_t> ev(2 * reps);
    for (auto &evt : ev) CHECK(hipEventCreate(&evt));
    std::vector<std::vector<double>> us(vs.size());
    int rot = 0;
    for (int r = 0; r < rounds + 1; ++r) {
        for (size_t v = 0; v < vs.size(); ++v) {
            for (int k = 0; k < reps; ++k) vs[v].run(S[rot++ % sets], st, ev[2 * k], ev[2 * k + 1]);
            CHECK(hipStreamSynchronize(st));
            if (r == 0) continue;
            for (int k = 0; k < reps; ++k) {
                float ms;
                CHECK(hipEventElapsedTime(&ms, ev[2 * k], ev[2 * k + 1]));
                us[v].push_back(1e3 * ms);
            }
        }
    }
    const char *pol = getenv("DPWA_LERP_POLICY");
    printf("numel %lld (%.1f MB per operand), %d rotating sets, %d rounds x %d launches, DPWA_LERP_POLICY=%s\n",
           (long long)n, bytes / 1e6, sets, rounds, reps, pol ? pol : "(product)");
    for (size_t v = 0; v < vs.size(); ++v) {
        auto x = us[v];
        std::sort(x.begin(), x.end());
        double mean = 0;
        for (double y : x) mean += y;
        mean /= x.size();
        const double gb = vs[v].factor * bytes;
        printf("%-50s mean %8.2f us  %7.1f GB/s (%5.1f%%)  median %8.2f\n", vs[v].name.c_str(), mean, gb / mean / 1e3,
               100.0 * gb / mean / 1e3 / 8000.0, x[x.size() / 2]);
    }
    return 0;
}
