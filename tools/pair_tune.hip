// pair_tune.hip -- two co-resident resident learners that average with each other (the N=1 bench
// loop: A reads B's published slot, B reads A's) in one dispatch, by block-to-span mapping and load
// policy (not part of the product).  Both averages of a round read the same two snapshots; with
// the product mapping (entry = block % 2) the two reads of a span run on different XCDs, so the
// second one cannot hit the first one's L2.  Variants:
//   rr-nt      product: entry = b % 2, span = b / 2, loads nt
//   rr-def     the same with default-policy loads
//   xcd-nt     entry = (b / 8) % 2, span = (b / 16) * 8 + b % 8: blocks b and b + 8 (same XCD under
//              round-robin dispatch) take the two entries of one span; loads nt
//   xcd-def    the same with default-policy loads (the first read allocates in L2)
//   fused      one workgroup per span computes both averages (2 loads, 2 stores): the floor
// "loop" mode alternates the direction over four slots as the bench loop does (round r reads
// A, B and writes A', B'; round r + 1 the reverse); "cold" mode rotates over > 1.5 GB of sets.
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -o tools/pair_tune tools/pair_tune.hip
// Run:   tools/pair_tune [numel] [rounds]
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
        hipError_t err_ = (x);                                                                \
        if (err_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(err_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int NT = 2, SC1 = 16, DEF = 0;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, int64_t off, int64_t total)
{
    const int64_t rem = total - off;
    const int num = rem <= 0 ? 0 : (rem < 1024 ? (int)rem : 1024);
    return __builtin_amdgcn_make_buffer_rsrc((void *)((const char *)p + off), 0, num, 0x00020000);
}
template <int AUX>
__device__ __forceinline__ f32x4 ld(__amdgpu_buffer_rsrc_t r, int off)
{
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX));
}
__device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, int off, f32x4 v)
{
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, SC1);
}

struct Pair {
    const float *a, *b;   // the two published slots (A's parameters, B's parameters)
    float *a2, *b2;       // their next slots
    int64_t bytes;
    int64_t spans;
};

// MAP 0: entry = b % 2; MAP 1: XCD-paired.  AUX: both loads; AUXP/AUXQ: own / peer load
template <int MAP, int AUX, int AUXP = AUX, int AUXQ = AUX>
__global__ __launch_bounds__(64) void k_pair(Pair p)
{
    uint32_t e, s;
    if (MAP == 0) {
        e = blockIdx.x & 1u;
        s = blockIdx.x >> 1;
    } else {
        e = (blockIdx.x >> 3) & 1u;
        s = (blockIdx.x >> 4) * 8u + (blockIdx.x & 7u);
    }
    if (s >= p.spans) return;
    const int64_t off = (int64_t)s * 1024;
    const float *mine = e ? p.b : p.a;
    const float *peer = e ? p.a : p.b;
    float *out = e ? p.b2 : p.a2;
    const f32x4 q = ld<AUXQ>(rsrc(peer, off, p.bytes), threadIdx.x * 16);
    const f32x4 x = ld<AUXP>(rsrc(mine, off, p.bytes), threadIdx.x * 16);
    st(rsrc(out, off, p.bytes), threadIdx.x * 16, 0.5f * q + 0.5f * x);
}

__global__ __launch_bounds__(64) void k_pair_fused(Pair p)
{
    const int64_t off = (int64_t)blockIdx.x * 1024;
    const f32x4 x = ld<NT>(rsrc(p.a, off, p.bytes), threadIdx.x * 16);
    const f32x4 y = ld<NT>(rsrc(p.b, off, p.bytes), threadIdx.x * 16);
    st(rsrc(p.a2, off, p.bytes), threadIdx.x * 16, 0.5f * y + 0.5f * x);
    st(rsrc(p.b2, off, p.bytes), threadIdx.x * 16, 0.25f * x + 0.75f * y);
}

struct Variant {
    const char *name;
    int kind;    // 0..3 k_pair<MAP, AUX>, 4 fused
};

static void launch(int kind, const Pair &p, hipStream_t s, hipEvent_t e0, hipEvent_t e1)
{
    const int spans = (int)p.spans;
    const int g2 = ((spans + 7) / 8) * 16;   // XCD map covers whole groups of 8 spans
    switch (kind) {
    case 0: hipExtLaunchKernelGGL((k_pair<0, NT>), dim3(2 * spans), dim3(64), 0, s, e0, e1, 0, p); break;
    case 1: hipExtLaunchKernelGGL((k_pair<0, DEF>), dim3(2 * spans), dim3(64), 0, s, e0, e1, 0, p); break;
    case 2: hipExtLaunchKernelGGL((k_pair<1, NT>), dim3(g2), dim3(64), 0, s, e0, e1, 0, p); break;
    case 3: hipExtLaunchKernelGGL((k_pair<1, DEF>), dim3(g2), dim3(64), 0, s, e0, e1, 0, p); break;
    case 5: hipExtLaunchKernelGGL((k_pair<1, NT, DEF, NT>), dim3(g2), dim3(64), 0, s, e0, e1, 0, p); break;
    case 6: hipExtLaunchKernelGGL((k_pair<1, NT, NT, DEF>), dim3(g2), dim3(64), 0, s, e0, e1, 0, p); break;
    default: hipExtLaunchKernelGGL(k_pair_fused, dim3(spans), dim3(64), 0, s, e0, e1, 0, p); break;
    }
}

int main(int argc, char **argv)
{
    int64_t n = argc > 1 ? atoll(argv[1]) : 11173962;
    const int rounds = argc > 2 ? atoi(argv[2]) : 12;
    n = n / 4 * 4;
    const int64_t bytes = n * 4;
    const int64_t spans = (bytes + 1023) / 1024;
    // cold sets: 4 slots each, > 1.5 GB in all
    const int sets = (int)std::max<int64_t>(3, (int64_t)(1.5e9 / (4.0 * bytes)) + 1);
    std::vector<float *> slots(4 * sets);
    std::vector<float> h((size_t)n);
    uint32_t x = 12345u;
    for (auto &v : h) {
        x = x * 1664525u + 1013904223u;
        v = (float)((int32_t)(x >> 8) - (1 << 23)) / (float)(1 << 23);
    }
    for (auto &p : slots) {
        CHECK(hipMalloc(&p, bytes));
        CHECK(hipMemcpy(p, h.data(), bytes, hipMemcpyHostToDevice));
    }
    const Variant vs[] = {{"rr-nt (product map)", 0}, {"rr-def", 1}, {"xcd-nt", 2}, {"xcd-def", 3},
                          {"xcd own-def peer-nt", 5}, {"xcd own-nt peer-def", 6}, {"fused (1 WG, 2R 2W)", 4}};
    const int nv = 7;
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    const int reps = 8;
    std::vector<hipEvent_t> ev(2 * reps);
    for (auto &evt : ev) CHECK(hipEventCreate(&evt));
    for (int mode = 0; mode < 2; ++mode) {   // 0 cold (rotating sets), 1 loop (one set, alternating)
        std::vector<std::vector<double>> us(nv);
        int rot = 0;
        for (int r = 0; r < rounds + 1; ++r) {
            for (int v = 0; v < nv; ++v) {
                for (int k = 0; k < reps; ++k) {
                    const int set = mode == 0 ? (rot++ % sets) : 0;
                    float **q = &slots[4 * set];
                    const bool flip = mode == 1 && (k & 1);
                    Pair p{flip ? q[2] : q[0], flip ? q[3] : q[1], flip ? q[0] : q[2], flip ? q[1] : q[3], bytes, spans};
                    launch(vs[v].kind, p, s, ev[2 * k], ev[2 * k + 1]);
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
        printf("%s: numel %lld (%.1f MB per slot), %d rounds x %d launches%s\n", mode ? "LOOP" : "COLD", (long long)n,
               bytes / 1e6, rounds, reps, mode ? "" : " over rotating sets");
        for (int v = 0; v < nv; ++v) {
            auto t = us[v];
            std::sort(t.begin(), t.end());
            double mean = 0;
            for (double y : t) mean += y;
            mean /= t.size();
            // two averagings: 6*N*s algorithmic (each reads two slots, writes one); 4*N*s distinct
            printf("  %-22s mean %8.2f us  median %8.2f  2x3Ns %7.1f GB/s  distinct 4Ns %7.1f GB/s (%5.1f%% of 8 TB/s)\n",
                   vs[v].name, mean, t[t.size() / 2], 6.0 * bytes / mean / 1e3, 4.0 * bytes / mean / 1e3,
                   100.0 * 4.0 * bytes / mean / 1e3 / 8000.0);
        }
    }
    return 0;
}
