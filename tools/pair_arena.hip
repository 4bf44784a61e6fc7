// pair_arena.hip -- the resident mutual-pair dispatch (dpwa_average_many_resident, XCD-grouped)
// by how the two learners' four slots were allocated, on a heap churned first the way a bench
// process churns it (not part of the product):
//   malloc   one hipMalloc per learner ([slot|slot], learner.cpp's layout)
//   contig   the same from hipExtMallocWithFlags(hipDeviceMallocContiguous)
//   arena    ONE contiguous allocation holding both learners' four slots
// REPS pairs of each kind are allocated (interleaved kinds), each timed twice in the gossip loop.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -o tools/pair_arena tools/pair_arena.hip
//        -Ldpwa_amd -ldpwa_hip -Wl,-rpath,'$ORIGIN/../dpwa_amd'
// Run:   tools/pair_arena [numel] [reps] [rounds] [churn 0|1]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "dpwa_hip.h"

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t err_ = (x);                                                                \
        if (err_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(err_)); \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

constexpr size_t kOff = DPWA_SLOT_PAYLOAD_OFFSET;

struct Pair {
    int kind;
    char *slot[2][2];
    std::vector<void *> allocs;
    std::vector<double> us;
};

int main(int argc, char **argv)
{
    const int64_t n = argc > 1 ? atoll(argv[1]) : 11173962;
    const int reps = argc > 2 ? atoi(argv[2]) : 4;
    const int rounds = argc > 3 ? atoi(argv[3]) : 400;
    const int churn = argc > 4 ? atoi(argv[4]) : 1;
    const size_t payload = (size_t)n * 4;
    const size_t stride = (kOff + payload + 4095) / 4096 * 4096;
    const char *kinds[3] = {"malloc", "contig", "arena"};
    std::vector<void *> keep;
    if (churn) {   // mixed sizes, half freed, as learners, staging buffers and torch blocks come and go
        uint32_t x = 7u;
        std::vector<void *> tmp;
        for (int i = 0; i < 60; ++i) {
            x = x * 1664525u + 1013904223u;
            const size_t mb = 2 + (x >> 8) % 190;
            void *p;
            CHECK(hipMalloc(&p, mb << 20));
            tmp.push_back(p);
        }
        for (size_t i = 0; i < tmp.size(); ++i)
            if (i % 2) CHECK(hipFree(tmp[i]));
            else keep.push_back(tmp[i]);
    }
    std::vector<float> h((size_t)n, 0.5f);
    std::vector<Pair> pairs;
    for (int r = 0; r < reps; ++r)
        for (int k = 0; k < 3; ++k) {
            Pair P;
            P.kind = k;
            if (k == 2) {
                void *p;
                CHECK(hipExtMallocWithFlags(&p, 4 * stride, hipDeviceMallocContiguous));
                P.allocs.push_back(p);
                for (int a = 0; a < 2; ++a)
                    for (int s = 0; s < 2; ++s) P.slot[a][s] = (char *)p + (2 * a + s) * stride;
            } else {
                for (int a = 0; a < 2; ++a) {
                    void *p;
                    if (k == 1) CHECK(hipExtMallocWithFlags(&p, 2 * stride, hipDeviceMallocContiguous));
                    else CHECK(hipMalloc(&p, 2 * stride));
                    P.allocs.push_back(p);
                    for (int s = 0; s < 2; ++s) P.slot[a][s] = (char *)p + s * stride;
                }
            }
            for (auto &sl : P.slot)
                for (char *s : sl) {
                    CHECK(hipMemset(s, 0, kOff));
                    CHECK(hipMemcpy(s + kOff, h.data(), payload, hipMemcpyHostToDevice));
                }
            pairs.push_back(P);
        }
    double *clock;
    dpwa_coef *coef;
    CHECK(hipMalloc(&clock, 4 * sizeof(double)));
    CHECK(hipMalloc(&coef, 2 * sizeof(dpwa_coef)));
    CHECK(hipMemset(clock, 0, 4 * sizeof(double)));
    static dpwa_interp cfg{DPWA_INTERP_CONSTANT, 0, 0.5, 0.0};
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int pass = 0; pass < 2; ++pass)
        for (auto &P : pairs) {
            CHECK(hipStreamSynchronize(st));
            for (int r = 0; r < rounds; ++r) {
                const int k = r & 1;
                dpwa_average_desc d[2];
                for (int a = 0; a < 2; ++a)
                    d[a] = dpwa_average_desc{P.slot[a][k] + kOff, P.slot[1 - a][k], n, clock + 2 * a, 1.0, coef + a,
                                             P.slot[a][1 - k] + kOff};
                if (r == rounds / 4) CHECK(hipEventRecord(e0, st));
                if (dpwa_average_many_resident(DPWA_F32, d, 2, &cfg, st, nullptr, nullptr)) {
                    fprintf(stderr, "%s\n", dpwa_last_error());
                    return 1;
                }
            }
            CHECK(hipEventRecord(e1, st));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            P.us.push_back(1e3 * ms / (rounds - rounds / 4));
        }
    for (int k = 0; k < 3; ++k) {
        printf("%-7s", kinds[k]);
        for (auto &P : pairs)
            if (P.kind == k) printf("  %.2f/%.2f", P.us[0], P.us[1]);
        printf("   (us per round, pass 0/pass 1, per pair)\n");
    }
    return 0;
}
