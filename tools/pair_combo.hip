// pair_combo.hip -- does the resident pair dispatch's speed depend on WHICH buffers the two
// learners got (their physical placement), stably per combination?  Allocates L learner-layout
// buffers ([slot|slot] each, as learner.cpp) and times the product's mutual-pair dispatch
// (dpwa_average_many_resident, XCD-grouped) in the gossip loop for many (A, B) combinations, each
// measured twice in separate passes (not part of the product).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -o tools/pair_combo tools/pair_combo.hip
//        -Ldpwa_amd -ldpwa_hip -Wl,-rpath,'$ORIGIN/../dpwa_amd'
// Run:   tools/pair_combo [numel] [learners] [rounds] [frag_kib] [contig]
//   frag_kib > 0: first fill 1.5 GB of the heap with frag_kib-KiB allocations and free every other
//   one (holes the learners' buffers may be assembled from: small TLB fragments); contig 1: the
//   learners' buffers from hipExtMallocWithFlags(hipDeviceMallocContiguous)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <utility>
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

int main(int argc, char **argv)
{
    const int64_t n = argc > 1 ? atoll(argv[1]) : 11173962;
    const int L = argc > 2 ? atoi(argv[2]) : 8;
    const int rounds = argc > 3 ? atoi(argv[3]) : 400;
    const size_t payload = (size_t)n * 4;
    const size_t stride = (kOff + payload + 4095) / 4096 * 4096;
    std::vector<float> h((size_t)n, 0.5f);
    const int frag_kib = argc > 4 ? atoi(argv[4]) : 0;
    const int contig = argc > 5 ? atoi(argv[5]) : 0;
    std::vector<void *> frag;
    if (frag_kib > 0) {
        const size_t fb = (size_t)frag_kib << 10;
        frag.resize((size_t)(1.5e9 / fb));
        for (auto &f : frag) CHECK(hipMalloc(&f, fb));
        for (size_t i = 0; i < frag.size(); i += 2) CHECK(hipFree(frag[i]));
    }
    std::vector<char *> base(L);
    for (auto &p : base) {
        if (contig)
            CHECK(hipExtMallocWithFlags((void **)&p, 2 * stride, hipDeviceMallocContiguous));
        else
            CHECK(hipMalloc(&p, 2 * stride));
        for (int k = 0; k < 2; ++k) {
            CHECK(hipMemset(p + k * stride, 0, kOff));
            CHECK(hipMemcpy(p + k * stride + kOff, h.data(), payload, hipMemcpyHostToDevice));
        }
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
    std::vector<std::pair<int, int>> combos;
    for (int a = 0; a < L; ++a)
        for (int b = a + 1; b < L; ++b) combos.push_back({a, b});
    std::vector<std::vector<double>> res(combos.size());
    for (int pass = 0; pass < 2; ++pass)
        for (size_t c = 0; c < combos.size(); ++c) {
            char *s[2][2];
            for (int x = 0; x < 2; ++x)
                for (int k = 0; k < 2; ++k) s[x][k] = base[x ? combos[c].second : combos[c].first] + k * stride;
            CHECK(hipStreamSynchronize(st));
            for (int r = 0; r < rounds; ++r) {
                const int k = r & 1;
                dpwa_average_desc d[2];
                for (int a = 0; a < 2; ++a)
                    d[a] = dpwa_average_desc{s[a][k] + kOff, s[1 - a][k], n, clock + 2 * a, 1.0, coef + a,
                                             s[a][1 - k] + kOff};
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
            res[c].push_back(1e3 * ms / (rounds - rounds / 4));
        }
    std::vector<size_t> order(combos.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = i;
    std::sort(order.begin(), order.end(), [&](size_t x, size_t y) { return res[x][0] < res[y][0]; });
    double sum = 0;
    for (auto &r : res) sum += r[0] + r[1];
    printf("frag_kib %d contig %d: mean over combinations %.2f us\n", frag_kib, contig, sum / (2.0 * res.size()));
    for (size_t i : order)
        printf("A %d B %d  pass0 %6.2f us  pass1 %6.2f us   (A %p B %p)\n", combos[i].first, combos[i].second,
               res[i][0], res[i][1], (void *)base[combos[i].first], (void *)base[combos[i].second]);
    return 0;
}
