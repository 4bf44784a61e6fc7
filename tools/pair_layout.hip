// pair_layout.hip -- the product's resident pair dispatch (dpwa_average_many_resident over two
// learners that average with each other, k_lerp_batch's XCD-grouped order) by buffer layout, in the
// gossip loop (each round reads the two published slots and writes the two other slots, then the
// roles swap) -- not part of the product.
//   sep      four separate hipMallocs, one per slot (tools/pair_tune.hip's layout)
//   learner  two hipMallocs of two slots each, [hdr|payload] x 2 at the learner's slot stride
//            (learner.cpp's layout)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -o tools/pair_layout tools/pair_layout.hip
//        -Ldpwa_amd -ldpwa_hip -Wl,-rpath,'$ORIGIN/../dpwa_amd'
// Run:   tools/pair_layout [numel] [rounds] [data 0|1|2]
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

int main(int argc, char **argv)
{
    const int64_t n = argc > 1 ? atoll(argv[1]) : 11173962;
    const int rounds = argc > 2 ? atoi(argv[2]) : 400;
    const size_t payload = (size_t)n * 4;
    const size_t stride = (kOff + payload + 4095) / 4096 * 4096;
    // data: 0 all 0.5f, 1 random normal-ish floats (every mantissa bit toggles), 2 random in
    // [0.5, 1) rounded to 8 mantissa bits
    const int data = argc > 3 ? atoi(argv[3]) : 0;
    std::vector<float> h((size_t)n, 0.5f);
    uint32_t x = 12345u;
    for (auto &v : h) {
        if (!data) break;
        x = x * 1664525u + 1013904223u;
        const float u = (float)(x >> 8) / (float)(1 << 24);
        v = data == 1 ? (u - 0.5f) * 3.4f : 0.5f + (float)((int)(u * 256.f)) / 512.f;
    }
    struct Layout {
        const char *name;
        char *slot[2][2];    // [learner][slot]
    };
    // A heap with 2 MiB holes first: 1024 x 2 MiB, every other one freed, so that later
    // allocations may be assembled from small physical blocks (small TLB fragments).
    std::vector<void *> frag(1024);
    for (auto &f : frag) CHECK(hipMalloc(&f, 2 << 20));
    for (size_t i = 0; i < frag.size(); i += 2) CHECK(hipFree(frag[i]));
    std::vector<Layout> ls(5);
    ls[0].name = "sep (4 hipMallocs)";
    for (int a = 0; a < 2; ++a)
        for (int k = 0; k < 2; ++k) CHECK(hipMalloc(&ls[0].slot[a][k], stride));
    ls[1].name = "learner (2 x [slot|slot])";
    for (int a = 0; a < 2; ++a) {
        char *p;
        CHECK(hipMalloc(&p, 2 * stride));
        ls[1].slot[a][0] = p;
        ls[1].slot[a][1] = p + stride;
    }
    ls[2].name = "learner, B offset 1 MiB";
    for (int a = 0; a < 2; ++a) {
        char *p;
        CHECK(hipMalloc(&p, 2 * stride + (1 << 20)));
        p += a ? (1 << 20) : 0;
        ls[2].slot[a][0] = p;
        ls[2].slot[a][1] = p + stride;
    }
    ls[3].name = "learner, after 2 MiB holes";
    for (int a = 0; a < 2; ++a) {
        char *p;
        CHECK(hipMalloc(&p, 2 * stride));
        ls[3].slot[a][0] = p;
        ls[3].slot[a][1] = p + stride;
    }
    ls[4].name = "learner, contiguous flag";
    for (int a = 0; a < 2; ++a) {
        void *p;
        CHECK(hipExtMallocWithFlags(&p, 2 * stride, hipDeviceMallocContiguous));
        ls[4].slot[a][0] = (char *)p;
        ls[4].slot[a][1] = (char *)p + stride;
    }
    for (auto &L : ls)
        for (auto &sl : L.slot)
            for (char *s : sl) {
                CHECK(hipMemset(s, 0, kOff));
                CHECK(hipMemcpy(s + kOff, h.data(), payload, hipMemcpyHostToDevice));
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
        for (auto &L : ls) {
            std::vector<double> us;
            for (int r = 0; r < rounds; ++r) {
                const int k = r & 1;    // published slot this round; the average writes the other
                dpwa_average_desc d[2];
                for (int a = 0; a < 2; ++a)
                    d[a] = dpwa_average_desc{L.slot[a][k] + kOff, L.slot[1 - a][k], n, clock + 2 * a, 1.0, coef + a,
                                             L.slot[a][1 - k] + kOff};
                const bool timed = r >= rounds / 2 && (r % 4) == 0;
                if (dpwa_average_many_resident(DPWA_F32, d, 2, &cfg, st, timed ? e0 : nullptr, timed ? e1 : nullptr)) {
                    fprintf(stderr, "%s\n", dpwa_last_error());
                    return 1;
                }
                if (timed) {
                    CHECK(hipEventSynchronize(e1));
                    float ms;
                    CHECK(hipEventElapsedTime(&ms, e0, e1));
                    us.push_back(1e3 * ms);
                }
            }
            CHECK(hipStreamSynchronize(st));
            std::sort(us.begin(), us.end());
            double mean = 0;
            for (double y : us) mean += y;
            mean /= us.size();
            printf("pass %d %-28s loop: mean %7.2f us  median %7.2f  (4Ns %6.1f GB/s)  slots A %p %p B %p %p\n", pass,
                   L.name, mean, us[us.size() / 2], 4.0 * payload / mean / 1e3, (void *)L.slot[0][0],
                   (void *)L.slot[0][1], (void *)L.slot[1][0], (void *)L.slot[1][1]);
        }
    return 0;
}
