// Host-only stress of the scheduler's C ABI (dpwa_amd/csrc/sched.cpp) for the sanitizer
// build in tests/test_native_sanitizers.py: random sequences of every entry point, with the
// invariants of conn.py:178-317 checked after each call and malformed calls expected to fail
// cleanly.  Exit status 0 = every check held (ASan/UBSan abort on their own findings).
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "../../include/dpwa_hip.h"

namespace dpwa {
int set_error(int code, const char *, ...) { return code; }   // learner.cpp's, not linked here
}  // namespace dpwa

#define CHECK(c)                                                                    \
    do {                                                                            \
        if (!(c)) {                                                                 \
            std::fprintf(stderr, "%s:%d check failed: %s\n", __FILE__, __LINE__, #c); \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

static void check_scores(dpwa_sched *s, int n, const std::vector<char> &removed)
{
    int live = 0;
    for (int p = 0; p < n; ++p) {
        int sc = 0;
        CHECK(dpwa_sched_score(s, p, &sc) == DPWA_OK);
        if (removed[p]) {
            CHECK(sc == -1);
        } else {
            CHECK(sc >= 10 && sc <= 1000);   // conn.py:264-272 bounds
            ++live;
        }
    }
    int nl = -1;
    CHECK(dpwa_sched_n_live(s, &nl) == DPWA_OK && nl == live);
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? std::atoi(argv[1]) : 200;
    std::mt19937 rng(12345);
    auto uni = [&](int a, int b) { return std::uniform_int_distribution<int>(a, b)(rng); };
    for (int it = 0; it < iters; ++it) {
        const int n = uni(0, 9);
        std::vector<uint32_t> key(uni(0, 3));
        for (auto &w : key) w = rng();
        dpwa_sched *s = nullptr;
        const double fp = uni(0, 4) / 4.0;
        CHECK(dpwa_sched_create(&s, n, key.data(), (int)key.size(), fp) == DPWA_OK && s);
        std::vector<char> removed((size_t)n, 0);
        for (int step = 0; step < 300; ++step) {
            switch (uni(0, 7)) {
            case 0: {   // one whole fetch loop against a random static status
                std::vector<int32_t> st((size_t)(n > 0 ? n : 1));
                for (auto &x : st) x = uni(DPWA_PEER_READY, DPWA_PEER_DEAD);
                int peer = -2, att = -1;
                CHECK(dpwa_sched_fetch(s, st.data(), 50, &peer, &att) == DPWA_OK);
                CHECK(att >= 0 && att <= 50);
                CHECK(peer == -1 || (peer >= 0 && peer < n && st[peer] == DPWA_PEER_READY));
                for (int p = 0; p < n; ++p) {
                    int sc = 0;
                    dpwa_sched_score(s, p, &sc);
                    if (sc == -1) removed[p] = 1;
                }
                break;
            }
            case 1: {   // pick + report, the way node.cpp drives it
                int peer = -2, connected = -1;
                CHECK(dpwa_sched_pick(s, &peer, &connected) == DPWA_OK);
                int nl = 0;
                dpwa_sched_n_live(s, &nl);
                CHECK((peer == -1) == (nl == 0));
                if (peer < 0) break;
                CHECK(peer < n && !removed[peer]);
                int done = 0, data = 0;
                if (!connected) {
                    const int c = uni(DPWA_CONNECT_OK, DPWA_CONNECT_ERROR);
                    CHECK(dpwa_sched_report(s, peer, c, &done, &data) == DPWA_OK);
                    CHECK(!data);
                    if (c == DPWA_CONNECT_ERROR) removed[peer] = 1;
                    if (done) break;
                }
                const int r = uni(DPWA_REPLY_PAYLOAD, DPWA_REPLY_ERROR);
                CHECK(dpwa_sched_report(s, peer, r, &done, &data) == DPWA_OK);
                CHECK(data == (r == DPWA_REPLY_PAYLOAD));
                if (r == DPWA_REPLY_ERROR) removed[peer] = 1;
                break;
            }
            case 2: {
                if (n == 0) break;
                const int p = uni(0, n - 1);
                CHECK(dpwa_sched_remove(s, p) == DPWA_OK || removed[p]);
                removed[p] = 1;
                break;
            }
            case 3: {
                if (n == 0) break;
                const int p = uni(0, n - 1);
                CHECK(dpwa_sched_add(s, p) == DPWA_OK);
                removed[p] = 0;
                int sc = 0;
                CHECK(dpwa_sched_score(s, p, &sc) == DPWA_OK && sc == 1000);   // conn.py:190
                break;
            }
            case 4: {
                int f = -1;
                CHECK(dpwa_sched_bernoulli(s, &f) == DPWA_OK && (f == 0 || f == 1));
                if (fp == 0.0) CHECK(f == 0);
                if (fp == 1.0) CHECK(f == 1);
                double x = -1;
                CHECK(dpwa_sched_random(s, &x) == DPWA_OK && x >= 0.0 && x < 1.0);
                break;
            }
            case 5: {
                const int64_t a = uni(-5, 5), b = a + uni(0, 2000);
                int64_t v = 0;
                CHECK(dpwa_sched_randint(s, a, b, &v) == DPWA_OK && v >= a && v <= b);
                break;
            }
            case 6: {   // checkpoint: a twin restored from the state continues identically; damaged
                        // or truncated states fail without changing the scheduler they were given to
                int nw = 0;
                CHECK(dpwa_sched_get_state(s, nullptr, 0, &nw) == DPWA_OK && nw > 0);
                std::vector<uint32_t> st((size_t)nw);
                CHECK(dpwa_sched_get_state(s, st.data(), nw - 1, &nw) != DPWA_OK);
                CHECK(dpwa_sched_get_state(s, st.data(), nw, &nw) == DPWA_OK);
                dpwa_sched *t = nullptr;
                const uint32_t other = (uint32_t)rng();
                CHECK(dpwa_sched_create(&t, n, &other, 1, fp) == DPWA_OK && t);
                int tw = 0;    // t's own size: all its peers are live, s's may not be
                CHECK(dpwa_sched_get_state(t, nullptr, 0, &tw) == DPWA_OK);
                std::vector<uint32_t> before((size_t)tw), after((size_t)tw);
                CHECK(dpwa_sched_get_state(t, before.data(), tw, &tw) == DPWA_OK);
                std::vector<uint32_t> bad = st;
                const int cut = uni(0, nw - 1);
                if (uni(0, 1)) {
                    bad.resize((size_t)cut);           // truncated
                } else {                               // one word damaged
                    bad[(size_t)cut] ^= (uint32_t)uni(1, 0x7fffffff);
                }
                const int rc = dpwa_sched_set_state(t, bad.data(), (int)bad.size());
                if (rc != DPWA_OK) {
                    int aw = 0;
                    CHECK(dpwa_sched_get_state(t, after.data(), tw, &aw) == DPWA_OK && aw == tw);
                    CHECK(after == before);
                }
                CHECK(dpwa_sched_set_state(t, st.data(), nw) == DPWA_OK);
                for (int j = 0; j < 20; ++j) {
                    int pa = -2, pb = -2, ca = -1, cb = -1;
                    CHECK(dpwa_sched_pick(s, &pa, &ca) == DPWA_OK && dpwa_sched_pick(t, &pb, &cb) == DPWA_OK);
                    CHECK(pa == pb && ca == cb);
                    if (pa >= 0) {
                        const int r = uni(DPWA_REPLY_PAYLOAD, DPWA_REPLY_TIMEOUT);
                        int d1 = 0, d2 = 0, x1 = 0, x2 = 0;
                        CHECK(dpwa_sched_report(s, pa, r, &d1, &x1) == DPWA_OK);
                        CHECK(dpwa_sched_report(t, pb, r, &d2, &x2) == DPWA_OK);
                        CHECK(d1 == d2 && x1 == x2);
                    }
                    double xa = 0, xb = 1;
                    CHECK(dpwa_sched_random(s, &xa) == DPWA_OK && dpwa_sched_random(t, &xb) == DPWA_OK && xa == xb);
                }
                CHECK(dpwa_sched_destroy(t) == DPWA_OK);
                break;
            }
            default: {   // malformed calls fail cleanly
                int x = 0, y = 0;
                int64_t v = 0;
                CHECK(dpwa_sched_score(s, n + uni(0, 3), &x) != DPWA_OK);
                CHECK(dpwa_sched_score(s, -1 - uni(0, 3), &x) != DPWA_OK);
                CHECK(dpwa_sched_report(s, n + 1, DPWA_REPLY_PAYLOAD, &x, &y) != DPWA_OK);
                CHECK(dpwa_sched_add(s, n + uni(0, 3)) != DPWA_OK);
                CHECK(dpwa_sched_pick(nullptr, &x, &y) != DPWA_OK);
                CHECK(dpwa_sched_randint(s, 5, 4, &v) != DPWA_OK);
                break;
            }
            }
            check_scores(s, n, removed);
        }
        CHECK(dpwa_sched_destroy(s) == DPWA_OK);
    }
    std::printf("sched stress ok: %d schedulers\n", iters);
    return 0;
}
