// node_tsan.cpp -- TEST INFRASTRUCTURE: node.cpp + sched.cpp (the host scheduler and the per-round
// logic) built with ThreadSanitizer over the host-only learner stand-in (fake_learner.cpp).  The
// C ABI promises that calls are reentrant per handle: different handles may be driven from
// different threads at once (one DpwaConnection per thread, or the ranks of a job in one process).
// T threads each drive their own group of G lock-step nodes for `rounds` rounds -- random stalls,
// rescue lanes, faults, flow control, add/remove of peers, the Bernoulli gate at p < 1 -- with the
// roctx trace hooks live, so every piece of state the library shares between handles (error
// strings, the trace switch, statics of the scheduler and the node) is touched concurrently.  The
// races the reference has (conn.py:106 have_state read outside the lock, :240 peers read outside
// peers_lock, :259/:313 remove_peer from inside the Tx loop) have no counterpart if TSan stays
// silent here.  Exit 0 and "node tsan ok" on success; TSan reports make the run fail (halt_on_error).
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../../include/dpwa_hip.h"

extern "C" {
int fake_stall(dpwa_learner *l, int n);
int fake_land_all(dpwa_learner *l);
int fake_counts(dpwa_learner *l, int *out);
int fake_lanes(dpwa_learner *l, int cap, int land_after);
}

namespace {

std::atomic<int> g_failed{0};
std::atomic<long> g_rounds{0};

struct Rng {
    uint64_t s;
    uint64_t next()
    {
        uint64_t z = (s += 0x9e3779b97f4a7c15ULL);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
        return z ^ (z >> 31);
    }
};

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        const int rc_ = (x);                                                                       \
        if (rc_) {                                                                                 \
            fprintf(stderr, "thread %d: %s:%d %s = %d (%s)\n", t, __FILE__, __LINE__, #x, rc_,     \
                    dpwa_last_error());                                                            \
            g_failed++;                                                                            \
            return;                                                                                \
        }                                                                                          \
    } while (0)
#define EXPECT(c)                                                                                  \
    do {                                                                                           \
        if (!(c)) {                                                                                \
            fprintf(stderr, "thread %d: %s:%d invariant failed: %s\n", t, __FILE__, __LINE__, #c); \
            g_failed++;                                                                            \
            return;                                                                                \
        }                                                                                          \
    } while (0)

void group(int t, int G, int rounds)
{
    Rng rng{0x5eedULL + 1000003ULL * (uint64_t)t};
    const double fp = (t % 2) ? 0.7 : 1.0;
    const dpwa_interp cfg{DPWA_INTERP_CONSTANT, 0, 0.5, 0.0};
    std::vector<dpwa_node *> nodes(G, nullptr);
    std::vector<dpwa_learner *> learners(G, nullptr);
    std::vector<dpwa_sched *> scheds(G, nullptr);
    for (int g = 0; g < G; ++g) {
        const uint32_t key[2] = {(uint32_t)t, (uint32_t)g};
        CHECK(dpwa_node_create(&nodes[g], G - 1, key, 2, fp, &cfg));
        CHECK(dpwa_node_bind(nodes[g], 0, 1000, DPWA_F32));
        CHECK(dpwa_node_handles(nodes[g], &learners[g], &scheds[g]));
        CHECK(dpwa_node_set_timeout(nodes[g], 5));
    }
    for (int g = 0; g < G; ++g)
        for (int k = 0, j = 0; j < G; ++j)
            if (j != g) CHECK(dpwa_node_set_peer(nodes[g], k++, DPWA_NODE_PEER_LOCAL, nodes[j]));
    for (int r = 0; r < rounds; ++r) {
        std::vector<int> fetching(G);
        for (int g = 0; g < G; ++g) {
            const uint64_t u = rng.next() % 100;
            CHECK(fake_stall(learners[g], u < 70 ? 0 : u < 85 ? 1 : u < 95 ? 3 : 9));
            int lanes_now[5];
            CHECK(fake_counts(learners[g], lanes_now));
            int cap = (g % 2) ? 3 : 8;
            if (cap < lanes_now[2]) cap = lanes_now[2];
            CHECK(fake_lanes(learners[g], cap, 2));
            // faults on all but one live peer at most (a round where every live peer is slow or
            // empty spins for ever in the reference's TxThread, conn.py:286-313)
            int keep = -1;
            for (int k = 0; k < G - 1; ++k) {
                int sc = 0;
                CHECK(dpwa_sched_score(scheds[g], k, &sc));
                if (sc >= 0 && keep < 0) keep = k;
            }
            for (int k = 0; k < G - 1; ++k) {
                int f = -1;
                if (k != keep && rng.next() % 100 < 20) {
                    const uint64_t v = rng.next() % 100;
                    f = v < 20 ? DPWA_PEER_DOWN : v < 60 ? DPWA_PEER_SLOW : DPWA_PEER_NO_STATE;
                }
                CHECK(dpwa_node_set_fault(nodes[g], k, f));
            }
        }
        for (int g = 0; g < G; ++g)
            CHECK(dpwa_node_update_send(nodes[g], nullptr, 1.0, nullptr, 0, nullptr, &fetching[g]));
        for (int g = 0; g < G; ++g) {
            int peer = -2;
            CHECK(dpwa_node_update_wait_average(nodes[g], nullptr, 1.0, nullptr, 0, nullptr, &peer));
            EXPECT(peer >= -1 && peer < G - 1);
            EXPECT(fetching[g] || peer < 0);
            for (int k = 0; k < G - 1; ++k) {
                int sc = 0;
                CHECK(dpwa_sched_score(scheds[g], k, &sc));
                EXPECT(sc == -1 || (sc >= 10 && sc <= 1000));
            }
        }
        for (int g = 0; g < G; ++g) CHECK(fake_land_all(learners[g]));
        // an error string on this thread while the others write theirs
        if (dpwa_node_bind(nodes[0], 0, 1, DPWA_F32) == DPWA_OK) EXPECT(false);
        EXPECT(dpwa_last_error()[0] != 0);
        dpwa_trace_push("node_tsan.round");
        dpwa_trace_pop();
        g_rounds++;
    }
    for (int g = 0; g < G; ++g) CHECK(dpwa_node_destroy(nodes[g]));
}

}  // namespace

// The control: two threads bump one plain int (what the reference's peers dict and have_state
// are to its threads).  TSan must report it, or this build is not instrumented.
int g_unguarded = 0;

void racy(int n)
{
    for (int i = 0; i < n; ++i) g_unguarded++;
}

int main(int argc, char **argv)
{
    if (argc > 1 && argv[1][0] == 'r') {   // "racy": the control
        std::thread a(racy, 100000), b(racy, 100000);
        a.join();
        b.join();
        printf("racy control ran (%d)\n", g_unguarded);
        return 0;
    }
    const int T = argc > 1 ? atoi(argv[1]) : 4;
    const int G = argc > 2 ? atoi(argv[2]) : 4;
    const int rounds = argc > 3 ? atoi(argv[3]) : 2000;
    if (T < 1 || T > 64 || G < 2 || G > 16 || rounds < 1) return 1;
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(group, t, G, rounds);
    for (auto &x : th) x.join();
    if (g_failed.load()) return 2;
    printf("node tsan ok: %d threads x %d learners x %d rounds (%ld rounds), trace %s\n", T, G, rounds,
           g_rounds.load(), dpwa_trace_enabled() ? "on" : "off");
    return 0;
}
