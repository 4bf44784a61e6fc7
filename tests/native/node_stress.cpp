// node_stress.cpp -- TEST INFRASTRUCTURE: node.cpp's per-round logic (DpwaConnection.update_send /
// update_wait, dpwa.py:104-156, with TxThread's fetch loop, conn.py:277-315) over the host-only
// fake learner (fake_learner.cpp) and the real scheduler (sched.cpp), built with the sanitizers.
// G lock-step learners, `rounds` rounds; in every round each learner's first `stall` pulls stall
// (the count drawn from a seeded generator, 0-12, mostly 0): the node must judge the side pull
// timed out, re-select into rescue lanes, keep re-selecting while a lane's pull stalls too -- with
// every lane taken (8, or 3 where lane allocations fail) waiting for one to land, and ending the
// round without data only when no lane lands within DPWA_RESCUE_WAIT_MS (a stuck transport).  Prints one JSON object per
// (round, learner) -- the script and what the node did -- for tests/test_node_host.py to replay in
// oracle/policy.py, and checks invariants on the way.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/dpwa_hip.h"

extern "C" {
int fake_stall(dpwa_learner *l, int n);
int fake_land_all(dpwa_learner *l);
int fake_counts(dpwa_learner *l, int *out);
int fake_lanes(dpwa_learner *l, int cap, int land_after);
}

static uint64_t g_rng = 0;
static uint64_t next_u64()
{
    uint64_t z = (g_rng += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

#define CHECK(x)                                                                             \
    do {                                                                                     \
        const int rc_ = (x);                                                                 \
        if (rc_) {                                                                           \
            fprintf(stderr, "%s:%d %s = %d (%s)\n", __FILE__, __LINE__, #x, rc_, dpwa_last_error()); \
            return 2;                                                                        \
        }                                                                                    \
    } while (0)
#define EXPECT(c)                                                                            \
    do {                                                                                     \
        if (!(c)) {                                                                          \
            fprintf(stderr, "%s:%d invariant failed: %s\n", __FILE__, __LINE__, #c);         \
            return 3;                                                                        \
        }                                                                                    \
    } while (0)

int main(int argc, char **argv)
{
    const int G = argc > 1 ? atoi(argv[1]) : 4;
    const int rounds = argc > 2 ? atoi(argv[2]) : 40;
    const uint32_t seed0 = argc > 3 ? (uint32_t)atoi(argv[3]) : 100;
    const double fp = argc > 4 ? atof(argv[4]) : 1.0;
    const int fault_pct = argc > 5 ? atoi(argv[5]) : 0;     // % of (round, learner, peer) with a fault
    const int prefetch = argc > 6 ? atoi(argv[6]) : 0;       // start every granted fetch once all have published
    g_rng = seed0 * 7919ULL + (uint64_t)G;
    if (G < 2 || G > 16 || rounds < 1) return 1;
    const dpwa_interp cfg{DPWA_INTERP_CONSTANT, 0, 0.5, 0.0};
    std::vector<dpwa_node *> nodes(G, nullptr);
    std::vector<dpwa_learner *> learners(G, nullptr);
    std::vector<dpwa_sched *> scheds(G, nullptr);
    for (int g = 0; g < G; ++g) {
        const uint32_t key = seed0 + (uint32_t)g;
        CHECK(dpwa_node_create(&nodes[g], G - 1, &key, 1, fp, &cfg));
        CHECK(dpwa_node_bind(nodes[g], 0, 1000, DPWA_F32));
        CHECK(dpwa_node_handles(nodes[g], &learners[g], &scheds[g]));
        CHECK(dpwa_node_set_timeout(nodes[g], 5));
    }
    for (int g = 0; g < G; ++g)   // peer k of g = the k-th other node, in node order
        for (int k = 0, j = 0; j < G; ++j)
            if (j != g) CHECK(dpwa_node_set_peer(nodes[g], k++, DPWA_NODE_PEER_LOCAL, nodes[j]));
    printf("[\n");
    bool first = true;
    for (int r = 0; r < rounds; ++r) {
        std::vector<int> stall(G), fetching(G), cap(G), stuck(G);
        std::vector<std::vector<int>> fault(G, std::vector<int>(G - 1, -1));
        for (int g = 0; g < G; ++g) {
            const uint64_t u = next_u64() % 100;
            stall[g] = u < 60 ? 0 : u < 70 ? 1 : u < 76 ? 2 : u < 81 ? 3 : u < 85 ? 4 : u < 89 ? 5 :
                       u < 94 ? 6 + (int)(next_u64() % 4) : 10 + (int)(next_u64() % 3);
            CHECK(fake_stall(learners[g], stall[g]));
            // odd learners: lane allocations fail after 3 lanes; a quarter of the rounds with every
            // lane stalled have a stuck transport (no lane ever lands), the rest a held-up one
            int lanes_now[5];
            CHECK(fake_counts(learners[g], lanes_now));
            cap[g] = (g % 2) ? 3 : 8;
            if (cap[g] < lanes_now[2]) cap[g] = lanes_now[2];
            stuck[g] = (next_u64() % 4) == 0;
            CHECK(fake_lanes(learners[g], cap[g], stuck[g] ? -1 : 2));
            for (int k = 0; k < G - 1; ++k) {   // what a request to peer k meets this round
                if ((int)(next_u64() % 100) < fault_pct) {
                    const uint64_t v = next_u64() % 100;
                    fault[g][k] = v < 15 ? DPWA_PEER_DOWN : v < 55 ? DPWA_PEER_SLOW : v < 98 ? DPWA_PEER_NO_STATE
                                                                                      : DPWA_PEER_DEAD;
                }
            }
            // at least one live peer answers normally (a round in which every live peer is slow or
            // has no state spins for ever in the reference's TxThread, conn.py:286-313)
            int live_ok = 0, first_live = -1;
            for (int k = 0; k < G - 1; ++k) {
                int sc = 0;
                CHECK(dpwa_sched_score(scheds[g], k, &sc));
                if (sc < 0) continue;
                if (first_live < 0) first_live = k;
                live_ok += fault[g][k] < 0;
            }
            if (!live_ok && first_live >= 0) fault[g][first_live] = -1;
            for (int k = 0; k < G - 1; ++k) CHECK(dpwa_node_set_fault(nodes[g], k, fault[g][k]));
        }
        for (int g = 0; g < G; ++g)
            CHECK(dpwa_node_update_send(nodes[g], nullptr, 1.0, nullptr, 0, nullptr, &fetching[g]));
        if (prefetch)   // LocalGroup(prefetch=True): the pulls start before the training step
            for (int g = 0; g < G; ++g) CHECK(dpwa_node_start_fetch(nodes[g], 0, nullptr));
        for (int g = 0; g < G; ++g) {
            int before[5], after[5], peer = -2, f = 0, fp_ = 0, att = 0;
            uint64_t fv = 0;
            CHECK(fake_counts(learners[g], before));
            CHECK(dpwa_node_update_wait_average(nodes[g], nullptr, 1.0, nullptr, 0, nullptr, &peer));
            CHECK(fake_counts(learners[g], after));
            CHECK(dpwa_node_info(nodes[g], &f, &fp_, &fv, &att));
            EXPECT(peer >= -1 && peer < G - 1);
            EXPECT(after[3] - before[3] == (peer >= 0 ? 1 : 0));            // averaged iff data
            EXPECT(after[2] <= cap[g]);                                      // lanes within the cap
            EXPECT(fetching[g] || peer < 0);
            if (!fetching[g]) att = 0;                                       // (info keeps the last fetch's count)
            EXPECT(after[0] - before[0] <= att);                             // a pull per attempt at most
            printf("%s{\"round\": %d, \"learner\": %d, \"stall\": %d, \"fetching\": %d, \"peer\": %d, \"attempts\": %d, "
                   "\"pulls\": %d, \"rescue_pulls\": %d, \"lanes\": %d, \"cap\": %d, \"stuck\": %d, \"scores\": [",
                   first ? "" : ",\n", r, g, stall[g], fetching[g], peer, att, after[0] - before[0],
                   after[1] - before[1], after[2], cap[g], stuck[g]);
            first = false;
            for (int k = 0; k < G - 1; ++k) {
                int sc = 0;
                CHECK(dpwa_sched_score(scheds[g], k, &sc));
                EXPECT(sc == -1 || (sc >= 10 && sc <= 1000));
                printf("%s%d", k ? ", " : "", sc);
            }
            printf("], \"faults\": [");
            for (int k = 0; k < G - 1; ++k) printf("%s%d", k ? ", " : "", fault[g][k]);
            printf("]}");
        }
        for (int g = 0; g < G; ++g) CHECK(fake_land_all(learners[g]));
    }
    printf("\n]\n");
    for (int g = 0; g < G; ++g) CHECK(dpwa_node_destroy(nodes[g]));
    fprintf(stderr, "node stress ok\n");
    return 0;
}
