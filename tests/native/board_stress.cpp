// Host-only stress of the gossip board (dpwa_amd/csrc/board.cpp) for the sanitizer builds in
// tests/test_native_sanitizers.py.  Each thread is one rank of one board: it publishes its
// snapshots into two host slots under the board's publish rule (publish_wait, write the slot,
// advertise) and, between publishes, reads a random peer's newest snapshot seqlock-style
// (acquire, read the slot, release) -- the free-running gossip of AsyncDistGroup with the
// device steps done on the host.  Checks: a read never sees a torn or rewritten snapshot, the
// versions of a peer never go backwards, no wait times out.  (ThreadSanitizer cannot follow
// this protocol: every rank maps the shared block at its own address, and TSan pairs atomics
// by virtual address, so it reports the slot accesses as races; the torn-snapshot check is the
// race check here.)
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <thread>
#include <unistd.h>
#include <vector>

#include "../../dpwa_amd/csrc/kernels.hpp"

namespace dpwa {
int set_error(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    std::vfprintf(stderr, fmt, ap);
    va_end(ap);
    std::fputc('\n', stderr);
    return code;
}
// stream-ordered board stores are device work; this test only uses the host forms
hipError_t launch_store_u64(uint64_t *, uint64_t, hipStream_t) { return hipErrorInvalidValue; }
}  // namespace dpwa

#define CHECK(c)                                                                    \
    do {                                                                            \
        if (!(c)) {                                                                 \
            std::fprintf(stderr, "%s:%d check failed: %s\n", __FILE__, __LINE__, #c); \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

constexpr int kWords = 512;

struct Rank {
    std::vector<uint64_t> slot[2];
};

static uint64_t stamp(int rank, uint64_t version, int i) { return (uint64_t)rank << 48 ^ version << 12 ^ (uint64_t)i; }

int main(int argc, char **argv)
{
    const int world = argc > 1 ? std::atoi(argv[1]) : 4;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 2000;
    const std::string name = "/dpwa_board_stress_" + std::to_string(getpid());
    std::vector<Rank> ranks((size_t)world);
    for (auto &r : ranks)
        for (auto &s : r.slot) s.assign(kWords, 0);
    std::vector<dpwa_board *> boards((size_t)world, nullptr);
    CHECK(dpwa_board_open(&boards[0], name.c_str(), world, 0, 1) == DPWA_OK);
    for (int r = 1; r < world; ++r) CHECK(dpwa_board_open(&boards[r], name.c_str(), world, r, 0) == DPWA_OK);
    CHECK(dpwa_board_unlink(name.c_str()) == DPWA_OK);
    std::atomic<long> reads{0}, empty{0};
    auto run = [&](int me) {
        dpwa_board *b = boards[me];
        std::mt19937 rng(1000 + me);
        std::vector<uint64_t> last((size_t)world, 0);
        for (uint64_t v = 1; v <= (uint64_t)rounds; ++v) {
            // publish v: wait out readers of the slot it rewrites (that of v - 2), fill, announce
            CHECK(dpwa_board_publish_wait(b, v, 20000) == DPWA_OK);
            std::vector<uint64_t> &slot = ranks[me].slot[(v - 1) % 2];
            for (int i = 0; i < kWords; ++i) slot[i] = stamp(me, v, i);
            CHECK(dpwa_board_advertise(b, v, nullptr, 1) == DPWA_OK);
            // read a random peer's newest snapshot
            int r = (int)(rng() % (uint32_t)(world - 1));
            if (r >= me) ++r;
            int32_t st = -1;
            CHECK(dpwa_board_status(b, r, &st) == DPWA_OK);
            uint64_t got = 0;
            CHECK(dpwa_board_acquire(b, r, &got) == DPWA_OK);
            if (got == 0) {
                empty++;
                continue;
            }
            CHECK(got >= last[r]);
            last[r] = got;
            const std::vector<uint64_t> &src = ranks[r].slot[(got - 1) % 2];
            uint64_t bad = 0;
            for (int i = 0; i < kWords; ++i) bad += src[i] != stamp(r, got, i);
            CHECK(bad == 0);
            if (rng() % 4 == 0) std::this_thread::yield();   // a slow reader now and then
            uint64_t mine = 0;
            CHECK(dpwa_board_read(b, r, nullptr, &mine, nullptr) == DPWA_OK && mine == got);
            CHECK(dpwa_board_release(b, r, nullptr, 1) == DPWA_OK);
            reads++;
        }
    };
    std::vector<std::thread> th;
    for (int r = 0; r < world; ++r) th.emplace_back(run, r);
    for (auto &t : th) t.join();
    for (int r = 0; r < world; ++r) CHECK(dpwa_board_close(boards[r]) == DPWA_OK);
    CHECK(reads.load() > 0);
    std::printf("board stress ok: %d ranks x %d rounds, %ld reads, %ld found nothing\n", world, rounds, reads.load(),
                empty.load());
    return 0;
}
