// board.cpp -- the gossip board: free-running (asynchronous) rounds across processes.
//
// The reference's learners never wait for each other: RxThread serves whatever snapshot
// its node published last (conn.py:73-79, 98-110), under a Lock that makes a publish wait
// while a reply is being sent (conn.py:76-79 vs 109-110), and a fetch to a process that is
// gone meets ConnectionRefusedError (conn.py:253-256).  The lock-step DistGroup replaces
// all of that with one barrier per round; the board restores the free-running behaviour
// without any collective on the data path:
//
//   * one POSIX shared-memory block per node set (all ranks of a node), mapped by every
//     rank and registered with HIP so a stream can write into it;
//   * version[p]   -- the newest *complete* snapshot of publisher p.  Written by p's stream
//                     (a one-wave release-store kernel) after the publish kernel and its
//                     system-scope release, so a reader never sees a version before its bytes;
//   * reading[p][r] -- the version of p that reader r is pulling (0 = none).  Set by r's
//                     host before the pull is enqueued, cleared by r's side stream after
//                     the pull has landed;
//   * pid / closed -- liveness: a closed board entry or a dead pid is a refused connection.
//
// Publisher p, before its publish number v (which rewrites the slot of v-2, learner.cpp):
// waits until version[p] == v-1 (its own last publish is out) and then until no live
// reader holds v-2 -- the reference's Lock, blocking a publish only while a peer still
// reads the snapshot it would destroy.  Reader r acquires a version of p seqlock-style:
// v = version[p]; reading[p][r] = v; re-read version[p]; accept when unchanged.  If
// version[p] moved to v+1, p may already be checking readers for v+2 (which rewrites v's
// slot) without having seen our mark, so the reader retries with the newer version; if it
// is still v, p has not finished publishing v+1, so its check for v+2 comes later and
// sees the mark.
//
// A reader clears its mark from its side stream, after the pull, while its host may already
// be in the next round.  If the next round picks the same publisher, the new mark must not
// be wiped by that still-queued clear of the old one (the old store of 0 would land after
// the new mark and let the publisher rewrite the slot mid-pull).  So every stream-ordered
// release records an event, and the next acquire of the same publisher first waits for it:
// a reader holds at most one mark per publisher, and marks are only ever cleared by the
// release of the acquisition that set them.
#include <hip/hip_runtime.h>

#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <fcntl.h>
#include <new>
#include <signal.h>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

#include "common.hpp"
#include "kernels.hpp"

using namespace dpwa;

namespace {

constexpr uint64_t kBoardMagic = 0x445057414252440aULL;   // "DPWABRD\n"

struct alignas(64) BoardHead {
    uint64_t magic;
    int32_t world;
    int32_t pad;
};

struct alignas(64) NodeRec {
    uint64_t version;   // newest complete publish (device-written)
    int32_t pid;
    int32_t closed;
};

size_t board_bytes(int world)
{
    const size_t raw = sizeof(BoardHead) + sizeof(NodeRec) * (size_t)world + 8 * (size_t)world * (size_t)world;
    const size_t page = (size_t)sysconf(_SC_PAGESIZE);
    return (raw + page - 1) / page * page;
}

template <class T>
T load(const T *p)
{
    return __atomic_load_n(p, __ATOMIC_SEQ_CST);
}

template <class T>
void store(T *p, T v)
{
    __atomic_store_n(p, v, __ATOMIC_SEQ_CST);
}

}  // namespace

struct dpwa_board {
    int world = 0, rank = 0;
    std::string name;
    char *base = nullptr;
    size_t bytes = 0;
    BoardHead *head = nullptr;
    NodeRec *nodes = nullptr;
    uint64_t *reading = nullptr;   // [publisher * world + reader]
    char *dev_base = nullptr;      // device alias of `base` once registered
    int device = -1;
    // per publisher: the event recorded after our last stream-ordered release of its mark
    std::vector<hipEvent_t> released;
    std::vector<char> release_pending;

    uint64_t *dev(const void *host_ptr) const
    {
        return (uint64_t *)(dev_base + ((const char *)host_ptr - base));
    }

    bool alive(int r) const
    {
        if (load(&nodes[r].closed)) return false;
        const int32_t pid = load(&nodes[r].pid);
        if (pid <= 0) return false;
        return !(kill(pid, 0) == -1 && errno == ESRCH);
    }
};

// Stream-ordered store into the board: a one-wave kernel (a release store at system scope)
// by default; DPWA_BOARD_WRITE=value uses hipStreamWriteValue64 instead (comparison).
static hipError_t stream_store(uint64_t *dev_ptr, uint64_t v, hipStream_t s)
{
    static const bool write_value = [] {
        const char *e = getenv("DPWA_BOARD_WRITE");
        return e && std::string(e) == "value";
    }();
    if (write_value) return hipStreamWriteValue64(s, dev_ptr, v, 0);
    return launch_store_u64(dev_ptr, v, s);
}

extern "C" {

int dpwa_board_open(dpwa_board **out, const char *name, int world, int rank, int create)
{
    if (!out || !name || name[0] != '/' || world < 1 || rank < 0 || rank >= world)
        return set_error(DPWA_ERR_ARG, "dpwa_board_open: bad arguments");
    const size_t bytes = board_bytes(world);
    const int fd = shm_open(name, create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
    if (fd < 0) return set_error(DPWA_ERR_ARG, "dpwa_board_open: shm_open(%s): %s", name, strerror(errno));
    if (create && ftruncate(fd, (off_t)bytes) != 0) {
        const int e = errno;
        close(fd);
        shm_unlink(name);
        return set_error(DPWA_ERR_NOMEM, "dpwa_board_open: ftruncate: %s", strerror(e));
    }
    struct stat st;
    if (fstat(fd, &st) != 0 || (size_t)st.st_size < bytes) {
        close(fd);
        return set_error(DPWA_ERR_ARG, "dpwa_board_open: %s is not a board for %d ranks", name, world);
    }
    void *p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) return set_error(DPWA_ERR_NOMEM, "dpwa_board_open: mmap: %s", strerror(errno));
    dpwa_board *b = new (std::nothrow) dpwa_board();
    if (!b) {
        munmap(p, bytes);
        return set_error(DPWA_ERR_NOMEM, "dpwa_board_open: out of memory");
    }
    b->world = world;
    b->rank = rank;
    b->name = name;
    b->base = (char *)p;
    b->bytes = bytes;
    b->head = (BoardHead *)p;
    b->nodes = (NodeRec *)(b->base + sizeof(BoardHead));
    b->reading = (uint64_t *)(b->base + sizeof(BoardHead) + sizeof(NodeRec) * (size_t)world);
    if (create) {   // ftruncate zero-filled the block
        b->head->world = world;
        store(&b->head->magic, kBoardMagic);
    } else if (load(&b->head->magic) != kBoardMagic || b->head->world != world) {
        munmap(p, bytes);
        delete b;
        return set_error(DPWA_ERR_ARG, "dpwa_board_open: %s is not a board for %d ranks", name, world);
    }
    store(&b->nodes[rank].version, (uint64_t)0);
    for (int r = 0; r < world; ++r) store(&b->reading[(size_t)rank * world + r], (uint64_t)0);
    store(&b->nodes[rank].closed, 0);
    store(&b->nodes[rank].pid, (int32_t)getpid());
    *out = b;
    return DPWA_OK;
}

int dpwa_board_unlink(const char *name)
{
    if (!name) return set_error(DPWA_ERR_ARG, "dpwa_board_unlink: NULL name");
    if (shm_unlink(name) != 0 && errno != ENOENT)
        return set_error(DPWA_ERR_ARG, "dpwa_board_unlink(%s): %s", name, strerror(errno));
    return DPWA_OK;
}

int dpwa_board_close(dpwa_board *b)
{
    if (!b) return DPWA_OK;
    // From here on peers see a refused connection.  Readers that marked a snapshot before
    // they could see that are waited for (bounded), so the slots outlive their pulls.
    store(&b->nodes[b->rank].closed, 1);
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < b->world; ++r) {
        const uint64_t *mark = &b->reading[(size_t)b->rank * b->world + r];
        while (r != b->rank && load(mark) != 0 && b->alive(r) &&
               std::chrono::steady_clock::now() - t0 < std::chrono::seconds(10))
            std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    if (b->dev_base) {
        int prev = 0;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(b->device);
        for (hipEvent_t ev : b->released)
            if (ev) {
                (void)hipEventSynchronize(ev);
                (void)hipEventDestroy(ev);
            }
        (void)hipHostUnregister(b->base);
        (void)hipSetDevice(prev);
    }
    munmap(b->base, b->bytes);
    delete b;
    return DPWA_OK;
}

int dpwa_board_register(dpwa_board *b, int device)
{
    if (!b) return set_error(DPWA_ERR_ARG, "dpwa_board_register: NULL board");
    if (b->dev_base) return DPWA_OK;
    int prev = 0;
    HIP_TRY(hipGetDevice(&prev));
    HIP_TRY(hipSetDevice(device));
    hipError_t e = hipHostRegister(b->base, b->bytes, hipHostRegisterMapped);
    void *d = nullptr;
    if (e == hipSuccess) e = hipHostGetDevicePointer(&d, b->base, 0);
    (void)hipSetDevice(prev);
    if (e != hipSuccess) return set_error(DPWA_ERR_HIP, "dpwa_board_register: %s", hipGetErrorString(e));
    b->dev_base = (char *)d;
    b->device = device;
    b->released.assign((size_t)b->world, nullptr);
    b->release_pending.assign((size_t)b->world, 0);
    return DPWA_OK;
}

// What a TxThread request to rank r would meet (conn.py:246-313): refused when the node is
// gone, an empty reply before its first publish, data otherwise.
int dpwa_board_status(dpwa_board *b, int r, int32_t *status)
{
    if (!b || r < 0 || r >= b->world || !status) return set_error(DPWA_ERR_ARG, "dpwa_board_status: bad arguments");
    if (!b->alive(r))
        *status = DPWA_PEER_DOWN;
    else
        *status = load(&b->nodes[r].version) == 0 ? DPWA_PEER_NO_STATE : DPWA_PEER_READY;
    return DPWA_OK;
}

int dpwa_board_read(dpwa_board *b, int r, uint64_t *version, uint64_t *reading_by_me, int32_t *alive)
{
    if (!b || r < 0 || r >= b->world) return set_error(DPWA_ERR_ARG, "dpwa_board_read: bad arguments");
    if (version) *version = load(&b->nodes[r].version);
    if (reading_by_me) *reading_by_me = load(&b->reading[(size_t)r * b->world + b->rank]);
    if (alive) *alive = b->alive(r) ? 1 : 0;
    return DPWA_OK;
}

// Reader side: a version of r's snapshot that r will not rewrite until we release it
// (0 = r has not published, or has closed).
int dpwa_board_acquire(dpwa_board *b, int r, uint64_t *version)
{
    if (!b || r < 0 || r >= b->world || r == b->rank || !version)
        return set_error(DPWA_ERR_ARG, "dpwa_board_acquire: bad arguments");
    uint64_t *mark = &b->reading[(size_t)r * b->world + b->rank];
    if (!b->release_pending.empty() && b->release_pending[r]) {
        // our previous mark on r is cleared by a store still queued on a stream: let it land
        // first, or it would wipe the mark set below
        HIP_TRY(hipEventSynchronize(b->released[r]));
        b->release_pending[r] = 0;
    }
    uint64_t v = load(&b->nodes[r].version);
    for (int tries = 0; tries < 1000000; ++tries) {
        if (v == 0) {
            store(mark, (uint64_t)0);
            *version = 0;
            return DPWA_OK;
        }
        store(mark, v);
        if (!b->alive(r)) {   // r closed after the pick: it drains only marks it can see
            store(mark, (uint64_t)0);
            *version = 0;
            return DPWA_OK;
        }
        const uint64_t again = load(&b->nodes[r].version);
        if (again == v) {
            *version = v;
            return DPWA_OK;
        }
        v = again;
    }
    store(mark, (uint64_t)0);
    return set_error(DPWA_ERR_STATE, "dpwa_board_acquire: rank %d publishes faster than it can be read", r);
}

// Clears our read mark on r once everything enqueued on `stream` so far is done (stream
// NULL + host != 0: right now, from the host).
int dpwa_board_release(dpwa_board *b, int r, dpwa_stream_t stream, int host)
{
    if (!b || r < 0 || r >= b->world) return set_error(DPWA_ERR_ARG, "dpwa_board_release: bad arguments");
    uint64_t *mark = &b->reading[(size_t)r * b->world + b->rank];
    if (host) {
        store(mark, (uint64_t)0);
        return DPWA_OK;
    }
    if (!b->dev_base) return set_error(DPWA_ERR_STATE, "dpwa_board_release: board not registered with a device");
    HIP_TRY(stream_store(b->dev(mark), 0, (hipStream_t)stream));
    if (!b->released[r]) {
        int prev = 0;
        HIP_TRY(hipGetDevice(&prev));
        HIP_TRY(hipSetDevice(b->device));
        const hipError_t e = hipEventCreateWithFlags(&b->released[r], hipEventDisableTiming);
        (void)hipSetDevice(prev);
        if (e != hipSuccess) return set_error(DPWA_ERR_HIP, "dpwa_board_release: %s", hipGetErrorString(e));
    }
    HIP_TRY(hipEventRecord(b->released[r], (hipStream_t)stream));
    b->release_pending[r] = 1;
    return DPWA_OK;
}

// Publisher side, before publish number `next`: our previous publish is out, and no live
// reader still holds the snapshot that `next` overwrites (next - 2).
int dpwa_board_publish_wait(dpwa_board *b, uint64_t next, int timeout_ms)
{
    if (!b || next == 0) return set_error(DPWA_ERR_ARG, "dpwa_board_publish_wait: bad arguments");
    const auto t0 = std::chrono::steady_clock::now();
    auto expired = [&]() {
        return timeout_ms >= 0 &&
               std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms);
    };
    // What is waited for is GPU progress (our advertise, peers' read releases), typically tens
    // of microseconds: spin on the CPU for the first 200 us (a sleep costs the kernel's ~50 us
    // timer slack), then back off to short sleeps.
    auto pause = [&]() {
        if (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(200))
            __builtin_ia32_pause();
        else
            std::this_thread::sleep_for(std::chrono::microseconds(20));
    };
    while (load(&b->nodes[b->rank].version) + 1 < next) {
        if (expired())
            return set_error(DPWA_ERR_STATE, "dpwa_board_publish_wait: publish %llu never completed",
                             (unsigned long long)(next - 1));
        pause();
    }
    if (next < 3) return DPWA_OK;
    for (int r = 0; r < b->world; ++r) {
        if (r == b->rank) continue;
        const uint64_t *mark = &b->reading[(size_t)b->rank * b->world + r];
        while (load(mark) == next - 2 && b->alive(r)) {
            if (expired())
                return set_error(DPWA_ERR_STATE, "dpwa_board_publish_wait: rank %d still reads snapshot %llu",
                                 r, (unsigned long long)(next - 2));
            pause();
        }
    }
    return DPWA_OK;
}

// Announce publish `version` once everything enqueued on `stream` so far is done (stream
// NULL + host != 0: right now).
int dpwa_board_advertise(dpwa_board *b, uint64_t version, dpwa_stream_t stream, int host)
{
    if (!b) return set_error(DPWA_ERR_ARG, "dpwa_board_advertise: NULL board");
    uint64_t *v = &b->nodes[b->rank].version;
    if (host) {
        store(v, version);
        return DPWA_OK;
    }
    if (!b->dev_base) return set_error(DPWA_ERR_STATE, "dpwa_board_advertise: board not registered with a device");
    HIP_TRY(stream_store(b->dev(v), version, (hipStream_t)stream));
    return DPWA_OK;
}

}  // extern "C"
