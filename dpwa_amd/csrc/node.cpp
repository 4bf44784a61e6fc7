// node.cpp -- one gossip node = DpwaConnection's per-round logic in native code.
//
// A node owns the scheduler (TxThread's peer choice + flow control + the Bernoulli gate,
// sched.cpp) and, once bound to a flat buffer, a learner (learner.cpp), and knows how to
// reach each peer.  update_send / update_wait(_average) run a whole half-round in one call
// so the host cost of a round is a few microseconds plus two kernel launches:
//   update_send          dpwa/dpwa.py:104-123  (+ the fetch of conn.py:277-315 when eager)
//   update_wait          dpwa/dpwa.py:125-156  (factor only; the lerp follows separately)
//   update_wait_average  dpwa/dpwa.py:125-156 + dpwa/adapters/pytorch.py:60-68 in one kernel
// Built only on the public C ABI of the learner and the scheduler.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "common.hpp"

namespace {

enum PeerKind { PEER_UNSET = 0, PEER_LOCAL = 1, PEER_REMOTE = 2 };

struct PeerRef {
    int kind = PEER_UNSET;
    dpwa_node *node = nullptr;   // PEER_LOCAL
    int fault = -1;              // forced DPWA_PEER_* status, -1 = none
};

}  // namespace

struct dpwa_node {
    dpwa_sched *sched = nullptr;
    dpwa_learner *learner = nullptr;
    dpwa_interp cfg{};
    std::vector<PeerRef> peers;
    std::vector<int32_t> status;
    std::vector<char> attached;    // learner-level attach done for local peers
    std::vector<dpwa_learner *> attached_to;
    bool fetching = false;
    bool fetch_started = false;
    int fetch_peer = -1;
    uint64_t fetch_version = 0;
    int last_attempts = 0;
    bool awaiting_lerp = false;    // update_wait (split) done, lerp not yet issued
    // free-running rounds (board.cpp): REMOTE peers are read through the board
    dpwa_board *board = nullptr;
    std::vector<int32_t> board_rank;
    int publish_timeout_ms = -1;
    // fetch timeout (conn.py:249, 304-309): the reply of a judged pull is reported when
    // update_wait polls it (reply_pending), as data or as a timeout
    int timeout_ms = -1;
    bool reply_pending = false;
    // how long a re-selected request waits for a free rescue lane (every lane still pulling) before
    // it is given up: DPWA_RESCUE_WAIT_MS, default 60 s
    int64_t rescue_wait_ms = 60000;
};

using namespace dpwa;

// TxThread's loop ends only on data, on "no peer" or when every peer is gone (conn.py:286-313);
// with every live peer answering empty it would spin for ever: bounded here.
constexpr int kMaxFetchAttempts = 100000;

static uint64_t learner_version(dpwa_learner *l)
{
    uint64_t v = 0;
    if (l) dpwa_learner_version(l, &v);
    return v;
}

// Slot the learner's resident parameters are in, -1 when it is not resident.
static int resident_slot(dpwa_learner *l)
{
    void *p = nullptr;
    int k = -1;
    if (l) dpwa_learner_resident_params(l, &p, &k);
    return k;
}

extern "C" {

int dpwa_node_create(dpwa_node **out, int n_peers, const uint32_t *seed_key, int key_len, double fetch_probability,
                     const dpwa_interp *cfg)
{
    if (!out || n_peers < 0 || !cfg) return set_error(DPWA_ERR_ARG, "dpwa_node_create: bad arguments");
    if (cfg->method < 0 || cfg->method > 2) return set_error(DPWA_ERR_ARG, "dpwa_node_create: unknown method");
    dpwa_node *n = new (std::nothrow) dpwa_node();
    if (!n) return set_error(DPWA_ERR_NOMEM, "dpwa_node_create: out of memory");
    int rc = dpwa_sched_create(&n->sched, n_peers, seed_key, key_len, fetch_probability);
    if (rc) {
        delete n;
        return rc;
    }
    n->cfg = *cfg;
    if (const char *w = getenv("DPWA_RESCUE_WAIT_MS")) n->rescue_wait_ms = std::max(0LL, atoll(w));
    n->peers.assign((size_t)n_peers, PeerRef());
    n->status.assign((size_t)(n_peers > 0 ? n_peers : 1), DPWA_PEER_DOWN);
    n->attached.assign((size_t)n_peers, 0);
    n->attached_to.assign((size_t)n_peers, nullptr);
    *out = n;
    return DPWA_OK;
}

int dpwa_node_destroy(dpwa_node *n)
{
    if (!n) return DPWA_OK;
    if (n->learner) dpwa_learner_destroy(n->learner);
    dpwa_sched_destroy(n->sched);
    delete n;
    return DPWA_OK;
}

int dpwa_node_bind(dpwa_node *n, int device, int64_t numel, int32_t dtype)
{
    if (!n) return set_error(DPWA_ERR_ARG, "dpwa_node_bind: NULL node");
    if (n->learner) return set_error(DPWA_ERR_STATE, "dpwa_node_bind: already bound");
    return dpwa_learner_create(&n->learner, device, numel, dtype, &n->cfg);
}

int dpwa_node_handles(dpwa_node *n, dpwa_learner **learner, dpwa_sched **sched)
{
    if (!n) return set_error(DPWA_ERR_ARG, "dpwa_node_handles: NULL node");
    if (learner) *learner = n->learner;
    if (sched) *sched = n->sched;
    return DPWA_OK;
}

// A LOCAL peer may be the node itself: a YAML node entry at this node's own host:port is its own
// RxThread, which the reference's TxThread dials like any other (conn.py:246-251, 98-110), so the
// node averages with the snapshot it published (configs[1]'s self-peer).
int dpwa_node_set_peer(dpwa_node *n, int peer, int kind, dpwa_node *local)
{
    if (!n || peer < 0 || (size_t)peer >= n->peers.size() || kind < PEER_UNSET || kind > PEER_REMOTE ||
        (kind == PEER_LOCAL && !local))
        return set_error(DPWA_ERR_ARG, "dpwa_node_set_peer: bad arguments");
    PeerRef &p = n->peers[peer];
    p.kind = kind;
    p.node = kind == PEER_LOCAL ? local : nullptr;
    n->attached[peer] = 0;
    n->attached_to[peer] = nullptr;
    return DPWA_OK;
}

int dpwa_node_set_board(dpwa_node *n, dpwa_board *board, const int32_t *peer_ranks, int publish_timeout_ms)
{
    if (!n || (board && !peer_ranks)) return set_error(DPWA_ERR_ARG, "dpwa_node_set_board: bad arguments");
    n->board = board;
    n->board_rank.assign(peer_ranks && board ? peer_ranks : (const int32_t *)nullptr,
                         peer_ranks && board ? peer_ranks + n->peers.size() : (const int32_t *)nullptr);
    n->publish_timeout_ms = publish_timeout_ms;
    return DPWA_OK;
}

int dpwa_node_set_fault(dpwa_node *n, int peer, int status)
{
    if (!n || peer < 0 || (size_t)peer >= n->peers.size() || status < -1 || status > DPWA_PEER_DEAD)
        return set_error(DPWA_ERR_ARG, "dpwa_node_set_fault: bad arguments");
    n->peers[peer].fault = status;
    return DPWA_OK;
}

// What a TxThread request to this peer would meet right now (conn.py:246-313 outcomes).
static int32_t peer_status(const dpwa_node *n, size_t k)
{
    const PeerRef &p = n->peers[k];
    if (p.fault >= 0) return p.fault;
    if (p.kind == PEER_REMOTE && n->board) {             // free-running: what the board says
        int32_t st = DPWA_PEER_DOWN;
        return dpwa_board_status(n->board, n->board_rank[k], &st) == DPWA_OK ? st : DPWA_PEER_DOWN;
    }
    if (p.kind == PEER_REMOTE) return DPWA_PEER_READY;   // lock-step: published this round
    if (p.kind != PEER_LOCAL) return DPWA_PEER_DOWN;     // not listening: ConnectionRefused
    if (!p.node->learner || learner_version(p.node->learner) == 0) return DPWA_PEER_NO_STATE;
    return DPWA_PEER_READY;
}

static int64_t now_ms()
{
    return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// Moves peer `peer`'s snapshot towards this node's learner (or, PICK_ONLY, just records the
// pick for a transport that moves the bytes itself).  board_version: the version the board
// handed out (free-running), else unused.  rescue: into the rescue buffer on its own stream.
static int issue_pull(dpwa_node *n, int peer, uint64_t board_version, int flags, dpwa_stream_t stream, bool rescue)
{
    PeerRef &p = n->peers[peer];
    const bool via_board = n->board && p.kind == PEER_REMOTE;
    uint64_t version;
    int fflags;
    int rc;
    if (via_board) {
        // a completed publish (the board advertised it): the pull needs no ordering after `stream`
        version = board_version;
        fflags = DPWA_FETCH_PUBLISHED;
    } else if (p.kind == PEER_LOCAL) {
        dpwa_learner *pl = p.node->learner;
        if (n->attached_to[peer] != pl) {
            if ((rc = dpwa_learner_attach_local(n->learner, peer, pl))) return rc;
            n->attached_to[peer] = pl;
        }
        version = learner_version(pl);
        fflags = (flags & DPWA_FLAG_ZERO_COPY) ? DPWA_FETCH_ZERO_COPY : 0;
    } else {
        version = learner_version(n->learner);   // lock-step: every node publishes once per round
        fflags = 0;
    }
    if (flags & DPWA_FLAG_PICK_ONLY) {   // the transport moves the bytes (relay)
        n->fetch_peer = peer;
        n->fetch_version = version;
        return DPWA_OK;
    }
    if (rescue) fflags = (fflags & DPWA_FETCH_PUBLISHED) | DPWA_FETCH_RESCUE;
    if ((rc = dpwa_learner_fetch(n->learner, peer, version, fflags, stream))) {
        if (via_board) dpwa_board_release(n->board, n->board_rank[peer], nullptr, 1);
        return rc;
    }
    if (via_board) {   // our read mark is cleared once the pull has landed
        dpwa_stream_t fs = nullptr;
        if ((rc = dpwa_learner_fetch_stream(n->learner, &fs)) ||
            (rc = dpwa_board_release(n->board, n->board_rank[peer], fs, 0)))
            return rc;
    }
    n->fetch_peer = peer;
    n->fetch_version = version;
    return DPWA_OK;
}

// Host poll of a rescue pull (the abnormal path only): until it lands or timeout_ms after it was
// issued, as the reference's receive blocks up to its socket timeout.
static int wait_pull(dpwa_node *n, int *state)
{
    for (;;) {
        int rc = dpwa_learner_fetch_state(n->learner, n->timeout_ms, state);
        if (rc || *state != DPWA_FETCH_IN_FLIGHT) return rc;
        std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

// TxThread.run's loop for one queue item (conn.py:277-315): pick (conn.py:224-240), lazy
// connect (conn.py:245-260), request, reply.  The reply of a judged pull (a copying pull from a
// local peer or through the board, with a timeout set) is not reported here but when update_wait
// polls it (judge_pending); after a timeout the loop runs again with rescue = true, each
// re-selected pull going to the rescue buffer and being polled to its deadline on the host.
// Free-running rounds read REMOTE peers through the board: a READY peer's snapshot is acquired
// *before* the outcome is reported, so a peer that closed between its status read and the acquire
// counts as gone -- refused when not yet connected (conn.py:253-256), an error when it was
// (conn.py:311-313) -- and never as a reply with data.
static int fetch_loop(dpwa_node *n, int flags, dpwa_stream_t stream, bool rescue)
{
    TraceRange tr(rescue ? "dpwa.fetch_loop.rescue" : "dpwa.fetch_loop");
    int attempts = 0;
    int rc = DPWA_OK;
    while (attempts < kMaxFetchAttempts) {
        int peer, connected, done = 0, data = 0;
        if ((rc = dpwa_sched_pick(n->sched, &peer, &connected))) break;
        if (peer < 0) break;
        attempts++;
        const PeerRef &p = n->peers[peer];
        const bool via_board = n->board && p.kind == PEER_REMOTE;
        int32_t st = n->status[peer];
        uint64_t v = 0;
        if (st == DPWA_PEER_READY && via_board) {
            if (flags & DPWA_FLAG_PICK_ONLY) {
                rc = set_error(DPWA_ERR_STATE, "the relay transport needs lock-step rounds, not a board");
                break;
            }
            if ((rc = dpwa_board_acquire(n->board, n->board_rank[peer], &v))) break;
            if (v == 0) st = DPWA_PEER_DOWN;      // closed since its status was read
        }
        if (!connected) {
            int c = DPWA_CONNECT_OK;
            if (st == DPWA_PEER_DOWN) c = DPWA_CONNECT_REFUSED;
            else if (st == DPWA_PEER_DEAD) c = DPWA_CONNECT_ERROR;
            if ((rc = dpwa_sched_report(n->sched, peer, c, &done, &data))) break;
            if (done) break;
        }
        if (st == DPWA_PEER_READY) {
            const bool judged = n->timeout_ms >= 0 && !(flags & DPWA_FLAG_PICK_ONLY) &&
                                (p.kind == PEER_LOCAL || via_board);
            int state = DPWA_FETCH_LANDED;
            if (rescue && judged) {
                // a rescue lane must be free: its last pull landed, or another lane can be made
                // (up to 8, memory permitting).  With every lane's pull still in flight it is this
                // learner's own transport that is held up, not the peer: the request waits for a
                // lane to land before it goes out, unjudged -- the reference's timeout bounds only
                // the reply (conn.py:249) -- and TxThread's loop goes on (conn.py:286-313).  Only a
                // transport stuck for rescue_wait_ms gives the request up as a timeout and ends
                // the round without data.
                int free_ = 1;
                const int64_t t0 = now_ms();
                while ((rc = dpwa_learner_rescue_free(n->learner, &free_)) == DPWA_OK && !free_ &&
                       now_ms() - t0 < n->rescue_wait_ms)
                    std::this_thread::sleep_for(std::chrono::microseconds(50));
                if (rc) break;
                if (!free_) {
                    if (via_board) dpwa_board_release(n->board, n->board_rank[peer], nullptr, 1);
                    rc = dpwa_sched_report(n->sched, peer, DPWA_REPLY_TIMEOUT, &done, &data);
                    break;
                }
            }
            if ((rc = issue_pull(n, peer, v, flags, stream, rescue && judged))) break;
            if (judged && !rescue) {
                n->reply_pending = true;         // judged when update_wait polls it
                break;
            }
            if (judged && (rc = wait_pull(n, &state))) break;
            if (state == DPWA_FETCH_TIMED_OUT) {
                dpwa_learner_cancel(n->learner);
                n->fetch_peer = -1;
                if ((rc = dpwa_sched_report(n->sched, peer, DPWA_REPLY_TIMEOUT, &done, &data))) break;
                continue;
            }
            if ((rc = dpwa_sched_report(n->sched, peer, DPWA_REPLY_PAYLOAD, &done, &data))) break;
            break;
        }
        int r;
        switch (st) {
        case DPWA_PEER_NO_STATE: r = DPWA_REPLY_EMPTY; break;
        case DPWA_PEER_SLOW: r = DPWA_REPLY_TIMEOUT; break;
        default: r = DPWA_REPLY_ERROR; break;   // DOWN while connected (reset) or DEAD
        }
        if ((rc = dpwa_sched_report(n->sched, peer, r, &done, &data))) break;
        if (done) break;
    }
    n->last_attempts += attempts;
    return rc;
}

static void refresh_status(dpwa_node *n)
{
    for (size_t k = 0; k < n->peers.size(); ++k) n->status[k] = peer_status(n, k);
}

static int start_fetch(dpwa_node *n, int flags, dpwa_stream_t stream)
{
    n->fetch_started = true;
    n->fetch_peer = -1;
    n->reply_pending = false;
    n->last_attempts = 0;
    refresh_status(n);
    return fetch_loop(n, flags, stream, false);
}

// update_wait's verdict on a judged pull (conn.py:298-309): landed, or still within its
// timeout (then the device waits for it) -> the reply with data; else a socket timeout and the
// loop picks again.
static int judge_pending(dpwa_node *n, int flags, dpwa_stream_t stream)
{
    n->reply_pending = false;
    int state = DPWA_FETCH_LANDED, done = 0, data = 0;
    int rc = dpwa_learner_fetch_state(n->learner, n->timeout_ms, &state);
    if (rc) return rc;
    const int peer = n->fetch_peer;
    if (state != DPWA_FETCH_TIMED_OUT) return dpwa_sched_report(n->sched, peer, DPWA_REPLY_PAYLOAD, &done, &data);
    dpwa_learner_cancel(n->learner);          // the stalled pull still lands, into a buffer nobody reads
    n->fetch_peer = -1;
    if ((rc = dpwa_sched_report(n->sched, peer, DPWA_REPLY_TIMEOUT, &done, &data))) return rc;
    refresh_status(n);
    return fetch_loop(n, flags, stream, true);
}

int dpwa_node_set_timeout(dpwa_node *n, int timeout_ms)
{
    if (!n) return set_error(DPWA_ERR_ARG, "dpwa_node_set_timeout: NULL node");
    n->timeout_ms = timeout_ms < 0 ? -1 : timeout_ms;
    return DPWA_OK;
}

int dpwa_node_publish(dpwa_node *n, const void *flat, double loss, const double *loss_dev, int flags,
                      dpwa_stream_t stream)
{
    if (!n || !n->learner) return set_error(DPWA_ERR_STATE, "dpwa_node_publish: node not bound");
    TraceRange tr("dpwa.publish");
    if (n->awaiting_lerp) {   // update_wait() was not followed by a lerp: abandon that fetch
        dpwa_learner_cancel(n->learner);
        n->awaiting_lerp = false;
    }
    if (n->reply_pending) {   // update_wait never came: the reply arrived meanwhile (TxThread ran on)
        int done = 0, data = 0;
        n->reply_pending = false;
        int rc = dpwa_sched_report(n->sched, n->fetch_peer, DPWA_REPLY_PAYLOAD, &done, &data);
        if (rc) return rc;
        dpwa_learner_cancel(n->learner);
    }
    n->fetch_started = false;
    n->fetch_peer = -1;
    if (n->board) {   // free-running: wait out readers of the slot we rewrite, then announce
        // (after a write-through average the wait already happened there and returns at once)
        const uint64_t next = learner_version(n->learner) + 1;
        int rc = dpwa_board_publish_wait(n->board, next, n->publish_timeout_ms);
        if (!rc)
            rc = (flags & DPWA_FLAG_REUSE_SNAPSHOT) ? dpwa_learner_publish_reuse(n->learner, flat, loss, loss_dev, stream)
                                                     : dpwa_learner_publish(n->learner, flat, loss, loss_dev, stream);
        if (!rc) rc = dpwa_board_advertise(n->board, next, stream, 0);
        return rc;
    }
    if (flags & DPWA_FLAG_REUSE_SNAPSHOT) return dpwa_learner_publish_reuse(n->learner, flat, loss, loss_dev, stream);
    return dpwa_learner_publish(n->learner, flat, loss, loss_dev, stream);
}

int dpwa_node_gate(dpwa_node *n, int flags, dpwa_stream_t stream, int *fetching)
{
    if (!n || !n->learner || !fetching) return set_error(DPWA_ERR_STATE, "dpwa_node_gate: node not bound");
    int f = 0;
    int rc = dpwa_sched_bernoulli(n->sched, &f);   // dpwa.py:118
    if (rc) return rc;
    n->fetching = f != 0;
    *fetching = f;
    if (f && (flags & DPWA_FLAG_EAGER)) return start_fetch(n, flags, stream);
    return DPWA_OK;
}

int dpwa_node_update_send(dpwa_node *n, const void *flat, double loss, const double *loss_dev, int flags,
                          dpwa_stream_t stream, int *fetching)
{
    TraceRange tr("dpwa.update_send");
    int rc = dpwa_node_publish(n, flat, loss, loss_dev, flags, stream);
    if (rc) return rc;
    return dpwa_node_gate(n, flags, stream, fetching);
}

int dpwa_node_start_fetch(dpwa_node *n, int flags, dpwa_stream_t stream)
{
    if (!n || !n->learner) return set_error(DPWA_ERR_STATE, "dpwa_node_start_fetch: node not bound");
    if (!n->fetching || n->fetch_started) return DPWA_OK;
    return start_fetch(n, flags, stream);
}

// dpwa.py:130-137: *peer = -1 means (None, 0).
static int finish_fetch(dpwa_node *n, int flags, dpwa_stream_t stream, int *peer)
{
    *peer = -1;
    if (!n->fetching) return DPWA_OK;
    n->fetching = false;
    if (!n->fetch_started) {
        int rc = start_fetch(n, flags, stream);
        if (rc) return rc;
    }
    if (n->reply_pending) {
        int rc = judge_pending(n, flags, stream);
        if (rc) return rc;
    }
    *peer = n->fetch_peer;
    return DPWA_OK;
}

int dpwa_node_update_wait(dpwa_node *n, double loss, const double *loss_dev, int flags, dpwa_stream_t stream,
                          int *peer)
{
    if (!n || !n->learner || !peer) return set_error(DPWA_ERR_STATE, "dpwa_node_update_wait: node not bound");
    TraceRange tr("dpwa.update_wait");
    if (resident_slot(n->learner) >= 0)
        return set_error(DPWA_ERR_STATE, "dpwa_node_update_wait: a resident node averages with update_wait_average");
    int rc = finish_fetch(n, flags, stream, peer);
    if (rc || *peer < 0) return rc;
    if ((rc = dpwa_learner_factor(n->learner, loss, loss_dev, stream))) return rc;
    n->awaiting_lerp = true;
    return DPWA_OK;
}

int dpwa_node_lerp(dpwa_node *n, void *flat, dpwa_stream_t stream)
{
    if (!n || !n->learner) return set_error(DPWA_ERR_STATE, "dpwa_node_lerp: node not bound");
    int rc = dpwa_learner_lerp(n->learner, flat, stream);
    if (!rc) n->awaiting_lerp = false;
    return rc;
}

// A resident node's round without an average: its parameters leave the published slot (one
// copy into the next publish's slot, whose readers the board must have released first).
static int relocate(dpwa_node *n, dpwa_stream_t stream)
{
    const int k = resident_slot(n->learner);
    const uint64_t v = learner_version(n->learner);
    if (k < 0 || (uint64_t)k == v % 2) return DPWA_OK;
    if (n->board) {
        const int rc = dpwa_board_publish_wait(n->board, v + 1, n->publish_timeout_ms);
        if (rc) return rc;
    }
    return dpwa_learner_relocate(n->learner, stream);
}

int dpwa_node_set_resident(dpwa_node *n, const void *init, dpwa_stream_t stream)
{
    if (!n || !n->learner) return set_error(DPWA_ERR_STATE, "dpwa_node_set_resident: node not bound");
    return dpwa_learner_set_resident(n->learner, init, stream);
}

int dpwa_node_update_wait_average(dpwa_node *n, void *flat, double loss, const double *loss_dev, int flags,
                                  dpwa_stream_t stream, int *peer)
{
    if (!n || !n->learner || !peer) return set_error(DPWA_ERR_STATE, "dpwa_node_update_wait_average: node not bound");
    TraceRange tr("dpwa.update_wait_average");
    int rc = finish_fetch(n, flags, stream, peer);
    if (rc) return rc;
    const bool resident = resident_slot(n->learner) >= 0;
    if (*peer < 0) return resident ? relocate(n, stream) : DPWA_OK;
    if ((flags & DPWA_FLAG_WRITE_THROUGH) || resident) {
        if (n->board) {
            // the average rewrites the slot of the NEXT publish (that of publish v-1): the
            // board's publish rule -- our publish v is visible, no live reader holds v-1 --
            // must hold before the kernel is enqueued, not only before the next update_send
            if ((rc = dpwa_board_publish_wait(n->board, learner_version(n->learner) + 1, n->publish_timeout_ms)))
                return rc;
        }
        return dpwa_learner_average_through(n->learner, flat, loss, loss_dev, stream);
    }
    return dpwa_learner_average(n->learner, flat, loss, loss_dev, stream);
}

int dpwa_node_update_wait_average_many(dpwa_node *const *nodes, void *const *flats, const double *loss,
                                       const double *const *loss_dev, int count, int flags, dpwa_stream_t stream,
                                       int *peers)
{
    if (count < 0 || (count > 0 && (!nodes || !flats || !loss || !peers)))
        return set_error(DPWA_ERR_ARG, "dpwa_node_update_wait_average_many: bad arguments");
    TraceRange tr("dpwa.update_wait_average_many");
    std::vector<dpwa_learner *> ls;
    std::vector<void *> fl;
    std::vector<double> lo;
    std::vector<const double *> ld;
    std::vector<int> wt;
    const bool through = (flags & DPWA_FLAG_WRITE_THROUGH) != 0;
    for (int i = 0; i < count; ++i) peers[i] = -1;
    for (int i = 0; i < count; ++i) {
        dpwa_node *n = nodes[i];
        if (!n || !n->learner) return set_error(DPWA_ERR_STATE, "dpwa_node_update_wait_average_many: node %d not bound", i);
        int rc = finish_fetch(n, flags, stream, &peers[i]);   // dpwa.py:130-137, node by node
        if (rc) return rc;
        const bool resident = resident_slot(n->learner) >= 0;
        if (peers[i] < 0) {
            if (resident && (rc = relocate(n, stream))) return rc;
            continue;
        }
        if ((through || resident) && n->board &&
            (rc = dpwa_board_publish_wait(n->board, learner_version(n->learner) + 1, n->publish_timeout_ms)))
            return rc;
        ls.push_back(n->learner);
        fl.push_back(flats[i]);
        lo.push_back(loss[i]);
        ld.push_back(loss_dev ? loss_dev[i] : nullptr);
        wt.push_back(through || resident ? 1 : 0);
    }
    if (ls.empty()) return DPWA_OK;
    return dpwa_learner_average_many(ls.data(), fl.data(), lo.data(), ld.data(), wt.data(), (int)ls.size(), stream);
}

int dpwa_node_info(const dpwa_node *n, int *fetching, int *fetch_peer, uint64_t *fetch_version, int *last_attempts)
{
    if (!n) return set_error(DPWA_ERR_ARG, "dpwa_node_info: NULL node");
    if (fetching) *fetching = n->fetching ? 1 : 0;
    if (fetch_peer) *fetch_peer = n->fetch_peer;
    if (fetch_version) *fetch_version = n->fetch_version;
    if (last_attempts) *last_attempts = n->last_attempts;
    return DPWA_OK;
}

}  // extern "C"
