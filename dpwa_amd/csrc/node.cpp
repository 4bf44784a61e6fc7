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
#include <cstring>
#include <new>
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

int dpwa_node_set_peer(dpwa_node *n, int peer, int kind, dpwa_node *local)
{
    if (!n || peer < 0 || (size_t)peer >= n->peers.size() || kind < PEER_UNSET || kind > PEER_REMOTE ||
        (kind == PEER_LOCAL && (!local || local == n)))
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

// Free-running rounds: TxThread's loop (conn.py:277-315, as dpwa_sched_fetch runs it) with
// the board standing in for the peers' RxThreads.  A READY peer's snapshot is acquired
// *before* the outcome is reported, so a peer that closed between its status read and the
// acquire counts as gone -- refused when not yet connected (conn.py:253-256), an error when
// it was (conn.py:311-313) -- and never as a reply with data.
static int board_fetch(dpwa_node *n, int flags, int *peer_out, uint64_t *version_out, int *attempts_out)
{
    *peer_out = -1;
    *version_out = 0;
    int attempts = 0;
    while (attempts < kMaxFetchAttempts) {
        int peer, connected, done = 0, data = 0;
        int rc = dpwa_sched_pick(n->sched, &peer, &connected);
        if (rc) return rc;
        if (peer < 0) break;
        attempts++;
        int32_t st = n->status[peer];
        uint64_t v = 0;
        if (st == DPWA_PEER_READY && n->peers[peer].kind == PEER_REMOTE) {
            if (flags & DPWA_FLAG_PICK_ONLY)
                return set_error(DPWA_ERR_STATE, "the relay transport needs lock-step rounds, not a board");
            if ((rc = dpwa_board_acquire(n->board, n->board_rank[peer], &v))) return rc;
            if (v == 0) st = DPWA_PEER_DOWN;      // closed since its status was read
        }
        if (!connected) {
            int c = DPWA_CONNECT_OK;
            if (st == DPWA_PEER_DOWN) c = DPWA_CONNECT_REFUSED;
            else if (st == DPWA_PEER_DEAD) c = DPWA_CONNECT_ERROR;
            if ((rc = dpwa_sched_report(n->sched, peer, c, &done, &data))) return rc;
            if (done) break;
        }
        int r;
        switch (st) {
        case DPWA_PEER_READY: r = DPWA_REPLY_PAYLOAD; break;
        case DPWA_PEER_NO_STATE: r = DPWA_REPLY_EMPTY; break;
        case DPWA_PEER_SLOW: r = DPWA_REPLY_TIMEOUT; break;
        default: r = DPWA_REPLY_ERROR; break;
        }
        if ((rc = dpwa_sched_report(n->sched, peer, r, &done, &data))) return rc;
        if (data) {
            *peer_out = peer;
            *version_out = v;
            break;
        }
        if (done) break;
    }
    *attempts_out = attempts;
    return DPWA_OK;
}

static int start_fetch(dpwa_node *n, int flags, dpwa_stream_t stream)
{
    int zero_copy = (flags & DPWA_FLAG_ZERO_COPY) ? 1 : 0;
    n->fetch_started = true;
    n->fetch_peer = -1;
    for (size_t k = 0; k < n->peers.size(); ++k) n->status[k] = peer_status(n, k);
    int peer = -1, attempts = 0;
    int rc;
    if (n->board) {
        // free-running: the newest complete publish, held against rewrite until our pull lands
        uint64_t version = 0;
        if ((rc = board_fetch(n, flags, &peer, &version, &attempts))) return rc;
        n->last_attempts = attempts;
        if (peer < 0) return DPWA_OK;
        const int r = n->board_rank[peer];
        // a completed publish (the board advertised it): the pull needs no ordering after `stream`
        if ((rc = dpwa_learner_fetch(n->learner, peer, version, DPWA_FETCH_PUBLISHED, stream))) {
            dpwa_board_release(n->board, r, nullptr, 1);
            return rc;
        }
        dpwa_stream_t side = nullptr;
        if ((rc = dpwa_learner_side_stream(n->learner, &side)) ||
            (rc = dpwa_board_release(n->board, r, side, 0)))
            return rc;
        n->fetch_peer = peer;
        n->fetch_version = version;
        return DPWA_OK;
    }
    if ((rc = dpwa_sched_fetch(n->sched, n->status.data(), kMaxFetchAttempts, &peer, &attempts))) return rc;
    n->last_attempts = attempts;
    if (peer < 0) return DPWA_OK;
    PeerRef &p = n->peers[peer];
    uint64_t version;
    if (p.kind == PEER_LOCAL) {
        dpwa_learner *pl = p.node->learner;
        if (n->attached_to[peer] != pl) {
            if ((rc = dpwa_learner_attach_local(n->learner, peer, pl))) return rc;
            n->attached_to[peer] = pl;
        }
        version = learner_version(pl);
    } else {
        version = learner_version(n->learner);   // lock-step: every node publishes once per round
        zero_copy = 0;
    }
    if (flags & DPWA_FLAG_PICK_ONLY) {   // the transport moves the bytes (relay)
        n->fetch_peer = peer;
        n->fetch_version = version;
        return DPWA_OK;
    }
    if ((rc = dpwa_learner_fetch(n->learner, peer, version, zero_copy, stream))) return rc;
    n->fetch_peer = peer;
    n->fetch_version = version;
    return DPWA_OK;
}

int dpwa_node_publish(dpwa_node *n, const void *flat, double loss, const double *loss_dev, int flags,
                      dpwa_stream_t stream)
{
    if (!n || !n->learner) return set_error(DPWA_ERR_STATE, "dpwa_node_publish: node not bound");
    if (n->awaiting_lerp) {   // update_wait() was not followed by a lerp: abandon that fetch
        dpwa_learner_cancel(n->learner);
        n->awaiting_lerp = false;
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
    *peer = n->fetch_peer;
    return DPWA_OK;
}

int dpwa_node_update_wait(dpwa_node *n, double loss, const double *loss_dev, int flags, dpwa_stream_t stream,
                          int *peer)
{
    if (!n || !n->learner || !peer) return set_error(DPWA_ERR_STATE, "dpwa_node_update_wait: node not bound");
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

int dpwa_node_update_wait_average(dpwa_node *n, void *flat, double loss, const double *loss_dev, int flags,
                                  dpwa_stream_t stream, int *peer)
{
    if (!n || !n->learner || !peer) return set_error(DPWA_ERR_STATE, "dpwa_node_update_wait_average: node not bound");
    int rc = finish_fetch(n, flags, stream, peer);
    if (rc || *peer < 0) return rc;
    if (flags & DPWA_FLAG_WRITE_THROUGH) {
        if (n->board) {
            // the average rewrites the slot of the NEXT publish (that of publish v-1): the
            // board's publish rule -- our publish v is visible, no live reader holds v-1 --
            // must hold before the kernel is enqueued, not only before the next update_send
            const int rc = dpwa_board_publish_wait(n->board, learner_version(n->learner) + 1, n->publish_timeout_ms);
            if (rc) return rc;
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
        if (peers[i] < 0) continue;
        if (through && n->board &&
            (rc = dpwa_board_publish_wait(n->board, learner_version(n->learner) + 1, n->publish_timeout_ms)))
            return rc;
        ls.push_back(n->learner);
        fl.push_back(flats[i]);
        lo.push_back(loss[i]);
        ld.push_back(loss_dev ? loss_dev[i] : nullptr);
        wt.push_back(through ? 1 : 0);
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
