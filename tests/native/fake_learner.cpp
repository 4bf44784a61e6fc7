// fake_learner.cpp -- TEST INFRASTRUCTURE: a host-only stand-in for the learner runtime
// (dpwa_amd/csrc/learner.cpp) and the gossip board, so node.cpp's per-round logic -- TxThread's
// fetch loop (conn.py:277-315) with its timeout judging and rescue lanes -- can be built with g++
// and the sanitizers, and driven from a CPU test against the oracle policy
// (tests/test_node_host.py).  Nothing here touches a GPU: a "pull" is a record; whether it
// stalls is scripted per learner (fake_stall): a stalled pull never lands, so update_wait judges
// it timed out, and a stalled rescue pull keeps its lane taken until fake_land_all() -- or, with
// every lane taken, until the node has polled for a free lane `land_after` times (fake_lanes; the
// lane cap there also stands in for a lane allocation that fails).
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/dpwa_hip.h"

namespace dpwa {

static thread_local std::string g_last_error;

int set_error(int code, const char *fmt, ...)
{
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

}  // namespace dpwa

using dpwa::set_error;

namespace {
constexpr int kMaxLanes = 8;   // as learner.cpp kMaxRescueLanes
}

struct dpwa_learner {
    int64_t n = 0;
    uint64_t version = 0;
    int stall_next = 0;          // the next `stall_next` pulls issued stall
    bool have_fetch = false;
    bool fetch_stalled = false;
    int lanes = 0;               // rescue lanes allocated
    int lanes_stalled = 0;       // of them, holding a stalled pull
    int cap = kMaxLanes;         // lanes that can be made (a lower cap: the next allocation fails)
    int land_after = -1;         // with every lane stalled: one lands after this many polls (-1 never)
    int polls = 0;               // rescue_free polls that found no lane since the last landing
    int peer = -1;
    uint64_t peer_version = 0;
    int pulls = 0, rescue_pulls = 0, averages = 0, relocations = 0;
};

extern "C" {

const char *dpwa_last_error(void) { return dpwa::g_last_error.c_str(); }

// -- test controls -------------------------------------------------------------------------
int fake_stall(dpwa_learner *l, int n)
{
    if (!l || n < 0) return DPWA_ERR_ARG;
    l->stall_next = n;
    return DPWA_OK;
}

int fake_land_all(dpwa_learner *l)      // every stalled pull lands (the end of a round)
{
    if (!l) return DPWA_ERR_ARG;
    l->lanes_stalled = 0;
    l->fetch_stalled = false;
    return DPWA_OK;
}

int fake_lanes(dpwa_learner *l, int cap, int land_after)   // lane cap; polls until a stalled lane lands
{
    if (!l || cap < 0 || cap > kMaxLanes) return DPWA_ERR_ARG;
    l->cap = cap < l->lanes ? l->lanes : cap;
    l->land_after = land_after;
    l->polls = 0;
    return DPWA_OK;
}

int fake_counts(dpwa_learner *l, int *out)   // pulls, rescue pulls, lanes, averages, relocations
{
    if (!l || !out) return DPWA_ERR_ARG;
    out[0] = l->pulls;
    out[1] = l->rescue_pulls;
    out[2] = l->lanes;
    out[3] = l->averages;
    out[4] = l->relocations;
    return DPWA_OK;
}

// -- the learner ABI node.cpp uses -----------------------------------------------------------
int dpwa_learner_create(dpwa_learner **out, int, int64_t n, int32_t dtype, const dpwa_interp *)
{
    if (!out || n < 0 || (dtype != DPWA_F32 && dtype != DPWA_BF16)) return set_error(DPWA_ERR_ARG, "create");
    *out = new dpwa_learner();
    (*out)->n = n;
    return DPWA_OK;
}

int dpwa_learner_destroy(dpwa_learner *l)
{
    delete l;
    return DPWA_OK;
}

int dpwa_learner_version(const dpwa_learner *l, uint64_t *v)
{
    if (!l || !v) return set_error(DPWA_ERR_ARG, "version");
    *v = l->version;
    return DPWA_OK;
}

int dpwa_learner_resident_params(dpwa_learner *l, void **params, int *slot)
{
    if (!l || !params) return set_error(DPWA_ERR_ARG, "resident_params");
    *params = nullptr;
    if (slot) *slot = -1;
    return DPWA_OK;
}

int dpwa_learner_publish(dpwa_learner *l, const void *, double, const double *, dpwa_stream_t)
{
    if (!l) return set_error(DPWA_ERR_ARG, "publish");
    l->version++;
    return DPWA_OK;
}

int dpwa_learner_publish_reuse(dpwa_learner *l, const void *f, double loss, const double *d, dpwa_stream_t s)
{
    return dpwa_learner_publish(l, f, loss, d, s);
}

int dpwa_learner_attach_local(dpwa_learner *l, int, dpwa_learner *peer)
{
    if (!l || !peer || peer == l) return set_error(DPWA_ERR_ARG, "attach_local");
    return DPWA_OK;
}

int dpwa_learner_fetch(dpwa_learner *l, int peer_id, uint64_t peer_version, int flags, dpwa_stream_t)
{
    if (!l) return set_error(DPWA_ERR_ARG, "fetch");
    if (peer_version == 0) return set_error(DPWA_ERR_STATE, "fetch: peer %d has not published", peer_id);
    const bool stalled = l->stall_next > 0;
    if (stalled) l->stall_next--;
    if (flags & DPWA_FETCH_RESCUE) {
        // as learner.cpp: rescue_free made a lane when none was free, so one is free here
        if (l->lanes_stalled >= l->lanes) return set_error(DPWA_ERR_STATE, "fetch: no free rescue lane");
        if (stalled) l->lanes_stalled++;
        l->rescue_pulls++;
    }
    l->pulls++;
    l->have_fetch = true;
    l->fetch_stalled = stalled;
    l->peer = peer_id;
    l->peer_version = peer_version;
    return DPWA_OK;
}

int dpwa_learner_fetch_state(dpwa_learner *l, int64_t, int *state)
{
    if (!l || !state) return set_error(DPWA_ERR_ARG, "fetch_state");
    *state = l->have_fetch && l->fetch_stalled ? DPWA_FETCH_TIMED_OUT : DPWA_FETCH_LANDED;
    return DPWA_OK;
}

int dpwa_learner_rescue_free(dpwa_learner *l, int *free_out)
{
    if (!l || !free_out) return set_error(DPWA_ERR_ARG, "rescue_free");
    *free_out = 1;
    if (l->lanes_stalled < l->lanes) return DPWA_OK;          // a lane's pull landed
    if (l->lanes < l->cap) {                                   // make one (learner.cpp rescue_lane)
        l->lanes++;
        return DPWA_OK;
    }
    // every lane still pulling: one lands after `land_after` polls (a transport that was held up),
    // or never (a stuck one: the node gives up after DPWA_RESCUE_WAIT_MS)
    if (l->land_after >= 0 && ++l->polls > l->land_after) {
        l->lanes_stalled--;
        l->polls = 0;
        return DPWA_OK;
    }
    *free_out = 0;
    return DPWA_OK;
}

int dpwa_learner_fetch_stream(dpwa_learner *l, dpwa_stream_t *s)
{
    if (!l || !s) return set_error(DPWA_ERR_ARG, "fetch_stream");
    *s = nullptr;
    return DPWA_OK;
}

int dpwa_learner_cancel(dpwa_learner *l)
{
    if (!l) return set_error(DPWA_ERR_ARG, "cancel");
    l->have_fetch = false;
    return DPWA_OK;
}

static int averaged(dpwa_learner *l)
{
    if (!l) return set_error(DPWA_ERR_ARG, "average");
    if (!l->have_fetch) return set_error(DPWA_ERR_STATE, "average: no fetch in flight");
    l->have_fetch = false;
    l->averages++;
    return DPWA_OK;
}

int dpwa_learner_factor(dpwa_learner *l, double, const double *, dpwa_stream_t)
{
    return l && l->have_fetch ? DPWA_OK : set_error(DPWA_ERR_STATE, "factor");
}
int dpwa_learner_lerp(dpwa_learner *l, void *, dpwa_stream_t) { return averaged(l); }
int dpwa_learner_average(dpwa_learner *l, void *, double, const double *, dpwa_stream_t) { return averaged(l); }
int dpwa_learner_average_through(dpwa_learner *l, void *, double, const double *, dpwa_stream_t) { return averaged(l); }

int dpwa_learner_average_many(dpwa_learner *const *ls, void *const *, const double *, const double *const *,
                              const int *, int count, dpwa_stream_t)
{
    for (int i = 0; i < count; ++i) {
        const int rc = averaged(ls[i]);
        if (rc) return rc;
    }
    return DPWA_OK;
}

int dpwa_learner_relocate(dpwa_learner *l, dpwa_stream_t)
{
    if (!l) return set_error(DPWA_ERR_ARG, "relocate");
    l->relocations++;
    return DPWA_OK;
}

int dpwa_learner_set_resident(dpwa_learner *, const void *, dpwa_stream_t)
{
    return set_error(DPWA_ERR_STATE, "set_resident: not in the host-only build");
}

// -- the gossip board is not part of this build (no node here is given one) -----------------
int dpwa_board_status(dpwa_board *, int, int32_t *) { return set_error(DPWA_ERR_STATE, "no board"); }
int dpwa_board_acquire(dpwa_board *, int, uint64_t *) { return set_error(DPWA_ERR_STATE, "no board"); }
int dpwa_board_release(dpwa_board *, int, dpwa_stream_t, int) { return set_error(DPWA_ERR_STATE, "no board"); }
int dpwa_board_publish_wait(dpwa_board *, uint64_t, int) { return set_error(DPWA_ERR_STATE, "no board"); }
int dpwa_board_advertise(dpwa_board *, uint64_t, dpwa_stream_t, int) { return set_error(DPWA_ERR_STATE, "no board"); }

}  // extern "C"
