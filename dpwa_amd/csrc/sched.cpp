// sched.cpp -- host-side gossip scheduler: the reference TxThread's peer choice and flow
// control (dpwa/conn.py:178-317) and DpwaConnection's Bernoulli fetch gate
// (dpwa/dpwa.py:101-102, 118-123), driven by an MT19937 that reproduces CPython 3.10's
// `random` module draw for draw (Modules/_randommodule.c + Lib/random.py), so a learner
// seeded like `random.seed(seed)` picks exactly the peers the reference picks.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <new>
#include <random>
#include <vector>

#include "common.hpp"

namespace dpwa {

// CPython's MT19937 (_randommodule.c): init_genrand / init_by_array / genrand_uint32.
class PyMT {
public:
    static constexpr int N = 624;
    static constexpr int M = 397;

    void seed_by_array(const uint32_t *key, size_t key_len)
    {
        uint32_t zero = 0;
        if (key_len == 0) {  // random.seed(0): keyused = 1, key[0] = 0
            key = &zero;
            key_len = 1;
        }
        init_genrand(19650218U);
        size_t i = 1, j = 0;
        size_t k = (N > key_len ? N : key_len);
        for (; k; k--) {
            mt_[i] = (mt_[i] ^ ((mt_[i - 1] ^ (mt_[i - 1] >> 30)) * 1664525U)) + key[j] + (uint32_t)j;
            i++;
            j++;
            if (i >= (size_t)N) {
                mt_[0] = mt_[N - 1];
                i = 1;
            }
            if (j >= key_len) j = 0;
        }
        for (k = N - 1; k; k--) {
            mt_[i] = (mt_[i] ^ ((mt_[i - 1] ^ (mt_[i - 1] >> 30)) * 1566083941U)) - (uint32_t)i;
            i++;
            if (i >= (size_t)N) {
                mt_[0] = mt_[N - 1];
                i = 1;
            }
        }
        mt_[0] = 0x80000000U;
    }

    uint32_t next_u32()
    {
        static const uint32_t mag01[2] = {0x0U, 0x9908b0dfU};
        uint32_t y;
        if (idx_ >= N) {
            int kk;
            for (kk = 0; kk < N - M; kk++) {
                y = (mt_[kk] & 0x80000000U) | (mt_[kk + 1] & 0x7fffffffU);
                mt_[kk] = mt_[kk + M] ^ (y >> 1) ^ mag01[y & 0x1U];
            }
            for (; kk < N - 1; kk++) {
                y = (mt_[kk] & 0x80000000U) | (mt_[kk + 1] & 0x7fffffffU);
                mt_[kk] = mt_[kk + (M - N)] ^ (y >> 1) ^ mag01[y & 0x1U];
            }
            y = (mt_[N - 1] & 0x80000000U) | (mt_[0] & 0x7fffffffU);
            mt_[N - 1] = mt_[M - 1] ^ (y >> 1) ^ mag01[y & 0x1U];
            idx_ = 0;
        }
        y = mt_[idx_++];
        y ^= (y >> 11);
        y ^= (y << 7) & 0x9d2c5680U;
        y ^= (y << 15) & 0xefc60000U;
        y ^= (y >> 18);
        return y;
    }

    // random.random(): 53-bit double from two words (random_random)
    double random()
    {
        uint32_t a = next_u32() >> 5, b = next_u32() >> 6;
        return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
    }

    // random.getrandbits(k), 0 <= k <= 32 (random_getrandbits fast path)
    uint32_t getrandbits(int k)
    {
        if (k == 0) return 0;
        return next_u32() >> (32 - k);
    }

    // Random._randbelow_with_getrandbits(n) (Lib/random.py, CPython 3.10), n < 2**32
    uint64_t randbelow(uint64_t n)
    {
        if (n == 0) return 0;
        int k = 0;
        for (uint64_t t = n; t; t >>= 1) k++;  // n.bit_length()
        uint64_t r = getrandbits(k);
        while (r >= n) r = getrandbits(k);
        return r;
    }

    // random.randint(a, b) == randrange(a, b + 1) == a + _randbelow(b - a + 1)
    int64_t randint(int64_t a, int64_t b) { return a + (int64_t)randbelow((uint64_t)(b - a + 1)); }

    // The generator's state in CPython's random.getstate() order: the 624 words, then the
    // position (getstate()[1] == (*mt, pos)).
    void get_state(uint32_t *out) const
    {
        for (int i = 0; i < N; ++i) out[i] = mt_[i];
        out[N] = (uint32_t)idx_;
    }
    bool set_state(const uint32_t *in)
    {
        if (in[N] > (uint32_t)N) return false;     // CPython's setstate rejects pos > N too
        for (int i = 0; i < N; ++i) mt_[i] = in[i];
        idx_ = (int)in[N];
        return true;
    }

private:
    void init_genrand(uint32_t s)
    {
        mt_[0] = s;
        for (int i = 1; i < N; i++) mt_[i] = (1812433253U * (mt_[i - 1] ^ (mt_[i - 1] >> 30)) + (uint32_t)i);
        idx_ = N;
    }

    uint32_t mt_[N];
    int idx_ = N + 1;
};

// conn.py:178-181
constexpr int kFlowMin = 10;
constexpr int kFlowMax = 1000;
constexpr int kFlowInc = 10;
constexpr int kFlowDec = 100;

struct PeerEntry {
    int score = kFlowMax;      // WorkerConn.flow_control_score (conn.py:190)
    bool connected = false;    // lazy connection (conn.py:193)
    bool live = true;          // false after remove_peer (conn.py:215-222)
};

}  // namespace dpwa

struct dpwa_sched {
    dpwa::PyMT rng;
    double fetch_probability = 1.0;
    std::vector<dpwa::PeerEntry> peers;   // indexed by peer id (YAML order minus self)
    std::vector<int> order;               // live peers in TxThread.peers' dict order: YAML order,
                                          // removals dropped, re-added peers at the end
    std::vector<int64_t> draw;            // scratch: scores of this pick
};

using namespace dpwa;

extern "C" {

int dpwa_sched_create(dpwa_sched **out, int n_peers, const uint32_t *seed_key, int key_len,
                      double fetch_probability)
{
    if (!out || n_peers < 0) return set_error(DPWA_ERR_ARG, "dpwa_sched_create: bad arguments");
    if (key_len > 0 && !seed_key) return set_error(DPWA_ERR_ARG, "dpwa_sched_create: seed_key is NULL");
    dpwa_sched *s = new (std::nothrow) dpwa_sched();
    if (!s) return set_error(DPWA_ERR_NOMEM, "dpwa_sched_create: out of memory");
    if (key_len < 0) {  // random.seed(None): OS entropy
        std::random_device rd;
        std::vector<uint32_t> key(PyMT::N);
        for (auto &k : key) k = rd();
        s->rng.seed_by_array(key.data(), key.size());
    } else {
        s->rng.seed_by_array(seed_key, (size_t)key_len);
    }
    s->fetch_probability = fetch_probability;
    s->peers.assign((size_t)n_peers, PeerEntry());
    for (int k = 0; k < n_peers; ++k) s->order.push_back(k);
    *out = s;
    return DPWA_OK;
}

int dpwa_sched_destroy(dpwa_sched *s)
{
    delete s;
    return DPWA_OK;
}

int dpwa_sched_bernoulli(dpwa_sched *s, int *fetching)
{
    if (!s || !fetching) return set_error(DPWA_ERR_ARG, "dpwa_sched_bernoulli: NULL argument");
    *fetching = s->rng.random() < s->fetch_probability ? 1 : 0;
    return DPWA_OK;
}

int dpwa_sched_pick(dpwa_sched *s, int *peer, int *connected)
{
    if (!s || !peer || !connected) return set_error(DPWA_ERR_ARG, "dpwa_sched_pick: NULL argument");
    // conn.py:227-229: one randint(10, 1000) per live peer, in dict (insertion) order
    int64_t best = -1;
    int n_best = 0;
    s->draw.assign(s->peers.size(), -1);
    for (int k : s->order) {
        int64_t v = s->peers[k].score + s->rng.randint(kFlowMin, kFlowMax);
        s->draw[k] = v;
        if (v > best) {
            best = v;
            n_best = 1;
        } else if (v == best) {
            n_best++;
        }
    }
    if (n_best == 0) {  // conn.py:231-233: no peers
        *peer = -1;
        *connected = 0;
        return DPWA_OK;
    }
    // conn.py:238-239: ties in insertion order, chosen by randint(0, k-1) (always drawn)
    int64_t which = s->rng.randint(0, n_best - 1);
    for (int k : s->order) {
        if (s->draw[k] == best) {
            if (which == 0) {
                *peer = k;
                *connected = s->peers[k].connected ? 1 : 0;
                return DPWA_OK;
            }
            which--;
        }
    }
    return set_error(DPWA_ERR_STATE, "dpwa_sched_pick: internal error");
}

// TxThread.remove_peer (conn.py:215-222): `del self.peers[name]`.
static void drop_peer(dpwa_sched *s, int peer)
{
    s->peers[peer].live = false;
    s->peers[peer].connected = false;
    s->order.erase(std::remove(s->order.begin(), s->order.end(), peer), s->order.end());
}

int dpwa_sched_report(dpwa_sched *s, int peer, int outcome, int *round_done, int *got_data)
{
    if (!s || !round_done || !got_data || peer < 0 || (size_t)peer >= s->peers.size() || !s->peers[peer].live)
        return set_error(DPWA_ERR_ARG, "dpwa_sched_report: bad peer");
    PeerEntry &p = s->peers[peer];
    *round_done = 0;
    *got_data = 0;
    switch (outcome) {
    case DPWA_CONNECT_OK:
        p.connected = true;
        break;
    case DPWA_CONNECT_REFUSED:   // conn.py:253-256
        p.score = p.score - kFlowDec > kFlowMin ? p.score - kFlowDec : kFlowMin;
        *round_done = 1;
        break;
    case DPWA_CONNECT_ERROR:     // conn.py:257-260
        drop_peer(s, peer);
        *round_done = 1;
        break;
    case DPWA_REPLY_PAYLOAD:     // conn.py:301-302
        p.score = p.score + kFlowInc < kFlowMax ? p.score + kFlowInc : kFlowMax;
        *round_done = 1;
        *got_data = 1;
        break;
    case DPWA_REPLY_EMPTY:
        p.score = p.score + kFlowInc < kFlowMax ? p.score + kFlowInc : kFlowMax;
        break;
    case DPWA_REPLY_TIMEOUT:     // conn.py:304-309
        p.score = p.score - kFlowDec > kFlowMin ? p.score - kFlowDec : kFlowMin;
        p.connected = false;
        break;
    case DPWA_REPLY_ERROR:       // conn.py:311-313
        drop_peer(s, peer);
        break;
    default:
        return set_error(DPWA_ERR_ARG, "dpwa_sched_report: unknown outcome");
    }
    return DPWA_OK;
}

int dpwa_sched_fetch(dpwa_sched *s, const int32_t *peer_status, int max_attempts, int *peer_out,
                     int *attempts_out)
{
    if (!s || !peer_status || !peer_out || !attempts_out || max_attempts <= 0)
        return set_error(DPWA_ERR_ARG, "dpwa_sched_fetch: bad arguments");
    *peer_out = -1;
    int attempts = 0;
    while (attempts < max_attempts) {
        int peer, connected, done = 0, data = 0;
        int rc = dpwa_sched_pick(s, &peer, &connected);
        if (rc) return rc;
        if (peer < 0) break;
        attempts++;
        const int32_t st = peer_status[peer];
        if (!connected) {
            int c = DPWA_CONNECT_OK;
            if (st == DPWA_PEER_DOWN) c = DPWA_CONNECT_REFUSED;
            else if (st == DPWA_PEER_DEAD) c = DPWA_CONNECT_ERROR;
            if ((rc = dpwa_sched_report(s, peer, c, &done, &data))) return rc;
            if (done) break;
        }
        int r;
        switch (st) {
        case DPWA_PEER_READY: r = DPWA_REPLY_PAYLOAD; break;
        case DPWA_PEER_NO_STATE: r = DPWA_REPLY_EMPTY; break;
        case DPWA_PEER_SLOW: r = DPWA_REPLY_TIMEOUT; break;
        default: r = DPWA_REPLY_ERROR; break;   // DOWN while connected (reset) or DEAD
        }
        if ((rc = dpwa_sched_report(s, peer, r, &done, &data))) return rc;
        if (data) {
            *peer_out = peer;
            break;
        }
        if (done) break;
    }
    *attempts_out = attempts;
    return DPWA_OK;
}

int dpwa_sched_score(const dpwa_sched *s, int peer, int *score)
{
    if (!s || !score || peer < 0 || (size_t)peer >= s->peers.size())
        return set_error(DPWA_ERR_ARG, "dpwa_sched_score: bad peer");
    *score = s->peers[peer].live ? s->peers[peer].score : -1;
    return DPWA_OK;
}

int dpwa_sched_remove(dpwa_sched *s, int peer)
{
    if (!s || peer < 0 || (size_t)peer >= s->peers.size() || !s->peers[peer].live)
        return set_error(DPWA_ERR_ARG, "dpwa_sched_remove: bad peer");
    drop_peer(s, peer);
    return DPWA_OK;
}

// TxThread.add_peer (conn.py:208-213): `self.peers[name] = WorkerConn(...)` -- a fresh record
// (score 1000, not connected).  A live peer keeps its place in the dict order; a removed one
// is inserted again, at the end.
int dpwa_sched_add(dpwa_sched *s, int peer)
{
    if (!s || peer < 0 || (size_t)peer >= s->peers.size()) return set_error(DPWA_ERR_ARG, "dpwa_sched_add: bad peer");
    PeerEntry &p = s->peers[peer];
    if (!p.live) s->order.push_back(peer);
    p = PeerEntry();
    return DPWA_OK;
}

int dpwa_sched_n_live(const dpwa_sched *s, int *n_live)
{
    if (!s || !n_live) return set_error(DPWA_ERR_ARG, "dpwa_sched_n_live: NULL argument");
    int n = 0;
    for (const auto &p : s->peers) n += p.live ? 1 : 0;
    *n_live = n;
    return DPWA_OK;
}

// ---- gossip-state checkpoint (SURVEY §5 checkpoint/resume).  The reference keeps no gossip state
// across a restart (dpwa.py:59 starts the clock at 0; `random` starts from its seed again); here a
// resumed job can continue the scheduler exactly where it stopped.  Layout, 32-bit words:
//   magic 'DPWS', format 1, MT19937 state (624 words + position, CPython getstate() order),
//   n_peers, per peer {score, flags: 1 connected | 2 live}, n_order, order[n_order]
constexpr uint32_t kStateMagic = 0x53575044u;   // "DPWS" little-endian
constexpr uint32_t kStateFormat = 1;

static int state_words(const dpwa_sched *s)
{
    return 2 + PyMT::N + 1 + 1 + 2 * (int)s->peers.size() + 1 + (int)s->order.size();
}

int dpwa_sched_get_state(const dpwa_sched *s, uint32_t *words, int max_words, int *n_words)
{
    if (!s || !n_words) return set_error(DPWA_ERR_ARG, "dpwa_sched_get_state: NULL argument");
    const int n = state_words(s);
    *n_words = n;
    if (!words) return DPWA_OK;                   // size query
    if (max_words < n) return set_error(DPWA_ERR_ARG, "dpwa_sched_get_state: %d words needed, %d given", n, max_words);
    int w = 0;
    words[w++] = kStateMagic;
    words[w++] = kStateFormat;
    s->rng.get_state(words + w);
    w += PyMT::N + 1;
    words[w++] = (uint32_t)s->peers.size();
    for (const PeerEntry &p : s->peers) {
        words[w++] = (uint32_t)p.score;
        words[w++] = (p.connected ? 1u : 0u) | (p.live ? 2u : 0u);
    }
    words[w++] = (uint32_t)s->order.size();
    for (int k : s->order) words[w++] = (uint32_t)k;
    return DPWA_OK;
}

int dpwa_sched_set_state(dpwa_sched *s, const uint32_t *words, int n_words)
{
    if (!s || !words) return set_error(DPWA_ERR_ARG, "dpwa_sched_set_state: NULL argument");
    const int fixed = 2 + PyMT::N + 1 + 1;
    if (n_words < fixed + 1 || words[0] != kStateMagic || words[1] != kStateFormat)
        return set_error(DPWA_ERR_ARG, "dpwa_sched_set_state: not a scheduler state (format %u)", kStateFormat);
    const uint32_t P = words[2 + PyMT::N + 1];
    if (P != s->peers.size())
        return set_error(DPWA_ERR_ARG, "dpwa_sched_set_state: state of %u peers, scheduler has %zu", P,
                         s->peers.size());
    if (n_words < fixed + 2 * (int)P + 1) return set_error(DPWA_ERR_ARG, "dpwa_sched_set_state: truncated state");
    const uint32_t n_order = words[fixed + 2 * P];
    if (n_words != fixed + 2 * (int)P + 1 + (int)n_order || n_order > P)
        return set_error(DPWA_ERR_ARG, "dpwa_sched_set_state: bad peer order length");
    // validate everything before changing anything
    std::vector<PeerEntry> peers(P);
    for (uint32_t k = 0; k < P; ++k) {
        const uint32_t sc = words[fixed + 2 * k], fl = words[fixed + 2 * k + 1];
        if (sc < (uint32_t)kFlowMin || sc > (uint32_t)kFlowMax || fl > 3)
            return set_error(DPWA_ERR_ARG, "dpwa_sched_set_state: peer %u: score %u flags %u out of range", k, sc, fl);
        peers[k].score = (int)sc;
        peers[k].connected = (fl & 1u) != 0;
        peers[k].live = (fl & 2u) != 0;
    }
    std::vector<int> order;
    std::vector<char> seen(P, 0);
    for (uint32_t j = 0; j < n_order; ++j) {
        const uint32_t k = words[fixed + 2 * P + 1 + j];
        if (k >= P || seen[k] || !peers[k].live)
            return set_error(DPWA_ERR_ARG, "dpwa_sched_set_state: bad peer order entry %u", k);
        seen[k] = 1;
        order.push_back((int)k);
    }
    for (uint32_t k = 0; k < P; ++k)
        if (peers[k].live && !seen[k]) return set_error(DPWA_ERR_ARG, "dpwa_sched_set_state: live peer %u not ordered", k);
    PyMT rng = s->rng;
    if (!rng.set_state(words + 2)) return set_error(DPWA_ERR_ARG, "dpwa_sched_set_state: generator position out of range");
    s->rng = rng;
    s->peers = peers;
    s->order = order;
    return DPWA_OK;
}

int dpwa_sched_random(dpwa_sched *s, double *out)
{
    if (!s || !out) return set_error(DPWA_ERR_ARG, "dpwa_sched_random: NULL argument");
    *out = s->rng.random();
    return DPWA_OK;
}

int dpwa_sched_randint(dpwa_sched *s, int64_t a, int64_t b, int64_t *out)
{
    if (!s || !out || b < a || (uint64_t)(b - a) >= 0xffffffffULL)
        return set_error(DPWA_ERR_ARG, "dpwa_sched_randint: bad range");
    *out = s->rng.randint(a, b);
    return DPWA_OK;
}

}  // extern "C"
