"""The C++ scheduler (product, dpwa_amd/csrc/sched.cpp) against the reference's own peer
choices and Bernoulli draws (tests/golden/*.json, produced by running the reference).
Host code only -- no GPU."""
import random

import pytest

from dpwa_amd import _lib
from dpwa_amd.sched import Scheduler, seed_key
from tests.helpers import load_json


@pytest.mark.parametrize("seed", [0, 1, 7, 1000, 2**32, 2**64 + 3, -9, 123456789012345678901234567890])
def test_mt19937_matches_cpython(seed):
    s, r = Scheduler(1, seed), random.Random(seed)
    for _ in range(700):            # crosses a 624-word regeneration
        assert s.random() == r.random()
    for a, b in [(10, 1000), (0, 0), (0, 1), (0, 6), (0, 2**31), (-5, 5)]:
        for _ in range(200):
            assert s.randint(a, b) == r.randint(a, b)


def test_seed_key_words():
    assert seed_key(0) == []
    assert seed_key(5) == [5]
    assert seed_key(2**32 + 1) == [1, 1]
    assert seed_key(-7) == [7]


def test_unseeded_is_entropy():
    a, b = Scheduler(2), Scheduler(2)
    assert [a.random() for _ in range(4)] != [b.random() for _ in range(4)]


OUT = {"ok": "connect_ok", "refused": "refused", "error": "connect_error"}


def replay_round(s, attempts):
    """Drives pick/report with the reference's recorded outcomes; returns (picks, data)."""
    picks = []
    i = 0
    data = False
    while True:
        k, connected = s.pick()
        if k < 0:
            break
        picks.append(k)
        a = attempts[i]
        i += 1
        if not connected:
            assert a["connect"] is not None
            done, data = s.report(k, OUT[a["connect"]])
            if done:
                break
        else:
            assert a["connect"] is None
        done, data = s.report(k, a["request"])
        if done:
            break
    assert i == len(attempts)
    return picks, data


def test_peer_selection_matches_reference():
    data = load_json("peer_select.json")
    n_rounds = 0
    for case in data["cases"]:
        peers = case["peers"]
        s = Scheduler(len(peers), case["seed"], case["fetch_probability"])
        for r in case["rounds"]:
            fetching = s.bernoulli()
            assert fetching == r["fetching"]
            if fetching:
                picks, got = replay_round(s, r["attempts"])
                assert [peers[k] for k in picks] == [a["peer"] for a in r["attempts"]]
                assert got == r["data"]
            assert s.scores() == r["scores"]
            n_rounds += 1
    assert n_rounds == 48 * 40


def test_bernoulli_matches_reference_policy_traces():
    data = load_json("policy.json")
    for case in data["cases"]:
        s = Scheduler(2, case["seed"], case["fetch_probability"])
        assert [s.bernoulli() for _ in case["rounds"]] == [r["fetching"] for r in case["rounds"]]


def test_static_fetch_matches_pick_report_loop():
    """dpwa_sched_fetch (one call) == the explicit pick/report loop for static statuses."""
    rng = random.Random(5)
    for trial in range(200):
        P = rng.randint(1, 8)
        status = [rng.choice([_lib.PEER_READY] * 3 + [_lib.PEER_NO_STATE, _lib.PEER_DOWN, _lib.PEER_SLOW,
                                                       _lib.PEER_DEAD]) for _ in range(P)]
        a, b = Scheduler(P, trial), Scheduler(P, trial)
        for _ in range(20):
            k1, att1 = a.fetch(status, 50)
            # explicit loop
            k2, att2 = -1, 0
            while att2 < 50:
                k, connected = b.pick()
                if k < 0:
                    break
                att2 += 1
                st = status[k]
                if not connected:
                    c = {_lib.PEER_DOWN: "refused", _lib.PEER_DEAD: "connect_error"}.get(st, "connect_ok")
                    done, _ = b.report(k, c)
                    if done:
                        break
                r = {_lib.PEER_READY: "payload", _lib.PEER_NO_STATE: "empty", _lib.PEER_SLOW: "timeout"}.get(st, "error")
                done, got = b.report(k, r)
                if got:
                    k2 = k
                    break
                if done:
                    break
            assert (k1, att1) == (k2, att2)
            assert a.scores() == b.scores()


def test_flow_control_bounds_and_removal():
    s = Scheduler(2, 0)
    for _ in range(30):
        s.report(0, "timeout")
    assert s.score(0) == 10
    for _ in range(200):
        s.report(0, "payload")
    assert s.score(0) == 1000
    s.report(1, "error")
    assert s.score(1) is None and s.n_live() == 1
    with pytest.raises(_lib.DpwaError):
        s.report(1, "payload")
    _lib.call("dpwa_sched_remove", s._h, 0)
    assert s.pick() == (-1, False)


def test_add_peer_matches_reference():
    """Peers removed by errors and put back with add_peer (dpwa.py:95-96 -> conn.py:208-213):
    fresh score, not connected, and a re-added peer draws its randint after the others --
    replayed against the real TxThread's picks and scores."""
    data = load_json("peer_add.json")
    reorders = 0
    for case in data["cases"]:
        peers = case["peers"]
        s = Scheduler(len(peers), case["seed"], case["fetch_probability"])
        for r in case["rounds"]:
            for name in r["add_peer"]:
                s.add(peers.index(name))
            fetching = s.bernoulli()
            assert fetching == r["fetching"]
            if fetching:
                picks, got = replay_round(s, r["attempts"])
                assert [peers[k] for k in picks] == [a["peer"] for a in r["attempts"]]
                assert got == r["data"]
            assert s.scores() == r["scores"]
            reorders += r["order"] != [p for p in peers if p in r["order"]]
    assert reorders > 0        # the fixture does exercise a changed pick order


def test_oracle_add_peer_matches_reference():
    from oracle.policy import OracleLearner
    data = load_json("peer_add.json")
    for case in data["cases"]:
        L = OracleLearner(case["me"], case["peers"], 1.0, "clock", None, 0.0, case["seed"])
        for r in case["rounds"]:
            for name in r["add_peer"]:
                L.add_peer(name)
            L.update_send(1.0)
            it = iter(r["attempts"])
            pending = []           # the attempt whose connect outcome was just replayed

            def conn_fn(peer):
                a = next(it)
                assert a["peer"] == peer
                if a["connect"] == "ok":
                    pending.append(a)
                return a["connect"]

            def req_fn(peer):
                a = pending.pop() if pending else next(it)
                assert a["peer"] == peer
                out = a["request"]
                return (out, {"clock": 1, "loss": 0.5}, b"x") if out == "payload" else (out, None, None)

            _, payload, att = L.fetch(conn_fn, req_fn)
            assert [a["peer"] for a in att] == [a["peer"] for a in r["attempts"]]
            assert (payload is not None) == r["data"]
            assert L.scores(case["peers"]) == r["scores"]
            assert list(L.peers) == r["order"]


def test_state_is_cpython_getstate_and_round_trips():
    """Gossip-state checkpoint (dpwa_sched_get_state / _set_state): words 2..626 are CPython's
    random.getstate()[1] after the same draws; a second scheduler given the state continues the
    first one's peer choices, scores and gate draws exactly, through removals and faults."""
    s = Scheduler(5, seed=1234, fetch_probability=0.7)
    r = random.Random(1234)
    for _ in range(37):
        assert s.random() == r.random()
    st = s.get_state()
    assert st[:2] == [0x53575044, 1] and tuple(st[2:2 + 625]) == r.getstate()[1]
    rng = random.Random(77)

    def rounds(sched, n, seed):
        g = random.Random(seed)           # the same scripted transport outcomes for both
        out = []
        for _ in range(n):
            status = [g.choice([0, 0, 0, 1, 2, 3]) for _ in range(5)]
            out.append((sched.bernoulli(), sched.fetch(status), sched.scores()))
        return out

    rounds(s, 40, 5)
    live = [k for k, sc in enumerate(s.scores()) if sc is not None]
    if len(live) > 1:
        s.remove(live[-1])                # remove_peer (conn.py:215-222) on top of the faults' removals
    s.add(0)                              # and put a peer back (add_peer), if it was gone
    rounds(s, 10, 6)
    saved = s.get_state()
    ahead = rounds(s, 60, 7)
    t = Scheduler(5, seed=rng.randrange(1 << 30), fetch_probability=0.7)
    t.set_state(saved)
    assert t.get_state() == saved
    assert rounds(t, 60, 7) == ahead


def test_state_is_validated_before_it_is_applied():
    s = Scheduler(3, seed=9)
    good = s.get_state()
    t = Scheduler(4, seed=9)
    with pytest.raises(_lib.DpwaError, match="peers"):
        t.set_state(good)                                   # another peer count
    bad = list(good)
    bad[2 + 625 + 1] = 5000                                 # peer 0's score out of [10, 1000]
    before = s.get_state()
    with pytest.raises(_lib.DpwaError, match="out of range"):
        s.set_state(bad)
    assert s.get_state() == before                          # nothing changed
    bad = list(good)
    bad[0] = 0
    with pytest.raises(_lib.DpwaError, match="not a scheduler state"):
        s.set_state(bad)
    bad = list(good)
    bad[2 + 624] = 625                                      # generator position past N
    with pytest.raises(_lib.DpwaError, match="position"):
        s.set_state(bad)
