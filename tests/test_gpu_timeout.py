"""The device path's fetch timeout (the reference's socket timeout: conn.py:249 sets it from the
YAML's timeout_ms; conn.py:304-309 handles it: score -100, disconnect, pick again).

A pull is held back on the learner's side stream by a long spin kernel queued ahead of it, and
update_wait polls it after the deadline: the round must score that peer -100, pick again, pull
the re-selected peer into a rescue lane and average with it -- peers, scores, clocks and
parameters against the oracle policy with that request scripted as a timeout.  A pull that is
merely slower than the host (the normal case) is never judged a timeout.

The margins come from a measurement, not from an assumed clock: the spin kernel's rate
(torch.cuda._sleep cycles per second) is measured on the box first, a hold is sized in seconds
from it, and every held round checks afterwards, from events around the spin, that the hold
outlasted the host's wait past the deadline by the stated factor (so a held pull was still in
flight when it was judged)."""
import ctypes

import numpy as np
import pytest
import torch

from dpwa_amd import DpwaConnection, _lib
from dpwa_amd.group import LocalGroup
from oracle import lerp as olerp
from oracle.policy import OracleLearner

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)
from tests.helpers import HOLD_S, HOST_WAIT_S, TIMEOUT_MS, Hold  # noqa: E402  (measured spin holds)


def write_cfg(path, names, timeout_ms, interp="clock"):
    lines = ["- nodes:"] + ["  - {name: %s, host: localhost, port: %d}" % (n, 47000 + i) for i, n in enumerate(names)]
    lines += ["- fetch_probability: 1", "- timeout_ms: %d" % timeout_ms, "- interpolation: %s" % interp,
              "- divergence_threshold: 0", "- constant: { value: 0.5 }", "- clock: 0", "- loss: 0"]
    path.write_text("\n".join(lines) + "\n")


def side_stream(conn):
    s = ctypes.c_void_p()
    _lib.call("dpwa_learner_side_stream", conn._learner.handle, ctypes.byref(s))
    return torch.cuda.ExternalStream(s.value, device=DEV)


def expected(names, init, send, wait, seeds, timeouts):
    """The oracle's rounds; timeouts = {(round, learner): k}: learner's k-th request of that
    round (1-based) times out."""
    G, T = len(names), len(send)
    idx = {nm: i for i, nm in enumerate(names)}
    L = [OracleLearner(names[g], [x for x in names if x != names[g]], 1.0, "clock", None, 0.0, seeds[g])
         for g in range(G)]
    params = init.copy()
    out = []
    for r in range(T):
        states = [L[g].update_send(send[r][g]) for g in range(G)]
        snaps = [params[g].copy() for g in range(G)]
        row = []
        for g in range(G):
            n_req = [0]

            def request(peer, g=g, r=r, n_req=n_req):
                n_req[0] += 1
                if timeouts.get((r, g)) == n_req[0]:
                    return "timeout", None, None
                return "payload", states[idx[peer]], snaps[idx[peer]]

            state, payload, attempts = L[g].fetch(lambda p: "ok", request)
            averaged, factor = L[g].update_wait(wait[r][g], state, payload is not None)
            if averaged:
                params[g] = olerp.lerp_f32(params[g], payload, factor)
            row.append((attempts[-1]["peer"] if payload is not None else "", [a["peer"] for a in attempts]))
        out.append((params.copy(), [L[g].clock for g in range(G)],
                    [L[g].scores([x for x in names if x != names[g]]) for g in range(G)], row))
    return out


@pytest.mark.parametrize("pull", ["copy", "kernel:256"])
@pytest.mark.parametrize("G", [2, 3])
def test_held_pull_times_out_and_the_loop_picks_again(tmp_path, pull, G):
    names = ["t%d" % g for g in range(G)]
    cfg = tmp_path / "to.yaml"
    write_cfg(cfg, names, timeout_ms=TIMEOUT_MS)
    rng = np.random.default_rng(3)
    n, T = 100_003, 4
    init = rng.standard_normal((G, n)).astype(np.float32)
    send = [[1.0 + 0.5 * g + r for g in range(G)] for r in range(T)]
    wait = [[1.0 + 0.25 * g + r for g in range(G)] for r in range(T)]
    seeds = [60 + g for g in range(G)]
    held = {(1, 0)}                                      # learner 0's first pull of round 1 is held
    exp = expected(names, init, send, wait, seeds, {(1, 0): 1})
    group = LocalGroup(prefetch=True, zero_copy=False)   # copying pulls, started at the last publish
    conns = [DpwaConnection(names[g], str(cfg), seed=seeds[g], group=group, pull=pull) for g in range(G)]
    flats = [torch.from_numpy(init[g]).to(DEV) for g in range(G)]
    import time
    for r in range(T):
        holds = [Hold(side_stream(conns[g])) for g in range(G) if (r, g) in held]   # the next pull queues behind it
        for g in range(G):
            conns[g].update_send(flats[g], send[r][g])
        if holds:
            time.sleep(HOST_WAIT_S)                      # past the deadline
        got = [conns[g].update_wait_average(flats[g], wait[r][g]) for g in range(G)]
        torch.cuda.synchronize()                         # (the held pull has landed before the next round)
        for h in holds:
            h.check(HOST_WAIT_S)
        params, clocks, scores, row = exp[r]
        for g in range(G):
            assert (got[g][0].peer if got[g][0] is not None else "") == row[g][0], (r, g)
            assert conns[g].last_fetch_attempts == len(row[g][1]), (r, g)
            assert conns[g].clock == clocks[g], (r, g)
            assert olerp.bits_equal(flats[g].cpu().numpy(), params[g]), (r, g)
            want = dict(zip([x for x in names if x != names[g]], scores[g]))
            assert conns[g].flow_control_scores() == want, (r, g)
    assert len(exp[1][3][0][1]) == 2                     # the oracle's round: a timeout, then data
    for c in conns:
        c.close()


def test_slow_but_in_time_pull_is_data(tmp_path):
    """A pull held for less than the timeout is awaited on the device, not judged: the rounds
    are the oracle's rounds with no timeout."""
    G = 3
    names = ["s%d" % g for g in range(G)]
    cfg = tmp_path / "slow.yaml"
    write_cfg(cfg, names, timeout_ms=5000)
    rng = np.random.default_rng(4)
    n, T = 50_001, 3
    init = rng.standard_normal((G, n)).astype(np.float32)
    send = [[1.0 + g + r for g in range(G)] for r in range(T)]
    wait = [[2.0 + g + r for g in range(G)] for r in range(T)]
    seeds = [80 + g for g in range(G)]
    exp = expected(names, init, send, wait, seeds, {})
    group = LocalGroup(prefetch=True, zero_copy=False)
    conns = [DpwaConnection(names[g], str(cfg), seed=seeds[g], group=group) for g in range(G)]
    flats = [torch.from_numpy(init[g]).to(DEV) for g in range(G)]
    for r in range(T):
        # ~20 ms: slower than the host, well inside the 5 s timeout
        holds = [Hold(side_stream(conns[g]), 0.02) for g in range(G)] if r > 0 else []
        for g in range(G):
            conns[g].update_send(flats[g], send[r][g])
        for g in range(G):
            conns[g].update_wait_average(flats[g], wait[r][g])
        torch.cuda.synchronize()
        for h in holds:
            held = h.a.elapsed_time(h.b)
            assert held < 5000 / 10, "the hold lasted %.0f ms, not well inside the 5000 ms timeout" % held
        params, clocks, scores, _ = exp[r]
        for g in range(G):
            assert olerp.bits_equal(flats[g].cpu().numpy(), params[g]), (r, g)
            assert conns[g].clock == clocks[g]
            assert conns[g].flow_control_scores() == dict(zip([x for x in names if x != names[g]], scores[g]))
    for c in conns:
        c.close()


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("pull", ["copy", "kernel:256"])
def test_board_pull_times_out_and_the_rescue_pull_reads_a_whole_snapshot(tmp_path, pull):
    """Free-running rounds over the gossip board, two ranks on one GPU: rank 0's pull of round 3
    is held past timeout_ms.  Its only peer is scored -100 and disconnected, picked again
    (reconnect: the board still shows it live), and the rescue pull's snapshot is a whole,
    consistent version: every average of rank 0 equals the oracle lerp with the version the
    board handed out (oracle/async_check.py), versions never go backwards, and the scores follow
    the reference's increments (+10 per reply, -100 for the timeout)."""
    import torch.multiprocessing as mp
    from oracle.async_check import AsyncRuns
    from tests import dist_worker
    world, n, T, hold = 2, 200_003, 8, 3
    names = ["r%d" % i for i in range(world)]
    cfg = str(tmp_path / "to_board.yaml")
    dist_worker.write_cfg(cfg, names, 1.0, "constant", 0.0)
    text = open(cfg).read().replace("- timeout_ms: 2500", "- timeout_ms: %d" % TIMEOUT_MS)
    open(cfg, "w").write(text)
    mp.spawn(dist_worker.async_timeout_worker, args=(world, _free_port(), cfg, str(tmp_path), n, T, hold, pull),
             nprocs=world, join=True)
    runs = {g: np.load(tmp_path / ("rank%d.npz" % g)) for g in range(world)}
    check = AsyncRuns(names, {g: runs[g]["peers"] for g in range(world)},
                      {g: runs[g]["versions"] for g in range(world)}, "constant", 0.5, 0.0)
    for g in range(world):
        bad = check.check_rank(g, runs[g]["params"], runs[g]["clocks"], n)
        assert not bad, (g, bad[:5])
    r0 = runs[0]
    assert int(r0["attempts"][hold]) == 2 and str(r0["peers"][hold]) == "r1"     # a timeout, then data
    # scores of r1 as seen by r0: 1000 (max) until the timeout, 1000 - 100 + 10 after it, +10 per
    # later reply (conn.py:264-272)
    seen = [int(x[0]) for x in r0["scores"]]
    exp, sc = [], 1000
    for r in range(T):
        if str(r0["peers"][r]) == "" and r != hold:
            exp.append(sc)       # (an empty reply before r1's first publish is +10 too: capped)
            continue
        if r == hold:
            sc = max(sc - 100, 10)
        sc = min(sc + 10, 1000)
        exp.append(sc)
    assert seen == exp, (seen, exp)


def _stalled_rescue(_rank, tmp, mode):
    """See test_stalled_rescue_pulls_take_the_next_lane.  Rounds (learner 0): 1: its side stream
    held -> timeout, the re-selected pull on rescue lane 0 -> data; 2: side stream and lane 0 held
    -> two timeouts, lane 1 -> data; 3: side, lanes 0 and 1 held -> three timeouts, lane 2 ->
    data; 4: side and all three lanes held -> four timeouts, then
      mode "grow":   a fourth lane is made -> data (TxThread keeps re-selecting, conn.py:286-313);
      mode "capped": the lane count is capped at 3 (dpwa_learner_set_rescue_cap, as after a failed
                     allocation): the request waits for lane 0's pull to land, then goes out -> data;
      mode "stuck":  capped, and DPWA_RESCUE_WAIT_MS is shorter than the holds: no lane lands in
                     time, that request times out and the round ends without data (five timeouts)."""
    import os
    import pathlib
    import time
    if mode == "stuck":
        os.environ["DPWA_RESCUE_WAIT_MS"] = "50"        # read at node creation
    tmp_path = pathlib.Path(tmp)
    G = 3
    names = ["x%d" % g for g in range(G)]
    cfg = tmp_path / ("stall_%s.yaml" % mode)
    write_cfg(cfg, names, timeout_ms=TIMEOUT_MS)
    rng = np.random.default_rng(5)
    n, T = 50_003, 5
    init = rng.standard_normal((G, n)).astype(np.float32)
    send = [[1.0 + g + r for g in range(G)] for r in range(T)]
    wait = [[2.0 + g + r for g in range(G)] for r in range(T)]
    seeds = [90 + g for g in range(G)]
    stuck = mode == "stuck"
    timeouts = {1: 1, 2: 2, 3: 3, 4: 5 if stuck else 4}   # learner 0: its first k requests of round r time out
    idx = {nm: i for i, nm in enumerate(names)}
    L = [OracleLearner(names[g], [x for x in names if x != names[g]], 1.0, "clock", None, 0.0, seeds[g])
         for g in range(G)]
    params = init.copy()
    exp = []
    for r in range(T):
        states = [L[g].update_send(send[r][g]) for g in range(G)]
        snaps = [params[g].copy() for g in range(G)]
        picks = []
        for g in range(G):
            n_req = [0]

            def request(peer, g=g, r=r, n_req=n_req):
                n_req[0] += 1
                if g == 0 and n_req[0] <= timeouts.get(r, 0):
                    return "timeout", None, None
                return "payload", states[idx[peer]], snaps[idx[peer]]

            state, payload, attempts = L[g].fetch(lambda p: "ok", request,
                                                  max_attempts=5 if (g == 0 and r == 4 and stuck) else None)
            averaged, factor = L[g].update_wait(wait[r][g], state, payload is not None)
            if averaged:
                params[g] = olerp.lerp_f32(params[g], payload, factor)
            picks.append([a["peer"] for a in attempts])
        exp.append((params.copy(), [L[g].clock for g in range(G)],
                    [L[g].scores([x for x in names if x != names[g]]) for g in range(G)], picks))
    group = LocalGroup(prefetch=True, zero_copy=False)
    conns = [DpwaConnection(names[g], str(cfg), seed=seeds[g], group=group) for g in range(G)]
    flats = [torch.from_numpy(init[g]).to(DEV) for g in range(G)]
    lanes = []                                      # rescue lane streams, in the order they appear
    for r in range(T):
        holds = []
        if r >= 1:
            holds.append(Hold(side_stream(conns[0])))
            # lane j's pull is judged after the side pull's HOST_WAIT_S and j earlier rescue polls
            holds += [Hold(s, HOLD_S + (j + 1) * 0.3) for j, s in enumerate(lanes[:r - 1])]
        for g in range(G):
            conns[g].update_send(flats[g], send[r][g])
        if r == 1 and mode != "grow":                # bound by now: at most three lanes from here on
            _lib.call("dpwa_learner_set_rescue_cap", conns[0]._learner.handle, 3)
        if r >= 1:
            time.sleep(HOST_WAIT_S)
        t_wait = time.perf_counter()
        got = [conns[g].update_wait_average(flats[g], wait[r][g]) for g in range(G)]
        t_wait = time.perf_counter() - t_wait
        s = ctypes.c_void_p()
        _lib.call("dpwa_learner_fetch_stream", conns[0]._learner.handle, ctypes.byref(s))
        if 1 <= r <= 3 or (r == 4 and mode == "grow"):   # the rescue pull that delivered: a new lane
            assert s.value not in [x.cuda_stream for x in lanes] + [side_stream(conns[0]).cuda_stream], r
            lanes.append(torch.cuda.ExternalStream(s.value, device=DEV))
        elif r == 4 and mode == "capped":                # ... or, capped, the lane that landed first
            assert s.value == lanes[0].cuda_stream
            assert t_wait >= 0.5, t_wait                 # it waited for that lane's hold, well past 3 timeouts
        torch.cuda.synchronize()
        if holds:
            holds[0].check(HOST_WAIT_S)
            for j, h in enumerate(holds[1:]):       # lane j's pull is judged HOST_WAIT_S + (j+1) timeouts in
                h.check(HOST_WAIT_S + (j + 1) * TIMEOUT_MS / 1e3)
        p_exp, c_exp, s_exp, pk_exp = exp[r]
        for g in range(G):
            peer = got[g][0].peer if got[g][0] is not None else ""
            want = pk_exp[g][-1] if (g or r != 4 or not stuck) else ""
            assert (peer, conns[g].last_fetch_attempts) == (want, len(pk_exp[g])), \
                (r, g, peer, conns[g].last_fetch_attempts, pk_exp[g])
            assert conns[g].flow_control_scores() == dict(zip([x for x in names if x != names[g]], s_exp[g])), (r, g)
            assert olerp.bits_equal(flats[g].cpu().numpy(), p_exp[g]), (r, g)
            assert conns[g].clock == c_exp[g], (r, g)
    nl, cap = ctypes.c_int(), ctypes.c_int()
    _lib.call("dpwa_learner_rescue_lanes", conns[0]._learner.handle, ctypes.byref(nl), ctypes.byref(cap))
    assert (nl.value, cap.value) == ((4, 8) if mode == "grow" else (3, 3)), (nl.value, cap.value)
    if mode == "grow":
        # lanes beyond the first two are given back once idle for 8 fetch rounds (learner.cpp
        # trim_lanes): nine plain rounds later the learner holds two lanes again
        for r in range(9):
            for g in range(G):
                conns[g].update_send(flats[g], 1.0)
            for g in range(G):
                conns[g].update_wait_average(flats[g], 1.0)
        torch.cuda.synchronize()
        _lib.call("dpwa_learner_rescue_lanes", conns[0]._learner.handle, ctypes.byref(nl), ctypes.byref(cap))
        assert (nl.value, cap.value) == (2, 8), (nl.value, cap.value)
    for c in conns:
        c.close()


@pytest.mark.parametrize("mode", ["grow", "capped", "stuck"])
def test_stalled_rescue_pulls_take_the_next_lane(tmp_path, mode):
    """TxThread keeps re-selecting after a timeout until data, no peer, or every peer removed
    (conn.py:286-313).  Here a re-selected pull whose rescue lane is stalled times out too and the
    next pick goes to another lane: with the side stream and one, two, then all three rescue lanes
    held, the round still ends with data from the next pick -- on a fourth lane made for it, or,
    with the lanes capped at three (as after a lane allocation that failed), on the first lane whose
    pull lands -- peers, attempts, scores, clocks and parameters as the oracle policy with those
    requests scripted as timeouts.  Only a transport stuck for DPWA_RESCUE_WAIT_MS (here 50 ms,
    shorter than the holds) gives the request up: five timeouts, -100 each, no data.  Each mode
    runs in a fresh process (a stream map of its own)."""
    import torch.multiprocessing as mp
    mp.spawn(_stalled_rescue, args=(str(tmp_path), mode), nprocs=1, join=True)


def test_backlog_on_the_callers_stream_is_not_the_peers_delay(tmp_path):
    """The reference's timeout bounds only the wait for the reply (conn.py:249).  Work the caller
    queued on its own stream before update_send -- here a spin several times timeout_ms long --
    holds back a local peer's pull (it is ordered after that stream), but the request has not gone
    out until the stream gets there: the healthy peer is data, scored +10, never -100 -- the
    oracle's rounds with no timeout, every round, at 2 and 3 learners."""
    import time
    for G in (2, 3):
        names = ["b%d" % g for g in range(G)]
        cfg = tmp_path / ("backlog_%d.yaml" % G)
        write_cfg(cfg, names, timeout_ms=TIMEOUT_MS)
        rng = np.random.default_rng(6 + G)
        n, T = 100_003, 3
        init = rng.standard_normal((G, n)).astype(np.float32)
        send = [[1.0 + g + r for g in range(G)] for r in range(T)]
        wait = [[2.0 + g + r for g in range(G)] for r in range(T)]
        seeds = [70 + g for g in range(G)]
        exp = expected(names, init, send, wait, seeds, {})
        group = LocalGroup(prefetch=True, zero_copy=False)
        conns = [DpwaConnection(names[g], str(cfg), seed=seeds[g], group=group) for g in range(G)]
        flats = [torch.from_numpy(init[g]).to(DEV) for g in range(G)]
        for r in range(T):
            hold = Hold(torch.cuda.current_stream(DEV)) if r >= 1 else None   # the caller's backlog
            for g in range(G):
                conns[g].update_send(flats[g], send[r][g])
            if hold is not None:
                time.sleep(HOST_WAIT_S)                  # past the deadline as the host counts it
            for g in range(G):
                conns[g].update_wait_average(flats[g], wait[r][g])
            torch.cuda.synchronize()
            if hold is not None:
                hold.check(HOST_WAIT_S)                  # the backlog outlasted the judging point
            params, clocks, scores, row = exp[r]
            for g in range(G):
                assert conns[g].last_fetch_attempts == 1, (G, r, g)
                assert conns[g].flow_control_scores() == dict(zip([x for x in names if x != names[g]], scores[g]))
                assert olerp.bits_equal(flats[g].cpu().numpy(), params[g]), (G, r, g)
                assert conns[g].clock == clocks[g]
        for c in conns:
            c.close()
