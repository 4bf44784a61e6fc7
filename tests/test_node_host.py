"""node.cpp's per-round logic on the CPU, under AddressSanitizer + UndefinedBehaviorSanitizer:
DpwaConnection.update_send / update_wait (dpwa.py:104-156) and TxThread's fetch loop
(conn.py:277-315) with the device path's timeout judging and rescue lanes, built with g++ over a
host-only stand-in for the learner runtime (tests/native/fake_learner.cpp: a "pull" is a record
whose stalling is scripted) and the real scheduler (sched.cpp).  tests/native/node_stress.cpp
runs G lock-step learners whose first k pulls of a round stall (k drawn per learner and round,
0-12) and prints what every node did; here each learner's rounds are replayed in the oracle policy
(oracle/policy.py, pinned to the reference's TxThread by tests/golden/peer_select.json) with its
first k requests scripted as timeouts: the node re-selects after every timeout -- the side pull,
then rescue lanes, one after another while their pulls stall too -- exactly as TxThread keeps
re-selecting.  With the side stream and every lane stalled (8 lanes, or 3 on learners whose lane
allocations fail) the next request waits for a lane to land and then goes out as the next of the
TxThread loop's requests (a held-up transport: the oracle's rounds are unchanged); only when no lane
lands within DPWA_RESCUE_WAIT_MS (a stuck transport) does that request time out and the round end
without data.  Peers, attempts and flow-control scores must match round by round."""
import json
import os
import shutil
import subprocess

import pytest

from oracle.policy import OracleLearner

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]


@pytest.fixture(scope="module")
def node_stress(tmp_path_factory):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path_factory.mktemp("node") / "node_stress")
    srcs = ["dpwa_amd/csrc/node.cpp", "dpwa_amd/csrc/sched.cpp", "dpwa_amd/csrc/trace.cpp",
            "tests/native/fake_learner.cpp", "tests/native/node_stress.cpp"]
    cmd = [gxx, "-std=c++17", "-O1", "-g", *SAN, "-I", os.path.join(ROOT, "include"),
           *[os.path.join(ROOT, s) for s in srcs], "-o", exe, "-ldl", "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0 and ("asan" in r.stderr or "ubsan" in r.stderr):
        pytest.skip("sanitizer runtime not installed: " + r.stderr[-200:])
    assert r.returncode == 0, r.stderr
    return exe


def _run(exe, G, rounds, seed, fp, fault_pct=0, prefetch=0):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0", UBSAN_OPTIONS="print_stacktrace=1",
               DPWA_RESCUE_WAIT_MS="20")
    r = subprocess.run([exe, str(G), str(rounds), str(seed), repr(fp), str(fault_pct), str(prefetch)],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "node stress ok" in r.stderr
    return json.loads(r.stdout)


READY, NO_STATE, DOWN, SLOW, DEAD = 0, 1, 2, 3, 4     # DPWA_PEER_*; -1 = no fault


@pytest.mark.parametrize("G,fp,seed,fault_pct,prefetch", [(2, 1.0, 100, 0, 0), (4, 1.0, 200, 0, 0), (5, 0.7, 300, 0, 0),
                                                          (8, 1.0, 400, 0, 0), (4, 1.0, 500, 12, 0), (6, 0.8, 600, 8, 0),
                                                          (4, 1.0, 700, 0, 1), (5, 0.8, 800, 10, 1)])
def test_node_fetch_loop_with_rescue_lanes_matches_oracle(node_stress, G, fp, seed, fault_pct, prefetch):
    """With fault_pct > 0 some requests also meet a faulted peer (refused or reset when down,
    empty with no state, timed out when slow, removed when dead; conn.py:246-313), mixed with the
    stalled pulls.  prefetch: every granted fetch starts once the round has published
    (dpwa_node_start_fetch, LocalGroup(prefetch=True)); its side pull is judged at update_wait."""
    rounds = 40
    recs = _run(node_stress, G, rounds, seed, fp, fault_pct, prefetch)
    assert len(recs) == G * rounds
    names = ["n%d" % g for g in range(G)]
    L = [OracleLearner(names[g], [x for x in names if x != names[g]], fp, "constant", 0.5, 0.0, seed + g)
         for g in range(G)]
    by = {(x["round"], x["learner"]): x for x in recs}
    seen = {"data after a stalled rescue pull": 0, "lanes exhausted": 0, "data after every lane stalled": 0,
            "lanes capped": 0, "faulted requests": 0}
    for r in range(rounds):
        for g in range(G):
            L[g].update_send(1.0)
        for g in range(G):
            rec = by[(r, g)]
            others = [x for x in names if x != names[g]]
            fault = dict(zip(others, rec["faults"]))
            stall, cap, stuck = rec["stall"], rec["cap"], rec["stuck"]
            exhausted = stuck and stall > cap       # side pull + every lane stalled, none ever lands
            pulls = [0]      # requests to a ready peer (each is a pull; the first `stall` stall)

            def connect(peer, fault=fault):
                return {DOWN: "refused", DEAD: "error"}.get(fault[peer], "ok")

            def request(peer, fault=fault, stall=stall, pulls=pulls, cap=cap, exhausted=exhausted):
                f = fault[peer]
                if f in (-1, READY):
                    pulls[0] += 1
                    # the first `stall` pulls stall; with a stuck transport and every lane stalled the
                    # next request finds no lane within the wait and times out too
                    if pulls[0] <= stall if not exhausted else pulls[0] <= cap + 2:
                        return "timeout", None, None
                    return "payload", {"clock": 1, "loss": 1.0}, b"x"
                seen["faulted requests"] += 1
                return {NO_STATE: ("empty", None, None), SLOW: ("timeout", None, None)}.get(f, ("error", None, None))

            assert rec["fetching"] == int(L[g].fetching), (r, g)
            if L[g].fetching:
                _, payload, attempts = L[g].fetch(connect, request, max_attempts=100_000,   # node.cpp's bound
                                                  stop=lambda pulls=pulls, cap=cap, ex=exhausted:
                                                  ex and pulls[0] >= cap + 2)
                want_peer = others.index(attempts[-1]["peer"]) if payload is not None else -1
                assert (rec["peer"], rec["attempts"]) == (want_peer, len(attempts)), (r, g, rec, attempts)
                L[g].update_wait(1.0, {"clock": 1, "loss": 1.0}, payload is not None)
                if payload is not None and pulls[0] >= 3:
                    seen["data after a stalled rescue pull"] += 1
                if payload is not None and pulls[0] > cap + 1:
                    seen["data after every lane stalled"] += 1
                    seen["lanes capped"] += cap < 8
                if exhausted and pulls[0] >= cap + 2:
                    seen["lanes exhausted"] += 1
                    # (a prefetched side pull was issued before update_wait, where the driver counts)
                    assert rec["pulls"] == cap + (0 if prefetch else 1) and rec["peer"] == -1
            else:
                assert rec["peer"] == -1 and rec["attempts"] == 0
            want_scores = [-1 if x is None else x for x in L[g].scores(others)]
            assert rec["scores"] == want_scores, (r, g, rec)
    assert seen["data after a stalled rescue pull"] > 0 and seen["data after every lane stalled"] > 0, seen
    assert (seen["faulted requests"] > 0) == (fault_pct > 0), seen


def test_lanes_exhausted_and_capped_both_occur(node_stress):
    """Over the parameter sets above, rounds in which every lane stalled end with data when the
    transport was only held up -- on 8-lane learners and on learners whose lane allocations fail
    after 3 -- and without data only when it stayed stuck."""
    seen = {"held": 0, "capped": 0, "stuck": 0}
    for G, fp, seed in ((4, 1.0, 200), (8, 1.0, 400), (6, 1.0, 900)):
        for rec in _run(node_stress, G, 40, seed, fp):
            if not rec["fetching"] or rec["stall"] <= rec["cap"]:
                continue
            if rec["stuck"]:
                assert rec["peer"] == -1
                seen["stuck"] += 1
            else:
                assert rec["peer"] >= 0, rec
                seen["held"] += 1
                seen["capped"] += rec["cap"] == 3
    assert all(v > 0 for v in seen.values()), seen
