"""Pins the CPU oracle (oracle/) against the golden fixtures produced by running the
reference (tests/golden/make_golden.py).  CPU only."""
import json

import numpy as np
import pytest

from oracle import gossip as ogossip
from oracle import lerp as olerp
from oracle import policy as opolicy
from tests.helpers import AttemptReplay, hexf, load_json, load_npz, num


def test_lerp_f32_numpy_matches_reference_adapter():
    z = load_npz("lerp_f32.npz")
    for f, out in zip(z["factors"], z["out"]):
        got = olerp.lerp_f32(z["param"], z["peer"], float(f))
        assert olerp.bits_equal(got, out), f


def test_lerp_f32_c_matches_reference_adapter():
    z = load_npz("lerp_f32.npz")
    for f, out in zip(z["factors"], z["out"]):
        p = z["param"].copy()
        olerp.c_lerp_f32_(p, z["peer"].copy(), float(f))
        assert olerp.bits_equal(p, out), f


def test_lerp_f32_fma_would_not_match():
    """The fixtures contain near-cancellation pairs on which a fused multiply-add differs:
    guards against a restatement (or kernel) that silently contracts."""
    z = load_npz("lerp_f32.npz")
    f = 1.0 / 3.0
    a, b = olerp.coefficients(f)
    p = z["param"].astype(np.float64)
    t = z["peer"].astype(np.float64)
    with np.errstate(all="ignore"):
        fused = (a * t + np.float32(b * z["param"]).astype(np.float64)).astype(np.float32)
    out = z["out"][list(z["factors"]).index(f)]
    assert not olerp.bits_equal(fused, out)
    del p


def test_lerp_bf16_matches_torch_eager():
    z = load_npz("lerp_bf16.npz")
    for f, out in zip(z["factors"], z["out"]):
        assert olerp.bits_equal(olerp.lerp_bf16(z["param"], z["peer"], float(f)), out), f
        p = z["param"].copy()
        olerp.c_lerp_bf16_(p, z["peer"].copy(), float(f))
        assert olerp.bits_equal(p, out), f


def test_factor_c_matches_python_restatement():
    lib = olerp.clib()
    import ctypes
    rng = np.random.default_rng(3)
    for _ in range(2000):
        m = int(rng.integers(0, 3))
        vals = rng.uniform(0, 3, 5)
        args = (m, float(vals[0] / 3), float(rng.choice([0.0, 0.5, 1.0])), float(vals[1]),
                float(vals[2]), float(vals[3]), float(vals[4]))
        fo, co = ctypes.c_double(), ctypes.c_double()
        rc = lib.dpwa_oracle_factor(*args, ctypes.byref(fo), ctypes.byref(co))
        f, c = opolicy.factor_and_clock(["constant", "clock", "loss"][m], args[1], args[2], args[3], args[4],
                                        args[5], args[6])
        assert rc == 0 and fo.value == f and co.value == c


def test_policy_traces_match_reference():
    data = load_json("policy.json")
    assert len(data["cases"]) == 40
    for case in data["cases"]:
        L = opolicy.OracleLearner("w2", ["w1", "w3"], case["fetch_probability"], case["interpolation"],
                                  case["value"], case["divergence_threshold"], case["seed"])
        for r in case["rounds"]:
            st = L.update_send(num(r["send_loss"]))
            assert L.fetching == r["fetching"]
            assert st["clock"] == r["pub_clock"] and st["loss"] == num(r["pub_loss"])
            peer = {"clock": num(r["peer_clock"]), "loss": num(r["peer_loss"])}
            if r["raises"]:
                with pytest.raises(ZeroDivisionError):
                    L.update_wait(num(r["wait_loss"]), peer, r["has_payload"])
                L.fetching = False
            else:
                averaged, factor = L.update_wait(num(r["wait_loss"]), peer, r["has_payload"])
                assert averaged == r["averaged"]
                assert float(factor) == hexf(r["factor_hex"])
            assert float(L.clock) == hexf(r["clock_hex"])


def test_peer_selection_matches_reference_txthread():
    data = load_json("peer_select.json")
    assert len(data["cases"]) == 48
    for case in data["cases"]:
        L = opolicy.OracleLearner(case["me"], case["peers"], case["fetch_probability"], "clock", None, 0.0,
                                  case["seed"])
        for r in case["rounds"]:
            L.update_send(1.0)
            assert L.fetching == r["fetching"]
            state, payload = None, None
            if L.fetching:
                rep = AttemptReplay(r["attempts"])
                state, payload, attempts = L.fetch(rep.connect, rep.request)
                assert rep.done()
                assert [a["peer"] for a in attempts] == [a["peer"] for a in r["attempts"]]
            else:
                assert r["attempts"] == []
            averaged, factor = L.update_wait(1.0, state, payload is not None)
            assert averaged == r["data"]
            assert float(factor) == hexf(r["factor_hex"])
            assert float(L.clock) == hexf(r["clock_hex"])
            assert L.scores(case["peers"]) == r["scores"]


def test_gossip_trajectories_match_reference():
    meta = load_json("gossip.json")
    z = load_npz("gossip.npz")
    for case in meta["cases"]:
        k = case["key"]
        res = ogossip.simulate(case["names"], z[k + "_init"], z[k + "_deltas"], case["send_loss"],
                               case["wait_loss"], case["interpolation"], case["value"],
                               case["divergence_threshold"], case["fetch_probability"], case["seeds"])
        assert res["picks"] == case["picks"], k
        assert np.array_equal(res["fetching"], z[k + "_fetching"]), k
        assert np.array_equal(res["factors"], z[k + "_factors"]), k
        assert np.array_equal(res["clocks"], z[k + "_clocks"]), k
        assert olerp.bits_equal(res["params"], z[k + "_params"]), k


def test_gossip_step_after_wait_trajectories_match_reference():
    """The resident loop order (update_send, update_wait, step) from reference runs
    (make_golden.py gen_gossip_step_after_wait: the real adapter, connection and TxThread driven
    in that order, pytorch.py:42-68, dpwa.py:104-156) against oracle/gossip.py
    train_after_wait=True, bit for bit; and the README-order oracle does not reproduce it."""
    meta = load_json("gossip_step_after_wait.json")
    z = load_npz("gossip_step_after_wait.npz")
    assert meta["order"] == "update_send, update_wait, step"
    assert {c["G"] for c in meta["cases"]} == {3, 4}
    assert {c["interpolation"] for c in meta["cases"]} == {"clock", "loss"}
    for case in meta["cases"]:
        k = case["key"]
        args = (case["names"], z[k + "_init"], z[k + "_deltas"], case["send_loss"], case["wait_loss"],
                case["interpolation"], case["value"], case["divergence_threshold"], case["fetch_probability"],
                case["seeds"])
        res = ogossip.simulate(*args, train_after_wait=True)
        assert res["picks"] == case["picks"], k
        assert np.array_equal(res["fetching"], z[k + "_fetching"]), k
        assert np.array_equal(res["factors"], z[k + "_factors"]), k
        assert np.array_equal(res["clocks"], z[k + "_clocks"]), k
        assert olerp.bits_equal(res["params"], z[k + "_params"]), k
        other = ogossip.simulate(*args)
        assert not olerp.bits_equal(other["params"], z[k + "_params"]), k


def test_self_peer_trajectories_match_reference():
    """configs[1]'s self-peer (make_golden.py gen_gossip_self: the real adapter, connection and
    TxThread of one learner whose YAML lists a second node entry at its own host:port, so every
    fetch reaches its own RxThread, conn.py:246-251 -> 98-110) against oracle/gossip.py with that
    node list, bit for bit -- constant, clock and loss interpolation, fetch_probability 1 and 0.7."""
    meta = load_json("gossip_self.json")
    z = load_npz("gossip_self.npz")
    assert meta["order"] == "update_send, step, update_wait"
    assert {c["interpolation"] for c in meta["cases"]} == {"constant", "clock", "loss"}
    for case in meta["cases"]:
        k = case["key"]
        assert case["nodes"] == ["w1", "w1-self"] and case["serves"] == {"w1-self": 0}
        res = ogossip.simulate(case["names"], z[k + "_init"], z[k + "_deltas"], case["send_loss"],
                               case["wait_loss"], case["interpolation"], case["value"],
                               case["divergence_threshold"], case["fetch_probability"], case["seeds"],
                               nodes=case["nodes"], serves=case["serves"])
        assert res["picks"] == case["picks"], k
        assert np.array_equal(res["fetching"], z[k + "_fetching"]), k
        assert np.array_equal(res["factors"], z[k + "_factors"]), k
        assert np.array_equal(res["clocks"], z[k + "_clocks"]), k
        assert olerp.bits_equal(res["params"], z[k + "_params"]), k


def test_fixture_files_are_data_only():
    """Fixtures are inputs/outputs (json/npz), never reference source."""
    import os
    from tests.helpers import GOLDEN
    for fn in os.listdir(GOLDEN):
        assert fn.endswith((".json", ".npz", ".py", ".md")), fn
        if fn.endswith(".json"):
            json.load(open(os.path.join(GOLDEN, fn)))


def test_async_checker_accepts_a_consistent_run_and_rejects_a_torn_one():
    """oracle/async_check.py (the free-running checker used by test_gpu_async.py and bench.py's
    parity leg): a CPU-made run in which every round reads a published version passes; a
    snapshot with one element of a different version, or a stale clock, fails."""
    from oracle.async_check import AsyncRuns, async_base
    names = ["r0", "r1", "r2"]
    n, T = 257, 9
    rng = np.random.default_rng(4)
    peers, versions = {}, {}
    for g in range(3):
        peers[g], versions[g] = [], []
        for r in range(T):
            if r == 0:
                peers[g].append("")
                versions[g].append(0)
                continue
            q = int(rng.choice([x for x in range(3) if x != g]))
            peers[g].append(names[q])
            versions[g].append(int(rng.integers(max(1, r - 1), r + 1)))    # q's publish r-1 or r
    for g in range(3):          # versions per peer must not go backwards
        last = {}
        for r in range(T):
            if peers[g][r]:
                q = peers[g][r]
                versions[g][r] = max(versions[g][r], last.get(q, 0))
                last[q] = versions[g][r]
    for interp, thr in (("constant", 0.0), ("clock", 0.0), ("loss", 0.5)):
        check = AsyncRuns(names, peers, versions, interp, 0.5, thr)
        for g in range(3):
            params = np.stack([check.expected_params(g, r, n) for r in range(T)])
            clocks = np.array([check.clock_after(g, r) for r in range(T)])
            assert check.check_rank(g, params, clocks, n) == []
            torn = params.copy()
            q, v = check.read(g, 5)
            torn[5, 100] = olerp.lerp_f32(async_base(g, 5, n), async_base(q, v, n), check.policy(g, 5)[0])[100]
            assert any("round 5" in b for b in check.check_rank(g, torn, clocks, n))
            if interp != "constant":
                stale = clocks.copy()
                stale[6] += 1.0
                assert any("round 6: clock" in b for b in check.check_rank(g, params, stale, n))


def test_async_checker_distributed_digests():
    """AsyncRuns.served / check_rank_digests (bench.py's write-through parity leg): the
    publisher vouches for the averages of its own versions; a consistent CPU-made run passes
    and a torn average fails."""
    from oracle.async_check import AsyncRuns, async_base
    names = ["r0", "r1"]
    n, T = 131, 7
    peers = {0: ["", "r1", "r1", "", "r1", "r1", "r1"], 1: ["r0", "r0", "", "r0", "r0", "r0", "r0"]}
    versions = {0: [0, 1, 2, 0, 4, 4, 6], 1: [1, 2, 0, 3, 4, 5, 6]}
    check = AsyncRuns(names, peers, versions, "clock", None, 0.0)
    # write-through runs: version v of rank q is q's parameters after its round v-2 (v=1: initial)
    params = {q: np.zeros((T, n), np.float32) for q in (0, 1)}
    order = sorted((r, q) for q in (0, 1) for r in range(T))

    def pub(q, v):
        return async_base(q, -1, n) if v == 1 else params[q][v - 2]

    for r, q in order:       # versions read never exceed the publisher's progress (v - 2 < r)
        got = check.read(q, r)
        params[q][r] = async_base(q, r, n) if got is None else \
            olerp.lerp_f32(async_base(q, r, n), pub(got[0], got[1]), check.policy(q, r)[0])
    expected = {}
    for q in (0, 1):
        expected.update(check.served(q, lambda v, q=q: pub(q, v), n))
    clocks = {q: np.array([check.clock_after(q, r) for r in range(T)]) for q in (0, 1)}
    for g in (0, 1):
        assert check.check_rank_digests(g, params[g], clocks[g], n, expected) == []
    torn = params[0].copy()
    torn[4, 7] += 1.0
    assert any("round 4" in b for b in check.check_rank_digests(0, torn, clocks[0], n, expected))


def test_bf16_training_add_matches_torch():
    """oracle.gossip.add_bf16 (the bf16 multi-process tests' training step) is torch's bf16
    add_ (no reference bf16 path exists; pinned to torch-eager like the bf16 lerp)."""
    from tests import dist_worker
    init, deltas, _, _ = dist_worker.inputs(2, 50_001, 3, dtype="bf16")
    for g in range(2):
        p = dist_worker.to_device(init[g].copy(), "cpu")     # from_numpy shares the array
        p.add_(dist_worker.to_device(deltas[1, g], "cpu"))
        assert np.array_equal(dist_worker.to_host(p), ogossip.add_bf16(init[g], deltas[1, g]))
