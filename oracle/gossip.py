"""Lock-step G-learner gossip on the CPU -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

One round per learner g, as the reference's README loop runs it (README.md:18-29):
``update_send(loss)`` (adapters/pytorch.py:42-53 -> dpwa.py:104-123) publishes a copy of
the parameters plus ``{clock, loss}``, draws the Bernoulli gate; the training step
changes the parameters; ``update_wait(loss)`` (pytorch.py:55-68 -> dpwa.py:125-156)
fetches one peer's published snapshot chosen by TxThread (conn.py:224-317), computes
the factor/clock and averages.  "Lock-step" = every learner publishes round r before
any fetch of round r is served, which is the schedule the GPU gossip group runs.
"""
import numpy as np

from .lerp import bf16_to_f32, f32_to_bf16, lerp_f32
from .policy import OracleLearner


def add_bf16(param_u16, delta_u16):
    """torch's bf16 ``param.add_(delta)``: both widened to fp32, one fp32 add, rounded to
    bf16 (RNE); arrays hold raw bf16 bits."""
    with np.errstate(all="ignore"):
        return f32_to_bf16(bf16_to_f32(param_u16) + bf16_to_f32(delta_u16))


def simulate(names, init, deltas, send_loss, wait_loss, method, value, threshold, fetch_probability,
             seeds, lerp=lerp_f32, add=None, train_after_wait=False, nodes=None, serves=None):
    """init (G, n) and deltas (T, G, n): fp32 arrays, or raw bf16 bits (uint16) with
    lerp=lerp_bf16, add=add_bf16.  train_after_wait: round r's training delta is applied after
    its update_wait instead of between update_send and update_wait (the order a loop with
    resident parameters must keep: update_send, update_wait, training step); out_params then
    holds the parameters after the average, before that delta.

    nodes (default `names`): the YAML's node list; each learner's peers are the nodes other than
    itself, by name (dpwa.py:65-72).  serves (default: each learner by its own name): node name ->
    index of the learner whose RxThread answers at that node's address -- TxThread dials
    (host, port) (conn.py:246-251), so a node entry at a learner's own address is that learner;
    {"w1-self": 0} with nodes ["w1", "w1-self"] is configs[1]'s self-peer."""
    G, n = init.shape
    T = deltas.shape[0]
    nodes = list(names) if nodes is None else list(nodes)
    idx = {nm: i for i, nm in enumerate(names)}
    if serves is not None:
        idx.update(serves)
    learners = [OracleLearner(names[g], [x for x in nodes if x != names[g]], fetch_probability,
                              method, value, threshold, seeds[g]) for g in range(G)]
    params = init.copy()
    out_params = np.zeros((T, G, n), init.dtype)
    clocks = np.zeros((T, G))
    factors = np.zeros((T, G))
    fetching = np.zeros((T, G), bool)
    picks = [[None] * G for _ in range(T)]
    for r in range(T):
        states, snaps = [], []
        for g in range(G):
            states.append(learners[g].update_send(send_loss[r][g]))
            snaps.append(params[g].copy())
            fetching[r, g] = learners[g].fetching
        def train():
            for g in range(G):
                params[g] = (np.add(params[g], deltas[r, g], dtype=params.dtype) if add is None
                             else add(params[g], deltas[r, g]))
        if not train_after_wait:
            train()
        for g in range(G):
            L = learners[g]
            state, payload, attempts = None, None, []
            if L.fetching:
                state, payload, attempts = L.fetch(
                    lambda peer: "ok",
                    lambda peer: ("payload", states[idx[peer]], snaps[idx[peer]]))
            averaged, factor = L.update_wait(wait_loss[r][g], state, payload is not None)
            if averaged:
                params[g] = lerp(params[g], payload, factor)
            picks[r][g] = [a["peer"] for a in attempts]
            factors[r, g] = factor
            clocks[r, g] = L.clock
            out_params[r, g] = params[g]
        if train_after_wait:
            train()
    return {"params": out_params, "clocks": clocks, "factors": factors, "fetching": fetching, "picks": picks}
