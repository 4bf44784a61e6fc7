"""The import-compatible `dpwa` package: a script written against the reference imports the
MI355X implementation unchanged (CPU: construction and framing only)."""
import socket

from tests.helpers import load_json


def test_reference_imports_resolve_here():
    import dpwa_amd
    from dpwa.adapters.pytorch import DpwaPyTorchAdapter
    from dpwa.dpwa import DpwaConfiguration, DpwaConnection
    from dpwa.interpolation import ClockWeightedInterpolation, ConstantInterpolation, LossInterpolation
    assert DpwaPyTorchAdapter is dpwa_amd.DpwaPyTorchAdapter
    assert DpwaConnection is dpwa_amd.DpwaConnection
    assert DpwaConfiguration.__module__ == "dpwa_amd.dpwa"
    assert ConstantInterpolation(0.5)(1, 2, 3, 4) == 0.5
    assert ClockWeightedInterpolation()(1, 3, 0, 0) == 0.75
    assert LossInterpolation()(1.0, 3.0, 1.0, 3.0) == 0.25


def test_messaging_names_frame_like_the_reference():
    import threading

    from dpwa.messaging import HEADER_LEN, recv_message, send_message
    assert HEADER_LEN == load_json("wire.json")["header_len"]
    for rec in load_json("wire.json")["samples"]:
        payload = None if rec["payload_hex"] is None else bytes.fromhex(rec["payload_hex"])
        a, b = socket.socketpair()
        try:
            th = threading.Thread(target=send_message, args=(a, rec["type"], rec["message"], payload))
            th.start()
            got = recv_message(b)
            th.join()
        finally:
            a.close()
            b.close()
        d = rec["decoded"]
        assert got[0] == d["type"] and got[1] == d["message"]
        assert (got[2].hex() if got[2] is not None else None) == d["payload_hex"]


def test_conn_constants_and_scheduler_bounds():
    """dpwa.conn's constants (conn.py:34, 40, 178-181), and the native scheduler honours the
    flow-control ones: a refused peer drops by DEC to no lower than MIN, a reply lifts it by
    INC up to MAX."""
    from dpwa.conn import (FLOW_CONTROL_DEC_SCORE, FLOW_CONTROL_INC_SCORE, FLOW_CONTROL_MAX_SCORE,
                           FLOW_CONTROL_MIN_SCORE, MESSAGE_TYPE_FETCH_PARAMETERS, TCP_SOCKET_BUFFER_SIZE)
    from dpwa_amd.sched import Scheduler
    assert (MESSAGE_TYPE_FETCH_PARAMETERS, TCP_SOCKET_BUFFER_SIZE) == (1, 8 * 1024 * 1024)
    s = Scheduler(1, seed=3)
    assert s.score(0) == FLOW_CONTROL_MAX_SCORE
    want = FLOW_CONTROL_MAX_SCORE
    for _ in range(12):
        peer, connected = s.pick()
        assert peer == 0 and not connected
        s.report(0, "refused")
        want = max(want - FLOW_CONTROL_DEC_SCORE, FLOW_CONTROL_MIN_SCORE)
        assert s.score(0) == want
    peer, connected = s.pick()
    s.report(0, "connect_ok")
    s.report(0, "payload")
    assert s.score(0) == min(want + FLOW_CONTROL_INC_SCORE, FLOW_CONTROL_MAX_SCORE)
