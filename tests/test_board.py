"""The gossip board (dpwa_amd/csrc/board.cpp) on the CPU: the free-running protocol that
replaces the reference's RxThread server and its publish Lock (conn.py:73-79, 98-110) and
its refused connections (conn.py:253-256).  Host-side advertise/release stand in for the
stream writes the GPU path uses; the protocol logic is the same code."""
import ctypes
import multiprocessing as mp
import os

import numpy as np
import pytest

from dpwa_amd import _lib


def _name():
    return "/dpwa_test_%d_%s" % (os.getpid(), os.urandom(4).hex())


def _open(name, world, rank, create):
    b = ctypes.c_void_p()
    _lib.call("dpwa_board_open", ctypes.byref(b), name.encode(), world, rank, 1 if create else 0)
    return b


def _status(b, r):
    st = ctypes.c_int32()
    _lib.call("dpwa_board_status", b, r, ctypes.byref(st))
    return st.value


def _acquire(b, r):
    v = ctypes.c_uint64()
    _lib.call("dpwa_board_acquire", b, r, ctypes.byref(v))
    return v.value


def _read(b, r):
    v, mark, alive = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int32()
    _lib.call("dpwa_board_read", b, r, ctypes.byref(v), ctypes.byref(mark), ctypes.byref(alive))
    return v.value, mark.value, alive.value


def test_states_acquire_release_and_publish_lock():
    name = _name()
    b0 = _open(name, 2, 0, True)
    b1 = _open(name, 2, 1, False)
    _lib.call("dpwa_board_unlink", name.encode())
    try:
        assert _status(b1, 0) == _lib.PEER_NO_STATE        # empty reply before the first publish
        assert _acquire(b1, 0) == 0
        _lib.call("dpwa_board_publish_wait", b0, 1, 0)
        _lib.call("dpwa_board_advertise", b0, 1, None, 1)
        assert _status(b1, 0) == _lib.PEER_READY
        assert _acquire(b1, 0) == 1
        assert _read(b1, 0) == (1, 1, 1)
        _lib.call("dpwa_board_publish_wait", b0, 2, 0)        # publish 2 rewrites no slot in use
        _lib.call("dpwa_board_advertise", b0, 2, None, 1)
        # publish 3 rewrites publish 1's slot, which rank 1 still reads: the Lock holds
        with pytest.raises(_lib.DpwaError, match="still reads snapshot 1"):
            _lib.call("dpwa_board_publish_wait", b0, 3, 30)
        _lib.call("dpwa_board_release", b1, 0, None, 1)
        _lib.call("dpwa_board_publish_wait", b0, 3, 0)
        # publish 4 before publish 3 is out is out of order
        with pytest.raises(_lib.DpwaError, match="never completed"):
            _lib.call("dpwa_board_publish_wait", b0, 4, 10)
    finally:
        _lib.call("dpwa_board_close", b1)
    assert _status(b0, 1) == _lib.PEER_DOWN                 # closed: ConnectionRefusedError
    _lib.call("dpwa_board_close", b0)


def test_open_errors():
    with pytest.raises(_lib.DpwaError):
        _open("/dpwa_test_missing_%s" % os.urandom(4).hex(), 2, 1, False)
    with pytest.raises(_lib.DpwaError):
        _open("no_slash", 2, 0, True)
    name = _name()
    b0 = _open(name, 3, 0, True)
    try:
        with pytest.raises(_lib.DpwaError, match="not a board for 2 ranks"):
            _open(name, 2, 1, False)
    finally:
        _lib.call("dpwa_board_unlink", name.encode())
        _lib.call("dpwa_board_close", b0)


def _die_reading(name):
    b = _open(name, 2, 1, False)
    assert _acquire(b, 0) == 1
    os._exit(0)          # dies holding the read mark, without closing


def test_dead_reader_does_not_block_and_reads_as_refused():
    name = _name()
    b0 = _open(name, 2, 0, True)
    try:
        _lib.call("dpwa_board_advertise", b0, 1, None, 1)
        p = mp.get_context("fork").Process(target=_die_reading, args=(name,))
        p.start()
        p.join(30)
        assert p.exitcode == 0
        _lib.call("dpwa_board_advertise", b0, 2, None, 1)
        v, _, alive = _read(b0, 1)
        assert alive == 0 and _status(b0, 1) == _lib.PEER_DOWN
        _lib.call("dpwa_board_publish_wait", b0, 3, 1000)      # the dead reader's mark is ignored
    finally:
        _lib.call("dpwa_board_unlink", name.encode())
        _lib.call("dpwa_board_close", b0)


SLOT_ELEMS = 4096


def _publisher(name, shm_name, rounds):
    from multiprocessing import shared_memory
    shm = shared_memory.SharedMemory(name=shm_name)
    slots = np.ndarray((2, SLOT_ELEMS), dtype=np.int64, buffer=shm.buf)
    b = _open(name, 2, 0, False)
    for v in range(1, rounds + 1):
        _lib.call("dpwa_board_publish_wait", b, v, 20000)
        slots[(v - 1) % 2, :] = v             # the publish: rewrites the slot of v - 2
        _lib.call("dpwa_board_advertise", b, v, None, 1)
    _lib.call("dpwa_board_close", b)
    del slots
    shm.close()


def test_free_running_reader_never_sees_a_torn_snapshot():
    """A publisher rewriting its two slots as fast as it can and a reader pulling them: every
    acquired version reads back whole (the WAR rule of the reference's Lock), and the
    versions a reader sees never go backwards."""
    from multiprocessing import shared_memory
    name = _name()
    shm = shared_memory.SharedMemory(create=True, size=2 * SLOT_ELEMS * 8)
    slots = np.ndarray((2, SLOT_ELEMS), dtype=np.int64, buffer=shm.buf)
    slots[:] = 0
    b0 = _open(name, 2, 0, True)      # rank 0's entry is re-opened by the publisher process
    b1 = _open(name, 2, 1, False)
    _lib.call("dpwa_board_close", b0)
    rounds = 3000
    p = mp.get_context("fork").Process(target=_publisher, args=(name, shm.name, rounds))
    p.start()
    try:
        seen, last = 0, 0
        while True:
            v = _acquire(b1, 0)
            if v:
                assert v >= last
                last = v
                for _ in range(3):        # a slow pull: read the slot several times
                    snap = slots[(v - 1) % 2].copy()
                    assert (snap == v).all(), (v, np.unique(snap))
                seen += 1
                _lib.call("dpwa_board_release", b1, 0, None, 1)
            if last == rounds or not p.is_alive():   # a closed publisher hands out nothing more
                break
        p.join(60)
        assert p.exitcode == 0
        assert seen > 10 and last > rounds // 4
    finally:
        _lib.call("dpwa_board_unlink", name.encode())
        _lib.call("dpwa_board_close", b1)
        del slots
        shm.close()
        shm.unlink()
