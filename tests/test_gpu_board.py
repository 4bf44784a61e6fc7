"""The gossip board's stream-ordered release on the GPU (dpwa_amd/csrc/board.cpp).

A reader clears its read mark from its side stream after the pull, while its host may already
be in the next round.  When the next round picks the same publisher, the new mark must survive
that still-queued clear of the old one -- otherwise the publisher sees no reader and rewrites
the slot mid-pull (a torn snapshot averaged without any error)."""
import ctypes
import os

import pytest
import torch

from dpwa_amd import _lib

pytestmark = pytest.mark.gpu


def _open(name, world, rank, create):
    b = ctypes.c_void_p()
    _lib.call("dpwa_board_open", ctypes.byref(b), name.encode(), world, rank, 1 if create else 0)
    return b


def _acquire(b, r):
    v = ctypes.c_uint64()
    _lib.call("dpwa_board_acquire", b, r, ctypes.byref(v))
    return v.value


def _mark(b, r):
    v, mark, alive = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int32()
    _lib.call("dpwa_board_read", b, r, ctypes.byref(v), ctypes.byref(mark), ctypes.byref(alive))
    return mark.value


def test_reacquire_survives_a_pending_stream_release():
    name = "/dpwa_test_gpu_%d_%s" % (os.getpid(), os.urandom(4).hex())
    b0 = _open(name, 2, 0, True)          # the publisher (host-side advertise)
    b1 = _open(name, 2, 1, False)         # the reader (stream-side release)
    _lib.call("dpwa_board_unlink", name.encode())
    try:
        _lib.call("dpwa_board_register", b1, 0)
        side = torch.cuda.Stream()
        _lib.call("dpwa_board_advertise", b0, 1, None, 1)
        assert _acquire(b1, 0) == 1
        with torch.cuda.stream(side):
            torch.cuda._sleep(200_000_000)                     # a long "pull" on the side stream
        _lib.call("dpwa_board_release", b1, 0, ctypes.c_void_p(side.cuda_stream), 0)
        _lib.call("dpwa_board_publish_wait", b0, 2, 0)
        _lib.call("dpwa_board_advertise", b0, 2, None, 1)
        assert _acquire(b1, 0) == 2        # waits for the queued clear of mark 1 before setting 2
        torch.cuda.synchronize()
        assert _mark(b1, 0) == 2           # the old clear did not wipe the new mark
        _lib.call("dpwa_board_publish_wait", b0, 3, 0)
        _lib.call("dpwa_board_advertise", b0, 3, None, 1)
        # publish 4 rewrites snapshot 2's slot, which rank 1 still reads: the publisher waits
        with pytest.raises(_lib.DpwaError, match="still reads snapshot 2"):
            _lib.call("dpwa_board_publish_wait", b0, 4, 50)
        _lib.call("dpwa_board_release", b1, 0, ctypes.c_void_p(side.cuda_stream), 0)
        torch.cuda.synchronize()
        _lib.call("dpwa_board_publish_wait", b0, 4, 1000)
    finally:
        torch.cuda.synchronize()
        _lib.call("dpwa_board_close", b1)
        _lib.call("dpwa_board_close", b0)
