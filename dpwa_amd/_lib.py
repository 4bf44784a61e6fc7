"""ctypes binding of libdpwa_hip.so (the C ABI declared in include/dpwa_hip.h).

This is the reference-side binding a maintainer would add: plain
pointers, sizes and opaque handles.  There is no fallback -- if the library is missing
or cannot be loaded, every entry point raises :class:`DpwaLibraryError`.

``torch`` is imported before the library is loaded so that the process has exactly one
HIP runtime: torch's bundled ``libamdhip64.so`` carries the soname ``libamdhip64.so.7``
that libdpwa_hip.so was linked against.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the dlopen below: one HIP runtime per process)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DPWA_HIP_LIB", os.path.join(_HERE, "libdpwa_hip.so"))
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "dpwa_hip.h")

# Constants mirrored from include/dpwa_hip.h
ABI_VERSION = 10
OK, ERR_ARG, ERR_HIP, ERR_STATE, ERR_NOMEM = 0, -1, -2, -3, -4
F32, BF16, F64 = 0, 1, 2
INTERP_CONSTANT, INTERP_CLOCK, INTERP_LOSS = 0, 1, 2
STATUS_OK, STATUS_ZERO_DIVISION = 0, 1
IPC_HANDLE_BYTES = 128
SLOT_PAYLOAD_OFFSET = 4096   # [dpwa_header | pad | payload]
CONNECT_OK, CONNECT_REFUSED, CONNECT_ERROR = 0, 1, 2
REPLY_PAYLOAD, REPLY_EMPTY, REPLY_TIMEOUT, REPLY_ERROR = 3, 4, 5, 6
PEER_READY, PEER_NO_STATE, PEER_DOWN, PEER_SLOW, PEER_DEAD = 0, 1, 2, 3, 4
NODE_PEER_UNSET, NODE_PEER_LOCAL, NODE_PEER_REMOTE = 0, 1, 2
PULL_COPY_ENGINE, PULL_KERNEL = 0, 1
FETCH_ZERO_COPY, FETCH_PUBLISHED, FETCH_RESCUE = 1, 2, 4
FETCH_LANDED, FETCH_IN_FLIGHT, FETCH_TIMED_OUT = 0, 1, 2
FLAG_EAGER, FLAG_ZERO_COPY, FLAG_REUSE_SNAPSHOT, FLAG_WRITE_THROUGH, FLAG_PICK_ONLY = 1, 2, 4, 8, 16


class DpwaLibraryError(RuntimeError):
    pass


class DpwaError(RuntimeError):
    """A libdpwa_hip call returned a negative status."""

    def __init__(self, fn, code, msg):
        super().__init__("%s failed (%d): %s" % (fn, code, msg))
        self.code = code


class Header(ctypes.Structure):
    _fields_ = [("clock", ctypes.c_double), ("loss", ctypes.c_double), ("version", ctypes.c_uint64),
                ("n", ctypes.c_int64), ("dtype", ctypes.c_int32), ("reserved0", ctypes.c_int32),
                ("pad", ctypes.c_uint8 * 216)]


class Coef(ctypes.Structure):
    _fields_ = [("factor", ctypes.c_double), ("new_clock", ctypes.c_double), ("a", ctypes.c_float),
                ("b", ctypes.c_float), ("status", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class AverageDesc(ctypes.Structure):
    _fields_ = [("param", ctypes.c_void_p), ("peer_slot", ctypes.c_void_p), ("n", ctypes.c_int64),
                ("clock_dev", ctypes.c_void_p), ("loss", ctypes.c_double), ("coef_dev", ctypes.c_void_p),
                ("snap_payload", ctypes.c_void_p)]


class Interp(ctypes.Structure):
    _fields_ = [("method", ctypes.c_int32), ("reserved", ctypes.c_int32), ("value", ctypes.c_double),
                ("divergence_threshold", ctypes.c_double)]


_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_int = ctypes.c_int
_dbl = ctypes.c_double
_u64 = ctypes.c_uint64
_pint = ctypes.POINTER(ctypes.c_int)

# name -> argtypes (every function returns int status unless listed in _RESTYPES)
SIGNATURES = {
    "dpwa_last_error": [],
    "dpwa_abi_version": [],
    "dpwa_sched_get_state": [_vp, ctypes.POINTER(ctypes.c_uint32), _int, _pint],
    "dpwa_sched_set_state": [_vp, ctypes.POINTER(ctypes.c_uint32), _int],
    "dpwa_trace_enabled": [],
    "dpwa_trace_push": [ctypes.c_char_p],
    "dpwa_trace_pop": [],
    "dpwa_last_words_set": [ctypes.c_int, ctypes.c_char_p, ctypes.c_int64],
    "dpwa_last_words_flush": [ctypes.POINTER(ctypes.c_int)],
    "dpwa_last_words_written": [ctypes.POINTER(ctypes.c_int)],
    "dpwa_lerp_f32": [_vp, _vp, _i64, _vp, _vp],
    "dpwa_lerp_bf16": [_vp, _vp, _i64, _vp, _vp],
    "dpwa_lerp_f32_host": [_vp, _vp, _i64, _dbl, _vp],
    "dpwa_lerp_bf16_host": [_vp, _vp, _i64, _dbl, _vp],
    "dpwa_factor": [ctypes.POINTER(Interp), _vp, _vp, _dbl, _vp, _vp, _vp],
    "dpwa_average": [_i32, _vp, _vp, _i64, ctypes.POINTER(Interp), _vp, _dbl, _vp, _vp, _vp, _vp, _vp],
    "dpwa_average_many": [_i32, _vp, _int, ctypes.POINTER(Interp), _vp, _vp, _vp],
    "dpwa_average_many_resident": [_i32, _vp, _int, ctypes.POINTER(Interp), _vp, _vp, _vp],
    "dpwa_learner_average_many": [_vp, _vp, _vp, _vp, _vp, _int, _vp],
    "dpwa_learner_set_header_publish": [_vp, _int],
    "dpwa_learner_set_reuse_guard": [_vp, _int],
    "dpwa_learner_reuse_guard_hits": [_vp, ctypes.POINTER(ctypes.c_uint32)],
    "dpwa_learner_window_hits": [_vp, ctypes.POINTER(ctypes.c_uint32)],
    "dpwa_learner_set_resident": [_vp, _vp, _vp],
    "dpwa_learner_resident_params": [_vp, ctypes.POINTER(_vp), _pint],
    "dpwa_learner_relocate": [_vp, _vp],
    "dpwa_node_set_resident": [_vp, _vp, _vp],
    "dpwa_learner_fetch_state": [_vp, _i64, _pint],
    "dpwa_stream_mix": [_vp, ctypes.c_int, _vp, ctypes.c_int, ctypes.c_int64, _vp, _vp, _vp],
    "dpwa_learner_rescue_free": [_vp, _pint],
    "dpwa_learner_rescue_lanes": [_vp, _pint, _pint],
    "dpwa_learner_set_rescue_cap": [_vp, ctypes.c_int],
    "dpwa_learner_fetch_stream": [_vp, ctypes.POINTER(_vp)],
    "dpwa_learner_copy_factor": [_vp, _vp, _vp],
    "dpwa_learner_copy_fetched": [_vp, _vp, _vp],
    "dpwa_learner_create": [ctypes.POINTER(_vp), _int, _i64, _i32, ctypes.POINTER(Interp)],
    "dpwa_learner_destroy": [_vp],
    "dpwa_learner_publish": [_vp, _vp, _dbl, _vp, _vp],
    "dpwa_learner_version": [_vp, ctypes.POINTER(_u64)],
    "dpwa_learner_attach_local": [_vp, _int, _vp],
    "dpwa_learner_ipc_handle": [_vp, _vp, _i64],
    "dpwa_learner_attach_ipc": [_vp, _int, _vp, _i64],
    "dpwa_learner_export_fds": [_vp, _int, _pint, _int, _pint, ctypes.POINTER(_i64)],
    "dpwa_learner_attach_fds": [_vp, _int, _vp, _i64, _pint, _int, _i64],
    "dpwa_learner_fetch": [_vp, _int, _u64, _int, _vp],
    "dpwa_learner_average": [_vp, _vp, _dbl, _vp, _vp],
    "dpwa_learner_average_through": [_vp, _vp, _dbl, _vp, _vp],
    "dpwa_learner_publish_reuse": [_vp, _vp, _dbl, _vp, _vp],
    "dpwa_learner_factor": [_vp, _dbl, _vp, _vp],
    "dpwa_learner_lerp": [_vp, _vp, _vp],
    "dpwa_learner_cancel": [_vp],
    "dpwa_learner_set_pull": [_vp, _int, _int],
    "dpwa_learner_set_loss_dtype": [_vp, _i32],
    "dpwa_learner_wait_fetch": [_vp, _vp],
    "dpwa_learner_read_snapshot": [_vp, _vp, _vp, _i64, ctypes.POINTER(_u64)],
    "dpwa_learner_relay_enable": [_vp, _int, _int],
    "dpwa_learner_relay_handle": [_vp, _vp, _i64],
    "dpwa_learner_relay_attach": [_vp, _int, _int, _vp, _i64],
    "dpwa_learner_relay_attach_fds": [_vp, _int, _int, _vp, _i64, _pint, _int, _i64],
    "dpwa_learner_relay_wait": [_vp, _vp],
    "dpwa_learner_relay_phase1": [_vp, _vp, _u64, _int, _vp],
    "dpwa_learner_relay_phase2": [_vp, _vp, _int, _u64, _int, _int],
    "dpwa_learner_side_stream": [_vp, ctypes.POINTER(_vp)],
    "dpwa_learner_time_fetches": [_vp, _int],
    "dpwa_learner_read_fetch_times": [_vp, ctypes.POINTER(ctypes.c_float), _int, ctypes.POINTER(_int)],
    "dpwa_learner_time_averages": [_vp, _int],
    "dpwa_learner_arm_timing": [_vp],
    "dpwa_learner_read_average_times": [_vp, ctypes.POINTER(ctypes.c_float), _int, ctypes.POINTER(_int)],
    "dpwa_learner_fetch_host": [_vp, _vp, _vp, _i64, _vp],
    "dpwa_learner_pointers": [_vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_vp),
                              ctypes.POINTER(_vp)],
    "dpwa_learner_status_word": [_vp, ctypes.POINTER(_vp)],
    "dpwa_learner_read_clock": [_vp, ctypes.POINTER(_dbl)],
    "dpwa_learner_write_clock": [_vp, _dbl],
    "dpwa_learner_read_coef": [_vp, ctypes.POINTER(Coef)],
    "dpwa_learner_poll_status": [_vp, _pint, ctypes.POINTER(_i32)],
    "dpwa_node_create": [ctypes.POINTER(_vp), _int, ctypes.POINTER(ctypes.c_uint32), _int, _dbl,
                         ctypes.POINTER(Interp)],
    "dpwa_node_destroy": [_vp],
    "dpwa_node_bind": [_vp, _int, _i64, _i32],
    "dpwa_node_handles": [_vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp)],
    "dpwa_node_set_peer": [_vp, _int, _int, _vp],
    "dpwa_node_set_fault": [_vp, _int, _int],
    "dpwa_node_set_board": [_vp, _vp, ctypes.POINTER(_i32), _int],
    "dpwa_node_set_timeout": [_vp, _int],
    "dpwa_board_open": [ctypes.POINTER(_vp), ctypes.c_char_p, _int, _int, _int],
    "dpwa_board_unlink": [ctypes.c_char_p],
    "dpwa_board_close": [_vp],
    "dpwa_board_register": [_vp, _int],
    "dpwa_board_status": [_vp, _int, ctypes.POINTER(_i32)],
    "dpwa_board_read": [_vp, _int, ctypes.POINTER(_u64), ctypes.POINTER(_u64), ctypes.POINTER(_i32)],
    "dpwa_board_acquire": [_vp, _int, ctypes.POINTER(_u64)],
    "dpwa_board_release": [_vp, _int, _vp, _int],
    "dpwa_board_publish_wait": [_vp, _u64, _int],
    "dpwa_board_advertise": [_vp, _u64, _vp, _int],
    "dpwa_node_update_send": [_vp, _vp, _dbl, _vp, _int, _vp, _pint],
    "dpwa_node_publish": [_vp, _vp, _dbl, _vp, _int, _vp],
    "dpwa_node_gate": [_vp, _int, _vp, _pint],
    "dpwa_node_start_fetch": [_vp, _int, _vp],
    "dpwa_node_update_wait": [_vp, _dbl, _vp, _int, _vp, _pint],
    "dpwa_node_lerp": [_vp, _vp, _vp],
    "dpwa_node_update_wait_average": [_vp, _vp, _dbl, _vp, _int, _vp, _pint],
    "dpwa_node_update_wait_average_many": [_vp, _vp, _vp, _vp, _int, _int, _vp, _vp],
    "dpwa_node_info": [_vp, _pint, _pint, ctypes.POINTER(_u64), _pint],
    "dpwa_sched_create": [ctypes.POINTER(_vp), _int, ctypes.POINTER(ctypes.c_uint32), _int, _dbl],
    "dpwa_sched_destroy": [_vp],
    "dpwa_sched_bernoulli": [_vp, _pint],
    "dpwa_sched_pick": [_vp, _pint, _pint],
    "dpwa_sched_report": [_vp, _int, _int, _pint, _pint],
    "dpwa_sched_fetch": [_vp, ctypes.POINTER(_i32), _int, _pint, _pint],
    "dpwa_sched_score": [_vp, _int, _pint],
    "dpwa_sched_remove": [_vp, _int],
    "dpwa_sched_add": [_vp, _int],
    "dpwa_sched_n_live": [_vp, _pint],
    "dpwa_sched_random": [_vp, ctypes.POINTER(_dbl)],
    "dpwa_sched_randint": [_vp, _i64, _i64, ctypes.POINTER(_i64)],
}
_RESTYPES = {"dpwa_last_error": ctypes.c_char_p}

_lib = None
_load_error = None


def load():
    """Loads (once) and returns the CDLL; raises DpwaLibraryError if it is unavailable."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise DpwaLibraryError(_load_error)
    if not os.path.exists(LIB_PATH):
        _load_error = ("libdpwa_hip.so not found at %s -- build it first "
                       "(python -c 'import __graft_entry__ as g; g.build()' or make -C dpwa_amd/csrc)" % LIB_PATH)
        raise DpwaLibraryError(_load_error)
    try:
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    except OSError as e:
        _load_error = "cannot load %s: %s" % (LIB_PATH, e)
        raise DpwaLibraryError(_load_error) from e
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = _RESTYPES.get(name, ctypes.c_int)
    if lib.dpwa_abi_version() != ABI_VERSION:
        _load_error = "ABI mismatch: library %d, binding %d" % (lib.dpwa_abi_version(), ABI_VERSION)
        raise DpwaLibraryError(_load_error)
    _lib = lib
    return lib


# roctx ranges (include/dpwa_hip.h dpwa_trace_*): read once, like the library does at load
TRACE = os.environ.get("DPWA_ROCTX") == "1"


class trace_range:
    """A named roctx range over a `with` block (only used when TRACE is set)."""

    def __init__(self, name):
        self.name = name.encode()

    def __enter__(self):
        load().dpwa_trace_push(self.name)
        return self

    def __exit__(self, *exc):
        load().dpwa_trace_pop()
        return False


def last_words(fd, line):
    """Registers `line` (str; "" clears it) to be written to `fd` if the process is ended by a
    signal or dies by one (include/dpwa_hip.h dpwa_last_words_set)."""
    data = line.encode() if line else b""
    call("dpwa_last_words_set", int(fd) if data else -1, data or None, len(data))


def last_words_flush():
    """Writes the registered line now, unless a signal already did; True when this call wrote it."""
    w = ctypes.c_int()
    call("dpwa_last_words_flush", ctypes.byref(w))
    return bool(w.value)


def last_words_written():
    w = ctypes.c_int()
    call("dpwa_last_words_written", ctypes.byref(w))
    return bool(w.value)


def call(name, *args):
    """Calls `name`, raising DpwaError on a negative status."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc < 0:
        raise DpwaError(name, rc, lib.dpwa_last_error().decode(errors="replace"))
    return rc


def exported_symbols():
    """Names every `dpwa_*` function declared in include/dpwa_hip.h."""
    import re
    with open(HEADER_PATH) as f:
        text = f.read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(dpwa_\w+)\s*\(", text, re.M)))


def stream_handle(stream):
    """hipStream_t of a torch stream (None -> the current stream of the current device)."""
    if stream is None:
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)
