"""The C-ABI library: loads, exports every symbol include/dpwa_hip.h declares, and its
structs match the header.  No compute calls (CPU container, no GPU)."""
import ctypes
import os
import re

import torch

from dpwa_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_loads_and_abi_version():
    lib = _lib.load()
    assert lib.dpwa_abi_version() == _lib.ABI_VERSION


def test_every_declared_symbol_is_exported():
    lib = _lib.load()
    declared = _lib.exported_symbols()
    assert len(declared) >= 30
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(_lib.SIGNATURES), set(declared) ^ set(_lib.SIGNATURES)


def test_struct_layouts():
    assert ctypes.sizeof(_lib.Header) == 256
    assert ctypes.sizeof(_lib.Coef) == 32
    assert ctypes.sizeof(_lib.Interp) == 24


def test_header_constants_match_binding():
    text = open(_lib.HEADER_PATH).read()
    consts = dict(re.findall(r"#define (DPWA_\w+) \(?(-?\d+)\)?", text))
    assert int(consts["DPWA_ABI_VERSION"]) == _lib.ABI_VERSION
    assert int(consts["DPWA_IPC_HANDLE_BYTES"]) == _lib.IPC_HANDLE_BYTES
    assert int(consts["DPWA_SLOT_PAYLOAD_OFFSET"]) == _lib.SLOT_PAYLOAD_OFFSET
    for c, v in [("DPWA_F32", _lib.F32), ("DPWA_BF16", _lib.BF16), ("DPWA_INTERP_LOSS", _lib.INTERP_LOSS),
                 ("DPWA_STATUS_ZERO_DIVISION", _lib.STATUS_ZERO_DIVISION), ("DPWA_REPLY_ERROR", _lib.REPLY_ERROR),
                 ("DPWA_PEER_DEAD", _lib.PEER_DEAD), ("DPWA_ERR_STATE", _lib.ERR_STATE)]:
        assert int(consts[c]) == v, c


def test_argument_errors_are_reported_not_crashing():
    lib = _lib.load()
    rc = lib.dpwa_lerp_f32(None, None, -1, None, None)
    assert rc == _lib.ERR_ARG
    assert b"dpwa_lerp_f32" in lib.dpwa_last_error()


def test_no_gpu_fails_loudly():
    """Without a device the product path raises instead of falling back to the CPU."""
    if torch.cuda.is_available():
        return
    import pytest
    from dpwa_amd.learner import Learner
    from dpwa_amd.interpolation import ConstantInterpolation
    with pytest.raises(_lib.DpwaError):
        Learner(torch.device("cuda", 0), 16, torch.float32, ConstantInterpolation(0.5).device_config(0.0))


def test_binding_arity_matches_header_declarations():
    """Every entry point's ctypes argument list has as many entries as its declaration in
    include/dpwa_hip.h has parameters (a signature changed on one side only would pass the
    symbol check and then misread its arguments)."""
    text = re.sub(r"/\*.*?\*/", "", open(_lib.HEADER_PATH).read(), flags=re.S)
    decls = re.findall(r"\b(?:int|int32_t|void|const char \*)\s*\**(dpwa_\w+)\s*\(([^)]*)\)\s*;", text)
    assert len(decls) >= 80
    for name, params in decls:
        params = params.strip()
        count = 0 if params in ("", "void") else params.count(",") + 1
        assert name in _lib.SIGNATURES, name
        assert len(_lib.SIGNATURES[name]) == count, (name, count, len(_lib.SIGNATURES[name]))


def test_trace_switch_is_read_at_load():
    """roctx ranges (include/dpwa_hip.h dpwa_trace_*): off unless DPWA_ROCTX=1 when the library
    loads; on, push/pop go through the profiler SDK's roctx (no-ops without a profiler), and the
    Python layer's switch follows the same variable.  Separate processes: the switch is fixed at load."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); from dpwa_amd import _lib; lib = _lib.load(); "
            "print(lib.dpwa_trace_enabled(), lib.dpwa_trace_push(b'x'), lib.dpwa_trace_pop(), int(_lib.TRACE))"
            % ROOT)
    outs = []
    for on in ("0", "1"):
        env = dict(os.environ, DPWA_ROCTX=on)
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)
        assert r.returncode == 0, r.stderr
        outs.append(r.stdout.split())
    assert outs[0] == ["0", "0", "0", "0"]
    assert outs[1] == ["1", "0", "0", "1"], outs[1]
