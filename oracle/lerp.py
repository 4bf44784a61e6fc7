"""Averaging arithmetic restated on the CPU -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Reference: dpwa/adapters/pytorch.py:68  ``param.data = factor * t + (1 - factor) * param.data``
evaluated by torch eager on fp32 tensors: a = f32(factor), b = f32(1.0 - factor) (the
subtraction happens in Python double), out = f32(f32(a*t) + f32(b*p)); no FMA.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libdpwa_oracle.so")
_lib = None


def coefficients(factor):
    """(a, b) exactly as torch eager forms them (pytorch.py:68)."""
    return np.float32(factor), np.float32(1.0 - float(factor))


def lerp_f32(param, peer, factor):
    """numpy restatement; returns a new array (pytorch.py:68 rebinds param.data)."""
    a, b = coefficients(factor)
    with np.errstate(all="ignore"):
        x = np.multiply(a, peer, dtype=np.float32)
        y = np.multiply(b, param, dtype=np.float32)
        return np.add(x, y, dtype=np.float32)


def bf16_to_f32(u16):
    return (np.asarray(u16, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


def f32_to_bf16(f32):
    """c10::BFloat16 round-to-nearest-even; NaN -> 0x7FC0."""
    u = np.asarray(f32, dtype=np.float32).view(np.uint32)
    r = ((u + np.uint32(0x7FFF) + ((u >> 16) & np.uint32(1))) >> 16).astype(np.uint16)
    nan = (u & np.uint32(0x7FFFFFFF)) > np.uint32(0x7F800000)
    r[nan] = 0x7FC0
    return r


def lerp_bf16(param_u16, peer_u16, factor):
    """torch-eager bf16 form: bf16(bf16(a*t) + bf16(b*p)); arrays hold raw bf16 bits."""
    a, b = coefficients(factor)
    with np.errstate(all="ignore"):
        x = bf16_to_f32(f32_to_bf16(a * bf16_to_f32(peer_u16)))
        y = bf16_to_f32(f32_to_bf16(b * bf16_to_f32(param_u16)))
        return f32_to_bf16(x + y)


def clib():
    """The C restatement (oracle/dpwa_oracle.c); builds it on first use if needed."""
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", _HERE])
        lib = ctypes.CDLL(_LIB_PATH)
        lib.dpwa_oracle_lerp_f32.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_double]
        lib.dpwa_oracle_lerp_bf16.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_double]
        lib.dpwa_oracle_publish.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
        lib.dpwa_oracle_factor.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                           ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                           ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]
        lib.dpwa_oracle_factor.restype = ctypes.c_int
        _lib = lib
    return _lib


def c_lerp_f32_(param, peer, factor):
    """In-place C restatement on contiguous float32 arrays."""
    assert param.dtype == np.float32 and peer.dtype == np.float32 and param.flags.c_contiguous
    assert peer.flags.c_contiguous and param.size == peer.size
    clib().dpwa_oracle_lerp_f32(param.ctypes.data, peer.ctypes.data, param.size, float(factor))
    return param


def c_lerp_bf16_(param_u16, peer_u16, factor):
    assert param_u16.dtype == np.uint16 and peer_u16.dtype == np.uint16
    assert param_u16.flags.c_contiguous and peer_u16.flags.c_contiguous and param_u16.size == peer_u16.size
    clib().dpwa_oracle_lerp_bf16(param_u16.ctypes.data, peer_u16.ctypes.data, param_u16.size, float(factor))
    return param_u16


def c_publish_(slot, flat):
    assert slot.nbytes == flat.nbytes
    clib().dpwa_oracle_publish(slot.ctypes.data, flat.ctypes.data, flat.nbytes)
    return slot


def bits_equal(x, y):
    """Bit equality with every NaN treated as equal (NaN payloads are not part of the contract)."""
    x = np.asarray(x)
    y = np.asarray(y)
    if x.dtype == np.uint16:
        xf, yf = bf16_to_f32(x), bf16_to_f32(y)
    else:
        xf, yf = x, y
    nx, ny = np.isnan(xf), np.isnan(yf)
    if not np.array_equal(nx, ny):
        return False
    if x.dtype == np.uint16:
        return bool(np.array_equal(x[~nx], y[~ny]))
    return bool(np.array_equal(x[~nx].view(np.uint32), y[~ny].view(np.uint32)))
