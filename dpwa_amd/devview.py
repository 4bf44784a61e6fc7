"""torch tensors over device memory the library owns (a learner's resident parameter slots).

The resident form keeps a learner's parameters in its own snapshot slots
(``dpwa_learner_set_resident``, include/dpwa_hip.h); the training loop needs them as a torch
tensor.  ``device_tensor`` wraps a device pointer through DLPack (``torch.from_dlpack`` of a
``dltensor`` capsule built here with ctypes): no copy, and torch never frees the memory -- the
descriptor has no deleter.  Each descriptor (80 bytes) lives in malloc'd memory that is never
freed, so torch may read it whenever it lets go of the tensor, interpreter shutdown included,
without calling back into Python (a learner makes two such views for its life).  The tensor
must not outlive the learner that owns the memory.
"""
import ctypes

import torch

KDL_CPU = 1
KDL_ROCM = 10             # DLPack's device type for AMD GPUs (torch maps it to "cuda")
_KDL_FLOAT, _KDL_BFLOAT = 2, 4


class DLDevice(ctypes.Structure):
    _fields_ = [("device_type", ctypes.c_int32), ("device_id", ctypes.c_int32)]


class DLDataType(ctypes.Structure):
    _fields_ = [("code", ctypes.c_uint8), ("bits", ctypes.c_uint8), ("lanes", ctypes.c_uint16)]


class DLTensor(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("device", DLDevice), ("ndim", ctypes.c_int32), ("dtype", DLDataType),
                ("shape", ctypes.POINTER(ctypes.c_int64)), ("strides", ctypes.POINTER(ctypes.c_int64)),
                ("byte_offset", ctypes.c_uint64)]


class DLManagedTensor(ctypes.Structure):
    pass


_DELETER = ctypes.CFUNCTYPE(None, ctypes.POINTER(DLManagedTensor))
DLManagedTensor._fields_ = [("dl_tensor", DLTensor), ("manager_ctx", ctypes.c_void_p), ("deleter", _DELETER)]

_DTYPES = {torch.float32: (_KDL_FLOAT, 32), torch.bfloat16: (_KDL_BFLOAT, 16), torch.uint8: (1, 8)}
_libc = ctypes.CDLL(None)
_libc.malloc.restype = ctypes.c_void_p
_libc.malloc.argtypes = [ctypes.c_size_t]
_DESC_BYTES = ctypes.sizeof(DLManagedTensor) + ctypes.sizeof(ctypes.c_int64)
made = [0]                # descriptors made (never freed)

_capsule_new = ctypes.pythonapi.PyCapsule_New
_capsule_new.restype = ctypes.py_object
_capsule_new.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]


def device_tensor(ptr, numel, dtype, device, device_type=KDL_ROCM):
    """A 1-D tensor of `numel` elements of `dtype` at device address `ptr` on `device` (a
    torch.device, or an int ordinal), sharing the memory."""
    if dtype not in _DTYPES:
        raise KeyError("device_tensor: unsupported dtype %s" % dtype)
    if not ptr and numel:
        raise ValueError("device_tensor: NULL pointer")
    index = device.index if isinstance(device, torch.device) else int(device)
    addr = _libc.malloc(_DESC_BYTES)
    if not addr:
        raise MemoryError("device_tensor: no memory for a DLPack descriptor")
    shape = ctypes.c_int64.from_address(addr + ctypes.sizeof(DLManagedTensor))
    shape.value = int(numel)
    m = DLManagedTensor.from_address(addr)
    code, bits = _DTYPES[dtype]
    m.dl_tensor = DLTensor(ctypes.c_void_p(ptr), DLDevice(device_type, index or 0), 1, DLDataType(code, bits, 1),
                           ctypes.pointer(shape), None, 0)
    m.manager_ctx = None
    m.deleter = _DELETER()          # NULL: torch frees nothing and calls nothing
    made[0] += 1
    return torch.utils.dlpack.from_dlpack(_capsule_new(addr, b"dltensor", None))
