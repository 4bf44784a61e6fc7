"""Python handle of one device-resident learner (dpwa_learner in include/dpwa_hip.h).

A learner owns two snapshot slots, a staging buffer and the device clock/coefficient
block on its GPU; this class only forwards torch tensors and streams to the C ABI.
It sits on the per-round path, so it keeps host work small: raw ctypes function
objects, a Python-side publish counter, validation only when the tensor changes.
"""
import ctypes

import torch

from . import _lib

DTYPES = {torch.float32: _lib.F32, torch.bfloat16: _lib.BF16}

_c_void_p = ctypes.c_void_p
MAX_FDS = 240          # chunks (1 GiB each) one exported allocation may have; < SCM_MAX_FD (253)


def loss_args(loss, device):
    """(host double, device pointer or None, keep-alive) for a loss given as a number or a
    device tensor (a device tensor is read by the kernels without a host sync)."""
    if isinstance(loss, torch.Tensor):
        if loss.device.type == "cuda":
            t = loss.detach().to(device=device, dtype=torch.float64).reshape(())
            return 0.0, _c_void_p(t.data_ptr()), t
        return float(loss.item()), None, None
    return float(loss), None, None


class Learner:
    def __init__(self, device, numel, dtype, interp_cfg=None, handle=None):
        """Creates a learner, or wraps (without owning) `handle` from dpwa_node_handles."""
        if dtype not in DTYPES:
            raise KeyError("dpwa averages float32 or bfloat16 parameters, got %s" % dtype)
        self.device = torch.device(device)
        self.numel = int(numel)
        self.dtype = dtype
        lib = _lib.load()
        self._lib = lib
        self._owned = handle is None
        if handle is None:
            self._h = ctypes.c_void_p()
            _lib.call("dpwa_learner_create", ctypes.byref(self._h), self.device.index, self.numel, DTYPES[dtype],
                      ctypes.byref(interp_cfg))
        else:
            self._h = ctypes.c_void_p(handle)
        clock, coef, sh, sp = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
        _lib.call("dpwa_learner_pointers", self._h, ctypes.byref(clock), ctypes.byref(coef), ctypes.byref(sh),
                  ctypes.byref(sp))
        self.coef_ptr = coef.value
        self.staging_header_ptr, self.staging_payload_ptr = sh.value, sp.value
        word = ctypes.c_void_p()
        _lib.call("dpwa_learner_status_word", self._h, ctypes.byref(word))
        self._status = ctypes.c_int32.from_address(word.value)
        self.version = 0                 # publishes so far (mirrors dpwa_learner_version)
        self._keep = None
        self._loss_dtype = _lib.F64      # what device loss pointers point at (native side)
        self._checked = (None, None)     # (id, data_ptr, numel, dtype) of the last two validated tensors
        self._f_publish = lib.dpwa_learner_publish
        self._f_fetch = lib.dpwa_learner_fetch
        self._f_average = lib.dpwa_learner_average
        self._f_factor = lib.dpwa_learner_factor
        self._f_lerp = lib.dpwa_learner_lerp
        # resident parameters: where they are, read once per round
        self._f_resident = lib.dpwa_learner_resident_params
        self._res_ptr, self._res_slot = ctypes.c_void_p(), ctypes.c_int()
        self._res_args = (ctypes.byref(self._res_ptr), ctypes.byref(self._res_slot))
        self._res_views = {}             # slot payload address -> tensor over it (two at most)

    @property
    def handle(self):
        return self._h

    def loss_args(self, loss):
        """(host double, device pointer or None, keep-alive) for a loss given as a number or a
        device tensor.  A one-element float32/float64 tensor on this learner's device is read
        by the kernels in place (no conversion kernel, no host sync); anything else on a GPU
        is converted to a float64 scalar first."""
        if isinstance(loss, torch.Tensor) and loss.device.type == "cuda":
            if loss.device == self.device and loss.numel() == 1 and loss.dtype in (torch.float32, torch.float64):
                want = _lib.F32 if loss.dtype == torch.float32 else _lib.F64
                if want != self._loss_dtype:
                    _lib.call("dpwa_learner_set_loss_dtype", self._h, want)
                    self._loss_dtype = want
                return 0.0, _c_void_p(loss.data_ptr()), loss
            if self._loss_dtype != _lib.F64:
                _lib.call("dpwa_learner_set_loss_dtype", self._h, _lib.F64)
                self._loss_dtype = _lib.F64
        return loss_args(loss, self.device)

    def close(self):
        if self._owned and self._h is not None and self._h.value and _lib._lib is not None:
            _lib._lib.dpwa_learner_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _ptr(self, t):
        if not isinstance(t, torch.Tensor):
            raise ValueError("expected a %s tensor on %s, got %s" % (self.dtype, self.device, type(t).__name__))
        # id and address alone can repeat for a new tensor (a freed one's id, the caching
        # allocator's block): size and dtype are part of the key, so such a tensor is checked
        # (the last two keys: resident parameters alternate between two tensors)
        key = (id(t), t.data_ptr(), t.numel(), t.dtype)
        if key not in self._checked:
            if t.device != self.device or t.dtype != self.dtype:
                raise ValueError("expected a %s tensor on %s" % (self.dtype, self.device))
            if not t.is_contiguous() or t.numel() != self.numel:
                raise ValueError("expected a contiguous tensor of %d elements, got %s" % (self.numel, tuple(t.shape)))
            self._checked = (self._checked[-1], key)
        return key[1]

    def _fail(self, name, rc):
        raise _lib.DpwaError(name, rc, self._lib.dpwa_last_error().decode(errors="replace"))

    def publish(self, flat, loss, stream):
        p = self._ptr(flat)
        h, d, self._keep = self.loss_args(loss)
        rc = self._f_publish(self._h, p, h, d, stream.cuda_stream)
        if rc:
            self._fail("dpwa_learner_publish", rc)
        self.version += 1

    def resident_params(self):
        """The tensor over the slot the resident parameters are in now (None when the learner is
        not resident); it changes at every average."""
        rc = self._f_resident(self._h, *self._res_args)
        if rc:
            self._fail("dpwa_learner_resident_params", rc)
        ptr = self._res_ptr.value
        if not ptr:
            return None
        t = self._res_views.get(ptr)
        if t is None:
            from .devview import device_tensor
            t = self._res_views[ptr] = device_tensor(ptr, self.numel, self.dtype, self.device)
        return t

    def native_version(self):
        """dpwa_learner_version: publishes issued so far (no device sync)."""
        v = ctypes.c_uint64()
        _lib.call("dpwa_learner_version", self._h, ctypes.byref(v))
        return v.value

    def attach_local(self, peer_id, other):
        _lib.call("dpwa_learner_attach_local", self._h, peer_id, other.handle)

    def ipc_handle(self):
        buf = ctypes.create_string_buffer(_lib.IPC_HANDLE_BYTES)
        _lib.call("dpwa_learner_ipc_handle", self._h, buf, _lib.IPC_HANDLE_BYTES)
        return buf.raw

    def attach_ipc(self, peer_id, handle):
        buf = ctypes.create_string_buffer(bytes(handle), _lib.IPC_HANDLE_BYTES)
        _lib.call("dpwa_learner_attach_ipc", self._h, peer_id, buf, _lib.IPC_HANDLE_BYTES)

    def export_fds(self, which=0):
        """(fds, chunk bytes) sharing this learner's snapshot slots (which=0) or relay buffer
        (which=1) when that allocation is VMM-backed (>= 1.5 GiB, or DPWA_VMM=1); ([], 0)
        for an ordinary allocation, shared by ipc_handle's hipIpc handle.  The caller closes
        the fds once the peers hold theirs."""
        arr = (ctypes.c_int * MAX_FDS)()
        n, chunk = ctypes.c_int(), ctypes.c_int64()
        _lib.call("dpwa_learner_export_fds", self._h, which, arr, MAX_FDS, ctypes.byref(n), ctypes.byref(chunk))
        return list(arr[:n.value]), chunk.value

    def attach_fds(self, peer_id, handle, fds, chunk):
        buf = ctypes.create_string_buffer(bytes(handle), _lib.IPC_HANDLE_BYTES)
        arr = (ctypes.c_int * max(1, len(fds)))(*fds)
        _lib.call("dpwa_learner_attach_fds", self._h, peer_id, buf, _lib.IPC_HANDLE_BYTES, arr, len(fds), chunk)

    def fetch(self, peer_id, peer_version, zero_copy, stream):
        rc = self._f_fetch(self._h, peer_id, peer_version, 1 if zero_copy else 0, stream.cuda_stream)
        if rc:
            self._fail("dpwa_learner_fetch", rc)

    def factor(self, loss, stream):
        h, d, self._keep = self.loss_args(loss)
        rc = self._f_factor(self._h, h, d, stream.cuda_stream)
        if rc:
            self._fail("dpwa_learner_factor", rc)

    def lerp(self, flat, stream):
        rc = self._f_lerp(self._h, self._ptr(flat), stream.cuda_stream)
        if rc:
            self._fail("dpwa_learner_lerp", rc)

    def cancel(self):
        _lib.call("dpwa_learner_cancel", self._h)

    def average(self, flat, loss, stream):
        """Fused factor + lerp (one kernel)."""
        p = self._ptr(flat)
        h, d, self._keep = self.loss_args(loss)
        rc = self._f_average(self._h, p, h, d, stream.cuda_stream)
        if rc:
            self._fail("dpwa_learner_average", rc)

    def take_status(self):
        """Sticky device-reported status (no sync): non-OK at most once per error."""
        st = self._status.value
        if st:
            self._status.value = 0
        return st

    def read_clock(self):
        c = ctypes.c_double()
        _lib.call("dpwa_learner_read_clock", self._h, ctypes.byref(c))
        return c.value

    def write_clock(self, value):
        _lib.call("dpwa_learner_write_clock", self._h, float(value))

    def read_coef(self):
        c = _lib.Coef()
        _lib.call("dpwa_learner_read_coef", self._h, ctypes.byref(c))
        return c

    def poll_status(self):
        done, st = ctypes.c_int(), ctypes.c_int32()
        _lib.call("dpwa_learner_poll_status", self._h, ctypes.byref(done), ctypes.byref(st))
        return bool(done.value), st.value
