"""One flat, 256-byte-aligned HBM buffer per learner holding every parameter.

The reference snapshots ``named_parameters()`` tensor by tensor into a dict of bytes and
averages them tensor by tensor (dpwa/adapters/pytorch.py:49-53, 66-68).  Here the
parameters are re-homed once into a single contiguous buffer -- each tensor starting on a
256-byte boundary, in ``named_parameters()`` order, gaps zero-filled -- and every
``param.data`` becomes a view into it, so publishing and averaging are one kernel each
over one buffer.  Gaps average to zero (0*a + 0*b).
"""
import torch

ALIGN_BYTES = 256


class FlatParameters:
    def __init__(self, named_parameters, device=None):
        """device: where the flat buffer lives (a config's per-node `gpu:` key); parameters on
        another device are moved there (create the optimizer afterwards, as the reference's
        trainer does: examples/pytorch-cifar/main.py:109-116)."""
        params = list(named_parameters)
        if not params:
            raise ValueError("the model has no parameters")
        dtypes = {p.dtype for _, p in params}
        devices = {p.device for _, p in params}
        if len(dtypes) != 1 or len(devices) != 1:
            raise TypeError("all parameters must share one dtype and one device, got %s on %s"
                            % (sorted(map(str, dtypes)), sorted(map(str, devices))))
        self.dtype = dtypes.pop()
        self.device = devices.pop() if device is None else torch.device(device)
        esize = torch.empty((), dtype=self.dtype).element_size()
        align = ALIGN_BYTES // esize
        self.names, self.params, self.offsets = [], [], []
        off = 0
        for name, p in params:
            self.names.append(name)
            self.params.append(p)
            self.offsets.append(off)
            off += (p.numel() + align - 1) // align * align
        self.numel = off
        self.buffer = torch.zeros(self.numel, dtype=self.dtype, device=self.device)
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                self.buffer[o:o + p.numel()].copy_(p.data.reshape(-1))
        self._rebind()

    def _rebind(self):
        self._ptrs = []
        for p, o in zip(self.params, self.offsets):
            p.data = self.buffer[o:o + p.numel()].view(p.shape)
            self._ptrs.append(p.data_ptr())

    def rehome(self, buffer):
        """Re-points every parameter into `buffer`, a tensor of this layout that already holds
        the values (a resident learner's slot, which alternates between two: their views are
        built once, so a move costs one ``.data`` assignment per parameter)."""
        if buffer is self.buffer:
            return
        if buffer.numel() != self.numel or buffer.dtype != self.dtype or buffer.device != self.device:
            raise ValueError("rehome: a %s buffer of %d elements on %s is needed" % (self.dtype, self.numel,
                                                                                     self.device))
        cache = self.__dict__.setdefault("_homes", {})
        key = buffer.data_ptr()
        views = cache.get(key)
        if views is None:
            if len(cache) >= 2:
                cache.clear()
            views = cache[key] = [buffer[o:o + p.numel()].view(p.shape) for p, o in zip(self.params, self.offsets)]
        self.buffer = buffer
        for p, v in zip(self.params, views):
            p.data = v
        self._ptrs = [v.data_ptr() for v in views]

    def resync(self):
        """Re-homes parameters whose ``.data`` was replaced since the last call (e.g. a
        user assigned ``param.data = ...``); returns the number re-homed."""
        if [p.data_ptr() for p in self.params] == self._ptrs:
            return 0          # the common case: one pointer read per parameter
        moved = 0
        with torch.no_grad():
            for i, (p, o) in enumerate(zip(self.params, self.offsets)):
                if p.data_ptr() != self._ptrs[i] or p.device != self.device or p.dtype != self.dtype:
                    self.buffer[o:o + p.numel()].copy_(p.data.reshape(-1))
                    p.data = self.buffer[o:o + p.numel()].view(p.shape)
                    self._ptrs[i] = p.data_ptr()
                    moved += 1
        return moved

    def view(self, name):
        i = self.names.index(name)
        return self.buffer[self.offsets[i]:self.offsets[i] + self.params[i].numel()].view(self.params[i].shape)
