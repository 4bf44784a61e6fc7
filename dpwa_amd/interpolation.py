"""Interpolation methods (mirror of dpwa/interpolation.py).

Same class names, constructor signatures and error behaviour as the reference, so a
config that the reference accepts (or rejects) behaves identically here.  The factor
itself is computed on the GPU by the factor kernel (dpwa_amd/csrc/kernels.hip
``k_factor``) from each object's :meth:`device_config`; ``__call__`` evaluates the same
formula on the host in Python floats and is what the host-side API reports.
"""
from . import _lib


class InterpolationBase:
    method = None

    def __call__(self, clock, peer_clock, loss, peer_loss):
        raise NotImplementedError

    def device_config(self, divergence_threshold):
        return _lib.Interp(self.method, 0, float(getattr(self, "_value", 0.0)), float(divergence_threshold))


class ConstantInterpolation(InterpolationBase):
    """interpolation.py:8-15."""
    method = _lib.INTERP_CONSTANT

    def __init__(self, value):
        assert (value <= 1) and (value >= 0)
        self._value = value

    def __call__(self, clock, peer_clock, loss, peer_loss):
        return self._value


class ClockWeightedInterpolation(InterpolationBase):
    """interpolation.py:18-24: the peer with the larger clock pulls harder."""
    method = _lib.INTERP_CLOCK

    def __init__(self):
        pass

    def __call__(self, clock, peer_clock, loss, peer_loss):
        return peer_clock / (clock + peer_clock)


class LossInterpolation(InterpolationBase):
    """interpolation.py:27-33: a larger own loss pulls harder toward the peer."""
    method = _lib.INTERP_LOSS

    def __init__(self):
        pass

    def __call__(self, clock, peer_clock, loss, peer_loss):
        k = loss / (loss + peer_loss)
        return k


INTERPOLATION_METHODS = {          # dpwa.py:11-15
    'constant': ConstantInterpolation,
    'clock': ClockWeightedInterpolation,
    'loss': LossInterpolation,
}
