"""DeviceFactor's host-side rules (CPU): the exact double through float(), and a factor
from an earlier round refuses to be read once a later update_send has started a new one."""
import pytest

from dpwa_amd.dpwa import DeviceFactor


class FakeLearner:
    def __init__(self, f):
        self.f, self.version, self._h = f, 3, object()

    def read_coef(self):
        class C:
            factor = self.f
            new_clock, a, b, status = 2.0, 0.0, 0.0, 0
        return C()


def test_float_reads_the_exact_double():
    f = 2.0 / 7.0
    assert float(DeviceFactor(FakeLearner(f))) == f
    assert DeviceFactor(FakeLearner(f)).coefficients()["factor"] == f


def test_stale_factor_raises():
    learner = FakeLearner(0.5)
    d = DeviceFactor(learner)
    learner.version += 1            # update_send of the next round
    with pytest.raises(RuntimeError):
        float(d)
    with pytest.raises(RuntimeError):
        d.coefficients()
    with pytest.raises(RuntimeError):
        d.tensor()
