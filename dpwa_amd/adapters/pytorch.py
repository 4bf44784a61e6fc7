"""DpwaPyTorchAdapter on MI355X (mirror of dpwa/adapters/pytorch.py).

Same constructor and methods.  Instead of pickling every parameter through the host
(pytorch.py:17-34, 49-53) and averaging tensor by tensor with three ATen kernels and
three temporaries each (pytorch.py:66-68), the parameters live in one flat HBM buffer
(dpwa_amd/flat.py); update_send publishes it with one kernel and update_wait averages it
in place with one fused HIP kernel whose coefficients come from the device factor.

Differences that are intentional: the average is written in place (the reference
rebinds ``param.data`` to a new tensor), and float32 *and* bfloat16 models are accepted
(the reference maps only FloatTensor, pytorch.py:11-14).
"""
import logging

from ..dpwa import DpwaConnection
from ..flat import FlatParameters

LOGGER = logging.getLogger(__name__)


class DpwaPyTorchAdapter:
    def __init__(self, net, name, config_file, **connection_kwargs):
        self._net = net
        self._flat = FlatParameters(net.named_parameters())
        self._conn = DpwaConnection(name, config_file, **connection_kwargs)

    def update_send(self, loss):
        """pytorch.py:42-53: publish the parameters and maybe start a fetch."""
        self._flat.resync()
        self._conn.update_send(self._flat.buffer, loss)

    def update_wait(self, loss):
        """pytorch.py:55-68: wait for the fetch and average in place."""
        self._conn.update_wait_average(self._flat.buffer, loss)

    # -- extensions -------------------------------------------------------------------
    @property
    def connection(self):
        return self._conn

    @property
    def flat(self):
        return self._flat
