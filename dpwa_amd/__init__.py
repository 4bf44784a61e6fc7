"""dpwa_amd -- MI355X-native pairwise-averaging (gossip) hot path of dpwa.

Drop-in for the reference's ``dpwa.adapters.pytorch.DpwaPyTorchAdapter`` and
``dpwa.dpwa.DpwaConnection``; the compute path is libdpwa_hip.so (HIP for gfx950).
"""
from .dpwa import DpwaConfiguration, DpwaConnection  # noqa: F401
from .adapters.pytorch import DpwaPyTorchAdapter  # noqa: F401

__all__ = ["DpwaConfiguration", "DpwaConnection", "DpwaPyTorchAdapter"]
