"""dpwa.dpwa (reference dpwa/dpwa.py) -> dpwa_amd.dpwa."""
from dpwa_amd.dpwa import DeviceFactor, DpwaConfiguration, DpwaConnection, PeerSnapshot, Struct  # noqa: F401
from dpwa_amd.interpolation import INTERPOLATION_METHODS  # noqa: F401
