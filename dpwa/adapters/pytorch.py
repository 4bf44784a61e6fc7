"""dpwa.adapters.pytorch (reference dpwa/adapters/pytorch.py) -> dpwa_amd.adapters.pytorch."""
from dpwa_amd.adapters.pytorch import DpwaPyTorchAdapter  # noqa: F401
