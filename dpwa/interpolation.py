"""dpwa.interpolation (reference dpwa/interpolation.py) -> dpwa_amd.interpolation."""
from dpwa_amd.interpolation import (ClockWeightedInterpolation, ConstantInterpolation,  # noqa: F401
                                    InterpolationBase, LossInterpolation)
