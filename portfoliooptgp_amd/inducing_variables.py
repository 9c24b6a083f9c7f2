"""gpflow.inducing_variables.InducingPoints: trainable inducing inputs Z [M, D]
(test_scripts/SVGP.py:464 passes ``np.linspace(0, 360, 120)[:, None]``, which GPflow wraps in
InducingPoints)."""
from __future__ import annotations

import numpy as np

from .parameter import ArrayParameter


class InducingPoints:
    def __init__(self, Z, name: str = "Z"):
        Z = np.array(Z, dtype=np.float64)
        if Z.ndim == 1:
            Z = Z[:, None]
        if Z.ndim != 2:
            raise ValueError("Z must be [M, D]")
        self.Z = ArrayParameter(Z, name=name)

    @property
    def num_inducing(self) -> int:
        return int(self.Z.shape[0])

    def __len__(self) -> int:
        return self.num_inducing

    @property
    def parameters(self):
        return (self.Z,)
