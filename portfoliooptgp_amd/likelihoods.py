"""gpflow.likelihoods.Gaussian: variance σn² with a 1e-6 lower bound
(``Gaussian(variance=1.0, variance_lower_bound=1e-6)``)."""
from __future__ import annotations

from .parameter import Parameter

DEFAULT_VARIANCE_LOWER_BOUND = 1e-6


class Gaussian:
    def __init__(self, variance: float = 1.0, variance_lower_bound: float = DEFAULT_VARIANCE_LOWER_BOUND):
        self.variance = Parameter(variance, lower=variance_lower_bound, name="variance")

    @property
    def parameters(self):
        return (self.variance,)

    @property
    def trainable_parameters(self):
        return tuple(p for p in self.parameters if p.trainable)

    @property
    def trainable_variables(self):
        return tuple(p.unconstrained_variable for p in self.trainable_parameters)
