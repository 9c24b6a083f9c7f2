"""Positive parameters with GPflow 2.9.1 semantics.

GPflow stores each positive parameter as an unconstrained tf.Variable u and exposes the
constrained value θ = lower + softplus(u) (tfp.bijectors.Softplus, chained with Shift(lower)
for the Gaussian likelihood variance, lower = 1e-6). ``gpflow.optimizers.Scipy`` optimises u
(GPR/model_trainer.py:18-19). ``Parameter.assign`` takes a constrained value
(GPR/model_trainer.py:16: ``model.likelihood.variance.assign(1e-5)``).
"""
from __future__ import annotations

import math

import numpy as np

_EPS = float(np.finfo(np.float64).eps)
_THRESH = math.log(_EPS) + 2.0  # tfp.math.softplus_inverse threshold


def softplus(u: float) -> float:
    """np.logaddexp(0, u) bit for bit: numpy's scalar npy_logaddexp with the same libm
    exp/log1p, without the ufunc dispatch (this runs once per parameter per evaluation)."""
    u = float(u)
    if u == 0.0:
        return math.log(2.0)
    if u < 0.0:
        return math.log1p(math.exp(u))
    if u > 0.0:
        return u + math.log1p(math.exp(-u))
    return u  # nan


def softplus_inverse(t: float) -> float:
    """tfp.math.softplus_inverse: log(expm1(t)) with its small/large-argument branches."""
    t = float(t)
    if t < math.exp(_THRESH):
        return math.log(t)
    if t > -_THRESH:
        return t
    return t + math.log(-math.expm1(-t))


def sigmoid(u: float) -> float:
    return 0.5 * (1.0 + math.tanh(0.5 * u))


class UnconstrainedVariable:
    """The tf.Variable-like handle that lands in ``model.trainable_variables``."""

    def __init__(self, param: "Parameter"):
        self._param = param

    @property
    def name(self) -> str:
        return f"{self._param.name}:0"

    @property
    def shape(self):
        return ()

    @property
    def dtype(self):
        return np.float64

    @property
    def trainable(self) -> bool:
        return self._param.trainable

    def numpy(self) -> np.ndarray:
        return np.asarray(self._param.unconstrained, dtype=np.float64)

    def assign(self, u) -> None:
        self._param.set_unconstrained(float(np.asarray(u, dtype=np.float64).reshape(())))

    def __repr__(self) -> str:
        return f"<UnconstrainedVariable {self.name} u={self._param.unconstrained!r}>"


class Parameter:
    """A scalar positive parameter (θ = lower + softplus(u))."""

    def __init__(self, value: float, lower: float = 0.0, trainable: bool = True, name: str = "parameter"):
        value = value if type(value) is float else float(np.asarray(value, dtype=np.float64).reshape(()))
        if not value > lower:
            raise ValueError(f"{name}: value {value} must be > {lower} (positive transform)")
        self.lower = float(lower)
        self.trainable = bool(trainable)
        self.name = name
        self._u = softplus_inverse(value - self.lower)
        self._variable = UnconstrainedVariable(self)

    # --- constrained view -------------------------------------------------------------
    @property
    def value(self) -> float:
        return self.lower + softplus(self._u)

    def numpy(self) -> np.float64:
        return np.float64(self.value)

    def assign(self, value) -> None:
        value = value if type(value) is float else float(np.asarray(value, dtype=np.float64).reshape(()))
        if not value > self.lower:
            raise ValueError(f"{self.name}: value {value} must be > {self.lower}")
        self._u = softplus_inverse(value - self.lower)

    # --- unconstrained view -----------------------------------------------------------
    @property
    def unconstrained(self) -> float:
        return self._u

    def set_unconstrained(self, u: float) -> None:
        self._u = float(u)

    @property
    def unconstrained_variable(self) -> UnconstrainedVariable:
        return self._variable

    def dtheta_du(self) -> float:
        return sigmoid(self._u)

    @property
    def transform_name(self) -> str:
        return "Softplus" if self.lower == 0.0 else "Softplus + Shift"

    def __float__(self) -> float:
        return self.value

    def __array__(self, dtype=None, copy=None):
        return np.asarray(self.value, dtype=dtype or np.float64)

    def __repr__(self) -> str:
        return f"<Parameter {self.name}={self.value!r} trainable={self.trainable}>"


# ----------------------------------------------------------------------------------------
# array-valued parameters (SVGP: inducing inputs Z, q_mu, q_sqrt)
# ----------------------------------------------------------------------------------------
_TRI_CACHE = {}


def _tri_index(n: int):
    """(flat positions of the lower triangle of an n×n matrix, the vector index stored at each)
    for tfp's fill_triangular layout, computed once per n (a gather/scatter pair then replaces
    the concatenate/reverse/reshape of the definition below)."""
    hit = _TRI_CACHE.get(n)
    if hit is None:
        m = n * (n + 1) // 2
        x = np.arange(m, dtype=np.float64)
        full = np.tril(np.concatenate([x[n:], x[::-1]]).reshape(n, n))
        r, c = np.tril_indices(n)
        flat = r * n + c
        hit = (flat, full.reshape(-1)[flat].astype(np.int64))
        _TRI_CACHE[n] = hit
    return hit


def fill_triangular(x: np.ndarray) -> np.ndarray:
    """tfp.math.fill_triangular(x, upper=False): the vector → lower-triangular layout that
    tfp.bijectors.FillTriangular (GPflow's ``triangular()`` transform of q_sqrt) uses:
    L = tril(reshape(concat(x[n:], reverse(x)), [n, n]))."""
    x = np.asarray(x, dtype=np.float64)
    m = x.shape[-1]
    n = (math.isqrt(8 * m + 1) - 1) // 2
    if n * (n + 1) // 2 != m:
        raise ValueError(f"fill_triangular: {m} is not a triangular number")
    flat, src = _tri_index(n)
    L = np.zeros(n * n)
    L[flat] = x[src]
    return L.reshape(n, n)


def fill_triangular_inverse(L: np.ndarray) -> np.ndarray:
    """tfp.math.fill_triangular_inverse(L, upper=False) (the lower triangle of L, gathered back
    into fill_triangular's vector order)."""
    L = np.asarray(L, dtype=np.float64)
    n = L.shape[-1]
    flat, src = _tri_index(n)
    x = np.empty(n * (n + 1) // 2)
    x[src] = L.reshape(-1)[flat]
    return x


class ArrayVariable:
    """Unconstrained tf.Variable-like handle of an ArrayParameter."""

    def __init__(self, param: "ArrayParameter"):
        self._param = param

    @property
    def name(self) -> str:
        return f"{self._param.name}:0"

    @property
    def shape(self):
        return self._param.unconstrained.shape

    @property
    def dtype(self):
        return np.float64

    @property
    def trainable(self) -> bool:
        return self._param.trainable

    def numpy(self) -> np.ndarray:
        return self._param.unconstrained.copy()

    def assign(self, u) -> None:
        self._param.set_unconstrained(np.asarray(u, dtype=np.float64).reshape(self.shape))


class ArrayParameter:
    """A GPflow Parameter holding an array with the identity transform (Z, q_mu) or
    FillTriangular (q_sqrt: constrained [1, M, M] lower-triangular, unconstrained
    [1, M(M+1)/2])."""

    def __init__(self, value, transform: str = "identity", trainable: bool = True,
                 name: str = "parameter"):
        self.transform = transform
        self.trainable = bool(trainable)
        self.name = name
        self.assign(value)
        self._variable = ArrayVariable(self)

    @property
    def value(self) -> np.ndarray:
        if self.transform == "triangular":
            return np.stack([fill_triangular(r) for r in self._u])
        return self._u.copy()

    def numpy(self) -> np.ndarray:
        return self.value

    def assign(self, value) -> None:
        v = np.array(value, dtype=np.float64)
        if self.transform == "triangular":
            if v.ndim == 2:
                v = v[None]
            self._u = np.stack([fill_triangular_inverse(np.tril(r)) for r in v])
        else:
            self._u = v

    @property
    def shape(self):
        return self.value.shape

    @property
    def unconstrained(self) -> np.ndarray:
        return self._u

    def set_unconstrained(self, u) -> None:
        self._u = np.array(u, dtype=np.float64).reshape(self._u.shape)

    @property
    def unconstrained_variable(self) -> ArrayVariable:
        return self._variable

    def grad_to_unconstrained(self, g: np.ndarray) -> np.ndarray:
        """Chain rule for the transform: ∂/∂u from ∂/∂value (same layout as ``unconstrained``)."""
        if self.transform == "triangular":
            g = np.asarray(g, dtype=np.float64)
            if g.ndim == 2:
                g = g[None]
            return np.stack([fill_triangular_inverse(np.tril(r)) for r in g])
        return np.asarray(g, dtype=np.float64).reshape(self._u.shape)

    @property
    def transform_name(self) -> str:
        return "FillTriangular" if self.transform == "triangular" else "Identity"

    def __array__(self, dtype=None, copy=None):
        return np.asarray(self.value, dtype=dtype or np.float64)

    def __repr__(self) -> str:
        return f"<ArrayParameter {self.name} shape={self.shape} trainable={self.trainable}>"
