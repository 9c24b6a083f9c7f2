"""CPU oracle for the exact-GPR hot path — TEST INFRASTRUCTURE ONLY.

This module is a numpy/scipy fp64 restatement of the GPflow 2.9.1 arithmetic that the
reference reaches from ``GPR/model_trainer.py:15-20`` and ``GPR/predictor.py:5-8``.
GPflow itself (pinned at ``Multi-Input_GPR/requirements.txt:37``, gpflow==2.9.1 on
tensorflow==2.16.1 / tensorflow-probability==0.24.0) is not vendored in the reference and is
not installable here, so this file restates its published semantics:

* kernels  — ``gpflow.kernels`` SquaredExponential, Matern12/32/52, Exponential,
  RationalQuadratic, Periodic(SE base), Linear, Sum, Product, with ``active_dims``
  (kernel list at ``GPR/main.py:105-114``; composite at ``Multi-Input_GPR/main.py:118-135``);
* parameters — softplus-constrained (``θ = lower + log(1+e^u)``; Gaussian likelihood uses
  lower = 1e-6), trainable variables ordered the way ``tf.Module`` flattens attributes
  (sorted attribute names; ``kernels`` lists in order);
* ``GPR.log_marginal_likelihood`` / ``training_loss`` and its gradient w.r.t. the
  unconstrained variables (what ``gpflow.optimizers.Scipy`` feeds to L-BFGS-B,
  ``GPR/model_trainer.py:18-19``);
* ``GPR.predict_f(full_cov=False)`` / ``predict_y`` (``GPR/predictor.py:6-7``);
* ``gpflow.optimizers.Scipy().minimize`` (scipy L-BFGS-B, ``options=dict(maxiter=100)``);
* the data preparation of ``GPR/data_handler.py:26-65`` (without the network fetch).

Who may import this: ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg,
and only as the checker / the timed CPU baseline. The product package never imports it.

Parity pinning: the reference's own tests mock the GP (``GPR/tests/test_model_trainer.py:11``),
so no reference golden vector exists for these numbers. This restatement is pinned by
(1) an independent torch-fp64 autograd restatement (``tests/test_oracle.py``), (2) central
finite differences, (3) closed-form known-answer cases (N=1, N=2), and (4) the survey-time
numbers for the AAPL N=89 series. It is *not* GPflow-verified
("parity unpinned" against GPflow itself).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np
import scipy.linalg as sla
import scipy.optimize

LOG2PI = math.log(2.0 * math.pi)


# ----------------------------------------------------------------------------------------
# softplus transform (tfp.bijectors.Softplus, optionally Chain(Shift(lower), Softplus))
# ----------------------------------------------------------------------------------------
def softplus(u):
    u = np.asarray(u, dtype=np.float64)
    return np.logaddexp(0.0, u)


def softplus_inverse(t):
    t = np.asarray(t, dtype=np.float64)
    # log(exp(t) - 1) computed stably
    with np.errstate(over="ignore"):
        return np.where(t > 30.0, t + np.log(-np.expm1(-t)), np.log(np.expm1(t)))


def sigmoid(u):
    u = np.asarray(u, dtype=np.float64)
    return 0.5 * (1.0 + np.tanh(0.5 * u))


@dataclass
class OParam:
    """A positive GPflow Parameter: θ = lower + softplus(u)."""
    name: str
    value: float
    lower: float = 0.0
    trainable: bool = True

    @property
    def u(self) -> float:
        return float(softplus_inverse(self.value - self.lower))

    def set_u(self, u: float) -> None:
        self.value = float(self.lower + softplus(u))

    def dtheta_du(self) -> float:
        return float(sigmoid(self.u))


# ----------------------------------------------------------------------------------------
# kernels
# ----------------------------------------------------------------------------------------
def _slice_dims(X: np.ndarray, active_dims) -> np.ndarray:
    if active_dims is None:
        return X
    if isinstance(active_dims, slice):
        return X[:, active_dims]
    return X[:, list(active_dims)]


class OKernel:
    def params(self) -> List[OParam]:
        raise NotImplementedError

    def K(self, X, X2=None) -> np.ndarray:
        raise NotImplementedError

    def K_diag(self, X) -> np.ndarray:
        raise NotImplementedError

    def dK(self, X) -> List[np.ndarray]:
        """dK(X,X)/dθ for each parameter in params() order (constrained space)."""
        raise NotImplementedError

    def dK_dX1(self, X, X2) -> np.ndarray:
        """∂K(x, x')/∂x for x in X, x' in X2: [n1, n2, D] over ALL input columns (zero
        outside active_dims). Used by the SVGP oracle for the inducing-point gradient."""
        raise NotImplementedError


# How the scaled squared distance r² is formed. "gpflow" (the default) is GPflow 2.9.1's
# ``Stationary.scale`` (X / ℓ) followed by ``gpflow.utilities.ops.square_distance``:
#     a = x/ℓ, b = x'/ℓ;   r² = (−2·(a·b)) + (‖a‖² + ‖b‖²)
# each operation rounded on its own (TF evaluates op by op, no FMA contraction). For D = 1 that
# order is fully determined; for D > 1 the dot product and the norms are summed over d in
# order (TF's matmul/reduce_sum order for a 2–7 wide inner dimension is not specified; any
# order differs by an ulp). The expansion loses ~eps·max‖a‖² absolutely to cancellation, which
# at C2 size (x up to 4095, ℓ ≈ 1) moves logML by ~3e-7 and the gradient by ~5e-6 relative
# against the direct form — so the GPU path computes r² the same way (gpx_kfun.h sqdist).
# "direct" = Σ_d ((x_d − x'_d)/ℓ)² as squared differences, kept as a documented alternate
# (more accurate in exact-arithmetic terms, not what GPflow computes).
R2_FORM = "gpflow"


def scaled_sqdist(A: np.ndarray, B: np.ndarray, ell: float, form: Optional[str] = None) -> np.ndarray:
    """r²(a_i, b_j) for rows of A [n1, D] and B [n2, D] (already sliced to active dims)."""
    form = R2_FORM if form is None else form
    A = np.asarray(A, np.float64)
    B = np.asarray(B, np.float64)
    if form == "direct":
        diff = A[:, None, :] - B[None, :, :]
        return np.sum(diff * diff, axis=-1) / (ell * ell)
    a = A / ell
    b = B / ell
    D = a.shape[1]
    sa = a[:, 0] * a[:, 0]
    sb = b[:, 0] * b[:, 0]
    dot = a[:, 0:1] * b[None, :, 0]
    for d in range(1, D):
        sa = sa + a[:, d] * a[:, d]
        sb = sb + b[:, d] * b[:, d]
        dot = dot + a[:, d:d + 1] * b[None, :, d]
    return -2.0 * dot + (sa[:, None] + sb[None, :])


class OStationary(OKernel):
    """IsotropicStationary: r² = Σ_d ((x_d - x'_d)/ℓ)² over active dims, formed as GPflow's
    ``scaled_squared_euclid_dist`` forms it (``scaled_sqdist``), r = sqrt(max(r², 1e-36)) for
    the K_r kernels."""

    kind = "stationary"

    def __init__(self, variance=1.0, lengthscales=1.0, active_dims=None):
        self.variance = OParam("variance", float(variance))
        self.lengthscales = OParam("lengthscales", float(lengthscales))
        self.active_dims = active_dims

    def params(self):
        return [self.lengthscales, self.variance]          # sorted attribute names

    def _r2(self, X, X2):
        A = _slice_dims(np.asarray(X, np.float64), self.active_dims)
        B = A if X2 is None else _slice_dims(np.asarray(X2, np.float64), self.active_dims)
        return scaled_sqdist(A, B, self.lengthscales.value)

    # shape functions of the scaled r² (unit variance)
    def _g(self, r2):
        raise NotImplementedError

    def _dg_dr2(self, r2):
        raise NotImplementedError

    def K(self, X, X2=None):
        return self.variance.value * self._g(self._r2(X, X2))

    def K_diag(self, X):
        return np.full(np.asarray(X).shape[0], self.variance.value)

    def dK(self, X):
        ell, var = self.lengthscales.value, self.variance.value
        r2 = self._r2(X, None)
        g = self._g(r2)
        dl = var * self._dg_dr2(r2) * (-2.0 * r2 / ell)     # d r²/dℓ = -2 r²/ℓ
        return [dl, g]

    def dK_dX1(self, X, X2):
        X = np.asarray(X, np.float64)
        X2 = np.asarray(X2, np.float64)
        ell, var = self.lengthscales.value, self.variance.value
        r2 = self._r2(X, X2)
        f = var * self._dg_dr2(r2) * 2.0 / (ell * ell)        # ∂k/∂x_d = f · (x_d − x'_d)
        out = np.zeros(X.shape[:1] + X2.shape[:1] + X.shape[1:])
        cols = np.arange(X.shape[1])
        if self.active_dims is not None:
            cols = cols[self.active_dims] if isinstance(self.active_dims, slice) else np.asarray(list(self.active_dims))
        for d in cols:
            out[:, :, d] = f * (X[:, None, d] - X2[None, :, d])
        return out


class OSquaredExponential(OStationary):
    def _g(self, r2):
        return np.exp(-0.5 * r2)

    def _dg_dr2(self, r2):
        return -0.5 * np.exp(-0.5 * r2)


class _OKr(OStationary):
    """Kernels defined through K_r(r) with r = sqrt(max(r², 1e-36))."""

    def _h(self, r):
        raise NotImplementedError

    def _dh(self, r):
        raise NotImplementedError

    def _g(self, r2):
        return self._h(np.sqrt(np.maximum(r2, 1e-36)))

    def _dg_dr2(self, r2):
        # d/dr² h(sqrt(max(r2,1e-36))) = h'(r)/(2r) where r2 > 1e-36, else 0 (max clamps)
        r = np.sqrt(np.maximum(r2, 1e-36))
        return np.where(r2 > 1e-36, self._dh(r) / (2.0 * r), 0.0)


class OMatern12(_OKr):
    def _h(self, r):
        return np.exp(-r)

    def _dh(self, r):
        return -np.exp(-r)


class OExponential(_OKr):
    """gpflow.kernels.Exponential: K_r = σ² exp(-r/2)."""

    def _h(self, r):
        return np.exp(-0.5 * r)

    def _dh(self, r):
        return -0.5 * np.exp(-0.5 * r)


class OMatern32(_OKr):
    def _h(self, r):
        s = math.sqrt(3.0)
        return (1.0 + s * r) * np.exp(-s * r)

    def _dh(self, r):
        s = math.sqrt(3.0)
        return -3.0 * r * np.exp(-s * r)


class OMatern52(_OKr):
    def _h(self, r):
        s = math.sqrt(5.0)
        return (1.0 + s * r + 5.0 / 3.0 * r * r) * np.exp(-s * r)

    def _dh(self, r):
        s = math.sqrt(5.0)
        return -(5.0 / 3.0) * r * (1.0 + s * r) * np.exp(-s * r)


class ORationalQuadratic(OStationary):
    """K = σ² (1 + r²/(2α))^(-α)."""

    def __init__(self, variance=1.0, lengthscales=1.0, alpha=1.0, active_dims=None):
        super().__init__(variance, lengthscales, active_dims)
        self.alpha = OParam("alpha", float(alpha))

    def params(self):
        return [self.alpha, self.lengthscales, self.variance]

    def _g(self, r2):
        a = self.alpha.value
        return (1.0 + 0.5 * r2 / a) ** (-a)

    def _dg_dr2(self, r2):
        a = self.alpha.value
        return -0.5 * (1.0 + 0.5 * r2 / a) ** (-a - 1.0)

    def dK(self, X):
        dl, dv = super().dK(X)
        a, var = self.alpha.value, self.variance.value
        r2 = self._r2(X, None)
        b = 1.0 + 0.5 * r2 / a
        # d/dα b^(-α) = b^(-α) (-log b + r²/(2α b))
        da = var * b ** (-a) * (-np.log(b) + 0.5 * r2 / (a * b))
        return [da, dl, dv]


class OPeriodic(OKernel):
    """gpflow.kernels.Periodic(SquaredExponential()): SE has no K_r, so the K_r2 path:
    K = σ² exp(-½ Σ_d (sin(π (x_d - x'_d)/p) / ℓ)²)."""

    def __init__(self, base: Optional[OSquaredExponential] = None, period=1.0):
        self.base = base if base is not None else OSquaredExponential()
        self.period = OParam("period", float(period))

    def params(self):
        return [self.base.lengthscales, self.base.variance, self.period]

    def _parts(self, X, X2):
        A = _slice_dims(np.asarray(X, np.float64), self.base.active_dims)
        B = A if X2 is None else _slice_dims(np.asarray(X2, np.float64), self.base.active_dims)
        diff = A[:, None, :] - B[None, :, :]
        arg = math.pi * diff / self.period.value
        return diff, arg

    def K(self, X, X2=None):
        _, arg = self._parts(X, X2)
        ell = self.base.lengthscales.value
        s2 = np.sum((np.sin(arg) / ell) ** 2, axis=-1)
        return self.base.variance.value * np.exp(-0.5 * s2)

    def K_diag(self, X):
        return np.full(np.asarray(X).shape[0], self.base.variance.value)

    def dK(self, X):
        diff, arg = self._parts(X, None)
        ell, var, p = self.base.lengthscales.value, self.base.variance.value, self.period.value
        sn = np.sin(arg)
        s2 = np.sum((sn / ell) ** 2, axis=-1)               # as K: Σ (sin/ℓ)²
        g = np.exp(-0.5 * s2)
        dl = var * g * s2 / ell
        # d s2/dp = Σ 2 sin cos (-π diff / p²) / ℓ²
        ds2dp = np.sum(2.0 * sn * np.cos(arg) * (-math.pi * diff / (p * p)), axis=-1) / (ell * ell)
        dp = var * g * (-0.5) * ds2dp
        return [dl, g, dp]

    def dK_dX1(self, X, X2):
        X = np.asarray(X, np.float64)
        _, arg = self._parts(X, X2)
        ell, p = self.base.lengthscales.value, self.period.value
        k = self.K(X, X2)
        # ∂k/∂x_d = k · (−½) · 2 sin cos · (π/p) / ℓ²
        part = -k[:, :, None] * np.sin(arg) * np.cos(arg) * (math.pi / p) / (ell * ell)
        out = np.zeros(k.shape + X.shape[1:])
        cols = np.arange(X.shape[1])
        ad = self.base.active_dims
        if ad is not None:
            cols = cols[ad] if isinstance(ad, slice) else np.asarray(list(ad))
        out[:, :, cols] = part
        return out


class OLinear(OKernel):
    def __init__(self, variance=1.0, active_dims=None):
        self.variance = OParam("variance", float(variance))
        self.active_dims = active_dims

    def params(self):
        return [self.variance]

    def _xx(self, X, X2, scale=1.0):
        """Σ_d (x_d·scale)·x'_d, summed over d in order (gpflow.kernels.Linear.K:
        ``tf.linalg.matmul(X * variance, X2, transpose_b=True)``)."""
        A = _slice_dims(np.asarray(X, np.float64), self.active_dims) * scale
        B = _slice_dims(np.asarray(X if X2 is None else X2, np.float64), self.active_dims)
        out = A[:, 0:1] * B[None, :, 0]
        for d in range(1, A.shape[1]):
            out = out + A[:, d:d + 1] * B[None, :, d]
        return out

    def K(self, X, X2=None):
        return self._xx(X, X2, self.variance.value)

    def K_diag(self, X):
        # Linear.K_diag: reduce_sum(square(X) * variance, -1)
        A = _slice_dims(np.asarray(X, np.float64), self.active_dims)
        sq = (A * A) * self.variance.value
        out = sq[:, 0]
        for d in range(1, sq.shape[1]):
            out = out + sq[:, d]
        return out

    def dK(self, X):
        return [self._xx(X, None)]

    def dK_dX1(self, X, X2):
        X = np.asarray(X, np.float64)
        X2 = np.asarray(X2, np.float64)
        out = np.zeros((X.shape[0], X2.shape[0], X.shape[1]))
        cols = np.arange(X.shape[1])
        if self.active_dims is not None:
            cols = cols[self.active_dims] if isinstance(self.active_dims, slice) else np.asarray(list(self.active_dims))
        for d in cols:
            out[:, :, d] = self.variance.value * X2[None, :, d]
        return out


class OSum(OKernel):
    def __init__(self, kernels: Sequence[OKernel]):
        self.kernels = list(kernels)

    def params(self):
        return [p for k in self.kernels for p in k.params()]

    def K(self, X, X2=None):
        return sum(k.K(X, X2) for k in self.kernels)

    def K_diag(self, X):
        return sum(k.K_diag(X) for k in self.kernels)

    def dK(self, X):
        return [d for k in self.kernels for d in k.dK(X)]

    def dK_dX1(self, X, X2):
        return sum(k.dK_dX1(X, X2) for k in self.kernels)


class OProduct(OKernel):
    def __init__(self, kernels: Sequence[OKernel]):
        self.kernels = list(kernels)

    def params(self):
        return [p for k in self.kernels for p in k.params()]

    def K(self, X, X2=None):
        out = None
        for k in self.kernels:
            out = k.K(X, X2) if out is None else out * k.K(X, X2)
        return out

    def K_diag(self, X):
        out = None
        for k in self.kernels:
            out = k.K_diag(X) if out is None else out * k.K_diag(X)
        return out

    def dK(self, X):
        Ks = [k.K(X) for k in self.kernels]
        res = []
        for t, k in enumerate(self.kernels):
            others = np.ones_like(Ks[0])
            for s, Ks_s in enumerate(Ks):
                if s != t:
                    others = others * Ks_s
            res.extend(others * d for d in k.dK(X))
        return res

    def dK_dX1(self, X, X2):
        Ks = [k.K(X, X2) for k in self.kernels]
        out = 0.0
        for t, k in enumerate(self.kernels):
            others = np.ones_like(Ks[0])
            for s_, Ks_s in enumerate(Ks):
                if s_ != t:
                    others = others * Ks_s
            out = out + others[:, :, None] * k.dK_dX1(X, X2)
        return out


# ----------------------------------------------------------------------------------------
# exact GPR (GPflow 2.9.1 models.GPR with Gaussian likelihood and Zero mean)
# ----------------------------------------------------------------------------------------
class OGPR:
    def __init__(self, X, Y, kernel: OKernel, noise_variance: Optional[float] = None):
        self.X = np.asarray(X, dtype=np.float64).reshape(len(X), -1)
        self.Y = np.asarray(Y, dtype=np.float64).reshape(-1, 1)
        self.kernel = kernel
        nv = 1.0 if noise_variance is None else float(noise_variance)
        self.noise = OParam("variance", nv, lower=1e-6)

    # ordering: kernel.* < likelihood.variance (sorted attribute names on GPR)
    def trainable_params(self) -> List[OParam]:
        ps = [p for p in self.kernel.params() if p.trainable]
        if self.noise.trainable:
            ps.append(self.noise)
        return ps

    def get_u(self) -> np.ndarray:
        return np.array([p.u for p in self.trainable_params()], dtype=np.float64)

    def set_u(self, u) -> None:
        for p, v in zip(self.trainable_params(), np.asarray(u, dtype=np.float64)):
            p.set_u(float(v))

    def _Ky(self):
        """K + σn²I; a NOT_PD outcome (np.linalg.LinAlgError, as the Cholesky would give) where it
        cannot be formed: a hyperparameter outside (0, inf) — e.g. a Periodic period or lengthscale
        driven to 0 by a chaotic L-BFGS-B path, where sin(π·Δ/p)/ℓ is 0/0 — or a non-finite entry.
        The device reports the same points as not positive definite (its pivot test !(p > 0) fails on
        NaN) or as out-of-domain hyperparameters (InvalidParameterError); GPflow's fit raises out of
        Scipy.minimize there (GPR/model_trainer.py:18-19 catches nothing)."""
        for prm in self.kernel.params() + [self.noise]:
            if not (np.isfinite(prm.value) and prm.value > 0.0):
                raise np.linalg.LinAlgError(f"hyperparameter {prm.name}={prm.value} outside (0, inf): not positive definite")
        with np.errstate(all="ignore"):
            K = self.kernel.K(self.X)
        if not np.all(np.isfinite(K)):
            raise np.linalg.LinAlgError("K has non-finite entries: not positive definite")
        return K + self.noise.value * np.eye(K.shape[0])

    def log_marginal_likelihood(self) -> float:
        """logML = -½‖L⁻¹y‖² - Σ log L_ii - (N/2) log 2π  (gpflow.logdensities.multivariate_normal)."""
        L = np.linalg.cholesky(self._Ky())
        a = sla.solve_triangular(L, self.Y, lower=True)
        n = self.Y.shape[0]
        return float(-0.5 * np.sum(a * a) - np.sum(np.log(np.diag(L))) - 0.5 * n * LOG2PI)

    def loss_and_grad_u(self):
        """training_loss = -logML and its gradient w.r.t. the unconstrained trainables.

        ∂logML/∂θ = ½ αᵀ(∂K/∂θ)α − ½ tr(K⁻¹ ∂K/∂θ),  α = K⁻¹y;  ∂θ/∂u = sigmoid(u).
        """
        Ky = self._Ky()
        n = Ky.shape[0]
        c, low = sla.cho_factor(Ky, lower=True, check_finite=False)
        alpha = sla.cho_solve((c, low), self.Y, check_finite=False)[:, 0]
        logdet_half = float(np.sum(np.log(np.diag(c))))
        lml = float(-0.5 * np.dot(self.Y[:, 0], alpha) - logdet_half - 0.5 * n * LOG2PI)
        # K⁻¹ via LAPACK potri on the factor
        Kinv, info = sla.lapack.dpotri(c, lower=1)
        if info != 0:
            raise np.linalg.LinAlgError(f"dpotri info={info}")
        Kinv = np.tril(Kinv) + np.tril(Kinv, -1).T
        Wm = np.outer(alpha, alpha) - Kinv
        grads = []
        kparams = self.kernel.params()
        # (at a degenerate θ — ℓ ~ 1e-300 after a chaotic path — a ∂K/∂θ entry can be 0·inf = NaN:
        # reported as such, the caller compares the finite components)
        with np.errstate(all="ignore"):
            dks = self.kernel.dK(self.X)
        for p, dk in zip(kparams, dks):
            if p.trainable:
                grads.append(0.5 * float(np.sum(Wm * dk)) * p.dtheta_du())
        if self.noise.trainable:
            grads.append(0.5 * float(np.trace(Wm)) * self.noise.dtheta_du())
        return -lml, -np.array(grads, dtype=np.float64)

    def loss_and_grad_u_extended(self):
        """loss_and_grad_u with the linear algebra in x87 extended precision (np.longdouble, a
        64-bit significand: ~2000x fp64's precision) on the SAME fp64 K and ∂K/∂θ. The fp64
        gradient ½Σ(ααᵀ − K⁻¹)∘∂K is a cancellation whose error grows with cond(K); this is the
        near-exact value of the fp64 problem, used to tell where the fp64 oracle itself is off
        (tests/golden/make_golden.py stores it per fixture). O(N³) numpy vector ops: N ≲ 512."""
        ld = np.longdouble
        Ky = self._Ky().astype(ld)
        n = Ky.shape[0]
        L = np.zeros((n, n), dtype=ld)
        for j in range(n):
            s = Ky[j:, j] - L[j:, :j] @ L[j, :j]
            if s[0] <= 0:
                raise np.linalg.LinAlgError("not positive definite (extended precision)")
            L[j, j] = np.sqrt(s[0])
            L[j + 1:, j] = s[1:] / L[j, j]
        W = np.zeros((n, n), dtype=ld)          # W = L⁻¹ by forward substitution, column by column
        for i in range(n):
            W[i, :] = -(L[i, :i] @ W[:i, :])
            W[i, i] += 1
            W[i, :] /= L[i, i]
        y = self.Y[:, 0].astype(ld)
        z = W @ y
        alpha = W.T @ z
        Kinv = W.T @ W
        lml = -0.5 * (z @ z) - np.sum(np.log(np.diag(L))) - ld(0.5) * n * ld(LOG2PI)
        Wm = np.outer(alpha, alpha) - Kinv
        grads = []
        with np.errstate(all="ignore"):
            dks = self.kernel.dK(self.X)
        for p, dk in zip(self.kernel.params(), dks):
            if p.trainable:
                grads.append(float(ld(0.5) * np.sum(Wm * dk.astype(ld))) * p.dtheta_du())
        if self.noise.trainable:
            grads.append(float(ld(0.5) * np.trace(Wm)) * self.noise.dtheta_du())
        return -float(lml), -np.array(grads, dtype=np.float64)

    def predict_f(self, Xnew, full_cov=False):
        """GPflow base_conditional(kmn, kmm+σ²I, knn, err, white=False)."""
        Xnew = np.asarray(Xnew, dtype=np.float64).reshape(len(Xnew), -1)
        Lm = np.linalg.cholesky(self._Ky())
        Kmn = self.kernel.K(self.X, Xnew)
        A = sla.solve_triangular(Lm, Kmn, lower=True)
        if full_cov:
            fvar = self.kernel.K(Xnew) - A.T @ A
        else:
            fvar = self.kernel.K_diag(Xnew) - np.sum(A * A, axis=0)
        A2 = sla.solve_triangular(Lm.T, A, lower=False)
        fmean = A2.T @ self.Y
        return fmean, (fvar if full_cov else fvar[:, None])

    def predict_y(self, Xnew):
        m, v = self.predict_f(Xnew)
        return m, v + self.noise.value


@dataclass
class OFitResult:
    fun: float
    x: np.ndarray
    nfev: int
    nit: int
    success: bool
    message: str = ""
    history: list = field(default_factory=list)


def scipy_minimize(model: OGPR, maxiter: Optional[int] = 100, on_not_pd: str = "raise") -> OFitResult:
    """gpflow.optimizers.Scipy().minimize(model.training_loss, model.trainable_variables,
    options=dict(maxiter=...)) — scipy L-BFGS-B with jac=True, scipy defaults otherwise.
    on_not_pd: "raise" (GPflow: a failed Cholesky escapes the fit) or "inf" (the product's
    documented opt-in, optimizers.Scipy(on_not_pd="inf"): an infinite loss and a zero gradient
    at that point, so the line search backs off)."""
    x0 = model.get_u()

    def func(u):
        model.set_u(u)
        if on_not_pd == "inf":
            try:
                return model.loss_and_grad_u()
            except np.linalg.LinAlgError:
                return float("inf"), np.zeros_like(np.asarray(u, dtype=np.float64))
        return model.loss_and_grad_u()

    options = {} if maxiter is None else dict(maxiter=maxiter)
    res = scipy.optimize.minimize(func, x0, jac=True, method="L-BFGS-B", options=options)
    model.set_u(res.x)
    return OFitResult(float(res.fun), np.array(res.x), int(res.nfev), int(res.nit), bool(res.success),
                      str(res.message))


# ----------------------------------------------------------------------------------------
# data preparation restated from GPR/data_handler.py:26-65 (no network fetch)
# ----------------------------------------------------------------------------------------
def prepare_series(csv_path: str, train_start_date: str = "2024-02-01", column: str = "return"):
    """Returns (X [N,1] day offsets, Y [N,1] z-scored, mean, std) exactly as
    ``DataHandler.process_data`` (``GPR/data_handler.py:28-40``) + ``normalize_and_reshape``
    (``:55-65``): day offset from train_start (unnormalised), pct_change with the NaN in row 0
    filled by row 1's return, z-score with pandas' ddof=1 std."""
    import pandas as pd

    df = pd.read_csv(csv_path)
    df["date"] = pd.to_datetime(df["date"])
    start = pd.Timestamp(train_start_date)
    df["day_of_year"] = (df["date"] - start).dt.days
    df["return"] = df["close"].pct_change()
    first_return = df["return"].iloc[1]
    df = df.fillna({"return": first_return})
    df["intraday_return"] = (df["close"] - df["open"]) / df["open"]
    mean = df[column].mean()
    std = df[column].std()
    y = ((df[column] - mean) / std).values.astype(np.float64)
    x = df["day_of_year"].values.astype(np.float64)
    return x.reshape(-1, 1), y.reshape(-1, 1), float(mean), float(std)


# ----------------------------------------------------------------------------------------
# synthetic C2/C3 inputs — the same generator the bench uses
# ----------------------------------------------------------------------------------------
def synthetic_series(n: int, seed: int = 0, lengthscale: float = 64.0, n_features: int = 2048,
                     noise_std: float = 0.1):
    """X = arange(N)[:,None]; Y = zscore(ddof=1) of a random-Fourier-feature draw from
    SE(σ²=1, ℓ) plus N(0, noise_std²) noise.  O(N·R), seeded by numpy default_rng(seed)."""
    rng = np.random.default_rng(seed)
    x = np.arange(n, dtype=np.float64)
    w = rng.standard_normal(n_features) / lengthscale
    b = rng.uniform(0.0, 2.0 * math.pi, n_features)
    coef = rng.standard_normal(n_features)
    f = np.sqrt(2.0 / n_features) * (np.cos(np.outer(x, w) + b) @ coef)
    y = f + noise_std * rng.standard_normal(n)
    y = (y - y.mean()) / y.std(ddof=1)
    return x.reshape(-1, 1), y.reshape(-1, 1)


def reference_kernel_list():
    """The 8 kernels of GPR/main.py:105-114, fresh GPflow defaults."""
    SE, M12, RQ, EXP = OSquaredExponential, OMatern12, ORationalQuadratic, OExponential
    return [
        SE(), M12(), RQ(), EXP(),
        OSum([SE(), M12()]),
        OSum([EXP(), OPeriodic(SE()), OLinear()]),
        OSum([EXP(), OPeriodic(SE())]),
        OProduct([SE(), M12()]),
    ]
