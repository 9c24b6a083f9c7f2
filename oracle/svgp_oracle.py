"""CPU oracle for the SVGP path — TEST INFRASTRUCTURE ONLY.

Restates GPflow 2.9.1 ``models.SVGP`` with a Gaussian likelihood, the defaults the reference
uses at ``test_scripts/SVGP.py:461-474`` (and ``test_scripts/GPR.py:118-138``):
``whiten=True``, full lower-triangular ``q_sqrt``, ``q_diag=False``, zero mean function,
``num_latent_gps=1``, inducing points ``Z`` trainable, likelihood variance frozen by the caller:

    Kmm   = k(Z, Z) + 1e-6 I            (gpflow.covariances.Kuu with default_jitter())
    L     = chol(Kmm);  A = L⁻¹ k(Z, X)
    μ     = Aᵀ q_mu
    v     = k_diag(X) − Σ_m A² + Σ_m (q_sqrtᵀ A)²          (conditionals.base_conditional, white)
    E_n   = −½ log 2π − ½ log σ² − ½ ((y_n − μ_n)² + v_n) / σ²   (Gaussian.variational_expectations)
    KL    = ½ (‖q_mu‖² + ‖q_sqrt‖_F² − M − Σ log q_sqrt_ii²)      (kullback_leiblers.gauss_kl, K=None)
    ELBO  = (num_data / N_batch) Σ_n E_n − KL;   training_loss = −ELBO

Trainable-variable order (tf.Module flattens attributes by sorted name):
``inducing_variable.Z`` < ``kernel.*`` < ``likelihood.variance`` < ``q_mu`` < ``q_sqrt``.
``q_sqrt`` is stored unconstrained through ``tfp.bijectors.FillTriangular`` (restated below as
``fill_triangular`` / ``fill_triangular_inverse``).

The gradients here are written out by hand the way reverse-mode autodiff would produce them
from the forward above (through L with the TF Cholesky gradient); they are pinned by central
finite differences of ``elbo`` in ``tests/test_svgp_oracle.py``. GPflow itself is not
importable here: no reference-run fixture exists for SVGP (parity is against this
restatement).
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import scipy.linalg as sla

from .gp_oracle import LOG2PI, OKernel, OParam, sigmoid

JITTER = 1e-6


def fill_triangular(x: np.ndarray) -> np.ndarray:
    """tfp.math.fill_triangular(x, upper=False)."""
    x = np.asarray(x, dtype=np.float64)
    m = x.shape[-1]
    n = int(math.isqrt(8 * m + 1) - 1) // 2
    if n * (n + 1) // 2 != m:
        raise ValueError("length is not a triangular number")
    full = np.concatenate([x[n:], x[::-1]]).reshape(n, n)
    return np.tril(full)


def fill_triangular_inverse(L: np.ndarray) -> np.ndarray:
    """tfp.math.fill_triangular_inverse(L, upper=False)."""
    L = np.asarray(L, dtype=np.float64)
    n = L.shape[-1]
    m = n * (n + 1) // 2
    initial = L[-1, ::-1]
    tri = L[:-1, :]
    consolidated = tri + tri[::-1, ::-1]
    return np.concatenate([initial, consolidated.reshape(-1)[: m - n]])


def cholesky_grad(L: np.ndarray, Lbar: np.ndarray) -> np.ndarray:
    """TF's gradient of cholesky (tensorflow/python/ops/linalg_grad.py _CholeskyGrad):
    Σ̄ = ½ (S + Sᵀ),  S = L⁻ᵀ Φ(Lᵀ L̄) L⁻¹,  Φ = lower triangle with halved diagonal."""
    Linv = sla.solve_triangular(L, np.eye(L.shape[0]), lower=True)
    middle = L.T @ Lbar
    middle = np.tril(middle)
    middle[np.diag_indices_from(middle)] *= 0.5
    g = Linv.T @ middle @ Linv
    return 0.5 * (g + g.T)


class OSVGP:
    def __init__(self, kernel: OKernel, Z, num_data: Optional[float] = None, noise_variance: float = 1.0,
                 q_mu=None, q_sqrt=None):
        self.kernel = kernel
        self.Z = np.array(Z, dtype=np.float64).reshape(len(Z), -1)
        M = self.Z.shape[0]
        self.num_data = num_data
        self.noise = OParam("variance", float(noise_variance), lower=1e-6)
        self.q_mu = np.zeros(M) if q_mu is None else np.array(q_mu, dtype=np.float64).reshape(M)
        self.q_sqrt = np.eye(M) if q_sqrt is None else np.tril(np.array(q_sqrt, dtype=np.float64).reshape(M, M))
        self.Z_trainable = True
        self.q_trainable = True

    # ---------------------------------------------------------------- forward ---------
    def _parts(self, X, Y):
        X = np.asarray(X, np.float64).reshape(len(X), -1)
        Y = np.asarray(Y, np.float64).reshape(-1)
        Z, m, R = self.Z, self.q_mu, np.tril(self.q_sqrt)
        M = Z.shape[0]
        Kmm = self.kernel.K(Z) + JITTER * np.eye(M)
        L = np.linalg.cholesky(Kmm)
        Kmn = self.kernel.K(Z, X)
        A = sla.solve_triangular(L, Kmn, lower=True)
        B = R.T @ A
        mu = A.T @ m
        v = self.kernel.K_diag(X) - np.sum(A * A, axis=0) + np.sum(B * B, axis=0)
        s2 = self.noise.value
        ve = -0.5 * LOG2PI - 0.5 * math.log(s2) - 0.5 * ((Y - mu) ** 2 + v) / s2
        scale = 1.0 if self.num_data is None else float(self.num_data) / X.shape[0]
        kl = 0.5 * (m @ m + np.sum(R * R) - M - np.sum(np.log(np.diag(R) ** 2)))
        elbo = scale * ve.sum() - kl
        return dict(X=X, Y=Y, Z=Z, m=m, R=R, L=L, Kmn=Kmn, A=A, B=B, mu=mu, v=v, s2=s2,
                    scale=scale, kl=kl, elbo=elbo)

    def elbo(self, X, Y) -> float:
        return float(self._parts(X, Y)["elbo"])

    def training_loss(self, X, Y) -> float:
        return -self.elbo(X, Y)

    def predict_f(self, Xnew):
        Xnew = np.asarray(Xnew, np.float64).reshape(len(Xnew), -1)
        M = self.Z.shape[0]
        L = np.linalg.cholesky(self.kernel.K(self.Z) + JITTER * np.eye(M))
        A = sla.solve_triangular(L, self.kernel.K(self.Z, Xnew), lower=True)
        B = np.tril(self.q_sqrt).T @ A
        mu = A.T @ self.q_mu
        v = self.kernel.K_diag(Xnew) - np.sum(A * A, axis=0) + np.sum(B * B, axis=0)
        return mu[:, None], v[:, None]

    def predict_y(self, Xnew):
        mu, v = self.predict_f(Xnew)
        return mu, v + self.noise.value

    # ---------------------------------------------------------------- gradients -------
    def elbo_and_grads(self, X, Y):
        """ELBO and its gradients in constrained space:
        dict(Z [M,D], theta [P] (kernel params order), noise, q_mu [M], q_sqrt [M,M] lower)."""
        p = self._parts(X, Y)
        X, Y, Z, m, R, L, Kmn, A, B = (p[k] for k in ("X", "Y", "Z", "m", "R", "L", "Kmn", "A", "B"))
        s, s2, mu, v = p["scale"], p["s2"], p["mu"], p["v"]
        M = Z.shape[0]
        g_mu = s * (Y - mu) / s2
        g_v = np.full_like(Y, -0.5 * s / s2)
        # A appears in μ = Aᵀm and v (−ΣA² + Σ(RᵀA)²)
        Abar = np.outer(m, g_mu) + (-2.0 * A + 2.0 * R @ B) * g_v[None, :]
        Rbar = 2.0 * (A * g_v[None, :]) @ B.T - R + np.diag(1.0 / np.diag(R))
        mbar = A @ g_mu - m
        # A = L⁻¹ Kmn
        Kmn_bar = sla.solve_triangular(L.T, Abar, lower=False)
        Lbar = -Kmn_bar @ A.T
        Kmm_bar = cholesky_grad(L, np.tril(Lbar))
        # kernel hyper-parameters through Kmm, Kmn and k_diag (one joint dK over [Z; X])
        XA = np.concatenate([Z, X])
        dKs = self.kernel.dK(XA)
        dtheta = np.array([np.sum(Kmm_bar * d[:M, :M]) + np.sum(Kmn_bar * d[:M, M:])
                           + np.sum(g_v * np.diag(d)[M:]) for d in dKs])
        # inducing inputs: ∂k(z_m, ·)/∂z_m
        dZ = np.einsum("mn,mnd->md", Kmn_bar, self.kernel.dK_dX1(Z, X))
        dZ += 2.0 * np.einsum("mj,mjd->md", Kmm_bar, self.kernel.dK_dX1(Z, Z))
        dnoise = s * np.sum(-0.5 / s2 + 0.5 * ((Y - mu) ** 2 + v) / (s2 * s2))
        return p["elbo"], dict(Z=dZ, theta=dtheta, noise=dnoise, q_mu=mbar, q_sqrt=np.tril(Rbar))

    # ---------------------------------------------------------------- unconstrained ---
    def trainable_params(self):
        return [q for q in self.kernel.params() if q.trainable] + ([self.noise] if self.noise.trainable else [])

    def get_u(self) -> np.ndarray:
        parts = []
        if self.Z_trainable:
            parts.append(self.Z.ravel())
        parts.append(np.array([q.u for q in self.trainable_params()]))
        if self.q_trainable:
            parts.append(self.q_mu.ravel())
            parts.append(fill_triangular_inverse(self.q_sqrt))
        return np.concatenate(parts)

    def set_u(self, u) -> None:
        u = np.asarray(u, dtype=np.float64)
        o = 0
        if self.Z_trainable:
            self.Z = u[o:o + self.Z.size].reshape(self.Z.shape).copy()
            o += self.Z.size
        for q in self.trainable_params():
            q.set_u(float(u[o]))
            o += 1
        if self.q_trainable:
            M = self.q_mu.size
            self.q_mu = u[o:o + M].copy()
            o += M
            self.q_sqrt = fill_triangular(u[o:o + M * (M + 1) // 2])

    def loss_and_grad_u(self, X, Y):
        """(training_loss, ∂loss/∂u) in the flattened trainable-variable order."""
        elbo, g = self.elbo_and_grads(X, Y)
        kp = self.kernel.params()
        parts = []
        if self.Z_trainable:
            parts.append(-g["Z"].ravel())
        gt = []
        for i, q in enumerate(kp):
            if q.trainable:
                gt.append(-g["theta"][i] * q.dtheta_du())
        if self.noise.trainable:
            gt.append(-g["noise"] * self.noise.dtheta_du())
        parts.append(np.array(gt))
        if self.q_trainable:
            parts.append(-g["q_mu"].ravel())
            parts.append(-fill_triangular_inverse(g["q_sqrt"]))
        return -float(elbo), np.concatenate(parts)
