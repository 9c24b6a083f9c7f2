"""Banded CPU restatement of the C2 evaluation — TEST INFRASTRUCTURE / CPU CONTEXT ONLY.

The same algorithm the device's band sweeps run, restated in numpy +
LAPACK on the CPU: K + σn²I of a SquaredExponential kernel on sorted 1-D inputs vanishes
exactly (fp64 exp underflow) beyond a band, so the evaluation is a block-banded Cholesky, a
banded solve and the selected inverse Z = K⁻¹ on the band (Takahashi recurrences), with the
gradient contraction ½Σ(ααᵀ − Z)∘∂K/∂θ over the band only. It computes what
``gp_oracle.OGPR.loss_and_grad_u`` computes (the GPflow 2.9.1 arithmetic of
``GPR/model_trainer.py:15-19``; r² in GPflow's ``square_distance`` form), differing only in
summation order; ``tests/test_band_oracle.py`` checks it against the dense oracle.

Why it exists: ``bench.py``'s ``cpu_baseline`` times the dense O(N³) oracle (the reference's
CPU path). That ratio mixes algorithm and hardware, so the bench also reports this
same-algorithm CPU figure beside it as context (VERDICT r03 "next" item 8): what the host
cores reach with the band algorithm, fits in parallel over the job's cores.

Who may import this: ``tests/`` and ``bench.py``'s cpu_baseline leg only. The product package
never imports it.
"""
from __future__ import annotations

import math
import time

import numpy as np
import scipy.linalg as sla
import scipy.optimize

from oracle.gp_oracle import LOG2PI, sigmoid, softplus, softplus_inverse

UNDERFLOW = 746.0  # exp(−a) is exactly 0.0 in fp64 for a ≥ 745.14 (DESIGN §3c's margin)


def _r2(a, b):
    """GPflow square_distance of pre-scaled 1-D inputs a = x/ℓ, b = x'/ℓ: −2ab + (a² + b²)."""
    return -2.0 * np.multiply.outer(a, b) + (np.add.outer(a * a, b * b))


def se1_half_band(x, ell):
    """Largest |i − j| with K_ij != 0 (exp(−r²/2) not underflowed) for sorted 1-D x."""
    a = np.asarray(x, np.float64).ravel() / ell
    n = a.size
    for d in range(1, n):
        r2 = -2.0 * (a[d:] * a[:-d]) + (a[d:] * a[d:] + a[:-d] * a[:-d])
        if np.all(0.5 * r2 >= UNDERFLOW):
            return d - 1
    return n - 1


def se1_band_eval(x, y, ell, var, noise):
    """logML, ∂logML/∂(ℓ, σ², σn²), α and diag(K⁻¹) of K = SE(ℓ, σ²)(x, x) + σn²I by the
    block-tridiagonal form (block size ≥ the half band), x sorted 1-D."""
    x = np.asarray(x, np.float64).ravel()
    y = np.asarray(y, np.float64).ravel()
    n = x.size
    w = se1_half_band(x, ell)
    bs = max(1, w)
    nb = -(-n // bs)
    npad = nb * bs
    a = np.zeros(npad)
    a[:n] = x / ell
    yp = np.zeros(npad)
    yp[:n] = y
    valid = np.arange(npad) < n

    def kblock(i, j):
        ri, rj = slice(i * bs, (i + 1) * bs), slice(j * bs, (j + 1) * bs)
        r2 = _r2(a[ri], a[rj])
        e = np.exp(-0.5 * r2)
        m = np.logical_and.outer(valid[ri], valid[rj])
        e = np.where(m, e, 0.0)
        return e, r2 * m

    # forward: L_kk, W_kk = L_kk⁻¹, P_k = L_{k+1,k}; z = L⁻¹y
    E, R2, Wd, Pd = [], [], [], []
    logdet = 0.0
    z = np.zeros(npad)
    carry = None
    for k in range(nb):
        e, r2 = kblock(k, k)
        E.append(e)
        R2.append(r2)
        A = var * e
        idx = np.arange(k * bs, (k + 1) * bs)
        A[np.diag_indices(bs)] += np.where(valid[idx], noise, 1.0)
        A[np.diag_indices(bs)] = np.where(valid[idx], A[np.diag_indices(bs)], 1.0)
        if carry is not None:
            A -= carry
        Lk = np.linalg.cholesky(A)
        W = sla.solve_triangular(Lk, np.eye(bs), lower=True)
        Wd.append(W)
        logdet += 2.0 * float(np.sum(np.log(np.diag(Lk)[valid[idx]])))
        rhs = yp[idx] - (Pd[-1] @ z[idx - bs] if k > 0 else 0.0)
        z[idx] = W @ rhs
        if k + 1 < nb:
            eo, r2o = kblock(k + 1, k)
            E.append(eo)
            R2.append(r2o)
            P = (var * eo) @ W.T
            Pd.append(P)
            carry = P @ P.T
    # α = L⁻ᵀ z
    alpha = np.zeros(npad)
    for k in range(nb - 1, -1, -1):
        idx = np.arange(k * bs, (k + 1) * bs)
        t = z[idx] - (Pd[k].T @ alpha[idx + bs] if k + 1 < nb else 0.0)
        alpha[idx] = Wd[k].T @ t
    # selected inverse (block tridiagonal Takahashi) + the gradient contraction over the band
    g_ell = g_var = g_noise = 0.0
    diagz = np.zeros(npad)
    Znext = None
    for k in range(nb - 1, -1, -1):
        W = Wd[k]
        idx = np.arange(k * bs, (k + 1) * bs)
        if k + 1 < nb:
            G = Pd[k] @ W
            Zoff = -Znext @ G                    # Z_{k+1,k}
            Zkk = W.T @ W - G.T @ Zoff
            eo, r2o = E[2 * k + 1], R2[2 * k + 1]
            V = np.outer(alpha[idx + bs], alpha[idx]) - Zoff
            Ko = var * eo
            g_ell += 2.0 * float(np.sum(V * Ko * r2o))
            g_var += 2.0 * float(np.sum(V * eo))
        else:
            Zkk = W.T @ W
        e, r2 = E[2 * k], R2[2 * k]
        V = np.outer(alpha[idx], alpha[idx]) - Zkk
        g_ell += float(np.sum(V * (var * e) * r2))
        g_var += float(np.sum(V * e))
        g_noise += float(np.sum(np.diag(V)[valid[idx]]))
        diagz[idx] = np.diag(Zkk)
        Znext = Zkk
    lml = -0.5 * float(z[:n] @ z[:n]) - 0.5 * logdet - 0.5 * n * LOG2PI
    grad = np.array([0.5 * g_ell / ell, 0.5 * g_var, 0.5 * g_noise])
    return lml, grad, alpha[:n], diagz[:n]


class OBandGPR:
    """GPR with SquaredExponential on sorted 1-D inputs evaluated by the band algorithm; the
    same interface as gp_oracle.OGPR for scipy_minimize (loss_and_grad_u over (ℓ, σ²) with
    σn² fixed, or (ℓ, σ², σn²) with noise trainable)."""

    def __init__(self, X, Y, noise_variance=1e-5, noise_trainable=False):
        self.x = np.asarray(X, np.float64).ravel()
        self.y = np.asarray(Y, np.float64).ravel()
        self.ell, self.var, self.noise = 1.0, 1.0, float(noise_variance)
        self.noise_trainable = noise_trainable

    def get_u(self):
        u = [float(softplus_inverse(self.ell)), float(softplus_inverse(self.var))]
        if self.noise_trainable:
            u.append(float(softplus_inverse(self.noise - 1e-6)))
        return np.array(u)

    def set_u(self, u):
        self.ell, self.var = float(softplus(u[0])), float(softplus(u[1]))
        if self.noise_trainable:
            self.noise = 1e-6 + float(softplus(u[2]))

    def loss_and_grad_u(self):
        u = self.get_u()
        lml, g, _, _ = se1_band_eval(self.x, self.y, self.ell, self.var, self.noise)
        gu = g[:len(u)] * sigmoid(u)
        return -lml, -gu

    def predict_f_train(self):
        """predict_f at the training inputs: mean = y − σn²α, var = σn² − σn⁴ diag(K⁻¹)."""
        _, _, alpha, dz = se1_band_eval(self.x, self.y, self.ell, self.var, self.noise)
        return self.y - self.noise * alpha, self.noise - self.noise ** 2 * dz


def fit(x, y, noise=1e-5, maxiter=100):
    """GPR/model_trainer.py:15-20 on the band algorithm: GPflow defaults, σn² fixed, scipy
    L-BFGS-B (maxiter 100), then predict_f at the training inputs. Returns (fun, x, nfev)."""
    m = OBandGPR(x, y, noise)

    def func(u):
        m.set_u(u)
        return m.loss_and_grad_u()

    r = scipy.optimize.minimize(func, m.get_u(), jac=True, method="L-BFGS-B", options=dict(maxiter=maxiter))
    m.set_u(r.x)
    m.predict_f_train()
    return float(r.fun), np.array(r.x), int(r.nfev)


def _fit_seed(args):
    n, seed, noise = args
    from oracle.gp_oracle import synthetic_series
    import threadpoolctl
    with threadpoolctl.threadpool_limits(limits=1):
        x, y = synthetic_series(n, seed)
        t0 = time.perf_counter()
        out = fit(x, y, noise)
        return out[2], time.perf_counter() - t0


def parallel_fits_per_s(n, seeds, workers, noise=1e-5):
    """Whole fits (band algorithm + L-BFGS-B + predict) of the C2 series `seeds`, one per
    process on `workers` processes (BLAS single-threaded in each): (fits/s, mean nfev,
    mean seconds per fit)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    with ctx.Pool(workers) as pool:
        pool.map(_fit_seed, [(256, 0, noise)] * workers)  # workers up, modules imported
        t0 = time.perf_counter()
        res = pool.map(_fit_seed, [(n, s, noise) for s in seeds], chunksize=1)
        dt = time.perf_counter() - t0
    return len(seeds) / dt, float(np.mean([r[0] for r in res])), float(np.mean([r[1] for r in res]))


if __name__ == "__main__":  # quick timing: python -m oracle.band_oracle
    import sys
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    from oracle.gp_oracle import synthetic_series
    x, y = synthetic_series(n, 0)
    t0 = time.perf_counter()
    for _ in range(5):
        se1_band_eval(x, y, 1.18, 1.0, 1e-5)
    print(f"N={n}: {(time.perf_counter() - t0) / 5 * 1e3:.2f} ms per eval, half band {se1_half_band(x, 1.18)}")
    t0 = time.perf_counter()
    print(fit(x, y), f"{time.perf_counter() - t0:.2f} s per fit")
