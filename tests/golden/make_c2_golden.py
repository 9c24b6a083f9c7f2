"""Full-size fixtures for the headline configuration C2 (BASELINE.json configs[1]):
synthetic 1-D series, N = 4096, X = day offsets 0..4095, Y = the C2 generator
(oracle.synthetic_series), SquaredExponential at GPflow defaults, σn² = 1e-5 fixed — the
protocol of GPR/model_trainer.py:15-20 that bench.py times.

Run in the build container (a few minutes on 8 cores; nothing here reads /root/reference):

    python tests/golden/make_c2_golden.py

Writes tests/golden/c2_n4096.npz with, per seed s in {0, 1} (keys prefixed "s<seed>|"):
  y                         the generated series (x is arange(4096))
  ell|<l>|loss, |grad_u     training_loss and ∂/∂u (u = [ℓ, σ²] unconstrained, noise fixed) at
                            θ = (ℓ, σ² = 1), ℓ ∈ {1, 1.18, 1.72}, r² formed as GPflow forms it
                            (oracle R2_FORM "gpflow": square_distance on X/ℓ)
  ell|<l>|grad_u_torch      the same gradient by torch-fp64 reverse-mode autodiff through the
                            GPflow-form K (an independent restatement; agreement is checked here)
  ell|<l>|loss_direct, |grad_u_direct   the same with r² from direct differences (documentation:
                            how far the two forms of r² move the numbers at this size)
  fit|x, fit|loss, fit|nfev, fit|nit, fit|theta   gpflow.optimizers.Scipy().minimize(maxiter=100)
  fit|hist_u, fit|hist_f    every evaluation the L-BFGS-B driver requested (u, loss), in order
  pred|fmean, pred|fvar     predict_f at the training inputs at the fitted θ
"""
from __future__ import annotations

import math
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle import gp_oracle as O  # noqa: E402

N = 4096
NOISE = 1e-5
SEEDS = (0, 1)
ELLS = (1.0, 1.18, 1.72)


def torch_grad(x, y, ell, var, noise):
    """∂training_loss/∂u by torch autograd through GPflow-form K (tests/test_oracle.py style)."""
    import torch
    torch.set_default_dtype(torch.float64)
    u = torch.tensor([float(O.softplus_inverse(ell)), float(O.softplus_inverse(var))], requires_grad=True)
    X = torch.tensor(x)
    Y = torch.tensor(y)
    el = torch.nn.functional.softplus(u[0])
    vr = torch.nn.functional.softplus(u[1])
    A = X / el
    s = (A * A).sum(-1, keepdim=True)
    r2 = -2.0 * (A @ A.T) + (s + s.T)
    K = vr * torch.exp(-0.5 * r2) + noise * torch.eye(len(x))
    L = torch.linalg.cholesky(K)
    a = torch.linalg.solve_triangular(L, Y, upper=False)
    lml = -0.5 * (a * a).sum() - torch.log(torch.diagonal(L)).sum() - 0.5 * len(x) * math.log(2 * math.pi)
    (-lml).backward()
    return u.grad.numpy().copy()


def main():
    out = {"n": np.array([N]), "noise": np.array([NOISE]), "ells": np.array(ELLS)}
    for seed in SEEDS:
        t0 = time.time()
        x, y = O.synthetic_series(N, seed)
        p = f"s{seed}|"
        out[p + "y"] = y[:, 0]
        for ell in ELLS:
            k = O.OSquaredExponential(lengthscales=ell)
            m = O.OGPR(x, y, k, noise_variance=NOISE)
            m.noise.trainable = False
            loss, g = m.loss_and_grad_u()
            q = f"{p}ell|{ell}|"
            out[q + "loss"] = np.array([loss])
            out[q + "grad_u"] = g
            gt = torch_grad(x, y, ell, 1.0, NOISE)
            out[q + "grad_u_torch"] = gt
            rel = np.max(np.abs(gt - g)) / np.max(np.abs(g))
            assert rel < 1e-7, (seed, ell, g, gt)
            O.R2_FORM = "direct"
            try:
                ld, gd = m.loss_and_grad_u()
            finally:
                O.R2_FORM = "gpflow"
            out[q + "loss_direct"] = np.array([ld])
            out[q + "grad_u_direct"] = gd
            print(f"seed {seed} ell {ell}: loss {loss:.12g} grad {g} | torch rel {rel:.2e} | "
                  f"direct form: loss rel {abs(ld - loss) / abs(loss):.2e}, "
                  f"grad rel {np.max(np.abs(gd - g)) / np.max(np.abs(g)):.2e}", flush=True)
        # the full fit, recording every requested evaluation
        k = O.OSquaredExponential()
        m = O.OGPR(x, y, k, noise_variance=1.0)
        m.noise.value = NOISE
        m.noise.trainable = False
        hist = []
        orig = m.loss_and_grad_u

        def rec():
            f, g = orig()
            hist.append((m.get_u().copy(), f))
            return f, g

        m.loss_and_grad_u = rec
        r = O.scipy_minimize(m, 100)
        out[p + "fit|x"] = np.asarray(r.x)
        out[p + "fit|loss"] = np.array([r.fun])
        out[p + "fit|nfev"] = np.array([r.nfev])
        out[p + "fit|nit"] = np.array([r.nit])
        out[p + "fit|theta"] = np.array([pp.value for pp in k.params()])
        out[p + "fit|hist_u"] = np.array([h[0] for h in hist])
        out[p + "fit|hist_f"] = np.array([h[1] for h in hist])
        mu, var = m.predict_f(x)
        out[p + "pred|fmean"] = mu[:, 0]
        out[p + "pred|fvar"] = var[:, 0]
        print(f"seed {seed}: fit loss {r.fun:.12g} theta {out[p + 'fit|theta']} nfev {r.nfev} nit {r.nit} "
              f"({time.time() - t0:.0f} s)", flush=True)
    np.savez_compressed(os.path.join(HERE, "c2_n4096.npz"), **out)


if __name__ == "__main__":
    main()
