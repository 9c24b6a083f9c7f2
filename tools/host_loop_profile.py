"""Host cost of the bench's fitting loop without a GPU: the stepped driver (minimize_stream over a
ModelStream of GPR models, as bench.py's FitWorker runs it) against a stand-in engine whose
"device call" is a few vectorised numpy lines, so everything measured is host work: model
construction, rebinds, θ rows, the L-BFGS-B steps, results and the predict bookkeeping.
Prints GPX_DRIVER_STATS-style phase totals per fit and evaluation, and optionally a cProfile.

usage: python tools/host_loop_profile.py [--fits 4096] [--width 1024] [--profile] [--python-loop]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("GPX_DRIVER_STATS", "1")
import portfoliooptgp_amd as gpx  # noqa: E402
from portfoliooptgp_amd import _native as N  # noqa: E402


class StandInEngine:
    """lml(θ) = −Σ_p (log θ_p − log t_p)², t from the bound series (the driver-test engine),
    evaluated for a whole call in numpy; predict_train returns [n, 1] tensors of θ."""

    def __init__(self, B, n):
        self.B, self.device, self.n = B, 0, n
        self.target = np.ones((B, 2))
        self.n_params = np.full(B, 2)
        self.mu = torch.zeros(B, n, 1, dtype=torch.float64)

    def rebind(self, b, X, Y, spec):
        y = np.asarray(Y[:64], dtype=np.float64).reshape(-1)
        self.target[b] = [1.0 + abs(y.mean()) * 3.0, 0.5 + y.std()]

    def lml_grad(self, rows, theta, wait_deferred=True):
        r = np.asarray(rows)
        lml = np.full(self.B, np.nan)
        grad = np.zeros((self.B, N.GPX_THETA_STRIDE))
        d = np.log(theta[r, :2]) - np.log(self.target[r])
        lml[r] = -np.sum(d * d, axis=1)
        grad[r, :2] = -2.0 * d / theta[r, :2]
        return lml, grad, np.zeros(self.B, dtype=np.int32)

    def _predict_train(self, rows, theta, add_noise, column=False):
        return [self.mu[r] for r in rows], [self.mu[r] for r in rows], None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fits", type=int, default=4096)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--profile", action="store_true")
    ap.add_argument("--python-loop", action="store_true", help="GPX_NATIVE_LBFGSB=0")
    a = ap.parse_args()
    if a.python_loop:
        os.environ["GPX_NATIVE_LBFGSB"] = "0"
    rng = np.random.default_rng(0)
    series = [(np.arange(a.n, dtype=np.float64)[:, None], rng.standard_normal((a.n, 1))) for _ in range(64)]

    def make_model(i):
        m = gpx.models.GPR(data=series[i % len(series)], kernel=gpx.kernels.SquaredExponential())
        m.likelihood.variance.assign(1e-5)
        gpx.set_trainable(m.likelihood.variance, False)
        return m

    eng = StandInEngine(a.width, a.n)
    opt = gpx.optimizers.Scipy()
    pr = cProfile.Profile() if a.profile else None
    models = gpx.optimizers.ModelStream(a.fits, make_model, input_dim=1, max_points=a.n)
    t0 = time.perf_counter()
    if pr:
        pr.enable()
    res, _ = opt.minimize_stream(models, width=a.width, engine=eng, predict_train=True, options=dict(maxiter=100))
    if pr:
        pr.disable()
    dt = time.perf_counter() - t0
    st = dict(opt.last_stats or {})
    ev = st.get("fit_evals", 0)
    print(f"fits {a.fits} in {dt:.3f} s: {dt / a.fits * 1e6:.1f} us per fit, evaluations {ev} "
          f"({ev / a.fits:.1f} per fit), rounds {st.get('rounds')}")
    for k, v in st.items():
        if isinstance(v, float):
            print(f"  {k:14s} {v:8.3f} s  {v / a.fits * 1e6:8.2f} us/fit  {v / max(ev, 1) * 1e6:8.3f} us/eval")
    if pr:
        s = pstats.Stats(pr)
        s.sort_stats("tottime").print_stats(35)


if __name__ == "__main__":
    main()
