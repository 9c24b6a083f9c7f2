"""Latency of the unbatched drop-in call pattern (GPR/model_trainer.py:15-20 as the reference
runs it: one model at a time) — per loss+gradient evaluation and per full fit, GPU vs the CPU
oracle, at the reference's own sizes (N = 89 / 19 / 5: AAPL d/w/m) and larger N.
usage: python tools/solo_latency.py [--n 5,19,89,256,1024]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import portfoliooptgp_amd as gpx  # noqa: E402
from oracle import gp_oracle as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="5,19,89,256,1024")
    ap.add_argument("--evals", type=int, default=200)
    a = ap.parse_args()
    for n in [int(v) for v in a.n.split(",")]:
        x, y = O.synthetic_series(n, seed=1)
        m = gpx.models.GPR((x, y), kernel=gpx.kernels.SquaredExponential())
        m.likelihood.variance.assign(1e-5)
        gpx.set_trainable(m.likelihood.variance, False)
        m.loss_and_grad_unconstrained()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.evals):
            m.loss_and_grad_unconstrained()
        ev_gpu = (time.perf_counter() - t0) / a.evals
        om = O.OGPR(x, y, O.OSquaredExponential(), noise_variance=1e-5)
        om.noise.trainable = False
        om.loss_and_grad_u()
        reps = max(3, min(a.evals, int(2e8 / n ** 3) + 3))
        t0 = time.perf_counter()
        for _ in range(reps):
            om.loss_and_grad_u()
        ev_cpu = (time.perf_counter() - t0) / reps
        m2 = gpx.models.GPR((x, y), kernel=gpx.kernels.SquaredExponential())
        m2.likelihood.variance.assign(1e-5)
        gpx.set_trainable(m2.likelihood.variance, False)
        t0 = time.perf_counter()
        r = gpx.optimizers.Scipy().minimize(m2.training_loss, m2.trainable_variables, options=dict(maxiter=100))
        m2.predict_f(x)
        fit_gpu = time.perf_counter() - t0
        print(json.dumps({"N": n, "eval_us_gpu": ev_gpu * 1e6, "eval_us_cpu_oracle": ev_cpu * 1e6,
                          "fit_ms_gpu": fit_gpu * 1e3, "nfev": int(r.nfev)}), flush=True)


if __name__ == "__main__":
    main()
