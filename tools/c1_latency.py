"""Where one small-N evaluation of the drop-in pattern spends its time: the
reference fits one GPR at a time (GPR/model_trainer.py:14-20) at N = 89 / 19 / 5 (AAPL d/w/m), so
each loss+gradient is one B = 1 device call. Per N, microseconds per evaluation of
  model   m.loss_and_grad_unconstrained()           (the whole Python + native path)
  engine  Engine.lml_grad([0], theta)               (the engine wrapper + native)
  native  the ctypes call of gpx_batch_lml_grad with prepared arguments (native + device)
and the CPU oracle's evaluation. usage: python tools/c1_latency.py [--n 5,19,89] [--evals 400]"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import portfoliooptgp_amd as gpx  # noqa: E402
from portfoliooptgp_amd import _native as N  # noqa: E402


def _med(f, reps, inner):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        for _ in range(inner):
            f()
        ts.append((time.perf_counter() - t0) / inner)
    return sorted(ts)[len(ts) // 2] * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", default="5,19,89")
    ap.add_argument("--evals", type=int, default=400)
    ap.add_argument("--oracle", type=int, default=1)
    a = ap.parse_args()
    d = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                             "kernel_cases.npz"))
    by_n = {int(d[f"data|aapl_{tf}|x"].shape[0]): (d[f"data|aapl_{tf}|x"], d[f"data|aapl_{tf}|y"]) for tf in "dwm"}
    for n in [int(v) for v in a.n.split(",")]:
        x, y = by_n[n]
        m = gpx.models.GPR((x, y), kernel=gpx.kernels.SquaredExponential())
        m.likelihood.variance.assign(1e-5)
        gpx.set_trainable(m.likelihood.variance, False)
        m.loss_and_grad_unconstrained()
        eng, b = m.engine()
        theta = np.ones((eng.B, N.GPX_THETA_STRIDE))
        theta[b] = m.theta_row()
        inner = max(1, a.evals // 5)
        t_model = _med(lambda: m.loss_and_grad_unconstrained(), 5, inner)
        t_eng = _med(lambda: eng.lml_grad([b], theta), 5, inner)
        act = np.array([b], dtype=np.int32)
        lml = np.zeros(eng.B)
        grad = np.zeros((eng.B, N.GPX_THETA_STRIDE))
        info = np.zeros(eng.B, dtype=np.int32)
        args = (eng.handle, 1, act.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                theta.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), lml.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                grad.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), info.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                eng._stream())
        f = eng.lib.gpx_batch_lml_grad
        t_native = _med(lambda: f(*args), 5, inner)
        out = {"N": n, "us_model": t_model, "us_engine": t_eng, "us_native": t_native}
        if a.oracle:
            from oracle import gp_oracle as O
            om = O.OGPR(x, y, O.OSquaredExponential(), noise_variance=1e-5)
            om.noise.trainable = False
            om.loss_and_grad_u()
            out["us_cpu_oracle"] = _med(lambda: om.loss_and_grad_u(), 5, inner)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
