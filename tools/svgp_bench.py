"""Time one SVGP ELBO+gradient evaluation at the C5 shape (N=65536, M=1024, D=1, SE) on one
GPU, and the predict at N* points. Usage: python tools/svgp_bench.py [--n N] [--m M] [--reps R]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import portfoliooptgp_amd as gpx  # noqa: E402
from portfoliooptgp_amd.engine import SVGPEngine  # noqa: E402
from portfoliooptgp_amd.kernels import compile_spec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--m", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu", action="store_true",
                    help="also time one ELBO+gradient evaluation of the CPU oracle (oracle/svgp_oracle.py)")
    a = ap.parse_args()
    n, M = a.n, a.m
    rng = np.random.default_rng(0)
    X = np.sort(rng.uniform(0, 360, (n, 1)), axis=0)
    Y = np.sin(X / 20.0) + 0.1 * rng.standard_normal((n, 1))
    Z = np.linspace(0, 360, M)[:, None]
    k = gpx.kernels.SquaredExponential(lengthscales=2.0, variance=1.0)
    eng = SVGPEngine(X, Y, compile_spec(k, 1), M, num_data=n)
    theta = np.ones(16)
    theta[:3] = [2.0, 1.0, 1e-4]
    q = rng.standard_normal(M) * 0.3
    R = np.tril(rng.standard_normal((M, M)) * 1e-3)
    R[np.diag_indices(M)] = rng.uniform(0.05, 0.2, M)
    eng.elbo_grad(theta, Z, q, R)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        eng.elbo_grad(theta, Z, q, R)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.reps
    Mp = (M + 63) // 64 * 64
    big = 3.0 * Mp * Mp * n          # G (SYRK, lower: M²N) + Y = 2c·P·Kmn (2M²N)
    small = 14.0 * Mp ** 3           # the O(M³) GEMMs + Cholesky-and-inverse
    xs = np.linspace(0, 360, 4096)[:, None]
    eng.predict(theta, Z, q, R, xs, False)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(a.reps):
        eng.predict(theta, Z, q, R, xs, False)
    torch.cuda.synchronize()
    dp = (time.perf_counter() - t1) / a.reps
    out = {"N": n, "M": M, "eval_ms": dt * 1e3, "alg_tflops": (big + small) / dt / 1e12,
           "big_gemm_flops": big, "predict_ms_4096": dp * 1e3}
    if a.cpu:  # CPU baseline: the oracle (test infrastructure) on the same inputs, one evaluation
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from oracle import gp_oracle as O
        from oracle import svgp_oracle as S
        osv = S.OSVGP(O.OSquaredExponential(lengthscales=2.0, variance=1.0), Z, num_data=n,
                      noise_variance=1e-4, q_mu=q, q_sqrt=R)
        t2 = time.perf_counter()
        elbo_cpu = osv.elbo_and_grads(X, Y)[0]
        out["cpu_eval_ms"] = (time.perf_counter() - t2) * 1e3
        out["cpu_threads"] = int(os.environ.get("OPENBLAS_NUM_THREADS") or os.cpu_count())
        out["elbo_rel_diff"] = abs(eng.elbo_grad(theta, Z, q, R)[0] - elbo_cpu) / abs(elbo_cpu)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
