"""Few-problem latency of the exact-GPR fit (the reference's own call pattern): one C2 fit at
N = 4096 from GPflow's defaults, as GPR/model_trainer.py:15-20 calls it (models.GPR +
Scipy().minimize(maxiter=100) + predict_f at the training inputs), and the C3 batch (20 series x
N = 2048 streamed through one band-storage engine, as bench.py secondary_c3). Prints JSON lines.

usage: python tools/latency.py [--solo-reps 5] [--c3-reps 3] [--evals 50]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402  (the C2 generator, shared with the bench)
import portfoliooptgp_amd as gpx  # noqa: E402


def solo(n, seed, reps, evals):
    x, y = bench.synthetic_series(n, seed)

    def model():
        m = gpx.models.GPR(data=(x, y), kernel=gpx.kernels.SquaredExponential())
        m.likelihood.variance.assign(1e-5)
        gpx.set_trainable(m.likelihood.variance, False)
        return m

    m = model()
    m.loss_and_grad_unconstrained()  # warm-up (engine creation, first gather)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(evals):
        m.loss_and_grad_unconstrained()
    ev = (time.perf_counter() - t0) / evals
    walls, nfev, fun = [], None, None
    for _ in range(reps + 1):
        m2 = model()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = gpx.optimizers.Scipy().minimize(m2.training_loss, m2.trainable_variables, options=dict(maxiter=100))
        mean, var = m2.predict_f(x)
        torch.cuda.synchronize()
        walls.append(time.perf_counter() - t0)
        nfev, fun = int(r.nfev), float(r.fun)
    walls = sorted(walls[1:])
    return {"case": "solo", "N": n, "seed": seed, "eval_ms": ev * 1e3, "fit_ms_median": 1e3 * walls[len(walls) // 2],
            "fit_ms_all": [round(1e3 * w, 3) for w in walls], "nfev": nfev, "loss": fun}


def c3(reps, groups=1):
    from portfoliooptgp_amd.engine import Engine
    from portfoliooptgp_amd.kernels import compile_spec
    out = {"case": "c3"}
    for k in (20, 3, 1):
        t = []
        for _ in range(reps + 1):
            import bench as B
            dev = "cuda:0"
            data = [B.synthetic_series(2048, s) for s in range(k)]
            data = [(torch.as_tensor(a, device=dev), torch.as_tensor(b, device=dev)) for a, b in data]
            spec = compile_spec(gpx.kernels.SquaredExponential(), 1)
            G = max(1, min(groups, k))
            eng = [Engine([d[0] for d in data[g::G]], [d[1] for d in data[g::G]], [spec] * len(data[g::G]), device=0,
                          band_storage=True) for g in range(G)]
            ms = []
            for i in range(k):
                m = gpx.models.GPR(data=data[i], kernel=gpx.kernels.SquaredExponential(), device=0)
                m.likelihood.variance.assign(1e-5)
                gpx.set_trainable(m.likelihood.variance, False)
                ms.append(m)
            torch.cuda.synchronize()
            os.environ["GPX_DRIVER_STATS"] = "1"
            opt = gpx.optimizers.Scipy()
            t0 = time.perf_counter()
            opt.minimize_stream(ms, width=k, engine=eng if G > 1 else eng[0], groups=G, predict_train=True,
                                options=dict(maxiter=100))
            torch.cuda.synchronize()
            t.append(time.perf_counter() - t0)
            os.environ.pop("GPX_DRIVER_STATS", None)
            st = dict(opt.last_stats or {})
        t = sorted(t[1:])
        out[f"wall_ms_{k}"] = 1e3 * t[len(t) // 2]
        if k == 20 and st.get("rounds"):  # the host loop's phases per round (the last run)
            out["per_round_ms_20"] = {kk: round(1e3 * v / st["rounds"], 4) for kk, v in st.items()
                                      if isinstance(v, float)}
            out["rounds_20"] = st["rounds"]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--solo-reps", type=int, default=5)
    ap.add_argument("--c3-reps", type=int, default=3)
    ap.add_argument("--c3-groups", type=int, default=1, help="device batches the C3 fits are split over")
    ap.add_argument("--c3-only", action="store_true")
    ap.add_argument("--evals", type=int, default=50)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--chain-only", action="store_true", help="only the per-evaluation device chain lines")
    a = ap.parse_args()
    from portfoliooptgp_amd import _native as N
    for mode, cap in (() if a.chain_only else (("bcr", None), ("sweeps", "0"))):
        if cap is None:
            os.environ.pop("GPX_BCR_MAX", None)
        else:
            os.environ["GPX_BCR_MAX"] = cap
        for seed in (() if a.c3_only else (0, 1)):
            r = solo(a.n, seed, a.solo_reps, a.evals)
            r["mode"] = mode
            print(json.dumps(r), flush=True)
        r = c3(a.c3_reps, a.c3_groups)
        r["mode"] = mode
        r["groups"] = a.c3_groups
        print(json.dumps(r), flush=True)
    if a.c3_only:
        return
    # device time of one reduction chain (profiling on: HIP events around the chain)
    os.environ.pop("GPX_BCR_MAX", None)
    N.Context.get(0).set_profiling(True)
    for n in (2048, 4096):
        x, y = bench.synthetic_series(n, 0)
        m = gpx.models.GPR(data=(x, y), kernel=gpx.kernels.SquaredExponential())
        m.likelihood.variance.assign(1e-5)
        gpx.set_trainable(m.likelihood.variance, False)
        from portfoliooptgp_amd.engine import solo_engine
        eng = solo_engine(m)
        for ell in (1.0, 1.18, 1.6, 1.9):
            m.kernel.lengthscales.assign(ell)
            m.loss_and_grad_unconstrained()
            eng.reset_timing()
            t0 = time.perf_counter()
            for _ in range(20):
                m.loss_and_grad_unconstrained()
            wall = (time.perf_counter() - t0) / 20
            t = eng.last_timing()
            print(json.dumps({"case": "chain", "N": n, "ell": ell, "bcr_ms": t.bcr_ms_total / max(t.bcr_calls, 1),
                              "eval_total_ms": t.eval_ms_total / max(t.evals, 1), "wall_ms": 1e3 * wall,
                              "bcr_calls": t.bcr_calls}), flush=True)


if __name__ == "__main__":
    main()
