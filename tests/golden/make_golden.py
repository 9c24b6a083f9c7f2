"""Generate the committed golden fixtures under tests/golden/ (run in the build container only:
it reads the reference's CSV data under /root/reference, which does not exist on the GPU box).

Fixtures are DATA: inputs derived from the reference's own market CSVs (through the restated
GPR/data_handler.py:26-65 transform) or seeded synthetic series, and the oracle's outputs on
them. GPflow itself is not installable here, so the expected values come from
oracle/gp_oracle.py, which tests/test_oracle.py cross-checks against an independent torch-fp64
autograd restatement, finite differences and closed forms.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import scipy

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle import gp_oracle as O  # noqa: E402

REF = "/root/reference"

# kernel families: name -> factory of the oracle kernel (fresh GPflow defaults)
FAMILIES = {
    "se": lambda: O.OSquaredExponential(),
    "m12": lambda: O.OMatern12(),
    "m32": lambda: O.OMatern32(),
    "m52": lambda: O.OMatern52(),
    "exp": lambda: O.OExponential(),
    "rq": lambda: O.ORationalQuadratic(),
    "per": lambda: O.OPeriodic(O.OSquaredExponential()),
    "lin": lambda: O.OLinear(),
    "se+m12": lambda: O.OSum([O.OSquaredExponential(), O.OMatern12()]),
    "exp+per+lin": lambda: O.OSum([O.OExponential(), O.OPeriodic(O.OSquaredExponential()), O.OLinear()]),
    "exp+per": lambda: O.OSum([O.OExponential(), O.OPeriodic(O.OSquaredExponential())]),
    "se*m12": lambda: O.OProduct([O.OSquaredExponential(), O.OMatern12()]),
}


def datasets():
    out = {}
    x, y, mean, std = O.prepare_series(f"{REF}/Stocks/AAPL_EOD/AAPL_us_d.csv")
    out["aapl_d"] = (x, y, dict(mean=mean, std=std, source="Stocks/AAPL_EOD/AAPL_us_d.csv"))
    for tf in ("w", "m"):
        x, y, mean, std = O.prepare_series(f"{REF}/Stocks/AAPL/AAPL_us_{tf}.csv")
        out[f"aapl_{tf}"] = (x, y, dict(mean=mean, std=std, source=f"Stocks/AAPL/AAPL_us_{tf}.csv"))
    rng = np.random.default_rng(1234)
    for n in (1, 2, 16):
        xs = np.sort(rng.uniform(0.0, 20.0, n))[:, None]
        ys = rng.standard_normal((n, 1))
        out[f"synth{n}"] = (xs, ys, dict(source=f"uniform/normal rng(1234) N={n}"))
    x, y = O.synthetic_series(256, seed=11)
    out["synth256"] = (x, y, dict(source="oracle.synthetic_series(256, seed=11)"))
    return out


def set_theta(kernel, values):
    for p, v in zip(kernel.params(), values):
        p.value = float(v)


def kernel_cases():
    """logML / grad / predictions per (family, dataset, theta choice)."""
    rng = np.random.default_rng(99)
    arrays, index = {}, []
    for dname, (x, y, meta) in datasets().items():
        xf = np.concatenate([x, x[-1:] + np.arange(1, 31, dtype=np.float64)[:, None]], axis=0)
        for fname, fac in FAMILIES.items():
            for tchoice in ("default", "random"):
                k = fac()
                if tchoice == "random":
                    vals = np.exp(rng.uniform(np.log(0.5), np.log(4.0), len(k.params())))
                    # keep the periodic kernel away from the integer-lattice degeneracy
                    set_theta(k, vals)
                noise = 1e-5 if dname.startswith("aapl") else 1e-3
                if fname in ("lin", "exp+per+lin") and dname.startswith("aapl"):
                    noise = 1e-3
                m = O.OGPR(x, y, k, noise_variance=noise)
                try:
                    loss, g = m.loss_and_grad_u()
                    _, g_hp = m.loss_and_grad_u_extended()
                    m.noise.trainable = False
                    loss_nt, g_nt = m.loss_and_grad_u()
                    _, g_nt_hp = m.loss_and_grad_u_extended()
                    cond = float(np.linalg.cond(m._Ky()))
                    m.noise.trainable = True
                    mu, var = m.predict_f(xf)
                    _, vary = m.predict_y(xf)
                except np.linalg.LinAlgError:
                    continue
                key = f"{dname}|{fname}|{tchoice}"
                arrays[key + "|theta"] = np.array([p.value for p in k.params()])
                arrays[key + "|noise"] = np.array([noise])
                arrays[key + "|loss"] = np.array([loss])
                arrays[key + "|grad_u"] = g              # noise trainable (last entry = noise)
                arrays[key + "|grad_u_fixed_noise"] = g_nt
                # the same gradients with extended-precision linear algebra on the same fp64
                # K and ∂K (oracle loss_and_grad_u_extended): where the fp64 oracle is off
                arrays[key + "|grad_u_hp"] = g_hp
                arrays[key + "|grad_u_fixed_noise_hp"] = g_nt_hp
                arrays[key + "|cond"] = np.array([cond])
                arrays[key + "|xnew"] = xf
                arrays[key + "|fmean"] = mu[:, 0]
                arrays[key + "|fvar"] = var[:, 0]
                arrays[key + "|yvar"] = vary[:, 0]
                index.append(key)
    for dname, (x, y, meta) in datasets().items():
        arrays[f"data|{dname}|x"] = x
        arrays[f"data|{dname}|y"] = y
    return arrays, index


def reference_sweep():
    """GPR/main.py:23-37 for AAPL with the 8 kernels of GPR/main.py:105-114 shared across the
    d -> w -> m calls (the aliasing of SURVEY D6), each fit as GPR/model_trainer.py:14-25."""
    ds = datasets()
    kernels = O.reference_kernel_list()
    out = {"scipy": scipy.__version__, "timeframes": {}}
    for tf in ("d", "w", "m"):
        x, y, meta = ds[f"aapl_{tf}"]
        rows = []
        best = (np.inf, -1)
        for i, k in enumerate(kernels):
            m = O.OGPR(x, y, k, noise_variance=1.0)
            m.noise.value = 1e-5
            m.noise.trainable = False
            r = O.scipy_minimize(m, 100)
            mu, _ = m.predict_f(x)
            mse = float(np.mean((y - mu) ** 2))
            rows.append(dict(theta=[p.value for p in k.params()], loss=r.fun, nfev=r.nfev, nit=r.nit,
                             mse=mse))
            if mse < best[0]:
                best = (mse, i)
        out["timeframes"][tf] = dict(fits=rows, best_index=best[1], best_mse=best[0])
    # fresh-default fits per kernel on the daily series (no aliasing)
    x, y, _ = ds["aapl_d"]
    fresh = []
    for k in O.reference_kernel_list():
        m = O.OGPR(x, y, k, noise_variance=1.0)
        m.noise.value = 1e-5
        m.noise.trainable = False
        r = O.scipy_minimize(m, 100)
        fresh.append(dict(theta=[p.value for p in k.params()], loss=r.fun, nfev=r.nfev, nit=r.nit))
    out["fresh_daily"] = fresh
    return out


def multi_input_case():
    """C4 shape: D=5 (4 z-scored features + z-scored time), Exponential(dims 0..3) *
    Exponential(dim 4) as Multi-Input_GPR/main.py:118-135, and Matern52 over all dims, N=67,
    noise 1e-3 fixed (main.py:422), plus the train_likelihood variant with trainable noise
    (keys tl|*)."""
    rng = np.random.default_rng(100)
    n = 67
    feats = np.cumsum(rng.standard_normal((n, 4)) * 0.01, axis=0)
    t = np.linspace(0.0, 1.0, n)
    X = np.column_stack([feats, t])
    X = (X - X.mean(0)) / X.std(0, ddof=1)
    f = np.sin(3 * X[:, 4]) + 0.5 * X[:, 0] - 0.3 * X[:, 2]
    Y = f + 0.1 * rng.standard_normal(n)
    Y = ((Y - Y.mean()) / Y.std(ddof=1))[:, None]
    arrays = {"X": X, "Y": Y}
    k1 = O.OProduct([O.OExponential(), O.OExponential()])
    k1.kernels[0].active_dims = slice(0, 4)
    k1.kernels[1].active_dims = slice(4, 5)
    k2 = O.OMatern52()
    for name, k in (("expexp", k1), ("m52", k2)):
        m = O.OGPR(X, Y, k, noise_variance=1e-3)
        m.noise.trainable = False
        loss, g = m.loss_and_grad_u()
        arrays[f"{name}|loss0"] = np.array([loss])
        arrays[f"{name}|grad0"] = g
        r = O.scipy_minimize(m, None)
        arrays[f"{name}|loss_fit"] = np.array([r.fun])
        arrays[f"{name}|theta_fit"] = np.array([p.value for p in k.params()])
        arrays[f"{name}|nfev"] = np.array([r.nfev])
        mu, var = m.predict_f(X)
        arrays[f"{name}|fmean"] = mu[:, 0]
        arrays[f"{name}|fvar"] = var[:, 0]
    # Multi-Input_GPR/models/model_trainer.py:26-54 train_likelihood on the reference's composite
    # kernel: for each starting noise variance a fresh GPR((X, Y), deepcopy(kernel),
    # noise_variance=v) with the likelihood trainable, Scipy().minimize at scipy's default
    # maxiter; the lowest opt_logs.fun wins (strict <, first wins)
    starts = [1e-5, 1e-3, 1e-1, 1.0]
    arrays["tl|starts"] = np.array(starts)
    best, best_loss = -1, np.inf
    for r_i, v in enumerate(starts):
        k = O.OProduct([O.OExponential(), O.OExponential()])
        k.kernels[0].active_dims = slice(0, 4)
        k.kernels[1].active_dims = slice(4, 5)
        m = O.OGPR(X, Y, k, noise_variance=v)
        m.noise.trainable = True
        r = O.scipy_minimize(m, None)
        arrays[f"tl|{r_i}|loss_fit"] = np.array([r.fun])
        arrays[f"tl|{r_i}|theta_fit"] = np.array([p.value for p in k.params()])
        arrays[f"tl|{r_i}|noise_fit"] = np.array([m.noise.value])
        arrays[f"tl|{r_i}|nfev"] = np.array([r.nfev])
        if r.fun < best_loss:
            best, best_loss = r_i, r.fun
    arrays["tl|best"] = np.array([best])
    arrays["tl|best_loss"] = np.array([best_loss])
    return arrays


def meta_sweep():
    """C1 real-data N≈252 variant: test_data/Stocks/META_EOD/meta_us_eod.csv (251
    rows, 2023-05-30..2024-05-28) through the restated GPR/data_handler.py:26-65 with
    train_start = the first date, and the 8-kernel sweep of GPR/model_trainer.py:14-25 with
    fresh GPflow defaults per kernel (noise 1e-5 fixed, maxiter 100, predict_f at X, MSE)."""
    x, y, mean, std = O.prepare_series(f"{REF}/test_data/Stocks/META_EOD/meta_us_eod.csv",
                                       train_start_date="2023-05-30")
    arrays = {"x": x, "y": y, "mean": np.array([mean]), "std": np.array([std])}
    best = (np.inf, -1)
    for i, k in enumerate(O.reference_kernel_list()):
        m = O.OGPR(x, y, k, noise_variance=1.0)
        m.noise.value = 1e-5
        m.noise.trainable = False
        loss0, g0 = m.loss_and_grad_u()
        arrays[f"{i}|loss0"] = np.array([loss0])
        arrays[f"{i}|grad0"] = g0
        r = O.scipy_minimize(m, 100)
        mu, var = m.predict_f(x)
        mse = float(np.mean((y - mu) ** 2))
        arrays[f"{i}|theta_fit"] = np.array([p.value for p in k.params()])
        arrays[f"{i}|loss_fit"] = np.array([r.fun])
        arrays[f"{i}|nfev"] = np.array([r.nfev])
        arrays[f"{i}|mse"] = np.array([mse])
        arrays[f"{i}|fmean"] = mu[:, 0]
        arrays[f"{i}|fvar"] = var[:, 0]
        if mse < best[0]:
            best = (mse, i)
    arrays["best_index"] = np.array([best[1]])
    return arrays


def tickers():
    """C3 real-data variant: the daily series of every ticker under Stocks/<T>/ at native N."""
    arrays = {}
    root = f"{REF}/Stocks"
    for t in sorted(os.listdir(root)):
        p = f"{root}/{t}/{t}_us_d.csv"
        if os.path.exists(p) and not t.endswith("_EOD"):
            x, y, mean, std = O.prepare_series(p, train_start_date="2024-02-01")
            arrays[f"{t}|x"] = x
            arrays[f"{t}|y"] = y
    return arrays


def main():
    arrays, index = kernel_cases()
    np.savez_compressed(os.path.join(HERE, "kernel_cases.npz"), **arrays)
    with open(os.path.join(HERE, "kernel_cases_index.json"), "w") as f:
        json.dump(index, f, indent=0)
    with open(os.path.join(HERE, "reference_sweep.json"), "w") as f:
        json.dump(reference_sweep(), f, indent=1)
    np.savez_compressed(os.path.join(HERE, "multi_input.npz"), **multi_input_case())
    np.savez_compressed(os.path.join(HERE, "tickers.npz"), **tickers())
    np.savez_compressed(os.path.join(HERE, "meta_sweep.npz"), **meta_sweep())
    ds = datasets()
    x, y, meta = ds["aapl_d"]
    pin = O.OGPR(x, y, O.OSquaredExponential(), noise_variance=1e-5)
    pin.noise.trainable = False
    loss, g = pin.loss_and_grad_u()
    with open(os.path.join(HERE, "aapl_pin.json"), "w") as f:
        json.dump(dict(n=len(x), mean=meta["mean"], std=meta["std"], y0=float(y[0, 0]), y1=float(y[1, 0]),
                       lml=-loss, grad_u=list(map(float, g)),
                       survey_lml=-180.01628691394865,
                       survey_grad_u=[230.60287644662168, -47.072957583506444]), f, indent=1)
    print("wrote", len(index), "kernel cases")


if __name__ == "__main__":
    main()
