"""Golden vectors for the rows either side of the hot path, computed by the
REFERENCE'S OWN importable host modules. Run in the build container only (it imports from
/root/reference, which does not exist on the GPU box):

    python tests/golden/make_ref_golden.py

* f1 — ``GPR/optimizer.py`` (``Optimizer.optimize_weights``, the α/β SLSQP of the timeframe
  blend; TF-free, importable here: SURVEY.md §8c) on fixed daily / weekly / monthly
  predictions:
    - "aapl": the GPR/main.py:47-56 flow on the reference's AAPL d/w/m series — the best model
      of each timeframe from the oracle's 8-kernel sweep with shared kernels
      (reference_sweep.json), ``predict_single`` at the training inputs, the weekly and monthly
      means upsampled to the daily grid (GPR/predictor.py:35-51, pandas reindex + linear
      interpolate), then ``Optimizer(lambda_=0.1)`` (GPR/main.py:116); and the
      ``predict_combined`` outputs (GPR/predictor.py:10-33) at the daily/weekly/monthly inputs
      extended by GPR/data_handler.py:67-90's future dates (30 days / 4 weeks / 1 month), from
      the oracle's predictions at the best models' θ;
    - "synth<k>": seeded random predictions (interior and constrained optima), λ = 0.01 / 0.1.
  -> tests/golden/blend.npz
* f3 — ``Multi-Input_GPR/optimization/optimizer.py`` (``set_predictions``, ``set_cml_log_return``,
  ``set_predictions_cml``) fed per day exactly as ``Portfolio.evaluate_portfolio`` indexes the
  gathered per-asset lists (Multi-Input_GPR/Portfolio/portfolio.py:111-124): returns[i][0][0],
  returns[i][:(day+1)], variances[i][day][0], on 5 assets × 5 days of seeded means/variances in
  the run_step_4 output format (lists of [1]-arrays, Multi-Input_GPR/main.py:453-456).
  -> tests/golden/portfolio.npz

The importer loads each reference file by path (importlib), never the reference's packages, and
nothing of the reference is copied: only inputs and outputs are stored.
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle import gp_oracle as O  # noqa: E402

REF = "/root/reference"


def load_ref(relpath, name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, relpath))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def upsample(x_daily, x_tf, pred):
    """GPR/predictor.py:35-51 for period 'w' / 'm' (restated: the reference module imports TF)."""
    s = pd.Series(np.asarray(pred).reshape(-1), index=np.asarray(x_tf).reshape(-1))
    return s.reindex(np.asarray(x_daily).reshape(-1)).interpolate(method="linear").values.reshape(-1, 1)


def future_x(csv, period, total_days=30, train_start="2024-02-01"):
    """GPR/data_handler.py:67-90 generate_future_dates (restated)."""
    df = pd.read_csv(csv)
    last = pd.to_datetime(df["date"]).max()
    if period == "d":
        dates = pd.date_range(start=last + pd.Timedelta(days=1), periods=total_days, freq="D")
    elif period == "w":
        dates = pd.date_range(start=last + pd.DateOffset(weeks=1), periods=total_days // 7, freq="W")
    else:
        dates = pd.date_range(start=last + pd.DateOffset(months=1), periods=total_days // 30, freq="ME")
    return np.asarray((dates - pd.Timestamp(train_start)).days, dtype=np.float64).reshape(-1, 1)


def blend_cases(ref_opt):
    out = {}
    # --- aapl: the GPR/main.py flow on the oracle's shared-kernel sweep
    csv = {"d": f"{REF}/Stocks/AAPL_EOD/AAPL_us_d.csv", "w": f"{REF}/Stocks/AAPL/AAPL_us_w.csv",
           "m": f"{REF}/Stocks/AAPL/AAPL_us_m.csv"}
    kernels = O.reference_kernel_list()
    best = {}
    data = {}
    for tf in ("d", "w", "m"):
        x, y, _, _ = O.prepare_series(csv[tf])
        data[tf] = (x, y)
        bmse, bi = np.inf, -1
        for i, k in enumerate(kernels):
            m = O.OGPR(x, y, k, noise_variance=1.0)
            m.noise.value = 1e-5
            m.noise.trainable = False
            O.scipy_minimize(m, 100)
            mu, _ = m.predict_f(x)
            mse = float(np.mean((y - mu) ** 2))
            if mse < bmse:
                bmse, bi = mse, i
        best[tf] = bi
    preds = {}
    for tf in ("d", "w", "m"):
        # main.py predicts after all three sweeps: each best model's kernel object is shared, so
        # its θ is whatever the later timeframes' fits left in it
        i = best[tf]
        th = [p.value for p in kernels[i].params()]
        k = O.reference_kernel_list()[i]
        for p, v in zip(k.params(), th):
            p.value = v
        x, y = data[tf]
        m = O.OGPR(x, y, k, noise_variance=1e-5)
        xc = np.vstack([x, future_x(csv[tf], tf)])
        fm, fv = m.predict_f(x)
        ym, yv = m.predict_y(x)
        cm, cv = m.predict_f(xc)
        cym, cyv = m.predict_y(xc)
        preds[tf] = dict(fm=fm, fv=fv, ym=ym, yv=yv, cm=cm, cv=cv, cym=cym, cyv=cyv, xc=xc)
        p = f"aapl|{tf}|"
        out[p + "x"], out[p + "y"], out[p + "xc"] = x, y, xc
        out[p + "kernel_index"] = np.array([i])
        out[p + "theta"] = np.array(th)
        for key in ("fm", "fv", "ym", "yv", "cm", "cv", "cym", "cyv"):
            out[p + key] = preds[tf][key]
    xd = data["d"][0]
    fw_up = upsample(xd, data["w"][0], preds["w"]["fm"])
    fm_up = upsample(xd, data["m"][0], preds["m"]["fm"])
    out["aapl|fw_up"], out["aapl|fm_up"] = fw_up, fm_up
    lam = 0.1                                   # GPR/main.py:116
    try:
        ab = ref_opt.Optimizer(lam).optimize_weights(data["d"][1], preds["d"]["fm"], fw_up, fm_up)
        out["aapl|alpha_beta"] = np.asarray(ab, dtype=np.float64)
        out["aapl|raises"] = np.array([0])
    except ValueError:                          # sklearn refuses NaN (leading rows before the first w/m point)
        out["aapl|alpha_beta"] = np.array([np.nan, np.nan])
        out["aapl|raises"] = np.array([1])
    out["aapl|lambda"] = np.array([lam])
    # predict_combined at the extended inputs with the golden α/β (positional upsampling of
    # all four outputs, GPR/predictor.py:10-33)
    a, b = (out["aapl|alpha_beta"] if not out["aapl|raises"][0] else np.array([0.33, 0.33]))
    xcd = preds["d"]["xc"]
    comb = {}
    for key in ("cm", "cv", "cym", "cyv"):
        w_up = upsample(xcd, preds["w"]["xc"], preds["w"][key])
        m_up = upsample(xcd, preds["m"]["xc"], preds["m"][key])
        comb[key] = a * preds["d"][key] + b * w_up + (1 - a - b) * m_up
        out["aapl|combined|" + key] = comb[key]
    out["aapl|combined|alpha_beta"] = np.array([a, b])
    # --- synthetic blends (no NaN), interior and constrained solutions
    rng = np.random.default_rng(2024)
    for c, lam in enumerate((0.01, 0.1, 0.01, 0.0)):
        n = 89
        fd, fw, fmn = (rng.standard_normal((n, 1)) for _ in range(3))
        w = [(0.5, 0.3), (0.2, 0.1), (0.9, 0.6), (0.0, 0.0)][c]
        Y = w[0] * fd + w[1] * fw + (1 - w[0] - w[1]) * fmn + 0.05 * rng.standard_normal((n, 1))
        ab = ref_opt.Optimizer(lam).optimize_weights(Y, fd, fw, fmn)
        p = f"synth{c}|"
        out[p + "Y"], out[p + "fd"], out[p + "fw"], out[p + "fm"] = Y, fd, fw, fmn
        out[p + "lambda"] = np.array([lam])
        out[p + "alpha_beta"] = np.asarray(ab, dtype=np.float64)
    return out


def portfolio_case(ref_port_opt):
    """5 assets x 5 days in run_step_4's output format, fed to the reference Optimizer day by day
    as Portfolio.evaluate_portfolio (portfolio.py:111-124) indexes the lists."""
    rng = np.random.default_rng(77)
    A, H = 5, 5
    means = rng.normal(0.0, 0.01, (A, H))
    varis = rng.uniform(1e-5, 4e-4, (A, H))
    ret = [[np.array([means[i, d]]) for d in range(H)] for i in range(A)]
    var = [[np.array([varis[i, d]]) for d in range(H)] for i in range(A)]
    out = {"means": means, "vars": varis}
    rf = 0.01 / 252
    for log_ret in (True, False):
        mus, sig, sd = [], [], []
        for day in range(H):
            opt = ref_port_opt.Optimizer()
            std_devs = []
            if day == 0:
                returns = [ret[i][0][0] for i in range(A)]
                vols = [var[i][0][0] for i in range(A)]
                std_devs = [np.sqrt(var[i][0][0]) for i in range(A)]
                opt.set_predictions(returns, vols, rf)
            else:
                returns = [ret[i][:(day + 1)] for i in range(A)]
                vols = [var[i][:(day + 1)] for i in range(A)]
                std_devs = [np.sqrt(var[i][day][0]) for i in range(A)]
                if log_ret:
                    opt.set_cml_log_return(returns, vols, rf)
                else:
                    opt.set_predictions_cml(returns, vols, rf)
            mus.append(np.asarray(opt.mu, dtype=np.float64).reshape(-1))
            sig.append(np.asarray(opt.Sigma, dtype=np.float64))
            sd.append(np.asarray(std_devs, dtype=np.float64))
        tag = "log" if log_ret else "cml"
        out[f"{tag}|mu"] = np.stack(mus)
        out[f"{tag}|Sigma"] = np.stack(sig)
        out[f"{tag}|std"] = np.stack(sd)
    return out


def main():
    ref_opt = load_ref("GPR/optimizer.py", "ref_gpr_optimizer")
    ref_port_opt = load_ref("Multi-Input_GPR/optimization/optimizer.py", "ref_portfolio_optimizer")
    b = blend_cases(ref_opt)
    np.savez_compressed(os.path.join(HERE, "blend.npz"), **b)
    p = portfolio_case(ref_port_opt)
    np.savez_compressed(os.path.join(HERE, "portfolio.npz"), **p)
    print(json.dumps({"aapl_alpha_beta": b["aapl|alpha_beta"].tolist(), "aapl_raises": int(b["aapl|raises"][0]),
                      "kernels": [int(b[f"aapl|{t}|kernel_index"][0]) for t in "dwm"],
                      "synth": [b[f"synth{c}|alpha_beta"].tolist() for c in range(4)]}))


if __name__ == "__main__":
    main()
