"""C2 fit parity in distribution: many seeds of the headline
configuration fitted through the bench's own path against the oracle's whole fits
(tests/golden/c2_dist_n4096.npz, tests/golden/make_c2_dist_golden.py).

Protocol: GPR/model_trainer.py:15-20 — GPflow defaults (σ² = ℓ = 1), σn² = 1e-5 fixed,
Scipy().minimize(maxiter=100), predict_f at the training inputs; inputs the C2 generator
(X = day offsets 0..4095). The path under test is bench.py's: band-storage slots, the band16
sweeps or block cyclic reduction (both routes, the `route` fixture), Scipy.minimize_stream over a
ModelStream in two device groups.

Asserted per seed: loss* within 1e-5 relative of the oracle's fit (SURVEY §8c's bar), θ* within
1e-4, and the GPU's loss and gradient at its own θ* equal to the CPU restatement's there (loss
1e-8 — DESIGN §5's κ-scaled logML bar (1e-9 + 1e-14·κ) at C2's κ ≈ 1e6; observed up to 3e-9 —,
gradient 1e-6·max(1, |g|); the CPU side is oracle/band_oracle.py, the band algorithm on
numpy/LAPACK, itself checked against the dense oracle in tests/test_band_oracle.py — the dense
oracle takes seconds per evaluation at N = 4096). Over the population: the mean number of
evaluations per fit (fits/s ∝ 1/nfev, so a device that stopped early would inflate the headline).

Individual fits' nfev differ between ANY two correct implementations: near this flat optimum
L-BFGS-B's stop test reacts to 1e-9-level differences of summation order, and which seeds take
40+ evaluations instead of ~15 moves between the dense oracle, the band oracle and the device
(all three on c2_dist_n4096.npz's seeds). So the mean is compared (a) on the dense oracle's 32
seeds within three standard errors of the difference, and (b) on a 512-seed population fitted
by the band oracle (c2_dist_band_n4096.npz, standard error 0.36 evaluations) within ±10 %.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import portfoliooptgp_amd as gpx  # noqa: E402
from portfoliooptgp_amd.engine import Engine  # noqa: E402
from portfoliooptgp_amd.kernels import compile_spec  # noqa: E402

K = gpx.kernels
NOISE = 1e-5


@pytest.fixture(params=["bcr", "sweeps"], autouse=True)
def route(request, monkeypatch):
    """Both banded routes of a call: block cyclic reduction for every call
    (GPX_BCR_MAX far above the problems per call) and the band16 sweeps (GPX_BCR_MAX=0). By default
    the library sends a call to BCR when it holds at most 32 band16 problems."""
    monkeypatch.setenv("GPX_BCR_MAX", "1000000" if request.param == "bcr" else "0")
    return request.param


def _check_route(engines, route):
    bcr = sum(e.last_timing().bcr_evals for e in engines)
    assert (bcr > 0) == (route == "bcr"), (route, bcr)


def test_c2_fits_in_distribution(golden_dir, route):
    from oracle import band_oracle as BO
    from oracle import gp_oracle as O
    fx = np.load(os.path.join(golden_dir, "c2_dist_n4096.npz"))
    n = int(fx["n"][0])
    seeds = [int(s) for s in fx["seeds"]]
    assert len(seeds) >= 16
    data = [O.synthetic_series(n, s) for s in seeds]

    def model(i):
        m = gpx.models.GPR(data=data[i], kernel=K.SquaredExponential())
        m.likelihood.variance.assign(NOISE)
        gpx.set_trainable(m.likelihood.variance, False)
        return m

    models = gpx.optimizers.ModelStream(len(seeds), model, input_dim=1, max_points=n)
    spec = compile_spec(K.SquaredExponential(), 1)
    engines = [Engine([data[g][0]], [data[g][1]], [spec], band_storage=True) for g in range(2)]
    for e in engines:
        e.ctx.set_profiling(True)
        e.reset_timing()
    res, _ = gpx.optimizers.Scipy().minimize_stream(models, width=len(seeds), engine=engines, groups=2,
                                                    predict_train=True, options=dict(maxiter=100))
    evals = sum(e.last_timing().evals for e in engines)
    assert sum(e.last_timing().band_evals for e in engines) == evals > 0
    _check_route(engines, route)
    nf_gpu, nf_ora = [], []
    worst = dict(loss=0.0, theta=0.0, at_loss=0.0, at_grad=0.0)
    for i, (s, r) in enumerate(zip(seeds, res)):
        m = models[i]
        theta = np.array([m.kernel.lengthscales.value, m.kernel.variance.value])
        lo, tho = float(fx["loss"][i]), fx["theta"][i]
        el = abs(r.fun - lo) / abs(lo)
        et = float(np.max(np.abs(theta - tho) / np.abs(tho)))
        assert el <= 1e-5, (s, r.fun, lo)
        assert et <= 1e-4, (s, theta, tho)
        # the restatement at the GPU's θ*
        bm = BO.OBandGPR(*data[i], NOISE)
        bm.ell, bm.var = float(theta[0]), float(theta[1])
        lb, gb = bm.loss_and_grad_u()
        ea = abs(r.fun - lb) / abs(lb)
        eg = float(np.abs(np.asarray(r.jac) - gb).max() / max(1.0, np.abs(gb).max()))
        assert ea <= 1e-8, (s, r.fun, lb)
        assert eg <= 1e-6, (s, r.jac, gb)
        for k, v in (("loss", el), ("theta", et), ("at_loss", ea), ("at_grad", eg)):
            worst[k] = max(worst[k], v)
        nf_gpu.append(int(r.nfev))
        nf_ora.append(int(fx["nfev"][i]))
    mg, mo = float(np.mean(nf_gpu)), float(np.mean(nf_ora))
    se = float(np.sqrt(np.var(nf_gpu, ddof=1) / len(nf_gpu) + np.var(nf_ora, ddof=1) / len(nf_ora)))
    print(f"C2 in distribution ({len(seeds)} seeds, N={n}): nfev mean GPU {mg:.2f} oracle {mo:.2f} "
          f"(standard error of the difference {se:.2f}; GPU {nf_gpu}, oracle {nf_ora}); worst rel: {worst}")
    assert abs(mg - mo) <= 3.0 * se, (mg, mo, se)


def _fit_on_device(data, n):
    def model(i):
        m = gpx.models.GPR(data=data[i], kernel=K.SquaredExponential())
        m.likelihood.variance.assign(NOISE)
        gpx.set_trainable(m.likelihood.variance, False)
        return m

    models = gpx.optimizers.ModelStream(len(data), model, input_dim=1, max_points=n)
    spec = compile_spec(K.SquaredExponential(), 1)
    engines = [Engine([data[g][0]], [data[g][1]], [spec], band_storage=True) for g in range(2)]
    for e in engines:
        e.ctx.set_profiling(True)
        e.reset_timing()
    res, _ = gpx.optimizers.Scipy().minimize_stream(models, width=len(data), engine=engines, groups=2,
                                                    predict_train=True, options=dict(maxiter=100))
    return models, res, engines


def test_c2_nfev_population_vs_band_oracle(golden_dir, route):
    """512 C2 seeds through the bench's path against the band oracle's fits of the same seeds:
    every fitted loss within 1e-5 and θ* within 1e-4, and the mean evaluations per fit within
    ±10 % (VERDICT r03 item 5's bar; the population's standard error is ~0.4 evaluations, ~2 %)."""
    from oracle import gp_oracle as O
    fx = np.load(os.path.join(golden_dir, "c2_dist_band_n4096.npz"))
    n = int(fx["n"][0])
    seeds = [int(s) for s in fx["seeds"]]
    data = [O.synthetic_series(n, s) for s in seeds]
    models, res, engines = _fit_on_device(data, n)
    _check_route(engines, route)
    nf = np.array([r.nfev for r in res], dtype=np.float64)
    worst_l = worst_t = 0.0
    for i, (s, r) in enumerate(zip(seeds, res)):
        theta = np.array([models[i].kernel.lengthscales.value, models[i].kernel.variance.value])
        el = abs(r.fun - float(fx["loss"][i])) / abs(float(fx["loss"][i]))
        et = float(np.max(np.abs(theta - fx["theta"][i]) / np.abs(fx["theta"][i])))
        worst_l, worst_t = max(worst_l, el), max(worst_t, et)
        assert el <= 1e-5, (s, r.fun, float(fx["loss"][i]))
        assert et <= 1e-4, (s, theta, fx["theta"][i])
    mg, mo = float(nf.mean()), float(fx["nfev"].mean())
    print(f"C2 population ({len(seeds)} seeds): nfev mean GPU {mg:.3f} band oracle {mo:.3f} "
          f"(GPU > 30: {int((nf > 30).sum())}, oracle > 30: {int((fx['nfev'] > 30).sum())}); "
          f"worst loss rel {worst_l:.2e}, theta rel {worst_t:.2e}")
    assert abs(mg - mo) <= 0.10 * mo, (mg, mo)
