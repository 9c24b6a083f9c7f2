"""C2 fit parity in distribution: many seeds of the headline
configuration fitted through the bench's own path against the oracle's whole fits
(tests/golden/c2_dist_n4096.npz, tests/golden/make_c2_dist_golden.py).

Protocol: GPR/model_trainer.py:15-20 — GPflow defaults (σ² = ℓ = 1), σn² = 1e-5 fixed,
Scipy().minimize(maxiter=100), predict_f at the training inputs; inputs the C2 generator
(X = day offsets 0..4095). The path under test is bench.py's: band-storage slots, the band16
sweeps, Scipy.minimize_stream over a ModelStream in two device groups.

Asserted per seed: loss* within 1e-5 relative of the oracle's fit (SURVEY §8c's bar), θ* within
1e-4, and the GPU's loss and gradient at its own θ* equal to the CPU restatement's there (loss
1e-8 — DESIGN §5's κ-scaled logML bar (1e-9 + 1e-14·κ) at C2's κ ≈ 1e6; observed up to 3e-9 —,
gradient 1e-6·max(1, |g|); the CPU side is oracle/band_oracle.py, the band algorithm on
numpy/LAPACK, itself checked against the dense oracle in tests/test_band_oracle.py — the dense
oracle takes seconds per evaluation at N = 4096). Over the population: the mean number of
evaluations per fit within ±10 % of the oracle's (fits/s ∝ 1/nfev, so a device that stopped
early would inflate the headline; individual fits differ — near this flat optimum L-BFGS-B's
stop test sees 1e-9-level differences of summation order).
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


def test_c2_fits_in_distribution(golden_dir):
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
    print(f"C2 in distribution ({len(seeds)} seeds, N={n}): nfev mean GPU {mg:.2f} oracle {mo:.2f} "
          f"(GPU {nf_gpu}, oracle {nf_ora}); worst rel: {worst}")
    assert abs(mg - mo) <= 0.10 * mo, (mg, mo)
