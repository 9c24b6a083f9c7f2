"""A fit's arithmetic does not depend on its call's size (VERDICT r05 "do this" 2).

The banded route of a band16 problem (the one-wavefront sweeps or block cyclic reduction; they
agree to ~1e-9 relative, not bit for bit) is a property of the ENGINE (include/gpx.h
gpx_batch_set_band_route), never of how many problems share a call. So the same C2 series fitted

  * alone — models.GPR + Scipy().minimize, one problem per call, as GPR/model_trainer.py:14-19
    runs the reference's loop — and
  * inside a 64-problem Scipy().minimize_stream, whose calls start at 64 problems and shrink
    through the round-5 threshold (32) to 1 as the fits converge (the drain),

gives the identical fun, x and nfev, and the identical prediction, under each route: the default
("sweeps") and the latency route ("bcr"). Both routes' parity with the oracle is in
tests/test_c2_parity_gpu.py and tests/test_c2_dist_gpu.py."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import portfoliooptgp_amd as gpx  # noqa: E402
from oracle import gp_oracle as O  # noqa: E402

K = gpx.kernels
N_C2 = 4096
NOISE = 1e-5
MAXITER = 100


def _model(seed):
    x, y = O.synthetic_series(N_C2, seed=seed)
    m = gpx.models.GPR(data=(x, y), kernel=K.SquaredExponential())
    m.likelihood.variance.assign(NOISE)
    gpx.set_trainable(m.likelihood.variance, False)
    return m


@pytest.fixture(params=["sweeps", "bcr"])
def band_route(request, monkeypatch):
    monkeypatch.delenv("GPX_BCR_MAX", raising=False)  # (the process-wide A/B override: not here)
    prev = gpx.set_default_band_route(request.param)
    yield request.param
    gpx.set_default_band_route(prev)


def test_solo_fit_equals_fit_in_a_draining_64_problem_stream(band_route, monkeypatch):
    monkeypatch.setenv("GPX_TRACE_ROUNDS", "1")  # (the driver records each call's size)
    target = 0
    solo = _model(target)
    eng, _ = solo.engine()
    assert eng.B == 1 and eng.band_route == band_route
    eng.ctx.set_profiling(True)
    eng.reset_timing()
    r1 = gpx.optimizers.Scipy().minimize(solo.training_loss, solo.trainable_variables,
                                         options=dict(maxiter=MAXITER))
    t = eng.last_timing()
    assert t.band_evals > 0 and t.band_fallbacks == 0
    assert (t.bcr_evals > 0) == (band_route == "bcr"), (band_route, t.bcr_evals)
    m1, v1 = solo.predict_f(solo.data[0])

    # the same series as fit 17 of 64 (seeds 100.. for the others), every slot resident at once
    models = [_model(100 + i) for i in range(64)]
    models[17] = _model(target)
    opt = gpx.optimizers.Scipy()
    res, preds = opt.minimize_stream(models, width=64, predict_train=True, options=dict(maxiter=MAXITER))
    trace = getattr(opt, "last_trace", None) or []
    r2 = res[17]
    assert r2.nfev == r1.nfev and r2.nit == r1.nit, (r1.nfev, r2.nfev)
    assert float(r2.fun) == float(r1.fun), (r1.fun, r2.fun)
    assert np.array_equal(np.asarray(r2.x), np.asarray(r1.x)), (r1.x, r2.x)
    m2, v2 = preds[17]
    assert np.array_equal(m2.reshape(-1).cpu().numpy(), m1.reshape(-1).cpu().numpy())
    assert np.array_equal(v2.reshape(-1).cpu().numpy(), v1.reshape(-1).cpu().numpy())
    # the stream's calls did shrink through the round-5 threshold (32) while fit 17 ran
    sizes = [int(e[-1]) for e in trace]
    assert sizes and max(sizes) > 32 and min(sizes) <= 32, sizes


def test_route_is_validated():
    m = _model(1)
    eng, _ = m.engine()
    with pytest.raises(ValueError):
        eng.set_band_route("fastest")
    with pytest.raises(ValueError):
        gpx.set_default_band_route("fastest")
