"""GPU parity of the block-cyclic-reduction path (csrc/gpx_bcr.hip): engines on the "bcr" route
(gpx_batch_set_band_route) evaluate their band16 problems by block cyclic reduction over the
block-tridiagonal band (log-depth levels instead of the one-wavefront sweeps' N/16 steps).

Against the band16 sweeps of the same build (GPX_BCR_MAX=0), the dense path and the oracle.
Both banded paths are exact restatements of the dense factorisation that differ
in summation order only: logML 1e-9 relative, gradient 1e-7·(1 + max|g|) between them, the
oracle bars of tests/test_gpu_parity.py against the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import portfoliooptgp_amd as gpx  # noqa: E402
from portfoliooptgp_amd import _native as N  # noqa: E402
from oracle import gp_oracle as O  # noqa: E402
from tests.test_band_gpu import _Dense, _Env, _engine, _theta, _cond  # noqa: E402
from tests.test_gpu_parity import check_grad, check_loss, check_mean, check_var, gpx_kernel, oracle_kernel  # noqa: E402

K = gpx.kernels


def _sweeps():
    return _Env("GPX_BCR_MAX", "0")


@pytest.fixture(autouse=True)
def _bcr_route(monkeypatch):
    """The engines of these tests take the BCR route (gpx_batch_set_band_route; the default is the
    sweeps); _sweeps() switches a block to the sweeps by the process-wide override."""
    monkeypatch.delenv("GPX_BCR_MAX", raising=False)
    prev = gpx.set_default_band_route("bcr")
    yield
    gpx.set_default_band_route(prev)


def _close(la, ga, lb, gb, P, what, rows=None):
    for b in (range(len(la)) if rows is None else rows):
        assert abs(la[b] - lb[b]) <= 1e-9 * abs(lb[b]), (what, b, la[b], lb[b])
        tol = 1e-7 * (1.0 + np.abs(gb[b, :P]).max())
        assert np.all(np.abs(ga[b, :P] - gb[b, :P]) <= tol), (what, b, ga[b, :P], gb[b, :P])


@pytest.mark.parametrize("n", [2048, 4096])
def test_bcr_equals_sweeps_and_dense(n):
    """C2/C3 sizes: ℓ giving band16 widths Q = 1..5 (one chain per width group), a ragged member;
    against the band16 sweeps and the dense path; predictions at the training inputs (α and
    diag(K⁻¹) of the selected inverse); a problem alone in its call gives the same bits as in the
    mixed call (its arithmetic depends on its own width only)."""
    data = [O.synthetic_series(n, seed=s) for s in range(7)]
    xs = [d[0] for d in data]
    ys = [d[1] for d in data]
    xs[5], ys[5] = xs[5][: n - 1095], ys[5][: n - 1095]
    eng = _engine(xs, ys, K.SquaredExponential())
    rows = [(0.3, 1.0, 1e-5), (0.7, 0.9, 1e-5), (1.0, 1.0, 1e-5), (1.1795, 0.5632, 1e-5),
            (1.6, 0.8649, 1e-5), (1.5, 0.7, 1e-5), (1.9, 1.1, 1e-5)]
    th = _theta(eng, rows)
    act = list(range(7))
    q = eng.band_class(act, th)
    assert set(int(c) for c in q) >= {1, 2, 3, 4, 5}, q
    eng.reset_timing()
    lb, gb, ib = eng.lml_grad(act, th)
    t = eng.last_timing()
    assert not ib.any()
    assert t.bcr_evals == 7 and t.band16_evals == 0 and t.band_fallbacks == 0, (t.bcr_evals, t.band16_evals)
    mb, vb, _ = eng._predict_train(np.arange(7, dtype=np.int32), th, False)
    with _sweeps():
        eng.reset_timing()
        ls, gs, i_s = eng.lml_grad(act, th)
        assert eng.last_timing().bcr_evals == 0 and eng.last_timing().band16_evals == 7
        ms, vs, _ = eng._predict_train(np.arange(7, dtype=np.int32), th, False)
    _close(lb, gb, ls, gs, 3, "bcr vs band16 sweeps")
    for b in range(7):
        np.testing.assert_allclose(mb[b].cpu().numpy(), ms[b].cpu().numpy(), rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(vb[b].cpu().numpy(), vs[b].cpu().numpy(), rtol=1e-7, atol=1e-13)
    with _Dense():
        ld, gd, idn = eng.lml_grad(act, th)
        assert not idn.any()
    _close(lb, gb, ld, gd, 3, "bcr vs dense")
    # batch composition: each problem alone in its call, the same bits
    for b in act:
        eng.reset_timing()
        l1, g1, _ = eng.lml_grad([b], th)
        assert eng.last_timing().bcr_evals == 1
        assert l1[b] == lb[b] and np.array_equal(g1[b, :3], gb[b, :3]), b


@pytest.mark.parametrize("fam,ell", [("se", 1.0), ("se", 1.4), ("m12", 0.02), ("m32", 0.05), ("m52", 0.06),
                                     ("exp", 0.01), ("se+m12", 0.05), ("se*m12", 0.9)])
def test_bcr_against_oracle_n1024(fam, ell):
    """logML, ∂loss/∂u and predict_f at the training inputs through the reduction vs the oracle
    (N = 1024, C2 data), single- and multi-term kernels: the drop-in pattern (one GPR, one call)."""
    x, y = O.synthetic_series(1024, seed=3)
    m = gpx.models.GPR((x, y), kernel=gpx_kernel(fam), noise_variance=1e-5)
    ko = oracle_kernel(fam)
    for p, po in zip(m.kernel.parameters, ko.params()):
        v = ell if "lengthscale" in p.name else 0.8
        p.assign(v)
        po.value = v
    om = O.OGPR(x, y, ko, noise_variance=1e-5)
    N.Context.get(0).set_profiling(True)
    from portfoliooptgp_amd.engine import solo_engine
    eng = solo_engine(m)
    eng.reset_timing()
    loss, g = m.loss_and_grad_unconstrained()
    assert eng.last_timing().bcr_evals == 1, "expected the reduction path"
    assert eng.last_timing().band_fallbacks == 0
    lo, go = om.loss_and_grad_u()
    cond = _cond(x, ko, 1e-5)
    check_loss(loss, lo, cond)
    check_grad(g, go)
    mu, var = m.predict_f(x)
    mo, vo = om.predict_f(x)
    check_mean(mu.numpy(), mo, cond, float(np.abs(y).max()))
    check_var(var.numpy(), vo, 1.0)


def test_bcr_two_dimensional_ragged():
    """D = 2 (time + a feature), Matern32 over both dims, n = 1000 (the last block padded)."""
    n = 1000
    rng = np.random.default_rng(5)
    t = np.arange(n, dtype=np.float64)
    f = np.cumsum(rng.standard_normal(n)) * 0.01
    x = np.stack([t, f], 1)
    y = rng.standard_normal((n, 1))
    m = gpx.models.GPR((x, y), kernel=K.Matern32(lengthscales=0.05, variance=1.1), noise_variance=1e-4)
    om = O.OGPR(x, y, O.OMatern32(lengthscales=0.05, variance=1.1), noise_variance=1e-4)
    N.Context.get(0).set_profiling(True)
    from portfoliooptgp_amd.engine import solo_engine
    eng = solo_engine(m)
    eng.reset_timing()
    loss, g = m.loss_and_grad_unconstrained()
    assert eng.last_timing().bcr_evals == 1
    lo, go = om.loss_and_grad_u()
    cond = _cond(x, O.OMatern32(lengthscales=0.05, variance=1.1), 1e-4)
    check_loss(loss, lo, cond)
    check_grad(g, go)


def test_bcr_irregular_spacing_matches_dense():
    """Irregularly spaced inputs (trading days with gaps): every K block differs from its
    neighbours, so a block read for the wrong node or level would show."""
    n = 4096
    rng = np.random.default_rng(11)
    xs, ys = [], []
    for s in range(4):
        gaps = 1.0 + rng.choice([0.0, 0.0, 0.0, 0.0, 2.0], size=n) + 0.3 * rng.random(n)
        xs.append(np.cumsum(gaps)[:, None] - 1.0)
        ys.append(O.synthetic_series(n, seed=20 + s)[1])
    eng = _engine(xs, ys, K.SquaredExponential())
    th = _theta(eng, [(1.0, 1.0, 1e-5), (1.4, 0.7, 1e-5), (1.6, 0.9, 1e-5), (1.2, 1.2, 1e-5)])
    act = [0, 1, 2, 3]
    eng.reset_timing()
    lb, gb, ib = eng.lml_grad(act, th)
    t = eng.last_timing()
    assert not ib.any() and t.bcr_evals == 4 and t.band_fallbacks == 0
    mb, vb, _ = eng._predict_train(np.arange(4, dtype=np.int32), th, False)
    with _Dense():
        ld, gd, _ = eng.lml_grad(act, th)
        md, vd, _ = eng._predict_train(np.arange(4, dtype=np.int32), th, False)
    _close(lb, gb, ld, gd, 3, "bcr vs dense (irregular)")
    for b in range(4):
        np.testing.assert_allclose(mb[b].cpu().numpy(), md[b].cpu().numpy(), rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(vb[b].cpu().numpy(), vd[b].cpu().numpy(), rtol=1e-7, atol=1e-13)


def test_bcr_not_positive_definite():
    """A NaN input row: the reduction reports a failing pivot (info > 0, NaN logML), as GPflow's
    Cholesky raises; the other problem of the call is unaffected."""
    n = 1024
    x = np.arange(n, dtype=np.float64)[:, None]
    xb = x.copy()
    xb[700] = np.nan
    y = np.random.default_rng(2).standard_normal((n, 1))
    eng = _engine([xb, x], [y, y], K.SquaredExponential())
    th = _theta(eng, [(1.0, 1.0, 1e-5), (1.0, 1.0, 1e-5)])
    eng.reset_timing()
    lml, grad, info = eng.lml_grad([0, 1], th)
    assert eng.last_timing().bcr_evals == 2
    assert info[0] > 0 and np.isnan(lml[0]) and info[1] == 0 and np.isfinite(lml[1])


def test_bcr_check_forced_failure_falls_back():
    """A band-check tolerance no evaluation can meet sends the problem to the dense
    re-evaluation in the same call: results are the dense path's."""
    x, y = O.synthetic_series(2048, seed=4)
    eng = _engine([x], [y], K.SquaredExponential())
    th = _theta(eng, [(1.2, 0.7, 1e-5)])
    with _Env("GPX_BAND_TOL", "1e-30"):
        eng.reset_timing()
        lb, gb, _ = eng.lml_grad([0], th)
        t = eng.last_timing()
        assert t.bcr_evals == 1 and t.band_fallbacks == 1
    with _Dense():
        ld, gd, _ = eng.lml_grad([0], th)
    assert lb[0] == ld[0] and np.array_equal(gb[0, :3], gd[0, :3])


def test_bcr_band_storage_matches_dense_layout():
    """Band-storage slots (the continuous-batching engine) through the reduction: the same bits as
    a dense-layout batch (the reduction reads X and Y, writes α / diag(Z) into either layout)."""
    n = 2048
    data = [O.synthetic_series(n, seed=40 + s) for s in range(3)]
    from portfoliooptgp_amd.engine import Engine
    from portfoliooptgp_amd.kernels import compile_spec
    spec = compile_spec(K.SquaredExponential(), 1)
    e1 = Engine([d[0] for d in data], [d[1] for d in data], [spec] * 3, band_storage=True)
    e2 = Engine([d[0] for d in data], [d[1] for d in data], [spec] * 3)
    e1.ctx.set_profiling(True)
    th = _theta(e1, [(1.18, 0.9, 1e-5), (1.6, 1.0, 1e-5), (1.0, 0.8, 1e-5)])
    e1.reset_timing()
    l1, g1, _ = e1.lml_grad([0, 1, 2], th)
    assert e1.last_timing().bcr_evals == 3
    l2, g2, _ = e2.lml_grad([0, 1, 2], th)
    assert np.array_equal(l1, l2) and np.array_equal(g1[:, :3], g2[:, :3])
    m1, v1, _ = e1._predict_train(np.arange(3, dtype=np.int32), th, False)
    m2, v2, _ = e2._predict_train(np.arange(3, dtype=np.int32), th, False)
    for b in range(3):
        assert np.array_equal(m1[b].cpu().numpy(), m2[b].cpu().numpy())
        assert np.array_equal(v1[b].cpu().numpy(), v2[b].cpu().numpy())


@pytest.mark.parametrize("n", [4096, 4001, 2048])
def test_bcr_wide_q6_to_q8(n):
    """on the reduction route the widths Q = 6..8 (ℓ ≥ 2.3 on unit-spaced day
    offsets, where the shared-kernel warm starts of GPR/main.py:105-114 drift) take ONE
    block-cyclic-reduction chain of block size 128 (gpx_bcr.hip bcrw_*) — before round 6 they went
    to the 64-row sweeps there. Against the dense path (logML 1e-9, gradient 1e-7·(1 + max|g|)),
    the one-wavefront Q = 6..8 sweeps of the default route, the 64-row p = 2 sweeps
    (GPX_BAND16_QMAX=5), the band oracle at ℓ ∈ {2.5, 3} (SURVEY §8c bars), predict at the
    training inputs against the dense factor, and each problem alone in its call (the same bits)."""
    from tests.test_band16_gpu import _band_oracle_loss_grad
    ells = [2.0, 2.3, 2.5, 2.7, 3.0]
    data = [O.synthetic_series(n, seed=70 + s) for s in range(len(ells))]
    eng = _engine([d[0] for d in data], [d[1] for d in data], K.SquaredExponential())
    assert eng.band_route == "bcr"
    th = _theta(eng, [(e, 0.9, 1e-5) for e in ells])
    act = list(range(len(ells)))
    cls = eng.band_class(act, th)
    assert int(cls[0]) == 5 and all(6 <= int(c) <= 8 for c in cls[1:]) and int(cls[-1]) == 8, cls
    eng.reset_timing()
    lb, gb, ib = eng.lml_grad(act, th)
    t = eng.last_timing()
    assert not ib.any() and t.bcr_wide_evals == 4 and t.bcr_evals >= 1 and t.band_fallbacks == 0, \
        (t.bcr_wide_evals, t.bcr_evals, t.band_fallbacks)
    assert t.band_fused_launches == 0 and t.band16_evals == 0, (t.band_fused_launches, t.band16_evals)
    mb, vb, _ = eng._predict_train(np.arange(len(ells), dtype=np.int32), th, False)
    for b in act:  # composition: alone in its call, the same bits
        l1, g1, _ = eng.lml_grad([b], th)
        assert l1[b] == lb[b] and np.array_equal(g1[b, :3], gb[b, :3]), b
    with _sweeps():  # the default route's one-wavefront sweeps (Q = 5..8)
        eng.reset_timing()
        ls, gs, i_s = eng.lml_grad(act, th)
        assert not i_s.any() and eng.last_timing().band16_evals == len(ells) and eng.last_timing().bcr_wide_evals == 0
    _close(lb, gb, ls, gs, 3, "bcr wide vs the Q = 6..8 sweeps")
    with _Dense():
        ld, gd, idn = eng.lml_grad(act, th)
        assert not idn.any()
        md, vd, _ = eng._predict_train(np.arange(len(ells), dtype=np.int32), th, False)
    _close(lb, gb, ld, gd, 3, "bcr wide vs dense")
    for b in range(len(ells)):
        np.testing.assert_allclose(mb[b].cpu().numpy(), md[b].cpu().numpy(), rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(vb[b].cpu().numpy(), vd[b].cpu().numpy(), rtol=1e-7, atol=1e-13)
    with _sweeps(), _Env("GPX_BAND16_QMAX", "5"):
        eng.reset_timing()
        l64, g64, i64 = eng.lml_grad(act, th)
        assert not i64.any() and eng.last_timing().band_fused_launches > 0
    _close(lb, gb, l64, g64, 3, "bcr wide vs the 64-row p = 2 sweeps")
    for b, e in enumerate(ells):
        if e not in (2.5, 3.0):
            continue
        m = gpx.models.GPR(data[b], kernel=K.SquaredExponential(lengthscales=e, variance=0.9), noise_variance=1e-5)
        gpx.set_trainable(m.likelihood.variance, False)
        loss, g = m.loss_and_grad_unconstrained(lml=lb[b], grad_theta=gb[b])
        lo, go = _band_oracle_loss_grad(*data[b], e, 0.9)
        assert abs(loss - lo) <= 1e-9 * abs(lo), (e, loss, lo)
        assert np.abs(g - go).max() <= 1e-6 * max(1.0, np.abs(go).max()), (e, g, go)


def test_bcr_wide_fit_matches_dense_fit():
    """A whole fit that starts in the wide classes (GPflow's L-BFGS-B from ℓ = 2.8 on a C2 series,
    as a warm start from a previous fit's kernel would, GPR/model_trainer.py:15) through the wide
    chain, against the same fit on the dense path: the fitted loss to 1e-5 relative."""
    x, y = O.synthetic_series(2048, seed=5)

    def fit(dense):
        m = gpx.models.GPR((x, y), kernel=K.SquaredExponential(lengthscales=2.8))
        m.likelihood.variance.assign(1e-5)
        gpx.set_trainable(m.likelihood.variance, False)
        if dense:
            with _Dense():
                return gpx.optimizers.Scipy().minimize(m.training_loss, m.trainable_variables,
                                                       options=dict(maxiter=100))
        return gpx.optimizers.Scipy().minimize(m.training_loss, m.trainable_variables, options=dict(maxiter=100))

    rb, rd = fit(False), fit(True)
    assert abs(rb.fun - rd.fun) <= 1e-5 * abs(rd.fun), (rb.fun, rd.fun)
