"""GPU parity of the 16-row-block banded sweeps (csrc/gpx_band16.hip: one wavefront per problem,
band of Q <= 4 16-blocks) against the 64-row fused sweeps of the same build (GPX_BAND16=0), the
dense path and the oracle.

The band16 class takes every p64 <= 1 problem whose band is at most 4 16-blocks: at the C2
inputs (day offsets, σn² = 1e-5) that is ℓ <= 1.68 — Q = 3 up to ℓ = 1.27, Q = 4 above.
Tolerances: logML 1e-9 relative and gradient 1e-7·(1 + max|g|) between the banded variants
(both are exact restatements of the dense factorisation), the oracle bars of
tests/test_gpu_parity.py against the oracle.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import portfoliooptgp_amd as gpx  # noqa: E402
from portfoliooptgp_amd import _native as N  # noqa: E402
from oracle import gp_oracle as O  # noqa: E402
from tests.test_band_gpu import _Dense, _Env, _engine, _theta, _cond  # noqa: E402
from tests.test_gpu_parity import check_grad, check_loss, check_mean, check_var, gpx_kernel, oracle_kernel  # noqa: E402

K = gpx.kernels


@pytest.fixture(autouse=True)
def _band16_sweeps(monkeypatch):
    """These tests are about the one-wavefront band16 sweeps: keep their small calls off the
    block-cyclic-reduction path (gpx_bcr.hip, tests/test_bcr_gpu.py), which takes calls of at most
    GPX_BCR_MAX band16 problems by default."""
    monkeypatch.setenv("GPX_BCR_MAX", "0")


def _no16():
    return _Env("GPX_BAND16", "0")


def _close(la, ga, lb, gb, P, what):
    for b in range(len(la)):
        assert abs(la[b] - lb[b]) <= 1e-9 * abs(lb[b]), (what, b, la[b], lb[b])
        tol = 1e-7 * (1.0 + np.abs(gb[b, :P]).max())
        assert np.all(np.abs(ga[b, :P] - gb[b, :P]) <= tol), (what, b, ga[b, :P], gb[b, :P])


def test_band16_equals_band64_and_dense_n4096():
    """C2 size: ℓ giving Q = 1, 2, 3, 4 (and a ragged n = 3001 member) through the band16 sweeps,
    against the 64-row sweeps and the dense path on the same batch; predictions at the training
    inputs (α and diag(K⁻¹) of the selected inverse) against the 64-row sweeps'."""
    n = 4096
    data = [O.synthetic_series(n, seed=s) for s in range(6)]
    xs = [d[0] for d in data]
    ys = [d[1] for d in data]
    xs[5], ys[5] = xs[5][:3001], ys[5][:3001]
    eng = _engine(xs, ys, K.SquaredExponential())
    rows = [(0.3, 1.0, 1e-5), (0.7, 0.9, 1e-5), (1.0, 1.0, 1e-5), (1.1795, 0.5632, 1e-5),
            (1.6, 0.8649, 1e-5), (1.5, 0.7, 1e-5)]
    th = _theta(eng, rows)
    act = list(range(6))
    eng.reset_timing()
    l16, g16, i16 = eng.lml_grad(act, th)
    t = eng.last_timing()
    assert not i16.any()
    assert t.band16_evals == 6 and t.band_evals == 6, (t.band16_evals, t.band_evals)
    assert t.band_fallbacks == 0, t.band_fallbacks  # every band check passed
    qs = t.band16_q_sum
    assert qs == 1 + 2 + 3 + 3 + 4 + 4, qs
    m16, v16, _ = eng._predict_train(np.arange(6, dtype=np.int32), th, False)
    with _no16():
        eng.reset_timing()
        l64, g64, i64 = eng.lml_grad(act, th)
        t = eng.last_timing()
        assert not i64.any() and t.band16_evals == 0 and t.band_evals == 6
        m64, v64, _ = eng._predict_train(np.arange(6, dtype=np.int32), th, False)
    _close(l16, g16, l64, g64, 3, "band16 vs band64")
    for b in range(6):
        a, c = m16[b].cpu().numpy(), m64[b].cpu().numpy()
        np.testing.assert_allclose(a, c, rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(v16[b].cpu().numpy(), v64[b].cpu().numpy(), rtol=1e-7, atol=1e-13)
    with _Dense():
        ld, gd, idn = eng.lml_grad(act, th)
        assert not idn.any()
    _close(l16, g16, ld, gd, 3, "band16 vs dense")
    # batch composition: a problem's result does not depend on the other problems of the call
    l3, g3, _ = eng.lml_grad([3], th)
    assert l3[3] == l16[3] and np.array_equal(g3[3, :3], g16[3, :3])


@pytest.mark.parametrize("fam,ell", [("se", 1.0), ("se", 1.4), ("m12", 0.02), ("m32", 0.05), ("m52", 0.06),
                                     ("exp", 0.01), ("se+m12", 0.05), ("se*m12", 0.9)])
def test_band16_against_oracle_n1024(fam, ell):
    """logML, ∂loss/∂u and predict_f at the training inputs through the band16 sweeps vs the
    oracle (N = 1024, C2 data), single- and multi-term kernels."""
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
    assert eng.last_timing().band16_evals == 1, "expected the band16 path"
    assert eng.last_timing().band_fallbacks == 0
    lo, go = om.loss_and_grad_u()
    cond = _cond(x, ko, 1e-5)
    check_loss(loss, lo, cond)
    check_grad(g, go)
    mu, var = m.predict_f(x)
    mo, vo = om.predict_f(x)
    check_mean(mu.numpy(), mo, cond, float(np.abs(y).max()))
    check_var(var.numpy(), vo, 1.0)


def test_band16_two_dimensional_and_ragged():
    """D = 2 (time + a feature), Matern32 over both dims, n = 1000 (not a multiple of 16): the
    staged X rows and the padding rows of the last block."""
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
    assert eng.last_timing().band16_evals == 1
    lo, go = om.loss_and_grad_u()
    cond = _cond(x, O.OMatern32(lengthscales=0.05, variance=1.1), 1e-4)
    check_loss(loss, lo, cond)
    check_grad(g, go)


def test_band16_not_positive_definite_reports_pivot():
    """A NaN input row makes pivot 701 fail inside a 16-block: LAPACK-style pivot as the dense
    path reports it."""
    n = 1024
    x = np.arange(n, dtype=np.float64)[:, None]
    x[700] = np.nan
    y = np.random.default_rng(2).standard_normal((n, 1))
    eng = _engine([x], [y], K.SquaredExponential())
    th = _theta(eng, [(1.0, 1.0, 1e-5)])
    eng.reset_timing()
    lml, grad, info = eng.lml_grad([0], th)
    assert eng.last_timing().band16_evals == 1
    assert info[0] == 701 and np.isnan(lml[0])


def test_band16_check_forced_failure_falls_back():
    """A band-check tolerance no evaluation can meet (GPX_BAND_TOL=1e-30) sends the band16
    problem to the dense re-evaluation in the same call: results are the dense path's."""
    n = 2048
    x, y = O.synthetic_series(n, seed=4)
    eng = _engine([x], [y], K.SquaredExponential())
    th = _theta(eng, [(1.2, 0.7, 1e-5)])
    with _Env("GPX_BAND_TOL", "1e-30"):
        eng.reset_timing()
        lb, gb, _ = eng.lml_grad([0], th)
        t = eng.last_timing()
        assert t.band16_evals == 1 and t.band_fallbacks == 1
    with _Dense():
        ld, gd, _ = eng.lml_grad([0], th)
    assert lb[0] == ld[0] and np.array_equal(gb[0, :3], gd[0, :3])


def test_band16_irregular_spacing_matches_dense():
    """Irregularly spaced inputs (trading days with gaps: every K tile differs from its
    neighbours, so a tile staged for the wrong block step would show): band16 vs the dense path
    at N = 4096 over the band16 widths, no band-check fallback."""
    n = 4096
    rng = np.random.default_rng(11)
    xs, ys = [], []
    for s in range(4):
        gaps = 1.0 + rng.choice([0.0, 0.0, 0.0, 0.0, 2.0], size=n) + 0.3 * rng.random(n)
        x = np.cumsum(gaps)[:, None] - 1.0
        xs.append(x)
        ys.append(O.synthetic_series(n, seed=20 + s)[1])
    eng = _engine(xs, ys, K.SquaredExponential())
    th = _theta(eng, [(1.0, 1.0, 1e-5), (1.4, 0.7, 1e-5), (1.6, 0.9, 1e-5), (1.2, 1.2, 1e-5)])
    act = [0, 1, 2, 3]
    eng.reset_timing()
    lb, gb, ib = eng.lml_grad(act, th)
    t = eng.last_timing()
    assert not ib.any() and t.band16_evals == 4 and t.band_fallbacks == 0, (t.band16_evals, t.band_fallbacks)
    mb, vb, _ = eng._predict_train(np.arange(4, dtype=np.int32), th, False)
    with _Dense():
        ld, gd, _ = eng.lml_grad(act, th)
        md, vd, _ = eng._predict_train(np.arange(4, dtype=np.int32), th, False)
    _close(lb, gb, ld, gd, 3, "band16 vs dense (irregular)")
    for b in range(4):
        np.testing.assert_allclose(mb[b].cpu().numpy(), md[b].cpu().numpy(), rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(vb[b].cpu().numpy(), vd[b].cpu().numpy(), rtol=1e-7, atol=1e-13)


def test_band16_wide_class_p64_2():
    """ℓ = 1.8 and 2.0 at the C2 inputs: p64 = 2 (K built with three 64-block diagonals) and
    Q = 5 (the generic-contraction sweep): band16 vs the 64-row p = 2 sweep and the dense path."""
    n = 4096
    data = [O.synthetic_series(n, seed=30 + s) for s in range(3)]
    eng = _engine([d[0] for d in data], [d[1] for d in data], K.SquaredExponential())
    th = _theta(eng, [(1.8, 0.9, 1e-5), (2.0, 1.1, 1e-5), (1.2, 0.8, 1e-5)])
    act = [0, 1, 2]
    eng.reset_timing()
    lb, gb, ib = eng.lml_grad(act, th)
    t = eng.last_timing()
    assert not ib.any() and t.band16_evals == 3 and t.band_fallbacks == 0, (t.band16_evals, t.band_fallbacks)
    assert t.band16_q_sum == 5 + 5 + 3, t.band16_q_sum
    with _no16():
        l64, g64, _ = eng.lml_grad(act, th)
    _close(lb, gb, l64, g64, 3, "band16 vs band64 (p = 2)")
    with _Dense():
        ld, gd, _ = eng.lml_grad(act, th)
    _close(lb, gb, ld, gd, 3, "band16 vs dense (p = 2)")


def _band_oracle_loss_grad(x, y, ell, var):
    """The band oracle (oracle/band_oracle.py: block-tridiagonal Cholesky + Takahashi on the
    exact-zero band, numpy/LAPACK, pinned against the dense oracle in tests/test_band_oracle.py)
    at (ℓ, σ²): loss and ∂loss/∂u for the two kernel parameters (σn² fixed)."""
    from oracle import band_oracle as BO
    bm = BO.OBandGPR(x, y, 1e-5)
    bm.ell, bm.var = float(ell), float(var)
    return bm.loss_and_grad_u()


def test_band16_se1_q6_to_q8_n4096():
    """ℓ ∈ {2, 2.3, 2.5, 2.8, 3} at the C2 inputs: bands of Q = 5..8 16-blocks (p64 = 2). SE1
    problems with K's tiles inline take the band16 sweeps (one wavefront per SIMD, window in VGPRs
    and AGPRs) — no 64-row sweep launch — and agree with the 64-row p = 2 sweeps
    (GPX_BAND16_QMAX=5 sends them there), the dense path, and the band oracle at ℓ ∈ {2, 2.5, 3}
    (logML 1e-9, ∂loss/∂u 1e-6·max(1, |g|): VERDICT r04 item 2)."""
    n = 4096
    ells = [2.0, 2.3, 2.5, 2.8, 3.0]
    data = [O.synthetic_series(n, seed=40 + s) for s in range(len(ells))]
    eng = _engine([d[0] for d in data], [d[1] for d in data], K.SquaredExponential())
    th = _theta(eng, [(e, 0.9, 1e-5) for e in ells])
    act = list(range(len(ells)))
    cls = eng.band_class(act, th)
    assert list(cls) == [5, 6, 6, 7, 8], cls  # (ℓ = 2: Q = 5, the widest class of any kernel family)
    eng.reset_timing()
    lb, gb, ib = eng.lml_grad(act, th)
    t = eng.last_timing()
    assert not ib.any() and t.band16_evals == len(ells) and t.band_fallbacks == 0, (t.band16_evals, t.band_fallbacks)
    assert t.band16_q_sum == int(sum(cls)) and t.band_fused_launches == 0, (t.band16_q_sum, t.band_fused_launches)
    m16, v16, _ = eng._predict_train(np.arange(len(ells), dtype=np.int32), th, False)
    with _Env("GPX_BAND16_QMAX", "5"):
        eng.reset_timing()
        l64, g64, i64 = eng.lml_grad(act, th)
        t = eng.last_timing()
        assert not i64.any() and t.band16_evals == 1 and t.band_fused_launches > 0  # (ℓ = 2 stays at Q = 5)
        m64, v64, _ = eng._predict_train(np.arange(len(ells), dtype=np.int32), th, False)
    _close(lb, gb, l64, g64, 3, "band16 Q 6-8 vs band64 p = 2")
    for b in range(len(ells)):
        np.testing.assert_allclose(m16[b].cpu().numpy(), m64[b].cpu().numpy(), rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(v16[b].cpu().numpy(), v64[b].cpu().numpy(), rtol=1e-7, atol=1e-13)
    with _Dense():
        ld, gd, idn = eng.lml_grad(act, th)
        assert not idn.any()
    _close(lb, gb, ld, gd, 3, "band16 Q 6-8 vs dense")
    for b, e in enumerate(ells):
        if e not in (2.0, 2.5, 3.0):
            continue
        m = gpx.models.GPR(data[b], kernel=K.SquaredExponential(lengthscales=e, variance=0.9), noise_variance=1e-5)
        gpx.set_trainable(m.likelihood.variance, False)
        loss, g = m.loss_and_grad_unconstrained(lml=lb[b], grad_theta=gb[b])
        lo, go = _band_oracle_loss_grad(*data[b], e, 0.9)
        assert abs(loss - lo) <= 1e-9 * abs(lo), (e, loss, lo)
        assert np.abs(g - go).max() <= 1e-6 * max(1.0, np.abs(go).max()), (e, g, go)


def test_mixed_ell_c2_call_band_storage_no_64row_sweeps():
    """A C2 call through band storage (the bench's slots) with ℓ from 1 to 3 (Q = 3..8): every
    evaluation on the band16 sweeps — no 64-row sweep launch, nothing on the fallback slots —
    and each problem's logML and gradient the same as in a call of its own (composition)."""
    from portfoliooptgp_amd.engine import Engine
    from portfoliooptgp_amd.kernels import compile_spec
    n = 4096
    ells = [1.0, 1.18, 1.5, 1.8, 2.0, 2.2, 2.5, 2.7, 3.0, 1.3, 2.9, 1.1]
    data = [O.synthetic_series(n, seed=60 + s) for s in range(len(ells))]
    spec = compile_spec(K.SquaredExponential(), 1)
    eng = Engine([d[0] for d in data], [d[1] for d in data], [spec] * len(ells), band_storage=True)
    eng.ctx.set_profiling(True)
    th = _theta(eng, [(e, 1.0, 1e-5) for e in ells])
    act = list(range(len(ells)))
    eng.reset_timing()
    l, g, info = eng.lml_grad(act, th)
    t = eng.last_timing()
    assert not info.any()
    assert t.band16_evals == len(ells) and t.shadow_evals == 0 and t.band_fused_launches == 0, \
        (t.band16_evals, t.shadow_evals, t.band_fused_launches)
    for b in (0, 4, 8, 10):
        l1, g1, _ = eng.lml_grad([b], th)
        assert l1[b] == l[b] and np.array_equal(g1[b, :3], g[b, :3]), b


def test_reduce_forms_bit_identical():
    """The reduce kernel forms a problem's four 64-lane partial sums with four waves at once in
    calls of at most 64 problems and with one wave, one after another, in larger calls
    (gpx_kernels.hip reduce_kernel<NW>): the same loops, butterflies and combine order, so a
    problem's logML and gradient carry the same bits in a call of 40 and in one of 80 (band16
    sweeps both times: each problem's arithmetic is its own wavefront's)."""
    n = 1024
    data = [O.synthetic_series(n, seed=s) for s in range(80)]
    eng = _engine([d[0] for d in data], [d[1] for d in data], K.SquaredExponential())
    ells = np.linspace(0.8, 1.6, 80)
    th = _theta(eng, [(l, 0.9, 1e-5) for l in ells])
    eng.reset_timing()
    l80, g80, i80 = eng.lml_grad(list(range(80)), th)
    assert eng.last_timing().band16_evals == 80
    for half in (range(0, 40), range(40, 80)):
        act = list(half)
        eng.reset_timing()
        l40, g40, i40 = eng.lml_grad(act, th)
        assert eng.last_timing().band16_evals == 40
        assert np.array_equal(l40[act], l80[act])
        assert np.array_equal(g40[act, :3], g80[act, :3])
        assert np.array_equal(i40[act], i80[act])
