"""Deferred completion of the slow evaluation classes (include/gpx.h gpx_batch_set_deferred):
the problems of a call that take the band16 sweeps wider than q 16-blocks, or the 64-row
sweeps, come back from a later complete (or gpx_batch_deferred_wait) with results identical,
bit for bit, to an undeferred evaluation; the rest of the call completes without them."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import portfoliooptgp_amd as gpx  # noqa: E402
from portfoliooptgp_amd import _native as N  # noqa: E402
from portfoliooptgp_amd.engine import Engine  # noqa: E402
from portfoliooptgp_amd.kernels import compile_spec  # noqa: E402
from oracle import gp_oracle as O  # noqa: E402

K = gpx.kernels


@pytest.fixture(autouse=True)
def _band16_sweeps(monkeypatch):
    """These tests are about the one-wavefront band16 sweeps: keep their small calls off the
    block-cyclic-reduction path (gpx_bcr.hip, tests/test_bcr_gpu.py), which takes calls of at most
    GPX_BCR_MAX band16 problems by default."""
    monkeypatch.setenv("GPX_BCR_MAX", "0")
# ℓ on unit-spaced day offsets -> band16 width Q (38.6 ℓ rows): 1.18 -> 3, 1.6 -> 4, 1.9 -> 5;
# 2.3 -> 89 rows: the 64-row sweeps (p = 2)
# Q = 3, 4, 5 and 6, 7 (SE1 with K inline: band16; GPX_BAND16_QMAX=5: the 64-row sweeps)
ELLS = [1.18, 1.6, 1.18, 1.9, 2.3, 1.0, 1.6, 1.9, 1.18, 2.8]


def _engine(n, data, defer):
    spec = compile_spec(K.SquaredExponential(), 1)
    eng = Engine([d[0] for d in data], [d[1] for d in data], [spec] * len(data), band_storage=True)
    if defer is not None:
        eng.set_deferred(defer)
    return eng


def _theta(ells):
    th = np.ones((len(ells), N.GPX_THETA_STRIDE))
    th[:, 0] = ells
    th[:, 1] = 0.7
    th[:, 2] = 1e-5
    return th


@pytest.mark.parametrize("qmax", ["8", "5"])
@pytest.mark.parametrize("n", [2048, 4096])
def test_deferred_results_equal_undeferred(n, qmax, monkeypatch):
    monkeypatch.setenv("GPX_BAND16_QMAX", qmax)
    data = [O.synthetic_series(n, s) for s in range(len(ELLS))]
    th = _theta(ELLS)
    ref = _engine(n, data, None)
    l0, g0, i0 = ref.lml_grad(list(range(len(ELLS))), th)
    assert not i0.any()
    cls = ref.band_class(list(range(len(ELLS))), th)
    slow = [b for b, c in enumerate(cls) if not (1 <= c <= 3)]
    fast = [b for b, c in enumerate(cls) if 1 <= c <= 3]
    assert len(slow) >= 4 and len(fast) >= 3
    # the deferred part holds the 64-row chain with the Q <= 5 limit, Q = 6, 7 band16 classes without
    assert any(c >= 32 for c in cls) if qmax == "5" else (6 in cls and 7 in cls and not any(c >= 32 for c in cls))
    eng = _engine(n, data, 3)
    eng.lml_grad_submit(list(range(len(ELLS))), th)
    l1, g1, i1 = eng.lml_grad_complete()
    got = {}
    for b in fast:
        assert i1[b] == 0 and l1[b] == l0[b] and np.array_equal(g1[b, :3], g0[b, :3])
    for b in slow:
        assert i1[b] in (N.INFO_DEFERRED, 0)
        if i1[b] == 0:
            got[b] = (l1[b], g1[b, :3].copy())
    # a deferred row may not be evaluated again before its delivery
    pend = [b for b in slow if i1[b] == N.INFO_DEFERRED]
    if pend:
        with pytest.raises(N.GPXError):
            eng.lml_grad_submit([pend[0]], th)
    # a second call of the fast rows alone may deliver the slow ones
    eng.lml_grad_submit(fast, th)
    l2, g2, i2 = eng.lml_grad_complete()
    for b in fast:
        assert i2[b] == 0 and l2[b] == l0[b]
    for b in slow:
        if b not in got and i2[b] == 0:
            got[b] = (l2[b], g2[b, :3].copy())
    l3, g3, i3 = eng.deferred_wait()
    for b in slow:
        if b not in got:
            assert i3[b] == 0
            got[b] = (l3[b], g3[b, :3].copy())
    for b in slow:
        assert got[b][0] == l0[b] and np.array_equal(got[b][1], g0[b, :3]), (b, ELLS[b])
    # nothing left in flight: every row can be evaluated again, and deferral can be turned off
    l4, _, i4 = eng.lml_grad(list(range(len(ELLS))), th)
    eng.deferred_wait()
    eng.set_deferred(-1)
    l5, _, i5 = eng.lml_grad(list(range(len(ELLS))), th)
    assert not i5.any() and np.array_equal(l5, l0)


def test_deferred_fits_equal_undeferred_fits():
    """C2 fits (N = 2048) through minimize_stream with deferral on: every fit's nfev, x and
    prediction bit-identical to the same fits without deferral."""
    n, F = 2048, 12
    data = [O.synthetic_series(n, 40 + s) for s in range(F)]

    def run(defer):
        def model(i):
            m = gpx.models.GPR(data=data[i], kernel=K.SquaredExponential())
            m.likelihood.variance.assign(1e-5)
            gpx.set_trainable(m.likelihood.variance, False)
            return m
        models = gpx.optimizers.ModelStream(F, model, input_dim=1, max_points=n)
        eng = _engine(n, data[:6], defer)
        return gpx.optimizers.Scipy().minimize_stream(models, width=6, engine=eng, predict_train=True,
                                                      options=dict(maxiter=100))

    r0, p0 = run(None)
    r1, p1 = run(3)
    for a, b, pa, pb in zip(r0, r1, p0, p1):
        assert a.nfev == b.nfev and np.array_equal(a.x, b.x) and a.fun == b.fun
        assert np.array_equal(pa[0].cpu().numpy(), pb[0].cpu().numpy())
        assert np.array_equal(pa[1].cpu().numpy(), pb[1].cpu().numpy())


def test_deferred_redo_path_and_wait_while_submitted():
    """a deferred row whose band check fails is re-evaluated densely when it is
    delivered (here every check fails: GPX_BAND_TOL=1e-30), with the results of the undeferred
    call at the same tolerance; deferred_wait is refused while an evaluation is submitted (the
    re-evaluation would need the batch), and works once it is completed."""
    import os
    # (a short fast problem, n = 600, whose synchronous dense redo in the complete is quick, and long
    # slow ones: the slow part is still in flight when the first complete returns — round 6's wide
    # classes take the short reduction chain, so at one size for all the part could finish first)
    n = 4096
    ells = [1.18, 1.6, 1.9, 2.3, 2.8, 1.6, 1.9]
    data = [O.synthetic_series(n, s) for s in range(len(ells))]
    data[0] = (data[0][0][:600], data[0][1][:600])
    th = _theta(ells)
    act = list(range(len(ells)))
    prev = os.environ.get("GPX_BAND_TOL")
    os.environ["GPX_BAND_TOL"] = "1e-30"
    try:
        ref = _engine(n, data, None)
        l0, g0, i0 = ref.lml_grad(act, th)
        assert not i0.any()
        slow = [b for b, c in enumerate(ref.band_class(act, th)) if not (1 <= c <= 3)]
        assert len(slow) == 6, slow
        for attempt in range(5):  # (until the first complete returns with the slow part in flight)
            eng = _engine(n, data, 3)
            eng.lml_grad_submit(act, th)
            rows = np.zeros(len(act), dtype=np.int32)
            k = eng.lib.gpx_batch_deferred_rows(eng.handle, rows.ctypes.data, len(act))
            assert sorted(rows[:k].tolist()) == slow, (rows[:k], slow)  # the slow classes were deferred
            l1, g1, i1 = eng.lml_grad_complete()
            pend = [b for b in act if i1[b] == N.INFO_DEFERRED]
            if pend:
                break
            for b in act:  # (delivered at once: the same results)
                assert i1[b] == 0 and l1[b] == l0[b] and np.array_equal(g1[b, :3], g0[b, :3]), (b, i1[b])
        assert pend
        fast = [b for b in act if b not in pend]
        eng.lml_grad_submit(fast, th)
        with pytest.raises(N.GPXError):
            eng.deferred_wait()
        l2, g2, i2 = eng.lml_grad_complete()
        for b in pend:  # delivered by the complete (its slow part had finished) or still in flight
            if i2[b] == 0:
                l1[b], g1[b], i1[b] = l2[b], g2[b], 0
        l3, g3, i3 = eng.deferred_wait()
        for b in pend:
            if i3[b] != N.INFO_UNSET:
                l1[b], g1[b], i1[b] = l3[b], g3[b], i3[b]
        for b in act:
            assert i1[b] == 0 and l1[b] == l0[b] and np.array_equal(g1[b, :3], g0[b, :3]), (b, i1[b])
    finally:
        if prev is None:
            os.environ.pop("GPX_BAND_TOL", None)
        else:
            os.environ["GPX_BAND_TOL"] = prev
