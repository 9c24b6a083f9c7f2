"""The streaming / lock-step drivers of optimizers.Scipy on the CPU with a stand-in engine:
every fit must see exactly the trajectory it would see alone, whatever the slot count, the
number of concurrent device batches, and the refill order (the device arithmetic is covered
by the GPU tests; this pins the host-side scheduling: barriers, rebinding, predict requests)."""
import numpy as np
import pytest
import scipy.optimize
import torch

import portfoliooptgp_amd as gpx
from portfoliooptgp_amd import _native as N


@pytest.fixture(params=["native", "python"], autouse=True)
def lbfgsb_loop(request, monkeypatch):
    """Every driver test with both L-BFGS-B loops: the C++ loop over a batch of fits
    (lbfgsb.BatchStepper, the default) and the Python stepper per fit (GPX_NATIVE_LBFGSB=0)."""
    from portfoliooptgp_amd.lbfgsb import BatchStepper
    if request.param == "native" and not BatchStepper.NATIVE:
        pytest.skip("portfoliooptgp_amd/_gpx_lbfgsb*.so is not built")
    monkeypatch.setenv("GPX_NATIVE_LBFGSB", "1" if request.param == "native" else "0")
    return request.param


class FakeEngine:
    """lml(θ) = −Σ_p (log θ_p − log t_p)² with per-problem targets t from the bound data."""

    def __init__(self, B):
        self.B, self.device = B, 0
        self.target = np.ones((B, 2))
        self.n_params = np.full(B, 2)
        self.calls = []

    def rebind(self, b, X, Y, spec):
        y = np.asarray(Y, dtype=np.float64).reshape(-1)
        self.target[b] = [1.0 + abs(y.mean()) * 3.0, 0.5 + y.std()]

    def lml_grad(self, rows, theta, wait_deferred=True):
        self.calls.append(len(rows))
        lml = np.full(self.B, np.nan)
        grad = np.full((self.B, N.GPX_THETA_STRIDE), np.nan)
        info = np.zeros(self.B, dtype=np.int32)
        for r in rows:
            d = np.log(theta[r, :2]) - np.log(self.target[r])
            lml[r] = -np.sum(d * d)
            grad[r] = 0.0
            grad[r, :2] = -2.0 * d / theta[r, :2]
        return lml, grad, info

    def predict(self, rows, theta, xs, add_noise):
        return ([torch.full((len(x),), float(theta[r, 0])) for r, x in zip(rows, xs)],
                [torch.full((len(x),), float(theta[r, 1])) for r, x in zip(rows, xs)], None)


def _models(k):
    rng = np.random.default_rng(0)
    out = []
    for i in range(k):
        x = np.arange(10.0)[:, None]
        y = rng.standard_normal((10, 1)) * (1 + i % 3) + 0.2 * i
        m = gpx.models.GPR((x, y), kernel=gpx.kernels.SquaredExponential())
        m.likelihood.variance.assign(1e-5)
        gpx.set_trainable(m.likelihood.variance, False)
        out.append(m)
    return out


def _solo(m):
    eng = FakeEngine(1)
    eng.rebind(0, m.data[0], m.data[1], None)
    v = m.trainable_variables

    def f(u):
        for var, ui in zip(v, u):
            var.assign(ui)
        th = np.ones((1, N.GPX_THETA_STRIDE))
        th[0] = m.theta_row()
        lml, g, _ = eng.lml_grad([0], th)
        return m.loss_and_grad_unconstrained(v, lml=lml[0], grad_theta=g[0])
    return scipy.optimize.minimize(f, np.array([x.numpy() for x in v], dtype=float), jac=True,
                                   method="L-BFGS-B")


@pytest.mark.parametrize("width,groups,engines", [(3, 1, 1), (4, 2, 1), (4, 2, 2), (6, 3, 3)])
def test_stream_equals_solo(width, groups, engines):
    ms = _models(11)
    ref = [_solo(m) for m in _models(11)]
    per = width // engines
    eng = [FakeEngine(per) for _ in range(engines)]
    res, preds = gpx.optimizers.Scipy().minimize_stream(
        ms, width=width, engine=eng if engines > 1 else eng[0], groups=groups, predict_train=True)
    for r, r0, m, p in zip(res, ref, ms, preds):
        assert r.nfev == r0.nfev
        np.testing.assert_allclose(r.x, r0.x, rtol=0, atol=0)
        assert float(p[0][0, 0]) == pytest.approx(m.kernel.lengthscales.value)
    assert max(max(e.calls) for e in eng) <= per


class NotPDEngine(FakeEngine):
    """As FakeEngine, but K + σn²I 'fails to factor' once the lengthscale passes 2.5."""

    def lml_grad(self, rows, theta, wait_deferred=True):
        lml, grad, info = super().lml_grad(rows, theta)
        for r in rows:
            if theta[r, 0] > 2.5:
                info[r] = 7
        return lml, grad, info


def test_not_positive_definite_raises_like_gpflow_or_backs_off():
    """Default: a failed factorisation raises (GPflow: tf.linalg.cholesky's InvalidArgumentError
    escapes Scipy.minimize). on_not_pd="inf": the point gets an infinite loss, L-BFGS-B's line
    search backs off and the fit ends inside the factorisable region."""
    ms = _models(4)
    for m in ms:
        m.kernel.lengthscales.assign(1.0)
    with pytest.raises(N.NotPositiveDefiniteError):
        gpx.optimizers.Scipy().minimize_stream(_models(4), width=2, engine=NotPDEngine(2))
    res, _ = gpx.optimizers.Scipy().minimize_stream(ms, width=2, engine=NotPDEngine(2), on_not_pd="inf")
    for r, m in zip(res, ms):
        assert np.isfinite(r.fun)
        assert m.kernel.lengthscales.value <= 2.5
    with pytest.raises(ValueError):
        gpx.optimizers.Scipy().minimize_stream(_models(1), width=1, engine=NotPDEngine(1), on_not_pd="ignore")


class BadThetaEngine(FakeEngine):
    """As FakeEngine, but the lengthscale counts as out of (0, ∞) once it passes 2.5 (the
    device engine's host-side screen marks such rows INFO_BAD_THETA and skips them)."""

    def lml_grad(self, rows, theta, wait_deferred=True):
        lml, grad, info = super().lml_grad(rows, theta)
        for r in rows:
            if theta[r, 0] > 2.5:
                info[r] = N.INFO_BAD_THETA
        return lml, grad, info


def test_out_of_domain_hyperparameters_fail_one_fit_only():
    """A fit whose θ leaves (0, ∞) raises InvalidParameterError (default) or backs off
    (on_not_pd="inf"); with "inf" every fit of the batch finishes."""
    with pytest.raises(N.InvalidParameterError):
        gpx.optimizers.Scipy().minimize_stream(_models(4), width=2, engine=BadThetaEngine(2))
    ms = _models(4)
    res, _ = gpx.optimizers.Scipy().minimize_stream(ms, width=2, engine=BadThetaEngine(2), on_not_pd="inf")
    for r, m in zip(res, ms):
        assert np.isfinite(r.fun) and m.kernel.lengthscales.value <= 2.5


def test_screen_theta():
    from portfoliooptgp_amd.engine import screen_theta
    th = np.ones((4, N.GPX_THETA_STRIDE))
    th[1, 0] = 0.0          # softplus underflow
    th[2, 2] = np.nan       # beyond problem 2's parameters (n_params=1: θ0, σn² at index 1) ...
    th[3, 1] = np.inf       # ... σn² of problem 3
    info = np.zeros(4, dtype=np.int32)
    act = screen_theta(np.arange(4, dtype=np.int32), th, np.array([2, 2, 1, 1]), info)
    assert list(act) == [0, 2] and list(info) == [0, N.INFO_BAD_THETA, 0, N.INFO_BAD_THETA]


def test_lbfgsb_stepper_is_scipy():
    """The reverse-communication driver makes exactly scipy.optimize.minimize's setulb calls:
    same x, fun, jac, nfev, nit, status and message, including maxiter / maxfun stops and an
    infinite-loss region (the on_not_pd="inf" back-off)."""
    from portfoliooptgp_amd.lbfgsb import LbfgsbStepper

    def rosen(x):
        return scipy.optimize.rosen(x), scipy.optimize.rosen_der(x)

    def walled(x):
        if x[0] > 2.0:
            return float("inf"), np.zeros_like(x)
        return float(-x[0] + (x[1] - 1.0) ** 2), np.array([-1.0, 2.0 * (x[1] - 1.0)])

    cases = [(rosen, [-1.2, 1.0, 0.3, 2.0], {}), (rosen, [0.0] * 7, dict(maxiter=15)),
             (rosen, [3.0, -2.0], dict(maxfun=20)), (walled, [0.0, 0.0], dict(maxiter=100)),
             (rosen, [0.5413248546129181] * 2, dict(maxiter=100, ftol=1e-12, gtol=1e-9, maxcor=5, maxls=10))]
    for fn, x0, opts in cases:
        r0 = scipy.optimize.minimize(fn, np.array(x0), jac=True, method="L-BFGS-B", options=opts)
        st = LbfgsbStepper(np.array(x0), opts)
        while not st.done:
            st.tell(*fn(st.x.copy()))
        r1 = st.result()
        np.testing.assert_array_equal(r1.x, r0.x)
        np.testing.assert_array_equal(r1.jac, r0.jac)
        assert (r1.fun, r1.nfev, r1.njev, r1.nit, r1.status, r1.message) == \
               (r0.fun, r0.nfev, r0.njev, r0.nit, r0.status, r0.message)


def test_batch_stepper_is_scipy(lbfgsb_loop):
    """The C++ loop (lbfgsb.BatchStepper: scipy's setulb called from gpx_lbfgsb_host.cpp, a whole
    round of fits per call) against scipy.optimize.minimize, atol = 0: the cases of
    test_lbfgsb_stepper_is_scipy, each one run in several slots of one batch stepped together,
    a slot reused for a second fit, and the L-BFGS memory (hess_inv) as well."""
    if lbfgsb_loop != "native":
        pytest.skip("the native loop's own test")
    from portfoliooptgp_amd.lbfgsb import BatchStepper

    def rosen(x):
        return scipy.optimize.rosen(x), scipy.optimize.rosen_der(x)

    def walled(x):
        if x[0] > 2.0:
            return float("inf"), np.zeros_like(x)
        return float(-x[0] + (x[1] - 1.0) ** 2), np.array([-1.0, 2.0 * (x[1] - 1.0)])

    cases = [(rosen, [-1.2, 1.0, 0.3, 2.0], {}), (rosen, [0.0] * 7, dict(maxiter=15)),
             (rosen, [3.0, -2.0], dict(maxfun=20)), (walled, [0.0, 0.0], dict(maxiter=100)),
             (rosen, [0.5413248546129181] * 2, dict(maxiter=100, ftol=1e-12, gtol=1e-9, maxcor=5, maxls=10))]
    for fn, x0, opts in cases:
        n = len(x0)
        starts = [np.array(x0) + 0.25 * k for k in range(3)]
        refs = [scipy.optimize.minimize(fn, s0, jac=True, method="L-BFGS-B", options=opts) for s0 in starts]
        b = BatchStepper(3, n, opts)
        # slot 2 first runs another fit to its end, then the case's third start: a reused slot
        b.start(2, np.array(x0) - 0.5)
        for phase in (0, 1):
            rows = [2] if phase == 0 else [0, 1, 2]
            if phase == 1:
                for k in rows:
                    b.start(k, starts[k])
            act = np.array(rows, dtype=np.int32)
            while len(act):
                U = np.empty((len(act), n))
                b.gather(act, U)
                F, G = np.empty(len(act)), np.empty((len(act), n))
                for j in range(len(act)):
                    F[j], G[j] = fn(U[j].copy())
                d = np.zeros(len(act), np.uint8)
                b.tell(act, F, G, d)
                act = act[d == 0]
        for k, r0 in enumerate(refs):
            r1 = b.result(k)
            np.testing.assert_array_equal(r1.x, r0.x)
            np.testing.assert_array_equal(r1.jac, r0.jac)
            assert (r1.fun, r1.nfev, r1.njev, r1.nit, r1.status, r1.message) == \
                   (r0.fun, r0.nfev, r0.njev, r0.nit, r0.status, r0.message)
            np.testing.assert_array_equal(r1.hess_inv.sk, r0.hess_inv.sk)
            np.testing.assert_array_equal(r1.hess_inv.yk, r0.hess_inv.yk)


def test_stream_driver_uses_the_native_loop(lbfgsb_loop, monkeypatch):
    """By default the stepped driver advances its fits through BatchStepper.tell (one call per
    pack of a round), and GPX_NATIVE_LBFGSB=0 keeps it on the per-fit Python stepper."""
    from portfoliooptgp_amd import lbfgsb
    calls = []
    real = lbfgsb.BatchStepper.__init__

    def init(self, *a, **k):
        real(self, *a, **k)
        t = self.tell
        self.tell = lambda *x: (calls.append(len(x[0])), t(*x))[1]
    monkeypatch.setattr(lbfgsb.BatchStepper, "__init__", init)
    res, _ = gpx.optimizers.Scipy().minimize_stream(_models(6), width=3, engine=FakeEngine(3))
    assert all(r.success for r in res)
    assert (sum(calls) > 0) == (lbfgsb_loop == "native")


def test_batch_equals_solo():
    """minimize_batch (lock-step, model i in row i) gives every fit its solo trajectory."""
    ms = _models(5)
    ref = [_solo(m) for m in _models(5)]
    eng = FakeEngine(5)
    for b, m in enumerate(ms):
        eng.rebind(b, m.data[0], m.data[1], None)
    res = gpx.optimizers.Scipy().minimize_batch(ms, engine=eng)
    for r, r0 in zip(res, ref):
        assert r.nfev == r0.nfev and r.message == r0.message
        np.testing.assert_allclose(r.x, r0.x, rtol=0, atol=0)
    assert eng.calls[0] == 5


def test_model_without_trainable_variables_fails_alone():
    """A fit that cannot start (nothing trainable) raises ValueError after the others finish,
    in both the lock-step and the streaming driver."""
    for stream in (False, True):
        ms = _models(3)
        gpx.set_trainable(ms[1].kernel.lengthscales, False)
        gpx.set_trainable(ms[1].kernel.variance, False)
        eng = FakeEngine(3)
        for b, m in enumerate(ms):
            eng.rebind(b, m.data[0], m.data[1], None)
        with pytest.raises(ValueError, match="no trainable variables"):
            if stream:
                gpx.optimizers.Scipy().minimize_stream(ms, width=2, engine=FakeEngine(2))
            else:
                gpx.optimizers.Scipy().minimize_batch(ms, engine=eng)
        assert ms[0].kernel.lengthscales.value != 1.0 and ms[2].kernel.lengthscales.value != 1.0


@pytest.mark.parametrize("width,engines_b,expect", [(5, (3, 2), [3, 2]), (3, (2, 1), [2, 1]),
                                                    (4, (3, 2), [2, 2]), (2, (3, 2), [1, 1])])
def test_stream_uses_every_engine_row(width, engines_b, expect):
    """Unequal engines (the last of a ceil split is smaller) contribute all their rows, and the
    width cap deals the slots round-robin over the groups: `width` slots in total, not
    groups x the smallest engine."""
    from portfoliooptgp_amd.optimizers import _SteppedDriver
    ms = _models(9)
    eng = [FakeEngine(b) for b in engines_b]
    drv = _SteppedDriver(ms, eng, len(eng), {}, False, 1, width=width)
    assert [len(rows) for _, rows, _, _ in drv.groups] == expect
    ref = [_solo(m) for m in _models(9)]
    res, _ = gpx.optimizers.Scipy().minimize_stream(ms, width=width, engine=eng, groups=len(eng))
    for r, r0 in zip(res, ref):
        assert r.nfev == r0.nfev
        np.testing.assert_allclose(r.x, r0.x, rtol=0, atol=0)


class AsyncFakeEngine(FakeEngine):
    """FakeEngine with the submit / complete halves: the driver then steps every group from
    one host thread (optimizers._SteppedDriver._pipeline)."""

    def lml_grad_submit(self, rows, theta):
        self._sub = self.lml_grad(rows, theta.copy())

    def lml_grad_complete(self):
        out, self._sub = self._sub, None
        return out


@pytest.mark.parametrize("width,engines", [(4, 2), (6, 3), (5, 2)])
def test_pipelined_groups_equal_solo(width, engines):
    ms = _models(13)
    ref = [_solo(m) for m in _models(13)]
    per = -(-width // engines)
    eng = [AsyncFakeEngine(per) for _ in range(engines)]
    res, preds = gpx.optimizers.Scipy().minimize_stream(ms, width=width, engine=eng, groups=engines,
                                                        predict_train=True)
    for r, r0, m, p in zip(res, ref, ms, preds):
        assert r.nfev == r0.nfev
        np.testing.assert_allclose(r.x, r0.x, rtol=0, atol=0)
        assert float(p[0][0, 0]) == pytest.approx(m.kernel.lengthscales.value)
    assert sum(sum(e.calls) for e in eng) == sum(r.nfev for r in res)


class BandFakeEngine(AsyncFakeEngine):
    """AsyncFakeEngine that also answers the band-width routing query: 'wide' (p = 2) when
    the requested lengthscale exceeds 1.5, so fits cross between the narrow and wide batches."""

    def band_width(self, rows, theta):
        return np.array([2 if theta[r, 0] > 1.5 else 1 for r in rows], dtype=np.int32)

    def lml_grad(self, rows, theta, wait_deferred=True):
        self.classes = getattr(self, "classes", []) + [self.band_width(rows, theta)]
        return super().lml_grad(rows, theta)


def test_wide_group_routing_keeps_trajectories():
    ms = _models(17)
    ref = [_solo(m) for m in _models(17)]
    eng = [BandFakeEngine(4), BandFakeEngine(4), BandFakeEngine(3)]
    opt = gpx.optimizers.Scipy()
    res, preds = opt.minimize_stream(ms, width=11, engine=eng, groups=3, predict_train=True, wide_group=True)
    for r, r0, m, p in zip(res, ref, ms, preds):
        assert r.nfev == r0.nfev
        np.testing.assert_allclose(r.x, r0.x, rtol=0, atol=0)
        assert float(p[0][0, 0]) == pytest.approx(m.kernel.lengthscales.value)
    # fits did move into the wide batch, which evaluated mostly wide points (a fit with no
    # free narrow slot to go back to is evaluated where it is)
    wide_pts = np.concatenate(getattr(eng[2], "classes", [np.zeros(0, np.int32)]))
    assert len(wide_pts) > 0 and (wide_pts == 2).mean() > 0.5


@pytest.mark.parametrize("engines", [1, 3])
def test_model_stream_builds_on_demand_and_keeps_trajectories(engines):
    # a ModelStream (models built when a slot takes them, or while the host waits for the
    # device) gives the same fits as the list of the same models, each model built once
    src = _models(13)
    ref = [_solo(m) for m in _models(13)]
    calls = []

    def factory(i):
        calls.append(i)
        return src[i]
    ms = gpx.optimizers.ModelStream(13, factory, input_dim=1, max_points=10)
    assert len(ms) == 13 and calls == []
    eng = [AsyncFakeEngine(2) for _ in range(engines)] if engines > 1 else FakeEngine(4)
    res, preds = gpx.optimizers.Scipy().minimize_stream(ms, width=4 if engines == 1 else 6, engine=eng,
                                                        groups=engines, predict_train=True)
    assert sorted(calls) == list(range(13))
    for r, r0, m, p in zip(res, ref, ms, preds):
        assert r.nfev == r0.nfev
        np.testing.assert_allclose(r.x, r0.x, rtol=0, atol=0)
        assert float(p[0][0, 0]) == pytest.approx(m.kernel.lengthscales.value)
    with pytest.raises(IndexError):
        ms[13]


def test_stepper_result_reads_as_scipys():
    # the stepper's result builds hess_inv lazily; keys, `in`, attribute and item access and
    # the operator itself are scipy's
    from portfoliooptgp_amd import lbfgsb

    def f(x):
        return float(((x - np.arange(3)) ** 2).sum() + np.sin(x).sum()), 2 * (x - np.arange(3)) + np.cos(x)
    st = lbfgsb.LbfgsbStepper(np.zeros(3))
    while not st.done:
        st.tell(*f(st.x))
    r = st.result()
    r0 = scipy.optimize.minimize(f, np.zeros(3), jac=True, method="L-BFGS-B")
    assert "hess_inv" in r and sorted(r.keys()) == sorted(r0.keys())
    np.testing.assert_array_equal(r.hess_inv.todense(), r0.hess_inv.todense())
    assert r["hess_inv"] is r.hess_inv
    np.testing.assert_array_equal(r.x, r0.x)


class AsyncFakeEngine(FakeEngine):
    """FakeEngine with the split submit / complete calls of Engine; like gpx_batch it holds ONE
    pending evaluation (a second submit before the complete is refused)."""

    def __init__(self, B):
        super().__init__(B)
        self._pending = None

    def lml_grad_submit(self, rows, theta):
        if self._pending is not None:
            raise N.GPXError("an evaluation is already submitted on this batch")
        self._pending = self.lml_grad(list(rows), np.array(theta, copy=True))

    def lml_grad_ready(self):
        return True

    def lml_grad_complete(self):
        out, self._pending = self._pending, None
        return out


@pytest.mark.parametrize("engines", [1, 2])
def test_groups_on_one_engine_with_submit(engines):
    """two groups that are row ranges of ONE engine with submit support
    must not go through the one-thread pipeline (both groups would submit on the same batch);
    distinct engines do. Either way every fit equals its solo fit."""
    ms = _models(9)
    ref = [_solo(m) for m in _models(9)]
    eng = [AsyncFakeEngine(4 // engines) for _ in range(engines)]
    res, _ = gpx.optimizers.Scipy().minimize_stream(ms, width=4, engine=eng if engines > 1 else eng[0],
                                                    groups=2)
    for r, r0 in zip(res, ref):
        assert r.nfev == r0.nfev
        np.testing.assert_allclose(r.x, r0.x, rtol=0, atol=0)


class CachedPredictEngine(FakeEngine):
    """FakeEngine with a rough (noisy) objective, so that L-BFGS-B's line search sometimes backs
    off and returns a point other than the last one evaluated, and a predict at the training
    inputs that, like the band-storage engine's, is only served from the factor of the row's
    LAST evaluated θ (it records any other request)."""

    def __init__(self, B):
        super().__init__(B)
        self.last_theta = {}
        self.uncached = 0

    def lml_grad(self, rows, theta, wait_deferred=True):
        lml, grad, info = super().lml_grad(rows, theta)
        for r in rows:
            lml[r] += 1e-7 * np.sin(1e9 * theta[r, 0])     # rounding-level roughness
            self.last_theta[r] = theta[r].copy()
        return lml, grad, info

    def _predict_train(self, rows, theta, add_noise, column=False):
        for r in rows:
            if not np.array_equal(theta[r], self.last_theta.get(r)):
                self.uncached += 1
        mu = [torch.full((10, 1), float(theta[r, 0]), dtype=torch.float64) for r in rows]
        var = [torch.full((10, 1), float(theta[r, 1]), dtype=torch.float64) for r in rows]
        return mu, var, None


def test_predict_after_backed_off_line_search_uses_a_fresh_evaluation():
    """A fit whose result is not its last evaluated point gets one more (batched) evaluation at
    the result's x before its predict, so the predict at the training inputs always finds the
    factor of its θ; the results (x, nfev) are scipy's, untouched."""
    ms = _models(12)
    for m in ms:
        m.kernel.lengthscales.assign(3.0)
    eng = CachedPredictEngine(4)
    res, preds = gpx.optimizers.Scipy().minimize_stream(ms, width=4, engine=eng, predict_train=True)
    assert eng.uncached == 0
    assert sum(eng.calls) > sum(r.nfev for r in res)      # some fits were evaluated once more
    for r, m, p in zip(res, ms, preds):
        assert float(p[0][0, 0]) == m.kernel.lengthscales.value
        assert m.kernel.lengthscales.unconstrained == r.x[0]


def test_blas_thread_limit_is_process_wide_and_counted():
    """Overlapping single-thread-BLAS contexts (concurrent fits): the limit holds until the
    last one exits, then the previous count comes back."""
    from portfoliooptgp_amd.optimizers import _BlasThreads

    class Lib:
        def __init__(self):
            self.n = 8

        def get_num_threads(self):
            return self.n

        def set_num_threads(self, n):
            self.n = n
    lib = Lib()
    a, b = _BlasThreads([lib]), _BlasThreads([lib])
    a.__enter__()
    assert lib.n == 1
    b.__enter__()
    a.__exit__(None, None, None)
    assert lib.n == 1          # b still stepping
    b.__exit__(None, None, None)
    assert lib.n == 8


class ClassFakeEngine(AsyncFakeEngine):
    """AsyncFakeEngine answering the band-class query (Engine.band_class): band16 width 3
    below ℓ = 1.5, 5 above (slower: wide at the default GPX_NARROW_Q = 3), and a not-yet-known
    class (-2) for ℓ in a narrow window, which must leave the fit where it is."""

    def band_class(self, rows, theta):
        return np.array([-2 if 1.49 < theta[r, 0] <= 1.5 else (5 if theta[r, 0] > 1.5 else 3) for r in rows],
                        dtype=np.int32)

    def lml_grad(self, rows, theta, wait_deferred=True):
        self.classes = getattr(self, "classes", []) + [self.band_class(rows, theta)]
        return super().lml_grad(rows, theta)


def test_wide_group_by_band16_class_keeps_trajectories():
    """The wide batch by band16 class (ClassFakeEngine): fits cross between the narrow and the
    wide batch with their L-BFGS-B state, and every trajectory is the solo one."""
    ms = _models(17)
    ref = [_solo(m) for m in _models(17)]
    eng = [ClassFakeEngine(4), ClassFakeEngine(4), ClassFakeEngine(3)]
    res, preds = gpx.optimizers.Scipy().minimize_stream(ms, width=11, engine=eng, groups=3, predict_train=True,
                                                        wide_group=True)
    for r, r0, m, p in zip(res, ref, ms, preds):
        assert r.nfev == r0.nfev
        np.testing.assert_allclose(r.x, r0.x, rtol=0, atol=0)
        assert float(p[0][0, 0]) == pytest.approx(m.kernel.lengthscales.value)
    wide_pts = np.concatenate(getattr(eng[2], "classes", [np.zeros(0, np.int32)]))
    assert len(wide_pts) > 0 and (wide_pts == 5).mean() > 0.5


class DeferringFakeEngine(FakeEngine):
    """FakeEngine with deferred completion (Engine.set_deferred): a row whose requested
    lengthscale exceeds 1.5 comes back INFO_DEFERRED and is delivered by the NEXT complete (or by
    deferred_wait); a deferred row may not be submitted or rebound before its delivery."""

    deferral = 3

    def __init__(self, B):
        super().__init__(B)
        self._late = {}      # row -> (lml, grad row) of a deferred evaluation
        self._sub = None
        self.deferred_total = 0

    def rebind(self, b, X, Y, spec):
        assert b not in self._late, "rebind of a row with a deferred evaluation"
        super().rebind(b, X, Y, spec)

    def lml_grad_submit(self, rows, theta):
        rows = list(rows)
        assert self._sub is None and not (set(rows) & set(self._late)), "a deferred row was submitted again"
        th = np.array(theta, copy=True)
        self._sub = (rows, th, FakeEngine.lml_grad(self, rows, th))

    def lml_grad_ready(self):
        return True

    def lml_grad_complete(self):
        (rows, th, (lml, grad, _)), self._sub = self._sub, None
        info = np.full(self.B, N.INFO_UNSET, dtype=np.int32)
        for r, (l, g) in self._late.items():  # the last call's deferred rows arrive now
            lml[r], grad[r], info[r] = l, g, 0
        self._late = {}
        for r in rows:
            if th[r, 0] > 1.5:
                self._late[r] = (lml[r], grad[r].copy())
                lml[r], grad[r], info[r] = np.nan, np.nan, N.INFO_DEFERRED
                self.deferred_total += 1
            else:
                info[r] = 0
        return lml, grad, info

    def lml_grad(self, rows, theta, wait_deferred=True):
        self.lml_grad_submit(rows, theta)
        return self.lml_grad_complete()

    def deferred_wait(self):
        lml = np.full(self.B, np.nan)
        grad = np.full((self.B, N.GPX_THETA_STRIDE), np.nan)
        info = np.full(self.B, N.INFO_UNSET, dtype=np.int32)
        for r, (l, g) in self._late.items():
            lml[r], grad[r], info[r] = l, g, 0
        self._late = {}
        return lml, grad, info


@pytest.mark.parametrize("engines", [1, 2])
def test_deferred_rows_keep_trajectories(engines):
    """Rows deferred by the engine (results one call later, drained at the end) are stepped when
    they arrive: every fit's trajectory and prediction is the solo one, each fit is evaluated
    exactly nfev times, and the deferral did happen."""
    ms = _models(17)
    ref = [_solo(m) for m in _models(17)]
    eng = [DeferringFakeEngine(5) for _ in range(engines)]
    res, preds = gpx.optimizers.Scipy().minimize_stream(ms, width=5 * engines, engine=eng if engines > 1 else eng[0],
                                                        groups=engines, predict_train=True)
    for r, r0, m, p in zip(res, ref, ms, preds):
        assert r.nfev == r0.nfev
        np.testing.assert_allclose(r.x, r0.x, rtol=0, atol=0)
        assert float(p[0][0, 0]) == pytest.approx(m.kernel.lengthscales.value)
    assert sum(sum(e.calls) for e in eng) == sum(r.nfev for r in res)
    assert sum(e.deferred_total for e in eng) > 0


class HoldFakeEngine(DeferringFakeEngine):
    """DeferringFakeEngine answering the band-class query: band16 width 6 (a wide sweep) above
    ℓ = 2, 3 below; records each call's classes."""

    def band_class(self, rows, theta):
        return np.array([6 if theta[r, 0] > 2.0 else 3 for r in rows], dtype=np.int32)

    def lml_grad_submit(self, rows, theta):
        self.classes = getattr(self, "classes", []) + [self.band_class(list(rows), theta)]
        super().lml_grad_submit(rows, theta)


def test_hold_wide_keeps_trajectories(monkeypatch):
    """GPX_HOLD_WIDE (default 6:3): on a deferring batch, the rows whose next point is band16
    width >= 6 are submitted only in every H-th round (never all rows held). The schedule
    changes — fewer calls carry a wide row — and every fit's trajectory is still the solo one."""
    ref = [_solo(m) for m in _models(17)]
    share = {}
    for hold in ("0", "6:3", "6/2"):
        monkeypatch.setenv("GPX_HOLD_WIDE", hold)
        eng = HoldFakeEngine(6)
        res, _ = gpx.optimizers.Scipy().minimize_stream(_models(17), width=6, engine=eng, predict_train=True)
        for r, r0 in zip(res, ref):
            assert r.nfev == r0.nfev
            np.testing.assert_allclose(r.x, r0.x, rtol=0, atol=0)
        assert any((c == 6).any() for c in eng.classes)
        share[hold] = np.mean([(c == 6).any() for c in eng.classes])
    assert share["6:3"] < share["0"] and share["6/2"] < share["0"], share


class _CountingAdmission:
    """DeviceAdmission's interface over a plain semaphore, counting the places held at once; a
    blocking acquire that cannot be served fails the test instead of hanging it."""

    def __init__(self, places):
        import threading
        self.places, self.held, self.peak = places, 0, 0
        self._sem = threading.BoundedSemaphore(places)

    def acquire(self):
        assert self._sem.acquire(timeout=5.0), "admission deadlock: no place came back"
        self.held += 1
        self.peak = max(self.peak, self.held)

    def release(self):
        self.held -= 1
        self._sem.release()


@pytest.mark.parametrize("places,engines", [(1, 2), (1, 3), (2, 3)])
def test_admission_one_place_per_pipeline(places, engines):
    """A pipelined driver (one host thread, several device batches) with fewer admission places
    than batches: it holds one place while any of its calls is in flight (a place per
    group deadlocked), and the fits keep their solo trajectories."""
    ms = _models(9)
    ref = [_solo(m) for m in _models(9)]
    eng = [AsyncFakeEngine(2) for _ in range(engines)]
    adm = _CountingAdmission(places)
    res, _ = gpx.optimizers.Scipy().minimize_stream(ms, width=2 * engines, engine=eng, groups=engines,
                                                    admission=adm)
    for r, r0 in zip(res, ref):
        assert r.nfev == r0.nfev
        np.testing.assert_allclose(r.x, r0.x, rtol=0, atol=0)
    assert adm.peak == 1 and adm.held == 0


class _Var:
    """A variable the optimizer surface accepts (numpy / assign / shape), holding one vector."""

    def __init__(self, v):
        self.v = np.array(v, dtype=np.float64)
        self.shape = self.v.shape

    def numpy(self):
        return self.v

    def assign(self, x):
        self.v = np.array(x, dtype=np.float64).reshape(self.shape)


def test_solo_minimize_is_scipy(monkeypatch):
    """Scipy().minimize on one model (the drop-in pattern, GPR/model_trainer.py:18-19) drives scipy's
    setulb through the native loop (round 6): the OptimizeResult is scipy.optimize.minimize's, atol = 0,
    with and without the stepper (GPX_SOLO_STEPPER=0), for a converging, a maxiter-limited and a
    backed-off (infinite loss) run."""
    import portfoliooptgp_amd as gpx

    def rosen(x):
        return float(scipy.optimize.rosen(x)), scipy.optimize.rosen_der(x)

    def walled(x):
        if x[0] > 2.0:
            return float("inf"), np.zeros_like(x)
        return float(-x[0] + (x[1] - 1.0) ** 2), np.array([-1.0, 2.0 * (x[1] - 1.0)])

    for fn, x0, opts in ((rosen, [-1.2, 1.0, 0.3], dict(maxiter=100)), (rosen, [0.0] * 5, dict(maxiter=7)),
                         (walled, [0.0, 0.0], dict(maxiter=100))):
        ref = scipy.optimize.minimize(fn, np.array(x0), jac=True, method="L-BFGS-B", options=opts)
        for stepper in ("1", "0"):
            monkeypatch.setenv("GPX_SOLO_STEPPER", stepper)
            var = _Var(x0)

            def closure():
                raise AssertionError("not called: the optimizer uses _gpx_loss_and_grad")
            closure._gpx_loss_and_grad = lambda variables: fn(variables[0].numpy())
            res = gpx.optimizers.Scipy().minimize(closure, [var], options=opts)
            assert res.nfev == ref.nfev and res.nit == ref.nit and res.message == ref.message, (stepper, res, ref)
            assert res.fun == ref.fun and np.array_equal(res.x, ref.x) and np.array_equal(res.jac, ref.jac)
            assert np.array_equal(var.numpy(), ref.x)
