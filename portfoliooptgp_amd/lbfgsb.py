"""scipy's L-BFGS-B, driven by reverse communication instead of a callback.

``scipy.optimize.minimize(fun, x0, jac=True, method="L-BFGS-B", options=...)`` (what
``gpflow.optimizers.Scipy`` calls, GPR/model_trainer.py:18-19) is a Python loop around the
compiled L-BFGS-B routine ``setulb``: ``setulb`` asks for f and g at a point, the loop calls
``fun`` there, and repeats until ``setulb`` reports convergence, or until ``maxiter`` / ``maxfun``
stops it. ``LbfgsbStepper`` runs that same loop (scipy 1.15's ``_minimize_lbfgsb`` with no
bounds and no callback) as a generator. The caller reads the requested point, evaluates it
and passes ``(f, g)`` back. Many fits can then be stepped from ONE host thread, and every
request of a round is evaluated in one batched device call.

The memoisation follows scipy's ``ScalarFunction`` / ``MemoizeJac``: a point equal to the last
evaluated one is not evaluated again. ``nfev``, ``nit``, the messages and the returned fields
are scipy's. Each fit's sequence of ``setulb`` calls is therefore exactly the one
``scipy.optimize.minimize`` makes, so its trajectory is bit-identical
(``tests/test_stream_driver.py`` compares against scipy itself with atol=0).
"""
from __future__ import annotations

from typing import Optional

import numpy as np
from scipy.optimize import OptimizeResult

try:  # scipy ≥ 1.15: the C port of L-BFGS-B (task codes as int32 pairs)
    from scipy.optimize import _lbfgsb
    from scipy.optimize._lbfgsb_py import LbfgsInvHessProduct, status_messages, task_messages
    AVAILABLE = hasattr(_lbfgsb, "setulb") and isinstance(status_messages, dict)
except Exception:  # pragma: no cover - older scipy: callers use the threaded driver
    AVAILABLE = False
try:  # the same loop in C++ over a batch of fits (csrc/gpx_lbfgsb_host.cpp), when built
    from . import _gpx_lbfgsb as _native_loop
except ImportError:  # pragma: no cover - the Python stepper serves
    _native_loop = None
if not AVAILABLE:  # pragma: no cover - said once, at import: the fits still run, more slowly
    import warnings
    warnings.warn("scipy's L-BFGS-B routine setulb (scipy >= 1.15 layout) is not available: batched fits use the "
                  "threaded driver (one host thread per fit; same results, several times slower)", RuntimeWarning)

# scipy 1.15 _minimize_lbfgsb defaults
_DEFAULTS = dict(maxcor=10, ftol=2.2204460492503131e-09, gtol=1e-5, maxfun=15000, maxiter=15000, maxls=20)
# options accepted by _minimize_lbfgsb that have no effect with jac=True and no bounds
_INERT = {"disp", "iprint", "eps", "finite_diff_rel_step"}


def supports(method: str, scipy_kwargs: dict) -> bool:
    """True when minimize(..., method, **scipy_kwargs) is a plain unbounded L-BFGS-B run
    that the stepper reproduces exactly."""
    if not AVAILABLE or str(method).lower() != "l-bfgs-b":
        return False
    if set(scipy_kwargs) - {"options"}:
        return False  # bounds, callback, tol, ... : leave those to scipy itself
    opts = scipy_kwargs.get("options") or {}
    return not (set(opts) - set(_DEFAULTS) - _INERT)


class _Result(OptimizeResult):
    """scipy's OptimizeResult whose ``hess_inv`` (an LbfgsInvHessProduct: ≈9 µs to construct,
    most of a finished fit's host cost, rarely read) is built on first access. Every dict view
    (keys, items, iteration, repr, ``in``) builds it first, so the result reads as scipy's."""

    def _hess(self):
        if not dict.__contains__(self, "hess_inv"):
            s, y = dict.pop(self, "_sy")
            dict.__setitem__(self, "hess_inv", LbfgsInvHessProduct(s, y))

    def __missing__(self, key):
        if key == "hess_inv" and dict.__contains__(self, "_sy"):
            self._hess()
            return dict.__getitem__(self, "hess_inv")
        raise KeyError(key)

    def _views(name):  # noqa: N805 - method factory
        def f(self, *a, **k):
            if dict.__contains__(self, "_sy"):
                self._hess()
            return getattr(OptimizeResult, name)(self, *a, **k)
        f.__name__ = name
        return f

    for _n in ("keys", "items", "values", "__iter__", "__len__", "__repr__", "__contains__", "get",
               "copy", "__eq__", "__reduce__", "__dir__", "pop", "__str__"):
        locals()[_n] = _views(_n)
    del _n, _views


class LbfgsbStepper:
    """One L-BFGS-B minimisation. ``x`` is the point whose (f, g) is wanted next (None once
    finished); ``tell(f, g)`` supplies it; ``result()`` is scipy's OptimizeResult."""

    def __init__(self, x0, options: Optional[dict] = None):
        opts = dict(_DEFAULTS)
        opts.update({k: v for k, v in (options or {}).items() if k in _DEFAULTS})
        x0 = _x0(x0)
        if not opts["maxls"] > 0:
            raise ValueError("maxls must be positive.")
        self.nfev = 0
        self._res: Optional[OptimizeResult] = None
        self._gen = self._run(x0.ravel(), opts)
        self.x: Optional[np.ndarray] = next(self._gen)

    @property
    def done(self) -> bool:
        return self.x is None

    def tell(self, f, g) -> None:
        try:
            self.x = self._gen.send((f, g))
        except StopIteration:
            self.x = None

    def result(self) -> OptimizeResult:
        return self._res

    @staticmethod
    def _scalar(fx):
        if type(fx) is float:
            return fx
        if not np.isscalar(fx):
            try:
                fx = np.asarray(fx).item()
            except (TypeError, ValueError) as e:
                raise ValueError("The user-provided objective function must return a scalar value.") from e
        return fx

    def _run(self, x0, o):
        m, pgtol = o["maxcor"], o["gtol"]
        factr = o["ftol"] / np.finfo(float).eps
        n, = x0.shape
        # ScalarFunction: f and g at x0 up front (one evaluation), then memoised on x
        sf_x = np.atleast_1d(x0).astype(np.float64)
        fx, gx = yield sf_x.copy()
        self.nfev = 1
        sf_f, sf_g = self._scalar(fx), np.atleast_1d(gx)

        nbd = np.zeros(n, np.int32)
        low_bnd = np.zeros(n, np.float64)
        upper_bnd = np.zeros(n, np.float64)
        x = np.array(x0, dtype=np.float64)
        f = np.array(0.0, dtype=np.int32)
        g = np.zeros((n,), dtype=np.int32)
        wa = np.zeros(2 * m * n + 5 * n + 11 * m * m + 8 * m, np.float64)
        iwa = np.zeros(3 * n, dtype=np.int32)
        task = np.zeros(2, dtype=np.int32)
        ln_task = np.zeros(2, dtype=np.int32)
        lsave = np.zeros(4, dtype=np.int32)
        isave = np.zeros(44, dtype=np.int32)
        dsave = np.zeros(29, dtype=np.float64)
        n_iterations = 0
        maxiter, maxfun, maxls = o["maxiter"], o["maxfun"], o["maxls"]
        setulb = _lbfgsb.setulb
        sf_key = sf_x.tolist()
        while True:
            if g.dtype != np.float64:  # scipy re-casts g every pass; only the first is not f64
                g = g.astype(np.float64)
            setulb(m, x, low_bnd, upper_bnd, nbd, f, g, factr, pgtol, wa,
                   iwa, task, lsave, isave, dsave, maxls, ln_task)
            t0 = task[0]
            if t0 == 3:  # f and g wanted at x
                # np.array_equal(x, sf_x) for two float64 vectors of one shape: Python float
                # equality of the elements (0.0 == -0.0; NaN unequal: tolist() makes new objects)
                key = x.tolist()
                if key != sf_key:
                    sf_x = x.copy()
                    sf_key = key
                    fx, gx = yield sf_x
                    self.nfev += 1
                    # np.atleast_1d(gx), without its dispatch for the usual 1-D float64 row
                    sf_f = self._scalar(fx)
                    sf_g = gx if type(gx) is np.ndarray and gx.ndim == 1 else np.atleast_1d(gx)
                f, g = sf_f, sf_g.copy()  # setulb gets its own g, as scipy's per-pass astype copy
            elif t0 == 1:  # new iteration
                n_iterations += 1
                if n_iterations >= maxiter:
                    task[0], task[1] = 5, 504
                elif self.nfev > maxfun:
                    task[0], task[1] = 5, 502
            else:
                break
        if task[0] == 4:
            warnflag = 0
        elif self.nfev > o["maxfun"] or n_iterations >= o["maxiter"]:
            warnflag = 1
        else:
            warnflag = 2
        self._res = _result(x, f, g, wa, task, isave, m, n, self.nfev, n_iterations, warnflag)


def _result(x, f, g, wa, task, isave, m, n, nfev, nit, warnflag, copy=False):
    """scipy's OptimizeResult of a finished run from its work arrays (_minimize_lbfgsb's tail);
    copy=True when the arrays belong to a reused batch slot."""
    s = wa[0: m * n].reshape(m, n)
    y = wa[m * n: 2 * m * n].reshape(m, n)
    n_corrs = min(isave[30], m)
    msg = status_messages[task[0]] + ": " + task_messages[task[1]]
    if copy:
        x, g, s, y = x.copy(), g.copy(), s[:n_corrs].copy(), y[:n_corrs].copy()
    else:
        s, y = s[:n_corrs], y[:n_corrs]
    return _Result(fun=f, jac=g, nfev=nfev, njev=nfev, nit=nit, status=warnflag, message=msg, x=x,
                   success=(warnflag == 0), _sy=(s, y))


def _x0(x0):
    x0 = np.atleast_1d(np.asarray(x0))
    if x0.ndim != 1:
        raise ValueError("'x0' must only have one dimension.")
    if x0.dtype.kind in np.typecodes["AllInteger"]:
        x0 = np.asarray(x0, dtype=float)
    return x0


class BatchStepper:
    """``cap`` L-BFGS-B runs of dimension ``n`` with common options, advanced by the C++ loop of
    csrc/gpx_lbfgsb_host.cpp (``_gpx_lbfgsb``): the same loop as LbfgsbStepper around scipy's own
    ``setulb``, for a whole round of fits in one call (``tell``), so the per-evaluation host cost
    is the setulb calls themselves. Slot ``i`` holds one run at a time (``start``); ``gather``
    reads the rows' requested points, ``tell`` hands back their (f, g) and flags the finished
    ones; ``stepper(i)`` is the LbfgsbStepper-shaped view of one slot."""

    NATIVE = _native_loop is not None

    def __init__(self, cap: int, n: int, options: Optional[dict] = None):
        if _native_loop is None:
            raise RuntimeError("the native L-BFGS-B loop (portfoliooptgp_amd/_gpx_lbfgsb*.so) is not built")
        o = dict(_DEFAULTS)
        o.update({k: v for k, v in (options or {}).items() if k in _DEFAULTS})
        if not o["maxls"] > 0:
            raise ValueError("maxls must be positive.")
        self.o, self.n, self.m = o, n, o["maxcor"]
        m = self.m
        # _minimize_lbfgsb's work arrays (dtypes and sizes), per slot; the bounds stay zero (none)
        self.arrays = [(np.zeros(n), np.zeros(n), np.zeros(n), np.zeros(n, np.int32), np.zeros(n),
                        np.zeros(2 * m * n + 5 * n + 11 * m * m + 8 * m), np.zeros(3 * n, np.int32),
                        np.zeros(2, np.int32), np.zeros(4, np.int32), np.zeros(44, np.int32), np.zeros(29),
                        np.zeros(2, np.int32)) for _ in range(cap)]
        factr = o["ftol"] / np.finfo(float).eps
        self._b = _native_loop.Batch(_lbfgsb.setulb, cap, n, m, float(factr), float(o["gtol"]), int(o["maxls"]),
                                     int(o["maxiter"]), int(o["maxfun"]), self.arrays)
        self.gather = self._b.gather  # gather(rows int32[k], out float64[k, n])
        self.tell = self._b.tell      # tell(rows int32[k], f float64[k], g float64[k, n], done uint8[k])

    def start(self, slot: int, x0) -> "_SlotStepper":
        x0 = _x0(x0).ravel()
        if x0.shape[0] != self.n:
            raise ValueError(f"x0 has {x0.shape[0]} elements, the batch {self.n}")
        self._b.start(slot, np.ascontiguousarray(x0, dtype=np.float64))
        return _SlotStepper(self, slot)

    def request(self, slot: int) -> np.ndarray:
        return np.frombuffer(self._b.request(slot), dtype=np.float64)

    def result(self, slot: int) -> OptimizeResult:
        state, nfev, nit, f = self._b.state(slot)
        x, _, _, _, g, wa, _, task, _, isave, _, _ = self.arrays[slot]
        o = self.o
        if task[0] == 4:
            warnflag = 0
        elif nfev > o["maxfun"] or nit >= o["maxiter"]:
            warnflag = 1
        else:
            warnflag = 2
        return _result(x, f, g, wa, task, isave, self.m, self.n, nfev, nit, warnflag, copy=True)


class _SlotStepper:
    """LbfgsbStepper's interface over one BatchStepper slot."""
    __slots__ = ("b", "slot", "_res")

    def __init__(self, b: BatchStepper, slot: int):
        self.b, self.slot, self._res = b, slot, None

    @property
    def x(self):
        return None if self.done else self.b.request(self.slot)

    @property
    def done(self) -> bool:
        return self.b._b.state(self.slot)[0] == 3

    @property
    def nfev(self) -> int:
        return self.b._b.state(self.slot)[1]

    def tell(self, f, g) -> None:
        self.b._b.tell_one(self.slot, float(LbfgsbStepper._scalar(f)),
                           np.ascontiguousarray(np.atleast_1d(g), dtype=np.float64))

    def result(self) -> OptimizeResult:
        if self._res is None and self.done:
            self._res = self.b.result(self.slot)
        return self._res
