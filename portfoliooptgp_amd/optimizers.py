"""gpflow.optimizers.Scipy with the same call surface, plus a lock-step batched driver.

``Scipy().minimize(model.training_loss, model.trainable_variables, options=dict(maxiter=100))``
(GPR/model_trainer.py:18-19) runs scipy's L-BFGS-B (jac=True) over the concatenated
unconstrained variables and writes the result back, returning scipy's OptimizeResult
(``.fun``, ``.x``, ``.nfev``, ``.nit``; ``opt_logs.fun`` at
Multi-Input_GPR/models/model_trainer.py:40).

``minimize_batch`` / ``minimize_stream`` run one scipy L-BFGS-B per model and evaluate the
points the fits are waiting for together, in ONE batched device pass (gpx_batch_lml_grad).
Each optimiser sees exactly the values a solo run would see, so trajectories are per-fit
identical to sequential fitting while the device works on all fits at once. For plain
L-BFGS-B runs (the reference's) the fits are stepped by reverse communication
(``lbfgsb.LbfgsbStepper``: scipy's own ``setulb`` calls, no callback) from one host thread per
device batch (``_SteppedDriver``). Other methods or options, or GPX_THREADED_DRIVER=1, run
each fit's ``scipy.optimize.minimize`` in its own host thread around a barrier
(``_LockstepEvaluator``).
"""
from __future__ import annotations

import contextlib
import gc
import os
import sys
import queue
import threading
import time
from typing import Callable, List, Optional, Sequence

import numpy as np
import scipy.optimize
import torch

from . import _native as N
from . import lbfgsb
from .engine import Engine
from .kernels import compile_spec
from .parameter import UnconstrainedVariable


# GPX_THREADED_DRIVER=1: one host thread per fit/slot around scipy.optimize.minimize (the
# generic path, always used for methods/options the reverse-communication stepper does not cover)
_THREADED = os.environ.get("GPX_THREADED_DRIVER", "0") not in ("", "0")


class ModelStream(Sequence):
    """``n`` models built on demand by ``factory(i)``, for ``minimize_stream``.

    The reference builds each GPR right before fitting it, inside its per-ticker loop
    (GPR/model_trainer.py:14-15). A list of thousands of models built up front keeps the device
    idle for the whole construction (≈35 µs per GPR). Given a ModelStream, ``minimize_stream``
    builds model i when a slot takes it, or earlier while its host thread waits for the device,
    so construction overlaps device work. ``input_dim`` and ``max_points`` size the device slots
    without building every model first; a model that does not fit them fails alone (its
    rebind raises)."""

    def __init__(self, n: int, factory: Callable[[int], object], input_dim: int, max_points: int,
                 device: Optional[int] = None):
        self._n, self._factory = int(n), factory
        self.input_dim, self.max_points, self.device = int(input_dim), int(max_points), device
        self._built: List[object] = [None] * self._n
        self.next_unbuilt = 0  # every model below this index is built

    def __len__(self) -> int:
        return self._n

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(self._n))]
        if i < 0:
            i += self._n
        if not 0 <= i < self._n:
            raise IndexError(i)
        m = self._built[i]
        if m is None:
            m = self._built[i] = self._factory(i)
        return m

    def build_ahead(self) -> bool:
        """Build the lowest-indexed model not built yet; False when all are built."""
        while self.next_unbuilt < self._n and self._built[self.next_unbuilt] is not None:
            self.next_unbuilt += 1
        if self.next_unbuilt >= self._n:
            return False
        self[self.next_unbuilt]
        return True


def _new_stream(device):
    """A HIP stream from torch's pool (None without a device: the CPU test doubles)."""
    return torch.cuda.Stream(device=device) if torch.cuda.is_available() else None


def _stream_ctx(stream):
    return torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()


def _resolve_model(closure):
    if hasattr(closure, "_gpx_loss_and_grad"):  # closures that carry their data (SVGP)
        return closure
    m = getattr(closure, "_gpx_model", None)
    if m is None:
        m = getattr(closure, "__self__", None)
    if m is None or not hasattr(m, "loss_and_grad_unconstrained"):
        raise TypeError("closure must be a portfoliooptgp_amd model's training_loss "
                        "(or training_loss_closure()); gradients come from the GPU engine, "
                        "there is no autodiff of arbitrary Python closures")
    return m


def _not_pd_policy(on_not_pd: str):
    """GPflow/TF raise when the Cholesky of K + σn²I fails (tf.linalg.cholesky →
    InvalidArgumentError inside Scipy.minimize); on_not_pd="inf" instead reports an infinite
    loss (zero gradient) for that point, so L-BFGS-B's line search backs off and the fit goes on.
    The same holds for a point whose constrained hyperparameters left (0, inf) (softplus
    underflow after an extreme step: InvalidParameterError)."""
    if on_not_pd not in ("raise", "inf"):
        raise ValueError("on_not_pd must be 'raise' (GPflow's behaviour) or 'inf'")
    return on_not_pd == "inf"


def _guarded(fn, as_inf: bool):
    if not as_inf:
        return fn

    def g(x):
        try:
            return fn(x)
        except (N.NotPositiveDefiniteError, N.InvalidParameterError):
            return float("inf"), np.zeros_like(np.asarray(x, dtype=np.float64))
    return g


def _pack(variables) -> np.ndarray:
    if all(type(v) is UnconstrainedVariable for v in variables):  # scalar parameters: their u as stored
        return np.array([v._param._u for v in variables], dtype=np.float64)
    return np.concatenate([np.atleast_1d(v.numpy()).ravel() for v in variables]).astype(np.float64)


def _unpack(variables, x) -> None:
    x = np.asarray(x, dtype=np.float64)
    if all(type(v) is UnconstrainedVariable for v in variables) and x.shape == (len(variables),):
        for v, u in zip(variables, x.tolist()):  # (UnconstrainedVariable.assign: the same float)
            v._param._u = u
        return
    o = 0
    for v in variables:
        shape = tuple(v.shape)
        n = int(np.prod(shape)) if shape else 1
        v.assign(x[o] if not shape else x[o:o + n].reshape(shape))
        o += n


_TPC = None


def _single_thread_blas():
    """Context in which BLAS/LAPACK run single-threaded. scipy's L-BFGS-B calls them on
    n-vectors and m×m matrices; a multi-threaded OpenBLAS hands each of those tiny calls to its
    thread pool, which costs ≈10× the call itself (423 → 41 µs per step measured)."""
    global _TPC
    try:
        if _TPC is None:  # the BLAS libraries' thread controls, found once
            from threadpoolctl import ThreadpoolController
            _TPC = ThreadpoolController().select(user_api="blas").lib_controllers
        return _BlasThreads(_TPC)
    except Exception:  # pragma: no cover - threadpoolctl missing
        return contextlib.nullcontext()


class _BlasThreads:
    """set_num_threads(1) on each BLAS library while any fit steps (direct calls, not a fresh
    threadpool_limits scan: this wraps every single-model minimize). Process-wide and counted:
    with fits stepping concurrently (threaded driver, user threads) the first context to enter
    sets one thread and the last to exit restores the previous counts, so one fit finishing
    does not hand the others a multi-threaded BLAS mid-run."""

    _lock = threading.Lock()
    _active = 0
    _prev: list = []

    def __init__(self, libs):
        self.libs = libs

    def __enter__(self):
        cls = _BlasThreads
        with cls._lock:
            if cls._active == 0:
                cls._prev = []
                for lib in self.libs:
                    n = lib.get_num_threads()
                    cls._prev.append((lib, n))
                    if n != 1:
                        lib.set_num_threads(1)
            cls._active += 1
        return self

    def __exit__(self, *exc):
        cls = _BlasThreads
        with cls._lock:
            cls._active -= 1
            if cls._active == 0:
                for lib, n in cls._prev:
                    if n != 1:
                        lib.set_num_threads(n)
                cls._prev = []
        return False


class Scipy:
    def minimize(self, closure: Callable, variables: Sequence, method: str = "L-BFGS-B",
                 step_callback=None, compile: bool = True, allow_unused_variables: bool = False,
                 tf_fun_args=None, track_loss_history: bool = False, on_not_pd: str = "raise",
                 **scipy_kwargs):
        as_inf = _not_pd_policy(on_not_pd)
        if not callable(closure):
            raise TypeError("The 'closure' argument is expected to be a callable object.")
        variables = tuple(variables)
        if not variables:
            raise ValueError("The 'variables' argument is expected to only contain Variable instances")
        model = _resolve_model(closure)
        history: List[float] = []

        lg = getattr(model, "_gpx_loss_and_grad", None) or model.loss_and_grad_unconstrained

        def func(x):
            _unpack(variables, x)
            loss, g = lg(variables)
            if track_loss_history:
                history.append(loss)
            return loss, g

        callback = None
        if step_callback is not None:
            def callback(xk, *args):
                step_callback(len(history), variables, [np.asarray(v) for v in xk])
        x0 = _pack(variables)
        if (step_callback is None and lbfgsb.supports(method, scipy_kwargs) and not _THREADED
                and os.environ.get("GPX_SOLO_STEPPER", "1") != "0"):
            # the drop-in pattern (GPR/model_trainer.py:18-19, one model at a time): scipy's own
            # setulb driven by the C++ loop (lbfgsb.BatchStepper, one slot) instead of
            # scipy.optimize.minimize's Python loop — the same setulb calls in the same order, so
            # the same trajectory and OptimizeResult bit for bit (tests/test_stream_driver.py),
            # at a few µs of host time per evaluation instead of tens
            opts = scipy_kwargs.get("options") or {}
            st = (lbfgsb.BatchStepper(1, len(x0), opts).start(0, x0) if lbfgsb.BatchStepper.NATIVE
                  else lbfgsb.LbfgsbStepper(x0, opts))
            fg = _guarded(func, as_inf)
            with _single_thread_blas():
                while not st.done:
                    loss, g = fg(st.x)
                    st.tell(loss, g)
            res = st.result()
            _unpack(variables, res.x)
            if track_loss_history:
                res.loss_history = history
            return res
        with _single_thread_blas():
            res = scipy.optimize.minimize(_guarded(func, as_inf), x0, jac=True, method=method,
                                          callback=callback, **scipy_kwargs)
        _unpack(variables, res.x)
        if track_loss_history:
            res.loss_history = history
        return res

    def minimize_batch(self, models: Sequence, method: str = "L-BFGS-B",
                       engine: Optional[Engine] = None, device: Optional[int] = None,
                       on_not_pd: str = "raise", **scipy_kwargs) -> List[scipy.optimize.OptimizeResult]:
        """Fit several GPR models concurrently (their trainable_variables), lock-step batched."""
        as_inf = _not_pd_policy(on_not_pd)
        models = list(models)
        if not models:
            return []
        if engine is None:
            engine = Engine([m.data[0] for m in models], [m.data[1] for m in models],
                            [compile_spec(m.kernel, m.data[0].shape[1]) for m in models],
                            device=device if device is not None else models[0].device)
        for i, m in enumerate(models):
            m._attach(engine, i)
        if lbfgsb.supports(method, scipy_kwargs) and not _THREADED:
            drv = _SteppedDriver(models, [engine], 1, scipy_kwargs.get("options") or {}, as_inf,
                                 models[0].data[0].shape[1], fixed=True)
            drv.run()
            self.last_trace = drv.trace
            self.last_stats = drv.stats
            for e in drv.errors:
                if e is not None:
                    raise e
            return drv.results
        step = _LockstepEvaluator(engine, models)
        results: List[Optional[scipy.optimize.OptimizeResult]] = [None] * len(models)
        errors: List[Optional[BaseException]] = [None] * len(models)

        def worker(i: int):
            try:
                m = models[i]
                variables = m.trainable_variables
                if not variables:
                    raise ValueError("model has no trainable variables")

                def func(x):
                    _unpack(variables, x)
                    return step.request(i, variables)

                res = scipy.optimize.minimize(_guarded(func, as_inf), _pack(variables), jac=True,
                                              method=method, **scipy_kwargs)
                _unpack(variables, res.x)
                results[i] = res
            except BaseException as e:  # re-raised on the caller's thread
                errors[i] = e
            finally:
                step.finish(i)

        threads = [threading.Thread(target=worker, args=(i,), daemon=True) for i in range(len(models))]
        for t in threads:
            t.start()
        step.serve()
        for t in threads:
            t.join()
        for e in errors:
            if e is not None:
                raise e
        return results  # type: ignore[return-value]


    def minimize_stream(self, models: Sequence, width: int, method: str = "L-BFGS-B",
                        device: Optional[int] = None, predict_train: bool = False,
                        engine=None, groups: int = 1,
                        predict_inputs: Optional[Sequence] = None, on_not_pd: str = "raise",
                        wide_group: bool = False, admission=None, **scipy_kwargs):
        """Continuous batching: fit many models through ``width`` resident device slots.

        Every model still runs its own unmodified scipy L-BFGS-B; at most ``width`` are
        resident, and a slot is refilled from the queue as soon as its fit has converged, so
        the batched evaluations stay wide until the queue drains (a lock-step batch shrinks
        as its fits finish). With ``predict_train`` each model's predict_f at its training
        inputs (or at ``predict_inputs[i]`` when given) runs before its slot is released.

        ``groups`` > 1 splits the slots into that many independent device batches, each its
        own engine (gpx_batch) evaluated from its own server thread on its own HIP stream:
        the groups' evaluations run concurrently on the GPU (one group's latency-bound
        phases overlap another's large GEMMs) and one group's host work overlaps the others'
        device work. ``engine`` may be one Engine (groups then alternate on it) or a list of
        ``groups`` Engines. ``wide_group``: the last engine only evaluates points whose
        kernel band is wider than one 64-block (or dense) and the others only narrow ones; a
        fit moves between them (its series rebound, its L-BFGS-B state kept) when its next
        point changes class, so the narrow batches' calls never wait for the slower wide
        sweeps. ``admission``: a DeviceAdmission (or any object with acquire/release) shared
        by the processes that fit through the same GPU; each evaluation call holds one of its
        places from just before its submit until its results are back (see DeviceAdmission).
        Returns (results, predictions|None); models are detached afterwards.
        """
        as_inf = _not_pd_policy(on_not_pd)
        lazy = isinstance(models, ModelStream)
        if not lazy:
            models = list(models)
        if len(models) == 0:
            return [], ([] if predict_train else None)
        width = max(1, min(int(width), len(models)))
        groups = max(1, min(int(groups), width))
        if lazy:  # slot shapes from the stream's declaration, not from building every model
            D, nmax = models.input_dim, models.max_points
        else:
            D = models[0].data[0].shape[1]
            if any(m.data[0].shape[1] != D for m in models):
                raise ValueError("all models must have the same input dimension")
            nmax = max(m.data[0].shape[0] for m in models)
        if device is not None:
            dev = device
        else:
            dev = models.device if lazy and models.device is not None else models[0].device
        if engine is None:
            # slot shapes sized for the largest problem; one engine per group
            per = -(-width // groups)
            engines = []
            for g in range(groups):
                seed = models[g * per:(g + 1) * per] or models[:1]
                engines.append(Engine([np.zeros((nmax, D)) for _ in seed], [np.zeros((nmax, 1)) for _ in seed],
                                      [compile_spec(m.kernel, D) for m in seed], device=dev))
        else:
            engines = list(engine) if isinstance(engine, (list, tuple)) else [engine]
        if predict_inputs is not None and len(predict_inputs) != len(models):
            raise ValueError("predict_inputs needs one Xnew per model")
        if lbfgsb.supports(method, scipy_kwargs) and not _THREADED:
            drv = _SteppedDriver(models, engines, groups, scipy_kwargs.get("options") or {}, as_inf, D,
                                 predict_train=predict_train or predict_inputs is not None,
                                 predict_inputs=predict_inputs, width=width, wide_group=wide_group,
                                 admission=admission)
            t_run = time.perf_counter()
            drv.run()
            if drv.stats is not None:  # the whole run, phases or not (the gaps are the loop itself)
                drv.stats["run_total"] = time.perf_counter() - t_run
            self.last_trace = drv.trace
            self.last_stats = drv.stats
            for e in drv.errors:
                if e is not None:
                    raise e
            return drv.results, drv.preds
        step = _LockstepEvaluator(engines, None, total=len(models), groups=groups)
        results = [None] * len(models)
        if predict_inputs is not None:
            predict_train = True
            if len(predict_inputs) != len(models):
                raise ValueError("predict_inputs needs one Xnew per model")
        preds = [None] * len(models) if predict_train else None
        errors: List[Optional[BaseException]] = [None] * len(models)

        order: "queue.Queue[int]" = queue.Queue()
        for i in range(len(models)):
            order.put(i)

        def slot_worker(slot: int):
            # one host thread per device slot (not per model): it fits the queued models one
            # after another in its slot, so the thread count is the slot count however many
            # models are streamed
            while True:
                try:
                    i = order.get_nowait()
                except queue.Empty:
                    return
                fit_in_slot(i, slot)

        def fit_in_slot(i: int, slot: int):
            m = models[i]
            eng, local, lock = step.slot_engine(slot)
            try:
                # the slot is idle, so loading the new problem needs no engine lock: its copies
                # run on a side stream while the group's evaluation of other slots proceeds
                with _stream_ctx(_new_stream(eng.device)):
                    eng.rebind(local, m.data[0], m.data[1], compile_spec(m.kernel, D))
                m._attach(eng, local)
                step.bind(slot, m)
                variables = m.trainable_variables
                if not variables:
                    raise ValueError("model has no trainable variables")

                def func(x):
                    _unpack(variables, x)
                    return step.request(slot, variables)

                res = scipy.optimize.minimize(_guarded(func, as_inf), _pack(variables), jac=True,
                                              method=method, **scipy_kwargs)
                _unpack(variables, res.x)
                results[i] = res
                if predict_train:
                    step.unbind(slot)  # leave the lock-step set before the predict call
                    xp = m.data[0] if predict_inputs is None else predict_inputs[i]
                    # executed by the slot's server thread between its device calls
                    mu, var = step.predict(slot, m.theta_row(), xp)
                    preds[i] = (mu.reshape(-1, 1), var.reshape(-1, 1))
            except BaseException as e:
                errors[i] = e
            finally:
                m._engine = None
                step.finish(slot)

        n_workers = min(step.n_slots, len(models))
        threads = [threading.Thread(target=slot_worker, args=(s,), daemon=True) for s in range(n_workers)]
        for t in threads:
            t.start()
        step.serve()
        for t in threads:
            t.join()
        self.last_trace = step.trace
        for e in errors:
            if e is not None:
                raise e
        return results, preds


class _LockstepEvaluator:
    """Barrier between the optimiser threads and the device: evaluates all pending points in
    one gpx_batch_lml_grad call once every running optimiser has posted one."""

    def __init__(self, engine, models, total: Optional[int] = None, groups: int = 1):
        # engine: one Engine (slots = its rows; groups alternate on it) or a list of Engines
        # (one per group; global slot s lives in engines[s % G] at row s // G)
        self.engines = list(engine) if isinstance(engine, (list, tuple)) else [engine]
        self.engine = self.engines[0]
        if len(self.engines) > 1:
            G = len(self.engines)
            self.n_slots = G * min(e.B for e in self.engines)
            self.locks = [threading.Lock() for _ in self.engines]
            self.streams = [_new_stream(e.device) for e in self.engines]
        else:
            self.n_slots = self.engine.B
            self.locks = [threading.Lock()]
            self.streams = [None]
        if models is None:
            models = [None] * self.n_slots
        self.models = list(models)
        # slots are split into `groups` (slot % groups); each group has its own server thread
        # and device calls, so one group's host-side work (scipy steps, result unpacking)
        # overlaps the other group's device evaluation
        self.groups = len(self.engines) if len(self.engines) > 1 else max(1, int(groups))
        self.cv = threading.Condition()
        self.lib_lock = self.locks[0]
        if total is None:  # fixed lock-step batch: every slot runs from the start
            self.running = set(range(len(self.models)))
            self.remaining = len(self.models)
            self.initial = len(self.models)
        else:              # streaming: slots join via bind() and leave via finish()
            self.running = set()
            self.remaining = total
            self.initial = min(len(self.models), total)
        self.pending = {}
        self.results = {}
        self.ready_ev = {}  # slot -> threading.Event set when its result is posted
        self.rounds = 0
        # predict requests of finished fits, run by the slot's server thread between device
        # calls (no engine-lock wait behind a whole evaluation)
        self.admin = [[] for _ in range(self.groups)]
        # stagger: group g ≥ 1 starts its first device call g/G of a group-0 call after group 0's
        # first call returns, so the concurrent batches run out of phase (one batch's
        # latency-bound recursion levels under the other's large GEMMs); started in phase they
        # stay in phase
        self.rounds_g = [0] * self.groups
        self.first_call = threading.Event()
        self.first_call_s = 0.0
        # slots of the previous device call; only these (if still running) are waited for —
        # a fit bound since then joins whichever round it posts in time for, so rebinding a
        # slot never stalls the device
        self.last_batch = [None] * self.groups
        # GPX_TRACE_ROUNDS=1: (time, batch size) per device call, for bench diagnostics
        self.trace = [] if os.environ.get("GPX_TRACE_ROUNDS") else None

    def slot_engine(self, s: int):
        """(engine, row in that engine, its lock) of global slot s."""
        if len(self.engines) == 1:
            return self.engine, s, self.locks[0]
        G = len(self.engines)
        return self.engines[s % G], s // G, self.locks[s % G]

    def bind(self, slot: int, model):
        with self.cv:
            self.models[slot] = model
            self.running.add(slot)
            self.cv.notify_all()

    def unbind(self, slot: int):
        with self.cv:
            self.running.discard(slot)
            self.cv.notify_all()

    def _slot_event(self, i: int) -> threading.Event:
        ev = self.ready_ev.get(i)
        if ev is None:
            ev = self.ready_ev.setdefault(i, threading.Event())
        return ev

    def request(self, i: int, variables):
        # the optimiser thread waits on its own slot's event: the condition variable only
        # wakes the server threads (with hundreds of optimiser threads on one condition,
        # every notify_all woke them all)
        ev = self._slot_event(i)
        ev.clear()
        with self.cv:
            self.pending[i] = variables
            self.cv.notify_all()
        ev.wait()
        with self.cv:
            res = self.results.pop(i)
        if isinstance(res, BaseException):
            raise res
        return res

    def predict(self, slot: int, theta_row, Xnew):
        G = self.groups
        job = {"slot": slot, "theta": np.asarray(theta_row, dtype=np.float64), "x": Xnew, "out": None,
               "done": threading.Event()}
        with self.cv:
            self.admin[slot % G].append(job)
            self.cv.notify_all()
        job["done"].wait()
        if isinstance(job["out"], BaseException):
            raise job["out"]
        return job["out"]

    def _run_admin(self, g: int, eng, lock, multi: bool):
        with self.cv:
            jobs, self.admin[g] = self.admin[g], []
        G = self.groups
        for job in jobs:
            try:
                row = job["slot"] // G if multi else job["slot"]
                theta = np.ones((eng.B, N.GPX_THETA_STRIDE))
                theta[row] = job["theta"]
                with lock:
                    mu, var, _ = eng.predict([row], theta, [job["x"]], False)
                job["out"] = (mu[0], var[0])
            except BaseException as e:
                job["out"] = e
            job["done"].set()

    def finish(self, i: int):
        with self.cv:
            self.running.discard(i)
            self.remaining -= 1
            self.cv.notify_all()

    def _ready(self, g: int) -> bool:
        G = self.groups
        if not any(i % G == g for i in self.pending):
            return False
        run = {i for i in self.running if i % G == g}
        if self.last_batch[g] is None:  # first round: wait for the group's initial slots
            init = sum(1 for s in range(self.initial) if s % G == g)
            return len(run) >= min(init, self.remaining) and all(i in self.pending for i in run)
        return all(i in self.pending for i in self.last_batch[g] & run)

    def serve(self):
        if self.groups == 1:
            return self._serve(0)
        errs = []

        def run(g):
            try:
                self._serve(g)
            except BaseException as e:  # pragma: no cover - surfaced below
                errs.append(e)
        helpers = [threading.Thread(target=run, args=(g,), daemon=True) for g in range(1, self.groups)]
        for t in helpers:
            t.start()
        run(0)
        for t in helpers:
            t.join()
        if errs:
            raise errs[0]

    def _serve(self, g: int):
        # group 0 is served on the caller's thread: restore its current stream afterwards
        prev = torch.cuda.current_stream() if (len(self.engines) > 1 and self.streams[g] is not None) else None
        try:
            self._serve_loop(g)
        finally:
            if prev is not None:
                torch.cuda.set_stream(prev)
            if g == 0:
                self.first_call.set()

    def _serve_loop(self, g: int):
        G = self.groups
        multi = len(self.engines) > 1
        eng = self.engines[g] if multi else self.engine
        lock = self.locks[g] if multi else self.locks[0]
        if multi and self.streams[g] is not None:
            torch.cuda.set_stream(self.streams[g])  # this thread's device calls use stream g
        while True:
            with self.cv:
                while self.remaining > 0 and not self._ready(g) and not self.admin[g]:
                    self.cv.wait()
                if self.remaining <= 0 and not self.admin[g]:
                    return
                run_admin = bool(self.admin[g])
            if run_admin:
                self._run_admin(g, eng, lock, multi)
                continue
            with self.cv:
                if not self._ready(g):
                    continue
                batch = {i: self.pending.pop(i) for i in [i for i in self.pending if i % G == g]}
                self.last_batch[g] = set(batch)
            if multi and g > 0 and self.rounds_g[g] == 0:
                self.first_call.wait(timeout=10.0)
                time.sleep(self.first_call_s * g / G)
            active = sorted(batch)
            if self.trace is not None:
                self.trace.append((time.perf_counter(), len(active)))
            t_call = time.perf_counter()
            rows = [i // G for i in active] if multi else active
            theta = np.ones((eng.B, N.GPX_THETA_STRIDE))
            for i, r in zip(active, rows):
                theta[r] = self.models[i].theta_row()
            out = {}
            try:
                with lock:
                    lml, grad, info = eng.lml_grad(rows, theta)
                for i, r in zip(active, rows):
                    if info[r] == N.INFO_BAD_THETA:
                        out[i] = N.InvalidParameterError(
                            f"model {i}: hyperparameters out of (0, inf): {theta[r, :eng.n_params[r] + 1]}")
                    elif info[r] != 0:
                        out[i] = N.NotPositiveDefiniteError(
                            f"Cholesky decomposition was not successful (model {i}, pivot "
                            f"{int(info[r])}): K + noise I is not positive definite", info[r])
                    else:
                        out[i] = self.models[i].loss_and_grad_unconstrained(
                            batch[i], lml=lml[r], grad_theta=grad[r])
            except BaseException as e:
                for i in active:
                    out[i] = e
            if g == 0 and self.rounds_g[0] == 0:
                self.first_call_s = time.perf_counter() - t_call
                self.first_call.set()
            self.rounds_g[g] += 1
            with self.cv:
                self.rounds += 1
                self.results.update(out)
                self.cv.notify_all()
            for i in out:
                self._slot_event(i).set()


class DeviceAdmission:
    """Admission control for several host processes that evaluate batches on ONE GPU: at most
    ``places`` evaluation calls are on the device at a time; a process takes a place just before
    its submit and gives it back when its results are home (Scipy.minimize_stream(admission=)).

    Why: each process alternates a device call (its ~1000 problems, one wavefront each) and a
    host phase (its fits' L-BFGS-B steps). The GPU serves concurrent calls interleaved, so
    calls submitted together also finish together and their processes then step on the host at
    the same time, leaving the GPU idle ("convoys": the band16 wave trace of round 4 showed
    fewer than 256 of the 2048 sweep places filled for 30 % of the run). With a few places the
    device serves the calls nearly first-come first-served: they complete one after another,
    so the host phases interleave with the other processes' device work.

    A pipelined driver (several device batches from one host thread) holds ONE place while any
    of its calls is in flight, so a process never waits for a place while holding one.

    Create it in the parent before the helper processes are spawned (a multiprocessing
    semaphore crosses a spawn only as a Process argument)."""

    def __init__(self, places: int, ctx=None):
        import multiprocessing as mp
        if int(places) < 1:
            raise ValueError("DeviceAdmission needs at least one place")
        self.places = int(places)
        self._sem = (ctx or mp.get_context("spawn")).BoundedSemaphore(self.places)

    def acquire(self):
        self._sem.acquire()

    def release(self):
        self._sem.release()


class _SteppedDriver:
    """Single-threaded-per-group fitting with reverse-communication L-BFGS-B (lbfgsb.py).

    Device slots are split into groups; each group has (engine, rows, lock) and ONE host
    thread (group 0: the caller's) that loops: refill idle rows from the shared queue, evaluate
    every active fit's requested point in one ``lml_grad`` call, pass each fit its (loss, grad),
    and predict + release the fits that finished. Per-fit trajectories are exactly scipy's
    (same setulb calls); there are no per-fit threads, events or condition variables, so the
    host cost of a round is just the fits' L-BFGS-B steps. ``fixed=True`` (minimize_batch):
    model i stays in row i of the single engine, nothing is rebound."""

    def __init__(self, models, engines, groups: int, options: dict, as_inf: bool, D: int,
                 predict_train: bool = False, predict_inputs=None, width: Optional[int] = None,
                 fixed: bool = False, wide_group: bool = False, admission=None):
        self.models, self.options, self.as_inf, self.D = models, options, as_inf, D
        self.admission = admission
        self.predict_train, self.predict_inputs, self.fixed = predict_train, predict_inputs, fixed
        G = max(1, groups)
        # group g: rows of its engine (one engine per group, or one engine split row-wise)
        if len(engines) > 1:
            G = len(engines)
            # every row of every engine is a slot (the last engine of a ceil split may be
            # smaller); the width cap below trims the total
            self.groups = [(engines[g], list(range(engines[g].B)), threading.Lock(),
                            _new_stream(engines[g].device)) for g in range(G)]
        else:
            e = engines[0]
            lock = threading.Lock()
            # (a stream of its own for one group too: on the caller's default stream a predict is
            # synchronous — gpx_batch_predict_train returns early only on an explicit stream — and
            # with deferred slow parts in the stream that wait is the slow part's whole duration)
            own = G > 1 or os.environ.get("GPX_DRIVER_CALLER_STREAM", "0") != "1"
            self.groups = [(e, list(range(g, e.B, G)), lock, _new_stream(e.device) if own else None)
                           for g in range(G)]
        if width is not None:  # at most `width` slots in total, dealt round-robin over groups
            keep = [[] for _ in self.groups]
            flat = [(g, r) for k in range(max(len(x[1]) for x in self.groups))
                    for g, x in enumerate(self.groups) if k < len(x[1]) for r in [x[1][k]]]
            for g, r in flat[:width]:
                keep[g].append(r)
            self.groups = [(e, keep[g], lk, s) for g, (e, _, lk, s) in enumerate(self.groups)]
        self.queue = list(range(len(models)))
        self.qlock = threading.Lock()
        self.results = [None] * len(models)
        self.preds = [None] * len(models) if predict_train else None
        self.errors: List[Optional[BaseException]] = [None] * len(models)
        self.trace = [] if os.environ.get("GPX_TRACE_ROUNDS") else None
        self.first_call = threading.Event()
        self.first_call_s = 0.0
        self._theta = {}  # id(engine) -> [B, 16] θ rows (one array per engine, slots disjoint)
        # GPX_DRIVER_STATS=1: wall time per phase (bind, theta, device call, steps, finish) summed
        # over the groups' threads, in Scipy().last_stats
        self.stats = {} if os.environ.get("GPX_DRIVER_STATS") else None
        # wide_group: the last device batch takes the evaluations whose band is wider than one
        # 64-block (or dense): a fit is moved between batches (rebind of its series, stepper
        # state kept) when its next point changes class and the other side has a free slot, so
        # the narrow batches' calls are not held up by the slower wide sweeps
        self.wide = (wide_group and not fixed and len(self.groups) > 1
                     and all(hasattr(e, "band_width") or hasattr(e, "band_class") for e, _, _, _ in self.groups))
        self.moves = 0
        self._narrow_q = int(os.environ.get("GPX_NARROW_Q", "3"))
        # GPX_HOLD_WIDE="Q:H" (or Q/H; default 6:3, 0 = off): on a batch with deferred completion,
        # a fit whose next point takes the band16 sweeps Q or more 16-blocks wide is submitted only
        # every H-th round of its batch (held, its point unchanged, in the others), so those rare,
        # long sweeps (one per SIMD, 7-8 ms) lengthen the deferred part's wide launch in one round
        # of H instead of in most rounds — the deferred parts follow each other on one stream, so
        # their length is what deferred fits wait (+2 % on the bench, profiles/r06_ab.md).
        # Scheduling only: each fit's evaluations, and so its trajectory, are the same bits.
        hq = os.environ.get("GPX_HOLD_WIDE", "6:3").replace("/", ":").split(":")
        self._hold_q = int(hq[0] or 0)
        self._hold_every = max(1, int(hq[1])) if len(hq) > 1 else 2
        self.held = 0
        # the fits' L-BFGS-B loops advanced a round at a time by the C++ loop around scipy's
        # setulb (lbfgsb.BatchStepper; GPX_NATIVE_LBFGSB=0: the Python stepper per fit). Not with
        # wide-group routing, which moves a fit's loop state between batches
        self.native = (lbfgsb.BatchStepper.NATIVE and not self.wide
                       and os.environ.get("GPX_NATIVE_LBFGSB", "1") != "0")

    def _next(self) -> Optional[int]:
        with self.qlock:
            return self.queue.pop(0) if self.queue else None

    def run(self):
        # scipy's L-BFGS-B calls BLAS/LAPACK on n-vectors and m×m matrices; a multi-threaded
        # OpenBLAS hands each of those tiny calls to its thread pool (≈10× the cost of the call
        # itself on this host), so the fits' host steps run with single-threaded BLAS
        # the cyclic garbage collector's full passes over a heap of thousands of live models
        # stall the single host thread for milliseconds at a time; the driver's own garbage is
        # acyclic (refcounting frees it), so the collector is paused for the run
        gc_on = gc.isenabled() and os.environ.get("GPX_DRIVER_GC", "0") != "1"
        if gc_on:
            gc.disable()
        try:
            with _single_thread_blas():
                self._run_all()
            # predictions from cached factors return without waiting for the device (in their
            # group stream's order); the caller reads them on its own stream
            # (every device the groups' engines live on, not only the first group's)
            if self.predict_train and torch.cuda.is_available():
                for dev in sorted({int(e.device) for e, _, _, _ in self.groups}):
                    torch.cuda.synchronize(dev)
        finally:
            if gc_on:
                gc.enable()

    def _run_all(self):
        G = len(self.groups)
        errs = []
        # the groups' host work shares the GIL: a thread whose device call has returned must not
        # wait out another group's whole 5 ms switch interval before stepping its fits
        # several device batches: one host thread submits and completes their evaluations in
        # turn (GPX_PIPELINE=0: one thread per batch instead)
        # (only when every group has an engine of its own: the groups of ONE engine split
        # row-wise would each submit on the same batch, which holds one pending evaluation)
        if (G > 1 and os.environ.get("GPX_PIPELINE", "1") != "0"
                and len({id(e) for e, _, _, _ in self.groups}) == G
                and all(hasattr(e, "lml_grad_submit") for e, _, _, _ in self.groups)):
            try:
                self._pipeline()
            finally:
                self.first_call.set()
            return
        self.wide = False  # class routing needs the one-thread pipeline
        self._run_groups(G, errs)
        if errs:
            raise errs[0]

    def _run_groups(self, G, errs):

        def run_group(g):
            try:
                self._serve(g)
            except BaseException as e:  # pragma: no cover - surfaced below
                errs.append(e)
            finally:
                if g == 0:
                    self.first_call.set()
        helpers = [threading.Thread(target=run_group, args=(g,), daemon=True) for g in range(1, G)]
        for t in helpers:
            t.start()
        run_group(0)
        for t in helpers:
            t.join()

    def _serve(self, g: int):
        eng, rows, lock, stream = self.groups[g]
        if stream is None:
            return self._loop(g, eng, rows, lock)
        prev = torch.cuda.current_stream()
        torch.cuda.set_stream(stream)  # this group's device calls use its own stream
        try:
            return self._loop(g, eng, rows, lock)
        finally:
            torch.cuda.set_stream(prev)

    def _bind(self, i: int, eng, row: int, lock, gs=None):
        m = self.models[i]
        if not self.fixed:
            t0 = time.perf_counter()
            # (the model compiled its kernel's spec for its own input width at construction)
            spec = m._spec if (getattr(m, "_spec", None) is not None and m.data[0].shape[-1] == self.D) \
                else compile_spec(m.kernel, self.D)
            with lock:
                eng.rebind(row, m.data[0], m.data[1], spec)
            if self.stats is not None:
                self.stats["bind_rebind"] = self.stats.get("bind_rebind", 0.0) + (time.perf_counter() - t0)
            m._attach(eng, row)
        variables = m.trainable_variables
        if not variables:
            raise ValueError("model has no trainable variables")
        cols, lower = m.theta_layout(variables)
        # the slot's θ row: fixed parameters now, the trainable columns rewritten every round
        self._theta_of(eng)[row] = m.theta_row()
        x0 = _pack(variables)
        native = gs is not None and self.native
        st = gs.batch(self, len(x0)).start(row, x0) if native else lbfgsb.LbfgsbStepper(x0, self.options)
        return {"i": i, "m": m, "v": variables, "st": st, "native": native,
                "cols": cols, "lower": lower, "key": (len(cols), cols.tobytes(), lower.tobytes())}

    def _theta_of(self, eng) -> np.ndarray:
        th = self._theta.get(id(eng))
        if th is None:
            th = self._theta[id(eng)] = np.ones((eng.B, N.GPX_THETA_STRIDE))
        return th

    class _Group:
        """One device batch's host-side state: its slots, active fits and current request."""

        def __init__(self, drv, g, eng, rows, lock, stream):
            self.g, self.eng, self.lock, self.stream = g, eng, lock, stream
            self.free = list(rows) if not drv.fixed else []
            self.active = {}
            self.batches = {}   # P -> lbfgsb.BatchStepper over the engine's rows (drv.native)
            self.reeval = set()  # rows held for one more evaluation at their result's x (_finish)
            if drv.fixed:
                for r in rows:
                    if r < len(drv.models):
                        try:
                            self.active[r] = drv._bind(r, eng, r, lock, self)
                        except BaseException as e:
                            drv.errors[r] = e
            self.theta = drv._theta_of(eng)
            # rows whose evaluation the engine deferred (info INFO_DEFERRED, Engine.set_deferred):
            # row -> (P, the requested point, layout columns), stepped when a later complete
            # (or a drain) delivers their result
            self.pending = {}
            self.wide = drv.wide and g == len(drv.groups) - 1
            self.n_calls = 0
            self.act = self.packs = None
            self.t_call = 0.0

        def batch(self, drv, P: int):
            b = self.batches.get(P)
            if b is None:
                b = self.batches[P] = lbfgsb.BatchStepper(self.eng.B, P, drv.options)
            return b

    def _tick(self, key, t0):
        if self.stats is not None:
            self.stats[key] = self.stats.get(key, 0.0) + (time.perf_counter() - t0)

    def _prepare(self, gs) -> bool:
        """Fill free slots from the queue, then the θ rows of every active fit's requested
        point. False when the group has nothing left to evaluate."""
        clk = time.perf_counter
        t0 = clk()
        while gs.free and not gs.wide:
            i = self._next()
            if i is None:
                break
            r = gs.free.pop(0)
            try:
                gs.active[r] = self._bind(i, gs.eng, r, gs.lock, gs)
            except BaseException as e:
                self.errors[i] = e
                self.models[i]._engine = None
                gs.free.insert(0, r)
        if not gs.active:
            return False
        self._tick("bind", t0)
        t0 = clk()
        lib = N.load_library()
        active = gs.active
        # θ rows of every requested point in one native call per variable layout (the same
        # libm softplus as Parameter.value, so the values are those of the per-model path)
        for moved in (False, True):
            gs.act = sorted(r for r in active if r not in gs.pending) if gs.pending else sorted(active)
            layouts = {}
            for r in gs.act:
                layouts.setdefault(active[r]["key"], []).append(r)
            gs.packs = []
            for key, rs in layouts.items():
                s0 = active[rs[0]]
                P = key[0]
                R = np.asarray(rs, dtype=np.int32)
                if s0["native"]:
                    U = np.empty((len(rs), P))
                    gs.batches[P].gather(R, U)
                    for k in ([k for k, r in enumerate(rs) if r in gs.reeval] if gs.reeval else ()):
                        U[k] = active[rs[k]]["reeval"]
                else:
                    # a finished fit held for one more evaluation at its result's x (see _finish)
                    U = np.array([active[r]["st"].x if active[r].get("reeval") is None else active[r]["reeval"]
                                  for r in rs], dtype=np.float64).reshape(len(rs), P)
                if not moved:
                    lib.gpx_host_theta_rows(len(rs), P, U.ctypes.data, R.ctypes.data, s0["cols"].ctypes.data,
                                            s0["lower"].ctypes.data, gs.theta.ctypes.data)
                gs.packs.append((rs, P, U, R, s0["cols"]))
            if moved or not self.wide or not self._migrate(gs):
                break
        if (self._hold_q > 0 and len(gs.act) > 1 and gs.n_calls % self._hold_every
                and getattr(gs.eng, "deferral", -1) >= 0):
            self._hold(gs)
        self._tick("theta", t0)
        return bool(gs.act)

    def _hold(self, gs):
        """GPX_HOLD_WIDE: leave this round's rows of band16 width >= the hold width out of the
        call (never all of them); their θ rows and requested points stay for the next round."""
        cls_fn = getattr(gs.eng, "band_class", None)
        if cls_fn is None:
            return
        c = cls_fn(gs.act, gs.theta)
        hold = (c >= self._hold_q) & (c < 16)
        if not hold.any() or hold.all():
            return
        held = {r for r, h in zip(gs.act, hold) if h}
        gs.act = [r for r in gs.act if r not in held]
        packs = []
        for rs, P, U, R, cols in gs.packs:
            keep = np.fromiter((r not in held for r in rs), dtype=bool, count=len(rs))
            if keep.all():
                packs.append((rs, P, U, R, cols))
            elif keep.any():
                packs.append(([r for r, k in zip(rs, keep) if k], P, U[keep], R[keep], cols))
        gs.packs = packs
        self.held += len(held)

    def _wide_classes(self, gs):
        """Per active row of the group: True (wide), False (narrow) or None (not known yet).
        With band16 tables (Engine.band_class) the narrow class is the band16 sweeps of at
        most GPX_NARROW_Q 16-blocks (default 3: the bulk of C2's evaluations, ~1.3-1.5 ms per
        sweep); everything slower — the wider band16 sweeps (one wavefront per SIMD), the 64-row
        sweeps (73 KiB of LDS per workgroup: they wait for whole CUs under a band16 load) and the
        dense path — is wide, so a call of the narrow batch never waits for it. Without band16
        tables: band width <= 1 64-block is narrow."""
        cls_fn = getattr(gs.eng, "band_class", None)
        if cls_fn is not None:
            c = cls_fn(gs.act, gs.theta)
            nq = self._narrow_q
            # 1..15 band16 width (wide above nq); 16 + p: 64-row band without band16 tables (wide
            # above p = 1); 32 + p (64-row band despite band16 tables) and -1 (dense): wide;
            # -2: band tables not known yet (a rebind waiting for its gather)
            wide = np.where(c < 16, c > nq, np.where(c < 32, c - 16 > 1, True)) | (c == -1)
            return wide, c == -2
        p = gs.eng.band_width(gs.act, gs.theta)
        return (p > 1) | (p == -1), p == -2

    def _migrate(self, gs) -> bool:
        """Move the fits whose requested point belongs to the other class (_wide_classes) to a
        free slot of a batch of that class. A fit with no free slot on the other side is
        evaluated where it is. True if any moved."""
        moved = False
        wide, unknown = self._wide_classes(gs)
        cand = np.nonzero((wide != gs.wide) & ~unknown)[0]
        for k in cand:
            r, want_wide = gs.act[k], bool(wide[k])
            if want_wide:
                tg = self._gss[-1]
            else:
                tg = max((x for x in self._gss if not x.wide), key=lambda x: len(x.free))
            if not tg.free:
                continue
            st = gs.active.pop(r)
            gs.free.append(r)
            r2 = tg.free.pop(0)
            m = st["m"]
            with tg.lock:
                tg.eng.rebind(r2, m.data[0], m.data[1], compile_spec(m.kernel, self.D))
            m._attach(tg.eng, r2)
            tg.theta[r2] = m.theta_row()
            tg.active[r2] = st
            self.moves += 1
            moved = True
        return moved

    def _consume(self, gs, lml, grad, info, t_call_end):
        """Hand every fit its (loss, grad), predict + release the finished ones."""
        clk = time.perf_counter
        lib = N.load_library()
        eng, active = gs.eng, gs.active
        t0 = clk()
        gs.n_calls += 1
        done = []
        for rs, P, U, R, cols in gs.packs:
            loss = np.empty(len(rs))
            gu = np.empty((len(rs), P))
            lib.gpx_host_loss_grad_u(len(rs), P, U.ctypes.data, R.ctypes.data, cols.ctypes.data,
                                     lml.ctypes.data, grad.ctypes.data, loss.ctypes.data, gu.ctypes.data)
            rest = range(len(rs))
            if active[rs[0]]["native"]:
                rest = self._tell_native(gs, P, R, U, loss, gu, info, done)
            for k in rest:
                r = rs[k]
                if info[r] == N.INFO_DEFERRED:
                    gs.pending[r] = (P, U[k].copy(), cols)
                    continue
                self._take(gs, r, P, U[k], loss[k], gu[k], info[r], done)
        if gs.pending:
            # deferred rows of earlier calls that this complete (or drain) delivered: per variable
            # layout one native chain rule and one batched step, as for the call's own rows
            got = [r for r in gs.pending if info[r] != N.INFO_UNSET and info[r] != N.INFO_DEFERRED]
            lays = {}
            for r in got:
                P, u, cols = gs.pending.pop(r)
                ent = lays.setdefault((P, cols.tobytes()), (P, cols, [], []))
                ent[2].append(r)
                ent[3].append(u)
            for P, cols, rows, us in lays.values():
                R = np.asarray(rows, dtype=np.int32)
                U = np.array(us, dtype=np.float64).reshape(len(rows), P)
                loss = np.empty(len(rows))
                gu = np.empty((len(rows), P))
                lib.gpx_host_loss_grad_u(len(rows), P, U.ctypes.data, R.ctypes.data, cols.ctypes.data, lml.ctypes.data,
                                         grad.ctypes.data, loss.ctypes.data, gu.ctypes.data)
                rest = range(len(rows))
                if active[rows[0]]["native"]:
                    rest = self._tell_native(gs, P, R, U, loss, gu, info, done)
                for k in rest:
                    self._take(gs, rows[k], P, U[k], loss[k], gu[k], info[rows[k]], done)
        self._tick("steps", t0)
        t_steps = clk()
        held = self._finish(eng, gs.lock, active, done, gs)
        self._tick("finish", t_steps)
        if self.trace is not None:  # GPX_TRACE_ROUNDS: (group, call start, call end, steps end, finish end, n)
            self.trace.append((gs.g, gs.t_call, t_call_end, t_steps, clk(), len(gs.act)))
        if self.stats is not None:
            self.stats["rounds"] = self.stats.get("rounds", 0) + 1
            self.stats["fit_evals"] = self.stats.get("fit_evals", 0) + len(gs.act)
        for r, _ in done:
            if r in held:
                continue
            gs.reeval.discard(r)
            del active[r]
            if not self.fixed:
                gs.free.append(r)

    def _tell_native(self, gs, P, R, U, loss, gu, info, done):
        """The pack's ordinary rows (a result, no deferral, no pending re-evaluation) through one
        BatchStepper.tell; returns the pack positions left for _take."""
        normal = info[R] == 0
        if gs.reeval:
            normal &= ~np.isin(R, np.fromiter(gs.reeval, dtype=np.int32))
        idx = np.flatnonzero(normal)
        if len(idx) == 0:
            return range(len(R))
        whole = len(idx) == len(R)
        Rn = R if whole else np.ascontiguousarray(R[idx])
        d = np.zeros(len(idx), np.uint8)
        err = None
        try:
            gs.batches[P].tell(Rn, loss if whole else np.ascontiguousarray(loss[idx]),
                               gu if whole else np.ascontiguousarray(gu[idx]), d)
        except BaseException as e:  # a Python error inside setulb at the row flagged 2
            err = e
        active = gs.active
        for j in np.flatnonzero(d == 1):
            r = int(Rn[j])
            active[r]["last_u"] = U[idx[j]]
            done.append((r, True))
        rest = list(np.flatnonzero(~normal))
        if err is not None:
            bad = np.flatnonzero(d == 2)
            j0 = int(bad[0]) if len(bad) else len(idx)
            for j in bad:
                self.errors[active[int(Rn[j])]["i"]] = err
                done.append((int(Rn[j]), False))
            rest += [int(idx[j]) for j in range(j0 + 1, len(idx))]  # untouched by the failed call
        return rest

    def _take(self, gs, r, P, u, loss, gu, inf, done):
        """One fit's (loss, grad) at its requested point u: the L-BFGS-B step, or its failure;
        appends (row, ok) to done when the fit is finished."""
        s = gs.active[r]
        if s.get("reeval") is not None:
            # the extra evaluation at the result's x (its factor serves the predict)
            done.append((r, inf == 0))
            return
        s["last_u"] = u
        try:
            if inf != 0:
                if inf == N.INFO_BAD_THETA:
                    err = N.InvalidParameterError(
                        f"model {s['i']}: hyperparameters out of (0, inf): {gs.theta[r, :gs.eng.n_params[r] + 1]}")
                else:
                    err = N.NotPositiveDefiniteError(
                        f"Cholesky decomposition was not successful (model {s['i']}, pivot "
                        f"{int(inf)}): K + noise I is not positive definite", inf)
                if not self.as_inf:
                    raise err
                s["st"].tell(float("inf"), np.zeros(P))
            else:
                s["st"].tell(float(loss), gu)
        except BaseException as e:
            self.errors[s["i"]] = e
            done.append((r, False))
            return
        if s["st"].done:
            done.append((r, True))

    def _drain(self, gs) -> None:
        """Wait for the group's deferred evaluations and step their fits (nothing else to run)."""
        with gs.lock:
            lml, grad, info = gs.eng.deferred_wait()
        gs.packs = []
        self._consume(gs, lml, grad, info, time.perf_counter())

    def _loop(self, g: int, eng, rows, lock):
        G = len(self.groups)
        gs = self._Group(self, g, eng, rows, lock, None)
        while True:
            if not self._prepare(gs):
                if gs.pending:
                    self._drain(gs)
                    continue
                return
            if g > 0 and gs.n_calls == 0 and G > 1:
                # stagger: start g/G of a group-0 call after group 0's first call returns, so the
                # concurrent batches run out of phase (one's latency-bound recursion levels under
                # the other's large GEMMs); started in phase they stay in phase
                self.first_call.wait(timeout=10.0)
                time.sleep(self.first_call_s * g / G)
            adm = self.admission
            if adm is not None:
                t_a = time.perf_counter()
                adm.acquire()
                self._tick("admission_wait", t_a)
            gs.t_call = time.perf_counter()
            try:
                with lock:
                    lml, grad, info = eng.lml_grad(gs.act, gs.theta, wait_deferred=False)
            finally:
                if adm is not None:
                    adm.release()
            self._tick("device_call", gs.t_call)
            t_end = time.perf_counter()
            if g == 0 and gs.n_calls == 0:
                self.first_call_s = t_end - gs.t_call
                self.first_call.set()
            self._consume(gs, lml, grad, info, t_end)

    def _pipeline(self):
        """All groups from ONE host thread: each group's evaluation is submitted
        (Engine.lml_grad_submit, on the group's stream) and completed in turn, so a group's
        host work (steps, predicts, rebinds) overlaps the other groups' device work without
        the threads' GIL hand-offs."""
        gss = self._gss = [self._Group(self, g, e, rows, lk, stm)
                           for g, (e, rows, lk, stm) in enumerate(self.groups)]
        inflight = []

        # admission: this pipeline holds at most ONE place, from the submit that finds nothing of
        # it in flight to the complete that leaves nothing in flight — a place per group would let
        # one thread wait on the semaphore while holding places that only its own completes give
        # back (places < groups across the processes: every process waits for ever)
        adm = self.admission
        held = [False]

        def take():
            if adm is not None and not held[0]:
                t_a = time.perf_counter()
                adm.acquire()
                held[0] = True
                self._tick("admission_wait", t_a)

        def give():
            if adm is not None and held[0] and not inflight:
                adm.release()
                held[0] = False

        def submit(gs):
            if not self._prepare(gs):
                return False
            take()
            gs.t_call = time.perf_counter()
            try:
                with torch.cuda.stream(gs.stream) if gs.stream is not None else contextlib.nullcontext():
                    gs.eng.lml_grad_submit(gs.act, gs.theta)
            except BaseException:
                give()
                raise
            self._tick("submit", gs.t_call)
            return True

        def submit_idle():
            # groups that are not in flight (e.g. the wide batch before any fit moved in)
            for x in gss:
                if x not in inflight and x.active and submit(x):
                    inflight.append(x)
        # a ModelStream's models are built while this thread waits for the device
        build_ahead = getattr(self.models, "build_ahead", None)
        for gs in gss:
            if submit(gs):
                inflight.append(gs)

        def drain_idle():
            # a group with nothing left to submit but deferred rows in flight: wait for them
            for x in gss:
                while x not in inflight and x.pending:
                    with torch.cuda.stream(x.stream) if x.stream is not None else contextlib.nullcontext():
                        self._drain(x)
                        if submit(x):
                            inflight.append(x)
        drain_idle()
        while inflight:
            # complete whichever batch finishes first (the wide batch's calls are longer)
            t0 = time.perf_counter()
            gs = None
            while gs is None:
                for x in inflight:
                    ready = getattr(x.eng, "lml_grad_ready", None)
                    if ready is None or ready():
                        gs = x
                        break
                else:
                    if build_ahead is not None and build_ahead():
                        continue
                    build_ahead = None
                    if len(inflight) == 1:
                        gs = inflight[0]
                    else:
                        time.sleep(2e-5)
            inflight.remove(gs)
            self._tick("device_wait", t0)
            t1 = time.perf_counter()
            try:
                lml, grad, info = gs.eng.lml_grad_complete()
            finally:
                give()
            t_end = time.perf_counter()
            self._tick("complete", t1)
            with torch.cuda.stream(gs.stream) if gs.stream is not None else contextlib.nullcontext():
                self._consume(gs, lml, grad, info, t_end)
                if submit(gs):
                    inflight.append(gs)
            if self.wide:
                submit_idle()
            drain_idle()

    def _finish(self, eng, lock, active, done, gs=None):
        """Results of the finished fits and their predictions. Returns the rows held back for
        one more evaluation: predict at the training inputs reuses the factor of the fit's last
        evaluated point, which is the result's x unless L-BFGS-B returned an earlier point (its
        line search backed off); such a fit is evaluated once more at its result's x in the
        next batched round (banded and asynchronous, like any other evaluation) instead of being
        re-factorised alone by the predict call."""
        pred_rows, xs, held, refit = [], [], set(), []
        for r, ok in done:
            s = active[r]
            if ok:
                res = s.get("res") or s["st"].result()
                if (self.predict_train and self.predict_inputs is None and s.get("reeval") is None
                        and s.get("last_u") is not None and not np.array_equal(res.x, s["last_u"])):
                    s["res"] = res
                    s["reeval"] = np.array(res.x, dtype=np.float64)
                    held.add(r)
                    if gs is not None:
                        gs.reeval.add(r)
                    continue
                _unpack(s["v"], res.x)
                self.results[s["i"]] = res
                if self.predict_train:
                    pred_rows.append(r)
                    xs.append(s["m"].data[0] if self.predict_inputs is None else self.predict_inputs[s["i"]])
            elif s.get("reeval") is not None:
                # the extra evaluation failed: the result stands, the predict re-factorises
                res = s["res"]
                _unpack(s["v"], res.x)
                self.results[s["i"]] = res
                pred_rows.append(r)
                refit.append(r)
                xs.append(s["m"].data[0])
            elif not self.fixed:
                s["m"]._engine = None
        if pred_rows:
            if gs is not None:
                # the group's θ rows hold each finished fit's last evaluated point, which is its
                # result's x (else it was held for one more evaluation above): the native θ rows
                # are Parameter.value's bits, and exactly what the cached factor was computed at
                theta = gs.theta
                for r in refit:
                    theta[r] = active[r]["m"].theta_row()
            else:
                theta = np.ones((eng.B, N.GPX_THETA_STRIDE))
                for r in pred_rows:
                    theta[r] = active[r]["m"].theta_row()
            try:
                with lock:
                    if self.predict_inputs is None and hasattr(eng, "_predict_train"):
                        # predict_f at each fit's own training inputs (GPR/model_trainer.py:20):
                        # known here, so the engine's input comparison is skipped
                        mu, var, _ = eng._predict_train(np.asarray(pred_rows, dtype=np.int32), theta, False,
                                                        column=True)
                    else:
                        mu, var, _ = eng.predict(pred_rows, theta, xs, False)
                        mu = [t.reshape(-1, 1) for t in mu]
                        var = [t.reshape(-1, 1) for t in var]
                for k, r in enumerate(pred_rows):
                    self.preds[active[r]["i"]] = (mu[k], var[k])
            except BaseException as e:
                for r in pred_rows:
                    self.errors[active[r]["i"]] = e
        if not self.fixed:
            for r, ok in done:
                if r not in held and (ok or active[r].get("reeval") is not None):
                    active[r]["m"]._engine = None
        return held
