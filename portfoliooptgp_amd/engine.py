"""Device engine: a ``gpx_batch`` (include/gpx.h) over a list of GPR problems.

One engine holds the problems' X/Y resident in HBM ([B, N_max, D] / [B, N_max] fp64, ragged
problems padded, the padding handled exactly inside the kernels) plus the library's
factorisation workspace. Evaluations run on the caller's current torch stream.
"""
from __future__ import annotations

import ctypes
import os
import weakref
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import _native as N


def default_device() -> int:
    """The HIP device this process uses: GPX_DEVICE, else LOCAL_RANK (one process per GPU),
    else 0."""
    for var in ("GPX_DEVICE", "LOCAL_RANK"):
        v = os.environ.get(var)
        if v is not None:
            return int(v)
    return 0


def require_gpu(device: Optional[int] = None) -> int:
    device = default_device() if device is None else int(device)
    if not torch.cuda.is_available():
        raise N.GPXError("portfoliooptgp_amd needs a HIP device (MI355X / gfx950); none is visible. "
                         "There is no CPU fallback.")
    return device


def to_device_f64(a, device: int) -> torch.Tensor:
    if isinstance(a, torch.Tensor):
        t = a.detach()
    else:
        t = torch.as_tensor(np.asarray(a, dtype=np.float64))
    return t.to(device=f"cuda:{device}", dtype=torch.float64).contiguous()


def _host_f64(a) -> np.ndarray:
    """fp64 host array of a (a device tensor is copied down)."""
    if isinstance(a, torch.Tensor):
        return a.detach().to(device="cpu", dtype=torch.float64).numpy()
    return np.asarray(a, dtype=np.float64)


def _rows(x: torch.Tensor, D: int) -> torch.Tensor:
    """[M, D] view of prediction inputs (a 1-D input is one column; an empty one has D columns)."""
    if x.numel() == 0:
        return x if x.ndim == 2 else x.reshape(0, D)
    return x.reshape(x.shape[0], -1)


def screen_theta(act: np.ndarray, theta: np.ndarray, n_params: np.ndarray, info: np.ndarray) -> np.ndarray:
    """Active rows whose constrained θ (kernel parameters + σn²) are all finite and > 0; the
    others get info = INFO_BAD_THETA and stay out of the device call, so one fit whose softplus
    underflowed does not fail its whole batch (gpx_batch_lml_grad rejects the call otherwise)."""
    if np.isfinite(theta).all() and (theta > 0.0).all():  # the usual case, one pass
        return act
    ok = np.array([bool(np.all(np.isfinite(theta[b, : n_params[b] + 1]) & (theta[b, : n_params[b] + 1] > 0.0)))
                   for b in act], dtype=bool)
    if ok.all():
        return act
    info[act[~ok]] = N.INFO_BAD_THETA
    return np.ascontiguousarray(act[ok])


# Per-16-row-block bounding boxes ([ceil(n/16)][D][2]) of device-resident series (the band
# tables' input), kept per series so that rebinding the same series into a slot again
# (continuous batching refits the same assets step after step) skips the gather's box download
# and stream synchronise. Only series declared immutable take part (mark_immutable: bench.py's
# resident series, data.load_batch's views): a tensor written through .data, DLPack or native
# code keeps its version counter, and stale boxes would give band tables that are too narrow.
# Entries live as long as the tensor (a weakref finalizer drops them), keyed by id() and checked
# against the tensor's storage pointer, shape and strides.
_IMMUTABLE = {}   # id(x) -> [weakref(x), (data_ptr, shape, stride), boxes or None]


def mark_immutable(*tensors) -> None:
    """Declare device series whose contents will not change while they are in use: their band
    tables' boxes are computed once and reused by every later rebind of the same tensor.
    Writing to a marked tensor afterwards is a contract violation (results could be wrong)."""
    import weakref
    for x in tensors:
        if not (isinstance(x, torch.Tensor) and x.is_cuda):
            continue
        k = id(x)
        sig = (x.data_ptr(), tuple(x.shape), tuple(x.stride()))
        ent = _IMMUTABLE.get(k)
        if ent is not None and ent[0]() is x and ent[1] == sig:
            continue
        _IMMUTABLE[k] = [weakref.ref(x), sig, None]
        weakref.finalize(x, _IMMUTABLE.pop, k, None)


def _immutable_entry(x: torch.Tensor):
    """The cache entry of a marked tensor whose storage is still the marked one, else None."""
    if os.environ.get("GPX_BOX_CACHE", "1") == "0":
        return None
    ent = _IMMUTABLE.get(id(x))
    if ent is None or ent[0]() is not x:
        return None
    if ent[1] != (x.data_ptr(), tuple(x.shape), tuple(x.stride())):
        return None
    return ent


# The banded route every new engine takes (include/gpx.h gpx_batch_set_band_route): "sweeps"
# (default), "bcr" or "auto". A property of the engine, never of a call, so a fit's bits do not
# depend on which other fits share its calls; GPX_BAND_ROUTE sets the process default.
_DEFAULT_BAND_ROUTE = os.environ.get("GPX_BAND_ROUTE", "sweeps")


def set_default_band_route(route: str) -> str:
    """Set the banded route of engines created from now on ("sweeps": the one-wavefront band16
    sweeps, throughput; "bcr": block cyclic reduction, latency for calls of a few problems;
    "auto": BCR for calls of at most 32 band16 problems — call-size dependent bits). Returns the
    previous default. Engines already created keep theirs (Engine.set_band_route)."""
    global _DEFAULT_BAND_ROUTE
    if route not in N.BAND_ROUTES:
        raise ValueError(f"band route must be one of {sorted(N.BAND_ROUTES)}")
    prev, _DEFAULT_BAND_ROUTE = _DEFAULT_BAND_ROUTE, route
    return prev


class Engine:
    def __init__(self, Xs: Sequence, Ys: Sequence, specs: Sequence[N.GpxKernelSpec],
                 device: Optional[int] = None, band_storage: bool = False, band_route: Optional[str] = None):
        """B problem slots (gpx_batch). ``band_storage``: the workspace keeps only the 64-block
        band of width 2 (gpx_batch_create_banded: 25 MiB per slot at N = 4096 instead of
        384 MiB), for many resident slots of banded fits; anything else runs on the batch's
        dense fallback slots. Same results either way. ``band_route``: see
        set_default_band_route (default: the process default, "sweeps")."""
        self.device = require_gpu(device)
        self.ctx = N.Context.get(self.device)
        self.lib = self.ctx.lib
        B = len(Xs)
        if B == 0 or len(Ys) != B or len(specs) != B:
            raise ValueError("Engine needs matching non-empty lists of X, Y and specs")
        xs = [to_device_f64(x, self.device) for x in Xs]
        xs = [x.reshape(x.shape[0], -1) for x in xs]
        ys = [to_device_f64(y, self.device).reshape(-1) for y in Ys]
        D = xs[0].shape[1]
        if any(x.shape[1] != D for x in xs):
            raise ValueError("all problems in one engine must have the same input dimension")
        if D > N.GPX_MAX_DIM:
            raise NotImplementedError(f"input dimension {D} > {N.GPX_MAX_DIM}")
        ns = [x.shape[0] for x in xs]
        if any(y.shape[0] != n for y, n in zip(ys, ns)):
            raise ValueError("X and Y must have the same number of rows")
        self.B, self.D, self.Nmax = B, D, max(ns)
        self.n = np.asarray(ns, dtype=np.int32)
        dev = f"cuda:{self.device}"
        self.X = torch.zeros(B, self.Nmax, D, dtype=torch.float64, device=dev)
        self.Y = torch.zeros(B, self.Nmax, dtype=torch.float64, device=dev)
        for b in range(B):
            self.X[b, : ns[b]] = xs[b]
            self.Y[b, : ns[b]] = ys[b]
        self.specs = (N.GpxKernelSpec * B)(*specs)
        torch.cuda.synchronize(self.device)
        h = ctypes.c_void_p()
        create = self.lib.gpx_batch_create_banded if band_storage else self.lib.gpx_batch_create
        self.band_storage = bool(band_storage)
        rc = create(
            self.ctx.handle, B, self.Nmax, D, ctypes.c_void_p(self.X.data_ptr()),
            ctypes.c_void_p(self.Y.data_ptr()),
            self.n.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), self.specs, ctypes.byref(h))
        if rc != N.GPX_OK:
            raise N.GPXError(f"gpx_batch_create failed ({rc}): {self.ctx.last_error()}")
        self.handle = h
        self.band_route = "sweeps"
        self.set_band_route(_DEFAULT_BAND_ROUTE if band_route is None else band_route)
        self.n_params = np.asarray([s.n_params for s in specs], dtype=np.int64)
        self.eval_count = 0
        self._rebound = {}  # slot -> device tensors of its last rebind (kept alive for the gather)
        # (id(X), id(Y)) -> what rebind derives from a device pair whose X is marked immutable
        # (mark_immutable): a series rebound again and again skips the tensor checks
        self._rb_cache = {}
        self._streams = {}
        self._box_want = {}  # slot -> (box key, X) of a device rebind whose boxes are not cached yet

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                self.lib.gpx_batch_destroy(h)
            except Exception:
                pass
            self.handle = None

    def _stream(self):
        # the current stream's HIP handle, memoised on torch's (id, device, type) of the stream
        # (torch.cuda.current_stream builds a Stream object per call: a rebind-per-fit cost)
        sd = torch._C._cuda_getCurrentStream(self.device)
        h = self._streams.get(sd)
        if h is None:
            h = self._streams[sd] = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        return h

    @staticmethod
    def _active(active) -> np.ndarray:
        return np.ascontiguousarray(np.asarray(active, dtype=np.int32))

    def _harvest_boxes(self) -> None:
        """After a device call gathered the pending rebinds: cache the boxes of the series that
        were not cached yet (gpx_batch_slot_boxes)."""
        if not self._box_want:
            return
        for b, ent in self._box_want.items():
            buf = np.empty(((int(self.n[b]) + 15) // 16) * self.D * 2, dtype=np.float64)  # 16-row boxes
            if self.lib.gpx_batch_slot_boxes(self.handle, int(b), buf.ctypes.data) == N.GPX_OK:
                ent[2] = buf
        self._box_want.clear()

    def lml_grad(self, active: Sequence[int], theta: np.ndarray, wait_deferred: bool = True):
        """logML [B], ∂logML/∂θ [B, 16], info [B] for the active rows (others untouched).
        info[b] > 0: the LAPACK-style failing pivot; info[b] == INFO_BAD_THETA: θ of problem b
        is not finite and > 0, so b was left out of the device call (the others still run).
        With deferral on (set_deferred), the rows of this call that the library deferred are
        waited for and merged in (wait_deferred, for callers that read info != 0 as a failure);
        the stepped driver passes wait_deferred=False and steps them when they arrive."""
        act = self._active(active)
        theta = np.ascontiguousarray(theta, dtype=np.float64)
        assert theta.shape == (self.B, N.GPX_THETA_STRIDE)
        lml = np.full(self.B, np.nan)
        grad = np.full((self.B, N.GPX_THETA_STRIDE), np.nan)
        info = np.full(self.B, N.INFO_UNSET if self.deferral >= 0 else 0, dtype=np.int32)
        act = screen_theta(act, theta, self.n_params, info)
        if len(act) == 0:
            return lml, grad, info
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int32)
        rc = self.lib.gpx_batch_lml_grad(self.handle, len(act), act.ctypes.data_as(ip),
                                         theta.ctypes.data_as(dp), lml.ctypes.data_as(dp),
                                         grad.ctypes.data_as(dp), info.ctypes.data_as(ip),
                                         self._stream())
        self._harvest_boxes()
        if rc not in (N.GPX_OK, N.GPX_NOT_PD):
            raise N.GPXError(f"gpx_batch_lml_grad failed ({rc}): {self.ctx.last_error()}")
        self.eval_count += self._count_reported(info) if self.deferral >= 0 else len(act)
        if wait_deferred and self.deferral >= 0 and (info[act] == N.INFO_DEFERRED).any():
            l2, g2, i2 = self.deferred_wait()
            got = (i2 != N.INFO_UNSET) & (i2 != N.INFO_DEFERRED)
            lml[got], grad[got], info[got] = l2[got], g2[got], i2[got]
        return lml, grad, info

    def lml_grad_row(self, b: int, row: np.ndarray):
        """lml_grad for ONE problem, the drop-in pattern's call (GPR/model_trainer.py:14-19 fits
        one model at a time, so every loss+gradient is a call of one problem): the same library
        call with buffers and argument pointers prepared once per engine, the θ check on the
        problem's own parameters only. Returns (logML, ∂logML/∂θ [16] (a copy), info)."""
        fp = getattr(self, "_row_fast", None)
        if fp is None:
            th = np.ones((self.B, N.GPX_THETA_STRIDE))
            lml = np.zeros(self.B)
            grad = np.zeros((self.B, N.GPX_THETA_STRIDE))
            info = np.zeros(self.B, dtype=np.int32)
            act = np.zeros(1, dtype=np.int32)
            vp = ctypes.c_void_p
            fn = ctypes.CFUNCTYPE(ctypes.c_int, vp, ctypes.c_int, vp, vp, vp, vp, vp, vp)(("gpx_batch_lml_grad", self.lib))
            fp = self._row_fast = (th, lml, grad, info, act, fn, act.ctypes.data, th.ctypes.data, lml.ctypes.data,
                                   grad.ctypes.data, info.ctypes.data)
        th, lml, grad, info, act, fn, pa, pt, pl, pg, pi = fp
        np_b = int(self.n_params[b])
        for v in row[:np_b + 1].tolist():
            if not (0.0 < v < float("inf")):
                info[b] = N.INFO_BAD_THETA
                return float("nan"), np.full(N.GPX_THETA_STRIDE, np.nan), N.INFO_BAD_THETA
        th[b] = row
        act[0] = b
        if self.deferral >= 0:  # (deferral: the general path, which waits for deferred rows)
            l, g, i = self.lml_grad([b], th)
            return float(l[b]), g[b].copy(), int(i[b])
        rc = fn(self.handle.value, 1, pa, pt, pl, pg, pi, self._stream().value)
        if self._box_want:
            self._harvest_boxes()
        if rc not in (N.GPX_OK, N.GPX_NOT_PD):
            raise N.GPXError(f"gpx_batch_lml_grad failed ({rc}): {self.ctx.last_error()}")
        self.eval_count += 1
        return float(lml[b]), grad[b].copy(), int(info[b])

    @staticmethod
    def _count_reported(info: np.ndarray) -> int:
        """Problem-evaluations a deferral-mode complete reported: the call's own rows that were not
        deferred and the earlier deferred rows it delivered (each evaluation counted once,
        whichever call delivers it)."""
        return int(((info != N.INFO_UNSET) & (info != N.INFO_DEFERRED) & (info != N.INFO_BAD_THETA)).sum())

    def lml_grad_submit(self, active: Sequence[int], theta: np.ndarray):
        """First half of lml_grad: enqueue the evaluation on the current stream and return at
        once (gpx_batch_lml_grad_submit); lml_grad_complete() waits and returns what lml_grad
        would. Lets one host thread keep several engines' evaluations in flight."""
        act = self._active(active)
        theta = np.ascontiguousarray(theta, dtype=np.float64)
        assert theta.shape == (self.B, N.GPX_THETA_STRIDE)
        lml = np.full(self.B, np.nan)
        grad = np.full((self.B, N.GPX_THETA_STRIDE), np.nan)
        # (with deferral a complete reports on the call's rows and on earlier deferred rows it
        # delivers; every other row keeps INFO_UNSET)
        info = np.full(self.B, N.INFO_UNSET if self.deferral >= 0 else 0, dtype=np.int32)
        act = screen_theta(act, theta, self.n_params, info)
        self._submitted = (act, lml, grad, info)
        if len(act) == 0:
            return
        ip = ctypes.POINTER(ctypes.c_int32)
        rc = self.lib.gpx_batch_lml_grad_submit(self.handle, len(act), act.ctypes.data_as(ip),
                                                theta.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                                self._stream())
        self._harvest_boxes()
        if rc != N.GPX_OK:
            self._submitted = None
            raise N.GPXError(f"gpx_batch_lml_grad_submit failed ({rc}): {self.ctx.last_error()}")

    def lml_grad_ready(self) -> bool:
        """True when the submitted evaluation has finished on the device."""
        rc = self.lib.gpx_batch_lml_grad_query(self.handle)
        if rc < 0:
            raise N.GPXError(f"gpx_batch_lml_grad_query failed ({rc}): {self.ctx.last_error()}")
        return rc == 1

    def band_width(self, rows, theta: np.ndarray) -> np.ndarray:
        """Per row, the band width (64-blocks) its evaluation at theta would take; -1 dense,
        -2 not known yet (host-side, no device work)."""
        rows = self._active(rows)
        theta = np.ascontiguousarray(theta, dtype=np.float64)
        out = np.zeros(len(rows), dtype=np.int32)
        ip = ctypes.POINTER(ctypes.c_int32)
        rc = self.lib.gpx_batch_band_width(self.handle, len(rows), rows.ctypes.data_as(ip),
                                           theta.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                           out.ctypes.data_as(ip))
        if rc != N.GPX_OK:
            raise N.GPXError(f"gpx_batch_band_width failed ({rc}): {self.ctx.last_error()}")
        return out

    def set_band_route(self, route: str) -> None:
        """This engine's banded route (include/gpx.h gpx_batch_set_band_route)."""
        if route not in N.BAND_ROUTES:
            raise ValueError(f"band route must be one of {sorted(N.BAND_ROUTES)}")
        rc = self.lib.gpx_batch_set_band_route(self.handle, N.BAND_ROUTES[route])
        if rc != N.GPX_OK:
            raise N.GPXError(f"gpx_batch_set_band_route failed ({rc}): {self.ctx.last_error()}")
        self.band_route = route

    deferral = -1

    def set_deferred(self, q: int) -> None:
        """Deferred completion of the slow evaluation classes (include/gpx.h
        gpx_batch_set_deferred): the problems of a call that take the band16 sweeps wider than q
        16-blocks or the 64-row sweeps come back from a later lml_grad_complete (info
        INFO_DEFERRED until then); q < 0 turns it off."""
        rc = self.lib.gpx_batch_set_deferred(self.handle, int(q))
        if rc != N.GPX_OK:
            raise N.GPXError(f"gpx_batch_set_deferred failed ({rc}): {self.ctx.last_error()}")
        self.deferral = int(q) if q >= 0 else -1

    def deferred_wait(self):
        """Every deferred row's result (blocking): (lml, grad, info) with info INFO_UNSET on the
        rows not delivered here."""
        lml = np.full(self.B, np.nan)
        grad = np.full((self.B, N.GPX_THETA_STRIDE), np.nan)
        info = np.full(self.B, N.INFO_UNSET, dtype=np.int32)
        rc = self.lib.gpx_batch_deferred_wait(self.handle, lml.ctypes.data, grad.ctypes.data, info.ctypes.data)
        if rc not in (N.GPX_OK, N.GPX_NOT_PD):
            raise N.GPXError(f"gpx_batch_deferred_wait failed ({rc}): {self.ctx.last_error()}")
        self.eval_count += self._count_reported(info)
        return lml, grad, info

    def band_class(self, rows, theta: np.ndarray) -> np.ndarray:
        """Per row, the path its evaluation at theta would take (include/gpx.h
        gpx_batch_band_class): 1..15 band16 width Q, 16 + p / 32 + p the 64-row banded path
        (without / despite band16 tables), -1 dense, -2 not known yet. Host-side."""
        rows = self._active(rows)
        theta = np.ascontiguousarray(theta, dtype=np.float64)
        out = np.zeros(len(rows), dtype=np.int32)
        rc = self.lib.gpx_batch_band_class(self.handle, len(rows), rows.ctypes.data, theta.ctypes.data,
                                           out.ctypes.data)
        if rc != N.GPX_OK:
            raise N.GPXError(f"gpx_batch_band_class failed ({rc}): {self.ctx.last_error()}")
        return out

    def lml_grad_complete(self):
        act, lml, grad, info = self._submitted
        self._submitted = None
        if len(act) == 0:
            return lml, grad, info
        dp = ctypes.POINTER(ctypes.c_double)
        rc = self.lib.gpx_batch_lml_grad_complete(self.handle, lml.ctypes.data_as(dp), grad.ctypes.data_as(dp),
                                                  info.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
        if rc not in (N.GPX_OK, N.GPX_NOT_PD):
            raise N.GPXError(f"gpx_batch_lml_grad_complete failed ({rc}): {self.ctx.last_error()}")
        self.eval_count += self._count_reported(info) if self.deferral >= 0 else len(act)
        return lml, grad, info

    def predict(self, active: Sequence[int], theta: np.ndarray, Xnew: Sequence, add_noise: bool,
                full_cov: bool = False):
        """Marginal posterior mean/var at Xnew[i] (for problem active[i]); returns lists of
        device tensors [M_i] and info. With full_cov the second list holds the posterior
        covariance matrices [M_i, M_i] (latent f only, as GPflow)."""
        if full_cov and add_noise:
            raise NotImplementedError("full covariance is only defined for predict_f")
        act = self._active(active)
        theta = np.ascontiguousarray(theta, dtype=np.float64)
        xs = [_rows(to_device_f64(x, self.device), self.D) for x in Xnew]
        if any(x.shape[1] != self.D for x in xs):
            raise ValueError(f"Xnew must have {self.D} columns")
        if not full_cov and all(
                x.shape[0] == self.n[b] and torch.equal(x, self.X[b, : self.n[b]]) for b, x in zip(act, xs)):
            return self._predict_train(act, theta, add_noise)
        M = max(x.shape[0] for x in xs)
        dev = f"cuda:{self.device}"
        if M == 0:  # every Xnew is empty: empty outputs, as GPflow returns [0, 1] tensors
            e = torch.empty(0, dtype=torch.float64, device=dev)
            ev = torch.empty(0, 0, dtype=torch.float64, device=dev) if full_cov else e
            return [e for _ in act], [ev for _ in act], np.zeros(self.B, dtype=np.int32)
        Xn = torch.zeros(self.B, M, self.D, dtype=torch.float64, device=dev)
        for b, x in zip(act, xs):
            Xn[b, : x.shape[0]] = x
        mean = torch.empty(self.B, M, dtype=torch.float64, device=dev)
        info = np.zeros(self.B, dtype=np.int32)
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int32)
        if full_cov:
            var = torch.empty(self.B, M, M, dtype=torch.float64, device=dev)
            rc = self.lib.gpx_batch_predict_full_cov(
                self.handle, len(act), act.ctypes.data_as(ip), theta.ctypes.data_as(dp),
                ctypes.c_void_p(Xn.data_ptr()), M, ctypes.c_void_p(mean.data_ptr()),
                ctypes.c_void_p(var.data_ptr()), info.ctypes.data_as(ip), self._stream())
        else:
            var = torch.empty(self.B, M, dtype=torch.float64, device=dev)
            rc = self.lib.gpx_batch_predict(self.handle, len(act), act.ctypes.data_as(ip),
                                            theta.ctypes.data_as(dp), ctypes.c_void_p(Xn.data_ptr()),
                                            M, 1 if add_noise else 0,
                                            ctypes.c_void_p(mean.data_ptr()),
                                            ctypes.c_void_p(var.data_ptr()),
                                            info.ctypes.data_as(ip), self._stream())
        self._harvest_boxes()
        if rc == N.GPX_NOT_PD:
            bad = [int(b) for b in act if info[b] != 0]
            raise N.NotPositiveDefiniteError(
                f"Cholesky decomposition was not successful (problems {bad}, pivots "
                f"{[int(info[b]) for b in bad]}): K + noise I is not positive definite", info)
        if rc != N.GPX_OK:
            raise N.GPXError(f"gpx_batch_predict failed ({rc}): {self.ctx.last_error()}")
        rows = act
        if len(act) < self.B:  # compact copies of the predicted rows (see _predict_train)
            idx = torch.as_tensor(np.asarray(act, dtype=np.int64), device=dev)
            mean, var = mean.index_select(0, idx), var.index_select(0, idx)
            rows = range(len(act))
        outs_m = [mean[k, : x.shape[0]] for k, x in zip(rows, xs)]
        if full_cov:
            outs_v = [var[k, : x.shape[0], : x.shape[0]] for k, x in zip(rows, xs)]
        else:
            outs_v = [var[k, : x.shape[0]] for k, x in zip(rows, xs)]
        return outs_m, outs_v, info

    def _predict_train(self, act: np.ndarray, theta: np.ndarray, add_noise: bool, column: bool = False):
        """predict at each problem's own training inputs: O(N²) from the cached factor
        (gpx_batch_predict_train). ``column``: each output as an [n, 1] view (GPflow's
        predict_f shape) made by one indexing op per problem."""
        dev = f"cuda:{self.device}"
        act = np.ascontiguousarray(act, dtype=np.int32)
        # the predicted rows only, packed by position (gpx_batch_predict_train_rows): a long run
        # keeps every fit's prediction, so views into [B, Nmax] buffers would keep whole batches'
        # buffers alive (64 MiB per call at B = 1024)
        mean = torch.empty(len(act), self.Nmax, dtype=torch.float64, device=dev)
        var = torch.empty(len(act), self.Nmax, dtype=torch.float64, device=dev)
        info = np.zeros(self.B, dtype=np.int32)
        dp = ctypes.POINTER(ctypes.c_double)
        ip = ctypes.POINTER(ctypes.c_int32)
        rc = self.lib.gpx_batch_predict_train_rows(self.handle, len(act), act.ctypes.data_as(ip),
                                                   theta.ctypes.data_as(dp), 1 if add_noise else 0,
                                                   ctypes.c_void_p(mean.data_ptr()), ctypes.c_void_p(var.data_ptr()),
                                                   info.ctypes.data_as(ip), self._stream())
        self._harvest_boxes()
        if rc == N.GPX_NOT_PD:
            bad = [int(b) for b in act if info[b] != 0]
            raise N.NotPositiveDefiniteError(
                f"Cholesky decomposition was not successful (problems {bad}): K + noise I is not "
                "positive definite", info)
        if rc != N.GPX_OK:
            raise N.GPXError(f"gpx_batch_predict_train failed ({rc}): {self.ctx.last_error()}")
        if column:
            mean, var = mean.unsqueeze(-1), var.unsqueeze(-1)
        # one view per problem: unbind makes them in one call, a slice only where n < Nmax
        ms, vs = mean.unbind(0), var.unbind(0)
        nb = self.n
        full = self.Nmax
        return ([m if nb[b] == full else m[: nb[b]] for m, b in zip(ms, act)],
                [v if nb[b] == full else v[: nb[b]] for v, b in zip(vs, act)], info)

    def rebind(self, b: int, X, Y, spec: N.GpxKernelSpec) -> None:
        """Load a new problem into slot b (continuous batching). Host inputs are staged in
        pinned memory at once (gpx_batch_rebind_host); device tensors are only recorded
        (gpx_batch_rebind_device) and gathered, with every other slot rebound since, by one
        kernel at the start of the next device call — so the slot keeps a reference to them
        until it is rebound again."""
        c = self._rb_cache.get((id(X), id(Y)))
        if (c is not None and c[0]() is X and c[1]() is Y and X.data_ptr() == c[2] and Y.data_ptr() == c[3]
                and _immutable_entry(X) is c[4]):
            # (views made afresh: the cache holds no tensor, so it never keeps a dropped series'
            # device storage alive)
            return self._rebind_dev(b, X.detach(), Y.detach().reshape(-1), c[5], spec, c[4])
        ok_dev = (isinstance(X, torch.Tensor) and isinstance(Y, torch.Tensor) and X.is_cuda and Y.is_cuda
                  and X.device.index == self.device and Y.device.index == self.device
                  and X.dtype == torch.float64 and Y.dtype == torch.float64)
        box = None
        if ok_dev:
            x = X.detach().contiguous()
            y = Y.detach().contiguous()
            x2 = x.reshape(x.shape[0], -1)
            n, D, ny = x2.shape[0], x2.shape[1], y.numel()
            fn = self.lib.gpx_batch_rebind_device
            ent = _immutable_entry(X) if X.is_contiguous() else None
            if ent is not None and ent[2] is not None and ent[2].shape[0] == ((n + 15) // 16) * D * 2:
                box = ent[2]
        else:
            x = np.ascontiguousarray(_host_f64(X))
            y = np.ascontiguousarray(_host_f64(Y)).reshape(-1)
            x2 = x.reshape(x.shape[0], -1)
            n, D, ny = x2.shape[0], x2.shape[1], y.shape[0]
            fn = self.lib.gpx_batch_rebind_host
        if D != self.D or n > self.Nmax or ny != n:
            raise ValueError(f"problem does not fit slot shape (N <= {self.Nmax}, D = {self.D})")
        if ok_dev and ent is not None:
            # only contiguous pairs are cached (x, y are then views of X, Y, re-derived on a hit):
            # the entry keeps weak references and scalars, never device storage, and a copy of a
            # strided Y would miss later in-place writes to it
            if X.is_contiguous() and Y.is_contiguous():
                if len(self._rb_cache) >= max(4 * self.B, 1024):
                    self._rb_cache.clear()
                self._rb_cache[(id(X), id(Y))] = (weakref.ref(X), weakref.ref(Y), X.data_ptr(), Y.data_ptr(), ent, n)
            return self._rebind_dev(b, x, y, n, spec, ent)
        self.specs[b] = spec
        self.n_params[b] = spec.n_params
        self.n[b] = n
        if box is not None:
            rc = self.lib.gpx_batch_rebind_device_boxed(
                self.handle, int(b), int(n), ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()),
                ctypes.byref(spec), box.ctypes.data, self._stream())
        else:
            rc = fn(self.handle, int(b), int(n), ctypes.c_void_p(x.data_ptr() if ok_dev else x.ctypes.data),
                    ctypes.c_void_p(y.data_ptr() if ok_dev else y.ctypes.data), ctypes.byref(spec), self._stream())
        if rc != N.GPX_OK:
            raise N.GPXError(f"gpx_batch_rebind failed ({rc}): {self.ctx.last_error()}")
        self._box_want.pop(b, None)
        if ok_dev:
            self._rebound[b] = (x, y)  # read by the deferred gather
            if box is None and ent is not None:
                self._box_want[b] = ent
        else:
            self._rebound.pop(b, None)

    def _rebind_dev(self, b, x, y, n, spec, ent) -> None:
        """rebind's device path for a series whose X is marked immutable (its boxes cached in
        ``ent`` once a call has gathered them)."""
        box = ent[2]
        if box is not None and box.shape[0] != ((n + 15) // 16) * self.D * 2:
            box = None
        if box is not None:
            if len(ent) < 4 or ent[3][0] is not box:  # (the boxes' address, once per array)
                del ent[3:]
                ent.append((box, box.ctypes.data))
            box_ptr = ent[3][1]
        self.specs[b] = spec
        self.n_params[b] = spec.n_params
        self.n[b] = n
        if box is not None:
            rc = self.lib.gpx_batch_rebind_device_boxed(self.handle, int(b), int(n), ctypes.c_void_p(x.data_ptr()),
                                                        ctypes.c_void_p(y.data_ptr()), ctypes.byref(spec),
                                                        box_ptr, self._stream())
        else:
            rc = self.lib.gpx_batch_rebind_device(self.handle, int(b), int(n), ctypes.c_void_p(x.data_ptr()),
                                                  ctypes.c_void_p(y.data_ptr()), ctypes.byref(spec), self._stream())
        if rc != N.GPX_OK:
            raise N.GPXError(f"gpx_batch_rebind failed ({rc}): {self.ctx.last_error()}")
        self._box_want.pop(b, None)
        self._rebound[b] = (x, y)  # read by the deferred gather
        if box is None:
            self._box_want[b] = ent

    def reset_timing(self) -> None:
        self.lib.gpx_batch_reset_timing(self.handle)

    def last_timing(self) -> N.GpxTiming:
        t = N.GpxTiming()
        self.lib.gpx_batch_last_timing(self.handle, ctypes.byref(t))
        return t

    def wave_trace(self, cap: int) -> None:
        """Diagnostic: record each band16 wavefront's residency (start, end, kind) in the device's
        100 MHz clock, room for `cap` records (0: off). include/gpx.h gpx_batch_wave_trace."""
        rc = self.lib.gpx_batch_wave_trace(self.handle, int(cap))
        if rc != N.GPX_OK:
            raise N.GPXError(f"gpx_batch_wave_trace failed ({rc}): {self.ctx.last_error()}")
        self._wtrace_cap = int(cap)

    def wave_trace_read(self) -> np.ndarray:
        """The records since the last read, [n, 3] uint64 (start, end, kind); restarts recording."""
        cap = getattr(self, "_wtrace_cap", 0)
        out = np.zeros((max(cap, 1), 3), dtype=np.uint64)
        n = ctypes.c_uint(0)
        rc = self.lib.gpx_batch_wave_trace_read(self.handle, out.ctypes.data, cap, ctypes.byref(n))
        if rc != N.GPX_OK:
            raise N.GPXError(f"gpx_batch_wave_trace_read failed ({rc}): {self.ctx.last_error()}")
        return out[:n.value]


class SVGPEngine:
    """Device state of one SVGP data shard (include/gpx.h gpx_svgp): X [N, D] / Y [N]
    resident in HBM, Kmn / workspace owned by the library, and the per-shard partial-sum
    buffer as a torch tensor (so torch.distributed can all-reduce it in place)."""

    def __init__(self, X, Y, spec: N.GpxKernelSpec, M: int, num_data: float,
                 n_total: Optional[int] = None, device: Optional[int] = None):
        self.device = require_gpu(device)
        self.ctx = N.Context.get(self.device)
        self.lib = self.ctx.lib
        x = to_device_f64(X, self.device)
        self.X = x.reshape(x.shape[0], -1).contiguous()
        self.Y = to_device_f64(Y, self.device).reshape(-1).contiguous()
        self.N, self.D = self.X.shape
        if self.Y.shape[0] != self.N:
            raise ValueError("X and Y must have the same number of rows")
        if self.D > N.GPX_MAX_DIM:
            raise NotImplementedError(f"input dimension {self.D} > {N.GPX_MAX_DIM}")
        self.M = int(M)
        self.n_total = int(self.N if n_total is None else n_total)
        self.spec = spec
        torch.cuda.synchronize(self.device)
        h = ctypes.c_void_p()
        rc = self.lib.gpx_svgp_create(self.ctx.handle, self.N, self.M, self.D,
                                      ctypes.c_void_p(self.X.data_ptr()), ctypes.c_void_p(self.Y.data_ptr()),
                                      ctypes.byref(self.spec), float(num_data), self.n_total, ctypes.byref(h))
        if rc != N.GPX_OK:
            raise N.GPXError(f"gpx_svgp_create failed ({rc}): {self.ctx.last_error()}")
        self.handle = h
        ptr, ln = ctypes.c_void_p(), ctypes.c_longlong()
        self.lib.gpx_svgp_partials(h, ctypes.byref(ptr), ctypes.byref(ln))
        self.partials = torch.zeros(int(ln.value), dtype=torch.float64, device=f"cuda:{self.device}")
        rc = self.lib.gpx_svgp_bind_partials(h, ctypes.c_void_p(self.partials.data_ptr()), int(ln.value))
        if rc != N.GPX_OK:
            raise N.GPXError(f"gpx_svgp_bind_partials failed ({rc}): {self.ctx.last_error()}")

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            try:
                self.lib.gpx_svgp_destroy(h)
            except Exception:
                pass
            self.handle = None

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    @staticmethod
    def _host(a, shape) -> np.ndarray:
        return np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(shape))

    def _args(self, theta, Z, q_mu, q_sqrt):
        M, D = self.M, self.D
        self._keep = (self._host(theta, (N.GPX_THETA_STRIDE,)), self._host(Z, (M, D)),
                      self._host(q_mu, (M,)), self._host(q_sqrt, (M, M)))
        dp = ctypes.POINTER(ctypes.c_double)
        return [a.ctypes.data_as(dp) for a in self._keep]

    def _raise(self, rc, what, info):
        if rc == N.GPX_NOT_PD:
            raise N.NotPositiveDefiniteError(
                f"Cholesky decomposition was not successful (pivot {int(info.value)}): "
                "Kuu + jitter I is not positive definite", int(info.value))
        if rc != N.GPX_OK:
            raise N.GPXError(f"{what} failed ({rc}): {self.ctx.last_error()}")

    def eval_local(self, theta, Z, q_mu, q_sqrt) -> None:
        info = ctypes.c_int32(0)
        rc = self.lib.gpx_svgp_eval_local(self.handle, *self._args(theta, Z, q_mu, q_sqrt),
                                          ctypes.byref(info), self._stream())
        self._raise(rc, "gpx_svgp_eval_local", info)

    def eval_finish(self):
        M, D = self.M, self.D
        elbo = np.zeros(1)
        gth = np.zeros(N.GPX_THETA_STRIDE)
        gZ = np.zeros((M, D))
        gq = np.zeros(M)
        gR = np.zeros((M, M))
        dp = ctypes.POINTER(ctypes.c_double)
        rc = self.lib.gpx_svgp_eval_finish(self.handle, elbo.ctypes.data_as(dp), gth.ctypes.data_as(dp),
                                           gZ.ctypes.data_as(dp), gq.ctypes.data_as(dp),
                                           gR.ctypes.data_as(dp), self._stream())
        if rc != N.GPX_OK:
            raise N.GPXError(f"gpx_svgp_eval_finish failed ({rc}): {self.ctx.last_error()}")
        return float(elbo[0]), gth, gZ, gq, gR

    def elbo_grad(self, theta, Z, q_mu, q_sqrt):
        """ELBO and ∂ELBO/∂(θ, Z, q_mu, q_sqrt) (constrained space) on this shard alone."""
        self.eval_local(theta, Z, q_mu, q_sqrt)
        return self.eval_finish()

    def predict(self, theta, Z, q_mu, q_sqrt, Xnew, add_noise: bool):
        x = _rows(to_device_f64(Xnew, self.device), self.D).contiguous()
        if x.shape[1] != self.D:
            raise ValueError(f"Xnew must have {self.D} columns")
        Mn = x.shape[0]
        mean = torch.empty(Mn, dtype=torch.float64, device=x.device)
        var = torch.empty(Mn, dtype=torch.float64, device=x.device)
        if Mn == 0:  # empty Xnew: empty outputs (GPflow returns [0, 1] tensors)
            return mean, var
        info = ctypes.c_int32(0)
        rc = self.lib.gpx_svgp_predict(self.handle, *self._args(theta, Z, q_mu, q_sqrt),
                                       ctypes.c_void_p(x.data_ptr()), Mn, 1 if add_noise else 0,
                                       ctypes.c_void_p(mean.data_ptr()), ctypes.c_void_p(var.data_ptr()),
                                       ctypes.byref(info), self._stream())
        self._raise(rc, "gpx_svgp_predict", info)
        return mean, var


# ----------------------------------------------------------------------------------------
# pooled single-problem engines for models used on their own (no batch engine attached)
# ----------------------------------------------------------------------------------------
_SOLO_POOL: "OrderedDict" = None
_SOLO_POOL_MAX = 8


def solo_engine(model) -> Engine:
    """A B=1 engine for `model`'s shape, shared by every model of that (device, padded N, D):
    the reference fits many models one after another (GPR/main.py's ticker × timeframe ×
    kernel loop), and a fresh N×N workspace per model would grow device memory without
    bound. The model's data is rebound into the slot when another model used it last (the
    cached factor is dropped then, so results never mix)."""
    global _SOLO_POOL
    c = getattr(model, "_solo_cache", None)
    if c is not None and c[1] == _DEFAULT_BAND_ROUTE:  # (this model was the slot's last user)
        eng = c[0]()
        if eng is not None and eng._owner is not None and eng._owner() is model and _SOLO_POOL.get(c[2]) is eng:
            return eng
    import weakref
    from collections import OrderedDict
    if _SOLO_POOL is None:
        _SOLO_POOL = OrderedDict()
    X, Y = model.data
    n, D = int(X.shape[0]), int(X.shape[1])
    key = (int(model.device), (n + 63) // 64 * 64, D, _DEFAULT_BAND_ROUTE)  # (the route: set_default_band_route)
    eng = _SOLO_POOL.get(key)
    if eng is None:
        npad = key[1]
        eng = Engine([torch.zeros(npad, D, dtype=torch.float64)], [torch.zeros(npad, 1, dtype=torch.float64)],
                     [model._spec], device=model.device)
        eng._owner = None
        _SOLO_POOL[key] = eng
        while len(_SOLO_POOL) > _SOLO_POOL_MAX:
            _SOLO_POOL.popitem(last=False)
    _SOLO_POOL.move_to_end(key)
    owner = eng._owner() if eng._owner is not None else None
    if owner is not model:
        eng.rebind(0, X, Y, model._spec)
        eng._owner = weakref.ref(model)
    model._solo_cache = (weakref.ref(eng), _DEFAULT_BAND_ROUTE, key)
    return eng
