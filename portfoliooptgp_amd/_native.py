"""ctypes binding of the C ABI in ``include/gpx.h`` (libgpx.so, built for gfx950).

There is no CPU fallback: importing the engine without the shared library, or evaluating
without a HIP device, raises. The oracle under ``oracle/`` is test infrastructure and is never
imported from here.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

GPX_OK, GPX_NOT_PD, GPX_BAD_ARG, GPX_HIP_ERROR = 0, 1, 2, 3
GPX_MAX_TERMS = 4
GPX_THETA_STRIDE = 16
GPX_MAX_DIM = 16

(GPX_SE, GPX_MATERN12, GPX_MATERN32, GPX_MATERN52, GPX_EXPONENTIAL, GPX_RQ, GPX_PERIODIC_SE,
 GPX_LINEAR) = range(1, 9)
GPX_SUM, GPX_PRODUCT = 0, 1
# gpx_batch_set_band_route (include/gpx.h)
BAND_ROUTES = {"sweeps": 0, "bcr": 1, "auto": 2}

# GPX_LIB: an alternative build of the library (A/B experiments); default the in-tree one
LIB_PATH = os.environ.get("GPX_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgpx.so")

# every symbol include/gpx.h declares (checked by tests/test_abi.py)
EXPORTED_SYMBOLS = (
    "gpx_version", "gpx_create", "gpx_destroy", "gpx_last_error", "gpx_batch_create", "gpx_batch_create_banded",
    "gpx_batch_rebind_host",
    "gpx_batch_rebind_device", "gpx_batch_rebind_device_boxed", "gpx_batch_slot_boxes",
    "gpx_batch_destroy", "gpx_batch_lml_grad", "gpx_batch_lml_grad_submit", "gpx_batch_lml_grad_complete",
    "gpx_batch_lml_grad_query", "gpx_batch_band_width",
    "gpx_batch_predict", "gpx_batch_predict_full_cov", "gpx_batch_predict_train", "gpx_batch_predict_train_rows",
    "gpx_batch_last_timing",
    "gpx_set_profiling", "gpx_batch_reset_timing", "gpx_batch_rebind",
    "gpx_batch_wave_trace", "gpx_batch_wave_trace_read", "gpx_batch_band_class",
    "gpx_batch_set_deferred", "gpx_batch_deferred_wait", "gpx_batch_deferred_rows",
    "gpx_batch_set_band_route",
    "gpx_svgp_create", "gpx_svgp_destroy", "gpx_svgp_partials", "gpx_svgp_bind_partials",
    "gpx_svgp_eval_local", "gpx_svgp_eval_finish", "gpx_svgp_elbo_grad", "gpx_svgp_predict",
    "gpx_host_theta_rows", "gpx_host_loss_grad_u",
)


class GpxTerm(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("dim_start", ctypes.c_int32),
                ("dim_count", ctypes.c_int32), ("param_offset", ctypes.c_int32)]


class GpxKernelSpec(ctypes.Structure):
    _fields_ = [("n_terms", ctypes.c_int32), ("combine", ctypes.c_int32),
                ("n_params", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("terms", GpxTerm * GPX_MAX_TERMS)]


class GpxTiming(ctypes.Structure):
    _fields_ = [("factor_ms", ctypes.c_double), ("alpha_ms", ctypes.c_double),
                ("grad_ms", ctypes.c_double), ("predict_ms", ctypes.c_double),
                ("total_ms", ctypes.c_double), ("gemm_flops", ctypes.c_double),
                ("contract_ms_total", ctypes.c_double), ("contract_launches", ctypes.c_double),
                ("contract_alg_flops", ctypes.c_double), ("eval_ms_total", ctypes.c_double),
                ("evals", ctypes.c_double), ("band_ms_total", ctypes.c_double),
                ("band_calls", ctypes.c_double), ("band_evals", ctypes.c_double),
                ("band_p_sum", ctypes.c_double), ("band_fwd_ms_total", ctypes.c_double),
                ("band_bwd_ms_total", ctypes.c_double), ("band_fused_launches", ctypes.c_double),
                ("band_fwd_flops", ctypes.c_double), ("band_bwd_flops", ctypes.c_double),
                ("band_fallbacks", ctypes.c_double), ("shadow_evals", ctypes.c_double),
                ("shadow_predicts", ctypes.c_double), ("band16_fwd_ms_total", ctypes.c_double),
                ("band16_bwd_ms_total", ctypes.c_double), ("band16_launches", ctypes.c_double),
                ("band16_evals", ctypes.c_double), ("band16_q_sum", ctypes.c_double),
                ("band16_fwd_flops", ctypes.c_double), ("band16_bwd_flops", ctypes.c_double),
                ("band16_wave_ms", ctypes.c_double), ("band16_wide_ms_total", ctypes.c_double),
                ("band16_wide_launches", ctypes.c_double), ("band16_wide_flops", ctypes.c_double),
                ("band16_wide_evals", ctypes.c_double), ("bcr_ms_total", ctypes.c_double),
                ("bcr_calls", ctypes.c_double), ("bcr_evals", ctypes.c_double),
                ("band_fused_p2_launches", ctypes.c_double), ("bcr_wide_evals", ctypes.c_double)]


class GPXError(RuntimeError):
    pass


INFO_BAD_THETA = -1  # info code of a problem whose θ was screened out on the host
INFO_DEFERRED = -1000  # GPX_INFO_DEFERRED: the problem's result comes with a later complete
INFO_UNSET = -2000  # (Python side) a row the last complete did not report on


class InvalidParameterError(GPXError):
    """A constrained hyperparameter left (0, ∞) — softplus(u) underflows to 0 for u < -745 after
    an extreme L-BFGS-B step. The problem is not evaluated (the rest of its batch is)."""


class NotPositiveDefiniteError(GPXError):
    """K + σn²I is not positive definite (GPflow raises tf.errors.InvalidArgumentError from
    tf.linalg.cholesky in the same situation)."""

    def __init__(self, msg, info=None):
        super().__init__(msg)
        self.info = info


_lib = None
_lib_lock = threading.Lock()


def load_library(path: Optional[str] = None) -> ctypes.CDLL:
    """Load libgpx.so and declare its signatures. Raises if the library is missing."""
    global _lib
    with _lib_lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise GPXError(
                f"libgpx.so not found at {p}: build it with `make` (or __graft_entry__.build()). "
                "portfoliooptgp_amd has no CPU fallback.")
        lib = ctypes.CDLL(p)
        c_int, c_void_p, c_double_p = ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)
        c_int_p = ctypes.POINTER(ctypes.c_int32)
        c_double = ctypes.c_double
        lib.gpx_version.restype = ctypes.c_char_p
        lib.gpx_version.argtypes = []
        lib.gpx_create.restype = c_int
        lib.gpx_create.argtypes = [c_int, ctypes.POINTER(c_void_p)]
        lib.gpx_destroy.restype = c_int
        lib.gpx_destroy.argtypes = [c_void_p]
        lib.gpx_last_error.restype = ctypes.c_char_p
        lib.gpx_last_error.argtypes = [c_void_p]
        lib.gpx_set_profiling.restype = c_int
        lib.gpx_set_profiling.argtypes = [c_void_p, c_int]
        lib.gpx_batch_create.restype = c_int
        lib.gpx_batch_create.argtypes = [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int_p,
                                         ctypes.POINTER(GpxKernelSpec), ctypes.POINTER(c_void_p)]
        lib.gpx_batch_create_banded.restype = c_int
        lib.gpx_batch_create_banded.argtypes = lib.gpx_batch_create.argtypes
        lib.gpx_batch_destroy.restype = c_int
        lib.gpx_batch_destroy.argtypes = [c_void_p]
        lib.gpx_batch_lml_grad.restype = c_int
        lib.gpx_batch_lml_grad.argtypes = [c_void_p, c_int, c_int_p, c_double_p, c_double_p,
                                           c_double_p, c_int_p, c_void_p]
        lib.gpx_batch_lml_grad_submit.restype = c_int
        lib.gpx_batch_lml_grad_submit.argtypes = [c_void_p, c_int, c_int_p, c_double_p, c_void_p]
        lib.gpx_batch_lml_grad_complete.restype = c_int
        lib.gpx_batch_lml_grad_complete.argtypes = [c_void_p, c_double_p, c_double_p, c_int_p]
        lib.gpx_batch_lml_grad_query.restype = c_int
        lib.gpx_batch_lml_grad_query.argtypes = [c_void_p]
        lib.gpx_batch_band_width.restype = c_int
        lib.gpx_batch_band_width.argtypes = [c_void_p, c_int, c_int_p, c_double_p, c_int_p]
        lib.gpx_batch_predict.restype = c_int
        lib.gpx_batch_predict.argtypes = [c_void_p, c_int, c_int_p, c_double_p, c_void_p, c_int,
                                          c_int, c_void_p, c_void_p, c_int_p, c_void_p]
        lib.gpx_batch_predict_full_cov.restype = c_int
        lib.gpx_batch_predict_full_cov.argtypes = [c_void_p, c_int, c_int_p, c_double_p, c_void_p,
                                                   c_int, c_void_p, c_void_p, c_int_p, c_void_p]
        lib.gpx_batch_predict_train.restype = c_int
        lib.gpx_batch_predict_train.argtypes = [c_void_p, c_int, c_int_p, c_double_p, c_int, c_void_p,
                                                c_void_p, c_int_p, c_void_p]
        lib.gpx_batch_predict_train_rows.restype = c_int
        lib.gpx_batch_predict_train_rows.argtypes = [c_void_p, c_int, c_int_p, c_double_p, c_int, c_void_p,
                                                     c_void_p, c_int_p, c_void_p]
        lib.gpx_batch_last_timing.restype = c_int
        lib.gpx_batch_last_timing.argtypes = [c_void_p, ctypes.POINTER(GpxTiming)]
        lib.gpx_batch_rebind.restype = c_int
        lib.gpx_batch_rebind.argtypes = [c_void_p, c_int, c_int, ctypes.POINTER(GpxKernelSpec)]
        lib.gpx_batch_rebind_host.restype = c_int
        lib.gpx_batch_rebind_host.argtypes = [c_void_p, c_int, c_int, c_void_p, c_void_p,
                                              ctypes.POINTER(GpxKernelSpec), c_void_p]
        lib.gpx_batch_rebind_device.restype = c_int
        lib.gpx_batch_rebind_device.argtypes = [c_void_p, c_int, c_int, c_void_p, c_void_p,
                                                ctypes.POINTER(GpxKernelSpec), c_void_p]
        lib.gpx_batch_rebind_device_boxed.restype = c_int
        lib.gpx_batch_rebind_device_boxed.argtypes = [c_void_p, c_int, c_int, c_void_p, c_void_p,
                                                      ctypes.POINTER(GpxKernelSpec), c_void_p, c_void_p]
        lib.gpx_batch_slot_boxes.restype = c_int
        lib.gpx_batch_slot_boxes.argtypes = [c_void_p, c_int, c_void_p]
        lib.gpx_batch_reset_timing.restype = c_int
        lib.gpx_batch_reset_timing.argtypes = [c_void_p]
        lib.gpx_batch_set_deferred.restype = c_int
        lib.gpx_batch_set_deferred.argtypes = [c_void_p, c_int]
        lib.gpx_batch_set_band_route.restype = c_int
        lib.gpx_batch_set_band_route.argtypes = [c_void_p, c_int]
        lib.gpx_batch_deferred_wait.restype = c_int
        lib.gpx_batch_deferred_wait.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p]
        lib.gpx_batch_deferred_rows.restype = c_int
        lib.gpx_batch_deferred_rows.argtypes = [c_void_p, c_void_p, c_int]
        lib.gpx_batch_band_class.restype = c_int
        lib.gpx_batch_band_class.argtypes = [c_void_p, c_int, c_void_p, c_void_p, c_void_p]
        lib.gpx_batch_wave_trace.restype = c_int
        lib.gpx_batch_wave_trace.argtypes = [c_void_p, ctypes.c_uint]
        lib.gpx_batch_wave_trace_read.restype = c_int
        lib.gpx_batch_wave_trace_read.argtypes = [c_void_p, c_void_p, ctypes.c_uint, ctypes.POINTER(ctypes.c_uint)]
        spec_p = ctypes.POINTER(GpxKernelSpec)
        lib.gpx_svgp_create.restype = c_int
        lib.gpx_svgp_create.argtypes = [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, spec_p,
                                        c_double, ctypes.c_longlong, ctypes.POINTER(c_void_p)]
        lib.gpx_svgp_destroy.restype = c_int
        lib.gpx_svgp_destroy.argtypes = [c_void_p]
        lib.gpx_svgp_partials.restype = c_int
        lib.gpx_svgp_partials.argtypes = [c_void_p, ctypes.POINTER(c_void_p), ctypes.POINTER(ctypes.c_longlong)]
        lib.gpx_svgp_bind_partials.restype = c_int
        lib.gpx_svgp_bind_partials.argtypes = [c_void_p, c_void_p, ctypes.c_longlong]
        lib.gpx_svgp_eval_local.restype = c_int
        lib.gpx_svgp_eval_local.argtypes = [c_void_p, c_double_p, c_double_p, c_double_p, c_double_p,
                                            c_int_p, c_void_p]
        lib.gpx_svgp_eval_finish.restype = c_int
        lib.gpx_svgp_eval_finish.argtypes = [c_void_p, c_double_p, c_double_p, c_double_p, c_double_p,
                                             c_double_p, c_void_p]
        lib.gpx_svgp_elbo_grad.restype = c_int
        lib.gpx_svgp_elbo_grad.argtypes = [c_void_p, c_double_p, c_double_p, c_double_p, c_double_p,
                                           c_double_p, c_double_p, c_double_p, c_double_p, c_double_p,
                                           c_int_p, c_void_p]
        lib.gpx_svgp_predict.restype = c_int
        lib.gpx_svgp_predict.argtypes = [c_void_p, c_double_p, c_double_p, c_double_p, c_double_p,
                                         c_void_p, c_int, c_int, c_void_p, c_void_p, c_int_p, c_void_p]
        lib.gpx_host_theta_rows.restype = c_int
        lib.gpx_host_theta_rows.argtypes = [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
        lib.gpx_host_loss_grad_u.restype = c_int
        lib.gpx_host_loss_grad_u.argtypes = [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                             c_void_p, c_void_p]
        if path is None:
            _lib = lib
        return lib


class Context:
    """One gpx context per HIP device (process-wide cache)."""

    _cache = {}

    def __init__(self, device: int):
        self.lib = load_library()
        self.device = device
        h = ctypes.c_void_p()
        rc = self.lib.gpx_create(device, ctypes.byref(h))
        if rc != GPX_OK:
            raise GPXError(f"gpx_create(device={device}) failed with code {rc}: no usable HIP device?")
        self.handle = h

    @classmethod
    def get(cls, device: int) -> "Context":
        if device not in cls._cache:
            cls._cache[device] = Context(device)
        return cls._cache[device]

    def last_error(self) -> str:
        return self.lib.gpx_last_error(self.handle).decode()

    def set_profiling(self, on: bool) -> None:
        self.lib.gpx_set_profiling(self.handle, 1 if on else 0)
