"""Covariance functions with the gpflow.kernels 2.9.1 constructor surface.

The objects only hold parameters and structure; they compile to a ``gpx_kernel_spec``
(include/gpx.h) that the HIP kernels evaluate on the device. Classes and defaults follow the
kernels the reference instantiates at GPR/main.py:105-114 (SE, Matern12, RationalQuadratic,
Exponential, SE+Matern12, Exponential+Periodic(SE)+Linear, Exponential+Periodic(SE),
SE*Matern12) and Multi-Input_GPR/main.py:118-135 (Exponential(active_dims) *
Exponential(active_dims)). Parameter order = GPflow's tf.Module flattening order
(sorted attribute names; Sum/Product kernels in list order).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

from . import _native as N
from .parameter import Parameter


def _normalise_active_dims(active_dims) -> Optional[Tuple[int, int]]:
    """Return (start, count) for a contiguous selection, None for 'all dims'."""
    if active_dims is None:
        return None
    if isinstance(active_dims, slice):
        if active_dims.step not in (None, 1):
            raise NotImplementedError("active_dims slices with a step are not supported")
        start = 0 if active_dims.start is None else int(active_dims.start)
        if active_dims.stop is None:
            return (start, -1)  # up to D, resolved at compile time
        return (start, int(active_dims.stop) - start)
    dims = [int(d) for d in list(active_dims)]
    if not dims or dims != list(range(dims[0], dims[0] + len(dims))):
        raise NotImplementedError("only contiguous active_dims are supported")
    return (dims[0], len(dims))


class Kernel:
    """Base class. ``parameters`` is the GPflow-ordered tuple of Parameter objects."""

    def __init__(self, active_dims=None, name: Optional[str] = None):
        self.active_dims = active_dims
        self._dims = _normalise_active_dims(active_dims)
        self.name = name or type(self).__name__.lower()

    # --- structure --------------------------------------------------------------------
    @property
    def parameters(self) -> Tuple[Parameter, ...]:
        raise NotImplementedError

    @property
    def trainable_parameters(self) -> Tuple[Parameter, ...]:
        return tuple(p for p in self.parameters if p.trainable)

    @property
    def trainable_variables(self):
        return tuple(p.unconstrained_variable for p in self.trainable_parameters)

    def _param_paths(self, prefix: str) -> List[Tuple[str, Parameter]]:
        raise NotImplementedError

    def _terms(self) -> List["Kernel"]:
        return [self]

    def _combine(self) -> int:
        return N.GPX_SUM

    # --- algebra (gpflow.kernels.Kernel.__add__/__mul__) -------------------------------
    def __add__(self, other: "Kernel") -> "Sum":
        return Sum([self, other])

    def __mul__(self, other: "Kernel") -> "Product":
        return Product([self, other])

    def __repr__(self) -> str:
        return f"<{type(self).__name__} " + ", ".join(
            f"{n}={p.value:.6g}" for n, p in self._param_paths("")) + ">"


class _Term(Kernel):
    kind = 0

    def _spec_term(self, D: int, offset: int) -> N.GpxTerm:
        if self._dims is None:
            start, count = 0, D
        else:
            start, count = self._dims
            if count < 0:
                count = D - start
        if start < 0 or count < 1 or start + count > D:
            raise ValueError(f"{self.name}: active_dims {self.active_dims} out of range for D={D}")
        return N.GpxTerm(self.kind, start, count, offset)


class Stationary(_Term):
    """IsotropicStationary: scalar lengthscale, params ordered [lengthscales, variance]."""

    def __init__(self, variance=1.0, lengthscales=1.0, active_dims=None, name=None):
        super().__init__(active_dims=active_dims, name=name)
        self.variance = Parameter(variance, name="variance")
        self.lengthscales = Parameter(lengthscales, name="lengthscales")

    @property
    def parameters(self):
        return (self.lengthscales, self.variance)

    def _param_paths(self, prefix):
        return [(prefix + "lengthscales", self.lengthscales), (prefix + "variance", self.variance)]


class SquaredExponential(Stationary):
    """σ² exp(−r²/2)."""
    kind = N.GPX_SE


RBF = SquaredExponential


class Matern12(Stationary):
    """σ² exp(−r)."""
    kind = N.GPX_MATERN12


class Matern32(Stationary):
    """σ² (1 + √3 r) exp(−√3 r)."""
    kind = N.GPX_MATERN32


class Matern52(Stationary):
    """σ² (1 + √5 r + 5r²/3) exp(−√5 r)."""
    kind = N.GPX_MATERN52


class Exponential(Stationary):
    """gpflow.kernels.Exponential: σ² exp(−r/2)."""
    kind = N.GPX_EXPONENTIAL


class RationalQuadratic(Stationary):
    """σ² (1 + r²/(2α))^(−α); params ordered [alpha, lengthscales, variance]."""
    kind = N.GPX_RQ

    def __init__(self, variance=1.0, lengthscales=1.0, alpha=1.0, active_dims=None, name=None):
        super().__init__(variance, lengthscales, active_dims, name)
        self.alpha = Parameter(alpha, name="alpha")

    @property
    def parameters(self):
        return (self.alpha, self.lengthscales, self.variance)

    def _param_paths(self, prefix):
        return [(prefix + "alpha", self.alpha)] + super()._param_paths(prefix)


class Linear(_Term):
    """σ² x·x' over the active dims; params [variance]."""
    kind = N.GPX_LINEAR

    def __init__(self, variance=1.0, active_dims=None, name=None):
        super().__init__(active_dims=active_dims, name=name)
        self.variance = Parameter(variance, name="variance")

    @property
    def parameters(self):
        return (self.variance,)

    def _param_paths(self, prefix):
        return [(prefix + "variance", self.variance)]


class Periodic(_Term):
    """gpflow.kernels.Periodic(base_kernel=SquaredExponential(), period=1.0):
    σ² exp(−½ Σ_d (sin(π(x_d−x'_d)/p)/ℓ)²); params [base.lengthscales, base.variance, period]."""
    kind = N.GPX_PERIODIC_SE

    def __init__(self, base_kernel: Optional[SquaredExponential] = None, period=1.0, name=None):
        base_kernel = base_kernel if base_kernel is not None else SquaredExponential()
        if type(base_kernel) is not SquaredExponential:
            raise NotImplementedError("Periodic is implemented for a SquaredExponential base kernel")
        super().__init__(active_dims=base_kernel.active_dims, name=name)
        self.base_kernel = base_kernel
        self.period = Parameter(period, name="period")

    @property
    def parameters(self):
        return (self.base_kernel.lengthscales, self.base_kernel.variance, self.period)

    def _param_paths(self, prefix):
        return self.base_kernel._param_paths(prefix + "base_kernel.") + [(prefix + "period", self.period)]


class Combination(Kernel):
    """Sum / Product; nested combinations of the same class are flattened like GPflow's
    Combination._set_kernels."""

    combine = N.GPX_SUM

    def __init__(self, kernels: Sequence[Kernel], name=None):
        super().__init__(name=name)
        flat: List[Kernel] = []
        for k in kernels:
            if not isinstance(k, Kernel):
                raise TypeError("can only combine Kernel instances")
            if isinstance(k, type(self)):
                flat.extend(k.kernels)
            else:
                flat.append(k)
        self.kernels = flat

    @property
    def parameters(self):
        return tuple(p for k in self.kernels for p in k.parameters)

    def _param_paths(self, prefix):
        out = []
        for i, k in enumerate(self.kernels):
            out.extend(k._param_paths(f"{prefix}kernels[{i}]."))
        return out

    def _terms(self):
        terms = []
        for k in self.kernels:
            if isinstance(k, Combination):
                raise NotImplementedError(
                    "nested Sum/Product mixes are not supported by the device spec; "
                    "use a flat Sum or a flat Product")
            terms.append(k)
        return terms

    def _combine(self):
        return self.combine


class Sum(Combination):
    combine = N.GPX_SUM


class Product(Combination):
    combine = N.GPX_PRODUCT


def compile_spec(kernel: Kernel, D: int) -> N.GpxKernelSpec:
    """Kernel object -> gpx_kernel_spec (parameter offsets in GPflow order)."""
    terms = kernel._terms()
    if len(terms) > N.GPX_MAX_TERMS:
        raise NotImplementedError(f"at most {N.GPX_MAX_TERMS} kernel terms are supported")
    spec = N.GpxKernelSpec()
    spec.n_terms = len(terms)
    spec.combine = kernel._combine()
    off = 0
    for t, term in enumerate(terms):
        spec.terms[t] = term._spec_term(D, off)
        off += len(term.parameters)
    if off + 1 > N.GPX_THETA_STRIDE:
        raise NotImplementedError("too many kernel parameters")
    spec.n_params = off
    return spec
