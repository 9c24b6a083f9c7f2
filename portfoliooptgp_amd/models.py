"""gpflow.models.GPR 2.9.1 surface backed by the HIP engine.

Reference call sites this serves: ``gpflow.models.GPR(data=(X_tf, Y_tf), kernel=kernel)``
(GPR/model_trainer.py:15), ``model.likelihood.variance.assign`` / ``set_trainable``
(:16-17), ``model.training_loss`` / ``model.trainable_variables`` (:19), ``model.predict_f``
(:20, GPR/predictor.py:6) and ``model.predict_y`` (GPR/predictor.py:7); and
``gpflow.models.GPR((X, Y), kernel=deepcopy(k), noise_variance=v)``
(Multi-Input_GPR/main.py:421-423, Multi-Input_GPR/models/model_trainer.py:31).

Arithmetic: every logML / gradient / prediction is computed by libgpx.so on the GPU. The
outputs are torch float64 tensors: on the CPU when the data came in as numpy / CPU tensors
(so ``.numpy()``, arithmetic and slicing work as on the tf tensors GPflow returns), else on
the GPU.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from . import _native as N
from .engine import Engine, default_device, solo_engine
from .kernels import Kernel, compile_spec
from .likelihoods import Gaussian
from .parameter import Parameter


class GPR:
    """Exact GP regression with a Gaussian likelihood and a zero mean function."""

    def __init__(self, data: Tuple, kernel: Kernel, mean_function=None,
                 noise_variance: Optional[float] = None, likelihood: Optional[Gaussian] = None,
                 device: Optional[int] = None):
        if mean_function is not None:
            raise NotImplementedError("only the zero mean function (GPflow default) is supported")
        X, Y = data
        self._out_cpu = not (isinstance(Y, torch.Tensor) and Y.is_cuda)
        Xt = X if isinstance(X, torch.Tensor) else torch.as_tensor(np.asarray(X, dtype=np.float64))
        Yt = Y if isinstance(Y, torch.Tensor) else torch.as_tensor(np.asarray(Y, dtype=np.float64))
        Xt = Xt.to(torch.float64)
        Yt = Yt.to(torch.float64)
        if Xt.ndim == 1:
            Xt = Xt[:, None]
        if Yt.ndim == 1:
            Yt = Yt[:, None]
        if Yt.shape[1] != 1:
            raise NotImplementedError("single-output GPR only (Y must be [N, 1])")
        if Xt.shape[0] != Yt.shape[0]:
            raise ValueError("X and Y must have the same number of rows")
        if Xt.shape[0] == 0:
            # GPflow would return the prior; the device engine needs at least one training point
            # (an empty factorisation has nothing to run on the GPU), so refuse it up front
            raise ValueError("GPR needs at least one training point (X has 0 rows)")
        self.data = (Xt, Yt)
        self.kernel = kernel
        if likelihood is None:
            likelihood = Gaussian(1.0 if noise_variance is None else noise_variance)
        elif noise_variance is not None:
            raise ValueError("give either noise_variance or likelihood")
        self.likelihood = likelihood
        self.mean_function = None
        self.num_latent_gps = 1
        self.device = default_device() if device is None else int(device)
        self._spec = compile_spec(kernel, Xt.shape[1])
        self._engine: Optional[Engine] = None
        self._engine_index = 0

    # ---------------------------------------------------------------- structure -------
    @property
    def parameters(self) -> Tuple[Parameter, ...]:
        # GPR attributes sorted: kernel < likelihood (< mean_function, which has none here)
        return tuple(self.kernel.parameters) + tuple(self.likelihood.parameters)

    @property
    def trainable_parameters(self) -> Tuple[Parameter, ...]:
        return tuple(p for p in self.parameters if p.trainable)

    @property
    def trainable_variables(self):
        return tuple(p.unconstrained_variable for p in self.trainable_parameters)

    def _param_paths(self):
        return ([("GPR.kernel." + n if n else "GPR.kernel", p) for n, p in self.kernel._param_paths("")]
                + [("GPR.likelihood.variance", self.likelihood.variance)])

    @property
    def n_kernel_params(self) -> int:
        return int(self._spec.n_params)

    def theta_row(self) -> np.ndarray:
        """Constrained θ in the gpx layout: kernel params, then σn² at index n_params."""
        row = np.ones(N.GPX_THETA_STRIDE, dtype=np.float64)
        kp = self.kernel.parameters
        for i, p in enumerate(kp):
            row[i] = p.value
        row[len(kp)] = self.likelihood.variance.value
        return row

    # ---------------------------------------------------------------- engine ----------
    def _attach(self, engine: Engine, index: int) -> None:
        self._engine, self._engine_index = engine, index

    def engine(self) -> Tuple[Engine, int]:
        """(engine, slot): the batch engine this model was attached to, else a pooled
        single-problem engine for its shape (engine.solo_engine)."""
        if self._engine is None:
            return solo_engine(self), 0
        return self._engine, self._engine_index

    def _wrap(self, t: torch.Tensor) -> torch.Tensor:
        t = t.reshape(-1, 1)
        return t.cpu() if self._out_cpu else t

    # ---------------------------------------------------------------- objective -------
    def _lml_and_grad_theta(self):
        eng, b = self.engine()
        row = self.theta_row()
        lml, grad, info = eng.lml_grad_row(b, row)
        if info == N.INFO_BAD_THETA:
            raise N.InvalidParameterError(f"hyperparameters out of (0, inf): {row[:eng.n_params[b] + 1]}")
        if info != 0:
            raise N.NotPositiveDefiniteError(
                f"Cholesky decomposition was not successful: pivot {int(info)} of K + noise I "
                "is not positive", info)
        return lml, grad

    def log_marginal_likelihood(self) -> torch.Tensor:
        return torch.tensor(self._lml_and_grad_theta()[0], dtype=torch.float64)

    def maximum_log_likelihood_objective(self) -> torch.Tensor:
        return self.log_marginal_likelihood()

    def training_loss(self) -> torch.Tensor:
        """−logML (no priors), the closure GPR/model_trainer.py:19 hands to Scipy."""
        return -self.log_marginal_likelihood()

    def training_loss_closure(self, compile: bool = True):
        def closure():
            return self.training_loss()
        closure._gpx_model = self
        return closure

    def _variable_map(self, variables):
        """(variables, θ-row index of each variable, its Parameter), cached for the variables
        object an optimiser passes on every call (kernel parameters, then σn² at n_params)."""
        cache = getattr(self, "_grad_map", None)
        if cache is None or cache[0] is not variables:
            pindex = {id(p): i for i, p in enumerate(self.kernel.parameters)}
            nk = len(self.kernel.parameters)
            rows = []
            for v in variables:
                p = v._param
                if p is self.likelihood.variance:
                    rows.append(nk)
                elif id(p) in pindex:
                    rows.append(pindex[id(p)])
                else:
                    raise ValueError(f"variable {v.name} is not a parameter of this model")
            cache = self._grad_map = (variables, rows, [v._param for v in variables])
        return cache

    def theta_layout(self, variables):
        """(cols int32 [P], lower float64 [P]): θ-row index and Shift of each variable, for the
        batched driver's native θ / chain-rule helpers (gpx_host_theta_rows / _loss_grad_u)."""
        _, rows, params = self._variable_map(variables)
        return (np.asarray(rows, dtype=np.int32), np.asarray([p.lower for p in params], dtype=np.float64))

    def loss_and_grad_unconstrained(self, variables=None, lml=None, grad_theta=None):
        """(−logML, ∂(−logML)/∂u) for ``variables`` (default: trainable_variables)."""
        if lml is None:
            lml, grad_theta = self._lml_and_grad_theta()
        variables = self.trainable_variables if variables is None else variables
        _, rows, params = self._variable_map(variables)
        g = np.empty(len(rows), dtype=np.float64)
        for k, (r, p) in enumerate(zip(rows, params)):
            g[k] = -grad_theta[r] * p.dtheta_du()
        return -float(lml), g

    # ---------------------------------------------------------------- prediction ------
    def predict_f(self, Xnew, full_cov: bool = False, full_output_cov: bool = False):
        """Posterior of the latent f: mean [N*,1] and var [N*,1], or with full_cov the
        covariance [1,N*,N*] (GPflow's layout with one latent GP; full_output_cov changes
        nothing for a single output)."""
        return self._predict(Xnew, add_noise=False, full_cov=full_cov)

    def predict_y(self, Xnew, full_cov: bool = False, full_output_cov: bool = False):
        if full_cov or full_output_cov:
            # GPflow 2.9 GPModel.predict_y raises for these too
            raise NotImplementedError("The predict_y method currently supports only the argument "
                                      "values full_cov=False and full_output_cov=False")
        return self._predict(Xnew, add_noise=True)

    def _predict(self, Xnew, add_noise: bool, full_cov: bool = False):
        eng, b = self.engine()
        theta = np.ones((eng.B, N.GPX_THETA_STRIDE))
        theta[b] = self.theta_row()
        cpu_out = not (isinstance(Xnew, torch.Tensor) and Xnew.is_cuda)
        m, v, _ = eng.predict([b], theta, [Xnew], add_noise, full_cov=full_cov)
        m = m[0].reshape(-1, 1)
        v = v[0].unsqueeze(0) if full_cov else v[0].reshape(-1, 1)
        if cpu_out:
            m, v = m.cpu(), v.cpu()
        return m, v


def predict_f_batch(models: Sequence[GPR], Xnews: Sequence, add_noise: bool = False):
    """predict_f (or predict_y) for several models sharing one engine, in one device pass.
    Models not attached to a shared batch engine are predicted one by one."""
    if any(m._engine is None for m in models):
        return [(m.predict_y(x) if add_noise else m.predict_f(x)) for m, x in zip(models, Xnews)]
    eng, _ = models[0].engine()
    idx = []
    for m in models:
        e, b = m.engine()
        if e is not eng:
            raise ValueError("models must share an engine (fit them with Scipy().minimize_batch)")
        idx.append(b)
    theta = np.ones((eng.B, N.GPX_THETA_STRIDE))
    for m, b in zip(models, idx):
        theta[b] = m.theta_row()
    ms, vs, _ = eng.predict(idx, theta, Xnews, add_noise)
    out = []
    for x, m, v in zip(Xnews, ms, vs):
        cpu_out = not (isinstance(x, torch.Tensor) and x.is_cuda)
        m, v = m.reshape(-1, 1), v.reshape(-1, 1)
        out.append((m.cpu(), v.cpu()) if cpu_out else (m, v))
    return out


class SVGP:
    """gpflow.models.SVGP with a Gaussian likelihood and GPflow's defaults (whiten=True, full
    q_sqrt, zero mean, one latent GP) — the cells at test_scripts/SVGP.py:461-478 and
    test_scripts/GPR.py:118-138::

        m = SVGP(kernel=k, likelihood=Gaussian(variance=1e-4), inducing_variable=Z, num_data=N)
        set_trainable(m.likelihood.variance, False)
        Scipy().minimize(m.training_loss_closure((X, Y)), m.trainable_variables,
                         options=dict(maxiter=100))
        mean, var = m.predict_f(X_test)

    ELBO, gradients and predictions come from libgpx.so (gpx_svgp_*); trainable variables
    are ordered as tf.Module flattens SVGP: inducing_variable.Z, kernel.*, likelihood.variance,
    q_mu, q_sqrt (FillTriangular-unconstrained)."""

    def __init__(self, kernel: Kernel, likelihood: Gaussian, inducing_variable, *, mean_function=None,
                 num_latent_gps: int = 1, q_diag: bool = False, q_mu=None, q_sqrt=None,
                 whiten: bool = True, num_data: Optional[int] = None, device: Optional[int] = None):
        from .inducing_variables import InducingPoints
        from .parameter import ArrayParameter
        if mean_function is not None:
            raise NotImplementedError("only the zero mean function (GPflow default) is supported")
        if num_latent_gps != 1 or q_diag or not whiten:
            raise NotImplementedError("SVGP supports GPflow's defaults: one latent GP, full q_sqrt, whiten=True")
        if not isinstance(likelihood, Gaussian):
            raise NotImplementedError("SVGP supports the Gaussian likelihood")
        self.kernel = kernel
        self.likelihood = likelihood
        self.inducing_variable = (inducing_variable if isinstance(inducing_variable, InducingPoints)
                                  else InducingPoints(inducing_variable))
        M = self.inducing_variable.num_inducing
        self.num_data = num_data
        self.num_latent_gps = 1
        self.whiten = True
        self.q_mu = ArrayParameter(np.zeros((M, 1)) if q_mu is None else np.asarray(q_mu).reshape(M, 1),
                                   name="q_mu")
        self.q_sqrt = ArrayParameter(np.eye(M)[None] if q_sqrt is None else q_sqrt,
                                     transform="triangular", name="q_sqrt")
        self.device = default_device() if device is None else int(device)
        self._engines = {}

    # ---------------------------------------------------------------- structure -------
    @property
    def parameters(self):
        return ((self.inducing_variable.Z,) + tuple(self.kernel.parameters)
                + tuple(self.likelihood.parameters) + (self.q_mu, self.q_sqrt))

    @property
    def trainable_parameters(self):
        return tuple(p for p in self.parameters if p.trainable)

    @property
    def trainable_variables(self):
        return tuple(p.unconstrained_variable for p in self.trainable_parameters)

    def _param_paths(self):
        return ([("SVGP.inducing_variable.Z", self.inducing_variable.Z)]
                + [("SVGP.kernel." + n if n else "SVGP.kernel", p) for n, p in self.kernel._param_paths("")]
                + [("SVGP.likelihood.variance", self.likelihood.variance),
                   ("SVGP.q_mu", self.q_mu), ("SVGP.q_sqrt", self.q_sqrt)])

    @property
    def M(self) -> int:
        return self.inducing_variable.num_inducing

    def theta_row(self) -> np.ndarray:
        row = np.ones(N.GPX_THETA_STRIDE, dtype=np.float64)
        kp = self.kernel.parameters
        for i, p in enumerate(kp):
            row[i] = p.value
        row[len(kp)] = self.likelihood.variance.value
        return row

    def _state(self):
        return (self.theta_row(), self.inducing_variable.Z.value, self.q_mu.value.reshape(-1),
                self.q_sqrt.value[0])

    # ---------------------------------------------------------------- engine ----------
    def engine(self, data=None) -> "SVGPEngine":
        from .engine import SVGPEngine
        if data is None:
            if self._engines:
                return next(iter(self._engines.values()))[0]
            Z = self.inducing_variable.Z.value
            data = (Z[:1], np.zeros((1, 1)))
        X, Y = data
        key = (id(X), id(Y))
        hit = self._engines.get(key)
        if hit is None or hit[1] is not X or hit[2] is not Y:
            Xa = X if isinstance(X, torch.Tensor) else np.asarray(X, dtype=np.float64)
            n = int(Xa.shape[0])
            D = 1 if Xa.ndim == 1 else int(Xa.shape[1])
            eng = SVGPEngine(X, Y, compile_spec(self.kernel, D), self.M,
                             num_data=float(self.num_data if self.num_data is not None else n),
                             device=self.device)
            hit = (eng, X, Y)
            self._engines = {key: hit}
        return hit[0]

    # ---------------------------------------------------------------- objective -------
    def _elbo_and_grads(self, data):
        eng = self.engine(data)
        return eng.elbo_grad(*self._state())

    def elbo(self, data) -> torch.Tensor:
        return torch.tensor(self._elbo_and_grads(data)[0], dtype=torch.float64)

    def maximum_log_likelihood_objective(self, data) -> torch.Tensor:
        return self.elbo(data)

    def training_loss(self, data) -> torch.Tensor:
        return -self.elbo(data)

    def training_loss_closure(self, data, compile: bool = True):
        def closure():
            return self.training_loss(data)
        closure._gpx_model = self
        closure._gpx_loss_and_grad = lambda variables=None: self.loss_and_grad_unconstrained(data, variables)
        return closure

    def grads_to_unconstrained(self, variables, elbo, gth, gZ, gq, gR):
        """(−ELBO, ∂(−ELBO)/∂u flattened in ``variables`` order)."""
        kp = self.kernel.parameters
        pindex = {id(p): i for i, p in enumerate(kp)}
        parts = []
        for v in variables:
            p = v._param
            if p is self.inducing_variable.Z:
                parts.append(-np.asarray(gZ).ravel())
            elif p is self.likelihood.variance:
                parts.append(np.array([-gth[len(kp)] * p.dtheta_du()]))
            elif id(p) in pindex:
                parts.append(np.array([-gth[pindex[id(p)]] * p.dtheta_du()]))
            elif p is self.q_mu:
                parts.append(-np.asarray(gq).ravel())
            elif p is self.q_sqrt:
                parts.append(-p.grad_to_unconstrained(gR).ravel())
            else:
                raise ValueError(f"variable {v.name} is not a parameter of this model")
        return -float(elbo), np.concatenate(parts)

    def loss_and_grad_unconstrained(self, data, variables=None):
        variables = self.trainable_variables if variables is None else variables
        return self.grads_to_unconstrained(variables, *self._elbo_and_grads(data))

    # ---------------------------------------------------------------- prediction ------
    def predict_f(self, Xnew, full_cov: bool = False, full_output_cov: bool = False):
        if full_cov or full_output_cov:
            raise NotImplementedError("SVGP.predict_f supports full_cov=False (marginals)")
        return self._predict(Xnew, False)

    def predict_y(self, Xnew, full_cov: bool = False, full_output_cov: bool = False):
        if full_cov or full_output_cov:
            raise NotImplementedError("The predict_y method currently supports only the argument "
                                      "values full_cov=False and full_output_cov=False")
        return self._predict(Xnew, True)

    def _predict(self, Xnew, add_noise: bool):
        cpu_out = not (isinstance(Xnew, torch.Tensor) and Xnew.is_cuda)
        m, v = self.engine().predict(*self._state(), Xnew, add_noise)
        m, v = m.reshape(-1, 1), v.reshape(-1, 1)
        if cpu_out:
            m, v = m.cpu(), v.cpu()
        return m, v
