"""Counterparts of the reference's callers of the GP hot path, batched on the device.

* ``ModelTrainer.train_model`` — GPR/model_trainer.py:10-26: for each kernel, GPR with the
  noise fixed at 1e-5, L-BFGS-B maxiter=100, predict_f at the training X, keep the minimum
  training MSE (strict ``<``, first wins). Here the kernel fits run concurrently in one
  lock-step batch; each is the same scipy trajectory it would be alone. Kernel objects are
  shared across calls exactly as in the reference (later fits warm-start from the
  previous optimum and earlier best models alias the mutated kernels).
* ``Predictor`` — GPR/predictor.py:4-51 (predict_single; predict_combined and
  upsample_predictions as host post-processing).
* ``MultiInputTrainer`` — Multi-Input_GPR/models/model_trainer.py:17-72 (train_model,
  train_likelihood with 4 noise restarts picking the lowest opt_logs.fun, train_best_model).
* ``BlendOptimizer`` — GPR/optimizer.py:5-28 (the α/β SLSQP of the timeframe blend).
* ``refit_steps`` — Multi-Input_GPR/main.py:414-456 (run_step_4's refit loop), batched.
"""
from __future__ import annotations

from copy import deepcopy
from typing import List, Optional, Sequence

import numpy as np
import torch

from . import models as M
from .optimizers import Scipy
from .utilities import print_summary, set_trainable


def _np(a) -> np.ndarray:
    if isinstance(a, torch.Tensor):
        return a.detach().cpu().numpy()
    return np.asarray(a)


def mean_squared_error(y_true, y_pred) -> float:
    """sklearn.metrics.mean_squared_error for [N,1] arrays (GPR/model_trainer.py:21)."""
    a, b = _np(y_true).reshape(len(_np(y_true)), -1), _np(y_pred).reshape(len(_np(y_pred)), -1)
    return float(np.average((a - b) ** 2, axis=0).mean())


class ModelTrainer:
    def __init__(self, kernel_combinations: Sequence, device: Optional[int] = None):
        self.kernel_combinations = list(kernel_combinations)
        self.device = device
        self.last_results = []
        self.last_models = []

    def train_model(self, X_tf, Y_tf, maxiter: int = 100):
        models = []
        for kernel in self.kernel_combinations:
            model = M.GPR(data=(X_tf, Y_tf), kernel=kernel, device=self.device)
            model.likelihood.variance.assign(1e-5)
            set_trainable(model.likelihood.variance, False)
            models.append(model)
        self.last_results = Scipy().minimize_batch(models, options=dict(maxiter=maxiter))
        self.last_models = models
        preds = M.predict_f_batch(models, [m.data[0] for m in models])
        best_kernel, best_mse, best_model = None, float("inf"), None
        for kernel, model, (mean, _) in zip(self.kernel_combinations, models, preds):
            mse = mean_squared_error(Y_tf, _np(mean))
            if mse < best_mse:
                best_mse, best_kernel, best_model = mse, kernel, model
        return best_kernel, best_mse, best_model


class Predictor:
    def predict_single(self, model, X):
        f_mean, f_var = model.predict_f(X, full_cov=False)
        y_mean, y_var = model.predict_y(X)
        return f_mean, f_var, y_mean, y_var

    def predict_combined(self, alpha, beta, daily_model, weekly_model, monthly_model, X_daily, X_weekly,
                         X_monthly):
        fd, vd, yd, yvd = self.predict_single(daily_model, X_daily)
        fw, vw, yw, yvw = self.predict_single(weekly_model, X_weekly)
        fm, vm, ym, yvm = self.predict_single(monthly_model, X_monthly)
        up = self.upsample_predictions
        fw, fm = up(X_daily, X_weekly, fw, "w"), up(X_daily, X_monthly, fm, "m")
        vw, vm = up(X_daily, X_weekly, vw, "w"), up(X_daily, X_monthly, vm, "m")
        yw, ym = up(X_daily, X_weekly, yw, "w"), up(X_daily, X_monthly, ym, "m")
        yvw, yvm = up(X_daily, X_weekly, yvw, "w"), up(X_daily, X_monthly, yvm, "m")
        g = 1.0 - alpha - beta
        return (alpha * fd + beta * fw + g * fm, alpha * vd + beta * vw + g * vm,
                alpha * yd + beta * yw + g * ym, alpha * yvd + beta * yvw + g * yvm)

    def upsample_predictions(self, X_daily_tf, X_tf, predictions, period="d"):
        """pandas Series(pred, index=X).reindex(X_daily).interpolate('linear') — positional
        linear interpolation over the reindexed rows, leading NaNs kept (GPR/predictor.py:35-51)."""
        if period not in ("w", "m"):
            return predictions
        import pandas as pd

        xd = _np(X_daily_tf).reshape(-1)
        xs = _np(X_tf).reshape(-1)
        p = _np(predictions).reshape(-1)
        s = pd.Series(p, index=xs).reindex(xd).interpolate(method="linear")
        return torch.as_tensor(s.values.reshape(-1, 1), dtype=torch.float64)


class BlendOptimizer:
    """Timeframe-blend weights (GPR/optimizer.py:5-28): SLSQP over (α, β) ∈ [0,1]², α + β ≤ 1,
    from (0.33, 0.33), minimising MSE(Y, α·f_d + β·f_w + (1−α−β)·f_m) + λ(|α| + |β|). Host
    code: two variables, evaluated on the blended device predictions."""

    def __init__(self, lambda_: float = 0.01):
        self.lambda_ = float(lambda_)
        self.initial_weights = [0.33, 0.33]
        self.bounds = [(0, 1), (0, 1)]
        self.constraints = {"type": "ineq", "fun": lambda w: 1 - sum(w)}

    def loss_fn(self, weights, Y, f_daily, f_weekly, f_monthly) -> float:
        a, b = weights
        y = _np(Y).reshape(len(_np(Y)), -1)
        blend = a * _np(f_daily) + b * _np(f_weekly) + (1.0 - a - b) * _np(f_monthly)
        return mean_squared_error(y, blend.reshape(y.shape)) + self.lambda_ * (abs(a) + abs(b))

    def optimize_weights(self, Y_tf, f_mean_daily, f_mean_weekly, f_mean_monthly) -> np.ndarray:
        import scipy.optimize
        res = scipy.optimize.minimize(
            lambda w: self.loss_fn(w, Y_tf, f_mean_daily, f_mean_weekly, f_mean_monthly),
            self.initial_weights, method="SLSQP", bounds=self.bounds, constraints=self.constraints)
        return res.x


class MultiInputTrainer:
    """Multi-Input_GPR/models/model_trainer.py (methods callable without an instance, as the
    reference calls them: ``ModelTrainer.train_model(model)``)."""

    def __init__(self, kernel_combinations: Sequence = ()):
        self.kernel_combinations = list(kernel_combinations)

    @staticmethod
    def train_model(model, verbose: bool = True):
        set_trainable(model.likelihood, False)
        Scipy().minimize(model.training_loss, model.trainable_variables)
        if verbose:
            print_summary(model)
        return model

    @staticmethod
    def train_likelihood(X, Y, composite_kernel, starting_variances=(1e-5, 1e-3, 1e-1, 1.0),
                         verbose: bool = True):
        """Four restarts with trainable noise, run as one lock-step batch; lowest final loss wins
        (strict ``<``, first wins, as Multi-Input_GPR/models/model_trainer.py:42-45)."""
        models = []
        for v in starting_variances:
            m = M.GPR((X, Y), kernel=deepcopy(composite_kernel), noise_variance=v)
            set_trainable(m.likelihood, True)
            models.append(m)
        logs = Scipy().minimize_batch(models)
        best_model, best_loss = None, float("inf")
        for m, r in zip(models, logs):
            if r.fun < best_loss:
                best_model, best_loss = m, r.fun
        if verbose:
            print("\nBest model:")
            print_summary(best_model)
            print(f"Best loss: {best_loss}")
        return best_model

    def train_best_model(self, X_tf, Y_tf):
        return ModelTrainer(self.kernel_combinations).train_model(X_tf, Y_tf)


def refit_steps(X_full, Y_full, n_train: int, composite_kernels: Sequence, is_fixed: bool = True,
                mean: float = 0.0, std: float = 1.0, noise_variance: float = 1e-3,
                starting_variances=(1e-5, 1e-3, 1e-1, 1.0)):
    """The iterative refit of Multi-Input_GPR/main.py:414-456 (``run_step_4``), batched.

    For every step i in [n_train, len(Y_full)) and every composite kernel, the reference fits a
    fresh GPR (``deepcopy(kernel)``) on the first i rows — noise fixed at 1e-3 and
    ``ModelTrainer.train_model`` (scipy defaults, no maxiter) when ``is_fixed``, else the
    4-restart ``train_likelihood`` — keeps the model of the LAST kernel of the loop, predicts
    f at the first i+1 rows and keeps the last row, de-normalised (mean·std + μ, var·std²).
    All (step × kernel × restart) fits are independent: here they run as ONE lock-step batch
    (ragged N = n_train … len−1), each the same scipy trajectory it would be alone.

    Returns (f_means, f_vars, actual_returns): lists of [1]-arrays, as run_step_4's first
    three outputs.
    """
    X_full = _np(X_full)
    Y_full = _np(Y_full).reshape(-1, 1)
    steps = list(range(n_train, len(Y_full)))
    kernels = list(composite_kernels)
    if not steps or not kernels:
        return [], [], []
    starts = [noise_variance] if is_fixed else list(starting_variances)
    models, index = [], []
    for si, i in enumerate(steps):
        for ki, k in enumerate(kernels):
            for v in starts:
                m = M.GPR((X_full[:i], Y_full[:i]), kernel=deepcopy(k), noise_variance=v)
                set_trainable(m.likelihood, not is_fixed)
                models.append(m)
                index.append((si, ki))
    logs = Scipy().minimize_batch(models)
    # per step: the last kernel's model (best restart by final loss, strict <, first wins)
    chosen = []
    for si in range(len(steps)):
        best, best_loss = None, float("inf")
        for m, r, (s, k) in zip(models, logs, index):
            if s == si and k == len(kernels) - 1 and r.fun < best_loss:
                best, best_loss = m, r.fun
        chosen.append(best)
    preds = M.predict_f_batch(chosen, [X_full[: i + 1] for i in steps])
    f_means, f_vars, actual = [], [], []
    for i, (fm, fv) in zip(steps, preds):
        fm, fv = _np(fm), _np(fv)
        f_means.append(fm[-1] * std + mean)
        f_vars.append(fv[-1] * std ** 2)
        actual.append(Y_full[i] * std + mean)
    return f_means, f_vars, actual
