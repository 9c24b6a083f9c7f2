/*
 * gpx_host_math.c — host-side helpers of the stepped L-BFGS-B driver (portfoliooptgp_amd/
 * optimizers.py): the softplus transform of the unconstrained variables into θ rows and the
 * chain rule of ∂logML/∂θ back to ∂loss/∂u, for every fit of a round in one call.
 *
 * GPflow 2.9.1 semantics (gpflow.optimizers.Scipy over softplus-transformed parameters,
 * GPR/model_trainer.py:18-19): θ = lower + softplus(u), ∂θ/∂u = sigmoid(u). The arithmetic is
 * exactly that of portfoliooptgp_amd/parameter.py (softplus = numpy's npy_logaddexp(0, u) with
 * libm exp/log1p; sigmoid = 0.5(1 + tanh(u/2))): the same libm functions in the same order, so a
 * fit's trajectory does not depend on which path computed its θ. Built with gcc -O2
 * -fno-builtin (no constant folding or vectorised libm variants).
 */
#include <math.h>
#include <stdint.h>

#include "../../include/gpx.h"

static double gpx_softplus(double u) {
  if (u == 0.0) return log(2.0);
  if (u < 0.0) return log1p(exp(u));
  if (u > 0.0) return u + log1p(exp(-u));
  return u; /* nan */
}

static double gpx_sigmoid(double u) { return 0.5 * (1.0 + tanh(0.5 * u)); }

int gpx_host_theta_rows(int n_fits, int n_vars, const double* u, const int32_t* rows,
                        const int32_t* cols, const double* lower, double* theta) {
  if (n_fits < 0 || n_vars < 0 || n_vars > GPX_THETA_STRIDE || (n_fits > 0 && (!u || !rows || !cols || !lower || !theta)))
    return GPX_BAD_ARG;
  for (int k = 0; k < n_fits; ++k) {
    double* th = theta + (int64_t)rows[k] * GPX_THETA_STRIDE;
    for (int v = 0; v < n_vars; ++v) th[cols[v]] = lower[v] + gpx_softplus(u[(int64_t)k * n_vars + v]);
  }
  return GPX_OK;
}

int gpx_host_loss_grad_u(int n_fits, int n_vars, const double* u, const int32_t* rows,
                         const int32_t* cols, const double* lml, const double* grad, double* loss,
                         double* grad_u) {
  if (n_fits < 0 || n_vars < 0 || n_vars > GPX_THETA_STRIDE ||
      (n_fits > 0 && (!u || !rows || !cols || !lml || !grad || !loss || !grad_u)))
    return GPX_BAD_ARG;
  for (int k = 0; k < n_fits; ++k) {
    const int64_t b = rows[k];
    loss[k] = -lml[b];
    for (int v = 0; v < n_vars; ++v)
      grad_u[(int64_t)k * n_vars + v] = -grad[b * GPX_THETA_STRIDE + cols[v]] * gpx_sigmoid(u[(int64_t)k * n_vars + v]);
  }
  return GPX_OK;
}
