// gpx_kfun.h — device-side covariance functions and their θ-derivatives.
//
// Restates the GPflow 2.9.1 kernels the reference builds at GPR/main.py:105-114 and
// Multi-Input_GPR/main.py:118-135 (formulas: SURVEY.md §8 a3). Distances are taken as direct
// differences Σ_d (x_d - x'_d)² (GPflow expands ‖x‖²+‖x'‖²-2x·x'; the two agree to rounding),
// and the K_r kernels use r = sqrt(max(r², 1e-36)) with zero r-gradient where clamped, as
// GPflow's IsotropicStationary.K_r2 does.
#pragma once
#include <hip/hip_runtime.h>
#include "../../include/gpx.h"

namespace gpx {

constexpr int kMaxParams = GPX_THETA_STRIDE;  // kernel params + noise

struct DevSpec {
  int n_terms, combine, n_params, reserved;
  gpx_term terms[GPX_MAX_TERMS];
};

__device__ __forceinline__ int term_nparams(int kind) {
  switch (kind) {
    case GPX_RQ: case GPX_PERIODIC_SE: return 3;
    case GPX_LINEAR: return 1;
    default: return 2;
  }
}

// Value and derivatives (w.r.t. the term's own params, GPflow order) of one term.
template <bool GRAD>
__device__ __forceinline__ double eval_term(const gpx_term& t, const double* __restrict__ th,
                                            const double* __restrict__ xi,
                                            const double* __restrict__ xj, double* dk) {
  const int d0 = t.dim_start, dn = t.dim_count;
  switch (t.kind) {
    case GPX_LINEAR: {
      double s = 0.0;
      for (int d = 0; d < dn; ++d) s = fma(xi[d0 + d], xj[d0 + d], s);
      if (GRAD) dk[0] = s;
      return th[0] * s;
    }
    case GPX_PERIODIC_SE: {
      const double ell = th[0], var = th[1], p = th[2];
      const double inv_l2 = 1.0 / (ell * ell);
      double s2 = 0.0, sc = 0.0;
      for (int d = 0; d < dn; ++d) {
        const double diff = xi[d0 + d] - xj[d0 + d];
        double sn, cs;
        sincos(M_PI * diff / p, &sn, &cs);
        s2 = fma(sn, sn, s2);
        if (GRAD) sc = fma(sn * cs, diff, sc);
      }
      s2 *= inv_l2;
      const double g = exp(-0.5 * s2);
      if (GRAD) {
        dk[0] = var * g * s2 / ell;
        dk[1] = g;
        dk[2] = var * g * (M_PI * sc * inv_l2 / (p * p));
      }
      return var * g;
    }
    default: break;
  }
  // isotropic stationary kernels
  const bool rq = (t.kind == GPX_RQ);
  const double ell = rq ? th[1] : th[0];
  const double var = rq ? th[2] : th[1];
  double d2 = 0.0;
  for (int d = 0; d < dn; ++d) {
    const double diff = xi[d0 + d] - xj[d0 + d];
    d2 = fma(diff, diff, d2);
  }
  const double r2 = d2 / (ell * ell);
  switch (t.kind) {
    case GPX_SE: {
      const double g = exp(-0.5 * r2);
      if (GRAD) { dk[0] = var * g * r2 / ell; dk[1] = g; }
      return var * g;
    }
    case GPX_RQ: {
      const double a = th[0];
      const double b = 1.0 + 0.5 * r2 / a;
      const double lb = log(b);
      const double g = exp(-a * lb);
      if (GRAD) {
        dk[0] = var * g * (-lb + 0.5 * r2 / (a * b));
        dk[1] = var * (g / b) * r2 / ell;
        dk[2] = g;
      }
      return var * g;
    }
    default: break;
  }
  const bool clamped = !(r2 > 1e-36);
  const double r = sqrt(clamped ? 1e-36 : r2);
  double g, dgdr;
  switch (t.kind) {
    case GPX_MATERN12: { g = exp(-r); dgdr = -g; break; }
    case GPX_EXPONENTIAL: { g = exp(-0.5 * r); dgdr = -0.5 * g; break; }
    case GPX_MATERN32: {
      const double s = 1.7320508075688772;  // sqrt(3)
      const double e = exp(-s * r);
      g = (1.0 + s * r) * e;
      dgdr = -3.0 * r * e;
      break;
    }
    default: {  // GPX_MATERN52
      const double s = 2.23606797749979;  // sqrt(5)
      const double e = exp(-s * r);
      g = (1.0 + s * r + (5.0 / 3.0) * r * r) * e;
      dgdr = -(5.0 / 3.0) * r * (1.0 + s * r) * e;
      break;
    }
  }
  if (GRAD) {
    // dr/dℓ = -r/ℓ; zero where the 1e-36 clamp is active
    dk[0] = clamped ? 0.0 : var * dgdr * (-r / ell);
    dk[1] = g;
  }
  return var * g;
}

// K(xi, xj) for a full spec.
__device__ __forceinline__ double eval_k(const DevSpec& s, const double* __restrict__ th,
                                         const double* __restrict__ xi,
                                         const double* __restrict__ xj) {
  double acc = (s.combine == GPX_PRODUCT && s.n_terms > 1) ? 1.0 : 0.0;
  for (int t = 0; t < s.n_terms; ++t) {
    const double v = eval_term<false>(s.terms[t], th + s.terms[t].param_offset, xi, xj, nullptr);
    if (s.combine == GPX_PRODUCT && s.n_terms > 1) acc *= v; else acc += v;
  }
  return acc;
}

// K(xi, xj) and its derivatives, kept per term in statically indexed registers:
// dk[t][q] = dK/dθ for parameter q of term t (θ index terms[t].param_offset + q).
template <int NT = GPX_MAX_TERMS>
__device__ __forceinline__ double eval_k_grad(const DevSpec& s, const double* __restrict__ th,
                                              const double* __restrict__ xi,
                                              const double* __restrict__ xj,
                                              double (&dk)[NT][3]) {
  const bool prod = (NT > 1 && s.combine == GPX_PRODUCT && s.n_terms > 1);
  double vals[NT];
  double acc = prod ? 1.0 : 0.0;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    dk[t][0] = dk[t][1] = dk[t][2] = 0.0;
    vals[t] = 1.0;
    if (t < s.n_terms) {
      vals[t] = eval_term<true>(s.terms[t], th + s.terms[t].param_offset, xi, xj, dk[t]);
      if (prod) acc *= vals[t]; else acc += vals[t];
    }
  }
  if (prod) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      double others = 1.0;
#pragma unroll
      for (int u = 0; u < NT; ++u) if (u != t) others *= vals[u];
      dk[t][0] *= others; dk[t][1] *= others; dk[t][2] *= others;
    }
  }
  return acc;
}

// K_diag(x): σ² for stationary terms, σ² Σ x² for Linear.
__device__ __forceinline__ double eval_kdiag(const DevSpec& s, const double* __restrict__ th,
                                             const double* __restrict__ x) {
  return eval_k(s, th, x, x);
}

}  // namespace gpx
