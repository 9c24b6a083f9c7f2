// gpx_kfun.h — device-side covariance functions and their θ-derivatives.
//
// Restates the GPflow 2.9.1 kernels the reference builds at GPR/main.py:105-114 and
// Multi-Input_GPR/main.py:118-135 (formulas: SURVEY.md §8 a3). Squared distances are formed the
// way GPflow forms them (Stationary.scale divides by ℓ, then utilities.ops.square_distance
// expands): a = x/ℓ, b = x'/ℓ, r² = (−2·(a·b)) + (‖a‖² + ‖b‖²), each operation rounded on its own
// (no FMA contraction), sums over d in order — the same arithmetic as oracle/gp_oracle.py
// scaled_sqdist. The K_r kernels use r = sqrt(max(r², 1e-36)) with zero r-gradient where
// clamped, as GPflow's IsotropicStationary.K_r2 does.
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

// GPflow's square_distance of two points already scaled by 1/ℓ (a, b: dn values each):
// (−2·Σ a_d b_d) + (Σ a_d² + Σ b_d²), every product and sum rounded separately.
__device__ __forceinline__ double sqdist_scaled(const double* __restrict__ a, const double* __restrict__ b,
                                                int dn) {
#pragma clang fp contract(off)
  double dot = a[0] * b[0], sa = a[0] * a[0], sb = b[0] * b[0];
  for (int d = 1; d < dn; ++d) {
    dot = dot + a[d] * b[d];
    sa = sa + a[d] * a[d];
    sb = sb + b[d] * b[d];
  }
  return -2.0 * dot + (sa + sb);
}
// the same for one active dimension: a = x/ℓ, b = x'/ℓ given
__device__ __forceinline__ double sqdist1(double a, double b) {
#pragma clang fp contract(off)
  return -2.0 * (a * b) + (a * a + b * b);
}
// sqdist1(a, b) from b's −2b and b², computed once per column: the same bits (a·(−2b) is
// −2·(a·b) exactly, a power-of-two scaling commuting with the rounding)
__device__ __forceinline__ double sqdist1_b(double a, double m2b, double b2) {
#pragma clang fp contract(off)
  return a * m2b + (a * a + b2);
}
// raw inputs: scale by 1/ℓ (a division, as Stationary.scale) on the fly
__device__ __forceinline__ double sqdist_gpflow(const double* __restrict__ xi, const double* __restrict__ xj,
                                                int dn, double ell) {
#pragma clang fp contract(off)
  double a = xi[0] / ell, b = xj[0] / ell;
  double dot = a * b, sa = a * a, sb = b * b;
  for (int d = 1; d < dn; ++d) {
    a = xi[d] / ell;
    b = xj[d] / ell;
    dot = dot + a * b;
    sa = sa + a * a;
    sb = sb + b * b;
  }
  return -2.0 * dot + (sa + sb);
}

// Value and derivatives (w.r.t. the term's own params, GPflow order) of one term.
// (ai, aj: the term's inputs already divided by its ℓ — the quotients sqdist_gpflow forms per
// pair, formed once per row by the caller — or null)
template <bool GRAD>
__device__ __forceinline__ double eval_term(const gpx_term& t, const double* __restrict__ th,
                                            const double* __restrict__ xi,
                                            const double* __restrict__ xj, double* dk,
                                            const double* __restrict__ ai = nullptr,
                                            const double* __restrict__ aj = nullptr) {
  const int d0 = t.dim_start, dn = t.dim_count;
  switch (t.kind) {
    case GPX_LINEAR: {
      // gpflow.kernels.Linear.K: matmul(X * variance, X2ᵀ) -> Σ_d (x_d σ²)·x'_d; ∂/∂σ² = Σ x_d x'_d
#pragma clang fp contract(off)
      double s = (xi[d0] * th[0]) * xj[d0], sd = xi[d0] * xj[d0];
      for (int d = 1; d < dn; ++d) {
        s = s + (xi[d0 + d] * th[0]) * xj[d0 + d];
        sd = sd + xi[d0 + d] * xj[d0 + d];
      }
      if (GRAD) dk[0] = sd;
      return s;
    }
    case GPX_PERIODIC_SE: {
      // Periodic.K: r = π(x − x')/p, s² = Σ (sin r / ℓ)², K = σ² exp(−s²/2)
      const double ell = th[0], var = th[1], p = th[2];
      const double inv_l2 = 1.0 / (ell * ell);
      double s2 = 0.0, sc = 0.0;
      for (int d = 0; d < dn; ++d) {
        const double diff = xi[d0 + d] - xj[d0 + d];
        double sn, cs;
        sincos(M_PI * diff / p, &sn, &cs);
        const double q = sn / ell;
        s2 = s2 + q * q;
        if (GRAD) sc = fma(sn * cs, diff, sc);
      }
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
  const double r2 = ai ? sqdist_scaled(ai, aj, dn) : sqdist_gpflow(xi + d0, xj + d0, dn, ell);
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

// value derivatives (∂K/∂ℓ, ∂K/∂σ²) of a single-term isotropic stationary kernel at r2 = d²/ℓ²,
// with 1/ℓ precomputed by the caller (same formulas and clamp as eval_term<true>)
__device__ __forceinline__ void stationary_grad(int kind, double r2, double var, double inv_ell,
                                                double (&dk)[3]) {
  dk[2] = 0.0;
  if (kind == GPX_SE) {
    const double g = exp(-0.5 * r2);
    dk[0] = var * g * r2 * inv_ell;
    dk[1] = g;
    return;
  }
  const bool clamped = !(r2 > 1e-36);
  const double r = sqrt(clamped ? 1e-36 : r2);
  double g, dgdr;
  if (kind == GPX_MATERN12) {
    g = exp(-r); dgdr = -g;
  } else if (kind == GPX_EXPONENTIAL) {
    g = exp(-0.5 * r); dgdr = -0.5 * g;
  } else if (kind == GPX_MATERN32) {
    const double sq3 = 1.7320508075688772, e = exp(-sq3 * r);
    g = (1.0 + sq3 * r) * e; dgdr = -3.0 * r * e;
  } else {
    const double sq5 = 2.23606797749979, e = exp(-sq5 * r);
    g = (1.0 + sq5 * r + (5.0 / 3.0) * r * r) * e;
    dgdr = -(5.0 / 3.0) * r * (1.0 + sq5 * r) * e;
  }
  dk[0] = clamped ? 0.0 : var * dgdr * (-r * inv_ell);
  dk[1] = g;
}

// K(xi, xj) for a full spec.
__device__ __forceinline__ double eval_k(const DevSpec& s, const double* __restrict__ th,
                                         const double* __restrict__ xi,
                                         const double* __restrict__ xj) {
  const bool prod = (s.combine == GPX_PRODUCT && s.n_terms > 1);
  double acc = prod ? 1.0 : 0.0;
  // static term index (a runtime-indexed register copy of the spec would live in scratch)
#pragma unroll
  for (int t = 0; t < GPX_MAX_TERMS; ++t) {
    if (t >= s.n_terms) break;
    const double v = eval_term<false>(s.terms[t], th + s.terms[t].param_offset, xi, xj, nullptr);
    if (prod) acc *= v; else acc += v;
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

// eval_k / eval_k_grad with pre-scaled inputs: term t's rows at sxs + soff[t] (row-major, the
// term's dim_count values per row; soff[t] < 0: that term reads X as usual). The same
// operations as eval_k / eval_k_grad, so the same bits, without two divisions per entry.
__device__ __forceinline__ bool term_prescaled(int kind) {
  return kind != GPX_LINEAR && kind != GPX_PERIODIC_SE;
}
// the θ slot of a pre-scaled term's ℓ (eval_term's: RQ keeps α first)
__device__ __forceinline__ int term_ell_slot(const gpx_term& t) {
  return t.param_offset + (t.kind == GPX_RQ ? 1 : 0);
}
__device__ __forceinline__ double eval_k_pre(const DevSpec& s, const double* __restrict__ th,
                                             const double* __restrict__ xi, const double* __restrict__ xj,
                                             const double* __restrict__ sxs, const int* __restrict__ soff,
                                             int i, int j) {
  const bool prod = (s.combine == GPX_PRODUCT && s.n_terms > 1);
  double acc = prod ? 1.0 : 0.0;
#pragma unroll
  for (int t = 0; t < GPX_MAX_TERMS; ++t) {
    if (t >= s.n_terms) break;
    const int o = soff[t], dn = s.terms[t].dim_count;
    const double v = eval_term<false>(s.terms[t], th + s.terms[t].param_offset, xi, xj, nullptr,
                                      o >= 0 ? sxs + o + i * dn : nullptr, o >= 0 ? sxs + o + j * dn : nullptr);
    if (prod) acc *= v; else acc += v;
  }
  return acc;
}
template <int NT = GPX_MAX_TERMS>
__device__ __forceinline__ double eval_k_grad_pre(const DevSpec& s, const double* __restrict__ th,
                                                  const double* __restrict__ xi, const double* __restrict__ xj,
                                                  const double* __restrict__ sxs, const int* __restrict__ soff,
                                                  int i, int j, double (&dk)[NT][3]) {
  const bool prod = (NT > 1 && s.combine == GPX_PRODUCT && s.n_terms > 1);
  double vals[NT];
  double acc = prod ? 1.0 : 0.0;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    dk[t][0] = dk[t][1] = dk[t][2] = 0.0;
    vals[t] = 1.0;
    if (t < s.n_terms) {
      const int o = soff[t], dn = s.terms[t].dim_count;
      vals[t] = eval_term<true>(s.terms[t], th + s.terms[t].param_offset, xi, xj, dk[t],
                                o >= 0 ? sxs + o + i * dn : nullptr, o >= 0 ? sxs + o + j * dn : nullptr);
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

// ∂K(xi, xj)/∂xi over the first DM input columns (zero outside each term's active dims);
// the SVGP inducing-point gradient. Product rule applied term by term:
// (P, G) ← (P·v_t, G·v_t + P·g_t).
template <int DM>
__device__ __forceinline__ double eval_term_dx1(const gpx_term& t, const double* __restrict__ th,
                                                const double* __restrict__ xi,
                                                const double* __restrict__ xj, double (&g)[DM]) {
  const int d0 = t.dim_start, dn = t.dim_count;
#pragma unroll
  for (int d = 0; d < DM; ++d) g[d] = 0.0;
  switch (t.kind) {
    case GPX_LINEAR: {
      double s = 0.0;
      for (int d = 0; d < dn; ++d) s = fma(xi[d0 + d], xj[d0 + d], s);
#pragma unroll
      for (int d = 0; d < DM; ++d)
        if (d >= d0 && d < d0 + dn) g[d] = th[0] * xj[d];
      return th[0] * s;
    }
    case GPX_PERIODIC_SE: {
      const double ell = th[0], var = th[1], p = th[2];
      const double inv_l2 = 1.0 / (ell * ell);
      double s2 = 0.0;
      for (int d = 0; d < dn; ++d) {
        const double q = sin(M_PI * (xi[d0 + d] - xj[d0 + d]) / p) / ell;
        s2 = s2 + q * q;
      }
      const double k = var * exp(-0.5 * s2);
#pragma unroll
      for (int d = 0; d < DM; ++d)
        if (d >= d0 && d < d0 + dn) {
          double sn, cs;
          sincos(M_PI * (xi[d] - xj[d]) / p, &sn, &cs);
          g[d] = -k * sn * cs * (M_PI / p) * inv_l2;
        }
      return k;
    }
    default: break;
  }
  const bool rq = (t.kind == GPX_RQ);
  const double ell = rq ? th[1] : th[0];
  const double var = rq ? th[2] : th[1];
  const double inv_l2 = 1.0 / (ell * ell);
  const double r2 = sqdist_gpflow(xi + d0, xj + d0, dn, ell);
  double k, dgdr2;  // K = var·g(r²), dgdr2 = var·g'(r²)
  switch (t.kind) {
    case GPX_SE: { k = var * exp(-0.5 * r2); dgdr2 = -0.5 * k; break; }
    case GPX_RQ: {
      const double a = th[0];
      const double b = 1.0 + 0.5 * r2 / a;
      k = var * exp(-a * log(b));
      dgdr2 = -0.5 * k / b;
      break;
    }
    default: {
      const bool clamped = !(r2 > 1e-36);
      const double r = sqrt(clamped ? 1e-36 : r2);
      double gv, dh;
      switch (t.kind) {
        case GPX_MATERN12: { gv = exp(-r); dh = -gv; break; }
        case GPX_EXPONENTIAL: { gv = exp(-0.5 * r); dh = -0.5 * gv; break; }
        case GPX_MATERN32: {
          const double sq3 = 1.7320508075688772, e = exp(-sq3 * r);
          gv = (1.0 + sq3 * r) * e; dh = -3.0 * r * e; break;
        }
        default: {
          const double sq5 = 2.23606797749979, e = exp(-sq5 * r);
          gv = (1.0 + sq5 * r + (5.0 / 3.0) * r * r) * e;
          dh = -(5.0 / 3.0) * r * (1.0 + sq5 * r) * e;
          break;
        }
      }
      k = var * gv;
      dgdr2 = clamped ? 0.0 : var * dh / (2.0 * r);
      break;
    }
  }
  const double f = 2.0 * dgdr2 * inv_l2;
#pragma unroll
  for (int d = 0; d < DM; ++d)
    if (d >= d0 && d < d0 + dn) g[d] = f * (xi[d] - xj[d]);
  return k;
}

template <int DM>
__device__ __forceinline__ double eval_k_dx1(const DevSpec& s, const double* __restrict__ th,
                                             const double* __restrict__ xi,
                                             const double* __restrict__ xj, double (&g)[DM]) {
  const bool prod = (s.combine == GPX_PRODUCT && s.n_terms > 1);
  double P = prod ? 1.0 : 0.0;
#pragma unroll
  for (int d = 0; d < DM; ++d) g[d] = 0.0;
#pragma unroll
  for (int t = 0; t < GPX_MAX_TERMS; ++t) {
    if (t >= s.n_terms) break;
    double gt[DM];
    const double v = eval_term_dx1<DM>(s.terms[t], th + s.terms[t].param_offset, xi, xj, gt);
    if (prod) {
#pragma unroll
      for (int d = 0; d < DM; ++d) g[d] = fma(g[d], v, P * gt[d]);
      P *= v;
    } else {
#pragma unroll
      for (int d = 0; d < DM; ++d) g[d] += gt[d];
      P += v;
    }
  }
  return P;
}

// K_diag(x) as GPflow's K_diag methods: σ² for the stationary terms (Stationary.K_diag fills the
// variance; Periodic takes its base kernel's), Σ_d (x_d²)·σ² for Linear (reduce_sum(square(X) *
// variance)); sums / products of the terms'.
__device__ __forceinline__ double eval_kdiag(const DevSpec& s, const double* __restrict__ th,
                                             const double* __restrict__ x) {
  const bool prod = (s.combine == GPX_PRODUCT && s.n_terms > 1);
  double acc = prod ? 1.0 : 0.0;
#pragma unroll
  for (int t = 0; t < GPX_MAX_TERMS; ++t) {
    if (t >= s.n_terms) break;
    const gpx_term& tm = s.terms[t];
    const double* tth = th + tm.param_offset;
    double v;
    if (tm.kind == GPX_LINEAR) {
#pragma clang fp contract(off)
      v = (x[tm.dim_start] * x[tm.dim_start]) * tth[0];
      for (int d = 1; d < tm.dim_count; ++d) v = v + (x[tm.dim_start + d] * x[tm.dim_start + d]) * tth[0];
    } else {
      v = tm.kind == GPX_RQ ? tth[2] : tth[1];
    }
    if (prod) acc *= v; else acc += v;
  }
  return acc;
}

// value of a single-term isotropic stationary kernel at scaled squared distance r2 = d²/ℓ²
// (same formulas and 1e-36 clamp as eval_term in gpx_kfun.h)
template <int KIND>
__device__ __forceinline__ double stationary_value(double r2, double var) {
  if constexpr (KIND == GPX_SE) {
    return var * exp(-0.5 * r2);
  } else {
    const double r = sqrt(r2 > 1e-36 ? r2 : 1e-36);
    if constexpr (KIND == GPX_MATERN12) return var * exp(-r);
    if constexpr (KIND == GPX_EXPONENTIAL) return var * exp(-0.5 * r);
    if constexpr (KIND == GPX_MATERN32) {
      const double s = 1.7320508075688772;
      return var * ((1.0 + s * r) * exp(-s * r));
    }
    if constexpr (KIND == GPX_MATERN52) {
      const double s = 2.23606797749979;
      return var * ((1.0 + s * r + (5.0 / 3.0) * r * r) * exp(-s * r));
    }
  }
  return 0.0;
}


}  // namespace gpx
