// gpx_leaf.h — the 64x64 Cholesky-and-inverse leaf on LDS, shared by leaf_kernel
// (gpx_kernels.hip) and the fused banded kernels (gpx_band.hip).
#pragma once
#include <hip/hip_runtime.h>
#include "gpx_internal.h"

namespace gpx {

__device__ __forceinline__ double readlane_d(double v, int l) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)(u & 0xffffffffu), l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// 1/sqrt(x) from the hardware estimate and two Newton steps (each doubles the ~22 correct bits):
// within an ulp or two of 1/sqrt, and one multiply gives sqrt(x) = x/sqrt(x). Replaces a
// correctly rounded sqrt and a division on the leaves' serial 16-step diagonal chain.
__device__ __forceinline__ double rsqrt_nr(double x) {
  double y = __builtin_amdgcn_rsq(x);
  y = y * fma(-0.5 * x, y * y, 1.5);
  y = y * fma(-0.5 * x, y * y, 1.5);
  return y;
}

// Factor the lower 64x64 block held in sA (row stride kLeafS, upper part ignored) and write
// W = L⁻¹ into sW (which must be zero on entry; zeros above the diagonal are kept). sA is
// destroyed. Writes log L_ii to ldiag[0..63]; *sfail (LDS, -1 on entry) gets the first
// failing local pivot. 256 threads; ends with a barrier.
constexpr int kLeafS = 66;  // row stride (doubles): 16 rows x 1 col fragment reads are conflict-free
__device__ __forceinline__ void leaf64_lds(double* __restrict__ sA, double* __restrict__ sW,
                                           double* __restrict__ ldiag, int* sfail) {
  constexpr int S = kLeafS;
  typedef double d4 __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l15 = lane & 15, l4 = lane >> 4;
  for (int jb = 0; jb < 4; ++jb) {
    const int c0 = jb * 16;
    if (wave == 0) {
      double r[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) r[k] = sA[(c0 + l15) * S + c0 + k];
      int fail = -1;
      double invd[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const double piv = readlane_d(r[j], j);
        if (!(piv > 0.0) && fail < 0) fail = j;
        const double inv = rsqrt_nr(piv);
        const double ljj = piv * inv;
        invd[j] = inv;
        r[j] = (l15 > j) ? r[j] * inv : ((l15 == j) ? ljj : 0.0);
#pragma unroll
        for (int k = j + 1; k < 16; ++k) r[k] = fma(-r[j], readlane_d(r[j], k), r[k]);
      }
      // lane l15 holds row l15 of L_jj (r[0..l15]); column l15 of D = L_jj⁻¹ by substitution
      double w[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        double sacc = (i == l15) ? 1.0 : 0.0;
#pragma unroll
        for (int k = 0; k < i; ++k) sacc = fma(-readlane_d(r[k], i), w[k], sacc);
        w[i] = sacc * invd[i];
      }
      if (lane < 16) {
#pragma unroll
        for (int i = 0; i < 16; ++i) sW[(c0 + i) * S + c0 + lane] = w[i];
        ldiag[c0 + lane] = log(r[lane & 15]);
      }
      if (lane == 0 && fail >= 0 && *sfail < 0) *sfail = c0 + fail;
    }
    __syncthreads();
    // panel: L_(ib,jb) = A_(ib,jb) · Dᵀ for ib = jb+1 .. 3, one wave per block
    const int nblk = 3 - jb;
    if (wave < nblk) {
      const int r0 = (jb + 1 + wave) * 16;
      d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const double av = sA[(r0 + l15) * S + c0 + 4 * kk + l4];
        const double bv = sW[(c0 + l15) * S + c0 + 4 * kk + l4];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) sA[(r0 + l4 + 4 * q) * S + c0 + l15] = acc[q];
    }
    __syncthreads();
    // trailing update of the lower blocks (ib, kb), jb < kb <= ib
    const int ntr = nblk * (nblk + 1) / 2;
    for (int t = wave; t < ntr; t += 4) {
      int p = 0;
      while ((p + 1) * (p + 2) / 2 <= t) ++p;
      const int q = t - p * (p + 1) / 2;
      const int ri = (jb + 1 + p) * 16, rk = (jb + 1 + q) * 16;
      d4 acc;
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = sA[(ri + l4 + 4 * u) * S + rk + l15];
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const double av = sA[(ri + l15) * S + c0 + 4 * kk + l4];
        const double bv = sA[(rk + l15) * S + c0 + 4 * kk + l4];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-av, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) sA[(ri + l4 + 4 * u) * S + rk + l15] = acc[u];
    }
    __syncthreads();
  }
  // W = L⁻¹: block rows 1..3, blocks j < i in parallel (wave j)
  for (int i = 1; i < 4; ++i) {
    if (wave < i) {
      const int j = wave;
      d4 t = {0.0, 0.0, 0.0, 0.0};
      for (int k = j; k < i; ++k) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const double av = sA[(i * 16 + l15) * S + k * 16 + 4 * kk + l4];   // L_ik[row][k']
          const double bv = sW[(k * 16 + 4 * kk + l4) * S + j * 16 + l15];   // W_kj[k'][col]
          t = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, t, 0, 0, 0);
        }
      }
      d4 wv = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const double av = sW[(i * 16 + l15) * S + i * 16 + 4 * kk + l4];     // D_i[row][k']
        wv = __builtin_amdgcn_mfma_f64_16x16x4f64(-av, t[kk], wv, 0, 0, 0);  // T[k'][col]
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) sW[(i * 16 + l4 + 4 * q) * S + j * 16 + l15] = wv[q];
    }
    __syncthreads();
  }
}

}  // namespace gpx
