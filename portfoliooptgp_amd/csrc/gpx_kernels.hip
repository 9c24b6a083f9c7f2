// gpx_kernels.hip — CDNA4 (gfx950) kernels of the exact-GP engine, all fp64.
//
// Per loss+gradient evaluation (one L-BFGS-B function call of gpflow.optimizers.Scipy,
// GPR/model_trainer.py:18-19) the host drives, for a batch of independent problems:
//   build_kernel        K = k(X,X) + σn² I, lower 64x64 tiles, identity padding to Np
//   leaf_kernel         64x64 diagonal block: Cholesky + triangular inverse, in LDS
//   gemm_kernel<...>    fp64 MFMA (v_mfma_f64_16x16x4_f64) tile GEMM, batched over problems:
//                       the TRMM/SYRK steps of the recursive Cholesky-and-inverse and the
//                       fused K⁻¹ = WᵀW formation + gradient contraction (EPI_CONTRACT)
//   trmv_n/trmv_t       z = W y, α = Wᵀ z  (W = L⁻¹)
//   reduce_kernel       logML and ½Σ(αα−K⁻¹)∘∂K/∂θ from per-tile partials (deterministic)
// and for predict_f: the cross-covariance build, mean = Kxsᵀα, and W·Kxs with a fused
// column-sum-of-squares epilogue (EPI_COLSUMSQ) for the variance.
#include <hip/hip_ext.h>
#include <cstdio>
#include <cstdlib>
#include "gpx_internal.h"
#include "gpx_leaf.h"

namespace gpx {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

// linear index -> (ti, tj) of the lower-triangular tile enumeration (ti >= tj), row-major:
// a row's tiles share their A panel and start their k loops together, so its panel k-slabs are
// served from L2 in step. (A grouped order — 8 rows taken column by column, fewer distinct
// panels resident — was measured 7 % slower on the contraction: tiles of different rows start
// at different k, so the shared column panels are no longer read in step.)
__device__ __forceinline__ void lower_tile(int idx, int& ti, int& tj) {
  int t = (int)((sqrt(8.0 * (double)idx + 1.0) - 1.0) * 0.5);
  while ((t + 1) * (t + 2) / 2 <= idx) ++t;
  while (t * (t + 1) / 2 > idx) --t;
  ti = t;
  tj = idx - t * (t + 1) / 2;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ======================================================================================
// K build (and cross-covariance Kxs for predict)
// ======================================================================================
template <int KIND>
__device__ __forceinline__ void build_stationary(const BuildArgs& a, const DevSpec& spec,
                                                 const double* sth, const double* sxi,
                                                 const double* sxj, double noise, int n, int ncol,
                                                 int ti, int tj, double* out) {
  // sxi / sxj hold the inputs already scaled by 1/ℓ (staged that way by build_kernel)
  const gpx_term& t = spec.terms[0];
  const double* th = sth + t.param_offset;
  const double var = th[1];
  const int D = a.D, d0 = t.dim_start, dn = t.dim_count;
  const int c = threadIdx.x & 63;
  const int gj = tj * 64 + c;
  for (int q = 0; q < 16; ++q) {
    const int r = (threadIdx.x >> 6) + 4 * q;
    const int gi = ti * 64 + r;
    double v;
    const bool valid = a.symmetric ? (gi < n && gj < n) : (gi < n && gj < ncol);
    if (valid) {
      const double r2 = dn == 1 ? sqdist1(sxi[r * D + d0], sxj[c * D + d0])
                                : sqdist_scaled(sxi + r * D + d0, sxj + c * D + d0, dn);
      v = stationary_value<KIND>(r2, var);
      if (a.symmetric && gi == gj) v += noise;
    } else {
      v = (a.symmetric && gi == gj) ? 1.0 : 0.0;
    }
    out[(long long)gi * a.ldo + gj] = v;
  }
}

__global__ __launch_bounds__(256) void build_kernel(BuildArgs a) {
  const int b = a.active[blockIdx.y];
  int ti, tj;
  if (a.symmetric && a.band1 > 0) {
    // block band: tile x = d·nb + k -> (k, k − d), d < band1 (tiles with k < d are empty)
    const int nb = a.rows / 64, d = blockIdx.x / nb;
    ti = blockIdx.x - d * nb;
    tj = ti - d;
    if (tj < 0) return;
  } else if (a.symmetric) {
    lower_tile(blockIdx.x, ti, tj);
  } else {
    const int ntj = a.cols / 64;
    ti = blockIdx.x / ntj;
    tj = blockIdx.x - ti * ntj;
  }
  __shared__ double sxi[64 * GPX_MAX_DIM];
  __shared__ double sxj[64 * GPX_MAX_DIM];
  __shared__ double sth[GPX_THETA_STRIDE];
  const int D = a.D, tid = threadIdx.x;
  const int n = a.rows_valid > 0 ? a.rows_valid : a.nvalid[b];
  const int ncol = a.symmetric ? n : a.m2;
  const double* X = a.X + (long long)b * a.sX;
  const double* X2 = a.symmetric ? X : a.X2 + (long long)b * a.sX2;
  const DevSpec spec = a.specs[b];
  // single-term isotropic stationary kernels (the reference's SE / Matern / Exponential sweeps)
  // take a compact loop on inputs staged pre-scaled by 1/ℓ (GPflow's Stationary.scale, one
  // division per staged value instead of two per element): the generic term interpreter below
  // unrolls into tens of KiB of code per kernel, which thrashed the instruction cache of this
  // HBM-write kernel
  const int k0 = spec.terms[0].kind;
  const bool fast = spec.n_terms == 1 && k0 >= GPX_SE && k0 <= GPX_EXPONENTIAL;
  const double fell = fast ? a.theta[b * GPX_THETA_STRIDE + spec.terms[0].param_offset] : 1.0;
  for (int e = tid; e < 64 * D; e += 256) {
    const int r = e / D, d = e - (e / D) * D;
    const int gi = ti * 64 + r, gj = tj * 64 + r;
    const double xi = gi < n ? X[(long long)gi * D + d] : 0.0;
    const double xj = gj < ncol ? X2[(long long)gj * D + d] : 0.0;
    sxi[e] = fast ? xi / fell : xi;
    sxj[e] = fast ? xj / fell : xj;
  }
  if (tid < GPX_THETA_STRIDE) sth[tid] = a.theta[b * GPX_THETA_STRIDE + tid];
  // the general path: each stationary term's inputs over its ℓ staged once per row (the quotients
  // sqdist_gpflow forms per pair: the same bits, eval_k_pre), term t's at soff[t] in sxp, the
  // tile's 64 rows then its 64 columns, while they fit GPX_MAX_DIM doubles per row
  __shared__ double sxp[128 * GPX_MAX_DIM];
  __shared__ int soff[GPX_MAX_TERMS];
  if (!fast) {
    const DevSpec* gs = a.specs + b;  // (dynamic term index: read from memory, not the register copy)
    int P = 0;
    for (int t = 0; t < gs->n_terms; ++t) P += term_prescaled(gs->terms[t].kind) ? gs->terms[t].dim_count : 0;
    if (P > GPX_MAX_DIM) P = 0;
    if (tid == 0) {  // (soff[t] < 0: term t reads X as eval_k does)
      int o = 0;
      for (int t = 0; t < GPX_MAX_TERMS; ++t) {
        const bool pre = P > 0 && t < gs->n_terms && term_prescaled(gs->terms[t].kind);
        soff[t] = pre ? 128 * o : -1;
        o += pre ? gs->terms[t].dim_count : 0;
      }
    }
    if (P > 0) {
      for (int t = 0, o = 0; t < gs->n_terms; ++t) {
        const gpx_term& tm = gs->terms[t];
        if (!term_prescaled(tm.kind)) continue;
        const double ell = a.theta[b * GPX_THETA_STRIDE + term_ell_slot(tm)];
        const int dn = tm.dim_count;
        for (int e = tid; e < 64 * dn; e += 256) {
          const int r = e / dn, d = tm.dim_start + (e - r * dn);
          const int gi = ti * 64 + r, gj = tj * 64 + r;
          sxp[128 * o + e] = (gi < n ? X[(long long)gi * D + d] : 0.0) / ell;
          sxp[128 * o + 64 * dn + e] = (gj < ncol ? X2[(long long)gj * D + d] : 0.0) / ell;
        }
        o += dn;
      }
    }
  }
  __syncthreads();
  const double noise = sth[spec.n_params];
  double* out = a.out + (long long)b * a.sOut;
  const int c = tid & 63;
  const int gj = tj * 64 + c;
  if (fast) {
    switch (k0) {
      case GPX_SE:          build_stationary<GPX_SE>(a, spec, sth, sxi, sxj, noise, n, ncol, ti, tj, out); return;
      case GPX_MATERN12:    build_stationary<GPX_MATERN12>(a, spec, sth, sxi, sxj, noise, n, ncol, ti, tj, out); return;
      case GPX_MATERN32:    build_stationary<GPX_MATERN32>(a, spec, sth, sxi, sxj, noise, n, ncol, ti, tj, out); return;
      case GPX_MATERN52:    build_stationary<GPX_MATERN52>(a, spec, sth, sxi, sxj, noise, n, ncol, ti, tj, out); return;
      default:              build_stationary<GPX_EXPONENTIAL>(a, spec, sth, sxi, sxj, noise, n, ncol, ti, tj, out); return;
    }
  }
#pragma unroll 1
  for (int q = 0; q < 16; ++q) {
    const int r = (tid >> 6) + 4 * q;
    const int gi = ti * 64 + r;
    double v;
    auto kv = [&]() { return eval_k_pre(spec, sth, sxi + r * D, sxj + c * D, sxp, soff, r, 64 + c); };
    if (a.symmetric) {
      if (gi < n && gj < n) {
        v = kv();
        if (gi == gj) v += noise;
      } else {
        v = (gi == gj) ? 1.0 : 0.0;
      }
    } else {
      v = (gi < n && gj < ncol) ? kv() : 0.0;
    }
    out[(long long)gi * a.ldo + gj] = v;
  }
}

void launch_build(const BuildArgs& a, int n_active, hipStream_t s) {
  const int ti = a.rows / 64, tj = a.cols / 64;
  const int ntiles = a.symmetric ? (a.band1 > 0 ? a.band1 * ti : ti * (ti + 1) / 2) : ti * tj;
  hipLaunchKernelGGL(build_kernel, dim3(ntiles, n_active), dim3(256), 0, s, a);
}

// ======================================================================================
// Leaf: Cholesky of the 64x64 diagonal block at (off, off) of the (already updated) K and
// W11 = L11⁻¹. One workgroup (4 waves) per problem, blocked in 4 panels of 16:
//   diag 16x16: wave 0 factors it and inverts it in registers (lane i = row i; broadcasts by
//               v_readlane, no barriers), giving L_jj (for log det) and D = L_jj⁻¹;
//   panel:      L_ij = A_ij · Dᵀ                          (f64 MFMA 16x16x4, one wave per block)
//   trailing:   A_ik -= L_ij · L_kjᵀ                      (f64 MFMA)
// then W = L⁻¹ block rows: W_ij = −D_i · Σ_{k=j}^{i−1} L_ik W_kj (f64 MFMA; the accumulator of
// the first product is the B operand of the second without an LDS round trip).
// 15 barriers in all. Writes W11 (zeros above the diagonal) and log L_ii.
// ======================================================================================
__global__ __launch_bounds__(256) void leaf_kernel(LeafArgs a) {
  constexpr int S = kLeafS;
  __shared__ __attribute__((aligned(16))) double sA[64 * S];
  __shared__ __attribute__((aligned(16))) double sW[64 * S];
  __shared__ int sfail;
  const int b = a.active[blockIdx.x];
  const double* K = a.K + (long long)b * a.sMat;
  double* W = a.W + (long long)b * a.sMat;
  const int ld = a.ld, off = a.off, tid = threadIdx.x;
  // 8 independent loads in flight per thread (a load-then-store loop serialises on latency)
#pragma unroll 1
  for (int e0 = tid; e0 < 4096; e0 += 256 * 8) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + 256 * u, r = e >> 6, c = e & 63;
      v[u] = (c <= r) ? K[(long long)(off + r) * ld + off + c] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + 256 * u, r = e >> 6, c = e & 63;
      sA[r * S + c] = v[u];
      sW[r * S + c] = 0.0;
    }
  }
  if (tid == 0) sfail = -1;
  __syncthreads();

  leaf64_lds(sA, sW, a.ldiag + (long long)b * a.sVec + off, &sfail);
  for (int e = tid; e < 4096; e += 256) {
    const int r = e >> 6, c = e & 63;
    W[(long long)(off + r) * ld + off + c] = sW[r * S + c];
  }
  if (tid == 0 && sfail >= 0 && a.info[b] == 0) a.info[b] = off + sfail + 1;
}

void launch_leaf(const LeafArgs& a, int n_active, hipStream_t s) {
  hipLaunchKernelGGL(leaf_kernel, dim3(n_active), dim3(256), 0, s, a);
}

// ======================================================================================
// Leaf128: Cholesky + triangular inverse of a 128x128 diagonal block in ONE launch (replaces
// two 64-leaves and the four 64x64 GEMMs of a 128-node of the recursion: 6 dependent launches
// of a latency-bound chain become 1). One 4-wave workgroup per problem. The lower 16x16 blocks
// live in ONE packed LDS array (36 blocks, rows padded to 17 doubles: 78 KiB), so the leaf fits
// on a CU beside a GEMM workgroup (73.7 KiB, 256 VGPRs per wave) of the concurrent batch or of
// the recursion's forked T product — a 153 KiB two-array version waited for wholly free CUs.
// Each slot holds A, then L (off-diagonal) or D_j = L_jj⁻¹ (diagonal; L_jj itself is only
// needed for log det), then W: right-looking over 8 block columns
//   diag:     wave 0 factors A_jj and inverts it in registers (as leaf_kernel) -> D_j
//   panel:    L_ij = A_ij · D_jᵀ                 (f64 MFMA)
//   trailing: A_ik -= L_ij · L_kjᵀ, j < k <= i   (f64 MFMA, blocks over the 4 waves)
// then W_ij = −D_i · Σ_{k=j}^{i−1} L_ik W_kj block row by block row (W_jj = D_j): a row's blocks
// are formed in registers, then written over that row's L blocks after a barrier.
// ======================================================================================
namespace {
constexpr int L8 = 8, LBS = 16 * 17;   // blocks per side, block stride (doubles)
__device__ __forceinline__ int lblk(int bi, int bj) { return (bi * (bi + 1) / 2 + bj) * LBS; }
}  // namespace

// The 128x128 Cholesky-and-inverse on the packed lower-block LDS array sS (A in; W = L⁻¹ out, in
// place): the first nbv 16-row blocks only (the ones that hold data; blocks past them must hold
// the identity on the diagonal and zeros elsewhere, which are their own W). log L_ii of those
// rows to ldg[], the first failing pivot to *sfail (which must start at −1). 256 or 512 threads; ends
// with a barrier. leaf128_kernel (nbv = 8) and small128_kernel.
__device__ __forceinline__ void leaf128_lds(double* __restrict__ sS, double* __restrict__ ldg, int* sfail, int nbv) {
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;  // (4 or 8 waves)
  const int l15 = lane & 15, l4 = lane >> 4;
  // the diagonal block jb: wave 0 factors it and inverts it in registers -> D_jb over A_jb,jb
  auto diag = [&](const int jb) __attribute__((always_inline)) {
    const int dj = lblk(jb, jb);
    double r[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) r[k] = sS[dj + l15 * 17 + k];
    int fail = -1;
    double invd[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const double piv = bc16(r[j], j);
      if (!(piv > 0.0) && fail < 0) fail = j;
      const double inv = rsqrt_nr(piv);
      const double ljj = piv * inv;
      invd[j] = inv;
      r[j] = (l15 > j) ? r[j] * inv : ((l15 == j) ? ljj : 0.0);
#pragma unroll
      for (int k = j + 1; k < 16; ++k) r[k] = fma(-r[j], bc16(r[j], k), r[k]);
    }
    double w[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) w[i] = (i == l15) ? 1.0 : 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      w[k] *= invd[k];
      // column k's broadcasts wait for w_k (else all 120 are hoisted: ~240 registers)
      double rk = r[k];
      asm volatile("" : "+v"(rk) : "v"(w[k]));
#pragma unroll
      for (int i = k + 1; i < 16; ++i) w[i] = fma(-bc16(rk, i), w[k], w[i]);
    }
    // D_j over A_jj (this wave read the whole block into registers above)
    if (lane < 16) {
#pragma unroll
      for (int i = 0; i < 16; ++i) sS[dj + i * 17 + lane] = w[i];
      ldg[jb * 16 + lane] = log(r[lane & 15]);
    }
    if (lane == 0 && fail >= 0 && *sfail < 0) *sfail = jb * 16 + fail;
  };
  // trailing tile t of step jb (tiles (jb+1+p, jb+1+q), q <= p, numbered row by row)
  auto trail = [&](const int jb, const int t) __attribute__((always_inline)) {
    int p = 0;
    while ((p + 1) * (p + 2) / 2 <= t) ++p;
    const int q = t - p * (p + 1) / 2;
    const int bi = jb + 1 + p, bk = jb + 1 + q;
    const int ob = lblk(bi, bk), li = lblk(bi, jb), lk = lblk(bk, jb);
    d4 acc;
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = sS[ob + (l4 + 4 * u) * 17 + l15];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const double av = sS[li + l15 * 17 + 4 * kk + l4];
      const double bv = sS[lk + l15 * 17 + 4 * kk + l4];
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 1);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) sS[ob + (l4 + 4 * u) * 17 + l15] = acc[u];
  };
  // right-looking over the block columns, the next diagonal block factored ahead: in step jb wave 0
  // updates tile (jb+1, jb+1) first and factors it while the other waves update the rest of the
  // trailing tiles (each tile's updates in the same order and form as one after another: the
  // same bits, a barrier per step less on the critical path)
  if (wave == 0) diag(0);
  __syncthreads();
  for (int jb = 0; jb < nbv; ++jb) {
    const int dj = lblk(jb, jb);
    // panel: L_(ib,jb) = A_(ib,jb) · D_jbᵀ, in place
    const int nblk = nbv - 1 - jb;
    for (int t = wave; t < nblk; t += nw) {
      const int pb = lblk(jb + 1 + t, jb);
      d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const double av = sS[pb + l15 * 17 + 4 * kk + l4];
        const double bv = sS[dj + l15 * 17 + 4 * kk + l4];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
      // the wave's operand reads precede its MFMA results: the in-place update is safe
#pragma unroll
      for (int q = 0; q < 4; ++q) sS[pb + (l4 + 4 * q) * 17 + l15] = acc[q];
    }
    __syncthreads();
    if (nblk == 0) break;
    const int ntr = nblk * (nblk + 1) / 2;
    if (wave == 0) {
      trail(jb, 0);
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");  // (its LDS writes before diag's reads)
      diag(jb + 1);
    } else {
      for (int t = wave; t < ntr; t += nw - 1) trail(jb, t);
    }
    __syncthreads();
  }
  // W = L⁻¹ block rows 1..7; blocks j < i of a row (j = wave, wave + nw) in registers first
  for (int i = 1; i < nbv; ++i) {
    d4 wv[2];
    const int di = lblk(i, i);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = wave + nw * h;
      wv[h] = (d4){0.0, 0.0, 0.0, 0.0};
      if (j < i) {
        d4 t = {0.0, 0.0, 0.0, 0.0};
        for (int k = j; k < i; ++k) {
          const int lik = lblk(i, k), wkj = lblk(k, j);   // L_ik; W_kj (row k < i done; W_jj = D_j)
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const double av = sS[lik + l15 * 17 + 4 * kk + l4];
            const double bv = sS[wkj + (4 * kk + l4) * 17 + l15];
            t = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, t, 0, 0, 0);
          }
        }
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const double av = sS[di + l15 * 17 + 4 * kk + l4];   // D_i[row][k']
          wv[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, t[kk], wv[h], 0, 0, 1);
        }
      }
    }
    __syncthreads();   // every wave has read row i's L blocks
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = wave + nw * h;
      if (j < i) {
        const int wij = lblk(i, j);
#pragma unroll
        for (int q = 0; q < 4; ++q) sS[wij + (l4 + 4 * q) * 17 + l15] = wv[h][q];
      }
    }
    __syncthreads();
  }
}

#ifndef GPX_LEAF128_WAVES
#define GPX_LEAF128_WAVES 8
#endif
constexpr int kLeaf128Waves = GPX_LEAF128_WAVES;  // (4: round 5's leaf; the same bits either way)
__global__ __launch_bounds__(64 * kLeaf128Waves) void leaf128_kernel(LeafArgs a) {
  __shared__ __attribute__((aligned(16))) double sS[36 * LBS];
  __shared__ int sfail;
  const int b = a.active[blockIdx.x];
  const double* K = a.K + (long long)b * a.sMat;
  double* W = a.W + (long long)b * a.sMat;
  const int ld = a.ld, off = a.off, tid = threadIdx.x;
  // lower 128x128 of A (row pieces of 128 B, coalesced); blocks above the diagonal not stored
  // 8 independent loads in flight per thread (a load-then-store loop serialises on latency)
#pragma unroll 1
  for (int e0 = tid; e0 < 128 * 128; e0 += 64 * kLeaf128Waves * 8) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + 64 * kLeaf128Waves * u, r = e >> 7, c = e & 127;
      v[u] = (c <= r) ? K[(long long)(off + r) * ld + off + c] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + 64 * kLeaf128Waves * u, r = e >> 7, c = e & 127;
      if (c <= (r | 15)) sS[lblk(r >> 4, c >> 4) + (r & 15) * 17 + (c & 15)] = v[u];
    }
  }
  if (tid == 0) sfail = -1;
  __syncthreads();

  leaf128_lds(sS, a.ldiag + (long long)b * a.sVec + off, &sfail, L8);
  // the whole 128x128 block of W, zeros above the diagonal
  for (int e = tid; e < 128 * 128; e += 64 * kLeaf128Waves) {
    const int r = e >> 7, c = e & 127;
    const double v = (c <= r) ? sS[lblk(r >> 4, c >> 4) + (r & 15) * 17 + (c & 15)] : 0.0;
    W[(long long)(off + r) * ld + off + c] = v;
  }
  if (tid == 0 && sfail >= 0 && a.info[b] == 0) a.info[b] = off + sfail + 1;
}

void launch_leaf128(const LeafArgs& a, int n_active, hipStream_t s) {
  hipLaunchKernelGGL(leaf128_kernel, dim3(n_active), dim3(64 * kLeaf128Waves), 0, s, a);
}

// ======================================================================================
// Batched fp64 MFMA GEMM: C(tile) = alpha * Σ_k opA(i,k) opB(k,j) + beta * C, with
// per-tile k-range restriction for triangular operands and three epilogues.
// 256 threads = 4 waves in a 2x2 arrangement, each wave (BM/2)x(BM/2) of 16x16 MFMA tiles.
// Operands are staged global -> registers -> LDS (double-buffered, one barrier per K-tile)
// into [k][row] images whose row stride S ≡ 16 (mod 32) doubles makes the fragment reads
// (lanes 0-15 consecutive rows, lanes 16-31 next k) bank-conflict free for ds_read_b64.
// v_mfma_f64_16x16x4_f64: lane l holds A[l&15][l>>4], B[l>>4][l&15]; result register r of
// lane l is C[(l>>4) + 4r][l&15] (verified on gfx950, tools/probe_f64.hip).
// ======================================================================================
// epilogues light enough for three workgroups per CU (168 VGPRs, no spills): the plain store
// and predict's column sums of squares. The contraction epilogue spills ~500 VGPRs at that cap
// (measured), so it keeps BK=16 and two workgroups per CU.
constexpr bool kLeanEpi(int epi) { return epi == EPI_STORE || epi == EPI_COLSUMSQ; }
#ifndef GPX_BK128
// K-tile depth of the plain-store 128-tile GEMMs (the recursion's TRMM/SYRK products): 8 halves
// their LDS (36 KiB), so THREE workgroups share a CU instead of two and the third covers the
// others' barrier/LDS bubbles: factor 101.7 -> 99.6 ms per B=128 evaluation (BK=16: 2 per CU).
// The contraction instances keep BK=16 (see kLeanEpi).
#define GPX_BK128 8
#endif
template <int BM, bool TA, bool TB, int EPI>
__global__ __launch_bounds__(256, BM == 128 ? (GPX_BK128 == 8 && kLeanEpi(EPI) ? 3 : 2) : 1)
void gemm_kernel(GemmArgs a) {
  constexpr int BN = BM, BK = (BM == 128 && kLeanEpi(EPI)) ? GPX_BK128 : 16, S = BM + 16;
  constexpr int KC = BK / 2;  // double2 chunks per operand row of a K-tile
  constexpr int WT = BM / 2;
  constexpr int MT = WT / 16;
  constexpr int NLD = BM * BK / 2 / 256;  // double2 chunks per thread per operand
  constexpr int kMainLds = 2 * 2 * BK * S;
  constexpr bool kContractEpi = EPI == EPI_CONTRACT || EPI == EPI_CONTRACT1 || EPI == EPI_CONTRACT2;
  constexpr int kEpiLds = (EPI == EPI_CONTRACT || EPI == EPI_CONTRACT1 || EPI == EPI_CONTRACT2)
      ? 4 * 16 * WT + 2 * BM * GPX_MAX_DIM + 2 * BM + GPX_THETA_STRIDE + 64 : 0;
  __shared__ __attribute__((aligned(16))) double smem[kMainLds > kEpiLds ? kMainLds : kEpiLds];

  // XCD-aware placement: workgroups are dealt round-robin over the 8 XCDs (block x lands on
  // XCD x % 8 — observed placement, used for speed only). The first 8·⌊na/8⌋ problems are
  // given to the XCDs whole (⌊na/8⌋ each), so every problem's operand panels stream through ONE
  // L2; the remaining na mod 8 problems have their tiles interleaved over all XCDs, which
  // balances the tiles' unequal K ranges (a single problem uses the whole chip).
  const int nti = a.M / BM, ntj = a.N / BN;
  const int ntl = a.lower_only ? nti * (nti + 1) / 2 : nti * ntj;
  const int q = a.n_active >> 3;
  const int xcd = blockIdx.x & 7, s = blockIdx.x >> 3;
  int pa, tile;
  if (s < q * ntl) {
    pa = xcd * q + s / ntl;
    tile = s % ntl;
  } else {
    const int g = (s - q * ntl) * 8 + xcd;
    pa = 8 * q + g / ntl;
    tile = g % ntl;
    if (pa >= a.n_active) return;
  }
  const int b = a.active[pa];
  int ti, tj;
  if (a.lower_only) {
    lower_tile(tile, ti, tj);
  } else {
    // make the index that sets a tile's K range the SLOW one and run the longest tiles first
    const int x = tile;
    switch (a.order) {
      case ORDER_COL_DESC: tj = ntj - 1 - x / nti; ti = x % nti; break;
      case ORDER_COL_ASC:  tj = x / nti; ti = x % nti; break;
      case ORDER_ROW_DESC: ti = nti - 1 - x / ntj; tj = x % ntj; break;
      default:             ti = x / ntj; tj = x % ntj; break;
    }
  }
  const int i0 = ti * BM, j0 = tj * BN;
  int kmin = 0, kmax = a.K;
  if (a.tri & TRI_KMAX_I) kmax = min(kmax, i0 + BM);
  if (a.tri & TRI_KMAX_J) kmax = min(kmax, j0 + BN);
  if (a.tri & TRI_KMIN_J) kmin = max(kmin, j0);
  if (a.tri & TRI_KMIN_I) kmin = max(kmin, i0);

  const double* __restrict__ A = a.A + (long long)b * a.sA;
  const double* __restrict__ B = a.Bm + (long long)b * a.sB;
  const long long lda = a.lda, ldb = a.ldb;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;

  d4 acc[MT][MT];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int n = 0; n < MT; ++n) acc[m][n] = (d4){0.0, 0.0, 0.0, 0.0};

  // Operand loads are buffer loads: the K-tile origin is a wave-uniform base (SGPR buffer
  // descriptor rebuilt per K-tile with scalar arithmetic) and each lane's byte offset inside
  // the tile is a loop-invariant 32-bit VGPR — no per-load 64-bit address arithmetic.
  d2 ra[NLD], rb[NLD];
  int offa[NLD], offb[NLD];
#pragma unroll
  for (int q = 0; q < NLD; ++q) {
    const int c = tid + 256 * q;
    if (!TA) offa[q] = (int)(((c / KC) * lda + (c % KC) * 2) * 8);
    else offa[q] = (int)(((c / (BM / 2)) * lda + (c % (BM / 2)) * 2) * 8);
    if (TB) offb[q] = (int)(((c / KC) * ldb + (c % KC) * 2) * 8);
    else offb[q] = (int)(((c / (BN / 2)) * ldb + (c % (BN / 2)) * 2) * 8);
  }
  auto gload = [&](int k0) {
    const double* pa = TA ? A + (long long)k0 * lda + i0 : A + (long long)i0 * lda + k0;
    const double* pb = TB ? B + (long long)j0 * ldb + k0 : B + (long long)k0 * ldb + j0;
    const auto rsa = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(pa), (short)0, 0x7fffffff, 0x00020000);
    const auto rsb = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(pb), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      ra[q] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(rsa, offa[q], 0, 0));
      rb[q] = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(rsb, offb[q], 0, 0));
    }
  };
  auto swrite = [&](int buf) {
    double* sA = smem + (buf * 2 + 0) * BK * S;
    double* sB = smem + (buf * 2 + 1) * BK * S;
#pragma unroll
    for (int q = 0; q < NLD; ++q) {
      const int c = tid + 256 * q;
      if (!TA) {
        const int row = c / KC, kc = (c % KC) * 2;
        // transposed write: XOR-swizzle the row inside its 16-row group by k (bank spread)
        sA[kc * S + (row ^ (kc & 15))] = ra[q].x;
        sA[(kc + 1) * S + (row ^ ((kc + 1) & 15))] = ra[q].y;
      } else {
        const int krow = c / (BM / 2), ic = (c % (BM / 2)) * 2;
        *reinterpret_cast<d2*>(sA + krow * S + ic) = ra[q];
      }
      if (TB) {
        const int row = c / KC, kc = (c % KC) * 2;
        sB[kc * S + (row ^ (kc & 15))] = rb[q].x;
        sB[(kc + 1) * S + (row ^ ((kc + 1) & 15))] = rb[q].y;
      } else {
        const int krow = c / (BN / 2), jc = (c % (BN / 2)) * 2;
        *reinterpret_cast<d2*>(sB + krow * S + jc) = rb[q];
      }
    }
  };

  // Fragment reads are software-pipelined one k-step ahead (two register sets), so the
  // LDS latency of step kk+1 hides under the 16 MFMAs of step kk.
  auto compute = [&](int cur) {
    const double* sA = smem + (cur * 2 + 0) * BK * S;
    const double* sB = smem + (cur * 2 + 1) * BK * S;
    double af[2][MT], bf[2][MT];
    auto fload = [&](int kk, int slot) {
      const int k = kk * 4 + (lane >> 4);
      const int kr = k * S + (lane & 15);
      const int krs = k * S + ((lane & 15) ^ (k & 15));  // swizzled image (transposed writes)
      const int ka = TA ? kr : krs, kb = TB ? krs : kr;
#pragma unroll
      for (int m = 0; m < MT; ++m) af[slot][m] = sA[ka + wr * WT + m * 16];
#pragma unroll
      for (int n = 0; n < MT; ++n) bf[slot][n] = sB[kb + wc * WT + n * 16];
    };
    fload(0, 0);
    // contraction instances: raise the wave's issue priority over its MFMA block (measured at
    // B=128: contraction −1.3 %; on the factor's GEMMs it cost +3.5 %, so only here)
    if constexpr (kContractEpi) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      if (kk + 1 < BK / 4) fload(kk + 1, (kk + 1) & 1);
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < MT; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[kk & 1][m], bf[kk & 1][n], acc[m][n], 0, 0, 0);
    }
    if constexpr (kContractEpi) __builtin_amdgcn_s_setprio(0);
  };

  // Register-staged double buffer; the last K-tile is peeled so the loop body has no
  // conditionals (a conditional prefetch made hipcc shuttle every accumulator between AGPRs
  // and VGPRs once per K-tile). Skipping a wave's all-zero k-tiles in triangular tiles (its
  // quadrant starts WT after the tile's k range) was measured twice and dropped: as a loop split
  // it cost 7 % on full GEMMs through the main loop's scheduling; as guarded peeled head/tail
  // iterations it left the body intact but gained < 1.5 % (the co-resident workgroup's waves,
  // barrier-coupled to their own tile, cannot use the freed MFMA slots).
  const int nk = (kmax - kmin) / BK;
  if (nk > 0) {
    gload(kmin);
    swrite(0);
    __syncthreads();
    int cur = 0;
    for (int kt = 0; kt < nk - 1; ++kt) {
      gload(kmin + (kt + 1) * BK);
      compute(cur);
      swrite(cur ^ 1);
      __syncthreads();
      cur ^= 1;
    }
    compute(cur);
  }

  if constexpr (EPI == EPI_STORE) {
    double* C = a.C + (long long)b * a.sC;
    const long long ldc = a.ldc;
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < MT; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = i0 + wr * WT + m * 16 + (lane >> 4) + 4 * r;
          const int j = j0 + wc * WT + n * 16 + (lane & 15);
          double v = a.alpha * acc[m][n][r];
          if (a.beta != 0.0) v = fma(a.beta, C[i * ldc + j], v);
          C[i * ldc + j] = v;
        }
  } else if constexpr (EPI == EPI_CONTRACT || EPI == EPI_CONTRACT1 || EPI == EPI_CONTRACT2) {
    // derivative registers sized for the batch's largest spec: 1 term (SE / Matern sweeps),
    // 2 terms (sums / products such as Multi-Input_GPR's Exponential x Exponential) or 4
    constexpr int NT = (EPI == EPI_CONTRACT1) ? 1 : (EPI == EPI_CONTRACT2) ? 2 : GPX_MAX_TERMS;
    // Gradient contraction over this lower tile of K⁻¹ = WᵀW (acc = K⁻¹_ij):
    //   g_θ += w_ij (α_i α_j − K⁻¹_ij) ∂K_ij/∂θ,  w = 2 below the diagonal, 1 on it.
    // The accumulators go through LDS in two halves so that the kernel-derivative code runs
    // as a compact loop (keeping its registers out of the MFMA main loop's budget).
    const int D = a.D;
    const int n = a.nvalid[b];
    const double* X = a.X + (long long)b * a.sX;
    const double* al = a.vec + (long long)b * a.sVec;
    const DevSpec spec = a.specs[b];
    // the general (term-interpreter) derivatives of the one- and two-term instances: each
    // stationary term's inputs divided by its ℓ once per row, as small128 does (the quotients its
    // sqdist forms per pair: the same bits), while they fit the GPX_MAX_DIM doubles a row has here
    // (not the fast single-term path below: it stages its inputs pre-scaled already)
    const bool fast1 = (NT == 1) && spec.n_terms == 1 && spec.terms[0].kind >= GPX_SE &&
                       spec.terms[0].kind <= GPX_EXPONENTIAL;
    __shared__ int soff[NT];  // (in LDS: the element loop's registers are at the cap)
    int P = 0;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const bool pre = NT <= 2 && !fast1 && t < spec.n_terms && term_prescaled(spec.terms[t].kind);
      P += pre ? spec.terms[t].dim_count : 0;
    }
    if (D + P > GPX_MAX_DIM) P = 0;
    if (tid == 0) {
      int o = 0;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const bool pre = P > 0 && !fast1 && t < spec.n_terms && term_prescaled(spec.terms[t].kind);
        soff[t] = pre ? (BM + BN) * o : -1;
        o += pre ? spec.terms[t].dim_count : 0;
      }
    }
    double* sacc = smem;                      // [4 waves][16][WT]
    double* sxi = sacc + 4 * 16 * WT;         // [BM][D]
    double* sxj = sxi + BM * D;               // [BN][D]
    // the pre-scaled terms' x/ℓ: term t's at soff[t], [BM + BN][its dims], the tile's rows i0.. then j0..
    double* sxp = sxj + BN * D;
    double* sai = sxp + (BM + BN) * P;        // [BM]
    double* saj = sai + BM;                   // [BN]
    double* sth = saj + BN;                   // [16]
    double* sred = sth + GPX_THETA_STRIDE;    // [4 waves][16]
    __syncthreads();
    // single-term isotropic stationary specs (the SE / Matern / Exponential fits): the inputs
    // are staged pre-scaled by 1/ℓ and ℓ-dependent factors hoisted out of the per-element
    // derivative (no division per element)
    const int fkind = spec.terms[0].kind;
    const bool fast = (NT == 1) && spec.n_terms == 1 && fkind >= GPX_SE && fkind <= GPX_EXPONENTIAL;
    const int fd0 = spec.terms[0].dim_start, fdn = spec.terms[0].dim_count;
    const double fell = a.theta[b * GPX_THETA_STRIDE + spec.terms[0].param_offset];
    const double fvar = a.theta[b * GPX_THETA_STRIDE + spec.terms[0].param_offset + 1];
    const double finv_ell = 1.0 / fell;
    for (int e = tid; e < BM * D; e += 256) {
      const int r = e / D, d = e - (e / D) * D;
      const double xi = (i0 + r < n) ? X[(long long)(i0 + r) * D + d] : 0.0;
      const double xj = (j0 + r < n) ? X[(long long)(j0 + r) * D + d] : 0.0;
      sxi[e] = fast ? xi / fell : xi;
      sxj[e] = fast ? xj / fell : xj;
    }
    if (tid < BM) { sai[tid] = al[i0 + tid]; saj[tid] = al[j0 + tid]; }
    if (tid < GPX_THETA_STRIDE) sth[tid] = a.theta[b * GPX_THETA_STRIDE + tid];
    if (P > 0) {
      const double* th = a.theta + b * GPX_THETA_STRIDE;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        if (soff[t] < 0) continue;
        const gpx_term& tm = spec.terms[t];
        const double ell = th[term_ell_slot(tm)];
        const int dn = tm.dim_count;
        for (int e = tid; e < BM * dn; e += 256) {
          const int r = e / dn, d = tm.dim_start + (e - r * dn);
          sxp[soff[t] + e] = ((i0 + r < n) ? X[(long long)(i0 + r) * D + d] : 0.0) / ell;
          sxp[soff[t] + BM * dn + e] = ((j0 + r < n) ? X[(long long)(j0 + r) * D + d] : 0.0) / ell;
        }
      }
    }
    double sums[NT][3];
#pragma unroll
    for (int t = 0; t < NT; ++t) sums[t][0] = sums[t][1] = sums[t][2] = 0.0;
    double snoise = 0.0;
    // wave-local image [16 rows][WT cols] of one MFMA row-tile per pass;
    // lane -> column cl, rows rg, rg + RG, ...
    constexpr int RG = 64 / WT;
    double* wacc = sacc + wave * (16 * WT);
    const int cl = lane % WT, rg = lane / WT;
    const int jl = wc * WT + cl;            // this lane's column within the tile
    const int j = j0 + jl;
#pragma unroll
    for (int h = 0; h < MT; ++h) {
#pragma unroll
      for (int nn = 0; nn < MT; ++nn)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          wacc[((lane >> 4) + 4 * r) * WT + nn * 16 + (lane & 15)] = acc[h][nn][r];
      __syncthreads();
      if (j < n) {
        const double aj = saj[jl];
#pragma unroll 1
        for (int rr = rg; rr < 16; rr += RG) {
          const int il = wr * WT + h * 16 + rr;
          const int i = i0 + il;
          if (i >= j && i < n) {
            const double w = (i == j) ? 1.0 : 2.0;
            const double v = w * fma(sai[il], aj, -wacc[rr * WT + cl]);
            double dk[NT][3];
            if (fast) {
              stationary_grad(fkind, sqdist_scaled(sxi + il * D + fd0, sxj + jl * D + fd0, fdn), fvar,
                              finv_ell, dk[0]);
            } else if constexpr (NT <= 2) {  // (soff[t] < 0: term t reads X as eval_k_grad does)
              eval_k_grad_pre<NT>(spec, sth, sxi + il * D, sxj + jl * D, sxp, soff, il, BM + jl, dk);
            } else {  // (the four-term instance: its registers are at the cap already)
              eval_k_grad<NT>(spec, sth, sxi + il * D, sxj + jl * D, dk);
            }
#pragma unroll
            for (int t = 0; t < NT; ++t) {
              sums[t][0] = fma(v, dk[t][0], sums[t][0]);
              sums[t][1] = fma(v, dk[t][1], sums[t][1]);
              sums[t][2] = fma(v, dk[t][2], sums[t][2]);
            }
            if (i == j) snoise += v;
          }
        }
      }
      __syncthreads();
    }
    // block reduction of the 13 sums, then scatter to θ positions
    double vals[GPX_MAX_TERMS * 3 + 1];
#pragma unroll
    for (int t = 0; t < GPX_MAX_TERMS; ++t)
#pragma unroll
      for (int q = 0; q < 3; ++q) vals[t * 3 + q] = t < NT ? wave_sum(sums[t][q]) : 0.0;
    vals[GPX_MAX_TERMS * 3] = wave_sum(snoise);
    if (lane == 0) {
#pragma unroll
      for (int v = 0; v < GPX_MAX_TERMS * 3 + 1; ++v) sred[wave * 16 + v] = vals[v];
    }
    __syncthreads();
    if (tid < GPX_THETA_STRIDE) {
      double* out = a.partial + (long long)b * a.sPartial + (long long)tile * GPX_THETA_STRIDE;
      // map slot tid -> θ index
      double s = 0.0;
      int slot = -1;
      if (tid == spec.n_params) {
        slot = GPX_MAX_TERMS * 3;
      } else {
        const DevSpec* gs = a.specs + b;  // dynamic term index: read from memory, not a register copy
        for (int t = 0; t < gs->n_terms; ++t) {
          const int o = gs->terms[t].param_offset, kind = gs->terms[t].kind;
          const int np = (kind == GPX_RQ || kind == GPX_PERIODIC_SE) ? 3 : (kind == GPX_LINEAR ? 1 : 2);
          if (tid >= o && tid < o + np) slot = t * 3 + (tid - o);
        }
      }
      if (slot >= 0) s = sred[slot] + sred[16 + slot] + sred[32 + slot] + sred[48 + slot];
      out[tid] = s;
    }
  } else {  // EPI_COLSUMSQ
    double* scol = smem;  // [2][BN]
    __syncthreads();
#pragma unroll
    for (int nn = 0; nn < MT; ++nn) {
      double s = 0.0;
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) s = fma(acc[m][nn][r], acc[m][nn][r], s);
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      if (lane < 16) scol[wr * BN + wc * WT + nn * 16 + lane] = s;
    }
    __syncthreads();
    if (tid < BN) {
      double* out = a.partial + (long long)b * a.sPartial + (long long)ti * a.ldc;
      out[j0 + tid] = scol[tid] + scol[BN + tid];
    }
  }
}

// 128x128 tiles for operands of at least 512x512, else 64x64 tiles (small recursion levels are
// latency-bound on a single CU per tile otherwise). For the contraction (its per-tile partials
// depend on the tile) the choice depends on the shape only. For store GEMMs (small_tiles: the
// recursion's panels, trailing updates and inverses, and the SVGP chain) it also depends on how
// many problems share the launch — 128-tiles only when they still put a workgroup on every CU —
// which leaves every stored entry's bits unchanged: an entry's sum runs over the same k in the
// same 4-wide MFMA chunks either way (gemm() in gpx_api.hip), so a problem's arithmetic — and
// therefore its fit — is bit-identical whichever other problems are batched with it.
int gemm_tile(const GemmArgs& a, int n_active) {
  if (a.M % 128 != 0 || a.N % 128 != 0) return 64;
  if (a.small_tiles) {
    // launches of a single problem (the SVGP's M x M chain): 128-tiles only when they still
    // put a workgroup on every CU — 64 tiles of 128 on 256 CUs left three quarters idle
    const long long t = a.lower_only ? (long long)(a.M / 128) * (a.M / 128 + 1) / 2
                                     : (long long)(a.M / 128) * (a.N / 128);
    return t * n_active >= 256 ? 128 : 64;
  }
  return (a.M >= 512 && a.N >= 512) ? 128 : 64;
}

template <int BM, int EPI>
static void launch_gemm_t(const GemmArgs& a0, bool ta, bool tb, int n_active, hipStream_t s) {
  GemmArgs a = a0;
  a.n_active = n_active;
  const int ti = a.M / BM, tj = a.N / BM;
  const int ntiles = a.lower_only ? ti * (ti + 1) / 2 : ti * tj;
  const int q = n_active / 8, r = n_active % 8;
  dim3 grid(8 * (q * ntiles + (r * ntiles + 7) / 8));
  if (a.ev_start) {
    auto k = (!ta && !tb) ? gemm_kernel<BM, false, false, EPI> : (!ta && tb) ? gemm_kernel<BM, false, true, EPI>
           : (ta && !tb) ? gemm_kernel<BM, true, false, EPI> : gemm_kernel<BM, true, true, EPI>;
    hipExtLaunchKernelGGL(k, grid, dim3(256), 0, s, a.ev_start, a.ev_stop, 0, a);
    return;
  }
  if (!ta && !tb) hipLaunchKernelGGL((gemm_kernel<BM, false, false, EPI>), grid, dim3(256), 0, s, a);
  else if (!ta && tb) hipLaunchKernelGGL((gemm_kernel<BM, false, true, EPI>), grid, dim3(256), 0, s, a);
  else if (ta && !tb) hipLaunchKernelGGL((gemm_kernel<BM, true, false, EPI>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((gemm_kernel<BM, true, true, EPI>), grid, dim3(256), 0, s, a);
}

void launch_gemm(const GemmArgs& a, int epi, bool ta, bool tb, int n_active, hipStream_t s) {
  // unreachable through the C ABI (shapes are checked against kGemmMaxLd at create/predict);
  // a silent zero-filled operand would be far worse than stopping here
  if (a.lda > kGemmMaxLd || a.ldb > kGemmMaxLd) {
    fprintf(stderr, "gpx: GEMM leading dimension %d/%d exceeds the buffer-load window (%lld)\n",
            a.lda, a.ldb, kGemmMaxLd);
    abort();
  }
  const int bm = gemm_tile(a, n_active);
  if (bm == 128) {
    if (epi == EPI_STORE) launch_gemm_t<128, EPI_STORE>(a, ta, tb, n_active, s);
    else if (epi == EPI_CONTRACT) launch_gemm_t<128, EPI_CONTRACT>(a, ta, tb, n_active, s);
    else if (epi == EPI_CONTRACT1) launch_gemm_t<128, EPI_CONTRACT1>(a, ta, tb, n_active, s);
    else if (epi == EPI_CONTRACT2) launch_gemm_t<128, EPI_CONTRACT2>(a, ta, tb, n_active, s);
    else launch_gemm_t<128, EPI_COLSUMSQ>(a, ta, tb, n_active, s);
  } else {
    if (epi == EPI_STORE) launch_gemm_t<64, EPI_STORE>(a, ta, tb, n_active, s);
    else if (epi == EPI_CONTRACT) launch_gemm_t<64, EPI_CONTRACT>(a, ta, tb, n_active, s);
    else if (epi == EPI_CONTRACT1) launch_gemm_t<64, EPI_CONTRACT1>(a, ta, tb, n_active, s);
    else if (epi == EPI_CONTRACT2) launch_gemm_t<64, EPI_CONTRACT2>(a, ta, tb, n_active, s);
    else launch_gemm_t<64, EPI_COLSUMSQ>(a, ta, tb, n_active, s);
  }
}

// ======================================================================================
// y = M x (row dot products; lower: k <= i). 64 rows per WG, 16 rows per wave.
// ======================================================================================
// Both matrix-vector kernels are HBM streams over W's lower triangle; a workgroup's rate is set
// by the loads each wave keeps in flight (latency-bound otherwise, and the long-row workgroups
// set the kernel's tail), so each wave runs 8 independent row (column) streams and the longest
// workgroups are dispatched first.
__global__ __launch_bounds__(256) void trmv_n_kernel(TrmvArgs a) {
  constexpr int R = 8;
  // 1-D grid, block index major: every problem's longest rows are dispatched before any
  // problem's shorter ones (no long-row workgroup is left for the tail)
  const int na = a.n_active, nb = (a.rows + 63) / 64;
  const int blk = (int)blockIdx.x / na;
  const int b = a.active[(int)blockIdx.x - blk * na];
  const double* M = a.Wm + (long long)b * a.sW;
  const double* x = a.x + (long long)b * a.sx;
  const int nx = a.nvalid ? a.nvalid[b] : a.cols;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rb = a.lower ? nb - 1 - blk : blk;  // longest rows first
  for (int rr = 0; rr < 16; rr += R) {
    const int i0 = rb * 64 + wave * 16 + rr;
    if (i0 >= a.rows) break;
    double s[R];
#pragma unroll
    for (int q = 0; q < R; ++q) s[q] = 0.0;
    const double* r0 = M + (long long)i0 * a.ld;
    // full part: k < i0 is inside every row's triangle (and k < cols), no per-row checks
    const int kfull = a.lower ? min(i0, a.cols) : a.cols;
    const bool rows_ok = i0 + R <= a.rows;
    int k = lane;
    if (rows_ok) {
      for (; k < kfull; k += 64) {
        const double xv = (k < nx) ? x[k] : 0.0;
        double m[R];
#pragma unroll
        for (int q = 0; q < R; ++q) m[q] = r0[(long long)q * a.ld + k];
#pragma unroll
        for (int q = 0; q < R; ++q) s[q] = fma(m[q], xv, s[q]);
      }
    }
    // remainder: entries above the diagonal and rows beyond a.rows read as zero
    const int kend = a.lower ? min(i0 + R, a.cols) : a.cols;
    for (; k < kend; k += 64) {
      const double xv = (k < nx) ? x[k] : 0.0;
#pragma unroll
      for (int q = 0; q < R; ++q)
        if (i0 + q < a.rows && (!a.lower || k <= i0 + q)) s[q] = fma(r0[(long long)q * a.ld + k], xv, s[q]);
    }
#pragma unroll
    for (int q = 0; q < R; ++q) s[q] = wave_sum(s[q]);
    if (lane == 0) {
      double* y = a.y + (long long)b * a.sy;
#pragma unroll
      for (int q = 0; q < R; ++q)
        if (i0 + q < a.rows) y[i0 + q] = s[q];
    }
  }
}

void launch_trmv_n(const TrmvArgs& a, int n_active, hipStream_t s) {
  TrmvArgs t = a;
  t.n_active = n_active;
  hipLaunchKernelGGL(trmv_n_kernel, dim3((a.rows + 63) / 64 * n_active), dim3(256), 0, s, t);
}

// y = Mᵀ x (column sums; lower: i >= j). 64 columns per WG, rows split over 4 waves, 8 row
// loads in flight per lane. Column block 0 (the longest) has the lowest block index.
__global__ __launch_bounds__(256) void trmv_t_kernel(TrmvArgs a) {
  constexpr int R = 8;
  // 1-D grid, column block major (block 0, the longest column, first for every problem)
  const int na = a.n_active;
  const int blk = (int)blockIdx.x / na;
  const int b = a.active[(int)blockIdx.x - blk * na];
  const double* M = a.Wm + (long long)b * a.sW;
  const double* x = a.x + (long long)b * a.sx;
  __shared__ double sred[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j0 = blk * 64, j = j0 + lane;
  const int istart = a.lower ? j0 : 0;
  double s[R];
#pragma unroll
  for (int q = 0; q < R; ++q) s[q] = 0.0;
  if (j < a.cols) {
    int i = istart + wave;
    for (; i + 4 * (R - 1) < a.rows; i += 4 * R) {
      double m[R], xv[R];
#pragma unroll
      for (int q = 0; q < R; ++q) { m[q] = M[(long long)(i + 4 * q) * a.ld + j]; xv[q] = x[i + 4 * q]; }
#pragma unroll
      for (int q = 0; q < R; ++q) s[q] = fma(m[q], xv[q], s[q]);
    }
    for (; i < a.rows; i += 4) s[0] = fma(M[(long long)i * a.ld + j], x[i], s[0]);
  }
  // fixed-order combine (deterministic)
  double t = 0.0;
#pragma unroll
  for (int q = 0; q < R; ++q) t += s[q];
  sred[wave][lane] = t;
  __syncthreads();
  if (wave == 0 && j < a.cols)
    a.y[(long long)b * a.sy + j] = sred[0][lane] + sred[1][lane] + sred[2][lane] + sred[3][lane];
}

__global__ __launch_bounds__(256) void train_pred_kernel(TrainPredArgs a) {
  // (K⁻¹)_jj = Σ_{i≥j} W_ij²: a column stream over W's lower triangle like trmv_t — 1-D grid,
  // column block major (the longest columns of every problem first), 8 loads in flight per lane
  constexpr int R = 8;
  const int na = a.n_active;
  const int blk = (int)blockIdx.x / na;
  const int b = a.active[(int)blockIdx.x - blk * na];
  const double* W = a.W + (long long)b * a.sW;
  __shared__ double sred[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = blk * 64 + lane;
  const int n = a.nvalid[b];
  double s[R];
#pragma unroll
  for (int q = 0; q < R; ++q) s[q] = 0.0;
  if (j < n) {
    int i = blk * 64 + wave;
    for (; i + 4 * (R - 1) < n; i += 4 * R) {
      double w[R];
#pragma unroll
      for (int q = 0; q < R; ++q) w[q] = W[(long long)(i + 4 * q) * a.ld + j];
#pragma unroll
      for (int q = 0; q < R; ++q) s[q] = fma(w[q], w[q], s[q]);
    }
    for (; i < n; i += 4) {
      const double w = W[(long long)i * a.ld + j];
      s[0] = fma(w, w, s[0]);
    }
  }
  double t = 0.0;
#pragma unroll
  for (int q = 0; q < R; ++q) t += s[q];
  sred[wave][lane] = t;
  __syncthreads();
  if (wave == 0 && j < n) {
    const double kinv = (sred[0][lane] + sred[1][lane]) + (sred[2][lane] + sred[3][lane]);
    const double s2 = a.theta[b * GPX_THETA_STRIDE + a.specs[b].n_params];
    const long long ro = (a.orow ? a.orow[b] : b) * a.sOut;
    a.mean[ro + j] = fma(-s2, a.alpha[(long long)b * a.sVec + j], a.Y[(long long)b * a.sY + j]);
    double v = fma(-s2 * s2, kinv, s2);
    if (a.add_noise) v += s2;
    a.var[ro + j] = v;
  }
}

void launch_train_pred(const TrainPredArgs& a, int n_active, int Np, hipStream_t s) {
  TrainPredArgs t = a;
  t.n_active = n_active;
  hipLaunchKernelGGL(train_pred_kernel, dim3(Np / 64 * n_active), dim3(256), 0, s, t);
}

void launch_trmv_t(const TrmvArgs& a, int n_active, hipStream_t s) {
  TrmvArgs t = a;
  t.n_active = n_active;
  hipLaunchKernelGGL(trmv_t_kernel, dim3((a.cols + 63) / 64 * n_active), dim3(256), 0, s, t);
}

// ======================================================================================
// logML and gradient from the per-tile partials: one WG per problem, fixed order.
// ======================================================================================
// The four 64-lane partial sums of a problem (virtual thread v·64 + lane, v = 0..3: the same
// loops, butterflies and combine order either way, so the same bits) formed by four waves at
// once (NW = 4), or by one wave one after another (NW = 1): a one-wave workgroup fits any free
// wave slot, while on a chip full of one-wave sweeps a four-wave one waits until four slots of
// one CU are free at once (≈ 1 ms per call in the call timeline). Calls with few problems (an
// idle chip) keep the four-wave form.
template <int NW>
__global__ __launch_bounds__(64 * NW) void reduce_kernel(ReduceArgs a) {
  const int b = a.active[blockIdx.x];
  const int lane = threadIdx.x & 63;
  __shared__ double sred[4][GPX_THETA_STRIDE + 2];
  const double* part = a.partial + (long long)b * a.sPartial;
  const double* z = a.z + (long long)b * a.sVec;
  const double* ld = a.ldiag + (long long)b * a.sVec;
#pragma unroll 1
  for (int wave = (int)threadIdx.x >> 6; wave < 4; wave += NW) {
    const int tid = wave * 64 + lane;
    double ps[GPX_THETA_STRIDE];
#pragma unroll
    for (int p = 0; p < GPX_THETA_STRIDE; ++p) ps[p] = 0.0;
    for (int t = tid; t < a.ntiles; t += 256) {
#pragma unroll
      for (int p = 0; p < GPX_THETA_STRIDE; ++p) ps[p] += part[(long long)t * GPX_THETA_STRIDE + p];
    }
    double zz = 0.0, sl = 0.0;
    for (int i = tid; i < a.Np; i += 256) {
      zz = fma(z[i], z[i], zz);
      sl += ld[i];
    }
#pragma unroll
    for (int p = 0; p < GPX_THETA_STRIDE; ++p) ps[p] = wave_sum(ps[p]);
    zz = wave_sum(zz);
    sl = wave_sum(sl);
    if (lane == 0) {
#pragma unroll
      for (int p = 0; p < GPX_THETA_STRIDE; ++p) sred[wave][p] = ps[p];
      sred[wave][GPX_THETA_STRIDE] = zz;
      sred[wave][GPX_THETA_STRIDE + 1] = sl;
    }
  }
  __syncthreads();
  const int tid = threadIdx.x;
  if (tid < GPX_THETA_STRIDE + 2) {
    const double v = sred[0][tid] + sred[1][tid] + sred[2][tid] + sred[3][tid];
    double* res = a.results + (long long)b * kResStride;
    if (tid < GPX_THETA_STRIDE) {
      res[1 + tid] = 0.5 * v;
    } else if (tid == GPX_THETA_STRIDE) {
      res[17] = v;
    } else {
      res[18] = v;
    }
  }
  if (tid == 0) {
    double* res = a.results + (long long)b * kResStride;
    const double zz2 = sred[0][GPX_THETA_STRIDE] + sred[1][GPX_THETA_STRIDE] +
                       sred[2][GPX_THETA_STRIDE] + sred[3][GPX_THETA_STRIDE];
    const double sl2 = sred[0][GPX_THETA_STRIDE + 1] + sred[1][GPX_THETA_STRIDE + 1] +
                       sred[2][GPX_THETA_STRIDE + 1] + sred[3][GPX_THETA_STRIDE + 1];
    const int n = a.nvalid[b];
    res[0] = -0.5 * zz2 - sl2 - 0.5 * (double)n * 1.8378770664093453;  // log(2π)
  }
}

void launch_reduce(const ReduceArgs& a, int n_active, hipStream_t s) {
  if (n_active <= 64)
    hipLaunchKernelGGL(reduce_kernel<4>, dim3(n_active), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(reduce_kernel<1>, dim3(n_active), dim3(64), 0, s, a);
}

// ======================================================================================
// Small problems (Np = 64: N <= 64, the reference's weekly and monthly series, N = 19 / 5, and
// every N <= 64 fit): the whole evaluation in ONE launch, one 4-wave workgroup per problem, K in
// LDS — instead of the six-launch chain (build, leaf, two trmv, contraction GEMM, reduce) whose
// launch gaps were most of a solo evaluation's device time at these sizes (VERDICT r05 item 6;
// the reference evaluates one such model at a time, GPR/model_trainer.py:14-19):
//   K = k(X,X) + σn²I (lower, identity padding) → leaf64_lds (Cholesky + W = L⁻¹, log L_ii)
//   z = W y, α = Wᵀ z, logML = −½‖z‖² − Σ log L_ii − n/2 log 2π
//   K⁻¹ = WᵀW (lower tiles on f64 MFMA) and ½ Σ (ααᵀ − K⁻¹) ∘ ∂K/∂θ (weight 2 off the diagonal)
// Writes what the chain writes: W (the 64x64 block, zeros above the diagonal), z, α, log L_ii,
// results [lml, grad, yᵀK⁻¹y, Σ log L_ii], info. A problem's arithmetic depends on its own
// data and Np only (the route is taken for every Np = 64 problem, whatever the call holds).
// grad = 0 (predict's re-factorisation): the factor, z and α only.
// ======================================================================================
// the last act of a small-problem workgroup whose caller polls (GPX_SMALL_POLL): every thread's
// writes to the coherent host block made visible system-wide, then one vector store of the call's
// tag — the host reads the results once all of the call's flags carry it, with no synchronise
__device__ __forceinline__ void small_done(const Small64Args& a) {
  if (!a.done) return;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) *reinterpret_cast<volatile int*>(a.done + blockIdx.x) = a.tag;
}

template <int NT>
__global__ __launch_bounds__(256) void small64_kernel(Small64Args a) {
  constexpr int S = kLeafS;
  __shared__ __attribute__((aligned(16))) double sA[64 * S];  // K, then L (diag), then K⁻¹ (lower tiles)
  __shared__ __attribute__((aligned(16))) double sW[64 * S];  // W = L⁻¹
  __shared__ double sx[64 * GPX_MAX_DIM];
  __shared__ double sth[GPX_THETA_STRIDE];
  __shared__ double sy[64], sz[64], sal[64], sld[64];
  __shared__ double sred[4][GPX_MAX_TERMS * 3 + 3];
  __shared__ int sfail;
  const int b = a.active[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l15 = lane & 15, l4 = lane >> 4;
  const int n = a.nvalid[b], D = a.D;
  const DevSpec spec = a.specs[b];
  const double* X = a.X + (long long)b * a.sX;
  for (int e = tid; e < 64 * D; e += 256) {
    const int r = e / D;
    sx[e] = r < n ? X[(long long)e] : 0.0;
  }
  if (tid < GPX_THETA_STRIDE) sth[tid] = a.theta[b * GPX_THETA_STRIDE + tid];
  if (tid < 64) sy[tid] = tid < n ? a.Y[(long long)b * a.sY + tid] : 0.0;
  if (tid == 0) sfail = -1;
  __syncthreads();
  const double noise = sth[spec.n_params];
  // the 16-blocks that hold data: the leaf skips the identity padding past them (a function of the
  // problem's own n)
  const int nbv = (n + 15) >> 4;
  // K's lower triangle (the identity in the padding); W's block zero (its identity padding blocks
  // past nbv carry their 1s already: the leaf does not visit them)
#pragma unroll 1
  for (int e = tid; e < 4096; e += 256) {
    const int r = e >> 6, c = e & 63;
    double v = 0.0;
    if (c <= r) {
      if (r < n) {
        v = eval_k(spec, sth, sx + r * D, sx + c * D);
        if (r == c) v += noise;
      } else {
        v = (r == c) ? 1.0 : 0.0;
      }
    }
    sA[r * S + c] = v;
    sW[r * S + c] = (r == c && r >= 16 * nbv) ? 1.0 : 0.0;
  }
  __syncthreads();
  switch (nbv) {  // (ends with a barrier; log L_ii in sld)
    case 1: leaf64_lds<true, LeafNoHook, 1>(sA, sW, sld, &sfail); break;
    case 2: leaf64_lds<true, LeafNoHook, 2>(sA, sW, sld, &sfail); break;
    case 3: leaf64_lds<true, LeafNoHook, 3>(sA, sW, sld, &sfail); break;
    default: leaf64_lds<true, LeafNoHook, 4>(sA, sW, sld, &sfail); break;
  }
  // z = W y (wave 0, row per lane), then α = Wᵀ z (column per lane): sequential sums over the
  // rows that hold data (the padding's y, z and W entries off the diagonal are zeros)
  if (wave == 0) {
    double t = 0.0;
    const int kend = lane < n ? lane : -1;
    for (int k = 0; k <= kend; ++k) t = fma(sW[lane * S + k], sy[k], t);
    sz[lane] = t;
  }
  __syncthreads();
  if (wave == 0) {
    double t = 0.0;
    for (int i = n - 1; i >= lane; --i) t = fma(sW[i * S + lane], sz[i], t);
    sal[lane] = t;
  }
  // the factor for predict (W's block, z, α, log L_ii)
  double* W = a.W + (long long)b * a.sMat;
  for (int e = tid; e < 4096; e += 256) {
    const int r = e >> 6, c = e & 63;
    W[(long long)r * a.ld + c] = sW[r * S + c];
  }
  __syncthreads();
  if (tid < 64) {
    a.z[(long long)b * a.sVec + tid] = sz[tid];
    a.alpha[(long long)b * a.sVec + tid] = sal[tid];
    a.ldiag[(long long)b * a.sVec + tid] = sld[tid];
  }
  if (tid == 0 && sfail >= 0 && a.info[b] == 0) a.info[b] = sfail + 1;
  if (!a.grad) return;
  // K⁻¹ = WᵀW on the lower 16x16 tiles (I >= J), k over rows max(I, J)·16 .. 63 (W is lower):
  // D[m][n] = Σ_k W[k][16I + m] W[k][16J + n]; the 10 tiles dealt over the 4 waves
  for (int t = wave; t < nbv * (nbv + 1) / 2; t += 4) {  // (tiles past the data are never read)
    int I = 0;
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    const int J = t - I * (I + 1) / 2;
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    for (int k0 = 16 * I; k0 < 64; k0 += 4) {
      const double av = sW[(k0 + l4) * S + 16 * I + l15];
      const double bv = sW[(k0 + l4) * S + 16 * J + l15];
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) sA[(16 * I + l4 + 4 * q) * S + 16 * J + l15] = acc[q];
  }
  __syncthreads();
  // ½ Σ_{i,j} (α_i α_j − K⁻¹_ij) ∂K_ij/∂θ over the lower triangle (weight 2 off the diagonal)
  double sums[NT][3];
#pragma unroll
  for (int t = 0; t < NT; ++t) sums[t][0] = sums[t][1] = sums[t][2] = 0.0;
  double snoise = 0.0, szz = 0.0, sl = 0.0;
#pragma unroll 1
  for (int e = tid; e < 4096; e += 256) {
    const int i = e >> 6, j = e & 63;
    if (j > i || i >= n) continue;
    const double w = (i == j) ? 1.0 : 2.0;
    const double v = w * fma(sal[i], sal[j], -sA[i * S + j]);
    double dk[NT][3];
    eval_k_grad<NT>(spec, sth, sx + i * D, sx + j * D, dk);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      sums[t][0] = fma(v, dk[t][0], sums[t][0]);
      sums[t][1] = fma(v, dk[t][1], sums[t][1]);
      sums[t][2] = fma(v, dk[t][2], sums[t][2]);
    }
    if (i == j) snoise += v;
  }
  if (tid < 64) {
    szz = sz[tid] * sz[tid];
    sl = sld[tid];
  }
  // fixed-order reduction: wave sums, then the four waves in turn
  constexpr int NV = GPX_MAX_TERMS * 3 + 3;
  double vals[NV];
#pragma unroll
  for (int t = 0; t < GPX_MAX_TERMS; ++t)
#pragma unroll
    for (int q = 0; q < 3; ++q) vals[t * 3 + q] = t < NT ? wave_sum(sums[t][q]) : 0.0;
  vals[NV - 3] = wave_sum(snoise);
  vals[NV - 2] = wave_sum(szz);
  vals[NV - 1] = wave_sum(sl);
  if (lane == 0) {
#pragma unroll
    for (int v = 0; v < NV; ++v) sred[wave][v] = vals[v];
  }
  __syncthreads();
  double* res = a.results + (long long)b * kResStride;
  if (tid < GPX_THETA_STRIDE) {
    int slot = -1;
    if (tid == spec.n_params) {
      slot = NV - 3;
    } else {
      const DevSpec* gs = a.specs + b;
      for (int t = 0; t < gs->n_terms; ++t) {
        const int o = gs->terms[t].param_offset, kind = gs->terms[t].kind;
        const int np = (kind == GPX_RQ || kind == GPX_PERIODIC_SE) ? 3 : (kind == GPX_LINEAR ? 1 : 2);
        if (tid >= o && tid < o + np) slot = t * 3 + (tid - o);
      }
    }
    const double sv = slot >= 0 ? ((sred[0][slot] + sred[1][slot]) + sred[2][slot]) + sred[3][slot] : 0.0;
    res[1 + tid] = 0.5 * sv;
  }
  if (tid == 0) {
    const double zz = ((sred[0][NV - 2] + sred[1][NV - 2]) + sred[2][NV - 2]) + sred[3][NV - 2];
    const double l = ((sred[0][NV - 1] + sred[1][NV - 1]) + sred[2][NV - 1]) + sred[3][NV - 1];
    res[0] = -0.5 * zz - l - 0.5 * (double)n * 1.8378770664093453;  // log(2π)
    res[17] = zz;
    res[18] = l;
  }
  small_done(a);
}

// Np = 128 (N = 65..128: the reference's daily series, N = 89): the same one-launch evaluation on
// eight waves (K's entries and the gradient's are the per-element work; the leaf runs on them too),
// K and then W = L⁻¹ in leaf128's packed lower-block LDS array (78 KiB: a second 128x128 array
// for K⁻¹ would not fit beside it), so the K⁻¹ = WᵀW tiles stay in registers and are contracted
// with (ααᵀ − K⁻¹) ∘ ∂K/∂θ where they are formed. Blocks past the data keep their identity
// padding (leaf128_lds walks the nbv blocks that hold rows < n).
constexpr int kS128Waves = 8;
template <int NT>
__global__ __launch_bounds__(512) void small128_kernel(Small64Args a) {
  __shared__ __attribute__((aligned(16))) double sS[36 * LBS];  // K, then W = L⁻¹ (packed lower blocks)
  __shared__ double sx[128 * GPX_MAX_DIM];
  __shared__ double sxs[128 * GPX_MAX_DIM];  // the stationary terms' inputs over their ℓ (eval_k_pre)
  __shared__ double sth[GPX_THETA_STRIDE];
  __shared__ double sy[128], sz[128], sal[128], sld[128];
  __shared__ double sred[kS128Waves][GPX_MAX_TERMS * 3 + 3];
  __shared__ int sfail, soff[GPX_MAX_TERMS];
  const int b = a.active[blockIdx.x];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l15 = lane & 15, l4 = lane >> 4;
  const int n = a.nvalid[b], D = a.D;
  const DevSpec spec = a.specs[b];
  const double* X = a.X + (long long)b * a.sX;
  for (int e = tid; e < 128 * D; e += 64 * kS128Waves) {
    const int r = e / D;
    sx[e] = r < n ? X[(long long)e] : 0.0;
  }
  if (tid < GPX_THETA_STRIDE) sth[tid] = a.theta[b * GPX_THETA_STRIDE + tid];
  if (tid < 128) {
    sy[tid] = tid < n ? a.Y[(long long)b * a.sY + tid] : 0.0;
    sld[tid] = 0.0;  // (log 1 for the padding rows the leaf does not visit)
  }
  if (tid == 0) {
    sfail = -1;
    // where each stationary term's scaled rows go (while they fit: GPX_MAX_DIM doubles per row)
    int o = 0;
    for (int t = 0; t < GPX_MAX_TERMS; ++t) {
      const int dn = t < spec.n_terms ? spec.terms[t].dim_count : 0;
      const bool pre = t < spec.n_terms && term_prescaled(spec.terms[t].kind) && o + dn <= GPX_MAX_DIM;
      soff[t] = pre ? 128 * o : -1;
      o += pre ? dn : 0;
    }
  }
  __syncthreads();
  // a = x/ℓ of each pre-scaled term, once per row (the quotient its sqdist forms per pair; the
  // one- and two-term instances only: the pointers cost the 3-4-term one registers past 256)
  if constexpr (NT <= 2)
  for (int t = 0; t < spec.n_terms; ++t) {
    if (soff[t] < 0) continue;
    const gpx_term& tm = spec.terms[t];
    const double ell = sth[tm.param_offset + (tm.kind == GPX_RQ ? 1 : 0)];
    for (int e = tid; e < 128 * tm.dim_count; e += 64 * kS128Waves) {
      const int r = e / tm.dim_count, dd = e - r * tm.dim_count;
      sxs[soff[t] + e] = sx[r * D + tm.dim_start + dd] / ell;
    }
  }
  __syncthreads();
  const double noise = sth[spec.n_params];
  const int nbv = (n + 15) >> 4;
  // K's lower blocks (the diagonal blocks whole: zeros above their diagonal), the identity in the
  // padding — which is also W there
#pragma unroll 1
  for (int e = tid; e < 128 * 128; e += 64 * kS128Waves) {
    const int r = e >> 7, c = e & 127;
    if (c > (r | 15)) continue;
    double v = 0.0;
    if (c <= r) {
      if (r < n) {
        if constexpr (NT <= 2)
          v = eval_k_pre(spec, sth, sx + r * D, sx + c * D, sxs, soff, r, c);
        else
          v = eval_k(spec, sth, sx + r * D, sx + c * D);
        if (r == c) v += noise;
      } else {
        v = (r == c) ? 1.0 : 0.0;
      }
    }
    sS[lblk(r >> 4, c >> 4) + (r & 15) * 17 + (c & 15)] = v;
  }
  __syncthreads();
  leaf128_lds(sS, sld, &sfail, nbv);
  auto wat = [&](int i, int k) { return sS[lblk(i >> 4, k >> 4) + (i & 15) * 17 + (k & 15)]; };  // W[i][k], k <= i
  // z = W y (row per thread), then α = Wᵀ z (column per thread), over the rows that hold data
  if (tid < 128) {
    double t = 0.0;
    const int kend = tid < n ? tid : -1;
    for (int k = 0; k <= kend; ++k) t = fma(wat(tid, k), sy[k], t);
    sz[tid] = t;
  }
  __syncthreads();
  if (tid < 128) {
    double t = 0.0;
    for (int i = n - 1; i >= tid; --i) t = fma(wat(i, tid), sz[i], t);
    sal[tid] = t;
  }
  // the factor for predict (W's block, zeros above the diagonal; z, α, log L_ii)
  double* W = a.W + (long long)b * a.sMat;
  for (int e = tid; e < 128 * 128; e += 64 * kS128Waves) {
    const int r = e >> 7, c = e & 127;
    W[(long long)r * a.ld + c] = (c <= r) ? wat(r, c) : 0.0;
  }
  __syncthreads();
  if (tid < 128) {
    a.z[(long long)b * a.sVec + tid] = sz[tid];
    a.alpha[(long long)b * a.sVec + tid] = sal[tid];
    a.ldiag[(long long)b * a.sVec + tid] = sld[tid];
  }
  if (tid == 0 && sfail >= 0 && a.info[b] == 0) a.info[b] = sfail + 1;
  if (!a.grad) return;
  // K⁻¹ = WᵀW on the lower 16x16 tiles (I >= J) of the data blocks, k over rows 16I .. 16nbv − 1
  // (W is lower; the padding rows add exact zeros): acc[q] = K⁻¹[16I + l4 + 4q][16J + l15], then
  // ½ Σ (α_i α_j − K⁻¹_ij) ∂K_ij/∂θ over the tile's lower-triangle entries (weight 2 off the diagonal)
  double sums[NT][3];
#pragma unroll
  for (int t = 0; t < NT; ++t) sums[t][0] = sums[t][1] = sums[t][2] = 0.0;
  double snoise = 0.0, szz = 0.0, sl = 0.0;
  for (int t = wave; t < nbv * (nbv + 1) / 2; t += kS128Waves) {
    int I = 0;
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    const int J = t - I * (I + 1) / 2;
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    for (int kb = I; kb < nbv; ++kb) {
      const int oi = lblk(kb, I), oj = lblk(kb, J);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const double av = sS[oi + (4 * kk + l4) * 17 + l15];
        const double bv = sS[oj + (4 * kk + l4) * 17 + l15];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = 16 * I + l4 + 4 * q, j = 16 * J + l15;
      if (j > i || i >= n) continue;
      const double w = (i == j) ? 1.0 : 2.0;
      const double v = w * fma(sal[i], sal[j], -acc[q]);
      double dk[NT][3];
      if constexpr (NT <= 2)
        eval_k_grad_pre<NT>(spec, sth, sx + i * D, sx + j * D, sxs, soff, i, j, dk);
      else
        eval_k_grad<NT>(spec, sth, sx + i * D, sx + j * D, dk);
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        sums[u][0] = fma(v, dk[u][0], sums[u][0]);
        sums[u][1] = fma(v, dk[u][1], sums[u][1]);
        sums[u][2] = fma(v, dk[u][2], sums[u][2]);
      }
      if (i == j) snoise += v;
    }
  }
  if (tid < 128) {
    szz = sz[tid] * sz[tid];
    sl = sld[tid];
  }
  // fixed-order reduction: wave sums, then the waves in turn
  constexpr int NV = GPX_MAX_TERMS * 3 + 3;
  double vals[NV];
#pragma unroll
  for (int t = 0; t < GPX_MAX_TERMS; ++t)
#pragma unroll
    for (int q = 0; q < 3; ++q) vals[t * 3 + q] = t < NT ? wave_sum(sums[t][q]) : 0.0;
  vals[NV - 3] = wave_sum(snoise);
  vals[NV - 2] = wave_sum(szz);
  vals[NV - 1] = wave_sum(sl);
  if (lane == 0) {
#pragma unroll
    for (int v = 0; v < NV; ++v) sred[wave][v] = vals[v];
  }
  __syncthreads();
  double* res = a.results + (long long)b * kResStride;
  if (tid < GPX_THETA_STRIDE) {
    int slot = -1;
    if (tid == spec.n_params) {
      slot = NV - 3;
    } else {
      const DevSpec* gs = a.specs + b;
      for (int t = 0; t < gs->n_terms; ++t) {
        const int o = gs->terms[t].param_offset, kind = gs->terms[t].kind;
        const int np = (kind == GPX_RQ || kind == GPX_PERIODIC_SE) ? 3 : (kind == GPX_LINEAR ? 1 : 2);
        if (tid >= o && tid < o + np) slot = t * 3 + (tid - o);
      }
    }
    double sv = 0.0;
    if (slot >= 0)
      for (int w = 0; w < kS128Waves; ++w) sv += sred[w][slot];
    res[1 + tid] = 0.5 * sv;
  }
  if (tid == 0) {
    double zz = 0.0, l = 0.0;
    for (int w = 0; w < kS128Waves; ++w) {
      zz += sred[w][NV - 2];
      l += sred[w][NV - 1];
    }
    res[0] = -0.5 * zz - l - 0.5 * (double)n * 1.8378770664093453;  // log(2π)
    res[17] = zz;
    res[18] = l;
  }
  small_done(a);
}

void launch_small128(const Small64Args& a, int max_terms, int n_active, hipStream_t s) {
  auto k = max_terms <= 1 ? small128_kernel<1> : (max_terms == 2 ? small128_kernel<2> : small128_kernel<GPX_MAX_TERMS>);
  hipLaunchKernelGGL(k, dim3(n_active), dim3(64 * kS128Waves), 0, s, a);
}

void launch_small64(const Small64Args& a, int max_terms, int n_active, hipStream_t s) {
  auto k = max_terms <= 1 ? small64_kernel<1> : (max_terms == 2 ? small64_kernel<2> : small64_kernel<GPX_MAX_TERMS>);
  hipLaunchKernelGGL(k, dim3(n_active), dim3(256), 0, s, a);
}

// var_j = k(x*_j, x*_j) − Σ_rowtiles colsum partials (+ σn² for predict_y)
__global__ __launch_bounds__(256) void predvar_kernel(PredVarArgs a) {
  const int b = a.active[blockIdx.y];
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= a.M) return;
  const DevSpec spec = a.specs[b];
  const double* th = a.theta + b * GPX_THETA_STRIDE;
  double thr[GPX_THETA_STRIDE];
#pragma unroll
  for (int p = 0; p < GPX_THETA_STRIDE; ++p) thr[p] = th[p];
  const double* x = a.Xnew + (long long)b * a.sXnew + (long long)j * a.D;
  double xl[GPX_MAX_DIM];
  for (int d = 0; d < a.D; ++d) xl[d] = x[d];
  double kss = eval_kdiag(spec, thr, xl);
  const double* part = a.partial + (long long)b * a.sPartial;
  double s = 0.0;
  for (int t = 0; t < a.nrowtiles; ++t) s += part[(long long)t * a.ldp + j];
  double v = kss - s;
  if (a.add_noise) v += thr[spec.n_params];
  a.var[(long long)b * a.sVar + j] = v;
}

void launch_predvar(const PredVarArgs& a, int n_active, hipStream_t s) {
  hipLaunchKernelGGL(predvar_kernel, dim3((a.M + 255) / 256, n_active), dim3(256), 0, s, a);
}

}  // namespace gpx
