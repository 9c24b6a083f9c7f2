// gpx_band.hip — kernels of the block-banded evaluation path (gfx950, fp64).
//
// When every entry of K = k(X,X) and of every ∂K/∂θ beyond p 64-blocks off the diagonal is
// EXACTLY zero in fp64 (the kernel's exp underflows: SE / Matern / Exponential with a
// lengthscale small against the spacing of sorted inputs — the reference's own regime of
// unnormalised day offsets and GPflow's default ℓ = 1, GPR/data_handler.py:42-44 +
// GPR/model_trainer.py:15), the logML and its gradient need only:
//   L      block-banded Cholesky factor (a dense factorisation produces exact zeros outside the
//          band, so restricting it to the band changes rounding order only),
//   α      K⁻¹y by banded block triangular solves,
//   Z      K⁻¹ restricted to the band (selected inversion, Takahashi recurrences), since
//          ½Σ(ααᵀ − K⁻¹)∘∂K/∂θ has ∂K = 0 outside it.
// Work is O(N·(p·64)²) instead of O(N³). The host (gpx_api.hip) runs the block steps with the
// existing leaf and MFMA GEMM kernels; this file holds the band-specific pieces:
//   band_solve_kernel      z = L⁻¹y and α = L⁻ᵀz over the block band (one workgroup per problem)
//   band_transpose_kernel  mirror a column of Z blocks above the diagonal (the next windows
//                          read Z blocks on both sides)
//   band_contract_kernel   ½Σ w(α_iα_j − Z_ij)∂K_ij/∂θ over the band's lower blocks
//   band_train_pred_kernel predict at the training inputs from α and diag(Z)
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include "gpx_internal.h"
#include "gpx_leaf.h"

namespace gpx {

// Phase timing of the fused sweeps (diagnostic build only: tools/band_phases.py links a
// libgpx_phases.so compiled with -DGPX_BAND_PHASES). Thread 0 of each workgroup adds the
// shader-clock cycles of each phase of its block steps into g_band_phase[kernel][phase].
#ifdef GPX_BAND_PHASES
__device__ unsigned long long g_band_phase[4][16];
#define PH_BEGIN unsigned long long ph_t = __builtin_amdgcn_s_memtime(), ph_acc[12] = {};
#define PH(i)                                                              \
  do {                                                                     \
    const unsigned long long ph_n = __builtin_amdgcn_s_memtime();          \
    ph_acc[i] += ph_n - ph_t;                                              \
    ph_t = ph_n;                                                           \
  } while (0)
#define PH_END(kid)                                                               \
  do {                                                                            \
    if (threadIdx.x == 0) {                                                       \
      for (int ph_i = 0; ph_i < 12; ++ph_i) atomicAdd(&g_band_phase[kid][ph_i], ph_acc[ph_i]); \
      atomicAdd(&g_band_phase[kid][15], 1ull);                                    \
    }                                                                             \
  } while (0)
#else
#define PH_BEGIN
#define PH(i) \
  do {        \
  } while (0)
#define PH_END(kid) \
  do {              \
  } while (0)
#endif

namespace {
__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
}  // namespace

// One workgroup (4 waves) per problem; z/α for the whole problem in LDS (Np doubles, dynamic).
// forward  z_k = W_kk (y_k − Σ_{j=k−p}^{k−1} L_kj z_j)
// backward α_k = W_kkᵀ (z_k − Σ_{i=k+1}^{k+p} L_ikᵀ α_i)     (α_k overwrites z_k in LDS)
// W_kk = L_kk⁻¹ (the leaves' diagonal blocks of W), L_ij the panels written into L.
__global__ __launch_bounds__(256) void band_solve_kernel(BandSolveArgs a) {
  extern __shared__ double sv[];          // [Np]: z, then α
  __shared__ double st[64];               // the current block's right-hand side
  __shared__ double sp[4][64];            // per-wave column partials (backward)
  const int b = a.active[blockIdx.x];
  const int Np = a.Np, nb = Np / 64, p = a.p, ld = a.ld;
  const double* W = a.W + (long long)b * a.sMat;
  const double* L = a.L + (long long)b * a.sMat;
  const double* y = a.Y + (long long)b * a.sY;
  const int n = a.nvalid[b];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // forward: rows of block k over the waves (16 each), columns over the lanes
  for (int k = 0; k < nb; ++k) {
    const int r0 = k * 64, lo = k - p > 0 ? k - p : 0;
    for (int rr = 0; rr < 16; ++rr) {
      const int r = r0 + wave * 16 + rr;
      double s = 0.0;
      const double* Lr = L + (long long)r * ld;
      for (int c = lo * 64 + lane; c < r0; c += 64) s = fma(Lr[c], sv[c], s);
      s = wsum(s);
      if (lane == 0) st[wave * 16 + rr] = (r < n ? y[r] : 0.0) - s;
    }
    __syncthreads();
    for (int rr = 0; rr < 16; ++rr) {
      const int rl = wave * 16 + rr;
      const double* Wr = W + (long long)(r0 + rl) * ld + r0;
      double s = (lane <= rl) ? Wr[lane] * st[lane] : 0.0;
      s = wsum(s);
      if (lane == 0) sv[r0 + rl] = s;
    }
    __syncthreads();
  }
  for (int i = tid; i < Np; i += 256) a.z[(long long)b * a.sVec + i] = sv[i];
  __syncthreads();
  // backward: columns of block k over the lanes, rows split over the waves
  for (int k = nb - 1; k >= 0; --k) {
    const int c0 = k * 64, hi = (k + p < nb - 1 ? k + p : nb - 1) * 64 + 64;
    double s = 0.0;
    for (int r = c0 + 64 + wave; r < hi; r += 4) s = fma(L[(long long)r * ld + c0 + lane], sv[r], s);
    sp[wave][lane] = s;
    __syncthreads();
    if (wave == 0) st[lane] = sv[c0 + lane] - ((sp[0][lane] + sp[1][lane]) + (sp[2][lane] + sp[3][lane]));
    __syncthreads();
    // α_k[c] = Σ_{r >= c} W_kk[r][c] t[r]
    s = 0.0;
    for (int r = wave; r < 64; r += 4) s = (r >= lane) ? fma(W[(long long)(c0 + r) * ld + c0 + lane], st[r], s) : s;
    sp[wave][lane] = s;
    __syncthreads();
    if (wave == 0) sv[c0 + lane] = (sp[0][lane] + sp[1][lane]) + (sp[2][lane] + sp[3][lane]);
    __syncthreads();
  }
  for (int i = tid; i < Np; i += 256) a.alpha[(long long)b * a.sVec + i] = sv[i];
}

void launch_band_solve(const BandSolveArgs& a, int n_active, hipStream_t s) {
  hipLaunchKernelGGL(band_solve_kernel, dim3(n_active), dim3(256), (size_t)a.Np * sizeof(double), s, a);
}

// Z[k][k+d] = Z[k+d][k]ᵀ for d = 1..q (64x64 blocks through LDS, coalesced both ways)
__global__ __launch_bounds__(256) void band_transpose_kernel(BandTransposeArgs a) {
  __shared__ double t[64][65];
  const int b = a.active[blockIdx.y];
  const int d = blockIdx.x + 1;
  double* Z = a.Z + (long long)b * a.sMat;
  const long long ld = a.ld;
  const int r0 = (a.k + d) * 64, c0 = a.k * 64;
  const int tid = threadIdx.x, c = tid & 63;
  for (int r = tid >> 6; r < 64; r += 4) t[r][c] = Z[(r0 + r) * ld + c0 + c];
  __syncthreads();
  for (int r = tid >> 6; r < 64; r += 4) Z[(c0 + r) * ld + r0 + c] = t[c][r];
}

void launch_band_transpose(const BandTransposeArgs& a, int q, int n_active, hipStream_t s) {
  hipLaunchKernelGGL(band_transpose_kernel, dim3(q, n_active), dim3(256), 0, s, a);
}

// Gradient contraction over the lower blocks of the band: block (k, k−d), tile t = d·nb + k
// (offset-major, so a tile's index does not depend on the launch's p). Writes the same
// [tile][16] θ-slot partials as the dense contraction epilogue; tiles with k < d are zero.
template <int NT>
__global__ __launch_bounds__(256) void band_contract_kernel(BandContractArgs a) {
  __shared__ double sxi[64 * GPX_MAX_DIM], sxj[64 * GPX_MAX_DIM];
  __shared__ double sai[64], saj[64], sth[GPX_THETA_STRIDE];
  __shared__ double sred[4][16];
  const int b = a.active[blockIdx.y];
  const int nb = a.Np / 64;
  const int tile = blockIdx.x, d = tile / nb, k = tile - d * nb;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  double* out = a.partial + (long long)b * a.sPartial + (long long)tile * GPX_THETA_STRIDE;
  if (k < d) {
    if (tid < GPX_THETA_STRIDE) out[tid] = 0.0;
    return;
  }
  const int i0 = k * 64, j0 = (k - d) * 64, D = a.D;
  const int n = a.nvalid[b];
  const double* X = a.X + (long long)b * a.sX;
  const double* al = a.alpha + (long long)b * a.sVec;
  const DevSpec spec = a.specs[b];
  const int fkind = spec.terms[0].kind;
  const bool fast = (NT == 1) && spec.n_terms == 1 && fkind >= GPX_SE && fkind <= GPX_EXPONENTIAL;
  const int fd0 = spec.terms[0].dim_start, fdn = spec.terms[0].dim_count;
  const double fell = a.theta[b * GPX_THETA_STRIDE + spec.terms[0].param_offset];
  const double fvar = a.theta[b * GPX_THETA_STRIDE + spec.terms[0].param_offset + 1];
  const double finv_ell = 1.0 / fell;
  // one stationary term: inputs staged pre-scaled by 1/ℓ (GPflow's Stationary.scale)
  for (int e = tid; e < 64 * D; e += 256) {
    const int r = e / D, dd = e - (e / D) * D;
    const double xi = (i0 + r < n) ? X[(long long)(i0 + r) * D + dd] : 0.0;
    const double xj = (j0 + r < n) ? X[(long long)(j0 + r) * D + dd] : 0.0;
    sxi[e] = fast ? xi / fell : xi;
    sxj[e] = fast ? xj / fell : xj;
  }
  if (tid < 64) { sai[tid] = al[i0 + tid]; saj[tid] = al[j0 + tid]; }
  if (tid < GPX_THETA_STRIDE) sth[tid] = a.theta[b * GPX_THETA_STRIDE + tid];
  __syncthreads();
  const double* Z = a.Z + (long long)b * a.sMat;
  double sums[NT][3];
#pragma unroll
  for (int t = 0; t < NT; ++t) sums[t][0] = sums[t][1] = sums[t][2] = 0.0;
  double snoise = 0.0;
  const int jl = lane, j = j0 + jl;
  if (j < n) {
    const double aj = saj[jl];
#pragma unroll 1
    for (int il = wave; il < 64; il += 4) {
      const int i = i0 + il;
      if (i >= n || (d == 0 && il < jl)) continue;
      const double w = (d == 0 && il == jl) ? 1.0 : 2.0;
      const double zij = Z[(long long)i * a.ld + j];
      const double v = w * fma(sai[il], aj, -zij);
      double dk[NT][3];
      double kij;
      if (fast) {
        stationary_grad(fkind, sqdist_scaled(sxi + il * D + fd0, sxj + jl * D + fd0, fdn), fvar, finv_ell, dk[0]);
        kij = fvar * dk[0][1];
      } else {
        kij = eval_k_grad<NT>(spec, sth, sxi + il * D, sxj + jl * D, dk);
      }
      // band check: Σ_i K_ji Z_ij for column j (and, by symmetry, column i)
      if (i == j) kij += sth[spec.n_params];
      const double kz = kij * zij;
      atomicAdd(a.colsum + (long long)b * a.sCol + j, kz);
      if (i != j) atomicAdd(a.colsum + (long long)b * a.sCol + i, kz);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        sums[t][0] = fma(v, dk[t][0], sums[t][0]);
        sums[t][1] = fma(v, dk[t][1], sums[t][1]);
        sums[t][2] = fma(v, dk[t][2], sums[t][2]);
      }
      if (i == j) snoise += v;
    }
  }
  double vals[GPX_MAX_TERMS * 3 + 1];
#pragma unroll
  for (int t = 0; t < GPX_MAX_TERMS; ++t)
#pragma unroll
    for (int q = 0; q < 3; ++q) vals[t * 3 + q] = t < NT ? wsum(sums[t][q]) : 0.0;
  vals[GPX_MAX_TERMS * 3] = wsum(snoise);
  if (lane == 0) {
#pragma unroll
    for (int v = 0; v < GPX_MAX_TERMS * 3 + 1; ++v) sred[wave][v] = vals[v];
  }
  __syncthreads();
  if (tid < GPX_THETA_STRIDE) {
    double s = 0.0;
    int slot = -1;
    if (tid == spec.n_params) {
      slot = GPX_MAX_TERMS * 3;
    } else {
      const DevSpec* gs = a.specs + b;
      for (int t = 0; t < gs->n_terms; ++t) {
        const int o = gs->terms[t].param_offset, kind = gs->terms[t].kind;
        const int np = (kind == GPX_RQ || kind == GPX_PERIODIC_SE) ? 3 : (kind == GPX_LINEAR ? 1 : 2);
        if (tid >= o && tid < o + np) slot = t * 3 + (tid - o);
      }
    }
    if (slot >= 0) s = (sred[0][slot] + sred[1][slot]) + (sred[2][slot] + sred[3][slot]);
    out[tid] = s;
  }
}

__global__ __launch_bounds__(256) void band_check_kernel(const int* active, const double* colsum, long long sCol,
                                                        const int* nvalid, double* results) {
  __shared__ double sm[4];
  const int b = active[blockIdx.x];
  const int n = nvalid[b], tid = threadIdx.x;
  double m = 0.0;
  for (int j = tid; j < n; j += 256) {
    const double r = fabs(colsum[(long long)b * sCol + j] - 1.0);
    m = (r == r) ? fmax(m, r) : INFINITY;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
  if ((tid & 63) == 0) sm[tid >> 6] = m;
  __syncthreads();
  if (tid == 0) results[(long long)b * kResStride + kResBandCheck] = fmax(fmax(sm[0], sm[1]), fmax(sm[2], sm[3]));
}

void launch_band_check(const int* active, const double* colsum, long long sCol, const int* nvalid,
                       double* results, int n_active, int Np, hipStream_t s) {
  (void)Np;
  hipLaunchKernelGGL(band_check_kernel, dim3(n_active), dim3(256), 0, s, active, colsum, sCol, nvalid, results);
}

void launch_band_contract(const BandContractArgs& a, int max_terms, int n_active, hipStream_t s) {
  const dim3 grid((a.p + 1) * (a.Np / 64), n_active);
  if (max_terms <= 1) hipLaunchKernelGGL(band_contract_kernel<1>, grid, dim3(256), 0, s, a);
  else if (max_terms == 2) hipLaunchKernelGGL(band_contract_kernel<2>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(band_contract_kernel<GPX_MAX_TERMS>, grid, dim3(256), 0, s, a);
}

// predict_f / predict_y at the training inputs from a banded factorisation:
//   mean_j = y_j − σn² α_j,  var_j = σn² − σn⁴ Z_jj  (+σn²)   (as train_pred_kernel, with the
// diagonal of K⁻¹ read from the selected inverse instead of Σ_i W_ij²)
// (one-wave workgroups, as the reduce kernel: they fit any free wave slot)
__global__ __launch_bounds__(64) void band_train_pred_kernel(TrainPredArgs a) {
  const int b = a.active[blockIdx.y];
  const int j = blockIdx.x * 64 + threadIdx.x;
  const int n = a.nvalid[b];
  if (j >= n) return;
  const double s2 = a.theta[b * GPX_THETA_STRIDE + a.specs[b].n_params];
  const double zjj = a.W[(long long)b * a.sW + (long long)j * a.ld + j];
  const long long ro = (a.orow ? a.orow[b] : b) * a.sOut;
    a.mean[ro + j] = fma(-s2, a.alpha[(long long)b * a.sVec + j], a.Y[(long long)b * a.sY + j]);
  double v = fma(-s2 * s2, zjj, s2);
  if (a.add_noise) v += s2;
  a.var[ro + j] = v;
}

void launch_band_train_pred(const TrainPredArgs& a, int n_active, int Np, hipStream_t s) {
  hipLaunchKernelGGL(band_train_pred_kernel, dim3((Np + 63) / 64, n_active), dim3(64), 0, s, a);
}

// =======================================================================================
// Fused banded evaluation, band width p <= 2 blocks (the C2 regime: p = 1 or 2 at ℓ ≈ 1-1.7):
// the whole per-problem block sweep in one workgroup, in two launches instead of ~9 per block.
//   band_fwd_kernel: for k = 0..nb−1: leaf on A_kk -> W_kk (and log L_ii); z_k = W_kk(y_k + u_k);
//                    panels P_i = A_{k+i,k} W_kkᵀ; u_{k+i} −= P_i z_k (right-looking solve);
//                    A_{k+i,k+j} −= P_i P_jᵀ
//   band_bwd_kernel: for k = nb−1..0: α_k = W_kkᵀ(z_k − Σ P_iᵀ α_{k+i}); G_i = P_i W_kk;
//                    Z_{k+i,k} = −Σ_j Z_{k+i,k+j} G_j; Z_kk = W_kkᵀW_kk − Σ G_iᵀ Z_{k+i,k};
//                    and the gradient contraction of the three new Z blocks on their registers
// 64x64 operands are staged in LDS (row stride kLeafS); every product is a 64³ f64-MFMA block
// product by the 4 waves (a 32x32 quadrant each).
// =======================================================================================
namespace {
typedef double bd4 __attribute__((ext_vector_type(4)));
constexpr int BS = kLeafS;

struct Frag {
  bd4 c[2][2];
};

__device__ __forceinline__ void frag_zero(Frag& f) {
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n) f.c[m][n] = (bd4){0.0, 0.0, 0.0, 0.0};
}

// threadIdx.x through an empty asm: address arithmetic built on it is recomputed where it is
// used instead of being hoisted out of the block-step loops (where the 64-bit row offsets of
// every 64x64 block access would otherwise pin ~30 registers and spill)
__device__ __forceinline__ int tid_fresh() {
  int t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

// f += ±opA·opB over 64 k; A and B 64x64 in LDS. TA: opA(i,k) = A[k][i]; TB: opB(k,j) = B[j][k].
template <bool TA, bool TB, int U = 4>
__device__ __forceinline__ void frag_mma(Frag& f, const double* __restrict__ sA, const double* __restrict__ sB,
                                         bool neg) {
  const int t = tid_fresh();
  const int lane = t & 63, wave = t >> 6;
  const int wr = wave >> 1, wc = wave & 1, l15 = lane & 15, l4 = lane >> 4;
  const double sg = neg ? -1.0 : 1.0;
#pragma unroll U
  for (int kk = 0; kk < 16; ++kk) {
    const int k = kk * 4 + l4;
    double av[2], bv[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int i = wr * 32 + m * 16 + l15;
      av[m] = sg * (TA ? sA[k * BS + i] : sA[i * BS + k]);
    }
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int j = wc * 32 + n * 16 + l15;
      bv[n] = TB ? sB[j * BS + k] : sB[k * BS + j];
    }
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n) f.c[m][n] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[m], bv[n], f.c[m][n], 0, 0, 0);
  }
}

// (row, col) of fragment element c[m][n][r] of this lane
__device__ __forceinline__ int frag_row(int m, int r) {
  return (threadIdx.x >> 7) * 32 + m * 16 + ((threadIdx.x & 63) >> 4) + 4 * r;
}
__device__ __forceinline__ int frag_col(int n) {
  return ((threadIdx.x >> 6) & 1) * 32 + n * 16 + (threadIdx.x & 15);
}

__device__ __forceinline__ void frag_load_global(Frag& f, const double* __restrict__ g, int ld) {
  const int t = tid_fresh();
  g += ((t >> 7) * 32 + ((t & 63) >> 4)) * ld + ((t >> 6) & 1) * 32 + (t & 15);
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) f.c[m][n][r] = g[(m * 16 + 4 * r) * ld + n * 16];
}
__device__ __forceinline__ void frag_store_global(const Frag& f, double* __restrict__ g, int ld) {
  const int t = tid_fresh();
  g += ((t >> 7) * 32 + ((t & 63) >> 4)) * ld + ((t >> 6) & 1) * 32 + (t & 15);
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) g[(m * 16 + 4 * r) * ld + n * 16] = f.c[m][n][r];
}
__device__ __forceinline__ void frag_store_lds(const Frag& f, double* __restrict__ s) {
  const int t = tid_fresh();
  s += ((t >> 7) * 32 + ((t & 63) >> 4)) * BS + ((t >> 6) & 1) * 32 + (t & 15);
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) s[(m * 16 + 4 * r) * BS + n * 16] = f.c[m][n][r];
}

// 64x64 block global -> registers (element e = tid + 256u: row e>>6, column e&63), so the loads can be issued a phase ahead and stored to LDS later
__device__ __forceinline__ void block_fetch(double (&v)[16], const double* __restrict__ g, int ld) {
  const int tid = tid_fresh();
  g += (tid >> 6) * ld + (tid & 63);
#pragma unroll
  for (int u = 0; u < 16; ++u) v[u] = g[4 * u * ld];
}
__device__ __forceinline__ void block_store_lds(const double (&v)[16], double* __restrict__ s) {
  const int tid = tid_fresh();
  s += (tid >> 6) * BS + (tid & 63);
#pragma unroll
  for (int u = 0; u < 16; ++u) s[4 * u * BS] = v[u];
}
// the diagonal of a fragment-held block -> global (the selected inverse's diag(K⁻¹), read by
// band_train_pred_kernel)
__device__ __forceinline__ void frag_store_diag(const Frag& f, double* __restrict__ g, int ld) {
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = frag_row(m, r), j = frag_col(n);
        if (i == j) g[i * ld + j] = f.c[m][n][r];
      }
}

// ---- 16x16-tile primitives of the p <= 1 sweeps (band_fwd1_kernel / band_bwd1_kernel) ----
// A tile's C fragment (v_mfma_f64_16x16x4_f64): lane holds rows l4 + 4r (r = 0..3), column l15.
__device__ __forceinline__ void tile_zero(bd4& c) { c = (bd4){0.0, 0.0, 0.0, 0.0}; }
__device__ __forceinline__ void tile_store_lds(const bd4& c, double* __restrict__ s, int i0, int j0) {
  const int lane = tid_fresh() & 63;
  double* p = s + (i0 + (lane >> 4)) * BS + j0 + (lane & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) p[4 * r * BS] = c[r];
}
// the tile's transpose at (j0, i0)
__device__ __forceinline__ void tile_store_lds_t(const bd4& c, double* __restrict__ s, int i0, int j0) {
  const int lane = tid_fresh() & 63;
  double* p = s + (j0 + (lane & 15)) * BS + i0 + (lane >> 4);
#pragma unroll
  for (int r = 0; r < 4; ++r) p[4 * r] = c[r];
}
__device__ __forceinline__ void tile_load_lds(bd4& c, const double* __restrict__ s, int i0, int j0) {
  const int lane = tid_fresh() & 63;
  const double* p = s + (i0 + (lane >> 4)) * BS + j0 + (lane & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) c[r] = p[4 * r * BS];
}
__device__ __forceinline__ void tile_load_global(bd4& c, const double* __restrict__ g, long long ld, int i0, int j0) {
  const int lane = tid_fresh() & 63;
  const double* p = g + (long long)(i0 + (lane >> 4)) * ld + j0 + (lane & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) c[r] = p[4 * r * ld];
}
__device__ __forceinline__ void tile_store_global(const bd4& c, double* __restrict__ g, long long ld, int i0, int j0) {
  const int lane = tid_fresh() & 63;
  double* p = g + (long long)(i0 + (lane >> 4)) * ld + j0 + (lane & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) p[4 * r * ld] = c[r];
}

// Tile row ib (tiles (ib, jb), jb = 0..3) of ±opA · opB over the 64 k, skipping the k-blocks a
// triangular operand makes exactly zero: MODE 0 every k-block; MODE 1 k-blocks kb <= jb
// (opB = Wᵀ, W lower triangular: P = A Wᵀ); MODE 2 kb >= jb (opB = W lower: G = P W). One wave;
// the A fragment of each k-step is shared by the row's tiles. TA: opA(i,k) = A[k][i];
// TB: opB(k,j) = B[j][k].
template <bool TA, bool TB, int MODE>
__device__ __forceinline__ void row_mma(bd4 (&c)[4], const double* __restrict__ sA, const double* __restrict__ sB,
                                        int i0, bool neg) {
  const int lane = tid_fresh() & 63, l15 = lane & 15, l4 = lane >> 4;
  const double sg = neg ? -1.0 : 1.0;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = kb * 16 + q * 4 + l4;
      const double av = sg * (TA ? sA[k * BS + i0 + l15] : sA[(i0 + l15) * BS + k]);
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        if (MODE == 1 && kb > jb) continue;
        if (MODE == 2 && kb < jb) continue;
        const double bv = TB ? sB[(jb * 16 + l15) * BS + k] : sB[k * BS + jb * 16 + l15];
        c[jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, c[jb], 0, 0, 0);
      }
    }
}

// The 10 lower 16x16 tiles of a symmetric 64x64 product over the 4 waves, up to 3 per wave
// (slot s of wave w: (ib, jb), ib >= jb), balanced for the backward sweep's Z_kk = WᵀW − GᵀZ1
// (WᵀW's tile (ib, jb) has 4 − ib nonzero k-blocks, W lower triangular): every wave 20 k-steps of
// WᵀW, 32 or 48 of GᵀZ1 (a 2x2-quadrant split: 64 and 64).
//   w0: (0,0) (3,0) | w1: (1,0) (2,0) | w2: (1,1) (3,1) (3,2) | w3: (2,1) (2,2) (3,3)
__device__ __forceinline__ bool sym_tile(int w, int s, int& ib, int& jb) {
  const unsigned long long T = 0x7a92e6960824180ull;  // 5 bits per (w, s): ib * 4 + jb, 16 = none
  const int v = (int)((T >> (5 * (w * 3 + s))) & 31ull);
  ib = v >> 2;
  jb = v & 3;
  return v < 16;
}

// c[s] += ±opA · opB on this wave's symmetric tiles; TRI: k-blocks from max(ib, jb) only
// (opA = Wᵀ, opB = W with W lower triangular: WᵀW)
template <bool TA, bool TB, bool TRI>
__device__ __forceinline__ void sym_mma(bd4 (&c)[3], const double* __restrict__ sA, const double* __restrict__ sB,
                                        int w, bool neg) {
  const int lane = tid_fresh() & 63, l15 = lane & 15, l4 = lane >> 4;
  const double sg = neg ? -1.0 : 1.0;
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    int ib, jb;
    if (!sym_tile(w, s, ib, jb)) continue;
    const int i0 = ib * 16, j0 = jb * 16, kb0 = TRI ? ib : 0;   // (ib >= jb: max(ib, jb) = ib)
#pragma unroll 1
    for (int kb = kb0; kb < 4; ++kb) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = kb * 16 + q * 4 + l4;
        const double av = sg * (TA ? sA[k * BS + i0 + l15] : sA[(i0 + l15) * BS + k]);
        const double bv = TB ? sB[(j0 + l15) * BS + k] : sB[k * BS + j0 + l15];
        c[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, c[s], 0, 0, 0);
      }
    }
  }
}
__device__ __forceinline__ void sym_zero(bd4 (&c)[3]) {
#pragma unroll
  for (int s = 0; s < 3; ++s) tile_zero(c[s]);
}
__device__ __forceinline__ void sym_load_global(bd4 (&c)[3], const double* __restrict__ g, long long ld, int w) {
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    int ib, jb;
    if (sym_tile(w, s, ib, jb)) tile_load_global(c[s], g, ld, ib * 16, jb * 16);
  }
}
// lower tiles only (the leaf reads the lower triangle of its input)
__device__ __forceinline__ void sym_store_lds(const bd4 (&c)[3], double* __restrict__ s, int w) {
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    int ib, jb;
    if (sym_tile(w, t, ib, jb)) tile_store_lds(c[t], s, ib * 16, jb * 16);
  }
}
// lower tiles and their mirror images: the full symmetric matrix
__device__ __forceinline__ void sym_store_lds_full(const bd4 (&c)[3], double* __restrict__ s, int w) {
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    int ib, jb;
    if (!sym_tile(w, t, ib, jb)) continue;
    tile_store_lds(c[t], s, ib * 16, jb * 16);
    if (ib != jb) tile_store_lds_t(c[t], s, ib * 16, jb * 16);
  }
}
// the diagonal of the matrix (its diagonal tiles') -> g[i * ld + i]
__device__ __forceinline__ void sym_store_diag(const bd4 (&c)[3], double* __restrict__ g, long long ld, int w) {
  const int lane = tid_fresh() & 63, l15 = lane & 15, l4 = lane >> 4;
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    int ib, jb;
    if (!sym_tile(w, t, ib, jb) || ib != jb) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (l4 + 4 * r == l15) g[(long long)(ib * 16 + l15) * ld + ib * 16 + l15] = c[t][r];
  }
}

// X rows of one 64-row block -> LDS in two parts: xrows_fetch loads the first 256 elements
// (all of it for D <= 4) into a register a phase ahead, from a clamped (always valid) address
// and without a branch, so the load stays in flight; xrows_store writes it and loads any rest
__device__ __forceinline__ double xrows_fetch(const double* __restrict__ X, int r0, int n, int D) {
  const int e = tid_fresh();
  const int idx = min(r0 * D + e, n * D - 1);
  const double v = X[idx];
  return (e < 64 * D && r0 + e / D < n) ? v : 0.0;
}
// (scaled by 1/ell, a division as GPflow's Stationary.scale; ell = 1 stores them as they are)
__device__ __forceinline__ void xrows_store(double xr, double* __restrict__ s, const double* __restrict__ X,
                                            int r0, int n, int D, double ell) {
  const int nx = 64 * D, tid = threadIdx.x;
  if (tid < nx) s[tid] = xr / ell;
  for (int e = tid + 256; e < nx; e += 256) s[e] = (r0 + e / D < n) ? X[r0 * D + e] / ell : 0.0;
}

// Kernel-function context of one problem's gradient contraction
template <int NT>
struct ContractCtx {
  const DevSpec* spec;
  const double* sth;
  int D, n, fkind, fd0, fdn;
  bool fast;  // one stationary term (SE / Matern / Exponential): closed form below
  double fvar, finv_ell, noise;
  double xscale;  // the X rows in LDS are divided by this: ℓ when fast, else 1
  double sums[NT][3];
  double snoise;
};

// Gradient contraction of one 64x64 Z block staged in LDS (rows i0.., columns j0..; lanes over
// the columns, each wave over 16 rows): Σ w (α_i α_j − Z_ij) ∂K_ij/∂θ into cx.sums, and the
// products K_ij Z_ij into colacc (this thread's column). A diagonal block is taken whole (both
// triangles, w = 1: Z_kk and K_kk are symmetric); an off-diagonal block stands for itself and
// its mirror (w = 2), and its K_ij Z_ij overwrite Z in place for the row sums (block_rowsum).
// Inputs come from LDS: Z, the α slices and the X rows of both blocks (sxi, sxj; pre-scaled by
// 1/ℓ when cx.fast).
// The same for the reference's kernel (one SquaredExponential term on one input column), as
// straight-line code: r² = sqdist1(a_i, a_j) (GPflow's square_distance), g = exp(−r²/2),
// ∂K/∂ℓ = σ² g r²/ℓ, ∂K/∂σ² = g (stationary_grad's SE case, operation for operation)
template <int NT>
__device__ __forceinline__ void contract_block_se1(ContractCtx<NT>& cx, double* __restrict__ sZ,
                                                   const double* __restrict__ sxi, const double* __restrict__ sxj,
                                                   int i0, int j0, const double* __restrict__ ai,
                                                   const double* __restrict__ aj, bool diag, double& colacc) {
  const int lane = threadIdx.x & 63, part = threadIdx.x >> 6;
  const int jl = lane, j = j0 + jl, D = cx.D, d0 = cx.fd0;
  const double ajl = aj[jl], w = diag ? 1.0 : 2.0, xj = sxj[jl * D + d0];
  const double var = cx.fvar, inv_ell = cx.finv_ell;
  const bool jok = j < cx.n;
  double s0 = 0.0, s1 = 0.0, sn = 0.0, ca = 0.0;
#pragma unroll 4
  for (int t = 0; t < 16; ++t) {
    const int il = part * 16 + t, i = i0 + il;
    const double zij = sZ[il * BS + jl];
    const double r2 = sqdist1(sxi[il * D + d0], xj);
    const double g = exp(-0.5 * r2);
    const double v = w * fma(ai[il], ajl, -zij);
    const bool ok = jok && i < cx.n;
    const double kij = var * g + (i == j ? cx.noise : 0.0);
    const double kz = ok ? kij * zij : 0.0;
    s0 = ok ? fma(v, var * g * r2 * inv_ell, s0) : s0;
    s1 = ok ? fma(v, g, s1) : s1;
    sn = (ok && i == j) ? sn + v : sn;
    ca += kz;
    if (!diag) sZ[il * BS + jl] = kz;
  }
  cx.sums[0][0] += s0;
  cx.sums[0][1] += s1;
  cx.snoise += sn;
  colacc += ca;
}

template <int NT>
__device__ __forceinline__ void contract_block(ContractCtx<NT>& cx, double* __restrict__ sZ,
                                               const double* __restrict__ sxi, const double* __restrict__ sxj,
                                               int i0, int j0, const double* __restrict__ ai,
                                               const double* __restrict__ aj, bool diag, double& colacc) {
  if (cx.fast && cx.fkind == GPX_SE && cx.fdn == 1) {
    contract_block_se1<NT>(cx, sZ, sxi, sxj, i0, j0, ai, aj, diag, colacc);
    return;
  }
  const int lane = threadIdx.x & 63, part = threadIdx.x >> 6;
  const int jl = lane, j = j0 + jl, D = cx.D;
  const double ajl = aj[jl], w = diag ? 1.0 : 2.0;
  const double* xj = sxj + jl * D;
  const bool jok = j < cx.n;
#pragma unroll 2
  for (int t = 0; t < 16; ++t) {
    const int il = part * 16 + t, i = i0 + il;
    const double zij = sZ[il * BS + jl];
    double kz = 0.0;
    if (jok && i < cx.n) {
      const double v = w * fma(ai[il], ajl, -zij);
      const double* xi = sxi + il * D;
      double dk[NT][3];
      double kij;
      if (cx.fast) {
        stationary_grad(cx.fkind, sqdist_scaled(xi + cx.fd0, xj + cx.fd0, cx.fdn), cx.fvar, cx.finv_ell, dk[0]);
        kij = cx.fvar * dk[0][1];  // ∂K/∂σ² = K/σ² for a single stationary term
      } else {
        kij = eval_k_grad<NT>(*cx.spec, cx.sth, xi, xj, dk);
      }
      if (i == j) {
        kij += cx.noise;
        cx.snoise += v;
      }
      kz = kij * zij;
#pragma unroll
      for (int q = 0; q < NT; ++q) {
        cx.sums[q][0] = fma(v, dk[q][0], cx.sums[q][0]);
        cx.sums[q][1] = fma(v, dk[q][1], cx.sums[q][1]);
        cx.sums[q][2] = fma(v, dk[q][2], cx.sums[q][2]);
      }
    }
    colacc += kz;
    if (!diag) sZ[il * BS + jl] = kz;
  }
}

// Row sums of a K∘Z block left in LDS by contract_block: row r by threads 4r..4r+3 (16 columns
// each); returns the sum on the thread with (tid & 3) == 0, row tid >> 2
__device__ __forceinline__ double block_rowsum(const double* __restrict__ sKZ) {
  const int r = threadIdx.x >> 2, seg = threadIdx.x & 3;
  double s = 0.0;
#pragma unroll
  for (int c = 0; c < 16; ++c) s += sKZ[r * BS + seg * 16 + c];
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  return s;
}
}  // namespace

// The window's trailing-updated blocks stay in registers between steps (fragments D1 = A_kk,
// E1 = A_{k+1,k}, D2 = A_{k+1,k+1}); the original blocks entering the window at step k
// (A_{k+2,k}, A_{k+2,k+1}, A_{k+2,k+2}) are fetched before the leaf.
__global__ __launch_bounds__(256, 1) void band_fwd_kernel(BandFusedArgs a) {
  __shared__ __attribute__((aligned(16))) double sA[64 * BS];
  __shared__ __attribute__((aligned(16))) double sW[64 * BS];
  __shared__ __attribute__((aligned(16))) double sX[64 * BS];
  __shared__ __attribute__((aligned(16))) double sY[64 * BS];
  __shared__ double sv[3][64];        // y_k + u_k -> z_k, u_{k+1}, u_{k+2}
  __shared__ double spart[2][4][64];
  __shared__ int sfail;
  const int b = a.active[blockIdx.x];
  const int p = a.bandp[b], Np = a.Np, nb = Np / 64;
  const long long ld = a.ld;
  const double* K = a.K + (long long)b * a.sMat;
  double* L = a.L + (long long)b * a.sMat;
  double* W = a.W + (long long)b * a.sMat;
  double* z = a.z + (long long)b * a.sVec;
  double* ldiag = a.ldiag + (long long)b * a.sVec;
  const double* y = a.Y + (long long)b * a.sY;
  const int n = a.nvalid[b];
  const int tid = threadIdx.x, lane = tid & 63, part = tid >> 6;
  if (tid < 64) { sv[1][tid] = 0.0; sv[2][tid] = 0.0; }
  if (tid == 0) sfail = -1;
  int gfail = 0;
  Frag d1, e1, d2, f21, f22;
  double a20[16];
  frag_load_global(d1, K, ld);                                         // A_00
  if (nb > 1) {
    frag_load_global(d2, K + (long long)64 * ld + 64, ld);             // A_11
    if (p >= 1) frag_load_global(e1, K + (long long)64 * ld, ld);      // A_10
  }
  PH_BEGIN
  for (int k = 0; k < nb; ++k) {
    const int q = min(p, nb - 1 - k), k64 = k * 64;
    // originals entering the window at this step
    if (k + 2 < nb) {
      frag_load_global(f22, K + (long long)(k64 + 128) * ld + k64 + 128, ld);
      if (p >= 1) frag_load_global(f21, K + (long long)(k64 + 128) * ld + k64 + 64, ld);
      if (q >= 2) block_fetch(a20, K + (long long)(k64 + 128) * ld + k64, ld);
    }
    const double yk = (tid < 64 && k64 + tid < n) ? y[k64 + tid] : 0.0;
    frag_store_lds(d1, sA);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = tid + 256 * u;
      sW[(e >> 6) * BS + (e & 63)] = 0.0;
    }
    if (q >= 1) frag_store_lds(e1, sX);
    if (tid < 64) sv[0][tid] = yk + sv[1][tid];
    __syncthreads();
    PH(0);
    leaf64_lds<false>(sA, sW, ldiag + k64, &sfail);
    PH(1);
    if (tid == 0 && sfail >= 0) {
      if (gfail == 0) gfail = k64 + sfail + 1;
      sfail = -1;
    }
    {
      double* Wk = W + (long long)k64 * ld + k64;
      for (int e = tid; e < 4096; e += 256) Wk[(e >> 6) * ld + (e & 63)] = sW[(e >> 6) * BS + (e & 63)];
    }
    {  // z_k = W_kk (y_k + u_k)
      double s = 0.0;
      for (int c = part; c <= lane; c += 4) s = fma(sW[lane * BS + c], sv[0][c], s);
      spart[0][part][lane] = s;
    }
    if (q >= 2) block_store_lds(a20, sY);
    __syncthreads();
    if (tid < 64) {
      const double zk = (spart[0][0][tid] + spart[0][1][tid]) + (spart[0][2][tid] + spart[0][3][tid]);
      sv[0][tid] = zk;
      z[k64 + tid] = zk;
    }
    PH(2);
    // panels P_i = A_{k+i,k} W_kkᵀ -> L (global) and sX / sY
    Frag f1, f2;
    if (q >= 1) { frag_zero(f1); frag_mma<false, true, 16>(f1, sX, sW, false); }
    if (q >= 2) { frag_zero(f2); frag_mma<false, true, 16>(f2, sY, sW, false); }
    __syncthreads();
    if (q >= 1) {
      frag_store_lds(f1, sX);
      frag_store_global(f1, L + (long long)(k64 + 64) * ld + k64, ld);
    }
    if (q >= 2) {
      frag_store_lds(f2, sY);
      frag_store_global(f2, L + (long long)(k64 + 128) * ld + k64, ld);
    }
    __syncthreads();
    PH(3);
    // right-looking solve: u_{k+1} = u_{k+2} − P_1 z_k, u_{k+2} = −P_2 z_k
    if (q >= 1) {
      double s1 = 0.0, s2 = 0.0;
      for (int c = part; c < 64; c += 4) {
        s1 = fma(sX[lane * BS + c], sv[0][c], s1);
        if (q >= 2) s2 = fma(sY[lane * BS + c], sv[0][c], s2);
      }
      spart[0][part][lane] = s1;
      spart[1][part][lane] = s2;
    }
    // window update in registers: D2 −= P1 P1ᵀ, A_{k+2,k+1} −= P2 P1ᵀ, A_{k+2,k+2} −= P2 P2ᵀ
    if (q >= 1) frag_mma<false, true, 16>(d2, sX, sX, true);
    if (q >= 2) {
      frag_mma<false, true, 16>(f21, sY, sX, true);
      frag_mma<false, true, 16>(f22, sY, sY, true);
    }
    __syncthreads();
    if (tid < 64) {
      const double s1 = (spart[0][0][tid] + spart[0][1][tid]) + (spart[0][2][tid] + spart[0][3][tid]);
      const double s2 = (spart[1][0][tid] + spart[1][1][tid]) + (spart[1][2][tid] + spart[1][3][tid]);
      sv[1][tid] = q >= 1 ? sv[2][tid] - s1 : 0.0;
      sv[2][tid] = q >= 2 ? -s2 : 0.0;
    }
    // roll the window: (D1, E1, D2) <- (D2, A_{k+2,k+1}, A_{k+2,k+2})
    d1 = d2;
    e1 = f21;
    d2 = f22;
    __syncthreads();
    PH(4);
  }
  PH_END(2);
  if (tid == 0 && gfail > 0 && a.info[b] == 0) a.info[b] = gfail;
}

template <int NT>
__global__ __launch_bounds__(256, 1) void band_bwd_kernel(BandFusedArgs a) {
  __shared__ __attribute__((aligned(16))) double sA[64 * BS];
  __shared__ __attribute__((aligned(16))) double sW[64 * BS];
  __shared__ __attribute__((aligned(16))) double sX[64 * BS];
  __shared__ __attribute__((aligned(16))) double sY[64 * BS];
  __shared__ double sal[3][64];       // α_k, α_{k+1}, α_{k+2}
  __shared__ double st[64];
  __shared__ double spart[2][4][64];
  __shared__ double sth[GPX_THETA_STRIDE];
  __shared__ double sred[4][16];
  __shared__ double sres[3][64];      // Σ_i K_ji Z_ij for the columns of blocks k, k+1, k+2
  extern __shared__ double sxr[];     // [3][64·D] X rows, block k in slot k % 3
  const int b = a.active[blockIdx.x];
  const int p = a.bandp[b], Np = a.Np, nb = Np / 64;
  const long long ld = a.ld;
  double* K = a.K + (long long)b * a.sMat;
  const double* L = a.L + (long long)b * a.sMat;
  const double* W = a.W + (long long)b * a.sMat;
  const double* z = a.z + (long long)b * a.sVec;
  double* alpha = a.alpha + (long long)b * a.sVec;
  const double* X = a.X + (long long)b * a.sX;
  const int n = a.nvalid[b], D = a.D;
  const int tid = threadIdx.x, lane = tid & 63, part = tid >> 6;
  if (tid < 64) { sal[1][tid] = 0.0; sal[2][tid] = 0.0; sres[0][tid] = sres[1][tid] = sres[2][tid] = 0.0; }
  {  // the forward sweep left L_ii in ldiag: log det's terms (read by the reduce kernel)
    double* ldg = a.ldiag + (long long)b * a.sVec;
    for (int e = tid; e < Np; e += 256) ldg[e] = log(ldg[e]);
  }
  if (tid < GPX_THETA_STRIDE) sth[tid] = a.theta[b * GPX_THETA_STRIDE + tid];
  __syncthreads();
  const DevSpec spec = a.specs[b];
  const int nx = 64 * D;
  double resmax = 0.0;  // max |Σ_i K_ji Z_ij − 1| over the completed columns (this thread's share)
  ContractCtx<NT> cx;
  cx.spec = &spec; cx.sth = sth; cx.D = D; cx.n = n;
  cx.fkind = spec.terms[0].kind;
  cx.fast = (NT == 1) && spec.n_terms == 1 && cx.fkind >= GPX_SE && cx.fkind <= GPX_EXPONENTIAL;
  cx.fd0 = spec.terms[0].dim_start; cx.fdn = spec.terms[0].dim_count;
  cx.fvar = sth[spec.terms[0].param_offset + 1];
  cx.finv_ell = 1.0 / sth[spec.terms[0].param_offset];
  cx.xscale = cx.fast ? sth[spec.terms[0].param_offset] : 1.0;
  cx.noise = sth[spec.n_params];
#pragma unroll
  for (int t = 0; t < NT; ++t) cx.sums[t][0] = cx.sums[t][1] = cx.sums[t][2] = 0.0;
  cx.snoise = 0.0;
  // the first step's inputs (k = nb − 1 has no panels); the Z window (Z_{k+1,k+1},
  // Z_{k+2,k+1}, Z_{k+2,k+2}) rides in registers from step to step
  double pw[16], p1[16], p2[16];
  block_fetch(pw, W + (long long)(nb - 1) * 64 * ld + (nb - 1) * 64, ld);
  double zpre = z[(nb - 1) * 64 + lane];
  double xr = xrows_fetch(X, (nb - 1) * 64, n, D);
  Frag zA, zB, zC;
  frag_zero(zA);
  frag_zero(zB);
  frag_zero(zC);
  PH_BEGIN
  for (int k = nb - 1; k >= 0; --k) {
    const int q = min(p, nb - 1 - k), k64 = k * 64;
    const int s0 = k % 3, s1 = (k + 1) % 3, s2 = (k + 2) % 3;
    // α_k = W_kkᵀ (z_k − P_1ᵀ α_{k+1} − P_2ᵀ α_{k+2}): partials from the fetched registers
    {
      double s = 0.0;
      if (q >= 1) {
#pragma unroll
        for (int u = 0; u < 16; ++u) s = fma(p1[u], sal[1][part + 4 * u], s);
      }
      if (q >= 2) {
#pragma unroll
        for (int u = 0; u < 16; ++u) s = fma(p2[u], sal[2][part + 4 * u], s);
      }
      spart[0][part][lane] = s;
    }
    block_store_lds(pw, sW);
    if (q >= 1) block_store_lds(p1, sX);
    if (q >= 2) block_store_lds(p2, sY);
    xrows_store(xr, sxr + s0 * nx, X, k64, n, D, cx.xscale);
    __syncthreads();
    if (tid < 64) st[tid] = zpre - ((spart[0][0][tid] + spart[0][1][tid]) + (spart[0][2][tid] + spart[0][3][tid]));
    __syncthreads();
    {
      double s = 0.0;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int r = part + 4 * u;
        s = (r >= lane) ? fma(pw[u], st[r], s) : s;
      }
      spart[1][part][lane] = s;  // summed after the MFMAs' barrier below (no barrier of its own)
    }
    PH(0);
    // G_i = P_i W_kk;  Z_{k+i,k} = −Σ_j Z_{k+i,k+j} G_j  (Z_{k+1,k+2} = Z_{k+2,k+1}ᵀ);
    // Z_kk = W_kkᵀ W_kk − Σ_i G_iᵀ Z_{k+i,k}
    Frag g1, g2, z1, z2, zk;
    frag_zero(zk);
    frag_mma<true, false, 16>(zk, sW, sW, false);
    if (q >= 1) { frag_zero(g1); frag_mma<false, false, 16>(g1, sX, sW, false); }
    if (q >= 2) { frag_zero(g2); frag_mma<false, false, 16>(g2, sY, sW, false); }
    __syncthreads();
    if (tid < 64) {
      const double ak = (spart[1][0][tid] + spart[1][1][tid]) + (spart[1][2][tid] + spart[1][3][tid]);
      sal[0][tid] = ak;
      alpha[k64 + tid] = ak;
    }
    PH(1);
    frag_zero(z1);
    frag_zero(z2);
    if (q >= 1) {
      frag_store_lds(g1, sX);
      if (q >= 2) {
        frag_store_lds(g2, sY);
        frag_store_lds(zB, sA);
        frag_store_lds(zC, sW);
      }
      __syncthreads();
      if (q >= 2) {
        frag_mma<true, false, 16>(z1, sA, sY, true);
        frag_mma<false, false, 16>(z2, sA, sX, true);
        frag_mma<false, false, 16>(z2, sW, sY, true);
        __syncthreads();
      }
      frag_store_lds(zA, sA);
      __syncthreads();
      frag_mma<false, false, 16>(z1, sA, sX, true);
      __syncthreads();
      frag_store_lds(z1, sA);
      if (q >= 2) frag_store_lds(z2, sW);
      __syncthreads();
      frag_mma<true, false, 16>(zk, sX, sA, true);
      if (q >= 2) frag_mma<true, false, 16>(zk, sY, sW, true);
      __syncthreads();                   // every wave is done reading G_1 (sX)
      frag_store_lds(zk, sX);            // contraction: Z_kk in sX, Z_{k+1,k} in sA, Z_{k+2,k} in sW
    } else {
      frag_store_lds(zk, sX);
    }
    PH(2);
    frag_store_diag(zk, K + (long long)k64 * ld + k64, ld);
    // the next step's inputs, in flight during the contraction
    if (k > 0) {
      const int k1 = k64 - 64;
      block_fetch(pw, W + (long long)k1 * ld + k1, ld);
      block_fetch(p1, L + (long long)k64 * ld + k1, ld);
      if (k + 1 < nb) block_fetch(p2, L + (long long)(k64 + 64) * ld + k1, ld);
    }
    __syncthreads();
    PH(3);
    double colacc = 0.0;
    contract_block<NT>(cx, sX, sxr + s0 * nx, sxr + s0 * nx, k64, k64, sal[0], sal[0], true, colacc);
    if (q >= 1)
      contract_block<NT>(cx, sA, sxr + s1 * nx, sxr + s0 * nx, k64 + 64, k64, sal[1], sal[0], false, colacc);
    if (q >= 2)
      contract_block<NT>(cx, sW, sxr + s2 * nx, sxr + s0 * nx, k64 + 128, k64, sal[2], sal[0], false, colacc);
    PH(4);
    spart[0][part][lane] = colacc;
    if (k > 0) {
      zpre = z[k64 - 64 + lane];
      xr = xrows_fetch(X, k64 - 64, n, D);
    }
    __syncthreads();
    if (tid < 64) sres[0][tid] += (spart[0][0][tid] + spart[0][1][tid]) + (spart[0][2][tid] + spart[0][3][tid]);
    if (q >= 1) {
      const double rs = block_rowsum(sA);
      if ((tid & 3) == 0) sres[1][tid >> 2] += rs;
    }
    if (q >= 2) {
      const double rs = block_rowsum(sW);
      if ((tid & 3) == 0) sres[2][tid >> 2] += rs;
    }
    // roll the Z window: (Z_{k,k}, Z_{k+1,k}, Z_{k+1,k+1}) are the next step's (A, B, C)
    zC = zA;
    zB = z1;
    zA = zk;
    __syncthreads();
    // block k + p has all its band contributions now (later steps touch blocks < k + p only)
    if (tid < 64) {
      const int cb = k + p;
      if (cb < nb && cb * 64 + tid < n) resmax = fmax(resmax, fabs(sres[p][tid] - 1.0));
      sal[2][tid] = sal[1][tid];
      sal[1][tid] = sal[0][tid];
      sres[2][tid] = sres[1][tid];
      sres[1][tid] = sres[0][tid];
      sres[0][tid] = 0.0;
    }
    __syncthreads();
    PH(5);
  }
  PH_END(3);
  // blocks 0 .. p−1 complete at the end (rolled into slots 1 .. p)
  if (tid < 64)
    for (int cb = 0; cb < p && cb < nb; ++cb)
      if (cb * 64 + tid < n) resmax = fmax(resmax, fabs(sres[cb + 1][tid] - 1.0));
  // the band check: max over the workgroup (NaN propagates as a failure)
  {
    double rm = (resmax == resmax) ? resmax : INFINITY;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) rm = fmax(rm, __shfl_xor(rm, o, 64));
    if (lane == 0) sred[part][15] = rm;
    __syncthreads();
    if (tid == 0)
      a.results[(long long)b * kResStride + kResBandCheck] =
          fmax(fmax(sred[0][15], sred[1][15]), fmax(sred[2][15], sred[3][15]));
    __syncthreads();
  }
  // block reduction of the θ sums into the problem's single partial row
  double vals[GPX_MAX_TERMS * 3 + 1];
#pragma unroll
  for (int t = 0; t < GPX_MAX_TERMS; ++t)
#pragma unroll
    for (int q = 0; q < 3; ++q) vals[t * 3 + q] = t < NT ? wsum(cx.sums[t][q]) : 0.0;
  vals[GPX_MAX_TERMS * 3] = wsum(cx.snoise);
  if (lane == 0) {
#pragma unroll
    for (int v = 0; v < GPX_MAX_TERMS * 3 + 1; ++v) sred[part][v] = vals[v];
  }
  __syncthreads();
  if (tid < GPX_THETA_STRIDE) {
    double* out = a.partial + (long long)b * a.sPartial;
    double s = 0.0;
    int slot = -1;
    if (tid == spec.n_params) {
      slot = GPX_MAX_TERMS * 3;
    } else {
      const DevSpec* gs = a.specs + b;
      for (int t = 0; t < gs->n_terms; ++t) {
        const int o = gs->terms[t].param_offset, kind = gs->terms[t].kind;
        const int np = (kind == GPX_RQ || kind == GPX_PERIODIC_SE) ? 3 : (kind == GPX_LINEAR ? 1 : 2);
        if (tid >= o && tid < o + np) slot = t * 3 + (tid - o);
      }
    }
    if (slot >= 0) s = (sred[0][slot] + sred[1][slot]) + (sred[2][slot] + sred[3][slot]);
    out[tid] = s;
  }
}

void launch_band_fused(const BandFusedArgs& a, int max_terms, int n_active, hipStream_t s,
                       hipEvent_t* ev) {
  auto bwd = max_terms <= 1 ? band_bwd_kernel<1> : max_terms == 2 ? band_bwd_kernel<2>
                                                                   : band_bwd_kernel<GPX_MAX_TERMS>;
  const size_t xs = 3 * 64 * (size_t)a.D * sizeof(double);  // X-row slots of the backward sweep
  if (ev) {  // timestamped at the kernels' actual start and end (profiling)
    hipExtLaunchKernelGGL(band_fwd_kernel, dim3(n_active), dim3(256), 0, s, ev[0], ev[1], 0, a);
    hipExtLaunchKernelGGL(bwd, dim3(n_active), dim3(256), xs, s, ev[2], ev[3], 0, a);
    return;
  }
  hipLaunchKernelGGL(band_fwd_kernel, dim3(n_active), dim3(256), 0, s, a);
  hipLaunchKernelGGL(bwd, dim3(n_active), dim3(256), xs, s, a);
}

}  // namespace gpx

// =======================================================================================
// p <= 1 (91 % of the C2 evaluations): the same sweeps with two 64x64 LDS blocks (68 KiB), so
// two problems share a CU and interleave their latency chains (the leaf's serial diagonal, the
// barriers, the global round trips); the p = 2 kernels above hold four blocks (one per CU).
// =======================================================================================
namespace gpx {

// The trailing-updated diagonal block A_{k+1,k+1} stays in registers (each wave its lower 16x16
// tiles, sym_tile) and is the next leaf's input (no global round trip); the original blocks
// A_{k+1,k} and A_{k+1,k+1} are fetched during the leaf's inverse phase. The products skip what
// is exactly zero or redundant: the panel P = A_{k+1,k}W_kkᵀ only the k-blocks below W's
// diagonal (tile row per wave, 40 of 64 k-steps), the update A_{k+1,k+1} −= PPᵀ only its 10 lower
// tiles (at most 48 k-steps per wave). Sums are unchanged: the skipped terms are exact zeros
// (W's upper triangle) or the upper tiles the leaf never reads.
__global__ __launch_bounds__(256, 2) void band_fwd1_kernel(BandFusedArgs a) {
  __shared__ __attribute__((aligned(16))) double sA[64 * BS];   // A_kk -> (leaf) -> A_{k+1,k} -> P
  __shared__ __attribute__((aligned(16))) double sW[64 * BS];   // W_kk
  __shared__ double sv[2][64];        // y_k + u_k -> z_k, u_{k+1}
  __shared__ double spart[4][64];
  __shared__ int sfail;
  const int b = a.active[blockIdx.x];
  const int p = a.bandp[b], Np = a.Np, nb = Np / 64;
  const long long ld = a.ld;
  const double* K = a.K + (long long)b * a.sMat;
  double* L = a.L + (long long)b * a.sMat;
  double* W = a.W + (long long)b * a.sMat;
  double* z = a.z + (long long)b * a.sVec;
  double* ldiag = a.ldiag + (long long)b * a.sVec;
  const double* y = a.Y + (long long)b * a.sY;
  const int n = a.nvalid[b];
  const int tid = threadIdx.x, lane = tid & 63, part = tid >> 6;
  if (tid < 64) sv[1][tid] = 0.0;
  if (tid == 0) sfail = -1;
  int gfail = 0;
  bd4 cur[3], nxt[3];
  double pa[16];
  sym_load_global(cur, K, ld, part);  // A_00 (this wave's lower tiles)
  PH_BEGIN
  for (int k = 0; k < nb; ++k) {
    const int q = min(p, nb - 1 - k), k64 = k * 64;
    const double yk = (tid < 64 && k64 + tid < n) ? y[k64 + tid] : 0.0;
    sym_store_lds(cur, sA, part);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int e = tid + 256 * u;
      sW[(e >> 6) * BS + (e & 63)] = 0.0;
    }
    if (tid < 64) sv[0][tid] = yk + sv[1][tid];
    __syncthreads();
    PH(0);
    // this step's panel block and the next diagonal block, in flight during the leaf's inverse
    leaf64_lds<false>(sA, sW, ldiag + k64, &sfail, [&]() {
      if (q >= 1) block_fetch(pa, K + (long long)(k64 + 64) * ld + k64, ld);
      if (k + 1 < nb) sym_load_global(nxt, K + (long long)(k64 + 64) * ld + k64 + 64, ld, part);
    }, (int)(blockIdx.x & 3));
    PH(1);
    if (tid == 0 && sfail >= 0) {
      if (gfail == 0) gfail = k64 + sfail + 1;
      sfail = -1;
    }
    // W_kk -> global (the backward sweep reads it); z_k partials; the panel block -> sA
    {
      const int t = tid_fresh();
      double* Wk = W + (long long)k64 * ld + k64 + (t >> 6) * ld + (t & 63);
      const double* sWt = sW + (t >> 6) * BS + (t & 63);
#pragma unroll
      for (int u = 0; u < 16; ++u) Wk[4 * u * ld] = sWt[4 * u * BS];
    }
    {
      double s = 0.0;
      for (int c = part; c <= lane; c += 4) s = fma(sW[lane * BS + c], sv[0][c], s);
      spart[part][lane] = s;
    }
    if (q >= 1) block_store_lds(pa, sA);
    __syncthreads();
    if (tid < 64) {
      const double zk = (spart[0][tid] + spart[1][tid]) + (spart[2][tid] + spart[3][tid]);
      sv[0][tid] = zk;
      z[k64 + tid] = zk;
    }
    PH(2);
    if (q >= 1) {
      bd4 prow[4];
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) tile_zero(prow[jb]);
      row_mma<false, true, 1>(prow, sA, sW, part * 16, false);   // P = A_{k+1,k} W_kkᵀ (tile row)
      __syncthreads();
      PH(3);
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        tile_store_lds(prow[jb], sA, part * 16, jb * 16);
        tile_store_global(prow[jb], L + (long long)(k64 + 64) * ld + k64, ld, part * 16, jb * 16);
      }
      __syncthreads();
      PH(4);
      {  // u_{k+1} = −P z_k
        double s1 = 0.0;
        for (int c = part; c < 64; c += 4) s1 = fma(sA[lane * BS + c], sv[0][c], s1);
        spart[part][lane] = s1;
      }
      sym_mma<false, true, false>(nxt, sA, sA, part, true);    // A_{k+1,k+1} −= P Pᵀ (lower tiles)
      __syncthreads();
      if (tid < 64) sv[1][tid] = -((spart[0][tid] + spart[1][tid]) + (spart[2][tid] + spart[3][tid]));
      PH(5);
    } else if (tid < 64) {
      sv[1][tid] = 0.0;
    }
#pragma unroll
    for (int t = 0; t < 3; ++t) cur[t] = nxt[t];
    __syncthreads();
    PH(6);
  }
  PH_END(0);
  if (tid == 0 && gfail > 0 && a.info[b] == 0) a.info[b] = gfail;
}

// The backward sweep takes Z_{k+1,k+1} (the previous step's Z_kk) from LDS, fetches the next
// step's W_kk, P and X rows into registers during the contraction, and contracts from LDS with the X
// rows staged there (dynamic LDS: two 64·D slots, block k in slot k & 1).
template <int NT>
__global__ __launch_bounds__(256, 2) void band_bwd1_kernel(BandFusedArgs a) {
  __shared__ __attribute__((aligned(16))) double sA[64 * BS];   // P -> G -> Z_kk
  __shared__ __attribute__((aligned(16))) double sW[64 * BS];   // W_kk -> Z_{k+1,k+1} -> Z_{k+1,k} -> K∘Z
  extern __shared__ double sxr[];     // [2][64·D] X rows, block k in slot k & 1
  __shared__ double sal[2][64];       // α ring: α_k in slot k & 1
  __shared__ double st[64];
  __shared__ double spart[4][64];
  __shared__ double sth[GPX_THETA_STRIDE];
  __shared__ double sred[4][16];
  __shared__ double sres[2][64];      // Σ_i K_ji Z_ij ring: the columns of block k in slot k & 1
  const int b = a.active[blockIdx.x];
  const int p = a.bandp[b], Np = a.Np, nb = Np / 64;
  const long long ld = a.ld;
  double* K = a.K + (long long)b * a.sMat;
  const double* L = a.L + (long long)b * a.sMat;
  const double* W = a.W + (long long)b * a.sMat;
  const double* z = a.z + (long long)b * a.sVec;
  double* alpha = a.alpha + (long long)b * a.sVec;
  const double* X = a.X + (long long)b * a.sX;
  const int n = a.nvalid[b], D = a.D, nx = 64 * D;
  const int tid = threadIdx.x, lane = tid & 63, part = tid >> 6;
  if (tid < 64) { sal[0][tid] = sal[1][tid] = 0.0; sres[0][tid] = sres[1][tid] = 0.0; }
  {  // the forward sweep left L_ii in ldiag: log det's terms (read by the reduce kernel)
    double* ldg = a.ldiag + (long long)b * a.sVec;
    for (int e = tid; e < Np; e += 256) ldg[e] = log(ldg[e]);
  }
  if (tid < GPX_THETA_STRIDE) sth[tid] = a.theta[b * GPX_THETA_STRIDE + tid];
  // the first step's inputs (k = nb − 1 has no panel)
  double pw[16], pp[16];
  block_fetch(pw, W + (long long)(nb - 1) * 64 * ld + (nb - 1) * 64, ld);
  double zpre = z[(nb - 1) * 64 + lane];
  double xr = xrows_fetch(X, (nb - 1) * 64, n, D);
  __syncthreads();
  const DevSpec spec = a.specs[b];
  ContractCtx<NT> cx;
  cx.spec = &spec; cx.sth = sth; cx.D = D; cx.n = n;
  cx.fkind = spec.terms[0].kind;
  cx.fast = (NT == 1) && spec.n_terms == 1 && cx.fkind >= GPX_SE && cx.fkind <= GPX_EXPONENTIAL;
  cx.fd0 = spec.terms[0].dim_start; cx.fdn = spec.terms[0].dim_count;
  cx.fvar = sth[spec.terms[0].param_offset + 1];
  cx.finv_ell = 1.0 / sth[spec.terms[0].param_offset];
  cx.xscale = cx.fast ? sth[spec.terms[0].param_offset] : 1.0;
  cx.noise = sth[spec.n_params];
#pragma unroll
  for (int t = 0; t < NT; ++t) cx.sums[t][0] = cx.sums[t][1] = cx.sums[t][2] = 0.0;
  cx.snoise = 0.0;
  double resmax = 0.0;
  bd4 zrow[4];  // this wave's tile row of Z_{k+1,k+1}
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) tile_zero(zrow[jb]);
  PH_BEGIN
  for (int k = nb - 1; k >= 0; --k) {
    const int q = min(p, nb - 1 - k), k64 = k * 64, cs = k & 1, ns = cs ^ 1;
    // α_k = W_kkᵀ (z_k − Pᵀ α_{k+1}): partials straight from the fetched registers (thread
    // (part, lane) holds rows part + 4u of column lane)
    {
      double s = 0.0;
      if (q >= 1) {
#pragma unroll
        for (int u = 0; u < 16; ++u) s = fma(pp[u], sal[ns][part + 4 * u], s);
      }
      spart[part][lane] = s;
    }
    block_store_lds(pw, sW);
    if (q >= 1) block_store_lds(pp, sA);
    xrows_store(xr, sxr + cs * nx, X, k64, n, D, cx.xscale);
    __syncthreads();
    if (tid < 64) st[tid] = zpre - ((spart[0][tid] + spart[1][tid]) + (spart[2][tid] + spart[3][tid]));
    __syncthreads();
    {  // W_kkᵀ st partials; their sum (α_k) is taken after the next barrier, so the MFMAs
       // below issue without a barrier of their own for it
      double s = 0.0;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int r = part + 4 * u;
        s = (r >= lane) ? fma(pw[u], st[r], s) : s;
      }
      spart[part][lane] = s;
    }
    auto alpha_out = [&]() {  // after a barrier that follows the partials' stores
      if (tid < 64) {
        const double ak = (spart[0][tid] + spart[1][tid]) + (spart[2][tid] + spart[3][tid]);
        sal[cs][tid] = ak;
        alpha[k64 + tid] = ak;
      }
    };
    PH(0);
    // Z_kk = W_kkᵀW_kk − Gᵀ Z_{k+1,k}, Z_{k+1,k} = −Z_{k+1,k+1} G, G = P W_kk, by 16x16 tiles:
    // G and Z_{k+1,k} a tile row per wave (G only the k-blocks below W's diagonal), Z_kk (symmetric)
    // only its 10 lower tiles (WᵀW only the k-blocks below W's diagonal), mirrored into LDS
    bd4 zk[3];
    sym_zero(zk);
    sym_mma<true, false, true>(zk, sW, sW, part, false);         // WᵀW
    if (q >= 1) {
      bd4 g[4];
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) tile_zero(g[jb]);
      row_mma<false, false, 2>(g, sA, sW, part * 16, false);     // G = P W (tile row)
      __syncthreads();
      alpha_out();
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) {
        tile_store_lds(g[jb], sA, part * 16, jb * 16);
        tile_store_lds(zrow[jb], sW, part * 16, jb * 16);        // Z_{k+1,k+1}
      }
      __syncthreads();
      PH(1);
      bd4 z1[4];
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) tile_zero(z1[jb]);
      row_mma<false, false, 0>(z1, sW, sA, part * 16, true);     // Z_{k+1,k} = −Z_{k+1,k+1} G
      __syncthreads();
#pragma unroll
      for (int jb = 0; jb < 4; ++jb) tile_store_lds(z1[jb], sW, part * 16, jb * 16);
      __syncthreads();
      sym_mma<true, false, false>(zk, sA, sW, part, true);       // − Gᵀ Z_{k+1,k}
    }
    __syncthreads();                     // every wave is done reading G (sA)
    if (q == 0) alpha_out();
    PH(2);
    sym_store_lds_full(zk, sA, part);
    sym_store_diag(zk, K + (long long)k64 * ld + k64, ld, part);
    // the next step's inputs, in flight during the contraction
    if (k > 0) {
      const int k1 = k64 - 64;
      block_fetch(pw, W + (long long)k1 * ld + k1, ld);
      if (p >= 1) block_fetch(pp, L + (long long)k64 * ld + k1, ld);
    }
    __syncthreads();
    PH(3);
    double colacc = 0.0;
    contract_block<NT>(cx, sA, sxr + cs * nx, sxr + cs * nx, k64, k64, sal[cs], sal[cs], true, colacc);
    PH(4);
    if (q >= 1)
      contract_block<NT>(cx, sW, sxr + ns * nx, sxr + cs * nx, k64 + 64, k64, sal[ns], sal[cs], false, colacc);
    spart[part][lane] = colacc;
    if (k > 0) {  // (after the contraction: fewer registers live)
      zpre = z[k64 - 64 + lane];
      xr = xrows_fetch(X, k64 - 64, n, D);
    }
    __syncthreads();
    PH(5);
    if (tid < 64) sres[cs][tid] += (spart[0][tid] + spart[1][tid]) + (spart[2][tid] + spart[3][tid]);
    if (q >= 1) {
      const double rs = block_rowsum(sW);
      if ((tid & 3) == 0) sres[ns][tid >> 2] += rs;
    }
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) tile_load_lds(zrow[jb], sA, part * 16, jb * 16);  // the next Z_{k+1,k+1}
    __syncthreads();
    // block k + p has all its band contributions now; slot ns is block k − 1's next
    if (tid < 64) {
      const int cb = k + p;
      if (cb < nb && cb * 64 + tid < n) resmax = fmax(resmax, fabs(sres[cb & 1][tid] - 1.0));
      sres[ns][tid] = 0.0;
    }
    PH(6);
  }
  PH_END(1);
  if (tid < 64 && p >= 1 && tid < n) resmax = fmax(resmax, fabs(sres[0][tid] - 1.0));  // block 0
  {
    double rm = (resmax == resmax) ? resmax : INFINITY;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) rm = fmax(rm, __shfl_xor(rm, o, 64));
    if (lane == 0) sred[part][15] = rm;
    __syncthreads();
    if (tid == 0)
      a.results[(long long)b * kResStride + kResBandCheck] =
          fmax(fmax(sred[0][15], sred[1][15]), fmax(sred[2][15], sred[3][15]));
    __syncthreads();
  }
  double vals[GPX_MAX_TERMS * 3 + 1];
#pragma unroll
  for (int t = 0; t < GPX_MAX_TERMS; ++t)
#pragma unroll
    for (int q = 0; q < 3; ++q) vals[t * 3 + q] = t < NT ? wsum(cx.sums[t][q]) : 0.0;
  vals[GPX_MAX_TERMS * 3] = wsum(cx.snoise);
  if (lane == 0) {
#pragma unroll
    for (int v = 0; v < GPX_MAX_TERMS * 3 + 1; ++v) sred[part][v] = vals[v];
  }
  __syncthreads();
  if (tid < GPX_THETA_STRIDE) {
    double* out = a.partial + (long long)b * a.sPartial;
    double s = 0.0;
    int slot = -1;
    if (tid == spec.n_params) {
      slot = GPX_MAX_TERMS * 3;
    } else {
      const DevSpec* gs = a.specs + b;
      for (int t = 0; t < gs->n_terms; ++t) {
        const int o = gs->terms[t].param_offset, kind = gs->terms[t].kind;
        const int np = (kind == GPX_RQ || kind == GPX_PERIODIC_SE) ? 3 : (kind == GPX_LINEAR ? 1 : 2);
        if (tid >= o && tid < o + np) slot = t * 3 + (tid - o);
      }
    }
    if (slot >= 0) s = (sred[0][slot] + sred[1][slot]) + (sred[2][slot] + sred[3][slot]);
    out[tid] = s;
  }
}

void launch_band_fused1(const BandFusedArgs& a, int max_terms, int n_active, hipStream_t s, hipEvent_t* ev) {
  auto bwd = max_terms <= 1 ? band_bwd1_kernel<1> : max_terms == 2 ? band_bwd1_kernel<2>
                                                                    : band_bwd1_kernel<GPX_MAX_TERMS>;
  const size_t xs = 2 * 64 * (size_t)a.D * sizeof(double);  // X-row slots of the backward sweep
  if (ev) {
    hipExtLaunchKernelGGL(band_fwd1_kernel, dim3(n_active), dim3(256), 0, s, ev[0], ev[1], 0, a);
    hipExtLaunchKernelGGL(bwd, dim3(n_active), dim3(256), xs, s, ev[2], ev[3], 0, a);
    return;
  }
  hipLaunchKernelGGL(band_fwd1_kernel, dim3(n_active), dim3(256), 0, s, a);
  hipLaunchKernelGGL(bwd, dim3(n_active), dim3(256), xs, s, a);
}

}  // namespace gpx

namespace gpx {
// flush_rebinds' gather: one workgroup per rebound slot
// (one-wave workgroups: they fit any free wave slot beside the other processes' sweeps)
__global__ __launch_bounds__(64) void rebind_gather_kernel(const RebindDesc* desc, int Nmax, int D, double* box) {
  const RebindDesc d = desc[blockIdx.x];
  const int tid = threadIdx.x, n = d.n, nx = Nmax * D, nv = n * D;
  for (int e = tid; e < nx; e += 64) d.dx[e] = e < nv ? d.x[e] : 0.0;
  for (int e = tid; e < Nmax; e += 64) d.dy[e] = e < n ? d.y[e] : 0.0;
  if (d.box < 0) return;
  const int nb = (Nmax + 15) / 16;  // 16-row boxes (kBox)
  double* out = box + (size_t)d.box * nb * D * 2;
  for (int t = tid; t < nb * D; t += 64) {
    const int k = t / D, q = t - k * D;
    double lo = INFINITY, hi = -INFINITY;
    for (int r = k * 16; r < min(n, k * 16 + 16); ++r) {
      const double v = d.x[(size_t)r * D + q];
      lo = fmin(lo, v);
      hi = fmax(hi, v);
    }
    out[(size_t)t * 2] = lo;
    out[(size_t)t * 2 + 1] = hi;
  }
}

void launch_rebind_gather(const RebindDesc* desc, int m, int Nmax, int D, double* box, hipStream_t s) {
  hipLaunchKernelGGL(rebind_gather_kernel, dim3(m), dim3(64), 0, s, desc, Nmax, D, box);
}
}  // namespace gpx

#ifdef GPX_BAND_PHASES
// out[72] <- g_band_phase (kernel-major, 16 slots each: phases 0..11, [15] = workgroups) and
// g_leaf_phase (diag chain, panel, trailing, inverse, ..., [7] = leaves); reset != 0 zeroes
// both afterwards. Diagnostic build only (not in include/gpx.h).
extern "C" int gpx_debug_band_phases(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gpx::g_band_phase), sizeof(gpx::g_band_phase)) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out + 64, HIP_SYMBOL(gpx::g_leaf_phase), sizeof(gpx::g_leaf_phase)) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long zero[4][16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(gpx::g_band_phase), zero, sizeof(zero)) != hipSuccess) return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(gpx::g_leaf_phase), zero, 8 * sizeof(unsigned long long)) != hipSuccess) return -1;
  }
  return 0;
}
#endif
