// gpx_bcr.hip — the banded evaluation for calls with few problems: block cyclic reduction over
// the block-tridiagonal form of the band (gfx950, fp64).
//
// The band16 sweeps (gpx_band16.hip) walk a problem's 16-row blocks in order on ONE wavefront:
// N/16 dependent steps (256 at N = 4096, ≈ 1.3 ms forward + 1.4 ms backward per evaluation).
// That shape fills the chip when thousands of problems are in flight (the C2 bench) and leaves
// it empty for the reference's own calls, which carry 1-20 problems at a time: one GPR at a time
// inside the kernel loop (GPR/model_trainer.py:14-19), 2 tickers x 3 timeframes
// (GPR/main.py:23-37), 5 assets (Multi-Input_GPR/main.py:535-552), 20 tickers in BASELINE
// config 3. This path computes the same quantities with log-depth parallelism inside ONE problem:
//
//   * K + σn²I vanishes exactly beyond Q 16-blocks of the diagonal, so it is block
//     TRIDIAGONAL in blocks of bs = 16Q rows: tile (m, m − d) is zero for d > Q.
//   * Block cyclic reduction is the Cholesky factorisation of that matrix in odd-even order. At
//     level l the nodes are the original blocks j·2^l (j < m_l = ⌈n0 / 2^l⌉); the nodes at odd j
//     are eliminated all at once, one workgroup each: L_XX = chol(A_X), the panels
//     P_I = L(I,X), P_K = L(K,X) towards the two neighbours, whose Schur updates ΔA_I = P_I P_Iᵀ,
//     ΔA_K = P_K P_Kᵀ and new coupling E_KI = −P_K P_Iᵀ make the even nodes a block-tridiagonal
//     system of half the size. ⌈log2 n0⌉ + 1 levels (8 at N = 4096, Q = 3).
//   * z = L⁻¹(P y) rides along as one more right-hand side, log det = 2 Σ log L_ii; neither depends
//     on the elimination order, so −½‖z‖² − Σ log L_ii − n/2 log 2π is GPflow's logML.
//   * Selected inversion (Takahashi) runs the levels backwards: a node eliminated at level l needs
//     Z on its neighbours' blocks and on their coupling, all formed at coarser levels:
//       G_S = P_S W_X,  Z_{S,X} = −Z_{S,S'} G_{S'},  Z_XX = W_Xᵀ W_X − Σ_S G_Sᵀ Z_{S,X}  (S ∈ {I, K}),
//     and α_X = W_Xᵀ (z_X − P_Iᵀ α_I − P_Kᵀ α_K). Level 0 leaves Z_jj and Z_{j+1,j} for every
//     block: the band of K⁻¹ the gradient contraction ½ Σ (ααᵀ − Z) ∘ ∂K/∂θ reads.
//
// Outputs are those of the band16 sweeps, so the rest of the call (the reduce kernel, the band
// check, predict at the training inputs, the factor cache) is unchanged: z and log L_ii for the
// reduce kernel, α, diag(Z) on K's diagonal (band_train_pred_kernel), the problem's [16]
// gradient row, results[kResBandCheck] = max_j |Σ_i K_ji Z_ij − 1| (the same stability check:
// failing problems are re-evaluated densely), info (a failing pivot, 1-based row).
//
// Work is ~2.5x the sequential sweep's (every panel is a dense bs x bs block), but the chain is
// ⌈log2 n0⌉ levels of a bs-block elimination instead of N/16 16-row steps.
//
// Layout. Every bs x bs block lives row-major in a per-problem workspace (BcrLayout); inside a
// workgroup the blocks are row-major in LDS with a row stride ≡ 18 (mod 32) doubles, so both the
// C fragment of a tile and the C fragment of its transpose are read with at most a 2-way bank
// conflict (ds_read_b64 banks (a/4) mod 64 per 32-lane half). A workgroup has Q wavefronts and
// wave w owns tile column w of every right-hand side and of every product it forms, so no tile
// is computed twice and the results of a phase meet in LDS behind one barrier.
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>
#include <unordered_map>

#include "gpx_internal.h"
#include "gpx_b16core.h"
#include "gpx_host.h"

namespace gpx {

// Phase timing (diagnostic build only, -DGPX_BCR_PHASES: libgpx_phases.so, tools/bcr_phases.py):
// thread 0 of each workgroup adds the shader-clock cycles of its phases into
// g_bcr_phase[kernel][level][phase] ([..][..][15] counts workgroups); kernel 0 = forward levels,
// 1 = backward levels, 2 = contraction (level 0)
#ifdef GPX_BCR_PHASES
__device__ unsigned long long g_bcr_phase[3][16][16];
#define BP_BEGIN unsigned long long bp_t = __builtin_amdgcn_s_memtime(), bp_acc[8] = {};
#define BP(i)                                                          \
  do {                                                                 \
    const unsigned long long bp_n = __builtin_amdgcn_s_memtime();      \
    bp_acc[i] += bp_n - bp_t;                                          \
    bp_t = bp_n;                                                       \
  } while (0)
#define BP_END(kid, lev)                                                             \
  do {                                                                               \
    if (threadIdx.x == 0) {                                                          \
      for (int bp_i = 0; bp_i < 8; ++bp_i) atomicAdd(&g_bcr_phase[kid][lev][bp_i], bp_acc[bp_i]); \
      atomicAdd(&g_bcr_phase[kid][lev][15], 1ull);                                   \
    }                                                                                \
  } while (0)
#else
#define BP_BEGIN
#define BP(i) \
  do {        \
  } while (0)
#define BP_END(kid, lev) \
  do {                   \
  } while (0)
#endif

namespace {

template <int Q>
struct Bcr {
  static constexpr int bs = 16 * Q;
  static constexpr int rs = bs + (((18 - bs) % 32) + 32) % 32;  // LDS row stride ≡ 18 (mod 32)
  static constexpr int mat = bs * rs;
  static constexpr int BB = bs * bs;
};

// nodes at level l, and the level whose single node is the top of the reduction
__device__ __forceinline__ int lvl_m(int n0, int l) { return (n0 + (1 << l) - 1) >> l; }
__device__ __forceinline__ int lvl_top(int n0) {
  int l = 0;
  while (lvl_m(n0, l) > 1) ++l;
  return l;
}

// C fragment of tile (ti, tj) of a row-major matrix with leading dimension ld, and of its transpose
__device__ __forceinline__ t4 fr(const double* __restrict__ M, int ld, int ti, int tj, int l15, int l4) {
  const double* p = M + (16 * ti + l4) * ld + 16 * tj + l15;
  t4 t;
#pragma unroll
  for (int r = 0; r < 4; ++r) t[r] = p[4 * r * ld];
  return t;
}
__device__ __forceinline__ t4 frT(const double* __restrict__ M, int ld, int ti, int tj, int l15, int l4) {
  const double* p = M + (16 * ti + l15) * ld + 16 * tj + l4;
  t4 t;
#pragma unroll
  for (int r = 0; r < 4; ++r) t[r] = p[4 * r];
  return t;
}
// store a C fragment as tile (ti, tj), or its transpose as tile (tj, ti)
__device__ __forceinline__ void fst(double* __restrict__ M, int ld, int ti, int tj, const t4& c, int l15, int l4) {
  double* p = M + (16 * ti + l4) * ld + 16 * tj + l15;
#pragma unroll
  for (int r = 0; r < 4; ++r) p[4 * r * ld] = c[r];
}
__device__ __forceinline__ void fstT(double* __restrict__ M, int ld, int ti, int tj, const t4& c, int l15, int l4) {
  double* p = M + (16 * tj + l15) * ld + 16 * ti + l4;
#pragma unroll
  for (int r = 0; r < 4; ++r) p[4 * r] = c[r];
}

// K + σn²I of the problem at rows gi, gj (the identity in the padding rows)
__device__ __forceinline__ double kval(const DevSpec& spec, const double* __restrict__ th, double noise,
                                       const double* __restrict__ Xb, int D, int n, int gi, int gj) {
  if (gi >= n || gj >= n) return gi == gj ? 1.0 : 0.0;
  const double v = eval_k(spec, th, Xb + (long long)gi * D, Xb + (long long)gj * D);
  return gi == gj ? v + noise : v;
}

constexpr int kXs = 8;  // row stride of the staged x/ℓ rows (the band16 classes have D <= kBand16MaxD = 8)

// a single-term isotropic stationary kernel (SE / Matern / Exponential: the band path's kinds),
// evaluated from rows already scaled by 1/ℓ — the operations of eval_k (GPflow's Stationary.scale
// divides each input by ℓ; sqdist_scaled and stationary_value are eval_term's operations on the
// scaled values), so the same bits with one division per row instead of two per entry
struct KSt1 {
  bool on;
  int kind, d0, dn;
  double var, ell, inv_ell;
  __device__ __forceinline__ double val(double r2) const {
    switch (kind) {
      case GPX_SE: return stationary_value<GPX_SE>(r2, var);
      case GPX_MATERN12: return stationary_value<GPX_MATERN12>(r2, var);
      case GPX_MATERN32: return stationary_value<GPX_MATERN32>(r2, var);
      case GPX_MATERN52: return stationary_value<GPX_MATERN52>(r2, var);
      default: return stationary_value<GPX_EXPONENTIAL>(r2, var);
    }
  }
};
__device__ __forceinline__ KSt1 kst1(const DevSpec& s, const double* __restrict__ th) {
  KSt1 k;
  const gpx_term& t = s.terms[0];
  k.kind = t.kind;
  k.on = s.n_terms == 1 && t.kind >= GPX_SE && t.kind <= GPX_EXPONENTIAL && t.dim_count <= kXs;
  k.d0 = t.dim_start;
  k.dn = t.dim_count;
  k.ell = th[t.param_offset];
  k.var = th[t.param_offset + 1];
  k.inv_ell = 1.0 / k.ell;
  return k;
}
// x/ℓ of the rows of blocks b0, b1, b2 (b < 0: skipped) into slots 0, 1, 2 of sx ([3·bs][kXs])
__device__ __forceinline__ void stage_scaled(double* __restrict__ sx, const double* __restrict__ Xb, int D, int n,
                                             const KSt1& k1, int bs, int b0, int b1, int b2, int tid, int nt) {
  for (int e = tid; e < 3 * bs * k1.dn; e += nt) {
    const int slot = e / (bs * k1.dn), rem = e - slot * bs * k1.dn, r = rem / k1.dn, d = rem - r * k1.dn;
    const int blk = slot == 0 ? b0 : (slot == 1 ? b1 : b2);
    if (blk < 0) continue;
    const int g = blk * bs + r;
    sx[(slot * bs + r) * kXs + d] = g < n ? Xb[(long long)g * D + k1.d0 + d] / k1.ell : 0.0;
  }
}

}  // namespace

// ---------------------------------------------------------------------------------------
// The level-0 blocks from the inputs (grid: blocks J x 2 parts x problems, 256 threads):
// part 0 the lower tiles of A_J = K_JJ + σn²I (the identity in the padding) and y_J, part 1 the
// coupling C_J = K_{J,J−1}. Single-term stationary kernels from rows scaled once by 1/ℓ (KSt1).
// ---------------------------------------------------------------------------------------
template <int Q>
__global__ __launch_bounds__(256) void bcr_build_kernel(BcrArgs a) {
  constexpr int bs = Bcr<Q>::bs, BB = Bcr<Q>::BB;
  __shared__ double sx[2 * bs * kXs];  // x/ℓ of blocks J−1 (slot 0) and J (slot 1)
  const int p = blockIdx.z, b = a.active[p], part = blockIdx.y;
  const int n = a.nvalid[b], n0 = (n + bs - 1) / bs, J = blockIdx.x;
  if (J >= n0 || (part == 1 && J == 0)) return;
  const BcrLayout Lw(bs, a.nbm);
  double* ws = a.ws + (long long)p * a.sWs;
  const int tid = threadIdx.x;
  const DevSpec spec = a.specs[b];
  const double* th = a.theta + (long long)b * GPX_THETA_STRIDE;
  const double noise = th[spec.n_params];
  const double* Xb = a.X + (long long)b * a.sX;
  const int D = a.D;
  const KSt1 k1 = kst1(spec, th);
  if (k1.on) {
    for (int e = tid; e < 2 * bs * k1.dn; e += 256) {
      const int slot = e / (bs * k1.dn), rem = e - slot * bs * k1.dn, r = rem / k1.dn, d = rem - r * k1.dn;
      const int g = (J - 1 + slot) * bs + r;
      if (g >= 0) sx[(slot * bs + r) * kXs + d] = g < n ? Xb[(long long)g * D + k1.d0 + d] / k1.ell : 0.0;
    }
    __syncthreads();
  }
  double* out = ws + (part == 0 ? Lw.A : Lw.C) + (long long)J * BB;
  const int c0 = (part == 0 ? J : J - 1) * bs;
  for (int e = tid; e < BB; e += 256) {
    const int r = e / bs, c = e - r * bs;
    if (part == 0 && (r >> 4) < (c >> 4)) continue;
    const int gi = J * bs + r, gj = c0 + c;
    double v;
    if (gi >= n || gj >= n) {
      v = gi == gj ? 1.0 : 0.0;
    } else if (k1.on) {
      v = k1.val(sqdist_scaled(sx + (bs + r) * kXs, sx + ((part == 0 ? bs : 0) + c) * kXs, k1.dn));
      if (gi == gj) v += noise;
    } else {
      v = kval(spec, th, noise, Xb, D, n, gi, gj);
    }
    out[e] = v;
  }
  if (part == 0 && tid < bs) {
    const int g = J * bs + tid;
    ws[Lw.y + g] = g < n ? a.Y[(long long)b * a.sY + g] : 0.0;
  }
}

// ---------------------------------------------------------------------------------------
// Forward level l (grid: node positions j < m_l x problems). Odd j (and the top node): eliminate
// node X = j·2^l with neighbours I = X − 2^l, K = X + 2^l (if K < n0):
//   A_X (+ the level l−1 updates still pending on it) into LDS; right-hand sides
//   [E_XI | E_KXᵀ | I | y_X] into registers (wave w: tile column w of each, wave Q−1 the y column);
//   right-looking Cholesky of A_X over its Q tile columns, each step's W_tt = L_tt⁻¹ (leaf16m)
//   applied to the right-hand sides as it goes: afterwards they hold P_Iᵀ = L⁻¹E_XI, P_Kᵀ, W_X,
//   z_X; then ΔA_I = P_I P_Iᵀ, ΔA_K = P_K P_Kᵀ (lower tiles), E_KI = −P_K P_Iᵀ (-> C[K]) and the
//   y updates P_I z_X, P_K z_X.
// Even j: the node survives; at level l > 0 the updates of its two level l−1 neighbours are
// applied in place (the level-0 blocks come from bcr_build_kernel).
// ---------------------------------------------------------------------------------------
template <int Q>
__global__ __launch_bounds__(64 * Q) void bcr_fwd_kernel(BcrArgs a) {
  constexpr int bs = Bcr<Q>::bs, rs = Bcr<Q>::rs, BB = Bcr<Q>::BB, NT = 64 * Q, PER = BB / NT;
  __shared__ __attribute__((aligned(16))) double lds[2 * Bcr<Q>::mat + bs + 16 * kSC];
  double* sA = lds;                    // A_X -> L (W_tt on the diagonal) during the sweep, then P_Iᵀ
  double* sB = lds + Bcr<Q>::mat;      // P_Kᵀ
  double* sz = lds + 2 * Bcr<Q>::mat;  // y_X, then z_X
  double* sc = sz + bs;                // leaf16m's scratch
  const int p = blockIdx.y, b = a.active[p];
  const int n = a.nvalid[b], n0 = (n + bs - 1) / bs, l = a.level;
  const int m = lvl_m(n0, l), top = lvl_top(n0);
  const int j = blockIdx.x;
  if (l > top || j >= m) return;
  const bool is_top = l == top;
  const bool elim = is_top || (j & 1);
  if (l == 0 && !elim) return;  // (bcr_build_kernel wrote the level-0 blocks)
  BP_BEGIN
  const int X = j << l, h = l > 0 ? 1 << (l - 1) : 0;
  // updates pending on X from its level l−1 neighbours X − h (ΔR of that node) and X + h (ΔL)
  const bool pl = l > 0 && X > 0, pr = l > 0 && X + h < n0;
  const BcrLayout Lw(bs, a.nbm);
  double* ws = a.ws + (long long)p * a.sWs;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, l15 = lane & 15, l4 = lane >> 4;
  const int K = X + (1 << l);
  const bool hasI = elim && !is_top, hasK = elim && !is_top && K < n0;
  double* Ag = ws + Lw.A + (long long)X * BB;
  double* yg = ws + Lw.y + (long long)X * bs;
  const double* CX = ws + Lw.C + (long long)X * BB;
  const double* CK = ws + Lw.C + (long long)K * BB;
  // A_X − (ΔR of X − h + ΔL of X + h), y likewise, and the couplings E_XI, E_KX: every load
  // issued before the first use
  t4 R1[Q], R2[Q], R3[Q], RY[Q];
  {
    const double* dR = ws + Lw.DR + (long long)(X - h) * BB;
    const double* dL = ws + Lw.DL + (long long)(X + h) * BB;
    double va[PER], vr[PER], vl[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = tid + k * NT;
      va[k] = Ag[e];
      vr[k] = pl ? dR[e] : 0.0;
      vl[k] = pr ? dL[e] : 0.0;
    }
    double vy = 0.0;
    if (tid < bs) {
      const double yr = pl ? ws[Lw.dyR + (long long)(X - h) * bs + tid] : 0.0;
      const double yl = pr ? ws[Lw.dyL + (long long)(X + h) * bs + tid] : 0.0;
      vy = yg[tid] - (yr + yl);
    }
    // right-hand sides, tile column w of each: R1 = E_XI, R2 = E_KXᵀ, R3 = I, RY = y (wave Q−1)
    if (elim) {
#pragma unroll
      for (int t = 0; t < Q; ++t) {
        R1[t] = hasI ? fr(CX, bs, t, w, l15, l4) : tzero();
        R2[t] = hasK ? frT(CK, bs, w, t, l15, l4) : tzero();
      }
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = tid + k * NT, r = e / bs, c = e - r * bs;
      const double v = va[k] - (vr[k] + vl[k]);
      if (elim)
        sA[r * rs + c] = v;
      else
        Ag[e] = v;
    }
    if (tid < bs) {
      if (elim)
        sz[tid] = vy;
      else
        yg[tid] = vy;
    }
  }
  if (!elim) return;
  __syncthreads();
  BP(0);
#pragma unroll
  for (int t = 0; t < Q; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      R3[t][r] = (t == w && 4 * r + l4 == l15) ? 1.0 : 0.0;
      RY[t][r] = (w == Q - 1 && l15 == 0) ? sz[16 * t + 4 * r + l4] : 0.0;
    }
  }
  BP(1);
  // right-looking Cholesky of A_X over its tile columns, with the right-hand sides
#pragma unroll
  for (int t = 0; t < Q; ++t) {
    if (w == t) {  // the diagonal tile (read mirrored from its lower triangle)
      t4 Ad, V, Wr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = l15, cc = 4 * r + l4;
        Ad[r] = rr >= cc ? sA[(16 * t + rr) * rs + 16 * t + cc] : sA[(16 * t + cc) * rs + 16 * t + rr];
      }
      double lii;
      int fl;
      leaf16m(Ad, V, Wr, lii, fl, sc, l15, l4);
      fst(sA, rs, t, t, Wr, l15, l4);  // W_tt
      const int g = X * bs + 16 * t + l15;
      if (l4 == 0 && g < a.Np) a.ldiag[(long long)b * a.sVec + g] = log(lii);
      if (fl >= 0 && lane == 0) atomicCAS(a.info + b, 0, X * bs + 16 * t + fl + 1);
    }
    __syncthreads();
    const t4 WtT = frT(sA, rs, t, t, l15, l4);  // fragment of W_ttᵀ: the x operand of W_tt · Y
    if (w > t) {  // panel L(w, t) = A(w, t) W_ttᵀ
      t4 c = tzero();
      mma(c, frT(sA, rs, w, t, l15, l4), WtT);
      fst(sA, rs, w, t, c, l15, l4);
    }
    {  // the right-hand sides' block row t: X(t) = W_tt · R(t)
      t4 c1 = tzero(), c2 = tzero(), c3 = tzero(), cy = tzero();
      if (hasI) mma(c1, WtT, R1[t]);
      if (hasK) mma(c2, WtT, R2[t]);
      if (t >= w) mma(c3, WtT, R3[t]);
      if (w == Q - 1) mma(cy, WtT, RY[t]);
      R1[t] = c1;
      R2[t] = c2;
      R3[t] = c3;
      RY[t] = cy;
    }
    __syncthreads();
    // trailing update A(s, r) −= L(s, t) L(r, t)ᵀ, t < r <= s (tiles dealt to the waves in turn)
    {
      int idx = 0;
#pragma unroll
      for (int s = t + 1; s < Q; ++s)
#pragma unroll
        for (int r = t + 1; r <= s; ++r, ++idx)
          if (idx % Q == w) {
            t4 c = fr(sA, rs, s, r, l15, l4);
            mms(c, frT(sA, rs, s, t, l15, l4), frT(sA, rs, r, t, l15, l4));
            fst(sA, rs, s, r, c, l15, l4);
          }
    }
    // the right-hand sides' rows below: R(s) −= L(s, t) X(t)
#pragma unroll
    for (int s = t + 1; s < Q; ++s) {
      const t4 Ls = frT(sA, rs, s, t, l15, l4);
      if (hasI) mms(R1[s], Ls, R1[t]);
      if (hasK) mms(R2[s], Ls, R2[t]);
      if (t >= w) mms(R3[s], Ls, R3[t]);
      if (w == Q - 1) mms(RY[s], Ls, RY[t]);
    }
    __syncthreads();
  }
  BP(2);
  // the factor for the backward levels: W_X (lower tiles), P_Iᵀ, P_Kᵀ, z_X
  double* Wg = ws + Lw.Wm + (long long)X * BB;
  double* PIg = ws + Lw.PI + (long long)X * BB;
  double* PKg = ws + Lw.PK + (long long)X * BB;
#pragma unroll
  for (int t = 0; t < Q; ++t) {
    if (t >= w) fst(Wg, bs, t, w, R3[t], l15, l4);
    if (hasI) {
      fst(PIg, bs, t, w, R1[t], l15, l4);
      fst(sA, rs, t, w, R1[t], l15, l4);
    }
    if (hasK) {
      fst(PKg, bs, t, w, R2[t], l15, l4);
      fst(sB, rs, t, w, R2[t], l15, l4);
    }
  }
  if (w == Q - 1 && l15 == 0) {
#pragma unroll
    for (int t = 0; t < Q; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * t + 4 * r + l4, g = X * bs + i;
        sz[i] = RY[t][r];
        ws[Lw.z + g] = RY[t][r];
        if (g < a.Np) a.z[(long long)b * a.sVec + g] = RY[t][r];
      }
  }
  __syncthreads();
  BP(3);
  // the neighbours' updates (column w of each; the Δ's lower tiles only)
  if (hasI) {
    double* dLo = ws + Lw.DL + (long long)X * BB;
#pragma unroll
    for (int i = 0; i < Q; ++i) {
      if (i < w) continue;
      t4 c = tzero();
#pragma unroll
      for (int k = 0; k < Q; ++k) mma(c, fr(sA, rs, k, i, l15, l4), R1[k]);
      fst(dLo, bs, i, w, c, l15, l4);
    }
    // y_I −= P_I z_X: row 16w + l15 of P_I z = column of P_Iᵀ dotted with z
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < Q; ++k)
#pragma unroll
      for (int r = 0; r < 4; ++r) s = fma(R1[k][r], sz[16 * k + 4 * r + l4], s);
    s = sum4(s);
    if (l4 == 0) ws[Lw.dyL + (long long)X * bs + 16 * w + l15] = s;
  }
  if (hasK) {
    double* dRo = ws + Lw.DR + (long long)X * BB;
    double* CKo = ws + Lw.C + (long long)K * BB;  // becomes E_KI (K's left neighbour is I now)
#pragma unroll
    for (int i = 0; i < Q; ++i) {
      t4 e = tzero();
#pragma unroll
      for (int k = 0; k < Q; ++k) mms(e, fr(sB, rs, k, i, l15, l4), R1[k]);
      fst(CKo, bs, i, w, e, l15, l4);
      if (i < w) continue;
      t4 c = tzero();
#pragma unroll
      for (int k = 0; k < Q; ++k) mma(c, fr(sB, rs, k, i, l15, l4), R2[k]);
      fst(dRo, bs, i, w, c, l15, l4);
    }
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < Q; ++k)
#pragma unroll
      for (int r = 0; r < 4; ++r) s = fma(R2[k][r], sz[16 * k + 4 * r + l4], s);
    s = sum4(s);
    if (l4 == 0) ws[Lw.dyR + (long long)X * bs + 16 * w + l15] = s;
  }
  BP(4);
  BP_END(0, l);
}

// ---------------------------------------------------------------------------------------
// Backward level l (grid: eliminated positions j = 2x + 1, or the top node, x problems): for node
// X eliminated at level l with neighbours I, K (Z_II, Z_KK and their coupling Z_KI formed at the
// coarser levels):
//   α_X = W_Xᵀ (z_X − P_Iᵀ α_I − P_Kᵀ α_K)
//   G_I = P_I W_X, G_K = P_K W_X                   (wave w: column w)
//   Z_IX = −(Z_II G_I + Z_KIᵀ G_K),  Z_KX = −(Z_KI G_I + Z_KK G_K)
//   Z_XX = W_Xᵀ W_X − G_Iᵀ Z_IX − G_Kᵀ Z_KX         (wave w: row w)
// Z_XX overwrites A[X] (ZD), Z_{X,I} = Z_IXᵀ goes to C[X] and Z_{K,X} to C[K] (ZC[Y] = the coupling
// of node Y with its left neighbour at the finest level formed so far).
// ---------------------------------------------------------------------------------------
template <int Q>
__global__ __launch_bounds__(64 * Q) void bcr_bwd_kernel(BcrArgs a) {
  constexpr int bs = Bcr<Q>::bs, rs = Bcr<Q>::rs, BB = Bcr<Q>::BB, NT = 64 * Q, PER = BB / NT;
  __shared__ __attribute__((aligned(16))) double lds[3 * Bcr<Q>::mat + 4 * bs];
  double* s0 = lds;                    // W_X, then Z_II, then Z_IX
  double* s1 = lds + Bcr<Q>::mat;      // P_Iᵀ, then Z_KK, then Z_KX
  double* s2 = lds + 2 * Bcr<Q>::mat;  // P_Kᵀ, then Z_KI
  double* sz = lds + 3 * Bcr<Q>::mat;
  double* saI = sz + bs;
  double* saK = saI + bs;
  double* st = saK + bs;
  const int p = blockIdx.y, b = a.active[p];
  const int n = a.nvalid[b], n0 = (n + bs - 1) / bs, l = a.level;
  const int m = lvl_m(n0, l), top = lvl_top(n0);
  if (l > top) return;
  const bool is_top = l == top;
  int X = 0;
  if (is_top) {
    if (blockIdx.x != 0) return;
  } else {
    const int j = 2 * blockIdx.x + 1;
    if (j >= m) return;
    X = j << l;
  }
  const int I = X - (1 << l), K = X + (1 << l);
  const bool hasI = !is_top, hasK = !is_top && K < n0;
  BP_BEGIN
  const BcrLayout Lw(bs, a.nbm);
  double* ws = a.ws + (long long)p * a.sWs;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, l15 = lane & 15, l4 = lane >> 4;
  const double* Wg = ws + Lw.Wm + (long long)X * BB;
  const double* PIg = ws + Lw.PI + (long long)X * BB;
  const double* PKg = ws + Lw.PK + (long long)X * BB;
  double* al = ws + Lw.al;
  {  // W_X, P_Iᵀ, P_Kᵀ, z_X, α_I, α_K: every load issued before the first store
    double vw[PER], vi[PER], vk[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = tid + k * NT;
      vw[k] = Wg[e];
      vi[k] = hasI ? PIg[e] : 0.0;
      vk[k] = hasK ? PKg[e] : 0.0;
    }
    double v0 = 0.0, v1 = 0.0, v2 = 0.0;
    if (tid < bs) {
      v0 = ws[Lw.z + (long long)X * bs + tid];
      v1 = hasI ? al[(long long)I * bs + tid] : 0.0;
      v2 = hasK ? al[(long long)K * bs + tid] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = tid + k * NT, r = e / bs, c = e - r * bs;
      s0[r * rs + c] = (r >> 4) >= (c >> 4) ? vw[k] : 0.0;
      s1[r * rs + c] = vi[k];
      s2[r * rs + c] = vk[k];
    }
    if (tid < bs) {
      sz[tid] = v0;
      saI[tid] = v1;
      saK[tid] = v2;
    }
  }
  __syncthreads();
  BP(0);
  // α_X = W_Xᵀ (z_X − P_Iᵀ α_I − P_Kᵀ α_K): four threads per row (NT = 4·bs), each a quarter of
  // the dot products, summed over the four lanes in a fixed order
  {
    const int i = tid >> 2, q = tid & 3;
    double t = 0.0;
    if (hasI)
      for (int c = q; c < bs; c += 4) t = fma(s1[i * rs + c], saI[c], t);
    if (hasK)
      for (int c = q; c < bs; c += 4) t = fma(s2[i * rs + c], saK[c], t);
    t += __shfl_xor(t, 1, 64);
    t += __shfl_xor(t, 2, 64);
    if (q == 0) st[i] = sz[i] - t;
  }
  __syncthreads();
  {
    const int i = tid >> 2, q = tid & 3;
    double v = 0.0;
    for (int r = i + q; r < bs; r += 4) v = fma(s0[r * rs + i], st[r], v);
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    if (q == 0) al[(long long)X * bs + i] = v;
  }
  BP(1);
  // G_I, G_K (column w) and row w of W_Xᵀ W_X
  t4 GI[Q], GK[Q], Zr[Q];
#pragma unroll
  for (int k = 0; k < Q; ++k) {
    GI[k] = tzero();
    GK[k] = tzero();
    Zr[k] = tzero();
#pragma unroll
    for (int mm = 0; mm < Q; ++mm) {
      if (mm < w) continue;
      const t4 Wm = fr(s0, rs, mm, w, l15, l4);
      if (hasI) mma(GI[k], fr(s1, rs, mm, k, l15, l4), Wm);
      if (hasK) mma(GK[k], fr(s2, rs, mm, k, l15, l4), Wm);
      if (mm >= k) mma(Zr[k], Wm, fr(s0, rs, mm, k, l15, l4));
    }
  }
  BP(2);
  double* ZC = ws + Lw.C;
  __syncthreads();
  if (!is_top) {
    const double* ZI = ws + Lw.A + (long long)I * BB;
    const double* ZK = ws + Lw.A + (long long)K * BB;
    const double* ZKI = ZC + (long long)K * BB;
    double v0[PER], v1[PER], v2[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = tid + k * NT;
      v0[k] = ZI[e];
      v1[k] = hasK ? ZK[e] : 0.0;
      v2[k] = hasK ? ZKI[e] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int e = tid + k * NT, r = e / bs, c = e - r * bs;
      s0[r * rs + c] = v0[k];
      s1[r * rs + c] = v1[k];
      s2[r * rs + c] = v2[k];
    }
    __syncthreads();
    BP(3);
    t4 ZIX[Q], ZKX[Q];
#pragma unroll
    for (int i = 0; i < Q; ++i) {
      ZIX[i] = tzero();
      ZKX[i] = tzero();
#pragma unroll
      for (int k = 0; k < Q; ++k) {
        mms(ZIX[i], frT(s0, rs, i, k, l15, l4), GI[k]);
        if (hasK) {
          mms(ZIX[i], fr(s2, rs, k, i, l15, l4), GK[k]);
          mms(ZKX[i], frT(s2, rs, i, k, l15, l4), GI[k]);
          mms(ZKX[i], frT(s1, rs, i, k, l15, l4), GK[k]);
        }
      }
    }
    __syncthreads();
    BP(4);
    double* ZCX = ZC + (long long)X * BB;
    double* ZCK = ZC + (long long)K * BB;
#pragma unroll
    for (int i = 0; i < Q; ++i) {
      fst(s0, rs, i, w, ZIX[i], l15, l4);
      fstT(ZCX, bs, i, w, ZIX[i], l15, l4);
      if (hasK) {
        fst(s1, rs, i, w, ZKX[i], l15, l4);
        fst(ZCK, bs, i, w, ZKX[i], l15, l4);
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < Q; ++i)
#pragma unroll
      for (int k = 0; k < Q; ++k) {
        mms(Zr[i], GI[k], fr(s0, rs, k, i, l15, l4));
        if (hasK) mms(Zr[i], GK[k], fr(s1, rs, k, i, l15, l4));
      }
  }
  double* ZX = ws + Lw.A + (long long)X * BB;
#pragma unroll
  for (int i = 0; i < Q; ++i) fst(ZX, bs, w, i, Zr[i], l15, l4);
  BP(6);
  BP_END(1, l);
}

// ---------------------------------------------------------------------------------------
// Gradient contraction and band check over block J (grid: blocks x problems, 256 threads):
// thread (g, u) owns row/column u of block J and takes every G-th entry of its other index:
//   (J, J)     Z_JJ[v][u]        weight 1 (the whole block), the noise term on the diagonal
//   (J+1, J)   Z_{J+1,J}[v][u]   weight 2
//   (J, J−1)   Z_{J,J−1}[u][v]   band check only (its gradient share is block J−1's)
// r_u = Σ K∘Z over the three blocks is row J·bs + u of K·Z (the band check); the block's [16]
// gradient row and its check maximum go to the workspace for bcr_finish_kernel; diag(Z_JJ) onto
// K's diagonal and α into the batch's α vector.
// ---------------------------------------------------------------------------------------
// GZ (the bs = 128 reduction of the wide classes): Z_JJ, Z_{J+1,J} and Z_{J,J−1} are read from the
// workspace where they lie instead of being staged in LDS (2 x 128 KB) and registers
template <int Q, int NTm, bool GZ = false>
__global__ __launch_bounds__(256) void bcr_contract_kernel(BcrArgs a) {
  constexpr int bs = Bcr<Q>::bs, BB = Bcr<Q>::BB, G = 256 / bs;
  constexpr int NV = GPX_MAX_TERMS * 3 + 1;
  __shared__ double scs[G][bs];
  __shared__ double sred[4][NV];
  __shared__ double smax[4];
  __shared__ double sx[3 * bs * kXs];  // single-term stationary kernels: x/ℓ of blocks J−1, J, J+1
  __shared__ double sZs[GZ ? 1 : 2 * BB];  // Z_JJ, Z_{J+1,J}
  __shared__ double sal[2 * bs];       // α of blocks J, J+1
  constexpr int VM = (bs + G - 1) / G;  // entries per thread of each block's column (and of Z_{J,J−1}'s check part)
  constexpr int VMC = GZ ? 1 : VM;      // (GZ: Z_{J,J−1} read in place, not held in registers)
  const int p = blockIdx.y, b = a.active[p];
  const int n = a.nvalid[b], n0 = (n + bs - 1) / bs, J = blockIdx.x;
  if (J >= n0) return;
  BP_BEGIN
  const BcrLayout Lw(bs, a.nbm);
  const double* ws = a.ws + (long long)p * a.sWs;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int u = tid % bs, g = tid / bs;
  const DevSpec spec = a.specs[b];
  const double* th = a.theta + (long long)b * GPX_THETA_STRIDE;
  const double noise = th[spec.n_params];
  const double* Xb = a.X + (long long)b * a.sX;
  const int D = a.D;
  const KSt1 k1 = kst1(spec, th);
  const double* al = ws + Lw.al;
  const double* ZD = ws + Lw.A + (long long)J * BB;
  const double* ZCJ = ws + Lw.C + (long long)J * BB;         // Z_{J,J−1} (J >= 1)
  const double* ZCJ1 = ws + Lw.C + (long long)(J + 1) * BB;  // Z_{J+1,J} (J + 1 < n0)
  // the block's Z tiles and α rows into LDS, its share of Z_{J,J−1} into registers: every load
  // issued before the first use
  double zc[VMC];
  const double* sZD = GZ ? ZD : sZs;
  const double* sZ1 = GZ ? ZCJ1 : sZs + BB;
  if constexpr (GZ) {
    const double a0 = tid < 2 * bs ? al[(long long)J * bs + tid] : 0.0;  // (block J+1 past n0: zeros)
    if (k1.on) stage_scaled(sx, Xb, D, n, k1, bs, J - 1, J, J + 1 < n0 ? J + 1 : -1, tid, 256);
    if (tid < 2 * bs) sal[tid] = a0;
  } else {
    constexpr int PERC = BB / 256;
    double v0[PERC], v1[PERC];
#pragma unroll
    for (int k = 0; k < PERC; ++k) {
      v0[k] = ZD[tid + k * 256];
      v1[k] = J + 1 < n0 ? ZCJ1[tid + k * 256] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < VM; ++k) {
      const int v = g + k * G;
      zc[k] = (k1.on && J >= 1 && g < G && v < bs) ? ZCJ[u * bs + v] : 0.0;
    }
    const double a0 = tid < 2 * bs ? al[(long long)J * bs + tid] : 0.0;  // (block J+1 past n0: zeros)
    if (k1.on) stage_scaled(sx, Xb, D, n, k1, bs, J - 1, J, J + 1 < n0 ? J + 1 : -1, tid, 256);
    double* sw = sZs;
#pragma unroll
    for (int k = 0; k < PERC; ++k) {
      sw[tid + k * 256] = v0[k];
      sw[BB + tid + k * 256] = v1[k];
    }
    if (tid < 2 * bs) sal[tid] = a0;
  }
  __syncthreads();
  BP(0);
  double sums[NTm][3];
#pragma unroll
  for (int t = 0; t < NTm; ++t) sums[t][0] = sums[t][1] = sums[t][2] = 0.0;
  double snoise = 0.0, cs = 0.0;
  const int ju = J * bs + u;
  // K_ij and its θ-derivatives (dk[t][q], eval_k_grad's layout); the fast form for single-term
  // stationary kernels (stationary_grad on the staged rows, as the band16 sweeps' generic path)
  auto kgrad = [&](int si, int gi, int sj, int gj, double (&dk)[NTm][3]) {
    if (k1.on) {
      double d1[3];
      stationary_grad(k1.kind, sqdist_scaled(sx + (si * bs + gi % bs) * kXs, sx + (sj * bs + gj % bs) * kXs, k1.dn),
                      k1.var, k1.inv_ell, d1);
#pragma unroll
      for (int t = 0; t < NTm; ++t) dk[t][0] = dk[t][1] = dk[t][2] = 0.0;
      dk[0][0] = d1[0];
      dk[0][1] = d1[1];
      return k1.var * d1[1];
    }
    return eval_k_grad<NTm>(spec, th, Xb + (long long)gi * D, Xb + (long long)gj * D, dk);
  };
  if (g < G && ju < n) {
    const double aj = sal[u];
    for (int k = 0; k < VM; ++k) {
      const int v = g + k * G;
      if (v >= bs) continue;
      double dk[NTm][3];
      {  // (J, J)
        const int i = J * bs + v;
        if (i < n) {
          const double z = sZD[v * bs + u];
          double kv = kgrad(1, i, 1, ju, dk);
          const double vv = fma(sal[v], aj, -z);
#pragma unroll
          for (int t = 0; t < NTm; ++t)
#pragma unroll
            for (int q = 0; q < 3; ++q) sums[t][q] = fma(vv, dk[t][q], sums[t][q]);
          if (i == ju) {
            kv += noise;
            snoise += vv;
          }
          cs = fma(kv, z, cs);
        }
      }
      if (J + 1 < n0) {  // (J+1, J)
        const int i = (J + 1) * bs + v;
        if (i < n) {
          const double z = sZ1[v * bs + u];  // (GZ: read only when block J+1 exists)
          const double kv = kgrad(2, i, 1, ju, dk);
          const double vv = 2.0 * fma(sal[bs + v], aj, -z);
#pragma unroll
          for (int t = 0; t < NTm; ++t)
#pragma unroll
            for (int q = 0; q < 3; ++q) sums[t][q] = fma(vv, dk[t][q], sums[t][q]);
          cs = fma(kv, z, cs);
        }
      }
    }
    // (J, J−1): the check only (its gradient share is block J−1's)
    if (J >= 1) {
      if (k1.on && GZ) {
        for (int v = g; v < bs; v += G) cs = fma(k1.val(sqdist_scaled(sx + (bs + u) * kXs, sx + v * kXs, k1.dn)), ZCJ[u * bs + v], cs);
      } else if (!GZ && k1.on) {
#pragma unroll
        for (int k = 0; k < VMC; ++k) {
          const int v = g + k * G;
          if (v < bs) cs = fma(k1.val(sqdist_scaled(sx + (bs + u) * kXs, sx + v * kXs, k1.dn)), zc[k], cs);
        }
      } else {
        for (int v = g; v < bs; v += G)
          cs = fma(eval_k(spec, th, Xb + (long long)ju * D, Xb + (long long)((J - 1) * bs + v) * D), ZCJ[u * bs + v],
                   cs);
      }
    }
  }
  if (g < G) scs[g][u] = cs;
  // the block's gradient sums, fixed order: wave sums, then the four waves in turn
  double vals[NV];
#pragma unroll
  for (int t = 0; t < GPX_MAX_TERMS; ++t)
#pragma unroll
    for (int q = 0; q < 3; ++q) vals[t * 3 + q] = t < NTm ? wsum64(sums[t][q]) : 0.0;
  vals[NV - 1] = wsum64(snoise);
  if (lane == 0) {
#pragma unroll
    for (int v = 0; v < NV; ++v) sred[wave][v] = vals[v];
  }
  __syncthreads();
  BP(1);
  double* part = const_cast<double*>(ws) + Lw.part + (long long)J * GPX_THETA_STRIDE;
  if (tid < GPX_THETA_STRIDE) {
    int slot = -1;
    if (tid == spec.n_params) {
      slot = NV - 1;
    } else {
      for (int t = 0; t < spec.n_terms; ++t) {
        const int o = a.specs[b].terms[t].param_offset, kind = a.specs[b].terms[t].kind;
        const int np = (kind == GPX_RQ || kind == GPX_PERIODIC_SE) ? 3 : (kind == GPX_LINEAR ? 1 : 2);
        if (tid >= o && tid < o + np) slot = t * 3 + (tid - o);
      }
    }
    double sv = 0.0;
    if (slot >= 0) sv = ((sred[0][slot] + sred[1][slot]) + sred[2][slot]) + sred[3][slot];
    part[tid] = sv;
  }
  // the band check over the block's rows; diag(Z) and α out
  double res = 0.0;
  if (tid < bs) {
    double tot = 0.0;
#pragma unroll
    for (int gg = 0; gg < G; ++gg) tot += scs[gg][tid];
    const int row = J * bs + tid;
    if (row < n) {
      res = (tot == tot) ? fabs(tot - 1.0) : INFINITY;
      a.Kd[(long long)b * a.sMat + (long long)row * a.ld + row] = sZD[tid * bs + tid];
    }
    if (row < a.Np) a.alpha[(long long)b * a.sVec + row] = row < n ? sal[tid] : 0.0;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) res = fmax(res, __shfl_xor(res, o, 64));
  if (lane == 0) smax[wave] = res;
  __syncthreads();
  if (tid == 0) const_cast<double*>(ws)[Lw.chk + J] = fmax(fmax(smax[0], smax[1]), fmax(smax[2], smax[3]));
  BP(2);
  BP_END(2, 0);
}

// ---------------------------------------------------------------------------------------
// The wide classes (band16 widths Q = 6..8) as ONE reduction of block size
// bs = 128 (kBcrWideQ = 8: a band of at most 8 16-blocks is block tridiagonal in 128-row blocks,
// whatever its own width). The Q <= 5 kernels above keep every block of a node in LDS and every
// right-hand side in registers; at bs = 128 one block is 128 x 146 doubles (150 KB of the 160 KB
// LDS) and the four right-hand sides 256 VGPRs per wave, so these kernels split the work:
//   bcrw_fwd_factor  A_X in LDS; the Cholesky sweep with the couplings' solves (P_Iᵀ, P_Kᵀ) in
//                    registers, then a second substitution pass for W_X and z from the L left in
//                    LDS (read-only there: no barriers)
//   bcrw_fwd_delta   the neighbours' Δ updates and the new coupling from P_Iᵀ / P_Kᵀ as the
//                    factor launch left them in the workspace (C fragments read from L2)
//   bcrw_bwd         α, G, the Z panels and Z_XX with every block operand read from the workspace;
//                    Z_IX / Z_KX meet the other waves through the workspace behind a barrier
//   bcrw_contract    bcr_contract_kernel with Z read from the workspace instead of LDS
// Same mathematics as the Q <= 5 kernels (block cyclic reduction + Takahashi's selected inverse);
// a problem's arithmetic depends on its own data only (every Q = 6..8 problem takes bs = 128).
// ---------------------------------------------------------------------------------------
template <int Q>
__global__ __launch_bounds__(64 * Q) void bcrw_fwd_factor_kernel(BcrArgs a) {
  constexpr int bs = Bcr<Q>::bs, rs = Bcr<Q>::rs, BB = Bcr<Q>::BB, NT = 64 * Q;
  __shared__ __attribute__((aligned(16))) double lds[Bcr<Q>::mat + bs + 16 * kSC];
  double* sA = lds;                  // A_X -> L (W_tt on the diagonal tiles)
  double* sz = lds + Bcr<Q>::mat;    // y_X
  double* sc = sz + bs;              // leaf16m's scratch
  const int p = blockIdx.y, b = a.active[p];
  const int n = a.nvalid[b], n0 = (n + bs - 1) / bs, l = a.level;
  const int m = lvl_m(n0, l), top = lvl_top(n0);
  const int j = blockIdx.x;
  if (l > top || j >= m) return;
  const bool is_top = l == top;
  const bool elim = is_top || (j & 1);
  if (l == 0 && !elim) return;
  const int X = j << l, h = l > 0 ? 1 << (l - 1) : 0;
  const bool pl = l > 0 && X > 0, pr = l > 0 && X + h < n0;
  const BcrLayout Lw(bs, a.nbm);
  double* ws = a.ws + (long long)p * a.sWs;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, l15 = lane & 15, l4 = lane >> 4;
  const int K = X + (1 << l);
  const bool hasI = elim && !is_top, hasK = elim && !is_top && K < n0;
  double* Ag = ws + Lw.A + (long long)X * BB;
  double* yg = ws + Lw.y + (long long)X * bs;
  const double* CX = ws + Lw.C + (long long)X * BB;
  const double* CK = ws + Lw.C + (long long)K * BB;
  {  // A_X − (ΔR of X − h + ΔL of X + h), eight loads of each in flight per thread
    const double* dR = ws + Lw.DR + (long long)(X - h) * BB;
    const double* dL = ws + Lw.DL + (long long)(X + h) * BB;
    constexpr int CH = 8;
#pragma unroll 1
    for (int e0 = tid; e0 < BB; e0 += CH * NT) {
      double va[CH], vr[CH], vl[CH];
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        const int e = e0 + k * NT;
        va[k] = Ag[e];
        vr[k] = pl ? dR[e] : 0.0;
        vl[k] = pr ? dL[e] : 0.0;
      }
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        const int e = e0 + k * NT, r = e / bs, c = e - r * bs;
        const double v = va[k] - (vr[k] + vl[k]);
        if (elim)
          sA[r * rs + c] = v;
        else
          Ag[e] = v;
      }
    }
    if (tid < bs) {
      const double yr = pl ? ws[Lw.dyR + (long long)(X - h) * bs + tid] : 0.0;
      const double yl = pr ? ws[Lw.dyL + (long long)(X + h) * bs + tid] : 0.0;
      const double vy = yg[tid] - (yr + yl);
      if (elim)
        sz[tid] = vy;
      else
        yg[tid] = vy;
    }
  }
  if (!elim) return;
  // the couplings' right-hand sides, tile column w: R1 = E_XI, R2 = E_KXᵀ
  t4 R1[Q], R2[Q];
#pragma unroll
  for (int t = 0; t < Q; ++t) {
    R1[t] = hasI ? fr(CX, bs, t, w, l15, l4) : tzero();
    R2[t] = hasK ? frT(CK, bs, w, t, l15, l4) : tzero();
  }
  __syncthreads();
  // pass 1: right-looking Cholesky of A_X over its tile columns, with R1, R2
#pragma unroll
  for (int t = 0; t < Q; ++t) {
    if (w == t) {
      t4 Ad, V, Wr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = l15, cc = 4 * r + l4;
        Ad[r] = rr >= cc ? sA[(16 * t + rr) * rs + 16 * t + cc] : sA[(16 * t + cc) * rs + 16 * t + rr];
      }
      double lii;
      int fl;
      leaf16m(Ad, V, Wr, lii, fl, sc, l15, l4);
      fst(sA, rs, t, t, Wr, l15, l4);  // W_tt
      const int g = X * bs + 16 * t + l15;
      if (l4 == 0 && g < a.Np) a.ldiag[(long long)b * a.sVec + g] = log(lii);
      if (fl >= 0 && lane == 0) atomicCAS(a.info + b, 0, X * bs + 16 * t + fl + 1);
    }
    __syncthreads();
    const t4 WtT = frT(sA, rs, t, t, l15, l4);
    if (w > t) {  // panel L(w, t) = A(w, t) W_ttᵀ
      t4 c = tzero();
      mma(c, frT(sA, rs, w, t, l15, l4), WtT);
      fst(sA, rs, w, t, c, l15, l4);
    }
    {
      t4 c1 = tzero(), c2 = tzero();
      if (hasI) mma(c1, WtT, R1[t]);
      if (hasK) mma(c2, WtT, R2[t]);
      R1[t] = c1;
      R2[t] = c2;
    }
    __syncthreads();
    {
      int idx = 0;
#pragma unroll
      for (int s2 = t + 1; s2 < Q; ++s2)
#pragma unroll
        for (int r = t + 1; r <= s2; ++r, ++idx)
          if (idx % Q == w) {
            t4 c = fr(sA, rs, s2, r, l15, l4);
            mms(c, frT(sA, rs, s2, t, l15, l4), frT(sA, rs, r, t, l15, l4));
            fst(sA, rs, s2, r, c, l15, l4);
          }
    }
#pragma unroll
    for (int s2 = t + 1; s2 < Q; ++s2) {
      const t4 Ls = frT(sA, rs, s2, t, l15, l4);
      if (hasI) mms(R1[s2], Ls, R1[t]);
      if (hasK) mms(R2[s2], Ls, R2[t]);
    }
    __syncthreads();
  }
  double* PIg = ws + Lw.PI + (long long)X * BB;
  double* PKg = ws + Lw.PK + (long long)X * BB;
#pragma unroll
  for (int t = 0; t < Q; ++t) {
    if (hasI) fst(PIg, bs, t, w, R1[t], l15, l4);
    if (hasK) fst(PKg, bs, t, w, R2[t], l15, l4);
  }
  // pass 2: W_X = L⁻¹ (tile column w) and z_X = L⁻¹ y_X (wave Q−1) by substitution with the L in
  // LDS (read-only from here on)
  t4 R3[Q], RY[Q];
#pragma unroll
  for (int t = 0; t < Q; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      R3[t][r] = (t == w && 4 * r + l4 == l15) ? 1.0 : 0.0;
      RY[t][r] = (w == Q - 1 && l15 == 0) ? sz[16 * t + 4 * r + l4] : 0.0;
    }
  }
#pragma unroll
  for (int t = 0; t < Q; ++t) {
    const t4 WtT = frT(sA, rs, t, t, l15, l4);
    t4 c3 = tzero(), cy = tzero();
    if (t >= w) mma(c3, WtT, R3[t]);
    if (w == Q - 1) mma(cy, WtT, RY[t]);
    R3[t] = c3;
    RY[t] = cy;
#pragma unroll
    for (int s2 = t + 1; s2 < Q; ++s2) {
      const t4 Ls = frT(sA, rs, s2, t, l15, l4);
      if (t >= w) mms(R3[s2], Ls, R3[t]);
      if (w == Q - 1) mms(RY[s2], Ls, RY[t]);
    }
  }
  double* Wg = ws + Lw.Wm + (long long)X * BB;
#pragma unroll
  for (int t = 0; t < Q; ++t)
    if (t >= w) fst(Wg, bs, t, w, R3[t], l15, l4);
  if (w == Q - 1 && l15 == 0) {
#pragma unroll
    for (int t = 0; t < Q; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * t + 4 * r + l4, g = X * bs + i;
        ws[Lw.z + g] = RY[t][r];
        if (g < a.Np) a.z[(long long)b * a.sVec + g] = RY[t][r];
      }
  }
}

// the eliminated node's updates of its neighbours from the P_Iᵀ, P_Kᵀ, z_X the factor launch wrote
template <int Q>
__global__ __launch_bounds__(64 * Q) void bcrw_fwd_delta_kernel(BcrArgs a) {
  constexpr int bs = Bcr<Q>::bs, BB = Bcr<Q>::BB;
  const int p = blockIdx.y, b = a.active[p];
  const int n = a.nvalid[b], n0 = (n + bs - 1) / bs, l = a.level;
  const int m = lvl_m(n0, l), top = lvl_top(n0);
  const int j = blockIdx.x;
  if (l >= top || j >= m || !(j & 1)) return;  // (eliminated nodes below the top)
  const int X = j << l, K = X + (1 << l);
  const bool hasK = K < n0;
  const BcrLayout Lw(bs, a.nbm);
  double* ws = a.ws + (long long)p * a.sWs;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, l15 = lane & 15, l4 = lane >> 4;
  const double* PIg = ws + Lw.PI + (long long)X * BB;
  const double* PKg = ws + Lw.PK + (long long)X * BB;
  __shared__ double sz[bs];
  if (tid < bs) sz[tid] = ws[Lw.z + (long long)X * bs + tid];
  t4 R1[Q], R2[Q];
#pragma unroll
  for (int k = 0; k < Q; ++k) {
    R1[k] = fr(PIg, bs, k, w, l15, l4);
    R2[k] = hasK ? fr(PKg, bs, k, w, l15, l4) : tzero();
  }
  __syncthreads();
  {  // ΔA_I = P_I P_Iᵀ (lower tiles, column w) and y_I −= P_I z_X
    double* dLo = ws + Lw.DL + (long long)X * BB;
#pragma unroll
    for (int i = 0; i < Q; ++i) {
      if (i < w) continue;
      t4 c = tzero();
#pragma unroll
      for (int k = 0; k < Q; ++k) mma(c, fr(PIg, bs, k, i, l15, l4), R1[k]);
      fst(dLo, bs, i, w, c, l15, l4);
    }
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < Q; ++k)
#pragma unroll
      for (int r = 0; r < 4; ++r) s = fma(R1[k][r], sz[16 * k + 4 * r + l4], s);
    s = sum4(s);
    if (l4 == 0) ws[Lw.dyL + (long long)X * bs + 16 * w + l15] = s;
  }
  if (hasK) {  // ΔA_K = P_K P_Kᵀ, the new coupling E_KI = −P_K P_Iᵀ (-> C[K]), y_K −= P_K z_X
    double* dRo = ws + Lw.DR + (long long)X * BB;
    double* CKo = ws + Lw.C + (long long)K * BB;
#pragma unroll
    for (int i = 0; i < Q; ++i) {
      t4 e = tzero();
#pragma unroll
      for (int k = 0; k < Q; ++k) mms(e, fr(PKg, bs, k, i, l15, l4), R1[k]);
      fst(CKo, bs, i, w, e, l15, l4);
      if (i < w) continue;
      t4 c = tzero();
#pragma unroll
      for (int k = 0; k < Q; ++k) mma(c, fr(PKg, bs, k, i, l15, l4), R2[k]);
      fst(dRo, bs, i, w, c, l15, l4);
    }
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < Q; ++k)
#pragma unroll
      for (int r = 0; r < 4; ++r) s = fma(R2[k][r], sz[16 * k + 4 * r + l4], s);
    s = sum4(s);
    if (l4 == 0) ws[Lw.dyR + (long long)X * bs + 16 * w + l15] = s;
  }
}

// backward level l for bs = 128 (see bcr_bwd_kernel for the recurrences)
template <int Q>
__global__ __launch_bounds__(64 * Q) void bcrw_bwd_kernel(BcrArgs a) {
  constexpr int bs = Bcr<Q>::bs, BB = Bcr<Q>::BB;
  __shared__ double sz[bs], saI[bs], saK[bs], st[bs];
  const int p = blockIdx.y, b = a.active[p];
  const int n = a.nvalid[b], n0 = (n + bs - 1) / bs, l = a.level;
  const int m = lvl_m(n0, l), top = lvl_top(n0);
  if (l > top) return;
  const bool is_top = l == top;
  int X = 0;
  if (is_top) {
    if (blockIdx.x != 0) return;
  } else {
    const int j = 2 * blockIdx.x + 1;
    if (j >= m) return;
    X = j << l;
  }
  const int I = X - (1 << l), K = X + (1 << l);
  const bool hasI = !is_top, hasK = !is_top && K < n0;
  const BcrLayout Lw(bs, a.nbm);
  double* ws = a.ws + (long long)p * a.sWs;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, l15 = lane & 15, l4 = lane >> 4;
  const double* Wg = ws + Lw.Wm + (long long)X * BB;
  const double* PIg = ws + Lw.PI + (long long)X * BB;
  const double* PKg = ws + Lw.PK + (long long)X * BB;
  double* al = ws + Lw.al;
  if (tid < bs) {
    sz[tid] = ws[Lw.z + (long long)X * bs + tid];
    saI[tid] = hasI ? al[(long long)I * bs + tid] : 0.0;
    saK[tid] = hasK ? al[(long long)K * bs + tid] : 0.0;
  }
  __syncthreads();
  // α_X = W_Xᵀ (z_X − P_Iᵀ α_I − P_Kᵀ α_K): four threads per row (NT = 4·bs)
  {
    const int i = tid >> 2, q = tid & 3;
    double t = 0.0;
    if (hasI)
      for (int c = q; c < bs; c += 4) t = fma(PIg[i * bs + c], saI[c], t);
    if (hasK)
      for (int c = q; c < bs; c += 4) t = fma(PKg[i * bs + c], saK[c], t);
    t += __shfl_xor(t, 1, 64);
    t += __shfl_xor(t, 2, 64);
    if (q == 0) st[i] = sz[i] - t;
  }
  __syncthreads();
  {
    const int i = tid >> 2, q = tid & 3;
    double v = 0.0;
    for (int r = i + q; r < bs; r += 4) v = fma(Wg[r * bs + i], st[r], v);
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    if (q == 0) al[(long long)X * bs + i] = v;
  }
  // G_I = P_I W_X, G_K = P_K W_X (column w)
  t4 GI[Q], GK[Q];
#pragma unroll
  for (int k = 0; k < Q; ++k) {
    GI[k] = tzero();
    GK[k] = tzero();
  }
  if (hasI) {
#pragma unroll
    for (int mm = 0; mm < Q; ++mm) {
      if (mm < w) continue;
      const t4 Wm = fr(Wg, bs, mm, w, l15, l4);
#pragma unroll
      for (int k = 0; k < Q; ++k) {
        mma(GI[k], fr(PIg, bs, mm, k, l15, l4), Wm);
        if (hasK) mma(GK[k], fr(PKg, bs, mm, k, l15, l4), Wm);
      }
    }
  }
  double* ZC = ws + Lw.C;
  double* ZCX = ZC + (long long)X * BB;
  double* ZCK = ZC + (long long)K * BB;
  if (!is_top) {
    const double* ZI = ws + Lw.A + (long long)I * BB;
    const double* ZK = ws + Lw.A + (long long)K * BB;
    const double* ZKI = ZC + (long long)K * BB;
    t4 Z1[Q];
    // Z_IX = −(Z_II G_I + Z_KIᵀ G_K) -> C[X] as Z_{X,I} = Z_IXᵀ
#pragma unroll
    for (int i = 0; i < Q; ++i) {
      Z1[i] = tzero();
#pragma unroll
      for (int k = 0; k < Q; ++k) {
        mms(Z1[i], frT(ZI, bs, i, k, l15, l4), GI[k]);
        if (hasK) mms(Z1[i], fr(ZKI, bs, k, i, l15, l4), GK[k]);
      }
    }
#pragma unroll
    for (int i = 0; i < Q; ++i) fstT(ZCX, bs, i, w, Z1[i], l15, l4);
    // Z_KX = −(Z_KI G_I + Z_KK G_K) -> C[K], once every wave has read Z_KI out of it
    if (hasK) {
#pragma unroll
      for (int i = 0; i < Q; ++i) {
        Z1[i] = tzero();
#pragma unroll
        for (int k = 0; k < Q; ++k) {
          mms(Z1[i], frT(ZKI, bs, i, k, l15, l4), GI[k]);
          mms(Z1[i], frT(ZK, bs, i, k, l15, l4), GK[k]);
        }
      }
    }
    __syncthreads();
    if (hasK) {
#pragma unroll
      for (int i = 0; i < Q; ++i) fst(ZCK, bs, i, w, Z1[i], l15, l4);
    }
    __syncthreads();
  }
  // Z_XX row w = W_Xᵀ W_X − G_Iᵀ Z_IX − G_Kᵀ Z_KX
  t4 Zr[Q];
#pragma unroll
  for (int i = 0; i < Q; ++i) {
    Zr[i] = tzero();
#pragma unroll
    for (int mm = 0; mm < Q; ++mm) {
      if (mm < w || mm < i) continue;
      mma(Zr[i], fr(Wg, bs, mm, w, l15, l4), fr(Wg, bs, mm, i, l15, l4));
    }
    if (!is_top) {
#pragma unroll
      for (int k = 0; k < Q; ++k) {
        mms(Zr[i], GI[k], frT(ZCX, bs, i, k, l15, l4));
        if (hasK) mms(Zr[i], GK[k], fr(ZCK, bs, k, i, l15, l4));
      }
    }
  }
  double* ZX = ws + Lw.A + (long long)X * BB;
#pragma unroll
  for (int i = 0; i < Q; ++i) fst(ZX, bs, w, i, Zr[i], l15, l4);
}

// per problem: the [16] gradient row (Σ over blocks, in a fixed order) for the reduce kernel, the
// band check's maximum, and zeros in z / log L_ii / α past the last block (rows < Np). 256
// threads: thread t sums blocks t, t + 16, ... of parameter t % 16 (all loads in flight at once).
__global__ __launch_bounds__(256) void bcr_finish_kernel(BcrArgs a) {
  __shared__ double sp[16][GPX_THETA_STRIDE + 1];
  __shared__ double sm[256];
  const int p = blockIdx.x, b = a.active[p], bs = a.bs;
  const int n = a.nvalid[b], n0 = (n + bs - 1) / bs;
  const BcrLayout Lw(bs, a.nbm);
  const double* ws = a.ws + (long long)p * a.sWs;
  const int tid = threadIdx.x, q = tid & 15, jg = tid >> 4;
  double s = 0.0;
  for (int J = jg; J < n0; J += 16) s += ws[Lw.part + (long long)J * GPX_THETA_STRIDE + q];
  sp[jg][q] = s;
  double mx = 0.0;
  for (int J = tid; J < n0; J += 256) mx = fmax(mx, ws[Lw.chk + J]);
  sm[tid] = mx;
  for (int r = n0 * bs + tid; r < a.Np; r += 256) {
    a.z[(long long)b * a.sVec + r] = 0.0;
    a.ldiag[(long long)b * a.sVec + r] = 0.0;
    a.alpha[(long long)b * a.sVec + r] = 0.0;
  }
  __syncthreads();
  if (tid < GPX_THETA_STRIDE) {
    double t = 0.0;
    for (int k = 0; k < 16; ++k) t += sp[k][tid];
    a.partial[(long long)b * a.sPartial + tid] = t;
  }
  if (tid == 64) {
    double m = 0.0;
    for (int k = 0; k < 256; ++k) m = fmax(m, sm[k]);
    a.results[(long long)b * kResStride + kResBandCheck] = m;
  }
}

long long bcr_ws_doubles(int Q, int Nmax) {
  const int bs = 16 * (Q > kBcrMaxQ ? kBcrWideQ : Q);  // (the wide classes share bs = 128)
  return BcrLayout(bs, (Nmax + bs - 1) / bs).total;
}

template <int Q>
static void launch_bcr_q(BcrArgs a, int max_terms, int np, int Nmax, hipStream_t s) {
  constexpr int bs = 16 * Q;
  const int nbm = (Nmax + bs - 1) / bs;
  a.nbm = nbm;
  a.bs = bs;
  int top = 0;
  while (((nbm + (1 << top) - 1) >> top) > 1) ++top;
  hipLaunchKernelGGL(bcr_build_kernel<Q>, dim3(nbm, 2, np), dim3(256), 0, s, a);
  constexpr bool wide = Q > kBcrMaxQ;
  for (int l = 0; l <= top; ++l) {
    a.level = l;
    const dim3 grid((nbm + (1 << l) - 1) >> l, np);
    if constexpr (wide) {
      hipLaunchKernelGGL(bcrw_fwd_factor_kernel<Q>, grid, dim3(64 * Q), 0, s, a);
      if (l < top) hipLaunchKernelGGL(bcrw_fwd_delta_kernel<Q>, grid, dim3(64 * Q), 0, s, a);
    } else {
      hipLaunchKernelGGL(bcr_fwd_kernel<Q>, grid, dim3(64 * Q), 0, s, a);
    }
  }
  for (int l = top; l >= 0; --l) {
    a.level = l;
    const int m = (nbm + (1 << l) - 1) >> l;
    if constexpr (wide)
      hipLaunchKernelGGL(bcrw_bwd_kernel<Q>, dim3(std::max(1, m / 2), np), dim3(64 * Q), 0, s, a);
    else
      hipLaunchKernelGGL(bcr_bwd_kernel<Q>, dim3(std::max(1, m / 2), np), dim3(64 * Q), 0, s, a);
  }
  auto ck = max_terms <= 1 ? bcr_contract_kernel<Q, 1, wide>
                           : (max_terms == 2 ? bcr_contract_kernel<Q, 2, wide> : bcr_contract_kernel<Q, GPX_MAX_TERMS, wide>);
  hipLaunchKernelGGL(ck, dim3(nbm, np), dim3(256), 0, s, a);
  hipLaunchKernelGGL(bcr_finish_kernel, dim3(np), dim3(256), 0, s, a);
}

static void launch_bcr_direct(const BcrArgs& a, int Q, int max_terms, int np, int Nmax, hipStream_t s) {
  switch (Q) {
    case 1: launch_bcr_q<1>(a, max_terms, np, Nmax, s); break;
    case 2: launch_bcr_q<2>(a, max_terms, np, Nmax, s); break;
    case 3: launch_bcr_q<3>(a, max_terms, np, Nmax, s); break;
    case 4: launch_bcr_q<4>(a, max_terms, np, Nmax, s); break;
    case 5: launch_bcr_q<5>(a, max_terms, np, Nmax, s); break;
    default: launch_bcr_q<kBcrWideQ>(a, max_terms, np, Nmax, s); break;  // (Q = 6..8: bs = 128)
  }
}

// The chain as a HIP graph. A call of few problems is launch-bound on the host: ~20 dependent
// launches (build, ⌈log2 n0⌉ + 1 forward and as many backward levels, contraction, finish) cost
// ~0.1 ms of submit time per call, a quarter of the device chain. The chain's launches are a pure
// function of (Q, terms, problems, N_max) and the argument block (device pointers into the
// batch's buffers, which stay put between calls), so it is captured once per distinct key and
// replayed: the same kernels with the same arguments, one launch. GPX_BCR_GRAPH=0: direct launches.
// The graphs belong to the batch whose buffers they point into (gpx_batch::bcr_graphs): created on
// its first reduction call, destroyed with it (gpx_batch_destroy → bcr_graph_cache_free).
namespace {
struct BcrGraphKey {
  int device, Q, max_terms, np, Nmax, D, Np, ld;
  long long sX, sY, sWs, sVec, sMat, sPartial;
  const void* p[14];
  bool operator==(const BcrGraphKey& o) const { return std::memcmp(this, &o, sizeof(*this)) == 0; }
};
struct BcrGraphHash {
  size_t operator()(const BcrGraphKey& k) const {
    const unsigned char* b = reinterpret_cast<const unsigned char*>(&k);
    size_t h = 1469598103934665603ull;
    for (size_t i = 0; i < sizeof(k); ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
  }
};
struct BcrGraphCache {
  std::mutex mu;
  std::unordered_map<BcrGraphKey, hipGraphExec_t, BcrGraphHash> m;
};
// distinct chains kept per batch (keys shift with the call's width mix and the offset of each width
// group in the call's active list; beyond the cap: direct launches)
constexpr size_t kBcrGraphCap = 1024;
}  // namespace

void bcr_graph_cache_free(void* cache) {
  BcrGraphCache* c = static_cast<BcrGraphCache*>(cache);
  if (!c) return;
  for (auto& kv : c->m) (void)hipGraphExecDestroy(kv.second);
  delete c;
}

void launch_bcr(const BcrArgs& a, int Q, int max_terms, int np, int Nmax, hipStream_t s, void** cache) {
  static const bool graphs = [] {
    const char* e = getenv("GPX_BCR_GRAPH");
    return !(e && atoi(e) == 0);
  }();
  if (!graphs || !cache) return launch_bcr_direct(a, Q, max_terms, np, Nmax, s);
  if (!*cache) *cache = new BcrGraphCache();
  BcrGraphCache& gc = *static_cast<BcrGraphCache*>(*cache);
  BcrGraphKey k;
  std::memset(&k, 0, sizeof(k));  // (padding included: the key is compared and hashed bytewise)
  (void)hipGetDevice(&k.device);
  k.Q = Q; k.max_terms = max_terms; k.np = np; k.Nmax = Nmax; k.D = a.D; k.Np = a.Np; k.ld = a.ld;
  k.sX = a.sX; k.sY = a.sY; k.sWs = a.sWs; k.sVec = a.sVec; k.sMat = a.sMat; k.sPartial = a.sPartial;
  const void* ptrs[14] = {a.active, a.specs, a.theta, a.nvalid, a.X, a.Y, a.ws, a.info,
                          a.z, a.ldiag, a.alpha, a.Kd, a.partial, a.results};
  std::memcpy(k.p, ptrs, sizeof(ptrs));
  hipGraphExec_t exec = nullptr;
  {
    std::lock_guard<std::mutex> lk(gc.mu);
    auto it = gc.m.find(k);
    if (it != gc.m.end()) exec = it->second;
    else if (gc.m.size() >= kBcrGraphCap) return launch_bcr_direct(a, Q, max_terms, np, Nmax, s);
  }
  if (!exec) {
    hipGraph_t g = nullptr;
    if (hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed) != hipSuccess)
      return launch_bcr_direct(a, Q, max_terms, np, Nmax, s);
    BcrArgs c = a;
    c.level = 0;
    launch_bcr_direct(c, Q, max_terms, np, Nmax, s);
    if (hipStreamEndCapture(s, &g) != hipSuccess || !g ||
        hipGraphInstantiate(&exec, g, nullptr, nullptr, 0) != hipSuccess) {
      if (g) (void)hipGraphDestroy(g);
      (void)hipGetLastError();
      return launch_bcr_direct(a, Q, max_terms, np, Nmax, s);
    }
    (void)hipGraphDestroy(g);
    std::lock_guard<std::mutex> lk(gc.mu);
    gc.m.emplace(k, exec);
  }
  (void)hipGraphLaunch(exec, s);
}

}  // namespace gpx

#ifdef GPX_BCR_PHASES
// out[3*16*16] <- g_bcr_phase; reset != 0 zeroes it afterwards. Diagnostic build only.
extern "C" int gpx_debug_bcr_phases(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gpx::g_bcr_phase), sizeof(gpx::g_bcr_phase)) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long zero[3][16][16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(gpx::g_bcr_phase), zero, sizeof(zero)) != hipSuccess) return -1;
  }
  return 0;
}
#endif
