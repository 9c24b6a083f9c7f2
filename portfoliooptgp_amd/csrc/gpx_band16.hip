// gpx_band16.hip — the block-banded evaluation by 16-row blocks, one wavefront per problem
// (gfx950, fp64).
//
// Same mathematics as the 64-row fused sweeps of gpx_band.hip: a block-banded
// Cholesky of K + σn²I, z = L⁻¹y, α = L⁻ᵀz, the selected inverse Z = K⁻¹ on the band (Takahashi
// recurrences) and the gradient contraction ½Σ(ααᵀ − Z)∘∂K/∂θ over it, all exact because K and
// every ∂K/∂θ vanish exactly (exp underflow) outside the band. What changes is the granularity:
//
//   * blocks are 16 rows, one v_mfma_f64_16x16x4_f64 tile, and the band is Q 16-blocks wide
//     (Q = 1..5 for every band kernel family, 6..8 for SE1 problems with K's tiles computed in the
//     sweeps (ℓ up to ≈ 3.3 at unit spacing); at the reference's day-offset inputs and ℓ ∈ [1, 1.68], the band of exact
//     nonzeros is 39-65 entries: Q = 3-4 instead of the 64-row kernels' 128-wide two-block band,
//     so a step multiplies ~(56/96)² of the 64-row kernels' block entries and none of the
//     exactly-zero triangles of the 64-row blocks);
//   * one wavefront walks a whole problem, so a block step has no workgroup barrier: the
//     64-row kernels' steps were latency chains of 4 waves meeting at 8-10 barriers per step.
//     Independent problems on the same SIMD (2-3 waves) fill each other's MFMA / VALU gaps;
//   * every operand lives in registers as an MFMA C fragment (lane (l15, l4), register r holds
//     element (4r + l4, l15) of the tile). A C fragment is directly a valid A operand of the
//     tile's transpose and a B operand of the tile itself, so a chain of four MFMAs computes
//     Xᵀ·Y from the fragments of X and Y (mma / mms). The algebra below is arranged so that
//     every product has that form: the forward window holds Aᵀ blocks and W_kkᵀ, the panels
//     come out as Pᵀ; the backward sweep loads W_kk and Pᵀ from global memory in the
//     orientation it needs (a fragment load of a tile or of its transpose costs the same) and
//     transposes the window's off-diagonal Z tiles through a 2 KiB LDS scratch;
//   * the 16x16 diagonal Cholesky-and-inverse (leaf16m) runs on the matrix cores: four rank-4
//     steps, each a uniform 4x4 factorisation and two MFMAs (trailing update, L⁻¹ alongside).
//
// Inputs / outputs are those of band_fwd1_kernel / band_bwd1_kernel (the host picks this class
// for problems with p64 <= 2 and Q <= 5): K's band as built with kband = p64max + 1 64-block
// diagonals (entries in 64-block offset >= kband are read as the exact zeros they are), z,
// log L_ii, α, diag(Z) on K's diagonal (band_train_pred_kernel), the per-problem [16] gradient
// partial row, results[kResBandCheck] = max_j |Σ_i K_ji Z_ij − 1|, info (first failing pivot).
// The factor itself (W_kk = L_kk⁻¹ and the panels P_i = L_{k+i,k}) goes from the forward to the
// backward sweep through L's workspace in a private tile layout (frag_store below); the W
// workspace is not used.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include "gpx_internal.h"
#include "gpx_leaf.h"
#include "gpx_b16core.h"

namespace gpx {


// Phase timing (diagnostic build only, -DGPX_BAND_PHASES: libgpx_phases.so, tools/band16_phases.py):
// each wave adds the shader-clock cycles of its steps' phases into g_b16_phase[kernel][phase]
// ([kernel][15] counts waves).
#ifdef GPX_BAND_PHASES
__device__ unsigned long long g_b16_phase[2][16];
#define Q_BEGIN unsigned long long qp_t = __builtin_amdgcn_s_memtime(), qp_acc[12] = {};
#define QP(i)                                                        \
  do {                                                               \
    const unsigned long long qp_n = __builtin_amdgcn_s_memtime();    \
    qp_acc[i] += qp_n - qp_t;                                        \
    qp_t = qp_n;                                                     \
  } while (0)
#define Q_END(kid)                                                                 \
  do {                                                                             \
    if (threadIdx.x == 0) {                                                        \
      for (int qp_i = 0; qp_i < 12; ++qp_i) atomicAdd(&g_b16_phase[kid][qp_i], qp_acc[qp_i]); \
      atomicAdd(&g_b16_phase[kid][15], 1ull);                                      \
    }                                                                              \
  } while (0)
#else
#define Q_BEGIN
#define QP(i) \
  do {        \
  } while (0)
#define Q_END(kid) \
  do {             \
  } while (0)
#endif

namespace {

// frag of A_{bi,bj}ᵀ (bi >= bj, 16-blocks) from K's stored lower band; entries in 64-block
// offset >= kband (beyond the built band) read as 0 (exact: the class's p64 < kband); the
// diagonal tile from its lower triangle
__device__ __forceinline__ t4 ktile_t(const double* __restrict__ K, long long ld, int bi, int bj, int l15, int l4,
                                      int kband) {
  t4 t;
  const int gi = bi * 16 + l15;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int gj = bj * 16 + 4 * r + l4;
    const int i0 = max(gi, gj), j0 = min(gi, gj);
    const bool z = (i0 >> 6) - (j0 >> 6) >= kband;
    const double v = K[(long long)i0 * ld + (z ? i0 : j0)];
    t[r] = z ? 0.0 : v;
  }
  return t;
}

constexpr __host__ __device__ int wid(int i, int j) { return i * (i + 1) / 2 + j; }  // lower (i, j), j <= i

// Four exps in lockstep, as the device library computes exp (the sequence of the gfx950
// __ocml_exp_f64 code: a rndne(x·log2 e) reduction in two fma steps, a degree-12 polynomial,
// ldexp, the overflow and underflow selects — the same operations on the same constants, so the
// same bits; tests/test_inline_k_gpu.py checks them against the build kernel's exp). The library's
// exp alone is compiled with literal constants and v_fmac, whose accumulator must be a fresh
// vector copy of each constant: 14 v_mov_b64 per exp inside the sweeps' loops (≈ 230 per step).
// Four at a time, each constant is put in a register once for the four.
__device__ __forceinline__ void exp4(const double (&x)[4], double (&e)[4]) {
  constexpr double c[13] = {0x1.71547652b82fep+0, -0x1.62e42fefa39efp-1, -0x1.abc9e3b39803fp-56,
                            0x1.ade156a5dcb37p-26, 0x1.28af3fca7ab0cp-22, 0x1.71dee623fde64p-19,
                            0x1.a01997c89e6b0p-16, 0x1.a01a014761f6ep-13, 0x1.6c16c1852b7b0p-10,
                            0x1.1111111122322p-7, 0x1.55555555502a1p-5, 0x1.5555555555511p-3,
                            0x1.000000000000bp-1};
  double k[4], r[4], p[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    k[q] = __builtin_rint(x[q] * c[0]);
    r[q] = __builtin_fma(k[q], c[1], x[q]);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) r[q] = __builtin_fma(k[q], c[2], r[q]);
#pragma unroll
  for (int q = 0; q < 4; ++q) p[q] = __builtin_fma(r[q], c[3], c[4]);
#pragma unroll
  for (int i = 5; i <= 12; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) p[q] = __builtin_fma(r[q], p[q], c[i]);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    p[q] = __builtin_fma(r[q], p[q], 1.0);
    p[q] = __builtin_fma(r[q], p[q], 1.0);
    // (the library's overflow select, x > 1024 -> inf, is left out: here x = −½r² of finite inputs,
    // and for any x in (709.8, 2^31/log2 e) ldexp already overflows to the same inf — so the same
    // bits with one compare and one 64-bit select less per entry)
    const double v = __builtin_amdgcn_ldexp(p[q], (int)k[q]);
    e[q] = !(x[q] < -1075.0) ? v : 0.0;
  }
}
// the K tiles' exp: one at a time (the library's), or a tile's four together (exp4)
struct ExpLib {
  __device__ __forceinline__ void load() {}
  __device__ __forceinline__ double exp(double x) const { return ::exp(x); }
  __device__ __forceinline__ void exp4(const double (&x)[4], double (&e)[4]) const { gpx::exp4(x, e); }
};

// K_ij of the reference's kernel (SE1: one SquaredExponential term on one input column) from the
// scaled inputs a = x/ℓ, computed where a sweep needs it (KIN) instead of read from a K band that
// band16_build_kernel wrote: σ²·exp(−½ r²) with GPflow's r² (sqdist1), σn² added on the diagonal,
// the identity in the padding — the build kernel's operations, so the same bits (sqdist1 is
// symmetric in its arguments bit for bit, so no tile needs mirroring)
// (the row's −2a_i and a_i² formed once per row: sqdist1_b, the same bits as sqdist1(a_i, a_j))
template <class EXP>
__device__ __forceinline__ double k_se1(double m2ai, double ai2, double aj, bool ok, bool diag, double var,
                                       double noise, const EXP& E) {
  if (!ok) return diag ? 1.0 : 0.0;
  const double v = var * E.exp(-0.5 * sqdist1_b(aj, m2ai, ai2));  // (stationary_value<GPX_SE>'s operations)
  return diag ? v + noise : v;
}
// a tile in fragment-of-transpose layout (t[r] = A[bi·16 + l15][bj·16 + 4r + l4], as ktile_t reads
// it) into the row-major band where band16_build_kernel would have written it
__device__ __forceinline__ void ktile_store(double* __restrict__ K, long long ld, int bi, int bj, const t4& t, int l15,
                                            int l4) {
  double* p = K + (long long)(bi * 16 + l15) * ld + bj * 16 + l4;
#pragma unroll
  for (int r = 0; r < 4; ++r) p[4 * r] = t[r];
}
// index of element il of a 16-row block in the "row-quad" order (il & 3)·4 + (il >> 2): lane
// (l15, l4) finds the values of rows 4r + l4, r = 0..3, at 4·l4 .. 4·l4 + 3 (two ds_read_b128)
__device__ __forceinline__ int rq(int il) { return (il & 3) * 4 + (il >> 2); }

}  // namespace

// ---------------------------------------------------------------------------------------
// Forward sweep, k = 0 .. nb−1 (right-looking; window T_ij = fragment of A_{k+i,k+j}ᵀ,
// 0 <= j <= i <= Q, with the updates of the previous steps applied):
//   leaf(A_kk) -> V = W_kkᵀ, L_ii;  z_k = W_kk (y_k + u_k)
//   Q_i = Vᵀ T_i0 = P_iᵀ (P_i = A_{k+i,k} W_kkᵀ = L_{k+i,k});  u_{k+i} −= P_i z_k
//   T_ij −= Q_jᵀ Q_i   (A_{k+i,k+j} −= P_i P_jᵀ), 1 <= j <= i <= Q
// then the window moves down one block; its new row (block k+Q+1) is loaded during the step.
// ---------------------------------------------------------------------------------------
#ifndef GPX_B16_FWD3_WAVES
#define GPX_B16_FWD3_WAVES 2  // waves per SIMD the Q <= 3 forward sweep is compiled for
#endif
// KIN (SE1 problems only): the window's K tiles are computed in the sweep from X (k_se1) instead
// of read from the K band band16_build_kernel wrote — no build launch, and K's band never goes
// through HBM (2·(Q+1)·16·N doubles less per evaluation); the inputs of the last Q+1 blocks sit
// scaled (x/ℓ) in a small LDS ring.
// The sweeps are device functions over an LDS block the caller owns, so the forward and backward
// sweeps of one problem can run in one wavefront (band16_fused_kernel) on one LDS allocation.
template <int Q, bool KIN>
struct Fwd16 {  // the forward sweep's LDS, in doubles: scratch | the entering row (glds) | x/ℓ ring (KIN)
  static constexpr int kNew = 16 * kSC, kXa = kNew + (KIN ? 1 : Q + 1) * 256, size = kXa + (KIN ? Q + 1 : 1) * 16;
};
template <int Q, bool KIN>
__device__ __forceinline__ void fwd_sweep(const BandFusedArgs& a, double* __restrict__ lds) {
  double* sc = lds;
  double(*snew)[256] = reinterpret_cast<double(*)[256]>(lds + Fwd16<Q, KIN>::kNew);  // the entering row, staged by glds
  double(*sxa)[16] = reinterpret_cast<double(*)[16]>(lds + Fwd16<Q, KIN>::kXa);  // KIN: x/ℓ of blocks m, slot m % (Q+1), rq order
  const unsigned long long wt0 = a.wtrace ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const int b = a.active[blockIdx.x];
  const int Np = a.Np, nb = Np >> 4;
  const long long ld = a.ld;
  double* K = a.K + (long long)b * a.sMat;  // (KIN with kstore: written, otherwise read)
  double* L = a.L + (long long)b * a.sMat;
  double* z = a.z + (long long)b * a.sVec;
  double* ldiag = a.ldiag + (long long)b * a.sVec;
  const bool kst = KIN && a.kstore;
  const double* y = a.Y + (long long)b * a.sY;
  const int n = a.nvalid[b];
  const int lane = threadIdx.x, l15 = lane & 15, l4 = lane >> 4;
  constexpr int NW = (Q + 1) * (Q + 2) / 2;
  // KIN: the SE1 term's column, ℓ, σ², σn²
  const double* X = a.X + (long long)b * a.sX;
  int xd0 = 0;
  double kell = 1.0, kvar = 1.0, knoise = 0.0;
  ExpLib E;
  if constexpr (KIN) {
    E.load();
    const gpx_term& tm = a.specs[b].terms[0];
    const double* th = a.theta + (long long)b * GPX_THETA_STRIDE;
    xd0 = tm.dim_start;
    kell = th[tm.param_offset];
    kvar = th[tm.param_offset + 1];
    knoise = th[a.specs[b].n_params];
  }
  const int D = a.D;
  auto xval = [&](int g) { return X[(long long)min(g, n - 1) * D + xd0]; };  // (clamped into the slot's rows)
  t4 T[NW];
  double u[Q + 1];
  if constexpr (KIN) {
    // blocks 0..Q: the ring and the first window, computed
    if (l4 == 0) {
#pragma unroll
      for (int m = 0; m <= Q; ++m) sxa[m][rq(l15)] = m < nb ? xval(m * 16 + l15) / kell : 0.0;
    }
    wsync();
#pragma unroll
    for (int i = 0; i <= Q; ++i) {
      u[i] = 0.0;
      const double ar = i < nb ? xval(i * 16 + l15) / kell : 0.0;
      const int gi = i * 16 + l15;
#pragma unroll
      for (int j = 0; j <= i; ++j) {
        t4 t = tzero();
        if (i < nb) {
          const t4 ac = *reinterpret_cast<const t4*>(&sxa[j][4 * l4]);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int gj = j * 16 + 4 * r + l4;
            const bool zero = (gi >> 6) - (gj >> 6) >= a.kband;
            t[r] = zero ? 0.0 : k_se1(-2.0 * ar, ar * ar, ac[r], gi < n && gj < n, gi == gj, kvar, knoise, E);
          }
          if (kst) ktile_store(K, ld, i, j, t, l15, l4);
        }
        T[wid(i, j)] = t;
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i <= Q; ++i) {
      u[i] = 0.0;
#pragma unroll
      for (int j = 0; j <= i; ++j) T[wid(i, j)] = (i < nb) ? ktile_t(K, ld, i, j, l15, l4, a.kband) : tzero();
    }
  }
  int gfail = 0;
  Q_BEGIN
  // one block step; qkc = the window rows below the diagonal block (Q but in the last Q steps),
  // fullc: a new row enters (all but the last Q + 1 steps). The steps with both constant run
  // as a loop of their own, free of the edge conditions and their branches
  auto step = [&](const int k, const auto qkc, const auto fullc) __attribute__((always_inline)) {
    const int qk = qkc, k16 = k * 16;
    // the row entering the window after this step (block bn = k+Q+1): global -> LDS, in flight
    // during the step (the previous step's reads of snew are done: program order + wsync);
    // KIN: only its inputs (one value per row, into a register)
    const int bn = k + Q + 1;
    const bool newrow = decltype(fullc)::value || bn < nb;
    double xn = 0.0;
    if constexpr (KIN) {
      if (newrow) xn = xval(bn * 16 + l15);
    } else {
      wsync();
      lds_drain();  // the previous step's reads of snew have completed
      if (newrow) {
#pragma unroll
        for (int j = 0; j <= Q; ++j) tile_glds_swz(K + (long long)(bn * 16) * ld + (k + 1 + j) * 16, ld, snew[j], lane);
      }
    }
    // y_k in the row layout of u (lane l15 holds row l15)
    double yl = y[min(k16 + l15, n - 1)];
    yl = k16 + l15 < n ? yl : 0.0;
    QP(0);
    t4 V;
    double lii;
    int fl;
    double* Lk = L + (long long)k * ((Q + 1) * 256);  // this step's tiles (private layout above)
    double zr[4];  // z_k[4r + l4] (the panels' layout), on every lane of the row
    {
      t4 Wr;
      leaf16m(T[wid(0, 0)], V, Wr, lii, fl, sc, l15, l4);
      frag_store(Wr, Lk, lane);  // W_kk
      QP(1);
      // z_k = W_kk (y_k + u_k): Wr[r] = W_kk[4r+l4][l15], so each row is a 16-lane sum (DPP
      // butterfly) of Wr[r]·(y + u)[l15], with y and u already in that lane layout
      const double yu = yl + u[0];
#pragma unroll
      for (int r = 0; r < 4; ++r) zr[r] = sum16(Wr[r] * yu);
    }
    if (fl >= 0 && gfail == 0) gfail = k16 + fl + 1;
    QP(2);
    // panels: Q_i = Vᵀ T_i0 (= P_iᵀ), stored as P_i = L_{k+i,k}; u_{k+i} −= P_i z_k
#pragma unroll
    for (int i = 1; i <= Q; ++i) {
      if (i <= qk) {
        t4 c = tzero();
        mma(c, V, T[wid(i, 0)]);
        T[wid(i, 0)] = c;
        double s = 0.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) s = fma(c[r], zr[r], s);
        u[i] -= sum4(s);
      }
    }
    QP(3);
    // trailing update of the window
#pragma unroll
    for (int i = 1; i <= Q; ++i)
#pragma unroll
      for (int j = 1; j <= i; ++j)
        if (i <= qk) mms(T[wid(i, j)], T[wid(j, 0)], T[wid(i, 0)]);
    QP(4);
    // the new row has landed (this also retires W_kk's store, issued right after the leaf); the
    // panels, L_ii and z_k go out now, so that the next step's wait does not cover them early
    vm_drain();
    wsync();
    QP(6);
#pragma unroll
    for (int i = 1; i <= Q; ++i)
      if (i <= qk) frag_store(T[wid(i, 0)], Lk + i * 256, lane);  // P_iᵀ
    if (l4 == 0) ldiag[k16 + l15] = lii;
    if (l15 == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) z[k16 + 4 * r + l4] = zr[r];
    }
    // move the window down one block; its new row from LDS (fragments of A_{bn, k+1+j}ᵀ, entries
    // in 64-block offset >= 2 as exact zeros, the diagonal tile mirrored from its lower triangle)
#pragma unroll
    for (int i = 0; i < Q; ++i) {
#pragma unroll
      for (int j = 0; j <= i; ++j) T[wid(i, j)] = T[wid(i + 1, j + 1)];
      u[i] = u[i + 1];
    }
    u[Q] = 0.0;
    QP(7);
    if constexpr (KIN) {
      // block bn's inputs join the ring (in the slot of block k, whose last reads were at the
      // previous step's end), then the new row's tiles (bn, k+1+j) from x/ℓ
      const double ar = xn / kell, m2ar = -2.0 * ar, ar2 = ar * ar;
      if (newrow && l4 == 0) sxa[bn % (Q + 1)][rq(l15)] = ar;
      wsync();
      const int gi = bn * 16 + l15;
#pragma unroll
      for (int j = 0; j <= Q; ++j) {
        t4 t = tzero();
        const int c = k + 1 + j;
        // (16-row blocks sit inside one 64-block: the 64-block offset is uniform over the tile)
        if (newrow && (bn >> 2) - (c >> 2) < a.kband) {
          const t4 ac = *reinterpret_cast<const t4*>(&sxa[c % (Q + 1)][4 * l4]);
          // the tile's four exps together (k_se1's operations, element by element)
          double xe[4], ev[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) xe[r] = -0.5 * sqdist1_b(ac[r], m2ar, ar2);
          E.exp4(xe, ev);
          if (bn * 16 + 16 <= n) {
            // (uniform) every row of block bn holds data, so every entry of its tiles does: only
            // the diagonal tile's diagonal takes σn² — the general form below without its selects
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const double v = kvar * ev[r];
              t[r] = (j == Q && 4 * r + l4 == l15) ? v + knoise : v;
            }
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int gj = c * 16 + 4 * r + l4;
              const double v = kvar * ev[r];
              t[r] = !(gi < n && gj < n) ? (gi == gj ? 1.0 : 0.0) : (gi == gj ? v + knoise : v);
            }
          }
          if (kst) ktile_store(K, ld, bn, c, t, l15, l4);
        }
        T[wid(Q, j)] = t;
      }
    } else {
#pragma unroll
      for (int j = 0; j <= Q; ++j) {
        t4 t = tzero();
        if (newrow) {
          // (16-row blocks sit inside one 64-block: the 64-block offset is uniform over the tile)
          const bool zero = (bn >> 2) - ((k + 1 + j) >> 2) >= a.kband;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int cl = 4 * r + l4;
            const double v = (j == Q && cl > l15) ? snew[j][swz16(cl, l15)] : snew[j][swz16(l15, cl)];
            t[r] = zero ? 0.0 : v;
          }
        }
        T[wid(Q, j)] = t;
      }
    }
    QP(5);
  };
  int k = 0;
  // (not the two-wave Q = 4 sweep: its two copies of the step no longer fit 256 registers)
  if constexpr (Q != 4)
    for (; k < nb - Q - 1; ++k) step(k, std::integral_constant<int, Q>{}, std::true_type{});
  for (; k < nb; ++k) step(k, min(Q, nb - 1 - k), std::false_type{});
  Q_END(0);
  if (lane == 0 && gfail > 0 && a.info[b] == 0) a.info[b] = gfail;
  wave_trace_put(a, wt0, Q);
}

template <int Q, bool KIN>
__global__ __launch_bounds__(64, Q <= 3 ? GPX_B16_FWD3_WAVES : (Q <= 4 ? 2 : 1)) void band16_fwd_kernel(BandFusedArgs a) {
  __shared__ __attribute__((aligned(16))) double lds[Fwd16<Q, KIN>::size];
  fwd_sweep<Q, KIN>(a, lds);
}

// ---------------------------------------------------------------------------------------
// Backward sweep, k = nb−1 .. 0 (window S_ij = fragment of Z_{k+i,k+j}, 1 <= j <= i <= Q):
//   α_k = W_kkᵀ (z_k − Σ_i P_iᵀ α_{k+i})
//   G_i = P_i W_kk                                   (Xᵀ·Y with X = P_iᵀ, Y = W_kk)
//   Z_{k+i,k} = −Σ_j Z_{k+i,k+j} G_j                 (X = Z_{k+j,k+i}: S_ji, or S_ijᵀ when j < i)
//   Z_kk = W_kkᵀ W_kk − Σ_i G_iᵀ Z_{k+i,k}
//   contraction of Z_kk (whole, weight 1) and Z_{k+i,k} (weight 2), the band check's K∘Z sums
// The window then moves up one block (Z_kk and Z_{k+i,k} enter, row k+Q leaves).
// Band check: column j of block k gets its lower-band sums at step k (column sums of the
// step's tiles) and its upper-band sums from the row sums of tiles (k, k−m), m = 1..Q, at the
// following steps: complete after step k−Q (kept in LDS rings, rows/columns by 16-lane sums).
// ---------------------------------------------------------------------------------------
// SE1: every problem of the launch is the reference's kernel (one SquaredExponential term on one
// input column): the contraction is a straight-line loop (contract_block_se1's operations).
#ifndef GPX_B16_BWD_2W_QMAX
#define GPX_B16_BWD_2W_QMAX 3  // widest band the SE1 backward sweep is compiled for two waves per SIMD
#endif
// KIN (SE1 only): K_ij computed from the r² the contraction forms anyway (k_se1's operations)
// instead of fetched from the built K band: no K traffic and no 16 KiB K-tile double buffer.
template <int Q, int NT, bool SE1, bool KIN>
struct Bwd16 {  // the backward sweep's LDS, in doubles
  // scratch [16][kSC] (SE1: θ at [0, 16) before the loop and the final sums at [16, 30) after it)
  static constexpr int kZ = 16 * kSC;
  // SE1: the K tiles (k+i, k) as built, double-buffered by step parity (the next step's are
  // fetched by glds while this step's are contracted; not KIN); otherwise the step's Z tiles
  // for the runtime contraction loop
  static constexpr int nZ = SE1 ? (KIN ? 0 : 2 * (Q + 1)) : Q + 1;
  static constexpr int kAl = kZ + nZ * 256;                     // α ring (not SE1)
  // SE1: the α and x values of block m's rows in the contraction's lane order (lane (l15, l4)
  // takes rows 4r + l4: element of row il at (il & 3)·4 + (il >> 2)), so a lane reads its four
  // with two ds_read_b128 instead of four strided reads
  static constexpr int kAlT = kAl + (SE1 ? 0 : (Q + 1) * 16);
  static constexpr int kXT = kAlT + (SE1 ? (Q + 1) * 16 : 0);
  static constexpr int kCs = kXT + (SE1 ? (Q + 1) * 16 : 0);   // band check: column sums ring
  static constexpr int kTh = kCs + (Q + 1) * 16;                // θ (not SE1: the term interpreter reads it in the loop)
  static constexpr int kRed = kTh + (SE1 ? 0 : 16);
  // LP (the Q = 4 inline-K sweep): the next step's W_kk and P_iᵀ staged in LDS by glds instead
  // of registers — 40 VGPRs fewer, so the sweep fits two waves per SIMD without spilling
  static constexpr bool LP = SE1 && KIN && Q == 4;
  static constexpr int kPf = kRed + (SE1 ? 0 : 16);
  static constexpr int size = kPf + (LP ? (Q + 1) * 256 : 0);
};
template <int Q, int NT, bool SE1, bool KIN>
__device__ __forceinline__ void bwd_sweep(const BandFusedArgs& a, double* __restrict__ lds, double* __restrict__ sx) {
  static_assert(!SE1 || KIN || Q <= 5, "the SE1 sweep double-buffers its K tiles in LDS: Q <= 5");
  static_assert(!KIN || SE1, "inline K tiles: SE1 sweeps only");
  using Ly = Bwd16<Q, NT, SE1, KIN>;
  // sx: X ring [Q+1][16·D] (block m in slot m % (Q+1); not SE1)
  double* sc = lds;
  double(*sz)[256] = reinterpret_cast<double(*)[256]>(lds + Ly::kZ);
  double(*sal)[16] = reinterpret_cast<double(*)[16]>(lds + Ly::kAl);
  double(*salT)[16] = reinterpret_cast<double(*)[16]>(lds + Ly::kAlT);
  double(*sxT)[16] = reinterpret_cast<double(*)[16]>(lds + Ly::kXT);
  double(*scs)[16] = reinterpret_cast<double(*)[16]>(lds + Ly::kCs);
  double* sth = SE1 ? lds : lds + Ly::kTh;
  double* sred = SE1 ? lds + 16 : lds + Ly::kRed;
  const unsigned long long wt0 = a.wtrace ? __builtin_amdgcn_s_memrealtime() : 0ull;
  const int b = a.active[blockIdx.x];
  const int Np = a.Np, nb = Np >> 4;
  const long long ld = a.ld;
  double* Kd = a.K + (long long)b * a.sMat;           // diag(Z) goes on K's diagonal
  const double* L = a.L + (long long)b * a.sMat;
  const double* z = a.z + (long long)b * a.sVec;
  double* alpha = a.alpha + (long long)b * a.sVec;
  const double* X = a.X + (long long)b * a.sX;
  const int n = a.nvalid[b], D = a.D, nx = 16 * D;
  const int lane = threadIdx.x, l15 = lane & 15, l4 = lane >> 4;
  // inputs of a step: z_k and the block's X rows into registers (and, SE1, the K tiles by glds),
  // issued at the start of the step before
  auto fetch = [&](int kk, double (&zr)[4], double (&xr)[2]) {
    const int q1 = min(Q, nb - 1 - kk), c16 = kk * 16;
    if constexpr (SE1 && !KIN) {
#pragma unroll
      for (int i = 0; i <= Q; ++i)
        if (i <= q1) tile_glds_swz(Kd + (long long)(c16 + 16 * i) * ld + c16, ld, sz[(kk & 1) * (Q + 1) + i], lane);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) zr[r] = z[c16 + 4 * r + l4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // the first 128 values of the rows (all of them for D <= 8)
      const int e = lane + 64 * h;
      xr[h] = X[min((long long)c16 * D + e, (long long)n * D - 1)];  // (clamped into the slot's rows)
    }
  };
  // W_kk and P_iᵀ (the forward sweep's tiles, frag_store layout) straight into registers: two
  // 16-byte loads per lane and tile, issued once this step's P/G registers are dead (after Z_kk),
  // so the prefetch needs no LDS and no extra registers
  constexpr bool LP = Ly::LP;
  double* spf = lds + Ly::kPf;  // LP: tile i (W_kk, P_iᵀ) as two 1 KiB halves (a lane's 16-byte pieces)
  auto fetch_f = [&](int kk, t4& Wn, t4 (&Pn)[Q + 1]) {
    const int q1 = min(Q, nb - 1 - kk);
    const double* Lk = L + (long long)kk * ((Q + 1) * 256) + 4 * lane;
    if constexpr (LP) {
#pragma unroll
      for (int i = 0; i <= Q; ++i)
        if (i <= q1) {
          __builtin_amdgcn_global_load_lds(Lk + i * 256, spf + i * 256, 16, 0, 0);
          __builtin_amdgcn_global_load_lds(Lk + i * 256 + 2, spf + i * 256 + 128, 16, 0, 0);
        }
    } else {
      Wn = *reinterpret_cast<const t4*>(Lk);
#pragma unroll
      for (int i = 1; i <= Q; ++i) Pn[i] = (i <= q1) ? *reinterpret_cast<const t4*>(Lk + i * 256) : tzero();
    }
  };
  // LP: tile i back from the staging buffer (lane's 4 doubles as they lie in the frag layout)
  auto lds_tile = [&](int i) {
    const double2 a0 = *reinterpret_cast<const double2*>(spf + i * 256 + 2 * lane);
    const double2 a1 = *reinterpret_cast<const double2*>(spf + i * 256 + 128 + 2 * lane);
    return (t4){a0.x, a0.y, a1.x, a1.y};
  };
  double zr[4], xr[2];
  t4 Wn, Pn[Q + 1];
  fetch(nb - 1, zr, xr);
  fetch_f(nb - 1, Wn, Pn);
  {  // the forward sweep left L_ii: log det's terms (read by the reduce kernel)
    double* ldg = a.ldiag + (long long)b * a.sVec;
    for (int e = lane; e < Np; e += 64) ldg[e] = log(ldg[e]);
  }
  if (lane < GPX_THETA_STRIDE) sth[lane] = a.theta[b * GPX_THETA_STRIDE + lane];
  if (lane < 16) {
#pragma unroll
    for (int m = 0; m <= Q; ++m) {
      scs[m][lane] = 0.0;
      if constexpr (SE1) {
        salT[m][lane] = 0.0;
        sxT[m][lane] = 0.0;
      } else {
        sal[m][lane] = 0.0;
      }
    }
  }
  vm_drain();
  wsync();
  const DevSpec spec = a.specs[b];
  const int fkind = spec.terms[0].kind, fd0 = spec.terms[0].dim_start, fdn = spec.terms[0].dim_count;
  const bool fast = (NT == 1) && spec.n_terms == 1 && fkind >= GPX_SE && fkind <= GPX_EXPONENTIAL;
  const double fvar = sth[spec.terms[0].param_offset + 1];
  const double finv_ell = 1.0 / sth[spec.terms[0].param_offset];
  const double xscale = fast ? sth[spec.terms[0].param_offset] : 1.0;
  const double noise = sth[spec.n_params];
  double sums[NT][3];
#pragma unroll
  for (int t = 0; t < NT; ++t) sums[t][0] = sums[t][1] = sums[t][2] = 0.0;
  double snoise = 0.0, resmax = 0.0;
  constexpr int NS = Q * (Q + 1) / 2;  // window tiles S_ij, 1 <= j <= i <= Q  ->  S[wid(i-1, j-1)]
  t4 S[NS];
#pragma unroll
  for (int e = 0; e < NS; ++e) S[e] = tzero();
  double al[Q + 1];  // α_{k+i}[l15], i = 1..Q
  t4 R[Q + 1];       // band check: row-sum partials of blocks k+i (rows 4r + l4, unreduced over l15)
#pragma unroll
  for (int i = 0; i <= Q; ++i) {
    al[i] = 0.0;
    R[i] = tzero();
  }
  Q_BEGIN
  for (int k = nb - 1; k >= 0; --k) {
    const int qk = min(Q, nb - 1 - k), k16 = k * 16, cs = k % (Q + 1);
    // this step's W_kk and P_iᵀ (loaded during the previous step)
    t4 Wf, P[Q + 1];  // P_iᵀ, then G_i
    if constexpr (LP) {
      vm_drain();  // (the staged tiles have landed; this step's reads precede the next fetch_f)
      wsync();
      Wf = lds_tile(0);
#pragma unroll
      for (int i = 1; i <= Q; ++i) P[i] = (i <= qk) ? lds_tile(i) : tzero();
    } else {
      Wf = Wn;
#pragma unroll
      for (int i = 1; i <= Q; ++i) P[i] = Pn[i];
    }
    // X rows of block k -> ring slot cs (scaled by 1/ℓ as GPflow's Stationary.scale when fast)
    if constexpr (!SE1) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int e = lane + 64 * h;
        if (e < nx) sx[cs * nx + e] = (k16 + e / D < n) ? xr[h] / xscale : 0.0;
      }
      for (int e = lane + 128; e < nx; e += 64) sx[cs * nx + e] = (k16 + e / D < n) ? X[(long long)k16 * D + e] / xscale : 0.0;
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int e = lane + 64 * h, il = e / D;
        if (e < nx && e - il * D == fd0) sxT[cs][(il & 3) * 4 + (il >> 2)] = (k16 + il < n) ? xr[h] / xscale : 0.0;
      }
    }
    const double zc[4] = {zr[0], zr[1], zr[2], zr[3]};
    lds_drain();
    wsync();
    // the next step's inputs, in flight during this step
    if (k > 0) fetch(k - 1, zr, xr);
    QP(0);
    // α_k = W_kkᵀ (z_k − Σ_i P_iᵀ α_{k+i})
    // (no edge conditions in this step's products: the window's tiles beyond the last block
    // are exact zeros — P_i past qk is loaded as 0, so G_i, Z_{k+i,k} and every S tile that
    // reaches past the matrix stay 0 — and adding their zero products leaves every value as is)
    double t[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int i = 1; i <= Q; ++i) {
      // (LP: α_{k+i}[l15] from the ring the contraction reads — the value al[i] holds, without
      // its registers and shifts)
      double ai;
      if constexpr (LP)
        ai = salT[(k + i) % (Q + 1)][(l15 & 3) * 4 + (l15 >> 2)];
      else
        ai = al[i];
#pragma unroll
      for (int r = 0; r < 4; ++r) t[r] = fma(P[i][r], ai, t[r]);
    }
    double ap = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) ap = fma(Wf[r], zc[r] - sum16(t[r]), ap);
    ap = sum4(ap);
    al[0] = ap;
    if (l4 == 0) {
      if constexpr (SE1)
        salT[cs][(l15 & 3) * 4 + (l15 >> 2)] = ap;
      else
        sal[cs][l15] = ap;
    }
    QP(1);
    // G_i = P_i W_kk
#pragma unroll
    for (int i = 1; i <= Q; ++i) {
      t4 g = tzero();
      mma(g, P[i], Wf);
      P[i] = g;
    }
    QP(2);
    // Z_{k+i,k} = −Σ_j Z_{k+i,k+j} G_j
    t4 Zn[Q + 1];
#pragma unroll
    for (int i = 1; i <= Q; ++i) {
      Zn[i] = tzero();
#pragma unroll
      for (int j = 1; j <= Q; ++j) {
        if (j >= i) {
          mms(Zn[i], S[wid(j - 1, i - 1)], P[j]);
        } else {
          const t4 tt = tile_transpose(S[wid(i - 1, j - 1)], sc, l15, l4);
          mms(Zn[i], tt, P[j]);
        }
      }
    }
    QP(3);
    // the next step's W_kk and P_iᵀ, in flight during Z_kk and the contraction (issued ahead of
    // Z_kk's MFMA chain, which holds the wave's issue for ~1k cycles)
    if (k > 0) fetch_f(k - 1, Wn, Pn);
    // Z_kk = W_kkᵀ W_kk − Σ_i G_iᵀ Z_{k+i,k}
    t4 Zk = tzero();
    mma(Zk, Wf, Wf);
#pragma unroll
    for (int i = 1; i <= Q; ++i) mms(Zk, P[i], Zn[i]);
    wsync();
    QP(4);
    // gradient contraction and the band check's K∘Z sums over tile i (0: Z_kk whole, weight 1;
    // i >= 1: Z_{k+i,k}, weight 2): lane (l15, l4) takes rows 4r + l4 of column l15
    const int gj = k16 + l15;
    const bool jok = gj < n;
    const double* xj = sx + cs * nx + l15 * D;
    double colacc = 0.0;
    if constexpr (SE1) {
      // K_ij from the built band (the same var·exp(−r²/2) bits the exp would give; entries in
      // 64-block offset >= kband are the exact zeros of the class; the diagonal tile mirrored
      // from its lower triangle): ∂K/∂ℓ = K r²/ℓ, and Σ v ∂K/∂σ² = (Σ v K)/σ² at the end
      const double xjv = sxT[cs][(l15 & 3) * 4 + (l15 >> 2)];
      const double m2xj = -2.0 * xjv, xj2 = xjv * xjv;
#pragma unroll
      for (int i = 0; i <= Q; ++i) {
        if (i > qk) continue;
        const t4& Zt = (i == 0) ? Zk : Zn[i];
        const int si = (k + i) % (Q + 1);
        const double w = i == 0 ? 1.0 : 2.0;
        const t4 a4 = *reinterpret_cast<const t4*>(&salT[si][4 * l4]);  // α of rows 4r + l4
        const t4 x4 = *reinterpret_cast<const t4*>(&sxT[si][4 * l4]);   // x of rows 4r + l4
        const bool zero = ((k + i) >> 2) - (k >> 2) >= a.kband;  // (uniform, see the forward sweep)
        double r2v[4], kexp[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int r = 0; r < 4; ++r) r2v[r] = sqdist1_b(x4[r], m2xj, xj2);
        if constexpr (KIN) {
          if (!zero) {
            double xe[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) xe[r] = -0.5 * r2v[r];
            exp4(xe, kexp);
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int il = 4 * r + l4, gi = (k + i) * 16 + il;
          const double zij = Zt[r];
          const double ai = a4[r];
          const double r2 = r2v[r];
          const bool dg = i == 0 && il == l15;
          double kraw;
          if constexpr (KIN) {
            // (a zero tile's kexp stays 0: kraw is 0.0 there, as the built band holds. Rows past
            // n: on the diagonal tile `ok` masks them; off it their α (the ring holds 0) and Z
            // entries are exact zeros, so each of their terms below adds ±0 to a sum that starts
            // at +0 and only meets finite values — the sums' bits are those of the masked form)
            kraw = 0.0;
            if (!zero) {
              const double kv = fvar * kexp[r];  // (stationary_value<GPX_SE>'s operations)
              kraw = dg ? kv + noise : kv;
            }
          } else {
            const bool up = i == 0 && il < l15;
            kraw = sz[(k & 1) * (Q + 1) + i][up ? swz16(l15, il) : swz16(il, l15)];  // (swizzled rows)
          }
          const double v = w * fma(ai, ap, -zij);
          // rows or columns past n: off the diagonal tile the built band holds exact zeros there
          // (the padding is the identity), so only the diagonal tile needs the mask
          const bool ok = i > 0 || (jok && gi < n);
          const double kij = KIN ? (ok ? kraw : 0.0) : ((zero || !ok) ? 0.0 : kraw);
          const double kg = i > 0 ? kij : (ok ? (dg ? fvar : kij) : 0.0);  // σ²·g (the noise is not part of ∂K/∂θ)
          sums[0][0] = fma(v, kg * r2, sums[0][0]);  // (× 1/ℓ once, at the end)
          sums[0][1] = fma(v, kg, sums[0][1]);
          snoise = (ok && dg) ? snoise + v : snoise;
          const double kz = kij * zij;
          colacc += kz;
          if (i > 0) R[i][r] += kz;
        }
      }
    } else {
      // generic kernels: the step's tiles through LDS and a runtime loop (the term interpreter
      // is large; unrolled per tile it would not fit the registers)
#pragma unroll
      for (int i = 0; i <= Q; ++i)
        if (i <= qk) {
          const t4& Zt = (i == 0) ? Zk : Zn[i];
#pragma unroll
          for (int r = 0; r < 4; ++r) sz[i][(4 * r + l4) * 16 + l15] = Zt[r];
        }
      wsync();
      double rowp[Q + 1][4];
#pragma unroll
      for (int i = 0; i <= Q; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) rowp[i][r] = 0.0;
      for (int i = 0; i <= qk; ++i) {
        const int si = (k + i) % (Q + 1);
        const double w = i == 0 ? 1.0 : 2.0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int il = 4 * r + l4, gi = (k + i) * 16 + il;
          const double zij = sz[i][il * 16 + l15];
          const double ai = sal[si][il];
          const double* xi = sx + si * nx + il * D;
          const bool ok = jok && gi < n;
          const bool dg = i == 0 && gi == gj;
          const double v = w * fma(ai, ap, -zij);
          double kij = 0.0;
          if (ok) {
            double dk[NT][3];
            if (fast) {
              double d1[3];
              stationary_grad(fkind, sqdist_scaled(xi + fd0, xj + fd0, fdn), fvar, finv_ell, d1);
              dk[0][0] = d1[0]; dk[0][1] = d1[1]; dk[0][2] = d1[2];
              kij = fvar * d1[1];
            } else {
              kij = eval_k_grad<NT>(spec, sth, xi, xj, dk);
            }
#pragma unroll
            for (int q = 0; q < NT; ++q) {
              sums[q][0] = fma(v, dk[q][0], sums[q][0]);
              sums[q][1] = fma(v, dk[q][1], sums[q][1]);
              sums[q][2] = fma(v, dk[q][2], sums[q][2]);
            }
          }
          if (dg) kij += noise;
          snoise = (ok && dg) ? snoise + v : snoise;
          const double kz = ok ? kij * zij : 0.0;
          colacc += kz;
          // (runtime i: the row partials go to a statically indexed slot)
#pragma unroll
          for (int q = 1; q <= Q; ++q) rowp[q][r] = (q == i) ? kz : rowp[q][r];
        }
      }
#pragma unroll
      for (int i = 1; i <= Q; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) R[i][r] += rowp[i][r];
    }
    QP(5);
    // band check: block k's lower-band column sums; block k+Q is complete (its last upper-band
    // tile was (k+Q, k)): its row sums (R[Q], reduced over the row's 16 lanes) + column sums
    colacc = sum4(colacc);
    if (l4 == 0) scs[cs][l15] = colacc;
    // Rm: block m's upper-band row partials (unreduced over the 16 lanes of a row): through the
    // scratch as a 16x16 tile, each of lanes 0..15 sums one row
    auto finish = [&](int m, const t4& Rm) {
      const int sm = m % (Q + 1);
      wsync();
#pragma unroll
      for (int r = 0; r < 4; ++r) sc[(4 * r + l4) * kSC + l15] = Rm[r];
      wsync();
      if (lane < 16) {
        double rs = 0.0;
#pragma unroll
        for (int c = 0; c < 16; ++c) rs += sc[lane * kSC + c];
        const int g = m * 16 + lane;
        const double tot = scs[sm][lane] + rs;
        if (g < n) resmax = (tot == tot) ? fmax(resmax, fabs(tot - 1.0)) : INFINITY;
        scs[sm][lane] = 0.0;
      }
    };
    if (k + Q < nb) finish(k + Q, R[Q]);
    if (k == 0) {
#pragma unroll
      for (int m = Q - 1; m >= 0; --m)
        if (m < nb) finish(m, R[m]);
    }
    QP(7);
    // this step's inputs for the next one have landed; this step's outputs go out after the
    // wait (α_k, diag(Z_kk) on K's diagonal for band_train_pred_kernel)
    vm_drain();
    wsync();
    QP(8);
    if (l4 == 0) alpha[k16 + l15] = ap;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (4 * r + l4 == l15) Kd[(long long)(k16 + l15) * ld + k16 + l15] = Zk[r];
    // move the window up one block: S'_{11} = Z_kk, S'_{i+1,1} = Z_{k+i,k}, S'_{i+1,j+1} = S_ij
#pragma unroll
    for (int i = Q; i >= 2; --i) {
#pragma unroll
      for (int j = i; j >= 2; --j) S[wid(i - 1, j - 1)] = S[wid(i - 2, j - 2)];
      S[wid(i - 1, 0)] = Zn[i - 1];
    }
    S[wid(0, 0)] = Zk;
#pragma unroll
    for (int i = Q; i >= 1; --i) {
      if constexpr (!LP) al[i] = al[i - 1];
      R[i] = R[i - 1];
    }
    R[1] = tzero();
    QP(6);
  }
  Q_END(1);
  // band check result and the gradient partials (one [16] row per problem, as band_bwd1_kernel)
  {
    double rm = (resmax == resmax) ? resmax : INFINITY;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) rm = fmax(rm, __shfl_xor(rm, o, 64));
    if (lane == 0) a.results[(long long)b * kResStride + kResBandCheck] = rm;
  }
  double vals[GPX_MAX_TERMS * 3 + 1];
#pragma unroll
  for (int t = 0; t < GPX_MAX_TERMS; ++t)
#pragma unroll
    for (int q = 0; q < 3; ++q) vals[t * 3 + q] = t < NT ? wsum64(sums[t][q]) : 0.0;
  if (SE1) {
    vals[0] *= finv_ell;  // Σ v K r² -> Σ v ∂K/∂ℓ
    vals[1] /= fvar;      // Σ v σ² g -> Σ v ∂K/∂σ²
  }
  vals[GPX_MAX_TERMS * 3] = wsum64(snoise);
  if (lane == 0) {
#pragma unroll
    for (int v = 0; v < GPX_MAX_TERMS * 3 + 1; ++v) sred[v] = vals[v];
  }
  wsync();
  if (lane < GPX_THETA_STRIDE) {
    double* out = a.partial + (long long)b * a.sPartial;
    double s = 0.0;
    int slot = -1;
    const DevSpec* gs = a.specs + b;  // (runtime term index: read from global, not the register copy)
    if (lane == gs->n_params) {
      slot = GPX_MAX_TERMS * 3;
    } else {
      for (int t = 0; t < gs->n_terms; ++t) {
        const int o = gs->terms[t].param_offset, kind = gs->terms[t].kind;
        const int np = (kind == GPX_RQ || kind == GPX_PERIODIC_SE) ? 3 : (kind == GPX_LINEAR ? 1 : 2);
        if (lane >= o && lane < o + np) slot = t * 3 + (lane - o);
      }
    }
    if (slot >= 0) s = sred[slot];
    out[lane] = s;
  }
  wave_trace_put(a, wt0, 16 + Q);
}

template <int Q, int NT, bool SE1, bool KIN>
__global__ __launch_bounds__(64, ((Q <= GPX_B16_BWD_2W_QMAX && SE1) || Bwd16<Q, NT, SE1, KIN>::LP) ? 2 : 1)
void band16_bwd_kernel(BandFusedArgs a) {
  extern __shared__ double sx[];
  __shared__ __attribute__((aligned(16))) double lds[Bwd16<Q, NT, SE1, KIN>::size];
  bwd_sweep<Q, NT, SE1, KIN>(a, lds, sx);
}

// Both sweeps of a problem in one wavefront (SE1 classes): one launch per width class, and each
// problem's backward sweep starts when its own forward sweep ends instead of when the launch's
// last one does; the two sweeps share one LDS block.
template <int Q, bool KIN_F, bool KIN_B>
__global__ __launch_bounds__(64, (Q <= GPX_B16_BWD_2W_QMAX) ? 2 : 1) void band16_fused_kernel(BandFusedArgs a) {
  constexpr int nf = Fwd16<Q, KIN_F>::size, nbk = Bwd16<Q, 1, true, KIN_B>::size;
  __shared__ __attribute__((aligned(16))) double lds[nf > nbk ? nf : nbk];
  fwd_sweep<Q, KIN_F>(a, lds);
  // the factor tiles, z and L_ii this wavefront stored are read back by it: its stores are
  // complete and visible to its own loads
  vm_drain();
  __threadfence();
  wsync();
  bwd_sweep<Q, 1, true, KIN_B>(a, lds, nullptr);
}

// ---------------------------------------------------------------------------------------
// K's band for the band16 sweeps: the 16x16 tiles (m, m − d), d = 0..Q, of every 16-row block m
// (the diagonal tile whole), lane (r, c4) of a wavefront computing row r, columns 4·c4 .. 4·c4 + 3
// of a tile — the same values, by the same operations, as build_kernel (inputs scaled by 1/ℓ
// with one division each for single-term stationary kernels, σn² on the diagonal, the identity in
// the padding), written to the same band-storage positions. Each wavefront computes kB16Tiles
// consecutive tiles (one tile per wavefront made a call of ~1000 problems ~1M tiny wavefronts:
// the dispatch, not the exp work, set the kernel's time, 4-9 ms per call in the round-4 wave
// trace, and the sweeps of the call waited for it).
// ---------------------------------------------------------------------------------------
constexpr int kB16Tiles = 16;
__global__ __launch_bounds__(256) void band16_build_kernel(BuildArgs a, int Q) {
  const int b = a.active[blockIdx.y];
  const int nb = a.rows >> 4, ntiles = nb * (Q + 1);
  const int lane = threadIdx.x & 63;
  const int t0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * kB16Tiles;
  if (t0 >= ntiles) return;
  const int n = a.nvalid[b], D = a.D;
  const double* X = a.X + (long long)b * a.sX;
  const double* th = a.theta + (long long)b * GPX_THETA_STRIDE;
  const DevSpec& spec = a.specs[b];
  const int k0 = spec.terms[0].kind;
  const bool fast = spec.n_terms == 1 && k0 >= GPX_SE && k0 <= GPX_EXPONENTIAL;
  const double noise = th[spec.n_params];
  const gpx_term& tm = spec.terms[0];
  const double ell = th[tm.param_offset], var = th[tm.param_offset + 1];
  const int d0 = tm.dim_start, dn = tm.dim_count;
  for (int t = t0; t < min(t0 + kB16Tiles, ntiles); ++t) {
    const int m = t / (Q + 1), d = t - m * (Q + 1);
    if (m < d) continue;
    const int gi = m * 16 + (lane >> 2), gj0 = (m - d) * 16 + (lane & 3) * 4;
    double* out = a.out + (long long)b * a.sOut + (long long)gi * a.ldo + gj0;
    double v[4];
    if (fast) {
      const double* xi = X + (long long)min(gi, n - 1) * D + d0;  // (padding rows: not read)
      const double xi0 = gi < n ? xi[0] / ell : 0.0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int gj = gj0 + q;
        if (gi < n && gj < n) {
          const double* xj = X + (long long)gj * D + d0;
          // (x/ℓ by one division per value, as build_kernel stages them)
          const double r2 = dn == 1 ? sqdist1(xi0, xj[0] / ell) : sqdist_gpflow(xi, xj, dn, ell);
          switch (k0) {
            case GPX_SE: v[q] = stationary_value<GPX_SE>(r2, var); break;
            case GPX_MATERN12: v[q] = stationary_value<GPX_MATERN12>(r2, var); break;
            case GPX_MATERN32: v[q] = stationary_value<GPX_MATERN32>(r2, var); break;
            case GPX_MATERN52: v[q] = stationary_value<GPX_MATERN52>(r2, var); break;
            default: v[q] = stationary_value<GPX_EXPONENTIAL>(r2, var); break;
          }
          if (gi == gj) v[q] += noise;
        } else {
          v[q] = gi == gj ? 1.0 : 0.0;
        }
      }
    } else {
      const DevSpec sp = spec;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int gj = gj0 + q;
        if (gi < n && gj < n) {
          v[q] = eval_k(sp, th, X + (long long)gi * D, X + (long long)gj * D);
          if (gi == gj) v[q] += noise;
        } else {
          v[q] = gi == gj ? 1.0 : 0.0;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) out[q] = v[q];
  }
}

// a deferred slow part's results, gathered for one download: rows act[i] of the batch's result
// block and info into compact [n][stride] / [n] buffers
__global__ __launch_bounds__(64) void slow_gather_kernel(const int* __restrict__ act, int n,
                                                          const double* __restrict__ res, int stride,
                                                          double* __restrict__ out, const int* __restrict__ info,
                                                          int* __restrict__ info_out) {
  const int t = blockIdx.x * 64 + threadIdx.x;
  if (t >= n * stride) return;
  const int i = t / stride, c = t - i * stride, b = act[i];
  out[t] = res[(long long)b * stride + c];
  if (c == 0) info_out[i] = info[b];
  __threadfence_system();  // (out / info_out may be coherent host memory: GPX_SLOW_DIRECT)
}

__global__ __launch_bounds__(64) void slow_inputs_kernel(const int* __restrict__ act, int n, int* __restrict__ act_out,
                                                         const double* __restrict__ theta, double* __restrict__ theta_out,
                                                         const int* __restrict__ bandp, int* __restrict__ bandp_out,
                                                         int* __restrict__ info_out, int B, int r0, int r1) {
  const int t = blockIdx.x * 64 + threadIdx.x;
  if (t < B * GPX_THETA_STRIDE) theta_out[t] = theta[t];
  if (t < n) act_out[t] = (t >= r0 && t < r1) ? act[r0 + r1 - 1 - t] : act[t];
  if (t < B) {
    bandp_out[t] = bandp[t];
    info_out[t] = 0;
  }
}

void launch_slow_inputs(const int* act, int n, int* act_out, const double* theta, double* theta_out, const int* bandp,
                        int* bandp_out, int* info_out, int B, hipStream_t s, int r0, int r1) {
  const int m = std::max(B * GPX_THETA_STRIDE, n);
  hipLaunchKernelGGL(slow_inputs_kernel, dim3((m + 63) / 64), dim3(64), 0, s, act, n, act_out, theta, theta_out, bandp,
                     bandp_out, info_out, B, r0, r1);
}

void launch_slow_gather(const int* act, int n, const double* res, int stride, double* out, const int* info,
                        int* info_out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(slow_gather_kernel, dim3((n * stride + 63) / 64), dim3(64), 0, s, act, n, res, stride, out,
                     info, info_out);
}

// diagnostic (GPX_SLOW_DELAY_US): a one-wave kernel that spins for us microseconds on the device's
// 100 MHz clock — lengthens a deferred part by a known amount to measure how the line depends on it
__global__ __launch_bounds__(64) void spin_us_kernel(int us) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < 100ull * (unsigned long long)us) {
  }
}
void launch_spin_us(int us, hipStream_t s) { hipLaunchKernelGGL(spin_us_kernel, dim3(1), dim3(64), 0, s, us); }

// a one-wave kernel that appends a stream-order marker {t, t, kind} to the wave trace: where a
// call's device work stands when the stream reaches it (kinds >= 32, gpx_api.hip trace_mark)
__global__ __launch_bounds__(64) void wave_marker_kernel(BandFusedArgs a, int kind) {
  wave_trace_put(a, __builtin_amdgcn_s_memrealtime(), kind);
}

void launch_wave_marker(unsigned long long* wt, unsigned int* wn, unsigned int cap, int kind, hipStream_t s) {
  BandFusedArgs a{};
  a.wtrace = wt;
  a.wtrace_n = wn;
  a.wtrace_cap = cap;
  hipLaunchKernelGGL(wave_marker_kernel, dim3(1), dim3(64), 0, s, a, kind);
}

void launch_band16_build(const BuildArgs& a, int Q, int n_active, hipStream_t s) {
  const int tiles = (a.rows >> 4) * (Q + 1), per_wg = 4 * kB16Tiles;
  hipLaunchKernelGGL(band16_build_kernel, dim3((tiles + per_wg - 1) / per_wg, n_active), dim3(256), 0, s, a, Q);
}

// The wide classes (Q = 4, 5: one wavefront per SIMD either way) of a call as ONE launch, each
// wavefront running both sweeps of its problem at its own width (bandp): a single launch instead
// of a build / forward / backward chain per class, so a call's few wide problems cost one wave
// latency instead of one per class. SE1 problems only.
template <int Q, bool KF, bool KB>
__device__ __forceinline__ void fused_sweeps(const BandFusedArgs& a, double* __restrict__ lds) {
  fwd_sweep<Q, KF>(a, lds);
  vm_drain();
  __threadfence();
  wsync();
  bwd_sweep<Q, 1, true, KB>(a, lds, nullptr);
}
template <int Q, bool KF, bool KB>
constexpr int fused_lds() {
  return Fwd16<Q, KF>::size > Bwd16<Q, 1, true, KB>::size ? Fwd16<Q, KF>::size : Bwd16<Q, 1, true, KB>::size;
}
// WQ = 8 (K inline in both sweeps only): the Q = 6..8 classes in the same launch
template <bool KF, bool KB, int WQ>
__global__ __launch_bounds__(64, 1) void band16_wide_kernel(BandFusedArgs a) {
  constexpr int n4 = fused_lds<4, KF, KB>(), n5 = fused_lds<5, KF, KB>();
  constexpr int n8 = WQ > 5 ? fused_lds<8, KF, KB>() : 0;
  constexpr int n45 = n4 > n5 ? n4 : n5;
  __shared__ __attribute__((aligned(16))) double lds[n45 > n8 ? n45 : n8];
  const int Q = a.bandp[a.active[blockIdx.x]];
  if constexpr (WQ > 5) {
    if (Q == 8) return fused_sweeps<8, KF, KB>(a, lds);
    if (Q == 7) return fused_sweeps<7, KF, KB>(a, lds);
    if (Q == 6) return fused_sweeps<6, KF, KB>(a, lds);
  }
  if (Q == 5)
    fused_sweeps<5, KF, KB>(a, lds);
  else
    fused_sweeps<4, KF, KB>(a, lds);
}

void launch_band16_wide(const BandFusedArgs& a, int kin, int n_active, hipStream_t s, hipEvent_t* ev, int wq) {
  auto k = (kin & 1) ? ((kin & 2) ? (wq > 5 ? band16_wide_kernel<true, true, 8> : band16_wide_kernel<true, true, 5>)
                                  : band16_wide_kernel<true, false, 5>)
                     : ((kin & 2) ? band16_wide_kernel<false, true, 5> : band16_wide_kernel<false, false, 5>);
  if (ev) {
    hipExtLaunchKernelGGL(k, dim3(n_active), dim3(64), 0, s, ev[0], ev[1], 0, a);
    (void)hipEventRecord(ev[2], s);
    (void)hipEventRecord(ev[3], s);
    return;
  }
  hipLaunchKernelGGL(k, dim3(n_active), dim3(64), 0, s, a);
}

template <int Q>
static void launch16_q(const BandFusedArgs& a, int max_terms, bool se1, int kin, int n_active, hipStream_t s,
                       hipEvent_t* ev) {
  kin = se1 ? kin : 0;
  // GPX_B16_FUSED=1: the SE1 classes' sweeps as one fused launch (fwd then bwd per wavefront)
  static const bool fused = [] {
    const char* e = getenv("GPX_B16_FUSED");
    return e && atoi(e) != 0;
  }();
  if (se1 && fused) {
    auto fk = (kin & 1) ? ((kin & 2) ? band16_fused_kernel<Q, true, true> : band16_fused_kernel<Q, true, false>)
                        : ((kin & 2) ? band16_fused_kernel<Q, false, true> : band16_fused_kernel<Q, false, false>);
    if (ev) {
      hipExtLaunchKernelGGL(fk, dim3(n_active), dim3(64), 0, s, ev[0], ev[1], 0, a);
      (void)hipEventRecord(ev[2], s);  // (the backward sweeps' share is inside ev[0] .. ev[1])
      (void)hipEventRecord(ev[3], s);
      return;
    }
    hipLaunchKernelGGL(fk, dim3(n_active), dim3(64), 0, s, a);
    return;
  }
  auto fwd = (kin & 1) ? band16_fwd_kernel<Q, true> : band16_fwd_kernel<Q, false>;
  auto bwd = se1 ? ((kin & 2) ? band16_bwd_kernel<Q, 1, true, true> : band16_bwd_kernel<Q, 1, true, false>)
                 : max_terms <= 1 ? band16_bwd_kernel<Q, 1, false, false>
                                  : max_terms == 2 ? band16_bwd_kernel<Q, 2, false, false>
                                                   : band16_bwd_kernel<Q, GPX_MAX_TERMS, false, false>;
  const size_t xs = se1 ? 0 : (size_t)(Q + 1) * 16 * a.D * sizeof(double);
  if (ev) {
    hipExtLaunchKernelGGL(fwd, dim3(n_active), dim3(64), 0, s, ev[0], ev[1], 0, a);
    hipExtLaunchKernelGGL(bwd, dim3(n_active), dim3(64), xs, s, ev[2], ev[3], 0, a);
    return;
  }
  hipLaunchKernelGGL(fwd, dim3(n_active), dim3(64), 0, s, a);
  hipLaunchKernelGGL(bwd, dim3(n_active), dim3(64), xs, s, a);
}

// Q = 6..8 (the routing sends only SE1 problems with both sweeps computing K inline): one
// wavefront per SIMD whose window tiles fill VGPRs and AGPRs — 28 / 36 / 45 forward window
// tiles; Q = 6 fits (241 + 256 registers, no scratch), Q = 7 and 8 spill (240-920 B per lane),
// still one launch pair per class instead of the 64-row p = 2 sweeps' 73 KiB workgroups
template <int Q>
static void launch16_wide_q(const BandFusedArgs& a, int n_active, hipStream_t s, hipEvent_t* ev) {
  auto fwd = band16_fwd_kernel<Q, true>;
  auto bwd = band16_bwd_kernel<Q, 1, true, true>;
  if (ev) {
    hipExtLaunchKernelGGL(fwd, dim3(n_active), dim3(64), 0, s, ev[0], ev[1], 0, a);
    hipExtLaunchKernelGGL(bwd, dim3(n_active), dim3(64), 0, s, ev[2], ev[3], 0, a);
    return;
  }
  hipLaunchKernelGGL(fwd, dim3(n_active), dim3(64), 0, s, a);
  hipLaunchKernelGGL(bwd, dim3(n_active), dim3(64), 0, s, a);
}

void launch_band16(const BandFusedArgs& a, int Q, int max_terms, bool se1, int kin, int n_active, hipStream_t s,
                   hipEvent_t* ev) {
  switch (Q) {
    case 1: launch16_q<1>(a, max_terms, se1, kin, n_active, s, ev); break;
    case 2: launch16_q<2>(a, max_terms, se1, kin, n_active, s, ev); break;
    case 3: launch16_q<3>(a, max_terms, se1, kin, n_active, s, ev); break;
    case 4: launch16_q<4>(a, max_terms, se1, kin, n_active, s, ev); break;
    case 5: launch16_q<5>(a, max_terms, se1, kin, n_active, s, ev); break;
    case 6: launch16_wide_q<6>(a, n_active, s, ev); break;
    case 7: launch16_wide_q<7>(a, n_active, s, ev); break;
    default: launch16_wide_q<8>(a, n_active, s, ev); break;
  }
}

}  // namespace gpx

#ifdef GPX_BAND_PHASES
// out[32] <- g_b16_phase (fwd, bwd: phases 0..11, [15] = waves); reset != 0 zeroes it afterwards.
// Diagnostic build only (not in include/gpx.h).
extern "C" int gpx_debug_band16_phases(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(gpx::g_b16_phase), sizeof(gpx::g_b16_phase)) != hipSuccess) return -1;
  if (reset) {
    static const unsigned long long zero[2][16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(gpx::g_b16_phase), zero, sizeof(zero)) != hipSuccess) return -1;
  }
  return 0;
}
#endif
