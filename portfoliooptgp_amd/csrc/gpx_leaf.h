// gpx_leaf.h — the 64x64 Cholesky-and-inverse leaf on LDS, shared by leaf_kernel
// (gpx_kernels.hip) and the fused banded kernels (gpx_band.hip).
#pragma once
#include <hip/hip_runtime.h>
#include "gpx_internal.h"

namespace gpx {

// sub-phase timing of the leaf (diagnostic build of gpx_band.hip only, see GPX_BAND_PHASES)
#ifdef GPX_BAND_PHASES
__device__ unsigned long long g_leaf_phase[8];
#define LEAF_PH_BEGIN unsigned long long lph_t = __builtin_amdgcn_s_memtime(), lph_acc[4] = {};
#define LEAF_PH(i)                                                \
  do {                                                            \
    const unsigned long long lph_n = __builtin_amdgcn_s_memtime(); \
    lph_acc[i] += lph_n - lph_t;                                  \
    lph_t = lph_n;                                                \
  } while (0)
#define LEAF_PH_END                                                                          \
  do {                                                                                       \
    if (threadIdx.x == 0) {                                                                  \
      for (int lph_i = 0; lph_i < 4; ++lph_i) atomicAdd(&g_leaf_phase[lph_i], lph_acc[lph_i]); \
      atomicAdd(&g_leaf_phase[7], 1ull);                                                     \
    }                                                                                        \
  } while (0)
#else
#define LEAF_PH_BEGIN
#define LEAF_PH(i) \
  do {             \
  } while (0)
#define LEAF_PH_END \
  do {              \
  } while (0)
#endif

__device__ __forceinline__ double readlane_d(double v, int l) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)(u & 0xffffffffu), l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// v of lane k of this lane's 16-lane row (DPP row_newbcast: one v_mov_b64_dpp, no SGPR round
// trip as readlane_d needs). k must fold to a constant (unrolled loops); rows of 16 lanes that
// hold the same 16 values (lane & 15) all see lane k's.
__device__ __forceinline__ double bc16(double v, int k) {
// mov_dpp (no "old" operand: every lane is written, so no zeroing move per broadcast)
#define GPX_BC16(K) \
  case K:           \
    return __builtin_amdgcn_mov_dpp(v, 0x150 + K, 0xf, 0xf, true);
  switch (k) {
    GPX_BC16(0) GPX_BC16(1) GPX_BC16(2) GPX_BC16(3) GPX_BC16(4) GPX_BC16(5) GPX_BC16(6) GPX_BC16(7)
    GPX_BC16(8) GPX_BC16(9) GPX_BC16(10) GPX_BC16(11) GPX_BC16(12) GPX_BC16(13) GPX_BC16(14)
    default: return __builtin_amdgcn_mov_dpp(v, 0x150 + 15, 0xf, 0xf, true);
  }
#undef GPX_BC16
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
// pre_inverse() is called by every thread between the factorisation and the W = L⁻¹ block
// rows: a caller issues its next global loads there, when the diagonal factor's registers
// are free again.
struct LeafNoHook {
  __device__ void operator()() const {}
};
// kLog = false: ldiag gets L_ii itself (the banded sweeps take the logs once per problem, in
// their backward kernels, instead of on every step's critical path)
// rot: the hardware wave that plays wave 0 (the serial diagonal chain) is (rot & 3); callers
// with several workgroups per CU pass a per-workgroup rotation so co-resident workgroups'
// diagonal chains tend to sit on different SIMDs
// NB < 4 (the small-problem kernel, gpx_kernels.hip small64_kernel): only the leading NB 16-blocks
// hold data — the rest of the block is the identity padding, whose factor and inverse are the
// identity (the caller puts 1s on sW's diagonal there; sA's diagonal holds them already, so their
// logs come out 0) — and the steps on the padding blocks are skipped. NB = 4 is the full leaf.
template <bool kLog = true, class PreInverse = LeafNoHook, int NB = 4>
__device__ __forceinline__ void leaf64_lds(double* __restrict__ sA, double* __restrict__ sW,
                                           double* __restrict__ ldiag, int* sfail,
                                           PreInverse pre_inverse = PreInverse(), int rot = 0) {
  constexpr int S = kLeafS;
  typedef double d4 __attribute__((ext_vector_type(4)));
  // threadIdx.x through an empty asm: the leaf's LDS addresses are formed per call instead of
  // being hoisted out of a caller's block-step loop (where they would pin registers and spill)
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63, wave = ((tid >> 6) - rot) & 3;
  const int l15 = lane & 15, l4 = lane >> 4;
  LEAF_PH_BEGIN
  // wave 0's 16x16 diagonal step on block jb: L_jj, D_j = L_jj⁻¹ (-> sW), L_ii (-> ldiag / sA)
  auto diag = [&](int jb) {
    const int c0 = jb * 16;
    double r[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) r[k] = sA[(c0 + l15) * S + c0 + k];
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
    // lane l15 holds row l15 of L_jj (r[0..l15]); column l15 of D = L_jj⁻¹ by substitution,
    // right-looking so the 16 steps' FMAs are independent across i
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
    if (lane < 16) {
#pragma unroll
      for (int i = 0; i < 16; ++i) sW[(c0 + i) * S + c0 + lane] = w[i];
      if (kLog)
        sA[(c0 + lane) * S + c0 + lane] = r[lane & 15];   // L_ii, for log det at the end
      else
        ldiag[c0 + lane] = r[lane & 15];
    }
    if (lane == 0 && fail >= 0 && *sfail < 0) *sfail = c0 + fail;
  };
  // A_ik −= L_ij L_kjᵀ on one 16x16 tile (rows ri, columns rk; column block c0 of L)
  auto tile_update = [&](int ri, int rk, int c0) {
    d4 acc;
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = sA[(ri + l4 + 4 * u) * S + rk + l15];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const double av = sA[(ri + l15) * S + c0 + 4 * kk + l4];
      const double bv = sA[(rk + l15) * S + c0 + 4 * kk + l4];
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 1);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) sA[(ri + l4 + 4 * u) * S + rk + l15] = acc[u];
  };
  // Right-looking over the 4 column blocks with look-ahead: wave 0 computes the next diagonal
  // tile's update itself (from the panel tile it just produced) and factors it while waves
  // 1-3 apply the rest of the trailing update, so that update is off the diagonal chain.
  if (wave == 0) diag(0);
  for (int jb = 0; jb < NB; ++jb) {
    const int c0 = jb * 16;
    __syncthreads();
    LEAF_PH(0);
    // panel: L_(ib,jb) = A_(ib,jb) · Dᵀ for ib = jb+1 .. NB−1, one wave per block (wave 0 takes
    // ib = jb + 1, the tile its look-ahead needs)
    const int nblk = NB - 1 - jb;
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
    LEAF_PH(1);
    // trailing update of the lower blocks (ib, kb), jb < kb <= ib: tile 0 = (jb+1, jb+1) by
    // wave 0 with the next diagonal step, the others over waves 1..3
    const int ntr = nblk * (nblk + 1) / 2;
    if (wave == 0) {
      if (jb < NB - 1) {
        tile_update((jb + 1) * 16, (jb + 1) * 16, c0);
        diag(jb + 1);
      }
    } else {
      for (int t = wave; t < ntr; t += 3) {
        int p = 0;
        while ((p + 1) * (p + 2) / 2 <= t) ++p;
        const int q = t - p * (p + 1) / 2;
        tile_update((jb + 1 + p) * 16, (jb + 1 + q) * 16, c0);
      }
    }
    LEAF_PH(2);
  }
  __syncthreads();
  pre_inverse();
  // W = L⁻¹: block rows 1..NB−1, blocks j < i in parallel (wave j); the idle wave 3 takes the
  // logs of L's diagonal (left on sA's diagonal by the diagonal steps)
  if (kLog && NB == 1 && wave == 3) ldiag[lane] = log(sA[lane * S + lane]);
  for (int i = 1; i < NB; ++i) {
    if (kLog && i == NB - 1 && wave == 3) ldiag[lane] = log(sA[lane * S + lane]);
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
        wv = __builtin_amdgcn_mfma_f64_16x16x4f64(av, t[kk], wv, 0, 0, 1);  // T[k'][col]
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) sW[(i * 16 + l4 + 4 * q) * S + j * 16 + l15] = wv[q];
    }
    __syncthreads();
  }
  LEAF_PH(3);
  LEAF_PH_END;
}

}  // namespace gpx
