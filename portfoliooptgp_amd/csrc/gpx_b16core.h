// gpx_b16core.h — the register-tile toolkit of the 16-row banded kernels (gfx950, fp64), shared by
// the one-wavefront band16 sweeps (gpx_band16.hip) and the block-cyclic-reduction path
// (gpx_bcr.hip): 16x16 tiles held as v_mfma_f64_16x16x4_f64 C fragments (lane (l15, l4),
// register r holds element (4r + l4, l15)), the Xᵀ·Y product of two fragments, 16- and 64-lane
// sums, wave-level LDS ordering, and leaf16m, the 16x16 Cholesky-and-inverse on the matrix cores.
#pragma once
#include <hip/hip_runtime.h>
#include "gpx_internal.h"
#include "gpx_leaf.h"

namespace gpx {

namespace {

typedef double t4 __attribute__((ext_vector_type(4)));
constexpr int kSC = 18;  // LDS scratch row stride (doubles): 16-byte aligned rows

__device__ __forceinline__ t4 tzero() { return (t4){0.0, 0.0, 0.0, 0.0}; }

// c += Xᵀ·Y (X, Y: C fragments of 16x16 tiles)
__device__ __forceinline__ void mma(t4& c, const t4& x, const t4& y) {
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) c = __builtin_amdgcn_mfma_f64_16x16x4f64(x[kk], y[kk], c, 0, 0, 0);
}
// c −= Xᵀ·Y (blgp = 1 on an f64 MFMA is its neg modifier on A: −X exactly, no sign-flip VALU op)
__device__ __forceinline__ void mms(t4& c, const t4& x, const t4& y) {
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) c = __builtin_amdgcn_mfma_f64_16x16x4f64(x[kk], y[kk], c, 0, 0, 1);
}

// sums over the 4 lanes l4 = 0..3 of a column (lanes l15 + 16·l4), no LDS round trip: with both
// operands holding v, v_permlane32_swap leaves [A|A] and [B|B] (A, B: the wave's lower and upper
// 32 lanes), whose sum is A + B on every lane; v_permlane16_swap does the same for adjacent
// 16-lane rows. Every lane ends with the same bits (each add is commutative).
__device__ __forceinline__ double swap_add(double v, bool sw32) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
  const auto a = sw32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                      : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = sw32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                      : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const double p = __longlong_as_double(((unsigned long long)b[0] << 32) | a[0]);
  const double q = __longlong_as_double(((unsigned long long)b[1] << 32) | a[1]);
  return p + q;
}
__device__ __forceinline__ double sum4(double v) { return swap_add(swap_add(v, true), false); }
// butterfly over the 16 lanes of a row: DPP quad_perm xor 1, xor 2, row_half_mirror, row_mirror
// (four v_mov_b64_dpp + four adds; every lane ends with the same bits: each add is commutative)
__device__ __forceinline__ double sum16(double v) {
  v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, true);
  v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, true);
  v += __builtin_amdgcn_mov_dpp(v, 0x141, 0xf, 0xf, true);
  v += __builtin_amdgcn_mov_dpp(v, 0x140, 0xf, 0xf, true);
  return v;
}
__device__ __forceinline__ double wsum64(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// LDS ordering point of the single-wave workgroup: a wave's LDS operations execute in issue
// order, so only the compiler has to be kept from moving them across (no barrier, no wait)
__device__ __forceinline__ void wsync() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); }
// wait for this wave's global -> LDS copies (and its other vector memory operations)
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// wait for this wave's LDS operations
__device__ __forceinline__ void lds_drain() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// async copy of a 16x16 tile (row-major, leading dimension ld) into a 16x16 LDS tile: two
// 16-byte global_load_lds per lane (8 rows each; LDS destination = base + lane·16 B), the 16-byte
// column pairs of row r XOR-swizzled by (r >> 1) & 7 so that transposed fragment reads (lane
// (l15, l4) reading row l15: sixteen rows 128 B apart, i.e. the same LDS banks) spread over all
// banks; element (r, c) sits at swz16(r, c)
__device__ __forceinline__ int swz16(int r, int c) { return r * 16 + ((((c >> 1) ^ (r >> 1)) & 7) << 1) + (c & 1); }
__device__ __forceinline__ void tile_glds_swz(const double* __restrict__ g, long long ld, double* __restrict__ s,
                                              int lane) {
  const int row = lane >> 3, q = lane & 7;
  __builtin_amdgcn_global_load_lds(g + (long long)row * ld + 2 * (q ^ ((row >> 1) & 7)), s, 16, 0, 0);
  __builtin_amdgcn_global_load_lds(g + (long long)(row + 8) * ld + 2 * (q ^ (((row + 8) >> 1) & 7)), s + 128, 16, 0, 0);
}

// band16's private factor layout (forward sweep -> backward sweep; nothing else reads it): per
// block step k, Q + 1 tiles of 256 doubles at L + (k·(Q+1) + i)·256 (i = 0: W_kk, i >= 1: P_iᵀ),
// each stored as its C fragment with a lane's 4 doubles contiguous: a tile is one coalesced 2 KiB
// store and one coalesced 2 KiB load (two 16-byte accesses per lane), straight into registers
__device__ __forceinline__ void frag_store(const t4& t, double* __restrict__ g, int lane) {
  *reinterpret_cast<t4*>(g + 4 * lane) = t;
}
// transpose of a tile through the scratch
__device__ __forceinline__ t4 tile_transpose(const t4& t, double* __restrict__ sc, int l15, int l4) {
  wsync();
#pragma unroll
  for (int r = 0; r < 4; ++r) sc[(4 * r + l4) * kSC + l15] = t[r];
  wsync();
  t4 o;
#pragma unroll
  for (int r = 0; r < 4; ++r) o[r] = sc[l15 * kSC + 4 * r + l4];
  return o;
}

// 16x16 Cholesky-and-inverse on the matrix cores: four 4-column steps, each a 4x4 diagonal
// factorisation (every lane, uniform values from LDS), the 16x4 panel by the diagonal block's
// inverse, ONE v_mfma_f64_16x16x4_f64 for the rank-4 trailing update of the tile and one for the
// rank-4 update of L⁻¹ (built alongside, right-looking: W := Li·W_jb on block row jb, then
// W_below −= L_below,jb · W_jb). A (symmetric) is read through its column blocks: fragment
// register c at lane (l15, l4) is A[l15][4c + l4]. Returns V = fragment of (L⁻¹)ᵀ (through one LDS
// transpose), Wr = fragment of L⁻¹ (rows: register r holds rows 4r + l4), lii = L[l15][l15] and
// fail = the first pivot that is not > 0 (or −1).
__device__ __forceinline__ void leaf16m(t4 A, t4& V, t4& Wr, double& lii, int& fail, double* __restrict__ sc,
                                        int l15, int l4) {
#pragma unroll
  for (int r = 0; r < 4; ++r) Wr[r] = (4 * r + l4 == l15) ? 1.0 : 0.0;
  fail = -1;
  lii = 0.0;
  double* sm = sc;       // [16][4] column block of A
  double* sw = sc + 64;  // [16][4] block row of W, transposed: sw[j][b] = W[4jb + b][j]
#pragma unroll
  for (int jb = 0; jb < 4; ++jb) {
    wsync();
    sm[l15 * 4 + l4] = A[jb];
    sw[l15 * 4 + l4] = Wr[jb];
    wsync();
    double m[4], wv[4], d[4][4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      m[c] = sm[l15 * 4 + c];
      wv[c] = sw[l15 * 4 + c];
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c <= a; ++c) d[a][c] = sm[(4 * jb + a) * 4 + c];  // (same address on every lane)
    // 4x4 Cholesky L_d and its inverse Li (uniform)
    double l[4][4], iv[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
#pragma unroll
      for (int c = 0; c < a; ++c) {
        double t = d[a][c];
#pragma unroll
        for (int e = 0; e < c; ++e) t = fma(-l[a][e], l[c][e], t);
        l[a][c] = t * iv[c];
      }
      double pv = d[a][a];
#pragma unroll
      for (int e = 0; e < a; ++e) pv = fma(-l[a][e], l[a][e], pv);
      if (!(pv > 0.0) && fail < 0) fail = 4 * jb + a;
      iv[a] = rsqrt_nr(pv);
      l[a][a] = pv * iv[a];
    }
    if ((l15 >> 2) == jb) {
      const int a = l15 & 3;
      lii = a == 0 ? l[0][0] : a == 1 ? l[1][1] : a == 2 ? l[2][2] : l[3][3];
    }
    // panel column block jb of L: rows below the block m·Li_dᵀ, rows of the block L_d, above 0.
    // lrow = row l4 of Li = L_d⁻¹ (0 for c > l4), by substitution along the row (Li·L_d = I:
    // Li[a][c] = −iv[c] Σ_{e=c+1}^{a} Li[a][e] l[e][c]), each lane its own row: no 4x4 inverse
    double lrow[4];
    lrow[3] = l4 == 3 ? iv[3] : 0.0;
#pragma unroll
    for (int c = 2; c >= 0; --c) {
      double t = lrow[c + 1] * l[c + 1][c];
#pragma unroll
      for (int e = c + 2; e < 4; ++e) t = fma(lrow[e], l[e][c], t);
      lrow[c] = l4 == c ? iv[c] : (l4 > c ? -iv[c] * t : 0.0);
    }
    double xb = 0.0;
#pragma unroll
    for (int c = 0; c < 4; ++c) xb = fma(m[c], lrow[c], xb);
    // rows below the block only: the update of the block's own rows and columns (L_d L_dᵀ) is
    // never read again, so the block rows of the panel are left at 0
    xb = l15 - 4 * jb >= 4 ? xb : 0.0;
    A = __builtin_amdgcn_mfma_f64_16x16x4f64(xb, xb, A, 0, 0, 1);  // trailing update (rank 4)
    // block row jb of L⁻¹: Li · (its current rows), then the rows below
    double wn = 0.0;
#pragma unroll
    for (int c = 0; c < 4; ++c) wn = fma(lrow[c], wv[c], wn);
    Wr[jb] = wn;
    // (at jb = 3 no row lies below the block: xb is all zeros, the update adds exact zeros to
    // entries that are finite or +0, so it is left out — the same bits, one MFMA less per leaf)
    if (jb < 3) Wr = __builtin_amdgcn_mfma_f64_16x16x4f64(xb, wn, Wr, 0, 0, 1);
  }
  // V = fragment of (L⁻¹)ᵀ
  wsync();
#pragma unroll
  for (int r = 0; r < 4; ++r) sc[(4 * r + l4) * kSC + l15] = Wr[r];
  wsync();
#pragma unroll
  for (int r = 0; r < 4; ++r) V[r] = sc[l15 * kSC + 4 * r + l4];
}

}  // namespace

}  // namespace gpx
