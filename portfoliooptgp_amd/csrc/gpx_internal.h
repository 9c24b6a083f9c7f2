// gpx_internal.h — launch arguments and launcher entry points shared by gpx_api.hip and
// gpx_kernels.hip. Not part of the public ABI (include/gpx.h is).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "gpx_kfun.h"

namespace gpx {

constexpr int kLeaf = 64;      // diagonal-block size of the recursive Cholesky-and-inverse
constexpr int kResStride = 32; // results row: [0]=lml, [1..16]=grad, [17]=yᵀK⁻¹y, [18]=Σlog L_ii,
                               // [19]=banded path check: max_j |Σ_i K_ji Z_ij − 1| (Z = K⁻¹ on the band)
constexpr int kResBandCheck = 19;

// ---- K / cross-covariance build -------------------------------------------------------
struct BuildArgs {
  const int* active;
  const DevSpec* specs;
  const double* theta;     // [B][16] device
  const int* nvalid;       // [B] valid rows (training points)
  const double* X; long long sX;   // row points: X + b*sX, [rows][D]
  const double* X2; long long sX2; // column points (cross mode)
  int D;
  int m2;                  // valid columns in cross mode
  double* out; long long sOut; int ldo;
  int rows, cols;          // padded, multiples of 64
  int symmetric;           // 1: lower tiles of K(X,X)+σn²I with identity padding
  int rows_valid;          // >0: valid rows for every problem (K(X*,X*)), else nvalid[b]
  int band1;               // symmetric only: >0 builds just the 64-blocks (k, k−d), d < band1
};

// ---- leaf: 64x64 Cholesky + triangular inverse in LDS --------------------------------
struct LeafArgs {
  const int* active;
  const double* K; double* W; long long sMat; int ld; int off;
  double* ldiag; long long sVec;   // log L_ii, [B][Np]
  int* info;                       // [B], first failing pivot (1-based), 0 = ok
};

// ---- batched fp64 MFMA GEMM -----------------------------------------------------------
enum : int { TRI_KMAX_I = 1, TRI_KMAX_J = 2, TRI_KMIN_J = 4, TRI_KMIN_I = 8 };
// EPI_CONTRACT1: EPI_CONTRACT specialised for single-term kernels (every active spec has
// n_terms == 1): a quarter of the derivative registers, no spills in the epilogue.
enum : int { EPI_STORE = 0, EPI_CONTRACT = 1, EPI_COLSUMSQ = 2, EPI_CONTRACT1 = 3, EPI_CONTRACT2 = 4 };
// tile enumeration for rectangular launches (see gemm_kernel)
enum : int { ORDER_ROW_ASC = 0, ORDER_COL_DESC = 1, ORDER_ROW_DESC = 2, ORDER_COL_ASC = 3 };

struct GemmArgs {
  const int* active;
  const double* A; long long sA; int lda;   // opA(i,k) = A[i*lda+k] (N) or A[k*lda+i] (T)
  const double* Bm; long long sB; int ldb;  // opB(k,j) = B[k*ldb+j] (N) or B[j*ldb+k] (T)
  double* C; long long sC; int ldc;
  int M, N, K;
  int tri;            // TRI_* flags restricting the k range per tile
  int lower_only;     // only tiles with ti >= tj
  int order;          // ORDER_* tile enumeration (rectangular launches)
  int small_tiles;    // pick the tile size by workgroup count (single-problem launches: SVGP)
  int n_active;       // set by the launcher (XCD-aware problem placement)
  double alpha, beta;
  // EPI_CONTRACT
  const double* vec; long long sVec;        // α vectors [B][Np]
  const double* X; long long sX; int D;
  const DevSpec* specs; const double* theta; const int* nvalid;
  double* partial; long long sPartial;      // [B][ntiles][16] / [B][rowtiles][ldc]
  // host-side only: when set, the launch is timestamped at the kernel's actual start and end
  // (hipExtLaunchKernel), excluding any wait for resources held by other streams
  hipEvent_t ev_start, ev_stop;
};

// ---- vectors --------------------------------------------------------------------------
struct TrmvArgs {
  const int* active;
  const double* Wm; long long sW; int ld;
  const double* x; long long sx;   // input vector
  const int* nvalid;               // mask input x beyond n (for y); may be null
  double* y; long long sy;         // output
  int rows, cols;                  // operator dims
  int lower;                       // 1: triangular (skip known zeros)
  int n_active;                    // set by the launcher (1-D grid: blocks x problems)
};

// predict_f / predict_y at the training inputs from the cached factor, O(N²):
//   mean_j = y_j − σn² α_j,  var_j = σn² − σn⁴ [K_y⁻¹]_jj  (+σn² for predict_y),
// [K_y⁻¹]_jj = Σ_i W_ij² — algebraically GPflow's Kxsᵀα and k_jj − colsum((L⁻¹Kxs)²) with
// Kxs = K_y − σn²I.
struct TrainPredArgs {
  const int* active;
  const double* W; long long sW; int ld;
  const double* alpha; long long sVec;
  const double* Y; long long sY;
  const int* nvalid;
  const DevSpec* specs; const double* theta;
  int add_noise;
  double* mean; double* var; long long sOut;
  const int* orow;  // output row of slot b (null: row b) — gpx_batch_predict_train_rows
  int n_active;                    // set by the launcher (1-D grid: blocks x problems)
};

struct ReduceArgs {
  const int* active;
  const double* partial; long long sPartial; int ntiles;
  const double* z; long long sVec;
  const double* ldiag;
  const int* nvalid;
  const DevSpec* specs;
  double* results;   // [B][kResStride]
  int Np;
};

// ---- small problems (Np = 64 / 128): one fused launch per evaluation (small64_kernel, small128_kernel)
struct Small64Args {
  const int* active;
  const DevSpec* specs; const double* theta; const int* nvalid;
  const double* X; long long sX; int D;
  const double* Y; long long sY;
  double* W; long long sMat; int ld;          // the factor W = L⁻¹ (64x64 block at the origin)
  double* z; double* alpha; double* ldiag; long long sVec;
  int* info;
  double* results;                            // [B][kResStride]
  int grad;                                   // 0: factor, z, α only (predict's re-factorisation)
  int* done; int tag;                         // done != null: workgroup i writes tag to done[i] last
};
void launch_small64(const Small64Args& a, int max_terms, int n_active, hipStream_t s);
void launch_small128(const Small64Args& a, int max_terms, int n_active, hipStream_t s);  // Np = 128

struct PredVarArgs {
  const int* active;
  const double* partial; long long sPartial; int nrowtiles; int ldp;
  const double* Xnew; long long sXnew; int D;
  const DevSpec* specs; const double* theta;
  int M; int add_noise;
  double* var; long long sVar;
};

// ---- block-banded path (gpx_band.hip) --------------------------------------------------
struct BandSolveArgs {
  const int* active;
  const double* W; const double* L; long long sMat; int ld;   // diagonal W_kk blocks, L panels
  const double* Y; long long sY; const int* nvalid;
  double* z; double* alpha; long long sVec;
  int Np, p;                       // p: band width in 64-blocks
};
struct BandTransposeArgs {
  const int* active;
  double* Z; long long sMat; int ld;
  int k;                           // mirror blocks (k+d, k) -> (k, k+d), d = 1..q
};
struct BandContractArgs {
  const int* active;
  const double* Z; long long sMat; int ld;       // selected inverse (band blocks of K⁻¹)
  const double* alpha; long long sVec;
  const double* X; long long sX; int D;
  const DevSpec* specs; const double* theta; const int* nvalid;
  double* partial; long long sPartial;           // [B][(p+1)·nb][16], tile = d·nb + k
  double* colsum; long long sCol;                // [B][Np]: Σ_i K_ji Z_ij accumulated (atomics)
  int Np, p;
};
// fused per-problem sweep for band width p <= 2 (gpx_band.hip: band_fwd_kernel, band_bwd_kernel)
// one slot rebind of flush_rebinds' gather: n rows of X [n][D] and Y [n] from x / y (device
// memory or pinned host staging) into the slot's dx [Nmax][D] / dy [Nmax] (zero padded); with
// box >= 0 also the per-64-block lo/hi of X into box row `box` of the batch's box table
struct RebindDesc {
  const double* x; const double* y; double* dx; double* dy;
  int n; int box;
};
void launch_rebind_gather(const RebindDesc* desc, int m, int Nmax, int D, double* box, hipStream_t s);

struct BandFusedArgs {
  const int* active; const int* bandp;           // per-problem band width p (64-blocks), <= 2
  double* K; double* L; double* W; long long sMat;
  const double* Y; long long sY; const int* nvalid;
  double* z; double* alpha; double* ldiag; long long sVec;
  const double* X; long long sX; int D;
  const DevSpec* specs; const double* theta;
  double* partial; long long sPartial;           // one [16] row per problem (tile 0)
  int* info;
  double* results;                               // [B][kResStride]: writes [kResBandCheck]
  int Np;
  int ld;                                        // leading dimension of K/L/W (Np, or band storage's)
  int kband;                                     // band16: K's band was built with this many 64-block
                                                 // diagonals; entries beyond read as 0 (exact)
  int kstore;                                    // band16 SE1, forward computing K's tiles (KIN): it
                                                 // also writes them into K's band for the backward
  // wave residency trace (gpx_batch_wave_trace; nullptr: off): each band16 wavefront appends
  // {start, end, kind} in the device's constant 100 MHz clock (s_memrealtime), kind = Q for the
  // forward sweep, 16 + Q for the backward
  unsigned long long* wtrace; unsigned int* wtrace_n; unsigned int wtrace_cap;
};
// one wavefront's residency record (lane 0 appends; a vector atomic on the counter)
__device__ __forceinline__ void wave_trace_put(const BandFusedArgs& a, unsigned long long t0, int kind) {
  if (a.wtrace == nullptr) return;
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63) == 0) {
    const unsigned int i = atomicAdd(a.wtrace_n, 1u);
    if (i < a.wtrace_cap) {
      a.wtrace[3ull * i] = t0;
      a.wtrace[3ull * i + 1] = t1;
      a.wtrace[3ull * i + 2] = (unsigned long long)kind;
    }
  }
}
void launch_band_fused(const BandFusedArgs& a, int max_terms, int n_active, hipStream_t s,
                       hipEvent_t* ev = nullptr);  // ev[4]: fwd start/stop, bwd start/stop
// the same for problems with p <= 1 (two LDS blocks per workgroup: two problems per CU)
void launch_band_fused1(const BandFusedArgs& a, int max_terms, int n_active, hipStream_t s,
                        hipEvent_t* ev = nullptr);
// 16-row blocks, one wavefront per problem (gpx_band16.hip); bandp holds each problem's band in
// 16-blocks, all <= Q; se1: every problem is one SquaredExponential term on one input column
// K's band as the band16 sweeps read it: per 16-row block m the tiles (m, m − d), d = 0..Q,
// one wavefront per tile (half the entries of the two 64-block diagonals launch_build writes)
void launch_band16_build(const BuildArgs& a, int Q, int n_active, hipStream_t s);
void launch_wave_marker(unsigned long long* wt, unsigned int* wn, unsigned int cap, int kind, hipStream_t s);
// SE1 band16 problems of widths Q = 4 and 5 (bandp) in one launch, both sweeps per wavefront
void launch_band16_wide(const BandFusedArgs& a, int kin, int n_active, hipStream_t s, hipEvent_t* ev, int wq = 5);
// the deferred part's private copies of the call's active rows, θ and widths, and its zeroed
// info block, in one launch of one-wave workgroups
void launch_slow_inputs(const int* act, int n, int* act_out, const double* theta, double* theta_out, const int* bandp,
                        int* bandp_out, int* info_out, int B, hipStream_t s,
                        int r0 = 0, int r1 = 0);
void launch_spin_us(int us, hipStream_t s);  // diagnostic delay (GPX_SLOW_DELAY_US)
void launch_slow_gather(const int* act, int n, const double* res, int stride, double* out, const int* info,
                        int* info_out, hipStream_t s);
void launch_band16(const BandFusedArgs& a, int Q, int max_terms, bool se1, int kin, int n_active, hipStream_t s,
                   hipEvent_t* ev = nullptr);
// ---- block cyclic reduction over the band (gpx_bcr.hip): calls with few problems -------------
// per-problem workspace, nbm blocks of bs = 16Q rows: the blocks A (then Z_XX), C (the coupling
// with the left neighbour: E, then Z), the neighbours' updates ΔL / ΔR, the factor W_X, P_Iᵀ,
// P_Kᵀ; the vectors y, the y updates, z, α; per block a [16] gradient row and a check maximum
struct BcrLayout {
  long long A, C, DL, DR, Wm, PI, PK, y, dyL, dyR, z, al, part, chk, ctr, total;
  __host__ __device__ BcrLayout(int bs, int nbm) {
    const long long M = (long long)bs * bs * nbm, V = (long long)bs * nbm;
    A = 0; C = M; DL = 2 * M; DR = 3 * M; Wm = 4 * M; PI = 5 * M; PK = 6 * M;
    y = 7 * M; dyL = y + V; dyR = dyL + V; z = dyR + V; al = z + V;
    part = al + V; chk = part + (long long)GPX_THETA_STRIDE * nbm; ctr = chk + nbm; total = ctr + 1;
  }
};
struct BcrArgs {
  const int* active;                 // the class's problems (workspace index = position here)
  const DevSpec* specs; const double* theta; const int* nvalid;
  const double* X; long long sX; int D;
  const double* Y; long long sY;
  double* ws; long long sWs;         // per-problem workspace (bcr_ws_doubles)
  int nbm, bs;                       // blocks per problem in the layout, block rows (set by the launcher)
  int* info;
  double* z; double* ldiag; double* alpha; long long sVec; int Np;   // the reduce kernel's inputs, α
  double* Kd; long long sMat; int ld;                                 // diag(Z) onto K's diagonal
  double* partial; long long sPartial;                                // the [16] gradient row (tile 0)
  double* results;                                                    // [kResBandCheck]
  int level;
};
long long bcr_ws_doubles(int Q, int Nmax);
// the whole evaluation of np problems of band width <= Q 16-blocks (Q <= 5): forward levels,
// backward levels, contraction, per-problem finish; the reduce kernel follows (launch_reduce)
// cache: the batch's captured chains (gpx_batch::bcr_graphs; created on first use), or nullptr
void launch_bcr(const BcrArgs& a, int Q, int max_terms, int np, int Nmax, hipStream_t s, void** cache);
void bcr_graph_cache_free(void* cache);

void launch_band_solve(const BandSolveArgs& a, int n_active, hipStream_t s);
void launch_band_transpose(const BandTransposeArgs& a, int q, int n_active, hipStream_t s);
void launch_band_contract(const BandContractArgs& a, int max_terms, int n_active, hipStream_t s);
// results[b][kResBandCheck] = max_{j<n} |colsum[b][j] − 1|
void launch_band_check(const int* active, const double* colsum, long long sCol, const int* nvalid,
                       double* results, int n_active, int Np, hipStream_t s);
void launch_band_train_pred(const TrainPredArgs& a, int n_active, int Np, hipStream_t s);

void launch_build(const BuildArgs& a, int n_active, hipStream_t s);
void launch_leaf(const LeafArgs& a, int n_active, hipStream_t s);
void launch_leaf128(const LeafArgs& a, int n_active, hipStream_t s);  // 128x128 block, fused
void launch_gemm(const GemmArgs& a, int epi, bool ta, bool tb, int n_active, hipStream_t s);
void launch_trmv_n(const TrmvArgs& a, int n_active, hipStream_t s);   // y = M x   (row dots)
void launch_trmv_t(const TrmvArgs& a, int n_active, hipStream_t s);   // y = Mᵀ x  (column sums)
void launch_reduce(const ReduceArgs& a, int n_active, hipStream_t s);
void launch_train_pred(const TrainPredArgs& a, int n_active, int Np, hipStream_t s);
void launch_predvar(const PredVarArgs& a, int n_active, hipStream_t s);
int gemm_tile(const GemmArgs& a, int n_active);  // tile edge the launcher will use (64 or 128)
// The GEMM stages operands with buffer loads: a per-K-tile base plus a 32-bit per-lane byte
// offset, inside a 0x7fffffff-byte buffer window. The farthest element a tile reads is
// (128 - 1) rows * ld * 8 B + one 128-wide row, so every leading dimension must satisfy
// 127 * ld * 8 + 1024 < 2^31 (ld <= 2,113,662 doubles). Out-of-window buffer loads return 0
// without faulting, so the API rejects larger shapes (GPX_BAD_ARG) and the launcher asserts.
constexpr long long kGemmMaxLd = (0x7fffffffLL - 1024) / (127LL * 8);

// ---- SVGP (gpx_svgp_kernels.hip) -----------------------------------------------------
// Row-organised derivative contraction over an M×N (or M×M) index set:
//   Kbar_ij = u_i g_j (optional) + Y_ij (or ½(Y_ij + Y_ji) when sym)
//   θ:  Σ_ij Kbar_ij ∂k(z_i, x_j)/∂θ          -> part_theta [blocks][16]
//   z:  zscale Σ_j Kbar_ij ∂k(z_i, x_j)/∂z_i  -> part_z [chunks][Mp*D]
//   w:  Σ_j k(z_i, x_j) g_j (optional)         -> part_w [chunks][Mp]
struct RowsArgs {
  const double* Zr; const double* Xc; int D;
  int nrows, ncols;
  const double* Y; int ldy; int sym;
  const double* u; const double* g;
  double zscale;
  const DevSpec* spec; const double* theta;
  int chunk;
  double* part_theta; double* part_z; double* part_w;
  int Mp;
};

// g_j = s (y_j − μ_j)/σ²; block partials [blocks][kResidW]: 0..15 c Σ ∂k_jj/∂θ (θ layout),
// 16 Σ (y−μ)², 17 Σ k_jj.
constexpr int kResidW = 20;
struct ResidArgs {
  const double* X; const double* Y; const double* mu; int D; int n; int npad;
  const DevSpec* spec; const double* theta;
  double scale;            // num_data / n_total
  double* g;               // [npad], zero beyond n
  double* part;            // [blocks][kResidW]
};

// dst[c] (+)= Σ_b src[b*stride + c], c < width
struct SumArgs {
  const double* src; long long stride; int nb; long long width;
  double* dst; int accumulate;
};

// Elementwise M×M tail of the ELBO gradient (valid i, j < m):
//   Phi = Φ(−(q âᵀ + 2c X1)), Rbar = tril(2c GR − R + diag(1/R_ii)), trace partials of Sm1∘Ĝ
struct SvgpFinalArgs {
  const double* X1; const double* GR; const double* R; const double* Sm1; const double* Gh;
  const double* q; const double* ahat; double c2;
  int m, ld;
  double* Phi; double* Rbar; double* part_tr;   // part_tr [blocks]
};

struct SvgpPredVarArgs {
  const double* pA; const double* pB; int nrt; int ldp;   // COLSUMSQ partials [nrt][ldp]
  const double* Xnew; int D; int M;
  const DevSpec* spec; const double* theta; int add_noise;
  double* var;
};

void launch_rows(const RowsArgs& a, bool single_term, hipStream_t s);
int rows_chunk_for(int D);              // column chunk for RowsArgs.chunk
int rows_blocks(const RowsArgs& a);     // number of part_theta rows written
int rows_chunks(const RowsArgs& a);     // number of part_z / part_w chunks written
void launch_resid(const ResidArgs& a, hipStream_t s);
int resid_blocks(int npad);
void launch_sum(const SumArgs& a, hipStream_t s);
void launch_svgp_final(const SvgpFinalArgs& a, hipStream_t s);
int svgp_final_blocks(int m);
void launch_diag_add(double* A, int ld, int n, double v, hipStream_t s);
void launch_symmetrize_lower(double* A, int ld, int n, hipStream_t s);
void launch_svgp_predvar(const SvgpPredVarArgs& a, hipStream_t s);

}  // namespace gpx
