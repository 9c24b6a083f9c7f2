// gpx_api.hip — C ABI (include/gpx.h) and host orchestration of the exact-GP engine.
//
// One evaluation of logML and ∂logML/∂θ for B problems (the closure gpflow.optimizers.Scipy
// calls from GPR/model_trainer.py:19) runs, all on one stream:
//   1. K = k(X,X) + σn²I                                      build_kernel
//   2. (L, W = L⁻¹) by recursive blocked Cholesky-and-inverse  leaf + MFMA TRMM/SYRK GEMMs
//        chol_inv(A):  (L11,W11) = chol_inv(A11);  L21 = A21 W11ᵀ;  A22 -= L21 L21ᵀ;
//                      (L22,W22) = chol_inv(A22);  W21 = −W22 (L21 W11)
//   3. z = W y, α = Wᵀ z                                      trmv kernels
//   4. K⁻¹ = WᵀW formed tile by tile and contracted on the fly with (ααᵀ − K⁻¹)∘∂K/∂θ
//   5. logML = −½‖z‖² − Σ log L_ii − (n/2) log 2π;  ∂logML/∂θ = ½ Σ (ααᵀ − K⁻¹)∘∂K/∂θ
// Algorithmic flops per problem: N³/3 (potrf) + N³/3 (trtri) + N³/3 (WᵀW) ≈ N³.
#include <hip/hip_runtime.h>
#include <cfloat>
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <string>
#include <chrono>
#include <vector>
#include "gpx_host.h"

using namespace gpx;

namespace gpx {

const char* kVersion = "gpx 0.1.0 (gfx950, fp64 MFMA)";

std::string& last_error_slot() {
  static thread_local std::string msg;
  return msg;
}


// MFMA flops the GEMM launcher will issue for these args (bench / roofline bookkeeping)
double gemm_issued_flops(const GemmArgs& a, int na) {
  const int bm = gemm_tile(a, na);
  const int ti = a.M / bm, tj = a.N / bm;
  double f = 0.0;
  for (int x = 0; x < ti; ++x)
    for (int y = 0; y < tj; ++y) {
      if (a.lower_only && y > x) continue;
      const int i0 = x * bm, j0 = y * bm;
      int kmin = 0, kmax = a.K;
      if (a.tri & TRI_KMAX_I) kmax = std::min(kmax, i0 + bm);
      if (a.tri & TRI_KMAX_J) kmax = std::min(kmax, j0 + bm);
      if (a.tri & TRI_KMIN_J) kmin = std::max(kmin, j0);
      if (a.tri & TRI_KMIN_I) kmin = std::max(kmin, i0);
      if (kmax > kmin) f += 2.0 * bm * bm * (kmax - kmin);
    }
  return f * na;
}

void gemm(const Run& r, GemmArgs a, int epi, bool ta, bool tb) {
  a.active = r.d_act;
  // store GEMMs (the recursion's panels, trailing updates and inverses) pick 128-tiles only when
  // the launch still has a workgroup per CU (64-tiles otherwise: 4x the workgroups for the
  // recursion's lower levels in calls of few problems). An entry's sum runs over the same k in
  // the same 4-wide MFMA chunks either way — a wider tile's k-range only adds products with the
  // triangular operand's exact zeros, each ±0 onto a sum that is +0 until its first nonzero —
  // so a problem's arithmetic still does not depend on its call (tests/test_gpu_parity.py).
  // The contraction's per-tile partials do depend on the tile: it keeps the shape-only rule.
  a.small_tiles = r.bt->small_tiles || epi == EPI_STORE;
  launch_gemm(a, epi, ta, tb, r.na, r.s);
  if (r.bt->ctx->profiling) r.bt->flops_acc += gemm_issued_flops(a, r.na);
}

GemmArgs gemm_args(const double* A, int lda, const double* B, int ldb, double* C, int ldc,
                   long long stride, int M, int N, int K, int tri, int lower, double alpha,
                   double beta) {
  GemmArgs g{};
  // longest-K tiles first, with the K-determining tile index as the slow one
  g.order = (tri & TRI_KMAX_J) ? ORDER_COL_DESC : (tri & TRI_KMIN_J) ? ORDER_COL_ASC
          : (tri & TRI_KMAX_I) ? ORDER_ROW_DESC : ORDER_ROW_ASC;
  g.A = A; g.sA = stride; g.lda = lda;
  g.Bm = B; g.sB = stride; g.ldb = ldb;
  g.C = C; g.sC = stride; g.ldc = ldc;
  g.M = M; g.N = N; g.K = K; g.tri = tri; g.lower_only = lower;
  g.alpha = alpha; g.beta = beta;
  return g;
}

// Recursive Cholesky-and-inverse on the diagonal block [off, off+n) of every problem of r.
void chol_inv(const Run& r, int off, int n, int depth) {
  gpx_batch* bt = r.bt;
  const int Np = bt->Np;
  const long long st = mat_stride(bt);
  // GPX_LEAF128=0 recurses down to 64-leaves instead (A/B measurements)
  static const bool leaf128 = [] {
    const char* e = getenv("GPX_LEAF128");
    return !(e && atoi(e) == 0);
  }();
  if (n == kLeaf || (leaf128 && n == 2 * kLeaf)) {
    LeafArgs la{};
    la.active = r.d_act; la.K = bt->K; la.W = bt->W; la.sMat = st; la.ld = Np; la.off = off;
    la.ldiag = bt->ldiag; la.sVec = Np; la.info = bt->d_info;
    // a 128-node is factored and inverted by one fused kernel (no 64x64 GEMM launches)
    if (n == kLeaf) launch_leaf(la, r.na, r.s);
    else launch_leaf128(la, r.na, r.s);
    return;
  }
  int n1 = ((n / 2 + kLeaf - 1) / kLeaf) * kLeaf;
  if (n1 >= n) n1 = n - kLeaf;
  const int n2 = n - n1;
  chol_inv(r, off, n1, depth + 1);
  const long long o11 = (long long)off * Np + off;
  const long long o21 = (long long)(off + n1) * Np + off;
  const long long o22 = (long long)(off + n1) * Np + off + n1;
  // L21 = A21 · W11ᵀ          (opB(k,j) = W11[j][k], nonzero for k <= j)
  gemm(r, gemm_args(bt->K + o21, Np, bt->W + o11, Np, bt->L + o21, Np, st, n2, n1, n1,
                    TRI_KMAX_J, 0, 1.0, 0.0), EPI_STORE, false, true);
  // T = L21 · W11 → the dead A21 region of K   (opB(k,j) = W11[k][j], nonzero for k >= j).
  // T depends only on L21 and W11, so at the top depths it runs on an auxiliary stream
  // concurrently with the (latency-bound) recursion on A22 below.
  const GemmArgs targs = gemm_args(bt->L + o21, Np, bt->W + o11, Np, bt->K + o21, Np, st, n2, n1,
                                   n1, TRI_KMIN_J, 0, 1.0, 0.0);
  const bool fork = r.dag && depth < kAux && r.next_event && *r.next_event + 2 <= kEvents;
  hipEvent_t eT = nullptr;
  if (fork) {
    hipEvent_t eL = bt->ev[(*r.next_event)++];
    eT = bt->ev[(*r.next_event)++];
    Run ra = r;
    ra.s = bt->aux[depth];
    (void)hipEventRecord(eL, r.s);
    (void)hipStreamWaitEvent(ra.s, eL, 0);
    gemm(ra, targs, EPI_STORE, false, false);
    (void)hipEventRecord(eT, ra.s);
  } else {
    gemm(r, targs, EPI_STORE, false, false);
  }
  // A22 -= L21 · L21ᵀ         (lower tiles only)
  gemm(r, gemm_args(bt->L + o21, Np, bt->L + o21, Np, bt->K + o22, Np, st, n2, n2, n1, 0, 1,
                    -1.0, 1.0), EPI_STORE, false, true);
  chol_inv(r, off + n1, n2, depth + 1);
  if (fork) (void)hipStreamWaitEvent(r.s, eT, 0);
  // W21 = −W22 · T             (opA(i,k) = W22[i][k], nonzero for k <= i)
  gemm(r, gemm_args(bt->W + o22, Np, bt->K + o21, Np, bt->W + o21, Np, st, n2, n1, n2,
                    TRI_KMAX_I, 0, -1.0, 0.0), EPI_STORE, false, false);
}

// K build + recursive factor for the problems of r.
void factor(const Run& r) {
  gpx_batch* bt = r.bt;
  BuildArgs ba{};
  ba.active = r.d_act; ba.specs = bt->d_specs; ba.theta = bt->d_theta; ba.nvalid = bt->d_n;
  ba.X = bt->X; ba.sX = (long long)bt->Nmax * bt->D; ba.X2 = bt->X; ba.sX2 = ba.sX; ba.D = bt->D;
  ba.m2 = 0; ba.out = bt->K; ba.sOut = mat_stride(bt); ba.ldo = bt->Np; ba.rows = ba.cols = bt->Np;
  ba.symmetric = 1;
  launch_build(ba, r.na, r.s);
  chol_inv(r, 0, bt->Np);
}

// z = W y, α = Wᵀ z
void alpha_solve(const Run& r) {
  gpx_batch* bt = r.bt;
  const long long st = mat_stride(bt);
  TrmvArgs t{};
  t.active = r.d_act; t.Wm = bt->W; t.sW = st; t.ld = bt->Np;
  t.x = bt->Y; t.sx = bt->Nmax; t.nvalid = bt->d_n; t.y = bt->z; t.sy = bt->Np;
  t.rows = t.cols = bt->Np; t.lower = 1;
  launch_trmv_n(t, r.na, r.s);
  TrmvArgs u{};
  u.active = r.d_act; u.Wm = bt->W; u.sW = st; u.ld = bt->Np;
  u.x = bt->z; u.sx = bt->Np; u.nvalid = nullptr; u.y = bt->alpha; u.sy = bt->Np;
  u.rows = u.cols = bt->Np; u.lower = 1;
  launch_trmv_t(u, r.na, r.s);
}

// fused K⁻¹ = WᵀW formation + gradient contraction over lower tiles, then the reduction
void contract(const Run& r, int max_terms, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr) {
  gpx_batch* bt = r.bt;
  GemmArgs g = gemm_args(bt->W, bt->Np, bt->W, bt->Np, nullptr, 0, mat_stride(bt), bt->Np, bt->Np,
                         bt->Np, TRI_KMIN_I, 1, 1.0, 0.0);
  g.vec = bt->alpha; g.sVec = bt->Np; g.X = bt->X; g.sX = (long long)bt->Nmax * bt->D; g.D = bt->D;
  g.specs = bt->d_specs; g.theta = bt->d_theta; g.nvalid = bt->d_n;
  g.partial = bt->partial; g.sPartial = bt->partial_stride;
  g.ev_start = ev0; g.ev_stop = ev1;
  gemm(r, g, max_terms <= 1 ? EPI_CONTRACT1 : max_terms == 2 ? EPI_CONTRACT2 : EPI_CONTRACT, true, false);
}

void reduce(const Run& r) {
  gpx_batch* bt = r.bt;
  GemmArgs g{};
  g.M = g.N = bt->Np; g.lower_only = 1; g.small_tiles = bt->small_tiles;  // as gemm() launches it
  const int bm = gemm_tile(g, r.na), tt = bt->Np / bm;
  ReduceArgs ra{};
  ra.active = r.d_act; ra.partial = bt->partial; ra.sPartial = bt->partial_stride;
  ra.ntiles = tt * (tt + 1) / 2; ra.z = bt->z; ra.sVec = bt->Np; ra.ldiag = bt->ldiag;
  ra.nvalid = bt->d_n; ra.specs = bt->d_specs; ra.results = bt->results; ra.Np = bt->Np;
  launch_reduce(ra, r.na, r.s);
}


// Np = 64 and Np = 128 batches: every dense evaluation is one fused launch (small64_kernel,
// small128_kernel; GPX_SMALL64=0 / GPX_SMALL128=0: the six-launch chain, for A/B). Which path runs
// depends on Np only, never on the call.
bool small64_on(const gpx_batch* bt) {
  static const bool on64 = [] {
    const char* e = getenv("GPX_SMALL64");
    return !(e && atoi(e) == 0);
  }();
  static const bool on128 = [] {
    const char* e = getenv("GPX_SMALL128");
    return !(e && atoi(e) == 0);
  }();
  return (on64 && bt->Np == kLeaf) || (on128 && bt->Np == 2 * kLeaf);
}

// the fused small-problem evaluation (grad: the gradient and logML too) for the problems of r;
// sio: the call's I/O block in coherent pinned memory (active list, θ, info, results read and
// written there by the kernel), else the device I/O block
void small64_eval(const Run& r, bool grad, char* sio = nullptr, int tag = 0) {
  gpx_batch* bt = r.bt;
  Small64Args a{};
  a.active = r.d_act; a.specs = bt->d_specs; a.theta = bt->d_theta; a.nvalid = bt->d_n;
  a.X = bt->X; a.sX = (long long)bt->Nmax * bt->D; a.D = bt->D; a.Y = bt->Y; a.sY = bt->Nmax;
  a.W = bt->W; a.sMat = mat_stride(bt); a.ld = bt->Np;
  a.z = bt->z; a.alpha = bt->alpha; a.ldiag = bt->ldiag; a.sVec = bt->Np;
  a.info = bt->d_info; a.results = bt->results; a.grad = grad ? 1 : 0;
  if (sio) {
    a.active = reinterpret_cast<const int*>(sio);
    a.info = reinterpret_cast<int*>(sio + bt->io_info_off);
    a.theta = reinterpret_cast<const double*>(sio + bt->io_theta_off);
    a.results = reinterpret_cast<double*>(sio + bt->io_res_off);
    if (tag > 0) {
      a.done = reinterpret_cast<int*>(sio + bt->io_flag_off);
      a.tag = tag;
    }
  }
  int max_terms = 1;
  for (int b = 0; b < bt->B; ++b) max_terms = std::max(max_terms, (int)bt->specs[b].n_terms);
  if (bt->Np == kLeaf)
    launch_small64(a, max_terms, r.na, r.s);
  else
    launch_small128(a, max_terms, r.na, r.s);
}

// ---------------------------------------------------------------------------------------
// Block-banded path (kernels in gpx_band.hip)
// ---------------------------------------------------------------------------------------
// Exactness: for the monotone stationary kernels (SE, Matern12/32/52, Exponential) every value
// and θ-derivative carries the factor exp(−a(s)), s = r/ℓ, with a(s) = s²/2, s, s/2, √3 s or
// √5 s. When a(s) ≥ 746 that factor is exactly 0 in fp64 (exp underflows below 2^-1075 at
// 745.13) and so is the whole entry (0 times a finite polynomial). band_rmin bounds r from
// below for every pair of points in blocks (k, k − d) (bounding boxes of the blocks' valid
// rows, per term's active dims); the margin 746 − 745.13 covers the rounding of r²/ℓ² on the
// device many times over. The device forms r² as GPflow does, (−2a·b) + (‖a‖² + ‖b‖²) with
// a = x/ℓ, which can fall short of the true (Δx/ℓ)² by cancellation, by at most a few
// eps·(‖a‖² + ‖b‖² + ‖a−b‖·max‖a‖): band_width shaves 64 eps·(M² + sM + 1) off s² (M = the
// largest ‖x/ℓ‖ of the problem's valid rows, kept in slot 0 of each term's table).
// A sum vanishes when all its terms do, a product when any does.
namespace {
bool band_kind(int kind) { return kind >= GPX_SE && kind <= GPX_EXPONENTIAL; }

double band_arg(int kind, double s) {
  switch (kind) {
    case GPX_SE: return 0.5 * s * s;
    case GPX_MATERN12: return s;
    case GPX_EXPONENTIAL: return 0.5 * s;
    case GPX_MATERN32: return 1.7320508075688772 * s;
    default: return 2.23606797749979 * s;  // GPX_MATERN52
  }
}
}  // namespace

// band_rmin of problem b at block size bs (64: band_rmin, 16: band_rmin16) from the per-block
// boxes lo/hi [nvb][D] of its valid rows (blocks of bs rows)
// The widest band offset (in blocks of bs rows) any routing decision distinguishes: the 64-row
// paths take p <= band_limit <= Np/256, the band16 path Q <= kBand16MaxQ; a table entry beyond
// it only has to say "still nonzero" correctly, which a lower bound does.
static int band_table_cap(const gpx_batch* bt, int bs) {
  if (bs != kLeaf) return kBand16MaxQ + 1;
  const char* ep = getenv("GPX_BAND_PMAX");  // (band_limit's override, when it raises the limit)
  return std::max(bt->Np / kLeaf / 4, ep ? atoi(ep) : 0) + 1;
}

static void band_tables_lohi(gpx_batch* bt, int b, int bs, const std::vector<double>& lo,
                             const std::vector<double>& hi) {
  const int nb = bt->Np / bs, D = bt->D, n = bt->n[b];
  std::vector<double>& tabv = bs == kLeaf ? bt->band_rmin : bt->band_rmin16;
  double* out = tabv.data() + (size_t)b * GPX_MAX_TERMS * nb;
  std::fill(out, out + (size_t)GPX_MAX_TERMS * nb, INFINITY);
  int* tail = (bs == kLeaf ? bt->band_tail : bt->band_tail16).data() + (size_t)b * GPX_MAX_TERMS;
  std::fill(tail, tail + GPX_MAX_TERMS, nb);
  const gpx_kernel_spec& sp = bt->specs[b];
  const int nvb = (n + bs - 1) / bs;  // blocks holding valid rows
  const int cap = band_table_cap(bt, bs);
  for (int t = 0; t < sp.n_terms; ++t) {
    const int d0 = sp.terms[t].dim_start, dn = sp.terms[t].dim_count;
    double* rt = out + (size_t)t * nb;
    // one active dimension with the blocks' boxes in increasing order (day offsets): the gap
    // between blocks k and k − dd is lo[k] − hi[k − dd], nondecreasing in dd for every k, so
    // rmin is nondecreasing and rmin[cap] bounds every later entry from below
    bool sorted = dn == 1;
    for (int k = 1; sorted && k < nvb; ++k) sorted = hi[(size_t)(k - 1) * D + d0] <= lo[(size_t)k * D + d0];
    const int ddmax = sorted ? std::min(nvb - 1, cap) : nvb - 1;
    double m2 = 0.0;  // max ‖x‖² over the valid rows (active dims), bounded by the boxes
    for (int k = 0; k < nvb; ++k) {
      double s2 = 0.0;
      for (int d = d0; d < d0 + dn; ++d) {
        const double mx = std::max(std::fabs(lo[(size_t)k * D + d]), std::fabs(hi[(size_t)k * D + d]));
        s2 += mx * mx;
      }
      m2 = std::max(m2, s2);
    }
    rt[0] = std::sqrt(m2) * (1.0 + 1e-12);
    for (int dd = 1; dd <= ddmax; ++dd) {
      double m = INFINITY;
      for (int k = dd; k < nvb; ++k) {
        double g2 = 0.0;
        for (int d = d0; d < d0 + dn; ++d) {
          const double g = std::max(0.0, std::max(lo[(size_t)k * D + d] - hi[(size_t)(k - dd) * D + d],
                                                  lo[(size_t)(k - dd) * D + d] - hi[(size_t)k * D + d]));
          g2 += g * g;
        }
        m = std::min(m, g2);
      }
      // the box gap is exact in real arithmetic; shave a relative 1e-12 off for the rounding
      // of the sums above
      rt[dd] = std::sqrt(m) * (1.0 - 1e-12);
    }
    if (ddmax < nvb - 1) {
      for (int dd = ddmax + 1; dd < nvb; ++dd) rt[dd] = rt[ddmax];
      tail[t] = ddmax;
    }
  }
}

// both tables from the 16-row boxes box[nvb16][D][2] of problem b (the 64-row boxes are their
// unions); band_rmin16 is kept only where the 16-row path can run (Np <= kBand16MaxNp)
void band_tables_boxes(gpx_batch* bt, int b, const double* box) {
  const int D = bt->D, n = bt->n[b];
  const int nv16 = (n + kBox - 1) / kBox, nv64 = (n + kLeaf - 1) / kLeaf;
  std::vector<double> lo((size_t)nv64 * D, INFINITY), hi((size_t)nv64 * D, -INFINITY);
  for (int k = 0; k < nv16; ++k)
    for (int d = 0; d < D; ++d) {
      const size_t e = (size_t)k * D + d, f = (size_t)(k / (kLeaf / kBox)) * D + d;
      lo[f] = std::min(lo[f], box[2 * e]);
      hi[f] = std::max(hi[f], box[2 * e + 1]);
    }
  band_tables_lohi(bt, b, kLeaf, lo, hi);
  if (!bt->band_rmin16.empty()) {
    std::vector<double> lo16((size_t)nv16 * D), hi16((size_t)nv16 * D);
    for (size_t e = 0; e < (size_t)nv16 * D; ++e) {
      lo16[e] = box[2 * e];
      hi16[e] = box[2 * e + 1];
    }
    band_tables_lohi(bt, b, kBox, lo16, hi16);
  }
}

void band_tables(gpx_batch* bt, int b, const double* hostX) {
  const int D = bt->D, n = bt->n[b];
  const int nvb = (n + kBox - 1) / kBox;
  std::vector<double> box((size_t)nvb * D * 2);
  for (int k = 0; k < nvb; ++k)
    for (int d = 0; d < D; ++d) {
      double a = INFINITY, z = -INFINITY;
      for (int r = k * kBox; r < std::min(n, (k + 1) * kBox); ++r) {
        a = std::min(a, hostX[(size_t)r * D + d]);
        z = std::max(z, hostX[(size_t)r * D + d]);
      }
      box[2 * ((size_t)k * D + d)] = a;
      box[2 * ((size_t)k * D + d) + 1] = z;
    }
  band_tables_boxes(bt, b, box.data());
}

static int band_width_bs(const gpx_batch* bt, int b, const double* th, int bs) {
  const gpx_kernel_spec& sp = bt->specs[b];
  for (int t = 0; t < sp.n_terms; ++t)
    if (!band_kind(sp.terms[t].kind)) return -1;
  const int nb = bt->Np / bs;
  const double* tab = (bs == kLeaf ? bt->band_rmin : bt->band_rmin16).data() + (size_t)b * GPX_MAX_TERMS * nb;
  const int* tail = (bs == kLeaf ? bt->band_tail : bt->band_tail16).data() + (size_t)b * GPX_MAX_TERMS;
  const bool prod = sp.n_terms > 1 && sp.combine == GPX_PRODUCT;
  auto nz_at = [&](int d) {
    bool nz = prod;
    for (int t = 0; t < sp.n_terms; ++t) {
      const double ell = th[sp.terms[t].param_offset];
      const double r = tab[(size_t)t * nb + d];
      bool term_nz = false;
      if (r != INFINITY) {
        const double sv = r / ell, M = tab[(size_t)t * nb] / ell;
        const double s2 = sv * sv - 64.0 * DBL_EPSILON * (M * M + sv * M + 1.0);
        term_nz = !(band_arg(sp.terms[t].kind, s2 > 0.0 ? std::sqrt(s2) : 0.0) >= 746.0);
      }
      nz = prod ? (nz && term_nz) : (nz || term_nz);
    }
    return nz;
  };
  // beyond the largest tail offset every term's entry repeats, so the scan from the top gives the
  // same answer as testing that offset once
  int top = nb - 1, tmax = 0;
  for (int t = 0; t < sp.n_terms; ++t) tmax = std::max(tmax, tail[t]);
  if (tmax >= 1 && tmax < nb - 1) {
    if (nz_at(tmax)) return nb - 1;
    top = tmax - 1;
  }
  for (int d = top; d >= 1; --d)
    if (nz_at(d)) return d;
  return 0;
}

int band_width(const gpx_batch* bt, int b, const double* th) { return band_width_bs(bt, b, th, kLeaf); }

// the band width in 16-row blocks (band16 kernels), or -1 when the tables are not kept
int band_width16(const gpx_batch* bt, int b, const double* th) {
  if (bt->band_rmin16.empty()) return -1;
  return band_width_bs(bt, b, th, kBox);
}

// the 16-row path (gpx_band16.hip) takes p64 <= 1 problems whose band is at most this many
// 16-blocks (GPX_BAND16=0 disables it)
int band16_limit(const gpx_batch* bt) {
  const char* e = getenv("GPX_BAND16");
  if (e && atoi(e) == 0) return -1;
  if (bt->band_rmin16.empty() || bt->D > kBand16MaxD) return -1;
  return kBand16MaxQ;
}

// shapes the banded path handles: ≥ 8 blocks (smaller problems are a few leaves densely) and
// z in LDS for the solve. Band tables are kept for every such batch, whatever GPX_BAND says.
bool band_shape(const gpx_batch* bt) { return bt->Np / kLeaf >= 8 && bt->Np <= 8192; }

int band_limit(const gpx_batch* bt) {
  // read per call (cheap), so a process can compare the paths on the same problems
  const char* em = getenv("GPX_BAND");
  const char* ep = getenv("GPX_BAND_PMAX");
  const int mode = em ? atoi(em) : 1;
  const int pmax_env = ep ? atoi(ep) : -1;
  if (mode == 0 || bt->force_dense || !band_shape(bt)) return -1;
  return pmax_env >= 0 ? pmax_env : bt->Np / kLeaf / 4;
}

void band_eval(const Run& r, int p, int max_terms) {
  gpx_batch* bt = r.bt;
  const int Np = bt->Np, nb = Np / kLeaf;
  const long long st = mat_stride(bt);
  const long long rowb = (long long)kLeaf * Np;  // one block row
  BuildArgs ba{};
  ba.active = r.d_act; ba.specs = bt->d_specs; ba.theta = bt->d_theta; ba.nvalid = bt->d_n;
  ba.X = bt->X; ba.sX = (long long)bt->Nmax * bt->D; ba.X2 = bt->X; ba.sX2 = ba.sX; ba.D = bt->D;
  ba.m2 = 0; ba.out = bt->K; ba.sOut = st; ba.ldo = Np; ba.rows = ba.cols = Np;
  ba.symmetric = 1; ba.band1 = p + 1;
  launch_build(ba, r.na, r.s);
  // forward: right-looking block Cholesky over the band; W_kk = L_kk⁻¹ from the leaf
  LeafArgs la{};
  la.active = r.d_act; la.K = bt->K; la.W = bt->W; la.sMat = st; la.ld = Np;
  la.ldiag = bt->ldiag; la.sVec = Np; la.info = bt->d_info;
  for (int k = 0; k < nb; ++k) {
    la.off = k * kLeaf;
    launch_leaf(la, r.na, r.s);
    const int q = std::min(p, nb - 1 - k);
    if (q == 0) continue;
    const long long okk = k * rowb + k * kLeaf, opan = (k + 1) * rowb + k * kLeaf,
                    owin = (k + 1) * rowb + (k + 1) * kLeaf;
    // L_panel = A_panel · W_kkᵀ
    gemm(r, gemm_args(bt->K + opan, Np, bt->W + okk, Np, bt->L + opan, Np, st, q * kLeaf, kLeaf, kLeaf,
                      TRI_KMAX_J, 0, 1.0, 0.0), EPI_STORE, false, true);
    // A_window −= L_panel L_panelᵀ (lower tiles)
    gemm(r, gemm_args(bt->L + opan, Np, bt->L + opan, Np, bt->K + owin, Np, st, q * kLeaf, q * kLeaf,
                      kLeaf, 0, 1, -1.0, 1.0), EPI_STORE, false, true);
  }
  BandSolveArgs sa{};
  sa.active = r.d_act; sa.W = bt->W; sa.L = bt->L; sa.sMat = st; sa.ld = Np;
  sa.Y = bt->Y; sa.sY = bt->Nmax; sa.nvalid = bt->d_n; sa.z = bt->z; sa.alpha = bt->alpha; sa.sVec = Np;
  sa.Np = Np; sa.p = p;
  launch_band_solve(sa, r.na, r.s);
  // backward: selected inversion into K's band blocks (K is dead after the leaves read it)
  //   G = L_panel W_kk (in place over the panel), Z_panel = −Z_window G,
  //   Z_kk = W_kkᵀ W_kk − Gᵀ Z_panel, and the panel mirrored above the diagonal
  BandTransposeArgs ta{};
  ta.active = r.d_act; ta.Z = bt->K; ta.sMat = st; ta.ld = Np;
  for (int k = nb - 1; k >= 0; --k) {
    const int q = std::min(p, nb - 1 - k);
    const long long okk = k * rowb + k * kLeaf, opan = (k + 1) * rowb + k * kLeaf,
                    owin = (k + 1) * rowb + (k + 1) * kLeaf;
    gemm(r, gemm_args(bt->W + okk, Np, bt->W + okk, Np, bt->K + okk, Np, st, kLeaf, kLeaf, kLeaf, 0, 0,
                      1.0, 0.0), EPI_STORE, true, false);
    if (q == 0) continue;
    gemm(r, gemm_args(bt->L + opan, Np, bt->W + okk, Np, bt->L + opan, Np, st, q * kLeaf, kLeaf, kLeaf,
                      TRI_KMIN_J, 0, 1.0, 0.0), EPI_STORE, false, false);
    gemm(r, gemm_args(bt->K + owin, Np, bt->L + opan, Np, bt->K + opan, Np, st, q * kLeaf, kLeaf,
                      q * kLeaf, 0, 0, -1.0, 0.0), EPI_STORE, false, false);
    ta.k = k;
    launch_band_transpose(ta, q, r.na, r.s);
    gemm(r, gemm_args(bt->L + opan, Np, bt->K + opan, Np, bt->K + okk, Np, st, kLeaf, kLeaf, q * kLeaf,
                      0, 0, -1.0, 1.0), EPI_STORE, true, false);
  }
  BandContractArgs ca{};
  ca.active = r.d_act; ca.Z = bt->K; ca.sMat = st; ca.ld = Np; ca.alpha = bt->alpha; ca.sVec = Np;
  ca.X = bt->X; ca.sX = (long long)bt->Nmax * bt->D; ca.D = bt->D; ca.specs = bt->d_specs;
  ca.theta = bt->d_theta; ca.nvalid = bt->d_n; ca.partial = bt->partial; ca.sPartial = bt->partial_stride;
  ca.Np = Np; ca.p = p;
  // column sums of K∘Z for the band check (the batch-wide buffer is grown on first use;
  // gpx_batch_lml_grad checked the allocation before launching anything)
  (void)hipMemsetAsync(bt->bres, 0, sizeof(double) * (size_t)bt->B * Np, r.s);
  ca.colsum = bt->bres; ca.sCol = Np;
  launch_band_contract(ca, max_terms, r.na, r.s);
  launch_band_check(r.d_act, bt->bres, Np, bt->d_n, bt->results, r.na, Np, r.s);
  ReduceArgs ra{};
  ra.active = r.d_act; ra.partial = bt->partial; ra.sPartial = bt->partial_stride;
  ra.ntiles = (p + 1) * nb; ra.z = bt->z; ra.sVec = Np; ra.ldiag = bt->ldiag;
  ra.nvalid = bt->d_n; ra.specs = bt->d_specs; ra.results = bt->results; ra.Np = Np;
  launch_reduce(ra, r.na, r.s);
}

// Routing of one evaluation call: the block-banded path when K and every ∂K/∂θ vanish exactly
// beyond a band of p <= band_limit 64-blocks at this θ (gpx_band.hip), the dense recursion
// otherwise. p <= 2 problems whose band is at most band16_limit 16-blocks take the band16
// sweeps (grouped by width Q), other p <= 2 problems the 64-row fused sweeps; band storage runs
// everything else on its dense fallback slots. Pure host logic over the band tables (writes
// h_bandp; tests/c/host_harness.cpp runs it under ASan/UBSan).
RouteLimits route_limits(const gpx_batch* bt) {
  RouteLimits L;
  L.plim = band_limit(bt);
  if (bt->compact) L.plim = std::min(L.plim, kBandStoreP);
  const char* ef = getenv("GPX_BAND_FUSED");  // 0: p <= 2 problems take the per-block launches too
  L.fused_on = !(ef && atoi(ef) == 0);
  L.q16lim = L.fused_on ? band16_limit(bt) : -1;
  // the widest SE1 band16 class (GPX_BAND16_QMAX, default kBand16MaxQ): only with both sweeps
  // computing K's tiles inline
  const char* eq = getenv("GPX_BAND16_QMAX");
  L.q16wide = b16_inline_k() == 3 ? std::min(kBand16MaxQ, eq ? atoi(eq) : kBand16MaxQ) : kBand16MaxQAny;
  return L;
}

// one problem's path at θ (route_call and gpx_batch_band_class)
RouteKind route_one(const gpx_batch* bt, int b, const double* thb, const RouteLimits& L, int& w) {
  const int p = L.plim >= 0 ? band_width(bt, b, thb) : -1;
  w = p;
  if (p >= 0 && p <= L.plim) {
    // p <= 2 problems whose band is at most kBand16MaxQ 16-blocks: the band16 sweeps
    int q16 = (p <= 2 && L.q16lim > 0) ? band_width16(bt, b, thb) : -1;
    // Q = 6..8 (a one-wave sweep whose window fills the register file): SE1 problems whose K
    // tiles both sweeps compute inline (their LDS holds no K tiles), up to GPX_BAND16_QMAX
    if (q16 > kBand16MaxQAny && !(q16 <= L.q16wide && se1_spec(bt->specs[b]))) q16 = -1;
    if (q16 >= 0 && q16 <= L.q16lim) {
      w = std::max(q16, 1);
      return kRouteBand16;
    }
    // (the p = 2 sweep holds four 64x64 LDS blocks plus three 64·D X-row slots: <= 160 KiB)
    if (L.fused_on && (p <= 1 || (p == 2 && bt->D <= 12))) return kRouteFused;
    return bt->compact ? kRouteShadow : kRouteBand;  // band storage runs the fused sweeps only
  }
  return bt->compact ? kRouteShadow : kRouteDense;   // (band storage: dense on the fallback slots)
}

void route_call(gpx_batch* bt, int n_active, const int32_t* active, const double* theta, Route& rt,
                int q16wide_cap) {
  std::vector<int32_t>& order = rt.order;
  order.clear();
  order.reserve(n_active);
  rt.shadow_ids.clear();
  std::vector<int32_t> band_ids, fused_ids;
  int pband = 0;
  RouteLimits L = route_limits(bt);
  L.q16wide = std::min(L.q16wide, q16wide_cap);
  std::vector<int32_t> b16_ids[kBand16MaxQ + 1];  // band16 class by width Q (16-blocks)
  bool b16_p2 = false;                             // ... holding p = 2 problems (K band of 3 diagonals)
  for (int i = 0; i < n_active; ++i) {
    const int b = active[i];
    const double* thb = theta + (size_t)b * GPX_THETA_STRIDE;
    int w = -1;
    switch (route_one(bt, b, thb, L, w)) {
      case kRouteBand16:
        bt->h_bandp[b] = w;
        b16_ids[w].push_back(b);
        b16_p2 = b16_p2 || band_width(bt, b, thb) == 2;
        break;
      case kRouteFused:
        bt->h_bandp[b] = w;
        fused_ids.push_back(b);
        break;
      case kRouteBand:
        bt->h_bandp[b] = w;
        band_ids.push_back(b);
        pband = std::max(pband, w);
        break;
      case kRouteShadow:
        if (w >= 0 && w <= L.plim) bt->h_bandp[b] = w;
        rt.shadow_ids.push_back(b);
        break;
      default:
        order.push_back(b);
    }
  }
  rt.n16 = 0;
  for (int q = 1; q <= kBand16MaxQ; ++q) rt.n16 += (int)b16_ids[q].size();
  rt.n_dense = (int)order.size();
  rt.n_band = (int)band_ids.size();
  rt.n_fused = (int)fused_ids.size() + rt.n16;
  rt.pband = pband;
  rt.b16_p2 = b16_p2;
  order.insert(order.end(), band_ids.begin(), band_ids.end());
  // fused problems: the band16 class first (by width), then p <= 1 (its own two-blocks-per-CU
  // kernels), then p = 2
  rt.n_g16 = 0;
  for (int q = 1; q <= kBand16MaxQ; ++q)
    if (!b16_ids[q].empty()) {
      order.insert(order.end(), b16_ids[q].begin(), b16_ids[q].end());
      rt.g16_q[rt.n_g16] = q;
      rt.g16_n[rt.n_g16++] = (int)b16_ids[q].size();
    }
  rt.n_fused1 = 0;
  for (int b : fused_ids)
    if (bt->h_bandp[b] <= 1) order.push_back(b), ++rt.n_fused1;
  for (int b : fused_ids)
    if (bt->h_bandp[b] > 1) order.push_back(b);
}

// Band width <= 2 blocks: the whole sweep per problem in two fused kernels (gpx_band.hip),
// each problem with its own p (d_bandp); K's band is built for the widest.
double band_fused_flops(int Np, int p, bool fwd) {
  const double U = 2.0 * kLeaf * kLeaf * kLeaf;  // one 64³ block product
  const int nb = Np / kLeaf;
  double f = 0.0;
  for (int k = 0; k < nb; ++k) {
    const double q = std::min(p, nb - 1 - k);
    f += fwd ? (2.0 / 3.0 + q + q * (q + 1) / 2.0) * U   // leaf, panels, window update
             : (1.0 + q + q * q + q) * U;               // WᵀW, G, Z panel, Gᵀ Z
  }
  return f;
}

// MFMA flops the band16 sweeps issue per problem (2·16³ per 16x16x16 tile product; the leaves'
// 16x16 factorisations are VALU work and not counted)
double band16_flops(int Np, int Q, bool fwd) {
  const double U = 2.0 * 16 * 16 * 16;
  const int nb = Np / 16;
  double f = 0.0;
  for (int k = 0; k < nb; ++k) {
    const double q = std::min(Q, nb - 1 - k);
    f += fwd ? (q + q * (q + 1) / 2.0) * U          // panels, window update
             : (q + q * q + 1.0 + q) * U;           // G, Z panel, WᵀW, GᵀZ
  }
  return f;
}

// which SE1 band16 sweeps compute their K tiles from X (bit 0: forward, bit 1: backward;
// GPX_B16_INLINE_K, read once): a sweep that does not reads K's band. Same bits every way.
// the same for the wide launch of a deferred part (GPX_B16_INLINE_K_WIDE, default: as above)
int b16_inline_k_wide() {
  static const int kin = [] {
    const char* e = getenv("GPX_B16_INLINE_K_WIDE");
    return e ? (atoi(e) & 3) : b16_inline_k();
  }();
  return kin;
}

// the widest band16 class a deferred part's wide launch takes: 5, or 8 (GPX_WIDE_QMAX, default
// 8) for SE1 parts whose sweeps compute K inline
int wide_qmax(bool se1) {
  static const int wq = [] {
    const char* e = getenv("GPX_WIDE_QMAX");
    return e ? std::max(5, std::min(8, atoi(e))) : 8;
  }();
  return (se1 && b16_inline_k_wide() == 3) ? wq : 5;
}

// band16 widths Q > kBcrMaxQ (6..8) by the block-cyclic-reduction chain of block size 128
// (gpx_bcr.hip bcrw_*; GPX_WIDE_BCR): 1 (default) in calls on the reduction route (the batch's
// band route "bcr": latency — before round 6 these widths went to the 64-row sweeps there),
// 2 in every call, 0 never. Measured in the C2 bench's layout (8 host processes, thousands of
// problems in flight) mode 2 loses 35 % with deferral and 12 % without (profiles/r06_ab.md: the
// chain's 8-wave, 150 KB-LDS workgroups wait for an empty CU behind the other processes' sweeps),
// so the sweeps route keeps its one-wavefront Q = 6..8 sweeps. Either way a problem's path is a
// function of its own width and the batch's route, never of the call.
// GPX_SLOW_DIRECT (default 0 until measured): a deferred part's results written by its gather
// kernel into coherent pinned host buffers instead of two copy-engine downloads
static bool slow_direct() {
  static const bool on = [] {
    const char* e = getenv("GPX_SLOW_DIRECT");
    return e && atoi(e) != 0;
  }();
  return on;
}

int wide_bcr_mode() {
  static const int m = [] {
    const char* e = getenv("GPX_WIDE_BCR");
    return e ? std::max(0, std::min(2, atoi(e))) : 1;
  }();
  return m;
}
bool wide_bcr_on(bool bcr_route) { return wide_bcr_mode() == 2 || (wide_bcr_mode() == 1 && bcr_route); }

// the widest class a deferred part's wide launch (band16_wide_kernel) takes (deferred parts
// exist on the sweeps route only)
static int wide_launch_qmax(bool se1) { return wide_bcr_on(false) ? std::min(wide_qmax(se1), kBcrMaxQ) : wide_qmax(se1); }

// reduction workspace of band16 groups g0 .. g1-1 (each problem in slots of its group's layout)
long long bcr_ws_need(const int* q, const int* cnt, int g0, int g1, int Nmax) {
  long long t = 0;
  for (int g = g0; g < g1; ++g) t += (long long)cnt[g] * bcr_ws_doubles(q[g], Nmax);
  return t;
}

int b16_inline_k() {
  static const int kin = [] {
    const char* e = getenv("GPX_B16_INLINE_K");
    return e ? (atoi(e) & 3) : 3;  // default: both (round 4: +4-7 % on the C2 bench, K's band never in HBM)
  }();
  return kin;
}

// the reference's kernel: one SquaredExponential term on one input column (the band16 sweeps'
// straight-line contraction, and the only family of the Q > kBand16MaxQAny classes)
bool se1_spec(const gpx_kernel_spec& sp) {
  return sp.n_terms == 1 && sp.terms[0].kind == GPX_SE && sp.terms[0].dim_count == 1;
}

// the most band16 problems a call may hold for them to take the block-cyclic-reduction path
// (gpx_bcr.hip) instead of the one-wavefront sweeps: the batch's route (gpx_batch_set_band_route:
// sweeps 0, BCR every call, AUTO GPX_BCR_MAX or 32), unless GPX_BCR_MAX is set, which overrides
// it for the whole process (read per call: a process can compare the paths)
static int bcr_max_problems(const gpx_batch* bt) {
  const char* e = getenv("GPX_BCR_MAX");
  if (e) return atoi(e);
  switch (bt->band_route) {
    case GPX_BAND_ROUTE_BCR: return 1 << 30;
    case GPX_BAND_ROUTE_AUTO: return 32;
    default: return 0;
  }
}

// stream-order markers in the wave trace (diagnostic; no-op unless gpx_batch_wave_trace is on):
// 38 submit reached the device, 39 rebind gather done, 40 band16 work starts, 43 a lane's K band
// built, 41 the lanes joined, 42 reduce done, 44 the results' download done
static void trace_mark(gpx_batch* bt, int kind, hipStream_t s) {
  if (bt->d_wtrace) launch_wave_marker(bt->d_wtrace, bt->d_wtrace_n, bt->wtrace_cap, kind, s);
}

int band_fused_eval(const Run& r, int n16, int n_g16, const int* g16_q, const int* g16_n, bool se1, int kband16,
                     int n1, int max_terms, hipEvent_t* ev, hipEvent_t (*ev16)[4]) {
  // r's active range is [band16 problems (n16, by width group) | p <= 1 problems (n1) | p = 2
  // problems]; the p = 2 class runs as a separate launch pair on an auxiliary stream concurrently
  gpx_batch* bt = r.bt;
  const int Np = bt->Np;
  const long long st = mat_stride(bt);
  const int nlo = n16 + n1;  // the classes whose K band is two 64-block diagonals
  // K's band is built per class on that class's stream (2 block diagonals for p <= 1, 3 for
  // p = 2), so the p <= 1 build does not pay for the wider class and the two overlap
  BuildArgs ba{};
  ba.active = r.d_act; ba.specs = bt->d_specs; ba.theta = r.theta ? r.theta : bt->d_theta; ba.nvalid = bt->d_n;
  ba.X = bt->X; ba.sX = (long long)bt->Nmax * bt->D; ba.X2 = bt->X; ba.sX2 = ba.sX; ba.D = bt->D;
  ba.m2 = 0; ba.out = bt->K; ba.sOut = st; ba.ldo = mat_ld(bt); ba.rows = ba.cols = Np;
  ba.symmetric = 1;
  BandFusedArgs fa{};
  fa.active = r.d_act; fa.bandp = r.bandp ? r.bandp : bt->d_bandp; fa.K = bt->K; fa.L = bt->L; fa.W = bt->W; fa.sMat = st;
  fa.Y = bt->Y; fa.sY = bt->Nmax; fa.nvalid = bt->d_n; fa.z = bt->z; fa.alpha = bt->alpha;
  fa.ldiag = bt->ldiag; fa.sVec = Np; fa.X = bt->X; fa.sX = (long long)bt->Nmax * bt->D; fa.D = bt->D;
  fa.specs = bt->d_specs; fa.theta = r.theta ? r.theta : bt->d_theta; fa.partial = bt->partial;
  fa.sPartial = bt->partial_stride;
  fa.info = r.info ? r.info : bt->d_info; fa.results = bt->results; fa.Np = Np; fa.ld = mat_ld(bt);
  fa.wtrace = bt->d_wtrace; fa.wtrace_n = bt->d_wtrace_n; fa.wtrace_cap = bt->wtrace_cap;
  // The width classes of the call are independent: each class's chain (its K band build, then
  // its sweeps) is a *lane*, and the lanes run concurrently — the largest on the call's stream,
  // the others on the batch's auxiliary streams, joined before the reduction. Serialised on one
  // stream (GPX_BAND_LANES=0, the round-3 order) every class's sweeps — about the same latency
  // whatever their problem count — followed each other, so a call lasted ~2 sweeps per class
  // while the small classes held few waves.
  // Lane kinds: band16 width group g (K's band as its sweeps read it: the 16-row tiles (m, m − d),
  // d <= Q; kband16 — 2, or 3 when the class holds p = 2 problems — still tells the sweeps which
  // entries are exact zeros by the 64-row bound), the 64-row p <= 1 class (two 64-block
  // diagonals), the 64-row p = 2 class (three).
  const int wq = wide_qmax(se1);  // the widest class a deferred part's wide launch takes
  struct Lane { int kind, g, n, off, g_end; long long wso; };
  Lane lanes[kBand16MaxQ + 2];
  int nl = 0;
  {
    int off = 0;
    long long wso = 0;  // (the reduction lanes' workspace offsets, in group order)
    // (r.bcr_q: each band16 width group as a block-cyclic-reduction chain of its own width,
    // gpx_bcr.hip: a problem's arithmetic depends on its own width only, not on the call's mix)
    int g = 0;
    for (; g < n_g16 && r.bcr_q > 0 && g16_q[g] <= kBcrMaxQ; ++g) {
      lanes[nl++] = Lane{4, g, g16_n[g], off, g + 1, wso};
      off += g16_n[g];
      wso += (long long)g16_n[g] * bcr_ws_doubles(g16_q[g], bt->Nmax);
    }
    for (; g < n_g16; ++g) {
      if (wide_bcr_on(r.bcr_q > 0) && g16_q[g] > kBcrMaxQ) {
        // the widths 6..8 (always the tail of the groups) as ONE reduction chain of block size 128
        if (nl > 0 && lanes[nl - 1].kind == 5) {
          lanes[nl - 1].n += g16_n[g];
          lanes[nl - 1].g_end = g + 1;
        } else {
          lanes[nl++] = Lane{5, g, g16_n[g], off, g + 1, wso};
        }
        wso += (long long)g16_n[g] * bcr_ws_doubles(g16_q[g], bt->Nmax);
        if (bt->ctx->profiling) bt->timing.bcr_wide_evals += g16_n[g];
      } else if (r.wide_from > 0 && se1 && g16_q[g] >= std::max(r.wide_from, 4) && g16_q[g] <= wq && nl > 0 &&
          lanes[nl - 1].kind == 3) {
        // (r.wide_from: the SE1 groups of width 4 and 5 as one lane, one band16_wide_kernel launch)
        lanes[nl - 1].n += g16_n[g];
        lanes[nl - 1].g_end = g + 1;
      } else if (r.wide_from > 0 && se1 && g16_q[g] >= std::max(r.wide_from, 4) && g16_q[g] <= wq) {
        lanes[nl++] = Lane{3, g, g16_n[g], off, g + 1, 0};
      } else {
        lanes[nl++] = Lane{0, g, g16_n[g], off, g + 1, 0};
      }
      off += g16_n[g];
    }
    if (n1 > 0) lanes[nl++] = Lane{1, 0, n1, n16, 0, 0};
    if (nlo < r.na) lanes[nl++] = Lane{2, 0, r.na - nlo, nlo, 0, 0};
  }
  // GPX_LANE_ORDER=1: the small (slow-class) lanes are enqueued first, ahead of the bulk lane,
  // so their wavefronts reach the dispatcher before the bulk lane's fill the chip
  static const int lane_order = [] {
    const char* e = getenv("GPX_LANE_ORDER");
    return e ? atoi(e) : 0;
  }();
  {  // the reduction lanes' workspace (grow-only; their offsets were laid out in group order)
    long long need = 0;
    for (int i = 0; i < nl; ++i)
      if (lanes[i].kind == 4 || lanes[i].kind == 5)
        need = std::max(need, lanes[i].wso + (long long)lanes[i].n *
                                  bcr_ws_doubles(lanes[i].kind == 5 ? kBcrWideQ : g16_q[lanes[i].g], bt->Nmax));
    if (need > 0 && (size_t)need > *r.bcr_capp) {  // (grown with headroom: each regrowth frees, which synchronises)
      const int e = ensure(bt->ctx, *r.bcr_wsp, *r.bcr_capp, (size_t)need * 3 / 2);
      if (e != GPX_OK) return e;
    }
  }
  std::sort(lanes, lanes + nl, [](const Lane& x, const Lane& y) { return x.n > y.n; });
  if (lane_order == 1 && nl > 1) std::rotate(lanes, lanes + 1, lanes + nl);  // bulk lane last (on an aux stream)
  trace_mark(bt, 40, r.s);
  static const bool lanes_on = [] {
    const char* e = getenv("GPX_BAND_LANES");
    return !(e && atoi(e) == 0);
  }();
  // which SE1 band16 sweeps compute their K tiles from X (bit 0: forward, bit 1: backward;
  // GPX_B16_INLINE_K): a sweep that does not reads K's band — written by band16_build_kernel
  // when the forward reads it too, by the forward itself when only the backward reads it (1:
  // each K tile's exp once, the band through HBM once each way). Same bits every way.
  static const int kin = b16_inline_k();
  // the same for the wide launch (the Q = 4, 5 classes of a deferred part, one wavefront per SIMD:
  // there the exp on each sweep's chain costs more than a build launch; GPX_B16_INLINE_K_WIDE,
  // default: as GPX_B16_INLINE_K)
  static const int kin_wide = b16_inline_k_wide();
  // GPX_BAND_LANE_STREAMS: streams the lanes are spread over (the bulk lane alone on the call's
  // stream, the others round-robin on the rest). A process gets GPU_MAX_HW_QUEUES hardware
  // queues (the bench: 2, so that 8 processes stay within the 16 the GPU maps without
  // time-slicing) and streams beyond that share queues, where their kernels run in order
  static const int lane_streams = [] {
    const char* e = getenv("GPX_BAND_LANE_STREAMS");
    return e ? std::max(1, atoi(e)) : 1 + kAux;
  }();
  const int nstreams = (lanes_on && !r.one_stream) ? std::min(std::min(nl, 1 + kAux), lane_streams) : 1;
  auto lane_stream = [&](int i) { return (i == 0 || nstreams == 1) ? r.s : bt->aux[(i - 1) % (nstreams - 1)]; };
  const bool bcr_timed = r.bcr_q > 0 && bt->ctx->profiling && bt->bcr_ev[0];
  if (bcr_timed) (void)hipEventRecord(bt->bcr_ev[0], r.s);
  if (nstreams > 1) {
    (void)hipEventRecord(bt->ev[kEvents - 2], r.s);   // the call's uploads are in
    for (int i = 1; i < nstreams; ++i) (void)hipStreamWaitEvent(bt->aux[i - 1], bt->ev[kEvents - 2], 0);
  }
  for (int i = 0; i < nl; ++i) {
    const Lane& l = lanes[i];
    hipStream_t ls = lane_stream(i);
    if (l.kind == 0) {
      // SE1 classes compute their K tiles inside the sweeps (band16 KIN): no build launch (a
      // forward computing them while the backward reads the band writes the band itself). The
      // Q > kBand16MaxQAny classes hold SE1 problems only and always compute K inline, whatever
      // the rest of the call holds (se1 is the whole call's), so they never need the build.
      if (!(se1 && (kin & 1)) && g16_q[l.g] <= kBand16MaxQAny) {
        BuildArgs bg = ba;
        bg.active = r.d_act + l.off;
        launch_band16_build(bg, g16_q[l.g], l.n, ls);
        trace_mark(bt, 43, ls);
      }
      BandFusedArgs f16 = fa;
      f16.kband = kband16;
      f16.active = r.d_act + l.off;
      f16.kstore = se1 && (kin & 1) && !(kin & 2);
      launch_band16(f16, g16_q[l.g], max_terms, se1, kin, l.n, ls, ev16 ? ev16[l.g - r.ev16_g0] : nullptr);
    } else if (l.kind == 3) {
      // the wide SE1 groups: their K bands (unless computed in the sweeps), then one launch
      int goff = l.off;
      for (int g = l.g; g < l.g_end; ++g) {
        if (!(kin_wide & 1)) {
          BuildArgs bg = ba;
          bg.active = r.d_act + goff;
          launch_band16_build(bg, g16_q[g], g16_n[g], ls);
        }
        goff += g16_n[g];
      }
      BandFusedArgs f16 = fa;
      f16.kband = kband16;
      f16.active = r.d_act + l.off;
      f16.kstore = (kin_wide & 1) && !(kin_wide & 2);
      if (ev16)
        for (int g = l.g + 1; g < l.g_end; ++g) (void)hipEventRecord(ev16[g - r.ev16_g0][0], ls);
      launch_band16_wide(f16, kin_wide, l.n, ls, ev16 ? ev16[l.g - r.ev16_g0] : nullptr, g16_q[l.g_end - 1]);
      if (ev16)
        for (int g = l.g + 1; g < l.g_end; ++g)
          for (int e = 1; e < 4; ++e) (void)hipEventRecord(ev16[g - r.ev16_g0][e], ls);
    } else if (l.kind == 4 || l.kind == 5) {
      // a reduction chain: the group's width (kind 4), or the widths 6..8 at block size 128 (kind 5)
      const int qc = l.kind == 5 ? kBcrWideQ : g16_q[l.g];
      BcrArgs ca{};
      ca.active = r.d_act + l.off; ca.specs = bt->d_specs; ca.theta = fa.theta; ca.nvalid = bt->d_n;
      ca.X = bt->X; ca.sX = (long long)bt->Nmax * bt->D; ca.D = bt->D; ca.Y = bt->Y; ca.sY = bt->Nmax;
      // (workspace: the lane's problems in slots of its layout, at the lane's offset)
      ca.sWs = bcr_ws_doubles(qc, bt->Nmax);
      ca.ws = *r.bcr_wsp + l.wso; ca.info = fa.info;
      ca.z = bt->z; ca.ldiag = bt->ldiag; ca.alpha = bt->alpha; ca.sVec = Np; ca.Np = Np;
      ca.Kd = bt->K; ca.sMat = st; ca.ld = mat_ld(bt);
      ca.partial = bt->partial; ca.sPartial = bt->partial_stride; ca.results = bt->results;
      launch_bcr(ca, qc, max_terms, l.n, bt->Nmax, ls, &bt->bcr_graphs);
    } else if (l.kind == 1) {
      BuildArgs b1 = ba;
      b1.active = r.d_act + l.off;
      b1.band1 = 2;
      launch_build(b1, l.n, ls);
      BandFusedArgs f1 = fa;
      f1.active = r.d_act + l.off;
      launch_band_fused1(f1, max_terms, l.n, ls, ev);
    } else {
      BuildArgs b2 = ba;
      b2.active = r.d_act + l.off;
      b2.band1 = 3;
      launch_build(b2, l.n, ls);
      BandFusedArgs f2 = fa;
      f2.active = r.d_act + l.off;
      launch_band_fused(f2, max_terms, l.n, ls, n1 == 0 ? ev : nullptr);
    }
  }
  for (int i = 1; i < nstreams; ++i) {
    (void)hipEventRecord(bt->ev[kEvents - 4 - i], bt->aux[i - 1]);
    (void)hipStreamWaitEvent(r.s, bt->ev[kEvents - 4 - i], 0);
  }
  if (bcr_timed) (void)hipEventRecord(bt->bcr_ev[1], r.s);
  trace_mark(bt, 41, r.s);
  ReduceArgs ra{};
  ra.active = r.d_act; ra.partial = bt->partial; ra.sPartial = bt->partial_stride;
  ra.ntiles = 1; ra.z = bt->z; ra.sVec = Np; ra.ldiag = bt->ldiag;
  ra.nvalid = bt->d_n; ra.specs = bt->d_specs; ra.results = bt->results; ra.Np = Np;
  launch_reduce(ra, r.na, r.s);
  trace_mark(bt, 42, r.s);
  return GPX_OK;
}

// The batch's auxiliary streams (the forked T products of the recursion) take the priority of
// the stream the caller evaluates on, so a batch submitted on a high-priority stream is high
// priority throughout. Called at the start of an evaluation, when the aux streams are idle (the
// previous evaluation joined them before returning).
int match_aux_priority(gpx_batch* bt, hipStream_t s) {
  int p = 0;
  if (hipStreamGetPriority(s, &p) != hipSuccess) p = 0;
  if (p == bt->aux_priority) return GPX_OK;
  for (int g = 0; g < kAux; ++g) {
    if (bt->aux[g]) HIPX(bt->ctx, hipStreamDestroy(bt->aux[g]));
    bt->aux[g] = nullptr;
    HIPX(bt->ctx, hipStreamCreateWithPriority(&bt->aux[g], hipStreamNonBlocking, p));
  }
  bt->aux_priority = p;
  return GPX_OK;
}

// pinned n[] / specs[] mirrors and the dirty flags of the deferred rebinds (first rebind)
int ensure_rebind_meta(gpx_batch* bt) {
  gpx_ctx* ctx = bt->ctx;
  if (!bt->h_nmeta) {
    HIPX(ctx, hipHostMalloc(&bt->h_nmeta, sizeof(int) * bt->B, hipHostMallocNonCoherent));
    HIPX(ctx, hipHostMalloc(&bt->h_specs, sizeof(DevSpec) * bt->B, hipHostMallocNonCoherent));
  }
  if (bt->dirty.empty()) {
    bt->dirty.assign(bt->B, 0);
    bt->n_dirty = 0;
  }
  return GPX_OK;
}

// remember slot b's per-block X boxes (rows of its valid blocks; the rest of the slot's row
// is left as it was)
void keep_slot_box(gpx_batch* bt, int b, const double* box) {
  const int nbx = (bt->Nmax + kBox - 1) / kBox;
  const size_t row = (size_t)nbx * bt->D * 2;
  if (bt->slot_box.empty()) {
    bt->slot_box.assign(row * bt->B, 0.0);
    bt->slot_box_ok.assign(bt->B, 0);
  }
  const int nvb = (bt->n[b] + kBox - 1) / kBox;
  std::memcpy(bt->slot_box.data() + row * b, box, sizeof(double) * (size_t)nvb * bt->D * 2);
  bt->slot_box_ok[b] = 1;
}

// GPX_SUBMIT_STATS: wall-clock phase accumulators of the submit/complete calls (host profiling)
static bool submit_stats_on() {
  static const bool on = [] {
    const char* e = getenv("GPX_SUBMIT_STATS");
    return e && atoi(e) != 0;
  }();
  return on;
}
void print_submit_stats(const gpx_batch* bt) {
  fprintf(stderr, "[gpx submit stats] batch B=%d calls=%lld flush=%.3f route=%.3f upload=%.3f launch=%.3f "
          "download=%.3f complete_sync=%.3f (flush: wait_io=%.3f box_sync=%.3f over %lld syncs) "
          "predict=%.3f (io wait %.3f, shadow slots %.3f, %.0f shadow predicts) s\n", bt->B,
          bt->sub_calls, bt->sub_s[0], bt->sub_s[1], bt->sub_s[2], bt->sub_s[3], bt->sub_s[4], bt->sub_s[5],
          bt->sub_s[6], bt->sub_s[7], bt->box_syncs, bt->sub_s[8], bt->sub_s[9], bt->sub_s[10],
          bt->timing.shadow_predicts);
}
struct SubClock {
  gpx_batch* bt;
  bool on;
  std::chrono::steady_clock::time_point t;
  explicit SubClock(gpx_batch* b) : bt(b), on(submit_stats_on()) {
    if (on) t = std::chrono::steady_clock::now();
  }
  void skip() {
    if (on) t = std::chrono::steady_clock::now();
  }
  void lap(int i) {
    if (!on) return;
    const auto n = std::chrono::steady_clock::now();
    bt->sub_s[i] += std::chrono::duration<double>(n - t).count();
    t = n;
  }
};

int wait_io(gpx_batch* bt) {
  if (!bt->io_pending) return GPX_OK;
  gpx_ctx* ctx = bt->ctx;
  HIPX(ctx, hipEventSynchronize(bt->io_ev));
  bt->io_pending = false;
  return GPX_OK;
}

// An asynchronous predict (predict_impl, `async`) left kernels in flight on bt->io_stream that
// read the batch's device I/O block, n / specs and the predicted slots' factors. Every later
// writer of that state on another stream (the uploads and rebind gathers of the next call, and
// through their order that call's kernels, which overwrite the factors of rebound slots) first
// waits for those kernels on the device — no host synchronisation. On the same stream the order
// is already the stream's.
int fence_io(gpx_batch* bt, hipStream_t s) {
  if (!bt->io_pending || bt->io_stream == s) return GPX_OK;
  HIPX(bt->ctx, hipStreamWaitEvent(s, bt->io_ev, 0));
  return GPX_OK;
}

int flush_rebinds(gpx_batch* bt, hipStream_t s) {
  if (bt->n_dirty == 0 && bt->pend.empty()) return GPX_OK;
  gpx_ctx* ctx = bt->ctx;
  {
    const int e = fence_io(bt, s);
    if (e != GPX_OK) return e;
  }
  SubClock fc(bt);
  {
    const int e = wait_io(bt);
    if (e != GPX_OK) return e;
  }
  fc.lap(6);
  {
    const int rc = ensure_rebind_meta(bt);
    if (rc != GPX_OK) return rc;
  }
  const size_t nx = (size_t)bt->Nmax * bt->D, ny = bt->Nmax;
  const int nbx = (bt->Nmax + kBox - 1) / kBox;
  if (!bt->h_rdesc) {
    HIPX(ctx, hipHostMalloc(&bt->h_rdesc, sizeof(RebindDesc) * bt->B, hipHostMallocCoherent));
    HIPX(ctx, hipMalloc(&bt->d_box, sizeof(double) * (size_t)bt->B * nbx * bt->D * 2));
    HIPX(ctx, hipHostMalloc(&bt->h_box, sizeof(double) * (size_t)bt->B * nbx * bt->D * 2, hipHostMallocNonCoherent));
  }
  // host-staged slots: DMA from their pinned regions (non-coherent host memory: DMA, not
  // kernel reads, is what sees the CPU's writes whole)
  for (int b = 0; b < bt->B && bt->n_dirty > 0; ++b) {
    if (!bt->dirty[b]) continue;
    const double* hx = bt->h_stage + (size_t)b * bt->stage_stride;
    HIPX(ctx, hipMemcpyAsync(const_cast<double*>(bt->X) + (size_t)b * nx, hx, sizeof(double) * nx,
                             hipMemcpyHostToDevice, s));
    HIPX(ctx, hipMemcpyAsync(const_cast<double*>(bt->Y) + (size_t)b * ny, hx + nx, sizeof(double) * ny,
                             hipMemcpyHostToDevice, s));
    bt->dirty[b] = 0;
    --bt->n_dirty;
  }
  bt->n_dirty = 0;
  // device sources: one gather kernel for all of them (descriptors in coherent pinned memory),
  // which also returns their X boxes for the band tables
  int m = 0;
  const bool tables = band_shape(bt);
  int nbox = 0;
  for (const auto& e : bt->pend)
    bt->h_rdesc[m++] = RebindDesc{e.x, e.y, const_cast<double*>(bt->X) + (size_t)e.b * nx,
                                  const_cast<double*>(bt->Y) + (size_t)e.b * ny, e.n,
                                  tables && !e.boxed ? nbox++ : -1};
  for (auto& w : bt->rebind_waits)  // the device sources' producers (gpx_batch_rebind_device)
    if (w.armed) {
      if (w.s != s) HIPX(ctx, hipStreamWaitEvent(s, w.ev, 0));
      w.armed = false;
    }
  if (m > 0) {
    launch_rebind_gather(bt->h_rdesc, m, bt->Nmax, bt->D, bt->d_box, s);
    HIPX(ctx, hipGetLastError());
  }
  if (nbox > 0) {
    const size_t row = (size_t)nbx * bt->D * 2;
    HIPX(ctx, hipMemcpyAsync(bt->h_box, bt->d_box, sizeof(double) * row * nbox, hipMemcpyDeviceToHost, s));
    fc.skip();
    HIPX(ctx, hipStreamSynchronize(s));
    fc.lap(7);
    ++bt->box_syncs;
    int i = 0;
    for (const auto& e : bt->pend) {
      if (e.boxed) continue;
      const double* box = bt->h_box + row * i++;
      band_tables_boxes(bt, e.b, box);
      keep_slot_box(bt, e.b, box);
    }
  }
  bt->pend.clear();
  for (int b = 0; b < bt->B; ++b) {
    bt->h_nmeta[b] = bt->n[b];
    std::memcpy(&bt->h_specs[b], &bt->specs[b], sizeof(DevSpec));
  }
  HIPX(ctx, hipMemcpyAsync(bt->d_n, bt->h_nmeta, sizeof(int) * bt->B, hipMemcpyHostToDevice, s));
  HIPX(ctx, hipMemcpyAsync(bt->d_specs, bt->h_specs, sizeof(DevSpec) * bt->B, hipMemcpyHostToDevice, s));
  return GPX_OK;
}

// the active set and every active row's θ (kernel parameters + σn²: finite and > 0)
int check_active_theta(gpx_batch* bt, int n_active, const int32_t* active, const double* theta) {
  gpx_ctx* ctx = bt->ctx;
  if (n_active <= 0 || n_active > bt->B || !active || !theta)
    return fail(ctx, GPX_BAD_ARG, "bad active set / theta");
  for (int i = 0; i < n_active; ++i)
    if (active[i] < 0 || active[i] >= bt->B) return fail(ctx, GPX_BAD_ARG, "active index out of range");
  for (int i = 0; i < n_active; ++i) {
    const int b = active[i];
    const int np = bt->specs[b].n_params;
    for (int p = 0; p <= np; ++p) {
      const double v = theta[(size_t)b * GPX_THETA_STRIDE + p];
      if (!(v > 0.0) || !std::isfinite(v))
        return fail(ctx, GPX_BAD_ARG, "theta must be finite and > 0 (constrained space)");
    }
  }
  return GPX_OK;
}

int upload_common(gpx_batch* bt, int n_active, const int32_t* active, const double* theta,
                  hipStream_t s, bool predict_block) {
  gpx_ctx* ctx = bt->ctx;
  {
    const int e = check_active_theta(bt, n_active, active, theta);
    if (e != GPX_OK) return e;
  }
  {
    const int e = flush_rebinds(bt, s);
    if (e != GPX_OK) return e;
  }
  {  // (the rebind flush above host-waits for it when it had work; here without rebinds)
    const int e = fence_io(bt, s);
    if (e != GPX_OK) return e;
  }
  // a deferred slow part copies the active list, θ and band widths it runs on out of the I/O
  // block on its own stream: this upload may overwrite them only after those copies
  if (bt->slow_in_armed) HIPX(bt->ctx, hipStreamWaitEvent(s, bt->slow_in, 0));
  char* hio = bt->h_io;
  if (predict_block) {  // (the last asynchronous predict's upload out of it has completed)
    SubClock pc(bt);
    const int e = wait_io(bt);
    pc.lap(9);
    if (e != GPX_OK) return e;
    if (!bt->h_io_pred) HIPX(ctx, hipHostMalloc(&bt->h_io_pred, bt->io_bytes, hipHostMallocNonCoherent));
    hio = bt->h_io_pred;
  }
  // one DMA from the pinned block (allocated non-coherent: the host reads and writes it as
  // ordinary cached memory, the DMAs at the call boundaries see it whole):
  // [active | info = 0 | bandp | theta] (every call ends with a stream synchronize, so the previous call's transfers out of h_io have completed; bandp is
  // written into h_bandp by gpx_batch_lml_grad before this)
  std::memcpy(hio, active, sizeof(int) * n_active);
  std::memset(hio + bt->io_info_off, 0, sizeof(int) * bt->B);
  std::memcpy(hio + bt->io_theta_off, theta, sizeof(double) * GPX_THETA_STRIDE * bt->B);
  HIPX(ctx, hipMemcpyAsync(bt->d_io, hio, bt->io_res_off, hipMemcpyHostToDevice, s));
  return GPX_OK;
}

}  // namespace gpx


extern "C" {

const char* gpx_version(void) { return kVersion; }

int gpx_create(int device, gpx_ctx** out) {
  if (!out) return GPX_BAD_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return GPX_HIP_ERROR;
  if (device < 0 || device >= ndev) return GPX_BAD_ARG;
  if (hipSetDevice(device) != hipSuccess) return GPX_HIP_ERROR;
  gpx_ctx* c = new gpx_ctx();
  c->device = device;
  const bool ok = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess;
  if (!ok) {
    delete c;
    return GPX_HIP_ERROR;
  }
  *out = c;
  return GPX_OK;
}

int gpx_destroy(gpx_ctx* ctx) {
  if (!ctx) return GPX_BAD_ARG;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return GPX_OK;
}

const char* gpx_last_error(const gpx_ctx* ctx) {
  (void)ctx;
  return last_error_slot().c_str();
}

int gpx_set_profiling(gpx_ctx* ctx, int enabled) {
  if (!ctx) return GPX_BAD_ARG;
  ctx->profiling = enabled;
  return GPX_OK;
}

static int batch_create(gpx_ctx* ctx, int B, int N_max, int D, const double* X, const double* Y,
                        const int32_t* n, const gpx_kernel_spec* specs, bool compact, gpx_batch** out) {
  if (!ctx || !out) return GPX_BAD_ARG;
  *out = nullptr;
  if (B <= 0 || N_max <= 0 || D <= 0 || D > GPX_MAX_DIM || !X || !Y || !n || !specs)
    return fail(ctx, GPX_BAD_ARG, "bad batch dimensions or null pointer");
  for (int b = 0; b < B; ++b) {
    if (n[b] < 1 || n[b] > N_max) return fail(ctx, GPX_BAD_ARG, "n[b] must be in [1, N_max]");
    const gpx_kernel_spec& sp = specs[b];
    if (sp.n_terms < 1 || sp.n_terms > GPX_MAX_TERMS || sp.n_params < 1 ||
        sp.n_params >= GPX_THETA_STRIDE)
      return fail(ctx, GPX_BAD_ARG, "bad kernel spec");
    for (int t = 0; t < sp.n_terms; ++t) {
      const gpx_term& tm = sp.terms[t];
      const int np = (tm.kind == GPX_RQ || tm.kind == GPX_PERIODIC_SE) ? 3 : (tm.kind == GPX_LINEAR ? 1 : 2);
      if (tm.kind < GPX_SE || tm.kind > GPX_LINEAR || tm.dim_start < 0 || tm.dim_count < 1 ||
          tm.dim_start + tm.dim_count > D || tm.param_offset < 0 || tm.param_offset + np > sp.n_params)
        return fail(ctx, GPX_BAD_ARG, "bad kernel term");
    }
  }
  if (((long long)N_max + kLeaf - 1) / kLeaf * kLeaf > kGemmMaxLd)
    return fail(ctx, GPX_BAD_ARG, "N_max exceeds the GEMM buffer-load window (kGemmMaxLd)");
  if (compact && (N_max < 8 * kLeaf - (kLeaf - 1) || N_max > 8192))
    return fail(ctx, GPX_BAD_ARG, "band storage needs 449 <= N_max <= 8192 (8 to 128 64-blocks)");
  HIPX(ctx, hipSetDevice(ctx->device));
  gpx_batch* bt = new gpx_batch();
  bt->ctx = ctx; bt->B = B; bt->Nmax = N_max; bt->D = D;
  bt->Np = ((N_max + kLeaf - 1) / kLeaf) * kLeaf;
  bt->X = X; bt->Y = Y;
  bt->n.assign(n, n + B);
  bt->specs.assign(specs, specs + B);
  // band storage: rows of ldm + 1 doubles holding columns i − 64·(kBandStoreP+1) .. i + 63
  // (band_c0 = the column offset of the diagonal in a row), plus a 64-double guard
  const long long band_c0 = 64LL * kBandStoreP + 64;
  if (compact) {
    bt->compact = 1;
    bt->ldm = 64 * (kBandStoreP + 2);
    bt->smat = (long long)bt->Np * (bt->ldm + 1);
  }
  const size_t mat = ((size_t)B * mat_stride(bt) + (compact ? 64 : 0)) * sizeof(double);
  const size_t vec = (size_t)B * bt->Np * sizeof(double);
  const int t64 = bt->Np / 64;
  // the dense contraction writes one row of partials per lower 64-tile; the fused band
  // sweeps (band storage's only path) one row per problem
  bt->partial_stride = compact ? GPX_THETA_STRIDE : (long long)t64 * (t64 + 1) / 2 * GPX_THETA_STRIDE;
  auto cleanup = [&](const std::string& m) {
    gpx_batch_destroy(bt);
    return fail(ctx, GPX_HIP_ERROR, m);
  };
  if (hipMalloc(&bt->K, mat) != hipSuccess || hipMalloc(&bt->L, mat) != hipSuccess ||
      hipMalloc(&bt->W, mat) != hipSuccess)
    return cleanup("out of device memory for K/L/W workspace");
  if (hipMalloc(&bt->z, vec) != hipSuccess || hipMalloc(&bt->alpha, vec) != hipSuccess ||
      hipMalloc(&bt->ldiag, vec) != hipSuccess ||
      hipMalloc(&bt->partial, (size_t)B * bt->partial_stride * sizeof(double)) != hipSuccess ||
      hipMalloc(&bt->d_n, sizeof(int) * B) != hipSuccess ||
      hipMalloc(&bt->d_orow, sizeof(int) * B) != hipSuccess ||
      hipMalloc(&bt->d_specs, sizeof(DevSpec) * B) != hipSuccess)
    return cleanup("out of device memory for batch vectors");
  {
    const size_t ints = ((size_t)B * sizeof(int) + 7) / 8 * 8;
    bt->io_info_off = ints;
    bt->io_bandp_off = 2 * ints;
    bt->io_theta_off = 3 * ints;
    bt->io_res_off = bt->io_theta_off + (size_t)B * GPX_THETA_STRIDE * sizeof(double);
    bt->io_flag_off = bt->io_res_off + (size_t)B * kResStride * sizeof(double);
    bt->io_bytes = bt->io_flag_off + ints;
    if (hipMalloc(&bt->d_io, bt->io_bytes) != hipSuccess ||
        hipHostMalloc(&bt->h_io, bt->io_bytes, hipHostMallocNonCoherent) != hipSuccess)
      return cleanup("out of memory for the batch I/O block");
    std::memset(bt->h_io, 0, bt->io_bytes);
    bt->d_active = reinterpret_cast<int*>(bt->d_io);
    bt->d_info = reinterpret_cast<int*>(bt->d_io + bt->io_info_off);
    bt->d_bandp = reinterpret_cast<int*>(bt->d_io + bt->io_bandp_off);
    bt->h_bandp = reinterpret_cast<int*>(bt->h_io + bt->io_bandp_off);
    bt->d_theta = reinterpret_cast<double*>(bt->d_io + bt->io_theta_off);
    bt->results = reinterpret_cast<double*>(bt->d_io + bt->io_res_off);
    bt->h_info = reinterpret_cast<int*>(bt->h_io + bt->io_info_off);
    bt->h_results = reinterpret_cast<double*>(bt->h_io + bt->io_res_off);
  }
  // W and L upper triangles must read as exact zeros (never written afterwards)
  if (hipMemset(bt->W, 0, mat) != hipSuccess || hipMemset(bt->L, 0, mat) != hipSuccess ||
      hipMemset(bt->K, 0, mat) != hipSuccess)
    return cleanup("memset failed");
  if (compact) {
    bt->Kraw = bt->K; bt->Lraw = bt->L; bt->Wraw = bt->W;
    bt->K += band_c0; bt->L += band_c0; bt->W += band_c0;
  }
  for (int g = 0; g < kAux; ++g)
    if (hipStreamCreateWithFlags(&bt->aux[g], hipStreamNonBlocking) != hipSuccess)
      return cleanup("stream creation failed");
  for (int e = 0; e < kEvents; ++e)
    if (hipEventCreateWithFlags(&bt->ev[e], hipEventDisableTiming) != hipSuccess)
      return cleanup("event creation failed");
  std::vector<DevSpec> ds(B);
  for (int b = 0; b < B; ++b) std::memcpy(&ds[b], &specs[b], sizeof(DevSpec));
  static_assert(sizeof(DevSpec) == sizeof(gpx_kernel_spec), "spec layout");
  if (hipMemcpy(bt->d_specs, ds.data(), sizeof(DevSpec) * B, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(bt->d_n, n, sizeof(int) * B, hipMemcpyHostToDevice) != hipSuccess)
    return cleanup("upload failed");
  bt->fac_theta.assign((size_t)B * GPX_THETA_STRIDE, 0.0);
  bt->fac_valid.assign(B, 0);
  bt->fac_band.assign(B, 0);
  bt->band_rmin.assign((size_t)B * GPX_MAX_TERMS * (bt->Np / kLeaf), INFINITY);
  bt->band_tail.assign((size_t)B * GPX_MAX_TERMS, bt->Np / kLeaf);
  if (bt->Np <= kBand16MaxNp) {
    bt->band_rmin16.assign((size_t)B * GPX_MAX_TERMS * (bt->Np / kBox), INFINITY);
    bt->band_tail16.assign((size_t)B * GPX_MAX_TERMS, bt->Np / kBox);
  }
  if (band_shape(bt)) {
    std::vector<double> hx((size_t)B * N_max * D);
    if (hipMemcpy(hx.data(), X, sizeof(double) * hx.size(), hipMemcpyDeviceToHost) != hipSuccess)
      return cleanup("upload failed");
    for (int b = 0; b < B; ++b) band_tables(bt, b, hx.data() + (size_t)b * N_max * D);
  }
  if (compact) {
    // the dense fallback: kShadowSlots ordinary slots with their own X / Y rows
    const size_t nx = (size_t)kShadowSlots * N_max * D, ny = (size_t)kShadowSlots * N_max;
    if (hipMalloc(&bt->shX, nx * sizeof(double)) != hipSuccess ||
        hipMalloc(&bt->shY, ny * sizeof(double)) != hipSuccess ||
        hipMemset(bt->shX, 0, nx * sizeof(double)) != hipSuccess ||
        hipMemset(bt->shY, 0, ny * sizeof(double)) != hipSuccess)
      return cleanup("out of device memory for the dense fallback slots");
    std::vector<int32_t> n1(kShadowSlots, 1);
    std::vector<gpx_kernel_spec> sp1(kShadowSlots, specs[0]);
    const int rc = batch_create(ctx, kShadowSlots, N_max, D, bt->shX, bt->shY, n1.data(), sp1.data(), false,
                                &bt->shadow);
    if (rc != GPX_OK) {
      const std::string m = last_error_slot();
      gpx_batch_destroy(bt);
      return fail(ctx, rc, "dense fallback slots: " + m);
    }
    bt->shadow->force_dense = 1;
  }
  *out = bt;
  return GPX_OK;
}

int gpx_batch_create(gpx_ctx* ctx, int B, int N_max, int D, const double* X, const double* Y,
                     const int32_t* n, const gpx_kernel_spec* specs, gpx_batch** out) {
  return batch_create(ctx, B, N_max, D, X, Y, n, specs, false, out);
}

int gpx_batch_create_banded(gpx_ctx* ctx, int B, int N_max, int D, const double* X, const double* Y,
                            const int32_t* n, const gpx_kernel_spec* specs, gpx_batch** out) {
  return batch_create(ctx, B, N_max, D, X, Y, n, specs, true, out);
}

int gpx_batch_destroy(gpx_batch* bt) {
  if (!bt) return GPX_BAD_ARG;
  (void)hipSetDevice(bt->ctx->device);
  if (bt->pending_eval) {  // a submitted evaluation still reads and writes the buffers below
    (void)hipStreamSynchronize(bt->pending_eval->s);
    bt->pending_eval.reset();
  }
  if (submit_stats_on() && bt->sub_calls > 0) print_submit_stats(bt);
  if (!bt->slow_out.empty() || bt->slow_s || bt->d_slow_res) {  // deferred slow parts use the buffers below
    for (auto& r : bt->slow_out) (void)hipEventSynchronize(r->done);
    if (bt->slow_s) (void)hipStreamSynchronize(bt->slow_s);
    bt->slow_out.clear();
    bt->slow_pool.clear();
    if (bt->slow_s) (void)hipStreamDestroy(bt->slow_s);
    for (hipEvent_t e : {bt->slow_in, bt->slow_up, bt->bulk_ev})
      if (e) (void)hipEventDestroy(e);
    for (void* q : {(void*)bt->d_slow_act, (void*)bt->d_slow_theta, (void*)bt->d_slow_bandp, (void*)bt->d_slow_info,
                    (void*)bt->d_slow_res, (void*)bt->d_slow_info_c})
      if (q) (void)hipFree(q);
  }
  if (bt->shadow) gpx_batch_destroy(bt->shadow);  // waits for its own submitted evaluation
  if (bt->shadow_s) (void)hipStreamDestroy(bt->shadow_s);
  if (bt->shadow_ev) (void)hipEventDestroy(bt->shadow_ev);
  for (auto& w : bt->rebind_waits) (void)hipEventDestroy(w.ev);
  if (bt->io_ev) {
    (void)hipEventSynchronize(bt->io_ev);
    (void)hipEventDestroy(bt->io_ev);
  }
  if (bt->compact && bt->Kraw) {  // K/L/W point into the raw allocations (band storage's row offset)
    bt->K = bt->Kraw; bt->L = bt->Lraw; bt->W = bt->Wraw;
  }
  for (void* p : {(void*)bt->shX, (void*)bt->shY, (void*)bt->d_wtrace, (void*)bt->d_wtrace_n})
    if (p) (void)hipFree(p);
  for (void* p : {(void*)bt->K, (void*)bt->L, (void*)bt->W, (void*)bt->z, (void*)bt->alpha,
                  (void*)bt->ldiag, (void*)bt->partial, (void*)bt->d_io, (void*)bt->d_n, (void*)bt->d_orow,
                  (void*)bt->d_specs, (void*)bt->kxs, (void*)bt->pvp, (void*)bt->abuf, (void*)bt->covw,
                  (void*)bt->bres, (void*)bt->bcr_ws, (void*)bt->bcr_ws_slow})
    if (p) (void)hipFree(p);
  for (hipEvent_t e : bt->bcr_ev)
    if (e) (void)hipEventDestroy(e);
  bcr_graph_cache_free(bt->bcr_graphs);  // (every stream of the batch has drained above)
  bt->bcr_graphs = nullptr;
  if (bt->h_io) (void)hipHostFree(bt->h_io);
  if (bt->h_sio) (void)hipHostFree(bt->h_sio);
  if (bt->h_io_pred) (void)hipHostFree(bt->h_io_pred);
  if (bt->h_stage) (void)hipHostFree(bt->h_stage);
  if (bt->h_rdesc) (void)hipHostFree(bt->h_rdesc);
  if (bt->h_box) (void)hipHostFree(bt->h_box);
  if (bt->d_box) (void)hipFree(bt->d_box);
  if (bt->h_nmeta) (void)hipHostFree(bt->h_nmeta);
  if (bt->h_specs) (void)hipHostFree(bt->h_specs);
  for (int g = 0; g < kAux; ++g)
    if (bt->aux[g]) (void)hipStreamDestroy(bt->aux[g]);
  if (bt->hp) (void)hipStreamDestroy(bt->hp);
  for (int g = 0; g < kGroups; ++g) {
    if (bt->workers[g]) (void)hipStreamDestroy(bt->workers[g]);
    if (bt->join[g]) (void)hipEventDestroy(bt->join[g]);
  }
  if (bt->fork) (void)hipEventDestroy(bt->fork);
  for (int e = 0; e < kEvents; ++e)
    if (bt->ev[e]) (void)hipEventDestroy(bt->ev[e]);
  delete bt;
  return GPX_OK;
}

static int check_rebind(gpx_batch* bt, int b, int n, const gpx_kernel_spec* spec) {
  gpx_ctx* ctx = bt->ctx;
  if (b < 0 || b >= bt->B || n < 1 || n > bt->Nmax || !spec)
    return fail(ctx, GPX_BAD_ARG, "bad rebind arguments");
  const gpx_kernel_spec& sp = *spec;
  if (sp.n_terms < 1 || sp.n_terms > GPX_MAX_TERMS || sp.n_params < 1 || sp.n_params >= GPX_THETA_STRIDE)
    return fail(ctx, GPX_BAD_ARG, "bad kernel spec");
  for (int t = 0; t < sp.n_terms; ++t) {
    const gpx_term& tm = sp.terms[t];
    const int np = (tm.kind == GPX_RQ || tm.kind == GPX_PERIODIC_SE) ? 3 : (tm.kind == GPX_LINEAR ? 1 : 2);
    if (tm.kind < GPX_SE || tm.kind > GPX_LINEAR || tm.dim_start < 0 || tm.dim_count < 1 ||
        tm.dim_start + tm.dim_count > bt->D || tm.param_offset < 0 || tm.param_offset + np > sp.n_params)
      return fail(ctx, GPX_BAD_ARG, "bad kernel term");
  }
  if (!bt->deferred.empty() && b >= 0 && b < bt->B && bt->deferred[b])
    return fail(ctx, GPX_BAD_ARG, "slot has a deferred evaluation in flight (gpx_batch_deferred_wait)");
  return GPX_OK;
}

int gpx_batch_rebind(gpx_batch* bt, int b, int n, const gpx_kernel_spec* spec) {
  if (!bt) return GPX_BAD_ARG;
  gpx_ctx* ctx = bt->ctx;
  int rc = check_rebind(bt, b, n, spec);
  if (rc != GPX_OK) return rc;
  const gpx_kernel_spec& sp = *spec;
  HIPX(ctx, hipSetDevice(ctx->device));
  bt->n[b] = n;
  bt->specs[b] = sp;
  bt->fac_valid[b] = 0;
  bt->fac_band[b] = 0;
  if (!bt->dirty.empty() && bt->dirty[b]) {  // the caller's own device data supersedes a staged one
    bt->dirty[b] = 0;
    --bt->n_dirty;
  }
  for (size_t i = 0; i < bt->pend.size(); ++i)
    if (bt->pend[i].b == b) {
      bt->pend.erase(bt->pend.begin() + i);
      break;
    }
  HIPX(ctx, hipMemcpy(bt->d_n + b, &n, sizeof(int), hipMemcpyHostToDevice));
  HIPX(ctx, hipMemcpy(bt->d_specs + b, &sp, sizeof(DevSpec), hipMemcpyHostToDevice));
  if (band_shape(bt)) {
    std::vector<double> hx((size_t)n * bt->D);
    HIPX(ctx, hipMemcpy(hx.data(), bt->X + (size_t)b * bt->Nmax * bt->D, sizeof(double) * hx.size(),
                        hipMemcpyDeviceToHost));
    band_tables(bt, b, hx.data());
  }
  return GPX_OK;
}

static int stage_slot(gpx_batch* bt, int b, double** hx, double** hy) {
  gpx_ctx* ctx = bt->ctx;
  const size_t nx = (size_t)bt->Nmax * bt->D, ny = bt->Nmax;
  constexpr size_t kSpecDoubles = (sizeof(DevSpec) + sizeof(double) - 1) / sizeof(double);
  if (!bt->h_stage) {
    bt->stage_stride = nx + ny + 1 + kSpecDoubles;
    HIPX(ctx, hipHostMalloc(&bt->h_stage, sizeof(double) * bt->stage_stride * bt->B, hipHostMallocNonCoherent));
  }
  const int rc = ensure_rebind_meta(bt);
  if (rc != GPX_OK) return rc;
  *hx = bt->h_stage + (size_t)b * bt->stage_stride;
  *hy = *hx + nx;
  return GPX_OK;
}

int gpx_batch_rebind_device(gpx_batch* bt, int b, int n, const double* X, const double* Y,
                            const gpx_kernel_spec* spec, void* stream) {
  if (!bt) return GPX_BAD_ARG;
  gpx_ctx* ctx = bt->ctx;
  if (!X || !Y) return fail(ctx, GPX_BAD_ARG, "null device inputs");
  int rc = check_rebind(bt, b, n, spec);
  if (rc != GPX_OK) return rc;
  // recorded only: the next device call's flush_rebinds gathers every pending slot in one
  // kernel on that call's stream (X and Y must stay valid until then). X and Y are ready in
  // the order of `stream` (the caller's current stream, where their producers ran): an event
  // recorded on it now orders the gather after them, whichever stream the gather runs on
  if (stream) {
    HIPX(ctx, hipSetDevice(ctx->device));
    const hipStream_t s = (hipStream_t)stream;
    gpx_batch::RebindWait* w = nullptr;
    for (auto& x : bt->rebind_waits)
      if (x.s == s) w = &x;
    if (!w) {
      hipEvent_t ev;
      HIPX(ctx, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      bt->rebind_waits.push_back(gpx_batch::RebindWait{s, ev, false});
      w = &bt->rebind_waits.back();
    }
    HIPX(ctx, hipEventRecord(w->ev, s));
    w->armed = true;
  }
  bt->n[b] = n;
  bt->specs[b] = *spec;
  bt->fac_valid[b] = 0;
  bt->fac_band[b] = 0;
  if (!bt->dirty.empty() && bt->dirty[b]) {  // supersedes a host-staged rebind of the slot
    bt->dirty[b] = 0;
    --bt->n_dirty;
  }
  if (!bt->slot_box_ok.empty()) bt->slot_box_ok[b] = 0;
  for (auto& e : bt->pend)
    if (e.b == b) {
      e = gpx_batch::PendingRebind{b, n, X, Y, false};
      return GPX_OK;
    }
  bt->pend.push_back(gpx_batch::PendingRebind{b, n, X, Y, false});
  return GPX_OK;
}

int gpx_batch_rebind_device_boxed(gpx_batch* bt, int b, int n, const double* X, const double* Y,
                                  const gpx_kernel_spec* spec, const double* box, void* stream) {
  if (!bt) return GPX_BAD_ARG;
  if (!box) return fail(bt->ctx, GPX_BAD_ARG, "null boxes");
  const int rc = gpx_batch_rebind_device(bt, b, n, X, Y, spec, stream);
  if (rc != GPX_OK) return rc;
  for (auto& e : bt->pend)
    if (e.b == b) e.boxed = true;
  if (band_shape(bt)) {  // the band tables now, from the caller's boxes: no download at the gather
    band_tables_boxes(bt, b, box);
    keep_slot_box(bt, b, box);
  }
  return GPX_OK;
}

int gpx_batch_slot_boxes(const gpx_batch* bt, int b, double* out) {
  if (!bt || !out || b < 0 || b >= bt->B) return GPX_BAD_ARG;
  if (bt->slot_box_ok.empty() || !bt->slot_box_ok[b] || !bt->pend.empty()) return GPX_BAD_ARG;
  const int nbx = (bt->Nmax + kBox - 1) / kBox;
  const size_t row = (size_t)nbx * bt->D * 2;
  const int nvb = (bt->n[b] + kBox - 1) / kBox;
  std::memcpy(out, bt->slot_box.data() + row * b, sizeof(double) * (size_t)nvb * bt->D * 2);
  return GPX_OK;
}

int gpx_batch_rebind_host(gpx_batch* bt, int b, int n, const double* X, const double* Y,
                          const gpx_kernel_spec* spec, void* stream) {
  if (!bt) return GPX_BAD_ARG;
  gpx_ctx* ctx = bt->ctx;
  if (!X || !Y) return fail(ctx, GPX_BAD_ARG, "null host inputs");
  int rc = check_rebind(bt, b, n, spec);
  if (rc != GPX_OK) return rc;
  HIPX(ctx, hipSetDevice(ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  const size_t nx = (size_t)bt->Nmax * bt->D, ny = bt->Nmax;
  double *hx, *hy;
  rc = stage_slot(bt, b, &hx, &hy);
  if (rc != GPX_OK) return rc;
  for (size_t i = 0; i < bt->pend.size(); ++i)
    if (bt->pend[i].b == b) {
      bt->pend.erase(bt->pend.begin() + i);
      break;
    }
  if (hx != X) std::memcpy(hx, X, sizeof(double) * (size_t)n * bt->D);
  std::memset(hx + (size_t)n * bt->D, 0, sizeof(double) * (nx - (size_t)n * bt->D));
  if (hy != Y) std::memcpy(hy, Y, sizeof(double) * n);
  std::memset(hy + n, 0, sizeof(double) * (ny - n));
  // the copies go out with the next device call (flush_rebinds)
  bt->n[b] = n;
  bt->specs[b] = *spec;
  bt->fac_valid[b] = 0;
  bt->fac_band[b] = 0;
  if (!bt->dirty[b]) {
    bt->dirty[b] = 1;
    ++bt->n_dirty;
  }
  (void)s;
  if (!bt->slot_box_ok.empty()) bt->slot_box_ok[b] = 0;
  if (band_shape(bt)) band_tables(bt, b, hx);
  return GPX_OK;
}

// Band storage's dense fallback: problem b of bt is rebound to a slot of bt->shadow (its X / Y
// rows gathered device to device by the shadow's next call) and evaluated there, in chunks of
// kShadowSlots; outputs land at row b as gpx_batch_lml_grad writes them.
static int shadow_lml_grad(gpx_batch* bt, const std::vector<int32_t>& ids, const double* theta,
                           double* lml, double* grad, int32_t* info, hipStream_t s) {
  gpx_batch* sh = bt->shadow;
  const size_t nx = (size_t)bt->Nmax * bt->D;
  std::vector<double> th((size_t)kShadowSlots * GPX_THETA_STRIDE, 1.0), l(kShadowSlots);
  std::vector<double> g((size_t)kShadowSlots * GPX_THETA_STRIDE);
  std::vector<int32_t> inf(kShadowSlots), act(kShadowSlots);
  int status = GPX_OK;
  for (size_t c = 0; c < ids.size(); c += kShadowSlots) {
    const int cnt = (int)std::min<size_t>(kShadowSlots, ids.size() - c);
    for (int k = 0; k < cnt; ++k) {
      const int b = ids[c + k];
      const int rc = gpx_batch_rebind_device(sh, k, bt->n[b], bt->X + b * nx, bt->Y + (size_t)b * bt->Nmax,
                                             &bt->specs[b], s);
      if (rc != GPX_OK) return rc;
      std::memcpy(&th[(size_t)k * GPX_THETA_STRIDE], theta + (size_t)b * GPX_THETA_STRIDE,
                  sizeof(double) * GPX_THETA_STRIDE);
      act[k] = k;
    }
    const int rc = gpx_batch_lml_grad(sh, cnt, act.data(), th.data(), l.data(), g.data(), inf.data(), s);
    if (rc != GPX_OK && rc != GPX_NOT_PD) return rc;
    bt->timing.shadow_evals += cnt;
    for (int k = 0; k < cnt; ++k) {
      const int b = ids[c + k];
      info[b] = inf[k];
      if (inf[k] != 0) status = GPX_NOT_PD;
      lml[b] = l[k];
      for (int p = 0; p <= bt->specs[b].n_params; ++p)
        grad[(size_t)b * GPX_THETA_STRIDE + p] = g[(size_t)k * GPX_THETA_STRIDE + p];
      bt->fac_valid[b] = 0;  // no factor of b is kept in bt
      bt->fac_band[b] = 0;
    }
  }
  if (status == GPX_NOT_PD) last_error_slot() = "K + noise*I is not positive definite for some problem";
  return status;
}

// Band storage: up to kShadowSlots fallback problems are submitted on the batch's fallback
// stream at _submit (after the call's rebind gather on s, which their inputs come from), so the
// dense evaluation runs beside the band sweeps; _complete collects it.
static int shadow_submit(gpx_batch* bt, const std::vector<int32_t>& ids, const double* theta, hipStream_t s) {
  gpx_ctx* ctx = bt->ctx;
  gpx_batch* sh = bt->shadow;
  if (!bt->shadow_s) {
    HIPX(ctx, hipStreamCreateWithFlags(&bt->shadow_s, hipStreamNonBlocking));
    HIPX(ctx, hipEventCreateWithFlags(&bt->shadow_ev, hipEventDisableTiming));
  }
  HIPX(ctx, hipEventRecord(bt->shadow_ev, s));
  HIPX(ctx, hipStreamWaitEvent(bt->shadow_s, bt->shadow_ev, 0));
  const size_t nx = (size_t)bt->Nmax * bt->D;
  std::vector<double> th((size_t)kShadowSlots * GPX_THETA_STRIDE, 1.0);
  std::vector<int32_t> act(ids.size());
  for (size_t k = 0; k < ids.size(); ++k) {
    const int b = ids[k];
    const int rc = gpx_batch_rebind_device(sh, (int)k, bt->n[b], bt->X + b * nx, bt->Y + (size_t)b * bt->Nmax,
                                           &bt->specs[b], bt->shadow_s);
    if (rc != GPX_OK) return rc;
    std::memcpy(&th[k * GPX_THETA_STRIDE], theta + (size_t)b * GPX_THETA_STRIDE, sizeof(double) * GPX_THETA_STRIDE);
    act[k] = (int32_t)k;
  }
  return gpx_batch_lml_grad_submit(sh, (int)ids.size(), act.data(), th.data(), bt->shadow_s);
}

static int shadow_collect(gpx_batch* bt, const std::vector<int32_t>& ids, double* lml, double* grad,
                          int32_t* info) {
  gpx_batch* sh = bt->shadow;
  std::vector<double> l(kShadowSlots), g((size_t)kShadowSlots * GPX_THETA_STRIDE);
  std::vector<int32_t> inf(kShadowSlots);
  const int rc = gpx_batch_lml_grad_complete(sh, l.data(), g.data(), inf.data());
  if (rc != GPX_OK && rc != GPX_NOT_PD) return rc;
  bt->timing.shadow_evals += (double)ids.size();
  int status = GPX_OK;
  for (size_t k = 0; k < ids.size(); ++k) {
    const int b = ids[k];
    info[b] = inf[k];
    if (inf[k] != 0) status = GPX_NOT_PD;
    lml[b] = l[k];
    for (int p = 0; p <= bt->specs[b].n_params; ++p)
      grad[(size_t)b * GPX_THETA_STRIDE + p] = g[k * GPX_THETA_STRIDE + p];
    bt->fac_valid[b] = 0;
    bt->fac_band[b] = 0;
  }
  return status;
}

// ---- deferred completion of the slow classes (gpx_batch_set_deferred) ----
// By default the slow part runs on a stream of its own, from copies of the call's inputs, so the
// next call's work does not queue behind it (the C2 bench: +14-18 % over the same-stream variant
// once the driver's calls are on a stream of their own). GPX_DEFER_STREAM=0: it
// follows the call's own work on the call's stream, after the call's download (the call
// completes at an event there), and delays the next call.
static bool defer_own_stream() {
  static const bool on = [] {
    const char* e = getenv("GPX_DEFER_STREAM");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

static int slow_setup(gpx_batch* bt) {
  gpx_ctx* ctx = bt->ctx;
  const size_t B = bt->B;
  if (!bt->d_slow_res) {
    HIPX(ctx, hipMalloc(&bt->d_slow_res, sizeof(double) * B * kResStride));
    HIPX(ctx, hipMalloc(&bt->d_slow_info_c, sizeof(int) * B));
  }
  if (!bt->slow_in) HIPX(ctx, hipEventCreateWithFlags(&bt->slow_in, hipEventDisableTiming));
  if (!defer_own_stream() || bt->slow_s) return GPX_OK;
  // GPX_SLOW_PRIORITY: the slow stream at the device's lowest (-1) or highest (1) stream priority
  // (streams of another priority take hardware queues of their own); 0 / unset: the default
  static const int prio = [] {
    const char* e = getenv("GPX_SLOW_PRIORITY");
    return e ? atoi(e) : 0;
  }();
  if (prio != 0) {
    int least = 0, greatest = 0;
    HIPX(ctx, hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIPX(ctx, hipStreamCreateWithPriority(&bt->slow_s, hipStreamNonBlocking, prio > 0 ? greatest : least));
  } else {
    HIPX(ctx, hipStreamCreateWithFlags(&bt->slow_s, hipStreamNonBlocking));
  }
  HIPX(ctx, hipEventCreateWithFlags(&bt->slow_up, hipEventDisableTiming));
  HIPX(ctx, hipMalloc(&bt->d_slow_act, sizeof(int) * B));
  HIPX(ctx, hipMalloc(&bt->d_slow_theta, sizeof(double) * B * GPX_THETA_STRIDE));
  HIPX(ctx, hipMalloc(&bt->d_slow_bandp, sizeof(int) * B));
  HIPX(ctx, hipMalloc(&bt->d_slow_info, sizeof(int) * B));
  return GPX_OK;
}

// The slow part of a call: problems order[off .. off + n) of the uploaded active list (band16
// groups q/cnt, then the 64-row sweeps' p <= 1 problems (n1) and p = 2 ones), on slow_s, from
// copies of the active list / θ / widths so the next call's upload cannot change them under it
static int submit_slow(gpx_batch* bt, hipStream_t s, const int32_t* ids, int off, int n, int n_g16, const int* q,
                       const int* cnt, int n16, int n1, bool se1, int kband16, int max_terms, const double* theta) {
  gpx_ctx* ctx = bt->ctx;
  {
    const int e = slow_setup(bt);
    if (e != GPX_OK) return e;
  }
  std::unique_ptr<gpx_batch::SlowRec> rec;
  if (!bt->slow_pool.empty()) {
    rec = std::move(bt->slow_pool.back());
    bt->slow_pool.pop_back();
  } else {
    rec.reset(new gpx_batch::SlowRec());
    HIPX(ctx, hipEventCreateWithFlags(&rec->done, hipEventDisableTiming));
    const unsigned fl = slow_direct() ? hipHostMallocCoherent : hipHostMallocDefault;
    HIPX(ctx, hipHostMalloc(&rec->h_res, sizeof(double) * bt->B * kResStride, fl));
    HIPX(ctx, hipHostMalloc(&rec->h_info, sizeof(int) * bt->B, fl));
  }
  rec->ids.assign(ids, ids + n);
  // The wide launch's waves in reverse order, widest first (GPX_WIDE_REVERSE=0: ascending): its
  // workgroups are dispatched in index order as wave slots free up under the other processes'
  // sweeps, and a Q = 6..8 wave — 2-3x a Q = 4 / 5 wave's time — dispatched last used to end the
  // launch alone. Each wave's arithmetic is its own problem's, so the bits are unchanged; the
  // part's active copy and its result gather (rec->ids) take the same order.
  static const bool wide_rev = [] {
    const char* e = getenv("GPX_WIDE_REVERSE");
    return !(e && atoi(e) == 0);
  }();
  int r0 = 0, r1 = 0;
  {
    static const bool wide_on = [] {
      const char* e = getenv("GPX_DEFER_WIDE");
      return !(e && atoi(e) == 0);
    }();
    const int wq = wide_launch_qmax(se1);
    if (wide_rev && wide_on && se1 && defer_own_stream()) {
      int o = 0;
      r0 = r1 = -1;
      for (int g = 0; g < n_g16; ++g) {
        if (q[g] >= 4 && q[g] <= wq) {
          if (r0 < 0) r0 = o;
          r1 = o + cnt[g];
        }
        o += cnt[g];
      }
      if (r0 < 0) r0 = r1 = 0;
      std::reverse(rec->ids.begin() + r0, rec->ids.begin() + r1);
    }
  }
  rec->theta.assign(theta, theta + (size_t)bt->B * GPX_THETA_STRIDE);
  rec->clear_events();
  // (the swept groups: the wide ones, Q > kBcrMaxQ, run as a reduction chain without band16 events)
  int g_sw = n_g16;
  while (wide_bcr_on(false) && g_sw > 0 && q[g_sw - 1] > kBcrMaxQ) --g_sw;
  rec->n_g16 = g_sw;
  rec->se1 = se1;
  for (int g = 0; g < n_g16; ++g) {
    rec->g16_q[g] = q[g];
    rec->g16_n[g] = cnt[g];
  }
  rec->p64.clear();
  const bool own = defer_own_stream();
  hipStream_t ss = own ? bt->slow_s : s;
  if (own) {
    HIPX(ctx, hipEventRecord(bt->slow_up, s));
    HIPX(ctx, hipStreamWaitEvent(ss, bt->slow_up, 0));
    // one launch of one-wave workgroups, not the runtime's three copies and a fill: its blit
    // kernels' multi-wave workgroups wait for free CU space behind the other processes' sweeps
    // (+2.8 % on the bench, profiles/r05_ab.md)
    launch_slow_inputs(bt->d_active + off, n, bt->d_slow_act, bt->d_theta, bt->d_slow_theta, bt->d_bandp,
                       bt->d_slow_bandp, bt->d_slow_info, bt->B, ss, r0, r1);
    HIPX(ctx, hipGetLastError());
    HIPX(ctx, hipEventRecord(bt->slow_in, ss));
    bt->slow_in_armed = true;
  }
  const bool fused64 = n > n16;
  if (ctx->profiling) {
    for (int g = 0; g < g_sw; ++g)
      for (int e = 0; e < 4; ++e) HIPX(ctx, hipEventCreate(&rec->fq16[g][e]));
    if (fused64) {
      for (int e = 0; e < 4; ++e) HIPX(ctx, hipEventCreate(&rec->fq[e]));
      // (the timed 64-row pair is the p <= 1 class's when there is one, else the p = 2 class's)
      const int t0 = n16, t1 = n1 > 0 ? n16 + n1 : n;
      for (int i = t0; i < t1; ++i) rec->p64.push_back(bt->h_bandp[ids[i]]);
    }
  }
  // (on the call's stream, after its download: the next call's upload follows this part in the
  // stream's order, so the part reads the call's own active list, θ and widths in place)
  Run r{bt, own ? bt->d_slow_act : bt->d_active + off, n, ss};
  r.bcr_wsp = &bt->bcr_ws_slow;
  r.bcr_capp = &bt->bcr_ws_slow_cap;
  if (own) {
    r.theta = bt->d_slow_theta;
    r.bandp = bt->d_slow_bandp;
    r.info = bt->d_slow_info;
  }
  // GPX_DEFER_LANES=1: the part's lanes (the wide band16 launch; the 64-row sweeps) on the
  // batch's lane streams, joined on ss, instead of one after another on ss
  static const bool lanes = [] {
    const char* e = getenv("GPX_DEFER_LANES");
    return e && atoi(e) != 0;
  }();
  r.one_stream = !lanes;
  // the part's band16 classes as one launch (band16_wide_kernel), or (GPX_DEFER_WIDE=0) one
  // forward and one backward launch per class, each at its own occupancy
  static const bool wide = [] {
    const char* e = getenv("GPX_DEFER_WIDE");
    return !(e && atoi(e) == 0);
  }();
  r.wide_from = wide ? 1 : 0;
  {
    const int e = band_fused_eval(r, n16, n_g16, q, cnt, se1, kband16, n1, max_terms,
                                  (ctx->profiling && fused64) ? rec->fq : nullptr, ctx->profiling ? rec->fq16 : nullptr);
    if (e != GPX_OK) return e;
  }
  static const int slow_delay = [] {
    const char* e = getenv("GPX_SLOW_DELAY_US");
    return e ? atoi(e) : 0;
  }();
  if (slow_delay > 0) launch_spin_us(slow_delay, ss);
  if (slow_direct()) {
    // the gather writes the part's result rows straight into the record's coherent pinned
    // buffers: no copy-engine download on the slow stream, whose deferred parts follow each
    // other (their length is what deferred fits wait)
    launch_slow_gather(r.d_act, n, bt->results, kResStride, rec->h_res, own ? bt->d_slow_info : bt->d_info,
                       rec->h_info, ss);
  } else {
    launch_slow_gather(r.d_act, n, bt->results, kResStride, bt->d_slow_res, own ? bt->d_slow_info : bt->d_info,
                       bt->d_slow_info_c, ss);
    HIPX(ctx, hipMemcpyAsync(rec->h_res, bt->d_slow_res, sizeof(double) * n * kResStride, hipMemcpyDeviceToHost, ss));
    HIPX(ctx, hipMemcpyAsync(rec->h_info, bt->d_slow_info_c, sizeof(int) * n, hipMemcpyDeviceToHost, ss));
  }
  HIPX(ctx, hipEventRecord(rec->done, ss));
  if (!own) {
    // same-stream mode reads the call's active list, θ, widths and info in place: the next
    // upload into them (from any stream) waits for the part to finish (upload_common)
    HIPX(ctx, hipEventRecord(bt->slow_in, ss));
    bt->slow_in_armed = true;
  }
  HIPX(ctx, hipGetLastError());
  if (bt->deferred.size() != (size_t)bt->B) bt->deferred.assign(bt->B, 0);
  for (int i = 0; i < n; ++i) {
    bt->deferred[ids[i]] = 1;
    bt->fac_valid[ids[i]] = 0;
  }
  bt->slow_out.push_back(std::move(rec));
  return GPX_OK;
}

// A finished slow part's results into the caller's arrays, as _complete reports its own rows
// (band-check failures re-evaluated densely here)
static int deliver_slow(gpx_batch* bt, gpx_batch::SlowRec& rec, double* lml, double* grad, int32_t* info) {
  gpx_ctx* ctx = bt->ctx;
  const char* et = getenv("GPX_BAND_TOL");
  const double band_tol = et ? atof(et) : 1e-6;
  int status = GPX_OK;
  std::vector<int32_t> redo;
  const int n = (int)rec.ids.size();
  for (int i = 0; i < n; ++i) {
    const int b = rec.ids[i];
    bt->deferred[b] = 0;
    const double* res = rec.h_res + (size_t)i * kResStride;
    const int np = bt->specs[b].n_params;
    if (rec.h_info[i] == 0 && !(res[kResBandCheck] <= band_tol)) {
      redo.push_back(b);  // (its info is written by the dense re-evaluation, once that succeeds)
      continue;
    }
    info[b] = rec.h_info[i];
    if (info[b] != 0) {
      status = GPX_NOT_PD;
      lml[b] = NAN;
      for (int p = 0; p <= np; ++p) grad[(size_t)b * GPX_THETA_STRIDE + p] = NAN;
      bt->fac_valid[b] = 0;
      continue;
    }
    lml[b] = res[0];
    for (int p = 0; p <= np; ++p) grad[(size_t)b * GPX_THETA_STRIDE + p] = res[1 + p];
    std::memcpy(&bt->fac_theta[(size_t)b * GPX_THETA_STRIDE], rec.theta.data() + (size_t)b * GPX_THETA_STRIDE,
                sizeof(double) * GPX_THETA_STRIDE);
    bt->fac_valid[b] = 1;
    bt->fac_band[b] = 1;
  }
  if (ctx->profiling) {
    bt->timing.band_evals += n;
    bt->timing.evals += n;
    bool wide_seen = false;
    for (int g = 0; g < rec.n_g16; ++g) {
      float f0 = 0.f, f1 = 0.f;
      (void)hipEventElapsedTime(&f0, rec.fq16[g][0], rec.fq16[g][1]);
      (void)hipEventElapsedTime(&f1, rec.fq16[g][2], rec.fq16[g][3]);
      const int n = rec.g16_n[g], q = rec.g16_q[g];
      const double fl = n * (band16_flops(bt->Np, q, true) + band16_flops(bt->Np, q, false));
      if (rec.se1 && q >= 4 && q <= wide_qmax(true) && (q <= 5 || b16_inline_k_wide() == 3)) {
        // the wide launch (band_fused_eval's kind-3 lane): every one of its groups' events spans
        // the one kernel, so it is counted once, apart from the per-class launches
        if (!wide_seen) {
          bt->timing.band16_wide_ms_total += f0;
          bt->timing.band16_wide_launches += 1.0;
          wide_seen = true;
        }
        bt->timing.band16_wide_flops += fl;
        bt->timing.band16_wide_evals += n;
        bt->timing.band16_wave_ms += (double)n * (double)f0;
      } else {
        bt->timing.band16_fwd_ms_total += f0;
        bt->timing.band16_bwd_ms_total += f1;
        bt->timing.band16_wave_ms += (double)n * ((double)f0 + (double)f1);
        bt->timing.band16_launches += 1.0;
        bt->timing.band16_fwd_flops += n * band16_flops(bt->Np, q, true);
        bt->timing.band16_bwd_flops += n * band16_flops(bt->Np, q, false);
      }
      bt->timing.band16_evals += n;
      bt->timing.band16_q_sum += (double)q * n;
      bt->timing.band_p_sum += n;
    }
    if (rec.fq[0]) {
      float f0 = 0.f, f1 = 0.f;
      (void)hipEventElapsedTime(&f0, rec.fq[0], rec.fq[1]);
      (void)hipEventElapsedTime(&f1, rec.fq[2], rec.fq[3]);
      bt->timing.band_fwd_ms_total += f0;
      bt->timing.band_bwd_ms_total += f1;
      bt->timing.band_fused_launches += 1.0;
      bool p2 = !rec.p64.empty();
      for (int pb : rec.p64) p2 = p2 && pb == 2;
      if (p2) bt->timing.band_fused_p2_launches += 1.0;
      for (int pb : rec.p64) {
        bt->timing.band_fwd_flops += band_fused_flops(bt->Np, pb, true);
        bt->timing.band_bwd_flops += band_fused_flops(bt->Np, pb, false);
        bt->timing.band_p_sum += pb;
      }
    }
  }
  if (!redo.empty()) {
    if (ctx->profiling) bt->timing.band_fallbacks += (double)redo.size();
    int rc2;
    if (bt->compact) {
      rc2 = shadow_lml_grad(bt, redo, rec.theta.data(), lml, grad, info, bt->slow_s ? bt->slow_s : ctx->stream);
    } else {
      bt->force_dense = 1;
      rc2 = gpx_batch_lml_grad(bt, (int)redo.size(), redo.data(), rec.theta.data(), lml, grad, info,
                               bt->slow_s ? bt->slow_s : ctx->stream);
      bt->force_dense = 0;
    }
    if (rc2 != GPX_OK && rc2 != GPX_NOT_PD) return rc2;
    if (rc2 == GPX_NOT_PD) status = GPX_NOT_PD;
  }
  return status;
}

// every slow part that has finished (block: all of them, waiting), oldest first
static int deliver_ready(gpx_batch* bt, double* lml, double* grad, int32_t* info, bool block) {
  gpx_ctx* ctx = bt->ctx;
  int status = GPX_OK;
  while (!bt->slow_out.empty()) {
    gpx_batch::SlowRec& rec = *bt->slow_out.front();
    if (block) {
      HIPX(ctx, hipEventSynchronize(rec.done));
    } else {
      const hipError_t e = hipEventQuery(rec.done);
      if (e == hipErrorNotReady) break;
      if (e != hipSuccess) return fail(ctx, GPX_HIP_ERROR, std::string("hipEventQuery: ") + hipGetErrorString(e));
    }
    std::unique_ptr<gpx_batch::SlowRec> done = std::move(bt->slow_out.front());
    bt->slow_out.erase(bt->slow_out.begin());
    const int rc = deliver_slow(bt, *done, lml, grad, info);
    done->clear_events();
    bt->slow_pool.push_back(std::move(done));
    if (rc != GPX_OK && rc != GPX_NOT_PD) return rc;
    if (rc == GPX_NOT_PD) status = GPX_NOT_PD;
  }
  if (status == GPX_NOT_PD) last_error_slot() = "K + noise*I is not positive definite for some problem";
  return status;
}

int gpx_batch_lml_grad_submit(gpx_batch* bt, int n_active, const int32_t* active, const double* theta,
                              void* stream) {
  if (!bt) return GPX_BAD_ARG;
  gpx_ctx* ctx = bt->ctx;
  if (bt->pending_eval) return fail(ctx, GPX_BAD_ARG, "an evaluation is already submitted on this batch");
  {  // every argument check before anything is routed or submitted (the fallback slots included)
    const int e = check_active_theta(bt, n_active, active, theta);
    if (e != GPX_OK) return e;
  }
  if (!bt->deferred.empty())
    for (int i = 0; i < n_active; ++i)
      if (bt->deferred[active[i]])
        return fail(ctx, GPX_BAD_ARG, "a problem of the call has a deferred evaluation in flight");
  HIPX(ctx, hipSetDevice(ctx->device));
  SubClock sc(bt);
  ++bt->sub_calls;
  if (submit_stats_on() && bt->sub_calls % 256 == 0) print_submit_stats(bt);  // (runs that never destroy it)

  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  trace_mark(bt, 38, s);
  {  // slots rebound since the last call land first: their band tables (from the gather's
     // X boxes) decide the routing below
    const int rc0 = flush_rebinds(bt, s);
    if (rc0 != GPX_OK) return rc0;
  }
  trace_mark(bt, 39, s);
  sc.lap(0);
  // Route each problem (route_call: the dense recursion, the per-block banded launches, the
  // band16 sweeps by width, the 64-row fused sweeps, or the fallback slots of band storage)
  Route rt;
  route_call(bt, n_active, active, theta, rt);
  // a call with few band16 problems takes them by block cyclic reduction (gpx_bcr.hip, Q <= 5):
  // there its p64 = 2 problems go back to the 64-row sweeps (a Q = 6..8 one-wave sweep is the
  // throughput choice, but its N/16-step chain is 2-3x the 64-row sweeps' latency)
  const int bcr_max = bcr_max_problems(bt);
  if (!wide_bcr_on(true) && rt.n16 > 0 && rt.n16 <= bcr_max && rt.n_g16 > 0 && rt.g16_q[rt.n_g16 - 1] > kBcrMaxQ)
    route_call(bt, n_active, active, theta, rt, kBcrMaxQ);
  std::vector<int32_t>& order = rt.order;
  std::vector<int32_t>& shadow_ids = rt.shadow_ids;
  const int n_dense = rt.n_dense, n_band = rt.n_band, n_fused = rt.n_fused, n16 = rt.n16;
  const int pband = rt.pband, n_g16 = rt.n_g16, n_fused1 = rt.n_fused1;
  const int* g16_q = rt.g16_q;
  const int* g16_n = rt.g16_n;
  const bool b16_p2 = rt.b16_p2;
  // a call with few band16 problems takes them by block cyclic reduction (gpx_bcr.hip): the
  // one-wavefront sweeps' N/16-step chain would be the whole call's latency
  const int bcr_q = (n16 > 0 && n16 <= bcr_max) ? 1 : 0;
  // (the width groups of Q <= kBcrMaxQ: the reduction; wider ones keep their sweeps, so a
  // problem's arithmetic depends on its own width and the call's size only)
  int g_bcr = 0, n16_bcr = 0;
  while (bcr_q > 0 && g_bcr < n_g16 && g16_q[g_bcr] <= kBcrMaxQ) n16_bcr += g16_n[g_bcr++];
  // the problems launched by this call (band storage: without the shadowed ones)
  n_active = n_dense + n_band + n_fused;
  // band storage: a few fallback problems go out at once on the fallback stream (more than the
  // fallback slots hold run in chunks at _complete)
  const bool shadow_async = !shadow_ids.empty() && (int)shadow_ids.size() <= kShadowSlots;
  // a failure after the fallback evaluation went out leaves nothing pending on the fallback
  // slots: drain its stream and drop its state, so later calls are not refused
  auto drop_shadow = [&](int rc) {
    if (shadow_async && bt->shadow && bt->shadow->pending_eval) {
      (void)hipStreamSynchronize(bt->shadow->pending_eval->s);
      bt->shadow->pending_eval.reset();
    }
    return rc;
  };
  if (shadow_async) {
    const int rcs = shadow_submit(bt, shadow_ids, theta, s);
    if (rcs != GPX_OK) return drop_shadow(rcs);
  }
  if (n_active == 0) {  // everything on the dense fallback (the rebinds landed above)
    std::unique_ptr<gpx_batch::PendingEval> pe0(new gpx_batch::PendingEval());
    pe0->s = s;
    pe0->theta.assign(theta, theta + (size_t)bt->B * GPX_THETA_STRIDE);
    pe0->total.reset(new PhaseTimer(false, s));
    pe0->ct.reset(new PhaseTimer(false, s));
    pe0->bp.reset(new PhaseTimer(false, s));
    pe0->shadow_ids = std::move(shadow_ids);
    pe0->shadow_async = shadow_async;
    bt->pending_eval = std::move(pe0);
    return GPX_OK;
  }
  if (n_band > 0) {
    const int e = ensure(ctx, bt->bres, bt->bres_cap, (size_t)bt->B * bt->Np);
    if (e != GPX_OK) return drop_shadow(e);
  }
  // the wide groups (Q > kBcrMaxQ, a suffix of the groups) on the bs = 128 reduction
  int g_wide = n_g16;
  while (wide_bcr_on(bcr_q > 0) && g_wide > 0 && g16_q[g_wide - 1] > kBcrMaxQ) --g_wide;
  if (n16_bcr > 0 || g_wide < n_g16) {  // (the workspace is sized by band_fused_eval for what it launches)
    if (ctx->profiling && !bt->bcr_ev[0])
      for (auto& e2 : bt->bcr_ev) HIPX(ctx, hipEventCreate(&e2));
  }
  sc.lap(1);
  // a small-problem call (Np = 64, every problem on the one fused kernel): its I/O straight through
  // coherent pinned memory — no upload or download DMA, the kernel launch and the synchronise
  // are the call's whole device round trip (the drop-in pattern's solo calls, VERDICT r05 item 6;
  // GPX_SMALL_DIRECT=0: the DMA'd I/O block)
  static const bool small_direct = [] {
    const char* e = getenv("GPX_SMALL_DIRECT");
    return !(e && atoi(e) == 0);
  }();
  if (small_direct && small64_on(bt) && n_dense == n_active && !shadow_async && shadow_ids.empty()) {
    if (!bt->h_sio) HIPX(ctx, hipHostMalloc(&bt->h_sio, bt->io_bytes, hipHostMallocCoherent));
    {
      const int e = fence_io(bt, s);
      if (e != GPX_OK) return e;
    }
    std::memcpy(bt->h_sio, order.data(), sizeof(int) * n_active);
    std::memset(bt->h_sio + bt->io_info_off, 0, sizeof(int) * bt->B);
    std::memcpy(bt->h_sio + bt->io_theta_off, theta, sizeof(double) * GPX_THETA_STRIDE * bt->B);
    std::unique_ptr<gpx_batch::PendingEval> pd(new gpx_batch::PendingEval());
    pd->s = s;
    pd->n_active = n_active;
    pd->n_dense = n_active;
    pd->direct = true;
    pd->theta.assign(theta, theta + (size_t)bt->B * GPX_THETA_STRIDE);
    pd->total.reset(new PhaseTimer(ctx->profiling != 0, s));
    pd->ct.reset(new PhaseTimer(false, s));
    pd->bp.reset(new PhaseTimer(false, s));
    // completion by polling the workgroups' flags (GPX_SMALL_POLL, default on; not when profiling,
    // whose events complete reads): a launch + synchronise round trip costs ≈ 12 µs, a launch and
    // a polled flag ≈ 7 (tools/micro/launch_roundtrip.hip)
    static const bool poll = [] {
      const char* e = getenv("GPX_SMALL_POLL");
      return !(e && atoi(e) == 0);
    }();
    if (poll && !ctx->profiling) {
      bt->direct_tag = bt->direct_tag >= (1 << 30) ? 1 : bt->direct_tag + 1;
      pd->poll_tag = bt->direct_tag;
    }
    pd->total->mark();
    small64_eval(Run{bt, reinterpret_cast<const int*>(bt->h_sio), n_active, s}, true, bt->h_sio, pd->poll_tag);
    pd->total->mark();
    HIPX(ctx, hipGetLastError());
    pd->order = std::move(order);
    bt->pending_eval = std::move(pd);
    sc.lap(4);
    return GPX_OK;
  }
  int rc = upload_common(bt, n_active, order.data(), theta, s);
  if (rc != GPX_OK) return drop_shadow(rc);
  sc.lap(2);
  rc = match_aux_priority(bt, s);
  if (rc != GPX_OK) return drop_shadow(rc);
  bt->flops_acc = 0.0;
  std::unique_ptr<gpx_batch::PendingEval> pe(new gpx_batch::PendingEval());
  pe->s = s;
  pe->n_active = n_active;
  pe->theta.assign(theta, theta + (size_t)bt->B * GPX_THETA_STRIDE);
  pe->total.reset(new PhaseTimer(ctx->profiling != 0, s));
  PhaseTimer& total = *pe->total;
  total.mark();
  hipEvent_t* kev = pe->kev;
  int& ng = pe->ng;
  std::vector<PhaseTimer>& pts = pe->pts;
  pe->ct.reset(new PhaseTimer(ctx->profiling != 0 && n_dense > 0, s));
  PhaseTimer& ct = *pe->ct;
  if (n_dense > 0 && small64_on(bt)) {
    // Np = 64: the whole evaluation of every dense problem in one launch
    small64_eval(Run{bt, bt->d_active, n_dense, s}, true);
  } else if (n_dense > 0) {
    // Split the dense problems into up to kGroups ranges, each running the whole pipeline on
    // its own stream: one group's latency-bound phases (64x64 leaves, small recursion levels)
    // overlap another group's large MFMA GEMMs.
    // Default: one pipeline whose recursion forks the top-level T products onto aux streams
    // (concurrency inside the DAG). GPX_GROUPS=g instead splits the problems into g pipelines.
    ng = 1;
    if (const char* e = getenv("GPX_GROUPS")) ng = atoi(e);
    ng = std::max(1, std::min(std::min(ng, kGroups), n_dense));
    if (ng > 1 && !bt->fork) {
      HIPX(ctx, hipEventCreateWithFlags(&bt->fork, hipEventDisableTiming));
      for (int g = 0; g < kGroups; ++g) {
        HIPX(ctx, hipStreamCreateWithFlags(&bt->workers[g], hipStreamNonBlocking));
        HIPX(ctx, hipEventCreateWithFlags(&bt->join[g], hipEventDisableTiming));
      }
    }
    int next_event = 0;
    Run runs[kGroups];
    int start = 0;
    for (int g = 0; g < ng; ++g) {
      const int cnt = n_dense / ng + (g < n_dense % ng ? 1 : 0);
      runs[g] = Run{bt, bt->d_active + start, cnt, ng == 1 ? s : bt->workers[g], ng == 1, &next_event};
      start += cnt;
    }
    if (ng > 1) {
      HIPX(ctx, hipEventRecord(bt->fork, s));
      for (int g = 0; g < ng; ++g) HIPX(ctx, hipStreamWaitEvent(runs[g].s, bt->fork, 0));
    }
    pts.reserve(ng);
    for (int g = 0; g < ng; ++g) pts.emplace_back(ctx->profiling != 0, runs[g].s);
    for (int g = 0; g < ng; ++g) {
      const Run& r = runs[g];
      pts[g].mark();
      factor(r);
      pts[g].mark();
      alpha_solve(r);
      pts[g].mark();
    }
    if (ng > 1) {
      for (int g = 0; g < ng; ++g) {
        HIPX(ctx, hipEventRecord(bt->join[g], runs[g].s));
        HIPX(ctx, hipStreamWaitEvent(s, bt->join[g], 0));
      }
    }
    // The contraction fills the chip by itself (Np²/2/128² tiles per problem): one launch over
    // every dense problem, alone on the stream.
    const Run all{bt, bt->d_active, n_dense, s};
    int max_terms = 1;
    for (int i = 0; i < n_dense; ++i) max_terms = std::max(max_terms, (int)bt->specs[order[i]].n_terms);
    // the contraction kernel is timestamped at its actual start/end (hipExtLaunchKernel), so
    // its duration excludes any wait behind kernels of other streams (concurrent batches)
    if (ctx->profiling) {
      HIPX(ctx, hipEventCreate(&kev[0]));
      HIPX(ctx, hipEventCreate(&kev[1]));
    }
    // optional: run the contraction on a highest-priority stream so that, with several batches
    // evaluating concurrently, its workgroups are dispatched ahead of the other batches' kernels
    static const bool prio = [] {
      const char* e = getenv("GPX_CONTRACT_PRIORITY");
      return e && atoi(e) != 0;
    }();
    Run cr = all;
    if (prio) {
      if (!bt->hp) {
        int lo = 0, hi = 0;
        HIPX(ctx, hipDeviceGetStreamPriorityRange(&lo, &hi));
        HIPX(ctx, hipStreamCreateWithPriority(&bt->hp, hipStreamNonBlocking, hi));
      }
      HIPX(ctx, hipEventRecord(bt->ev[kEvents - 4], s));
      HIPX(ctx, hipStreamWaitEvent(bt->hp, bt->ev[kEvents - 4], 0));
      cr.s = bt->hp;
    }
    ct.mark();
    contract(cr, max_terms, kev[0], kev[1]);
    ct.mark();
    reduce(cr);
    if (prio) {
      HIPX(ctx, hipEventRecord(bt->ev[kEvents - 3], bt->hp));
      HIPX(ctx, hipStreamWaitEvent(s, bt->ev[kEvents - 3], 0));
    }
    ct.mark();
  }
  pe->bp.reset(new PhaseTimer(ctx->profiling != 0, s));
  PhaseTimer& bp = *pe->bp;
  bp.mark();
  if (n_band > 0) {
    int max_terms = 1;
    for (int i = n_dense; i < n_dense + n_band; ++i) max_terms = std::max(max_terms, (int)bt->specs[order[i]].n_terms);
    band_eval(Run{bt, bt->d_active + n_dense, n_band, s}, pband, max_terms);
  }
  hipEvent_t* fqe = pe->fq;
  // deferred completion: the slow classes (band16 wider than defer_q, then the 64-row sweeps) are
  // the tail of the fused range; they go out as a slow part and this call completes without them
  int n_slow = 0, n_g16_run = n_g16, n16_run = n16, n_fused1_run = n_fused1;
  struct SlowArgs { int off, n_g16, g0, n16, n1; bool se1; int max_terms; };
  SlowArgs slow_args{-1, 0, 0, 0, 0, true, 1};
  if (bt->defer_q >= 0 && n_fused > 0 && bcr_q == 0) {
    int k = 0, nb16 = 0;
    while (k < n_g16 && g16_q[k] <= bt->defer_q) nb16 += g16_n[k++];
    if (n_fused > nb16 && n_dense + n_band + nb16 > 0) {  // (a call of slow problems only just runs)
      n_slow = n_fused - nb16;
      n_g16_run = k;
      n16_run = nb16;
      n_fused1_run = 0;
    }
  }
  const int n_fused_run = n_fused - n_slow;
  if (n_slow > 0) {
    int max_terms = 1;
    bool se1s = true;
    const int off = n_active - n_slow;
    for (int i = off; i < n_active; ++i) max_terms = std::max(max_terms, (int)bt->specs[order[i]].n_terms);
    for (int i = off; i < off + (n16 - n16_run); ++i) {
      const gpx_kernel_spec& sp = bt->specs[order[i]];
      se1s = se1s && se1_spec(sp);
    }
    if (defer_own_stream()) {
      const int rcs = submit_slow(bt, s, order.data() + off, off, n_slow, n_g16 - n_g16_run, g16_q + n_g16_run,
                                  g16_n + n_g16_run, n16 - n16_run, n_fused1, se1s, b16_p2 ? 3 : 2, max_terms, theta);
      if (rcs != GPX_OK) return drop_shadow(rcs);
    } else {
      slow_args = SlowArgs{off, n_g16 - n_g16_run, n_g16_run, n16 - n16_run, n_fused1, se1s, max_terms};
    }
  }
  if (n_fused_run > 0) {
    const int n_fused = n_fused_run, n16 = n16_run, n_g16 = n_g16_run, n_fused1 = n_fused1_run;
    const int n_active = n_dense + n_band + n_fused;
    int max_terms = 1;
    for (int i = n_dense + n_band; i < n_active; ++i) max_terms = std::max(max_terms, (int)bt->specs[order[i]].n_terms);
    const bool old_fused = n_fused > n16;  // the 64-row fused kernels run too
    if (ctx->profiling && old_fused)
      for (int e = 0; e < 4; ++e) HIPX(ctx, hipEventCreate(&fqe[e]));
    pe->n_band16 = n16;
    // (timing: the swept groups g_bcr .. g_wide only; the reductions' chains have their own events)
    pe->n_g16 = std::min(n_g16, g_wide) - g_bcr;
    pe->n_bcr = n16_bcr;
    for (int g = 0; g < pe->n_g16; ++g) {
      pe->g16_q[g] = g16_q[g_bcr + g];
      pe->g16_n[g] = g16_n[g_bcr + g];
      if (ctx->profiling)
        for (int e = 0; e < 4; ++e) HIPX(ctx, hipEventCreate(&pe->fq16[g][e]));
    }
    // the reference's kernel (one SquaredExponential term on one column) everywhere in the band16
    // class: its backward sweep's straight-line contraction
    bool se1 = true;
    for (int i = n_dense + n_band; i < n_dense + n_band + n16; ++i) {
      const gpx_kernel_spec& sp = bt->specs[order[i]];
      se1 = se1 && se1_spec(sp);
    }
    Run rf{bt, bt->d_active + n_dense + n_band, n_fused, s};
    rf.bcr_q = bcr_q;
    rf.bcr_wsp = &bt->bcr_ws;
    rf.bcr_capp = &bt->bcr_ws_cap;
    rf.ev16_g0 = g_bcr;
    const int ebf = band_fused_eval(rf, n16, n_g16, g16_q, g16_n, se1,
                    b16_p2 ? 3 : 2, n_fused1,
                    max_terms, (ctx->profiling && old_fused) ? fqe : nullptr, ctx->profiling ? pe->fq16 : nullptr);
    if (ebf != GPX_OK) return drop_shadow(ebf);
  }
  bp.mark();
  total.mark();
  HIPX(ctx, hipGetLastError());
  sc.lap(3);
  // one DMA into the pinned block: [info | theta (unchanged) | results]
  HIPX(ctx, hipMemcpyAsync(bt->h_io + bt->io_info_off, bt->d_io + bt->io_info_off,
                           bt->io_bytes - bt->io_info_off, hipMemcpyDeviceToHost, s));
  trace_mark(bt, 44, s);
  if (slow_args.off >= 0) {
    // the call completes here; its slow part follows on the same stream
    if (!bt->bulk_ev) HIPX(ctx, hipEventCreateWithFlags(&bt->bulk_ev, hipEventDisableTiming));
    HIPX(ctx, hipEventRecord(bt->bulk_ev, s));
    pe->bulk_done = bt->bulk_ev;
    const SlowArgs& a = slow_args;
    const int rcs = submit_slow(bt, s, order.data() + a.off, a.off, n_slow, a.n_g16, g16_q + a.g0, g16_n + a.g0, a.n16,
                                a.n1, a.se1, b16_p2 ? 3 : 2, a.max_terms, theta);
    if (rcs != GPX_OK) return drop_shadow(rcs);
  }
  sc.lap(4);
  if (n_slow > 0) {  // the call's own problems: [dense | band | bulk band16]
    pe->deferred_ids.assign(order.end() - n_slow, order.end());
    order.resize(order.size() - n_slow);
    pe->n_active = n_active - n_slow;
  }
  pe->order = std::move(order);
  pe->n_dense = n_dense;
  pe->n_band = n_band;
  pe->n_fused = n_fused_run;
  pe->n_fused1 = n_fused1_run;
  pe->shadow_ids = std::move(shadow_ids);
  pe->shadow_async = shadow_async;
  bt->pending_eval = std::move(pe);
  return GPX_OK;
}

int gpx_batch_lml_grad_complete(gpx_batch* bt, double* lml, double* grad, int32_t* info) {
  if (!bt) return GPX_BAD_ARG;
  gpx_ctx* ctx = bt->ctx;
  if (!bt->pending_eval) return fail(ctx, GPX_BAD_ARG, "no evaluation submitted on this batch");
  std::unique_ptr<gpx_batch::PendingEval> pe = std::move(bt->pending_eval);
  if (!lml || !grad || !info) return fail(ctx, GPX_BAD_ARG, "null output");
  HIPX(ctx, hipSetDevice(ctx->device));
  hipStream_t s = pe->s;
  SubClock sc(bt);
  if (pe->poll_tag > 0) {
    // a small-problem call: wait for every workgroup's flag (each is written after its results, a
    // system-scope fence between); the stream is asked now and then, so a failed launch ends the
    // wait with its error instead of a spin
    const volatile int* flags = reinterpret_cast<const volatile int*>(bt->h_sio + bt->io_flag_off);
    for (int i = 0, spins = 0; i < pe->n_active;) {
      if (flags[i] == pe->poll_tag) {
        ++i;
        continue;
      }
      if (++spins % 4096 == 0) {
        const hipError_t q = hipStreamQuery(s);
        if (q != hipErrorNotReady && q != hipSuccess) HIPX(ctx, q);
        if (q == hipSuccess && flags[i] != pe->poll_tag) {  // (finished without its flag: not expected)
          HIPX(ctx, hipStreamSynchronize(s));
          break;
        }
      }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
  } else if (pe->bulk_done) {  // (a slow part follows the call on its stream)
    HIPX(ctx, hipEventSynchronize(pe->bulk_done));
  } else {
    HIPX(ctx, hipStreamSynchronize(s));
  }
  if (pe->direct) {  // (the kernel wrote info and results into the coherent block)
    for (int i = 0; i < pe->n_active; ++i) {
      const int b = pe->order[i];
      bt->h_info[b] = reinterpret_cast<const int*>(bt->h_sio + bt->io_info_off)[b];
      std::memcpy(bt->h_results + (size_t)b * kResStride,
                  reinterpret_cast<const double*>(bt->h_sio + bt->io_res_off) + (size_t)b * kResStride,
                  sizeof(double) * kResStride);
    }
  }
  sc.lap(5);
  const int n_active = pe->n_active, n_dense = pe->n_dense, n_band = pe->n_band, n_fused = pe->n_fused;
  const int n_fused1 = pe->n_fused1, ng = pe->ng;
  const std::vector<int32_t>& order = pe->order;
  const double* theta = pe->theta.data();
  PhaseTimer& total = *pe->total;
  PhaseTimer& ct = *pe->ct;
  PhaseTimer& bp = *pe->bp;
  std::vector<PhaseTimer>& pts = pe->pts;
  hipEvent_t* kev = pe->kev;
  hipEvent_t* fqe = pe->fq;
  if (total.on) {
    bt->timing.factor_ms = bt->timing.alpha_ms = 0.0;
    for (int g = 0; g < ng; ++g) {
      bt->timing.factor_ms += pts[g].ms(0, 1) / ng;
      bt->timing.alpha_ms += pts[g].ms(1, 2) / ng;
    }
    // (the small-problem kernel of Np = 64 batches has no separate contraction launch to time)
    bt->timing.grad_ms = (n_dense > 0 && ct.ev.size() >= 3) ? ct.ms(0, 2) : 0.0;
    if (n_dense > 0 && kev[0]) {
      float kms = 0.f;
      (void)hipEventElapsedTime(&kms, kev[0], kev[1]);
      bt->timing.contract_ms_total += kms;
      bt->timing.contract_launches += 1.0;
      double f = 0.0;
      for (int i = 0; i < bt->Np; ++i) f += 2.0 * (i + 1) * (double)(bt->Np - i);
      bt->timing.contract_alg_flops += n_dense * f;
    }
    if (n_band + n_fused > 0) {
      bt->timing.band_ms_total += bp.ms(0, 1);
      bt->timing.band_calls += 1.0;
      bt->timing.band_evals += n_band + n_fused;
      for (int i = n_dense; i < n_active; ++i)
        bt->timing.band_p_sum += (i >= n_dense + n_band && i < n_dense + n_band + pe->n_band16) ? 1 : bt->h_bandp[order[i]];
    }
    if (pe->n_bcr > 0 && bt->bcr_ev[0]) {
      float fb = 0.f;
      (void)hipEventElapsedTime(&fb, bt->bcr_ev[0], bt->bcr_ev[1]);
      bt->timing.bcr_ms_total += fb;
      bt->timing.bcr_calls += 1.0;
      bt->timing.bcr_evals += pe->n_bcr;
    }
    for (int g = 0; g < pe->n_g16; ++g) {
      float f0 = 0.f, f1 = 0.f;
      (void)hipEventElapsedTime(&f0, pe->fq16[g][0], pe->fq16[g][1]);
      (void)hipEventElapsedTime(&f1, pe->fq16[g][2], pe->fq16[g][3]);
      bt->timing.band16_fwd_ms_total += f0;
      bt->timing.band16_bwd_ms_total += f1;
      bt->timing.band16_wave_ms += (double)pe->g16_n[g] * ((double)f0 + (double)f1);
      bt->timing.band16_launches += 1.0;
      bt->timing.band16_evals += pe->g16_n[g];
      bt->timing.band16_q_sum += (double)pe->g16_q[g] * pe->g16_n[g];
      bt->timing.band16_fwd_flops += pe->g16_n[g] * band16_flops(bt->Np, pe->g16_q[g], true);
      bt->timing.band16_bwd_flops += pe->g16_n[g] * band16_flops(bt->Np, pe->g16_q[g], false);
    }
    if (n_fused > pe->n_band16) {
      float f0 = 0.f, f1 = 0.f;
      (void)hipEventElapsedTime(&f0, fqe[0], fqe[1]);
      (void)hipEventElapsedTime(&f1, fqe[2], fqe[3]);
      bt->timing.band_fwd_ms_total += f0;
      bt->timing.band_bwd_ms_total += f1;
      bt->timing.band_fused_launches += 1.0;
      if (n_fused1 == 0) bt->timing.band_fused_p2_launches += 1.0;
      // the timed launch pair is the p <= 1 class's when there is one, else the p = 2 class's
      const int t0 = n_dense + n_band + pe->n_band16, t1 = n_fused1 > 0 ? t0 + n_fused1 : n_active;
      for (int i = t0; i < t1; ++i) {
        const int pb = bt->h_bandp[order[i]];
        bt->timing.band_fwd_flops += band_fused_flops(bt->Np, pb, true);
        bt->timing.band_bwd_flops += band_fused_flops(bt->Np, pb, false);
      }
    }
    bt->timing.predict_ms = 0.0;
    bt->timing.total_ms = total.ms(0, 1);
    bt->timing.gemm_flops = bt->flops_acc;
    bt->timing.eval_ms_total += total.ms(0, 1);
    bt->timing.evals += n_active;
  }
  int status = GPX_OK;
  // banded evaluations whose check failed are redone on the dense path below
  const char* et = getenv("GPX_BAND_TOL");
  const double band_tol = et ? atof(et) : 1e-6;
  std::vector<int32_t> redo;
  for (int i = 0; i < n_active; ++i) {
    const int b = order[i];
    const double* res = bt->h_results + (size_t)b * kResStride;
    info[b] = bt->h_info[b];
    const int np = bt->specs[b].n_params;
    if (i >= n_dense && info[b] == 0 && !(res[kResBandCheck] <= band_tol)) {
      redo.push_back(b);
      continue;
    }
    if (info[b] != 0) {
      status = GPX_NOT_PD;
      lml[b] = NAN;
      for (int p = 0; p <= np; ++p) grad[(size_t)b * GPX_THETA_STRIDE + p] = NAN;
      bt->fac_valid[b] = 0;
      continue;
    }
    lml[b] = res[0];
    for (int p = 0; p <= np; ++p) grad[(size_t)b * GPX_THETA_STRIDE + p] = res[1 + p];
    std::memcpy(&bt->fac_theta[(size_t)b * GPX_THETA_STRIDE], theta + (size_t)b * GPX_THETA_STRIDE,
                sizeof(double) * GPX_THETA_STRIDE);
    bt->fac_valid[b] = 1;
    bt->fac_band[b] = i >= n_dense;
  }
  for (int b : pe->deferred_ids) {  // (their results come with a later _complete / deferred_wait)
    info[b] = GPX_INFO_DEFERRED;
    lml[b] = NAN;
    for (int p = 0; p <= bt->specs[b].n_params; ++p) grad[(size_t)b * GPX_THETA_STRIDE + p] = NAN;
  }
  if (!bt->slow_out.empty()) {  // earlier calls' slow parts that have finished by now
    const int rcd = deliver_ready(bt, lml, grad, info, false);
    if (rcd != GPX_OK && rcd != GPX_NOT_PD) return rcd;
    if (rcd == GPX_NOT_PD) status = GPX_NOT_PD;
  }
  if (status == GPX_NOT_PD) last_error_slot() = "K + noise*I is not positive definite for some problem";
  if (bt->compact) {
    // band storage: the problems routed dense and those whose band check failed run on the
    // dense fallback slots
    if (total.on) bt->timing.band_fallbacks += (double)redo.size();
    std::vector<int32_t> ids;
    if (pe->shadow_async) {
      const int rc1 = shadow_collect(bt, pe->shadow_ids, lml, grad, info);
      if (rc1 != GPX_OK && rc1 != GPX_NOT_PD) return rc1;
      if (rc1 == GPX_NOT_PD) status = GPX_NOT_PD;
    } else {
      ids = pe->shadow_ids;
    }
    ids.insert(ids.end(), redo.begin(), redo.end());
    if (!ids.empty()) {
      const int rc2 = shadow_lml_grad(bt, ids, theta, lml, grad, info, s);
      if (rc2 != GPX_OK && rc2 != GPX_NOT_PD) return rc2;
      if (rc2 == GPX_NOT_PD) status = GPX_NOT_PD;
    }
    return status;
  }
  if (!redo.empty()) {
    if (total.on) bt->timing.band_fallbacks += (double)redo.size();
    bt->force_dense = 1;
    const int rc2 = gpx_batch_lml_grad(bt, (int)redo.size(), redo.data(), theta, lml, grad, info, s);
    bt->force_dense = 0;
    if (rc2 != GPX_OK && rc2 != GPX_NOT_PD) return rc2;
    if (rc2 == GPX_NOT_PD) status = GPX_NOT_PD;
  }
  return status;
}


int gpx_batch_lml_grad_query(gpx_batch* bt) {
  if (!bt) return GPX_BAD_ARG;
  if (!bt->pending_eval) return 1;
  hipError_t e = bt->pending_eval->bulk_done ? hipEventQuery(bt->pending_eval->bulk_done)
                                              : hipStreamQuery(bt->pending_eval->s);
  if (e == hipSuccess && bt->pending_eval->shadow_async) e = hipStreamQuery(bt->shadow_s);
  if (e == hipSuccess) return 1;
  if (e == hipErrorNotReady) return 0;
  return fail(bt->ctx, GPX_HIP_ERROR, std::string("hipStreamQuery: ") + hipGetErrorString(e));
}

int gpx_batch_band_width(gpx_batch* bt, int n_rows, const int32_t* rows, const double* theta, int32_t* p_out) {
  if (!bt) return GPX_BAD_ARG;
  if (n_rows < 0 || (n_rows > 0 && (!rows || !theta || !p_out))) return fail(bt->ctx, GPX_BAD_ARG, "bad band-width query");
  const int plim = band_limit(bt);
  for (int i = 0; i < n_rows; ++i) {
    const int b = rows[i];
    if (b < 0 || b >= bt->B) return fail(bt->ctx, GPX_BAD_ARG, "row out of range");
    bool pending = false;
    for (const auto& e : bt->pend) pending = pending || e.b == b;
    if (pending) {  // its band tables arrive with the next call's gather
      p_out[i] = -2;
      continue;
    }
    const int p = plim >= 0 ? band_width(bt, b, theta + (size_t)b * GPX_THETA_STRIDE) : -1;
    p_out[i] = (p >= 0 && p <= plim) ? p : -1;
  }
  return GPX_OK;
}

int gpx_batch_band_class(gpx_batch* bt, int n_rows, const int32_t* rows, const double* theta, int32_t* cls_out) {
  if (!bt) return GPX_BAD_ARG;
  if (n_rows < 0 || (n_rows > 0 && (!rows || !theta || !cls_out)))
    return fail(bt->ctx, GPX_BAD_ARG, "bad band-class query");
  const RouteLimits L = route_limits(bt);
  for (int i = 0; i < n_rows; ++i) {
    const int b = rows[i];
    if (b < 0 || b >= bt->B) return fail(bt->ctx, GPX_BAD_ARG, "row out of range");
    bool pending = false;
    for (const auto& e : bt->pend) pending = pending || e.b == b;
    if (pending) {
      cls_out[i] = -2;
      continue;
    }
    int w = -1;
    const RouteKind k = route_one(bt, b, theta + (size_t)b * GPX_THETA_STRIDE, L, w);
    cls_out[i] = k == kRouteBand16 ? w : (k == kRouteFused || k == kRouteBand) ? (L.q16lim > 0 ? 32 : 16) + w : -1;
  }
  return GPX_OK;
}

int gpx_batch_lml_grad(gpx_batch* bt, int n_active, const int32_t* active, const double* theta,
                       double* lml, double* grad, int32_t* info, void* stream) {
  if (!bt) return GPX_BAD_ARG;
  if (!lml || !grad || !info) return fail(bt->ctx, GPX_BAD_ARG, "null output");
  const int rc = gpx_batch_lml_grad_submit(bt, n_active, active, theta, stream);
  if (rc != GPX_OK) return rc;
  return gpx_batch_lml_grad_complete(bt, lml, grad, info);
}

// Shared body of gpx_batch_predict (var != nullptr) and gpx_batch_predict_full_cov
// (cov != nullptr).
static int predict_impl(gpx_batch* bt, int n_active, const int32_t* active, const double* theta,
                        const double* Xnew, int M, int add_noise, double* mean, double* var,
                        double* cov, int32_t* info, void* stream, bool train = false, bool rows = false) {
  if (!bt) return GPX_BAD_ARG;
  gpx_ctx* ctx = bt->ctx;
  if ((!train && (!Xnew || M <= 0)) || !mean || !(var || cov) || !info)
    return fail(ctx, GPX_BAD_ARG, "bad predict args");
  if (!train && ((long long)M + 63) / 64 * 64 > kGemmMaxLd)
    return fail(ctx, GPX_BAD_ARG, "too many prediction points for one call (kGemmMaxLd): split Xnew");
  if (!bt->deferred.empty() && active)
    for (int i = 0; i < n_active; ++i)
      if (active[i] >= 0 && active[i] < bt->B && bt->deferred[active[i]])
        return fail(ctx, GPX_BAD_ARG, "a problem has a deferred evaluation in flight");
  HIPX(ctx, hipSetDevice(ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  SubClock pclk(bt);
  struct PredLap {  // (GPX_SUBMIT_STATS: the call's host time, whatever path it returns by)
    SubClock& c;
    ~PredLap() { c.lap(8); }
  } plap{pclk};
  // band storage: only predict at the training inputs from a cached banded factor at exactly
  // this θ stays here; every other problem is predicted on the dense fallback slots, one by one
  std::vector<int32_t> keep;
  int shadow_status = GPX_OK;
  // rows (train only): outputs [n_active, Nmax], row i for active[i]; orow[b] = i
  std::vector<int32_t> orow;
  if (rows) {
    if (!train || n_active <= 0 || n_active > bt->B || !active) return fail(ctx, GPX_BAD_ARG, "bad active set");
    orow.assign(bt->B, -1);
    for (int i = 0; i < n_active; ++i) {
      if (active[i] < 0 || active[i] >= bt->B) return fail(ctx, GPX_BAD_ARG, "active index out of range");
      // a slot listed twice would leave an earlier output row unwritten (uninitialised memory
      // returned as a prediction)
      if (orow[active[i]] >= 0) return fail(ctx, GPX_BAD_ARG, "a slot appears twice in the active set");
      orow[active[i]] = i;
    }
    for (int& o : orow) o = std::max(o, 0);  // (rows not in the call are never read)
  }
  auto out_row = [&](int b) -> size_t { return rows ? (size_t)orow[b] : (size_t)b; };
  if (bt->compact) {
    if (n_active <= 0 || n_active > bt->B || !active || !theta)
      return fail(ctx, GPX_BAD_ARG, "bad active set / theta");
    gpx_batch* sh = bt->shadow;
    const size_t nx = (size_t)bt->Nmax * bt->D;
    std::vector<double> th((size_t)kShadowSlots * GPX_THETA_STRIDE, 1.0);
    std::vector<int32_t> inf(kShadowSlots, 0);
    const int32_t act0 = 0;
    for (int i = 0; i < n_active; ++i) {
      const int b = active[i];
      if (b < 0 || b >= bt->B) return fail(ctx, GPX_BAD_ARG, "active index out of range");
      const bool cached = train && bt->fac_valid[b] && bt->fac_band[b] &&
                          std::memcmp(&bt->fac_theta[(size_t)b * GPX_THETA_STRIDE],
                                      theta + (size_t)b * GPX_THETA_STRIDE,
                                      sizeof(double) * GPX_THETA_STRIDE) == 0;
      if (cached) {
        keep.push_back(b);
        continue;
      }
      int rc = gpx_batch_rebind_device(sh, 0, bt->n[b], bt->X + b * nx, bt->Y + (size_t)b * bt->Nmax,
                                       &bt->specs[b], s);
      if (rc != GPX_OK) return rc;
      std::memcpy(th.data(), theta + (size_t)b * GPX_THETA_STRIDE, sizeof(double) * GPX_THETA_STRIDE);
      inf[0] = 0;
      if (train)
        rc = predict_impl(sh, 1, &act0, th.data(), nullptr, 0, add_noise, mean + out_row(b) * bt->Nmax,
                          var + out_row(b) * bt->Nmax, nullptr, inf.data(), s, true);
      else
        rc = predict_impl(sh, 1, &act0, th.data(), Xnew + (size_t)b * M * bt->D, M, add_noise,
                          mean + (size_t)b * M, var ? var + (size_t)b * M : nullptr,
                          cov ? cov + (size_t)b * M * M : nullptr, inf.data(), s);
      if (rc != GPX_OK && rc != GPX_NOT_PD) return rc;
      bt->timing.shadow_predicts += 1;
      info[b] = inf[0];
      if (rc == GPX_NOT_PD) shadow_status = GPX_NOT_PD;
    }
    if (n_active > (int)keep.size()) {
      SubClock sc2(bt);
      sc2.t = pclk.t;
      sc2.lap(10);  // (from the call's start: the shadow slots' synchronous predicts)
    }
    if (keep.empty()) return shadow_status;
    active = keep.data();
    n_active = (int)keep.size();
  }
  int rc = upload_common(bt, n_active, active, theta, s, true);
  if (rc != GPX_OK) return rc;
  // re-factorise the problems whose cached factor is not at exactly this theta. A cached
  // block-banded factorisation (gpx_band.hip) serves predict at the training inputs (it holds
  // α and the diagonal of K⁻¹); any other predict re-factorises densely.
  std::vector<int> refac, band_cached;
  for (int i = 0; i < n_active; ++i) {
    const int b = active[i];
    const bool same = bt->fac_valid[b] &&
                      std::memcmp(&bt->fac_theta[(size_t)b * GPX_THETA_STRIDE],
                                  theta + (size_t)b * GPX_THETA_STRIDE,
                                  sizeof(double) * GPX_THETA_STRIDE) == 0;
    if (!same || (bt->fac_band[b] && !train)) refac.push_back(b);
    else if (bt->fac_band[b]) band_cached.push_back(b);
  }
  // the asynchronous case (see below) records no phase events: destroying an event the device
  // has not reached yet would wait for it
  const bool async = train && refac.empty() && stream;
  PhaseTimer pt(ctx->profiling != 0 && !async, s);
  bt->flops_acc = 0.0;
  pt.mark();
  // device active list: [dense-factored problems | band-cached problems]
  std::vector<int32_t> order;
  order.reserve(n_active);
  for (int i = 0; i < n_active; ++i)
    if (std::find(band_cached.begin(), band_cached.end(), active[i]) == band_cached.end())
      order.push_back(active[i]);
  const int n_dense = (int)order.size();
  order.insert(order.end(), band_cached.begin(), band_cached.end());
  if (!refac.empty()) {
    HIPX(ctx, hipMemcpyAsync(bt->d_active, refac.data(), sizeof(int) * refac.size(),
                             hipMemcpyHostToDevice, s));
    const Run rr{bt, bt->d_active, (int)refac.size(), s};
    if (small64_on(bt)) {
      small64_eval(rr, false);
    } else {
      factor(rr);
      alpha_solve(rr);
    }
  }
  if (!refac.empty() || n_dense < n_active)
    HIPX(ctx, hipMemcpyAsync(bt->d_active, order.data(), sizeof(int) * n_active, hipMemcpyHostToDevice, s));
  pt.mark();
  const int Np = bt->Np;
  if (train) {
    TrainPredArgs ta{};
    ta.active = bt->d_active; ta.W = bt->W; ta.sW = mat_stride(bt); ta.ld = Np;
    ta.alpha = bt->alpha; ta.sVec = Np; ta.Y = bt->Y; ta.sY = bt->Nmax; ta.nvalid = bt->d_n;
    ta.specs = bt->d_specs; ta.theta = bt->d_theta; ta.add_noise = add_noise;
    ta.mean = mean; ta.var = var; ta.sOut = bt->Nmax;
    if (rows) {
      HIPX(ctx, hipMemcpyAsync(bt->d_orow, orow.data(), sizeof(int) * bt->B, hipMemcpyHostToDevice, s));
      ta.orow = bt->d_orow;
    }
    if (n_dense > 0) launch_train_pred(ta, n_dense, Np, s);
    if (n_dense < n_active) {
      // banded: diag(K⁻¹) from the selected inverse in K's diagonal blocks
      TrainPredArgs tb = ta;
      tb.active = bt->d_active + n_dense; tb.W = bt->K; tb.ld = mat_ld(bt);
      launch_band_train_pred(tb, n_active - n_dense, Np, s);
    }
  } else {
  const int Mp = ((M + 63) / 64) * 64;
  // cross-covariance workspace [B][Np][Mp]
  const size_t need = (size_t)bt->B * Np * Mp;
  double* kxs;
  if ((size_t)Mp <= (size_t)Np) {
    kxs = bt->L;  // L is dead once W is formed
  } else {
    const int e = ensure(ctx, bt->kxs, bt->kxs_cap, need);
    if (e != GPX_OK) return e;
    kxs = bt->kxs;
  }
  const long long skx = (long long)Np * Mp;
  BuildArgs ba{};
  ba.active = bt->d_active; ba.specs = bt->d_specs; ba.theta = bt->d_theta; ba.nvalid = bt->d_n;
  ba.X = bt->X; ba.sX = (long long)bt->Nmax * bt->D; ba.X2 = Xnew; ba.sX2 = (long long)M * bt->D;
  ba.D = bt->D; ba.m2 = M; ba.out = kxs; ba.sOut = skx; ba.ldo = Mp; ba.rows = Np; ba.cols = Mp;
  ba.symmetric = 0;
  launch_build(ba, n_active, s);
  // mean = Kxsᵀ α
  TrmvArgs t{};
  t.active = bt->d_active; t.Wm = kxs; t.sW = skx; t.ld = Mp; t.x = bt->alpha; t.sx = Np;
  t.nvalid = nullptr; t.y = mean; t.sy = M; t.rows = Np; t.cols = M; t.lower = 0;
  launch_trmv_t(t, n_active, s);
  if (cov) {
    // A = W · Kxs stored; cov = K(X*,X*) − AᵀA (padded rows/cols of A are exactly zero)
    double* abuf;
    if ((size_t)Mp <= (size_t)Np) {
      abuf = bt->K;  // K is dead once W is formed
    } else {
      const int e = ensure(ctx, bt->abuf, bt->abuf_cap, need);
      if (e != GPX_OK) return e;
      abuf = bt->abuf;
    }
    const long long scv = (long long)Mp * Mp;
    {
      const int e = ensure(ctx, bt->covw, bt->covw_cap, (size_t)bt->B * scv);
      if (e != GPX_OK) return e;
    }
    BuildArgs kb = ba;
    kb.X = Xnew; kb.sX = (long long)M * bt->D; kb.rows_valid = M; kb.out = bt->covw; kb.sOut = scv;
    kb.ldo = Mp; kb.rows = Mp; kb.cols = Mp;
    launch_build(kb, n_active, s);
    const Run rr{bt, bt->d_active, n_active, s};
    GemmArgs ga = gemm_args(bt->W, Np, kxs, Mp, abuf, Mp, 0, Np, Mp, Np, TRI_KMAX_I, 0, 1.0, 0.0);
    ga.sA = mat_stride(bt); ga.sB = skx; ga.sC = skx;
    gemm(rr, ga, EPI_STORE, false, false);
    GemmArgs gc = gemm_args(abuf, Mp, abuf, Mp, bt->covw, Mp, 0, Mp, Mp, Np, 0, 0, -1.0, 1.0);
    gc.sA = skx; gc.sB = skx; gc.sC = scv;
    gemm(rr, gc, EPI_STORE, true, false);
    for (int i = 0; i < n_active; ++i) {
      const int b = active[i];
      HIPX(ctx, hipMemcpy2DAsync(cov + (size_t)b * M * M, sizeof(double) * M,
                                 bt->covw + (size_t)b * scv, sizeof(double) * Mp,
                                 sizeof(double) * M, M, hipMemcpyDeviceToDevice, s));
    }
  } else {
  // A = W · Kxs with fused column sum of squares
  GemmArgs g = gemm_args(bt->W, Np, kxs, Mp, nullptr, Mp, 0, Np, Mp, Np, TRI_KMAX_I, 0, 1.0, 0.0);
  g.sA = mat_stride(bt); g.sB = skx; g.sC = 0;
  g.small_tiles = bt->small_tiles;  // the tile size gemm() will launch with
  const int bm = gemm_tile(g, n_active);
  const int nrt = Np / bm;
  const size_t pneed = (size_t)bt->B * nrt * Mp;
  {
    const int e = ensure(ctx, bt->pvp, bt->pvp_cap, pneed);
    if (e != GPX_OK) return e;
  }
  g.partial = bt->pvp; g.sPartial = (long long)nrt * Mp;
  gemm(Run{bt, bt->d_active, n_active, s}, g, EPI_COLSUMSQ, false, false);
  PredVarArgs pv{};
  pv.active = bt->d_active; pv.partial = bt->pvp; pv.sPartial = (long long)nrt * Mp;
  pv.nrowtiles = nrt; pv.ldp = Mp; pv.Xnew = Xnew; pv.sXnew = (long long)M * bt->D; pv.D = bt->D;
  pv.specs = bt->d_specs; pv.theta = bt->d_theta; pv.M = M; pv.add_noise = add_noise;
  pv.var = var; pv.sVar = M;
  launch_predvar(pv, n_active, s);
  }
  }
  pt.mark();
  HIPX(ctx, hipGetLastError());
  if (async) {
    // every problem predicted from its cached factor at exactly this θ (the fit's last
    // evaluation): nothing can fail, so the call returns without waiting for the device — the
    // outputs are ready in the order of the CALLER's stream (not with stream == NULL: the
    // library's own non-blocking stream is not ordered with the caller's default stream);
    // the upload out of h_io is fenced by io_ev
    if (!bt->io_ev) HIPX(ctx, hipEventCreateWithFlags(&bt->io_ev, hipEventDisableTiming));
    HIPX(ctx, hipEventRecord(bt->io_ev, s));
    bt->io_pending = true;
    bt->io_stream = s;
    for (int i = 0; i < n_active; ++i) info[active[i]] = 0;
    if (shadow_status == GPX_NOT_PD) last_error_slot() = "K + noise*I is not positive definite for some problem";
    return shadow_status;
  }
  HIPX(ctx, hipMemcpyAsync(bt->h_info, bt->d_info, sizeof(int) * bt->B, hipMemcpyDeviceToHost, s));
  HIPX(ctx, hipStreamSynchronize(s));
  if (pt.on) {
    bt->timing.factor_ms = pt.ms(0, 1);
    bt->timing.alpha_ms = 0.0;
    bt->timing.grad_ms = 0.0;
    bt->timing.predict_ms = pt.ms(1, 2);
    bt->timing.total_ms = pt.ms(0, 2);
    bt->timing.gemm_flops = bt->flops_acc;
  }
  int status = GPX_OK;
  for (int i = 0; i < n_active; ++i) {
    const int b = active[i];
    // info is only (re)computed for re-factorised problems; cached ones were OK
    const bool was_refac = std::find(refac.begin(), refac.end(), b) != refac.end();
    info[b] = was_refac ? bt->h_info[b] : 0;
    if (info[b] != 0) {
      status = GPX_NOT_PD;
      bt->fac_valid[b] = 0;
    } else if (was_refac) {
      std::memcpy(&bt->fac_theta[(size_t)b * GPX_THETA_STRIDE], theta + (size_t)b * GPX_THETA_STRIDE,
                  sizeof(double) * GPX_THETA_STRIDE);
      bt->fac_valid[b] = 1;
      bt->fac_band[b] = 0;
    }
  }
  if (shadow_status == GPX_NOT_PD) status = GPX_NOT_PD;
  if (status == GPX_NOT_PD) last_error_slot() = "K + noise*I is not positive definite for some problem";
  return status;
}

int gpx_batch_predict(gpx_batch* bt, int n_active, const int32_t* active, const double* theta,
                      const double* Xnew, int M, int add_noise, double* mean, double* var,
                      int32_t* info, void* stream) {
  if (!var) return bt ? fail(bt->ctx, GPX_BAD_ARG, "bad predict args") : GPX_BAD_ARG;
  return predict_impl(bt, n_active, active, theta, Xnew, M, add_noise, mean, var, nullptr, info,
                      stream);
}

int gpx_batch_predict_train(gpx_batch* bt, int n_active, const int32_t* active, const double* theta,
                            int add_noise, double* mean, double* var, int32_t* info, void* stream) {
  return predict_impl(bt, n_active, active, theta, nullptr, 0, add_noise, mean, var, nullptr, info,
                      stream, true);
}

int gpx_batch_predict_train_rows(gpx_batch* bt, int n_active, const int32_t* active, const double* theta,
                                 int add_noise, double* mean, double* var, int32_t* info, void* stream) {
  return predict_impl(bt, n_active, active, theta, nullptr, 0, add_noise, mean, var, nullptr, info,
                      stream, true, true);
}

int gpx_batch_predict_full_cov(gpx_batch* bt, int n_active, const int32_t* active,
                               const double* theta, const double* Xnew, int M, double* mean,
                               double* cov, int32_t* info, void* stream) {
  if (!cov) return bt ? fail(bt->ctx, GPX_BAD_ARG, "bad predict args") : GPX_BAD_ARG;
  return predict_impl(bt, n_active, active, theta, Xnew, M, 0, mean, nullptr, cov, info, stream);
}

int gpx_batch_reset_timing(gpx_batch* bt) {
  if (!bt) return GPX_BAD_ARG;
  bt->timing = gpx_timing{};
  for (double& v : bt->sub_s) v = 0.0;
  bt->sub_calls = bt->box_syncs = 0;
  return GPX_OK;
}

int gpx_batch_last_timing(const gpx_batch* bt, gpx_timing* out) {
  if (!bt || !out) return GPX_BAD_ARG;
  *out = bt->timing;
  return GPX_OK;
}

int gpx_batch_set_deferred(gpx_batch* bt, int q) {
  if (!bt) return GPX_BAD_ARG;
  if (q < 0 && !bt->slow_out.empty())
    return fail(bt->ctx, GPX_BAD_ARG, "deferred evaluations in flight (gpx_batch_deferred_wait first)");
  bt->defer_q = q < 0 ? -1 : q;
  if (bt->deferred.size() != (size_t)bt->B) bt->deferred.assign(bt->B, 0);
  return GPX_OK;
}

int gpx_batch_set_band_route(gpx_batch* bt, int route) {
  if (!bt) return GPX_BAD_ARG;
  if (route != GPX_BAND_ROUTE_SWEEPS && route != GPX_BAND_ROUTE_BCR && route != GPX_BAND_ROUTE_AUTO)
    return fail(bt->ctx, GPX_BAD_ARG, "unknown band route");
  if (bt->pending_eval) return fail(bt->ctx, GPX_BAD_ARG, "an evaluation is submitted on this batch");
  bt->band_route = route;
  return GPX_OK;
}

int gpx_batch_deferred_wait(gpx_batch* bt, double* lml, double* grad, int32_t* info) {
  if (!bt) return GPX_BAD_ARG;
  if (!lml || !grad || !info) return fail(bt->ctx, GPX_BAD_ARG, "null output");
  // a delivered row whose band check failed is re-evaluated densely through this batch (or its
  // fallback slots), which an evaluation still submitted on it would refuse: refuse before any
  // slow part is taken off the queue, so nothing is lost
  if (bt->pending_eval)
    return fail(bt->ctx, GPX_BAD_ARG, "an evaluation is submitted on this batch: complete it before deferred_wait");
  HIPX(bt->ctx, hipSetDevice(bt->ctx->device));
  return deliver_ready(bt, lml, grad, info, true);
}

int gpx_batch_deferred_rows(const gpx_batch* bt, int32_t* rows, int cap) {
  if (!bt) return 0;
  int n = 0;
  for (const auto& r : bt->slow_out)
    for (int b : r->ids) {
      if (rows && n < cap) rows[n] = b;
      ++n;
    }
  return n;
}

// Diagnostic: the band16 sweeps' per-wavefront residency records (BandFusedArgs::wtrace)
int gpx_batch_wave_trace(gpx_batch* bt, unsigned int cap) {
  if (!bt) return GPX_BAD_ARG;
  gpx_ctx* ctx = bt->ctx;
  HIPX(ctx, hipSetDevice(ctx->device));
  HIPX(ctx, hipDeviceSynchronize());  // no sweep is writing the old buffer
  if (bt->d_wtrace) (void)hipFree(bt->d_wtrace);
  if (bt->d_wtrace_n) (void)hipFree(bt->d_wtrace_n);
  bt->d_wtrace = nullptr;
  bt->d_wtrace_n = nullptr;
  bt->wtrace_cap = 0;
  if (cap == 0) return GPX_OK;
  HIPX(ctx, hipMalloc(&bt->d_wtrace, sizeof(unsigned long long) * 3 * (size_t)cap));
  HIPX(ctx, hipMalloc(&bt->d_wtrace_n, sizeof(unsigned int)));
  HIPX(ctx, hipMemset(bt->d_wtrace_n, 0, sizeof(unsigned int)));
  bt->wtrace_cap = cap;
  return GPX_OK;
}

int gpx_batch_wave_trace_read(gpx_batch* bt, unsigned long long* out, unsigned int cap, unsigned int* n_out) {
  if (!bt || !n_out || (cap > 0 && !out)) return GPX_BAD_ARG;
  gpx_ctx* ctx = bt->ctx;
  *n_out = 0;
  if (!bt->d_wtrace) return GPX_OK;
  HIPX(ctx, hipSetDevice(ctx->device));
  HIPX(ctx, hipDeviceSynchronize());
  unsigned int n = 0;
  HIPX(ctx, hipMemcpy(&n, bt->d_wtrace_n, sizeof(n), hipMemcpyDeviceToHost));
  n = std::min(n, std::min(cap, bt->wtrace_cap));
  if (n > 0) HIPX(ctx, hipMemcpy(out, bt->d_wtrace, sizeof(unsigned long long) * 3 * (size_t)n, hipMemcpyDeviceToHost));
  HIPX(ctx, hipMemset(bt->d_wtrace_n, 0, sizeof(unsigned int)));
  *n_out = n;
  return GPX_OK;
}

}  // extern "C"
