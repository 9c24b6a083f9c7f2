// gpx_svgp.hip — C ABI and host orchestration of the SVGP ELBO / gradient / predict path
// (the reference's gpflow.models.SVGP at test_scripts/SVGP.py:461-478 and
// test_scripts/GPR.py:118-138: whitened q(u) = N(q_mu, q_sqrt q_sqrtᵀ), Gaussian likelihood).
//
// With W = L⁻¹ (L = chol(Kmm + 1e-6 I)), u = Wᵀ q_mu, S = q_sqrt q_sqrtᵀ, P = Wᵀ(S − I)W,
// G = Kmn Kmnᵀ, Ĝ = W G Wᵀ, c = −s/(2σ²), s = num_data / n_total:
//   μ = Kmnᵀ u,   Σ_n v_n = Σ k_nn + tr((S − I) Ĝ)
//   ELBO = s (−n/2 log 2πσ² − (Σ(y−μ)² + Σ v)/(2σ²)) − KL
//   K̄mn  = u g_μᵀ + 2c P Kmn            (g_μ = s (y − μ)/σ²)
//   Lᵀ L̄ = −(q_mu âᵀ + 2c (S − I) Ĝ)   (â = W Kmn g_μ), K̄mm = sym(Wᵀ Φ(Lᵀ L̄) W)
//   ∂q_mu = â − q_mu,  ∂q_sqrt = tril(2c Ĝ q_sqrt − q_sqrt + diag(1/q_sqrt_ii))
//   ∂θ = Σ K̄mn ∘ ∂Kmn + Σ K̄mm ∘ ∂Kmm + c Σ ∂k_nn;   ∂Z likewise through ∂k/∂z
// (derivation checked against the autodiff-shaped oracle/svgp_oracle.py, which is pinned by
// finite differences). The data-size work is two MFMA GEMMs of M²N (split-K SYRK for G,
// Y = 2c P Kmn) plus O(MN) element passes; everything after the per-shard partial sums is
// O(M³) and replicated, so N shards over GPUs with one all-reduce of the partial buffer.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>
#include "gpx_host.h"

using namespace gpx;

namespace {
constexpr double kJitter = 1e-6;  // gpflow.config.default_jitter()
constexpr int kScalars = 4;       // Σ(y−μ)², Σ k_nn, n_local, 0
}  // namespace

struct gpx_svgp {
  gpx_ctx* ctx = nullptr;
  int N = 0, M = 0, D = 0, Mp = 0, Ncols = 0, nc = 1, chunkK = 64, rows_chunk = 64;
  const double* X = nullptr;
  const double* Y = nullptr;
  gpx_kernel_spec spec{};
  double num_data = 0.0;
  long long n_total = 0;
  gpx_batch* kmm = nullptr;  // Kmm factorisation (B = 1, X = Z)
  double *dZ = nullptr, *dYdummy = nullptr, *d_theta = nullptr;
  double *dq = nullptr, *dR = nullptr, *u = nullptr, *mu = nullptr, *g = nullptr;
  double *Sm1 = nullptr, *T = nullptr, *P = nullptr, *Gh = nullptr, *X1 = nullptr, *GR = nullptr;
  double *Phi = nullptr, *Sb = nullptr, *ahat = nullptr, *Rbar = nullptr;
  double *Kmn = nullptr, *Ybuf = nullptr, *Gpart = nullptr;
  double *part = nullptr;     // the all-reduced per-shard partial sums
  bool own_part = true;       // false once the caller bound its own buffer
  long long off_G = 0, off_w = 0, off_th = 0, off_z = 0, off_sc = 0, part_len = 0;
  double *pth = nullptr, *pz = nullptr, *pw = nullptr, *pres = nullptr, *ptr = nullptr, *fin = nullptr;
  size_t pth_cap = 0, pz_cap = 0, pw_cap = 0;
  int* d_iota = nullptr;
  // predict workspace
  double *Kms = nullptr, *V = nullptr, *pA = nullptr, *pB = nullptr;
  size_t kms_cap = 0, pa_cap = 0, pb_cap = 0;
  // host staging
  std::vector<double> h_q, h_part_small, h_fin, h_ahat;
  double* h_R = nullptr;     // pinned [Mp][Mp] q_sqrt staging (upper part stays zero)
  double* h_Rbar = nullptr;  // pinned [Mp][Mp] ∂ELBO/∂q_sqrt staging
  std::vector<double> h_theta;
  double h_nloc = 0.0;
  int h_info = 0;
  bool local_done = false;
};

namespace {

int rows_alloc(gpx_svgp* sv, const RowsArgs& ra) {
  int e = ensure(sv->ctx, sv->pth, sv->pth_cap, (size_t)rows_blocks(ra) * GPX_THETA_STRIDE);
  if (e != GPX_OK) return e;
  e = ensure(sv->ctx, sv->pz, sv->pz_cap, (size_t)rows_chunks(ra) * sv->Mp * sv->D);
  if (e != GPX_OK) return e;
  return ensure(sv->ctx, sv->pw, sv->pw_cap, (size_t)rows_chunks(ra) * sv->Mp);
}

void sum_into(const double* src, long long stride, int nb, long long width, double* dst, int acc,
              hipStream_t s) {
  SumArgs a{src, stride, nb, width, dst, acc};
  launch_sum(a, s);
}

// theta check + uploads shared by the ELBO and predict paths (all on stream s).
int prelude(gpx_svgp* sv, const double* theta, const double* Z, const double* q_mu,
            const double* q_sqrt, hipStream_t s) {
  gpx_ctx* ctx = sv->ctx;
  if (!theta || !Z || !q_mu || !q_sqrt) return fail(ctx, GPX_BAD_ARG, "null svgp argument");
  const int np = sv->spec.n_params, M = sv->M, Mp = sv->Mp;
  for (int p = 0; p <= np; ++p)
    if (!(theta[p] > 0.0) || !std::isfinite(theta[p]))
      return fail(ctx, GPX_BAD_ARG, "theta must be finite and > 0 (constrained space)");
  for (int i = 0; i < M; ++i)
    if (!(q_sqrt[(size_t)i * M + i] != 0.0)) return fail(ctx, GPX_BAD_ARG, "q_sqrt has a zero diagonal");
  sv->h_theta.assign(theta, theta + GPX_THETA_STRIDE);
  std::vector<double> th_kmm(sv->h_theta);
  th_kmm[np] = kJitter;
  const int32_t act0 = 0;
  int rc = upload_common(sv->kmm, 1, &act0, th_kmm.data(), s);
  if (rc != GPX_OK) return rc;
  HIPX(ctx, hipMemcpyAsync(sv->d_theta, sv->h_theta.data(), sizeof(double) * GPX_THETA_STRIDE,
                           hipMemcpyHostToDevice, s));
  HIPX(ctx, hipMemcpyAsync(sv->dZ, Z, sizeof(double) * M * sv->D, hipMemcpyHostToDevice, s));
  sv->h_q.assign(Mp, 0.0);
  std::memcpy(sv->h_q.data(), q_mu, sizeof(double) * M);
  for (int i = 0; i < M; ++i)
    std::memcpy(&sv->h_R[(size_t)i * Mp], q_sqrt + (size_t)i * M, sizeof(double) * (i + 1));
  HIPX(ctx, hipMemcpyAsync(sv->dq, sv->h_q.data(), sizeof(double) * Mp, hipMemcpyHostToDevice, s));
  HIPX(ctx, hipMemcpyAsync(sv->dR, sv->h_R, sizeof(double) * Mp * Mp, hipMemcpyHostToDevice, s));
  return GPX_OK;
}

// Kmm = k(Z,Z) + jitter I -> W = L⁻¹ (recursive Cholesky-and-inverse), u = Wᵀ q_mu.
void factor_u(gpx_svgp* sv, hipStream_t s) {
  const Run r{sv->kmm, sv->kmm->d_active, 1, s};
  factor(r);
  TrmvArgs t{};
  t.active = sv->kmm->d_active; t.Wm = sv->kmm->W; t.sW = 0; t.ld = sv->Mp; t.x = sv->dq; t.sx = 0;
  t.nvalid = nullptr; t.y = sv->u; t.sy = 0; t.rows = t.cols = sv->Mp; t.lower = 1;
  launch_trmv_t(t, 1, s);
}

bool single_term(const gpx_svgp* sv) { return sv->spec.n_terms == 1; }

int check_info(gpx_svgp* sv, int32_t* info, hipStream_t s) {
  gpx_ctx* ctx = sv->ctx;
  HIPX(ctx, hipMemcpyAsync(&sv->h_info, sv->kmm->d_info, sizeof(int), hipMemcpyDeviceToHost, s));
  HIPX(ctx, hipStreamSynchronize(s));
  if (info) *info = sv->h_info;
  if (sv->h_info != 0) return fail(ctx, GPX_NOT_PD, "Kmm + jitter I is not positive definite");
  return GPX_OK;
}

}  // namespace

extern "C" {

int gpx_svgp_create(gpx_ctx* ctx, int N, int M, int D, const double* X, const double* Y,
                    const gpx_kernel_spec* spec, double num_data, long long n_total,
                    gpx_svgp** out) {
  if (!ctx || !out) return GPX_BAD_ARG;
  *out = nullptr;
  if (N < 1 || M < 1 || D < 1 || D > GPX_MAX_DIM || !X || !Y || !spec || !(num_data > 0.0) ||
      n_total < N)
    return fail(ctx, GPX_BAD_ARG, "bad svgp dimensions or null pointer");
  HIPX(ctx, hipSetDevice(ctx->device));
  gpx_svgp* sv = new gpx_svgp();
  sv->ctx = ctx; sv->N = N; sv->M = M; sv->D = D; sv->X = X; sv->Y = Y; sv->spec = *spec;
  sv->num_data = num_data; sv->n_total = n_total;
  sv->Mp = ((M + kLeaf - 1) / kLeaf) * kLeaf;
  const int Mp = sv->Mp;
  // split-K chunks for G = Kmn Kmnᵀ: enough (problem, tile) pairs to fill the chip
  const int n64 = (N + 63) / 64 * 64;
  sv->nc = std::max(1, std::min(32, n64 / 1024));
  sv->chunkK = ((n64 + sv->nc - 1) / sv->nc + 63) / 64 * 64;
  sv->Ncols = sv->nc * sv->chunkK;
  sv->rows_chunk = rows_chunk_for(D);
  if (sv->Ncols > kGemmMaxLd || Mp > kGemmMaxLd) {
    delete sv;
    return fail(ctx, GPX_BAD_ARG, "svgp shard too large for the GEMM buffer-load window "
                                  "(N <= ~2.1M rows per gpx_svgp): shard the data over more objects");
  }
  auto bail = [&](const std::string& m) {
    gpx_svgp_destroy(sv);
    return fail(ctx, GPX_HIP_ERROR, m);
  };
  if (hipMalloc(&sv->dZ, sizeof(double) * Mp * D) != hipSuccess ||
      hipMalloc(&sv->dYdummy, sizeof(double) * Mp) != hipSuccess)
    return bail("out of device memory");
  if (hipMemset(sv->dZ, 0, sizeof(double) * Mp * D) != hipSuccess ||
      hipMemset(sv->dYdummy, 0, sizeof(double) * Mp) != hipSuccess)
    return bail("memset failed");
  const int32_t nM = M;
  int rc = gpx_batch_create(ctx, 1, M, D, sv->dZ, sv->dYdummy, &nM, spec, &sv->kmm);
  if (rc != GPX_OK) {
    gpx_svgp_destroy(sv);
    return rc;
  }
  sv->kmm->small_tiles = 1;   // every M x M launch here is one problem: size tiles to fill the chip
  const size_t mm = (size_t)Mp * Mp;
  sv->off_G = 0;
  sv->off_w = (long long)mm;
  sv->off_th = sv->off_w + Mp;
  sv->off_z = sv->off_th + GPX_THETA_STRIDE;
  sv->off_sc = sv->off_z + (long long)Mp * D;
  sv->part_len = sv->off_sc + kScalars;
  double** mats[] = {&sv->Sm1, &sv->T, &sv->P, &sv->Gh, &sv->X1, &sv->GR, &sv->Phi, &sv->Sb, &sv->Rbar, &sv->dR};
  for (double** p : mats)
    if (hipMalloc(p, sizeof(double) * mm) != hipSuccess || hipMemset(*p, 0, sizeof(double) * mm) != hipSuccess)
      return bail("out of device memory for M x M workspace");
  double** vecs[] = {&sv->dq, &sv->u, &sv->ahat};
  for (double** p : vecs)
    if (hipMalloc(p, sizeof(double) * Mp) != hipSuccess || hipMemset(*p, 0, sizeof(double) * Mp) != hipSuccess)
      return bail("out of device memory for M vectors");
  if (hipHostMalloc(&sv->h_R, sizeof(double) * mm, hipHostMallocNonCoherent) != hipSuccess ||
      hipHostMalloc(&sv->h_Rbar, sizeof(double) * mm, hipHostMallocNonCoherent) != hipSuccess)
    return bail("out of pinned host memory");
  std::memset(sv->h_R, 0, sizeof(double) * mm);
  const size_t mn = (size_t)Mp * sv->Ncols;
  if (hipMalloc(&sv->Kmn, sizeof(double) * mn) != hipSuccess ||
      hipMalloc(&sv->Ybuf, sizeof(double) * mn) != hipSuccess ||
      hipMalloc(&sv->Gpart, sizeof(double) * mm * sv->nc) != hipSuccess ||
      hipMalloc(&sv->mu, sizeof(double) * sv->Ncols) != hipSuccess ||
      hipMalloc(&sv->g, sizeof(double) * sv->Ncols) != hipSuccess ||
      hipMalloc(&sv->part, sizeof(double) * sv->part_len) != hipSuccess ||
      hipMalloc(&sv->pres, sizeof(double) * resid_blocks(sv->Ncols) * kResidW) != hipSuccess ||
      hipMalloc(&sv->ptr, sizeof(double) * svgp_final_blocks(M)) != hipSuccess ||
      hipMalloc(&sv->fin, sizeof(double) * (GPX_THETA_STRIDE + (size_t)Mp * D + 1)) != hipSuccess ||
      hipMalloc(&sv->d_theta, sizeof(double) * GPX_THETA_STRIDE) != hipSuccess ||
      hipMalloc(&sv->d_iota, sizeof(int) * sv->nc) != hipSuccess)
    return bail("out of device memory for N-sized workspace");
  // upper tiles of the split-K partials are never written: keep them zero
  if (hipMemset(sv->Gpart, 0, sizeof(double) * mm * sv->nc) != hipSuccess ||
      hipMemset(sv->g, 0, sizeof(double) * sv->Ncols) != hipSuccess)
    return bail("memset failed");
  std::vector<int> iota(sv->nc);
  for (int i = 0; i < sv->nc; ++i) iota[i] = i;
  if (hipMemcpy(sv->d_iota, iota.data(), sizeof(int) * sv->nc, hipMemcpyHostToDevice) != hipSuccess)
    return bail("upload failed");
  sv->h_nloc = (double)N;
  *out = sv;
  return GPX_OK;
}

int gpx_svgp_destroy(gpx_svgp* sv) {
  if (!sv) return GPX_BAD_ARG;
  (void)hipSetDevice(sv->ctx->device);
  if (sv->kmm) gpx_batch_destroy(sv->kmm);
  if (sv->h_R) (void)hipHostFree(sv->h_R);
  if (sv->h_Rbar) (void)hipHostFree(sv->h_Rbar);
  for (void* p : {(void*)sv->dZ, (void*)sv->dYdummy, (void*)sv->d_theta, (void*)sv->dq, (void*)sv->dR,
                  (void*)sv->u, (void*)sv->mu, (void*)sv->g, (void*)sv->Sm1, (void*)sv->T, (void*)sv->P,
                  (void*)sv->Gh, (void*)sv->X1, (void*)sv->GR, (void*)sv->Phi, (void*)sv->Sb,
                  (void*)sv->ahat, (void*)sv->Rbar, (void*)sv->Kmn, (void*)sv->Ybuf, (void*)sv->Gpart,
                  (void*)(sv->own_part ? sv->part : nullptr), (void*)sv->pth, (void*)sv->pz, (void*)sv->pw, (void*)sv->pres,
                  (void*)sv->ptr, (void*)sv->fin, (void*)sv->d_iota, (void*)sv->Kms, (void*)sv->V,
                  (void*)sv->pA, (void*)sv->pB})
    if (p) (void)hipFree(p);
  delete sv;
  return GPX_OK;
}

int gpx_svgp_partials(gpx_svgp* sv, double** dev_ptr, long long* len) {
  if (!sv || !dev_ptr || !len) return GPX_BAD_ARG;
  *dev_ptr = sv->part;
  *len = sv->part_len;
  return GPX_OK;
}

int gpx_svgp_bind_partials(gpx_svgp* sv, double* dev_ptr, long long len) {
  if (!sv || !dev_ptr) return GPX_BAD_ARG;
  if (len < sv->part_len) return fail(sv->ctx, GPX_BAD_ARG, "partial buffer too small");
  if (sv->own_part && sv->part) (void)hipFree(sv->part);
  sv->part = dev_ptr;
  sv->own_part = false;
  sv->local_done = false;
  return GPX_OK;
}

int gpx_svgp_eval_local(gpx_svgp* sv, const double* theta, const double* Z, const double* q_mu,
                        const double* q_sqrt, int32_t* info, void* stream) {
  if (!sv) return GPX_BAD_ARG;
  gpx_ctx* ctx = sv->ctx;
  HIPX(ctx, hipSetDevice(ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  sv->local_done = false;
  int rc = prelude(sv, theta, Z, q_mu, q_sqrt, s);
  if (rc != GPX_OK) return rc;
  const int M = sv->M, Mp = sv->Mp, Nc = sv->Ncols, D = sv->D;
  const double s2 = theta[sv->spec.n_params];
  const double scale = sv->num_data / (double)sv->n_total;
  const double c2 = -scale / s2;  // 2c
  const Run r{sv->kmm, sv->kmm->d_active, 1, s};
  double* W = sv->kmm->W;
  hipStream_t sa = sv->kmm->aux[0];
  hipEvent_t e_up = sv->kmm->ev[kEvents - 2], e_m = sv->kmm->ev[kEvents - 1];
  HIPX(ctx, hipEventRecord(e_up, s));
  // Kmn = k(Z, X) (rows ≥ M and columns ≥ N are zero)
  BuildArgs ba{};
  ba.active = sv->kmm->d_active; ba.specs = sv->kmm->d_specs; ba.theta = sv->d_theta;
  ba.nvalid = sv->kmm->d_n; ba.X = sv->dZ; ba.sX = 0; ba.X2 = sv->X; ba.sX2 = 0; ba.D = D;
  ba.m2 = sv->N; ba.out = sv->Kmn; ba.sOut = 0; ba.ldo = Nc; ba.rows = Mp; ba.cols = Nc;
  ba.symmetric = 0; ba.rows_valid = 0;
  launch_build(ba, 1, s);
  // G = Kmn Kmnᵀ (lower), split-K over nc column chunks, then summed
  {
    const Run rk{sv->kmm, sv->d_iota, sv->nc, s};
    GemmArgs gg = gemm_args(sv->Kmn, Nc, sv->Kmn, Nc, sv->Gpart, Mp, 0, Mp, Mp, sv->chunkK, 0, 1, 1.0, 0.0);
    gg.sA = sv->chunkK; gg.sB = sv->chunkK; gg.sC = (long long)Mp * Mp;
    gemm(rk, gg, EPI_STORE, false, true);
    sum_into(sv->Gpart, (long long)Mp * Mp, sv->nc, (long long)Mp * Mp, sv->part + sv->off_G, 0, s);
  }
  // The M×M chain (latency-bound recursive factorisation, then S − I and P) runs on an
  // auxiliary stream while the main stream builds Kmn and runs the split-K SYRK for G
  // (enqueued first, so the chain's many small launches do not delay the big ones).
  HIPX(ctx, hipStreamWaitEvent(sa, e_up, 0));
  {
    const Run ra{sv->kmm, sv->kmm->d_active, 1, sa};
    factor_u(sv, sa);
    // S − I = q_sqrt q_sqrtᵀ − I;  P = Wᵀ (S − I) W
    gemm(ra, gemm_args(sv->dR, Mp, sv->dR, Mp, sv->Sm1, Mp, 0, Mp, Mp, Mp, TRI_KMAX_I | TRI_KMAX_J, 0,
                       1.0, 0.0), EPI_STORE, false, true);
    launch_diag_add(sv->Sm1, Mp, M, -1.0, sa);
    gemm(ra, gemm_args(sv->Sm1, Mp, W, Mp, sv->T, Mp, 0, Mp, Mp, Mp, TRI_KMIN_J, 0, 1.0, 0.0), EPI_STORE,
         false, false);
    gemm(ra, gemm_args(W, Mp, sv->T, Mp, sv->P, Mp, 0, Mp, Mp, Mp, TRI_KMIN_I, 0, 1.0, 0.0), EPI_STORE,
         true, false);
    HIPX(ctx, hipEventRecord(e_m, sa));
  }
  HIPX(ctx, hipStreamWaitEvent(s, e_m, 0));
  // μ = Kmnᵀ u
  TrmvArgs t{};
  t.active = sv->kmm->d_active; t.Wm = sv->Kmn; t.sW = 0; t.ld = Nc; t.x = sv->u; t.sx = 0;
  t.nvalid = nullptr; t.y = sv->mu; t.sy = 0; t.rows = Mp; t.cols = Nc; t.lower = 0;
  launch_trmv_t(t, 1, s);
  // g_μ, Σ(y−μ)², Σ k_nn, c Σ ∂k_nn/∂θ
  ResidArgs ra{};
  ra.X = sv->X; ra.Y = sv->Y; ra.mu = sv->mu; ra.D = D; ra.n = sv->N; ra.npad = Nc;
  ra.spec = sv->kmm->d_specs; ra.theta = sv->d_theta; ra.scale = scale; ra.g = sv->g; ra.part = sv->pres;
  launch_resid(ra, s);
  const int nrb = resid_blocks(Nc);
  sum_into(sv->pres, kResidW, nrb, GPX_THETA_STRIDE, sv->part + sv->off_th, 0, s);
  sum_into(sv->pres + 16, kResidW, nrb, 2, sv->part + sv->off_sc, 0, s);
  HIPX(ctx, hipMemcpyAsync(sv->part + sv->off_sc + 2, &sv->h_nloc, sizeof(double), hipMemcpyHostToDevice, s));
  // Y = 2c P Kmn
  gemm(r, gemm_args(sv->P, Mp, sv->Kmn, Nc, sv->Ybuf, Nc, 0, Mp, Nc, Mp, 0, 0, c2, 0.0), EPI_STORE,
       false, false);
  // K̄mn = u g_μᵀ + Y contracted with ∂Kmn/∂θ, ∂Kmn/∂Z; w = Kmn g_μ
  RowsArgs ro{};
  ro.Zr = sv->dZ; ro.Xc = sv->X; ro.D = D; ro.nrows = M; ro.ncols = sv->N; ro.Y = sv->Ybuf; ro.ldy = Nc;
  ro.sym = 0; ro.u = sv->u; ro.g = sv->g; ro.zscale = 1.0; ro.spec = sv->kmm->d_specs;
  ro.theta = sv->d_theta; ro.chunk = sv->rows_chunk; ro.Mp = Mp;
  rc = rows_alloc(sv, ro);
  if (rc != GPX_OK) return rc;
  ro.part_theta = sv->pth; ro.part_z = sv->pz; ro.part_w = sv->pw;
  HIPX(ctx, hipMemsetAsync(sv->pz, 0, sizeof(double) * rows_chunks(ro) * Mp * D, s));
  HIPX(ctx, hipMemsetAsync(sv->pw, 0, sizeof(double) * rows_chunks(ro) * Mp, s));
  launch_rows(ro, single_term(sv), s);
  sum_into(sv->pth, GPX_THETA_STRIDE, rows_blocks(ro), GPX_THETA_STRIDE, sv->part + sv->off_th, 1, s);
  sum_into(sv->pz, (long long)Mp * D, rows_chunks(ro), (long long)Mp * D, sv->part + sv->off_z, 0, s);
  sum_into(sv->pw, Mp, rows_chunks(ro), Mp, sv->part + sv->off_w, 0, s);
  HIPX(ctx, hipGetLastError());
  rc = check_info(sv, info, s);
  if (rc != GPX_OK) return rc;
  sv->local_done = true;
  return GPX_OK;
}

int gpx_svgp_eval_finish(gpx_svgp* sv, double* elbo, double* grad_theta, double* grad_Z,
                         double* grad_qmu, double* grad_qsqrt, void* stream) {
  if (!sv) return GPX_BAD_ARG;
  gpx_ctx* ctx = sv->ctx;
  if (!sv->local_done) return fail(ctx, GPX_BAD_ARG, "gpx_svgp_eval_local must succeed first");
  if (!elbo || !grad_theta || !grad_Z || !grad_qmu || !grad_qsqrt) return fail(ctx, GPX_BAD_ARG, "null output");
  HIPX(ctx, hipSetDevice(ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  const int M = sv->M, Mp = sv->Mp, D = sv->D, np = sv->spec.n_params;
  const double s2 = sv->h_theta[np];
  const double scale = sv->num_data / (double)sv->n_total;
  const double c2 = -scale / s2;
  const Run r{sv->kmm, sv->kmm->d_active, 1, s};
  double* W = sv->kmm->W;
  double* G = sv->part + sv->off_G;
  launch_symmetrize_lower(G, Mp, M, s);
  // Ĝ = W G Wᵀ,  â = W w
  gemm(r, gemm_args(W, Mp, G, Mp, sv->T, Mp, 0, Mp, Mp, Mp, TRI_KMAX_I, 0, 1.0, 0.0), EPI_STORE, false, false);
  gemm(r, gemm_args(sv->T, Mp, W, Mp, sv->Gh, Mp, 0, Mp, Mp, Mp, TRI_KMAX_J, 0, 1.0, 0.0), EPI_STORE,
       false, true);
  TrmvArgs t{};
  t.active = sv->kmm->d_active; t.Wm = W; t.sW = 0; t.ld = Mp; t.x = sv->part + sv->off_w; t.sx = 0;
  t.nvalid = nullptr; t.y = sv->ahat; t.sy = 0; t.rows = t.cols = Mp; t.lower = 1;
  launch_trmv_n(t, 1, s);
  // X1 = (S − I) Ĝ,  GR = Ĝ q_sqrt
  gemm(r, gemm_args(sv->Sm1, Mp, sv->Gh, Mp, sv->X1, Mp, 0, Mp, Mp, Mp, 0, 0, 1.0, 0.0), EPI_STORE, false, false);
  gemm(r, gemm_args(sv->Gh, Mp, sv->dR, Mp, sv->GR, Mp, 0, Mp, Mp, Mp, TRI_KMIN_J, 0, 1.0, 0.0), EPI_STORE,
       false, false);
  SvgpFinalArgs fa{};
  fa.X1 = sv->X1; fa.GR = sv->GR; fa.R = sv->dR; fa.Sm1 = sv->Sm1; fa.Gh = sv->Gh; fa.q = sv->dq;
  fa.ahat = sv->ahat; fa.c2 = c2; fa.m = M; fa.ld = Mp; fa.Phi = sv->Phi; fa.Rbar = sv->Rbar; fa.part_tr = sv->ptr;
  launch_svgp_final(fa, s);
  // K̄mm' = Wᵀ Φ W (symmetrised inside the contraction)
  gemm(r, gemm_args(W, Mp, sv->Phi, Mp, sv->T, Mp, 0, Mp, Mp, Mp, TRI_KMIN_I | TRI_KMIN_J, 0, 1.0, 0.0),
       EPI_STORE, true, false);
  gemm(r, gemm_args(sv->T, Mp, W, Mp, sv->Sb, Mp, 0, Mp, Mp, Mp, TRI_KMIN_J, 0, 1.0, 0.0), EPI_STORE,
       false, false);
  RowsArgs ro{};
  ro.Zr = sv->dZ; ro.Xc = sv->dZ; ro.D = D; ro.nrows = M; ro.ncols = M; ro.Y = sv->Sb; ro.ldy = Mp;
  ro.sym = 1; ro.u = nullptr; ro.g = nullptr; ro.zscale = 2.0; ro.spec = sv->kmm->d_specs;
  ro.theta = sv->d_theta; ro.chunk = sv->rows_chunk; ro.Mp = Mp;
  int rc = rows_alloc(sv, ro);
  if (rc != GPX_OK) return rc;
  ro.part_theta = sv->pth; ro.part_z = sv->pz; ro.part_w = nullptr;
  HIPX(ctx, hipMemsetAsync(sv->pz, 0, sizeof(double) * rows_chunks(ro) * Mp * D, s));
  launch_rows(ro, single_term(sv), s);
  sum_into(sv->pth, GPX_THETA_STRIDE, rows_blocks(ro), GPX_THETA_STRIDE, sv->fin, 0, s);
  sum_into(sv->pz, (long long)Mp * D, rows_chunks(ro), (long long)Mp * D, sv->fin + GPX_THETA_STRIDE, 0, s);
  sum_into(sv->ptr, 1, svgp_final_blocks(M), 1, sv->fin + GPX_THETA_STRIDE + (long long)Mp * D, 0, s);
  HIPX(ctx, hipGetLastError());
  // results to the host
  const size_t small = GPX_THETA_STRIDE + (size_t)Mp * D + kScalars;
  sv->h_part_small.resize(small);
  HIPX(ctx, hipMemcpyAsync(sv->h_part_small.data(), sv->part + sv->off_th, sizeof(double) * small,
                           hipMemcpyDeviceToHost, s));
  sv->h_fin.resize(GPX_THETA_STRIDE + (size_t)Mp * D + 1);
  HIPX(ctx, hipMemcpyAsync(sv->h_fin.data(), sv->fin, sizeof(double) * sv->h_fin.size(), hipMemcpyDeviceToHost, s));
  sv->h_ahat.resize(Mp);
  HIPX(ctx, hipMemcpyAsync(sv->h_ahat.data(), sv->ahat, sizeof(double) * Mp, hipMemcpyDeviceToHost, s));
  HIPX(ctx, hipMemcpyAsync(sv->h_Rbar, sv->Rbar, sizeof(double) * Mp * Mp, hipMemcpyDeviceToHost, s));
  HIPX(ctx, hipStreamSynchronize(s));
  const double* pth = sv->h_part_small.data();
  const double* pz = pth + GPX_THETA_STRIDE;
  const double* sc = pz + (size_t)Mp * D;
  const double* fth = sv->h_fin.data();
  const double* fz = fth + GPX_THETA_STRIDE;
  const double trace = fz[(size_t)Mp * D];
  if (std::llround(sc[2]) != sv->n_total)
    return fail(ctx, GPX_BAD_ARG, "partial sums do not cover n_total rows (missing all-reduce?)");
  const double ntot = (double)sv->n_total;
  const double sumv = sc[1] + trace;
  double kl = -M;
  for (int i = 0; i < M; ++i) {
    kl += sv->h_q[i] * sv->h_q[i];
    for (int j = 0; j <= i; ++j) {
      const double v = sv->h_R[(size_t)i * Mp + j];
      kl += v * v;
    }
    kl -= std::log(sv->h_R[(size_t)i * Mp + i] * sv->h_R[(size_t)i * Mp + i]);
  }
  kl *= 0.5;
  *elbo = scale * (-0.5 * ntot * std::log(2.0 * M_PI * s2) - (sc[0] + sumv) / (2.0 * s2)) - kl;
  for (int p = 0; p < GPX_THETA_STRIDE; ++p) grad_theta[p] = (p < np) ? pth[p] + fth[p] : 0.0;
  grad_theta[np] = scale * (-0.5 * ntot / s2 + 0.5 * (sc[0] + sumv) / (s2 * s2));
  for (int m = 0; m < M; ++m)
    for (int d = 0; d < D; ++d) grad_Z[(size_t)m * D + d] = pz[(size_t)m * D + d] + fz[(size_t)m * D + d];
  for (int m = 0; m < M; ++m) grad_qmu[m] = sv->h_ahat[m] - sv->h_q[m];
  for (int i = 0; i < M; ++i) {
    std::memcpy(grad_qsqrt + (size_t)i * M, sv->h_Rbar + (size_t)i * Mp, sizeof(double) * (i + 1));
    std::memset(grad_qsqrt + (size_t)i * M + i + 1, 0, sizeof(double) * (M - i - 1));
  }
  return GPX_OK;
}

int gpx_svgp_elbo_grad(gpx_svgp* sv, const double* theta, const double* Z, const double* q_mu,
                       const double* q_sqrt, double* elbo, double* grad_theta, double* grad_Z,
                       double* grad_qmu, double* grad_qsqrt, int32_t* info, void* stream) {
  if (!sv) return GPX_BAD_ARG;
  if (sv->n_total != sv->N)
    return fail(sv->ctx, GPX_BAD_ARG, "sharded svgp: use eval_local + all-reduce + eval_finish");
  const int rc = gpx_svgp_eval_local(sv, theta, Z, q_mu, q_sqrt, info, stream);
  if (rc != GPX_OK) return rc;
  return gpx_svgp_eval_finish(sv, elbo, grad_theta, grad_Z, grad_qmu, grad_qsqrt, stream);
}

int gpx_svgp_predict(gpx_svgp* sv, const double* theta, const double* Z, const double* q_mu,
                     const double* q_sqrt, const double* Xnew, int Mn, int add_noise, double* mean,
                     double* var, int32_t* info, void* stream) {
  if (!sv) return GPX_BAD_ARG;
  gpx_ctx* ctx = sv->ctx;
  if (!Xnew || Mn < 1 || !mean || !var) return fail(ctx, GPX_BAD_ARG, "bad predict args");
  if (((long long)Mn + 63) / 64 * 64 > kGemmMaxLd)
    return fail(ctx, GPX_BAD_ARG, "too many prediction points for one call (kGemmMaxLd): split Xnew");
  HIPX(ctx, hipSetDevice(ctx->device));
  hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
  sv->local_done = false;
  int rc = prelude(sv, theta, Z, q_mu, q_sqrt, s);
  if (rc != GPX_OK) return rc;
  factor_u(sv, s);
  const int Mp = sv->Mp, D = sv->D;
  const int Mnp = (Mn + 63) / 64 * 64;
  const Run r{sv->kmm, sv->kmm->d_active, 1, s};
  double* W = sv->kmm->W;
  if (!sv->V) HIPX(ctx, hipMalloc(&sv->V, sizeof(double) * Mp * Mp));
  // V = q_sqrtᵀ W  (so that q_sqrtᵀ A = V Kms)
  gemm(r, gemm_args(sv->dR, Mp, W, Mp, sv->V, Mp, 0, Mp, Mp, Mp, TRI_KMIN_I | TRI_KMIN_J, 0, 1.0, 0.0),
       EPI_STORE, true, false);
  rc = ensure(ctx, sv->Kms, sv->kms_cap, (size_t)Mp * Mnp);
  if (rc != GPX_OK) return rc;
  BuildArgs ba{};
  ba.active = sv->kmm->d_active; ba.specs = sv->kmm->d_specs; ba.theta = sv->d_theta;
  ba.nvalid = sv->kmm->d_n; ba.X = sv->dZ; ba.sX = 0; ba.X2 = Xnew; ba.sX2 = 0; ba.D = D;
  ba.m2 = Mn; ba.out = sv->Kms; ba.sOut = 0; ba.ldo = Mnp; ba.rows = Mp; ba.cols = Mnp;
  ba.symmetric = 0; ba.rows_valid = 0;
  launch_build(ba, 1, s);
  TrmvArgs t{};
  t.active = sv->kmm->d_active; t.Wm = sv->Kms; t.sW = 0; t.ld = Mnp; t.x = sv->u; t.sx = 0;
  t.nvalid = nullptr; t.y = mean; t.sy = 0; t.rows = Mp; t.cols = Mn; t.lower = 0;
  launch_trmv_t(t, 1, s);
  // column sums of squares of A = W Kms and B = V Kms
  GemmArgs ga = gemm_args(W, Mp, sv->Kms, Mnp, nullptr, Mnp, 0, Mp, Mnp, Mp, TRI_KMAX_I, 0, 1.0, 0.0);
  ga.small_tiles = sv->kmm->small_tiles;  // the tile size gemm() will launch with
  const int nrt = Mp / gemm_tile(ga, 1);
  rc = ensure(ctx, sv->pA, sv->pa_cap, (size_t)nrt * Mnp);
  if (rc != GPX_OK) return rc;
  rc = ensure(ctx, sv->pB, sv->pb_cap, (size_t)nrt * Mnp);
  if (rc != GPX_OK) return rc;
  ga.partial = sv->pA; ga.sPartial = 0;
  gemm(r, ga, EPI_COLSUMSQ, false, false);
  GemmArgs gb = gemm_args(sv->V, Mp, sv->Kms, Mnp, nullptr, Mnp, 0, Mp, Mnp, Mp, 0, 0, 1.0, 0.0);
  gb.partial = sv->pB; gb.sPartial = 0;
  gemm(r, gb, EPI_COLSUMSQ, false, false);
  SvgpPredVarArgs pv{};
  pv.pA = sv->pA; pv.pB = sv->pB; pv.nrt = nrt; pv.ldp = Mnp; pv.Xnew = Xnew; pv.D = D; pv.M = Mn;
  pv.spec = sv->kmm->d_specs; pv.theta = sv->d_theta; pv.add_noise = add_noise; pv.var = var;
  launch_svgp_predvar(pv, s);
  HIPX(ctx, hipGetLastError());
  return check_info(sv, info, s);
}

}  // extern "C"
