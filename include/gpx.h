/*
 * gpx.h — C ABI of the MI355X exact-GP regression engine (libgpx.so, gfx950).
 *
 * This is the drop-in boundary for the reference's GP hot path. The reference has no FFI of
 * its own: its seam is the duck-typed GPflow model it calls from Python
 * (SURVEY.md §8b). Each entry point below replaces one piece of GPflow 2.9.1 arithmetic at a
 * reference call site:
 *
 *   gpx_batch_lml_grad  <- model.training_loss + its gradient inside
 *                          gpflow.optimizers.Scipy().minimize(...)   GPR/model_trainer.py:18-19
 *                          (also Multi-Input_GPR/models/model_trainer.py:20-21, 36-37)
 *   gpx_batch_predict   <- model.predict_f(X, full_cov=False)        GPR/model_trainer.py:20,
 *                          GPR/predictor.py:6;  model.predict_y(X)   GPR/predictor.py:7
 *   gpx_batch_predict_full_cov <- model.predict_f(X, full_cov=True)  test_scripts/GPR_Entropy.py:373
 *   gpx_kernel_spec     <- the kernel objects of GPR/main.py:105-114 and the composite
 *                          Exponential*Exponential of Multi-Input_GPR/main.py:118-135
 *
 * Evaluation paths (chosen per problem and per call, results agree to rounding): the dense
 * recursive Cholesky-and-inverse, or — when K and every ∂K/∂θ are exactly zero in fp64 beyond a
 * band of 64-blocks (SE / Matern / Exponential with a lengthscale small against the spacing of
 * sorted inputs, e.g. GPflow's default ℓ = 1 on the reference's integer day offsets) — a
 * block-banded Cholesky, banded solves and selected inversion of K⁻¹ on the band, O(N·bw²).
 * Every banded evaluation checks itself: max_j |Σ_i K_ji Z_ij − 1| over the band (Z the selected
 * inverse) must be <= GPX_BAND_TOL (default 1e-6), else that problem is re-evaluated densely in
 * the same call (selected inversion loses accuracy for very smooth kernels with wide bands).
 * GPX_BAND=0 in the environment forces the dense path.
 *
 * Conventions
 *  - All arithmetic is fp64. X, Y, Xnew and the predict outputs are caller-owned DEVICE
 *    pointers (e.g. torch tensors' data_ptr()); the library never frees them.
 *  - theta / lml / grad / info of gpx_batch_lml_grad are HOST arrays; the call returns when
 *    they are filled (the L-BFGS-B driver on the host needs them immediately).
 *  - theta is in constrained space (θ > 0), row stride GPX_THETA_STRIDE per problem:
 *    theta[b*GPX_THETA_STRIDE + p] for the kernel parameters p < spec.n_params, followed by the
 *    Gaussian noise variance σn² at p = spec.n_params. grad has the same layout and holds
 *    ∂logML/∂θ (the chain rule to the unconstrained variables is the caller's job).
 *  - Per-term parameter order follows GPflow's tf.Module flattening (sorted attribute names):
 *      SE/Matern12/Matern32/Matern52/Exponential : [lengthscales, variance]
 *      RationalQuadratic                         : [alpha, lengthscales, variance]
 *      Periodic(SquaredExponential)              : [base.lengthscales, base.variance, period]
 *      Linear                                    : [variance]
 *  - Return codes: GPX_OK, GPX_NOT_PD (some problem's K+σn²I is not positive definite; its
 *    info[b] holds the 1-based index of the first failing pivot, like LAPACK potrf),
 *    GPX_BAD_ARG, GPX_HIP_ERROR. No C++ exception crosses this boundary.
 *  - A context is bound to one device. Several threads may use one context at the same time
 *    as long as each thread works on its own batch / svgp object (all per-evaluation streams,
 *    events and workspace belong to the batch); a single batch is NOT thread-safe.
 *    gpx_last_error returns the calling thread's most recent failure message (errno-like).
 *    A NULL stream means the context's own stream, which concurrent threads then share
 *    (correct, but their evaluations serialise): pass one stream per thread instead.
 */
#ifndef GPX_H_
#define GPX_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPX_OK 0
#define GPX_NOT_PD 1
#define GPX_BAD_ARG 2
#define GPX_HIP_ERROR 3
/* info[b] of a problem whose evaluation was deferred (gpx_batch_set_deferred): its result comes
 * with a later gpx_batch_lml_grad_complete or gpx_batch_deferred_wait */
#define GPX_INFO_DEFERRED (-1000)

#define GPX_MAX_TERMS 4
#define GPX_THETA_STRIDE 16 /* kernel params + 1 noise slot, per problem */
#define GPX_MAX_DIM 16      /* input dimension D limit */

typedef enum {
  GPX_SE = 1,          /* σ² exp(-r²/2)                         gpflow.kernels.SquaredExponential */
  GPX_MATERN12 = 2,    /* σ² exp(-r)                            gpflow.kernels.Matern12 */
  GPX_MATERN32 = 3,    /* σ² (1+√3r) exp(-√3r)                  gpflow.kernels.Matern32 */
  GPX_MATERN52 = 4,    /* σ² (1+√5r+5r²/3) exp(-√5r)            gpflow.kernels.Matern52 */
  GPX_EXPONENTIAL = 5, /* σ² exp(-r/2)                          gpflow.kernels.Exponential */
  GPX_RQ = 6,          /* σ² (1+r²/(2α))^(-α)                   gpflow.kernels.RationalQuadratic */
  GPX_PERIODIC_SE = 7, /* σ² exp(-½Σ(sin(πΔ/p)/ℓ)²)             gpflow.kernels.Periodic(SE) */
  GPX_LINEAR = 8       /* σ² x·x'                               gpflow.kernels.Linear */
} gpx_term_kind;

typedef enum { GPX_SUM = 0, GPX_PRODUCT = 1 } gpx_combine;

typedef struct {
  int32_t kind;         /* gpx_term_kind */
  int32_t dim_start;    /* active_dims = slice(dim_start, dim_start + dim_count) */
  int32_t dim_count;
  int32_t param_offset; /* index of this term's first parameter in the theta row */
} gpx_term;

typedef struct {
  int32_t n_terms;      /* 1..GPX_MAX_TERMS */
  int32_t combine;      /* gpx_combine (ignored when n_terms == 1) */
  int32_t n_params;     /* kernel parameters; the noise variance sits at theta[n_params] */
  int32_t reserved;
  gpx_term terms[GPX_MAX_TERMS];
} gpx_kernel_spec;

typedef struct gpx_ctx gpx_ctx;
typedef struct gpx_batch gpx_batch;

const char* gpx_version(void);

/* One context per device. */
int gpx_create(int device, gpx_ctx** out);
int gpx_destroy(gpx_ctx* ctx);
const char* gpx_last_error(const gpx_ctx* ctx);

/*
 * A batch of B independent GPR problems (the per-asset / per-kernel fits of
 * GPR/main.py:23-37 x GPR/model_trainer.py:14). Problem b has n[b] <= N_max points.
 *   X : device fp64 [B, N_max, D] row-major;  Y : device fp64 [B, N_max].
 *   n : host int32 [B];  specs : host [B].
 * The batch keeps pointers to X and Y (they must outlive it) and owns its HBM workspace
 * (about 4 * B * Np^2 * 8 bytes, Np = N_max rounded up to 64).
 */
int gpx_batch_create(gpx_ctx* ctx, int B, int N_max, int D, const double* X, const double* Y,
                     const int32_t* n, const gpx_kernel_spec* specs, gpx_batch** out);
/*
 * gpx_batch_create with BAND STORAGE, for many resident slots of banded problems (the
 * continuous-batching fits of configuration C2: SE / Matern / Exponential kernels on sorted
 * day offsets, GPR/data_handler.py:42-44 + GPR/model_trainer.py:15, whose K is exactly zero in
 * fp64 beyond one or two 64-blocks off the diagonal). The workspace keeps only the band of two
 * 64-blocks: 3 * Np * 257 * 8 bytes per slot (25 MiB at N = 4096 instead of 384 MiB), so ~10x
 * more slots fit in HBM. Same calls and results as a gpx_batch_create batch; evaluations the
 * fused banded sweeps cannot take (a wider band, another kernel family, a failed band check)
 * and predictions that need a fresh factor run densely on 4 internal fallback slots in the
 * same call. 449 <= N_max <= 8192.
 */
int gpx_batch_create_banded(gpx_ctx* ctx, int B, int N_max, int D, const double* X, const double* Y,
                            const int32_t* n, const gpx_kernel_spec* specs, gpx_batch** out);
int gpx_batch_destroy(gpx_batch* batch);

/*
 * Rebind slot b to a new problem: the caller has already written its inputs into row b of
 * the X / Y arrays given at creation (n <= N_max valid points); this updates n[b] and the
 * kernel spec and invalidates the slot's cached factor. Used to stream many fits through a
 * fixed set of device slots (continuous batching).
 */
int gpx_batch_rebind(gpx_batch* batch, int b, int n, const gpx_kernel_spec* spec);

/*
 * gpx_batch_rebind with the problem's inputs given on the HOST (X [n, D], Y [n], fp64): they are
 * copied into the slot's pinned staging region at once (the host buffers may be reused on
 * return) and reach slot b of the batch's X / Y arrays by DMA at the start of the next device
 * call on the batch, on that call's stream. Rows n .. N_max-1 of the slot are zeroed.
 * `stream` is unused (kept for the ABI).
 */
int gpx_batch_rebind_host(gpx_batch* batch, int b, int n, const double* X, const double* Y,
                          const gpx_kernel_spec* spec, void* stream);
/* The same with the inputs in DEVICE memory (X [n, D], Y [n], e.g. a model's resident tensors):
 * only recorded; the next device call on the batch gathers every pending slot in one kernel on
 * its stream (which also returns the per-16-row-block boxes of X for the band tables), so X and Y
 * must stay valid and unchanged until that call has been issued and completed. `stream` (may be
 * NULL) is the stream in whose order X and Y are ready (their producer's): an event recorded on
 * it here is waited on by the gather when that runs on another stream. */
int gpx_batch_rebind_device(gpx_batch* batch, int b, int n, const double* X, const double* Y,
                            const gpx_kernel_spec* spec, void* stream);
/* gpx_batch_rebind_device with the per-16-row-block bounding boxes of X supplied by the caller
 * (host array, for each of the ceil(n/16) blocks and each of the D columns the pair (min, max)
 * of that column over the block's rows: [ceil(n/16)][D][2]), as gpx_batch_slot_boxes returned
 * them for the same X earlier: the band tables are computed here and the next call's gather
 * needs no box download (and no stream synchronise) for this slot. */
int gpx_batch_rebind_device_boxed(gpx_batch* batch, int b, int n, const double* X, const double* Y,
                                  const gpx_kernel_spec* spec, const double* boxes, void* stream);
/* The boxes of slot b's X (layout as above) as computed when its inputs were last gathered;
 * GPX_BAD_ARG if unknown (not gathered yet, host-staged, or no band tables for this batch's
 * shape). For a caller that caches them per series. */
int gpx_batch_slot_boxes(const gpx_batch* batch, int b, double* boxes);

/*
 * logML and ∂logML/∂θ at theta for the n_active problems listed in active (host int32).
 * Outputs are written at each active problem's row: lml[b], grad[b*GPX_THETA_STRIDE + p],
 * info[b]. stream may be NULL (library stream). Returns after the outputs are on the host.
 */
int gpx_batch_lml_grad(gpx_batch* batch, int n_active, const int32_t* active, const double* theta,
                       double* lml, double* grad, int32_t* info, void* stream);

/*
 * gpx_batch_lml_grad in two halves, so one host thread can keep several batches in flight:
 * _submit validates, routes and enqueues the whole evaluation (uploads, kernels and the
 * download of the results into pinned memory) on `stream` and returns without waiting;
 * _complete waits for it, writes lml / grad / info exactly as gpx_batch_lml_grad does (and
 * re-evaluates densely, synchronously, any banded problem whose check failed). One submitted
 * evaluation per batch at a time; the batch must not be used in between (other batches may).
 * theta is copied by _submit. gpx_batch_lml_grad = _submit + _complete.
 */
int gpx_batch_lml_grad_submit(gpx_batch* batch, int n_active, const int32_t* active, const double* theta,
                              void* stream);
int gpx_batch_lml_grad_complete(gpx_batch* batch, double* lml, double* grad, int32_t* info);
/* 1 when the submitted evaluation (if any) has finished on the device (complete will not
 * wait), 0 while it runs; < 0 on error. */
int gpx_batch_lml_grad_query(gpx_batch* batch);
/*
 * Host-side routing query: for rows[i] at theta (the gpx_batch_lml_grad layout), the band
 * width in 64-blocks the evaluation would take (>= 0: the block-banded path), -1 for the
 * dense path, -2 when the row's band tables are not known yet (a device rebind still waiting
 * for the next call's gather). No device work.
 */
int gpx_batch_band_width(gpx_batch* batch, int n_rows, const int32_t* rows, const double* theta, int32_t* p_out);
/* The path an evaluation of each row at theta would take, host-side (no device work), as
 * gpx_batch_lml_grad_submit routes it: 1..15 = the band16 sweeps with a band of that many 16-row
 * blocks; 16 + p = the 64-row banded path with p 64-blocks in a batch without band16 tables;
 * 32 + p = the 64-row banded path although the batch has band16 tables (the band is wider than
 * the band16 sweeps take); -1 = dense (or, band storage, the fallback slots); -2 = not known yet
 * (a rebind whose gather runs with the next call). Callers that keep several batches use it to
 * evaluate the slow classes apart from the fast ones (Scipy.minimize_stream wide_group). */
int gpx_batch_band_class(gpx_batch* batch, int n_rows, const int32_t* rows, const double* theta, int32_t* cls_out);
/* Deferred completion of the slow evaluation classes. With q >= 0, the problems of a call whose
 * evaluation takes the band16 sweeps wider than q 16-row blocks, or the 64-row banded sweeps,
 * run on a stream of their own and gpx_batch_lml_grad_complete returns without waiting for them:
 * it reports info[b] = GPX_INFO_DEFERRED for those rows, and delivers (lml, grad, info) of
 * deferred rows of earlier calls whose work has finished by then (rows of neither kind are not
 * written). A deferred row may not be evaluated, predicted or rebound until it is delivered;
 * gpx_batch_deferred_wait blocks until every deferred row is delivered (into its arrays; it is
 * refused, GPX_BAD_ARG, while an evaluation is submitted on the batch and not completed). The
 * call's other problems never wait for the slow classes, whose sweeps (one wavefront per SIMD,
 * or 73 KiB of LDS per workgroup) start late under a full band16 load. Same results, bit for
 * bit, as without deferral. q < 0 turns it off (the default). */
/* Which banded route the batch's band16 problems take (GPX_BAND_ROUTE_*), a property of the batch,
 * never of a call: a problem's arithmetic then depends on its own data, θ and this setting only —
 * not on how many problems share its call — so a fit reproduces bit for bit whichever fits run
 * beside it (the solo GPR of GPR/model_trainer.py:15-19 and the same series inside a batch of
 * thousands give the same trajectory).
 *   SWEEPS (0, the default): the one-wavefront band16 sweeps (throughput: thousands of problems
 *     in flight fill the chip);
 *   BCR (1): block cyclic reduction for the widths it covers (Q <= 5; log-depth latency for calls
 *     of a few problems, ~4x the sweeps' work), wider problems on the 64-row sweeps;
 *   AUTO (2): BCR for calls of at most GPX_BCR_MAX (default 32) band16 problems, else the sweeps —
 *     the round-5 rule, whose results depend on the call's size (the two routes agree to ~1e-9
 *     relative, not bit for bit).
 * The environment variable GPX_BCR_MAX, when set, overrides the setting for every batch of the
 * process (0: sweeps, a large value: BCR; the A/B knob of the tests and tools). */
#define GPX_BAND_ROUTE_SWEEPS 0
#define GPX_BAND_ROUTE_BCR 1
#define GPX_BAND_ROUTE_AUTO 2
int gpx_batch_set_band_route(gpx_batch* batch, int route);
int gpx_batch_set_deferred(gpx_batch* batch, int q);
int gpx_batch_deferred_wait(gpx_batch* batch, double* lml, double* grad, int32_t* info);
/* rows with a deferred evaluation in flight: writes up to cap slot indices, returns the count */
int gpx_batch_deferred_rows(const gpx_batch* batch, int32_t* rows, int cap);

/*
 * Posterior marginals at Xnew for the active problems: GPflow GPR.predict_f(full_cov=False)
 * (add_noise = 0) or predict_y (add_noise = 1: variance + σn²).
 *   Xnew : device fp64 [B, M, D];  mean, var : device fp64 [B, M] (caller-owned).
 * theta/info are host arrays as above. Re-factorises K+σn²I at theta like GPflow (no caching
 * across calls unless theta is bit-identical to the last factorisation of that problem).
 */
int gpx_batch_predict(gpx_batch* batch, int n_active, const int32_t* active, const double* theta,
                      const double* Xnew, int M, int add_noise, double* mean, double* var,
                      int32_t* info, void* stream);

/*
 * gpx_batch_predict at each problem's own training inputs (GPR/model_trainer.py:20,
 * predict_f(X_train)) in O(N²) from the factor: with Kxs = K_y − σn²I, GPflow's
 * Kxsᵀα = y − σn²α and k_jj − colsum((L⁻¹Kxs)²)_j = σn² − σn⁴ [K_y⁻¹]_jj exactly.
 *   mean, var : device fp64 [B, N_max] (rows < n[b] written).
 */
int gpx_batch_predict_train(gpx_batch* batch, int n_active, const int32_t* active,
                            const double* theta, int add_noise, double* mean, double* var,
                            int32_t* info, void* stream);

/*
 * gpx_batch_predict_train with the outputs packed by position: mean, var : device fp64
 * [n_active, N_max], row i for problem active[i] (rows < n[active[i]] written). A caller that
 * keeps each fit's prediction (the stepped drivers: a few dozen finished fits per round of a
 * 1024-slot batch) allocates only those rows. Same values as gpx_batch_predict_train.
 */
int gpx_batch_predict_train_rows(gpx_batch* batch, int n_active, const int32_t* active,
                                 const double* theta, int add_noise, double* mean, double* var,
                                 int32_t* info, void* stream);

/*
 * Posterior mean and FULL covariance at Xnew: GPflow GPR.predict_f(Xnew, full_cov=True)
 * (GPflow returns the covariance as [1, M, M]; predict_y has no full_cov form in GPflow).
 *   Xnew : device fp64 [B, M, D];  mean : device fp64 [B, M];  cov : device fp64 [B, M, M].
 * cov[b] = k(X*,X*) − Kxsᵀ (K+σn²I)⁻¹ Kxs, formed as k(X*,X*) − AᵀA with A = L⁻¹·Kxs (MFMA).
 */
int gpx_batch_predict_full_cov(gpx_batch* batch, int n_active, const int32_t* active,
                               const double* theta, const double* Xnew, int M, double* mean,
                               double* cov, int32_t* info, void* stream);

/* Timing hooks for bench.py: total device time (ms) of the last call's kernels, measured with
 * HIP events on the stream they ran on, split by phase. */
typedef struct {
  double factor_ms;   /* K build + recursive Cholesky-and-inverse */
  double alpha_ms;    /* the two triangular matrix-vector products */
  double grad_ms;     /* fused K^-1 = W^T W formation + gradient contraction + reduce */
  double predict_ms;  /* predict-only kernels */
  double total_ms;
  double gemm_flops;  /* MFMA flops issued by the GEMM kernels of the last call */
  /* cumulative since the last gpx_batch_reset_timing, profiling enabled only: the fused
   * K^-1 = W^T W + gradient-contraction kernel (one launch per gpx_batch_lml_grad call) */
  double contract_ms_total;
  double contract_launches;
  double contract_alg_flops;  /* algorithmic flops of those launches: n_active * sum_i 2(i+1)(Np-i) */
  double eval_ms_total;       /* whole gpx_batch_lml_grad device time */
  double evals;               /* problem-evaluations (sum of n_active) */
  /* block-banded path (cumulative, profiling enabled only): device time of its part of the
   * calls, calls that had banded problems, banded problem-evaluations, Σ band width p (64-blocks)
   * over those evaluations */
  double band_ms_total;
  double band_calls;
  double band_evals;
  double band_p_sum;
  /* fused banded kernels (p <= 2), each launch timestamped at its actual start and end:
   * summed durations, launches, and block-product flops issued (2·64³ per 64³ product, the
   * leaf counted as 2/3 of one) */
  double band_fwd_ms_total;
  double band_bwd_ms_total;
  double band_fused_launches;
  double band_fwd_flops;
  double band_bwd_flops;
  double band_fallbacks;      /* banded evaluations whose check failed, redone densely */
  double shadow_evals;        /* band storage: evaluations run on the dense fallback slots */
  double shadow_predicts;     /* band storage: predictions run on the dense fallback slots */
  /* 16-row-block banded sweeps (one wavefront per problem, band of Q <= 4 16-blocks): summed
   * launch durations, launch pairs, problem-evaluations, Σ Q, and the MFMA flops they issue
   * (2·16³ per tile product) */
  double band16_fwd_ms_total;
  double band16_bwd_ms_total;
  double band16_launches;
  double band16_evals;
  double band16_q_sum;
  double band16_fwd_flops;
  double band16_bwd_flops;
  /* Σ over band16 launches of (problems in the launch) × (its duration, ms): the wave-ms the
   * sweeps held (one wavefront per problem); ÷ (wave slots × wall ms) = their occupancy */
  double band16_wave_ms;
  /* the deferred part's wide launches (band16_wide_kernel: the Q = 4 and 5 classes of a call, both
   * sweeps per wavefront): their durations, count, MFMA flops and problems — kept out of the
   * band16 forward/backward launch figures above (which count the per-class launches only) */
  double band16_wide_ms_total, band16_wide_launches, band16_wide_flops, band16_wide_evals;
  /* block cyclic reduction (calls with at most GPX_BCR_MAX band16 problems): the device time of
   * the reduction chains (forward and backward levels, contraction), chains, problem-evaluations */
  double bcr_ms_total, bcr_calls, bcr_evals;
  /* of band_fused_launches: the timed 64-row launch pairs that were the p = 2 class's
   * (band_fwd_kernel / band_bwd_kernel) rather than the p <= 1 class's (band_fwd1_kernel / band_bwd1_kernel) */
  double band_fused_p2_launches;
  /* band16 problem-evaluations of widths Q = 6..8 taken by the block-cyclic-reduction chain of block
   * size 128 (whatever the batch's route; they no longer run as one-wavefront sweeps) */
  double bcr_wide_evals;
} gpx_timing;
int gpx_batch_last_timing(const gpx_batch* batch, gpx_timing* out);
int gpx_batch_reset_timing(gpx_batch* batch);
/* Diagnostic: per-wavefront residency records of the band16 sweeps (one wavefront walks one
 * problem), for occupancy timelines across processes sharing a GPU. cap > 0 allocates room for
 * cap records and turns recording on; 0 frees it and turns it off (both synchronise the device).
 * Each record is three uint64: start and end in the device's constant 100 MHz clock
 * (s_memrealtime, one clock for every process on the GPU) and kind = Q (forward sweep) or
 * 16 + Q (backward sweep). _read synchronises the device, copies up to cap records into out,
 * sets *n_out and restarts the recording. */
int gpx_batch_wave_trace(gpx_batch* batch, unsigned int cap);
int gpx_batch_wave_trace_read(gpx_batch* batch, unsigned long long* out, unsigned int cap, unsigned int* n_out);
int gpx_set_profiling(gpx_ctx* ctx, int enabled);

/* ---------------------------------------------------------------------------------------
 * SVGP: gpflow.models.SVGP(kernel, Gaussian(σn²), inducing_variable=Z, num_data=...) with
 * GPflow's defaults (whiten=True, full lower-triangular q_sqrt, zero mean, one latent GP) —
 * test_scripts/SVGP.py:461-478 (M=120), :515-540 (M=20), test_scripts/GPR.py:118-138.
 *   gpx_svgp_elbo_grad  <- training_loss_closure((X, Y)) value + gradient, fed to
 *                          gpflow.optimizers.Scipy().minimize (test_scripts/SVGP.py:471-474)
 *   gpx_svgp_predict    <- model.predict_f(X_test) / predict_y          (SVGP.py:478)
 *
 * One gpx_svgp holds one shard of the data: X [N, D] and Y [N] (device, fp64, caller-owned).
 * n_total = rows over all shards (= N on one GPU); the ELBO's data term is scaled by
 * num_data / n_total like GPflow's minibatch scaling. Per evaluation:
 *   theta  host [16]: kernel params (gpx_kernel_spec layout) then σn² at theta[n_params]
 *   Z      host [M, D]   inducing inputs;   q_mu host [M];   q_sqrt host [M, M] row-major,
 *          lower triangle used (the FillTriangular-constrained value)
 * Outputs (host): elbo; grad_theta [16] (∂ELBO/∂θ constrained, σn² at n_params);
 *   grad_Z [M, D]; grad_qmu [M]; grad_qsqrt [M, M] (lower triangle, upper zero).
 * Sharded use: gpx_svgp_eval_local on every shard, sum the gpx_svgp_partials() device
 * buffers over shards (one all-reduce), then gpx_svgp_eval_finish. gpx_svgp_elbo_grad is
 * local + finish for the unsharded case (n_total == N).
 */
typedef struct gpx_svgp gpx_svgp;
int gpx_svgp_create(gpx_ctx* ctx, int N, int M, int D, const double* X, const double* Y,
                    const gpx_kernel_spec* spec, double num_data, long long n_total,
                    gpx_svgp** out);
int gpx_svgp_destroy(gpx_svgp* svgp);
/* the partial-sum buffer (device, fp64, len doubles) and a way to substitute a caller-owned
 * one (e.g. a torch tensor that torch.distributed all-reduces in place) */
int gpx_svgp_partials(gpx_svgp* svgp, double** dev_ptr, long long* len);
int gpx_svgp_bind_partials(gpx_svgp* svgp, double* dev_ptr, long long len);
int gpx_svgp_eval_local(gpx_svgp* svgp, const double* theta, const double* Z, const double* q_mu,
                        const double* q_sqrt, int32_t* info, void* stream);
int gpx_svgp_eval_finish(gpx_svgp* svgp, double* elbo, double* grad_theta, double* grad_Z,
                         double* grad_qmu, double* grad_qsqrt, void* stream);
int gpx_svgp_elbo_grad(gpx_svgp* svgp, const double* theta, const double* Z, const double* q_mu,
                       const double* q_sqrt, double* elbo, double* grad_theta, double* grad_Z,
                       double* grad_qmu, double* grad_qsqrt, int32_t* info, void* stream);
/* predict_f (add_noise = 0) / predict_y (1) at Xnew (device [Mn, D]) -> mean, var (device [Mn]) */
int gpx_svgp_predict(gpx_svgp* svgp, const double* theta, const double* Z, const double* q_mu,
                     const double* q_sqrt, const double* Xnew, int Mn, int add_noise, double* mean,
                     double* var, int32_t* info, void* stream);

/* ---------------------------------------------------------------------------------------
 * Host helpers of the batched L-BFGS-B driver (no device work): for the n_fits fits of one
 * round, u [n_fits, n_vars] are the unconstrained variables (gpflow.optimizers.Scipy's x,
 * GPR/model_trainer.py:18-19), rows [n_fits] their batch slots, cols [n_vars] the θ index of each
 * variable, lower [n_vars] its Shift (1e-6 for the Gaussian likelihood variance, else 0).
 *   gpx_host_theta_rows   theta[rows[k]][cols[v]] = lower[v] + softplus(u[k][v])
 *   gpx_host_loss_grad_u  loss[k] = −lml[rows[k]];
 *                         grad_u[k][v] = −grad[rows[k]][cols[v]] · sigmoid(u[k][v])
 * theta / grad rows have GPX_THETA_STRIDE entries (gpx_batch_lml_grad's layout).
 */
int gpx_host_theta_rows(int n_fits, int n_vars, const double* u, const int32_t* rows,
                        const int32_t* cols, const double* lower, double* theta);
int gpx_host_loss_grad_u(int n_fits, int n_vars, const double* u, const int32_t* rows,
                         const int32_t* cols, const double* lml, const double* grad, double* loss,
                         double* grad_u);

#ifdef __cplusplus
}
#endif
#endif /* GPX_H_ */
