// gpx_host.h — host-side internals shared by the exact-GP (gpx_api.hip) and SVGP
// (gpx_svgp.hip) orchestration: context / batch state, error plumbing and the device
// building blocks (K build + recursive Cholesky-and-inverse, batched MFMA GEMM).
#pragma once
#include <hip/hip_runtime.h>
#include <memory>
#include <string>
#include <vector>
#include "gpx_internal.h"

constexpr int kGroups = 4;  // max concurrent pipelines per evaluation (HIP streams)
constexpr int kAux = 3;     // auxiliary streams for the T = L21·W11 products of depths 0..2
constexpr int kEvents = 64;

// A context only names the device and holds its default stream (used when a call passes a
// NULL stream). Every piece of per-evaluation state (worker / aux streams, fork and join
// events, workspace) lives in the batch, so threads that evaluate different batches of one
// context never share mutable state; error messages are per calling thread (gpx::fail).
struct gpx_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int profiling = 0;
};

struct gpx_batch {
  gpx_ctx* ctx = nullptr;
  int B = 0, Nmax = 0, D = 0, Np = 0;
  const double* X = nullptr;
  const double* Y = nullptr;
  std::vector<int> n;
  std::vector<gpx_kernel_spec> specs;
  int* d_n = nullptr;
  gpx::DevSpec* d_specs = nullptr;
  double* d_theta = nullptr;
  int* d_active = nullptr;
  int* d_orow = nullptr;  // gpx_batch_predict_train_rows: output row of each slot
  int* d_info = nullptr;
  double *K = nullptr, *L = nullptr, *W = nullptr;     // [B][Np][Np] (band storage: see below)
  // band storage (gpx_batch_create_banded): K, L, W keep only the 64-block band of width
  // kBandStoreP; element (i, j) of problem b lives at X_b + i·ldm + j with ldm = 64·(kBandStoreP+2)
  // and X_b = raw + b·smat + band_c0, i.e. row i occupies [i·(ldm+1), (i+1)·(ldm+1)) of the slot
  // for j − i in [−64·(kBandStoreP+1), 63]: 257 doubles per row instead of Np. Problems that
  // need the dense path run on `shadow`, a small dense batch inside this one.
  int compact = 0;
  int ldm = 0;                     // leading dimension of K/L/W (0: Np)
  long long smat = 0;              // per-problem stride of K/L/W in doubles (0: Np²)
  double *Kraw = nullptr, *Lraw = nullptr, *Wraw = nullptr;
  gpx_batch* shadow = nullptr;     // dense fallback slots (band storage only)
  double *shX = nullptr, *shY = nullptr;
  hipStream_t shadow_s = nullptr;  // the fallback evaluation runs here, beside the band sweeps
  hipEvent_t shadow_ev = nullptr;
  double *z = nullptr, *alpha = nullptr, *ldiag = nullptr;  // [B][Np]
  double* partial = nullptr;       // [B][ntiles64][16]
  long long partial_stride = 0;
  double* results = nullptr;       // [B][kResStride]
  // predict workspace
  double* kxs = nullptr; size_t kxs_cap = 0;
  double* pvp = nullptr; size_t pvp_cap = 0;
  double* abuf = nullptr; size_t abuf_cap = 0;   // A = W·Kxs (full_cov, Mp > Np)
  double* covw = nullptr; size_t covw_cap = 0;   // padded [B][Mp][Mp] covariance
  // factor cache: theta row of the last factorisation per problem
  std::vector<double> fac_theta;
  std::vector<char> fac_valid;
  std::vector<char> fac_band;      // the cached factorisation is the block-banded one (gpx_band.hip)
  // block-band eligibility (see band_width): per problem, per kernel term, per block offset d,
  // a lower bound on the distance between any point of block k and any point of block k − d
  // over the term's active dims, [B][GPX_MAX_TERMS][Np/64]; computed when a problem is bound
  std::vector<double> band_rmin;
  std::vector<double> band_rmin16;  // the same per 16-row block, [B][GPX_MAX_TERMS][Np/16] (band16 path)
  // [B][GPX_MAX_TERMS]: the offset from which a term's table holds one repeated value (a lower
  // bound: inputs sorted along the term's single dimension make the table nondecreasing, so it is
  // computed exactly only up to the widest band any path takes and repeated beyond; see
  // band_tables_lohi), or Np/bs when every entry is exact
  std::vector<int> band_tail;
  std::vector<int> band_tail16;
  double* bres = nullptr; size_t bres_cap = 0;  // [B][Np] band-check column sums (per-block path)
  // block-cyclic-reduction workspace (gpx_bcr.hip: calls with few band16 problems), grow-only
  double* bcr_ws = nullptr; size_t bcr_ws_cap = 0;
  double* bcr_ws_slow = nullptr; size_t bcr_ws_slow_cap = 0;  // the deferred parts' wide reductions (slow_s)
  hipEvent_t bcr_ev[2] = {};       // profiling: the last call's reduction chain, start / end
  void* bcr_graphs = nullptr;      // the reduction chains captured as HIP graphs (gpx_bcr.hip), freed with the batch
  int force_dense = 0;         // re-evaluation of problems whose band check failed
  // pinned staging for gpx_batch_rebind_host, one region per slot ([Nmax*D] X, [Nmax] Y, n and
  // the spec): a slot's previous copies have completed before it is rebound (every evaluation
  // synchronises its stream), so no region is reused while a DMA may still read it
  double* h_stage = nullptr;
  size_t stage_stride = 0;      // doubles per slot
  // gpx_batch_rebind_host only stages; the copies of every slot rebound since the last device
  // call go out at the start of the next one (flush_rebinds), ordered before its kernels
  std::vector<char> dirty;
  int n_dirty = 0;
  int* h_nmeta = nullptr;       // pinned copies of n[] and specs[] for those uploads
  gpx::DevSpec* h_specs = nullptr;
  // gpx_batch_rebind_device only records the source pointers; flush_rebinds copies every
  // pending slot (device sources and host-staged ones) with ONE gather kernel that also takes
  // the per-64-block bounding boxes of X for the band tables (one small download per call)
  struct PendingRebind { int b, n; const double* x; const double* y; bool boxed; };
  // the per-64-block boxes of each slot's X as last bound ([B][nbx][D][2], valid where
  // slot_box_ok): a caller that rebinds the same series again hands them back
  // (gpx_batch_rebind_device_boxed) and the gather needs no box download + synchronise
  std::vector<double> slot_box;
  std::vector<char> slot_box_ok;
  // the evaluation submitted by gpx_batch_lml_grad_submit, completed by _complete (gpx_api.hip)
  struct PendingEval;
  std::unique_ptr<PendingEval> pending_eval;
  std::vector<PendingRebind> pend;
  // the streams the pending device sources were rebound on (their producers' order): an event
  // recorded there at the rebind, waited on by flush_rebinds' gather stream
  struct RebindWait { hipStream_t s; hipEvent_t ev; bool armed; };
  // a call that returns without synchronising its stream (predict at the training inputs from
  // cached factors) leaves its upload DMA out of h_io in flight: the next writer of the pinned
  // blocks waits on this event first (wait_io)
  // io_stream is the stream that call ran on: its kernels still read the device side of the
  // block (active list, θ, n, specs) and the slots' factors, so a writer of those on ANOTHER
  // stream waits for io_ev on the device first (fence_io)
  hipEvent_t io_ev = nullptr;
  bool io_pending = false;
  hipStream_t io_stream = nullptr;
  // predict calls upload [active | info | bandp | theta] from their own pinned block, so an
  // asynchronous predict's upload never holds up the next evaluation's (which writes h_io)
  char* h_io_pred = nullptr;
  std::vector<RebindWait> rebind_waits;
  gpx::RebindDesc* h_rdesc = nullptr;   // pinned (coherent), one per slot
  double* d_box = nullptr;               // [B][nb][D][2] per-block lo/hi of X
  double* h_box = nullptr;               // pinned mirror of the rows of one flush
  // per-call I/O in ONE device block mirrored by ONE pinned host block, laid out
  //   [active: B ints][info: B ints][bandp: B ints][theta: B×16][results: B×kResStride]
  // so an evaluation uploads [active, info=0, theta] in one DMA and downloads [info ..
  // results] in one DMA (was 2 pageable copies + a memset up, 2 pageable copies down)
  char* d_io = nullptr;
  char* h_io = nullptr;       // pinned
  // the same layout in COHERENT pinned memory, for small-problem calls (Np = 64) whose one kernel
  // reads its active list / θ and writes info / results here directly: no DMA either way
  char* h_sio = nullptr;
  size_t io_info_off = 0, io_bandp_off = 0, io_theta_off = 0, io_res_off = 0, io_flag_off = 0, io_bytes = 0;
  int direct_tag = 0;  // the last small-problem call's completion tag (h_sio flags, GPX_SMALL_POLL)
  int* d_bandp = nullptr;     // [B] band width (64-blocks) of the banded problems of the call
  int* h_bandp = nullptr;
  double* h_results = nullptr;  // views into h_io
  int* h_info = nullptr;
  gpx_timing timing{};
  double flops_acc = 0.0;
  // deferred completion of the slow width classes (gpx_batch_set_deferred): the band16 classes
  // wider than defer_q 16-blocks and the 64-row sweeps of a call run on slow_s from copies of
  // the call's active list / θ / widths (d_slow_*), and their results come back with a later
  // _complete (or gpx_batch_deferred_wait); the call itself completes with the rest
  int defer_q = -1;
  int band_route = GPX_BAND_ROUTE_SWEEPS;  // gpx_batch_set_band_route
  hipStream_t slow_s = nullptr;
  hipEvent_t slow_in = nullptr;       // the latest slow part's copies are done (the next upload waits)
  hipEvent_t slow_up = nullptr;       // the call's upload (and rebind gather) are in: the slow part may start
  hipEvent_t bulk_ev = nullptr;       // same-stream deferral: the call's own results are downloaded
  bool slow_in_armed = false;
  int* d_slow_act = nullptr;
  double* d_slow_theta = nullptr;
  int* d_slow_bandp = nullptr;
  int* d_slow_info = nullptr;
  double* d_slow_res = nullptr;       // the slow problems' result rows, gathered for one download
  int* d_slow_info_c = nullptr;
  struct SlowRec;
  std::vector<std::unique_ptr<SlowRec>> slow_out;   // in flight, oldest first
  std::vector<std::unique_ptr<SlowRec>> slow_pool;  // delivered, reused (pinned buffers)
  std::vector<char> deferred;         // [B]: the slot's evaluation is in flight in a slow part
  // wave residency trace of the band16 sweeps (gpx_batch_wave_trace; off when null)
  unsigned long long* d_wtrace = nullptr;
  unsigned int* d_wtrace_n = nullptr;
  unsigned int wtrace_cap = 0;
  // per-batch auxiliary streams and events (the recursion's T-product forks), so that
  // independent batches of one context can evaluate concurrently on different streams
  int aux_priority = 0;       // priority the aux streams were created with
  int small_tiles = 0;        // GEMM tiles by workgroup count (set for the SVGP's B=1 Kmm batch)
  hipStream_t aux[kAux] = {};
  hipEvent_t ev[kEvents] = {};
  hipStream_t hp = nullptr;   // highest-priority stream for the contraction (GPX_CONTRACT_PRIORITY)
  // GPX_GROUPS > 1: per-batch pipelines (created on first use)
  hipStream_t workers[kGroups] = {};
  hipEvent_t fork = nullptr, join[kGroups] = {};
  // GPX_SUBMIT_STATS=1: host wall seconds of gpx_batch_lml_grad_submit's phases (rebind flush,
  // routing, upload, launches, download enqueue) and of _complete's wait, printed at destroy
  double sub_s[12] = {};  // (GPX_SUBMIT_STATS: 0-7 the submit phases, 8-10 predict: total, its I/O wait, shadow slots)
  long long sub_calls = 0, box_syncs = 0;
};

namespace gpx {

// The last error message of the calling thread (errno-like): a context may be used by
// several threads at once (one batch each), so the message cannot live in the context.
std::string& last_error_slot();

inline int fail(gpx_ctx* ctx, int code, const std::string& msg) {
  (void)ctx;
  last_error_slot() = msg;
  return code;
}

#define HIPX(ctx, expr)                                                               \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess)                                                             \
      return fail(ctx, GPX_HIP_ERROR, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

inline long long mat_stride(const gpx_batch* bt) { return bt->smat ? bt->smat : (long long)bt->Np * bt->Np; }
inline int mat_ld(const gpx_batch* bt) { return bt->ldm ? bt->ldm : bt->Np; }
constexpr int kBandStoreP = 2;     // band width (64-blocks) held by band storage
constexpr int kBox = 16;           // rows per bounding box of the band tables (16: the band16 path's block)
constexpr int kBand16MaxQ = 8;     // widest band (16-blocks) of the band16 kernels (gpx_band16.hip)
constexpr int kBand16MaxQAny = 5;  // ... for any kernel family; Q = 6..8 only for SE1 problems with K inline
constexpr int kBcrMaxQ = 5;        // widest band (16-blocks) of the block-cyclic-reduction kernels that keep a node in LDS
constexpr int kBcrWideQ = 8;       // the wide classes Q = 6..8: one reduction of block size 16·8 = 128 (gpx_bcr.hip bcrw_*)
constexpr int kBand16MaxD = 8;     // input columns the band16 backward sweep stages per block
constexpr int kBand16MaxNp = 8192;
constexpr int kShadowSlots = 4;    // dense fallback slots of a band-storage batch

// One pipeline instance: a contiguous range of the device active list on one stream.
struct Run {
  gpx_batch* bt;
  const int* d_act;  // device pointer into the uploaded active list
  int na;            // problems in this range
  hipStream_t s;
  bool dag = false;  // run the T products of the top recursion levels on the aux streams
  int* next_event = nullptr;
  // the deferred (slow-class) part of a call reads its own copies of the call's θ rows and band
  // widths and writes its own info block, and keeps all its lanes on its one stream
  const double* theta = nullptr;
  const int* bandp = nullptr;
  int* info = nullptr;
  bool one_stream = false;
  int wide_from = 0;  // > 0: the band16 groups of at least this width run as ONE launch (band16_wide_kernel)
  int bcr_q = 0;      // > 0: the band16 width groups of Q <= kBcrMaxQ run as block cyclic reduction
                      // (gpx_bcr.hip), each at its width; wider groups keep their sweeps
  int ev16_g0 = 0;    // the band16 group the ev16 timing events start at (the first swept group)
  // the reduction chains' grow-only workspace for this range (the call's, or the slow part's),
  // sized by band_fused_eval for the lanes it actually launches
  double** bcr_wsp = nullptr;
  size_t* bcr_capp = nullptr;
};

struct PhaseTimer {
  bool on;
  hipStream_t s;
  std::vector<hipEvent_t> ev;
  PhaseTimer(bool enabled, hipStream_t st) : on(enabled), s(st) {}
  void mark() {
    if (!on) return;
    hipEvent_t e;
    (void)hipEventCreate(&e);
    (void)hipEventRecord(e, s);
    ev.push_back(e);
  }
  double ms(int i, int j) {
    float t = 0.f;
    (void)hipEventElapsedTime(&t, ev[i], ev[j]);
    return t;
  }
  ~PhaseTimer() {
    for (auto e : ev) (void)hipEventDestroy(e);
  }
};

// grow-only device workspace
inline int ensure(gpx_ctx* ctx, double*& p, size_t& cap, size_t need) {
  if (cap >= need) return GPX_OK;
  if (p) (void)hipFree(p);
  p = nullptr; cap = 0;
  HIPX(ctx, hipMalloc(&p, need * sizeof(double)));
  cap = need;
  return GPX_OK;
}

double gemm_issued_flops(const GemmArgs& a, int na);
void gemm(const Run& r, GemmArgs a, int epi, bool ta, bool tb);
GemmArgs gemm_args(const double* A, int lda, const double* B, int ldb, double* C, int ldc,
                   long long stride, int M, int N, int K, int tri, int lower, double alpha,
                   double beta);
void chol_inv(const Run& r, int off, int n, int depth = 0);
void band_tables(gpx_batch* bt, int b, const double* hostX);  // fills band_rmin for problem b
// the same from per-64-block boxes of X ([nb][D][2]: lo, hi over the block's valid rows)
void band_tables_boxes(gpx_batch* bt, int b, const double* box);
int band_width(const gpx_batch* bt, int b, const double* theta_row);  // p in 64-blocks, or -1
int band_width16(const gpx_batch* bt, int b, const double* theta_row);  // the same in 16-row blocks
int band16_limit(const gpx_batch* bt);  // widest band16 class (16-blocks), -1: off
bool band_shape(const gpx_batch* bt);  // the banded path handles this batch's padded size
int band_limit(const gpx_batch* bt);  // largest p the banded path takes (-1: path disabled)
void band_eval(const Run& r, int p, int max_terms);  // build .. reduce for a banded active set
// the routing of one evaluation call (gpx_batch_lml_grad_submit), pure host logic: the device
// active list [dense | per-block band | band16 by width Q | 64-row fused p <= 1 | p = 2], the
// band-storage fallback problems, the class sizes; writes h_bandp of the routed problems
struct Route {
  std::vector<int32_t> order;
  std::vector<int32_t> shadow_ids;
  int n_dense = 0, n_band = 0, n_fused = 0, n16 = 0, n_fused1 = 0, pband = 0;
  int n_g16 = 0, g16_q[kBand16MaxQ] = {}, g16_n[kBand16MaxQ] = {};
  bool b16_p2 = false;
};
// q16wide_cap: the widest SE1 band16 class this call may use (a latency-bound call of few problems
// keeps its p64 = 2 problems on the 64-row sweeps: one wavefront walking N/16 steps is slower there)
void route_call(gpx_batch* bt, int n_active, const int32_t* active, const double* theta, Route& rt,
                int q16wide_cap = kBand16MaxQ);
// the per-call limits of the routing, and one problem's path under them (w: its band width, in
// 16-blocks for kRouteBand16, in 64-blocks otherwise, -1 when not banded)
struct RouteLimits { int plim = -1, q16lim = -1, q16wide = -1; bool fused_on = true; };
int b16_inline_k();                            // GPX_B16_INLINE_K (bit 0 forward, bit 1 backward)
int b16_inline_k_wide();                       // ... for the wide launch (GPX_B16_INLINE_K_WIDE)
int wide_bcr_mode();                            // GPX_WIDE_BCR: 0 never, 1 on the reduction route (default), 2 always
bool wide_bcr_on(bool bcr_route);               // band16 widths Q > kBcrMaxQ by the bs = 128 reduction in this call
long long bcr_ws_need(const int* q, const int* cnt, int g0, int g1, int Nmax);  // workspace of groups g0..g1-1
int wide_qmax(bool se1);                       // widest class of the wide launch (5, or 8: GPX_WIDE_QMAX)
bool se1_spec(const gpx_kernel_spec& sp);     // one SquaredExponential term on one column
enum RouteKind { kRouteDense, kRouteShadow, kRouteBand, kRouteFused, kRouteBand16 };
RouteLimits route_limits(const gpx_batch* bt);
RouteKind route_one(const gpx_batch* bt, int b, const double* theta_row, const RouteLimits& L, int& w);
// p <= 2: [band16 groups (sizes g16_n, widths g16_q; K band of kband16 64-block diagonals) |
// p<=1 (n1) | p=2]
int band_fused_eval(const Run& r, int n16, int n_g16, const int* g16_q, const int* g16_n, bool se1, int kband16,
                     int n1, int max_terms, hipEvent_t* ev = nullptr, hipEvent_t (*ev16)[4] = nullptr);
double band_fused_flops(int Np, int p, bool fwd);  // block-product flops of one problem's sweep
void factor(const Run& r);       // K build + recursive Cholesky-and-inverse (W = L⁻¹)
void alpha_solve(const Run& r);  // z = W y, α = Wᵀ z
int upload_common(gpx_batch* bt, int n_active, const int32_t* active, const double* theta,
                  hipStream_t s, bool predict_block = false);
int flush_rebinds(gpx_batch* bt, hipStream_t s);  // pending rebinds -> device (one gather on s)
int wait_io(gpx_batch* bt);                        // the last asynchronous call's uploads have left h_io
int fence_io(gpx_batch* bt, hipStream_t s);        // s waits (on the device) for that call's kernels
int ensure_rebind_meta(gpx_batch* bt);             // pinned n/spec mirrors + dirty flags

}  // namespace gpx

// A deferred slow part (gpx_batch_set_deferred) between its submit and its delivery
struct gpx_batch::SlowRec {
  std::vector<int32_t> ids;           // its problems, in launch order
  std::vector<double> theta;          // the call's θ rows (B × GPX_THETA_STRIDE)
  hipEvent_t done = nullptr;          // its results are in h_res / h_info
  double* h_res = nullptr;            // pinned [B][kResStride] (the first ids.size() rows used)
  int* h_info = nullptr;              // pinned [B]
  // profiling: its band16 groups and 64-row sweep pair, as PendingEval records them
  int n_g16 = 0, g16_q[gpx::kBand16MaxQ] = {}, g16_n[gpx::kBand16MaxQ] = {};
  bool se1 = false;                   // (its Q = 4, 5 groups ran as one band16_wide_kernel launch)
  hipEvent_t fq16[gpx::kBand16MaxQ][4] = {};
  hipEvent_t fq[4] = {};
  std::vector<int> p64;               // band widths of the timed 64-row launch pair's problems
  void clear_events() {
    for (auto& g : fq16)
      for (auto& x : g)
        if (x) (void)hipEventDestroy(x), x = nullptr;
    for (auto& x : fq)
      if (x) (void)hipEventDestroy(x), x = nullptr;
  }
  ~SlowRec() {
    clear_events();
    if (done) (void)hipEventDestroy(done);
    if (h_res) (void)hipHostFree(h_res);
    if (h_info) (void)hipHostFree(h_info);
  }
};

// State of a submitted evaluation between gpx_batch_lml_grad_submit and _complete: the
// routing, a copy of θ (the factor cache records it), and the timing events
struct gpx_batch::PendingEval {
  hipStream_t s = nullptr;
  int n_active = 0, n_dense = 0, n_band = 0, n_fused = 0, n_fused1 = 0, ng = 0;
  std::vector<int32_t> order;
  std::vector<int32_t> shadow_ids;  // band storage: problems evaluated on the dense shadow
  std::vector<int32_t> deferred_ids;  // problems of the call whose results come later (slow part)
  hipEvent_t bulk_done = nullptr;     // (not owned) the call's results are in h_io; a slow part may follow
  bool shadow_async = false;         // shadow_ids were submitted on bt->shadow_s by _submit
  std::vector<double> theta;
  std::unique_ptr<gpx::PhaseTimer> total, ct, bp;
  std::vector<gpx::PhaseTimer> pts;
  hipEvent_t kev[2] = {nullptr, nullptr};
  hipEvent_t fq[4] = {nullptr, nullptr, nullptr, nullptr};
  // band16 class: problems [n_band16] at the head of the fused range, grouped by band width Q
  // (one launch pair per group, timestamped when profiling)
  int n_band16 = 0;
  int g16_q[gpx::kBand16MaxQ] = {}, g16_n[gpx::kBand16MaxQ] = {}, n_g16 = 0;
  hipEvent_t fq16[gpx::kBand16MaxQ][4] = {};
  int n_bcr = 0;                      // problems of the call on the block-cyclic-reduction path (bcr_ev timed)
  bool direct = false;                // small-problem call with its I/O in h_sio (no DMA): copied to h_io at _complete
  int poll_tag = 0;                   // > 0: its workgroups write this tag to h_sio's flags when done (polled)
  ~PendingEval() {
    for (auto x : kev)
      if (x) (void)hipEventDestroy(x);
    for (auto x : fq)
      if (x) (void)hipEventDestroy(x);
    for (auto& g : fq16)
      for (auto x : g)
        if (x) (void)hipEventDestroy(x);
  }
};

