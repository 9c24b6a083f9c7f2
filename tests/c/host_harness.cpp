// Host-logic harness for the C ABI's pure host parts (SURVEY §5 sanitizers),
// built with AddressSanitizer + UndefinedBehaviorSanitizer on the HOST code only (hipcc
// --offload-host-only: no device code object at all, so nothing here can run on a GPU) and run
// by tests/test_host_harness.py on the CPU.
//
// What it checks, on seeded random batches:
//   * band_tables / band_tables_boxes (the per-block lower bounds on point distances the
//     banded routing rests on) — the two agree bit for bit;
//   * band_width / band_width16 are SAFE: every kernel entry beyond the reported band is an
//     exact fp64 zero by the device's own formula (GPflow's r², the term's exp argument), and
//     tight for sorted 1-D inputs (at most one block wider than the true band);
//   * route_call (gpx_batch_lml_grad_submit's routing) puts every active problem exactly once
//     in [dense | per-block band | band16 by width | fused p <= 1 | fused p = 2] or on the
//     band-storage fallback, with class sizes, widths and h_bandp consistent, under the
//     GPX_BAND / GPX_BAND16 / GPX_BAND_FUSED switches.
// Exit status 0 and a final "OK" line when every check holds.
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <random>
#include <vector>

#include "../../portfoliooptgp_amd/csrc/gpx_host.h"

using namespace gpx;

static int g_fail = 0;
#define CHECK(cond, ...)                        \
  do {                                          \
    if (!(cond)) {                              \
      if (g_fail < 20) {                        \
        std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
        std::fprintf(stderr, __VA_ARGS__);      \
        std::fprintf(stderr, "\n");             \
      }                                         \
      ++g_fail;                                 \
    }                                           \
  } while (0)

static double exp_arg(int kind, double s) {  // the term's exp argument a(s), s = r/ℓ
  switch (kind) {
    case GPX_SE: return 0.5 * s * s;
    case GPX_MATERN12: return s;
    case GPX_EXPONENTIAL: return 0.5 * s;
    case GPX_MATERN32: return std::sqrt(3.0) * s;
    default: return std::sqrt(5.0) * s;
  }
}

// is K_ij (and every ∂K/∂θ) nonzero by the device's formula: r² as GPflow's square_distance
// forms it on x/ℓ, r = sqrt(max(r², 1e-36)); a sum is nonzero when any term is, a product
// when all are
static bool entry_nz(const gpx_kernel_spec& sp, const double* th, const double* xi, const double* xj) {
  const bool prod = sp.n_terms > 1 && sp.combine == GPX_PRODUCT;
  bool nz = prod;
  for (int t = 0; t < sp.n_terms; ++t) {
    const gpx_term& tm = sp.terms[t];
    const double ell = th[tm.param_offset];
    double dot = 0.0, sa = 0.0, sb = 0.0;
    for (int d = tm.dim_start; d < tm.dim_start + tm.dim_count; ++d) {
      const double a = xi[d] / ell, b = xj[d] / ell;
      dot += a * b;
      sa += a * a;
      sb += b * b;
    }
    double r2 = -2.0 * dot + (sa + sb);
    r2 = r2 > 1e-36 ? r2 : 1e-36;
    const bool tnz = std::exp(-exp_arg(tm.kind, std::sqrt(r2))) != 0.0;
    nz = prod ? (nz && tnz) : (nz || tnz);
  }
  return nz;
}

struct Problem {
  gpx_kernel_spec sp{};
  std::vector<double> x;  // [n][D]
  int n = 0;
  bool sorted1d = false;
};

static gpx_kernel_spec make_spec(std::mt19937_64& rng, int D) {
  gpx_kernel_spec sp{};
  std::uniform_int_distribution<int> nt(1, 3), kind(GPX_SE, GPX_PERIODIC_SE), comb(0, 1);
  sp.n_terms = nt(rng);
  sp.combine = comb(rng);
  int off = 0;
  for (int t = 0; t < sp.n_terms; ++t) {
    int k = kind(rng);
    if (k == GPX_RQ && (rng() & 1)) k = GPX_SE;
    std::uniform_int_distribution<int> ds(0, D - 1);
    const int d0 = ds(rng);
    std::uniform_int_distribution<int> dc(1, D - d0);
    sp.terms[t] = gpx_term{k, d0, dc(rng), off};
    off += (k == GPX_RQ || k == GPX_PERIODIC_SE) ? 3 : 2;
  }
  sp.n_params = off;
  return sp;
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 40;
  std::mt19937_64 rng(20261017);
  long long checked_pairs = 0, routed = 0, band16_routed = 0, tight_checked = 0;
  for (int round = 0; round < rounds; ++round) {
    const int D = 1 + (int)(rng() % 3);
    const int Nmax = (round % 4 == 0) ? 4096 : 512 + 64 * (int)(rng() % 24);
    const int B = 6;
    gpx_batch bt;
    bt.B = B;
    bt.Nmax = Nmax;
    bt.D = D;
    bt.Np = (Nmax + 63) / 64 * 64;
    bt.compact = (round % 3 == 1);
    bt.n.assign(B, 0);
    bt.specs.assign(B, gpx_kernel_spec{});
    bt.band_rmin.assign((size_t)B * GPX_MAX_TERMS * (bt.Np / kLeaf), INFINITY);
    bt.band_tail.assign((size_t)B * GPX_MAX_TERMS, bt.Np / kLeaf);
    bt.band_rmin16.assign((size_t)B * GPX_MAX_TERMS * (bt.Np / kBox), INFINITY);
    bt.band_tail16.assign((size_t)B * GPX_MAX_TERMS, bt.Np / kBox);
    std::vector<int> bandp(B, -7);
    bt.h_bandp = bandp.data();
    std::vector<Problem> pr(B);
    std::vector<double> theta((size_t)B * GPX_THETA_STRIDE, 1.0);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    for (int b = 0; b < B; ++b) {
      Problem& p = pr[b];
      p.n = (b == 0) ? Nmax : std::max(1, (int)(Nmax * (0.3 + 0.7 * U(rng))));
      // inputs: unit-spaced day offsets (the reference's), jittered sorted, scaled, or random
      // (problems 0, 1: the reference's kernel on day offsets, C2's regime)
      const int mode = b < 2 ? (int)(rng() % 2) : (int)(rng() % 4);
      if (mode == 3) p.n = std::min(p.n, 1024);  // (unsorted inputs: every pair is brute-forced)
      p.sorted1d = D == 1 && mode <= 2;
      p.x.assign((size_t)p.n * D, 0.0);
      const double scale = mode == 2 ? 0.05 + 3.0 * U(rng) : 1.0;
      for (int i = 0; i < p.n; ++i)
        for (int d = 0; d < D; ++d) {
          double v;
          if (mode == 0) v = (double)i;
          else if (mode == 1) v = i + 0.4 * U(rng);
          else if (mode == 2) v = i * scale;
          else v = 4096.0 * U(rng);
          p.x[(size_t)i * D + d] = (D > 1 && d > 0 && mode != 3) ? v + d : v;
        }
      p.sp = (b < 2) ? gpx_kernel_spec{1, 0, 2, 0, {gpx_term{GPX_SE, 0, 1, 0}}} : make_spec(rng, D);
      bt.n[b] = p.n;
      bt.specs[b] = p.sp;
      // θ: lengthscales from 0.3 to 60 (bands from one block to dense)
      double* th = theta.data() + (size_t)b * GPX_THETA_STRIDE;
      for (int q = 0; q < p.sp.n_params; ++q) th[q] = 0.5 + U(rng);
      for (int t = 0; t < p.sp.n_terms; ++t) th[p.sp.terms[t].param_offset] = 0.3 * std::pow(200.0, U(rng));
      if (b < 2) th[0] = 0.8 + 1.4 * U(rng);  // ℓ ∈ [0.8, 2.2]: band16 widths Q = 2..6
      th[p.sp.n_params] = 1e-5;
      band_tables(&bt, b, p.x.data());
      // the box path (gpx_batch_rebind_device's gather hands back 16-row boxes) gives the same tables
      {
        const int nv16 = (p.n + kBox - 1) / kBox;
        std::vector<double> box((size_t)nv16 * D * 2);
        for (int k = 0; k < nv16; ++k)
          for (int d = 0; d < D; ++d) {
            double a = INFINITY, z = -INFINITY;
            for (int r = k * kBox; r < std::min(p.n, (k + 1) * kBox); ++r) {
              a = std::min(a, p.x[(size_t)r * D + d]);
              z = std::max(z, p.x[(size_t)r * D + d]);
            }
            box[2 * ((size_t)k * D + d)] = a;
            box[2 * ((size_t)k * D + d) + 1] = z;
          }
        const size_t t64 = (size_t)GPX_MAX_TERMS * (bt.Np / kLeaf), t16 = (size_t)GPX_MAX_TERMS * (bt.Np / kBox);
        std::vector<double> r64(bt.band_rmin.begin() + b * t64, bt.band_rmin.begin() + (b + 1) * t64);
        std::vector<double> r16(bt.band_rmin16.begin() + b * t16, bt.band_rmin16.begin() + (b + 1) * t16);
        band_tables_boxes(&bt, b, box.data());
        bool same = true;
        for (size_t e = 0; e < t64; ++e) same = same && r64[e] == bt.band_rmin[b * t64 + e];
        for (size_t e = 0; e < t16; ++e) same = same && r16[e] == bt.band_rmin16[b * t16 + e];
        CHECK(same, "round %d problem %d: band_tables_boxes differs from band_tables", round, b);
      }
    }
    // widths: safe and (sorted 1-D) tight
    for (int b = 0; b < B; ++b) {
      const Problem& p = pr[b];
      const double* th = theta.data() + (size_t)b * GPX_THETA_STRIDE;
      const int w64 = band_width(&bt, b, th), w16 = band_width16(&bt, b, th);
      bool bandable = true;
      for (int t = 0; t < p.sp.n_terms; ++t) bandable = bandable && p.sp.terms[t].kind <= GPX_EXPONENTIAL;
      CHECK((w64 < 0) == !bandable, "round %d problem %d: band_width %d for a %s kernel", round, b, w64,
            bandable ? "band" : "non-band");
      if (!bandable) continue;
      // true widths from every pair (i > j) within reach: beyond the reported band every entry
      // must be an exact zero
      int t64 = 0, t16 = 0;
      const int reach = std::min(p.n, 64 * (w64 + 3));
      for (int i = 0; i < p.n; ++i) {
        const int j0 = p.sorted1d ? std::max(0, i - reach) : 0;
        for (int j = j0; j < i; ++j) {
          if ((i >> 6) - (j >> 6) <= t64 && (i >> 4) - (j >> 4) <= t16) continue;
          ++checked_pairs;
          if (entry_nz(p.sp, th, &p.x[(size_t)i * D], &p.x[(size_t)j * D])) {
            t64 = std::max(t64, (i >> 6) - (j >> 6));
            t16 = std::max(t16, (i >> 4) - (j >> 4));
          }
        }
      }
      CHECK(w64 >= t64, "round %d problem %d: band_width %d < true %d (nonzero entries beyond the band)", round, b,
            w64, t64);
      CHECK(w16 >= t16, "round %d problem %d: band_width16 %d < true %d", round, b, w16, t16);
      // tight for sorted 1-D inputs while the true band is inside the tables' exact range (beyond
      // the widest band any path routes the tables repeat a lower bound: "dense", by design)
      if (p.sorted1d && p.sp.n_terms == 1) {
        const int cap64 = bt.Np / kLeaf / 4 + 1, cap16 = kBand16MaxQ + 1;
        if (t64 + 1 < cap64)
          CHECK(w64 <= t64 + 1, "round %d problem %d: band_width %d loose (true %d)", round, b, w64, t64);
        if (t16 + 1 < cap16)
          CHECK(w16 <= t16 + 1, "round %d problem %d: band_width16 %d loose (true %d)", round, b, w16, t16);
        tight_checked += (t16 + 1 < cap16);
      }
    }
    // routing under the switches
    static const char* envs[][2] = {{"GPX_BAND", nullptr}, {"GPX_BAND16", "0"}, {"GPX_BAND_FUSED", "0"},
                                    {"GPX_BAND", "0"}};
    for (int v = 0; v < 4; ++v) {
      unsetenv("GPX_BAND");
      unsetenv("GPX_BAND16");
      unsetenv("GPX_BAND_FUSED");
      if (envs[v][1]) setenv(envs[v][0], envs[v][1], 1);
      std::vector<int32_t> active;
      for (int b = 0; b < B; ++b)
        if (v == 0 || (rng() & 3)) active.push_back(b);
      std::fill(bandp.begin(), bandp.end(), -7);
      Route rt;
      route_call(&bt, (int)active.size(), active.data(), theta.data(), rt);
      std::vector<int> seen(B, 0);
      for (int b : rt.order) seen[b]++;
      for (int b : rt.shadow_ids) seen[b]++;
      for (int b = 0; b < B; ++b) {
        const bool act = std::find(active.begin(), active.end(), b) != active.end();
        CHECK(seen[b] == (act ? 1 : 0), "round %d env %d: problem %d routed %d times", round, v, b, seen[b]);
      }
      CHECK((int)rt.order.size() == rt.n_dense + rt.n_band + rt.n_fused, "order size %zu vs classes", rt.order.size());
      CHECK(!bt.compact || (rt.n_dense == 0 && rt.n_band == 0), "band storage routed problems to dense/per-block");
      int s16 = 0;
      for (int g = 0; g < rt.n_g16; ++g) {
        s16 += rt.g16_n[g];
        CHECK(rt.g16_q[g] >= 1 && rt.g16_q[g] <= kBand16MaxQ && (g == 0 || rt.g16_q[g] > rt.g16_q[g - 1]),
              "band16 group widths not increasing in 1..%d", kBand16MaxQ);
      }
      CHECK(s16 == rt.n16, "band16 group sizes %d vs n16 %d", s16, rt.n16);
      CHECK(rt.n_fused1 <= rt.n_fused - rt.n16, "fused p<=1 count");
      // segment checks
      int pos = rt.n_dense + rt.n_band;
      for (int g = 0; g < rt.n_g16; ++g)
        for (int i = 0; i < rt.g16_n[g]; ++i, ++pos) {
          const int b = rt.order[pos];
          const double* th = theta.data() + (size_t)b * GPX_THETA_STRIDE;
          const int w16 = band_width16(&bt, b, th);
          CHECK(bandp[b] == rt.g16_q[g] && std::max(w16, 1) == rt.g16_q[g] && band_width(&bt, b, th) <= 2,
                "band16 problem %d: h_bandp %d, group Q %d, width16 %d", b, bandp[b], rt.g16_q[g], w16);
          ++band16_routed;
        }
      for (int i = 0; i < rt.n_fused - rt.n16; ++i, ++pos) {
        const int b = rt.order[pos];
        const int p = band_width(&bt, b, theta.data() + (size_t)b * GPX_THETA_STRIDE);
        CHECK(bandp[b] == p && p <= 2 && ((i < rt.n_fused1) == (p <= 1)), "fused problem %d: p %d bandp %d", b, p,
              bandp[b]);
      }
      // gpx_batch_band_class (the drivers' class query) agrees with the routing
      {
        std::vector<int32_t> cls(active.size());
        CHECK(gpx_batch_band_class(&bt, (int)active.size(), active.data(), theta.data(), cls.data()) == GPX_OK,
              "gpx_batch_band_class failed");
        const int q16lim = route_limits(&bt).q16lim;
        for (size_t i = 0; i < active.size(); ++i) {
          const int b = active[i];
          const auto at = std::find(rt.order.begin(), rt.order.end(), b) - rt.order.begin();
          const double* th = theta.data() + (size_t)b * GPX_THETA_STRIDE;
          int want;
          if (at >= (long)rt.order.size() || at < rt.n_dense) {
            want = -1;  // dense, or band storage's fallback slots
          } else if (at < rt.n_dense + rt.n_band || at >= rt.n_dense + rt.n_band + rt.n16) {
            want = (q16lim > 0 ? 32 : 16) + band_width(&bt, b, th);
          } else {
            want = bandp[b];
          }
          CHECK(cls[i] == want, "round %d env %d problem %d: band_class %d, routed as %d", round, v, b, cls[i], want);
        }
      }
      if (v == 1) CHECK(rt.n16 == 0, "GPX_BAND16=0 still routed %d problems to band16", rt.n16);
      if (v == 3) CHECK(rt.n16 + rt.n_band + rt.n_fused == 0 || bt.compact == 0 ? rt.n_band + rt.n_fused == 0 : true,
                        "GPX_BAND=0 still routed banded problems");
      routed += (long long)active.size();
    }
    unsetenv("GPX_BAND");
    unsetenv("GPX_BAND16");
    unsetenv("GPX_BAND_FUSED");
    bt.h_bandp = nullptr;
  }
  std::printf("pairs checked %lld, tight band16 widths %lld, problems routed %lld (band16 %lld), failures %d\n",
              checked_pairs, tight_checked, routed, band16_routed, g_fail);
  if (g_fail) return 1;
  std::printf("OK\n");
  return 0;
}
