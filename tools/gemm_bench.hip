// Standalone microbenchmark of gpx::launch_gemm (fp64 MFMA tile GEMM) on random data.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>
#include "../portfoliooptgp_amd/csrc/gpx_internal.h"
using namespace gpx;
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void fill(double* p, size_t n, unsigned seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed; x ^= x >> 13; x *= 0x5bd1e995; x ^= x >> 15;
    p[i] = (x & 0xffffff) / double(0x1000000) - 0.5;
  }
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 2048;
  const int B = argc > 2 ? atoi(argv[2]) : 8;
  // run only the cases with this name prefix ("all": every case)
  const char* only = (argc > 3 && std::string(argv[3]) != "all") ? argv[3] : nullptr;
  const int ld = n + (argc > 4 ? atoi(argv[4]) : 0);  // leading dimension (row padding test)
  const size_t sz = (size_t)n * ld;
  double *A, *Bm, *C;
  CK(hipMalloc(&A, sz * B * 8)); CK(hipMalloc(&Bm, sz * B * 8)); CK(hipMalloc(&C, sz * B * 8));
  fill<<<1024, 256>>>(A, sz * B, 1); fill<<<1024, 256>>>(Bm, sz * B, 2); fill<<<1024, 256>>>(C, sz * B, 3);
  int* act; CK(hipMalloc(&act, B * 4));
  std::vector<int> h(B); for (int i = 0; i < B; ++i) h[i] = i;
  CK(hipMemcpy(act, h.data(), B * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  struct Case { const char* name; bool ta, tb; int tri, lower; int kdiv = 1; };
  Case cases[] = {{"NT full K/2", false, true, 0, 0, 2}, {"NN full K/2", false, false, 0, 0, 2},{"NN full", false, false, 0, 0}, {"NT full", false, true, 0, 0}, {"TN full", true, false, 0, 0},
                  {"NT syrk(lower)", false, true, 0, 1}, {"NT trmm kmax_j", false, true, TRI_KMAX_J, 0},
                  {"NN trmm kmin_j", false, false, TRI_KMIN_J, 0}, {"NN trmm kmax_i", false, false, TRI_KMAX_I, 0},
                  {"TN lauum(lower,kmin_i)", true, false, TRI_KMIN_I, 1},
                  {"TN syrk(lower)", true, false, 0, 1}, {"NT lauum(lower,kmin_i)", false, true, TRI_KMIN_I, 1}};
  for (auto& c : cases) {
    if (only && std::string(c.name).rfind(only, 0) != 0) continue;
    GemmArgs g{};
    g.active = act; g.A = A; g.sA = sz; g.lda = ld; g.Bm = Bm; g.sB = sz; g.ldb = ld; g.C = C; g.sC = sz; g.ldc = ld;
    g.M = g.N = n; g.K = n / c.kdiv; g.tri = c.tri; g.lower_only = c.lower;
    g.order = (c.tri & TRI_KMAX_J) ? ORDER_COL_DESC : (c.tri & TRI_KMIN_J) ? ORDER_COL_ASC
            : (c.tri & TRI_KMAX_I) ? ORDER_ROW_DESC : ORDER_ROW_ASC; g.alpha = -1.0; g.beta = 1.0;
    // issued flops
    const int bm = gemm_tile(g, B);
    double f = 0;
    for (int x = 0; x < n / bm; ++x) for (int y = 0; y < n / bm; ++y) {
      if (c.lower && y > x) continue;
      int kmin = 0, kmax = n / c.kdiv, i0 = x * bm, j0 = y * bm;
      if (c.tri & TRI_KMAX_I) kmax = std::min(kmax, i0 + bm);
      if (c.tri & TRI_KMAX_J) kmax = std::min(kmax, j0 + bm);
      if (c.tri & TRI_KMIN_J) kmin = std::max(kmin, j0);
      if (c.tri & TRI_KMIN_I) kmin = std::max(kmin, i0);
      if (kmax > kmin) f += 2.0 * bm * bm * (kmax - kmin);
    }
    f *= B;
    for (int epi = 0; epi < (c.tri == TRI_KMIN_I ? 2 : 1); ++epi) {
      GemmArgs gg = g;
      if (epi == 1) {  // the fused gradient contraction on the same shape (SE kernel spec)
        static double *alpha = nullptr, *X = nullptr, *theta = nullptr, *partial = nullptr;
        static DevSpec* spec = nullptr; static int* nv = nullptr;
        if (!alpha) {
          CK(hipMalloc(&alpha, (size_t)B * n * 8)); fill<<<256, 256>>>(alpha, (size_t)B * n, 7);
          CK(hipMalloc(&X, (size_t)B * n * 8)); fill<<<256, 256>>>(X, (size_t)B * n, 8);
          CK(hipMalloc(&theta, B * 16 * 8)); std::vector<double> th(B * 16, 1.0);
          CK(hipMemcpy(theta, th.data(), B * 16 * 8, hipMemcpyHostToDevice));
          CK(hipMalloc(&partial, (size_t)B * 2080 * 16 * 8));
          DevSpec sp{}; sp.n_terms = 1; sp.combine = 0; sp.n_params = 2; sp.terms[0].kind = 1;
          sp.terms[0].dim_start = 0; sp.terms[0].dim_count = 1; sp.terms[0].param_offset = 0;
          std::vector<DevSpec> sps(B, sp); CK(hipMalloc(&spec, B * sizeof(DevSpec)));
          CK(hipMemcpy(spec, sps.data(), B * sizeof(DevSpec), hipMemcpyHostToDevice));
          std::vector<int> nn(B, n); CK(hipMalloc(&nv, B * 4)); CK(hipMemcpy(nv, nn.data(), B * 4, hipMemcpyHostToDevice));
        }
        gg.vec = alpha; gg.sVec = n; gg.X = X; gg.sX = n; gg.D = 1; gg.specs = spec; gg.theta = theta;
        gg.nvalid = nv; gg.partial = partial; gg.sPartial = 2080 * 16;
      }
      const int ep = epi ? EPI_CONTRACT1 : EPI_STORE;
      launch_gemm(gg, ep, c.ta, c.tb, B, 0);
      CK(hipDeviceSynchronize());
      const int reps = 5;
      CK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) launch_gemm(gg, ep, c.ta, c.tb, B, 0);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); ms /= reps;
      printf("%-22s%s n=%d ld=%d B=%d tile=%d: %8.3f ms  %6.2f TF/s (issued)\n", c.name, epi ? " +contract" : "", n, ld, B, bm, ms, f / ms / 1e9);
    }
  }
  return 0;
}
