/* A plain-C consumer of the C ABI (include/gpx.h), as a non-Python host of the reference would
 * bind it: device buffers from the HIP runtime API, one batch of two GPR problems, logML +
 * gradient, predict at new inputs, predict at the training inputs. Prints one JSON line; the
 * GPU test (tests/test_c_abi_gpu.py) checks it against the CPU oracle.
 * usage: gpx_c_smoke N   (problem 0: X = 0..N-1, Y = sin(x/7); problem 1: N/2 points, Matern52) */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "gpx.h"

#define CHECK(x)                                                              \
  do {                                                                        \
    int rc_ = (int)(x);                                                       \
    if (rc_ != 0) {                                                           \
      fprintf(stderr, "%s failed: %d (%s)\n", #x, rc_, ctx ? gpx_last_error(ctx) : ""); \
      return 1;                                                               \
    }                                                                         \
  } while (0)

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 89;
  const int B = 2, M = 7;
  gpx_ctx* ctx = NULL;
  if (N < 2) return 2;
  double* hX = calloc((size_t)B * N, sizeof(double));
  double* hY = calloc((size_t)B * N, sizeof(double));
  int32_t n[2] = {N, N / 2};
  for (int b = 0; b < B; ++b)
    for (int i = 0; i < n[b]; ++i) {
      hX[(size_t)b * N + i] = (double)i;
      hY[(size_t)b * N + i] = sin(i / 7.0) + (b ? 0.3 * cos(i / 3.0) : 0.0);
    }
  double hXn[7] = {-1.5, 0.0, 3.25, 10.0, 40.5, 88.0, 120.0};
  double *dX, *dY, *dXn, *dMean, *dVar;
  if (hipMalloc((void**)&dX, sizeof(double) * B * N) || hipMalloc((void**)&dY, sizeof(double) * B * N) ||
      hipMalloc((void**)&dXn, sizeof(double) * B * M) || hipMalloc((void**)&dMean, sizeof(double) * B * N) ||
      hipMalloc((void**)&dVar, sizeof(double) * B * N))
    return 3;
  hipMemcpy(dX, hX, sizeof(double) * B * N, hipMemcpyHostToDevice);
  hipMemcpy(dY, hY, sizeof(double) * B * N, hipMemcpyHostToDevice);
  for (int b = 0; b < B; ++b) hipMemcpy(dXn + b * M, hXn, sizeof(hXn), hipMemcpyHostToDevice);

  CHECK(gpx_create(0, &ctx));
  gpx_kernel_spec specs[2] = {
      {.n_terms = 1, .combine = GPX_SUM, .n_params = 2, .terms = {{GPX_SE, 0, 1, 0}}},
      {.n_terms = 1, .combine = GPX_SUM, .n_params = 2, .terms = {{GPX_MATERN52, 0, 1, 0}}}};
  gpx_batch* bt = NULL;
  CHECK(gpx_batch_create(ctx, B, N, 1, dX, dY, n, specs, &bt));
  double theta[2 * GPX_THETA_STRIDE];
  for (int i = 0; i < 2 * GPX_THETA_STRIDE; ++i) theta[i] = 1.0;
  theta[0] = 3.0; theta[1] = 1.5; theta[2] = 1e-2;                                         /* ℓ, σ², σn² */
  theta[GPX_THETA_STRIDE + 0] = 5.0; theta[GPX_THETA_STRIDE + 1] = 0.7; theta[GPX_THETA_STRIDE + 2] = 1e-3;
  int32_t act[2] = {0, 1}, info[2] = {0, 0};
  double lml[2], grad[2 * GPX_THETA_STRIDE];
  CHECK(gpx_batch_lml_grad(bt, B, act, theta, lml, grad, info, NULL));
  CHECK(gpx_batch_predict(bt, B, act, theta, dXn, M, 0, dMean, dVar, info, NULL));
  double mean[2 * 7], var[2 * 7];
  hipMemcpy(mean, dMean, sizeof(mean), hipMemcpyDeviceToHost);
  hipMemcpy(var, dVar, sizeof(var), hipMemcpyDeviceToHost);
  CHECK(gpx_batch_predict_train(bt, 1, act, theta, 1, dMean, dVar, info, NULL));
  double ytrain_var0;
  hipMemcpy(&ytrain_var0, dVar, sizeof(double), hipMemcpyDeviceToHost);
  /* the same prediction packed by position: problem 1's row lands in row 0 */
  const int32_t act1[1] = {1};
  CHECK(gpx_batch_predict_train(bt, 1, act1, theta, 1, dMean, dVar, info, NULL));
  double v1_full[2], v1_rows[2];
  hipMemcpy(v1_full, dVar + N, sizeof(v1_full), hipMemcpyDeviceToHost);
  CHECK(gpx_batch_predict_train_rows(bt, 1, act1, theta, 1, dMean, dVar, info, NULL));
  hipMemcpy(v1_rows, dVar, sizeof(v1_rows), hipMemcpyDeviceToHost);
  const int rows_match = v1_full[0] == v1_rows[0] && v1_full[1] == v1_rows[1];
  /* a bad argument comes back as a status code, never as a C++ exception */
  const int bad = gpx_batch_lml_grad(bt, 0, act, theta, lml, grad, info, NULL);

  printf("{\"version\": \"%s\", \"N\": %d, \"lml\": [%.17g, %.17g], \"grad\": [[%.17g, %.17g, %.17g], [%.17g, %.17g, %.17g]], ",
         gpx_version(), N, lml[0], lml[1], grad[0], grad[1], grad[2], grad[GPX_THETA_STRIDE],
         grad[GPX_THETA_STRIDE + 1], grad[GPX_THETA_STRIDE + 2]);
  printf("\"mean\": [");
  for (int i = 0; i < 2 * M; ++i) printf("%s%.17g", i ? ", " : "", mean[i]);
  printf("], \"var\": [");
  for (int i = 0; i < 2 * M; ++i) printf("%s%.17g", i ? ", " : "", var[i]);
  printf("], \"ytrain_var0\": %.17g, \"train_rows_match\": %d, \"bad_arg_status\": %d}\n", ytrain_var0,
         rows_match, bad);
  gpx_batch_destroy(bt);
  gpx_destroy(ctx);
  hipFree(dX); hipFree(dY); hipFree(dXn); hipFree(dMean); hipFree(dVar);
  free(hX); free(hY);
  return 0;
}
