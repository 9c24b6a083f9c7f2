// Probe: v_mfma_f64_16x16x4_f64 operand/result layout + FP64 MFMA and VALU throughput on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>

typedef double d4 __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// A: 16x4 row-major, B: 4x16 row-major. Hypothesis: lane l holds A[l&15][l>>4], B[l>>4][l&15];
// D[(l>>4)+4r][l&15] in reg r.
__global__ void layout_kernel(const double* A, const double* B, double* D) {
  int l = threadIdx.x;
  double a = A[(l & 15) * 4 + (l >> 4)];
  double b = B[(l >> 4) * 16 + (l & 15)];
  d4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[((l >> 4) + 4 * r) * 16 + (l & 15)] = c[r];
}

template <int NACC>
__global__ void mfma_tput(double* out, int iters, double seed) {
  double a = seed + threadIdx.x * 1e-3, b = seed - threadIdx.x * 1e-3;
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (d4){0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void fma_tput(double* out, int iters, double seed) {
  double x0 = seed + threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;
  const double m = 0.9999999, c = 1e-9;
  for (int it = 0; it < iters; ++it) {
    x0 = fma(x0, m, c); x1 = fma(x1, m, c); x2 = fma(x2, m, c); x3 = fma(x3, m, c);
    x4 = fma(x4, m, c); x5 = fma(x5, m, c); x6 = fma(x6, m, c); x7 = fma(x7, m, c);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
}

int main() {
  // layout
  std::vector<double> A(64), B(64), D(256), R(256, 0.0);
  for (int i = 0; i < 64; ++i) { A[i] = (i * 7 % 13) - 6; B[i] = (i * 5 % 11) - 5 + 0.5 * (i % 3); }
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) for (int k = 0; k < 4; ++k) R[i * 16 + j] += A[i * 4 + k] * B[k * 16 + j];
  double *dA, *dB, *dD, *dO;
  CK(hipMalloc(&dA, 64 * 8)); CK(hipMalloc(&dB, 64 * 8)); CK(hipMalloc(&dD, 256 * 8));
  CK(hipMemcpy(dA, A.data(), 512, hipMemcpyHostToDevice)); CK(hipMemcpy(dB, B.data(), 512, hipMemcpyHostToDevice));
  layout_kernel<<<1, 64>>>(dA, dB, dD);
  CK(hipMemcpy(D.data(), dD, 256 * 8, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < 256; ++i) if (D[i] != R[i]) ++bad;
  printf("layout mismatches: %d / 256\n", bad);

  int nblk = 256 * 8, thr = 256;
  CK(hipMalloc(&dO, (size_t)nblk * thr * 8));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  int iters = 4000;
  for (int rep = 0; rep < 2; ++rep) {
    mfma_tput<4><<<nblk, thr>>>(dO, 10, 1.0);
    CK(hipEventRecord(e0));
    mfma_tput<4><<<nblk, thr>>>(dO, iters, 1.0);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    double flops = (double)nblk * (thr / 64) * iters * 4 * 2048.0;
    printf("mfma_f64_16x16x4 (4 acc, %d WG x %d thr): %.3f ms, %.2f TFLOP/s\n", nblk, thr, ms, flops / ms / 1e9);
  }
  for (int rep = 0; rep < 2; ++rep) {
    mfma_tput<1><<<nblk, thr>>>(dO, 10, 1.0);
    CK(hipEventRecord(e0));
    mfma_tput<1><<<nblk, thr>>>(dO, iters, 1.0);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    double flops = (double)nblk * (thr / 64) * iters * 1 * 2048.0;
    printf("mfma_f64_16x16x4 (1 acc dependent chain): %.3f ms, %.2f TFLOP/s\n", ms, flops / ms / 1e9);
  }
  // single-wave-per-SIMD latency probe: 256 WG x 256 thr (1 wave per SIMD), 1 acc
  {
    mfma_tput<1><<<256, 256>>>(dO, 10, 1.0);
    CK(hipEventRecord(e0));
    mfma_tput<1><<<256, 256>>>(dO, iters, 1.0);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("1 wave/SIMD, 1 acc chain: %.1f ns per MFMA (~%.0f cycles at 2.4GHz)\n", ms * 1e6 / iters, ms * 1e6 / iters * 2.4);
    mfma_tput<4><<<256, 256>>>(dO, 10, 1.0);
    CK(hipEventRecord(e0));
    mfma_tput<4><<<256, 256>>>(dO, iters, 1.0);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("1 wave/SIMD, 4 acc: %.1f ns per MFMA (~%.0f cycles at 2.4GHz)\n", ms * 1e6 / iters / 4, ms * 1e6 / iters / 4 * 2.4);
  }
  for (int rep = 0; rep < 2; ++rep) {
    fma_tput<<<nblk, thr>>>(dO, 10, 1.0);
    CK(hipEventRecord(e0));
    fma_tput<<<nblk, thr>>>(dO, iters, 1.0);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    double flops = (double)nblk * thr * iters * 8 * 2.0;
    printf("v_fma_f64 VALU: %.3f ms, %.2f TFLOP/s\n", ms, flops / ms / 1e9);
  }
  return 0;
}
