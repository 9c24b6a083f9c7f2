// Does a v_fma_f64 chain cost less when only part of the wave is active (exec mask)?
// One wave per SIMD, cycles per FMA for 64 / 32 / 16 / 1 active lanes. usage: hipcc ... && ./exec_mask_f64
#include <hip/hip_runtime.h>
#include <cstdio>
constexpr int NV = 512, REP = 64;
__global__ __launch_bounds__(64, 1) void kern(const double* __restrict__ in, double* __restrict__ out,
                                              unsigned long long* __restrict__ cyc, int active) {
  const int lane = threadIdx.x;
  double a = in[lane], b = in[lane + 64];
  double v[8];
  for (int i = 0; i < 8; ++i) v[i] = a + i;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (lane < active) {
    for (int rep = 0; rep < REP; ++rep) {
#pragma unroll
      for (int j = 0; j < NV / 8; ++j)
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = __builtin_fma(v[q], a, b);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int i = 0; i < 8; ++i) s += v[i];
  out[blockIdx.x * 64 + lane] = s;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  double *in, *out;
  unsigned long long* cyc;
  (void)hipMalloc(&in, 128 * 8);
  (void)hipMemset(in, 0, 128 * 8);
  (void)hipMalloc(&out, 4096 * 64 * 8);
  (void)hipMalloc(&cyc, 4096 * 8);
  static unsigned long long h[4096];
  for (int blocks : {1024, 2048})
    for (int act : {64, 32, 16, 4, 1}) {
      kern<<<blocks, 64>>>(in, out, cyc, act);
      kern<<<blocks, 64>>>(in, out, cyc, act);
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
      double m = 0;
      for (int i = 0; i < blocks; ++i) m += h[i];
      m /= blocks;
      printf("blocks %5d active lanes %2d  cycles per v_fma_f64 %6.2f\n", blocks, act, m / REP / NV);
    }
  return 0;
}
