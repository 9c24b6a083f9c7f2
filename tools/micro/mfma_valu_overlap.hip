// Does an f64 MFMA chain overlap with independent f64 VALU work of the same wave on gfx950?
// Three kernels, one wave per SIMD (1024 single-wave workgroups), cycles by s_memtime per wave:
//   A: NM v_mfma_f64_16x16x4_f64 (4 independent accumulators)
//   B: NV v_fma_f64 (8 independent chains)
//   C: both, interleaved by sched_group_barrier (1 MFMA, then NV/NM FMAs)
// usage: hipcc --offload-arch=gfx950 -O3 mfma_valu_overlap.hip -o /tmp/ovl && /tmp/ovl
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double t4 __attribute__((ext_vector_type(4)));
constexpr int NM = 64, NV = 512, REP = 64;

template <bool DO_M, bool DO_V, bool SGB>
__global__ __launch_bounds__(64, 1) void kern(const double* __restrict__ in, double* __restrict__ out,
                                              unsigned long long* __restrict__ cyc) {
  const int lane = threadIdx.x;
  double a = in[lane], b = in[lane + 64];
  t4 c0 = {a, b, a, b}, c1 = c0 * 2.0, c2 = c0 * 3.0, c3 = c0 * 4.0;
  double v[8];
  for (int i = 0; i < 8; ++i) v[i] = a + i;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int rep = 0; rep < REP; ++rep) {
#pragma unroll
    for (int i = 0; i < NM / 4; ++i) {
      if (DO_M) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
      }
      if (DO_V) {
#pragma unroll
        for (int j = 0; j < NV / NM * 4 / 8; ++j)
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] = __builtin_fma(v[q], a, b);
      }
    }
    if (SGB) {
#pragma unroll
      for (int g = 0; g < NM; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, NV / NM, 0);
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = c0[0] + c1[1] + c2[2] + c3[3];
  for (int i = 0; i < 8; ++i) s += v[i];
  out[blockIdx.x * 64 + lane] = s;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <bool M, bool V, bool S>
static void run(const char* name, double* in, double* out, unsigned long long* cyc, int blocks) {
  kern<M, V, S><<<blocks, 64>>>(in, out, cyc);
  kern<M, V, S><<<blocks, 64>>>(in, out, cyc);
  hipDeviceSynchronize();
  static unsigned long long h[4096];
  hipMemcpy(h, cyc, blocks * 8, hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < blocks; ++i) m += h[i];
  m /= blocks;
  printf("%-28s blocks %5d  cycles/rep %8.1f  per MFMA %6.1f  per FMA %6.2f\n", name, blocks, m / REP, m / REP / NM,
         m / REP / NV);
}

int main() {
  double *in, *out;
  unsigned long long* cyc;
  hipMalloc(&in, 128 * 8);
  hipMemset(in, 0, 128 * 8);
  hipMalloc(&out, 4096 * 64 * 8);
  hipMalloc(&cyc, 4096 * 8);
  for (int blocks : {1024, 2048}) {
    run<true, false, false>("A mfma only", in, out, cyc, blocks);
    run<false, true, false>("B fma only", in, out, cyc, blocks);
    run<true, true, false>("C both (compiler order)", in, out, cyc, blocks);
    run<true, true, true>("C both (sched groups)", in, out, cyc, blocks);
  }
  return 0;
}
