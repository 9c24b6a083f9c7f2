// Probe: int8 MFMA on gfx950 (v_mfma_i32_32x32x32_i8) — operand/result layout, register-only
// throughput, and an LDS-tiled batched C = A·Bᵀ (int8 in, int32 accumulate, result reduced
// mod p to one byte, as an Ozaki-II residue product would be). Decides whether emulating the
// fp64 contraction on int8 MFMA (one GEMM per modulus) can beat the fp64 MFMA.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

typedef int i4 __attribute__((ext_vector_type(4)));
typedef int i16 __attribute__((ext_vector_type(16)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// A: 32x32 (row-major, k contiguous), B: 32x32 stored [n][k]. Hypothesis: lane l holds
// A[l&31][16(l>>5) + j] and B[n=l&31][16(l>>5) + j], j = 0..15 (bytes of the 4 dwords);
// D reg r of lane l: row (r&3) + 8(r>>2) + 4(l>>5), col l&31.
__global__ void layout_kernel(const int8_t* A, const int8_t* B, int* D) {
  const int l = threadIdx.x;
  i4 a = *reinterpret_cast<const i4*>(A + (l & 31) * 32 + 16 * (l >> 5));
  i4 b = *reinterpret_cast<const i4*>(B + (l & 31) * 32 + 16 * (l >> 5));
  i16 c = {};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) D[((r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 32 + (l & 31)] = c[r];
}

template <int NACC>
__global__ __launch_bounds__(256) void mfma_tput(int* out, int iters) {
  i4 a = {(int)threadIdx.x, 3, 5, 7}, b = {11, (int)threadIdx.x, 13, 17};
  i16 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (i16){};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[i], 0, 0, 0);
  }
  int s = 0;
  for (int i = 0; i < NACC; ++i) for (int r = 0; r < 16; ++r) s += acc[i][r];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// Batched C[b] = A[b] · B[b]ᵀ mod p, A [M][K], B [N][K] int8 (k contiguous), C uint8 [M][N].
// 256x256 tile per workgroup, 4 waves 2x2 of 128x128 (4x4 blocks of 32x32), BK = 64,
// register-staged double-buffered LDS, row stride 80 B (conflict-free ds_read_b128).
constexpr int TM = 256, BK = 64, LS = 80;
__global__ __launch_bounds__(256, 1) void gemm_i8(const int8_t* __restrict__ A, const int8_t* __restrict__ B,
                                                   uint8_t* __restrict__ C, int M, int N, int K, int p) {
  __shared__ __attribute__((aligned(16))) int8_t smem[2 * 2 * TM * LS];
  const int ntn = N / TM, ntiles = (M / TM) * ntn;
  const int b = blockIdx.x / ntiles, t = blockIdx.x % ntiles;
  const int m0 = (t / ntn) * TM, n0 = (t % ntn) * TM;
  const int8_t* Ab = A + (size_t)b * M * K;
  const int8_t* Bb = B + (size_t)b * N * K;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wr = wave >> 1, wc = wave & 1;
  i16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (i16){};
  i4 ra[4], rb[4];
  auto gload = [&](int k0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = tid + 256 * q, row = c >> 2, kc = (c & 3) * 16;
      ra[q] = *reinterpret_cast<const i4*>(Ab + (size_t)(m0 + row) * K + k0 + kc);
      rb[q] = *reinterpret_cast<const i4*>(Bb + (size_t)(n0 + row) * K + k0 + kc);
    }
  };
  auto swrite = [&](int buf) {
    int8_t* sA = smem + buf * 2 * TM * LS;
    int8_t* sB = sA + TM * LS;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = tid + 256 * q, row = c >> 2, kc = (c & 3) * 16;
      *reinterpret_cast<i4*>(sA + row * LS + kc) = ra[q];
      *reinterpret_cast<i4*>(sB + row * LS + kc) = rb[q];
    }
  };
  auto compute = [&](int buf) {
    const int8_t* sA = smem + buf * 2 * TM * LS;
    const int8_t* sB = sA + TM * LS;
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      i4 af[4], bf[4];
      const int ko = s * 32 + (lane >> 5) * 16;
#pragma unroll
      for (int m = 0; m < 4; ++m) af[m] = *reinterpret_cast<const i4*>(sA + (wr * 128 + m * 32 + (lane & 31)) * LS + ko);
#pragma unroll
      for (int n = 0; n < 4; ++n) bf[n] = *reinterpret_cast<const i4*>(sB + (wc * 128 + n * 32 + (lane & 31)) * LS + ko);
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[m], bf[n], acc[m][n], 0, 0, 0);
    }
  };
  const int nk = K / BK;
  gload(0);
  swrite(0);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk - 1; ++kt) {
    gload((kt + 1) * BK);
    compute(cur);
    swrite(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
  compute(cur);
  uint8_t* Cb = C + (size_t)b * M * N;
  const float inv_p = 1.0f / (float)p;
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wr * 128 + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int col = n0 + wc * 128 + n * 32 + (lane & 31);
        const int v = acc[m][n][r];
        int q = (int)((float)v * inv_p);
        int res = v - q * p;
        res += (res < 0) ? p : 0;
        res -= (res >= p) ? p : 0;
        Cb[(size_t)row * N + col] = (uint8_t)res;
      }
}

__global__ void fill_i8(int8_t* x, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed; h ^= h >> 13; h *= 0x5bd1e995; h ^= h >> 15;
    x[i] = (int8_t)((int)(h % 251) - 125);
  }
}

int main(int argc, char** argv) {
  // 1. layout
  std::vector<int8_t> A(1024), B(1024);
  std::vector<int> D(1024), R(1024, 0);
  for (int i = 0; i < 1024; ++i) { A[i] = (int8_t)((i * 7 % 23) - 11); B[i] = (int8_t)((i * 5 % 19) - 9 + (i % 3)); }
  for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) for (int k = 0; k < 32; ++k) R[i * 32 + j] += A[i * 32 + k] * B[j * 32 + k];
  int8_t *dA, *dB; int* dD;
  CK(hipMalloc(&dA, 1024)); CK(hipMalloc(&dB, 1024)); CK(hipMalloc(&dD, 4096));
  CK(hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice)); CK(hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice));
  layout_kernel<<<1, 64>>>(dA, dB, dD);
  CK(hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < 1024; ++i) bad += D[i] != R[i];
  printf("i8 32x32x32 layout mismatches: %d / 1024\n", bad);

  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  // 2. register-only rate
  int* dO; const int nblk = 256 * 4, thr = 256, iters = 2000;
  CK(hipMalloc(&dO, (size_t)nblk * thr * 4));
  for (int rep = 0; rep < 2; ++rep) {
    mfma_tput<4><<<nblk, thr>>>(dO, 10);
    CK(hipEventRecord(e0));
    mfma_tput<4><<<nblk, thr>>>(dO, iters);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double ops = (double)nblk * (thr / 64) * iters * 4 * 65536.0;
    printf("mfma_i32_32x32x32_i8 registers (4 acc, %d WG x %d thr): %.3f ms, %.1f TOPS\n", nblk, thr, ms, ops / ms / 1e9);
  }
  // 3. tiled batched GEMM with mod-p byte epilogue
  const int n = argc > 1 ? atoi(argv[1]) : 4096, batch = argc > 2 ? atoi(argv[2]) : 16;
  const size_t sz = (size_t)n * n;
  int8_t *GA, *GB; uint8_t* GC;
  CK(hipMalloc(&GA, sz * batch)); CK(hipMalloc(&GB, sz * batch)); CK(hipMalloc(&GC, sz * batch));
  fill_i8<<<2048, 256>>>(GA, sz * batch, 1); fill_i8<<<2048, 256>>>(GB, sz * batch, 2);
  const int grid = (n / TM) * (n / TM) * batch;
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0));
    gemm_i8<<<grid, 256>>>(GA, GB, GC, n, n, n, 251);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("gemm_i8 n=%d batch=%d: %.3f ms, %.1f TOPS\n", n, batch, ms, 2.0 * n * (double)n * n * batch / ms / 1e9);
  }
  // spot check a few outputs against the host
  std::vector<int8_t> hA(sz), hB(sz); std::vector<uint8_t> hC(sz);
  CK(hipMemcpy(hA.data(), GA, sz, hipMemcpyDeviceToHost)); CK(hipMemcpy(hB.data(), GB, sz, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hC.data(), GC, sz, hipMemcpyDeviceToHost));
  int wrong = 0;
  for (int s = 0; s < 64; ++s) {
    const int i = (s * 977) % n, j = (s * 1223 + 17) % n;
    long long v = 0;
    for (int k = 0; k < n; ++k) v += (int)hA[(size_t)i * n + k] * (int)hB[(size_t)j * n + k];
    const int r = (int)(((v % 251) + 251) % 251);
    wrong += r != hC[(size_t)i * n + j];
  }
  printf("gemm_i8 spot check: %d / 64 wrong\n", wrong);
  return 0;
}
