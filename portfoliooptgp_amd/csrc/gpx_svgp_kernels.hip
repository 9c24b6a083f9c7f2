// gpx_svgp_kernels.hip — device kernels of the SVGP ELBO path that are
// not GEMMs. The M²N work (G = Kmn Kmnᵀ, Y = 2c·P·Kmn) runs on the MFMA GEMM of
// gpx_kernels.hip; what is here is O(MN) element work: kernel-derivative contractions
// (exp-bound, one pass over Y and X), the residual / k_diag sums, split-K reductions and the
// O(M²) elementwise tail. All HBM streams are coalesced along the N (data) axis.
#include <hip/hip_runtime.h>
#include "gpx_internal.h"

namespace gpx {

namespace {

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

constexpr int kRowsPerBlock = 16;   // 4 waves x 4 rows
constexpr int kRowsLds = 4096;      // doubles of column points staged per block

__device__ int theta_slot(const DevSpec* gs, int p) {
  // θ index p -> (term, q) slot t*3+q of the per-term derivative sums, or -1
  for (int t = 0; t < gs->n_terms; ++t) {
    const int o = gs->terms[t].param_offset, kind = gs->terms[t].kind;
    const int np = (kind == GPX_RQ || kind == GPX_PERIODIC_SE) ? 3 : (kind == GPX_LINEAR ? 1 : 2);
    if (p >= o && p < o + np) return t * 3 + (p - o);
  }
  return -1;
}

// Block reduction of the per-lane sums[4][3] into out[16] (θ layout).
template <int NT>
__device__ void reduce_theta(double (&sums)[NT][3], const DevSpec* gs, double* sred, double* out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int t = 0; t < GPX_MAX_TERMS; ++t)
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const double v = t < NT ? wsum(sums[t < NT ? t : 0][q]) : 0.0;
      if (lane == 0) sred[wave * 16 + t * 3 + q] = v;
    }
  __syncthreads();
  if (threadIdx.x < GPX_THETA_STRIDE) {
    const int slot = theta_slot(gs, threadIdx.x);
    out[threadIdx.x] = slot >= 0 ? sred[slot] + sred[16 + slot] + sred[32 + slot] + sred[48 + slot] : 0.0;
  }
}

template <int DM, int NT>
__global__ __launch_bounds__(256) void rows_kernel(RowsArgs a) {
  __shared__ double sx[kRowsLds];
  __shared__ double sz[kRowsPerBlock * GPX_MAX_DIM];
  __shared__ double sth[GPX_THETA_STRIDE];
  __shared__ double sred[64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int D = a.D;
  const int r0 = blockIdx.x * kRowsPerBlock;
  const int c0 = blockIdx.y * a.chunk;
  const int c1 = min(c0 + a.chunk, a.ncols);
  for (int e = tid; e < (c1 - c0) * D; e += 256) sx[e] = a.Xc[(long long)c0 * D + e];
  for (int e = tid; e < kRowsPerBlock * D; e += 256) {
    const int r = r0 + e / D;
    sz[e] = r < a.nrows ? a.Zr[(long long)r0 * D + e] : 0.0;
  }
  if (tid < GPX_THETA_STRIDE) sth[tid] = a.theta[tid];
  __syncthreads();
  const DevSpec spec = *a.spec;
  double sums[NT][3];
#pragma unroll
  for (int t = 0; t < NT; ++t) sums[t][0] = sums[t][1] = sums[t][2] = 0.0;
  for (int rr = 0; rr < 4; ++rr) {
    const int il = wave * 4 + rr;
    const int i = r0 + il;
    if (i >= a.nrows) break;
    const double ui = a.u ? a.u[i] : 0.0;
    double dz[DM];
#pragma unroll
    for (int d = 0; d < DM; ++d) dz[d] = 0.0;
    double wrow = 0.0;
    for (int j = c0 + lane; j < c1; j += 64) {
      const double* xj = sx + (j - c0) * D;
      const double* zi = sz + il * D;
      const double gj = a.g ? a.g[j] : 0.0;
      double kb = ui * gj;
      if (a.Y) {
        const double y = a.Y[(long long)i * a.ldy + j];
        kb += a.sym ? 0.5 * (y + a.Y[(long long)j * a.ldy + i]) : y;
      }
      double dk[NT][3];
      const double kv = eval_k_grad<NT>(spec, sth, zi, xj, dk);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        sums[t][0] = fma(kb, dk[t][0], sums[t][0]);
        sums[t][1] = fma(kb, dk[t][1], sums[t][1]);
        sums[t][2] = fma(kb, dk[t][2], sums[t][2]);
      }
      wrow = fma(kv, gj, wrow);
      double gz[DM];
      eval_k_dx1<DM>(spec, sth, zi, xj, gz);
#pragma unroll
      for (int d = 0; d < DM; ++d) dz[d] = fma(kb, gz[d], dz[d]);
    }
    const long long zo = (long long)blockIdx.y * a.Mp * D + (long long)i * D;
#pragma unroll
    for (int d = 0; d < DM; ++d) {
      const double v = wsum(dz[d]);
      if (lane == 0 && d < D) a.part_z[zo + d] = a.zscale * v;
    }
    if (a.part_w) {
      const double v = wsum(wrow);
      if (lane == 0) a.part_w[(long long)blockIdx.y * a.Mp + i] = v;
    }
  }
  reduce_theta(sums, a.spec, sred,
               a.part_theta + ((long long)blockIdx.y * gridDim.x + blockIdx.x) * GPX_THETA_STRIDE);
}

__global__ __launch_bounds__(256) void resid_kernel(ResidArgs a) {
  __shared__ double sx[256 * GPX_MAX_DIM];
  __shared__ double sth[GPX_THETA_STRIDE];
  __shared__ double sred[4 * kResidW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j0 = blockIdx.x * 256, D = a.D;
  for (int e = tid; e < 256 * D; e += 256) {
    const int j = j0 + e / D;
    sx[e] = j < a.n ? a.X[(long long)j0 * D + e] : 0.0;
  }
  if (tid < GPX_THETA_STRIDE) sth[tid] = a.theta[tid];
  __syncthreads();
  const DevSpec spec = *a.spec;
  const double s2 = sth[spec.n_params];
  const double c = -0.5 * a.scale / s2;
  const int j = j0 + tid;
  double sums[GPX_MAX_TERMS][3];
#pragma unroll
  for (int t = 0; t < GPX_MAX_TERMS; ++t) sums[t][0] = sums[t][1] = sums[t][2] = 0.0;
  double sq = 0.0, kd = 0.0;
  if (j < a.n) {
    const double r = a.Y[j] - a.mu[j];
    a.g[j] = a.scale * r / s2;
    sq = r * r;
    double dk[GPX_MAX_TERMS][3];
    kd = eval_k_grad<GPX_MAX_TERMS>(spec, sth, sx + tid * D, sx + tid * D, dk);
#pragma unroll
    for (int t = 0; t < GPX_MAX_TERMS; ++t) {
      sums[t][0] = c * dk[t][0]; sums[t][1] = c * dk[t][1]; sums[t][2] = c * dk[t][2];
    }
  } else if (j < a.npad) {
    a.g[j] = 0.0;
  }
  double* out = a.part + (long long)blockIdx.x * kResidW;
  const double vsq = wsum(sq), vkd = wsum(kd);
  if (lane == 0) { sred[wave * 2] = vsq; sred[wave * 2 + 1] = vkd; }
  __syncthreads();
  double s_sq = 0.0, s_kd = 0.0;
  if (tid == 0) {
    for (int w = 0; w < 4; ++w) { s_sq += sred[w * 2]; s_kd += sred[w * 2 + 1]; }
  }
  __syncthreads();
  reduce_theta(sums, a.spec, sred, out);
  if (tid == 0) { out[16] = s_sq; out[17] = s_kd; out[18] = 0.0; out[19] = 0.0; }
}

// wide outputs: one thread per column, the nb rows unrolled by 4 (independent loads in flight)
__global__ __launch_bounds__(256) void sum_kernel(SumArgs a) {
  const long long c = (long long)blockIdx.x * 256 + threadIdx.x;
  if (c >= a.width) return;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  int b = 0;
  for (; b + 4 <= a.nb; b += 4) {
    s0 += a.src[(long long)b * a.stride + c];
    s1 += a.src[(long long)(b + 1) * a.stride + c];
    s2 += a.src[(long long)(b + 2) * a.stride + c];
    s3 += a.src[(long long)(b + 3) * a.stride + c];
  }
  for (; b < a.nb; ++b) s0 += a.src[(long long)b * a.stride + c];
  const double s = (s0 + s1) + (s2 + s3);
  a.dst[c] = a.accumulate ? a.dst[c] + s : s;
}

// narrow outputs over many rows (θ partials of thousands of blocks): one block per column,
// the rows strided over the block, fixed-order tree reduction
__global__ __launch_bounds__(256) void sum_narrow_kernel(SumArgs a) {
  __shared__ double sred[4];
  const long long c = blockIdx.x;
  double s = 0.0;
  for (int b = threadIdx.x; b < a.nb; b += 256) s += a.src[(long long)b * a.stride + c];
  s = wsum(s);
  if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double t = (sred[0] + sred[1]) + (sred[2] + sred[3]);
    a.dst[c] = a.accumulate ? a.dst[c] + t : t;
  }
}

__global__ __launch_bounds__(256) void svgp_final_kernel(SvgpFinalArgs a) {
  __shared__ double sred[4];
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  const int i = (int)(e / a.m), j = (int)(e - (long long)(e / a.m) * a.m);
  double tr = 0.0;
  if (i < a.m) {
    const long long o = (long long)i * a.ld + j;
    tr = a.Sm1[o] * a.Gh[o];
    if (j <= i) {
      const double F = -(a.q[i] * a.ahat[j] + a.c2 * a.X1[o]);
      a.Phi[o] = (i == j) ? 0.5 * F : F;
      a.Rbar[o] = a.c2 * a.GR[o] - a.R[o] + ((i == j) ? 1.0 / a.R[o] : 0.0);
    } else {
      a.Phi[o] = 0.0;
      a.Rbar[o] = 0.0;
    }
  }
  const double v = wsum(tr);
  if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) a.part_tr[blockIdx.x] = sred[0] + sred[1] + sred[2] + sred[3];
}

__global__ void diag_add_kernel(double* A, int ld, int n, double v) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) A[(long long)i * ld + i] += v;
}

__global__ void symmetrize_kernel(double* A, int ld, int n) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  const int i = (int)(e / n), j = (int)(e - (long long)(e / n) * n);
  if (i < n && j > i) A[(long long)i * ld + j] = A[(long long)j * ld + i];
}

__global__ __launch_bounds__(256) void svgp_predvar_kernel(SvgpPredVarArgs a) {
  __shared__ double sx[256 * GPX_MAX_DIM];
  __shared__ double sth[GPX_THETA_STRIDE];
  const int tid = threadIdx.x, j0 = blockIdx.x * 256, D = a.D;
  for (int e = tid; e < 256 * D; e += 256) {
    const int j = j0 + e / D;
    sx[e] = j < a.M ? a.Xnew[(long long)j0 * D + e] : 0.0;
  }
  if (tid < GPX_THETA_STRIDE) sth[tid] = a.theta[tid];
  __syncthreads();
  const int j = j0 + tid;
  if (j >= a.M) return;
  const DevSpec spec = *a.spec;
  double v = eval_kdiag(spec, sth, sx + tid * D);
  for (int r = 0; r < a.nrt; ++r) v += a.pB[(long long)r * a.ldp + j] - a.pA[(long long)r * a.ldp + j];
  if (a.add_noise) v += sth[spec.n_params];
  a.var[j] = v;
}

}  // namespace

int rows_chunk_for(int D) {
  const int dm = D <= 1 ? 1 : D <= 2 ? 2 : D <= 4 ? 4 : D <= 8 ? 8 : 16;
  return std::min(1024, (kRowsLds / dm) / 64 * 64);
}

int rows_blocks(const RowsArgs& a) {
  return ((a.nrows + kRowsPerBlock - 1) / kRowsPerBlock) * rows_chunks(a);
}

int rows_chunks(const RowsArgs& a) { return (a.ncols + a.chunk - 1) / a.chunk; }

template <int NT>
static void launch_rows_nt(const RowsArgs& a, hipStream_t s) {
  dim3 grid((a.nrows + kRowsPerBlock - 1) / kRowsPerBlock, rows_chunks(a));
  if (a.D <= 1) hipLaunchKernelGGL((rows_kernel<1, NT>), grid, dim3(256), 0, s, a);
  else if (a.D <= 2) hipLaunchKernelGGL((rows_kernel<2, NT>), grid, dim3(256), 0, s, a);
  else if (a.D <= 4) hipLaunchKernelGGL((rows_kernel<4, NT>), grid, dim3(256), 0, s, a);
  else if (a.D <= 8) hipLaunchKernelGGL((rows_kernel<8, NT>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((rows_kernel<16, NT>), grid, dim3(256), 0, s, a);
}

// single-term kernels (the common case) use the 1-term derivative path: a quarter of the
// derivative registers
void launch_rows(const RowsArgs& a, bool single_term, hipStream_t s) {
  if (single_term) launch_rows_nt<1>(a, s);
  else launch_rows_nt<GPX_MAX_TERMS>(a, s);
}

int resid_blocks(int npad) { return (npad + 255) / 256; }

void launch_resid(const ResidArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(resid_kernel, dim3(resid_blocks(a.npad)), dim3(256), 0, s, a);
}

void launch_sum(const SumArgs& a, hipStream_t s) {
  if (a.width <= 64 && a.nb > 64)
    hipLaunchKernelGGL(sum_narrow_kernel, dim3((unsigned)a.width), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(sum_kernel, dim3((unsigned)((a.width + 255) / 256)), dim3(256), 0, s, a);
}

int svgp_final_blocks(int m) { return (int)(((long long)m * m + 255) / 256); }

void launch_svgp_final(const SvgpFinalArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(svgp_final_kernel, dim3(svgp_final_blocks(a.m)), dim3(256), 0, s, a);
}

void launch_diag_add(double* A, int ld, int n, double v, hipStream_t s) {
  hipLaunchKernelGGL(diag_add_kernel, dim3((n + 255) / 256), dim3(256), 0, s, A, ld, n, v);
}

void launch_symmetrize_lower(double* A, int ld, int n, hipStream_t s) {
  hipLaunchKernelGGL(symmetrize_kernel, dim3((unsigned)(((long long)n * n + 255) / 256)), dim3(256), 0,
                     s, A, ld, n);
}

void launch_svgp_predvar(const SvgpPredVarArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(svgp_predvar_kernel, dim3((a.M + 255) / 256), dim3(256), 0, s, a);
}

}  // namespace gpx
