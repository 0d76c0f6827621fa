// dense_llt.hip -- dense Cholesky of the reduced (tag + camera) system on
// gfx950, replacing the Eigen::LLT that Ceres' DenseSchurComplementSolver
// runs on one CPU thread.
//
// Right-looking tiled factorization, 64x64 fp64 tiles, lower triangle of a
// row-major matrix:
//   for k:  POTRF(k,k)            one workgroup, tile in LDS
//           TRSM (i,k), i > k     one workgroup per tile
//           UPDATE (i,j), k<j<=i  A_ij -= L_ik L_jk^T on MFMA
//                                 (v_mfma_f64_16x16x4_f64, 4 waves x 32x32)
// The right-hand side rides along as row nF of the matrix (inside the padded
// last tile row), so the forward substitution L z = b falls out of the
// factorization; the backward solve L^T y = z is one launch per tile row.
//
// tile_nz (optional, T*T bytes) marks structurally non-zero tiles of L; a
// tile whose L_ik or L_jk factor is structurally zero contributes exactly 0
// to an update, so skipping it is bit-identical to the dense factorization.
#include "lm_internal.h"

#include <cmath>

namespace arslam {

namespace {

typedef double dbl4 __attribute__((ext_vector_type(4)));
typedef double dbl2 __attribute__((ext_vector_type(2)));

constexpr int T64 = kTile;
constexpr int LP = 65;   // LDS row pitch for the POTRF/TRSM tiles
constexpr int LM = 66;   // LDS row pitch for MFMA operand tiles (conflict-free ds_read_b64)

__device__ __forceinline__ bool tile_live(const uint8_t *nz, int T, int i, int j) {
  return nz == nullptr || nz[(long)i * T + j] != 0;
}

__global__ __launch_bounds__(256) void k_potrf(double *__restrict__ S, long lda, int k,
                                               int *__restrict__ flag) {
  __shared__ double A[T64][LP];
  if (*flag) return;
  const int tid = threadIdx.x;
  double *base = S + (long)k * T64 * lda + (long)k * T64;
  for (int e = tid; e < T64 * T64; e += 256) {
    const int r = e >> 6, c = e & 63;
    if (c <= r) A[r][c] = base[(long)r * lda + c];
  }
  __syncthreads();
  const int i = tid >> 2, cg = tid & 3;
  for (int j = 0; j < T64; ++j) {
    const double ajj = A[j][j];
    if (!(ajj > 0.0)) {
      if (tid == 0) atomicCAS(flag, 0, 1 + k * T64 + j);
      return;
    }
    const double inv = 1.0 / ajj;
    if (i > j) {
      const double aij = A[i][j] * inv;
      int c = j + 1 + ((cg - (j + 1)) & 3);
      for (; c <= i; c += 4) A[i][c] -= aij * A[c][j];
    }
    __syncthreads();
  }
  // L_ic = A_ic / sqrt(A_cc), L_ii = sqrt(A_ii)
  for (int c = cg; c <= i; c += 4) {
    const double d = sqrt(A[c][c]);
    base[(long)i * lda + c] = (c == i) ? d : A[i][c] / d;
  }
}

__global__ __launch_bounds__(256) void k_trsm(double *__restrict__ S, long lda, int k, int T,
                                              const uint8_t *__restrict__ nz,
                                              const int *__restrict__ flag) {
  __shared__ double Lk[T64][LP];
  __shared__ double X[T64][LP];
  if (*flag) return;
  const int ti = k + 1 + blockIdx.x;
  if (!tile_live(nz, T, ti, k)) return;
  const int tid = threadIdx.x;
  const double *lk = S + (long)k * T64 * lda + (long)k * T64;
  double *xt = S + (long)ti * T64 * lda + (long)k * T64;
  for (int e = tid; e < T64 * T64; e += 256) {
    const int r = e >> 6, c = e & 63;
    if (c <= r) Lk[r][c] = lk[(long)r * lda + c];
    X[r][c] = xt[(long)r * lda + c];
  }
  __syncthreads();
  // X L^T = A, column by column: x_rj = a_rj / L_jj ; a_rc -= x_rj L_cj (c > j)
  const int r = tid >> 2, cg = tid & 3;
  for (int j = 0; j < T64; ++j) {
    const double xrj = X[r][j] / Lk[j][j];
    int c = j + 1 + ((cg - (j + 1)) & 3);
    for (; c < T64; c += 4) X[r][c] -= xrj * Lk[c][j];
    __syncthreads();
  }
  for (int c = cg; c < T64; c += 4) xt[(long)r * lda + c] = X[r][c] / Lk[c][c];
}

// A_ij -= L_ik L_jk^T for every live tile pair k < j <= i < T.
__global__ __launch_bounds__(256) void k_update(double *__restrict__ S, long lda, int k, int T,
                                                const uint8_t *__restrict__ nz,
                                                const int *__restrict__ flag) {
  __shared__ __attribute__((aligned(16))) double sA[T64 * LM];
  __shared__ __attribute__((aligned(16))) double sB[T64 * LM];
  if (*flag) return;
  const long b = blockIdx.x;
  int ip = (int)((sqrt(8.0 * (double)b + 1.0) - 1.0) * 0.5);
  while ((long)ip * (ip + 1) / 2 > b) --ip;
  while ((long)(ip + 1) * (ip + 2) / 2 <= b) ++ip;
  const int jp = (int)(b - (long)ip * (ip + 1) / 2);
  const int ti = k + 1 + ip, tj = k + 1 + jp;
  if (!tile_live(nz, T, ti, k) || !tile_live(nz, T, tj, k)) return;
  const int tid = threadIdx.x;
  const double *Ai = S + (long)ti * T64 * lda + (long)k * T64;
  const double *Bj = S + (long)tj * T64 * lda + (long)k * T64;
  for (int e = tid; e < T64 * 32; e += 256) {
    const int r = e >> 5, c2 = (e & 31) * 2;
    const dbl2 va = *reinterpret_cast<const dbl2 *>(Ai + (long)r * lda + c2);
    const dbl2 vb = *reinterpret_cast<const dbl2 *>(Bj + (long)r * lda + c2);
    *reinterpret_cast<dbl2 *>(&sA[r * LM + c2]) = va;
    *reinterpret_cast<dbl2 *>(&sB[r * LM + c2]) = vb;
  }
  __syncthreads();
  const int w = tid >> 6, lane = tid & 63;
  const int r0 = (w >> 1) * 32, c0 = (w & 1) * 32;
  const int li = lane & 15, lk = lane >> 4;
  dbl4 acc00 = {0, 0, 0, 0}, acc01 = {0, 0, 0, 0}, acc10 = {0, 0, 0, 0}, acc11 = {0, 0, 0, 0};
#pragma unroll 4
  for (int kk = 0; kk < T64 / 4; ++kk) {
    const int kc = kk * 4 + lk;
    const double a0 = sA[(r0 + li) * LM + kc];
    const double a1 = sA[(r0 + 16 + li) * LM + kc];
    const double b0 = sB[(c0 + li) * LM + kc];
    const double b1 = sB[(c0 + 16 + li) * LM + kc];
    acc00 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc00, 0, 0, 0);
    acc01 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc01, 0, 0, 0);
    acc10 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc10, 0, 0, 0);
    acc11 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc11, 0, 0, 0);
  }
  // f64 MFMA C/D layout: col = lane & 15, row = (lane >> 4) + 4 * reg
  double *C = S + (long)ti * T64 * lda + (long)tj * T64;
  const dbl4 accs[4] = {acc00, acc01, acc10, acc11};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int rb = r0 + (q >> 1) * 16, cb = c0 + (q & 1) * 16;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int row = rb + lk + 4 * reg, col = cb + li;
      C[(long)row * lda + col] -= accs[q][reg];
    }
  }
}

// z[j] = S[nF][j] (the forward-substituted right-hand side)
__global__ void k_init_z(const double *__restrict__ S, long lda, long nF, long N,
                         double *__restrict__ z) {
  const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < N) z[j] = j < nF ? S[nF * lda + j] : 0.0;
}

// One tile row of L^T y = z: solve the 64x64 diagonal block (every workgroup,
// redundantly), then z_j -= L_kj^T y_k over this workgroup's columns j < 64k.
__global__ __launch_bounds__(256) void k_back_solve(const double *__restrict__ S, long lda, long nF,
                                                    int k, int T, const uint8_t *__restrict__ nz,
                                                    double *__restrict__ z, double *__restrict__ yF,
                                                    const int *__restrict__ flag) {
  __shared__ double Lk[T64][LP];
  __shared__ double y[T64];
  if (*flag) return;
  const int tid = threadIdx.x;
  const long row0 = (long)k * T64;
  const double *lk = S + row0 * lda + row0;
  for (int e = tid; e < T64 * T64; e += 256) {
    const int r = e >> 6, c = e & 63;
    if (c <= r) Lk[r][c] = lk[(long)r * lda + c];
  }
  __syncthreads();
  if (tid < 64) {
    double zr = (row0 + tid < nF) ? z[row0 + tid] : 0.0;
    double yv_own = 0.0;
    for (int rr = T64 - 1; rr >= 0; --rr) {
      double yv = __shfl(zr / Lk[rr][rr], rr, 64);
      if (row0 + rr >= nF) yv = 0.0;
      if (tid == rr) yv_own = yv;
      if (tid < rr) zr -= Lk[rr][tid] * yv;
    }
    y[tid] = yv_own;
    if (blockIdx.x == 0 && row0 + tid < nF) yF[row0 + tid] = yv_own;
  }
  __syncthreads();
  const long j = (long)blockIdx.x * 256 + tid;
  if (j < row0) {
    const int tj = (int)(j / T64);
    if (!tile_live(nz, T, k, tj)) return;
    double s = 0.0;
#pragma unroll 8
    for (int r = 0; r < T64; ++r) s += S[(row0 + r) * lda + j] * y[r];
    z[j] -= s;
  }
}

__global__ void k_zero_tiles(double *__restrict__ S, long lda, int T, const uint8_t *__restrict__ nz) {
  const long b = blockIdx.x;
  int ip = (int)((sqrt(8.0 * (double)b + 1.0) - 1.0) * 0.5);
  while ((long)ip * (ip + 1) / 2 > b) --ip;
  while ((long)(ip + 1) * (ip + 2) / 2 <= b) ++ip;
  const int jp = (int)(b - (long)ip * (ip + 1) / 2);
  if (!tile_live(nz, T, ip, jp) && ip != jp) return;
  double *t = S + (long)ip * T64 * lda + (long)jp * T64;
  for (int e = threadIdx.x; e < T64 * 32; e += blockDim.x) {
    const int r = e >> 5, c2 = (e & 31) * 2;
    *reinterpret_cast<dbl2 *>(t + (long)r * lda + c2) = dbl2{0.0, 0.0};
  }
}

}  // namespace

void launch_zero_lower(double *S, long N, long lda, const uint8_t *tile_nz, hipStream_t s) {
  const int T = (int)(N / T64);
  const long ntiles = (long)T * (T + 1) / 2;
  hipLaunchKernelGGL(k_zero_tiles, dim3((unsigned)ntiles), dim3(256), 0, s, S, lda, T, tile_nz);
}

void launch_dense_llt(double *S, long N, long lda, int *flag, const uint8_t *tile_nz, hipStream_t s,
                      LaunchTiming *timing) {
  const int T = (int)(N / T64);
  for (int k = 0; k < T; ++k) {
    hipLaunchKernelGGL(k_potrf, dim3(1), dim3(256), 0, s, S, lda, k, flag);
    const int m = T - k - 1;
    if (m == 0) break;
    hipLaunchKernelGGL(k_trsm, dim3(m), dim3(256), 0, s, S, lda, k, T, tile_nz, flag);
    const long nt = (long)m * (m + 1) / 2;
    const bool rec = timing && timing->used < timing->cap;
    if (rec) (void)hipEventRecord(timing->ev[2 * timing->used], s);
    hipLaunchKernelGGL(k_update, dim3((unsigned)nt), dim3(256), 0, s, S, lda, k, T, tile_nz, flag);
    if (rec) {
      (void)hipEventRecord(timing->ev[2 * timing->used + 1], s);
      timing->used++;
      // useful flops: off-diagonal tiles 2*64^3, diagonal tiles (lower incl. diagonal) 64*65*64
      timing->flops += 2.0 * T64 * T64 * T64 * ((double)m * (m - 1) / 2) + (double)T64 * (T64 + 1) * T64 * m;
    }
  }
}

void launch_dense_back_solve(const double *S, long N, long lda, long nF, double *z, double *yF,
                             const int *flag, const uint8_t *tile_nz, hipStream_t s) {
  const int T = (int)(N / T64);
  hipLaunchKernelGGL(k_init_z, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, S, lda, nF, N, z);
  for (int k = T - 1; k >= 0; --k) {
    const long cols = (long)k * T64;
    const unsigned grid = (unsigned)((cols + 255) / 256 > 0 ? (cols + 255) / 256 : 1);
    hipLaunchKernelGGL(k_back_solve, dim3(grid), dim3(256), 0, s, S, lda, nF, k, T, tile_nz, z, yF, flag);
  }
}

}  // namespace arslam
