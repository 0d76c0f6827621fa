// dense_llt.hip -- Cholesky of the reduced (tag + camera) system on gfx950,
// replacing the Eigen::LLT that Ceres' DenseSchurComplementSolver runs on one
// CPU thread.
//
// Storage: dense row-major N x N (lower triangle used), 64 x 64 fp64 tiles.
// Right-looking tiled factorization driven by a tile plan (LltPlan):
//   for k:  POTRF(k,k)            one wavefront, lane r owns row r in VGPRs
//           TRSM (i,k)            one wavefront per tile, rows in VGPRs,
//                                 L_kk^T in LDS (broadcast reads)
//           UPDATE (i,j)          A_ij -= L_ik L_jk^T on MFMA
//                                 (v_mfma_f64_16x16x4_f64, 4 waves x 32x32)
// The plan lists, per step k, the tiles the step touches.  A dense plan lists
// every lower tile; a sparse plan lists only the tiles of the symbolic
// Cholesky fill of the reduced system (tile level), so a structurally zero
// tile is never read or written.  A skipped update would have added exactly
// 0 (products with an all-zero tile), so the sparse plan computes the same
// factor as the dense plan on the same ordering.
//
// The right-hand side rides along as row nF of the matrix (inside the padded
// last tile row), so the forward substitution L z = b falls out of the
// factorization; the backward solve L^T y = z is one launch per tile row.
#include "lm_internal.h"

#include <cmath>
#include <cstdlib>

namespace arslam {

namespace {

typedef double dbl4 __attribute__((ext_vector_type(4)));
typedef double dbl2 __attribute__((ext_vector_type(2)));

constexpr int T64 = kTile;
constexpr int LP = 65;   // LDS row pitch (doubles) for row-per-lane tiles
constexpr int LM = 66;   // LDS row pitch for MFMA operand tiles (conflict-free ds_read_b64)

// Load a 64x64 tile (row-major, lda) into LDS with pitch LP using 64 lanes:
// 32 independent 16-byte loads per lane are issued before any LDS store.
__device__ __forceinline__ void load_tile64(const double *__restrict__ g, long lda, double *lds,
                                            int lane) {
  dbl2 v[32];
#pragma unroll
  for (int q = 0; q < 32; ++q) {
    const int e = q * 64 + lane, r = e >> 5, c2 = (e & 31) * 2;
    v[q] = *reinterpret_cast<const dbl2 *>(g + (long)r * lda + c2);
  }
#pragma unroll
  for (int q = 0; q < 32; ++q) {
    const int e = q * 64 + lane, r = e >> 5, c2 = (e & 31) * 2;
    lds[r * LP + c2] = v[q].x;
    lds[r * LP + c2 + 1] = v[q].y;
  }
}

// Store a 64x64 LDS tile (pitch LP) to global memory with 16-byte stores.
__device__ __forceinline__ void store_tile64(double *__restrict__ g, long lda, const double *lds,
                                             int lane) {
#pragma unroll
  for (int q = 0; q < 32; ++q) {
    const int e = q * 64 + lane, r = e >> 5, c2 = (e & 31) * 2;
    *reinterpret_cast<dbl2 *>(g + (long)r * lda + c2) = dbl2{lds[r * LP + c2], lds[r * LP + c2 + 1]};
  }
}

constexpr int LQ = 66;   // LDS pitch of the blocked panel kernel (16-lane row access and MFMA
                         // fragment reads both conflict-free)

// 256-thread load of a 64x64 tile into LDS (pitch LQ), all loads in flight.
__device__ __forceinline__ void load_tile_wg(const double *__restrict__ g, long lda, double *lds,
                                             int tid) {
  dbl2 v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = q * 256 + tid, r = e >> 5, c2 = (e & 31) * 2;
    v[q] = *reinterpret_cast<const dbl2 *>(g + (long)r * lda + c2);
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = q * 256 + tid, r = e >> 5, c2 = (e & 31) * 2;
    *reinterpret_cast<dbl2 *>(lds + r * LQ + c2) = v[q];
  }
}

// 256-thread store of the lower triangle (zeros above) of an LDS tile.
__device__ __forceinline__ void store_tile_wg(double *__restrict__ g, long lda, const double *lds,
                                              int tid, bool lower_only) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = q * 256 + tid, r = e >> 5, c2 = (e & 31) * 2;
    dbl2 v = *reinterpret_cast<const dbl2 *>(lds + r * LQ + c2);
    if (lower_only) {
      if (c2 > r) v.x = 0.0;
      if (c2 + 1 > r) v.y = 0.0;
    }
    *reinterpret_cast<dbl2 *>(g + (long)r * lda + c2) = v;
  }
}

__device__ __forceinline__ double readlane_d(double v, int l) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, l);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), l);
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// One wave: C(16x16) -= A(16 x K) B(16 x K)^T, operands in LDS (pitch LQ).
__device__ __forceinline__ void wave_gemm16_sub(double *C, const double *A, const double *B, int K,
                                                int lane) {
  const int li = lane & 15, lk = lane >> 4;
  dbl4 acc = {0, 0, 0, 0};
  for (int k4 = 0; k4 < K; k4 += 4) {
    const double a = A[li * LQ + k4 + lk];
    const double b = B[li * LQ + k4 + lk];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) C[(lk + 4 * reg) * LQ + li] -= acc[reg];
}

// In-LDS blocked Cholesky of the 64x64 tile D (256 threads).  Sub-panels of
// 16 columns: unblocked 16x16 factor (16 lanes of wave 0), row solve of the
// panel below (16 lanes per wave), MFMA rank-16 update of the trailing tile.
// Returns false (uniformly) if a pivot is not positive; inv[c] = 1 / L_cc.
template <int AB>
__device__ bool blocked_potrf64(double *D, double *inv, double *LTd, int *bad, int tid) {
  const int w = tid >> 6, lane = tid & 63;
  if (tid == 0) *bad = 0;
  __syncthreads();
  for (int p = 0; p < 4; ++p) {
    const int b0 = 16 * p;
    if (w == 0 && !(AB & 1)) {
      // 16x16 diagonal block, lane i < 16 owns row b0+i in registers.  LDL^T
      // form: a_ic -= (a_ij / a_jj) a_cj, so only a reciprocal sits on the
      // pivot chain (the square roots are taken once at the end); the pivot
      // is broadcast with v_readlane, the column through LDS.
      double x[16];
      double *cb = LTd;   // scratch column buffer (16 doubles)
      const int li = lane & 15;
      const int i = b0 + li;
#pragma unroll
      for (int c = 0; c < 16; ++c) x[c] = D[i * LQ + b0 + c];
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) {
        if (lane < 16) cb[lane] = x[jj];
        const double ajj = readlane_d(x[jj], jj);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        double r = __builtin_amdgcn_rcp(ajj);
        r = r * (2.0 - ajj * r);                    // Newton refinement of v_rcp_f64
        r = r * (2.0 - ajj * r);
        const double f = (lane > jj) ? x[jj] * r : 0.0;
#pragma unroll
        for (int c = jj + 1; c < 16; ++c) x[c] -= f * cb[c];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      // pivots are x_i[i]; L_ic = x_i[c] / sqrt(piv_c), L_ii = sqrt(piv_i)
      double piv = 0.0;
#pragma unroll
      for (int c = 0; c < 16; ++c) piv = (c == li) ? x[c] : piv;
      if (!(piv > 0.0) && lane < 16) *bad = 1;
      const double d = sqrt(piv), rd = 1.0 / d;
      if (lane < 16) { cb[16 + lane] = rd; inv[i] = rd; }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (lane < 16) {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          const double l = (c < li) ? x[c] * cb[16 + c] : (c == li ? d : 0.0);
          D[i * LQ + b0 + c] = l;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // transposed copy of the diagonal block for the row solves: LTd[p][j][c] = L[b0+c][b0+j]
      if (lane < 16) {
#pragma unroll
        for (int c = 0; c < 16; ++c) LTd[32 + p * 256 + lane * 16 + c] = D[(b0 + c) * LQ + b0 + lane];
      }
    }
    __syncthreads();
    // rows below the diagonal block: X L_pp^T = A_panel
    {
      const int i = b0 + 16 + w * 16 + lane;
      if (lane < 16 && i < 64 && !(AB & 2)) {
        double x[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) x[c] = D[i * LQ + b0 + c];
        const double *lt = LTd + 32 + p * 256;
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) {
          x[jj] *= inv[b0 + jj];
#pragma unroll
          for (int c = jj + 1; c < 16; ++c) x[c] -= x[jj] * lt[jj * 16 + c];
        }
#pragma unroll
        for (int c = 0; c < 16; ++c) D[i * LQ + b0 + c] = x[c];
      }
    }
    __syncthreads();
    // trailing update of blocks p+1..3 (lower tiles I >= C) with the panel
    const int m = 3 - p;
    const int ntl = (AB & 4) ? 0 : m * (m + 1) / 2;
    for (int t = w; t < ntl; t += 4) {
      int I = 0;
      while ((I + 1) * (I + 2) / 2 <= t) ++I;
      const int C = t - I * (I + 1) / 2;
      const int bi = 16 * (p + 1 + I), bc = 16 * (p + 1 + C);
      wave_gemm16_sub(D + bi * LQ + bc, D + bi * LQ + b0, D + bc * LQ + b0, 16, lane);
    }
    __syncthreads();
  }
  return *bad == 0;
}

// In-LDS blocked solve X L^T = A for a 64x64 tile X (256 threads), L from
// blocked_potrf64 (lower part of D, inv = 1 / diag).
template <int AB>
__device__ void blocked_trsm64(double *X, const double *D, const double *inv, const double *LTd,
                               int tid) {
  const int w = tid >> 6, lane = tid & 63;
  for (int p = 0; p < 4; ++p) {
    const int b0 = 16 * p;
    if (p > 0 && !(AB & 8))   // X[:, b0:b0+16] -= X[:, 0:b0] L[b0:b0+16, 0:b0]^T  (wave w: rows 16w..)
      wave_gemm16_sub(X + 16 * w * LQ + b0, X + 16 * w * LQ, D + b0 * LQ, b0, lane);
    __syncthreads();
    if (lane < 16 && !(AB & 16)) {
      const int r = 16 * w + lane;
      double x[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) x[c] = X[r * LQ + b0 + c];
      const double *lt = LTd + 32 + p * 256;
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) {
        x[jj] *= inv[b0 + jj];
#pragma unroll
        for (int c = jj + 1; c < 16; ++c) x[c] -= x[jj] * lt[jj * 16 + c];
      }
#pragma unroll
      for (int c = 0; c < 16; ++c) X[r * LQ + b0 + c] = x[c];
    }
    __syncthreads();
  }
}

// Panel of step k: workgroup 0 factors the diagonal tile (k,k) and stores
// L_kk; workgroup b > 0 factors it redundantly (no extra launch on the
// critical path) and solves tile (rows[b-1], k).
template <int AB>
__global__ __launch_bounds__(256) void k_panel(double *__restrict__ S, long lda, int k,
                                               const int *__restrict__ rows,
                                               int *__restrict__ flag) {
  __shared__ __attribute__((aligned(16))) double D[T64 * LQ];
  __shared__ __attribute__((aligned(16))) double X[T64 * LQ];
  __shared__ double inv[T64];
  __shared__ __attribute__((aligned(16))) double LTd[32 + 4 * 256];   // column scratch + transposed diagonal blocks
  __shared__ int bad;
  if (*flag) return;
  const int tid = threadIdx.x, b = blockIdx.x;
  const double *dk = S + (long)k * T64 * lda + (long)k * T64;
  double *xt = b > 0 ? S + (long)rows[b - 1] * T64 * lda + (long)k * T64 : nullptr;
  load_tile_wg(dk, lda, D, tid);
  if (b > 0) load_tile_wg(xt, lda, X, tid);
  __syncthreads();
  const bool ok = blocked_potrf64<AB>(D, inv, LTd, &bad, tid) || AB != 0;
  if (!ok) {
    if (b == 0 && tid == 0) {
      int first = 0;
      while (first < T64 && D[first * LQ + first] > 0.0) ++first;
      atomicCAS(flag, 0, 1 + k * T64 + first);
    }
    return;
  }
  if (b == 0) {
    store_tile_wg(const_cast<double *>(dk), lda, D, tid, true);
    return;
  }
  blocked_trsm64<AB>(X, D, inv, LTd, tid);
  store_tile_wg(xt, lda, X, tid, false);
}

// A_ij -= L_ik L_jk^T for the (i,j) tile pairs listed for step k.
__global__ __launch_bounds__(256) void k_update(double *__restrict__ S, long lda, int k,
                                                const int2 *__restrict__ pairs,
                                                const int *__restrict__ flag) {
  __shared__ __attribute__((aligned(16))) double sA[T64 * LM];
  __shared__ __attribute__((aligned(16))) double sB[T64 * LM];
  if (*flag) return;
  const int2 pr = pairs[blockIdx.x];
  const int ti = pr.x, tj = pr.y;
  const int tid = threadIdx.x;
  const double *Ai = S + (long)ti * T64 * lda + (long)k * T64;
  const double *Bj = S + (long)tj * T64 * lda + (long)k * T64;
  {
    dbl2 va[8], vb[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = q * 256 + tid, r = e >> 5, c2 = (e & 31) * 2;
      va[q] = *reinterpret_cast<const dbl2 *>(Ai + (long)r * lda + c2);
      vb[q] = *reinterpret_cast<const dbl2 *>(Bj + (long)r * lda + c2);
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int e = q * 256 + tid, r = e >> 5, c2 = (e & 31) * 2;
      *reinterpret_cast<dbl2 *>(&sA[r * LM + c2]) = va[q];
      *reinterpret_cast<dbl2 *>(&sB[r * LM + c2]) = vb[q];
    }
  }
  __syncthreads();
  const int w = tid >> 6, lane = tid & 63;
  const int r0 = (w >> 1) * 32, c0 = (w & 1) * 32;
  const int li = lane & 15, lk = lane >> 4;
  double *C = S + (long)ti * T64 * lda + (long)tj * T64;
  double cval[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int rb = r0 + (q >> 1) * 16, cb = c0 + (q & 1) * 16;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) cval[4 * q + reg] = C[(long)(rb + lk + 4 * reg) * lda + cb + li];
  }
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
  const dbl4 accs[4] = {acc00, acc01, acc10, acc11};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int rb = r0 + (q >> 1) * 16, cb = c0 + (q & 1) * 16;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int row = rb + lk + 4 * reg, col = cb + li;
      C[(long)row * lda + col] = cval[4 * q + reg] - accs[q][reg];
    }
  }
}

// z[j] = S[nF][j] (the forward-substituted right-hand side)
__global__ void k_init_z(const double *__restrict__ S, long lda, long nF, long N,
                         double *__restrict__ z) {
  const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (j < N) z[j] = j < nF ? S[nF * lda + j] : 0.0;
}

// One tile row k of L^T y = z.  Every workgroup solves the 64x64 diagonal
// block (redundantly; lane r owns z_r, blocked by 16 with scalar broadcasts),
// then z_j -= L_kj^T y_k over its listed tile column.  Workgroup 0 writes y_k.
__global__ __launch_bounds__(64) void k_back_solve(const double *__restrict__ S, long lda, long nF,
                                                   int k, const int *__restrict__ cols,
                                                   double *__restrict__ z, double *__restrict__ yF,
                                                   const int *__restrict__ flag) {
  __shared__ double Lk[T64 * LP];
  __shared__ double y[T64];
  if (*flag) return;
  const int lane = threadIdx.x;
  const long row0 = (long)k * T64;
  const double *lk = S + row0 * lda + row0;
  double zr = (row0 + lane < nF) ? z[row0 + lane] : 0.0;
  load_tile64(lk, lda, Lk, lane);
  __syncthreads();
  const double my_inv = (row0 + lane < nF) ? 1.0 / Lk[lane * LP + lane] : 0.0;   // y = 0 past nF
  double yv_own = 0.0;
  for (int p = 3; p >= 0; --p) {
    const int b0 = 16 * p;
    // 16x16 diagonal block: sequential over rows, scalar broadcast of y
    for (int rr = 15; rr >= 0; --rr) {
      const int r = b0 + rr;
      const double yv = readlane_d(zr * my_inv, r);
      if (lane == r) yv_own = yv;
      if (lane >= b0 && lane < r) zr -= Lk[r * LP + lane] * yv;
    }
    y[lane] = yv_own;
    __syncthreads();
    // rows above the block: z_i -= sum_r L[b0+r][i] y[b0+r]
    if (lane < b0) {
      double acc = 0.0;
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) acc += Lk[(b0 + rr) * LP + lane] * y[b0 + rr];
      zr -= acc;
    }
    __syncthreads();
  }
  y[lane] = yv_own;
  __syncthreads();
  if (blockIdx.x == 0) {
    if (row0 + lane < nF) yF[row0 + lane] = yv_own;
    return;
  }
  const long j = (long)cols[blockIdx.x - 1] * T64 + lane;
  double s0 = 0.0, s1 = 0.0;
#pragma unroll 8
  for (int r = 0; r < T64; r += 2) {
    s0 += S[(row0 + r) * lda + j] * y[r];
    s1 += S[(row0 + r + 1) * lda + j] * y[r + 1];
  }
  z[j] -= s0 + s1;
}

__global__ void k_zero_tiles(double *__restrict__ S, long lda, const int2 *__restrict__ tiles) {
  const int2 t = tiles[blockIdx.x];
  double *p = S + (long)t.x * T64 * lda + (long)t.y * T64;
  for (int e = threadIdx.x; e < T64 * 32; e += blockDim.x) {
    const int r = e >> 5, c2 = (e & 31) * 2;
    *reinterpret_cast<dbl2 *>(p + (long)r * lda + c2) = dbl2{0.0, 0.0};
  }
}

}  // namespace

static int panel_ablation() {
  static const int v = [] {
    const char *e = std::getenv("ARSLAM_PANEL_ABLATION");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

void launch_zero_tiles(const LltPlan &P, double *S, hipStream_t s) {
  if (P.n_tiles == 0) return;
  hipLaunchKernelGGL(k_zero_tiles, dim3((unsigned)P.n_tiles), dim3(256), 0, s, S, P.lda, P.tiles);
}

void launch_dense_llt(const LltPlan &P, double *S, int *flag, hipStream_t s, LaunchTiming *timing) {
  const int T = P.T;
  for (int k = 0; k < T; ++k) {
    const int nr = P.h_trsm_off[k + 1] - P.h_trsm_off[k];
    const dim3 g((unsigned)(nr + 1));
    const int *rows = P.trsm_rows + P.h_trsm_off[k];
    switch (panel_ablation()) {   // timing-only ablations (ARSLAM_PANEL_ABLATION), 0 = real kernel
      case 1: hipLaunchKernelGGL(k_panel<1>, g, dim3(256), 0, s, S, P.lda, k, rows, flag); break;
      case 2: hipLaunchKernelGGL(k_panel<2>, g, dim3(256), 0, s, S, P.lda, k, rows, flag); break;
      case 4: hipLaunchKernelGGL(k_panel<4>, g, dim3(256), 0, s, S, P.lda, k, rows, flag); break;
      case 8: hipLaunchKernelGGL(k_panel<8>, g, dim3(256), 0, s, S, P.lda, k, rows, flag); break;
      case 16: hipLaunchKernelGGL(k_panel<16>, g, dim3(256), 0, s, S, P.lda, k, rows, flag); break;
      case 31: hipLaunchKernelGGL(k_panel<31>, g, dim3(256), 0, s, S, P.lda, k, rows, flag); break;
      default: hipLaunchKernelGGL(k_panel<0>, g, dim3(256), 0, s, S, P.lda, k, rows, flag); break;
    }
    const long nu = P.h_upd_off[k + 1] - P.h_upd_off[k];
    if (nu > 0) {
      const bool rec = timing && timing->used < timing->cap;
      if (rec) (void)hipEventRecord(timing->ev[2 * timing->used], s);
      hipLaunchKernelGGL(k_update, dim3((unsigned)nu), dim3(256), 0, s, S, P.lda, k,
                         P.upd_pairs + P.h_upd_off[k], flag);
      if (rec) {
        (void)hipEventRecord(timing->ev[2 * timing->used + 1], s);
        timing->used++;
        timing->flops += P.h_upd_flops[k];
      }
    }
  }
}

void launch_dense_back_solve(const LltPlan &P, const double *S, long nF, double *z, double *yF,
                             const int *flag, hipStream_t s) {
  const long N = (long)P.T * T64;
  hipLaunchKernelGGL(k_init_z, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, S, P.lda, nF, N, z);
  for (int k = P.T - 1; k >= 0; --k) {
    const int nc = P.h_bs_off[k + 1] - P.h_bs_off[k];
    hipLaunchKernelGGL(k_back_solve, dim3((unsigned)(nc + 1)), dim3(64), 0, s, S, P.lda, nF, k,
                       P.bs_cols + P.h_bs_off[k], z, yF, flag);
  }
}

}  // namespace arslam
