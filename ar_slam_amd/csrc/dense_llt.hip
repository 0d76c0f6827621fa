// dense_llt.hip -- Cholesky of the reduced (tag + camera) system on gfx950,
// replacing the Eigen::LLT that Ceres' DenseSchurComplementSolver runs on one
// CPU thread.
//
// Storage: compact 64 x 64 fp64 tiles (only the tiles of the factor exist;
// tile (i,j) at S + tile_id[i*T+j] * 4096, assembled tiles first so the
// multi-GPU all-reduce of the Schur sums covers one contiguous prefix).
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

#include <algorithm>
#include <climits>
#include <cmath>
#include <utility>

namespace arslam {

namespace {

typedef double dbl4 __attribute__((ext_vector_type(4)));
typedef double dbl2 __attribute__((ext_vector_type(2)));

constexpr int T64 = kTile;

#ifdef ARSLAM_STAMPS
__device__ unsigned long long g_stamps[64];
#define STAMP(id)                                                                       \
  do {                                                                                  \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    unsigned long long _t;                                                              \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");        \
    if (blockIdx.x == 0 && threadIdx.x == 0) g_stamps[id] = _t;                         \
    __builtin_amdgcn_sched_barrier(0);                                                  \
  } while (0)
#else
#define STAMP(id) do {} while (0)
#endif
constexpr int LP = 65;   // LDS row pitch (doubles) for row-per-lane tiles
constexpr int LM = 66;   // LDS row pitch for MFMA operand tiles (conflict-free ds_read_b64)

// Compact tile storage: tile (i,j) of the factor is a contiguous 64x64
// row-major block at S + tid[i*T + j] * 4096 (tid = -1: structurally zero).
__device__ __forceinline__ double *tile_ptr(double *S, const int *tid, int T, int i, int j) {
  return S + (long)tid[(long)i * T + j] * (T64 * T64);
}
__device__ __forceinline__ const double *tile_ptr(const double *S, const int *tid, int T, int i, int j) {
  return S + (long)tid[(long)i * T + j] * (T64 * T64);
}

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

// A fast continuation (-DARSLAM_FAST_CONT, round 6, measured and not kept:
// DESIGN §9): a claimed continuation whose A_kk is in registers starts on
// waves 0, 2, 3 while wave 1 still waits for the solved tile's store
// acknowledgements -- no closing barriers, no start barriers
#ifdef ARSLAM_FAST_CONT
constexpr bool kFastCont = true;
#else
constexpr bool kFastCont = false;
#endif
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

// v of lane l of this lane's 16-lane row: one v_mov_b64_dpp row_newbcast:l.
// l must fold to a constant (unrolled loops; the switch then disappears), and
// the source lane must be active: call it outside divergent conditions.
__device__ __forceinline__ double bcast16(double v, int l) {
  switch (l) {
    case 0: return __builtin_amdgcn_mov_dpp(v, 0x150, 0xf, 0xf, false);
    case 1: return __builtin_amdgcn_mov_dpp(v, 0x151, 0xf, 0xf, false);
    case 2: return __builtin_amdgcn_mov_dpp(v, 0x152, 0xf, 0xf, false);
    case 3: return __builtin_amdgcn_mov_dpp(v, 0x153, 0xf, 0xf, false);
    case 4: return __builtin_amdgcn_mov_dpp(v, 0x154, 0xf, 0xf, false);
    case 5: return __builtin_amdgcn_mov_dpp(v, 0x155, 0xf, 0xf, false);
    case 6: return __builtin_amdgcn_mov_dpp(v, 0x156, 0xf, 0xf, false);
    case 7: return __builtin_amdgcn_mov_dpp(v, 0x157, 0xf, 0xf, false);
    case 8: return __builtin_amdgcn_mov_dpp(v, 0x158, 0xf, 0xf, false);
    case 9: return __builtin_amdgcn_mov_dpp(v, 0x159, 0xf, 0xf, false);
    case 10: return __builtin_amdgcn_mov_dpp(v, 0x15a, 0xf, 0xf, false);
    case 11: return __builtin_amdgcn_mov_dpp(v, 0x15b, 0xf, 0xf, false);
    case 12: return __builtin_amdgcn_mov_dpp(v, 0x15c, 0xf, 0xf, false);
    case 13: return __builtin_amdgcn_mov_dpp(v, 0x15d, 0xf, 0xf, false);
    case 14: return __builtin_amdgcn_mov_dpp(v, 0x15e, 0xf, 0xf, false);
    case 15: return __builtin_amdgcn_mov_dpp(v, 0x15f, 0xf, 0xf, false);
    default: return v;
  }
}

// One wave: C(16x16) -= A(16 x K) B(16 x K)^T, operands in LDS (pitch LQ;
// C never overlaps A or B).  C's four entries per lane are read before the
// MFMA chain: read after it, hipcc issued each read-subtract-write as its own
// LDS round trip (four in a row, ~300 cycles on the POTRF's chain per call).
__device__ __forceinline__ void wave_gemm16_sub(double *C, const double *A, const double *B, int K,
                                                int lane) {
  const int li = lane & 15, lk = lane >> 4;
  double c[4];
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) c[reg] = C[(lk + 4 * reg) * LQ + li];
  dbl4 acc = {0, 0, 0, 0};
#ifdef ARSLAM_GEMM_PF
  if (K == 64 && A == B) {   // (variant) the fold: every operand read before the chain
    double a[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) a[q] = A[li * LQ + 4 * q + lk];
#pragma unroll
    for (int q = 0; q < 16; ++q) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q], a[q], acc, 0, 0, 0);
  } else
#endif
  for (int k4 = 0; k4 < K; k4 += 4) {
    const double a = A[li * LQ + k4 + lk];
    const double b = B[li * LQ + k4 + lk];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) C[(lk + 4 * reg) * LQ + li] = c[reg] - acc[reg];
}

constexpr int LI = 18;   // LDS pitch of the 16x16 inverse diagonal blocks (conflict-free fragments)

// One wave: C(16x16) <- C Linv^T in place (the 16-column triangular solve
// X L^T = C as an MFMA product with the explicit inverse of the 16x16 block).
__device__ __forceinline__ void wave_apply_inv16(double *C, const double *Linv, int lane) {
  const int li = lane & 15, lk = lane >> 4;
  double a[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) a[q] = C[li * LQ + 4 * q + lk];
  __builtin_amdgcn_wave_barrier();
  dbl4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int q = 0; q < 4; ++q)
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q], Linv[li * LI + 4 * q + lk], acc, 0, 0, 0);
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) C[(lk + 4 * reg) * LQ + li] = acc[reg];
}

// v of DPP row g (16 lanes) of this wave, lane-wise, in every row: two
// v_permlane16_swap_b32 (within pairs of rows) then two v_permlane32_swap_b32
// (between the halves), picking the half that holds row g.  g must fold to
// a constant (unrolled loops).
__device__ __forceinline__ double rowbcast(double v, int g) {
  const unsigned long long u = __double_as_longlong(v);
  const unsigned lo0 = (unsigned)u, hi0 = (unsigned)(u >> 32);
  const auto a = __builtin_amdgcn_permlane16_swap(lo0, lo0, false, false);   // {even rows, odd rows} replicated per pair
  const auto b = __builtin_amdgcn_permlane16_swap(hi0, hi0, false, false);
  const unsigned lo1 = (g & 1) ? a[1] : a[0], hi1 = (g & 1) ? b[1] : b[0];
  const auto c = __builtin_amdgcn_permlane32_swap(lo1, lo1, false, false);   // {lower half, upper half} replicated
  const auto d = __builtin_amdgcn_permlane32_swap(hi1, hi1, false, false);
  const unsigned lo = (g & 2) ? c[1] : c[0], hi = (g & 2) ? d[1] : d[0];
  return __longlong_as_double(((unsigned long long)hi << 32) | lo);
}

// One elimination step of diag16 under an explicit exec mask (constant per
// pivot, so no per-lane selects): in the rows below the pivot,
// x_q += nf * xj_q and R += nf * rj; then, in the pivot column's group,
// register jq becomes nf.  The masks are 32-bit immediates per exec half
// (both halves of `below` are equal), so no SGPR pair holds a 64-bit mask
// constant across the unrolled pivots (those used to be spilled to VGPR lanes
// and reloaded with v_readlane inside the chain).  The caller's exec is
// restored at the end, and the trailing s_nop covers the wait states hipcc
// does not insert after an asm statement (exec write -> DPP, and the outputs
// -> the next pivot's DPP).
template <int j>
__device__ __forceinline__ void elim_step(double &x0, double &x1, double &x2, double &x3, double &R, double nf,
                                          double y0, double y1, double y2, double y3, double rj) {
  constexpr unsigned m = (0xffffu << (j + 1)) & 0xffffu;   // rows i > j of one 16-lane group
  constexpr unsigned BL = m | (m << 16);                    // `below`, per exec half
  constexpr int g = j >> 2;                                 // the group holding column j
  constexpr unsigned CL = g == 0 ? m : g == 1 ? (m << 16) : 0u;
  constexpr unsigned CH = g == 2 ? m : g == 3 ? (m << 16) : 0u;
  unsigned sl, sh;
#define ARSLAM_ELIM_ASM(XS)                                                                   \
  asm volatile("s_mov_b32 %[sl], exec_lo\n\t"                                                 \
               "s_mov_b32 %[sh], exec_hi\n\t"                                                 \
               "s_and_b32 exec_lo, %[sl], %[bl]\n\t"                                          \
               "s_and_b32 exec_hi, %[sh], %[bl]\n\t"                                          \
               "v_fma_f64 %[x0], %[nf], %[y0], %[x0]\n\t"                                     \
               "v_fma_f64 %[x1], %[nf], %[y1], %[x1]\n\t"                                     \
               "v_fma_f64 %[x2], %[nf], %[y2], %[x2]\n\t"                                     \
               "v_fma_f64 %[x3], %[nf], %[y3], %[x3]\n\t"                                     \
               "v_fma_f64 %[R], %[nf], %[rj], %[R]\n\t"                                       \
               "s_and_b32 exec_lo, %[sl], %[cl]\n\t"                                          \
               "s_and_b32 exec_hi, %[sh], %[ch]\n\t"                                          \
               "v_mov_b64 %[" XS "], %[nf]\n\t"                                               \
               "s_mov_b32 exec_lo, %[sl]\n\t"                                                 \
               "s_mov_b32 exec_hi, %[sh]\n\t"                                                 \
               "s_nop 4"   /* exec write -> DPP: 5 states; VGPR write -> DPP read: 2 */        \
               : [x0] "+v"(x0), [x1] "+v"(x1), [x2] "+v"(x2), [x3] "+v"(x3), [R] "+v"(R),      \
                 [sl] "=&s"(sl), [sh] "=&s"(sh)                                                \
               : [nf] "v"(nf), [y0] "v"(y0), [y1] "v"(y1), [y2] "v"(y2), [y3] "v"(y3),          \
                 [rj] "v"(rj), [bl] "i"(BL), [cl] "i"(CL), [ch] "i"(CH))
  switch (j & 3) {
    case 0: ARSLAM_ELIM_ASM("x0"); break;
    case 1: ARSLAM_ELIM_ASM("x1"); break;
    case 2: ARSLAM_ELIM_ASM("x2"); break;
    default: ARSLAM_ELIM_ASM("x3"); break;
  }
#undef ARSLAM_ELIM_ASM
}

// Pivot J of diag16 (a template, so every broadcast lane and exec mask is a
// compile-time constant however large the unrolled loop gets).
template <int j>
__device__ __forceinline__ void diag16_pivot(double (&x)[4], double &R, double &R2, double *colx, int lane) {
  const int i = lane & 15;
  const double ajj = bcast16(R, j);
  const double r0 = __builtin_amdgcn_rcp(ajj);
  const double e = __builtin_fma(-ajj, r0, 1.0);   // r0 (1 + e + e^2) = (1 - e^3) / ajj
  const double nf0 = -R * r0;
  const double pe = __builtin_fma(e, e, e);
  const double nf = __builtin_fma(nf0, pe, nf0);    // -f_ij (garbage in rows i <= j: masked below)
  double xj[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) xj[q] = bcast16(x[q], j);
  const double rj = j + 1 < 16 ? bcast16(R2, j) : 0.0;
  R = R2;
  // rows i > j only (exec = the lanes 16 g + i with i > j, a constant per
  // pivot); then column j of those rows (group j / 4) becomes -f_ij
  elim_step<j>(x[0], x[1], x[2], x[3], R, nf, xj[0], xj[1], xj[2], xj[3], rj);
  if (j + 2 < 16) {   // column j+2 after this pivot, a pivot before it is needed
    colx[lane] = x[(j + 2) & 3];
    R2 = colx[16 * ((j + 2) >> 2) + i];
  }
}

template <int... J>
__device__ __forceinline__ void diag16_pivots(double (&x)[4], double &R, double &R2, double *colx, int lane,
                                              std::integer_sequence<int, J...>) {
  (diag16_pivot<J>(x, R, R2, colx, lane), ...);
}

// 16x16 diagonal block (rows/cols b0..b0+15 of D, lower triangle) on one
// wave: L into D (zeros above the diagonal), L^{-1} into Li (pitch LI),
// 1/L_ii into inv.  Lane 16 g + i owns row i, columns 4g..4g+3.  One
// Gaussian elimination pass over A, in place: at pivot j the register of
// column j in the rows below becomes the multiplier -f_ij, so row i ends as
// U = Dg Lu^T (columns >= i) and Lu^{-1} (columns < i), with Lu unit lower
// and Dg the pivots; then L^T = Dg^{-1/2} U and L^{-1} = Dg^{-1/2} Lu^{-1}.
// Each pivot needs column j in every row; it is kept replicated one pivot
// ahead (R: column j, R2: column j+1), and column j+2 is fetched through the
// 64-double LDS scratch colx after pivot j's update, a pivot before it is
// needed.  Per pivot: DPP broadcast -> v_rcp_f64 -> two-term Newton
// correction -> multiplier -> update; about 20 VALU instructions, so the
// block is bound by one wave's issue rate (tools/lat_bench.hip).
__device__ __forceinline__ void diag16(double *D, int b0, double *inv, double *Li, int *bad, int lane,
                                       double *colx) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int g = lane >> 4, i = lane & 15;
  double x[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {   // the lower triangle is the valid half: mirror it
    const int c = 4 * g + q;
    x[q] = c <= i ? D[(b0 + i) * LQ + b0 + c] : D[(b0 + c) * LQ + b0 + i];
  }
  // replicated columns 0 and 1 (lower triangle mirrored)
  double R = D[(b0 + i) * LQ + b0];
  double R2 = i >= 1 ? D[(b0 + i) * LQ + b0 + 1] : D[(b0 + 1) * LQ + b0];
  diag16_pivots(x, R, R2, colx, lane, std::make_integer_sequence<int, 16>{});
  // pivot of row i: the diagonal entry of U, held by group i / 4
  __builtin_amdgcn_wave_barrier();
  if (g == (i >> 2)) colx[i] = (i & 3) == 0 ? x[0] : (i & 3) == 1 ? x[1] : (i & 3) == 2 ? x[2] : x[3];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const double piv = colx[i];
  if (!(piv > 0.0)) *bad = 1;
#ifdef ARSLAM_D16_RSQ
  // (variant) 1 / sqrt(piv) by v_rsq_f64 and two Newton steps, d = piv / sqrt(piv)
  double rd = __builtin_amdgcn_rsq(piv);
  rd = rd * __builtin_fma(-0.5 * piv * rd, rd, 1.5);
  rd = rd * __builtin_fma(-0.5 * piv * rd, rd, 1.5);
  const double d = piv * rd;
#else
  const double d = sqrt(piv), rd = 1.0 / d;
#endif
  // lane (g, i), column c = 4g+q:  L_{c,i} = U_i[c] / d_i (c > i),
  // (L^{-1})_{i,c} = Lu^{-1}_i[c] / d_i (c < i)
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = 4 * g + q;
    D[(b0 + c) * LQ + b0 + i] = c > i ? x[q] * rd : (c == i ? d : 0.0);
    Li[i * LI + c] = c < i ? x[q] * rd : (c == i ? rd : 0.0);
  }
  if (g == 0) inv[b0 + i] = rd;
}

// In-LDS blocked Cholesky of the 64x64 tile D (256 threads), right-looking
// over 16-column panels with a one-panel lookahead: wave 0 updates the next
// diagonal block first and factors it (diag16) while waves 1-3 apply the
// rest of the trailing update, so the critical chain is the four diag16
// calls plus one 16-row solve and one 16x16 update per panel.
// Returns false (uniformly) if a pivot is not positive; inv[c] = 1 / L_cc.
// idle(p, w, lane) runs on waves 1-3 beside wave 0's diagonal block p (after
// their share of the trailing update): the persistent executor fetches its
// fused TRSM's tile there.
// F (with fold / non-null): a 64x64 tile in LDS (pitch LQ) whose product F F^T is first
// subtracted from D -- the last update of the diagonal tile, folded into the
// factorization: wave 0 folds block (0,0) and goes straight on to its
// diag16 while waves 1-3 fold the other nine lower blocks beside it (the
// same MFMA products in the same order as a separate fold: bit-identical).
template <class Idle>
__device__ bool blocked_potrf64_idle(double *D, double *inv, double *LTd, int *bad, int tid, double *colx,
                                     Idle &&idle, const double *F = nullptr) {
  const int w = tid >> 6, lane = tid & 63;
  if (tid == 0) *bad = 0;
  __syncthreads();
  for (int p = 0; p < 4; ++p) {
    const int b0 = 16 * p;
    STAMP(10 + 4 * p);
    if (w == 0) {
      if (p == 0 && F) wave_gemm16_sub(D, F, F, 64, lane);
      if (p > 0) wave_gemm16_sub(D + b0 * LQ + b0, D + b0 * LQ + b0 - 16, D + b0 * LQ + b0 - 16, 16, lane);
      diag16(D, b0, inv, LTd + p * 16 * LI, bad, lane, colx);
    } else if (p == 0) {
      if (F) {
        // lower blocks 1..9 in row order (I, C), I >= C: (1,0) (1,1) (2,0) (2,1) (2,2) (3,0) ...
        for (int t = w; t < 10; t += 3) {
          int I = 0;
          while ((I + 1) * (I + 2) / 2 <= t) ++I;
          const int C = t - I * (I + 1) / 2;
          wave_gemm16_sub(D + 16 * I * LQ + 16 * C, F + 16 * I * LQ, F + 16 * C * LQ, 64, lane);
        }
      }
      idle(0, w, lane);
    } else {
      // panel p-1's update of blocks (I, C), I >= C >= p, except (p, p)
      const int m = 4 - p, ntl = m * (m + 1) / 2;
      for (int t = w; t < ntl; t += 3) {
        int I = 0;
        while ((I + 1) * (I + 2) / 2 <= t) ++I;
        const int C = t - I * (I + 1) / 2;
        const int bi = 16 * (p + I), bc = 16 * (p + C);
        wave_gemm16_sub(D + bi * LQ + bc, D + bi * LQ + b0 - 16, D + bc * LQ + b0 - 16, 16, lane);
      }
      idle(p, w, lane);
    }
    __syncthreads();
    STAMP(11 + 4 * p);
    if (p < 3) {
      // rows below the diagonal block: X L_pp^T = A_panel  ->  X = A_panel L_pp^{-T}
      if (w < 3 - p) wave_apply_inv16(D + (b0 + 16 + 16 * w) * LQ + b0, LTd + p * 16 * LI, lane);
      __syncthreads();
    }
    STAMP(12 + 4 * p);
    STAMP(13 + 4 * p);
  }
  return *bad == 0;
}

// LDS flags of the asynchronous panel pipeline below (one workgroup).  The
// volatile accesses go through LDS-typed pointers: a volatile access through a
// generic pointer stays a flat access (the address space is not inferred),
// and hipcc mis-selects the aperture compare of some of those.
typedef __attribute__((address_space(3))) volatile int lds_vint;
__device__ __forceinline__ lds_vint *as_lds(const int *f) { return (lds_vint *)(f); }
__device__ __forceinline__ void lds_set(int *f, int v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  *as_lds(f) = v;
}
__device__ __forceinline__ void lds_add(int *f, int lane) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (lane == 0) __hip_atomic_fetch_add(f, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int lds_get(const int *f) { return *as_lds(f); }
__device__ __forceinline__ void lds_wait(const int *f, int v) {
  while (*as_lds(f) < v) __builtin_amdgcn_s_sleep(0);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// The same factorization (same products in the same order: bit-identical) as
// blocked_potrf64_idle, without workgroup barriers on wave 0's chain.  Wave 0
// runs diag16(p) -> the next block's apply (p+1, p) -> the lookahead update of
// (p+1, p+1) -> diag16(p+1) ...; waves 1-3 apply the blocks further down and
// do the trailing updates of each panel (and the optional fold F F^T) beside
// it, synchronised through LDS counters: fl[0] = panels whose diagonal block is
// factored and next block applied (wave 0), fl[1] = applies done by waves 1-3,
// fl[2] = update rounds done by waves 1-3 (round 0 the fold, round p+1 panel
// p's trailing updates; three increments per round).  idle(p, w, lane) runs
// on waves 1-3 after round p (as beside panel p in the barrier version).
//
// With the fold, wave 0's first apply and lookahead need only blocks (1, 0)
// and (1, 1) folded -- the first blocks waves 1 and 2 fold -- not the whole
// round 0 (wave 3's third block made wave 0 wait ~500 cycles after diag16(0)):
// those two count in *fcnt, and waves 1-3 await the complete round 0
// themselves before their first applies.
//
// fsync (a fast continuation, k_factor_dag): the caller reset the flags
// before its last barrier and the waves arrive at different times, so there
// is no reset and no barrier here; fsync[0] = 1 once the flags are reset,
// fsync[1] = 2 once waves 2-3 have moved A_kk into D.
template <class Idle>
__device__ bool blocked_potrf64_async(double *D, double *inv, double *LTd, int *bad, int *fl, int tid,
                                      double *colx, Idle &&idle, const double *F = nullptr, bool fold = false,
                                      int *fcnt = nullptr, const int *fsync = nullptr) {
  const int w = tid >> 6, lane = tid & 63;
  const bool early = fold && fcnt;
  if (fsync) {
    lds_wait(fsync, 1);
    lds_wait(fsync + 1, 2);
  } else {
    if (tid == 0) {
      *bad = 0;
      fl[0] = fl[1] = fl[2] = fl[3] = 0;   // (fl[3]: the caller's prefetch count)
      if (fcnt) *fcnt = 0;
    }
    __syncthreads();
  }
  if (w == 0) {
    STAMP(30);
    for (int p = 0; p < 4; ++p) {
      const int b0 = 16 * p;
      if (p == 0 && fold) wave_gemm16_sub(D, F, F, 64, lane);
      // (p > 0: block (p, p) had panel p-1's lookahead update at the end of
      // iteration p-1, and rounds 0 .. p-1 were awaited there)
      STAMP(31 + 6 * p);
      STAMP(32 + 6 * p);
      diag16(D, b0, inv, LTd + p * 16 * LI, bad, lane, colx);
      STAMP(33 + 6 * p);
      if (p < 3) {
        if (p == 0 && early) lds_wait(fcnt, 2);   // blocks (1, 0) and (1, 1) folded
        else lds_wait(fl + 2, 3 * (p + 1));      // round p: block (p+1, p) has panel p-1's update
        STAMP(34 + 6 * p);
        // The block below the diagonal solved transposed, Y = L_pp^{-1} A^T
        // (the same products as A L_pp^{-T}, operands swapped: bit-identical),
        // so each lane holds X[i][lk + 4 reg] -- the MFMA operand layout of
        // X X^T: the next diagonal block's lookahead update runs from the
        // registers, without reading X back from LDS.
        const int li = lane & 15, lk = lane >> 4;
        double *Cb = D + (b0 + 16) * LQ + b0, *Cd = Cb + 16;
        const double *Linv = LTd + p * 16 * LI;
        double a[4], cd[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] = Cb[li * LQ + 4 * q + lk];
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) cd[reg] = Cd[(lk + 4 * reg) * LQ + li];
        __builtin_amdgcn_wave_barrier();
        dbl4 y = {0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < 4; ++q) y = __builtin_amdgcn_mfma_f64_16x16x4f64(Linv[li * LI + 4 * q + lk], a[q], y, 0, 0, 0);
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) Cb[li * LQ + lk + 4 * reg] = y[reg];
        lds_set(fl, p + 1);
        STAMP(35 + 6 * p);
        dbl4 g = {0, 0, 0, 0};
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) g = __builtin_amdgcn_mfma_f64_16x16x4f64(y[reg], y[reg], g, 0, 0, 0);
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) Cd[(lk + 4 * reg) * LQ + li] = cd[reg] - g[reg];
      }
    }
  } else {
    if (fold) {
      // the fold's lower blocks 1..9 in row order (I, C), I >= C: (1,0) (1,1) (2,0) (2,1) ...
      for (int t = w; t < 10; t += 3) {
        int I = 0;
        while ((I + 1) * (I + 2) / 2 <= t) ++I;
        const int C = t - I * (I + 1) / 2;
        wave_gemm16_sub(D + 16 * I * LQ + 16 * C, F + 16 * I * LQ, F + 16 * C * LQ, 64, lane);
        if (early && t <= 2) lds_add(fcnt, lane);   // (1, 0) by wave 1, (1, 1) by wave 2
      }
    }
    idle(0, w, lane);
    lds_add(fl + 2, lane);
    for (int p = 0; p < 3; ++p) {
      const int b0 = 16 * p;
      if (p == 0 && early) lds_wait(fl + 2, 3);   // every block folded (wave 0 no longer awaits it)
      lds_wait(fl, p + 1);                  // L_pp's block inverse, block (p+1, p) applied
      if (w < 3 - p - 1 + 1 && p + 1 + w <= 3)   // blocks (p+2 .. 3, p): wave w takes p + 1 + w
        wave_apply_inv16(D + (b0 + 16 * (1 + w)) * LQ + b0, LTd + p * 16 * LI, lane);
      lds_add(fl + 1, lane);
      lds_wait(fl + 1, 3 * (p + 1));        // every block of panel p applied
      // panel p's update of blocks (I, C), I >= C >= p + 1, except (p + 1, p + 1)
      const int m = 3 - p, ntl = m * (m + 1) / 2;
      for (int t = w; t < ntl; t += 3) {
        int I = 0;
        while ((I + 1) * (I + 2) / 2 <= t) ++I;
        const int C = t - I * (I + 1) / 2;
        const int bi = 16 * (p + 1 + I), bc = 16 * (p + 1 + C);
        wave_gemm16_sub(D + bi * LQ + bc, D + bi * LQ + b0, D + bc * LQ + b0, 16, lane);
      }
      idle(p + 1, w, lane);
      lds_add(fl + 2, lane);
    }
  }
  __syncthreads();
  return *bad == 0;
}

__device__ bool blocked_potrf64(double *D, double *inv, double *LTd, int *bad, int tid, double *colx) {
  return blocked_potrf64_idle(D, inv, LTd, bad, tid, colx, [](int, int, int) {});
}

// Column step p of the blocked solve X L^T = A for row block rb of X (one
// wave): X[rb, p] -= X[rb, 0:p] L[p, 0:p]^T, then X[rb, p] <- X[rb, p] L_pp^{-T}.
__device__ __forceinline__ void trsm_step(double *X, const double *D, const double *LTd, int rb, int p, int lane) {
  const int b0 = 16 * p;
  if (p > 0) wave_gemm16_sub(X + 16 * rb * LQ + b0, X + 16 * rb * LQ, D + b0 * LQ, b0, lane);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  wave_apply_inv16(X + 16 * rb * LQ + b0, LTd + p * 16 * LI, lane);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// In-LDS blocked solve X L^T = A for a 64x64 tile X (256 threads), L from
// blocked_potrf64 (lower part of D, inv = 1 / diag).
__device__ void blocked_trsm64(double *X, const double *D, const double *inv, const double *LTd,
                               int tid) {
  // row block w of X depends only on itself (and on D, LTd): the four
  // column steps need wave-local ordering only; one barrier at the end
  const int w = tid >> 6, lane = tid & 63;
  for (int p = 0; p < 4; ++p) trsm_step(X, D, LTd, w, p, lane);
  __syncthreads();
}

// Inverse X = L^{-1} of the 64x64 lower factor in D (after blocked_potrf64),
// built in LDS as its transpose XT (XT[c][r] = X[r][c]) from the 16x16
// diagonal-block inverses Li_p in LTd:  X_qq = Li_q,
//   X_pq = -Li_p sum_{r=q}^{p-1} L_pr X_rq   (p > q).
// Wave q owns column block q (three dependent 16x16 MFMA steps at most);
// its 16x16 scratch sits in a part of XT that stays structurally zero.
__device__ void blocked_trinv64(const double *D, const double *LTd, double *XT, int tid) {
  const int q = tid >> 6, lane = tid & 63;
  const int li = lane & 15, lk = lane >> 4;
  const double *Lq = LTd + q * 16 * LI;
#pragma unroll
  for (int e = 0; e < 4; ++e) {   // XT block (q,q) = Li_q^T
    const int idx = lane + 64 * e, i = idx >> 4, j = idx & 15;
    XT[(16 * q + j) * LQ + 16 * q + i] = (j <= i) ? Lq[i * LI + j] : 0.0;
  }
  double *scr = XT + (q == 0 ? 48 : 16 * q) * LQ;   // columns 0..15 of row block 3 (q=0) or q
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  for (int p = q + 1; p < 4; ++p) {
    dbl4 acc = {0, 0, 0, 0};
    for (int r = q; r < p; ++r)
#pragma unroll
      for (int k4 = 0; k4 < 4; ++k4) {
        const double a = D[(16 * p + li) * LQ + 16 * r + 4 * k4 + lk];
        const double b = XT[(16 * q + li) * LQ + 16 * r + 4 * k4 + lk];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
      }
    // acc[reg] = M[lk + 4 reg][li]; scratch rows = M^T rows
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) scr[li * LQ + lk + 4 * reg] = acc[reg];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    dbl4 x = {0, 0, 0, 0};
    const double *Lp = LTd + p * 16 * LI;
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4)
      x = __builtin_amdgcn_mfma_f64_16x16x4f64(Lp[li * LI + 4 * k4 + lk], scr[li * LQ + 4 * k4 + lk], x, 0, 0, 0);
    // x[reg] = (Li_p M)[lk + 4 reg][li] = -X_pq[...]
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) XT[(16 * q + li) * LQ + 16 * p + lk + 4 * reg] = -x[reg];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// Panel tasks of one level: task (i,k) factors the diagonal tile (k,k) (every
// task of column k does so redundantly, keeping the level to one launch) and
// either stores L_kk (i == k) or solves tile (i,k) against it.  L_kk goes to
// its own buffer Ld (64x64 per tile column), never over A_kk in S: the other
// tasks of the column may still be reading A_kk.
__global__ __launch_bounds__(256) void k_panel(double *__restrict__ S, const int *__restrict__ tid_map,
                                               int T, double *__restrict__ Ld,
                                               const int2 *__restrict__ tasks,
                                               int *__restrict__ flag) {
  __shared__ __attribute__((aligned(16))) double D[T64 * LQ];
  __shared__ __attribute__((aligned(16))) double X[T64 * LQ];
  __shared__ double inv[T64];
  __shared__ __attribute__((aligned(16))) double LTd[4 * 16 * LI];   // inverses of the 16x16 diagonal blocks
  __shared__ double colx[T64];
  __shared__ int bad;
  STAMP(0);
  if (*flag) return;
  const int tid = threadIdx.x;
  const int2 t = tasks[blockIdx.x];
  const int ti = t.x, k = t.y;
  const double *dk = tile_ptr(S, tid_map, T, k, k);
  double *xt = tile_ptr(S, tid_map, T, ti, k);
  load_tile_wg(dk, T64, D, tid);
  if (ti != k) load_tile_wg(xt, T64, X, tid);
  __syncthreads();
  STAMP(1);
  const bool ok = blocked_potrf64(D, inv, LTd, &bad, tid, colx);
  if (!ok) {
    if (ti == k && tid == 0) {
      int first = 0;
      while (first < T64 && D[first * LQ + first] > 0.0) ++first;
      atomicCAS(flag, 0, 1 + k * T64 + first);
    }
    return;
  }
  if (ti == k) {
    // L_kk, and its inverse (for the backward solve) while the column's
    // other tasks run their TRSMs
    store_tile_wg(Ld + (long)k * T64 * T64, T64, D, tid, true);
    blocked_trinv64(D, LTd, X, tid);
    __syncthreads();
    double *Xg = Ld + ((long)T + k) * T64 * T64;
#pragma unroll 4
    for (int m = 0; m < 16; ++m) {
      const int e = m * 256 + tid, r = e >> 6, c = e & 63;
      Xg[e] = (r >= c) ? X[c * LQ + r] : 0.0;
    }
    return;
  }
  STAMP(2);
  blocked_trsm64(X, D, inv, LTd, tid);
  STAMP(3);
  store_tile_wg(xt, T64, X, tid, false);
  STAMP(4);
}

// Update items of one level: tile (i,j) -= sum over the item's columns k of
// L_ik L_jk^T.  An unsplit target is one item (one workgroup writes the
// tile); a split target's chunks each store their partial product to a slot
// of `part`, and the chunk that arrives last sums the partials in chunk order
// and writes the tile (agent-scope release / acquire hand-off: correct for
// any placement of the chunks over XCDs).  4 waves x 32x32 on
// v_mfma_f64_16x16x4_f64, K = 64 per column; the next column's operand
// tiles are in flight while the current column's MFMAs run.
__global__ __launch_bounds__(256) void k_update(double *__restrict__ S, const int *__restrict__ tid_map,
                                                int T, const int2 *__restrict__ targets,
                                                const int4 *__restrict__ items,
                                                const int *__restrict__ ks,
                                                const int2 *__restrict__ split,
                                                double *__restrict__ part, int *__restrict__ cnt,
                                                const int *__restrict__ flag) {
  __shared__ __attribute__((aligned(16))) double sA[T64 * LM + 2];
  __shared__ __attribute__((aligned(16))) double sB[T64 * LM];
  if (*flag) return;
  const int4 it = items[blockIdx.x];
  const int2 pr = targets[it.x];
  const int ti = pr.x, tj = pr.y;
  const int q0 = it.y, q1 = it.z, sid = it.w;   // sid < 0: unsplit target
  const int tid = threadIdx.x;
  const int w = tid >> 6, lane = tid & 63;
  const int r0 = (w >> 1) * 32, c0 = (w & 1) * 32;
  const int li = lane & 15, lk = lane >> 4;
  dbl4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
  dbl2 va[8], vb[8];
  auto fetch = [&](int q) {
    const int k = ks[q];
    const double *Ai = tile_ptr(S, tid_map, T, ti, k);
    const double *Bj = tile_ptr(S, tid_map, T, tj, k);
#pragma unroll
    for (int e8 = 0; e8 < 8; ++e8) {
      const int e = e8 * 256 + tid, r = e >> 5, c2 = (e & 31) * 2;
      va[e8] = *reinterpret_cast<const dbl2 *>(Ai + r * T64 + c2);
      vb[e8] = *reinterpret_cast<const dbl2 *>(Bj + r * T64 + c2);
    }
  };
  if (q0 < q1) fetch(q0);
  for (int q = q0; q < q1; ++q) {
    if (q > q0) __syncthreads();   // previous column's fragments consumed
#pragma unroll
    for (int e8 = 0; e8 < 8; ++e8) {
      const int e = e8 * 256 + tid, r = e >> 5, c2 = (e & 31) * 2;
      *reinterpret_cast<dbl2 *>(&sA[r * LM + c2]) = va[e8];
      *reinterpret_cast<dbl2 *>(&sB[r * LM + c2]) = vb[e8];
    }
    __syncthreads();
    if (q + 1 < q1) fetch(q + 1);
#pragma unroll 4
    for (int kk = 0; kk < T64 / 4; ++kk) {
      const int kc = kk * 4 + lk;
      const double a0 = sA[(r0 + li) * LM + kc];
      const double a1 = sA[(r0 + 16 + li) * LM + kc];
      const double b0 = sB[(c0 + li) * LM + kc];
      const double b1 = sB[(c0 + 16 + li) * LM + kc];
      acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[1], 0, 0, 0);
      acc[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[2], 0, 0, 0);
      acc[3] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[3], 0, 0, 0);
    }
  }
  if (sid >= 0) {
    // split target (sid = split id << 8 | chunk): publish this chunk's partial
    // (fragment order, lane-contiguous 16-B stores), draw a ticket; the last
    // arriver sums every chunk's partial in chunk order
    const int2 sp = split[sid >> 8];   // {n_chunks, first slot}
    dbl2 *mine = reinterpret_cast<dbl2 *>(part + (long)(sp.y + (sid & 255)) * 4096);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      mine[(2 * q) * 256 + tid] = dbl2{acc[q][0], acc[q][1]};
      mine[(2 * q + 1) * 256 + tid] = dbl2{acc[q][2], acc[q][3]};
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int *is_last = reinterpret_cast<int *>(&sA[T64 * LM]);
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int old = __hip_atomic_fetch_add(cnt + (sid >> 8), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *is_last = old == sp.x - 1;
      if (old == sp.x - 1) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    __syncthreads();
    if (!*is_last) return;
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = dbl4{0, 0, 0, 0};
    for (int c = 0; c < sp.x; ++c) {
      const dbl2 *pc = reinterpret_cast<const dbl2 *>(part + (long)(sp.y + c) * 4096);
      dbl2 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = pc[u * 256 + tid];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc[q][0] += v[2 * q].x;
        acc[q][1] += v[2 * q].y;
        acc[q][2] += v[2 * q + 1].x;
        acc[q][3] += v[2 * q + 1].y;
      }
    }
  }
  // f64 MFMA C/D layout: col = lane & 15, row = (lane >> 4) + 4 * reg
  double *C = tile_ptr(S, tid_map, T, ti, tj);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int rb = r0 + (q >> 1) * 16, cb = c0 + (q & 1) * 16;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int row = rb + lk + 4 * reg, col = cb + li;
      C[row * T64 + col] -= acc[q][reg];
    }
  }
}

// ---------------------------------------------------------------------------
// Persistent task-graph executor of the same factorization.  Every workgroup
// loops: draw a ticket (tasks are in a topological order, dag_build), wait
// (thread 0, bounded spin) for the task's dependency counters, run it, and
// publish its result (stores drained, agent-scope release, counter update).
// A waited-on task always holds a smaller ticket, i.e. it was drawn by a
// running workgroup, so progress is guaranteed for any grid size; every
// spin is still bounded (kSpinCap) and raises the error flag if exceeded.
//   POTRF k   : L_kk and L_kk^{-1} into Ld (the column's TRSMs then need
//               only a GEMM with the inverse)
//   TRSM i,k  : L_ik = A_ik L_kk^{-T}  (MFMA, in place)
//   update    : the plan item's sum over its columns k of L_ik L_jk^T; split
//               items publish partials and the last arriver reduces them in
//               chunk order; the application to the target waits for the
//               target's earlier levels, so the summation order is fixed.
// ---------------------------------------------------------------------------
constexpr int kLtdSize = 4 * 16 * LI;   // 1152 doubles
// How long a dependency wait may last before it counts as a device fault: 50
// ms of the 100 MHz s_memrealtime clock (read every 16 polls), far beyond any
// legitimate wait (a whole factorization is < 1 ms).  A time limit, not a poll
// count: the chain tasks poll every unit and the update tasks every 16, so
// with a count the chain task waiting downstream of a stuck update gave up
// first and was the one reported; with the clock the earliest wait gives up
// first, i.e. the stuck task itself (its fault record names its counter).
constexpr unsigned long long kWaitCapTicks = 5000000ull;   // 50 ms at 100 MHz
// the bound on the poll count as well (the clock read is 1 in 16 polls)
constexpr long kSpinCap = 1L << 22;
__device__ __forceinline__ unsigned long long wait_clock() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}
// The time a wait has been *running*: the clock is read every 16th poll and
// each interval counts at most kGapTicks (1 ms; 16 polls take microseconds),
// so a wave descheduled by preemption (the hardware saves the whole dispatch's
// waves and restores them later) does not count the time it was off the
// machine, and a producer preempted with it is not reported as stuck.
constexpr unsigned long long kGapTicks = 100000ull;   // 1 ms at 100 MHz
struct WaitTimer {
  unsigned long long last, run = 0;
  __device__ __forceinline__ WaitTimer() : last(wait_clock()) {}
  // true once the wait has run kWaitCapTicks (checked on every 16th poll) or kSpinCap polls
  __device__ __forceinline__ bool expired(long spins) {
    if (spins > kSpinCap) return true;
    if ((spins & 15) != 0) return false;
    const unsigned long long now = wait_clock(), d = now - last;
    last = now;
    run += d < kGapTicks ? d : kGapTicks;
    return run > kWaitCapTicks;
  }
};
// s_sleep units (64 cycles) between two polls of a dependency counter.  Every
// poll is a device-scope atomic performed at the memory side; with a few
// hundred update tasks waiting at once, polling every 64 cycles slowed the
// whole factorization (the chain's own loads and hand-offs queue behind the
// polls): cfg3 k_factor_dag 796 -> 757 us with the update tasks polling
// every 16 units, flat from 16 to 32, worse at 64 (tools/variant_bench.sh).
// The chain tasks (POTRF, TRSM) and the backward solve keep polling fast.
#ifndef ARSLAM_POLL_SLEEP
#define ARSLAM_POLL_SLEEP 16
#endif
constexpr int kPollSleep = ARSLAM_POLL_SLEEP;   // update tasks
#ifndef ARSLAM_CHAIN_SLEEP
#define ARSLAM_CHAIN_SLEEP 1
#endif
constexpr int kChainSleep = ARSLAM_CHAIN_SLEEP;   // POTRF / TRSM tasks
constexpr int kBsolveSleep = 1;    // k_bsolve_dag (its waits are all on the chain)

// Poll a dependency counter with an atomic read-modify-write (+0): counters
// are advanced by device-scope atomic adds, and an RMW is performed where
// those are, so it observes them on every XCD.  (A plain relaxed load was
// observed to spin forever on a counter another task had already advanced.)
__device__ __forceinline__ int ld_acquire_relaxed(int *p) {
  // compare-and-swap that never matches (counters are >= 0): returns the value
  // without a write, and cannot be folded into a plain load as an RMW of 0 is
  int v = INT_MIN;
  __hip_atomic_compare_exchange_strong(p, &v, INT_MIN, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return v;
}

// Tile hand-offs between workgroups of the persistent kernel use the
// write-through form (MI355X_MICROARCH.md, visibility): every published
// tile is stored sc1 (8-byte agent-scope relaxed atomic stores) and every
// load of a tile that another workgroup may write in this launch is an sc1
// load, so no release or acquire fence is needed around the counters.
__device__ __forceinline__ void st_wt(double *p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long *>(p), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double *p) {
  return __longlong_as_double((long long)__hip_atomic_load(
      reinterpret_cast<const unsigned long long *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// 16-byte write-through store / sc1 loads (inline asm: hipcc has no 16-byte
// atomic form).  Loads are issued in groups inside ONE asm statement that
// also waits for them (vmcnt(0)), so the compiler never sees an asm output
// before its data has arrived.
// (the trailing s_nop: a VALU write of the data VGPRs right after a 128-bit
// store may land before the store has read them, and hipcc does not pad an
// asm statement; MI355X hazard rule, cdna_hip_programming.md §5.7)
__device__ __forceinline__ void st_wt16(double *p, dbl2 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}
// eight 16-byte sc1 loads p[k] -> v[k], waited
__device__ __forceinline__ void ld_wt16x8(const double *const p[8], dbl2 v[8]) {
  asm volatile(
      "global_load_dwordx4 %0, %8, off sc1\n\t"
      "global_load_dwordx4 %1, %9, off sc1\n\t"
      "global_load_dwordx4 %2, %10, off sc1\n\t"
      "global_load_dwordx4 %3, %11, off sc1\n\t"
      "global_load_dwordx4 %4, %12, off sc1\n\t"
      "global_load_dwordx4 %5, %13, off sc1\n\t"
      "global_load_dwordx4 %6, %14, off sc1\n\t"
      "global_load_dwordx4 %7, %15, off sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])
      : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]), "v"(p[6]), "v"(p[7])
      : "memory");
}
// sixteen 16-byte sc1 loads p[k] -> v[k], waited
__device__ __forceinline__ void ld_wt16x16(const double *const p[16], dbl2 v[16]) {
  asm volatile(
      "global_load_dwordx4 %0, %16, off sc1\n\t"
      "global_load_dwordx4 %1, %17, off sc1\n\t"
      "global_load_dwordx4 %2, %18, off sc1\n\t"
      "global_load_dwordx4 %3, %19, off sc1\n\t"
      "global_load_dwordx4 %4, %20, off sc1\n\t"
      "global_load_dwordx4 %5, %21, off sc1\n\t"
      "global_load_dwordx4 %6, %22, off sc1\n\t"
      "global_load_dwordx4 %7, %23, off sc1\n\t"
      "global_load_dwordx4 %8, %24, off sc1\n\t"
      "global_load_dwordx4 %9, %25, off sc1\n\t"
      "global_load_dwordx4 %10, %26, off sc1\n\t"
      "global_load_dwordx4 %11, %27, off sc1\n\t"
      "global_load_dwordx4 %12, %28, off sc1\n\t"
      "global_load_dwordx4 %13, %29, off sc1\n\t"
      "global_load_dwordx4 %14, %30, off sc1\n\t"
      "global_load_dwordx4 %15, %31, off sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7]),
        "=&v"(v[8]), "=&v"(v[9]), "=&v"(v[10]), "=&v"(v[11]), "=&v"(v[12]), "=&v"(v[13]), "=&v"(v[14]),
        "=&v"(v[15])
      : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]), "v"(p[6]), "v"(p[7]), "v"(p[8]),
        "v"(p[9]), "v"(p[10]), "v"(p[11]), "v"(p[12]), "v"(p[13]), "v"(p[14]), "v"(p[15])
      : "memory");
}
// 11 16-byte sc1 loads p[k] -> v[k] in one batch, waited
__device__ __forceinline__ void ld_wt16x11(const double *const p[11], dbl2 v[11]) {
  asm volatile(
      "global_load_dwordx4 %0, %11, off sc1\n\t"
      "global_load_dwordx4 %1, %12, off sc1\n\t"
      "global_load_dwordx4 %2, %13, off sc1\n\t"
      "global_load_dwordx4 %3, %14, off sc1\n\t"
      "global_load_dwordx4 %4, %15, off sc1\n\t"
      "global_load_dwordx4 %5, %16, off sc1\n\t"
      "global_load_dwordx4 %6, %17, off sc1\n\t"
      "global_load_dwordx4 %7, %18, off sc1\n\t"
      "global_load_dwordx4 %8, %19, off sc1\n\t"
      "global_load_dwordx4 %9, %20, off sc1\n\t"
      "global_load_dwordx4 %10, %21, off sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7]), "=&v"(v[8]), "=&v"(v[9]), "=&v"(v[10])
      : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]), "v"(p[6]), "v"(p[7]), "v"(p[8]), "v"(p[9]), "v"(p[10])
      : "memory");
}
// 19 16-byte sc1 loads p[k] -> v[k] in one batch, waited
__device__ __forceinline__ void ld_wt16x19(const double *const p[19], dbl2 v[19]) {
  asm volatile(
      "global_load_dwordx4 %0, %19, off sc1\n\t"
      "global_load_dwordx4 %1, %20, off sc1\n\t"
      "global_load_dwordx4 %2, %21, off sc1\n\t"
      "global_load_dwordx4 %3, %22, off sc1\n\t"
      "global_load_dwordx4 %4, %23, off sc1\n\t"
      "global_load_dwordx4 %5, %24, off sc1\n\t"
      "global_load_dwordx4 %6, %25, off sc1\n\t"
      "global_load_dwordx4 %7, %26, off sc1\n\t"
      "global_load_dwordx4 %8, %27, off sc1\n\t"
      "global_load_dwordx4 %9, %28, off sc1\n\t"
      "global_load_dwordx4 %10, %29, off sc1\n\t"
      "global_load_dwordx4 %11, %30, off sc1\n\t"
      "global_load_dwordx4 %12, %31, off sc1\n\t"
      "global_load_dwordx4 %13, %32, off sc1\n\t"
      "global_load_dwordx4 %14, %33, off sc1\n\t"
      "global_load_dwordx4 %15, %34, off sc1\n\t"
      "global_load_dwordx4 %16, %35, off sc1\n\t"
      "global_load_dwordx4 %17, %36, off sc1\n\t"
      "global_load_dwordx4 %18, %37, off sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7]), "=&v"(v[8]), "=&v"(v[9]), "=&v"(v[10]), "=&v"(v[11]), "=&v"(v[12]), "=&v"(v[13]), "=&v"(v[14]), "=&v"(v[15]), "=&v"(v[16]), "=&v"(v[17]), "=&v"(v[18])
      : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]), "v"(p[6]), "v"(p[7]), "v"(p[8]), "v"(p[9]), "v"(p[10]), "v"(p[11]), "v"(p[12]), "v"(p[13]), "v"(p[14]), "v"(p[15]), "v"(p[16]), "v"(p[17]), "v"(p[18])
      : "memory");
}
// A 64x64 tile g1 -> lds1 (and g2 -> lds2 if given) and a column's 16x16
// block inverses ltd_g -> LTd (1152 doubles): every sc1 load in flight at
// once, one round trip instead of one per array
__device__ __forceinline__ void load_tiles_ltd_wt(const double *__restrict__ g1, double *lds1,
                                                  const double *__restrict__ g2, double *lds2,
                                                  const double *__restrict__ ltd_g, double *LTd, int tid) {
  constexpr int kL = kLtdSize / 2;   // 16-byte elements of the block inverses (576)
  const double *p[19];
  dbl2 v[19];
  const int nt = g2 ? 16 : 8;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    p[q] = g1 + 2 * (q * 256 + tid);
    p[8 + q] = (g2 ? g2 : g1) + 2 * (q * 256 + tid);
  }
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int e = tid + 256 * u;
    p[16 + u] = ltd_g + 2 * (e < kL ? e : 0);
  }
  if (g2) {
    ld_wt16x19(p, v);
  } else {
    const double *p11[11] = {p[0], p[1], p[2], p[3], p[4], p[5], p[6], p[7], p[16], p[17], p[18]};
    dbl2 v11[11];
    ld_wt16x11(p11, v11);
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = v11[q];
#pragma unroll
    for (int u = 0; u < 3; ++u) v[16 + u] = v11[8 + u];
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = q * 256 + tid, r = e >> 5, c2 = (e & 31) * 2;
    *reinterpret_cast<dbl2 *>(lds1 + r * LQ + c2) = v[q];
    if (nt == 16) *reinterpret_cast<dbl2 *>(lds2 + r * LQ + c2) = v[8 + q];
  }
#pragma unroll
  for (int u = 0; u < 3; ++u) {
    const int e = tid + 256 * u;
    if (e < kL) *reinterpret_cast<dbl2 *>(LTd + 2 * e) = v[16 + u];
  }
}
// Half a 64x64 tile (128 threads, t2 = 0..127: 16-byte element u * 128 + t2
// into v[u]) as sixteen sc1 loads, ISSUED ONLY -- the registers hold the data
// after ld_wt16x16_wait, and nothing may read them before (the caller keeps
// them untouched; the pair shares one address, the second at +2048 bytes).
__device__ __forceinline__ void ld_wt16x16_issue(const double *__restrict__ g, int t2, dbl2 v[16]) {
  const double *p[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) p[m] = g + 2 * (2 * m * 128 + t2);
  asm volatile(
      "global_load_dwordx4 %0, %16, off sc1\n\t"
      "global_load_dwordx4 %1, %16, off offset:2048 sc1\n\t"
      "global_load_dwordx4 %2, %17, off sc1\n\t"
      "global_load_dwordx4 %3, %17, off offset:2048 sc1\n\t"
      "global_load_dwordx4 %4, %18, off sc1\n\t"
      "global_load_dwordx4 %5, %18, off offset:2048 sc1\n\t"
      "global_load_dwordx4 %6, %19, off sc1\n\t"
      "global_load_dwordx4 %7, %19, off offset:2048 sc1\n\t"
      "global_load_dwordx4 %8, %20, off sc1\n\t"
      "global_load_dwordx4 %9, %20, off offset:2048 sc1\n\t"
      "global_load_dwordx4 %10, %21, off sc1\n\t"
      "global_load_dwordx4 %11, %21, off offset:2048 sc1\n\t"
      "global_load_dwordx4 %12, %22, off sc1\n\t"
      "global_load_dwordx4 %13, %22, off offset:2048 sc1\n\t"
      "global_load_dwordx4 %14, %23, off sc1\n\t"
      "global_load_dwordx4 %15, %23, off offset:2048 sc1\n\t"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7]), "=&v"(v[8]), "=&v"(v[9]), "=&v"(v[10]), "=&v"(v[11]), "=&v"(v[12]), "=&v"(v[13]), "=&v"(v[14]), "=&v"(v[15])
      : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]), "v"(p[6]), "v"(p[7])
      : "memory");
}
__device__ __forceinline__ void ld_wt16x16_wait(dbl2 v[16]) {
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]), "+v"(v[8]), "+v"(v[9]), "+v"(v[10]), "+v"(v[11]), "+v"(v[12]), "+v"(v[13]), "+v"(v[14]), "+v"(v[15])::"memory");
}
// eight 8-byte sc1 loads, waited
__device__ __forceinline__ void ld_wt8x8(const double *const p[8], double v[8]) {
  asm volatile(
      "global_load_dwordx2 %0, %8, off sc1\n\t"
      "global_load_dwordx2 %1, %9, off sc1\n\t"
      "global_load_dwordx2 %2, %10, off sc1\n\t"
      "global_load_dwordx2 %3, %11, off sc1\n\t"
      "global_load_dwordx2 %4, %12, off sc1\n\t"
      "global_load_dwordx2 %5, %13, off sc1\n\t"
      "global_load_dwordx2 %6, %14, off sc1\n\t"
      "global_load_dwordx2 %7, %15, off sc1\n\t"
      "s_waitcnt vmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])
      : "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]), "v"(p[6]), "v"(p[7])
      : "memory");
}

// 256-thread sc1 load of a 64x64 row-major tile into LDS (pitch LQ)
__device__ __forceinline__ void load_tile_wt(const double *__restrict__ g, double *lds, int tid) {
  const double *p[8];
  dbl2 v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) p[q] = g + 2 * (q * 256 + tid);
  ld_wt16x8(p, v);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = q * 256 + tid, r = e >> 5, c2 = (e & 31) * 2;
    *reinterpret_cast<dbl2 *>(lds + r * LQ + c2) = v[q];
  }
}

// two tiles at once (both sets of sc1 loads in flight before either is stored)
__device__ __forceinline__ void load_two_tiles_wt(const double *__restrict__ g1, double *lds1,
                                                  const double *__restrict__ g2, double *lds2, int tid) {
  const double *p[16];
  dbl2 v[16];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    p[q] = g1 + 2 * (q * 256 + tid);
    p[8 + q] = g2 + 2 * (q * 256 + tid);
  }
  ld_wt16x16(p, v);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int e = q * 256 + tid, r = e >> 5, c2 = (e & 31) * 2;
    *reinterpret_cast<dbl2 *>(lds1 + r * LQ + c2) = v[q];
    *reinterpret_cast<dbl2 *>(lds2 + r * LQ + c2) = v[8 + q];
  }
}

// NT-thread write-through store of a 64x64 LDS tile (pitch LQ), optionally
// lower triangle only
template <int NT = 256>
__device__ __forceinline__ void store_tile_wt(double *__restrict__ g, const double *lds, int tid, bool lower) {
#pragma unroll
  for (int q = 0; q < 2048 / NT; ++q) {
    const int e = q * NT + tid, r = e >> 5, c2 = (e & 31) * 2;
    dbl2 v = *reinterpret_cast<const dbl2 *>(lds + r * LQ + c2);
    if (lower) {
      if (c2 > r) v.x = 0.0;
      if (c2 + 1 > r) v.y = 0.0;
    }
    st_wt16(g + 2 * e, v);
  }
}

// wave 0: spin until counter[idx] >= val for every wait; false on timeout,
// or at once when another workgroup already timed out (flag < 0), so a
// broken graph drains in one spin cap instead of one per task.  Lane q polls
// wait q (64 at a time), so a task's counters are read in one round trip, not
// one after another.
// On a timeout *unmet = {counter, value seen, value awaited} of the first
// wait still unmet (uniform over the wave), for the fault record; *expired:
// this wait ran out of time (false: it gave up because another one had).
__device__ bool dag_wait(int *counters, const int2 *waits, int w0, int w1, int *flag, int lane, bool chain,
                         int3 *unmet, bool *expired) {
  for (int base = w0; base < w1; base += 64) {
    const int w = base + lane;
    const bool mine = w < w1;
    const int2 cv = mine ? waits[w] : make_int2(0, 0);
    long spins = 0;
    WaitTimer tm;
    for (;;) {
      // (every lane re-polls each round: no loop-carried per-lane state)
      const int got = mine ? ld_acquire_relaxed(counters + cv.x) : 0;
      const unsigned long long m = __builtin_amdgcn_ballot_w64(mine && got < cv.y);
      if (m == 0) break;
      if (chain) __builtin_amdgcn_s_sleep(kChainSleep);
      else __builtin_amdgcn_s_sleep(kPollSleep);
      const bool exp = tm.expired(++spins);
      const bool give_up = exp || ((spins & 255) == 0 && __builtin_amdgcn_readfirstlane(ld_acquire_relaxed(flag)) < 0);
      if (give_up) {
        *expired = exp;
        const int l = __builtin_ctzll(m);
        *unmet = make_int3(__builtin_amdgcn_readlane(cv.x, l), __builtin_amdgcn_readlane(got, l),
                           __builtin_amdgcn_readlane(cv.y, l));
        return false;
      }
    }
  }
  return true;
}

// A wait of ticket t gave up (one thread): raise the launch's fault flag
// (-(kind * 1000000 + t)); the workgroup whose code wins it also fills the
// fault record (kDagFault*), which the host reads to name the stuck counter,
// its producers and how far the launch had drawn.  Plain agent-scope atomic
// stores: the record is read after the launch.
// Every wait that ran out of time (not one that gave up after another's
// fault) also records its ticket in kFaultFirstStuck (as INT_MAX - ticket,
// max-combined): the smallest stuck ticket, where a stuck chain starts.
__device__ void dag_fault(int *flag, int *counters, int n_tiles, const int *ticket, int kind, int t, int3 unmet,
                          bool expired) {
  int *f = counters + 2 * n_tiles + kDagOffFault;
  if (expired) __hip_atomic_fetch_max(f + kFaultFirstStuck, INT_MAX - t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (atomicCAS(flag, 0, -(kind * 1000000 + t)) != 0) return;
  const int v[kFaultFirstStuck] = {t, kind, unmet.x, unmet.y, unmet.z,
                                   ld_acquire_relaxed(const_cast<int *>(ticket)),
                                   ld_acquire_relaxed(counters + 2 * n_tiles + kDagOffInflight), (int)blockIdx.x};
#pragma unroll
  for (int i = 0; i < kFaultFirstStuck; ++i)   // (kFaultFirstStuck itself is max-combined above)
    __hip_atomic_store(f + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// all threads: drain this workgroup's write-through stores before thread 0
// bumps a counter
__device__ __forceinline__ void dag_release(int tid) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// C = A B^T for two 64x64 LDS tiles (pitch LQ), 4 waves x 32x32; acc layout
// of the f64 MFMA (col = lane & 15, row = (lane >> 4) + 4 reg)
__device__ __forceinline__ void gemm64_nt(const double *sA, const double *sB, int tid, dbl4 acc[4]) {
  const int w = tid >> 6, lane = tid & 63;
  const int r0 = (w >> 1) * 32, c0 = (w & 1) * 32;
  const int li = lane & 15, lk = lane >> 4;
#pragma unroll 4
  for (int kk = 0; kk < T64 / 4; ++kk) {
    const int kc = kk * 4 + lk;
    const double a0 = sA[(r0 + li) * LQ + kc];
    const double a1 = sA[(r0 + 16 + li) * LQ + kc];
    const double b0 = sB[(c0 + li) * LQ + kc];
    const double b1 = sB[(c0 + 16 + li) * LQ + kc];
    acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0], 0, 0, 0);
    acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[1], 0, 0, 0);
    acc[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[2], 0, 0, 0);
    acc[3] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[3], 0, 0, 0);
  }
}

// The first panel beside which the fused solve's steps may run (4: never).
// cfg3 k_factor_dag: 3 -> 660.8, 4 -> 665.1, 2 -> 676.1, 1 -> 683.8 us
// (interleaved, one box): waves 1-3 working beside the earlier panels slow
// wave 0's diagonal blocks (the same steps alone on the chip cost nothing,
// tools/pipe_bench.hip).
#ifndef ARSLAM_PIPE_FROM
#define ARSLAM_PIPE_FROM 3
#endif
constexpr int kPipeFrom = ARSLAM_PIPE_FROM;
#ifndef ARSLAM_PIPE_W2
#define ARSLAM_PIPE_W2 1
#endif
constexpr int kPipeW2 = ARSLAM_PIPE_W2;   // the wave (1-3) that also takes row block 3

struct DagArgs {
  double *S;
  int T;
  double *Ld;                 // [2T][4096]: L_kk then L_kk^{-1}
  double *ltd;                // [T][kLtdSize]: the 16x16 diagonal-block inverses of each L_kk
  // (the task, its fused TRSM, continuation, fold and update-item fields are
  // all in the ticket's record; LltPlan::dag_rec)
  const int *rec;             // [n_tasks][32] each ticket's record (DagRecField)
  const int2 *ks_tiles;       // [ks] operand tile ids of an update column
  const int *ks;              // [ks] the column of each (a multi-column fold's own term test)
  int *claimed;               // [n_tasks] continuation targets: claimed by the predecessor or the drawer
  const int2 *waits;          // wait lists {counter, value} (ranges in the records)
  int *counters;              // ready[n_tiles] | applied[n_tiles] | ticket
  int n_tiles;
  int n_tasks;
  double *part;
  int *split_cnt;
  int *flag;
  int t_begin, t_end;         // this launch's tickets (one phase of a multi-rank plan, or all)
  int *ticket;                // its ticket counter
  int *progress;              // debug: [grid][4] host-visible (ticket, phase, task type, spins)
  unsigned long long *trace;  // debug: [n_tasks][8] s_memrealtime at draw / waits met / end, workgroup, sub-phases
  // tiles >= first_store are fill tiles the Schur gather does not write -- S
  // never clears them, and their first update stores 0 - acc instead of
  // reading the tile (INT_MAX: every tile is cleared and read-modify-written)
  int first_store;
  int *started;               // workgroups of this launch that have started (the claim cap's base)
  int wg_limit;               // debug: workgroups with blockIdx.x >= wg_limit return at once (INT_MAX: none)
};

// A ticket's 32-int record: two scalar loads in flight, one wait (the record
// array is read-only in the launch).  From LDS for a claimed continuation
// (its predecessor copied it there beside its POTRF).
typedef int int16v __attribute__((ext_vector_type(16)));
struct DagRecV {
  int16v a, b;
  __device__ __forceinline__ int operator[](int i) const { return i < 16 ? a[i] : b[i - 16]; }
};
__device__ __forceinline__ DagRecV load_rec(const int *p) {
  DagRecV r;
  asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx16 %1, %2, 0x40\n\ts_waitcnt lgkmcnt(0)"
               : "=s"(r.a), "=s"(r.b)
               : "s"(p)
               : "memory");
  return r;
}
__device__ __forceinline__ DagRecV lds_rec(const int *s) {
  DagRecV r;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    r.a[i] = __builtin_amdgcn_readfirstlane(s[i]);
    r.b[i] = __builtin_amdgcn_readfirstlane(s[16 + i]);
  }
  return r;
}

__device__ __forceinline__ unsigned long long realtime() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

#define DAG_PROGRESS(slot, v)                                                                  \
  do {                                                                                         \
    if (a.progress && tid == 0)                                                                \
      __hip_atomic_store(a.progress + 4 * blockIdx.x + (slot), (v), __ATOMIC_RELAXED,          \
                         __HIP_MEMORY_SCOPE_SYSTEM);                                            \
  } while (0)

__global__ __launch_bounds__(256, kDagWorkgroupsPerCu) void k_factor_dag(DagArgs a) {
  // one LDS array carved per task type (POTRF: D, X, inv, LTd; GEMMs: sA, sB)
  __shared__ __attribute__((aligned(16))) double lds[2 * T64 * LQ + T64 + 4 * 16 * LI + 12 + 16 + T64];
  double *D = lds, *X = lds + T64 * LQ, *inv = X + T64 * LQ, *LTd = inv + T64;
  // [0] ticket, [1] bad, [2] ok, [3] last, [4] claimed continuation, [7] the POTRF fold's first blocks done,
  // [12..15] fused solve steps done,
  // [6] its fetch requested, [8..10] the POTRF pipeline's flags, [11] thirds of that tile loaded,
  // [16..17] the continuation's A_kk halves in D, [20..21] its early waits seen met by waves 2-3
  int *sh = reinterpret_cast<int *>(LTd + 4 * 16 * LI);
  int *sh_rec = sh + 24;                        // the claimed continuation's record
  double *colx = LTd + 4 * 16 * LI + 12 + 16;   // POTRF pivot scratch (X stays free for the prefetch)
  int *ready = a.counters, *applied = a.counters + a.n_tiles, *ticket = a.ticket;
  // claimed continuation targets in flight.  A target is claimed once its
  // EARLY waits are all drawn; its late waits may name undrawn tickets, so at
  // most half the grid may hold claimed targets: the other workgroups can
  // always draw the lowest unfinished ticket, whose producers are all done.
  //
  // "Half the grid" is not enough when fewer workgroups than the grid are
  // resident (another process on the GPU, several ranks sharing one): every
  // resident workgroup could then hold a claimed target while the ones that
  // would draw never start.  So the cap is half the workgroups that have
  // *started* (counted on entry, read at each claim): a started workgroup
  // stays resident until every ticket is drawn, so at least half of the
  // started ones hold no claimed target and can draw the lowest unfinished
  // ticket (dag_simulate's started-k schedules).
  int *inflight = a.counters + 2 * a.n_tiles + kDagOffInflight;
  if ((int)blockIdx.x >= a.wg_limit) return;   // (debug: only wg_limit workgroups ever start)
  if (threadIdx.x == 0) __hip_atomic_fetch_add(a.started, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // Per-CU "POTRF running" flags (performance only: a wrong or stale flag
  // costs a bounded pause, never a result).  The 64x64 POTRF is a chain of
  // dependent LDS/VALU steps on one wave; the other workgroup on its CU runs
  // update GEMMs that take SIMD issue and LDS bandwidth from it (the POTRF
  // phase takes ~11 us in the contended half of the factorization, 8.5
  // beside idle neighbours), so updates on that CU hold their next GEMM
  // (at most ~55 us) while the flag is up: cfg3 k_factor_dag 689 -> ~675 us.
  // A flag held across the POTRF task's late wait made it 2x slower (the
  // wait can need an update the flag holds).
  int *cu_flag = a.counters + 2 * a.n_tiles + kDagOffCuFlags;
  int cu_key = 0;
  {
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    cu_key = (int)(((xcc & 7u) << 8) | ((hw >> 8) & 0xffu));   // XCC, SE, SH, CU
  }
  // Continuation targets stay ordinary tickets with a claim flag.  The
  // predecessor's workgroup claims its target (before publishing the tile the
  // target waits for, so it wins whenever it claims) if every task the target
  // waits on has been drawn -- then the target only waits on running tasks --
  // and runs it at once, the folded tile still in LDS.  Otherwise the
  // workgroup that drew the target claims and runs it once its waits are met.
  int next = -1, prev_k = -1;
  bool next_met = false;   // a claimed continuation whose early waits were already seen met
  // A fast continuation: its predecessor's waves went straight on to it
  // without the predecessor's closing barriers (wave 1 still waiting for the
  // solved tile's store acknowledgements) -- see the end of the POTRF task.
  bool fast_next = false;
  for (;;) {
    // thread coordinates re-derived per task from a laundered threadIdx: the
    // per-lane LDS/tile addresses of every task type are then computed where
    // they are used instead of being hoisted out of the loop and spilled
    int tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    const int w = tid >> 6, lane = tid & 63;
    const int r0 = (w >> 1) * 32, c0 = (w & 1) * 32;
    const int li = lane & 15, lk = lane >> 4;
    const bool cont = next >= 0;
    if (!cont) {
      if (tid == 0) sh[0] = a.t_begin + atomicAdd(ticket, 1);
      __syncthreads();
      next = sh[0];
      __syncthreads();
    }
    const int t = __builtin_amdgcn_readfirstlane(next);
    const int pk = prev_k;   // a claimed continuation: the predecessor's column (its L_{k,pk} is in X)
    const bool premet = cont && next_met;   // (only for the claimed target it was polled for)
    const bool fast = cont && fast_next;
    next = -1;
    prev_k = -1;
    next_met = false;
    fast_next = false;
    DAG_PROGRESS(0, t);
    DAG_PROGRESS(1, 1);
    if (t >= a.t_end) break;
    const DagRecV r = cont ? lds_rec(sh_rec) : load_rec(a.rec + (long)t * kDagRecInts);
    const int4 task = make_int4(r[kRecType], r[kRecY], r[kRecZ], r[kRecW]);
    DAG_PROGRESS(2, task.x);
    if (a.trace && tid == 0) { a.trace[8L * t] = realtime(); a.trace[8L * t + 3] = blockIdx.x; }
    const int2 sub = make_int2(r[kRecSub], r[kRecLate]);
    if (w == 0) {
      // (sub.y: the end of the early waits; the late ones are a fused TRSM's,
      // or a folded TRSM's L_kk)
      int3 unmet;
      bool expired = false;
      const bool ok =
          premet || dag_wait(a.counters, a.waits, r[kRecWait0], sub.y, a.flag, lane, task.x != 2, &unmet, &expired);
      if (lane == 0) {
        if (!ok) dag_fault(a.flag, a.counters, a.n_tiles, ticket, 1, t, unmet, expired);   // stuck ticket, for diagnosis
        // a drawn continuation target: run it only if its predecessor did not claim it
        sh[2] = (cont || r[kRecMaxdep] < 0 || atomicCAS(a.claimed + t, 0, 1) == 0) ? 1 : 0;
      }
    }
    if (!fast) {
      __syncthreads();
      if (!sh[2]) continue;
    }
    DAG_PROGRESS(1, 2);
    if (a.trace && tid == 0) a.trace[8L * t + 1] = realtime();
    // the chain tasks (POTRF, TRSM) win SIMD arbitration over co-resident updates
    if (task.x != 2) __builtin_amdgcn_s_setprio(3);
    if (task.x == 0) {
      // ---- POTRF k: publish L_kk and its 16x16 block inverses, then (off the
      // critical path) the full inverse for the backward solve ----
      const int k = task.y;
      // The continuation's A_kk, prefetched by waves 2-3 into registers beside
      // the last POTRF panel once its early waits are met (apf: the target
      // folds this task's solved tile alone, so A_kk is all it loads).  This
      // task's tile stores are then made by waves 0-1 alone, so their release
      // (s_waitcnt vmcnt(0)) never waits for those loads; waves 2-3 move the
      // registers into D after the fused solve, as the target's A_kk.
      const int c = sub.x >= 0 ? r[kRecCont] : -1;
      const int apf_tile = sub.x >= 0 ? r[kRecContAkk] : -1;
      const bool apf = apf_tile >= 0;
      const double *apf_src = a.S + (long)max(apf_tile, 0) * (T64 * T64);
      bool ap_met = false;   // waves 2-3: the target's early waits seen met beside the last panel
      int c_rec = 0;         // wave 3 (lanes 0-31): the target's record, bound for sh_rec
      int2 c_wait = make_int2(0, 0);   // waves 2-3: lane q's early wait of the target
      dbl2 apv[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) apv[u] = dbl2{0.0, 0.0};
      bool ap_ok = false;
      // this CU's flag is up from the fold to the end of the factorization,
      // never across a wait (an update held on this CU may be what a wait
      // needs; the early waits are met here, the late ones come after)
      if (tid == 0)
        __hip_atomic_store(cu_flag + cu_key, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int4 fit = make_int4(0, r[kRecQ0], r[kRecQ1], 0);
      const bool akk_in_d = cont && sh[16] && sh[17];   // (its predecessor's waves 2-3 put A_kk in D)
      // a one-column folded update runs inside the factorization (fold_f: its
      // L_kj tile in X -- the predecessor's solved tile for a continuation,
      // else loaded beside A_kk); several columns fold first, as one GEMM pass
      const bool fold_in = task.z >= 0 && fit.z - fit.y == 1;
      if (fold_in) {
        const double *Akk = a.S + (long)task.w * (T64 * T64);
        if (cont && r[kRecFoldK0] == pk) {
          if (!akk_in_d) load_tile_wt(Akk, D, tid);
        } else load_two_tiles_wt(Akk, D, a.S + (long)r[kRecFoldTile0] * (T64 * T64), X, tid);
      } else if (task.z >= 0) {
        // folded final update: A_kk -= sum over the item's columns j of L_kj L_kj^T
        const int4 it = fit;
        dbl4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
        // A_kk (final: the task's waits are met) straight into the MFMA
        // accumulator layout, sc1 loads in flight during the fold's GEMMs
        double akk[16];
        {
          const double *Akk = a.S + (long)task.w * (T64 * T64);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int rb = r0 + (q >> 1) * 16, cb = c0 + (q & 1) * 16;
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) akk[4 * q + reg] = ld_wt(Akk + (rb + lk + 4 * reg) * T64 + cb + li);
          }
        }
        // (the same products in the same order whether the task was drawn
        // or claimed: a claimed continuation takes the term of its
        // predecessor's column from the tile that task just solved, still in X)
        for (int q = it.y; q < it.z; ++q) {
          if (cont && a.ks[q] == pk) {
            gemm64_nt(X, X, tid, acc);
            continue;
          }
          if (q > it.y) __syncthreads();
          load_tile_wt(a.S + (long)a.ks_tiles[q].x * (T64 * T64), D, tid);
          __syncthreads();
          gemm64_nt(D, D, tid, acc);
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rb = r0 + (q >> 1) * 16, cb = c0 + (q & 1) * 16;
#pragma unroll
          for (int reg = 0; reg < 4; ++reg) D[(rb + lk + 4 * reg) * LQ + cb + li] = akk[4 * q + reg] - acc[q][reg];
        }
      } else {
        load_tile_wt(a.S + (long)task.w * (T64 * T64), D, tid);
      }
      if (!fast) __syncthreads();
      if (a.trace && tid == 0) a.trace[8L * t + 4] = realtime();
      // The fused TRSM's tile: wave 1 fetches it into X while wave 0 factors
      // the first diagonal block, if its late waits are already met;
      // otherwise it is waited for and loaded after L_kk is published.
      const double *pf_src = sub.x >= 0 ? a.S + (long)sub.x * (T64 * T64) : nullptr;
      const int pw0 = sub.y, pw1 = r[kRecWait1];
      // lane q's late wait of the fused tile (loaded now, polled beside the panels)
      const int2 pw_wait = (sub.x >= 0 && pw0 + lane < pw1) ? a.waits[pw0 + lane] : make_int2(0, 0);
      // A tile whose waits were not met at panel 0 is polled again by wave 1
      // beside panels 1 and 2 (the request in sh[6]) and fetched by waves 1-3,
      // a third each, beside the next panel: on the late elimination-tree chain
      // the tile's last update lands a few microseconds into the POTRF
      // (cfg3 k_factor_dag 758 -> 736 us).
      if (tid == 0 && !fast) {   // (a fast continuation: reset by its predecessor)
        sh[6] = 0;
        sh[12] = sh[13] = sh[14] = sh[15] = 0;   // the fused solve's column steps done per row block
        sh[18] = 0;                              // beside the last panel: wave 1's take / skip (1 / 2)
      }
      // sh[11]: thirds of the tile loaded into X (3: all; set to 0 by the
      // pipeline's start).  Each wave decides for its own third: a wave that
      // reaches a panel late must not take another wave's completed third for
      // the whole tile.
      bool third_done = false;
      // The fused solve's first steps beside the last panel: once the whole
      // tile is in X, waves 1-3 apply the solve's column steps 0-2 while wave 0
      // factors the last diagonal block (wave w takes row block w - 1, and wave
      // kPipeW2 row block 3 as well), so only step 3 remains after the factorization (the
      // same products in the same order).  Beside the earlier panels they slow
      // the factorization more than they save (kPipeFrom).
      int sdone = 0;
      const bool ok = blocked_potrf64_async(D, inv, LTd, sh + 1, sh + 8, tid, colx, [&](int p, int wv, int ln) {
        auto fetch_third = [&]() {
        auto poll = [&]() {
          if (!pf_src || pw1 - pw0 > 64) return false;
          const int q = pw0 + ln;
          const int got = q < pw1 ? ld_acquire_relaxed(a.counters + pw_wait.x) : 0;
          return __builtin_amdgcn_ballot_w64(q < pw1 && got < pw_wait.y) == 0;
        };
        int lnl = ln;   // laundered: the prefetch addresses are formed here, not hoisted and spilled
        asm volatile("" : "+v"(lnl));
        if (p == 0) {   // (X may still hold the fold's operand: the thirds go out beside panel 1)
          if (wv == 1 && poll() && ln == 0) *as_lds(sh + 6) = -1;
          return;
        }
        if (third_done || lds_get(sh + 11) >= 3) return;
        const int req = lds_get(sh + 6);
        // not requested yet: wave 1 polls beside panels 1 and 2, and beside the
        // last panel for all three waves (sh[18]); each then takes its own third
        bool take = req != 0 && req < p;
        if (req == 0) {
          if (p < 3) {
            if (wv == 1 && poll() && ln == 0) *as_lds(sh + 6) = p;
          } else {
            // one decision for waves 1-3 (wave 1 polls), so that a wave that
            // takes its third knows the other two do as well
            if (!pf_src || pw1 - pw0 > 64) {
              take = false;
            } else if (wv == 1) {
              take = poll();
              lds_set(sh + 18, take ? 1 : 2);
            } else {
              lds_wait(sh + 18, 1);
              take = lds_get(sh + 18) == 1;
            }
          }
        }
        if (take) {   // the three thirds, one batch of sc1 loads each
          // 2048 16-byte elements of the 64x64 tile: wave w takes e in [(w-1)*683, min(w*683, 2048))
          const int e0 = (wv - 1) * 683, e1 = min(wv * 683, 2048);
          const double *p11[11];
          dbl2 v[11];
#pragma unroll
          for (int u = 0; u < 11; ++u) p11[u] = pf_src + 2 * min(e0 + u * 64 + lnl, e1 - 1);
          ld_wt16x11(p11, v);
#pragma unroll
          for (int u = 0; u < 11; ++u) {
            const int e = e0 + u * 64 + ln, r = e >> 5, c2 = (e & 31) * 2;
            if (e < e1) *reinterpret_cast<dbl2 *>(X + r * LQ + c2) = v[u];
          }
          third_done = true;
          lds_add(sh + 11, ln);
        }
        };
        // (beside the last panel the continuation's counters are read first,
        // so their round trip overlaps the fused tile's)
        int c_got = 0;
        bool c_mine = false;
        if (p == 3 && c >= 0 && wv >= 2 && r[kRecContLate] - r[kRecContWait0] <= 64) {
          const int q = r[kRecContWait0] + ln;
          c_mine = q < r[kRecContLate] && c_wait.x != sub.x;   // (the tile this task solves counts as met)
          if (c_mine) c_got = ld_acquire_relaxed(a.counters + c_wait.x);
        }
        fetch_third();
        // waves 2-3 and the continuation target: its record into LDS (wave 3,
        // issued beside panel 1, stored beside panel 2), its early-wait list
        // (beside panel 2) and their counters (beside panel 3, where wave 0
        // waits for nothing from them): loads in flight across a panel, so no
        // round trip delays an update round wave 0 waits for
        if (c >= 0 && wv >= 2) {
          const int cw0 = r[kRecContWait0], cw1 = r[kRecContLate];
          if (p == 1 && wv == 3 && ln < kDagRecInts) c_rec = a.rec[(long)c * kDagRecInts + ln];
          if (p == 2) {
            if (wv == 3 && ln < kDagRecInts) sh_rec[ln] = c_rec;
            const int q = cw0 + ln;
            if (q < cw1) c_wait = a.waits[q];
          }
          if (p == 3) {
            const bool met = cw1 - cw0 <= 64 && __builtin_amdgcn_ballot_w64(c_mine && c_got < c_wait.y) == 0;
            if (ln == 0) sh[20 + wv - 2] = met ? 1 : 0;
            ap_met = met && apf;
          }
        }
        // beside the last panel every wave that took its third waits for the
        // other two (they took theirs too), so the solve's steps 0-2 always run
        // here once the tile is in, not only when all thirds landed by chance
        // (cfg3 k_factor_dag 605.9 -> 601.3 us, cfg2 207.1 -> 205.6, same-box A/B)
        if (p == 3 && third_done && sdone < 3) lds_wait(sh + 11, 3);
        if (kPipeFrom <= 3 && pf_src && p >= kPipeFrom && sdone < p && lds_get(sh + 11) >= 3) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
          for (int st = sdone; st < p; ++st) {
            trsm_step(X, D, LTd, wv - 1, st, ln);
            if (wv == kPipeW2) trsm_step(X, D, LTd, 3, st, ln);
          }
          sdone = p;
          if (ln == 0) {
            sh[12 + wv - 1] = sdone;
            if (wv == kPipeW2) sh[15] = sdone;
          }
        }
      }, X, fold_in, sh + 7, fast ? sh + 22 : nullptr);   // (a flag, not a nullable LDS pointer: hipcc mis-selects that null check)
      // A fused solve whose tile is already in X has no wait: the CU's flag
      // stays up through it too (the solve is the link's next stretch of the
      // chain; cfg3 k_factor_dag 621.9 -> 604.2 us, same-box A/B)
      const bool keep_flag = sub.x >= 0 && sh[11] >= 3;
      if (tid == 0 && !keep_flag)
        __hip_atomic_store(cu_flag + cu_key, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (a.trace && tid == 0) a.trace[8L * t + 5] = realtime();
      if (!ok && tid == 0) {
        int first = 0;
        while (first < T64 && D[first * LQ + first] > 0.0) ++first;
        atomicCAS(a.flag, 0, 1 + k * T64 + first);
      }
      double *ltd_g = a.ltd + (long)k * kLtdSize;
      // (Measured slower: L_kk stored by one wave and released beside the
      // solve or by the continuation -- the other TRSMs of the column, on the
      // path to the continuation's fused tile, then start later.)
      store_tile_wt(a.Ld + (long)k * T64 * T64, D, tid, true);
      for (int e = tid; e < kLtdSize / 2; e += 256)
        st_wt16(ltd_g + 2 * e, *reinterpret_cast<const dbl2 *>(LTd + 2 * e));
      dag_release(tid);
      if (tid == 0) __hip_atomic_fetch_add(ready + task.w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (a.trace && tid == 0) a.trace[8L * t + 6] = realtime();
      if (sub.x >= 0) {
        // fused TRSM of the parent's tile against the L_kk still in LDS
        const bool pref = sh[11] >= 3;   // (written inside the POTRF, barriers since)
        if (!pref) {
          if (w == 0) {
            int3 unmet;
            bool expired = false;
            const bool ok2 = dag_wait(a.counters, a.waits, sub.y, r[kRecWait1], a.flag, lane, true, &unmet, &expired);
            if (!ok2 && lane == 0) dag_fault(a.flag, a.counters, a.n_tiles, ticket, 3, t, unmet, expired);
          }
          __syncthreads();
        }
        double *Ct = a.S + (long)sub.x * (T64 * T64);
        // The continuation claim's round trips ride along the solve instead of
        // following it: the ticket count and the in-flight reservation go out
        // now, the claim itself after the solve, answered during the tile's
        // stores (its target's early waits were polled beside the last POTRF
        // panel, sh[20..21]: a claimed target whose waits were seen met skips
        // its own poll).
        int tk_seen = 0, infl_old = 0, started_seen = 0;
        if (c >= 0 && tid == 0) {
          tk_seen = ld_acquire_relaxed(ticket);
          started_seen = ld_acquire_relaxed(a.started);
          infl_old = atomicAdd(inflight, 1);
        }
        if (!pref) load_tile_wt(Ct, X, tid);
        if (ap_met) {   // waves 2-3: the continuation's A_kk in flight during the solve
          int t2 = tid - 128;
          asm volatile("" : "+v"(t2));
          ld_wt16x16_issue(apf_src, t2, apv);
          ap_ok = true;
        }
        __syncthreads();
        // blocked_trsm64, its steps inline (row block w per wave), from the
        // first step not applied beside the last panel
        const int s0 = pref ? sh[12 + w] : 0;
        for (int st = s0; st < 2; ++st) trsm_step(X, D, LTd, w, st, lane);
        // claim the continuation target before the tile is published: its
        // drawer waits for this tile, so it cannot have claimed it yet.  (The
        // CAS goes out here and is answered beside the last two steps.)
        const bool want = c >= 0 && tid == 0 && a.t_begin + tk_seen > r[kRecContMaxdep] && infl_old < started_seen / 2;
        int cas_old = 1;
        if (want) cas_old = atomicCAS(a.claimed + c, 0, 1);
        for (int st = max(s0, 2); st < 4; ++st) trsm_step(X, D, LTd, w, st, lane);
        if (keep_flag && tid == 0)
          __hip_atomic_store(cu_flag + cu_key, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef ARSLAM_FAST_CONT
        // whether A_kk comes in D, before the barrier; the claim's answer (the
        // CAS issued beside steps 1-2) is read by tid 0 after it, while wave 1
        // issues the tile's stores and waves 2-3 move A_kk, and published in
        // sh[5] (1 + claimed target, 0 until then)
        if (tid == 0) sh[5] = sh[22] = sh[23] = 0;   // (a fast continuation's start flags, below)
        if (w >= 2 && lane == 0) sh[16 + w - 2] = ap_ok ? 1 : 0;
        __syncthreads();
        if (tid == 0) {
          const int cl = want && cas_old == 0 ? c : -1;
          if (c >= 0 && cl < 0) atomicSub(inflight, 1);
          sh[4] = cl;
          lds_set(sh + 5, 1);
        }
        // A fast continuation (the claimed target's early waits were seen met,
        // its A_kk is in registers, and it folds this task's column alone): the
        // waves go straight on to it.  Wave 1 stores the solved tile, waits
        // for the acknowledgements and publishes the tile -- at the time the
        // barrier version would -- while wave 0 starts the target's fold and
        // first diagonal block: the acknowledgement round trip and the two
        // closing barriers, the target's start barriers and its flag resets
        // leave the chain.  Waves 2-3 move A_kk into D (L_kk's last reader was
        // the solve) and count themselves in sh[23]; tid 0 resets the target's
        // POTRF flags now (every reader of them is past the barrier) and sets
        // sh[22].  Wave 1's first fold block, (1, 0), is needed only after wave
        // 0's first diagonal block.
        // wave 1 stores the solved tile, waves 2-3 move the continuation's
        // A_kk into D (free: L_kk's last reader was the solve)
        if (w == 1) store_tile_wt<64>(Ct, X, tid - 64, false);
        lds_wait(sh + 5, 1);
        const int claim = sh[4];
        const bool fc = kFastCont && claim >= 0 && sh[20] && sh[21] && sh[16] && sh[17] && sh_rec[kRecZ] >= 0 &&
                        sh_rec[kRecQ1] - sh_rec[kRecQ0] == 1 && sh_rec[kRecFoldK0] == k;
        if (w >= 2) {
          if (ap_ok) {
            ld_wt16x16_wait(apv);
            const int t2 = tid - 128;
#pragma unroll
            for (int u = 0; u < 16; ++u) {
              const int e = u * 128 + t2, row = e >> 5, c2 = (e & 31) * 2;
              *reinterpret_cast<dbl2 *>(D + row * LQ + c2) = apv[u];
            }
          }
          if (fc) lds_add(sh + 23, lane);
        }
        // (wave 1 alone waits for the stores' acknowledgements; releasing
        // the tile from the continuation instead was measured slower)
        if (w == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (fc) {
          if (w == 1 && lane == 0) {
            __hip_atomic_fetch_add(ready + sub.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (a.trace) a.trace[8L * t + 7] = realtime();
          }
          if (tid == 0) {
            sh[1] = 0;                                   // the target POTRF's bad flag
            sh[7] = sh[8] = sh[9] = sh[10] = sh[11] = 0;   // its fold count and pipeline flags
            sh[18] = 0;
            sh[6] = 0;
            sh[12] = sh[13] = sh[14] = sh[15] = 0;
            if (a.trace) a.trace[8L * t + 3] = blockIdx.x | ((unsigned long long)(1 | 2 | (pref ? 4 : 0) | 8 | 16 | 32) << 32);
            lds_set(sh + 22, 1);
          }
          fast_next = true;
        } else {
          __syncthreads();
          if (tid == 0) __hip_atomic_fetch_add(ready + sub.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (a.trace && tid == 0) {
            a.trace[8L * t + 7] = realtime();
            // (debug flags above the workgroup: premet, A_kk prefetched into D, fused tile prefetched,
            // the continuation's early waits seen met, claimed)
            const unsigned long long fl = (premet ? 1 : 0) | (akk_in_d ? 2 : 0) | (pref ? 4 : 0) |
                                          (sh[20] && sh[21] ? 8 : 0) | (sh[4] >= 0 ? 16 : 0);
            a.trace[8L * t + 3] = blockIdx.x | (fl << 32);
          }
          __syncthreads();
        }
        next = claim;
        next_met = next >= 0 && sh[20] && sh[21];
#else
        __syncthreads();
        // wave 1 stores the solved tile, waves 2-3 move the continuation's
        // A_kk into D (free: L_kk's last reader was the solve)
        if (w == 1) {
          store_tile_wt<64>(Ct, X, tid - 64, false);
        } else if (w >= 2) {
          if (ap_ok) {
            ld_wt16x16_wait(apv);
            const int t2 = tid - 128;
#pragma unroll
            for (int u = 0; u < 16; ++u) {
              const int e = u * 128 + t2, row = e >> 5, c2 = (e & 31) * 2;
              *reinterpret_cast<dbl2 *>(D + row * LQ + c2) = apv[u];
            }
          }
          if (lane == 0) sh[16 + w - 2] = ap_ok ? 1 : 0;
        }
        if (tid == 0) {
          const int claim = want && cas_old == 0 ? c : -1;
          if (c >= 0 && claim < 0) atomicSub(inflight, 1);
          sh[4] = claim;
        }
        // (wave 1 alone waits for the stores' acknowledgements; releasing
        // the tile from the continuation instead was measured slower)
        if (w == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_fetch_add(ready + sub.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.trace && tid == 0) {
          a.trace[8L * t + 7] = realtime();
          // (debug flags above the workgroup: premet, A_kk prefetched into D, fused tile prefetched,
          // the continuation's early waits seen met, claimed)
          const unsigned long long fl = (premet ? 1 : 0) | (akk_in_d ? 2 : 0) | (pref ? 4 : 0) |
                                        (sh[20] && sh[21] ? 8 : 0) | (sh[4] >= 0 ? 16 : 0);
          a.trace[8L * t + 3] = blockIdx.x | (fl << 32);
        }
        __syncthreads();
        next = sh[4];
        next_met = next >= 0 && sh[20] && sh[21];
#endif
        if (next >= 0) prev_k = k;
      }
    } else if (task.x == 3) {
      // ---- INV k: L_kk^{-1} for the backward solve (off the critical chain) ----
      const int k = task.y;
      load_tiles_ltd_wt(a.Ld + (long)k * T64 * T64, D, nullptr, nullptr, a.ltd + (long)k * kLtdSize, LTd, tid);
      __syncthreads();
      blocked_trinv64(D, LTd, X, tid);
      __syncthreads();
      double *Xg = a.Ld + ((long)a.T + k) * T64 * T64;
#pragma unroll 4
      for (int m = 0; m < 16; ++m) {
        const int e = m * 256 + tid, r = e >> 6, c = e & 63;
        Xg[e] = (r >= c) ? X[c * LQ + r] : 0.0;   // read by the next kernel only
      }
    } else if (task.x == 1) {
      // ---- TRSM i,k: L_ik L_kk^T = A_ik, blocked with the 16x16 inverses ----
      const int k = task.z;
      double *Ct = a.S + (long)task.w * (T64 * T64);
      // the tile, L_kk and its block inverses in one round trip
      load_tiles_ltd_wt(Ct, X, a.Ld + (long)k * T64 * T64, D, a.ltd + (long)k * kLtdSize, LTd, tid);
      __syncthreads();
      if (a.trace && tid == 0) a.trace[8L * t + 4] = realtime();
      blocked_trsm64(X, D, inv, LTd, tid);
      if (a.trace && tid == 0) a.trace[8L * t + 5] = realtime();
      store_tile_wt(Ct, X, tid, false);
      dag_release(tid);
      if (tid == 0) __hip_atomic_fetch_add(ready + task.w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      // ---- update item ----
      const int4 it = make_int4(0, r[kRecQ0], r[kRecQ1], r[kRecSid]);
      const int ti = r[kRecTi], tj = r[kRecTj], sid = it.w;
      dbl4 acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
      // The target's in-order wait (its earlier levels applied) is polled
      // beside the first operand fetch; when it is met then, the target's own
      // loads go out before the last GEMM and land during it (one round trip
      // fewer after the GEMM).  (Unsplit items: a split piece stores a partial.)
      double *C = a.S + (long)task.w * (T64 * T64);
      double cv[16];
      bool c_pre = false;
      if (task.z == 0 && task.w >= a.first_store) {   // (0 - acc below: the same bits)
#pragma unroll
        for (int u = 0; u < 16; ++u) cv[u] = 0.0;
        c_pre = true;
      }
      for (int q = it.y; q < it.z; ++q) {
        // (operand tile ids: the first column's in the record, no column -> tile lookup chain)
        const int2 kt = q == it.y ? make_int2(r[kRecTile0I], r[kRecTile0J]) : a.ks_tiles[q];
        if (q > it.y) __syncthreads();
        {   // hold the GEMM while a POTRF runs on this CU (bounded)
          if (tid == 0) {
            for (int spin = 0; spin < 256 &&
                               __hip_atomic_load(cu_flag + cu_key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                 ++spin)
              __builtin_amdgcn_s_sleep(8);
          }
          __syncthreads();
        }
        if (q == it.y && sid < 0 && tid == 0)
          sh[3] = (task.z == 0 || ld_acquire_relaxed(applied + task.w) >= task.z) ? 1 : 0;
        if (ti != tj)   // both operands in one round trip
          load_two_tiles_wt(a.S + (long)kt.x * (T64 * T64), D, a.S + (long)kt.y * (T64 * T64), X, tid);
        else
          load_tile_wt(a.S + (long)kt.x * (T64 * T64), D, tid);
        __syncthreads();
        const bool c_issue = q == it.z - 1 && sid < 0 && sh[3] && !c_pre;
        if (c_issue) {
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int rb = r0 + (u >> 1) * 16, cb = c0 + (u & 1) * 16;
#pragma unroll
            for (int reg = 0; reg < 4; ++reg) cv[4 * u + reg] = ld_wt(C + (rb + lk + 4 * reg) * T64 + cb + li);
          }
          c_pre = true;
        }
        gemm64_nt(D, ti != tj ? X : D, tid, acc);   // a diagonal target: one operand tile, fetched once
      }
      bool apply = true;
      if (sid >= 0) {
        const int2 sp = make_int2(r[kRecSplitN], r[kRecSplitP]);
        double *mine = a.part + (long)(sp.y + (sid & 255)) * 4096;
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int reg = 0; reg < 4; ++reg) st_wt(mine + (4 * q + reg) * 256 + tid, acc[q][reg]);
        dag_release(tid);
        if (tid == 0) {
          const int old = __hip_atomic_fetch_add(a.split_cnt + (sid >> 8), 1, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
          sh[3] = old == sp.x - 1;
        }
        __syncthreads();
        apply = sh[3] != 0;
        if (apply) {
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[q] = dbl4{0, 0, 0, 0};
          for (int c = 0; c < sp.x; ++c) {
            const double *pc = a.part + (long)(sp.y + c) * 4096;
            double v[16];
            const double *p8[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) p8[u] = pc + u * 256 + tid;
            ld_wt8x8(p8, v);
            ld_wt8x8(p8 + 8, v + 8);
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
              for (int reg = 0; reg < 4; ++reg) acc[q][reg] += v[4 * q + reg];
          }
        }
      }
      DAG_PROGRESS(1, 3);
      if (apply && !c_pre) {
        // in level order: wait until the target's earlier levels were applied
        if (tid == 0) {
          long spins = 0;
          int seen;
          WaitTimer tm;
          while ((seen = ld_acquire_relaxed(applied + task.w)) < task.z) {
            __builtin_amdgcn_s_sleep(kPollSleep);
            const bool exp = tm.expired(++spins);
            if (exp || (((spins & 255) == 0) && ld_acquire_relaxed(a.flag) < 0)) {
              dag_fault(a.flag, a.counters, a.n_tiles, ticket, 2, t, make_int3(a.n_tiles + task.w, seen, task.z), exp);
              break;
            }
          }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 4; ++q) {   // (sixteen loads in flight)
          const int rb = r0 + (q >> 1) * 16, cb = c0 + (q & 1) * 16;
#pragma unroll
          for (int reg = 0; reg < 4; ++reg) cv[4 * q + reg] = ld_wt(C + (rb + lk + 4 * reg) * T64 + cb + li);
        }
      }
      if (apply) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int rb = r0 + (q >> 1) * 16, cb = c0 + (q & 1) * 16;
#pragma unroll
          for (int reg = 0; reg < 4; ++reg)
            st_wt(C + (rb + lk + 4 * reg) * T64 + cb + li, cv[4 * q + reg] - acc[q][reg]);
        }
        dag_release(tid);
        if (tid == 0) __hip_atomic_fetch_add(applied + task.w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    DAG_PROGRESS(1, 4);
    if (cont && tid == 0) atomicSub(inflight, 1);   // this claimed target is done
    __builtin_amdgcn_s_setprio(0);
    if (a.trace && tid == 0) a.trace[8L * t + 2] = realtime();
  }
  {
    const int tid = threadIdx.x;
    DAG_PROGRESS(1, 9);
  }
}

// z[j] = L[nR][j], the forward-substituted right-hand side: from S for the
// tiles left of the rhs row's own tile, from that tile's diagonal factor in Ld.
__global__ void k_init_z(const double *__restrict__ S, const int *__restrict__ tid_map, int T,
                         const double *__restrict__ Ld, long nR, long N, double *__restrict__ z) {
  const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= N) return;
  const long kr = nR / T64;
  double v = 0.0;
  if (j < nR) {
    if (j >= kr * T64) v = Ld[kr * T64 * T64 + (nR - kr * T64) * T64 + (j - kr * T64)];
    else v = tile_ptr(S, tid_map, T, (int)kr, (int)(j / T64))[(nR - kr * T64) * T64 + (j % T64)];
  }
  z[j] = v;
}

// Backward solve L^T y = z, level by level from the root.  For a level:
//   k_bs_gather: one workgroup per gathered tile (i,k) (i > k, an ancestor
//     already solved): part_g = L_ik^T y_i, stored to its own slot;
//   k_bs_solve:  one workgroup per column k: sums its gathers' partials in
//     plan order (deterministic: every rank of a sharded solve computes the
//     same bits), then solves L_kk^T y_k = z_k - sum (lane r owns row r,
//     16-row blocks, scalar broadcasts of y).
__global__ __launch_bounds__(256) void k_bs_gather(const double *__restrict__ S,
                                                   const int *__restrict__ tid_map, int T, long nR,
                                                   const int2 *__restrict__ tasks,
                                                   const double *__restrict__ yF,
                                                   double *__restrict__ part_out,
                                                   const int *__restrict__ flag) {
  __shared__ double part[4][T64];
  if (*flag) return;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int2 t = tasks[blockIdx.x];
  const long ri = (long)t.x * T64;
  const double *Lik = tile_ptr(S, tid_map, T, t.x, t.y);
  double a0 = 0.0, a1 = 0.0;
#pragma unroll
  for (int r = w; r < T64; r += 8) {
    const double y0 = (ri + r < nR) ? yF[ri + r] : 0.0;
    const double y1 = (ri + r + 4 < nR) ? yF[ri + r + 4] : 0.0;
    a0 += Lik[r * T64 + lane] * y0;
    a1 += Lik[(r + 4) * T64 + lane] * y1;
  }
  part[w][lane] = a0 + a1;
  __syncthreads();
  if (w == 0) part_out[(long)blockIdx.x * T64 + lane] = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
}

// y_k = L_kk^{-T} (z_k - sum of the column's gathered partials), with the
// inverse X_kk from the panel: y[c] = sum_r X[r][c] acc[r] (4 waves x 16 rows,
// fixed-order combine).  Rows past nR carry acc = 0 and y = 0.
__global__ __launch_bounds__(256) void k_bs_solve(const double *__restrict__ Xinv, long nR,
                                                  const int *__restrict__ cols,
                                                  const int *__restrict__ gbeg,
                                                  const double *__restrict__ z,
                                                  const double *__restrict__ part,
                                                  double *__restrict__ yF,
                                                  const int *__restrict__ flag) {
  __shared__ double accs[T64];
  __shared__ double red[4][T64];
  if (*flag) return;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int k = cols[blockIdx.x];
  const long row0 = (long)k * T64;
  if (w == 0) {
    double acc = 0.0;
    const int ga = gbeg[blockIdx.x], gb = gbeg[blockIdx.x + 1];
    for (int g = ga; g < gb; g += 8) {   // 8 loads in flight, summed in plan order
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(long)min(g + u, gb - 1) * T64 + lane];
#pragma unroll
      for (int u = 0; u < 8; ++u) acc += (g + u < gb) ? v[u] : 0.0;
    }
    accs[lane] = (row0 + lane < nR) ? z[row0 + lane] - acc : 0.0;
  }
  __syncthreads();
  const double *X = Xinv + (long)k * T64 * T64;
  double s = 0.0;
#pragma unroll
  for (int rr = 0; rr < 16; ++rr) {
    const int r = 16 * w + rr;
    s += X[r * T64 + lane] * accs[r];
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && row0 + lane < nR) yF[row0 + lane] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// Persistent backward solve L^T y = z (the launch-per-level pair above as one
// launch).  Ticket b takes column bs_cols[b]; the columns are root level
// first, so every ancestor a column waits for holds an earlier ticket and was
// drawn by a running workgroup (deadlock-free for any grid).  A column task:
//   z_k      from the rhs row (as k_init_z);
//   gathers  nearest ancestor LAST (ancestors finish root-first, so all but
//            the parent's partial are summed while the parent is still being
//            solved): L_ik is prefetched into registers before the wait on
//            done[i], y_i is an sc1 load (written this launch), and the
//            partials are summed in this fixed order, so every rank of a
//            sharded solve computes the same bits;
//   solve    y_k = L_kk^{-T}(z_k - acc) with the prefetched inverse X_kk;
//            wave 0 stores y_k write-through, drains, bumps done[k].
__global__ __launch_bounds__(256) void k_bsolve_dag(const double *__restrict__ S, const int *__restrict__ tid_map,
                                                    int T, const double *__restrict__ Ld, long nR,
                                                    const int *__restrict__ cols, const int2 *__restrict__ gather,
                                                    const int *__restrict__ gbeg, int ncols, double *yF,
                                                    int *counters, int *flag) {
  __shared__ double red[4][T64];
  __shared__ double ys[T64];
  __shared__ int sh[2];
  if (*flag) return;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  int *ticket = counters + T;   // (counters[0..T) are unused: y entries are their own flags)
  const double *Xinv = Ld + (long)T * T64 * T64;
  const long kr = nR / T64;
  for (;;) {
    if (tid == 0) sh[0] = atomicAdd(ticket, 1);
    __syncthreads();
    const int b = sh[0];
    if (b >= ncols) break;
    const int k = cols[b];
    const long row0 = (long)k * T64;
    // the inverse's rows 16w..16w+15 for lane's column, in flight during the gathers
    const double *X = Xinv + (long)k * T64 * T64;
    double xv[16];
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) xv[rr] = X[(16 * w + rr) * T64 + lane];
    double acc = 0.0;   // wave 0: lane's row of sum_i L_ik^T y_i
    bool ok = true;
    for (int g = gbeg[b + 1] - 1; g >= gbeg[b]; --g) {
      const int i = gather[g].x;
      const long ri = (long)i * T64;
      const double *Lik = tile_ptr(S, tid_map, T, i, k);
      double lv[16];   // rows w, w+4, ..., lane's column
#pragma unroll
      for (int m = 0; m < 16; ++m) lv[m] = Lik[(w + 4 * m) * T64 + lane];
      if (w == 0) {
        // y_i is its own ready flag: the entries are kYSentinel until column
        // i's task stores them (8-byte write-through stores, never torn), so
        // the wait is the load itself -- no counter, no drain before it
        double yv = 0.0;
        bool mine = ri + lane < nR;
        long spins = 0;
        WaitTimer tm;
        for (;;) {
          if (mine) {
            yv = ld_wt(yF + ri + lane);
            mine = (unsigned long long)__double_as_longlong(yv) == kYSentinel;
          }
          if (__builtin_amdgcn_ballot_w64(mine) == 0) break;
          __builtin_amdgcn_s_sleep(kBsolveSleep);
          if (tm.expired(++spins) || (((spins & 255) == 0) &&
                                     __builtin_amdgcn_readfirstlane(ld_acquire_relaxed(flag)) != 0)) {
            if (lane == 0) atomicCAS(flag, 0, -(4000000 + b));
            ok = false;
            break;
          }
        }
        if (lane == 0) sh[1] = ok;
        ys[lane] = (ri + lane < nR) ? yv : 0.0;
      }
      __syncthreads();
      if (!sh[1]) break;
      double s = 0.0;
#pragma unroll
      for (int m = 0; m < 16; ++m) s += lv[m] * ys[w + 4 * m];
      red[w][lane] = s;
      __syncthreads();
      if (w == 0) acc += ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
    }
    if (w == 0) {
      double z = 0.0;
      if (row0 + lane < nR) {
        if (k == kr) z = Ld[kr * T64 * T64 + (nR - kr * T64) * T64 + lane];
        else z = tile_ptr(S, tid_map, T, (int)kr, k)[(nR - kr * T64) * T64 + lane];
      }
      ys[lane] = (row0 + lane < nR) ? z - acc : 0.0;
    }
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) s += xv[rr] * ys[16 * w + rr];
    red[w][lane] = s;
    __syncthreads();
    if (w == 0 && row0 + lane < nR)   // (published by the store itself; see the gathers)
      st_wt(yF + row0 + lane, ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane]);
  }
}

// tests only: copy the diagonal factors L_kk into their S tiles
__global__ void k_scatter_diag(double *__restrict__ S, const int *__restrict__ tid_map, int T,
                               const double *__restrict__ Ld) {
  const int k = blockIdx.x;
  double *t = tile_ptr(S, tid_map, T, k, k);
  for (int e = threadIdx.x; e < T64 * T64; e += blockDim.x) t[e] = Ld[(long)k * T64 * T64 + e];
}

}  // namespace

void launch_scatter_diag(const LltPlan &P, double *S, hipStream_t s) {
  hipLaunchKernelGGL(k_scatter_diag, dim3((unsigned)P.T), dim3(256), 0, s, S, P.tile_id, P.T, P.ldiag);
}

namespace {
// One launch zeroing the persistent executors' counters (and the step's
// failure flag) instead of a fill launch per array.
// (with ld.n > 0 also the step's LM diagonal: k_lm_diag's work, one launch less)
__global__ void k_exec_reset(int *flag, int *a, long na, int *b, long nb, int *c, long nc, int *d, long nd,
                             LmDiagArgs ld) {
  const long n = na + nb + nc + nd;
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < ld.nys; e += (long)gridDim.x * blockDim.x)
    ld.ysent[e] = __longlong_as_double((long long)kYSentinel);
  for (long e = (long)blockIdx.x * blockDim.x + threadIdx.x; e < n + ld.n; e += (long)gridDim.x * blockDim.x) {
    if (e < na) a[e] = 0;
    else if (e < na + nb) b[e - na] = 0;
    else if (e < na + nb + nc) c[e - na - nb] = 0;
    else if (e < n) d[e - na - nb - nc] = 0;
    else {
      const long i = e - n;
      const double v = ld.scale[i] * ld.scale[i] * ld.colnorm[i];   // squared column norm of J diag(s)
      ld.diag[i] = fmin(fmax(v, ld.dmin), ld.dmax);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *flag = 0;
}
}  // namespace

void launch_exec_reset(const LltPlan &P, int *flag, hipStream_t s, const LmDiagArgs *ld) {
  const long na = P.n_dag_tasks ? 2 * P.n_tiles + kDagCounterExtra : 0, nb = P.n_dag_tasks, nc = P.n_split,
             nd = P.h_bcols.empty() ? 0 : (long)P.T + 1;
  LmDiagArgs l{};
  if (ld) l = *ld;
  const long n = std::max(na + nb + nc + nd + l.n, l.nys);
  const unsigned grid = (unsigned)std::max<long>(1, std::min<long>((n + 255) / 256, 1024));
  hipLaunchKernelGGL(k_exec_reset, dim3(grid), dim3(256), 0, s, flag, P.dag_counters, na, P.dag_claimed, nb,
                     P.upd_cnt, nc, P.bs_counters, nd, l);
}

ExecReset exec_reset_args(const LltPlan &P, int *flag, double *ysent, long nys) {
  ExecReset r;
  r.flag = flag;
  r.na = P.n_dag_tasks ? 2 * P.n_tiles + kDagCounterExtra : 0;
  r.a = P.dag_counters;
  r.nb = P.n_dag_tasks;
  r.b = P.dag_claimed;
  r.nc = P.n_split;
  r.c = P.upd_cnt;
  r.nd = P.h_bcols.empty() ? 0 : (long)P.T + 1;
  r.d = P.bs_counters;
  r.ysent = ysent;
  r.nys = nys;
  return r;
}

void launch_zero_tiles(const LltPlan &P, double *S, hipStream_t s) {
  if (P.n_tiles) (void)hipMemsetAsync(S, 0, (size_t)P.n_tiles * T64 * T64 * sizeof(double), s);
}

void launch_dense_llt(const LltPlan &P, double *S, int *flag, hipStream_t s, LaunchTiming *timing) {
  if (P.n_split) (void)hipMemsetAsync(P.upd_cnt, 0, P.n_split * sizeof(int), s);
  for (int l = 0; l < P.nlev; ++l) {
    const int np = P.h_panel_off[l + 1] - P.h_panel_off[l];
    hipLaunchKernelGGL(k_panel, dim3((unsigned)np), dim3(256), 0, s, S, P.tile_id, P.T, P.ldiag,
                       P.panel + P.h_panel_off[l], flag);
    const int ni = P.h_item_off[l + 1] - P.h_item_off[l];
    if (ni > 0) {
      const bool rec = timing && timing->used < timing->cap;
      if (rec) (void)hipEventRecord(timing->ev[2 * timing->used], s);
      hipLaunchKernelGGL(k_update, dim3((unsigned)ni), dim3(256), 0, s, S, P.tile_id, P.T, P.upd_targets,
                         P.upd_items + P.h_item_off[l], P.upd_ks, P.upd_split, P.upd_part, P.upd_cnt, flag);
      if (rec) {
        (void)hipEventRecord(timing->ev[2 * timing->used + 1], s);
        timing->used++;
        timing->flops += P.h_upd_flops[l];
      }
    }
  }
}

static int g_dag_wg_limit = INT_MAX;   // debug (arslam_debug_dag_workgroup_limit), process-wide
void set_dag_workgroup_limit(int k) { g_dag_wg_limit = k > 0 ? k : INT_MAX; }

void launch_dense_llt_dag(const LltPlan &P, double *S, int *flag, hipStream_t s, int n_workgroups, int *progress,
                          unsigned long long *trace, bool reset, int phase, long first_store) {
  const int t_begin = phase == 1 ? (int)P.phase_split : 0;
  const int t_end = phase == 0 ? (int)P.phase_split : (int)P.n_dag_tasks;
  if (t_end <= t_begin) return;
  if (reset) {
    (void)hipMemsetAsync(P.dag_counters, 0, (2 * (size_t)P.n_tiles + kDagCounterExtra) * sizeof(int), s);
    (void)hipMemsetAsync(P.dag_claimed, 0, (size_t)P.n_dag_tasks * sizeof(int), s);
    if (P.n_split) (void)hipMemsetAsync(P.upd_cnt, 0, P.n_split * sizeof(int), s);
  }
  DagArgs a{S, P.T, P.ldiag, P.ldiag + 2L * P.T * T64 * T64, P.dag_rec, P.dag_ks_tiles, P.upd_ks, P.dag_claimed,
            P.dag_waits, P.dag_counters, (int)P.n_tiles, (int)P.n_dag_tasks, P.upd_part, P.upd_cnt, flag, t_begin, t_end,
            P.dag_counters + 2 * P.n_tiles + (phase == 1 ? kDagOffTicket1 : kDagOffTicket0), progress, trace,
            (int)std::min<long>(first_store, INT_MAX),
            P.dag_counters + 2 * P.n_tiles + (phase == 1 ? kDagOffStarted1 : kDagOffStarted0), g_dag_wg_limit};
  // A small task graph runs on fewer workgroups (a quarter of its tasks, at
  // least 64): its time is the elimination tree's chain, which runs faster
  // beside fewer co-resident update workgroups (cfg2, 580 tasks: 219.6 us on
  // 128 workgroups against 228.4 on 448; the incremental cfg2 flow's
  // minimizer 1.83 -> 1.79 ms per Solve).  cfg3 (12,625 tasks) keeps the full grid.
  const long ntk = t_end - t_begin;
  // (n_workgroups: at most the resident count, kDagWorkgroupsPerCu per CU --
  // the claim cap, half the grid, must leave resident workgroups free to draw;
  // DESIGN §8b.  The callers clamp it: a HIP query here would sit on the hot path)
  const int grid = (int)std::min<long>(n_workgroups, std::max<long>(std::min<long>(64, ntk), ntk / 4));
  hipLaunchKernelGGL(k_factor_dag, dim3((unsigned)grid), dim3(256), 0, s, a);
}

void launch_dense_back_solve_dag(const LltPlan &P, const double *S, long nR, double *yF, int *flag,
                                 hipStream_t s, int n_workgroups, bool reset) {
  const int ncols = (int)P.h_bcols.size();
  if (ncols == 0) return;
  if (reset) {
    (void)hipMemsetAsync(P.bs_counters, 0, ((size_t)P.T + 1) * sizeof(int), s);
    // y to the "not solved" pattern (both 32-bit halves of kYSentinel are equal)
    static_assert((kYSentinel >> 32) == (kYSentinel & 0xffffffffull), "kYSentinel halves");
    if (nR > 0) (void)hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(yF), (int)(kYSentinel & 0xffffffffull),
                                        2 * (size_t)nR, s);
  }
  const int grid = std::min(n_workgroups, ncols);
  hipLaunchKernelGGL(k_bsolve_dag, dim3((unsigned)grid), dim3(256), 0, s, S, P.tile_id, P.T, P.ldiag, nR, P.bs_cols,
                     P.bs_gather, P.bs_gbeg, ncols, yF, P.bs_counters, flag);
}

void launch_dense_back_solve(const LltPlan &P, const double *S, long nR, double *z, double *yF,
                             const int *flag, hipStream_t s) {
  const long N = (long)P.T * T64;
  hipLaunchKernelGGL(k_init_z, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, S, P.tile_id, P.T, P.ldiag,
                     nR, N, z);
  for (int l = 0; l < P.nlev; ++l) {
    const int g0 = P.h_bsg_off[l], ng = P.h_bsg_off[l + 1] - g0;
    if (ng > 0)
      hipLaunchKernelGGL(k_bs_gather, dim3((unsigned)ng), dim3(256), 0, s, S, P.tile_id, P.T, nR, P.bs_gather + g0, yF,
                         P.bs_part + (long)g0 * T64, flag);
    const int b0 = P.h_bs_off[l], nc = P.h_bs_off[l + 1] - b0;
    hipLaunchKernelGGL(k_bs_solve, dim3((unsigned)nc), dim3(256), 0, s, P.ldiag + (long)P.T * T64 * T64, nR,
                       P.bs_cols + b0,
                       P.bs_gbeg + b0, z, P.bs_part, yF, flag);
  }
}

}  // namespace arslam
