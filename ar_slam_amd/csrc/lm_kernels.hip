// lm_kernels.hip -- per-capture kernels of the LM step (fp64, gfx950).
//
// One 64-lane wavefront per capture (the eliminated Schur e-block).  Lane l
// of a 64-row chunk owns residual row l = 8*obs + 2*corner + {x,y} of that
// capture's observations, so the k = 8 observations of a synthetic capture
// are exactly one wave.  Each lane evaluates its row of the reference's
// residual (projectCorner, ar_slam_util.cpp:131-172; ArucoReprojectionError
// :198-211) and the analytic Jacobian into LDS; the
// wave then forms the capture's normal-equation blocks:
//   U_c = E'E + D_c^2 (6x6), W_c = E'F (6 x (1 + 6 n_tags)), F'F, E'r, F'r
// and writes its Schur contribution F'F - W'U^{-1}W (lower block triangle)
// and F'r - W'U^{-1}E'r to its block-packed slab slot; k_schur_gather sums
// the slab blocks of each destination in capture order into the compact
// tiles of the reduced system.
//
// Every sum is fixed-order (no atomics in any of them): the Schur gather, the
// reductions that feed an LM decision (cost, model cost change, step and
// gradient norms) and the factorization's split updates, so a solve is
// bit-identical run to run.
#include "lm_internal.h"
#include "projection.h"

#include <cfloat>
#include <mutex>
#include <string>
#include <vector>

#include "arslam_lm.h"
#include <cmath>

namespace arslam {

#ifdef ARSLAM_SCHUR_STAMPS
__device__ unsigned long long g_schur_ph[16];
#define SCHUR_STAMP_INIT unsigned long long _st0 = clock64()
#define SCHUR_STAMP(k)                                                         \
  do {                                                                         \
    const unsigned long long _n = clock64();                                   \
    if (threadIdx.x == 0) atomicAdd(&g_schur_ph[k], _n - _st0);                \
    _st0 = _n;                                                                 \
  } while (0)
void debug_read_schur_stamps(unsigned long long *out) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_schur_ph), sizeof(g_schur_ph));
}
#else
#define SCHUR_STAMP_INIT do {} while (0)
#define SCHUR_STAMP(k) do {} while (0)
void debug_read_schur_stamps(unsigned long long *out) {
  for (int i = 0; i < 16; ++i) out[i] = 0;
}
#endif

namespace {


__device__ __forceinline__ long slot_cap(const DevProblem &P, int c) { return 3 + 6L * c; }
__device__ __forceinline__ long slot_tag(const DevProblem &P, int t) { return 3 + 6L * P.nc + 6L * t; }

// does group c evaluate its residuals with the two poses exchanged (its e-block is a tag)?
__device__ __forceinline__ bool group_swapped(const DevProblem &P, int c) {
  return P.cap_kind ? P.cap_kind[c] == kMixTag : P.swap_roles != 0;
}
// a direct group of the mixed e-set (its own pose stays on the reduced side)?
__device__ __forceinline__ bool group_direct(const DevProblem &P, int c) {
  return P.cap_kind && P.cap_kind[c] == kMixDirect;
}

__device__ __forceinline__ double lm_d2(const double *diag, long slot, double radius) {
  const double d = sqrt(diag[slot] / radius);   // lm_diagonal_ = sqrt(diag / radius)
  return d * d;
}

// Fill LDS rows [nr][kRowStride] with rows [row0, row0 + nr) of capture c
// (nrows rows in all, observations from o0): 13 Jacobian entries (scaled by
// the Jacobi scale if scale != nullptr) and the residual in column 13.
// With gout, the unscaled rows are also stored there column-major per capture
// (entry (row, j) at gout + 8 o0 kJStored + jrow_col(j) nrows + row, the
// translation columns once): the Schur and back-substitution passes at the
// same point reload them instead of re-evaluating the projection.
__device__ __forceinline__ void fill_rows(const DevProblem &P, const double *x, const double *scale, int c,
                          int o0, int row0, int nr, int nrows, double *rows, double *gout = nullptr) {
  const double *cam = x;
  const double *cap = x + slot_cap(P, c);
  for (int lr = threadIdx.x; lr < nr; lr += kWave) {
    const int row = row0 + lr;
    const int q = row >> 3, corner = (row >> 1) & 3, comp = row & 1;
    const int obs = o0 + q;
    const int t = P.obs_tag[obs];
    const double *tag = x + slot_tag(P, t);
    double J[13];
    // (tag elimination: the e-block is the problem's tag -- projectCorner
    // still takes the capture first; the Jacobian halves come back as e|f)
    const bool sw = group_swapped(P, c);
    const double r = residual_jacobian_row(cam, sw ? tag : cap, sw ? cap : tag, corner, comp,
                                           P.corners[8L * obs + 2 * corner + comp], J);
    if (sw) {
#pragma unroll
      for (int j = 1; j < 7; ++j) {
        const double v = J[j];
        J[j] = J[j + 6];
        J[j + 6] = v;
      }
    }
    double *dst = rows + (long)lr * kRowStride;
    if (scale) {
      const double *sc = scale + slot_cap(P, c);
      const double *st = scale + slot_tag(P, t);
      dst[0] = J[0] * scale[0];
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        dst[1 + j] = J[1 + j] * sc[j];
        dst[7 + j] = J[7 + j] * st[j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < 13; ++j) dst[j] = J[j];
    }
    dst[13] = r;
    if (gout) {
      double *g = gout + 8L * o0 * kJStored + row;
#pragma unroll
      for (int j = 0; j < 13; ++j)
        if (j < 7 || j > 9) g[(long)jrow_col(j) * nrows] = J[j];
      g[(long)jrow_col(13) * nrows] = r;
    }
  }
}

// LDS rows [row0, row0 + nr) of capture c (nrows rows in all) from the copy
// fill_rows stored at the same point, Jacobi-scaled, and each row's
// reduced-side product
//   qv[row] = F_row . y_F = J_f y_f + J_t . y_F[tag rows]
// formed from the row the lane just scaled (its tag row and y_F loads go out
// beside the Jacobian loads instead of after a barrier).
__device__ __forceinline__ void load_rows_q(const DevProblem &P, const double *scale, const double *yF, double yf, int c, int o0,
                            int row0, int nr, int nrows, double *rows, double *qv) {
  const double *sc = scale + slot_cap(P, c);
  for (int lr = threadIdx.x; lr < nr; lr += kWave) {
    const int row = row0 + lr;
    const double *g = P.jrows + 8L * o0 * kJStored + row;
    const int t = P.obs_tag[o0 + (row >> 3)];
    const int tr = P.tag_row[t];
    double u[kJStored], v[14];
#pragma unroll
    for (int j = 0; j < kJStored; ++j) u[j] = g[(long)j * nrows];
#pragma unroll
    for (int j = 0; j < 14; ++j) v[j] = u[jrow_col(j)];
    const double *st = scale + slot_tag(P, t);
    double yt[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) yt[j] = tr >= 0 ? yF[tr + j] : 0.0;
    double *dst = rows + (long)lr * kRowStride;
    double d[14];
    d[0] = v[0] * scale[0];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      d[1 + j] = v[1 + j] * sc[j];
      d[7 + j] = v[7 + j] * st[j];
    }
    d[13] = v[13];
#pragma unroll
    for (int j = 0; j < 14; ++j) dst[j] = d[j];
    double q = d[0] * yf;
    if (tr >= 0) {
#pragma unroll
      for (int j = 0; j < 6; ++j) q += d[7 + j] * yt[j];
    }
    qv[lr] = q;
  }
}

#ifdef ARSLAM_BACKSUB_RECOMPUTE
// load_rows_q's rows evaluated again at x instead of read back (the same
// products in the same order: fill_rows scales J as load_rows_q scales the
// stored copy, and q is formed from the row as there)
__device__ __forceinline__ void eval_rows_q(const DevProblem &P, const double *x, const double *scale, const double *yF,
                                            double yf, int c, int o0, int row0, int nr, int nrows, double *rows,
                                            double *qv) {
  fill_rows(P, x, scale, c, o0, row0, nr, nrows, rows);
  for (int lr = threadIdx.x; lr < nr; lr += kWave) {
    const int row = row0 + lr;
    const int tr = P.tag_row[P.obs_tag[o0 + (row >> 3)]];
    const double *d = rows + (long)lr * kRowStride;
    double q = d[0] * yf;
    if (tr >= 0) {
#pragma unroll
      for (int j = 0; j < 6; ++j) q += d[7 + j] * yF[tr + j];
    }
    qv[lr] = q;
  }
}
#define ARSLAM_BACKSUB_ROWS(...) eval_rows_q(P, x, __VA_ARGS__)
#else
#define ARSLAM_BACKSUB_ROWS(...) load_rows_q(P, __VA_ARGS__)
#endif

// (a,b) of the e-th entry of the upper triangle of a 6x6 matrix, row-major
__device__ __forceinline__ void upper6(int e, int &a, int &b) {
  a = 0;
  int rem = e;
  while (rem >= 6 - a) { rem -= 6 - a; ++a; }
  b = a + rem;
}

// 6x6 SPD inverse by LLT + two triangular solves against I (Ceres'
// InvertPSDMatrix<full rank>); single lane.
__device__ void inv6(const double *U, double *Ui) {
  double L[36];
#pragma unroll
  for (int i = 0; i < 36; ++i) L[i] = U[i];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    double xj = L[6 * j + j];
#pragma unroll
    for (int p = 0; p < j; ++p) xj -= L[6 * j + p] * L[6 * j + p];
    const double d = sqrt(xj);
    L[6 * j + j] = d;
#pragma unroll
    for (int i = j + 1; i < 6; ++i) {
      double v = L[6 * i + j];
#pragma unroll
      for (int p = 0; p < j; ++p) v -= L[6 * i + p] * L[6 * j + p];
      L[6 * i + j] = v / d;
    }
  }
#pragma unroll
  for (int col = 0; col < 6; ++col) {
    double e[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      double v = (i == col) ? 1.0 : 0.0;
#pragma unroll
      for (int p = 0; p < i; ++p) v -= L[6 * i + p] * e[p];
      e[i] = v / L[6 * i + i];
    }
#pragma unroll
    for (int i = 5; i >= 0; --i) {
      double v = e[i];
#pragma unroll
      for (int p = i + 1; p < 6; ++p) v -= L[6 * p + i] * e[p];
      e[i] = v / L[6 * i + i];
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) Ui[6 * i + col] = e[i];
  }
}

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------

// rr[ca] * rr[cb], rounded before it is added (no FMA contraction: the
// per-capture sums of k_linearize have always rounded product and sum
// separately, the per-observation ones use FMAs; kept as they were)
__device__ __forceinline__ double row_prod(const double *rr, int ca, int cb) {
#pragma clang fp contract(off)
  return rr[ca] * rr[cb];
}

// The per-capture kernels k_linearize, k_cost and k_backsub come in two
// instances: kChunked = false, the main launch over every capture, which
// takes the captures of at most kObsChunk observations (one wave of rows, the
// code the usual capture runs) and skips the others when there are some;
// true, a second launch over those (DevProblem::chunk_caps), their rows
// through LDS 64 at a time.  The rare large capture's loops then cost the
// usual one no registers or branches.
template <bool kChunked>
__device__ __forceinline__ int chunk_capture(const DevProblem &P, int &k) {
  const int c = kChunked ? P.chunk_caps[blockIdx.x] : (int)blockIdx.x;
  k = P.cap_start[c + 1] - P.cap_start[c];
  return (!kChunked && k > kObsChunk) ? -1 : c;   // (-1: the chunked launch's)
}

// (4 waves per SIMD instead of the 3 its 143 VGPRs allow: a 28-byte spill,
// 84 -> 71 us on cfg3; 5 waves spills 148 bytes and is slower)
// Linearize at x: per-observation tag gradient/column norms, per-capture
// gradient/column norms, cost and camera partials.  Unscaled Jacobian.
template <bool kChunked>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_linearize(DevProblem P, const double *__restrict__ x,
                                                     double *__restrict__ g,
                                                     double *__restrict__ colnorm,
                                                     double *__restrict__ obs_tg,
                                                     double *__restrict__ parts) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int c = kChunked ? P.chunk_caps[blockIdx.x] : (int)blockIdx.x, lane = threadIdx.x;
  const int o0 = P.cap_start[c], k = P.cap_start[c + 1] - o0;
  if (!kChunked && k > kObsChunk) return;   // (the chunked launch's)
  const int nrows = 8 * k;
  // The rows go through LDS in chunks of kObsChunk observations (one wave's
  // 64 rows), so any number of observations per capture fits; every sum runs
  // on over the chunks in the same order as over the whole capture at once
  double *rows = sm;
  double *ocost = rows + (long)8 * kObsChunk * kRowStride;   // [kObsChunk]
  // the running sums carried over the chunks, in LDS (nothing held in
  // registers across the projection): lanes 0..13's per-capture sums, then
  // the active and fixed cost
  double *accs = ocost + kObsChunk;   // [16]
  // (one chunk -- the usual capture -- as its own specialised copy: the loop
  // around the projection cost the single-chunk code spills)
  auto chunk = [&](int q0) __attribute__((always_inline)) {
    const int kc = min(kObsChunk, k - q0), nr = 8 * kc;
    fill_rows(P, x, nullptr, c, o0, 8 * q0, nr, nrows, rows, P.jrows);
    __syncthreads();
    // Every sum below is over rows of one product of two LDS columns (ca, cb),
    // picked per lane up front: one code path for the whole wave (a divergent
    // if-chain ran each case's LDS round trips one after another)
    // per observation: cost (r'r), tag gradient (6: F_t'r), tag column norms (6)
    for (int e = lane; e < 13 * kc; e += kWave) {
      const int q = e / 13, it = e % 13;
      const double *rq = rows + (long)q * 8 * kRowStride;
      const int ca = it == 0 ? 13 : it <= 6 ? 6 + it : it, cb = it <= 6 ? 13 : it;
      double s = 0.0;
#pragma unroll
      for (int rr = 0; rr < 8; ++rr) s += rq[rr * kRowStride + ca] * rq[rr * kRowStride + cb];
      if (it == 0) ocost[q] = 0.5 * s;
      else obs_tg[12L * P.obs_tpos[o0 + q0 + q] + (it - 1)] = s;   // (tag-major: k_lin_reduce reads a tag's at once)
    }
    // per capture: capture gradient (6: E'r), capture column norms (6), f gradient, f column norm
    if (lane < 14) {
      const int ca = lane < 6 ? 1 + lane : lane < 12 ? lane - 5 : 0;
      const int cb = lane < 6 ? 13 : lane < 12 ? lane - 5 : lane == 12 ? 13 : 0;
      double ps = q0 ? accs[lane] : 0.0;
#pragma unroll 8
      for (int r = 0; r < nr; ++r) ps += row_prod(rows + (long)r * kRowStride, ca, cb);
      accs[lane] = ps;
    }
    __syncthreads();
    if (lane == 0) {
      double act = q0 ? accs[14] : 0.0, fix = q0 ? accs[15] : 0.0;
      for (int q = 0; q < kc; ++q) {
        if (P.obs_active[o0 + q0 + q]) act += ocost[q]; else fix += ocost[q];
      }
      accs[14] = act;
      accs[15] = fix;
    }
  };
  if (!kChunked) {   // (at most one chunk)
    chunk(0);
  } else {
    for (int q0 = 0; q0 < k; q0 += kObsChunk) {
      if (q0) __syncthreads();   // the previous chunk's LDS reads are done
      chunk(q0);
    }
  }
  if (lane < 14) {
    const double ps = k ? accs[lane] : 0.0;
    if (lane < 12) {
      const long slot = slot_cap(P, c) + (lane % 6);
      const double v = P.slot_free[slot] ? ps : 0.0;
      if (lane < 6) g[slot] = v; else colnorm[slot] = v;
    } else if (lane == 12) {
      parts[(long)P_GF * P.nc + c] = ps;
    } else {
      parts[(long)P_CF * P.nc + c] = ps;
    }
  }
  if (lane == 0) {
    parts[(long)P_COST * P.nc + c] = k ? accs[14] : 0.0;
    parts[(long)P_FIXED * P.nc + c] = k ? accs[15] : 0.0;
  }
}

// Per tag slot: the gradient / column-norm sums over the tag's observations
// (obs_tg from k_linearize), in observation order.  Element e = 12 t + j.
__device__ __forceinline__ void tag_reduce_elem(const DevProblem &P, const double *__restrict__ obs_tg, long e,
                                                double *__restrict__ g, double *__restrict__ colnorm) {
  if (e >= 12L * P.nt) return;
  const int t = (int)(e / 12), j = (int)(e % 12);
  double s = 0.0;
  const int qa = P.tag_start[t], qb = P.tag_start[t + 1];
  // (obs_tg is tag-major: the tag's observations, in observation order, are
  // contiguous -- no index load in front of the sums' loads)
  for (int q0 = qa; q0 < qb; q0 += 32) {   // 32 loads in flight; summed in observation order
    double v[32];
#pragma unroll
    for (int u = 0; u < 32; ++u) v[u] = obs_tg[12L * min(q0 + u, qb - 1) + j];
#pragma unroll
    for (int u = 0; u < 32; ++u) s += (q0 + u < qb) ? v[u] : 0.0;
  }
  const long slot = slot_tag(P, t) + (j % 6);
  if (P.f_alias) {
    // (mixed e-set) a capture on the reduced side with a direct group: that
    // group's sums over its own pose (k_linearize) belong to this block; the
    // group's slot gets the total too, so its scale and LM diagonal are the block's
    const int d = P.f_alias[t];
    if (d >= 0) {
      double *dv = (j < 6 ? g : colnorm) + slot_cap(P, d) + (j % 6);
      s += *dv;
      *dv = P.slot_free[slot] ? s : 0.0;
    }
  }
  const double v = P.slot_free[slot] ? s : 0.0;
  if (j < 6) g[slot] = v; else colnorm[slot] = v;
}

// (diag: also the LM diagonal clamp(s^2 colnorm, dmin, dmax) from the new scale: k_lm_diag's work)
__global__ void k_scale(long n, const unsigned char *__restrict__ free_, const double *__restrict__ colnorm,
                        int jacobi, double *__restrict__ scale, double dmin, double dmax, double *__restrict__ diag) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // jacobian_scaling = 1 / (1 + sqrt(SquaredColumnNorm)) at iteration 0
  const double sv = free_[i] ? (jacobi ? 1.0 / (1.0 + sqrt(colnorm[i])) : 1.0) : 0.0;
  scale[i] = sv;
  if (diag) diag[i] = fmin(fmax(sv * sv * colnorm[i], dmin), dmax);
}

__global__ void k_lm_diag(long n, const double *__restrict__ scale, const double *__restrict__ colnorm,
                          double dmin, double dmax, double *__restrict__ diag) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double d = scale[i] * scale[i] * colnorm[i];   // squared column norm of J * diag(s)
  diag[i] = fmin(fmax(d, dmin), dmax);
}

// A direct group of the mixed e-set (MixedProblem): residuals whose two poses
// are both on the reduced side, grouped by their capture, whose pose is the
// group's last local f-block (nblk - 1: no residual lists it, so its W, F'r and
// F'F entries stayed zero).  Nothing is eliminated: the stored local system is
// the plain normal-equation blocks of [f | tag blocks | own pose | r] (Ceres'
// SchurEliminator adds such rows to the reduced system as they are), the own
// pose's from the capture-wide sums U = E'E, E'f, E'F_u and E'r.
__device__ void store_direct_group(double *out, int nblk, int m, const double *U, const double *Etr, const double *W,
                                   const double *Ftr, const double *FF, double ff00, int lane) {
  const int own = nblk - 1;
  // local column x: 0 f, 1 a tag block's row, 2 the own pose's, 3 the rhs; u its block, i the row in it
  auto cls = [&](int x, int &u, int &i) {
    u = x >= 1 && x < m ? (x - 1) / 6 : 0;
    i = x >= 1 && x < m ? (x - 1) - 6 * u : 0;
    return x == 0 ? 0 : x == m ? 3 : (u == own ? 2 : 1);
  };
  for (int Ub = 0; Ub <= nblk + 1; ++Ub) {
    const int sU = schur_blk_size(Ub, nblk), p0 = schur_blk_start(Ub, nblk), ncol = p0 + sU;
    double *dst = out + schur_block_off(Ub, 0, nblk);
    for (int e = lane; e < sU * ncol; e += kWave) {
      const int ip = e / ncol, q = e - ip * ncol, p = p0 + ip;
      int ua, ia, ub, ib;
      int ka = cls(q, ua, ia), kb = cls(p, ub, ib);   // (the pair in f < tag < own < rhs order)
      if (ka > kb || (ka == kb && q > p)) {
        const int tk = ka, tu = ua, ti = ia;
        ka = kb; ua = ub; ia = ib;
        kb = tk; ub = tu; ib = ti;
      }
      double v = 0.0;
      if (ka == 0) {
        v = kb == 0 ? ff00 : kb == 1 ? FF[28 * ub + 21 + ib] : kb == 2 ? W[ib * m] : Ftr[0];
      } else if (ka == 1) {
        if (kb == 1) {
          if (ua == ub) {
            const int lo = min(ia, ib), hi = max(ia, ib);
            v = FF[28 * ua + lo * 6 - lo * (lo - 1) / 2 + (hi - lo)];
          }
        } else {
          v = kb == 2 ? W[ib * m + 1 + 6 * ua + ia] : Ftr[1 + 6 * ua + ia];
        }
      } else if (ka == 2) {
        v = kb == 2 ? U[6 * ia + ib] : Etr[ia];
      }
      const int V = schur_blk(q, m), q0V = schur_blk_start(V, nblk);
      dst[(long)sU * q0V + ip * schur_blk_size(V, nblk) + (q - q0V)] = v;
    }
  }
}

// Schur elimination of capture c (ComputeTrustRegionStep's DENSE_SCHUR
// eliminate step, one capture = one e-block; the normal-equation blocks from
// per-observation Gram matrices on MFMA): the packed local reduced system
//   [F'F - W' U^-1 W | F'r - W' U^-1 E'r],  U = E'E + D_c^2, W = E'F,
// over the local f-side columns (f, then 6 per distinct tag of the capture),
// stored for k_schur_gather.  One wave per capture.
// kBig = false: the main launch (captures of at most kSchurMfmaBlocks tags,
// the output as one MFMA product; the blocks past the captures clear S and
// reset the executors); true: the captures of more tags (cap_list), one block
// row of the output at a time.  Two instances, so the main one carries no
// registers for the other's path.
template <bool kBig>
__global__ __launch_bounds__(kWave) void k_schur(DevProblem P, const double *__restrict__ scale,
                                                 const double *__restrict__ diag, double radius,
                                                 double *__restrict__ zero_tiles, long n_zero, ExecReset er,
                                                 const int *__restrict__ cap_list) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  SCHUR_STAMP_INIT;
  // (cap_list: the second launch, over the captures with more than
  // kSchurMfmaBlocks distinct tags; the main launch then skips them)
  const int c = kBig ? cap_list[blockIdx.x] : (int)blockIdx.x, lane = threadIdx.x;
  if (c >= P.nc + n_zero) {
    // the blocks past the tiles: the persistent executors' reset (ExecReset;
    // launch_exec_reset's work when the LM diagonal needs no update)
    exec_reset_elem(er, (long)(c - P.nc - n_zero) * kWave + lane);
    return;
  }
  if (c >= P.nc) {
    // the blocks past the captures clear one 64x64 tile of S each (the gather
    // writes only the assembled blocks; the rest of S must be zero): the
    // stores overlap the latency-bound capture waves instead of a memset
    // launch of their own
    typedef double d2 __attribute__((ext_vector_type(2)));
    d2 *z = reinterpret_cast<d2 *>(zero_tiles + (long)(c - P.nc) * 4096);
#pragma unroll 8
    for (int e = lane; e < 2048; e += kWave) z[e] = d2{0.0, 0.0};
    return;
  }
  const int o0 = P.cap_start[c], k = P.cap_start[c + 1] - o0;
  if (k == 0) return;
  const int nrows = 8 * k;
  const int b0 = P.cap_blk_start[c], nblk = P.cap_blk_start[c + 1] - b0;
  if (!kBig && nblk > kSchurMfmaBlocks) return;   // (the second launch's)
  const int m = 1 + 6 * nblk;   // local f-side columns: f, then 6 per distinct tag
  // LDS (schur_lds_bytes): no copy of the Jacobian rows (they go from HBM
  // straight into the MFMA operand registers), so ~8 KB per wave at 8 tags:
  // 4-5 waves per SIMD instead of the 2.75 the 13.5 KB row-staging layout
  // allowed (latency-bound kernel)
  double *stage = sm;                            // 6 min(m + 1, 64): the MFMA product's Z operand
  double *tscale = stage + 6 * min(m + 1, kWave);   // 6 kObsChunk: the chunk's observations' tag column scales
  double *U = tscale + 6 * kObsChunk;            // 36
  double *Ui = U + 36;                           // 36
  double *Etr = Ui + 36;                         // 8
  double *W = Etr + 8;                           // 6*m
  double *Ftr = W + 6 * m;                       // m (+pad)
  double *FF = Ftr + m + (m & 1);                // 28 per tag block: F_u'F_u (21, packed), F_0'F_u (6), pad
  int *lblk = (int *)(FF + 28 * nblk);           // kObsChunk: the chunk's observations' tag blocks
  double *ff00 = reinterpret_cast<double *>(lblk + kObsChunk);     // F_0'F_0

  // the first eight observations' Jacobian rows (the Gram loop's operands
  // below) are loaded before the prologue's dependent loads (obs_tag -> the
  // tag scales), so the two latencies overlap
  const int li = lane & 15, lk = lane >> 4;
  const bool valid = li < 14;
  // (column li of the row is stored column jrow_col(li): lanes 7..9 read the
  // translation column lanes 1..3 read)
  const double *jb = P.jrows + 8L * o0 * kJStored + (long)jrow_col(min(li, 13)) * nrows;
  double jv[16];
#pragma unroll
  for (int u = 0; u < 8; ++u)
#pragma unroll
    for (int st = 0; st < 2; ++st)
      jv[2 * u + st] = (valid && u < k) ? jb[8 * u + 4 * st + lk] : 0.0;
  static_assert(kObsChunk == 8, "k_schur's operand registers hold eight observations");
  // the tag scales and blocks of a chunk of kObsChunk observations (reloaded
  // beside the operand registers in the Gram loop)
  auto stage_chunk = [&](int q0) {
    const int kc = min(kObsChunk, k - q0);
    if (lane < kc) lblk[lane] = P.obs_lblk[o0 + q0 + lane];
    if (lane < 6 * kc) tscale[lane] = scale[slot_tag(P, P.obs_tag[o0 + q0 + lane / 6]) + lane % 6];
  };
  stage_chunk(0);
  __syncthreads();
  SCHUR_STAMP(0);
  // Every product below is an entry of an observation's Gram matrix over its
  // 8 rows and 14 columns [f | E (capture) | F (tag) | r]: G_q = R_q' R_q, two
  // v_mfma_f64_16x16x4_f64 per observation (columns padded to 16; lane
  // (lk, li) supplies row 4s + lk, column li as both operands; the result is
  // G_q[lk + 4 reg][li]).  The capture-wide sums (U = E'E, E'r, E'f, f'r, f'f)
  // add the observations' Grams in observation order; the per-tag-block
  // products (W_u = E'F_u, F_u'r, F_u'F_u, f'F_u) are added into LDS per
  // observation (a tag seen twice in one capture sums into one block).
  {
    for (int e = lane; e < 6 * m + m + (m & 1) + 28 * nblk; e += kWave) W[e] = 0.0;   // W, Ftr, FF: contiguous
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    typedef double dbl4v __attribute__((ext_vector_type(4)));
    dbl4v tot = {0, 0, 0, 0};
    // lane (lk, li) reads column li of rows 8q + lk and 8q + 4 + lk from the
    // capture's column-major Jacobian block (load_rows' layout), eight
    // observations' loads in flight at once, and scales it as load_rows does
    // (the same products: the Grams are bit-identical)
    const double *sc = scale + slot_cap(P, c);
    const double cs = li == 0 ? scale[0] : li <= 6 ? sc[li - 1] : 1.0;   // (tag columns: tscale)
    const bool tagcol = li >= 7 && li <= 12;
    // Where this lane's Gram entries G[lk + 4 reg][li] go, as an LDS index
    // (W, Ftr and FF are contiguous) plus a stride per tag block u: one LDS
    // add per register and observation instead of a divergent if-chain
    //   E'F_u  : W[(r-1) m + 1 + 6u + (c-7)]          r 1..6,  c 7..12
    //   F_u'r  : Ftr[1 + 6u + (r-7)]                    r 7..12, c 13
    //   F_u'F_u: FF[28u + a*6 - a(a-1)/2 + (b-a)]       r 7..12, r <= c <= 12
    //   f'F_u  : FF[28u + 21 + (c-7)]                   r 0,     c 7..12
    int acc_off[4], acc_stride[4];
    const int w_base = (int)(W - sm);
    {
      const int c = li, ftr0 = 6 * m, ff0 = ftr0 + m + (m & 1);
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int r = lk + 4 * reg;
        int off = -1, st = 0;
        if (r >= 1 && r <= 6 && c >= 7 && c <= 12) { off = (r - 1) * m + 1 + (c - 7); st = 6; }
        else if (r >= 7 && r <= 12 && c == 13) { off = ftr0 + 1 + (r - 7); st = 6; }
        else if (r >= 7 && r <= 12 && c >= r && c <= 12) {
          const int a = r - 7, b = c - 7;
          off = ff0 + a * 6 - a * (a - 1) / 2 + (b - a); st = 28;
        } else if (r == 0 && c >= 7 && c <= 12) { off = ff0 + 21 + (c - 7); st = 28; }
        acc_off[reg] = off >= 0 ? w_base + off : 0;   // (no destination: stage[0], dead here)
        acc_stride[reg] = st;
      }
    }
    for (int q = 0; q < k; ++q) {
      if ((q & 7) == 0 && q > 0) {
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
          for (int st = 0; st < 2; ++st)
            jv[2 * u + st] = (valid && q + u < k) ? jb[8 * (q + u) + 4 * st + lk] : 0.0;
        stage_chunk(q);   // (the previous iteration ended at a wave barrier: its reads are done)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      dbl4v g = {0, 0, 0, 0};
      const double s = tagcol ? tscale[6 * (q & 7) + li - 7] : cs;
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        double v = 0.0;
        switch (q & 7) {   // (register array: constant indices only)
          case 0: v = jv[0 + st]; break;
          case 1: v = jv[2 + st]; break;
          case 2: v = jv[4 + st]; break;
          case 3: v = jv[6 + st]; break;
          case 4: v = jv[8 + st]; break;
          case 5: v = jv[10 + st]; break;
          case 6: v = jv[12 + st]; break;
          default: v = jv[14 + st]; break;
        }
        v = li == 13 ? v : v * s;   // the residual column is not scaled
        g = __builtin_amdgcn_mfma_f64_16x16x4f64(v, v, g, 0, 0, 0);
      }
      tot += g;
      const int u = lblk[q & 7] - 1;   // the observation's tag block
      // this lane's entries G[lk + 4 reg][li] (acc_off above): the four
      // destinations are distinct, so their reads go out together
      int di[4];
      double dv[4];
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        di[reg] = acc_off[reg] + acc_stride[reg] * u;
        dv[reg] = sm[di[reg]];
      }
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) sm[di[reg]] = dv[reg] + g[reg];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int r = lk + 4 * reg, c = li;
      const double v = tot[reg];
      if (r >= 1 && r <= 6 && c >= 1 && c <= 6) U[6 * (r - 1) + (c - 1)] = v;   // E'E
      else if (r >= 1 && r <= 6 && c == 13) Etr[r - 1] = v;                     // E'r
      else if (r >= 1 && r <= 6 && c == 0) W[(r - 1) * m] = v;                  // E'f
      else if (r == 0 && c == 13) Ftr[0] = v;                                   // f'r
      else if (r == 0 && c == 0) *ff00 = v;                                     // f'f
    }
  }
  __syncthreads();
  SCHUR_STAMP(1);
  if (group_direct(P, c)) {
    store_direct_group(P.slab + P.cap_off[c], nblk, m, U, Etr, W, Ftr, FF, *ff00, lane);
    return;
  }
  // (U + D_c^2)^{-1}: every lane factors U (one reciprocal per pivot), lane j
  // solves for column j
  {
    const long sc = slot_cap(P, c);
    double L[21];
    double rd[6];
    int e = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j <= i; ++j) L[e++] = U[6 * i + j] + (i == j ? lm_d2(diag, sc + i, radius) : 0.0);
#define LI6(i, j) L[(i) * ((i) + 1) / 2 + (j)]
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      double d = LI6(j, j);
#pragma unroll
      for (int p = 0; p < j; ++p) d -= LI6(j, p) * LI6(j, p);
      const double sd = sqrt(d);
      rd[j] = 1.0 / sd;
      LI6(j, j) = sd;
#pragma unroll
      for (int i = j + 1; i < 6; ++i) {
        double v = LI6(i, j);
#pragma unroll
        for (int p = 0; p < j; ++p) v -= LI6(i, p) * LI6(j, p);
        LI6(i, j) = v * rd[j];
      }
    }
    if (lane < 6) {
      double ev[6];
#pragma unroll
      for (int i = 0; i < 6; ++i) {
        double v = (i == lane) ? 1.0 : 0.0;
#pragma unroll
        for (int p = 0; p < i; ++p) v -= LI6(i, p) * ev[p];
        ev[i] = v * rd[i];
      }
#pragma unroll
      for (int i = 5; i >= 0; --i) {
        double v = ev[i];
#pragma unroll
        for (int p = i + 1; p < 6; ++p) v -= LI6(p, i) * ev[p];
        ev[i] = v * rd[i];
      }
#pragma unroll
      for (int i = 0; i < 6; ++i) Ui[6 * i + lane] = ev[i];
    }
#undef LI6
  }
  __syncthreads();
  if (lane < 36) P.cap_ui[36L * c + lane] = Ui[lane];   // reused by k_backsub
  SCHUR_STAMP(2);
  SCHUR_STAMP(3);
  // block-packed rows (row m is the rhs; entries of constant blocks are never
  // gathered; schur_block_off): lane q owns column q, z = (U + D_c^2)^{-1}
  // W[:, q] in registers; row p is wave-uniform, so its W column (the rhs
  // row: E'r) is an LDS broadcast.  One block row U at a time is staged in
  // LDS (over the dead Jacobian rows) in its final layout, then copied out
  // with contiguous stores.
  //   (p, q) = F_p'F_q - W_p' z_q,   (m, q) = F_q'r - (E'r)' z_q
  double *out = P.slab + P.cap_off[c];
  auto make_z = [&](int q, double z[6]) {
    if (q < m) {
      double wq[6];
#pragma unroll
      for (int b = 0; b < 6; ++b) wq[b] = W[b * m + q];
#pragma unroll
      for (int a = 0; a < 6; ++a) {
        double s = 0.0;
#pragma unroll
        for (int b = 0; b < 6; ++b) s += Ui[6 * a + b] * wq[b];
        z[a] = s;
      }
    } else {
#pragma unroll
      for (int a = 0; a < 6; ++a) z[a] = 0.0;
    }
  };
  const bool one_chunk = !kBig;   // (m + 1 <= kWave)
  double z[6];
  if (one_chunk) make_z(lane, z);
  if (one_chunk) {
    // All M = m + 1 local rows at once as one MFMA product C = Wx' Z (K = 6,
    // padded to 8), Wx = [W | E'r] (6 x M), Z = [z_0 .. z_{m-1} | 0] (6 x M):
    // C[p][q] = W_p' z_q, the rhs row's (E'r)' z_q at p = m.  Only the 16x16
    // tiles that hold stored (lower block-triangle) entries are formed; each
    // lane then writes its entries F_p'F_q - C[p][q] (the F'F / F'r / f'f
    // terms where they are nonzero) straight to their block-packed slab slots.
    const int M = m + 1;
    const int li = lane & 15, lk = lane >> 4;
    double *Zs = stage;   // 6 M doubles: Zs[a M + q]
    if (lane < M)
#pragma unroll
      for (int a = 0; a < 6; ++a) Zs[a * M + lane] = z[a];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double Aop[4][2], Bop[4][2];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        const int a = 4 * kb + lk, pq = 16 * r + li;
        const bool in = a < 6 && pq < M;
        Aop[r][kb] = in ? (pq < m ? W[a * m + pq] : Etr[a]) : 0.0;
        Bop[r][kb] = in ? Zs[a * M + pq] : 0.0;
      }
    typedef double dbl4v __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (16 * r >= M) break;
      // this lane's rows p = 16 r + lk + 4 reg: block row, row inside it, last stored column
      int pU[4], pI[4], pEnd[4];
      long pOff[4];
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int pp = 16 * r + lk + 4 * reg;
        const int up = pp >= 1 && pp < m ? (pp - 1) / 6 : -1;
        const int U = pp == 0 ? 0 : (pp < m ? 1 + up : nblk + 1);
        pU[reg] = U;
        pI[reg] = up >= 0 ? pp - 1 - 6 * up : 0;
        pEnd[reg] = pp == 0 ? 1 : (pp < m ? 7 + 6 * up : M);   // columns q < pEnd are stored
        pOff[reg] = schur_block_off(U, 0, nblk);               // the block row's first element
      }
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        if (cc > r + 1 || 16 * cc >= M) break;
        dbl4v acc = {0, 0, 0, 0};
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[r][0], Bop[cc][0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Aop[r][1], Bop[cc][1], acc, 0, 0, 0);
        const int q = 16 * cc + li;
        const int uq = q >= 1 && q < m ? (q - 1) / 6 : -1;   // q's tag block
        const int V = q == 0 ? 0 : (q < m ? 1 + uq : nblk + 1);
        const int sV = schur_blk_size(V, nblk), q0V = schur_blk_start(V, nblk);
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) {
          const int pp = 16 * r + lk + 4 * reg;
          if (pp >= M || q >= pEnd[reg]) continue;
          const int U = pU[reg], sU = schur_blk_size(U, nblk);
          double ff = 0.0;
          if (pp == 0) {
            ff = *ff00;                                     // (q == 0 only)
          } else if (pp == m) {
            ff = q < m ? Ftr[q] : 0.0;
          } else {
            const int up = U - 1, i = pI[reg];
            if (q == 0) {
              ff = FF[28 * up + 21 + i];                    // f'F_u
            } else if (uq == up) {                          // F_u'F_u packed upper (a <= b)
              const int iq = q - 1 - 6 * uq, lo = min(i, iq), hi = max(i, iq);
              ff = FF[28 * up + lo * 6 - lo * (lo - 1) / 2 + (hi - lo)];
            }
          }
          out[pOff[reg] + (long)sU * q0V + pI[reg] * sV + (q - q0V)] = ff - acc[reg];
        }
      }
    }
  } else
  for (int U = 0; U <= nblk + 1; ++U) {
    // (more than kSchurMfmaBlocks tags: one block row U at a time, each entry
    // stored straight to its block-packed slot)
    const int sU = schur_blk_size(U, nblk), p0U = schur_blk_start(U, nblk), ncol = p0U + sU;
    double *dst = out + schur_block_off(U, 0, nblk);
    for (int q0 = 0; q0 < ncol; q0 += kWave) {
      const int q = q0 + lane;
      if (!one_chunk) make_z(q, z);
      const int V = schur_blk(min(q, m), m), sV = schur_blk_size(V, nblk), q0V = schur_blk_start(V, nblk);
      const int uq = V - 1, iq = q - q0V;   // tag block and row inside it (V in 1..nblk)
      if (sU == 6) {
        // a tag block row: the 36 W entries of its six rows read up front
        // (independent broadcasts), then six rows of six FMAs
        const int up = U - 1;
        double wv[6][6];
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
          for (int a = 0; a < 6; ++a) wv[i][a] = W[a * m + p0U + i];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
          double s = 0.0;
#pragma unroll
          for (int a = 0; a < 6; ++a) s += wv[i][a] * z[a];
          double ff = 0.0;
          if (q == 0) {
            ff = FF[28 * up + 21 + i];
          } else if (uq == up) {   // F_u'F_u packed upper (a <= b)
            const int lo = min(i, iq), hi = max(i, iq);
            ff = FF[28 * up + lo * 6 - lo * (lo - 1) / 2 + (hi - lo)];
          }
          if (q < ncol) dst[6 * q0V + i * sV + (q - q0V)] = ff - s;
        }
      } else {   // the f row (p = 0) or the rhs row (p = m)
        const int p = p0U;
        const double *wp = p < m ? W + p : Etr;
        const int st = p < m ? m : 1;
        double s = 0.0;
#pragma unroll
        for (int a = 0; a < 6; ++a) s += wp[a * st] * z[a];
        double ff = 0.0;
        if (p == m) ff = q < m ? Ftr[q] : 0.0;
        else ff = *ff00;   // p == 0: only q == 0 is stored
        if (q < ncol) dst[q0V + (q - q0V)] = ff - s;
      }
    }
  }
  SCHUR_STAMP(4);
}

// Destination block geometry: E = sX sY elements (1 row for f and the rhs,
// 6 for a tag), G = 64 / E lane groups; lane -> (element (i, j), group).
struct GatherLane {
  int E, G, el, grp, i, j;
  __device__ GatherLane(const DevProblem &P, int2 rr, int lane) {
    const int sx = (rr.x == P.nR || rr.x == P.cam_row) ? 1 : 6;
    const int sy = rr.y == P.cam_row ? 1 : 6;
    E = sx * sy;
    G = kWave / E;
    el = lane % E;
    grp = lane / E;
    i = el / sy;
    j = el % sy;
  }
};

// Lanes < E of the wave: the sum of the groups' partials, in group order.
__device__ __forceinline__ double gather_groups(double s, const GatherLane &g, double *part, int lane) {
  if (g.G == 1) return s;
  part[lane] = s;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double t = 0.0;
  if (lane < g.E)
    for (int q = 0; q < g.G; ++q) t += part[q * g.E + lane];
  return t;
}

// Sum of the captures' packed local systems into the reduced tiles: one wave
// per work item (a destination block (rX, rY), or a <= 64-contribution piece
// of one).  The wave stages the item's contribution descriptors in LDS; the
// G lane groups stride over them with 8 slab loads in flight per lane, and
// the groups' partials are added in group order -- a fixed summation order,
// no atomics.  Pieces store partial sums for k_schur_combine.
// The D_f^2 of a reduced row's diagonal element (prep: the gather adds it when
// it writes the element, k_prep_reduced's work), else 0.
__device__ __forceinline__ double prep_d2(const DevProblem &P, const double *diag, double radius, long r,
                                          long col) {
  if (!diag || r != col || r >= P.nR) return 0.0;
  const int slot = P.row_slot[r];
  return slot >= 0 ? lm_d2(diag, slot, radius) : 0.0;
}

// k_prep_reduced's diagonal elements that no gather item writes: alignment
// padding and the rows past the rhs become identity rows, the rhs row a pivot
// large enough to stay positive (in prep mode the gather leaves the rhs-rhs
// element to this), the camera's l1/l2 rows get their D_f^2
__device__ __forceinline__ void prep_pad_row(const DevProblem &P, const double *diag, double radius, double *S,
                                             long i) {
  if (i >= P.N) return;
  if (i < P.nR && P.row_slot[i] >= 0) {
    // the camera's l1, l2 rows (zero Jacobian columns, no Schur block): D_f^2 only
    if (P.cam_row >= 0 && i > P.cam_row && i <= P.cam_row + 2)
      *reduced_elem(S, P, i, i) = lm_d2(diag, P.row_slot[i], radius);
    return;
  }
  *reduced_elem(S, P, i, i) = i == P.nR ? 1e300 : 1.0;
}

__global__ __launch_bounds__(256) void k_schur_gather(DevProblem P, double *__restrict__ S,
                                                      const double *__restrict__ diag, double radius) {
  __shared__ double part[4][kWave];
  __shared__ SchurContrib cts[4][kWave];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n_item_blocks = (P.n_items + 3) / 4;
  if (diag && (int)blockIdx.x >= n_item_blocks) {   // (prep) the rows no item writes
    prep_pad_row(P, diag, radius, S, (long)(blockIdx.x - n_item_blocks) * 256 + threadIdx.x);
    return;
  }
  const int it = blockIdx.x * 4 + w;
  if (it >= P.n_items) return;
  const int4 item = P.gather_items[it];
  const int2 rr = P.dest_row[item.x];
  const GatherLane g(P, rr, lane);
  const int nk = item.z - item.y;   // (gather_partition: <= 64, or <= 16 per lane group)
  const bool staged = nk <= kWave;
  if (staged && lane < nk) cts[w][lane] = P.contrib[item.y + lane];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  double s = 0.0;
  // (a long item -- a 1- or 6-element block summing up to 16 contributions
  // per group -- reads its descriptors itself; the same order either way)
  auto sum = [&](const SchurContrib *src) __attribute__((always_inline)) {
    for (int t0 = g.grp; t0 < nk; t0 += 8 * g.G) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int t = min(t0 + u * g.G, nk - 1);   // clamped: always a valid address
        const SchurContrib ct = src[t];
        v[u] = P.slab[ct.off + (ct.tr ? g.j * ct.ld + g.i : g.i * ct.ld + g.j)];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) s += (t0 + u * g.G < nk) ? v[u] : 0.0;
    }
  };
  if (g.grp < g.G) {
    if (staged) sum(cts[w]);
    else sum(P.contrib + item.y);
  }
  s = gather_groups(s, g, part[w], lane);
  if (lane >= g.E) return;
  if (item.w >= 0) {
    P.gather_part[(long)item.w * 36 + lane] = s;
  } else {
    const long r = rr.x + g.i, col = rr.y + g.j;
    if (r >= col && !(diag && r == P.nR && col == P.nR)) *reduced_elem(S, P, r, col) = s + prep_d2(P, diag, radius, r, col);
  }
}

// Split destinations: the pieces' partial sums, in piece order.
__global__ __launch_bounds__(256) void k_schur_combine(DevProblem P, double *__restrict__ S,
                                                       const double *__restrict__ diag, double radius) {
  __shared__ double part[4][kWave];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int sp = blockIdx.x * 4 + w;
  if (sp >= P.n_splits) return;
  const int4 split = P.gather_splits[sp];
  const int2 rr = P.dest_row[split.x];
  const GatherLane g(P, rr, lane);
  double s = 0.0;
  if (g.grp < g.G) {
    for (int t0 = g.grp; t0 < split.z; t0 += 8 * g.G) {
      double v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        v[u] = P.gather_part[(long)(split.y + min(t0 + u * g.G, split.z - 1)) * 36 + g.el];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += (t0 + u * g.G < split.z) ? v[u] : 0.0;
    }
  }
  s = gather_groups(s, g, part[w], lane);
  const long r = rr.x + g.i, col = rr.y + g.j;
  if (lane < g.E && r >= col && !(diag && r == P.nR && col == P.nR))
    *reduced_elem(S, P, r, col) = s + prep_d2(P, diag, radius, r, col);
}

// S[i][i] += D_f^2 for the reduced (tag + camera) rows; alignment padding and
// the rows past the rhs become identity rows; the rhs row gets a pivot large
// enough to stay positive (its factor row is L^{-1} b, its pivot unused).
__global__ void k_prep_reduced(DevProblem P, const double *__restrict__ diag, double radius,
                               double *__restrict__ S, int which) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P.N) return;
  if (which >= 0 && P.tile_class[i >> 6] != which) return;
  double *d = reduced_elem(S, P, i, i);
  if (i < P.nR) {
    const int slot = P.row_slot[i];
    if (slot >= 0) *d += lm_d2(diag, slot, radius);
    else *d = 1.0;
  } else if (i == P.nR) {
    *d = 1e300;
  } else {
    *d = 1.0;
  }
}

// multi-rank y: the rows this rank solved (own subtree; the top rows on rank 0
// only, or on every rank with keep_top), every other row 0
__global__ void k_mask_y(DevProblem P, double *__restrict__ yF, int rank, int keep_top) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P.nR) return;
  const int c = P.tile_class[i >> 6];
  if (!(c == 0 || (c == 1 && (rank == 0 || keep_top)))) yF[i] = 0.0;
}

__global__ void k_own_copy(DevProblem P, long first, long count, const double *__restrict__ src,
                           double *__restrict__ dst) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < count) dst[i] = P.f_own[first + i] ? src[i] : 0.0;
}

// Cost at x (candidate evaluation) of capture c: active / fixed cost,
// finiteness.  cap: the capture's 6 parameters (x's slot, or the candidate
// k_backsub just formed, held in LDS); camera and tags from x.
// (kChunked: a capture of more than kObsChunk observations, its rows 64 at a
// time; else at most one wave of rows)
template <bool kChunked>
__device__ __forceinline__ void capture_cost(const DevProblem &P, const double *__restrict__ x, const double *cap,
                                             int c, double *__restrict__ parts) {
  __shared__ double sq[kWave];
  __shared__ double ocost[kObsChunk];   // (per 64-row chunk; summed in observation order)
  const int lane = threadIdx.x;
  const int o0 = P.cap_start[c], k = P.cap_start[c + 1] - o0;
  const int nrows = 8 * k;
  const double *cam = x;
  const AngleAxis ac = aa_prepare(cap + 3);
  double bad = 0.0, act = 0.0, fix = 0.0;
  for (int base = 0; base < (kChunked ? nrows : 1); base += kWave) {
    const int row = base + lane;
    double r2 = 0.0;
    if (row < nrows) {
      const int q = row >> 3, corner = (row >> 1) & 3, comp = row & 1;
      const int obs = o0 + q;
      const double *tag = x + slot_tag(P, P.obs_tag[obs]);
      const AngleAxis at = aa_prepare(tag + 3);
      const double obsv = P.corners[8L * obs + 2 * corner + comp];
      const bool sw = group_swapped(P, c);   // tag e-block: the capture is the f-block
      const double r = residual_row(sw ? at : ac, sw ? tag : cap, sw ? ac : at, sw ? cap : tag, cam[0], corner,
                                    comp, obsv, nullptr, nullptr);
      if (!isfinite(r)) bad = 1.0;
      r2 = r * r;
    }
    sq[lane] = r2;
    __syncthreads();
    if (lane < 8 && base / 8 + lane < k) {
      double s = 0.0;
#pragma unroll
      for (int rr = 0; rr < 8; ++rr) s += sq[8 * lane + rr];
      ocost[lane] = 0.5 * s;
    }
    __syncthreads();
    if (kChunked && lane == 0)
      for (int q = base / 8; q < min(k, base / 8 + kObsChunk); ++q) {
        if (P.obs_active[o0 + q]) act += ocost[q - base / 8]; else fix += ocost[q - base / 8];
      }
  }
  if (!kChunked && lane == 0)
    for (int q = 0; q < k; ++q) {
      if (P.obs_active[o0 + q]) act += ocost[q]; else fix += ocost[q];
    }
  bad = wave_max(bad);
  if (lane == 0) {
    parts[(long)P_COST * P.nc + c] = act;
    parts[(long)P_FIXED * P.nc + c] = fix;
    parts[(long)P_CBAD * P.nc + c] = bad;
  }
}

template <bool kChunked>
__global__ __launch_bounds__(kWave) void k_cost(DevProblem P, const double *__restrict__ x,
                                                double *__restrict__ parts) {
  int k;
  const int c = chunk_capture<kChunked>(P, k);
  if (c < 0) return;
  capture_cost<kChunked>(P, x, x + slot_cap(P, c), c, parts);
}

// Back substitution for capture c, candidate update of its slots and its
// share of the model cost change.
template <bool kChunked>
__global__ __launch_bounds__(kWave) void k_backsub(DevProblem P, const double *__restrict__ x,
                                                   const double *__restrict__ scale,
                                                   const double *__restrict__ diag, double radius,
                                                   const double *__restrict__ yF,
                                                   double *__restrict__ xc,
                                                   double *__restrict__ parts, int reuse_ui, int with_cost) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  int k;
  const int c = chunk_capture<kChunked>(P, k), lane = threadIdx.x;
  if (c < 0) return;
  const int o0 = P.cap_start[c];
  const long sc = slot_cap(P, c);
  if (k == 0) {
    if (lane < 6) xc[sc + lane] = x[sc + lane];
    if (lane == 0) {
      parts[(long)P_MODEL * P.nc + c] = 0.0;
      parts[(long)P_STEP2 * P.nc + c] = 0.0;
      parts[(long)P_YBAD * P.nc + c] = 0.0;
      if (with_cost) {
        parts[(long)P_COST * P.nc + c] = 0.0;
        parts[(long)P_FIXED * P.nc + c] = 0.0;
        parts[(long)P_CBAD * P.nc + c] = 0.0;
      }
    }
    return;
  }
  const int nrows = 8 * k;
  // the rows go through LDS in chunks of one wave's 64 rows (kObsChunk
  // observations); each lane's running sum is carried over the chunks in row
  // order, as over the whole capture at once
  constexpr int kChunkRows = 8 * kObsChunk;
  double *rows = sm;
  double *qv = rows + (long)kChunkRows * kRowStride;   // [kChunkRows]
  double *U = qv + kChunkRows;                    // 36
  double *Ui = U + 36;                            // 36
  double *v = Ui + 36;                            // 8
  double *yc = v + 8;                             // 8
  const double yf = P.cam_row >= 0 ? yF[P.cam_row] : 0.0;
  if (reuse_ui && lane < 36) Ui[lane] = P.cap_ui[36L * c + lane];   // (U_c + D_c^2)^{-1} as k_schur formed it
  // lanes 0..20: U = E'E (upper triangle entry (a, b)); 21..26 (32..37 with
  // the stored inverse): v = E'(b - F z); each lane's sum runs on over the
  // chunks in LDS (U, v), nothing held in registers across the row loads
  auto chunk = [&](int r0) __attribute__((always_inline)) {
    const int nr = min(kChunkRows, nrows - r0);
    ARSLAM_BACKSUB_ROWS(scale, yF, yf, c, o0, r0, nr, nrows, rows, qv);
    __syncthreads();
    const int va = reuse_ui ? lane - 32 : lane - 21;
    if (!reuse_ui && lane < 21) {
      int a, b;
      upper6(lane, a, b);
      double s = r0 ? U[6 * a + b] : 0.0;
      for (int r = 0; r < nr; ++r) s += rows[(long)r * kRowStride + 1 + a] * rows[(long)r * kRowStride + 1 + b];
      U[6 * a + b] = s;
      U[6 * b + a] = s;
    } else if (va >= 0 && va < 6) {
      double s = r0 ? v[va] : 0.0;
      for (int r = 0; r < nr; ++r) {
        const double *rr = rows + (long)r * kRowStride;
        s += rr[1 + va] * (rr[13] - qv[r]);   // E'(b - F z)
      }
      v[va] = s;
    }
  };
  if (!kChunked) {   // (at most one chunk)
    chunk(0);
  } else {
    for (int r0 = 0; r0 < nrows; r0 += kChunkRows) {
      if (r0) __syncthreads();   // the previous chunk's LDS reads are done
      chunk(r0);
    }
  }
  __syncthreads();
  const bool direct = group_direct(P, c);
  if (direct) {
    // (mixed e-set) a direct group's own pose is a reduced-side block (its last
    // local block): its step is the reduced solution's, as k_update_f forms it
    if (lane < 6) {
      const int r0 = P.tag_row[P.blk_tag[P.cap_blk_start[c + 1] - 1]];
      yc[lane] = r0 >= 0 ? yF[r0 + lane] : 0.0;
    }
  } else if (reuse_ui) {
    if (lane < 6) {
      double t = 0.0;
#pragma unroll
      for (int b = 0; b < 6; ++b) t += Ui[6 * lane + b] * v[b];
      yc[lane] = t;
    }
  } else if (lane == 0) {
#pragma unroll
    for (int a = 0; a < 6; ++a) U[7 * a] += lm_d2(diag, sc + a, radius);
    inv6(U, Ui);
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      double t = 0.0;
#pragma unroll
      for (int b = 0; b < 6; ++b) t += Ui[6 * a + b] * v[b];
      yc[a] = t;
    }
  }
  __syncthreads();
  // model cost change share: p = Jt y (= -Jt step), sum p (r - p/2) (a capture
  // of more than one chunk loads its rows again)
  double mpart = 0.0;
  auto model = [&](int nr) __attribute__((always_inline)) {
    for (int row = lane; row < nr; row += kWave) {
      const double *rr = rows + (long)row * kRowStride;
      double p = qv[row];
#pragma unroll
      for (int a = 0; a < 6; ++a) p += rr[1 + a] * yc[a];
      mpart += p * (rr[13] - p / 2.0);
    }
  };
  if (!kChunked) {
    model(nrows);
  } else {
    for (int r0 = 0; r0 < nrows; r0 += kChunkRows) {
      const int nr = min(kChunkRows, nrows - r0);
      __syncthreads();
      ARSLAM_BACKSUB_ROWS(scale, yF, yf, c, o0, r0, nr, nrows, rows, qv);
      __syncthreads();
      model(nr);
    }
  }
  mpart = wave_sum(mpart);
  double st = 0.0, bad = 0.0;
  double *capc = v;   // (v is free again: the candidate capture pose, for the cost)
  if (lane < 6) {
    const double yv = yc[lane];
    const double d = -yv * scale[sc + lane];
    const double xo = x[sc + lane];
    const double xn = xo + d;
    xc[sc + lane] = xn;
    capc[lane] = xn;
    if (P.slot_free[sc + lane] && !direct) st = (xo - xn) * (xo - xn);   // (a direct group: counted on its f-block)
    bad = isfinite(yv) ? 0.0 : 1.0;
  }
  st = wave_sum(st);
  bad = wave_max(bad);
  if (lane == 0) {
    parts[(long)P_MODEL * P.nc + c] = mpart;
    parts[(long)P_STEP2 * P.nc + c] = st;
    parts[(long)P_YBAD * P.nc + c] = bad;
  }
  // the candidate's cost (k_cost fused): camera and tags of xc were written
  // by k_update_f, launched before this kernel
  if (with_cost) {
    __syncthreads();
    capture_cost<kChunked>(P, xc, capc, c, parts);
  }
}

// The levels of offset < 64 of a block's pairwise tree reduction
// red[t] = op(red[t], red[t + off]) (off = n/2 .. 1), on wave 0 by lane shifts
// instead of an LDS round trip and a block barrier per level: the same pairs
// in the same order, so the same bits.  v: lane t's red[t] after the level of
// offset 64 (n: the elements left, <= 64); the result lands in lane 0.  All of
// wave 0 must be active.
__device__ __forceinline__ double wave_tree_sum(double v, int n) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
    if (off < n) v += __shfl_down(v, off, kWave);
  return v;
}
__device__ __forceinline__ double wave_tree_max(double v, int n) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1)
    if (off < n) v = fmax(v, __shfl_down(v, off, kWave));
  return v;
}

// Candidate update of the tag and camera slots from the reduced solution
// (every f-side slot of xc is written, so xc needs no copy of x first:
// k_backsub writes every capture slot).
__global__ __launch_bounds__(256) void k_update_f(DevProblem P, const double *__restrict__ x,
                                                  const double *__restrict__ scale,
                                                  const double *__restrict__ yF,
                                                  double *__restrict__ xc,
                                                  double *__restrict__ fparts) {
  __shared__ double red[2][256];
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  double st = 0.0, bad = 0.0;
  const long slot = i < P.nR ? P.row_slot[i] : -1;
  if (slot >= 0) {   // reduced row i
    const double yv = yF[i];
    const double xo = x[slot];
    const double xn = xo + (-yv * scale[slot]);
    xc[slot] = xn;
    // (several ranks: each slot's step counted on the rank holding it)
    if (P.slot_free[slot] && (!P.f_own || P.f_own[slot])) st = (xo - xn) * (xo - xn);
    bad = isfinite(yv) ? 0.0 : 1.0;
  }
  if (i < P.nf && P.fslot_row[i] < 0) {   // f-side slot i outside the reduced system: unchanged
    const long fs = i < 3 ? i : 3 + 6L * P.nc + (i - 3);
    xc[fs] = x[fs];
  }
  if ((long)blockIdx.x * blockDim.x >= P.nR) return;   // (partials: one per 256 reduced rows)
  red[0][threadIdx.x] = st;
  red[1][threadIdx.x] = bad;
  __syncthreads();
  for (int off = 128; off >= kWave; off >>= 1) {
    if (threadIdx.x < off) {
      red[0][threadIdx.x] += red[0][threadIdx.x + off];
      red[1][threadIdx.x] = fmax(red[1][threadIdx.x], red[1][threadIdx.x + off]);
    }
    __syncthreads();
  }
  if (threadIdx.x < kWave) {
    const double s0 = wave_tree_sum(red[0][threadIdx.x], kWave);
    const double s1 = wave_tree_max(red[1][threadIdx.x], kWave);
    if (threadIdx.x == 0) {
      fparts[2L * blockIdx.x] = s0;
      fparts[2L * blockIdx.x + 1] = s1;
    }
  }
}

// Deterministic single-block reduction of the per-capture partials.
// out[p] for p < NPART: sum (max for the *BAD flags); out[NPART] = F-side step^2,
// out[NPART+1] = F-side non-finite flag.
// One block per LM scalar p (deterministic: fixed element -> thread
// assignment, fixed tree); 8 loads in flight per thread.
__device__ __forceinline__ void reduce_parts_block(int p, const double *__restrict__ parts, int nc,
                                                   const double *__restrict__ fparts, int nfparts,
                                                   double *__restrict__ out, const int *__restrict__ flag,
                                                   double *red, double *__restrict__ hout,
                                                   int *seq_done = nullptr, double seq = 0.0,
                                                   double *__restrict__ save = nullptr) {
  const int t = threadIdx.x;
  const bool is_max = (p == P_YBAD || p == P_CBAD || p == NPART + 1);
  const double *src = p < NPART ? parts + (long)p * nc : fparts;
  const int len = p < NPART ? nc : (fparts ? nfparts : 0);
  const int stride = p < NPART ? 1 : 2, off0 = p < NPART ? 0 : p - NPART;
  double acc = 0.0;
  for (int i0 = t; i0 < len; i0 += 8 * 1024) {
    double v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = src[(long)stride * min(i0 + u * 1024, len - 1) + off0];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const double w = (i0 + u * 1024 < len) ? v[u] : 0.0;
      acc = is_max ? fmax(acc, w) : acc + w;
    }
  }
  red[t] = acc;
  __syncthreads();
  for (int off = 512; off >= kWave; off >>= 1) {
    if (t < off) red[t] = is_max ? fmax(red[t], red[t + off]) : red[t] + red[t + off];
    __syncthreads();
  }
  if (t < kWave) {
    const double r = is_max ? wave_tree_max(red[t], kWave) : wave_tree_sum(red[t], kWave);
    if (t == 0) {
      out[p] = r;
      if (hout) hout[p] = r;
      if (save && p < 2) save[p] = r;   // (P_COST, P_FIXED)
    }
  }
  if (flag && p == 0 && t == 0) {   // rides along the step's one host read
    const int f = *flag;
    const double v[3] = {f > 0 ? 1.0 : 0.0,   // indefinite reduced system: an invalid LM step (max over ranks)
                         f < 0 ? 1.0 : 0.0,   // executor fault: an error, never a step (max over ranks)
                         (double)f};          // this rank's raw code, for the error message
    for (int q = 0; q < 3; ++q) {
      out[NPART + 2 + q] = v[q];
      if (hout) hout[NPART + 2 + q] = v[q];
    }
  }
  if (hout && t == 0) {
    // this block's host words out of its XCD's L2 (the blocks span XCDs);
    // then the last block to finish stores the sequence number
    __threadfence_system();
    // acq_rel at system scope: the last block acquires every other block's
    // fenced host stores before its release of the sequence word
    if (seq_done && seq > 0.0 &&
        __hip_atomic_fetch_add(seq_done, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM) == (int)gridDim.x - 1) {
      atomicExch(seq_done, 0);
      __hip_atomic_store(hout + kHostSeq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

__global__ __launch_bounds__(1024) void k_reduce_parts(const double *__restrict__ parts, int nc,
                                                       const double *__restrict__ fparts,
                                                       int nfparts, double *__restrict__ out,
                                                       const int *__restrict__ flag,
                                                       double *__restrict__ hout, int *seq_done, double seq) {
  __shared__ double red[1024];
  reduce_parts_block(blockIdx.x, parts, nc, fparts, nfparts, out, flag, red, hout, seq_done, seq);
}

// The linearization's two reductions of k_linearize's output in one launch
// (they are independent): blocks 0 .. NPART+1 reduce the per-capture partials
// (k_reduce_parts), the rest sum the tag slots (k_tag_reduce, 1024 slots each).
__global__ __launch_bounds__(1024) void k_lin_reduce(DevProblem P, const double *__restrict__ obs_tg,
                                                     double *__restrict__ g, double *__restrict__ colnorm,
                                                     const double *__restrict__ parts, double *__restrict__ out,
                                                     double *__restrict__ hout, double *__restrict__ save) {
  __shared__ double red[1024];
  if ((int)blockIdx.x < NPART + 2)
    reduce_parts_block(blockIdx.x, parts, P.nc, nullptr, 0, out, nullptr, red, hout, nullptr, 0.0, save);
  else
    tag_reduce_elem(P, obs_tg, (long)(blockIdx.x - (NPART + 2)) * 1024 + threadIdx.x, g, colnorm);
}

// Norms over free parameter slots, split into capture slots (out[0..2]) and
// camera + tag slots (out[3..5]): max |g|, sum g^2, sum x^2.  The split lets
// the capture-sharded path reduce only the disjoint capture part across ranks.

__global__ __launch_bounds__(256) void k_slot_norms(long n, long cap_lo, long cap_hi,
                                                    const unsigned char *__restrict__ free_,
                                                    const unsigned char *__restrict__ f_own,
                                                    double *__restrict__ g, double *__restrict__ colnorm,
                                                    const double *__restrict__ red,
                                                    const double *__restrict__ x,
                                                    double *__restrict__ out,
                                                    double *__restrict__ hout, const double *__restrict__ scale,
                                                    double dmin, double dmax, double *__restrict__ diag, double seq) {
  __shared__ double rs[6][256];
  __shared__ int last;
  const int t = threadIdx.x;
  // the camera slots from the reduced per-capture partials (f gradient and
  // column norm; l1, l2 have no Jacobian column): written once, and used here
  // in place of g[0..2]
  const double g0 = free_[0] ? red[P_GF] : 0.0;
  if (blockIdx.x == 0 && t == 0) {
    g[0] = g0;
    colnorm[0] = free_[0] ? red[P_CF] : 0.0;
    g[1] = g[2] = 0.0;
    colnorm[1] = colnorm[2] = 0.0;
  }
  const double cn0 = free_[0] ? red[P_CF] : 0.0;   // (colnorm[0], as block 0 writes it)
  double v[6] = {0, 0, 0, 0, 0, 0};
  for (long i = (long)blockIdx.x * 256 + t; i < n; i += (long)kNormBlocks * 256) {
    if (diag) {   // the LM diagonal of the new linearization (launch_exec_reset's k_lm_diag work)
      const double cn = i >= 3 ? colnorm[i] : (i == 0 ? cn0 : 0.0);
      diag[i] = fmin(fmax(scale[i] * scale[i] * cn, dmin), dmax);
    }
    // (several ranks: each slot counted on the rank holding it, DevProblem::f_own)
    if (!free_[i] || (f_own && !f_own[i])) continue;
    const int o = (i >= cap_lo && i < cap_hi) ? 0 : 3;
    const double gv = i >= 3 ? g[i] : (i == 0 ? g0 : 0.0), xv = x[i];
    v[o] = fmax(v[o], fabs(gv));
    v[o + 1] += gv * gv;
    v[o + 2] += xv * xv;
  }
  for (int q = 0; q < 6; ++q) rs[q][t] = v[q];
  __syncthreads();
  for (int off = 128; off >= kWave; off >>= 1) {
    if (t < off) {
      rs[0][t] = fmax(rs[0][t], rs[0][t + off]);
      rs[1][t] += rs[1][t + off];
      rs[2][t] += rs[2][t + off];
      rs[3][t] = fmax(rs[3][t], rs[3][t + off]);
      rs[4][t] += rs[4][t + off];
      rs[5][t] += rs[5][t + off];
    }
    __syncthreads();
  }
  if (t < kWave)
    for (int q = 0; q < 6; ++q) {
      const double r = (q % 3 == 0) ? wave_tree_max(rs[q][t], kWave) : wave_tree_sum(rs[q][t], kWave);
      if (t == 0) rs[q][0] = r;
    }
  // out[8 + 6 b + q]: block b's partials; out[7] (as an int): blocks done.
  // The last block to finish reduces the kNormBlocks partials over a fixed
  // tree (independent of which block is last) into out[0..5], and resets the
  // count for the next launch.
  double *part = out + 8;
  int *done = reinterpret_cast<int *>(out + 7);
  if (t == 0) {
    for (int q = 0; q < 6; ++q) part[6L * blockIdx.x + q] = rs[q][0];
    __threadfence();   // the partials before the count (agent scope: the blocks span XCDs)
    last = atomicAdd(done, 1) == kNormBlocks - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();     // every block's partials after the count
  if (t < kNormBlocks)
    for (int q = 0; q < 6; ++q) rs[q][t] = part[6L * t + q];
  __syncthreads();
  for (int off = kNormBlocks / 2; off >= kWave; off >>= 1) {
    if (t < off)
      for (int q = 0; q < 6; ++q)
        rs[q][t] = (q % 3 == 0) ? fmax(rs[q][t], rs[q][t + off]) : rs[q][t] + rs[q][t + off];
    __syncthreads();
  }
  if (t < kWave) {
    const int left = kNormBlocks < kWave ? kNormBlocks : kWave;
    double r6[6];
    for (int q = 0; q < 6; ++q) {
      const double v0 = t < left ? rs[q][t] : 0.0;
      r6[q] = (q % 3 == 0) ? wave_tree_max(v0, left) : wave_tree_sum(v0, left);
    }
    if (t == 0)
      for (int q = 0; q < 6; ++q) rs[q][0] = r6[q];
  }
  __syncthreads();
  if (t < 6) {
    out[t] = rs[t][0];
    if (hout) {
      hout[t] = rs[t][0];
      __threadfence_system();
    }
  }
  if (t == 0) atomicExch(done, 0);
  if (hout && seq > 0.0) {
    __syncthreads();
    if (t == 0) __hip_atomic_store(hout + kHostSeq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---- multi-rank exchange buffers (lm_solver.hip) ----
// Segments copied into (unpack = 0) or out of (1) one contiguous buffer, so
// several arrays cross the ranks in one all-reduce.
__global__ void k_pack(PackSegs sg, double *__restrict__ buf, int unpack) {
  long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (int q = 0; q < sg.n; ++q) {
    if (e < sg.len[q]) {
      if (unpack) sg.p[q][e] = buf[sg.off[q] + e];
      else buf[sg.off[q] + e] = sg.p[q][e];
      return;
    }
    e -= sg.len[q];
  }
}

__global__ void k_top_tail(const int *__restrict__ idx, int m, double *__restrict__ g, double *__restrict__ cn,
                           double *__restrict__ red, double *__restrict__ tail, int unpack) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= 2 * m + 2) return;
  double *v = e < m ? g + idx[e] : e < 2 * m ? cn + idx[e - m] : red + (e == 2 * m ? P_GF : P_CF);
  if (unpack) *v = tail[e];
  else tail[e] = *v;
}

// All-gather of a few scalars through one SUM all-reduce: this rank's fields
// (src[idx[f]]) into row `rank` of ag[nranks][kAgFields], every other row 0
// (x + 0 is exact, so the all-reduce hands every rank every rank's values)
__global__ void k_ag_put(const double *__restrict__ src, AgFields fl, double *__restrict__ ag, int nranks, int rank) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nranks * kAgFields) return;
  const int r = e / kAgFields, f = e % kAgFields;
  ag[e] = (r == rank && f < fl.n) ? src[fl.idx[f]] : 0.0;
}

// ... and their combination in rank order (sum, or max where fl.max bit f is
// set), the same bits on every rank, written back to dst[idx[f]]
__global__ void k_ag_reduce(const double *__restrict__ ag, AgFields fl, double *__restrict__ dst, int nranks,
                            HostOut ho) {
  const int f = threadIdx.x;
  if (f < fl.n) {
    const bool mx = (fl.max >> f) & 1u;
    double v = ag[f];
    for (int r = 1; r < nranks; ++r) {
      const double w = ag[r * kAgFields + f];
      v = mx ? fmax(v, w) : v + w;
    }
    dst[fl.idx[f]] = v;
  }
  if (!ho.seq_word) return;
  // the host's words (after every combined value: one block), fenced at
  // system scope, then the sequence number the host polls
  __syncthreads();
  for (int q = 0; q < ho.n; ++q)
    for (int e = f; e < ho.len[q]; e += blockDim.x) ho.dst[q][e] = ho.src[q][e];
  __threadfence_system();
  __syncthreads();
  if (f == 0) __hip_atomic_store(ho.seq_word, ho.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one thread per (observation, row): residual and 15-column Jacobian row
__global__ void k_debug_rj(int n, const double *__restrict__ cam, const double *__restrict__ cap,
                           const double *__restrict__ tag, const double *__restrict__ corners,
                           double *__restrict__ r, double *__restrict__ J) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= 8L * n) return;
  const long o = e / 8;
  const int row = (int)(e % 8), corner = row >> 1, comp = row & 1;
  double j13[13];
  r[e] = residual_jacobian_row(cam + 3 * o, cap + 6 * o, tag + 6 * o, corner, comp,
                               corners[8 * o + row], j13);
  double *out = J + e * 15;
  out[0] = j13[0];
  out[1] = 0.0;
  out[2] = 0.0;
  for (int j = 0; j < 12; ++j) out[3 + j] = j13[1 + j];
}

// AngleAxisRotatePoint of n (w, p) pairs with the branch each one took
// (1: theta^2 > DBL_EPSILON, Rodrigues; 0: x + w x p) -- parity of the
// small-angle branch, ar_slam_util.cpp:145,155.
__global__ void k_debug_aa(int n, const double *__restrict__ w, const double *__restrict__ p,
                           double *__restrict__ out, int *__restrict__ branch) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const AngleAxis a = aa_prepare(w + 3L * i);
  aa_rotate(a, p + 3L * i, out + 3L * i);
  branch[i] = a.big ? 1 : 0;
}

// test hook: S[row,row] = v after the LM diagonal was added (a forced
// indefinite reduced system, arslam_lm_debug_force_indefinite)
__global__ void k_debug_set_diag(DevProblem P, double *S, long row, double v) {
  if (threadIdx.x == 0) *reduced_elem(S, P, row, row) = v;
}

size_t lds_rows(int maxk) { return (size_t)8 * maxk * kRowStride * sizeof(double); }

}  // namespace

// ---------------------------------------------------------------------------
// launch wrappers
// ---------------------------------------------------------------------------

void launch_linearize(const DevProblem &P, const double *x, double *g, double *colnorm,
                      double *obs_tg, double *parts, hipStream_t s) {
  if (P.nc == 0) return;
  const size_t lds = lds_rows(kObsChunk) + sizeof(double) * (kObsChunk + 16);
  hipLaunchKernelGGL(k_linearize<false>, dim3(P.nc), dim3(kWave), lds, s, P, x, g, colnorm, obs_tg, parts);
  if (P.n_chunk_caps)
    hipLaunchKernelGGL(k_linearize<true>, dim3(P.n_chunk_caps), dim3(kWave), lds, s, P, x, g, colnorm, obs_tg, parts);
}

void launch_lin_reduce(const DevProblem &P, const double *obs_tg, double *g, double *colnorm,
                       const double *parts, double *out, hipStream_t s, double *hout, double *save) {
  const unsigned tag_blocks = (unsigned)((12L * P.nt + 1023) / 1024);
  hipLaunchKernelGGL(k_lin_reduce, dim3(NPART + 2 + tag_blocks), dim3(1024), 0, s, P, obs_tg, g, colnorm, parts,
                     out, hout, save);
}

void launch_scale(const DevProblem &P, const double *colnorm, int jacobi, double *scale, hipStream_t s,
                  const LmDiagArgs *ld) {
  hipLaunchKernelGGL(k_scale, dim3((unsigned)((P.n + 255) / 256)), dim3(256), 0, s, P.n, P.slot_free,
                     colnorm, jacobi, scale, ld ? ld->dmin : 0.0, ld ? ld->dmax : 0.0, ld ? ld->diag : nullptr);
}

void launch_lm_diag(const DevProblem &P, const double *scale, const double *colnorm, double dmin,
                    double dmax, double *diag, hipStream_t s) {
  hipLaunchKernelGGL(k_lm_diag, dim3((unsigned)((P.n + 255) / 256)), dim3(256), 0, s, P.n, scale,
                     colnorm, dmin, dmax, diag);
}

// k_schur<true>'s dynamic-LDS limit on the current device, once per device
// (the attribute is per device; several host threads may reach it at once): a
// failure is an error, not a launch that later fails for its LDS size.  Called
// where the device is made current (ensure_stream), not per launch.
void set_schur_big_lds_attribute() {
  static std::mutex m;
  static std::vector<char> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) throw ApiError(ARSLAM_E_HIP, "hipGetDevice");
  std::lock_guard<std::mutex> g(m);
  if ((int)done.size() <= dev) done.resize(dev + 1, 0);
  if (done[dev]) return;
  const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_schur<true>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)schur_lds_bytes(kMaxSchurBlocks));
  if (e != hipSuccess)
    throw ApiError(ARSLAM_E_HIP, std::string("hipFuncSetAttribute(k_schur, dynamic LDS): ") + hipGetErrorString(e));
  done[dev] = 1;
}

void launch_schur(const DevProblem &P, const double *x, const double *scale, const double *diag,
                  double radius, double *S, hipStream_t s, bool prep, long zero_tiles, const ExecReset *er) {
  const ExecReset r = er ? *er : ExecReset{};
  if (P.nc == 0) {
    if (zero_tiles) (void)hipMemsetAsync(S, 0, (size_t)zero_tiles * 4096 * sizeof(double), s);
    if (prep) launch_prep_reduced(P, diag, radius, S, s);
    return;
  }
  // the main launch: captures of at most kSchurMfmaBlocks distinct tags (and
  // the tile clears and the executor reset); a second one, its LDS sized for
  // them, takes the captures with more
  const size_t lds = schur_lds_bytes(std::min(P.max_blk_per_cap, kSchurMfmaBlocks));
  const long reset_blocks = (r.n() + kWave - 1) / kWave;
  hipLaunchKernelGGL(k_schur<false>, dim3((unsigned)(P.nc + zero_tiles + reset_blocks)), dim3(kWave), lds, s, P, scale,
                     diag, radius, S, zero_tiles, r, (const int *)nullptr);
  if (P.n_big_caps > 0) {
    const size_t lds_big = schur_lds_bytes(P.max_blk_per_cap);
    // (dynamic LDS past 64 KiB: set once per device by the caller, ensure_stream)
    hipLaunchKernelGGL(k_schur<true>, dim3((unsigned)P.n_big_caps), dim3(kWave), lds_big, s, P, scale, diag, radius, S,
                       0L, ExecReset{}, P.big_caps);
  }
  const double *pd = prep ? diag : nullptr;
  const unsigned gb = (unsigned)((P.n_items + 3) / 4) + (prep ? (unsigned)((P.N + 255) / 256) : 0u);
  if (gb) hipLaunchKernelGGL(k_schur_gather, dim3(gb), dim3(256), 0, s, P, S, pd, radius);
  if (P.n_splits)
    hipLaunchKernelGGL(k_schur_combine, dim3((unsigned)((P.n_splits + 3) / 4)), dim3(256), 0, s, P, S, pd,
                       radius);
}

void launch_prep_reduced(const DevProblem &P, const double *diag, double radius, double *S,
                         hipStream_t s, int which) {
  hipLaunchKernelGGL(k_prep_reduced, dim3((unsigned)((P.N + 255) / 256)), dim3(256), 0, s, P, diag,
                     radius, S, which);
}

void launch_mask_y(const DevProblem &P, double *yF, int rank, hipStream_t s, bool keep_top) {
  if (P.nR == 0) return;
  hipLaunchKernelGGL(k_mask_y, dim3((unsigned)((P.nR + 255) / 256)), dim3(256), 0, s, P, yF, rank, keep_top ? 1 : 0);
}

void launch_own_copy(const DevProblem &P, long first, long count, const double *src, double *dst, hipStream_t s) {
  if (count <= 0) return;
  hipLaunchKernelGGL(k_own_copy, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, P, first, count, src, dst);
}

void launch_backsub(const DevProblem &P, const double *x, const double *scale, const double *diag,
                    double radius, const double *yF, double *xc, double *parts, hipStream_t s,
                    bool reuse_ui, bool with_cost) {
  if (P.nc == 0) return;
  const size_t lds = lds_rows(kObsChunk) + sizeof(double) * (8L * kObsChunk + 36 + 36 + 16);
  hipLaunchKernelGGL(k_backsub<false>, dim3(P.nc), dim3(kWave), lds, s, P, x, scale, diag, radius, yF, xc, parts,
                     reuse_ui ? 1 : 0, with_cost ? 1 : 0);
  if (P.n_chunk_caps)
    hipLaunchKernelGGL(k_backsub<true>, dim3(P.n_chunk_caps), dim3(kWave), lds, s, P, x, scale, diag, radius, yF, xc,
                       parts, reuse_ui ? 1 : 0, with_cost ? 1 : 0);
}

void launch_update_f(const DevProblem &P, const double *x, const double *scale, const double *yF,
                     double *xc, double *fparts, hipStream_t s) {
  const long n = std::max<long>(P.nR, P.nf);
  if (n == 0) return;
  hipLaunchKernelGGL(k_update_f, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, P, x, scale, yF, xc, fparts);
}

void launch_cost(const DevProblem &P, const double *x, double *parts, hipStream_t s) {
  if (P.nc == 0) return;
  hipLaunchKernelGGL(k_cost<false>, dim3(P.nc), dim3(kWave), 0, s, P, x, parts);
  if (P.n_chunk_caps) hipLaunchKernelGGL(k_cost<true>, dim3(P.n_chunk_caps), dim3(kWave), 0, s, P, x, parts);
}

// The parameter download on one rank: a kernel stores x straight into the
// page-locked host buffer and the last block to finish stores the sequence
// number after every block's stores were made visible at system scope (the
// host polls that word, as in the LM loop) -- no copy engine, no event.
__global__ __launch_bounds__(256) void k_copy_out(const double *__restrict__ src, long n, double *__restrict__ dst,
                                                  int *seq_done, double *word, double seq) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) dst[i] = src[i];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0 &&
      __hip_atomic_fetch_add(seq_done, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM) == (int)gridDim.x - 1) {
    atomicExch(seq_done, 0);
    __hip_atomic_store(word, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

void launch_copy_out(const double *src, long n, double *dst, int *seq_done, double *word, double seq, hipStream_t s) {
  const unsigned blocks = (unsigned)std::min<long>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(k_copy_out, dim3(std::max(blocks, 1u)), dim3(256), 0, s, src, n, dst, seq_done, word, seq);
}

void launch_reduce_parts(const double *parts, int nc, const double *fparts, int nfparts, double *out,
                         hipStream_t s, const int *flag, double *hout, int *seq_done, double seq) {
  hipLaunchKernelGGL(k_reduce_parts, dim3(NPART + 2), dim3(1024), 0, s, parts, nc, fparts, nfparts, out, flag, hout,
                     seq_done, seq);
}

void launch_slot_norms(const DevProblem &P, const double *red, double *g, double *colnorm, const double *x,
                       double *out, hipStream_t s, double *hout, const LmDiagArgs *ld, double seq) {
  // out[0..5] results, out[7] the block count (zero between launches), out[8..] the per-block partials
  hipLaunchKernelGGL(k_slot_norms, dim3(kNormBlocks), dim3(256), 0, s, P.n, 3L, 3L + 6L * P.nc, P.slot_free, P.f_own, g,
                     colnorm, red, x, out, hout, ld ? ld->scale : nullptr, ld ? ld->dmin : 0.0,
                     ld ? ld->dmax : 0.0, ld ? ld->diag : nullptr, seq);
}

void launch_pack(const PackSegs &sg, double *buf, bool unpack, hipStream_t s) {
  long tot = 0;
  for (int q = 0; q < sg.n; ++q) tot += sg.len[q];
  if (tot == 0) return;
  hipLaunchKernelGGL(k_pack, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, sg, buf, unpack ? 1 : 0);
}

void launch_top_tail(const int *idx, int m, double *g, double *cn, double *red, double *tail, bool unpack,
                     hipStream_t s) {
  hipLaunchKernelGGL(k_top_tail, dim3((unsigned)((2 * m + 2 + 255) / 256)), dim3(256), 0, s, idx, m, g, cn, red, tail,
                     unpack ? 1 : 0);
}

void launch_ag_put(const double *src, const AgFields &fl, double *ag, int nranks, int rank, hipStream_t s) {
  hipLaunchKernelGGL(k_ag_put, dim3((unsigned)((nranks * kAgFields + 255) / 256)), dim3(256), 0, s, src, fl, ag,
                     nranks, rank);
}

void launch_ag_reduce(const double *ag, const AgFields &fl, double *dst, int nranks, hipStream_t s,
                      const HostOut *ho) {
  hipLaunchKernelGGL(k_ag_reduce, dim3(1), dim3(kAgFields), 0, s, ag, fl, dst, nranks, ho ? *ho : HostOut{});
}

void debug_residual_jacobian(int n, const double *cam, const double *cap, const double *tag,
                             const double *corners, double *r, double *J, hipStream_t s) {
  const long m = 8L * n;
  hipLaunchKernelGGL(k_debug_rj, dim3((unsigned)((m + 127) / 128)), dim3(128), 0, s, n, cam, cap, tag,
                     corners, r, J);
}

void debug_set_reduced_diag(const DevProblem &P, double *S, long row, double v, hipStream_t s) {
  hipLaunchKernelGGL(k_debug_set_diag, dim3(1), dim3(64), 0, s, P, S, row, v);
}

void debug_angle_axis(int n, const double *w, const double *p, double *out, int *branch, hipStream_t s) {
  hipLaunchKernelGGL(k_debug_aa, dim3((unsigned)((n + 127) / 128)), dim3(128), 0, s, n, w, p, out, branch);
}

}  // namespace arslam
