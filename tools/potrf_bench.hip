// Diagnostic micro-benchmark: blocked_potrf64 (dense_llt.hip) on one
// workgroup, alone on the chip, timed with s_memrealtime (100 MHz) around
// each call.  Build: hipcc --offload-arch=gfx950 -O3 -I include -I ar_slam_amd/csrc
//   tools/potrf_bench.hip -o tools/potrf_bench
#define ARSLAM_STAMPS 1
#include "../ar_slam_amd/csrc/dense_llt.hip"

#include <cstdio>
#include <vector>

using namespace arslam;

namespace {
__global__ __launch_bounds__(256) void k_bench(const double *A, int reps, unsigned long long *out, double *res,
                                               int prio) {
  __shared__ __attribute__((aligned(16))) double D[T64 * LQ];
  __shared__ double inv[T64];
  __shared__ __attribute__((aligned(16))) double LTd[4 * 16 * LI];
  __shared__ double colx[64];
  __shared__ int bad;
  const int tid = threadIdx.x;
  if (prio) __builtin_amdgcn_s_setprio(3);
  unsigned long long tot = 0, best = ~0ull;
  for (int r = 0; r < reps; ++r) {
    for (int e = tid; e < 4096; e += 256)   // lower triangle only, as in the factor's tiles
      D[(e >> 6) * LQ + (e & 63)] = (e & 63) <= (e >> 6) ? A[e] : -7.0;
    __syncthreads();
    const unsigned long long t0 = realtime();
    blocked_potrf64(D, inv, LTd, &bad, tid, colx);
    __syncthreads();
    const unsigned long long t1 = realtime();
    tot += t1 - t0;
    best = t1 - t0 < best ? t1 - t0 : best;
  }
  if (tid == 0) { out[0] = tot; out[1] = best; }
  for (int e = tid; e < 4096; e += 256) res[e] = D[(e >> 6) * LQ + (e & 63)];
}
}  // namespace

int main() {
  std::vector<double> h(4096);
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) h[i * 64 + j] = (i == j) ? 65.0 : 1.0 / (1.0 + i + j);
  double *A, *res;
  unsigned long long *out;
  hipMalloc(&A, 4096 * 8);
  hipMalloc(&res, 4096 * 8);
  hipMalloc(&out, 16);
  hipMemcpy(A, h.data(), 4096 * 8, hipMemcpyHostToDevice);
  const int reps = 200;
  hipLaunchKernelGGL(k_bench, dim3(1), dim3(256), 0, 0, A, reps, out, res, 0);
  unsigned long long o[2];
  hipMemcpy(o, out, 16, hipMemcpyDeviceToHost);
  std::vector<double> L(4096);
  hipMemcpy(L.data(), res, 4096 * 8, hipMemcpyDeviceToHost);
  double err = 0;   // |L L^T - A| on the lower triangle
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = 0;
      for (int k = 0; k <= j; ++k) s += L[i * 64 + k] * L[j * 64 + k];
      err = std::max(err, std::fabs(s - h[i * 64 + j]));
    }
  unsigned long long st[64];
  hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof(st));
  for (int p = 0; p < 4; ++p)
    printf("  p%d: [lookahead update +] diag factor+inv %llu, rows below %llu (s_memtime ticks)\n", p,
           st[11 + 4 * p] - st[10 + 4 * p], st[12 + 4 * p] - st[11 + 4 * p]);
  {   // host Cholesky, error per 16x16 block of L
    std::vector<double> Lh(4096, 0.0);
    for (int j = 0; j < 64; ++j) {
      double d = h[j * 64 + j];
      for (int k = 0; k < j; ++k) d -= Lh[j * 64 + k] * Lh[j * 64 + k];
      Lh[j * 64 + j] = std::sqrt(d);
      for (int i = j + 1; i < 64; ++i) {
        double v = h[i * 64 + j];
        for (int k = 0; k < j; ++k) v -= Lh[i * 64 + k] * Lh[j * 64 + k];
        Lh[i * 64 + j] = v / Lh[j * 64 + j];
      }
    }
    for (int I = 0; I < 4; ++I) {
      for (int J = 0; J <= I; ++J) {
        double e = 0;
        for (int i = 0; i < 16; ++i)
          for (int j = 0; j < 16; ++j) {
            const int r = 16 * I + i, c = 16 * J + j;
            if (r >= c) e = std::max(e, std::fabs(L[r * 64 + c] - Lh[r * 64 + c]));
          }
        printf(" %.1e", e);
      }
      printf("\n");
    }
    printf("L00 row 3: ");
    for (int c = 0; c < 5; ++c) printf("%.6f/%.6f ", L[3 * 64 + c], Lh[3 * 64 + c]);
    printf("\n");
  }
  printf("blocked_potrf64 alone: mean %.2f us, best %.2f us, max|LL'-A| %.2e\n", o[0] / 100.0 / reps, o[1] / 100.0, err);
  return 0;
}
