// Diagnostic micro-benchmark: the POTRF variants of dense_llt.hip on one
// workgroup alone on the chip, timed with s_memrealtime (100 MHz) per call:
//   v1       blocked_potrf64 (workgroup barriers between panels)
//   v2       blocked_potrf64_async (LDS counters)
//   v1+fold  blocked_potrf64_idle with the fold D -= F F^T
//   v2+fold  blocked_potrf64_async with the fold
//   diag16x4 the four diagonal-block factorizations alone (the chain's floor)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I ar_slam_amd/csrc
//   tools/potrf2_bench.hip -o tools/potrf2_bench
#include "../ar_slam_amd/csrc/dense_llt.hip"

#include <cstdio>
#include <vector>

using namespace arslam;

namespace {
__global__ __launch_bounds__(256) void k_bench(const double *A, const double *Fg, int reps, int variant,
                                               unsigned long long *out, double *res) {
  __shared__ __attribute__((aligned(16))) double D[T64 * LQ];
  __shared__ __attribute__((aligned(16))) double F[T64 * LQ];
  __shared__ double inv[T64];
  __shared__ __attribute__((aligned(16))) double LTd[4 * 16 * LI];
  __shared__ double colx[64];
  __shared__ int bad;
  __shared__ int fl[8];
  const int tid = threadIdx.x;
  __builtin_amdgcn_s_setprio(3);
  unsigned long long tot = 0, best = ~0ull;
  for (int e = tid; e < 4096; e += 256) F[(e >> 6) * LQ + (e & 63)] = Fg[e];
  for (int r = 0; r < reps; ++r) {
    for (int e = tid; e < 4096; e += 256)
      D[(e >> 6) * LQ + (e & 63)] = (e & 63) <= (e >> 6) ? A[e] : -7.0;
    __syncthreads();
    const unsigned long long t0 = realtime();
    const bool fold = variant == 2 || variant == 3;
    auto none = [](int, int, int) {};
    if (variant == 0) blocked_potrf64(D, inv, LTd, &bad, tid, colx);
    else if (variant == 1) blocked_potrf64_async(D, inv, LTd, &bad, fl, tid, colx, none);
    else if (variant == 2) blocked_potrf64_idle(D, inv, LTd, &bad, tid, colx, none, F);
    else if (variant == 3) blocked_potrf64_async(D, inv, LTd, &bad, fl, tid, colx, none, F, true, fl + 4);
    else if (tid < 64) {
      for (int p = 0; p < 4; ++p) diag16(D, 16 * p, inv, LTd + p * 16 * LI, &bad, tid, colx);
    }
    (void)fold;
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
  std::vector<double> h(4096), f(4096);
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) {
      h[i * 64 + j] = (i == j) ? 130.0 : 1.0 / (1.0 + i + j);
      f[i * 64 + j] = 0.05 * std::sin(1.0 + i * 0.3 + j * 0.7);
    }
  double *A, *Fg, *res;
  unsigned long long *out;
  hipMalloc(&A, 4096 * 8);
  hipMalloc(&Fg, 4096 * 8);
  hipMalloc(&res, 4096 * 8);
  hipMalloc(&out, 16);
  hipMemcpy(A, h.data(), 4096 * 8, hipMemcpyHostToDevice);
  hipMemcpy(Fg, f.data(), 4096 * 8, hipMemcpyHostToDevice);
  const int reps = 200;
  const char *names[] = {"v1", "v2", "v1+fold", "v2+fold", "diag16x4"};
  std::vector<double> ref;
  for (int v = 0; v < 5; ++v) {
    hipLaunchKernelGGL(k_bench, dim3(1), dim3(256), 0, 0, A, Fg, reps, v, out, res);
    unsigned long long o[2];
    hipMemcpy(o, out, 16, hipMemcpyDeviceToHost);
    std::vector<double> L(4096);
    hipMemcpy(L.data(), res, 4096 * 8, hipMemcpyDeviceToHost);
    double diff = 0;
    if (v == 1 || v == 3) {
      for (int i = 0; i < 64; ++i)
        for (int j = 0; j <= i; ++j) diff = std::max(diff, std::fabs(L[i * 64 + j] - ref[i * 64 + j]));
    }
    if (v == 0 || v == 2) ref = L;
    printf("%-9s mean %.2f us, best %.2f us%s %.1e\n", names[v], o[0] / 100.0 / reps, o[1] / 100.0,
           (v == 1 || v == 3) ? "  max|diff vs barrier version|" : "", diff);
  }
  return 0;
}
