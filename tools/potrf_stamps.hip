// Diagnostic micro-benchmark: where wave 0's time goes inside
// blocked_potrf64_async with the fold (the chain's POTRF of a claimed
// continuation), one workgroup alone on the chip: s_memtime stamps
// (ARSLAM_STAMPS) at each phase of wave 0, averaged over reps.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -DARSLAM_STAMPS -I include
//   -I ar_slam_amd/csrc tools/potrf_stamps.hip -o tools/potrf_stamps
#include "../ar_slam_amd/csrc/dense_llt.hip"

#include <cstdio>
#include <vector>

using namespace arslam;

namespace {
__global__ __launch_bounds__(256) void k_bench(const double *A, const double *Fg, int reps, unsigned long long *acc) {
  __shared__ __attribute__((aligned(16))) double D[T64 * LQ];
  __shared__ __attribute__((aligned(16))) double F[T64 * LQ];
  __shared__ double inv[T64];
  __shared__ __attribute__((aligned(16))) double LTd[4 * 16 * LI];
  __shared__ double colx[64];
  __shared__ int bad;
  __shared__ int fl[8];
  const int tid = threadIdx.x;
  __builtin_amdgcn_s_setprio(3);
  for (int e = tid; e < 4096; e += 256) F[(e >> 6) * LQ + (e & 63)] = Fg[e];
  for (int r = 0; r < reps; ++r) {
    for (int e = tid; e < 4096; e += 256) D[(e >> 6) * LQ + (e & 63)] = (e & 63) <= (e >> 6) ? A[e] : -7.0;
    __syncthreads();
    auto none = [](int, int, int) {};
    blocked_potrf64_async(D, inv, LTd, &bad, fl, tid, colx, none, F, true, fl + 4);
    __syncthreads();
    if (tid == 0 && r > 0)
      for (int i = 31; i < 54; ++i) acc[i] += g_stamps[i] - g_stamps[30];
  }
}
}  // namespace

int main() {
  std::vector<double> h(4096), f(4096);
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) {
      h[i * 64 + j] = (i == j) ? 130.0 : 1.0 / (1.0 + i + j);
      f[i * 64 + j] = 0.05 * std::sin(1.0 + i * 0.3 + j * 0.7);
    }
  double *A, *Fg;
  unsigned long long *acc;
  (void)hipMalloc(&A, 4096 * 8);
  (void)hipMalloc(&Fg, 4096 * 8);
  (void)hipMalloc(&acc, 64 * 8);
  (void)hipMemset(acc, 0, 64 * 8);
  (void)hipMemcpy(A, h.data(), 4096 * 8, hipMemcpyHostToDevice);
  (void)hipMemcpy(Fg, f.data(), 4096 * 8, hipMemcpyHostToDevice);
  const int reps = 201;
  hipLaunchKernelGGL(k_bench, dim3(1), dim3(256), 0, 0, A, Fg, reps, acc);
  unsigned long long o[64];
  (void)hipMemcpy(o, acc, 64 * 8, hipMemcpyDeviceToHost);
  const char *nm[6] = {"gemm/fold done", "waited rounds", "diag16 done", "waited round p+1", "apply done", ""};
  double prev = 0;
  for (int p = 0; p < 4; ++p)
    for (int q = 0; q < 5; ++q) {
      const int id = 31 + 6 * p + q;
      if (p == 3 && q > 2) continue;
      const double c = (double)o[id] / (reps - 1);
      printf("p%d %-18s at %7.0f cycles  (+%6.0f)\n", p, nm[q], c, c - prev);
      prev = c;
    }
  return 0;
}
