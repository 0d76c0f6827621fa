// Diagnostic micro-benchmark: one diag16 call (16x16 diagonal-block
// elimination of dense_llt.hip) on one wave, alone on the chip, in cycles
// (s_memtime) per call, plus its error against a host Cholesky.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I ar_slam_amd/csrc
//   tools/diag16_bench.hip -o tools/diag16_bench
#include "../ar_slam_amd/csrc/dense_llt.hip"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

using namespace arslam;

namespace {
__device__ __forceinline__ unsigned long long clk() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

__global__ __launch_bounds__(64) void k_bench(const double *A, int reps, unsigned long long *out, double *res) {
  __shared__ __attribute__((aligned(16))) double D[16 * LQ];
  __shared__ double inv[16];
  __shared__ __attribute__((aligned(16))) double Li[16 * LI];
  __shared__ double colx[64];
  __shared__ int bad;
  const int lane = threadIdx.x;
  unsigned long long tot = 0, best = ~0ull;
  for (int r = 0; r < reps; ++r) {
    for (int e = lane; e < 256; e += 64) D[(e >> 4) * LQ + (e & 15)] = A[e];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    const unsigned long long t0 = clk();
    diag16(D, 0, inv, Li, &bad, lane, colx);
    const unsigned long long t1 = clk();
    tot += t1 - t0;
    best = t1 - t0 < best ? t1 - t0 : best;
    __syncthreads();
  }
  if (lane == 0) { out[0] = tot; out[1] = best; }
  for (int e = lane; e < 256; e += 64) res[e] = D[(e >> 4) * LQ + (e & 15)];
}
}  // namespace

int main() {
  std::vector<double> h(256);
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) h[i * 16 + j] = (i == j) ? 17.0 : 1.0 / (1.0 + i + j);
  double *A, *res;
  unsigned long long *out;
  (void)hipMalloc(&A, 256 * 8);
  (void)hipMalloc(&res, 256 * 8);
  (void)hipMalloc(&out, 16);
  (void)hipMemcpy(A, h.data(), 256 * 8, hipMemcpyHostToDevice);
  const int reps = 500;
  hipLaunchKernelGGL(k_bench, dim3(1), dim3(64), 0, 0, A, reps, out, res);
  unsigned long long o[2];
  (void)hipMemcpy(o, out, 16, hipMemcpyDeviceToHost);
  std::vector<double> L(256);
  (void)hipMemcpy(L.data(), res, 256 * 8, hipMemcpyDeviceToHost);
  double err = 0;
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = 0;
      for (int k = 0; k <= j; ++k) s += L[i * 16 + k] * L[j * 16 + k];
      err = std::max(err, std::fabs(s - h[i * 16 + j]));
    }
  unsigned long long hsh = 1469598103934665603ull;   // the factor's bits (variant builds compare it)
  for (double v : L) {
    unsigned long long u;
    std::memcpy(&u, &v, 8);
    hsh = (hsh ^ u) * 1099511628211ull;
  }
  printf("diag16: mean %.0f cycles, best %llu cycles (%.1f per pivot), max|LL'-A| %.2e, factor hash %016llx\n",
         (double)o[0] / reps, o[1], o[1] / 16.0, err, hsh);
  return 0;
}
