// Diagnostic micro-benchmark (one workgroup alone on the chip): the 64x64
// POTRF followed by the fused solve X L^T = A of a second tile, against the
// same solve pipelined into the POTRF (waves 1-3 apply column step p of the
// solve beside the later panels, the last step after the factorization).
// Times in us (s_memrealtime, 100 MHz) from the start to X solved.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I ar_slam_amd/csrc
//   tools/pipe_bench.hip -o tools/pipe_bench
#include "../ar_slam_amd/csrc/dense_llt.hip"

#include <cstdio>
#include <vector>

using namespace arslam;

namespace {
__global__ __launch_bounds__(256) void k_bench(const double *A, const double *Xg, int reps, int variant,
                                               unsigned long long *out, double *res) {
  __shared__ __attribute__((aligned(16))) double D[T64 * LQ];
  __shared__ __attribute__((aligned(16))) double X[T64 * LQ];
  __shared__ double inv[T64];
  __shared__ __attribute__((aligned(16))) double LTd[4 * 16 * LI];
  __shared__ double colx[64];
  __shared__ int bad;
  __shared__ int fl[8];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  __builtin_amdgcn_s_setprio(3);
  unsigned long long tot = 0, best = ~0ull;
  for (int r = 0; r < reps; ++r) {
    for (int e = tid; e < 4096; e += 256) {
      D[(e >> 6) * LQ + (e & 63)] = (e & 63) <= (e >> 6) ? A[e] : -7.0;
      X[(e >> 6) * LQ + (e & 63)] = Xg[e];
    }
    __syncthreads();
    const unsigned long long t0 = realtime();
    if (variant == 0) {
      auto none = [](int, int, int) {};
      blocked_potrf64_async(D, inv, LTd, &bad, fl, tid, colx, none);
      blocked_trsm64(X, D, inv, LTd, tid);
    } else {
      // steps 0..2 beside the panels: idle(q) (q >= 1) follows panel q-1's
      // applies, so column step q-1 of the solve is possible there; wave 1
      // takes row blocks 0 and 3, waves 2 and 3 one each
      auto pipe = [&](int q, int wv, int ln) {
        if (q == 0) return;
        if (wv == 1) {
          trsm_step(X, D, LTd, 0, q - 1, ln);
          trsm_step(X, D, LTd, 3, q - 1, ln);
        } else {
          trsm_step(X, D, LTd, wv - 1, q - 1, ln);
        }
      };
      blocked_potrf64_async(D, inv, LTd, &bad, fl, tid, colx, pipe);
      trsm_step(X, D, LTd, w, 3, lane);   // the last step: after diag16(3)
      __syncthreads();
    }
    const unsigned long long t1 = realtime();
    tot += t1 - t0;
    best = t1 - t0 < best ? t1 - t0 : best;
    __syncthreads();
  }
  if (tid == 0) { out[0] = tot; out[1] = best; }
  for (int e = tid; e < 4096; e += 256) res[e] = X[(e >> 6) * LQ + (e & 63)];
}
}  // namespace

int main() {
  std::vector<double> h(4096), x(4096);
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) {
      h[i * 64 + j] = (i == j) ? 130.0 : 1.0 / (1.0 + i + j);
      x[i * 64 + j] = 0.05 * std::sin(1.0 + i * 0.3 + j * 0.7);
    }
  double *A, *Xg, *res;
  unsigned long long *out;
  hipMalloc(&A, 4096 * 8);
  hipMalloc(&Xg, 4096 * 8);
  hipMalloc(&res, 4096 * 8);
  hipMalloc(&out, 16);
  hipMemcpy(A, h.data(), 4096 * 8, hipMemcpyHostToDevice);
  hipMemcpy(Xg, x.data(), 4096 * 8, hipMemcpyHostToDevice);
  const int reps = 200;
  std::vector<double> ref(4096), got(4096);
  for (int v = 0; v < 2; ++v) {
    hipLaunchKernelGGL(k_bench, dim3(1), dim3(256), 0, 0, A, Xg, reps, v, out, res);
    unsigned long long o[2];
    hipMemcpy(o, out, 16, hipMemcpyDeviceToHost);
    hipMemcpy(v == 0 ? ref.data() : got.data(), res, 4096 * 8, hipMemcpyDeviceToHost);
    double diff = 0;
    if (v == 1)
      for (int e = 0; e < 4096; ++e) diff = std::max(diff, std::fabs(got[e] - ref[e]));
    printf("%-12s mean %.2f us, best %.2f us  max|diff| %.1e\n", v == 0 ? "potrf+trsm" : "pipelined",
           o[0] / 100.0 / reps, o[1] / 100.0, diff);
  }
  return 0;
}
