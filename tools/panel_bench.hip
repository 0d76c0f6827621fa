// Diagnostic micro-benchmark of the reduced-system panel kernel: one column
// with a diagonal tile and one tile below, timed with HIP events and with
// in-kernel s_memtime stamps (STAMP ids in dense_llt.hip).  Stamp shares only;
// the stamped build's absolute time is not the real kernel's.
#define ARSLAM_STAMPS 1
#include "../ar_slam_amd/csrc/dense_llt.hip"

#include <cstdio>
#include <vector>

using namespace arslam;

int main() {
  const int T = 2;
  const long N = T * 64;
  std::vector<double> h(N * N, 0.0);
  for (long i = 0; i < N; ++i)
    for (long j = 0; j <= i; ++j) h[i * N + j] = (i == j) ? N + 1.0 : 1.0 / (1.0 + i + j);
  double *S, *Ld;
  int *flag;
  int2 *tasks;
  hipMalloc(&S, N * N * 8);
  hipMalloc(&Ld, T * 64 * 64 * 8);
  hipMalloc(&flag, 4);
  hipMalloc(&tasks, 2 * sizeof(int2));
  int2 ht[2] = {make_int2(1, 0), make_int2(0, 0)};   // block 0 = the (1,0) solve task
  hipMemcpy(tasks, ht, sizeof(ht), hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e9;
  for (int rep = 0; rep < 20; ++rep) {
    hipMemcpy(S, h.data(), N * N * 8, hipMemcpyHostToDevice);
    hipMemset(flag, 0, 4);
    hipEventRecord(a, 0);
    hipLaunchKernelGGL(k_panel, dim3(2), dim3(256), 0, 0, S, N, Ld, tasks, flag);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  unsigned long long st[64];
  hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamps), sizeof(st));
  int fl;
  hipMemcpy(&fl, flag, 4, hipMemcpyDeviceToHost);
  printf("k_panel best %.2f us (flag %d)\n", best * 1e3, fl);
  const char *names[64] = {};
  names[1] = "load";
  for (int p = 0; p < 4; ++p) {
    static char buf[4][3][32];
    snprintf(buf[p][0], 32, "p%d diag factor", p);
    snprintf(buf[p][1], 32, "p%d rows below", p);
    snprintf(buf[p][2], 32, "p%d trailing mfma", p);
    names[11 + 4 * p] = buf[p][0];
    names[12 + 4 * p] = buf[p][1];
    names[13 + 4 * p] = buf[p][2];
  }
  names[2] = "potrf tail";
  names[3] = "trsm";
  names[4] = "store";
  const int order[] = {0, 1, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 2, 3, 4};
  for (size_t q = 1; q < sizeof(order) / sizeof(int); ++q) {
    const int id = order[q], prev = order[q - 1];
    if (st[id] && st[prev]) printf("  %-20s %8llu ticks\n", names[id] ? names[id] : "-", st[id] - st[prev]);
  }
  return 0;
}
