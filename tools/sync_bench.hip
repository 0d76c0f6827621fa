// Host round trip of one tiny kernel (debug micro-benchmark, alone on the chip): how long from
// enqueueing a kernel to the host seeing it done, by
//   event  hipEventRecord + a hipEventQuery spin (the LM loop's spin_sync)
//   sync   hipStreamSynchronize
//   flag   the kernel's last store (a sequence number in page-locked host memory, after a
//          system-scope release) seen by a host spin on that word
// usage: hipcc --offload-arch=gfx950 -O2 tools/sync_bench.hip -o tools/sync_bench && tools/sync_bench
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

__global__ void k_touch(double *dev, volatile double *host, double seq) {
  if (threadIdx.x == 0) {
    dev[0] += 1.0;
    if (host) {
      host[1] = seq * 2.0;   // a payload the host reads after the flag
      __threadfence_system();
      host[0] = seq;
    }
  }
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  double *dev;
  CK(hipMalloc(&dev, 64));
  CK(hipMemset(dev, 0, 64));
  double *host;
  CK(hipHostMalloc(&host, 64, hipHostMallocDefault));
  host[0] = host[1] = 0.0;
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const int N = 4000;
  for (int rep = 0; rep < 3; ++rep) {
    double t0 = now();
    for (int i = 0; i < N; ++i) {
      k_touch<<<1, 64, 0, s>>>(dev, nullptr, 0.0);
      CK(hipEventRecord(ev, s));
      hipError_t e;
      while ((e = hipEventQuery(ev)) == hipErrorNotReady) {
      }
      CK(e);
    }
    const double t_event = (now() - t0) / N;
    t0 = now();
    for (int i = 0; i < N; ++i) {
      k_touch<<<1, 64, 0, s>>>(dev, nullptr, 0.0);
      CK(hipStreamSynchronize(s));
    }
    const double t_sync = (now() - t0) / N;
    t0 = now();
    int bad = 0;
    for (int i = 0; i < N; ++i) {
      const double seq = 1.0 + rep * N + i;
      k_touch<<<1, 64, 0, s>>>(dev, host, seq);
      while (*(volatile double *)&host[0] != seq) {
      }
      if (*(volatile double *)&host[1] != 2.0 * seq) ++bad;
    }
    const double t_flag = (now() - t0) / N;
    CK(hipStreamSynchronize(s));
    std::printf("round trip per kernel: event %.2f us  sync %.2f us  flag %.2f us (payload late %d)\n",
                1e6 * t_event, 1e6 * t_sync, 1e6 * t_flag, bad);
  }
  return 0;
}
