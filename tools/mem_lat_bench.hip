// Diagnostic micro-benchmark: the memory round trips the persistent executor's
// hand-offs are made of, on MI355X.
//  1. dependent-chain load latency, one lane alone: agent-scope relaxed atomic
//     loads (what ld_wt emits: sc1, L2-bypassing across XCDs), plain loads
//     (L1/L2 hits after the first pass) and never-matching CAS (ld_acquire_relaxed);
//  2. ping-pong between two workgroups through agent-scope atomics, for a
//     partner on the same XCD and on another one (HW_REG_XCC_ID reported).
// Build: hipcc --offload-arch=gfx950 -O3 tools/mem_lat_bench.hip -o tools/mem_lat_bench
#include <hip/hip_runtime.h>
#include <climits>
#include <cstdio>
#include <vector>

__device__ __forceinline__ unsigned long long rt() {
  unsigned long long t;
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;   // 100 MHz
}

__global__ void k_chase(const long *next, int n, int mode, unsigned long long *out, long *sink) {
  if (threadIdx.x != 0) return;
  long p = 0;
  for (int i = 0; i < 64; ++i) p = next[p];   // warm
  const unsigned long long t0 = rt();
  for (int i = 0; i < n; ++i) {
    if (mode == 0) {
      p = __hip_atomic_load(next + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (mode == 1) {
      p = *(volatile const long *)(next + p);
    } else {
      long v = LONG_MIN;
      __hip_atomic_compare_exchange_strong(const_cast<long *>(next) + p, &v, LONG_MIN, __ATOMIC_RELAXED,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      p = v;
    }
  }
  out[0] = rt() - t0;
  sink[0] = p;
}

__global__ void k_pingpong(int *flags, int partner, int n, unsigned long long *out, int *xcc) {
  if (threadIdx.x != 0) return;
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  xcc[blockIdx.x] = (int)(x & 7);
  if (blockIdx.x != 0 && (int)blockIdx.x != partner) return;
  int *a = flags, *b = flags + 64;
  const bool first = blockIdx.x == 0;
  const unsigned long long t0 = rt();
  for (int i = 1; i <= n; ++i) {
    if (first) {
      __hip_atomic_store(a, i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      while (__hip_atomic_load(b, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < i) {}
    } else {
      while (__hip_atomic_load(a, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < i) {}
      __hip_atomic_store(b, i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (first) out[0] = rt() - t0;
}

int main() {
  const int nel = 1 << 14;   // 128 KB working set
  std::vector<long> h(nel);
  // a single random cycle over cache-line-spaced slots
  std::vector<int> perm(nel / 16);
  for (int i = 0; i < (int)perm.size(); ++i) perm[i] = i;
  unsigned s = 12345;
  for (int i = (int)perm.size() - 1; i > 0; --i) {
    s = s * 1103515245u + 12345u;
    std::swap(perm[i], perm[s % (i + 1)]);
  }
  for (int i = 0; i < (int)perm.size(); ++i) h[16 * perm[i]] = 16L * perm[(i + 1) % perm.size()];
  long *d, *sink;
  unsigned long long *out;
  int *flags, *xcc;
  hipMalloc(&d, nel * sizeof(long));
  hipMalloc(&sink, 64);
  hipMalloc(&out, 64);
  hipMalloc(&flags, 1024);
  hipMalloc(&xcc, 64 * sizeof(int));
  hipMemcpy(d, h.data(), nel * sizeof(long), hipMemcpyHostToDevice);
  const char *names[3] = {"agent-scope atomic load (sc1)", "plain volatile load", "never-matching CAS"};
  const int n = 2000;
  for (int m = 0; m < 3; ++m) {
    k_chase<<<1, 64>>>(d, n, m, out, sink);
    unsigned long long t;
    hipMemcpy(&t, out, 8, hipMemcpyDeviceToHost);
    std::printf("chase %-32s %7.1f ns per dependent load\n", names[m], t * 10.0 / n);
  }
  for (int partner : {1, 2, 8, 16, 9, 63}) {
    hipMemset(flags, 0, 1024);
    k_pingpong<<<64, 64>>>(flags, partner, n, out, xcc);
    unsigned long long t;
    int hx[64];
    hipMemcpy(&t, out, 8, hipMemcpyDeviceToHost);
    hipMemcpy(hx, xcc, sizeof(hx), hipMemcpyDeviceToHost);
    std::printf("ping-pong block 0 (XCC %d) <-> block %d (XCC %d): %7.1f ns per round trip\n", hx[0], partner,
                hx[partner], t * 10.0 / n);
  }
  return 0;
}
