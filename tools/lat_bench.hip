// Diagnostic micro-benchmark: dependent-chain latency (cycles, s_memtime) of
// the fp64 VALU / DPP / LDS operations the diagonal-block elimination of
// dense_llt.hip is built from, one wave alone on the chip.
// Build: hipcc --offload-arch=gfx950 -O3 tools/lat_bench.hip -o tools/lat_bench
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

#define N 64

__device__ __forceinline__ unsigned long long clk() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

__global__ void k_lat(double seed, unsigned long long *out, double *sink) {
  __shared__ double lds[128];
  const int lane = threadIdx.x;
  double x = seed + lane * 1e-3, y = 1.0 + lane * 1e-4;
  unsigned long long t0, t1;
  int slot = 0;
#define TIME(BODY)                                                           \
  do {                                                                       \
    t0 = clk();                                                              \
    _Pragma("unroll") for (int r = 0; r < N; ++r) { BODY; }                  \
    t1 = clk();                                                              \
    if (lane == 0) out[slot] = t1 - t0;                                       \
    ++slot;                                                                  \
  } while (0)
  // 0: dependent v_fma_f64
  TIME(asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(x) : "v"(y)));
  // 1: independent v_fma_f64 (4 chains interleaved, count per instruction)
  {
    double a = x, b = x + 1, c = x + 2, d = x + 3;
    TIME(asm volatile("v_fma_f64 %0, %0, %4, %4\n\tv_fma_f64 %1, %1, %4, %4\n\tv_fma_f64 %2, %2, %4, %4\n\tv_fma_f64 %3, %3, %4, %4"
                      : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(y)));
    x += a + b + c + d;
  }
  // 2: dependent v_rcp_f64
  TIME(asm volatile("v_rcp_f64 %0, %0" : "+v"(x)));
  // 3: dependent v_mov_b64_dpp row_newbcast:3
  TIME(asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %0 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(x)));
  // 4: dependent fma + dpp pair
  TIME(asm volatile("v_fma_f64 %0, %0, %1, %1\n\ts_nop 1\n\tv_mov_b64_dpp %0, %0 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(x) : "v"(y)));
  // 5: LDS write -> read round trip (dependent)
  TIME({
    lds[lane] = x;
    x = lds[(lane + 1) & 63] + 1.0;
  });
  // 6: dependent v_mul_f64
  TIME(asm volatile("v_mul_f64 %0, %0, %1" : "+v"(x) : "v"(y)));
  // 7: dependent v_fma_f32 (reference point)
  {
    float f = (float)x;
    TIME(asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f) : "v"((float)y)));
    x += f;
  }
  // 8: v_readlane x2 -> s -> v_mov (dependent through SGPR)
  {
    unsigned u = (unsigned)lane;
    TIME(asm volatile("v_readlane_b32 s2, %0, 3\n\ts_nop 3\n\tv_add_u32 %0, s2, %0" : "+v"(u)::"s2"));
    x += u;
  }
  // 9: permlane16_swap + permlane32_swap pair (dependent)
  {
    unsigned u = (unsigned)lane, v = u + 7;
    TIME(asm volatile("v_permlane16_swap_b32 %0, %1\n\ts_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(u), "+v"(v)));
    x += u + v;
  }
  sink[lane] = x;
  // v_rcp_f64 accuracy: max |a rcp(a) - 1| over 64 lanes x 256 values
  double emax = 0.0;
  for (int r = 0; r < 256; ++r) {
    const double a = 1e-3 + (double)((lane * 7919 + r * 104729) % 1000003) * 1.3e-3;
    const double e = __builtin_fma(-a, __builtin_amdgcn_rcp(a), 1.0);
    emax = fmax(emax, fabs(e));
  }
  for (int o = 32; o; o >>= 1) emax = fmax(emax, __shfl_xor(emax, o));
  if (lane == 0) sink[64] = emax;
}

int main() {
  unsigned long long *out;
  double *sink;
  hipMalloc(&out, 64 * 8);
  hipMalloc(&sink, 65 * 8);
  for (int rep = 0; rep < 2; ++rep) hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, 1.0001, out, sink);
  unsigned long long h[16];
  hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
  const char *names[] = {"dep v_fma_f64", "indep v_fma_f64 (per instr)", "dep v_rcp_f64", "dep dpp b64 (+s_nop 1)",
                         "dep fma+dpp pair", "lds write->read trip", "dep v_mul_f64", "dep v_fma_f32",
                         "readlane->salu->valu", "permlane16+32 swap pair"};
  for (int s = 0; s < 10; ++s) {
    const double per = (double)h[s] / N / (s == 1 ? 4 : 1);
    printf("%-30s %7.1f cycles\n", names[s], per);
  }
  double em;
  hipMemcpy(&em, sink + 64, 8, hipMemcpyDeviceToHost);
  printf("v_rcp_f64 max |a r - 1| = %.3e (2^%.1f)\n", em, std::log2(em));
  return 0;
}
