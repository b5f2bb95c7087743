// Throughput of the dropout random-bit generators on one MI355X (diagnostic).
// Every thread runs ITERS dependent Philox calls; cycles per call per wave are
// derived from the wall time, the SIMD count and the measured shader clock.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

template <int R, bool X3>
__device__ __forceinline__ uint4 philox(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    if (X3) c = make_uint4(xor3(hi1, c.y, k0), lo1, xor3(hi0, c.w, k1), lo0);
    else c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

template <int R, bool X3>
__global__ __launch_bounds__(256) void k_philox(uint32_t* out, int iters, uint32_t k0, uint32_t k1) {
  uint4 c = make_uint4(blockIdx.x * 256 + threadIdx.x, 0, 7, 0);
  uint32_t acc = 0;
  for (int i = 0; i < iters; ++i) {
    const uint4 r = philox<R, X3>(c, k0, k1);
    acc += r.x ^ r.y ^ r.z ^ r.w;
    c.y = i + 1;
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__global__ __launch_bounds__(256) void k_clock(unsigned long long* o) {
  unsigned long long a, b, ra, rb;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(a)::"memory");
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ra)::"memory");
  uint32_t x = threadIdx.x;
  for (int i = 0; i < 2000000; ++i) x = x * 1664525u + 1013904223u;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(b)::"memory");
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(rb)::"memory");
  if (threadIdx.x == 0 && blockIdx.x == 0) { o[0] = b - a; o[1] = rb - ra; }
  if (x == 12345u) o[2] = x;
}

template <typename K>
static float run(K kern, uint32_t* out, int blocks, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, 0x1234u, 0x5678u);
  hipEventRecord(a);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, out, iters, 0x1234u, 0x5678u);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main() {
  int cus = 0; hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int blocks = cus * 8, iters = 2000;
  uint32_t* out; hipMalloc(&out, (size_t)blocks * 256 * 4);
  unsigned long long* clk; hipMalloc(&clk, 32);
  hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, 0, clk);
  unsigned long long h[2]; hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
  const double ghz = (double)h[0] / (double)h[1] * 0.1;
  const double waves = blocks * 4.0, simds = cus * 4.0;
  auto rep = [&](const char* n, float ms) {
    const double cyc = ms * 1e-3 * ghz * 1e9;          // wall cycles
    const double per = cyc * simds / (waves * iters);   // SIMD cycles per call per wave
    printf("{\"variant\": \"%s\", \"ms\": %.3f, \"simd_cycles_per_call_per_wave\": %.1f}\n", n, ms, per);
  };
  printf("{\"cus\": %d, \"idle_clock_ghz\": %.3f}\n", cus, ghz);
  rep("philox10", run(k_philox<10, false>, out, blocks, iters));
  rep("philox10_xor3", run(k_philox<10, true>, out, blocks, iters));
  rep("philox7", run(k_philox<7, false>, out, blocks, iters));
  rep("philox7_xor3", run(k_philox<7, true>, out, blocks, iters));
  rep("philox10", run(k_philox<10, false>, out, blocks, iters));
  return 0;
}
