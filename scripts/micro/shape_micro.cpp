// fp32 MFMA shape micro-benchmark: the GEMM main loop's LDS-fragment + MFMA body with the
// 32x32x2 and the 16x16x4 f32 MFMA at the same 64x64 wave tile, every CU busy (3 workgroups of
// 4 waves per CU), random operands; prints TF/s and the clock the chip held (s_memtime over
// s_memrealtime, 100 MHz).  Build: make -C scripts/micro shape_micro.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int NT = 256, DK = 16, ITERS = 4000;

// LDS images like the GEMM's RK tiles: [128 rows][16 k] for A and B (8 KB each)
template <int SHAPE, int BAR = 0>
__global__ __launch_bounds__(NT, 3) void body(const float* __restrict__ src, float* __restrict__ out,
                                              unsigned long long* __restrict__ clk, const float* __restrict__ stream) {
  // 48 KB as in the GEMM (3 workgroups / CU): three [A | B] stages; the static fragments of the
  // non-ring variants are stage 0 (values are irrelevant: random operands either way)
  __shared__ __attribute__((aligned(16))) float S[3][2 * 128 * DK];
  float* const A = &S[0][0];
  float* const B = &S[0][128 * DK];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  // BAR == 2: per 16-k tile, the GEMM's DMA traffic (16 KB per workgroup, 4 x 1 KB per wave) streamed
  // from a 256 MB buffer into LDS two tiles ahead, waited for like the GEMM's ring
  auto dma = [&](int it) {
    const size_t base = ((size_t)blockIdx.x * ITERS + it) * 4096 % (64u << 20);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ins = wave * 4 + u;
      __builtin_amdgcn_global_load_lds((const void*)(stream + base + ins * 256 + lane * 4),
                                       (__attribute__((address_space(3))) void*)(&S[it % 3][ins * 256]), 16, 0, 0);
    }
  };
  if (BAR == 2) dma(0);
  if (BAR == 3) {
    dma(0);
    dma(1);
  }
  for (int i = t; i < 128 * DK; i += NT) {
    A[i] = src[(blockIdx.x * 7 + i) & 65535];
    B[i] = src[(blockIdx.x * 13 + i + 777) & 65535];
  }
  __syncthreads();
  const int wm = wave >> 1, wn = wave & 1;
  unsigned long long t0 = 0, r0 = 0;
  if (t == 0) {
    t0 = __builtin_amdgcn_s_memtime();
    r0 = __builtin_amdgcn_s_memrealtime();
  }
  float res = 0.f;
  if constexpr (SHAPE == 32) {
    f32x16 acc[2][2] = {};
    const int h = lane >> 5, c = lane & 31;
    for (int it = 0; it < ITERS; ++it) {
      const float* Ab = A;
      const float* Bb = B;
      if (BAR == 3) {
        // tile it landed once only tile it+1's 4 DMA instructions are outstanding
        if (it + 1 < ITERS) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (it + 2 < ITERS) dma(it + 2);
        Ab = &S[it % 3][0];
        Bb = &S[it % 3][128 * DK];
      } else if (BAR == 2) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (it + 1 < ITERS) dma(it + 1);
      } else if (BAR) {
        __syncthreads();
      }
      asm volatile("" ::: "memory");   // the fragments are re-read every iteration, as in the GEMM
#pragma unroll
      for (int j = 0; j < DK / 8; ++j) {
        f32x4 af[2], bf[2];
#pragma unroll
        for (int a = 0; a < 2; ++a) af[a] = *reinterpret_cast<const f32x4*>(Ab + (wm * 64 + a * 32 + c) * DK + (2 * j + h) * 4);
#pragma unroll
        for (int b = 0; b < 2; ++b) bf[b] = *reinterpret_cast<const f32x4*>(Bb + (wn * 64 + b * 32 + c) * DK + (2 * j + h) * 4);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a][s], bf[b][s], acc[a][b], 0, 0, 0);
      }
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) res += acc[a][b][r];
  } else {
    f32x4 acc[4][4] = {};
    const int q = lane >> 4, i = lane & 15;
    for (int it = 0; it < ITERS; ++it) {
      if (BAR == 2) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (it + 1 < ITERS) dma(it + 1);
      } else if (BAR) {
        __syncthreads();
      }
      asm volatile("" ::: "memory");
      f32x4 af[4], bf[4];   // one 16-k chunk: lane group q holds k = 4q + s
#pragma unroll
      for (int a = 0; a < 4; ++a) af[a] = *reinterpret_cast<const f32x4*>(A + (wm * 64 + a * 16 + i) * DK + q * 4);
#pragma unroll
      for (int b = 0; b < 4; ++b) bf[b] = *reinterpret_cast<const f32x4*>(B + (wn * 64 + b * 16 + i) * DK + q * 4);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[a][s], bf[b][s], acc[a][b], 0, 0, 0);
    }
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int r = 0; r < 4; ++r) res += acc[a][b][r];
  }
  if (t == 0) {
    clk[2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - t0;
    clk[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime() - r0;
  }
  out[blockIdx.x * NT + t] = res;
}

template <int SHAPE, int BAR = 0>
static void run(int grid, const float* src, float* out, unsigned long long* clk, const float* stream) {
  for (int w = 0; w < 3; ++w) body<SHAPE, BAR><<<grid, NT>>>(src, out, clk, stream);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int reps = 20;
  (void)hipEventRecord(a);
  for (int r = 0; r < reps; ++r) body<SHAPE, BAR><<<grid, NT>>>(src, out, clk, stream);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  ms /= reps;
  std::vector<unsigned long long> h(2 * grid);
  (void)hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost);
  double ghz = 0.0;
  for (int i = 0; i < grid; ++i) ghz += (double)h[2 * i] / (double)h[2 * i + 1] * 0.1;
  ghz /= grid;
  const double flops = (double)grid * 4 * 64.0 * 64.0 * 2.0 * DK * ITERS;
  printf("%dx%d f32 MFMA%s: %8.3f ms  %7.1f TF/s  held clock %.2f GHz\n", SHAPE, SHAPE, BAR == 3 ? " + GEMM ring (3 stages, DMA 2 ahead, fragments from the ring)" : BAR == 2 ? " + barrier + 16 KB DMA per 16-k tile" : BAR ? " + barrier per 16-k tile" : "", ms, flops / (ms * 1e-3) / 1e12,
         ghz);
}

int main() {
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int grid = 3 * cus;
  std::vector<float> h(65536);
  unsigned x = 12345u;
  for (auto& v : h) {
    x = x * 1664525u + 1013904223u;
    v = (float)((x >> 8) & 0xFFFF) / 65536.f - 0.5f;
  }
  float *src = nullptr, *out = nullptr;
  unsigned long long* clk = nullptr;
  (void)hipMalloc(&src, h.size() * 4);
  (void)hipMalloc(&out, (size_t)grid * NT * 4);
  (void)hipMalloc(&clk, (size_t)grid * 16);
  (void)hipMemcpy(src, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  float* stream = nullptr;
  (void)hipMalloc(&stream, (size_t)(64u << 20) * 4 + 65536 * 4);
  (void)hipMemset(stream, 0, (size_t)(64u << 20) * 4 + 65536 * 4);
  for (int rep = 0; rep < 2; ++rep) {
    run<32>(grid, src, out, clk, stream);
    run<32, 1>(grid, src, out, clk, stream);
    run<32, 2>(grid, src, out, clk, stream);
    run<32, 3>(grid, src, out, clk, stream);
  }
  return 0;
}
