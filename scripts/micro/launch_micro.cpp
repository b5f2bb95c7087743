// Fixed costs of small launches (the launch-lean L = 1 step's kernels take 8-19 us for a few us of
// work): back-to-back launches of 96 x 256-thread workgroups, hipEvents over 200 launches, eager
// and replayed from a hipGraph.  K0 empty; K1 + a 1.3 KB argument struct read through dependent
// scalar loads; K2 + 48 float4 weight loads per lane (192 KB per workgroup, L2-resident);
// K3 + 192 v_mfma_f32_16x16x4_f32 per wave on them; K4 = K3 + 2 syncthreads-separated LDS phases.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/micro/launch_micro.cpp -o scripts/micro/launch_micro
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
struct Big { const float* p[160]; int idx[8]; float* out; };

__global__ __launch_bounds__(256) void k0(float* out) {
  if (threadIdx.x == 0 && blockIdx.x == 1000000) out[0] = 1.f;
}
__global__ __launch_bounds__(256) void k1(const Big a) {
  const int i = a.idx[blockIdx.x & 7];
  const float* p = a.p[i];
  if (threadIdx.x == 0 && p == nullptr) a.out[0] = 1.f;
}
template <int MODE>
__global__ __launch_bounds__(256) void kw(const Big a) {
  __shared__ float lds[16 * 132];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const float* W = a.p[a.idx[blockIdx.x & 7]];
  float4 w[48];
#pragma unroll
  for (int i = 0; i < 48; ++i) w[i] = *reinterpret_cast<const float4*>(W + ((i * 256 + t) * 4) % (48 * 1024));
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (MODE >= 1) {
    float4 x = make_float4(t, t, t, t);
    if (MODE >= 2) {
      lds[t] = (float)t;
      __syncthreads();
      x.x = lds[(t + 1) & 255];
    }
#pragma unroll
    for (int i = 0; i < 48; ++i) {
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.x, w[i].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.y, w[i].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.z, w[i].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x.w, w[i].w, acc, 0, 0, 0);
    }
    if (MODE >= 2) {
      __syncthreads();
      lds[t] = acc[0];
      __syncthreads();
      acc[1] += lds[(t + 3) & 255];
    }
  } else {
#pragma unroll
    for (int i = 0; i < 48; ++i) acc[0] += w[i].x + w[i].y + w[i].z + w[i].w;
  }
  a.out[(blockIdx.x * 256 + t) * 4 % 65536] = acc[0] + acc[1] + acc[2] + acc[3];
}

template <typename F>
float timeit(F launch, hipStream_t st, bool graph) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int n = 200;
  if (graph) {
    hipGraph_t g; hipGraphExec_t ge;
    hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
    for (int i = 0; i < 20; ++i) launch();
    hipStreamEndCapture(st, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphLaunch(ge, st);
    hipStreamSynchronize(st);
    hipEventRecord(e0, st);
    for (int i = 0; i < n / 20; ++i) hipGraphLaunch(ge, st);
    hipEventRecord(e1, st);
  } else {
    for (int i = 0; i < 10; ++i) launch();
    hipStreamSynchronize(st);
    hipEventRecord(e0, st);
    for (int i = 0; i < n; ++i) launch();
    hipEventRecord(e1, st);
  }
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.f / n;
}

int main() {
  hipStream_t st;
  hipStreamCreate(&st);
  float *w, *out;
  hipMalloc(&w, 48 * 1024 * 4 * 8);
  hipMalloc(&out, 65536 * 4);
  hipMemset(w, 0, 48 * 1024 * 4 * 8);
  Big a;
  for (int i = 0; i < 160; ++i) a.p[i] = w + (i % 8) * 48 * 1024;
  for (int i = 0; i < 8; ++i) a.idx[i] = i;
  a.out = out;
  for (int grid : {96, 256, 1024}) {
    for (int graph = 0; graph < 2; ++graph) {
      const float t0 = timeit([&] { hipLaunchKernelGGL(k0, dim3(grid), dim3(256), 0, st, out); }, st, graph);
      const float t1 = timeit([&] { hipLaunchKernelGGL(k1, dim3(grid), dim3(256), 0, st, a); }, st, graph);
      const float t2 = timeit([&] { hipLaunchKernelGGL(kw<0>, dim3(grid), dim3(256), 0, st, a); }, st, graph);
      const float t3 = timeit([&] { hipLaunchKernelGGL(kw<1>, dim3(grid), dim3(256), 0, st, a); }, st, graph);
      const float t4 = timeit([&] { hipLaunchKernelGGL(kw<2>, dim3(grid), dim3(256), 0, st, a); }, st, graph);
      printf("grid %4d %s: empty %.2f  bigargs %.2f  +loads %.2f  +mfma %.2f  +lds/sync %.2f us per launch\n", grid,
             graph ? "graph" : "eager", t0, t1, t2, t3, t4);
    }
  }
  return 0;
}
