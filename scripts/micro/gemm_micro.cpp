// GEMM micro-benchmark at the C2 launch shapes (kernel-only timing, hipEvents).
// Build: make -C scripts/micro   Run (box): scripts/micro/gemm_micro
#include <cstdio>
#include <vector>

#include "capi_util.h"

using namespace mmf;


static float* dev(size_t n, float v = 0.01f) {
  float* p = nullptr;
  (void)hipMalloc(&p, n * 4);
  std::vector<float> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = v * (float)((i * 2654435761u) % 1000) / 1000.f;
  (void)hipMemcpy(p, h.data(), n * 4, hipMemcpyHostToDevice);
  return p;
}

static void run(const char* name, std::vector<GemmJob>& jobs, int am, int bm, double flops) {
  hipStream_t st;
  (void)hipStreamCreate(&st);
  for (int i = 0; i < 3; ++i) launch_gemm(jobs.data(), (int)jobs.size(), am, bm, 0.f, nullptr, st);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int reps = 20;
  (void)hipEventRecord(a, st);
  for (int i = 0; i < reps; ++i) launch_gemm(jobs.data(), (int)jobs.size(), am, bm, 0.f, nullptr, st);
  (void)hipEventRecord(b, st);
  (void)hipEventSynchronize(b);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, a, b);
  ms /= reps;
  printf("%-10s %8.1f us  %7.1f TF/s\n", name, ms * 1e3, flops / (ms * 1e-3) / 1e12);
}

int main() {
  const int R = 32768, H = 128;
  // fwd.qkv: 12 x (R x H) = P (R x H) W^T (+bias)
  {
    std::vector<GemmJob> jobs;
    float* P = dev((size_t)3 * R * H);
    float* W = dev((size_t)12 * H * H);
    float* bias = dev((size_t)12 * H);
    float* out = dev((size_t)12 * R * H);
    for (int g = 0; g < 12; ++g) {
      GemmJob j = make_job(R, H, out + (size_t)g * R * H, H, EPI_BIAS);
      j.g.bias = bias + g * H;
      add_src(j, opnd(P + (size_t)(g % 3) * R * H, H), opnd(W + (size_t)g * H * H, H), H);
      jobs.push_back(j);
    }
    run("qkv", jobs, MODE_RK, MODE_RK, 12.0 * 2 * R * H * H);
    std::vector<GemmJob> proj(jobs.begin(), jobs.begin() + 3);
    run("proj", proj, MODE_RK, MODE_RK, 3.0 * 2 * R * H * H);
  }
  // bwd.dZ: 3 x (R x H) = sum of 4 sources dQ/dK (R x H) . W (H x H) (KR)
  {
    std::vector<GemmJob> jobs;
    float* dq = dev((size_t)12 * R * H);
    float* W = dev((size_t)12 * H * H);
    float* out = dev((size_t)3 * R * H);
    for (int m = 0; m < 3; ++m) {
      GemmJob j = make_job(R, H, out + (size_t)m * R * H, H, 0);
      for (int s = 0; s < 4; ++s)
        add_src(j, opnd(dq + (size_t)(m * 4 + s) * R * H, H), opnd(W + (size_t)(m * 4 + s) * H * H, H), H);
      jobs.push_back(j);
    }
    run("dZ", jobs, MODE_RK, MODE_KR, 3.0 * 4 * 2 * R * H * H);
    // the same FLOPs as ONE source of K = 4H per output (source-switch cost)
    std::vector<GemmJob> one;
    float* a1 = dev((size_t)3 * R * 4 * H);
    float* w1 = dev((size_t)3 * 4 * H * H);
    for (int m = 0; m < 3; ++m) {
      GemmJob j = make_job(R, H, out + (size_t)m * R * H, H, 0);
      add_src(j, opnd(a1 + (size_t)m * R * 4 * H, 4 * H), opnd(w1 + (size_t)m * 4 * H * H, H), 4 * H);
      one.push_back(j);
    }
    run("dZ_1src", one, MODE_RK, MODE_KR, 3.0 * 4 * 2 * R * H * H);
    // marginal cost of the main loop: the same launch at K = 2H and K = 8H (fixed prologue /
    // epilogue, k-loop length x1/4 and x2)
    for (int K : {16, 32, 64, 128, 256, 1024}) {
      std::vector<GemmJob> kv;
      float* ak = dev((size_t)3 * R * K);
      float* wk = dev((size_t)3 * K * H);
      for (int m = 0; m < 3; ++m) {
        GemmJob j = make_job(R, H, out + (size_t)m * R * H, H, 0);
        add_src(j, opnd(ak + (size_t)m * R * K, K), opnd(wk + (size_t)m * K * H, H), K);
        kv.push_back(j);
      }
      char name[32];
      snprintf(name, sizeof(name), "dZ_K%d", K);
      run(name, kv, MODE_RK, MODE_KR, 3.0 * 2 * R * H * K);
      (void)hipFree(ak);
      (void)hipFree(wk);
    }
    // probe: the same FLOPs with every row tile reading the SAME 128 A rows (L2-resident):
    // if this is much faster, the real launch is bound by streaming A from HBM
    {
      std::vector<GemmJob> l2 = one;
      for (auto& j : l2) j.src[0].a.row_div = 128;   // row r -> stored row r / 128: 256 distinct rows
      run("dZ_Al2", l2, MODE_RK, MODE_KR, 3.0 * 4 * 2 * R * H * H);
      std::vector<GemmJob> l2b = one;
      for (auto& j : l2b) j.src[0].a.row_div = 32768;
      run("dZ_Al2one", l2b, MODE_RK, MODE_KR, 3.0 * 4 * 2 * R * H * H);
    }
    // RK B operand (W^T stored [j][kk]) instead of KR
    run("dZ_1srcRK", one, MODE_RK, MODE_RK, 3.0 * 4 * 2 * R * H * H);
    // the real epilogue: ReLU gate from P_m (EPI_GATE) + row-broadcast c_m / L (EPI_ROWADD)
    float* gate = dev((size_t)3 * R * H);
    float* cvec = dev((size_t)256 * 3 * H);
    std::vector<GemmJob> g = jobs;
    for (int m = 0; m < 3; ++m) {
      g[m].g.epi = EPI_GATE | EPI_ROWADD;
      g[m].g.gate = gate + (size_t)m * R * H; g[m].g.ld_gate = H; g[m].g.gate_scale = 1.f;
      g[m].g.rowadd = cvec + (size_t)m * H; g[m].g.ld_rowadd = 3 * H; g[m].g.rowadd_div = 128;
      g[m].g.rowadd_scale = 1.f / 128.f;
    }
    run("dZ_gate", g, MODE_RK, MODE_KR, 3.0 * 4 * 2 * R * H * H);
    // + E_m: 2 per-sample K = heads sources (pbar^T rows against dU_b, segment offsets)
    float* pbT = dev((size_t)2 * R * 4);
    float* du = dev((size_t)2 * 256 * 4 * H);
    std::vector<GemmJob> ge = g;
    for (int m = 0; m < 3; ++m) {
      ge[m].g.seg_rows = 128;
      for (int e = 0; e < 2; ++e) {
        Operand d = opnd(du + (size_t)e * 256 * 4 * H, H);
        d.seg_stride = 4 * H;
        add_src(ge[m], opnd(pbT + (size_t)e * R * 4, 4), d, 4);
      }
    }
    run("dZ_gate_em", ge, MODE_RK, MODE_KR, 3.0 * 4 * 2 * R * H * H);
  }
  // bwd.wgrad: 15 x (H x H) = dY^T X over R rows, split-K slabs
  {
    WgradPlan wp;
    size_t need = 0;
    {
      Bump bp(nullptr);
      WgradPlan tmp;
      for (int g = 0; g < 15; ++g) plan_wgrad(tmp, bp, H, H, R, opnd(nullptr, H), opnd(nullptr, H), nullptr, nullptr);
      need = bp.off + 256;
    }
    float* ws = dev(need / 4 + 64, 0.f);
    Bump bp(ws);
    float* dy = dev((size_t)15 * R * H);
    float* x = dev((size_t)3 * R * H);
    float* gw = dev((size_t)15 * H * H);
    float* gb = dev((size_t)15 * H);
    for (int g = 0; g < 15; ++g)
      plan_wgrad(wp, bp, H, H, R, opnd(dy + (size_t)g * R * H, H), opnd(x + (size_t)(g % 3) * R * H, H),
                 gw + (size_t)g * H * H, gb + g * H);
    run("wgrad", wp.jobs, MODE_KR, MODE_KR, 15.0 * 2 * R * H * H);
  }
  return 0;
}
