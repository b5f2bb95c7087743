// Attention with head_dim > 64 (the reference's heads ablation at hidden_dim 256:
// num_heads 1 / 2 -> head_dim 256 / 128, .github/workflows/parallel_run.yml:79-97,
// config/base.yaml:28-30).  The fused attention kernels keep a head's query /
// key fragments in registers, which caps them at head_dim 64; beyond that the
// scores are materialised: S = scale Q K^T and the contractions with V / dO / dS
// are grouped strided-batch MFMA GEMMs (gemm.hip, one group per (pair, head),
// batch = sample), and the row work between them runs here, one wave per row:
//   wide_softmax : P = softmax(S) over the unmasked keys (-inf -> NaN -> 0 for a
//                  fully masked row, src/attention.py:120-129) in place, plus the
//                  post-dropout P' (general plan) and the attention maps;
//   wide_colmean : pbar = mean_q P' and its (B, Lk, heads) transpose (pooled plan);
//   wide_dsoftmax: dS = P (dP - rowsum(P dP)) with dP = keep dP' / (1 - p), dP' = dO V^T
//                  (general) or dpbar / Lq (pooled: every query row of dP' is that).
// Dropout keep decisions are element ((b heads + h) Lq + i) Lk + j of the pair's
// probability tensor: the Philox stream of every other attention kernel.
#include <algorithm>
#include <cstring>

#include "capi_util.h"
#include "mmf_device.h"

namespace mmf {
namespace {

constexpr int WNT = 256;   // 4 waves = 4 rows per workgroup

struct WideRowArgs {
  WidePair p[WIDE_MAX_PAIRS];
  int32_t npairs, B, heads;
  float drop_p;
  const RngSnap* rng;
  int32_t pooled;
};

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ bool key_live(const WidePair& P, int b, int j) {
  if (P.kmask_mode == 1) return P.kmask[(int64_t)b * P.kmask_ld] != 0.f;
  if (P.kmask_mode == 2) return P.kmask[(int64_t)b * P.kmask_ld + j] != 0.f;
  return true;
}

// one wave per (b, h, i) row of pair blockIdx.y
__global__ __launch_bounds__(WNT) void wide_softmax_kernel(const WideRowArgs A) {
  const WidePair& P = A.p[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (WNT / 64) + (threadIdx.x >> 6);
  const int64_t nrows = (int64_t)A.B * A.heads * P.Lq;
  if (row >= nrows) return;
  const int b = (int)(row / ((int64_t)A.heads * P.Lq));
  const int Lk = P.Lk;
  float* s = P.P + row * Lk;
  RngSnap rs{0, 0};
  if (A.drop_p > 0.f && A.rng) rs = *A.rng;
  const float inv_keep = A.drop_p < 1.f ? 1.f / (1.f - A.drop_p) : 0.f;
  float mx = -INFINITY;
  for (int j = lane; j < Lk; j += 64)
    if (key_live(P, b, j)) mx = fmaxf(mx, s[j]);
  mx = wave_max(mx);
  float sum = 0.f;
  for (int j = lane; j < Lk; j += 64)
    if (key_live(P, b, j)) sum += __expf(s[j] - mx);
  sum = wave_sum(sum);
  // no live key: softmax of all -inf is NaN, nan_to_num -> 0 (src/attention.py:127-129)
  const float inv = mx == -INFINITY ? 0.f : 1.f / sum;
  for (int j = lane; j < Lk; j += 64) {
    const float pr = (mx != -INFINITY && key_live(P, b, j)) ? __expf(s[j] - mx) * inv : 0.f;
    s[j] = pr;
    float pd = pr;
    if (A.drop_p > 0.f) pd = keep1(rs, P.drop_site, (uint64_t)row * Lk + j, A.drop_p) ? pr * inv_keep : 0.f;
    if (P.Pd) P.Pd[row * Lk + j] = pd;
    if (P.probs) P.probs[row * Lk + j] = pd;
  }
}

// one thread per (b, h, j) of pair blockIdx.y: pbar = mean over queries of P'
__global__ __launch_bounds__(WNT) void wide_colmean_kernel(const WideRowArgs A) {
  const WidePair& P = A.p[blockIdx.y];
  const int64_t e = (int64_t)blockIdx.x * WNT + threadIdx.x;
  const int Lq = P.Lq, Lk = P.Lk;
  if (e >= (int64_t)A.B * A.heads * Lk) return;
  const int j = (int)(e % Lk);
  const int64_t bh = e / Lk;
  const int h = (int)(bh % A.heads), b = (int)(bh / A.heads);
  RngSnap rs{0, 0};
  if (A.drop_p > 0.f && A.rng) rs = *A.rng;
  const float inv_keep = A.drop_p < 1.f ? 1.f / (1.f - A.drop_p) : 0.f;
  float acc = 0.f;
  for (int i = 0; i < Lq; ++i) {
    const int64_t row = bh * Lq + i;
    float pr = P.P[row * Lk + j];
    if (A.drop_p > 0.f) pr = keep1(rs, P.drop_site, (uint64_t)row * Lk + j, A.drop_p) ? pr * inv_keep : 0.f;
    acc += pr;
  }
  const float v = acc * (1.f / (float)Lq);
  P.pbar[e] = v;
  if (P.pbarT) P.pbarT[((int64_t)b * Lk + j) * A.heads + h] = v;
}

// one wave per row: dS = P (dP - D), D = sum_j P dP
__global__ __launch_bounds__(WNT) void wide_dsoftmax_kernel(const WideRowArgs A) {
  const WidePair& P = A.p[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (WNT / 64) + (threadIdx.x >> 6);
  const int Lq = P.Lq, Lk = P.Lk;
  if (row >= (int64_t)A.B * A.heads * Lq) return;
  const int64_t bh = row / Lq;
  RngSnap rs{0, 0};
  if (A.drop_p > 0.f && A.rng) rs = *A.rng;
  const float inv_keep = A.drop_p < 1.f ? 1.f / (1.f - A.drop_p) : 0.f;
  const float* pr = P.P + row * Lk;
  const float inv_lq = 1.f / (float)Lq;
  auto dp_of = [&](int j) {
    float g = A.pooled ? P.dpbar[bh * Lk + j] * inv_lq : P.dPd[row * Lk + j];
    if (A.drop_p > 0.f) g = keep1(rs, P.drop_site, (uint64_t)row * Lk + j, A.drop_p) ? g * inv_keep : 0.f;
    return g;
  };
  float D = 0.f;
  for (int j = lane; j < Lk; j += 64) D += pr[j] * dp_of(j);
  D = wave_sum(D);
  for (int j = lane; j < Lk; j += 64) P.dS[row * Lk + j] = pr[j] * (dp_of(j) - D);
}

WideRowArgs row_args(const WidePair* pairs, int n, int B, int heads, float drop_p, const RngSnap* rng, bool pooled) {
  WideRowArgs a;
  memset(&a, 0, sizeof(a));
  for (int g = 0; g < n; ++g) a.p[g] = pairs[g];
  a.npairs = n; a.B = B; a.heads = heads; a.drop_p = drop_p; a.rng = rng; a.pooled = pooled;
  return a;
}

enum class RowKind { Softmax, Colmean, Dsoftmax };

hipError_t launch_rows(RowKind kind, const WidePair* pairs, int npairs, int B, int heads, float drop_p,
                       const RngSnap* rng, bool pooled, hipStream_t st) {
  for (int g0 = 0; g0 < npairs; g0 += WIDE_MAX_PAIRS) {
    const int n = std::min(WIDE_MAX_PAIRS, npairs - g0);
    const WideRowArgs a = row_args(pairs + g0, n, B, heads, drop_p, rng, pooled);
    int64_t maxw = 1;
    double by = 0.0;
    for (int g = 0; g < n; ++g) {
      const WidePair& P = pairs[g0 + g];
      const double elems = (double)B * heads * P.Lq * P.Lk;
      const int64_t w = kind == RowKind::Colmean ? (int64_t)B * heads * P.Lk : (int64_t)B * heads * P.Lq;
      maxw = std::max(maxw, w);
      by += kind == RowKind::Softmax ? 4.0 * elems * (2 + (P.Pd ? 1 : 0) + (P.probs ? 1 : 0))
          : kind == RowKind::Colmean ? 4.0 * (elems + 2.0 * B * heads * P.Lk)
                                     : 4.0 * elems * (pooled ? 2 : 3);
    }
    const int per = kind == RowKind::Colmean ? WNT : WNT / 64;
    const dim3 grid((unsigned)((maxw + per - 1) / per), n);
    if (kind == RowKind::Softmax) {
      ProfLaunch prof_(st, "wide_softmax_kernel", 0.0, by);
      mmf_launch(wide_softmax_kernel, grid, dim3(WNT), 0, st, a);
    } else if (kind == RowKind::Colmean) {
      ProfLaunch prof_(st, "wide_colmean_kernel", 0.0, by);
      mmf_launch(wide_colmean_kernel, grid, dim3(WNT), 0, st, a);
    } else {
      ProfLaunch prof_(st, "wide_dsoftmax_kernel", 0.0, by);
      mmf_launch(wide_dsoftmax_kernel, grid, dim3(WNT), 0, st, a);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// C (per pair and head, batched over samples) = alpha * A B: one group per (pair, head)
struct HeadGemm {
  int M, N, K;
  const float* a; int lda; int64_t bsa;   // per-sample stride
  const float* b; int ldb; int64_t bsb;
  float* c; int ldc; int64_t bsc;
  int64_t ha, hb, hc;                     // per-head offsets
};

hipError_t head_gemms(const std::vector<HeadGemm>& gs, int B, int heads, int amode, int bmode, float alpha,
                      hipStream_t st) {
  std::vector<GemmJob> jobs;
  for (const HeadGemm& g : gs)
    for (int h = 0; h < heads; ++h) {
      GemmJob j = make_job(g.M, g.N, g.c + h * g.hc, g.ldc, 0);
      j.g.alpha = alpha;
      j.g.nbatch = B;
      j.g.bs_a = (int32_t)g.bsa;
      j.g.bs_b = (int32_t)g.bsb;
      j.g.bs_c = (int32_t)g.bsc;
      Operand a = opnd(g.a + h * g.ha, g.lda), b = opnd(g.b + h * g.hb, g.ldb);
      // every batch element's rows must stay 16-B aligned for the vector paths
      a.vec = a.vec && (g.bsa % 4) == 0;
      b.vec = b.vec && (g.bsb % 4) == 0;
      add_src(j, a, b, g.K);
      jobs.push_back(j);
    }
  if (jobs.empty()) return hipSuccess;
  return launch_gemm(jobs.data(), (int)jobs.size(), amode, bmode, 0.f, nullptr, st);
}

}  // namespace

bool wide_supported(int B, int heads, int Lq, int Lk) {
  // strided-batch GEMM strides are int32
  return (int64_t)heads * Lq * Lk < (int64_t)1 << 31 && (int64_t)B * heads * Lq < (int64_t)1 << 40;
}

hipError_t launch_wide_fwd(const WidePair* pairs, int npairs, int B, int heads, int hd, float scale, float drop_p,
                           const RngSnap* rng, bool pooled, hipStream_t st) {
  if (npairs < 1) return hipErrorInvalidValue;
  // S = scale Q K^T  (A = Q [q][d] RK, B = K [k][d] NK), per (pair, head), batched over samples
  std::vector<HeadGemm> gs;
  for (int g = 0; g < npairs; ++g) {
    const WidePair& P = pairs[g];
    gs.push_back({P.Lq, P.Lk, hd, P.q, P.ldq, (int64_t)P.Lq * P.ldq, P.k, P.ldk, (int64_t)P.Lk * P.ldk,
                  P.P, P.Lk, (int64_t)heads * P.Lq * P.Lk, hd, hd, (int64_t)P.Lq * P.Lk});
  }
  hipError_t e = head_gemms(gs, B, heads, MODE_RK, MODE_RK, scale, st);
  if (e != hipSuccess) return e;
  e = launch_rows(RowKind::Softmax, pairs, npairs, B, heads, drop_p, rng, pooled, st);
  if (e != hipSuccess) return e;
  if (pooled) return launch_rows(RowKind::Colmean, pairs, npairs, B, heads, drop_p, rng, pooled, st);
  // O = P' V  (A = P' [q][k] RK, B = V [k][d] KN)
  gs.clear();
  for (int g = 0; g < npairs; ++g) {
    const WidePair& P = pairs[g];
    gs.push_back({P.Lq, hd, P.Lk, P.Pd, P.Lk, (int64_t)heads * P.Lq * P.Lk, P.v, P.ldv, (int64_t)P.Lk * P.ldv,
                  P.o, P.ldo, (int64_t)P.Lq * P.ldo, (int64_t)P.Lq * P.Lk, hd, hd});
  }
  return head_gemms(gs, B, heads, MODE_RK, MODE_KR, 1.f, st);
}

hipError_t launch_wide_bwd(const WidePair* pairs, int npairs, int B, int heads, int hd, float scale, float drop_p,
                           const RngSnap* rng, bool pooled, hipStream_t st) {
  if (npairs < 1) return hipErrorInvalidValue;
  std::vector<HeadGemm> gs;
  hipError_t e;
  if (!pooled) {
    // dP' = dO V^T  (A = dO [q][d] RK, B = V [k][d] NK)
    for (int g = 0; g < npairs; ++g) {
      const WidePair& P = pairs[g];
      gs.push_back({P.Lq, P.Lk, hd, P.dout, P.ldo, (int64_t)P.Lq * P.ldo, P.v, P.ldv, (int64_t)P.Lk * P.ldv,
                    P.dPd, P.Lk, (int64_t)heads * P.Lq * P.Lk, hd, hd, (int64_t)P.Lq * P.Lk});
    }
    if ((e = head_gemms(gs, B, heads, MODE_RK, MODE_RK, 1.f, st)) != hipSuccess) return e;
    // dV = P'^T dO  (A = P' stored [q][k]: KR; B = dO stored [q][d]: KN)
    gs.clear();
    for (int g = 0; g < npairs; ++g) {
      const WidePair& P = pairs[g];
      gs.push_back({P.Lk, hd, P.Lq, P.Pd, P.Lk, (int64_t)heads * P.Lq * P.Lk, P.dout, P.ldo, (int64_t)P.Lq * P.ldo,
                    P.dv, P.ldv, (int64_t)P.Lk * P.ldv, (int64_t)P.Lq * P.Lk, hd, hd});
    }
    if ((e = head_gemms(gs, B, heads, MODE_KR, MODE_KR, 1.f, st)) != hipSuccess) return e;
  }
  if ((e = launch_rows(RowKind::Dsoftmax, pairs, npairs, B, heads, drop_p, rng, pooled, st)) != hipSuccess) return e;
  // dQ = scale dS K  (A = dS [q][k] RK, B = K [k][d] KN)
  gs.clear();
  for (int g = 0; g < npairs; ++g) {
    const WidePair& P = pairs[g];
    gs.push_back({P.Lq, hd, P.Lk, P.dS, P.Lk, (int64_t)heads * P.Lq * P.Lk, P.k, P.ldk, (int64_t)P.Lk * P.ldk,
                  P.dq, P.ldq, (int64_t)P.Lq * P.ldq, (int64_t)P.Lq * P.Lk, hd, hd});
  }
  if ((e = head_gemms(gs, B, heads, MODE_RK, MODE_KR, scale, st)) != hipSuccess) return e;
  // dK = scale dS^T Q  (A = dS stored [q][k]: KR; B = Q stored [q][d]: KN)
  gs.clear();
  for (int g = 0; g < npairs; ++g) {
    const WidePair& P = pairs[g];
    gs.push_back({P.Lk, hd, P.Lq, P.dS, P.Lk, (int64_t)heads * P.Lq * P.Lk, P.q, P.ldq, (int64_t)P.Lq * P.ldq,
                  P.dk, P.ldk, (int64_t)P.Lk * P.ldk, (int64_t)P.Lq * P.Lk, hd, hd});
  }
  return head_gemms(gs, B, heads, MODE_KR, MODE_KR, scale, st);
}

}  // namespace mmf
