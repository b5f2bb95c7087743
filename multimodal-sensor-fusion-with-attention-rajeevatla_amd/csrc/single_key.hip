// Single-key attention (Lk == 1): the reference's 2-D-input case.
//
// With one key, softmax over the key axis is 1 for an unmasked key and
// -inf -> NaN -> nan_to_num -> 0 for a masked one (src/attention.py:118-129), so
// the post-dropout probability of (b, head, q) is
//     P'[b, h, q, 0] = [mask_b != 0] * keep(b, h, q) / (1 - p)
// independent of Q and K.  Q, K, QK^T and their gradients are dead: dS =
// P (dP - rowsum(P dP)) = P dP (1 - P) = 0 exactly, so query_proj / key_proj
// receive exactly zero gradient (as the reference's autograd produces).  These
// kernels produce what the rest of the path consumes instead:
//   sk_fwd : pbar[b, h] = mean_q P' (the pooled plan's query-mean probabilities,
//            also its (B, Lk, heads) transpose, the same layout at Lk = 1) and
//            the attention maps (B, h, Lq, 1);
//   sk_out : O[b, q, h*hd + d] = P'[b, h, q] V[b, 0, h*hd + d] (general plan,
//            standalone CrossModalAttention);
//   sk_dv  : dV[b, 0, c] = sum_q P'[b, h(c), q] dO[b, q, c]   (fixed order).
// The dropout keep decision of (b, h, q) is element ((b*heads + h)*Lq + q)*Lk + 0
// of the pair's probability tensor: the same Philox stream every attention kernel
// of the library draws (mmf_device.h keep1), so the HIP path and the Philox replay
// in tests/_philox.py agree.
#include <algorithm>
#include <cstring>

#include "mmf_device.h"

namespace mmf {
namespace {

__device__ __forceinline__ float sk_prob(const SkPair& P, const RngSnap& rs, int heads, int b, int h, int q,
                                         float pdrop, float inv_keep) {
  if (P.kmask_mode != 0 && P.kmask[(int64_t)b * P.kmask_ld] == 0.f) return 0.f;   // masked_fill(mask == 0)
  if (pdrop > 0.f)
    return keep1(rs, P.drop_site, ((uint64_t)b * heads + h) * (uint64_t)P.Lq + q, pdrop) ? inv_keep : 0.f;
  return 1.f;
}

// one thread per (b, head) of one pair (blockIdx.y): the query loop runs in order
__global__ __launch_bounds__(256) void sk_fwd_kernel(const SkArgs A) {
  const SkPair& P = A.p[blockIdx.y];
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= A.B * A.heads) return;
  const int b = i / A.heads, h = i % A.heads;
  RngSnap rs{0, 0};
  if (A.drop_p > 0.f && A.rng) rs = *A.rng;
  const float inv_keep = A.drop_p < 1.f ? 1.f / (1.f - A.drop_p) : 0.f;
  float sum = 0.f;
  for (int q = 0; q < P.Lq; ++q) {
    const float pk = sk_prob(P, rs, A.heads, b, h, q, A.drop_p, inv_keep);
    if (P.probs) P.probs[(int64_t)i * P.Lq + q] = pk;
    sum += pk;
  }
  const float v = sum * (1.f / (float)P.Lq);
  if (P.pbar) P.pbar[i] = v;
  if (P.pbarT) P.pbarT[i] = v;
}

// one thread per output element (b, q, c) of one pair
__global__ __launch_bounds__(256) void sk_out_kernel(const SkArgs A) {
  const SkPair& P = A.p[blockIdx.y];
  const int H = A.heads * A.hd;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)A.B * P.Lq * H) return;
  const int c = (int)(e % H);
  const int64_t r = e / H;
  const int q = (int)(r % P.Lq), b = (int)(r / P.Lq);
  RngSnap rs{0, 0};
  if (A.drop_p > 0.f && A.rng) rs = *A.rng;
  const float inv_keep = A.drop_p < 1.f ? 1.f / (1.f - A.drop_p) : 0.f;
  const float pk = sk_prob(P, rs, A.heads, b, c / A.hd, q, A.drop_p, inv_keep);
  P.o[((int64_t)b * P.Lq + q) * P.ldo + c] = pk * P.v[(int64_t)b * P.ldv + c];
}

// one thread per (b, c) of one pair
__global__ __launch_bounds__(256) void sk_dv_kernel(const SkArgs A) {
  const SkPair& P = A.p[blockIdx.y];
  const int H = A.heads * A.hd;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= A.B * H) return;
  const int b = i / H, c = i % H, h = c / A.hd;
  RngSnap rs{0, 0};
  if (A.drop_p > 0.f && A.rng) rs = *A.rng;
  const float inv_keep = A.drop_p < 1.f ? 1.f / (1.f - A.drop_p) : 0.f;
  float acc = 0.f;
  for (int q = 0; q < P.Lq; ++q) {
    const float pk = sk_prob(P, rs, A.heads, b, h, q, A.drop_p, inv_keep);
    acc = fmaf(pk, P.dout[((int64_t)b * P.Lq + q) * P.ldo + c], acc);
  }
  P.dv[(int64_t)b * P.ldv + c] = acc;
}

// zero-fill of up to 16 buffers of 4-byte words in one launch (a kernel node under graph capture)
constexpr int ZERO_MAX = 16;
struct ZeroArgs {
  float* p[ZERO_MAX];
  int64_t n[ZERO_MAX];
};
__global__ __launch_bounds__(256) void zero_fill_kernel(const ZeroArgs a) {
  float* p = a.p[blockIdx.y];
  const int64_t n = a.n[blockIdx.y];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) p[i] = 0.f;
}

SkArgs sk_args(const SkPair* pairs, int npairs, int B, int heads, int hd, float drop_p, const RngSnap* rng) {
  SkArgs a;
  memset(&a, 0, sizeof(a));
  for (int g = 0; g < npairs; ++g) a.p[g] = pairs[g];
  a.npairs = npairs; a.B = B; a.heads = heads; a.hd = hd; a.drop_p = drop_p; a.rng = rng;
  return a;
}

}  // namespace

hipError_t launch_sk_fwd(const SkPair* pairs, int npairs, int B, int heads, int hd, float drop_p,
                         const RngSnap* rng, hipStream_t st) {
  if (npairs < 1) return hipErrorInvalidValue;
  if (npairs > SK_MAX_PAIRS) {
    const hipError_t e = launch_sk_fwd(pairs, SK_MAX_PAIRS, B, heads, hd, drop_p, rng, st);
    return e != hipSuccess ? e : launch_sk_fwd(pairs + SK_MAX_PAIRS, npairs - SK_MAX_PAIRS, B, heads, hd, drop_p, rng, st);
  }
  const SkArgs a = sk_args(pairs, npairs, B, heads, hd, drop_p, rng);
  double by = 0.0;
  for (int g = 0; g < npairs; ++g)
    by += 4.0 * B * heads * ((pairs[g].probs ? pairs[g].Lq : 0) + (pairs[g].pbar ? 1 : 0) + (pairs[g].pbarT ? 1 : 0));
  ProfLaunch prof_(st, "sk_fwd_kernel", 0.0, by);
  mmf_launch(sk_fwd_kernel, dim3((B * heads + 255) / 256, npairs), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_sk_out(const SkPair* pairs, int npairs, int B, int heads, int hd, float drop_p,
                         const RngSnap* rng, hipStream_t st) {
  if (npairs < 1) return hipErrorInvalidValue;
  if (npairs > SK_MAX_PAIRS) {
    const hipError_t e = launch_sk_out(pairs, SK_MAX_PAIRS, B, heads, hd, drop_p, rng, st);
    return e != hipSuccess ? e : launch_sk_out(pairs + SK_MAX_PAIRS, npairs - SK_MAX_PAIRS, B, heads, hd, drop_p, rng, st);
  }
  const SkArgs a = sk_args(pairs, npairs, B, heads, hd, drop_p, rng);
  int64_t maxe = 1;
  double by = 0.0, fl = 0.0;
  for (int g = 0; g < npairs; ++g) {
    const int64_t e = (int64_t)B * pairs[g].Lq * heads * hd;
    maxe = e > maxe ? e : maxe;
    by += 4.0 * (e + (double)B * heads * hd);
    fl += (double)e;
  }
  ProfLaunch prof_(st, "sk_out_kernel", fl, by);
  mmf_launch(sk_out_kernel, dim3((unsigned)((maxe + 255) / 256), npairs), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_sk_dv(const SkPair* pairs, int npairs, int B, int heads, int hd, float drop_p,
                        const RngSnap* rng, hipStream_t st) {
  if (npairs < 1) return hipErrorInvalidValue;
  if (npairs > SK_MAX_PAIRS) {
    const hipError_t e = launch_sk_dv(pairs, SK_MAX_PAIRS, B, heads, hd, drop_p, rng, st);
    return e != hipSuccess ? e : launch_sk_dv(pairs + SK_MAX_PAIRS, npairs - SK_MAX_PAIRS, B, heads, hd, drop_p, rng, st);
  }
  const SkArgs a = sk_args(pairs, npairs, B, heads, hd, drop_p, rng);
  double by = 0.0, fl = 0.0;
  for (int g = 0; g < npairs; ++g) {
    by += 4.0 * ((double)B * pairs[g].Lq * heads * hd + (double)B * heads * hd);
    fl += 2.0 * B * pairs[g].Lq * heads * hd;
  }
  ProfLaunch prof_(st, "sk_dv_kernel", fl, by);
  mmf_launch(sk_dv_kernel, dim3((B * heads * hd + 255) / 256, npairs), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_zero_fill(float* const* ptrs, const int64_t* counts, int n, hipStream_t st) {
  ZeroArgs a;
  memset(&a, 0, sizeof(a));
  int m = 0;
  int64_t maxn = 0;
  for (int i = 0; i < n && m < ZERO_MAX; ++i)
    if (ptrs[i] && counts[i] > 0) {
      a.p[m] = ptrs[i];
      a.n[m] = counts[i];
      maxn = counts[i] > maxn ? counts[i] : maxn;
      ++m;
    }
  if (m == 0) return hipSuccess;
  if (n > ZERO_MAX) return hipErrorInvalidValue;
  const unsigned blocks = (unsigned)std::min<int64_t>((maxn + 255) / 256, 1024);
  ProfLaunch prof_(st, "zero_fill_kernel", 0.0, 4.0 * (double)maxn * m);
  mmf_launch(zero_fill_kernel, dim3(blocks, m), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace mmf
