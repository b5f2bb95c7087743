// Fused per-sample tail of the pooled HybridFusion plan (forward and backward).
//
// After the attention kernels, everything left in a HybridFusion step works on
// B rows: value/out projections of the query-mean (pooled plan, see
// attention.hip), the aggregation + gating + adaptive weighting
// (src/fusion.py:406-418, compute_adaptive_weights :429-479) and the
// classifier (src/fusion.py:323-328, 419).  As separate GEMM launches these
// are a dozen latency-bound kernels of 2-12 workgroups each.  Here ONE
// workgroup per sample runs the whole chain as GEMVs against L2-resident
// weights (a weight row is read with float4 loads by adjacent lanes), keeping
// every intermediate in LDS.  Nothing mixes samples, so the launch is B
// independent workgroups.
#include <cstdlib>
#include <cstring>

#include "mmf_device.h"

namespace mmf {

namespace {

constexpr int NT = 256;
constexpr int MAXM = 8;
constexpr int MAXHEADS = 8;

__device__ __forceinline__ float wsum(float v) { return sum64(v); }

// GEMVs against L2-resident weights, over S samples of one workgroup: each
// weight element is loaded once and feeds S accumulators.  Sample s's input
// starts at xs + s * xsamp, its output at y + s * ysamp.
// gemv_nt_s: y[n] = sum_k x(n)[k] * W[n][k] for n < N; x(n) = xs + (n / xdiv) * xstride
// (a per-head input when xdiv = head_dim).  Two adjacent lanes share an output
// (k halves, K % 16 == 0), their float4 loads of the W row all in flight.
template <int S>
__device__ __forceinline__ void gemv_nt_s(const float* xs, int xsamp, int xdiv, int xstride,
                                          const float* __restrict__ W, int N, int K, float* y, int ysamp) {
  const int t = threadIdx.x, half = t & 1;
  const int kh = K >> 1;
  for (int n = t >> 1; n < N; n += NT / 2) {
    const float* x0 = xs + (n / xdiv) * xstride + half * kh;
    const float* w = W + (int64_t)n * K + half * kh;
    float acc[S];
#pragma unroll
    for (int q = 0; q < S; ++q) acc[q] = 0.f;
#pragma unroll 4
    for (int k = 0; k < kh; k += 8) {
      const float4 a = *reinterpret_cast<const float4*>(w + k);
      const float4 b = *reinterpret_cast<const float4*>(w + k + 4);
#pragma unroll
      for (int q = 0; q < S; ++q) {
        const float4 xa = *reinterpret_cast<const float4*>(x0 + q * xsamp + k);
        const float4 xb = *reinterpret_cast<const float4*>(x0 + q * xsamp + k + 4);
        acc[q] += a.x * xa.x + a.y * xa.y + a.z * xa.z + a.w * xa.w + b.x * xb.x + b.y * xb.y + b.z * xb.z +
                  b.w * xb.w;
      }
    }
#pragma unroll
    for (int q = 0; q < S; ++q) {
      const float v = acc[q] + dpp<DPP_XOR1>(acc[q]);
      if (half == 0) y[q * ysamp + n] = v;
    }
  }
}

// y_s[k] = sum_{n < N} x_s[n] W[n][k]; red: S * NT floats
template <int S>
__device__ __forceinline__ void gemv_nn_s(const float* x, int xsamp, const float* __restrict__ W, int N, int K,
                                          float* y, int ysamp, float* red) {
  const int t = threadIdx.x, rh = t >> 7, kc = t & 127;
  const int nm = N >> 1;
  for (int k0 = 0; k0 < K; k0 += 128) {
    const int k = k0 + kc;
    float acc[S];
#pragma unroll
    for (int q = 0; q < S; ++q) acc[q] = 0.f;
    if (k < K) {
      const int a = rh ? nm : 0, e = rh ? N : nm;
#pragma unroll 4
      for (int n = a; n < e; ++n) {
        const float w = W[(int64_t)n * K + k];
#pragma unroll
        for (int q = 0; q < S; ++q) acc[q] += x[q * xsamp + n] * w;
      }
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < S; ++q) red[q * NT + t] = acc[q];
    __syncthreads();
    if (rh == 0 && k < K)
#pragma unroll
      for (int q = 0; q < S; ++q) y[q * ysamp + k] = red[q * NT + t] + red[q * NT + t + 128];
  }
}

// y_s[g][k] = sum_{n in segment g} x_s[n] W[n][k] (per-head row blocks of value_proj.weight)
template <int S>
__device__ __forceinline__ void gemv_nn_seg_s(const float* x, int xsamp, const float* __restrict__ W, int nseg,
                                              int seg, int K, float* y, int ysamp) {
  const int t = threadIdx.x, sg = t >> 7, kc = t & 127;
  for (int k0 = 0; k0 < K; k0 += 128) {
    const int k = k0 + kc;
    if (k >= K) continue;
    for (int sgi = sg; sgi < nseg; sgi += NT / 128) {
      const int n0 = sgi * seg;
      float acc[S];
#pragma unroll
      for (int q = 0; q < S; ++q) acc[q] = 0.f;
#pragma unroll 4
      for (int n = 0; n < seg; ++n) {
        const float w = W[(int64_t)(n0 + n) * K + k];
#pragma unroll
        for (int q = 0; q < S; ++q) acc[q] += x[q * xsamp + n0 + n] * w;
      }
#pragma unroll
      for (int q = 0; q < S; ++q) y[q * ysamp + sgi * K + k] = acc[q];
    }
  }
}

// Masked softmax over modalities + renormalisation / fallback (src/fusion.py:462-478);
// see head.hip adaptive_fwd (identical arithmetic).
__device__ float adaptive_w(int M, const float* score, const float* mask, float* sm, float* w) {
  float mx = -INFINITY;
  for (int m = 0; m < M; ++m)
    if (mask[m] > 0.f) mx = fmaxf(mx, score[m]);
  float z = 0.f;
  for (int m = 0; m < M; ++m) {
    sm[m] = (mask[m] > 0.f) ? __expf(score[m] - mx) : 0.f;
    z += sm[m];
  }
  float sw = 0.f, ms = 0.f;
  for (int m = 0; m < M; ++m) {
    sm[m] = (mx == -INFINITY) ? 0.f : sm[m] / z;
    w[m] = sm[m] * mask[m];
    sw += w[m];
    ms += mask[m];
  }
  if (sw > 0.f) {
    const float den = sw + 1e-8f;
    for (int m = 0; m < M; ++m) w[m] = w[m] / den;
  } else {
    for (int m = 0; m < M; ++m) w[m] = ms > 0.f ? mask[m] / (ms + 1e-8f) : 1.f / (float)M;
  }
  return sw;
}

// ---------------------------------------------------------------- per (pair, sample)
// Forward: U_h = pbar_h P_k (+ r_h = sum pbar_h), Obar = U W_v^T (per head) + r b_v,
// Abar = Obar W_o^T + b_o.  grid (B, npairs).
template <int S>
__global__ __launch_bounds__(NT) void tail_pair_fwd_kernel(const TailArgs a) {
  constexpr int TH = TAIL_MAX_H;
  __shared__ float pb_s[MAXHEADS * 128];
  __shared__ __attribute__((aligned(16))) float u_s[S * MAXHEADS * TH];
  __shared__ __attribute__((aligned(16))) float4 red4[NT];
  __shared__ __attribute__((aligned(16))) float v1[S * TH], v2[S * TH];
  __shared__ float r_s[S * MAXHEADS];
  const int b0 = blockIdx.x * S, ns = min(S, a.B - b0);
  const TailPair& P = a.p[blockIdx.y];
  const int t = threadIdx.x;
  const int H = a.H, nh = a.heads, hd = a.hd, Lk = P.Lk, H4 = H >> 2;
  MMF_STAMP(0)
  MMF_STAMP_ID()
  for (int si = 0; si < S; ++si) {
    float* us = u_s + si * nh * H;
    if (si >= ns) {   // no sample: zero inputs keep the batched GEMVs finite
      for (int i = t; i < nh * H; i += NT) us[i] = 0.f;
      if (t < nh) r_s[si * MAXHEADS + t] = 0.f;
      continue;
    }
    const int b = b0 + si;
    __syncthreads();   // pb_s of the previous sample consumed
    for (int i = t; i < nh * Lk; i += NT) pb_s[i] = P.pbar[(int64_t)b * nh * Lk + i];
    __syncthreads();
    if (t < nh) {
      float s = 0.f;
      for (int j = 0; j < Lk; ++j) s += pb_s[t * Lk + j];
      r_s[si * MAXHEADS + t] = s;
      P.r[(int64_t)b * nh + t] = s;
    }
    MMF_STAMP(1)
    // U: thread (float4 column c4, row group rg) loads each P_k float4 once and feeds
    // every head with it (one pass over P_k[b]); the RG row groups are summed in order
    const float* pk = P.Pk + (int64_t)b * Lk * H;
    const int RG = NT / H4;
    const int c4 = t % H4, rg = t / H4;
    float4 acc[MAXHEADS];
#pragma unroll
    for (int hh = 0; hh < MAXHEADS; ++hh) acc[hh] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 2
    for (int j = rg; j < Lk; j += RG) {
      const float4 v = *reinterpret_cast<const float4*>(pk + (int64_t)j * H + 4 * c4);
#pragma unroll
      for (int hh = 0; hh < MAXHEADS; ++hh) {
        if (hh < nh) {
          const float w = pb_s[hh * Lk + j];
          acc[hh].x += w * v.x; acc[hh].y += w * v.y; acc[hh].z += w * v.z; acc[hh].w += w * v.w;
        }
      }
    }
#pragma unroll
    for (int hh = 0; hh < MAXHEADS; ++hh) {
      if (hh < nh) {
        __syncthreads();
        red4[t] = acc[hh];
        __syncthreads();
        if (t < H4) {
          float4 sum = red4[t];
          for (int g = 1; g < RG; ++g) {
            const float4 v = red4[g * H4 + t];
            sum.x += v.x; sum.y += v.y; sum.z += v.z; sum.w += v.w;
          }
          *reinterpret_cast<float4*>(&us[hh * H + 4 * t]) = sum;
          *reinterpret_cast<float4*>(P.U + ((int64_t)b * nh + hh) * H + 4 * t) = sum;
        }
      }
    }
  }
  __syncthreads();
  MMF_STAMP(2)
  // Obar = U W_v^T (per head) + r b_v;  Abar = Obar W_o^T + b_o
  gemv_nt_s<S>(u_s, nh * H, hd, H, P.Wv, H, H, v1, TH);
  __syncthreads();
  MMF_STAMP(3)
  for (int i = t; i < S * H; i += NT) {
    const int si = i / H, n = i - si * H;
    const float o = v1[si * TH + n] + r_s[si * MAXHEADS + n / hd] * P.bv[n];
    v1[si * TH + n] = o;
    if (si < ns) P.Ob[(int64_t)(b0 + si) * H + n] = o;
  }
  __syncthreads();
  gemv_nt_s<S>(v1, TH, 1 << 30, 0, P.Wo, H, H, v2, TH);
  __syncthreads();
  MMF_STAMP(4)
  for (int i = t; i < ns * H; i += NT) {
    const int si = i / H, n = i - si * H;
    P.Ab[(int64_t)(b0 + si) * H + n] = v2[si * TH + n] + P.bo[n];
  }
  MMF_STAMP(5)
}

// Backward: dObar = cvec_q W_o; dU_h = dObar_h W_v[h rows];
// dpbar_h[j] = P_k[j] . dU_h + dObar_h . b_v,h.  grid (B, npairs).
template <int S>
__global__ __launch_bounds__(NT) void tail_pair_bwd_kernel(const TailArgs a) {
  constexpr int TH = TAIL_MAX_H;
  __shared__ __attribute__((aligned(16))) float c_s[S * TH], v1[S * TH];
  __shared__ __attribute__((aligned(16))) float du_s[S * MAXHEADS * TH];
  __shared__ float red[S * NT];
  __shared__ float dr_s[S * MAXHEADS];
  const int b0 = blockIdx.x * S, ns = min(S, a.B - b0);
  const TailPair& P = a.p[blockIdx.y];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int H = a.H, nh = a.heads, hd = a.hd, Lk = P.Lk, M = a.M;
  constexpr int DUS = MAXHEADS * TH;   // du_s stride per sample
  for (int i = t; i < S * H; i += NT) {
    const int si = i / H, n = i - si * H;
    c_s[si * TH + n] = si < ns ? a.cvec[((int64_t)(b0 + si) * M + P.q) * H + n] : 0.f;
  }
  __syncthreads();
  gemv_nn_s<S>(c_s, TH, P.Wo, H, H, v1, TH, red);
  __syncthreads();
  for (int i = t; i < ns * H; i += NT) {
    const int si = i / H, n = i - si * H;
    P.dOb[(int64_t)(b0 + si) * H + n] = v1[si * TH + n];
  }
  gemv_nn_seg_s<S>(v1, TH, P.Wv, nh, hd, H, du_s, DUS);
  for (int sh = wave; sh < S * nh; sh += NT / 64) {
    const int si = sh / nh, hh = sh - si * nh;
    float s = 0.f;
    for (int d = lane; d < hd; d += 64) s += v1[si * TH + hh * hd + d] * P.bv[hh * hd + d];
    s = wsum(s);
    if (lane == 0) dr_s[si * MAXHEADS + hh] = s;
  }
  __syncthreads();
  for (int i = t; i < ns * nh * H; i += NT) {
    const int si = i / (nh * H), r = i - si * nh * H;
    P.dU[(int64_t)(b0 + si) * nh * H + r] = du_s[si * DUS + r];
  }
  // dpbar: a wave takes two keys per step (lane halves), lanes stride the H/4 float4 columns
  const int half = lane >> 5, l32 = lane & 31;
  for (int si = 0; si < ns; ++si) {
    const int b = b0 + si;
    const float* pk = P.Pk + (int64_t)b * Lk * H;
    const float* du = du_s + si * DUS;
#pragma unroll 2
    for (int j0 = 2 * wave; j0 < Lk; j0 += 2 * (NT / 64)) {
      const int j = j0 + half;
      float acc[MAXHEADS];
#pragma unroll
      for (int hh = 0; hh < MAXHEADS; ++hh) acc[hh] = 0.f;
      if (j < Lk) {
        for (int c4 = l32; c4 < H / 4; c4 += 32) {
          const float4 v = *reinterpret_cast<const float4*>(pk + (int64_t)j * H + 4 * c4);
#pragma unroll
          for (int hh = 0; hh < MAXHEADS; ++hh) {
            if (hh < nh) {
              const float4 u = *reinterpret_cast<const float4*>(&du[hh * H + 4 * c4]);
              acc[hh] += v.x * u.x + v.y * u.y + v.z * u.z + v.w * u.w;
            }
          }
        }
      }
#pragma unroll
      for (int hh = 0; hh < MAXHEADS; ++hh) {
        if (hh < nh) {
          const float sv = sum32(acc[hh]);
          if (l32 == 0 && j < Lk) P.dpbar[((int64_t)b * nh + hh) * Lk + j] = sv + dr_s[si * MAXHEADS + hh];
        }
      }
    }
  }
}

// ---------------------------------------------------------------- per sample
// Forward head: pooled_m = mask_m / n_m (mean_L P_m + sum_{g: q(g)=m} Abar_g), gating
// scores, adaptive weights, fused, classifier.  grid (B).
__global__ __launch_bounds__(NT) void tail_head_fwd_kernel(const TailArgs a) {
  __shared__ __attribute__((aligned(16))) float pooled_s[MAXM * TAIL_MAX_H];
  __shared__ __attribute__((aligned(16))) float v1[TAIL_MAX_H], v2[TAIL_MAX_H];
  __shared__ __attribute__((aligned(16))) float4 red4[NT];
  __shared__ float score_s[MAXM], w_s[MAXM];
  const int b = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int M = a.M, H = a.H;
  const int H4 = H >> 2;

  // (1) mean over L of P_m (the modality's own entry of the aggregation list)
  for (int m = 0; m < M; ++m) {
    const int L = a.L[m];
    if (a.Pcol[m]) {
      // the projection GEMM's per-tile column sums: ncol rows per sample
      const int nc = a.ncol[m];
      const float* pc = a.Pcol[m] + (int64_t)b * nc * H;
      for (int n = t; n < H; n += NT) {
        float s = 0.f;
        for (int c = 0; c < nc; ++c) s += pc[(int64_t)c * H + n];
        pooled_s[m * H + n] = s * (1.f / (float)L);
      }
      __syncthreads();
      continue;
    }
    const float* base = a.P[m] + (int64_t)b * L * H;
    const int RG = NT / H4;
    const int c4 = t % H4, rg = t / H4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f), acc2 = acc;
    if (rg < RG) {
      int r = rg;
#pragma unroll 4
      for (; r + RG < L; r += 2 * RG) {
        const float4 v = *reinterpret_cast<const float4*>(base + (int64_t)r * H + 4 * c4);
        const float4 u = *reinterpret_cast<const float4*>(base + (int64_t)(r + RG) * H + 4 * c4);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        acc2.x += u.x; acc2.y += u.y; acc2.z += u.z; acc2.w += u.w;
      }
      if (r < L) {
        const float4 v = *reinterpret_cast<const float4*>(base + (int64_t)r * H + 4 * c4);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
    }
    red4[t] = make_float4(acc.x + acc2.x, acc.y + acc2.y, acc.z + acc2.z, acc.w + acc2.w);
    __syncthreads();
    if (t < H4) {
      float4 s = red4[t];
      for (int g = 1; g < RG; ++g) {
        const float4 v = red4[g * H4 + t];
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
      const float f = 1.f / (float)L;
      *reinterpret_cast<float4*>(&pooled_s[m * H + 4 * t]) = make_float4(s.x * f, s.y * f, s.z * f, s.w * f);
    }
    __syncthreads();
  }
  // (2) + the attended means of every pair whose query is m, then agg * mask / n_m
  for (int i = t; i < M * H; i += NT) {
    const int m = i / H, n = i - m * H;
    float v = pooled_s[i];
    for (int g = 0; g < a.npairs; ++g)
      if (a.p[g].q == m) v += a.p[g].Ab[(int64_t)b * H + n];
    v *= a.inv_cnt[m] * a.mask[(int64_t)b * M + m];
    pooled_s[i] = v;
    a.pooled[(int64_t)b * M * H + i] = v;
  }
  __syncthreads();
  // (3) gating scores (nn.Linear(H, 1), src/fusion.py:316-321,452-461), adaptive weights
  for (int m = wave; m < M; m += NT / 64) {
    float s = 0.f;
    for (int j = lane; j < H; j += 64) s += pooled_s[m * H + j] * a.gate_w[m][j];
    s = wsum(s);
    if (lane == 0) score_s[m] = s + a.gate_b[m][0];
  }
  __syncthreads();
  if (t == 0) {
    float msk[MAXM], sm[MAXM], w[MAXM];
    for (int m = 0; m < M; ++m) msk[m] = a.mask[(int64_t)b * M + m];
    adaptive_w(M, score_s, msk, sm, w);
    for (int m = 0; m < M; ++m) {
      w_s[m] = w[m];
      a.scores[(int64_t)b * M + m] = score_s[m];
      a.weights[(int64_t)b * M + m] = w[m];
      if (a.weights_out) a.weights_out[(int64_t)b * M + m] = w[m];
    }
  }
  __syncthreads();
  // (4) fused = sum_m w_m pooled_m; classifier Linear -> ReLU -> Dropout -> Linear
  for (int j = t; j < H; j += NT) {
    float f = 0.f;
    for (int m = 0; m < M; ++m) f += pooled_s[m * H + j] * w_s[m];
    v1[j] = f;
    a.fused[(int64_t)b * H + j] = f;
  }
  __syncthreads();
  gemv_nt_s<1>(v1, 0, 1 << 30, 0, a.W1, H, H, v2, 0);
  __syncthreads();
  const float p = a.drop_p;
  const bool drop = p > 0.f && a.rng != nullptr;
  RngSnap rs{0, 0};
  if (drop) rs = *a.rng;
  const float inv_keep = p < 1.f ? 1.f / (1.f - p) : 0.f;
  for (int n = t; n < H; n += NT) {
    float x = fmaxf(v2[n] + a.b1[n], 0.f);
    if (drop) x = keep1(rs, a.drop_site, (uint64_t)b * H + n, p) ? x * inv_keep : 0.f;
    v2[n] = x;
    a.h1[(int64_t)b * H + n] = x;
  }
  __syncthreads();
  for (int c = wave; c < a.C; c += NT / 64) {
    float s = 0.f;
    for (int j = lane; j < H; j += 64) s += v2[j] * a.W2[(int64_t)c * H + j];
    s = wsum(s);
    if (lane == 0) a.logits[(int64_t)b * a.C + c] = s + a.b2[c];
  }
}

// Backward head: dz1 = ReLU'/Dropout'(dlogits W2), dfused = dz1 W1, head backward
// (dscore, cvec = dpooled * mask / n).  grid (B).
__global__ __launch_bounds__(NT) void tail_head_bwd_kernel(const TailArgs a) {
  __shared__ __attribute__((aligned(16))) float pooled_s[MAXM * TAIL_MAX_H];
  __shared__ __attribute__((aligned(16))) float v1[TAIL_MAX_H], v2[TAIL_MAX_H], dl_s[256];
  __shared__ float red[NT];
  __shared__ float dw_s[MAXM], dscore_s[MAXM];
  const int b = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int M = a.M, H = a.H, C = a.C;

  for (int c = t; c < C; c += NT) dl_s[c] = a.dlogits[(int64_t)b * C + c];
  for (int i = t; i < M * H; i += NT) pooled_s[i] = a.pooled[(int64_t)b * M * H + i];
  __syncthreads();
  // the saved h1 is post-dropout, so h1 > 0 marks kept, active units (gscale = 1/(1-p))
  gemv_nn_s<1>(dl_s, 0, a.W2, C, H, v1, 0, red);
  __syncthreads();
  for (int n = t; n < H; n += NT) {
    const float z = a.h1[(int64_t)b * H + n] > 0.f ? v1[n] * a.gscale : 0.f;
    v1[n] = z;
    a.dz1[(int64_t)b * H + n] = z;
  }
  __syncthreads();
  gemv_nn_s<1>(v1, 0, a.W1, H, H, v2, 0, red);
  __syncthreads();
  // head backward (head.hip head_bwd_kernel): dw_m = dfused . pooled_m
  for (int m = wave; m < M; m += NT / 64) {
    float s = 0.f;
    for (int j = lane; j < H; j += 64) s += v2[j] * pooled_s[m * H + j];
    s = wsum(s);
    if (lane == 0) dw_s[m] = s;
  }
  __syncthreads();
  if (t == 0) {
    float msk[MAXM], sc[MAXM], sm[MAXM], w[MAXM], ds[MAXM];
    for (int m = 0; m < M; ++m) {
      msk[m] = a.mask[(int64_t)b * M + m];
      sc[m] = a.scores[(int64_t)b * M + m];
      ds[m] = 0.f;
    }
    const float sw = adaptive_w(M, sc, msk, sm, w);
    if (sw > 0.f) {
      const float S = sw + 1e-8f;
      float dot = 0.f;
      for (int m = 0; m < M; ++m) dot += dw_s[m] * sm[m] * msk[m];
      float dsm[MAXM], sdot = 0.f;
      for (int m = 0; m < M; ++m) {
        dsm[m] = (dw_s[m] / S - dot / (S * S)) * msk[m];
        sdot += sm[m] * dsm[m];
      }
      for (int m = 0; m < M; ++m) ds[m] = msk[m] > 0.f ? sm[m] * (dsm[m] - sdot) : 0.f;
    }
    for (int m = 0; m < M; ++m) {
      dscore_s[m] = ds[m];
      a.dscore[(int64_t)b * M + m] = ds[m];
    }
  }
  __syncthreads();
  for (int i = t; i < M * H; i += NT) {
    const int m = i / H, j = i - m * H;
    const float wm = a.weights[(int64_t)b * M + m];
    const float f = a.mask[(int64_t)b * M + m] * a.inv_cnt[m];
    a.cvec[(int64_t)b * M * H + i] = (wm * v2[j] + dscore_s[m] * a.gate_w[m][j]) * f;
  }
}

}  // namespace

// Samples per workgroup of the per-(pair, sample) kernels (MMF_TAIL_S = 2 or 4
// overrides, for tuning).  Measured at C2 (B = 256, 6 pairs): S = 1 / 2 / 4 ->
// pair bwd 52.7 / 70.3 / 120.1 us, pair fwd 45.6 / 50.7 / 76.2 us.  The chains
// are latency-bound, so the weight reuse of S > 1 loses to the parallelism it
// removes; S = 1 it is.
int tail_samples() {
  static int s = 0;
  if (s == 0) {
    const char* e = getenv("MMF_TAIL_S");
    s = e ? atoi(e) : 1;
    if (s != 1 && s != 2 && s != 4) s = 1;
  }
  return s;
}

bool tail_supported(int M, int H, int C, int heads, int hd, int npairs) {
  return M <= MAXM && heads <= MAXHEADS && H % 16 == 0 && H <= TAIL_MAX_H && C <= 256 &&
         npairs <= TAIL_MAX_PAIRS && hd % 8 == 0 && (NT % (H / 4)) == 0;
}

hipError_t launch_tail_fwd(const TailArgs& a, hipStream_t st) {
  if (!tail_supported(a.M, a.H, a.C, a.heads, a.hd, a.npairs)) return hipErrorInvalidValue;
  for (int g = 0; g < a.npairs; ++g)
    if (a.p[g].Lk > 128) return hipErrorInvalidValue;
  const double B = a.B, H = a.H;
  if (a.npairs) {
    // per pair: Vbar = U W_v^T (+ r b_v), Obar = Vbar W_o^T + b_o; weights read once
    ProfLaunch prof_(st, "tail_pair_fwd_kernel", 4.0 * B * H * H * a.npairs,
                     4.0 * a.npairs * (2 * H * H + B * (a.heads * H + 2 * H)));
    const int S = tail_samples();
    if (S == 4) hipLaunchKernelGGL(tail_pair_fwd_kernel<4>, dim3((a.B + 3) / 4, a.npairs), dim3(NT), 0, st, a);
    else if (S == 2) hipLaunchKernelGGL(tail_pair_fwd_kernel<2>, dim3((a.B + 1) / 2, a.npairs), dim3(NT), 0, st, a);
    else hipLaunchKernelGGL(tail_pair_fwd_kernel<1>, dim3(a.B, a.npairs), dim3(NT), 0, st, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  // pooling, gating, adaptive weights, weighted sum, classifier
  ProfLaunch prof_(st, "tail_head_fwd_kernel", 2.0 * B * H * (H + a.C) + 4.0 * a.M * B * H,
                   4.0 * (H * (H + a.C) + B * (a.M * H + a.C)));
  hipLaunchKernelGGL(tail_head_fwd_kernel, dim3(a.B), dim3(NT), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_tail_bwd(const TailArgs& a, hipStream_t st) {
  if (!tail_supported(a.M, a.H, a.C, a.heads, a.hd, a.npairs)) return hipErrorInvalidValue;
  const double B = a.B, H = a.H;
  {
    ProfLaunch prof_(st, "tail_head_bwd_kernel", 2.0 * B * H * (H + a.C) + 4.0 * a.M * B * H,
                     4.0 * (H * (H + a.C) + B * (a.M * H + a.C)));
    hipLaunchKernelGGL(tail_head_bwd_kernel, dim3(a.B), dim3(NT), 0, st, a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !a.npairs) return e;
  {
    ProfLaunch prof_(st, "tail_pair_bwd_kernel", 4.0 * B * H * H * a.npairs,
                     4.0 * a.npairs * (2 * H * H + B * (a.heads * H + 2 * H)));
    const int S = tail_samples();
    if (S == 4) hipLaunchKernelGGL(tail_pair_bwd_kernel<4>, dim3((a.B + 3) / 4, a.npairs), dim3(NT), 0, st, a);
    else if (S == 2) hipLaunchKernelGGL(tail_pair_bwd_kernel<2>, dim3((a.B + 1) / 2, a.npairs), dim3(NT), 0, st, a);
    else hipLaunchKernelGGL(tail_pair_bwd_kernel<1>, dim3(a.B, a.npairs), dim3(NT), 0, st, a);
  }
  return hipGetLastError();
}

}  // namespace mmf

#ifdef MMF_STAMPS
extern "C" int mmf_tail_stamps_read(void* out, size_t bytes) {   // tail_pair_fwd_kernel phases
  if (bytes > sizeof(mmf::g_mmf_stamps)) bytes = sizeof(mmf::g_mmf_stamps);
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mmf::g_mmf_stamps), bytes) == hipSuccess ? 0 : 3;
}
#endif
