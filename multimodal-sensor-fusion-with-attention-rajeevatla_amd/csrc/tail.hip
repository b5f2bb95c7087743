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
    for (int hh = t >> 6; hh < nh; hh += NT / 64) {   // r_h: one wave per head
      float s = 0.f;
      for (int j = t & 63; j < Lk; j += 64) s += pb_s[hh * Lk + j];
      s = wsum(s);
      if ((t & 63) == 0) {
        r_s[si * MAXHEADS + hh] = s;
        P.r[(int64_t)b * nh + hh] = s;
      }
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

// ---------------------------------------------------------------- MFMA pair tail
// The pair tail as two kinds of launch per direction, on fp32 MFMA tiles
// (v_mfma_f32_32x32x2_f32, exact f32 products) when hd % 32 == 0, H % 32 == 0
// and at most 32 (pair, head) rows share a key modality:
//  * P_k side, one workgroup per (sample, key modality k): every pair whose key
//    is k reads P_k[b] once.  Forward U_{g,h} = pbar_{g,h} P_k and r_{g,h} =
//    sum_j pbar_{g,h}[j]; backward dpbar_{g,h} = P_k dU_{g,h} + dObar_{g,h} . b_v,h.
//    The (pair, head) rows are one 32-row MFMA tile.
//  * weight side, one workgroup per (pair, 32 samples): forward Obar = U W_v^T
//    (per head) + r b_v, Abar = Obar W_o^T + b_o; backward dObar = c_q W_o and
//    dU_h = dObar_h W_v[h rows].  A weight element is read once per 32 samples
//    (the per-sample GEMV kernels above read the 128 KB of W_v, W_o per sample).
// MFMA k order: within each 8-deep chunk, lane half hf feeds k = 8 q + 4 hf + s at
// step s (one float4 per lane and chunk for row-contiguous operands).
constexpr int KG_ROWS = 32;

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

__device__ __forceinline__ f32x16 mfma4(const float4& a, const float4& b, f32x16 acc) {
  acc = mfma32(a.x, b.x, acc);
  acc = mfma32(a.y, b.y, acc);
  acc = mfma32(a.z, b.z, acc);
  return mfma32(a.w, b.w, acc);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.f;
  return z;
}

// Forward, P_k side: grid (B, key groups).  Thread (float4 column c4, row group rg)
// loads its Lk / RG rows of P_k[b] at once (before the pbar rows are staged) and
// accumulates eight (pair, head) rows per pass; the row groups are summed in order.
__global__ __launch_bounds__(NT, 3) void tail_u_kernel(const TailArgs a) {
  constexpr int PS = 128 + 4;   // pbar image pitch (keys <= 128)
  constexpr int RPT = 16;       // P_k rows per thread and batch
  __shared__ __attribute__((aligned(16))) float pb_s[KG_ROWS * PS];
  __shared__ __attribute__((aligned(16))) float4 red4[8 * NT];
  const int b = blockIdx.x, kg = blockIdx.y;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int H = a.H, nh = a.heads, R = a.kg_cnt[kg] * nh, H4 = H >> 2, RG = NT / H4;
  const int c4 = t % H4, rg = t / H4;
  const TailPair& P0 = a.p[a.kg_pair[kg][0]];
  const int Lk = P0.Lk;
  const float* pk = P0.Pk + (int64_t)b * Lk * H + 4 * c4;
  float4 v[RPT];
  auto load_rows = [&](int j0) {
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      // (unconditional, clamped: every use is guarded by j < Lk; a select here compiled to a
      // branch whose other side waited for the load before zeroing its registers)
      const int j = j0 + rg + RG * i;
      v[i] = ld4(pk + (int64_t)min(j, Lk - 1) * H);
    }
  };
  load_rows(0);
  const int per = nh * Lk;   // pbar floats of one pair for sample b (contiguous: (B, heads, Lk))
  if (per % 64 == 0) {
    // wave-uniform pair slot per chunk: its pbar pointer is a scalar load, every value load of
    // the staging issued before the first LDS write (a per-lane index into the pair table was a
    // vector load of the pointer and a wait, per element chunk)
    constexpr int U = 4;
    for (int i0 = 0; i0 < R * Lk; i0 += U * NT) {
      float vv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = min(i0 + u * NT + t, R * Lk - 1);
        const int slot = __builtin_amdgcn_readfirstlane(i / per);
        vv[u] = a.p[a.kg_pair[kg][slot]].pbar[(int64_t)b * per + (i - slot * per)];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * NT + t;
        if (i < R * Lk) {
          const int row = i / Lk, j = i - row * Lk;
          pb_s[row * PS + j] = vv[u];
        }
      }
    }
  } else {
    for (int i = t; i < R * Lk; i += NT) {
      const int row = i / Lk, j = i - row * Lk;
      pb_s[row * PS + j] = a.p[a.kg_pair[kg][row / nh]].pbar[((int64_t)b * nh + row % nh) * Lk + j];
    }
  }
  __syncthreads();
  for (int row = w; row < R; row += NT / 64) {   // r_{g,h}
    float s = 0.f;
    for (int j = lane; j < Lk; j += 64) s += pb_s[row * PS + j];
    s = wsum(s);
    if (lane == 0) a.p[a.kg_pair[kg][row / nh]].r[(int64_t)b * nh + row % nh] = s;
  }
  for (int r0 = 0; r0 < R; r0 += 8) {
    float4 acc[8];
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) acc[rr] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int j0 = 0; j0 < Lk; j0 += RG * RPT) {
      if (j0 > 0) load_rows(j0);
#pragma unroll
      for (int i = 0; i < RPT; ++i) {
        const int j = j0 + rg + RG * i;
        if (j < Lk) {
#pragma unroll
          for (int rr = 0; rr < 8; ++rr) {
            if (r0 + rr < R) {
              const float wgt = pb_s[(r0 + rr) * PS + j];
              acc[rr].x += wgt * v[i].x; acc[rr].y += wgt * v[i].y;
              acc[rr].z += wgt * v[i].z; acc[rr].w += wgt * v[i].w;
            }
          }
        }
      }
    }
    if (R > 8 && Lk > RG * RPT) load_rows(0);   // the next pass starts from the first batch again
#pragma unroll
    for (int rr = 0; rr < 8; ++rr) red4[rr * NT + t] = acc[rr];
    __syncthreads();
    for (int task = t; task < 8 * H4; task += NT) {
      const int rr = task / H4, cc = task - rr * H4;
      if (r0 + rr < R) {
        float4 s = red4[rr * NT + cc];
        for (int g = 1; g < RG; ++g) {
          const float4 u = red4[rr * NT + g * H4 + cc];
          s.x += u.x; s.y += u.y; s.z += u.z; s.w += u.w;
        }
        const int row = r0 + rr;
        *reinterpret_cast<float4*>(a.p[a.kg_pair[kg][row / nh]].U + ((int64_t)b * nh + row % nh) * H + 4 * cc) = s;
      }
    }
    __syncthreads();
  }
}

// Weight side (H = 128): 8 waves per workgroup of 32 samples.  Wave (ts, kq)
// owns output tile ts (32 features) over the K half kq; the upper half goes
// through LDS and the lower-half wave adds it (fixed order, deterministic).  Every
// global operand of both phases is loaded at kernel start (one round trip).
constexpr int NTW = 512;
constexpr int WH = 128;   // hidden size of the weight-side kernels

// acc += sum over 8 chunks of a[q] . b[q] (k = 8 q + 4 hf + s)
__device__ __forceinline__ f32x16 mfma8(const float4 (&a)[8], const float4 (&b)[8], f32x16 acc) {
#pragma unroll
  for (int q = 0; q < 8; ++q) acc = mfma4(a[q], b[q], acc);
  return acc;
}

// Finishes a split-K tile (every wave calls it: it holds a barrier).
__device__ __forceinline__ void split_reduce(float (*part)[16][64], f32x16& acc, int kq, int ts, int lane) {
  if (kq == 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) part[ts][r][lane] = acc[r];
  }
  __syncthreads();
  if (kq == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] += part[ts][r][lane];
  }
}

// Forward, weight side: grid (ceil(B / 32), pairs).  C[i = sample][j = feature].
__global__ __launch_bounds__(NTW) void tail_ob_mfma_kernel(const TailArgs a) {
  constexpr int OS = WH + 4;
  __shared__ __attribute__((aligned(16))) float ob_s[32 * OS];
  __shared__ float part[4][16][64];
  const TailPair& P = a.p[blockIdx.y];
  const int s0 = blockIdx.x * 32;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, hf = lane >> 5, c = lane & 31;
  const int ts = w & 3, kq = w >> 2, k0 = kq * 64 + 4 * hf;
  const int nh = a.heads, hd = a.hd, B = a.B;
  const int sa = min(s0 + c, B - 1);   // this lane's A row (rows past B are never stored)
  const int n = ts * 32 + c, hh = (ts * 32) / hd;
  float4 au[8], bv[8], bo[8];
  const float* urow = P.U + ((int64_t)sa * nh + hh) * WH + k0;
  const float* vrow = P.Wv + (int64_t)n * WH + k0;
  const float* orow = P.Wo + (int64_t)n * WH + k0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    au[q] = ld4(urow + 8 * q);
    bv[q] = ld4(vrow + 8 * q);
    bo[q] = ld4(orow + 8 * q);
  }
  float rs[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    // (unconditional, clamped: a row past B is computed but never stored; a guarded load was a
    // branch whose other side waited for every load in flight)
    const int s = s0 + acc_row(r, hf);
    rs[r] = P.r[(int64_t)min(s, B - 1) * nh + hh];
  }
  const float bvn = P.bv[n], bon = P.bo[n];
  __builtin_amdgcn_sched_barrier(0);   // (every load above in flight before the first MFMA)
  // Obar = U W_v^T + r b_v
  f32x16 acc = mfma8(au, bv, zero16());
  split_reduce(part, acc, kq, ts, lane);
  if (kq == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = acc_row(r, hf), s = s0 + i;
      const float o = acc[r] + rs[r] * bvn;
      ob_s[i * OS + n] = o;
      if (s < B) P.Ob[(int64_t)s * WH + n] = o;
    }
  }
  __syncthreads();
  // Abar = Obar W_o^T + b_o
  float4 ao[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) ao[q] = ld4(ob_s + c * OS + k0 + 8 * q);
  acc = mfma8(ao, bo, zero16());
  split_reduce(part, acc, kq, ts, lane);
  if (kq == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int s = s0 + acc_row(r, hf);
      if (s < B) P.Ab[(int64_t)s * WH + n] = acc[r] + bon;
    }
  }
}

// Backward, weight side: grid (ceil(B / 32), pairs).
__global__ __launch_bounds__(NTW) void tail_dob_mfma_kernel(const TailArgs a) {
  constexpr int OS = WH + 4;
  __shared__ __attribute__((aligned(16))) float dob_s[32 * OS];
  __shared__ float part[4][16][64];
  const TailPair& P = a.p[blockIdx.y];
  const int s0 = blockIdx.x * 32;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, hf = lane >> 5, c = lane & 31;
  const int ts = w & 3, kq = w >> 2, k0 = kq * 64 + 4 * hf;
  const int nh = a.heads, hd = a.hd, B = a.B, M = a.M;
  const int sa = min(s0 + c, B - 1);
  const int n = ts * 32 + c;
  // phase 1 operands: A = c_q row (k-contiguous), B = W_o column n (k-strided)
  float4 ac[8], bw[8];
  const float* crow = a.cvec + ((int64_t)sa * M + P.q) * WH + k0;
  const float* wcol = P.Wo + (int64_t)k0 * WH + n;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    ac[q] = ld4(crow + 8 * q);
    bw[q] = make_float4(wcol[(8 * q) * WH], wcol[(8 * q + 1) * WH], wcol[(8 * q + 2) * WH], wcol[(8 * q + 3) * WH]);
  }
  // phase 2 operands (dU tiles tt = w, w + 8 of nh x 4): W_v[h hd + kk][32 kt + c], kk < hd
  const int ntile = nh * (WH / 32);
  float4 bu[2][8];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int tt = w + 8 * u;
    const int hh = tt >> 2, kc = (tt & 3) * 32 + c;
    const float* vcol = P.Wv + (int64_t)(hh * hd + 4 * hf) * WH + kc;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      bu[u][q] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (tt < ntile && 8 * q < hd)
        bu[u][q] = make_float4(vcol[(8 * q) * WH], vcol[(8 * q + 1) * WH], vcol[(8 * q + 2) * WH],
                               vcol[(8 * q + 3) * WH]);
    }
  }
  // dObar = c_q W_o
  f32x16 acc = mfma8(ac, bw, zero16());
  split_reduce(part, acc, kq, ts, lane);
  if (kq == 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = acc_row(r, hf), s = s0 + i;
      dob_s[i * OS + n] = acc[r];
      if (s < B) P.dOb[(int64_t)s * WH + n] = acc[r];
    }
  }
  __syncthreads();
  // dU_h = dObar_h W_v[h hd : (h+1) hd, :]  (K = hd <= 64 here: 8 chunks cover it)
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int tt = w + 8 * u;
    if (tt >= ntile) break;
    const int hh = tt >> 2, kc = (tt & 3) * 32 + c;
    f32x16 acc2 = zero16();
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (8 * q < hd) acc2 = mfma4(ld4(dob_s + c * OS + hh * hd + 4 * hf + 8 * q), bu[u][q], acc2);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int s = s0 + acc_row(r, hf);
      if (s < B) P.dU[((int64_t)s * nh + hh) * WH + kc] = acc2[r];
    }
  }
}

// Backward, P_k side: grid (B, key groups).  C[i = key][j = (pair, head) row].
// The P_k rows of a wave's key tile are loaded before the dU rows are staged.
__global__ __launch_bounds__(NT) void tail_dpbar_mfma_kernel(const TailArgs a) {
  __shared__ __attribute__((aligned(16))) float du_s[KG_ROWS * (TAIL_MAX_H + 4)];
  __shared__ float dr_s[KG_ROWS];
  __shared__ float* rowp[KG_ROWS];
  const int b = blockIdx.x, kg = blockIdx.y;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, hf = lane >> 5, c = lane & 31;
  const int H = a.H, nh = a.heads, hd = a.hd, R = a.kg_cnt[kg] * nh, DS = H + 4;
  const TailPair& P0 = a.p[a.kg_pair[kg][0]];
  const int Lk = P0.Lk;
  const float* pk = P0.Pk + (int64_t)b * Lk * H;
  float4 av[16];
  auto load_a = [&](int mt, int k0) {   // P_k rows of key tile mt, features [k0, k0 + 128)
    const float* arow = pk + (int64_t)min(mt * 32 + c, Lk - 1) * H + k0 + 4 * hf;
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (k0 + 8 * q < H) av[q] = ld4(arow + 8 * q);
  };
  if (w * 32 < Lk) load_a(w, 0);
  const int H4 = H / 4, per = nh * H4;   // dU float4 of one pair for sample b (contiguous)
  if (per % 64 == 0) {
    // wave-uniform pair slot per chunk (see tail_u_kernel): rows past R are zero-filled
    constexpr int U = 4;
    for (int i0 = 0; i0 < KG_ROWS * H4; i0 += U * NT) {
      float4 vv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = min(i0 + u * NT + t, R * H4 - 1);
        const int slot = __builtin_amdgcn_readfirstlane(i / per);
        const int e = i - slot * per;
        vv[u] = ld4(a.p[a.kg_pair[kg][slot]].dU + (int64_t)b * nh * H + 4 * e);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * NT + t;
        if (i < KG_ROWS * H4) {
          const int row = i / H4, c4 = (i - row * H4) * 4;
          // (a native 4-vector store: one ds_write_b128, 8 lanes over 32 consecutive banks; the float4
          // struct's member-wise copy became two ds_write2_b32, 4-way bank-conflicted)
          const float4 q = row < R ? vv[u] : make_float4(0.f, 0.f, 0.f, 0.f);
          reinterpret_cast<f32x4v*>(du_s)[(row * DS + c4) >> 2] = f32x4v{q.x, q.y, q.z, q.w};
        }
      }
    }
  } else {
    for (int i = t; i < KG_ROWS * H4; i += NT) {
      const int row = i / H4, c4 = (i - row * H4) * 4;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row < R) v = ld4(a.p[a.kg_pair[kg][row / nh]].dU + ((int64_t)b * nh + row % nh) * H + c4);
      reinterpret_cast<f32x4v*>(du_s)[(row * DS + c4) >> 2] = f32x4v{v.x, v.y, v.z, v.w};
    }
  }
  if (t < R) rowp[t] = a.p[a.kg_pair[kg][t / nh]].dpbar + ((int64_t)b * nh + t % nh) * Lk;
  for (int row = w; row < R; row += NT / 64) {   // dr_{g,h} = dObar_{g,h} . b_v,h
    const TailPair& P = a.p[a.kg_pair[kg][row / nh]];
    const int hh = row % nh;
    float s = 0.f;
    for (int d = lane; d < hd; d += 64) s += P.dOb[(int64_t)b * H + hh * hd + d] * P.bv[hh * hd + d];
    s = wsum(s);
    if (lane == 0) dr_s[row] = s;
  }
  __syncthreads();
  const float* brow = du_s + c * DS + 4 * hf;
  for (int mt = w; mt * 32 < Lk; mt += NT / 64) {
    f32x16 acc = zero16();
    for (int k0 = 0; k0 < H; k0 += 128) {
      if (mt != w || k0 > 0) load_a(mt, k0);
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (k0 + 8 * q < H) acc = mfma4(av[q], ld4(brow + k0 + 8 * q), acc);
    }
    if (c < R) {
      float* outp = rowp[c];
      const float dr = dr_s[c];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kk = mt * 32 + acc_row(r, hf);
        if (kk < Lk) outp[kk] = acc[r] + dr;
      }
    }
  }
}

// ---------------------------------------------------------------- per sample
// PRE (H = 128, M <= 4, C <= 8): every weight element a thread's GEMVs / dot
// products read (W1 row half, gating row slice, W2 rows) is loaded at kernel
// start, beside the activations: one memory round trip instead of one per stage.
constexpr int PH = 128;

// y[n] = x . W[n] (N = K = 128): thread pair (n = t >> 1, k half t & 1), its 64 weights in wr
__device__ __forceinline__ void gemv128_pre(const float* x, const float4 (&wr)[16], float* y) {
  const int t = threadIdx.x, half = t & 1;
  const float* x0 = x + half * 64;
  float acc = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const float4 xv = *reinterpret_cast<const float4*>(x0 + 4 * q);
    acc += wr[q].x * xv.x + wr[q].y * xv.y + wr[q].z * xv.z + wr[q].w * xv.w;
  }
  const float v = acc + dpp<DPP_XOR1>(acc);
  if (half == 0) y[t >> 1] = v;
}

// y[k] = sum_n x[n] W[n][k] (K = 128): thread (k = t & 127, n half t >> 7) holds its cnt <= NW
// weights W[n0 + i][k] in wc; the halves are summed in order through red
template <int NW>
__device__ __forceinline__ void gemv_nn128_pre(const float* x, const float (&wc)[NW], int n0, int cnt, float* y,
                                               float* red) {
  const int t = threadIdx.x;
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i)
    if (i < cnt) acc += x[n0 + i] * wc[i];
  red[t] = acc;
  __syncthreads();
  if (t < 128) y[t] = red[t] + red[t + 128];
}

// Forward head: pooled_m = mask_m / n_m (mean_L P_m + sum_{g: q(g)=m} Abar_g), gating
// scores, adaptive weights, fused, classifier.  grid (B).
template <bool PRE>
__global__ __launch_bounds__(NT) void tail_head_fwd_kernel(const TailArgs a) {
  __shared__ __attribute__((aligned(16))) float pooled_s[MAXM * TAIL_MAX_H];
  __shared__ __attribute__((aligned(16))) float v1[TAIL_MAX_H], v2[TAIL_MAX_H];
  __shared__ __attribute__((aligned(16))) float4 red4[NT];
  __shared__ float score_s[MAXM], w_s[MAXM];
  const int b = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int M = a.M, H = a.H;
  const int H4 = H >> 2;
  float4 w1r[16];
  float gw[2] = {0.f, 0.f}, w2r[2][2] = {{0.f, 0.f}, {0.f, 0.f}}, b1n = 0.f;
  if constexpr (PRE) {
    const float* wr = a.W1 + (int64_t)(t >> 1) * PH + (t & 1) * 64;
#pragma unroll
    for (int q = 0; q < 16; ++q) w1r[q] = *reinterpret_cast<const float4*>(wr + 4 * q);
    if (wave < M) {
      gw[0] = a.gate_w[wave][lane];
      gw[1] = a.gate_w[wave][lane + 64];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (wave + 4 * u < a.C) {
        w2r[u][0] = a.W2[(int64_t)(wave + 4 * u) * PH + lane];
        w2r[u][1] = a.W2[(int64_t)(wave + 4 * u) * PH + lane + 64];
      }
    if (t < PH) b1n = a.b1[t];
  }
  if constexpr (PRE) {   // (head_pre: every modality has the projection GEMM's column sums)
    // (1 + 2) in one pass: mean_L P_m from the projection GEMM's per-tile column sums
    // (ncol rows per sample), + the attended means of every pair whose query is m,
    // then agg * mask / n_m
    // Every activation this thread's feature n needs (the column sums, the attended
    // means of every pair, the mask row) is loaded before the first store: one round
    // trip (the stores to `pooled` would otherwise order each modality's loads behind
    // the previous modality's stores).  head_pre: M <= 4, so at most 12 pairs.
    constexpr int PM = 4, PG = 12;
    const int n = t;   // H == PH <= NT
    if (n < H) {
      float pcs[PM], ab[PG], mk[PM];
#pragma unroll
      for (int m = 0; m < PM; ++m) {
        pcs[m] = 0.f;
        mk[m] = 0.f;
        if (m < M) {
          const int nc = a.ncol[m];
          const float* pc = a.Pcol[m] + (int64_t)b * nc * H + n;
          for (int c = 0; c < nc; ++c) pcs[m] += pc[(int64_t)c * H];
          mk[m] = a.mask[(int64_t)b * M + m];
        }
      }
#pragma unroll
      for (int g = 0; g < PG; ++g) ab[g] = g < a.npairs ? a.p[g].Ab[(int64_t)b * H + n] : 0.f;
#pragma unroll
      for (int m = 0; m < PM; ++m) {
        if (m >= M) break;
        const float f = a.inv_cnt[m] * mk[m], il = 1.f / (float)a.L[m];
        float v = pcs[m] * il;
#pragma unroll
        for (int g = 0; g < PG; ++g)
          if (g < a.npairs && a.p[g].q == m) v += ab[g];
        v *= f;
        pooled_s[m * H + n] = v;
        a.pooled[(int64_t)b * M * H + m * H + n] = v;
      }
    }
  } else {
    // (1) mean over L of P_m (the modality's own entry of the aggregation list)
    for (int m = 0; m < M; ++m) {
      const int L = a.L[m];
      if (a.Pcol[m]) {
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
  }
  __syncthreads();
  // (3) gating scores (nn.Linear(H, 1), src/fusion.py:316-321,452-461), adaptive weights
  if constexpr (PRE) {
    if (wave < M) {
      float s = pooled_s[wave * PH + lane] * gw[0] + pooled_s[wave * PH + lane + 64] * gw[1];
      s = wsum(s);
      if (lane == 0) score_s[wave] = s + a.gate_b[wave][0];
    }
  } else {
    for (int m = wave; m < M; m += NT / 64) {
      float s = 0.f;
      for (int j = lane; j < H; j += 64) s += pooled_s[m * H + j] * a.gate_w[m][j];
      s = wsum(s);
      if (lane == 0) score_s[m] = s + a.gate_b[m][0];
    }
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
  if constexpr (PRE) gemv128_pre(v1, w1r, v2);
  else gemv_nt_s<1>(v1, 0, 1 << 30, 0, a.W1, H, H, v2, 0);
  __syncthreads();
  const float p = a.drop_p;
  const bool drop = p > 0.f && a.rng != nullptr;
  RngSnap rs{0, 0};
  if (drop) rs = *a.rng;
  const float inv_keep = p < 1.f ? 1.f / (1.f - p) : 0.f;
  for (int n = t; n < H; n += NT) {
    float x = fmaxf(v2[n] + (PRE ? b1n : a.b1[n]), 0.f);
    if (drop) x = keep1(rs, a.drop_site, (uint64_t)b * H + n, p) ? x * inv_keep : 0.f;
    v2[n] = x;
    a.h1[(int64_t)b * H + n] = x;
  }
  __syncthreads();
  if constexpr (PRE) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = wave + 4 * u;
      if (c < a.C) {
        float s = v2[lane] * w2r[u][0] + v2[lane + 64] * w2r[u][1];
        s = wsum(s);
        if (lane == 0) a.logits[(int64_t)b * a.C + c] = s + a.b2[c];
      }
    }
  } else {
    for (int c = wave; c < a.C; c += NT / 64) {
      float s = 0.f;
      for (int j = lane; j < H; j += 64) s += v2[j] * a.W2[(int64_t)c * H + j];
      s = wsum(s);
      if (lane == 0) a.logits[(int64_t)b * a.C + c] = s + a.b2[c];
    }
  }
}

// Backward head: dz1 = ReLU'/Dropout'(dlogits W2), dfused = dz1 W1, head backward
// (dscore, cvec = dpooled * mask / n).  grid (B).
template <bool PRE>
__global__ __launch_bounds__(NT) void tail_head_bwd_kernel(const TailArgs a) {
  __shared__ __attribute__((aligned(16))) float pooled_s[MAXM * TAIL_MAX_H];
  __shared__ __attribute__((aligned(16))) float v1[TAIL_MAX_H], v2[TAIL_MAX_H], dl_s[256];
  __shared__ float red[NT];
  __shared__ float dw_s[MAXM], dscore_s[MAXM];
  const int b = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int M = a.M, H = a.H, C = a.C;
  // PRE: thread (k = t & 127, n half t >> 7) columns of W2 (rows [n0, n0 + cnt)) and
  // W1 (rows [64 rh, 64 rh + 64)); the gating weights of its cvec elements
  const int kc = t & 127, rh = t >> 7;
  const int c0 = rh ? (C >> 1) : 0, ccnt = rh ? C - (C >> 1) : (C >> 1);
  float w2c[4], w1c[64], gwc[2];
  if constexpr (PRE) {
#pragma unroll
    for (int i = 0; i < 4; ++i) w2c[i] = i < ccnt ? a.W2[(int64_t)(c0 + i) * PH + kc] : 0.f;
#pragma unroll
    for (int i = 0; i < 64; ++i) w1c[i] = a.W1[(int64_t)(rh * 64 + i) * PH + kc];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = t + u * NT;
      gwc[u] = i < M * PH ? a.gate_w[i / PH][i % PH] : 0.f;
    }
  }
  for (int c = t; c < C; c += NT) dl_s[c] = a.dlogits[(int64_t)b * C + c];
  for (int i = t; i < M * H; i += NT) pooled_s[i] = a.pooled[(int64_t)b * M * H + i];
  __syncthreads();
  // the saved h1 is post-dropout, so h1 > 0 marks kept, active units (gscale = 1/(1-p))
  if constexpr (PRE) gemv_nn128_pre<4>(dl_s, w2c, c0, ccnt, v1, red);
  else gemv_nn_s<1>(dl_s, 0, a.W2, C, H, v1, 0, red);
  __syncthreads();
  for (int n = t; n < H; n += NT) {
    const float z = a.h1[(int64_t)b * H + n] > 0.f ? v1[n] * a.gscale : 0.f;
    v1[n] = z;
    a.dz1[(int64_t)b * H + n] = z;
  }
  __syncthreads();
  if constexpr (PRE) gemv_nn128_pre<64>(v1, w1c, rh * 64, 64, v2, red);
  else gemv_nn_s<1>(v1, 0, a.W1, H, H, v2, 0, red);
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
  if constexpr (PRE) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = t + u * NT;
      if (i < M * PH) {
        const int m = i / PH, j = i - m * PH;
        const float wm = a.weights[(int64_t)b * M + m];
        const float f = a.mask[(int64_t)b * M + m] * a.inv_cnt[m];
        a.cvec[(int64_t)b * M * PH + i] = (wm * v2[j] + dscore_s[m] * gwc[u]) * f;
      }
    }
  } else {
    for (int i = t; i < M * H; i += NT) {
      const int m = i / H, j = i - m * H;
      const float wm = a.weights[(int64_t)b * M + m];
      const float f = a.mask[(int64_t)b * M + m] * a.inv_cnt[m];
      a.cvec[(int64_t)b * M * H + i] = (wm * v2[j] + dscore_s[m] * a.gate_w[m][j]) * f;
    }
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

// Prefetching head kernels (MMF_TAIL_GEMV=1 also selects the plain ones, for A/B)
static bool head_pre(const TailArgs& a) {
  static const bool gemv = getenv("MMF_TAIL_GEMV") != nullptr;
  bool allcol = true;
  for (int m = 0; m < a.M; ++m) allcol = allcol && a.Pcol[m] != nullptr;
  return !gemv && allcol && a.H == PH && a.M <= 4 && a.C <= 8;
}

// Groups the pairs by key modality into `m` and reports whether the MFMA pair
// tail applies (MMF_TAIL_GEMV=1 forces the per-sample GEMV kernels, for A/B).
static bool tail_mfma_groups(TailArgs& m) {
  static const bool gemv = getenv("MMF_TAIL_GEMV") != nullptr;
  if (gemv || m.H != WH || (m.hd != 32 && m.hd != 64)) return false;
  int mod_of[8];
  m.nkg = 0;
  for (int g = 0; g < m.npairs; ++g) {
    int i = 0;
    while (i < m.nkg && mod_of[i] != m.p[g].k) ++i;
    if (i == m.nkg) {
      if (m.nkg == 8) return false;
      mod_of[m.nkg] = m.p[g].k;
      m.kg_cnt[m.nkg++] = 0;
    }
    m.kg_pair[i][m.kg_cnt[i]++] = g;
  }
  for (int i = 0; i < m.nkg; ++i)
    if (m.kg_cnt[i] * m.heads > KG_ROWS) return false;
  return true;
}

hipError_t launch_tail_fwd(const TailArgs& a, hipStream_t st) {
  if (!tail_supported(a.M, a.H, a.C, a.heads, a.hd, a.npairs)) return hipErrorInvalidValue;
  for (int g = 0; g < a.npairs; ++g)
    if (a.p[g].Lk > 128) return hipErrorInvalidValue;
  const double B = a.B, H = a.H;
  TailArgs m = a;
  if (a.npairs && tail_mfma_groups(m)) {
    double fl = 0.0, by = 0.0;   // U = pbar P_k: P_k read once per key group
    for (int i = 0; i < m.nkg; ++i) {
      const double lk = m.p[m.kg_pair[i][0]].Lk, rows = (double)m.kg_cnt[i] * m.heads;
      fl += 2.0 * B * rows * lk * H;
      by += 4.0 * B * (lk * H + rows * (lk + H + 1));
    }
    {
      ProfLaunch prof_(st, "tail_u_kernel", fl, by);
      mmf_launch(tail_u_kernel, dim3(a.B, m.nkg), dim3(NT), 0, st, m);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    {
      // Obar = U W_v^T (+ r b_v), Abar = Obar W_o^T + b_o: weights read once per 32 samples
      ProfLaunch prof_(st, "tail_ob_mfma_kernel", 4.0 * B * H * H * a.npairs,
                       4.0 * a.npairs * (2 * H * H * ((a.B + 31) / 32) + B * (a.heads * H + 2 * H)));
      mmf_launch(tail_ob_mfma_kernel, dim3((a.B + 31) / 32, a.npairs), dim3(NTW), 0, st, m);
    }
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  } else if (a.npairs) {
    // per pair: Vbar = U W_v^T (+ r b_v), Obar = Vbar W_o^T + b_o; weights read once
    ProfLaunch prof_(st, "tail_pair_fwd_kernel", 4.0 * B * H * H * a.npairs,
                     4.0 * a.npairs * (2 * H * H + B * (a.heads * H + 2 * H)));
    // at H = 256 the forward's weight reads (2 x 256 KB per pair) outweigh the lost
    // parallelism: 2 samples per workgroup (C4: 42.2 -> 35.7 us; the backward stays at 1:
    // 45.3 -> 56.6 us at 2)
    const int S = getenv("MMF_TAIL_S") ? tail_samples() : (a.H >= 256 ? 2 : 1);
    if (S == 4) mmf_launch(tail_pair_fwd_kernel<4>, dim3((a.B + 3) / 4, a.npairs), dim3(NT), 0, st, a);
    else if (S == 2) mmf_launch(tail_pair_fwd_kernel<2>, dim3((a.B + 1) / 2, a.npairs), dim3(NT), 0, st, a);
    else mmf_launch(tail_pair_fwd_kernel<1>, dim3(a.B, a.npairs), dim3(NT), 0, st, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  // pooling, gating, adaptive weights, weighted sum, classifier: on 16-sample tiles where they
  // apply (l1.hip seq_head_kernel; a training step's loss and head backward in the same launch)
  if (seq_head_ok(a)) return launch_seq_head_fwd(a, st);
  if (a.labels) return hipErrorInvalidValue;   // (the caller checks seq_head_ok first)
  ProfLaunch prof_(st, head_pre(a) ? "tail_head_fwd_kernel<true>" : "tail_head_fwd_kernel<false>", 2.0 * B * H * (H + a.C) + 4.0 * a.M * B * H,
                   4.0 * (H * (H + a.C) + B * (a.M * H + a.C)));
  if (head_pre(a)) mmf_launch(tail_head_fwd_kernel<true>, dim3(a.B), dim3(NT), 0, st, a);
  else mmf_launch(tail_head_fwd_kernel<false>, dim3(a.B), dim3(NT), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_tail_bwd(const TailArgs& a, hipStream_t st) {
  if (!tail_supported(a.M, a.H, a.C, a.heads, a.hd, a.npairs)) return hipErrorInvalidValue;
  const double B = a.B, H = a.H;
  hipError_t e = hipSuccess;
  if (a.head_done) {
    // (the training step's head launch ran the head backward)
  } else if (seq_head_ok(a)) {
    e = launch_seq_head_bwd(a, st);
  } else {
    ProfLaunch prof_(st, head_pre(a) ? "tail_head_bwd_kernel<true>" : "tail_head_bwd_kernel<false>", 2.0 * B * H * (H + a.C) + 4.0 * a.M * B * H,
                     4.0 * (H * (H + a.C) + B * (a.M * H + a.C)));
    if (head_pre(a)) mmf_launch(tail_head_bwd_kernel<true>, dim3(a.B), dim3(NT), 0, st, a);
    else mmf_launch(tail_head_bwd_kernel<false>, dim3(a.B), dim3(NT), 0, st, a);
    e = hipGetLastError();
  }
  if (e != hipSuccess || !a.npairs) return e;
  TailArgs m = a;
  if (tail_mfma_groups(m)) {
    {
      // dObar = c_q W_o, dU_h = dObar_h W_v,h: weights read once per 32 samples
      ProfLaunch prof_(st, "tail_dob_mfma_kernel", 4.0 * B * H * H * a.npairs,
                       4.0 * a.npairs * (2 * H * H * ((a.B + 31) / 32) + B * (a.heads * H + 2 * H)));
      mmf_launch(tail_dob_mfma_kernel, dim3((a.B + 31) / 32, a.npairs), dim3(NTW), 0, st, m);
    }
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    double fl = 0.0, by = 0.0;   // dpbar = P_k dU + dr: P_k read once per key group
    for (int i = 0; i < m.nkg; ++i) {
      const double lk = m.p[m.kg_pair[i][0]].Lk, rows = (double)m.kg_cnt[i] * m.heads;
      fl += 2.0 * B * rows * lk * H;
      by += 4.0 * B * (lk * H + rows * (lk + H) + m.kg_cnt[i] * H);
    }
    ProfLaunch prof_(st, "tail_dpbar_mfma_kernel", fl, by);
    mmf_launch(tail_dpbar_mfma_kernel, dim3(a.B, m.nkg), dim3(NT), 0, st, m);
    return hipGetLastError();
  }
  {
    ProfLaunch prof_(st, "tail_pair_bwd_kernel", 4.0 * B * H * H * a.npairs,
                     4.0 * a.npairs * (2 * H * H + B * (a.heads * H + 2 * H)));
    const int S = tail_samples();
    if (S == 4) mmf_launch(tail_pair_bwd_kernel<4>, dim3((a.B + 3) / 4, a.npairs), dim3(NT), 0, st, a);
    else if (S == 2) mmf_launch(tail_pair_bwd_kernel<2>, dim3((a.B + 1) / 2, a.npairs), dim3(NT), 0, st, a);
    else mmf_launch(tail_pair_bwd_kernel<1>, dim3(a.B, a.npairs), dim3(NT), 0, st, a);
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
