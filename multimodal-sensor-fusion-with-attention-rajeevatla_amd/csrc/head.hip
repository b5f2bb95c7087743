// Fusion head kernels: per-modality aggregation + L mean-pool, gating scores,
// masked-softmax adaptive weights, weighted sum (forward) and their backward;
// plus the small training-step kernels (RNG snapshot, cross-entropy with label
// smoothing, AdamW).
//
// Reference: aggregation src/fusion.py:406-408; compute_adaptive_weights
// src/fusion.py:429-479; fused representation src/fusion.py:413-418;
// CrossEntropyLoss(label_smoothing) src/train.py:185-186,310.
// One workgroup per sample: nothing here mixes samples, so the data-parallel
// split over the batch needs no exchange.
#include <cstring>

#include "mmf_device.h"

namespace mmf {

namespace {

constexpr int NT = 256;
constexpr int HEAD_MAX_H = 1024;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Masked softmax over modalities + renormalisation / fallback, exactly as
// src/fusion.py:462-478 (scores of mask<=0 modalities are -inf; an all -inf row
// is NaN -> 0 -> fallback mask/(sum+1e-8) or uniform 1/M).
// Returns sw (> 0 iff the softmax branch was taken) and fills sm (softmax after
// nan_to_num), w (final weights).
__device__ float adaptive_fwd(int M, const float* score, const float* mask, float* sm, float* w) {
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
    sm[m] = (mx == -INFINITY) ? 0.f : sm[m] / z;   // nan_to_num of an all -inf row
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

__global__ __launch_bounds__(NT) void head_fwd_kernel(const HeadArgs a) {
  __shared__ __attribute__((aligned(16))) float pooled_s[8 * HEAD_MAX_H];
  __shared__ __attribute__((aligned(16))) float4 red4[NT];
  __shared__ float score_s[8], w_s[8], part_s[4][8];
  const int b = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int M = a.M, H = a.H;
  const int NCG = H / 4;
  const int RG = NT / NCG;   // host guarantees 4 <= H <= 1024, H % 4 == 0
  const int cg = t % NCG, rg = t / NCG;
  const bool active = rg < RG;

  for (int m = 0; m < M; ++m) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (active) {
      for (int si = 0; si < a.nsrc; ++si) {
        if (a.src_mod[si] != m) continue;
        const int L = a.src_L[si];
        const float sc = a.src_scale[si];
        const float* base = a.src[si] + (int64_t)b * L * H + 4 * cg;
        float4 part = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int r = rg; r < L; r += RG) {
          const float4 v = *reinterpret_cast<const float4*>(base + (int64_t)r * H);
          part.x += v.x; part.y += v.y; part.z += v.z; part.w += v.w;
        }
        acc.x += part.x * sc; acc.y += part.y * sc; acc.z += part.z * sc; acc.w += part.w * sc;
      }
    }
    red4[t] = acc;
    __syncthreads();
    if (t < NCG) {
      float4 s = red4[t];
      for (int g = 1; g < RG; ++g) {
        const float4 v = red4[g * NCG + t];
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
      const float f = a.inv_cnt[m] * (a.scale_by_mask ? a.mask[(int64_t)b * M + m] : 1.f);
      *reinterpret_cast<float4*>(&pooled_s[m * H + 4 * t]) = make_float4(s.x * f, s.y * f, s.z * f, s.w * f);
    }
    __syncthreads();
  }
  // gating scores (nn.Linear(H, 1) per modality, src/fusion.py:316-321,452-461)
  for (int m = wave; m < M; m += 4) {
    float s = 0.f;
    for (int j = lane; j < H; j += 64) s += pooled_s[m * H + j] * a.gate_w[m][j];
    s = wave_sum(s);
    if (lane == 0) score_s[m] = s + a.gate_b[m][0];
  }
  __syncthreads();
  if (t == 0) {
    float msk[8], sm[8], w[8];
    for (int m = 0; m < M; ++m) msk[m] = a.mask[(int64_t)b * M + m];
    adaptive_fwd(M, score_s, msk, sm, w);
    for (int m = 0; m < M; ++m) {
      w_s[m] = w[m];
      a.scores[(int64_t)b * M + m] = score_s[m];
      a.weights[(int64_t)b * M + m] = w[m];
      if (a.weights_out) a.weights_out[(int64_t)b * M + m] = w[m];
    }
  }
  __syncthreads();
  (void)part_s;
  for (int j = t; j < H; j += NT) {
    float f = 0.f;
    for (int m = 0; m < M; ++m) {
      const float v = pooled_s[m * H + j];
      f += v * w_s[m];
      a.pooled[((int64_t)b * M + m) * H + j] = v;
    }
    a.fused[(int64_t)b * H + j] = f;
  }
}

__global__ __launch_bounds__(NT) void head_bwd_kernel(const HeadArgs a) {
  __shared__ float dw_s[8], dscore_s[8];
  const int b = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int M = a.M, H = a.H;
  const float* df = a.dfused ? a.dfused + (int64_t)b * H : nullptr;
  const float* pooled = a.pooled + (int64_t)b * M * H;
  // dL/dw_m = dfused . pooled_m   (fused = sum_m w_m pooled_m), or given directly
  // (compute_adaptive_weights backward: dfused is null, dweights (B, M) the upstream grad)
  for (int m = wave; m < M; m += 4) {
    float s = 0.f;
    if (df) {
      for (int j = lane; j < H; j += 64) s += df[j] * pooled[m * H + j];
      s = wave_sum(s);
    } else {
      s = a.dweights[(int64_t)b * M + m];
    }
    if (lane == 0) dw_s[m] = s;
  }
  __syncthreads();
  if (t == 0) {
    float msk[8], sc[8], sm[8], w[8];
    for (int m = 0; m < M; ++m) {
      msk[m] = a.mask[(int64_t)b * M + m];
      sc[m] = a.scores[(int64_t)b * M + m];
    }
    const float sw = adaptive_fwd(M, sc, msk, sm, w);
    float ds[8];
    for (int m = 0; m < M; ++m) ds[m] = 0.f;
    if (sw > 0.f) {
      // w = wm / (sw + eps), wm = sm * mask  ->  d wm_i = dw_i/S - sum_j dw_j wm_j / S^2
      const float S = sw + 1e-8f;
      float dot = 0.f;
      for (int m = 0; m < M; ++m) dot += dw_s[m] * sm[m] * msk[m];
      float dsm[8], sdot = 0.f;
      for (int m = 0; m < M; ++m) {
        dsm[m] = (dw_s[m] / S - dot / (S * S)) * msk[m];
        sdot += sm[m] * dsm[m];
      }
      // softmax backward; masked_fill(mask<=0) zeroes the masked entries
      for (int m = 0; m < M; ++m) ds[m] = msk[m] > 0.f ? sm[m] * (dsm[m] - sdot) : 0.f;
    }
    for (int m = 0; m < M; ++m) {
      dscore_s[m] = ds[m];
      a.dscore[(int64_t)b * M + m] = ds[m];
    }
  }
  __syncthreads();
  for (int m = 0; m < M; ++m) {
    const float wm = a.weights[(int64_t)b * M + m];
    const float f = (a.scale_by_mask ? a.mask[(int64_t)b * M + m] : 1.f) * a.inv_cnt[m];
    const float dsm = dscore_s[m];
    const float* gw = a.gate_w[m];
    for (int j = t; j < H; j += NT) {
      const float dp = (df ? wm * df[j] : 0.f) + dsm * gw[j];
      a.cvec[((int64_t)b * M + m) * H + j] = dp * f;
    }
  }
}

struct GateWArgs {
  int32_t B, M, H;
  const float* dscore; const float* pooled;
  float* dgw[8]; float* dgb[8];
};

__global__ __launch_bounds__(NT) void gate_wgrad_kernel(const GateWArgs a) {
  const int idx = blockIdx.x * NT + threadIdx.x;
  const int per = a.H + 1;
  if (idx >= a.M * per) return;
  const int m = idx / per, j = idx % per;
  float s = 0.f;
  if (j < a.H) {
    for (int b = 0; b < a.B; ++b)
      s += a.dscore[(int64_t)b * a.M + m] * a.pooled[((int64_t)b * a.M + m) * a.H + j];
    a.dgw[m][j] = s;
  } else {
    for (int b = 0; b < a.B; ++b) s += a.dscore[(int64_t)b * a.M + m];
    a.dgb[m][0] = s;
  }
}

__global__ void rng_snapshot_kernel(uint64_t* state, RngSnap* snap) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    snap->seed = state[0];
    snap->offset = state[1];
    state[1] = state[1] + 1;
  }
}

// nn.CrossEntropyLoss(label_smoothing=eps), reduction='mean':
// loss_i = -(1-eps) log p_{y_i} - eps/C sum_c log p_c ; dlogits = (p - ((1-eps) onehot + eps/C)) / B
constexpr int64_t CE_IGNORE_INDEX = -100;   // torch.nn.CrossEntropyLoss(ignore_index=-100)

__global__ __launch_bounds__(NT) void cross_entropy_kernel(int B, int C, const float* logits,
                                                           const int64_t* labels, float eps,
                                                           float gscale, float* loss, float* dlogits) {
  __shared__ float red[NT];
  __shared__ int cnt[NT / 64];
  const int t = threadIdx.x;
  // torch's nn.CrossEntropyLoss defaults: rows labelled ignore_index (-100) add nothing and get a
  // zero gradient, the mean runs over the other rows (every row valid: the count is B, so the same
  // bits as a plain mean over B).  A label outside [0, C) (torch raises) makes the loss NaN and is
  // never used as an index.
  int nv = 0;
  for (int i = t; i < B; i += NT) nv += labels[i] != CE_IGNORE_INDEX;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) nv += __shfl_xor(nv, off);
  if ((t & 63) == 0) cnt[t >> 6] = nv;
  __syncthreads();
  const float nvalid = (float)((cnt[0] + cnt[1]) + (cnt[2] + cnt[3]));
  float acc = 0.f;
  for (int i = t; i < B; i += NT) {
    const float* z = logits + (int64_t)i * C;
    const int64_t yl = labels[i];
    float* d = dlogits + (int64_t)i * C;
    if (yl == CE_IGNORE_INDEX) {
      for (int c = 0; c < C; ++c) d[c] = 0.f;
      continue;
    }
    const bool bad = yl < 0 || yl >= C;
    const int y = bad ? 0 : (int)yl;
    float mx = -INFINITY;
    for (int c = 0; c < C; ++c) mx = fmaxf(mx, z[c]);
    float se = 0.f, sz = 0.f;
    for (int c = 0; c < C; ++c) { se += __expf(z[c] - mx); sz += z[c]; }
    const float lse = mx + __logf(se);
    // (an explicit fma: l1.hip loss_rows forms the same value bit for bit, whatever contraction
    // each context's compiler would choose)
    acc += bad ? NAN : __builtin_fmaf(1.f - eps, lse - z[y], eps * (lse - sz / (float)C));
    for (int c = 0; c < C; ++c) {
      const float pc = __expf(z[c] - lse);
      const float tgt = (c == y ? (1.f - eps) : 0.f) + eps / (float)C;
      d[c] = (pc - tgt) / nvalid * gscale;
    }
  }
  red[t] = acc;
  __syncthreads();
  for (int s = NT / 2; s > 0; s >>= 1) {
    if (t < s) red[t] += red[t + s];
    __syncthreads();
  }
  if (t == 0) loss[0] = red[0] / nvalid;
}

// Global gradient norm for clipping (torch.nn.utils.clip_grad_norm_, norm_type 2, as
// Lightning's gradient_clip_val applies it: src/train.py:416-430, config/base.yaml:74).
// Pass 1: CLIP_BLOCKS fixed partial sums of squares (grid-stride, fixed order);
// pass 2: one workgroup adds them in a fixed tree order -> deterministic.
constexpr int CLIP_BLOCKS = 256;
// The partials buffer holds CLIP_SLOTS = 4 CLIP_BLOCKS floats: grad_sumsq_kernel writes slots
// [0, CLIP_BLOCKS) and zeroes the rest; a producer with more pieces (the L = 1 weight-gradient launch,
// one slot per output tile) fills up to all of them.  Thread t of the clip reduction adds slots t,
// t + 256, t + 512, t + 768 in that order (in double: the zero slots add exact zeros).
constexpr int CLIP_SLOTS = 4 * CLIP_BLOCKS;
// (the L = 1 weight-gradient launch fills and zeroes CLIP_PARTIAL_SLOTS of them: the same count)
static_assert(CLIP_SLOTS == CLIP_PARTIAL_SLOTS, "clip partial slots out of sync with l1.hip's producer");

__global__ __launch_bounds__(NT) void grad_sumsq_kernel(int64_t n, const float* __restrict__ g,
                                                        float* __restrict__ partial, int64_t* step_incr) {
  __shared__ float red[NT / 64];
  const int t = threadIdx.x;
  // fused clip + AdamW: the step counter advances here, one launch before the update reads it
  if (step_incr && blockIdx.x == 0 && t == 0) *step_incr = *step_incr + 1;
  float acc = 0.f;
  const int64_t n4 = n / 4;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (int64_t i = (int64_t)blockIdx.x * NT + t; i < n4; i += (int64_t)CLIP_BLOCKS * NT) {
    const float4 v = g4[i];
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  if (blockIdx.x == 0)
    for (int64_t i = 4 * n4 + t; i < n; i += NT) acc += g[i] * g[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);   // fixed order per wave
  if ((t & 63) == 0) red[t >> 6] = acc;
  __syncthreads();
  if (t == 0) partial[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
  if (t >= 1 && t < CLIP_SLOTS / CLIP_BLOCKS) partial[blockIdx.x + t * CLIP_BLOCKS] = 0.f;
}

// total_norm = gscale * sqrt(sum); coef = min(1, max_norm / (total_norm + 1e-6)) (1 when max_norm <= 0;
// 0 when total_norm is not finite).
// Every thread of the block gets the same norm / coef: one partial per thread, a fixed
// xor-butterfly per wave, the four wave sums in a fixed order (the same bits in every block).
static_assert(CLIP_BLOCKS == NT, "one clip partial per thread");
constexpr int CLIP_PER_THREAD = CLIP_SLOTS / CLIP_BLOCKS;
// (from the thread's partials already in registers: clip_adamw_kernel issues their loads first)
__device__ __forceinline__ void clip_norm_coef_vals(const float (&pp)[CLIP_PER_THREAD], float gscale, float max_norm,
                                                    double* red, float& norm, float& coef) {
  const int t = threadIdx.x;
  double acc = (double)pp[0];
#pragma unroll
  for (int r = 1; r < CLIP_PER_THREAD; ++r) acc += (double)pp[r];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if ((t & 63) == 0) red[t >> 6] = acc;
  // LDS-only barrier (no vmcnt drain: clip_adamw_kernel's AdamW operand loads stay in flight)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  const double sum = (red[0] + red[1]) + (red[2] + red[3]);
  norm = (float)(sqrt(sum) * (double)gscale);
  coef = 1.f;
  if (max_norm > 0.f) coef = fminf(1.f, max_norm / (norm + 1e-6f));
  // a non-finite norm applies a zero gradient whether clipping is on or not: it is how a train
  // step whose bounded wait gave up (l1.hip: one +inf partial) keeps its incomplete gradient out of
  // the update (with clipping on, torch's max_norm / inf is 0 as well; fminf would keep 1 for NaN)
  if (!(norm <= 3.402823466e38f)) coef = 0.f;
}
__device__ __forceinline__ void clip_norm_coef(const float* __restrict__ partial, float gscale, float max_norm,
                                               double* red, float& norm, float& coef) {
  float pp[CLIP_PER_THREAD];
#pragma unroll
  for (int r = 0; r < CLIP_PER_THREAD; ++r) pp[r] = partial[threadIdx.x + r * CLIP_BLOCKS];
  clip_norm_coef_vals(pp, gscale, max_norm, red, norm, coef);
}

// One AdamW element update (shared by adamw_kernel and clip_adamw_kernel: the same
// float operations, so the fused and two-call paths agree bit for bit).  Contraction off: every
// product and sum rounds on its own, so the backend's fuse-or-not choice (which depends on the
// surrounding code, e.g. packed math in one caller) cannot make two callers differ.
__device__ __forceinline__ void adamw_elem(float& p, float g, float& m, float& v, float gs, float lr, float wd,
                                           float b1, float b2, float eps, float step_size, float bc2s) {
#pragma clang fp contract(off)
  const float gi = g * gs;
  float pi = p * (1.f - lr * wd);
  const float mi = b1 * m + (1.f - b1) * gi;
  const float vi = b2 * v + (1.f - b2) * gi * gi;
  m = mi;
  v = vi;
  pi -= step_size * mi / (sqrtf(vi) / bc2s + eps);
  p = pi;
}

// The update over [0, n): float4 slots grid-stride when every pointer is 16-B aligned
// (vec), then the scalar remainder; otherwise scalar throughout.
__device__ __forceinline__ void adamw_range(int64_t n, float* __restrict__ p, const float* __restrict__ g,
                                            float* __restrict__ m, float* __restrict__ v, bool vec, float gs,
                                            float lr, float wd, float b1, float b2, float eps, float step_size,
                                            float bc2s, int skip = 0) {
  const int64_t tid = (int64_t)blockIdx.x * NT + threadIdx.x, nth = (int64_t)gridDim.x * NT;
  int64_t done = 0;
  if (vec) {
    const int64_t n4 = n / 4;
    for (int64_t i = tid + skip * nth; i < n4; i += nth) {
      float4 pv = reinterpret_cast<float4*>(p)[i];
      const float4 gv = reinterpret_cast<const float4*>(g)[i];
      float4 mv = reinterpret_cast<float4*>(m)[i];
      float4 vv = reinterpret_cast<float4*>(v)[i];
      adamw_elem(pv.x, gv.x, mv.x, vv.x, gs, lr, wd, b1, b2, eps, step_size, bc2s);
      adamw_elem(pv.y, gv.y, mv.y, vv.y, gs, lr, wd, b1, b2, eps, step_size, bc2s);
      adamw_elem(pv.z, gv.z, mv.z, vv.z, gs, lr, wd, b1, b2, eps, step_size, bc2s);
      adamw_elem(pv.w, gv.w, mv.w, vv.w, gs, lr, wd, b1, b2, eps, step_size, bc2s);
      reinterpret_cast<float4*>(p)[i] = pv;
      reinterpret_cast<float4*>(m)[i] = mv;
      reinterpret_cast<float4*>(v)[i] = vv;
    }
    done = 4 * n4;
  }
  for (int64_t i = done + tid; i < n; i += nth) {
    float pi = p[i], mi = m[i], vi = v[i];
    adamw_elem(pi, g[i], mi, vi, gs, lr, wd, b1, b2, eps, step_size, bc2s);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}

__global__ __launch_bounds__(NT) void clip_coef_kernel(const float* __restrict__ partial, float gscale,
                                                       float max_norm, float* norm_out, float* coef_out) {
  __shared__ double red[NT / 64];
  float norm, coef;
  clip_norm_coef(partial, gscale, max_norm, red, norm, coef);
  if (threadIdx.x == 0) {
    if (norm_out) norm_out[0] = norm;
    coef_out[0] = coef;
  }
}

// torch.optim.AdamW (amsgrad=False, maximize=False): decoupled weight decay.
// lr_dev (optional) replaces lr and coef_dev (optional) multiplies the gradient
// scale, both read on the device so a captured step follows a scheduler / clipping.
__global__ __launch_bounds__(NT) void adamw_kernel(int64_t n, float* __restrict__ p,
                                                   const float* __restrict__ g, float* __restrict__ m,
                                                   float* __restrict__ v, const int64_t* step, float lr,
                                                   float b1, float b2, float eps, float wd, float gscale,
                                                   const float* __restrict__ lr_dev,
                                                   const float* __restrict__ coef_dev, int vec) {
  if (lr_dev) lr = lr_dev[0];
  if (coef_dev) gscale *= coef_dev[0];
  const double st = (double)(*step + 1);
  const float bc1 = (float)(1.0 - pow((double)b1, st));
  const float bc2s = (float)sqrt(1.0 - pow((double)b2, st));
  const float step_size = lr / bc1;
  adamw_range(n, p, g, m, v, vec != 0, gscale, lr, wd, b1, b2, eps, step_size, bc2s);
}

// (PF: the thread's first two float4 slots are loaded ahead of the clip reduction and the bias
// corrections, whose dependent chain -- partials -> double sums -> barrier -> pow -- then runs
// under the loads' latency; clamped addresses: unconditional loads, guarded stores.  Issue order is
// vmcnt order, so the partials go first and the reduction waits for them only.)
template <bool PF>
__device__ __forceinline__ void clip_adamw_body(int64_t n, float* __restrict__ p, const float* __restrict__ g,
                                                float* __restrict__ m, float* __restrict__ v, const int64_t* step,
                                                const float* __restrict__ lr_dev, float b1, float b2, float eps,
                                                float wd, float gscale, const float* __restrict__ partial,
                                                float max_norm, float* norm_out, float* coef_out, bool vec) {
  __shared__ double red[NT / 64];
  const int64_t tid = (int64_t)blockIdx.x * NT + threadIdx.x, nth = (int64_t)gridDim.x * NT;
  const int64_t n4 = n / 4;
  float pp[CLIP_PER_THREAD];
#pragma unroll
  for (int r = 0; r < CLIP_PER_THREAD; ++r) pp[r] = partial[threadIdx.x + r * CLIP_BLOCKS];
  const float lr = lr_dev[0];
  const double st = (double)(*step);
  float4 pv[2], gv[2], mv[2], vv[2];
  if constexpr (PF) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int64_t i = min(tid + s * nth, n4 - 1);
      pv[s] = reinterpret_cast<const float4*>(p)[i];
      gv[s] = reinterpret_cast<const float4*>(g)[i];
      mv[s] = reinterpret_cast<const float4*>(m)[i];
      vv[s] = reinterpret_cast<const float4*>(v)[i];
    }
  }
  float norm, coef;
  clip_norm_coef_vals(pp, gscale, max_norm, red, norm, coef);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (norm_out) norm_out[0] = norm;
    if (coef_out) coef_out[0] = coef;
  }
  const float bc1 = (float)(1.0 - pow((double)b1, st));
  const float bc2s = (float)sqrt(1.0 - pow((double)b2, st));
  const float step_size = lr / bc1;
  const float gs = gscale * coef;
  if constexpr (PF) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int64_t i = tid + s * nth;
      if (i >= n4) continue;
      adamw_elem(pv[s].x, gv[s].x, mv[s].x, vv[s].x, gs, lr, wd, b1, b2, eps, step_size, bc2s);
      adamw_elem(pv[s].y, gv[s].y, mv[s].y, vv[s].y, gs, lr, wd, b1, b2, eps, step_size, bc2s);
      adamw_elem(pv[s].z, gv[s].z, mv[s].z, vv[s].z, gs, lr, wd, b1, b2, eps, step_size, bc2s);
      adamw_elem(pv[s].w, gv[s].w, mv[s].w, vv[s].w, gs, lr, wd, b1, b2, eps, step_size, bc2s);
      reinterpret_cast<float4*>(p)[i] = pv[s];
      reinterpret_cast<float4*>(m)[i] = mv[s];
      reinterpret_cast<float4*>(v)[i] = vv[s];
    }
  }
  // the remaining float4 slots (all of them without PF) and the scalar tail
  adamw_range(n, p, g, m, v, vec, gs, lr, wd, b1, b2, eps, step_size, bc2s, PF ? 2 : 0);
}

// Clip + AdamW in one launch after grad_sumsq_kernel (which advanced *step): every
// block re-reduces the CLIP_BLOCKS partials itself (the same bits as clip_coef_kernel),
// block 0 publishes norm / coef.  Same update as adamw_kernel at step *step.
__global__ __launch_bounds__(NT) void clip_adamw_kernel(int64_t n, float* __restrict__ p,
                                                        const float* __restrict__ g, float* __restrict__ m,
                                                        float* __restrict__ v, const int64_t* step,
                                                        const float* __restrict__ lr_dev, float b1, float b2,
                                                        float eps, float wd, float gscale,
                                                        const float* __restrict__ partial, float max_norm,
                                                        float* norm_out, float* coef_out, int vec) {
  if (vec && n >= 4)
    clip_adamw_body<true>(n, p, g, m, v, step, lr_dev, b1, b2, eps, wd, gscale, partial, max_norm, norm_out,
                          coef_out, true);
  else
    clip_adamw_body<false>(n, p, g, m, v, step, lr_dev, b1, b2, eps, wd, gscale, partial, max_norm, norm_out,
                           coef_out, vec != 0);
}

__global__ void rng_advance_kernel(uint64_t* state) {
  if (threadIdx.x == 0 && blockIdx.x == 0) state[1] = state[1] + 1;
}

__global__ void step_incr_kernel(int64_t* step) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *step = *step + 1;
}

}  // namespace

hipError_t launch_head_fwd(const HeadArgs& a, hipStream_t st) {
  if (a.H % 4 != 0 || a.H > HEAD_MAX_H || a.H < 4 || a.M > 8) return hipErrorInvalidValue;
  ProfLaunch prof_(st, "head_fwd_kernel", 0.0, 0.0);
  mmf_launch(head_fwd_kernel, dim3(a.B), dim3(NT), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_head_bwd(const HeadArgs& a, hipStream_t st) {
  if (a.M > 8) return hipErrorInvalidValue;
  ProfLaunch prof_(st, "head_bwd_kernel", 0.0, 0.0);
  mmf_launch(head_bwd_kernel, dim3(a.B), dim3(NT), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_gate_wgrad(int B, int M, int H, const float* dscore, const float* pooled,
                             float* const* dgw, float* const* dgb, hipStream_t st) {
  GateWArgs a;
  memset(&a, 0, sizeof(a));
  a.B = B; a.M = M; a.H = H; a.dscore = dscore; a.pooled = pooled;
  for (int m = 0; m < M; ++m) { a.dgw[m] = dgw[m]; a.dgb[m] = dgb[m]; }
  const int n = M * (H + 1);
  ProfLaunch prof_(st, "gate_wgrad_kernel", 2.0 * B * M * H, 4.0 * B * M * (H + 1));
  mmf_launch(gate_wgrad_kernel, dim3((n + NT - 1) / NT), dim3(NT), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_rng_snapshot(const uint64_t* state, RngSnap* snap, hipStream_t st) {
  ProfLaunch prof_(st, "rng_snapshot_kernel", 0.0, 32.0);
  mmf_launch(rng_snapshot_kernel, dim3(1), dim3(64), 0, st, const_cast<uint64_t*>(state), snap);
  return hipGetLastError();
}

hipError_t launch_rng_advance(uint64_t* state, hipStream_t st) {
  ProfLaunch prof_(st, "rng_advance_kernel", 0.0, 16.0);
  mmf_launch(rng_advance_kernel, dim3(1), dim3(64), 0, st, state);
  return hipGetLastError();
}

hipError_t launch_cross_entropy(int B, int C, const float* logits, const int64_t* labels,
                                float smoothing, float grad_scale, float* loss, float* dlogits,
                                hipStream_t st) {
  ProfLaunch prof_(st, "cross_entropy_kernel", 0.0, 8.0 * B * C + 8.0 * B);
  mmf_launch(cross_entropy_kernel, dim3(1), dim3(NT), 0, st, B, C, logits, labels, smoothing,
                     grad_scale, loss, dlogits);
  return hipGetLastError();
}

size_t grad_clip_workspace_bytes() { return CLIP_SLOTS * sizeof(float); }

hipError_t launch_grad_clip_coef(int64_t n, const float* g, float gscale, float max_norm, float* norm_out,
                                 float* coef_out, float* partial, hipStream_t st) {
  {
    ProfLaunch prof_(st, "grad_sumsq_kernel", 2.0 * n, 4.0 * n);
    mmf_launch(grad_sumsq_kernel, dim3(CLIP_BLOCKS), dim3(NT), 0, st, n, g, partial, (int64_t*)nullptr);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  ProfLaunch prof_(st, "clip_coef_kernel", 0.0, 4.0 * CLIP_BLOCKS);
  mmf_launch(clip_coef_kernel, dim3(1), dim3(NT), 0, st, (const float*)partial, gscale, max_norm, norm_out,
                     coef_out);
  return hipGetLastError();
}

// float4 path when every operand is 16-B aligned; about two float4 slots per thread
// (every block re-reduces the clip partials, so fewer, fuller blocks)
static int adamw_vec(const float* p, const float* g, const float* m, const float* v) {
  return ((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0) ? 1 : 0;
}
static int64_t adamw_blocks(int64_t n, int vec) {
  const int64_t per_block = (int64_t)NT * (vec ? 8 : 2);
  int64_t blocks = (n + per_block - 1) / per_block;
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  return blocks;
}

// dst += src over a flat fp32 buffer (gradient accumulation over micro-batches, Lightning's
// accumulate_grad_batches, config/base.yaml:75): float4 body, scalar tail
__global__ __launch_bounds__(256) void grad_accum_kernel(int64_t n, const float* __restrict__ src,
                                                          float* __restrict__ dst) {
  const int64_t n4 = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 a = reinterpret_cast<const float4*>(src)[i];
    float4 b = reinterpret_cast<float4*>(dst)[i];
    b.x += a.x; b.y += a.y; b.z += a.z; b.w += a.w;
    reinterpret_cast<float4*>(dst)[i] = b;
  }
  for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    dst[i] += src[i];
}

hipError_t launch_grad_accum(int64_t n, const float* src, float* dst, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((n / 4 + 255) / 256 + 1, 4 * (int64_t)device_cu_count());
  ProfLaunch prof_(st, "grad_accum_kernel", (double)n, 12.0 * (double)n);
  mmf_launch(grad_accum_kernel, dim3((unsigned)blocks), dim3(256), 0, st, n, src, dst);
  return hipGetLastError();
}

hipError_t launch_adamw(int64_t n, float* p, const float* g, float* m, float* v, int64_t* step,
                        float lr, float b1, float b2, float eps, float wd, float gscale,
                        hipStream_t st, const float* lr_dev, const float* coef_dev) {
  const int vec = adamw_vec(p, g, m, v);
  const int64_t blocks = adamw_blocks(n, vec);
  ProfLaunch prof_(st, "adamw_kernel", 0.0, 28.0 * n);   // p m v read+write, g read
  mmf_launch(adamw_kernel, dim3((unsigned)blocks), dim3(NT), 0, st, n, p, g, m, v, step, lr, b1,
                     b2, eps, wd, gscale, lr_dev, coef_dev, vec);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  mmf_launch(step_incr_kernel, dim3(1), dim3(64), 0, st, step);
  return hipGetLastError();
}

// The squared-norm partials of a flat gradient (and the step counter advanced) for a later
// launch_clip_adamw_apply
hipError_t launch_grad_sumsq(int64_t n, const float* g, float* partial, int64_t* step, hipStream_t st) {
  ProfLaunch prof_(st, "grad_sumsq_kernel", 2.0 * n, 4.0 * n);
  mmf_launch(grad_sumsq_kernel, dim3(CLIP_BLOCKS), dim3(NT), 0, st, n, g, partial, step);
  return hipGetLastError();
}

// clip + AdamW from partials a producer already wrote (grad_sumsq_kernel, or the L = 1 weight-gradient
// launch), the step counter already advanced: the one launch of launch_clip_adamw's two
hipError_t launch_clip_adamw_apply(int64_t n, float* p, const float* g, float* m, float* v, const int64_t* step,
                                   const float* lr_dev, float b1, float b2, float eps, float wd, float gscale,
                                   float max_norm, float* norm_out, float* coef_out, const float* partial,
                                   hipStream_t st) {
  const int vec = adamw_vec(p, g, m, v);
  const int64_t blocks = adamw_blocks(n, vec);
  ProfLaunch prof_(st, "clip_adamw_kernel", 0.0, 28.0 * n);
  mmf_launch(clip_adamw_kernel, dim3((unsigned)blocks), dim3(NT), 0, st, n, p, g, m, v, step, lr_dev, b1, b2, eps,
             wd, gscale, partial, max_norm, norm_out, coef_out, vec);
  return hipGetLastError();
}

hipError_t launch_clip_adamw(int64_t n, float* p, const float* g, float* m, float* v, int64_t* step,
                             const float* lr_dev, float b1, float b2, float eps, float wd, float gscale,
                             float max_norm, float* norm_out, float* coef_out, float* partial, hipStream_t st) {
  {
    ProfLaunch prof_(st, "grad_sumsq_kernel", 2.0 * n, 4.0 * n);
    mmf_launch(grad_sumsq_kernel, dim3(CLIP_BLOCKS), dim3(NT), 0, st, n, g, partial, step);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int vec = adamw_vec(p, g, m, v);
  const int64_t blocks = adamw_blocks(n, vec);
  ProfLaunch prof_(st, "clip_adamw_kernel", 0.0, 28.0 * n);
  mmf_launch(clip_adamw_kernel, dim3((unsigned)blocks), dim3(NT), 0, st, n, p, g, m, v, (const int64_t*)step,
                     lr_dev, b1, b2, eps, wd, gscale, (const float*)partial, max_norm, norm_out, coef_out, vec);
  return hipGetLastError();
}

}  // namespace mmf
