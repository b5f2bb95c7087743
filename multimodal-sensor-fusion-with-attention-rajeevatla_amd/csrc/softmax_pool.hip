// Masked softmax weighting kernels beside the fused path:
//
//  * FrameEncoder.attention_pool (src/encoders.py:313-336): per sample,
//    s_t = x_t . u + c over the frames, -inf where mask == 0, softmax over t,
//    nan_to_num (an all-masked row gives weights 0), pooled = sum_t w_t x_t.
//    One workgroup per sample; the frame rows are read once for the scores and
//    once for the weighted sum (the second pass hits L2), coalesced along D.
//    Backward: g = dpooled, a_t = x_t . g, ds_t = w_t (a_t - sum w a),
//    dx_t = w_t g + ds_t u; du, dc are reduced over the batch from per-sample
//    partial rows by a fixed-order column sum (deterministic).
//
//  * LateFusion weighting (src/fusion.py:228-245): base = softmax(weight_logits),
//    w = base * mask, normalised by (sum + 1e-8) where the sum > 0 else 1/M,
//    fused = sum_m w_m logits_m.  Backward through the same branches
//    (torch.where passes the gradient of the selected branch only).
//
// All fp32; every entry point only enqueues on the caller's stream.
#include <cmath>

#include "capi_util.h"

namespace mmf {

namespace {

constexpr int NT = 256;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// block-wide reductions over NT threads (4 waves) through 4 LDS slots
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  return fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

struct PoolFwdArgs {
  int B, T, D;
  const float* x;      // (B, T, D)
  const float* u;      // (D)   attention.weight
  const float* c;      // (1)   attention.bias
  const float* mask;   // (B, T) or null
  float* pooled;       // (B, D)
  float* weights;      // (B, T)
};

// scores in LDS (T <= MAX_T)
constexpr int MAX_T = 8192;

__global__ __launch_bounds__(NT) void attn_pool_frames_fwd(PoolFwdArgs a) {
  __shared__ float sc[MAX_T];
  __shared__ float red[4];
  const int b = blockIdx.x;
  const int t0 = threadIdx.x, lane = t0 & 63, w = t0 >> 6;
  const float* xb = a.x + (int64_t)b * a.T * a.D;
  const float cb = a.c ? a.c[0] : 0.f;
  // scores: one wave per frame, lanes along D
  for (int t = w; t < a.T; t += 4) {
    const float* row = xb + (int64_t)t * a.D;
    float s = 0.f;
    for (int d = lane; d < a.D; d += 64) s = fmaf(row[d], a.u[d], s);
    s = wave_sum(s) + cb;
    if (lane == 0) {
      const bool keep = !a.mask || a.mask[(int64_t)b * a.T + t] != 0.f;
      sc[t] = keep ? s : -INFINITY;
    }
  }
  __syncthreads();
  float mx = -INFINITY;
  for (int t = t0; t < a.T; t += NT) mx = fmaxf(mx, sc[t]);
  mx = block_max(mx, red);
  float sum = 0.f;
  for (int t = t0; t < a.T; t += NT) {
    const float e = mx == -INFINITY ? 0.f : __expf(sc[t] - mx);
    sc[t] = e;
    sum += e;
  }
  sum = block_sum(sum, red);
  // all keys masked: softmax is NaN in the reference -> nan_to_num -> 0
  const float inv = sum > 0.f ? 1.f / sum : 0.f;
  for (int t = t0; t < a.T; t += NT) {
    const float wt = sc[t] * inv;
    sc[t] = wt;
    a.weights[(int64_t)b * a.T + t] = wt;
  }
  __syncthreads();
  for (int d = t0; d < a.D; d += NT) {
    float acc = 0.f;
    for (int t = 0; t < a.T; ++t) acc = fmaf(sc[t], xb[(int64_t)t * a.D + d], acc);
    a.pooled[(int64_t)b * a.D + d] = acc;
  }
}

struct PoolBwdArgs {
  int B, T, D;
  const float* x;        // (B, T, D)
  const float* u;        // (D)
  const float* weights;  // (B, T)
  const float* g;        // dpooled (B, D)
  float* dx;             // (B, T, D)
  float* part;           // (B, D + 1) per-sample du | dc partials
};

__global__ __launch_bounds__(NT) void attn_pool_frames_bwd(PoolBwdArgs a) {
  __shared__ float ds[MAX_T];
  __shared__ float red[4];
  const int b = blockIdx.x;
  const int t0 = threadIdx.x, lane = t0 & 63, w = t0 >> 6;
  const float* xb = a.x + (int64_t)b * a.T * a.D;
  const float* gb = a.g + (int64_t)b * a.D;
  const float* wb = a.weights + (int64_t)b * a.T;
  for (int t = w; t < a.T; t += 4) {
    const float* row = xb + (int64_t)t * a.D;
    float s = 0.f;
    for (int d = lane; d < a.D; d += 64) s = fmaf(row[d], gb[d], s);
    s = wave_sum(s);
    if (lane == 0) ds[t] = s;   // a_t = x_t . g
  }
  __syncthreads();
  float wa = 0.f;
  for (int t = t0; t < a.T; t += NT) wa = fmaf(wb[t], ds[t], wa);
  wa = block_sum(wa, red);
  float dcs = 0.f;
  for (int t = t0; t < a.T; t += NT) {
    const float v = wb[t] * (ds[t] - wa);
    ds[t] = v;
    dcs += v;
  }
  dcs = block_sum(dcs, red);   // also orders the ds[] writes before the reads below
  for (int d = t0; d < a.D; d += NT) {
    const float gd = gb[d], ud = a.u[d];
    float du = 0.f;
    for (int t = 0; t < a.T; ++t) {
      const int64_t o = (int64_t)t * a.D + d;
      a.dx[(int64_t)b * a.T * a.D + o] = fmaf(wb[t], gd, ds[t] * ud);
      du = fmaf(ds[t], xb[o], du);
    }
    a.part[(int64_t)b * (a.D + 1) + d] = du;
  }
  if (t0 == 0) a.part[(int64_t)b * (a.D + 1) + a.D] = dcs;
}

// out[j] = sum_b part[b][j], j < n (fixed order over b)
__global__ __launch_bounds__(NT) void column_sum(const float* part, int rows, int n, float* out0, int n0,
                                                 float* out1) {
  const int j = blockIdx.x * NT + threadIdx.x;
  if (j >= n) return;
  float s = 0.f;
  for (int r = 0; r < rows; ++r) s += part[(int64_t)r * n + j];
  if (j < n0) out0[j] = s;
  else if (out1) out1[j - n0] = s;
}

struct LateArgs {
  int B, M, C;
  const float* logits;   // (B, M, C) stacked per-modality logits
  const float* wl;       // (M) weight_logits
  const float* mask;     // (B, M) or null (ones)
  float* fused;          // (B, C)
  float* weights;        // (B, M) normalised weights
  // backward
  const float* dfused;   // (B, C)
  float* dlogits;        // (B, M, C)
  float* part;           // (B, M) per-sample d base
};

constexpr int LATE_MAX_M = 64;

// base = softmax(weight_logits) computed per block (M is small)
__device__ __forceinline__ void late_base(const LateArgs& a, float* base) {
  if (threadIdx.x == 0) {
    float mx = -INFINITY;
    for (int m = 0; m < a.M; ++m) mx = fmaxf(mx, a.wl[m]);
    float s = 0.f;
    for (int m = 0; m < a.M; ++m) {
      base[m] = __expf(a.wl[m] - mx);
      s += base[m];
    }
    for (int m = 0; m < a.M; ++m) base[m] /= s;
  }
}

__global__ __launch_bounds__(NT) void late_weights_fwd(LateArgs a) {
  __shared__ float base[LATE_MAX_M];
  __shared__ float nw[LATE_MAX_M];
  const int b = blockIdx.x;
  late_base(a, base);
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int m = 0; m < a.M; ++m) {
      const float mk = a.mask ? a.mask[(int64_t)b * a.M + m] : 1.f;
      nw[m] = base[m] * mk;
      s += nw[m];
    }
    for (int m = 0; m < a.M; ++m) {
      nw[m] = s > 0.f ? nw[m] / (s + 1e-8f) : 1.f / (float)a.M;
      a.weights[(int64_t)b * a.M + m] = nw[m];
    }
  }
  __syncthreads();
  for (int cidx = threadIdx.x; cidx < a.C; cidx += NT) {
    float acc = 0.f;
    for (int m = 0; m < a.M; ++m) acc += a.logits[((int64_t)b * a.M + m) * a.C + cidx] * nw[m];
    a.fused[(int64_t)b * a.C + cidx] = acc;
  }
}

__global__ __launch_bounds__(NT) void late_weights_bwd(LateArgs a) {
  __shared__ float base[LATE_MAX_M];
  __shared__ float dnw[LATE_MAX_M];
  __shared__ float red[4];
  const int b = blockIdx.x;
  late_base(a, base);
  __syncthreads();
  const float* nwb = a.weights + (int64_t)b * a.M;
  const float* gf = a.dfused + (int64_t)b * a.C;
  for (int m = 0; m < a.M; ++m) {
    float acc = 0.f;
    for (int cidx = threadIdx.x; cidx < a.C; cidx += NT) {
      const int64_t o = ((int64_t)b * a.M + m) * a.C + cidx;
      a.dlogits[o] = gf[cidx] * nwb[m];
      acc = fmaf(gf[cidx], a.logits[o], acc);
    }
    acc = block_sum(acc, red);
    if (threadIdx.x == 0) dnw[m] = acc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int m = 0; m < a.M; ++m) s += base[m] * (a.mask ? a.mask[(int64_t)b * a.M + m] : 1.f);
    // nw = w / (s + eps) where s > 0: dw_j = dnw_j / (s+eps) - sum_m dnw_m w_m / (s+eps)^2;
    // the uniform branch carries no gradient.  d base_j = dw_j * mask_j.
    float dot = 0.f;
    for (int m = 0; m < a.M; ++m) dot += dnw[m] * base[m] * (a.mask ? a.mask[(int64_t)b * a.M + m] : 1.f);
    const float se = s + 1e-8f;
    for (int m = 0; m < a.M; ++m) {
      const float mk = a.mask ? a.mask[(int64_t)b * a.M + m] : 1.f;
      const float dw = s > 0.f ? dnw[m] / se - dot / (se * se) : 0.f;
      a.part[(int64_t)b * a.M + m] = dw * mk;
    }
  }
}

// d weight_logits = softmax Jacobian^T (sum_b d base); one lane per modality
__global__ void late_logits_grad(const float* wl, const float* part, int B, int M, float* dwl) {
  __shared__ float base[LATE_MAX_M], db[LATE_MAX_M];
  const int m = threadIdx.x;
  if (m < M) {
    float mx = -INFINITY;
    for (int i = 0; i < M; ++i) mx = fmaxf(mx, wl[i]);
    float s = 0.f;
    for (int i = 0; i < M; ++i) s += __expf(wl[i] - mx);
    base[m] = __expf(wl[m] - mx) / s;
    float acc = 0.f;
    for (int r = 0; r < B; ++r) acc += part[(int64_t)r * M + m];
    db[m] = acc;
  }
  __syncthreads();
  if (m < M) {
    float dot = 0.f;
    for (int i = 0; i < M; ++i) dot += base[i] * db[i];
    dwl[m] = base[m] * (db[m] - dot);
  }
}

}  // namespace

}  // namespace mmf

using namespace mmf;

extern "C" {

size_t mmf_attention_pool_workspace_bytes(int32_t batch, int32_t dim) {
  return (size_t)batch * (dim + 1) * sizeof(float) + 256;
}

int mmf_attention_pool_forward(int32_t batch, int32_t frames, int32_t dim, const float* x, const float* score_w,
                               const float* score_b, const float* mask, float* pooled, float* weights,
                               void* stream) {
  if (batch < 0 || frames < 1 || dim < 1) return fail(MMF_EINVAL, "attention_pool: bad shape");
  if (frames > MAX_T) return fail(MMF_ELIMIT, "attention_pool: %d frames > %d", frames, MAX_T);
  if (batch == 0) return MMF_OK;
  hipStream_t st = (hipStream_t)stream;
  PoolFwdArgs a{batch, frames, dim, x, score_w, score_b, mask, pooled, weights};
  ProfLaunch prof_(st, "attn_pool_frames_fwd", 4.0 * batch * frames * dim, 4.0 * batch * frames * dim);
  mmf_launch(attn_pool_frames_fwd, dim3(batch), dim3(NT), 0, st, a);
  HIP_TRY(hipGetLastError());
  return MMF_OK;
}

int mmf_attention_pool_backward(int32_t batch, int32_t frames, int32_t dim, const float* x, const float* score_w,
                                const float* weights, const float* dpooled, float* dx, float* dscore_w,
                                float* dscore_b, void* workspace, void* stream) {
  if (batch < 0 || frames < 1 || dim < 1) return fail(MMF_EINVAL, "attention_pool: bad shape");
  if (frames > MAX_T) return fail(MMF_ELIMIT, "attention_pool: %d frames > %d", frames, MAX_T);
  hipStream_t st = (hipStream_t)stream;
  if (batch == 0) {
    float* zp[2] = {dscore_w, dscore_b};
    const int64_t zn[2] = {dim, 1};
    HIP_TRY(launch_zero_fill(zp, zn, 2, st));
    return MMF_OK;
  }
  float* part = (float*)workspace;
  PoolBwdArgs a{batch, frames, dim, x, score_w, weights, dpooled, dx, part};
  {
    ProfLaunch prof_(st, "attn_pool_frames_bwd", 6.0 * batch * frames * dim, 8.0 * batch * frames * dim);
    mmf_launch(attn_pool_frames_bwd, dim3(batch), dim3(NT), 0, st, a);
    HIP_TRY(hipGetLastError());
  }
  const int n = dim + 1;
  ProfLaunch prof_(st, "column_sum", (double)batch * n, 4.0 * batch * n);
  mmf_launch(column_sum, dim3((n + NT - 1) / NT), dim3(NT), 0, st, (const float*)part, batch, n, dscore_w,
                     dim, dscore_b);
  HIP_TRY(hipGetLastError());
  return MMF_OK;
}

size_t mmf_late_fusion_workspace_bytes(int32_t batch, int32_t num_modalities) {
  return (size_t)batch * num_modalities * sizeof(float) + 256;
}

int mmf_late_fusion_forward(int32_t batch, int32_t num_modalities, int32_t num_classes, const float* logits,
                            const float* weight_logits, const float* mask, float* fused, float* weights,
                            void* stream) {
  if (batch < 0 || num_modalities < 1 || num_classes < 1) return fail(MMF_EINVAL, "late fusion: bad shape");
  if (num_modalities > LATE_MAX_M) return fail(MMF_ELIMIT, "late fusion: more than %d modalities", LATE_MAX_M);
  if (batch == 0) return MMF_OK;
  hipStream_t st = (hipStream_t)stream;
  LateArgs a;
  memset(&a, 0, sizeof(a));
  a.B = batch; a.M = num_modalities; a.C = num_classes;
  a.logits = logits; a.wl = weight_logits; a.mask = mask; a.fused = fused; a.weights = weights;
  ProfLaunch prof_(st, "late_weights_fwd", 2.0 * batch * num_modalities * num_classes,
                   4.0 * batch * num_modalities * (num_classes + 2));
  mmf_launch(late_weights_fwd, dim3(batch), dim3(NT), 0, st, a);
  HIP_TRY(hipGetLastError());
  return MMF_OK;
}

int mmf_late_fusion_backward(int32_t batch, int32_t num_modalities, int32_t num_classes, const float* logits,
                             const float* weight_logits, const float* mask, const float* weights,
                             const float* dfused, float* dlogits, float* dweight_logits, void* workspace,
                             void* stream) {
  if (batch < 0 || num_modalities < 1 || num_classes < 1) return fail(MMF_EINVAL, "late fusion: bad shape");
  if (num_modalities > LATE_MAX_M) return fail(MMF_ELIMIT, "late fusion: more than %d modalities", LATE_MAX_M);
  hipStream_t st = (hipStream_t)stream;
  if (batch == 0) {
    float* zp[1] = {dweight_logits};
    const int64_t zn[1] = {num_modalities};
    HIP_TRY(launch_zero_fill(zp, zn, 1, st));
    return MMF_OK;
  }
  LateArgs a;
  memset(&a, 0, sizeof(a));
  a.B = batch; a.M = num_modalities; a.C = num_classes;
  a.logits = logits; a.wl = weight_logits; a.mask = mask; a.weights = (float*)weights;
  a.dfused = dfused; a.dlogits = dlogits; a.part = (float*)workspace;
  {
    ProfLaunch prof_(st, "late_weights_bwd", 4.0 * batch * num_modalities * num_classes,
                     4.0 * batch * num_modalities * (2 * num_classes + 2));
    mmf_launch(late_weights_bwd, dim3(batch), dim3(NT), 0, st, a);
    HIP_TRY(hipGetLastError());
  }
  ProfLaunch prof_(st, "late_logits_grad", 2.0 * batch * num_modalities, 4.0 * batch * num_modalities);
  mmf_launch(late_logits_grad, dim3(1), dim3(64), 0, st, weight_logits, (const float*)a.part, batch,
                     num_modalities, dweight_logits);
  HIP_TRY(hipGetLastError());
  return MMF_OK;
}

}  // extern "C"
