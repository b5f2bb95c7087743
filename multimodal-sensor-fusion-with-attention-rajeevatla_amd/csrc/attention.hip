// Flash-style cross-modal attention on CDNA4 fp32 matrix cores.
//
// Semantics (src/attention.py:118-139): scores = (q k^T) * hd^-0.5; keys with
// mask == 0 get -inf; softmax; a row whose keys are all masked is NaN in the
// reference and nan_to_num'd to 0 (src/attention.py:127-129), so here it
// produces P = 0, O = 0, LSE = -inf; Dropout(p) on the probabilities; attn @ v.
//
// Layout: one workgroup = 4 waves = 128 query rows (forward / dQ) or 128 keys
// (dK/dV) of one (pair, sample, head).  K/V (or Q/dO) chunks are staged in LDS
// with a 16-B row pad (conflict-free ds_read_b128 on the row-wise MFMA operand).
//
// MFMA orientation (v_mfma_f32_32x32x2_f32; C/D: col = lane&31, rows in regs):
//  * forward / dQ: S^T = K Q^T, so each lane owns ONE query row (col) and 16 of
//    the tile's 32 keys (regs; the other 16 sit in lane^32).  Row max / row sum
//    are in-register + one xor-32 shuffle.  The S^T accumulator registers are
//    directly the B operand of O^T += V^T P^T and dQ^T += K^T dS^T (no LDS trip).
//  * dK/dV: S = Q K^T (key on the lane); the accumulators are directly the A
//    operand of dV += P'^T dO and dK += dS^T Q.
// The head dimension is zero-padded to HDP (32 or 64); the MFMA contraction
// order over d is permuted (lane half h owns d in [h*HDP/2, (h+1)*HDP/2)) so
// each lane's operand is contiguous.
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "mmf_device.h"

namespace mmf {

namespace {

constexpr int NT = 256;


// Diagnostic stamps (make stamps / stampsf): the fused backward's phases, or with
// MMF_STAMPS_FWD the pooled forward's, into the TU's one stamp buffer.
#if defined(MMF_STAMPS) && defined(MMF_STAMPS_FWD)
#define FSTAMP(i) MMF_STAMP(i)
#define FSTAMP_RT(i) MMF_STAMP_RT(i)
#define FSTAMP_ID() MMF_STAMP_ID()
#define BSTAMP(i)
#define BSTAMP_RT(i)
#define BSTAMP_ID()
#else
#define FSTAMP(i)
#define FSTAMP_RT(i)
#define FSTAMP_ID()
#define BSTAMP(i) MMF_STAMP(i)
#define BSTAMP_RT(i) MMF_STAMP_RT(i)
#define BSTAMP_ID() MMF_STAMP_ID()
#endif

__device__ __forceinline__ float kmask_val(const AttnPair& P, int b, int key) {
  if (P.kmask_mode == 1) return P.kmask[(int64_t)b * P.kmask_ld];
  if (P.kmask_mode == 2) return P.kmask[(int64_t)b * P.kmask_ld + key];
  return 1.f;
}

// Load rows [r0, r0+ROWS) of a (B, L, ld) tensor's head slice into LDS [ROWS][LS]
// (cols >= hd and rows >= L are zero).
// With 16-B rows (vec) every global load of the image is issued before the
// first LDS write: written as one loop, the compiler put an s_waitcnt vmcnt(0)
// in front of each ds_write (a full HBM round trip per 4 KB, 8 in a row for the
// K and Q images of the fused backward: a third of its workgroup lifetime).
template <int ROWS, int HDP, int LS, bool BATCHED = true>
__device__ __forceinline__ void load_rows(float* S, const float* base, int L, int ld, int r0, int hd,
                                          bool vec) {
  constexpr int C4 = HDP / 4;
  if (BATCHED && vec) {
    static_assert((ROWS * C4) % NT == 0, "whole float4 slots per thread");
    constexpr int PER = ROWS * C4 / NT;
    constexpr int BATCH = PER < 4 ? PER : 4;   // 16 VGPRs of loads in flight (the long-key kernels
                                               // call this inside their chunk loops, beside live sums)
    static_assert(PER % BATCH == 0, "whole batches");
#pragma unroll
    for (int i0 = 0; i0 < PER; i0 += BATCH) {
      float4 v[BATCH];
#pragma unroll
      for (int i = 0; i < BATCH; ++i) {
        const int idx = threadIdx.x + (i0 + i) * NT;
        const int r = idx / C4, c4 = (idx % C4) * 4;
        const int row = r0 + r;
        v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (row < L && c4 < hd) v[i] = *reinterpret_cast<const float4*>(base + (int64_t)row * ld + c4);
      }
#pragma unroll
      for (int i = 0; i < BATCH; ++i) {
        const int idx = threadIdx.x + (i0 + i) * NT;
        *reinterpret_cast<float4*>(&S[(idx / C4) * LS + (idx % C4) * 4]) = v[i];
      }
    }
    return;
  }
  for (int idx = threadIdx.x; idx < ROWS * C4; idx += NT) {
    const int r = idx / C4, c4 = (idx % C4) * 4;
    const int row = r0 + r;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < L) {
      const float* p = base + (int64_t)row * ld + c4;
      if (vec && c4 + 3 < hd) {
        v = *reinterpret_cast<const float4*>(p);
      } else {
        if (c4 + 0 < hd) v.x = p[0];
        if (c4 + 1 < hd) v.y = p[1];
        if (c4 + 2 < hd) v.z = p[2];
        if (c4 + 3 < hd) v.w = p[3];
      }
    }
    *reinterpret_cast<float4*>(&S[r * LS + c4]) = v;
  }
}

template <int HALF>
__device__ __forceinline__ void load_frag(float* f, const float* row, int dbase, int hd, bool valid) {
#pragma unroll
  for (int s = 0; s < HALF; ++s) {
    const int d = dbase + s;
    f[s] = (valid && d < hd) ? row[d] : 0.f;
  }
}

// acc += A_lds_row(lane) . f   over the HALF-long contraction (row-wise LDS operand)
// (BF: bf16 MFMA operands, see mfma_k16 in mmf_device.h; eight k-steps per chain)
template <int HALF, int BF = 0>
__device__ __forceinline__ f32x16 dot_rows(const float* lds_row, const float* f, f32x16 acc) {
  static_assert(HALF % 8 == 0, "k chains of 8");
#pragma unroll
  for (int s8 = 0; s8 < HALF; s8 += 8) {
    const float4 a0 = *reinterpret_cast<const float4*>(lds_row + s8);
    const float4 a1 = *reinterpret_cast<const float4*>(lds_row + s8 + 4);
    const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    float bv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) bv[j] = f[s8 + j];
    acc = mfma_k16<BF>(av, bv, acc);
  }
  return acc;
}

// ACC += sum over the 16 accumulator-register steps r of AEXPR(r) x BEXPR(r)
// (one fp32 k-step per r), issued as two chains of eight (mfma_k16<BF>).
#define MMF_CHAIN16(ACC, AEXPR, BEXPR)                                  \
  _Pragma("unroll") for (int g_ = 0; g_ < 2; ++g_) {                    \
    float av_[8], bv_[8];                                               \
    _Pragma("unroll") for (int j_ = 0; j_ < 8; ++j_) {                  \
      const int r = 8 * g_ + j_;                                        \
      av_[j_] = (AEXPR);                                                \
      bv_[j_] = (BEXPR);                                                \
    }                                                                   \
    ACC = mfma_k16<BF>(av_, bv_, ACC);                                  \
  }

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.f;
  return z;
}

// ---------------------------------------------------------------------------
// Forward (MODE 0) and attention-probability output (MODE 1, needs LSE).
// ---------------------------------------------------------------------------
template <int HDP, int MODE, int BF>
__global__ __launch_bounds__(NT) void attn_fwd_kernel(const AttnArgs A) {
  constexpr int KC = HDP == 32 ? 128 : 64;
  constexpr int LS = HDP + 4;
  constexpr int HALF = HDP / 2;
  constexpr int NDT = HDP / 32;
  __shared__ __attribute__((aligned(16))) float Ks[KC * LS];
  __shared__ __attribute__((aligned(16))) float Vs[(MODE == 0 ? KC : 1) * LS];

  const AttnPair& P = A.p[blockIdx.y];
  const int qblocks = (P.Lq + 127) / 128;
  int bid = blockIdx.x;
  if (bid >= A.B * A.heads * qblocks) return;
  const int qb = bid % qblocks;
  bid /= qblocks;
  const int head = bid % A.heads, b = bid / A.heads;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, h = lane >> 5, c = lane & 31;
  const int hd = A.hd, col0 = head * hd;
  const int q = qb * 128 + w * 32 + c;
  const bool qvalid = q < P.Lq;
  const bool wave_active = qb * 128 + w * 32 < P.Lq;
  const int64_t rowidx = ((int64_t)b * A.heads + head) * P.Lq + q;   // (b, head, q)
  const int Lk = P.Lk;
  const float scale = A.scale;
  const float pdrop = A.drop_p;
  const float inv_keep = pdrop < 1.f ? 1.f / (1.f - pdrop) : 0.f;
  RngSnap rs{0, 0};
  if (pdrop > 0.f && A.rng) rs = *A.rng;

  // a fully masked sample (per-sample key mask == 0): P = 0, O = 0, LSE = -inf
  if (P.kmask_mode == 1 && P.kmask[(int64_t)b * P.kmask_ld] == 0.f) {
    if (MODE == 0) {
      if (qvalid) {
        float* orow = P.o + ((int64_t)b * P.Lq + q) * P.ldo + col0;
        for (int d = h; d < hd; d += 2) orow[d] = 0.f;
        if (h == 0) P.lse[rowidx] = -INFINITY;
      }
    } else if (qvalid) {
      float* prow = P.probs + rowidx * Lk;
      for (int k = h; k < Lk; k += 2) prow[k] = 0.f;
    }
    return;
  }

  const bool vq = (P.ldq % 4 == 0) && (hd % 4 == 0);
  const bool vk = (P.ldk % 4 == 0) && (hd % 4 == 0);
  const bool vv = (P.ldv % 4 == 0) && (hd % 4 == 0);
  (void)vq;

  float qf[HALF];
  {
    const float* qrow = P.q + ((int64_t)b * P.Lq + (qvalid ? q : 0)) * P.ldq + col0;
    load_frag<HALF>(qf, qrow, h * HALF, hd, qvalid);
  }
  float m = -INFINITY, l = 0.f, lse = 0.f;
  if (MODE == 1) lse = qvalid ? P.lse[rowidx] : -INFINITY;
  f32x16 o[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) o[dt] = zero16();

  const float* kbase_ptr = P.k + (int64_t)b * Lk * P.ldk + col0;
  const float* vbase_ptr = P.v + (int64_t)b * Lk * P.ldv + col0;

  for (int kbase = 0; kbase < Lk; kbase += KC) {
    __syncthreads();
    load_rows<KC, HDP, LS>(Ks, kbase_ptr, Lk, P.ldk, kbase, hd, vk);
    if (MODE == 0) load_rows<KC, HDP, LS>(Vs, vbase_ptr, Lk, P.ldv, kbase, hd, vv);
    __syncthreads();
    if (!wave_active) continue;
    const int nkt = (min(KC, Lk - kbase) + 31) / 32;
    for (int kt = 0; kt < nkt; ++kt) {
      f32x16 s = dot_rows<HALF, BF>(Ks + (kt * 32 + c) * LS + h * HALF, qf, zero16());
      float sv[16];
      float mx = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kbase + kt * 32 + acc_row(r, h);
        const bool valid = key < Lk && (P.kmask_mode != 2 || kmask_val(P, b, key) != 0.f);
        sv[r] = valid ? s[r] * scale : -INFINITY;
        mx = fmaxf(mx, sv[r]);
      }
      if (MODE == 0) {
        mx = max_xor32(mx);
        const float mnew = fmaxf(m, mx);
        const float alpha = (m == -INFINITY) ? 0.f : __expf(m - mnew);
        float ls = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          sv[r] = (sv[r] == -INFINITY) ? 0.f : __expf(sv[r] - mnew);
          ls += sv[r];
        }
        ls = sum_xor32(ls);
        l = l * alpha + ls;
        m = mnew;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r)
          sv[r] = (sv[r] == -INFINITY || lse == -INFINITY) ? 0.f : __expf(sv[r] - lse);
      }
      if (pdrop > 0.f && qvalid) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int key0 = kbase + kt * 32 + 8 * g + 4 * h;
          const uint32_t bits = keep4(rs, P.drop_site, (uint64_t)rowidx * Lk + key0, pdrop);
#pragma unroll
          for (int j = 0; j < 4; ++j) sv[4 * g + j] = ((bits >> j) & 1u) ? sv[4 * g + j] * inv_keep : 0.f;
        }
      }
      if (MODE == 0) {
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
MMF_CHAIN16(o[dt], Vs[(kt * 32 + acc_row(r, h)) * LS + dt * 32 + c], sv[r])
        }
      } else if (qvalid) {
        float* prow = P.probs + rowidx * Lk;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kbase + kt * 32 + acc_row(r, h);
          if (key < Lk) prow[key] = sv[r];
        }
      }
    }
  }
  if (MODE == 1 || !qvalid) return;
  const float inv_l = l > 0.f ? 1.f / l : 0.f;
  float* orow = P.o + ((int64_t)b * P.Lq + q) * P.ldo + col0;
  const bool vo = (P.ldo % 4 == 0) && (hd % 4 == 0);
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d0 = dt * 32 + 8 * g + 4 * h;
      if (vo && d0 + 3 < hd) {
        *reinterpret_cast<float4*>(orow + d0) =
            make_float4(o[dt][4 * g] * inv_l, o[dt][4 * g + 1] * inv_l, o[dt][4 * g + 2] * inv_l,
                        o[dt][4 * g + 3] * inv_l);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (d0 + j < hd) orow[d0 + j] = o[dt][4 * g + j] * inv_l;
      }
    }
  if (h == 0) P.lse[rowidx] = l > 0.f ? m + __logf(l) : -INFINITY;
}

// D[b, head, q] = sum_d dO * O  (rowsum(P' . dP') of the softmax backward).
// Vectorised form: one thread per float4 of a row, a head = G = hd/4 consecutive
// lanes reduced by xor-shuffles (needs hd % 4 == 0, G a power of two, ld % 4 == 0).
__global__ __launch_bounds__(NT) void attn_bwd_prep_vec_kernel(const AttnArgs A) {
  const AttnPair& P = A.p[blockIdx.y];
  const int hd = A.hd, G = hd / 4, H4 = (A.heads * hd) / 4;
  const int64_t n = (int64_t)A.B * P.Lq * H4;
  const int64_t idx = (int64_t)blockIdx.x * NT + threadIdx.x;
  float s = 0.f;
  int64_t row = 0;
  int c4 = 0;
  if (idx < n) {
    row = idx / H4;              // b*Lq + q
    c4 = (int)(idx % H4);
    const float4 x = *reinterpret_cast<const float4*>(P.dout + row * P.ldo + 4 * c4);
    const float4 y = *reinterpret_cast<const float4*>(P.o + row * P.ldo + 4 * c4);
    s = x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
  }
  for (int o = G >> 1; o >= 1; o >>= 1) s += __shfl_xor(s, o);
  if (idx < n && (c4 % G) == 0) {
    const int head = c4 / G;
    const int q = (int)(row % P.Lq), b = (int)(row / P.Lq);
    P.dsum[((int64_t)b * A.heads + head) * P.Lq + q] = s;
  }
}

__global__ __launch_bounds__(NT) void attn_bwd_prep_kernel(const AttnArgs A) {
  const AttnPair& P = A.p[blockIdx.y];
  const int64_t n = (int64_t)A.B * P.Lq * A.heads;
  const int64_t idx = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (idx >= n) return;
  const int head = (int)(idx % A.heads);
  const int64_t bq = idx / A.heads;   // b*Lq + q
  const int q = (int)(bq % P.Lq);
  const int b = (int)(bq / P.Lq);
  const float* dor = P.dout + bq * P.ldo + head * A.hd;
  const float* orr = P.o + bq * P.ldo + head * A.hd;
  float s = 0.f;
  for (int d = 0; d < A.hd; ++d) s += dor[d] * orr[d];
  P.dsum[((int64_t)b * A.heads + head) * P.Lq + q] = s;
}

// ---------------------------------------------------------------------------
// dK / dV: one workgroup = 128 keys (4 waves x 32, key on the lane).
// ---------------------------------------------------------------------------
template <int HDP, int BF>
__global__ __launch_bounds__(NT) void attn_bwd_dkv_kernel(const AttnArgs A) {
  constexpr int QC = HDP == 32 ? 128 : 64;
  constexpr int LS = HDP + 4;
  constexpr int HALF = HDP / 2;
  constexpr int NDT = HDP / 32;
  __shared__ __attribute__((aligned(16))) float Qs[QC * LS];
  __shared__ __attribute__((aligned(16))) float Ds[QC * LS];   // dO chunk
  __shared__ float lse_s[QC];
  __shared__ float dsum_s[QC];

  const AttnPair& P = A.p[blockIdx.y];
  const int kblocks = (P.Lk + 127) / 128;
  int bid = blockIdx.x;
  if (bid >= A.B * A.heads * kblocks) return;
  const int kb = bid % kblocks;
  bid /= kblocks;
  const int head = bid % A.heads, b = bid / A.heads;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, h = lane >> 5, c = lane & 31;
  const int hd = A.hd, col0 = head * hd;
  const int Lq = P.Lq, Lk = P.Lk;
  const int key = kb * 128 + w * 32 + c;
  const bool wave_active = kb * 128 + w * 32 < Lk;
  bool kvalid = key < Lk;
  if (kvalid && P.kmask_mode == 2) kvalid = kmask_val(P, b, key) != 0.f;
  const float scale = A.scale;
  const float pdrop = A.drop_p;
  const float inv_keep = pdrop < 1.f ? 1.f / (1.f - pdrop) : 0.f;
  RngSnap rs{0, 0};
  if (pdrop > 0.f && A.rng) rs = *A.rng;

  f32x16 dk[NDT], dv[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) { dk[dt] = zero16(); dv[dt] = zero16(); }

  const bool sample_masked = (P.kmask_mode == 1 && P.kmask[(int64_t)b * P.kmask_ld] == 0.f);
  if (!sample_masked) {
    float kf[HALF], vf[HALF];
    {
      const int kr = key < Lk ? key : 0;
      load_frag<HALF>(kf, P.k + ((int64_t)b * Lk + kr) * P.ldk + col0, h * HALF, hd, key < Lk);
      load_frag<HALF>(vf, P.v + ((int64_t)b * Lk + kr) * P.ldv + col0, h * HALF, hd, key < Lk);
    }
    const bool vq = (P.ldq % 4 == 0) && (hd % 4 == 0);
    const bool vo = (P.ldo % 4 == 0) && (hd % 4 == 0);
    const float* qbase_ptr = P.q + (int64_t)b * Lq * P.ldq + col0;
    const float* dobase_ptr = P.dout + (int64_t)b * Lq * P.ldo + col0;
    const float* lse_ptr = P.lse + ((int64_t)b * A.heads + head) * Lq;
    const float* ds_ptr = P.dsum + ((int64_t)b * A.heads + head) * Lq;
    for (int qbase = 0; qbase < Lq; qbase += QC) {
      __syncthreads();
      load_rows<QC, HDP, LS>(Qs, qbase_ptr, Lq, P.ldq, qbase, hd, vq);
      load_rows<QC, HDP, LS>(Ds, dobase_ptr, Lq, P.ldo, qbase, hd, vo);
      for (int i = t; i < QC; i += NT) {
        const int qq = qbase + i;
        lse_s[i] = qq < Lq ? lse_ptr[qq] : -INFINITY;
        dsum_s[i] = qq < Lq ? ds_ptr[qq] : 0.f;
      }
      __syncthreads();
      if (!wave_active) continue;
      const int nqt = (min(QC, Lq - qbase) + 31) / 32;
      for (int qt = 0; qt < nqt; ++qt) {
        f32x16 s = dot_rows<HALF, BF>(Qs + (qt * 32 + c) * LS + h * HALF, kf, zero16());
        f32x16 dp = dot_rows<HALF, BF>(Ds + (qt * 32 + c) * LS + h * HALF, vf, zero16());
        float pd[16], dsr[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ql = qt * 32 + acc_row(r, h);
          const float lq = lse_s[ql];
          const bool valid = kvalid && (lq != -INFINITY) && (qbase + ql < Lq);
          const float pr = valid ? __expf(s[r] * scale - lq) : 0.f;
          float pkeep = pr, dpk = dp[r];
          if (pdrop > 0.f) {
            const bool keep =
                valid && keep1(rs, P.drop_site,
                               (uint64_t)(((int64_t)b * A.heads + head) * Lq + qbase + ql) * Lk + key, pdrop);
            pkeep = keep ? pr * inv_keep : 0.f;
            dpk = keep ? dp[r] * inv_keep : 0.f;
          }
          pd[r] = pkeep;
          dsr[r] = pr * (dpk - dsum_s[ql]);
        }
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
MMF_CHAIN16(dv[dt], pd[r], Ds[(qt * 32 + acc_row(r, h)) * LS + dt * 32 + c])
          MMF_CHAIN16(dk[dt], dsr[r], Qs[(qt * 32 + acc_row(r, h)) * LS + dt * 32 + c])
        }
      }
    }
  }
  if (!wave_active) return;
  // C[i = key (regs)][j = d (lane)]
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
    const int d = dt * 32 + c;
    if (d >= hd) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int kr = kb * 128 + w * 32 + acc_row(r, h);
      if (kr >= Lk) continue;
      P.dk[((int64_t)b * Lk + kr) * P.ldk + col0 + d] = dk[dt][r] * scale;
      P.dv[((int64_t)b * Lk + kr) * P.ldv + col0 + d] = dv[dt][r];
    }
  }
}

// ---------------------------------------------------------------------------
// dQ: one workgroup = 128 queries (query on the lane, like the forward).
// ---------------------------------------------------------------------------
template <int HDP, int BF>
__global__ __launch_bounds__(NT) void attn_bwd_dq_kernel(const AttnArgs A) {
  constexpr int KC = HDP == 32 ? 128 : 64;
  constexpr int LS = HDP + 4;
  constexpr int HALF = HDP / 2;
  constexpr int NDT = HDP / 32;
  __shared__ __attribute__((aligned(16))) float Ks[KC * LS];
  __shared__ __attribute__((aligned(16))) float Vs[KC * LS];

  const AttnPair& P = A.p[blockIdx.y];
  const int qblocks = (P.Lq + 127) / 128;
  int bid = blockIdx.x;
  if (bid >= A.B * A.heads * qblocks) return;
  const int qb = bid % qblocks;
  bid /= qblocks;
  const int head = bid % A.heads, b = bid / A.heads;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, h = lane >> 5, c = lane & 31;
  const int hd = A.hd, col0 = head * hd;
  const int Lq = P.Lq, Lk = P.Lk;
  const int q = qb * 128 + w * 32 + c;
  const bool qvalid = q < Lq;
  const bool wave_active = qb * 128 + w * 32 < Lq;
  const int64_t rowidx = ((int64_t)b * A.heads + head) * Lq + q;
  const float scale = A.scale;
  const float pdrop = A.drop_p;
  const float inv_keep = pdrop < 1.f ? 1.f / (1.f - pdrop) : 0.f;
  RngSnap rs{0, 0};
  if (pdrop > 0.f && A.rng) rs = *A.rng;

  f32x16 dq[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) dq[dt] = zero16();

  const bool sample_masked = (P.kmask_mode == 1 && P.kmask[(int64_t)b * P.kmask_ld] == 0.f);
  const float lse = qvalid ? P.lse[rowidx] : -INFINITY;
  if (!sample_masked) {
    float qf[HALF], df[HALF];
    const int qr = qvalid ? q : 0;
    load_frag<HALF>(qf, P.q + ((int64_t)b * Lq + qr) * P.ldq + col0, h * HALF, hd, qvalid);
    load_frag<HALF>(df, P.dout + ((int64_t)b * Lq + qr) * P.ldo + col0, h * HALF, hd, qvalid);
    const float dsum = qvalid ? P.dsum[rowidx] : 0.f;
    const bool vk = (P.ldk % 4 == 0) && (hd % 4 == 0);
    const bool vv = (P.ldv % 4 == 0) && (hd % 4 == 0);
    const float* kbase_ptr = P.k + (int64_t)b * Lk * P.ldk + col0;
    const float* vbase_ptr = P.v + (int64_t)b * Lk * P.ldv + col0;
    for (int kbase = 0; kbase < Lk; kbase += KC) {
      __syncthreads();
      load_rows<KC, HDP, LS>(Ks, kbase_ptr, Lk, P.ldk, kbase, hd, vk);
      load_rows<KC, HDP, LS>(Vs, vbase_ptr, Lk, P.ldv, kbase, hd, vv);
      __syncthreads();
      if (!wave_active) continue;
      const int nkt = (min(KC, Lk - kbase) + 31) / 32;
      for (int kt = 0; kt < nkt; ++kt) {
        f32x16 s = dot_rows<HALF, BF>(Ks + (kt * 32 + c) * LS + h * HALF, qf, zero16());
        f32x16 dp = dot_rows<HALF, BF>(Vs + (kt * 32 + c) * LS + h * HALF, df, zero16());
        float dsr[16];
        uint32_t bits[4] = {0xFu, 0xFu, 0xFu, 0xFu};
        if (pdrop > 0.f && qvalid) {
#pragma unroll
          for (int g = 0; g < 4; ++g)
            bits[g] = keep4(rs, P.drop_site, (uint64_t)rowidx * Lk + kbase + kt * 32 + 8 * g + 4 * h, pdrop);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kbase + kt * 32 + acc_row(r, h);
          const bool valid = qvalid && key < Lk && lse != -INFINITY &&
                             (P.kmask_mode != 2 || kmask_val(P, b, key) != 0.f);
          const float pr = valid ? __expf(s[r] * scale - lse) : 0.f;
          float dpk = dp[r];
          if (pdrop > 0.f) dpk = ((bits[r >> 2] >> (r & 3)) & 1u) ? dp[r] * inv_keep : 0.f;
          dsr[r] = pr * (dpk - dsum);
        }
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
MMF_CHAIN16(dq[dt], Ks[(kt * 32 + acc_row(r, h)) * LS + dt * 32 + c], dsr[r])
        }
      }
    }
  }
  if (!qvalid) return;
  float* qrow = P.dq + ((int64_t)b * Lq + q) * P.ldq + col0;
  const bool vo = (P.ldq % 4 == 0) && (hd % 4 == 0);
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d0 = dt * 32 + 8 * g + 4 * h;
      if (vo && d0 + 3 < hd) {
        *reinterpret_cast<float4*>(qrow + d0) =
            make_float4(dq[dt][4 * g] * scale, dq[dt][4 * g + 1] * scale, dq[dt][4 * g + 2] * scale,
                        dq[dt][4 * g + 3] * scale);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (d0 + j < hd) qrow[d0 + j] = dq[dt][4 * g + j] * scale;
      }
    }
}

// ===========================================================================
// Pooled-output attention (HybridFusion).  HybridFusion consumes the attended
// features only through their mean over the query axis (agg -> mean-pool,
// src/fusion.py:406-408 + sequence-mode pooling) and out_proj / value_proj are
// affine, so
//     mean_q (P' V) W_o^T + b_o = (pbar V) W_o^T + b_o,   pbar = mean_q P'[q, :]
// and the (Lq x Lk) attention only has to deliver the column means pbar (and
// LSE for the backward).  In the backward every query row of dP' equals
// dpbar / Lq, so dP needs no MFMA: dS = P' * dpbar / Lq - P * D,
// D = rowsum(P' * dpbar) / Lq.  Limits: Lk <= 128 (one LDS chunk).
// ===========================================================================
constexpr int PKC = 128;

constexpr float LOG2E = 1.4426950408889634f;

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Column-sum of a 32x32 S^T tile over its 32 query lanes (reduce-scatter
// butterfly without LDS: permlane16_swap for the lane-16 stage, DPP row_ror:8 /
// row_half_mirror / quad_perm for the rest).  Returns, in lane c, the sum for
// tile row r = (c >> 1) & 15 (lanes c and c^1 hold the same value).
__device__ __forceinline__ float colsum_tile(const float (&v)[16], int c) {
  float a8[8], a4[4], a2[2];
  const bool b3 = c & 8, b2 = c & 4, b1 = c & 2;
#pragma unroll
  for (int i = 0; i < 8; ++i) {   // lane c < 16 keeps rows i, c >= 16 rows i + 8 (of the pair c, c ^ 16)
    float x = v[i], y = v[i + 8];
    swap16(x, y);
    a8[i] = x + y;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {   // partner c ^ 8
    const float lo = a8[i] + dpp<DPP_ROR8>(a8[i]);
    const float hi = a8[i + 4] + dpp<DPP_ROR8>(a8[i + 4]);
    a4[i] = b3 ? hi : lo;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {   // partner c ^ 7 (flips bit 2)
    const float lo = a4[i] + dpp<DPP_HALF_MIRROR>(a4[i]);
    const float hi = a4[i + 2] + dpp<DPP_HALF_MIRROR>(a4[i + 2]);
    a2[i] = b2 ? hi : lo;
  }
  const float lo = a2[0] + dpp<DPP_XOR2>(a2[0]);
  const float hi = a2[1] + dpp<DPP_XOR2>(a2[1]);
  const float a1 = b1 ? hi : lo;
  return a1 + dpp<DPP_XOR1>(a1);
}

template <int HDP, int BF>
__global__ __launch_bounds__(NT) void attn_pool_fwd_kernel(const AttnArgs A) {
  constexpr int LS = HDP + 4;
  constexpr int HALF = HDP / 2;
  constexpr int NKT = PKC / 32;
  __shared__ __attribute__((aligned(16))) float Ks[PKC * LS];
  __shared__ float cs[4][PKC];

  const AttnPair& P = A.p[blockIdx.y];
  int bid = blockIdx.x;
  if (bid >= A.B * A.heads) return;
  const int head = bid % A.heads, b = bid / A.heads;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, h = lane >> 5, c = lane & 31;
  const int hd = A.hd, col0 = head * hd;
  const int Lq = P.Lq, Lk = P.Lk;
  const float scale = A.scale, pdrop = A.drop_p;
  const float inv_keep = pdrop < 1.f ? 1.f / (1.f - pdrop) : 0.f;
  RngSnap rs{0, 0};
  if (pdrop > 0.f && A.rng) rs = *A.rng;
  const int64_t bh = (int64_t)b * A.heads + head;
  float* pbar = P.pbar + bh * Lk;

  if (P.kmask_mode == 1 && P.kmask[(int64_t)b * P.kmask_ld] == 0.f) {
    // masked key modality: softmax over all -inf -> NaN -> 0 (src/attention.py:127-129)
    for (int k = t; k < Lk; k += NT) pbar[k] = 0.f;
    if (P.pbarT)
      for (int k = t; k < Lk; k += NT) P.pbarT[((int64_t)b * Lk + k) * A.heads + head] = 0.f;
    for (int q = t; q < Lq; q += NT) P.lse[bh * Lq + q] = -INFINITY;
    if (P.keep_bits)
      for (int q = t; q < Lq; q += NT)
        *reinterpret_cast<uint4*>(P.keep_bits + (bh * Lq + q) * 4) = make_uint4(0, 0, 0, 0);
    return;
  }
  const bool vk = (P.ldk % 4 == 0) && (hd % 4 == 0);
  load_rows<PKC, HDP, LS>(Ks, P.k + (int64_t)b * Lk * P.ldk + col0, Lk, P.ldk, 0, hd, vk);
  for (int i = t; i < 4 * PKC; i += NT) (&cs[0][0])[i] = 0.f;
  __syncthreads();
  const int nkt = (Lk + 31) / 32;

  for (int q0 = 0; q0 < Lq; q0 += 128) {
    const int q = q0 + w * 32 + c;
    if (q0 + w * 32 >= Lq) continue;   // whole wave idle (no barrier below)
    const bool qvalid = q < Lq;
    float qf[HALF];
    load_frag<HALF>(qf, P.q + ((int64_t)b * Lq + (qvalid ? q : 0)) * P.ldq + col0, h * HALF, hd, qvalid);
    float sv[NKT][16];
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      if (kt < nkt) {
        f32x16 s = dot_rows<HALF, BF>(Ks + (kt * 32 + c) * LS + h * HALF, qf, zero16());
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kt * 32 + acc_row(r, h);
          const bool valid = key < Lk && (P.kmask_mode != 2 || kmask_val(P, b, key) != 0.f);
          sv[kt][r] = valid ? s[r] * scale : -INFINITY;
          mx = fmaxf(mx, sv[kt][r]);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) sv[kt][r] = -INFINITY;
      }
    }
    mx = max_xor32(mx);
    float l = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sv[kt][r] = (sv[kt][r] == -INFINITY) ? 0.f : __expf(sv[kt][r] - mx);
        l += sv[kt][r];
      }
    l = sum_xor32(l);
    const float inv_l = (l > 0.f && qvalid) ? 1.f / l : 0.f;
    const int64_t rowidx = bh * Lq + q;
    uint32_t words[NKT];
    const bool aligned8 = (Lk & 7) == 0;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      uint32_t kb16 = 0xFFFFu;   // bit r: reg r kept
      if (pdrop > 0.f && kt < nkt)
        kb16 = keep_tile16(rs, P.drop_site, (uint64_t)rowidx * Lk + kt * 32, pdrop, h, qvalid, aligned8);
      uint32_t bits = 0;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const uint32_t kb = (kb16 >> (4 * g)) & 0xFu;
        bits |= kb << (8 * g + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float pv = sv[kt][4 * g + j] * inv_l;
          sv[kt][4 * g + j] = (pdrop > 0.f) ? (((kb >> j) & 1u) ? pv * inv_keep : 0.f) : pv;
        }
      }
      words[kt] = or_xor32(bits);
      if (kt < nkt) {
        const float colsum = colsum_tile(sv[kt], c);
        if ((c & 1) == 0) cs[w][kt * 32 + acc_row((c >> 1) & 15, h)] += colsum;
      }
    }
    if (qvalid && h == 0) {
      P.lse[rowidx] = l > 0.f ? mx + __logf(l) : -INFINITY;
      if (P.keep_bits) {
        uint32_t wv[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt) wv[kt] = words[kt];
        *reinterpret_cast<uint4*>(P.keep_bits + rowidx * 4) = make_uint4(wv[0], wv[1], wv[2], wv[3]);
      }
    }
  }
  __syncthreads();
  const float inv_lq = 1.f / (float)Lq;
  for (int k = t; k < Lk; k += NT) {
    const float v = (cs[0][k] + cs[1][k] + cs[2][k] + cs[3][k]) * inv_lq;
    pbar[k] = v;
    if (P.pbarT) P.pbarT[((int64_t)b * Lk + k) * A.heads + head] = v;
  }
}

// Pooled backward, query on the lane: D = rowsum(P' dpbar)/Lq, dS, dQ.
template <int HDP, int BF>
__global__ __launch_bounds__(NT) void attn_pool_bwd_dq_kernel(const AttnArgs A) {
  constexpr int LS = HDP + 4;
  constexpr int HALF = HDP / 2;
  constexpr int NDT = HDP / 32;
  constexpr int NKT = PKC / 32;
  __shared__ __attribute__((aligned(16))) float Ks[PKC * LS];
  __shared__ float dpb[PKC];

  const AttnPair& P = A.p[blockIdx.y];
  const int qblocks = (P.Lq + 127) / 128;
  int bid = blockIdx.x;
  if (bid >= A.B * A.heads * qblocks) return;
  const int qb = bid % qblocks;
  bid /= qblocks;
  const int head = bid % A.heads, b = bid / A.heads;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, h = lane >> 5, c = lane & 31;
  const int hd = A.hd, col0 = head * hd;
  const int Lq = P.Lq, Lk = P.Lk;
  const int q = qb * 128 + w * 32 + c;
  const bool qvalid = q < Lq;
  const int64_t bh = (int64_t)b * A.heads + head;
  const int64_t rowidx = bh * Lq + q;
  const float scale = A.scale, pdrop = A.drop_p;
  const float inv_keep = pdrop < 1.f ? 1.f / (1.f - pdrop) : 0.f;
  const float inv_lq = 1.f / (float)Lq;
  float* qrow = P.dq + ((int64_t)b * Lq + (qvalid ? q : 0)) * P.ldq + col0;

  if (P.kmask_mode == 1 && P.kmask[(int64_t)b * P.kmask_ld] == 0.f) {
    if (qvalid) {
      for (int d = h; d < hd; d += 2) qrow[d] = 0.f;
      if (h == 0) P.dsum[rowidx] = 0.f;
    }
    return;
  }
  const bool vk = (P.ldk % 4 == 0) && (hd % 4 == 0);
  load_rows<PKC, HDP, LS>(Ks, P.k + (int64_t)b * Lk * P.ldk + col0, Lk, P.ldk, 0, hd, vk);
  for (int k = t; k < PKC; k += NT) dpb[k] = k < Lk ? P.dpbar[bh * Lk + k] : 0.f;
  __syncthreads();
  if (qb * 128 + w * 32 >= Lq) return;
  const int nkt = (Lk + 31) / 32;
  float qf[HALF];
  load_frag<HALF>(qf, P.q + ((int64_t)b * Lq + (qvalid ? q : 0)) * P.ldq + col0, h * HALF, hd, qvalid);
  const float lse = qvalid ? P.lse[rowidx] : -INFINITY;
  uint4 kw = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
  if (P.keep_bits && pdrop > 0.f && qvalid) kw = *reinterpret_cast<const uint4*>(P.keep_bits + rowidx * 4);
  const uint32_t kwa[4] = {kw.x, kw.y, kw.z, kw.w};
  float pr[NKT][16];
  float D = 0.f;
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    if (kt < nkt) {
      f32x16 s = dot_rows<HALF, BF>(Ks + (kt * 32 + c) * LS + h * HALF, qf, zero16());
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kt * 32 + acc_row(r, h);
        const bool valid = qvalid && key < Lk && lse != -INFINITY &&
                           (P.kmask_mode != 2 || kmask_val(P, b, key) != 0.f);
        const float p = valid ? __expf(s[r] * scale - lse) : 0.f;
        pr[kt][r] = p;
        const bool keep = pdrop <= 0.f || ((kwa[kt] >> (key & 31)) & 1u);
        D += keep ? p * inv_keep * dpb[key] : 0.f;
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) pr[kt][r] = 0.f;
    }
  }
  D = sum_xor32(D) * inv_lq;
  if (qvalid && h == 0) P.dsum[rowidx] = D;
  f32x16 dq[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) dq[dt] = zero16();
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    if (kt >= nkt) break;
    float ds[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kt * 32 + acc_row(r, h);
      const bool keep = pdrop <= 0.f || ((kwa[kt] >> (key & 31)) & 1u);
      const float pd = keep ? pr[kt][r] * inv_keep : 0.f;
      ds[r] = pd * dpb[key] * inv_lq - pr[kt][r] * D;
    }
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
MMF_CHAIN16(dq[dt], Ks[(kt * 32 + acc_row(r, h)) * LS + dt * 32 + c], ds[r])
  }
  if (!qvalid) return;
  const bool vo = (P.ldq % 4 == 0) && (hd % 4 == 0);
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d0 = dt * 32 + 8 * g + 4 * h;
      if (vo && d0 + 3 < hd) {
        *reinterpret_cast<float4*>(qrow + d0) =
            make_float4(dq[dt][4 * g] * scale, dq[dt][4 * g + 1] * scale, dq[dt][4 * g + 2] * scale,
                        dq[dt][4 * g + 3] * scale);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (d0 + j < hd) qrow[d0 + j] = dq[dt][4 * g + j] * scale;
      }
    }
}

// Pooled backward, key on the lane: dK = scale * dS^T Q (needs D from the dq kernel).
// bf16x3 at hd 64 (here and in attn_poolL_dq_kernel) runs at 3 waves / SIMD: at 4 its
// split operands spill 73-84 VGPRs (C5 "high": dK 2404 -> 1778 us, dQ 3126 -> 2657 us);
// bf16 keeps 4 (3 cost its dQ 2199 -> 2478 us).
template <int HDP, int BF>
__global__ __launch_bounds__(NT, (BF == 2 && HDP == 64) ? 3 : 4) void attn_pool_bwd_dk_kernel(const AttnArgs A) {
  constexpr int QC = 128;
  constexpr int LS = HDP + 4;
  constexpr int HALF = HDP / 2;
  constexpr int NDT = HDP / 32;
  __shared__ __attribute__((aligned(16))) float Qs[QC * LS];
  __shared__ __attribute__((aligned(16))) float lse_s[QC];        // log2 units; +inf: no probability
  __shared__ __attribute__((aligned(16))) float dsum_s[QC];
  __shared__ __attribute__((aligned(16))) uint32_t kw_s[4 * QC];   // [wave][query]: keep word of the wave's 32 keys

  const AttnPair& P = A.p[blockIdx.y];
  const int kblocks = (P.Lk + 127) / 128;
  int bid = blockIdx.x;
  if (bid >= A.B * A.heads * kblocks) return;
  const int kb = bid % kblocks;
  bid /= kblocks;
  const int head = bid % A.heads, b = bid / A.heads;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, h = lane >> 5, c = lane & 31;
  const int hd = A.hd, col0 = head * hd;
  const int Lq = P.Lq, Lk = P.Lk;
  const int key = kb * 128 + w * 32 + c;
  const bool wave_active = kb * 128 + w * 32 < Lk;
  bool kvalid = key < Lk;
  if (kvalid && P.kmask_mode == 2) kvalid = kmask_val(P, b, key) != 0.f;
  const int64_t bh = (int64_t)b * A.heads + head;
  const float scale = A.scale, pdrop = A.drop_p;
  const float inv_keep = pdrop < 1.f ? 1.f / (1.f - pdrop) : 0.f;
  const float inv_lq = 1.f / (float)Lq;
  const bool use_bits = P.keep_bits && pdrop > 0.f;
  const float sl2 = scale * LOG2E;

  f32x16 dk[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) dk[dt] = zero16();
  const bool sample_masked = (P.kmask_mode == 1 && P.kmask[(int64_t)b * P.kmask_ld] == 0.f);
  if (!sample_masked) {
    float kf[HALF];
    load_frag<HALF>(kf, P.k + ((int64_t)b * Lk + (key < Lk ? key : 0)) * P.ldk + col0, h * HALF, hd,
                    key < Lk);
    const float dpk = key < Lk ? P.dpbar[bh * Lk + key] * inv_lq * inv_keep : 0.f;
    const bool vq = (P.ldq % 4 == 0) && (hd % 4 == 0);
    for (int qbase = 0; qbase < Lq; qbase += QC) {
      __syncthreads();
      load_rows<QC, HDP, LS, HDP == 32>(Qs, P.q + (int64_t)b * Lq * P.ldq + col0, Lq, P.ldq, qbase, hd, vq);
      for (int i = t; i < QC; i += NT) {
        const int qq = qbase + i;
        const float l = qq < Lq ? P.lse[bh * Lq + qq] : -INFINITY;
        lse_s[i] = l == -INFINITY ? INFINITY : l * LOG2E;
        dsum_s[i] = qq < Lq ? P.dsum[bh * Lq + qq] : 0.f;
      }
      if (use_bits)
        for (int i = t; i < QC * 4; i += NT) {
          // this workgroup's four 32-key words of query qq (kw_ld words per query row)
          const int wv = i / QC, qq = qbase + (i % QC), wd = kb * 4 + wv;
          kw_s[i] = (qq < Lq && wd < P.kw_ld) ? P.keep_bits[(bh * Lq + qq) * P.kw_ld + wd] : 0u;
        }
      __syncthreads();
      if (!wave_active) continue;
      const int nqt = (min(QC, Lq - qbase) + 31) / 32;
      for (int qt = 0; qt < nqt; ++qt) {
        f32x16 s = dot_rows<HALF, BF>(Qs + (qt * 32 + c) * LS + h * HALF, kf, zero16());
        float ds[16];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int q0 = qt * 32 + 8 * g + 4 * h;   // regs 4g..4g+3: queries q0..q0+3
          const float4 l4 = *reinterpret_cast<const float4*>(lse_s + q0);
          const float4 d4 = *reinterpret_cast<const float4*>(dsum_s + q0);
          const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dv[4] = {d4.x, d4.y, d4.z, d4.w};
          uint32_t kv[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
          if (use_bits) {
            const uint4 k4 = *reinterpret_cast<const uint4*>(kw_s + w * QC + q0);
            kv[0] = k4.x; kv[1] = k4.y; kv[2] = k4.z; kv[3] = k4.w;
          }
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const float p = fast_exp2(s[4 * g + jj] * sl2 - lv[jj]);
            ds[4 * g + jj] = kvalid ? p * ((((kv[jj] >> c) & 1u) ? dpk : 0.f) - dv[jj]) : 0.f;
          }
        }
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
MMF_CHAIN16(dk[dt], ds[r], Qs[(qt * 32 + acc_row(r, h)) * LS + dt * 32 + c])
      }
    }
  }
  if (!wave_active) return;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
    const int d = dt * 32 + c;
    if (d >= hd) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int kr = kb * 128 + w * 32 + acc_row(r, h);
      if (kr < Lk) P.dk[((int64_t)b * Lk + kr) * P.ldk + col0 + d] = dk[dt][r] * scale;
    }
  }
}

// ---------------------------------------------------------------------------
// Long-key pooled kernels (Lk > 128, e.g. C5's T = 512): the same pooled
// formulation, with keys streamed through LDS in chunks instead of held whole.
//   fwd pass 1 (query on the lane): LSE by an online max / sum over key chunks,
//       and the dropout keep words (B, heads, Lq, kw_ld), bit k%32 of word k/32;
//   fwd pass 2 (key on the lane, queries streamed): pbar = colsum(P') / Lq;
//   bwd dQ (query on the lane, two passes over key chunks): D, then dS and dQ;
//   bwd dK: attn_pool_bwd_dk_kernel (key on the lane; any Lk).
// ---------------------------------------------------------------------------
// LEAN (launch-time: every pair has Lk % 32 == 0 and no per-key mask): whole key tiles
// only, so the per-register validity tests and the unaligned keep-bit path compile out.
template <int HDP, int BF, bool LEAN = false>
__global__ __launch_bounds__(NT) void attn_poolL_lse_kernel(const AttnArgs A) {
  constexpr int KC = 128;   // keys per LDS chunk (34 KB at HDP = 64: 4 workgroups / CU)
  constexpr int LS = HDP + 4;
  constexpr int HALF = HDP / 2;
  __shared__ __attribute__((aligned(16))) float Ks[KC * LS];

  const AttnPair& P = A.p[blockIdx.y];
  const int qblocks = (P.Lq + 127) / 128;
  int bid = blockIdx.x;
  if (bid >= A.B * A.heads * qblocks) return;
  const int qb = bid % qblocks;
  bid /= qblocks;
  const int head = bid % A.heads, b = bid / A.heads;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, h = lane >> 5, c = lane & 31;
  const int hd = A.hd, col0 = head * hd;
  const int Lq = P.Lq, Lk = P.Lk, kwl = P.kw_ld;
  const int q = qb * 128 + w * 32 + c;
  const bool qvalid = q < Lq;
  const bool wave_active = qb * 128 + w * 32 < Lq;
  const int64_t bh = (int64_t)b * A.heads + head;
  const int64_t rowidx = bh * Lq + q;
  const float pdrop = A.drop_p;
  RngSnap rs{0, 0};
  if (pdrop > 0.f && A.rng) rs = *A.rng;
  const bool bits_out = P.keep_bits != nullptr && pdrop > 0.f;

  // masked key modality: every probability is 0 (src/attention.py:127-129); the
  // keep words are never read when LSE = -inf
  if (P.kmask_mode == 1 && P.kmask[(int64_t)b * P.kmask_ld] == 0.f) {
    if (qvalid && h == 0) P.lse[rowidx] = -INFINITY;
    return;
  }
  const bool vk = (P.ldk % 4 == 0) && (hd % 4 == 0);
  float qf[HALF];
  load_frag<HALF>(qf, P.q + ((int64_t)b * Lq + (qvalid ? q : 0)) * P.ldq + col0, h * HALF, hd, qvalid);
  const float sl2 = A.scale * LOG2E;
  const bool aligned8 = (Lk & 7) == 0;
  float m = -INFINITY, l = 0.f;   // running max / sum, log2 domain
  for (int kbase = 0; kbase < Lk; kbase += KC) {
    __syncthreads();
    load_rows<KC, HDP, LS>(Ks, P.k + (int64_t)b * Lk * P.ldk + col0, Lk, P.ldk, kbase, hd, vk);
    __syncthreads();
    if (!wave_active) continue;
    const int nkt = (min(KC, Lk - kbase) + 31) / 32;
    for (int kt = 0; kt < nkt; ++kt) {
      const f32x16 s = dot_rows<HALF, BF>(Ks + (kt * 32 + c) * LS + h * HALF, qf, zero16());
      float sv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) sv[r] = s[r] * sl2;
      if (!LEAN && (kbase + kt * 32 + 32 > Lk || P.kmask_mode == 2)) {   // partial tile / per-key mask only
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kbase + kt * 32 + acc_row(r, h);
          if (!(key < Lk && (P.kmask_mode != 2 || kmask_val(P, b, key) != 0.f))) sv[r] = -INFINITY;
        }
      }
      float mx = sv[0];
#pragma unroll
      for (int r = 1; r < 16; ++r) mx = fmaxf(mx, sv[r]);
      mx = max_xor32(mx);
      const float mnew = fmaxf(m, mx);
      const float mref = mnew == -INFINITY ? 0.f : mnew;   // exp2(-inf - mref) = 0, no NaN
      float ls = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) ls += fast_exp2(sv[r] - mref);
      ls = sum_xor32(ls);
      l = l * fast_exp2(m - mref) + ls;
      m = mnew;
      if (bits_out) {
        // LEAN: invalid query lanes draw too (their words are never stored)
        const uint32_t kb16 = keep_tile16(rs, P.drop_site, (uint64_t)rowidx * Lk + kbase + kt * 32, pdrop, h,
                                          LEAN || qvalid, LEAN || aligned8);
        uint32_t bits = 0;
#pragma unroll
        for (int g = 0; g < 4; ++g) bits |= ((kb16 >> (4 * g)) & 0xFu) << (8 * g + 4 * h);
        bits = or_xor32(bits);
        if (qvalid && h == 0) P.keep_bits[rowidx * kwl + ((kbase >> 5) + kt)] = bits;
      }
    }
  }
  if (qvalid && h == 0) P.lse[rowidx] = l > 0.f ? (m + __log2f(l)) * (1.f / LOG2E) : -INFINITY;
}

template <int HDP, int BF>
__global__ __launch_bounds__(NT) void attn_poolL_colsum_kernel(const AttnArgs A) {
  constexpr int QC = 128;
  constexpr int LS = HDP + 4;
  constexpr int HALF = HDP / 2;
  __shared__ __attribute__((aligned(16))) float Qs[QC * LS];
  __shared__ __attribute__((aligned(16))) float lse_s[QC];        // log2 units; +inf: no probability
  __shared__ __attribute__((aligned(16))) uint32_t kw_s[4 * QC];   // [wave][query]: keep word of the wave's 32 keys

  const AttnPair& P = A.p[blockIdx.y];
  const int kblocks = (P.Lk + 127) / 128;
  int bid = blockIdx.x;
  if (bid >= A.B * A.heads * kblocks) return;
  const int kb = bid % kblocks;
  bid /= kblocks;
  const int head = bid % A.heads, b = bid / A.heads;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, h = lane >> 5, c = lane & 31;
  const int hd = A.hd, col0 = head * hd;
  const int Lq = P.Lq, Lk = P.Lk;
  const int key = kb * 128 + w * 32 + c;
  const bool wave_active = kb * 128 + w * 32 < Lk;
  bool kvalid = key < Lk;
  if (kvalid && P.kmask_mode == 2) kvalid = kmask_val(P, b, key) != 0.f;
  const int64_t bh = (int64_t)b * A.heads + head;
  const float pdrop = A.drop_p;
  const float inv_keep = pdrop > 0.f ? (pdrop < 1.f ? 1.f / (1.f - pdrop) : 0.f) : 1.f;
  const bool use_bits = P.keep_bits != nullptr && pdrop > 0.f;
  const float sl2 = A.scale * LOG2E;

  float cs = 0.f;
  const bool sample_masked = (P.kmask_mode == 1 && P.kmask[(int64_t)b * P.kmask_ld] == 0.f);
  if (!sample_masked) {
    float kf[HALF];
    load_frag<HALF>(kf, P.k + ((int64_t)b * Lk + (key < Lk ? key : 0)) * P.ldk + col0, h * HALF, hd, key < Lk);
    const bool vq = (P.ldq % 4 == 0) && (hd % 4 == 0);
    for (int qbase = 0; qbase < Lq; qbase += QC) {
      __syncthreads();
      load_rows<QC, HDP, LS>(Qs, P.q + (int64_t)b * Lq * P.ldq + col0, Lq, P.ldq, qbase, hd, vq);
      for (int i = t; i < QC; i += NT) {
        const int qq = qbase + i;
        const float l = qq < Lq ? P.lse[bh * Lq + qq] : -INFINITY;
        lse_s[i] = l == -INFINITY ? INFINITY : l * LOG2E;
      }
      if (use_bits)
        for (int i = t; i < QC * 4; i += NT) {
          const int wv = i / QC, qq = qbase + (i % QC), wd = kb * 4 + wv;
          kw_s[i] = (qq < Lq && wd < P.kw_ld) ? P.keep_bits[(bh * Lq + qq) * P.kw_ld + wd] : 0u;
        }
      __syncthreads();
      if (!wave_active) continue;
      const int nqt = (min(QC, Lq - qbase) + 31) / 32;
      for (int qt = 0; qt < nqt; ++qt) {
        const f32x16 s = dot_rows<HALF, BF>(Qs + (qt * 32 + c) * LS + h * HALF, kf, zero16());
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int q0 = qt * 32 + 8 * g + 4 * h;   // regs 4g..4g+3: queries q0..q0+3
          const float4 l4 = *reinterpret_cast<const float4*>(lse_s + q0);
          const float lv[4] = {l4.x, l4.y, l4.z, l4.w};
          uint32_t kv[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
          if (use_bits) {
            const uint4 k4 = *reinterpret_cast<const uint4*>(kw_s + w * QC + q0);
            kv[0] = k4.x; kv[1] = k4.y; kv[2] = k4.z; kv[3] = k4.w;
          }
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            cs += ((kv[jj] >> c) & 1u) ? fast_exp2(s[4 * g + jj] * sl2 - lv[jj]) : 0.f;
        }
      }
    }
  }
  if (!kvalid) cs = 0.f;
  cs = sum_xor32(cs) * inv_keep * (1.f / (float)Lq);
  if (wave_active && h == 0 && key < Lk) {
    P.pbar[bh * Lk + key] = cs;
    if (P.pbarT) P.pbarT[((int64_t)b * Lk + key) * A.heads + head] = cs;
  }
}

template <int HDP, int BF, bool LEAN = false>   // LEAN: as attn_poolL_lse_kernel
__global__ __launch_bounds__(NT, (BF == 2 && HDP == 64) ? 3 : 4) void attn_poolL_dq_kernel(const AttnArgs A) {
  constexpr int KC = 128;   // keys per LDS chunk (34 KB at HDP = 64: 4 workgroups / CU)
  constexpr int LS = HDP + 4;
  constexpr int HALF = HDP / 2;
  constexpr int NDT = HDP / 32;
  __shared__ __attribute__((aligned(16))) float Ks[KC * LS];
  __shared__ __attribute__((aligned(16))) float dpb[KC];

  const AttnPair& P = A.p[blockIdx.y];
  const int qblocks = (P.Lq + 127) / 128;
  int bid = blockIdx.x;
  if (bid >= A.B * A.heads * qblocks) return;
  const int qb = bid % qblocks;
  bid /= qblocks;
  const int head = bid % A.heads, b = bid / A.heads;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, h = lane >> 5, c = lane & 31;
  const int hd = A.hd, col0 = head * hd;
  const int Lq = P.Lq, Lk = P.Lk, kwl = P.kw_ld;
  const int q = qb * 128 + w * 32 + c;
  const bool qvalid = q < Lq;
  const bool wave_active = qb * 128 + w * 32 < Lq;
  const int64_t bh = (int64_t)b * A.heads + head;
  const int64_t rowidx = bh * Lq + q;
  const float scale = A.scale, pdrop = A.drop_p;
  const float inv_keep = pdrop > 0.f ? (pdrop < 1.f ? 1.f / (1.f - pdrop) : 0.f) : 1.f;
  const bool use_bits = P.keep_bits != nullptr && pdrop > 0.f;
  const float gscale = inv_keep / (float)Lq;   // dP'[q, k] = dpbar[k] / Lq, through the dropout scale
  float* qrow = P.dq + ((int64_t)b * Lq + (qvalid ? q : 0)) * P.ldq + col0;

  if (P.kmask_mode == 1 && P.kmask[(int64_t)b * P.kmask_ld] == 0.f) {
    if (qvalid) {
      for (int d = h; d < hd; d += 2) qrow[d] = 0.f;
      if (h == 0) P.dsum[rowidx] = 0.f;
    }
    return;
  }
  const bool vk = (P.ldk % 4 == 0) && (hd % 4 == 0);
  float qf[HALF];
  load_frag<HALF>(qf, P.q + ((int64_t)b * Lq + (qvalid ? q : 0)) * P.ldq + col0, h * HALF, hd, qvalid);
  const float sl2 = scale * LOG2E;
  // invalid query lanes (and fully masked rows) get LSE = +inf: every p = exp2(s - inf) = 0
  const float lse_q = qvalid ? P.lse[rowidx] : -INFINITY;
  const float lse2 = lse_q == -INFINITY ? INFINITY : lse_q * LOG2E;
  const float* kbase_ptr = P.k + (int64_t)b * Lk * P.ldk + col0;

  // pre-dropout probabilities of one 32-key tile and the lane's keep bits
  // (shifted so reg r's key is bit (r & 3) + 8 (r >> 2)); per-key validity
  // tests only on a partial last tile or with a per-key mask
  auto tile = [&](int kbase, int kt, float (&pr)[16], uint32_t& word) {
    const f32x16 s = dot_rows<HALF, BF>(Ks + (kt * 32 + c) * LS + h * HALF, qf, zero16());
#pragma unroll
    for (int r = 0; r < 16; ++r) pr[r] = fast_exp2(s[r] * sl2 - lse2);
    if (!LEAN && (kbase + kt * 32 + 32 > Lk || P.kmask_mode == 2)) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kbase + kt * 32 + acc_row(r, h);
        if (!(key < Lk && (P.kmask_mode != 2 || kmask_val(P, b, key) != 0.f))) pr[r] = 0.f;
      }
    }
    word = (use_bits && qvalid) ? P.keep_bits[rowidx * kwl + ((kbase >> 5) + kt)] >> (4 * h) : 0xFFFFFFFFu;
  };
  auto keep_of = [](uint32_t word, int r) { return ((word >> ((r & 3) + 8 * (r >> 2))) & 1u) != 0u; };
  auto stage = [&](int kbase) {
    __syncthreads();
    load_rows<KC, HDP, LS, HDP == 32>(Ks, kbase_ptr, Lk, P.ldk, kbase, hd, vk);
    for (int i = t; i < KC; i += NT) dpb[i] = kbase + i < Lk ? P.dpbar[bh * Lk + kbase + i] * gscale : 0.f;
    __syncthreads();
  };

  // pass A: D = sum_k P'[q, k] dP'[q, k]
  float D = 0.f;
  for (int kbase = 0; kbase < Lk; kbase += KC) {
    stage(kbase);
    if (!wave_active) continue;
    const int nkt = (min(KC, Lk - kbase) + 31) / 32;
    for (int kt = 0; kt < nkt; ++kt) {
      float pr[16];
      uint32_t word;
      tile(kbase, kt, pr, word);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 g4 = *reinterpret_cast<const float4*>(dpb + kt * 32 + 8 * g + 4 * h);
        const float gv[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) D += keep_of(word, 4 * g + j) ? pr[4 * g + j] * gv[j] : 0.f;
      }
    }
  }
  D = sum_xor32(D);
  if (qvalid && h == 0) P.dsum[rowidx] = D;

  // pass B: dS = P (dP - D), dQ = scale dS K
  f32x16 dq[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) dq[dt] = zero16();
  for (int kbase = 0; kbase < Lk; kbase += KC) {
    stage(kbase);
    if (!wave_active) continue;
    const int nkt = (min(KC, Lk - kbase) + 31) / 32;
    for (int kt = 0; kt < nkt; ++kt) {
      float pr[16], ds[16];
      uint32_t word;
      tile(kbase, kt, pr, word);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 g4 = *reinterpret_cast<const float4*>(dpb + kt * 32 + 8 * g + 4 * h);
        const float gv[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) ds[4 * g + j] = pr[4 * g + j] * ((keep_of(word, 4 * g + j) ? gv[j] : 0.f) - D);
      }
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
MMF_CHAIN16(dq[dt], Ks[(kt * 32 + acc_row(r, h)) * LS + dt * 32 + c], ds[r])
    }
  }
  if (!qvalid) return;
  const bool vo = (P.ldq % 4 == 0) && (hd % 4 == 0);
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d0 = dt * 32 + 8 * g + 4 * h;
      if (vo && d0 + 3 < hd) {
        *reinterpret_cast<float4*>(qrow + d0) =
            make_float4(dq[dt][4 * g] * scale, dq[dt][4 * g + 1] * scale, dq[dt][4 * g + 2] * scale,
                        dq[dt][4 * g + 3] * scale);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (d0 + j < hd) qrow[d0 + j] = dq[dt][4 * g + j] * scale;
      }
    }
}

// ---------------------------------------------------------------------------
// Lean pooled kernels: the same three passes for the common HybridFusion case
// (every key valid: Lk % 32 == 0, Lk <= 128, no per-key mask; float4-able
// rows), with the per-score work cut to a handful of VALU ops: scores stay in
// the exp2 domain (one FMA + v_exp per score), no per-element validity
// tests (invalid query lanes get a zero weight / +inf LSE), and per-key /
// per-query side data are read from LDS as broadcast float4s.
// ---------------------------------------------------------------------------

template <int HALF>
__device__ __forceinline__ void load_frag_vec(float* f, const float* row) {
#pragma unroll
  for (int s = 0; s < HALF; s += 4) {
    const float4 v = *reinterpret_cast<const float4*>(row + s);
    f[s] = v.x; f[s + 1] = v.y; f[s + 2] = v.z; f[s + 3] = v.w;
  }
}

// Packed keep words of one 32-query tile (query on the lane) of the lean forward:
// words[kt] bit 8g + 4h' + j = keep decision of key kt*32 + 8g + 4h' + j for the
// lane's query (the layout of the saved keep_bits rows); both lane halves end with
// the same words.  Every lane of the wave must call it (it shuffles).
template <int NKT, bool DROP>
__device__ __forceinline__ void lean_keep_words(uint32_t (&words)[NKT], const RngSnap& rs, uint32_t site,
                                                uint64_t rowbase, int nkt, float pdrop, int h) {
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    words[kt] = 0u;
    if (kt < nkt) {
      const uint32_t kb16 = DROP ? keep_tile16(rs, site, rowbase + kt * 32, pdrop, h, true, true) : 0xFFFFu;
      uint32_t bits = 0;
#pragma unroll
      for (int g = 0; g < 4; ++g) bits |= ((kb16 >> (4 * g)) & 0xFu) << (8 * g + 4 * h);
      words[kt] = or_xor32(bits);
    }
  }
}

// DROP (train mode with p > 0, launch-time choice): the loop body has no dropout
// branches.  KW: the keep words were drawn beforehand (attn_keep_words_kernel, on a side
// stream while the projection GEMMs run) -- read, not drawn, and not written back.
template <int HDP, int BF, bool DROP = true, bool PST = false, bool KW = false>
__global__ __launch_bounds__(NT, HDP == 32 ? 4 : 2) void attn_pool_fwd_lean(const AttnArgs A) {
  constexpr int LS = HDP + 4;
  constexpr int HALF = HDP / 2;
  constexpr int NKT = PKC / 32;
  __shared__ __attribute__((aligned(16))) float Ks[PKC * LS];
  __shared__ float cs[4][PKC];

  const AttnPair& P = A.p[blockIdx.y];
  const int bid = blockIdx.x;
  if (bid >= A.B * A.heads) return;
  const int head = bid % A.heads, b = bid / A.heads;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, h = lane >> 5, c = lane & 31;
  const int hd = A.hd, col0 = head * hd;
  const int Lq = P.Lq, Lk = P.Lk, nkt = Lk >> 5;
  const float pdrop = DROP ? A.drop_p : 0.f;
  const float inv_keep = pdrop < 1.f ? 1.f / (1.f - pdrop) : 0.f;
  RngSnap rs{0, 0};
  if (pdrop > 0.f && A.rng) rs = *A.rng;
  const int64_t bh = (int64_t)b * A.heads + head;
  float* pbar = P.pbar + bh * Lk;
  FSTAMP_RT(7)
  FSTAMP(0)
  FSTAMP_ID()

  // the sample mask, this wave's first query fragment and the K image in one round trip
  const float msk = P.kmask_mode == 1 ? P.kmask[(int64_t)b * P.kmask_ld] : 1.f;
  float qf[HALF];   // the query fragment of this wave's current tile (reloaded at the end of an iteration)
  load_frag_vec<HALF>(qf, P.q + ((int64_t)b * Lq + min(w * 32 + c, Lq - 1)) * P.ldq + col0 + h * HALF);
  constexpr int C4 = HDP / 4;
  constexpr int KPER = PKC * C4 / NT;   // float4 slots of the K image per thread
  float4 kv[KPER];
  {
    // branch-free: clamped addresses, out-of-image slots zeroed at the LDS write (a
    // guarded load per slot made the compiler drain vmcnt between the loads)
    const float* kb = P.k + (int64_t)b * Lk * P.ldk + col0;
#pragma unroll
    for (int i = 0; i < KPER; ++i) {
      const int idx = t + i * NT;
      const int r = min(idx / C4, Lk - 1), c4 = min((idx % C4) * 4, hd - 4);
      kv[i] = *reinterpret_cast<const float4*>(kb + (int64_t)r * P.ldk + c4);
    }
  }
  // the dropout keep words of the wave's first query tile do not depend on any load:
  // drawn while the loads above are in flight (Philox is ~20 % of the kernel's VALU work)
  uint32_t words[NKT];
  auto read_words = [&](int qrow) {   // KW: the row's words as the draws would give them
    const uint4 v = *reinterpret_cast<const uint4*>(P.keep_bits + (bh * Lq + qrow) * 4);
    const uint32_t a[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) words[kt] = kt < nkt ? a[kt] : 0u;
  };
  if constexpr (KW) read_words(min(w * 32 + c, Lq - 1));
  else lean_keep_words<NKT, DROP>(words, rs, P.drop_site, (uint64_t)(bh * Lq + min(w * 32 + c, Lq - 1)) * Lk, nkt,
                                  pdrop, h);
  if (msk == 0.f) {
    for (int k = t; k < Lk; k += NT) pbar[k] = 0.f;
    if (P.pbarT)
      for (int k = t; k < Lk; k += NT) P.pbarT[((int64_t)b * Lk + k) * A.heads + head] = 0.f;
    for (int q = t; q < Lq; q += NT) P.lse[bh * Lq + q] = -INFINITY;
    if (P.keep_bits && !KW)
      for (int q = t; q < Lq; q += NT)
        *reinterpret_cast<uint4*>(P.keep_bits + (bh * Lq + q) * 4) = make_uint4(0, 0, 0, 0);
    return;
  }
#pragma unroll
  for (int i = 0; i < KPER; ++i) {
    const int idx = t + i * NT;
    const bool in = idx / C4 < Lk && (idx % C4) * 4 < hd;
    *reinterpret_cast<float4*>(&Ks[(idx / C4) * LS + (idx % C4) * 4]) = in ? kv[i] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  FSTAMP(1)

  const float c2 = A.scale * LOG2E;
  float colacc[NKT];
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) colacc[kt] = 0.f;

  for (int qt = w; qt * 32 < Lq; qt += 4) {
    const int q = qt * 32 + c;
    const bool qvalid = q < Lq;
    const int qq = qvalid ? q : Lq - 1;
    const int64_t rowidx = bh * Lq + qq;
    float sv[NKT][16];
    uint32_t kb[NKT];   // keep bits of the lane's 16 registers per key tile
    float mx = -INFINITY;
    // the dropout draws do not depend on S: issued beside the S MFMAs
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      if (kt < nkt) {
        const f32x16 s = dot_rows<HALF, BF>(Ks + (kt * 32 + c) * LS + h * HALF, qf, zero16());
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          sv[kt][r] = s[r];
          mx = fmaxf(mx, s[r]);
        }
      } else {
        kb[kt] = 0u;
#pragma unroll
        for (int r = 0; r < 16; ++r) sv[kt][r] = 0.f;
      }
    }
    mx = max_xor32(mx);
    FSTAMP(2)
    const float mc = mx * c2;
    float l = 0.f;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      if (kt < nkt) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = fast_exp2(fmaf(sv[kt][r], c2, -mc));
          sv[kt][r] = e;
          l += e;
        }
      }
    }
    l = sum_xor32(l);
    FSTAMP(3)
    if constexpr (PST) {
      // P = e / l kept for the backward (fire-and-forget 1-KB wave stores in register order);
      // P' = keep ? P / (1 - p) : 0 into the column sums
      const float f = qvalid ? 1.f / l : 0.f;
      float* pst = P.pstore + ((bh * ((Lq + 31) / 32) + qt) * 4) * 1024 + lane * 4;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        if (kt < nkt) {
          const uint32_t wk = words[kt] >> (4 * h);
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            float pv[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) pv[j] = sv[kt][4 * g + j] * f;
            *reinterpret_cast<float4*>(pst + kt * 1024 + g * 256) = make_float4(pv[0], pv[1], pv[2], pv[3]);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int r = 4 * g + j;
              sv[kt][r] = (!DROP || ((wk >> (8 * g + j)) & 1u)) ? (DROP ? pv[j] * inv_keep : pv[j]) : 0.f;
            }
          }
          colacc[kt] += colsum_tile(sv[kt], c);
        }
      }
    } else {
      const float f = qvalid ? (pdrop > 0.f ? inv_keep : 1.f) / l : 0.f;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt) {
        if (kt < nkt) {
          const uint32_t wk = words[kt] >> (4 * h);   // reg r = 4g + j <-> key bit 8g + 4h + j
#pragma unroll
          for (int r = 0; r < 16; ++r) sv[kt][r] = keep_sel(wk, 8 * (r >> 2) + (r & 3), sv[kt][r] * f);
          colacc[kt] += colsum_tile(sv[kt], c);
        }
      }
    }
    if (qvalid && h == 0) {
      P.lse[rowidx] = mx * A.scale + __logf(l);
      if (!KW && P.keep_bits && pdrop > 0.f)
        *reinterpret_cast<uint4*>(P.keep_bits + rowidx * 4) =
            make_uint4(words[0], NKT > 1 ? words[1] : 0u, NKT > 2 ? words[2] : 0u, NKT > 3 ? words[3] : 0u);
    }
    FSTAMP(4)
    if ((qt + 4) * 32 < Lq) {
      const int qn = min((qt + 4) * 32 + c, Lq - 1);
      load_frag_vec<HALF>(qf, P.q + ((int64_t)b * Lq + qn) * P.ldq + col0 + h * HALF);
      if constexpr (KW) read_words(qn);
      else lean_keep_words<NKT, DROP>(words, rs, P.drop_site, (uint64_t)(bh * Lq + qn) * Lk, nkt, pdrop, h);
    }
  }
  if ((c & 1) == 0) {
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt)
      if (kt < nkt) cs[w][kt * 32 + acc_row((c >> 1) & 15, h)] = colacc[kt];
  }
  __syncthreads();
  const float inv_lq = 1.f / (float)Lq;
  for (int k = t; k < Lk; k += NT) {
    const float v = ((cs[0][k] + cs[1][k]) + (cs[2][k] + cs[3][k])) * inv_lq;
    pbar[k] = v;
    if (P.pbarT) P.pbarT[((int64_t)b * Lk + k) * A.heads + head] = v;
  }
  FSTAMP(5)
  FSTAMP_RT(8)
}

// dq pass, query on the lane: G[k] = keep ? dpbar[k] / ((1-p) Lq) : 0;
// D = rowsum(P . G) (saved for the dk pass); dS = P . (G - D); dQ = scale dS K.
template <int HDP, int BF>
__global__ __launch_bounds__(NT) void attn_pool_bwd_dq_lean(const AttnArgs A) {
  constexpr int LS = HDP + 4;
  constexpr int HALF = HDP / 2;
  constexpr int NDT = HDP / 32;
  constexpr int NKT = PKC / 32;
  __shared__ __attribute__((aligned(16))) float Ks[PKC * LS];
  __shared__ __attribute__((aligned(16))) float gk[PKC];

  const AttnPair& P = A.p[blockIdx.y];
  const int qblocks = (P.Lq + 127) / 128;
  int bid = blockIdx.x;
  if (bid >= A.B * A.heads * qblocks) return;
  const int qb = bid % qblocks;
  bid /= qblocks;
  const int head = bid % A.heads, b = bid / A.heads;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, h = lane >> 5, c = lane & 31;
  const int hd = A.hd, col0 = head * hd;
  const int Lq = P.Lq, Lk = P.Lk, nkt = Lk >> 5;
  const int q = qb * 128 + w * 32 + c;
  const bool qvalid = q < Lq;
  const int qq = qvalid ? q : Lq - 1;
  const int64_t bh = (int64_t)b * A.heads + head;
  const int64_t rowidx = bh * Lq + qq;
  const float pdrop = A.drop_p;
  const float inv_keep = pdrop > 0.f && pdrop < 1.f ? 1.f / (1.f - pdrop) : 1.f;
  const float inv_lq = 1.f / (float)Lq;
  float* qrow = P.dq + ((int64_t)b * Lq + qq) * P.ldq + col0;

  if (P.kmask_mode == 1 && P.kmask[(int64_t)b * P.kmask_ld] == 0.f) {
    if (qvalid) {
      for (int d = h; d < hd; d += 2) qrow[d] = 0.f;
      if (h == 0) P.dsum[rowidx] = 0.f;
    }
    return;
  }
  load_rows<PKC, HDP, LS>(Ks, P.k + (int64_t)b * Lk * P.ldk + col0, Lk, P.ldk, 0, hd, true);
  for (int k = t; k < PKC; k += NT) gk[k] = k < Lk ? P.dpbar[bh * Lk + k] * inv_keep * inv_lq : 0.f;
  __syncthreads();
  if (qb * 128 + w * 32 >= Lq) return;
  float qf[HALF];
  load_frag_vec<HALF>(qf, P.q + ((int64_t)b * Lq + qq) * P.ldq + col0 + h * HALF);
  const float lse = P.lse[rowidx];
  const float lse2 = (!qvalid || lse == -INFINITY) ? INFINITY : lse * LOG2E;
  const float c2 = A.scale * LOG2E;
  uint4 kw = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
  if (P.keep_bits && pdrop > 0.f) kw = *reinterpret_cast<const uint4*>(P.keep_bits + rowidx * 4);
  const uint32_t kwa[4] = {kw.x, kw.y, kw.z, kw.w};
  float pr[NKT][16];
  float D = 0.f;
  // software pipeline: the next key tile's S chain is issued before this tile's VALU work
  f32x16 s_nx = dot_rows<HALF, BF>(Ks + c * LS + h * HALF, qf, zero16());
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    if (kt < nkt) {
      const f32x16 s = s_nx;
      if (kt + 1 < nkt) s_nx = dot_rows<HALF, BF>(Ks + ((kt + 1) * 32 + c) * LS + h * HALF, qf, zero16());
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 gv = *reinterpret_cast<const float4*>(gk + kt * 32 + 8 * g + 4 * h);
        const float gg[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 4 * g + j;
          const float p = fast_exp2(fmaf(s[r], c2, -lse2));
          pr[kt][r] = p;
          const bool keep = (kwa[kt] >> (8 * g + 4 * h + j)) & 1u;
          D += keep ? p * gg[j] : 0.f;
        }
      }
    }
  }
  D = sum_xor32(D);
  if (qvalid && h == 0) P.dsum[rowidx] = D;
  f32x16 dq[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) dq[dt] = zero16();
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    if (kt >= nkt) break;
    float ds[16];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const float4 gv = *reinterpret_cast<const float4*>(gk + kt * 32 + 8 * g + 4 * h);
      const float gg[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = 4 * g + j;
        const bool keep = (kwa[kt] >> (8 * g + 4 * h + j)) & 1u;
        ds[r] = pr[kt][r] * ((keep ? gg[j] : 0.f) - D);
      }
    }
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
MMF_CHAIN16(dq[dt], Ks[(kt * 32 + acc_row(r, h)) * LS + dt * 32 + c], ds[r])
  }
  if (!qvalid) return;
  const float scale = A.scale;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d0 = dt * 32 + 8 * g + 4 * h;
      if (d0 + 3 < hd)
        *reinterpret_cast<float4*>(qrow + d0) = make_float4(dq[dt][4 * g] * scale, dq[dt][4 * g + 1] * scale,
                                                            dq[dt][4 * g + 2] * scale, dq[dt][4 * g + 3] * scale);
    }
}

// dk pass, key on the lane: dK = scale * dS^T Q, dS = P . (G - D).
template <int HDP, int BF>
__global__ __launch_bounds__(NT) void attn_pool_bwd_dk_lean(const AttnArgs A) {
  constexpr int QC = 128;
  constexpr int LS = HDP + 4;
  constexpr int HALF = HDP / 2;
  constexpr int NDT = HDP / 32;
  __shared__ __attribute__((aligned(16))) float Qs[QC * LS];
  __shared__ __attribute__((aligned(16))) float lse_s[QC];
  __shared__ __attribute__((aligned(16))) float dsum_s[QC];
  __shared__ __attribute__((aligned(16))) uint32_t kw_t[4 * QC];   // [key word][query]

  const AttnPair& P = A.p[blockIdx.y];
  const int bid = blockIdx.x;
  if (bid >= A.B * A.heads) return;
  const int head = bid % A.heads, b = bid / A.heads;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, h = lane >> 5, c = lane & 31;
  const int hd = A.hd, col0 = head * hd;
  const int Lq = P.Lq, Lk = P.Lk;
  const int key = w * 32 + c;
  const bool wave_active = w * 32 < Lk;
  const int kk = wave_active ? key : 0;
  const int64_t bh = (int64_t)b * A.heads + head;
  const float pdrop = A.drop_p;
  const bool use_bits = P.keep_bits && pdrop > 0.f;
  const float inv_keep = pdrop > 0.f && pdrop < 1.f ? 1.f / (1.f - pdrop) : 1.f;
  const float inv_lq = 1.f / (float)Lq;
  const float c2 = A.scale * LOG2E;

  f32x16 dk[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) dk[dt] = zero16();
  const bool sample_masked = (P.kmask_mode == 1 && P.kmask[(int64_t)b * P.kmask_ld] == 0.f);
  if (!sample_masked) {
    float kf[HALF];
    load_frag_vec<HALF>(kf, P.k + ((int64_t)b * Lk + kk) * P.ldk + col0 + h * HALF);
    const float gkey = P.dpbar[bh * Lk + kk] * inv_keep * inv_lq;
    for (int qbase = 0; qbase < Lq; qbase += QC) {
      __syncthreads();
      load_rows<QC, HDP, LS>(Qs, P.q + (int64_t)b * Lq * P.ldq + col0, Lq, P.ldq, qbase, hd, true);
      for (int i = t; i < QC; i += NT) {
        const int qq = qbase + i;
        const float lse = qq < Lq ? P.lse[bh * Lq + qq] : -INFINITY;
        lse_s[i] = lse == -INFINITY ? INFINITY : lse * LOG2E;
        dsum_s[i] = qq < Lq ? P.dsum[bh * Lq + qq] : 0.f;
      }
      for (int i = t; i < QC * 4; i += NT) {
        const int qi = i >> 2, wd = i & 3;
        kw_t[wd * QC + qi] = (use_bits && qbase + qi < Lq) ? P.keep_bits[(bh * Lq + qbase + qi) * 4 + wd] : 0xFFFFFFFFu;
      }
      __syncthreads();
      if (!wave_active) continue;
      const int nqt = (min(QC, Lq - qbase) + 31) / 32;
      // software pipeline: the next tile's S chain is issued before this tile's VALU work
      f32x16 s_nx = dot_rows<HALF, BF>(Qs + c * LS + h * HALF, kf, zero16());
      for (int qt = 0; qt < nqt; ++qt) {
        const f32x16 s = s_nx;
        if (qt + 1 < nqt) s_nx = dot_rows<HALF, BF>(Qs + ((qt + 1) * 32 + c) * LS + h * HALF, kf, zero16());
        float ds[16];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int q0 = qt * 32 + 8 * g + 4 * h;
          const float4 l4 = *reinterpret_cast<const float4*>(lse_s + q0);
          const float4 d4 = *reinterpret_cast<const float4*>(dsum_s + q0);
          const uint4 w4 = *reinterpret_cast<const uint4*>(kw_t + w * QC + q0);
          const float ll[4] = {l4.x, l4.y, l4.z, l4.w};
          const float dd[4] = {d4.x, d4.y, d4.z, d4.w};
          const uint32_t ww[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int r = 4 * g + j;
            const float p = fast_exp2(fmaf(s[r], c2, -ll[j]));
            const bool keep = (ww[j] >> c) & 1u;
            ds[r] = p * ((keep ? gkey : 0.f) - dd[j]);
          }
        }
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
MMF_CHAIN16(dk[dt], ds[r], Qs[(qt * 32 + acc_row(r, h)) * LS + dt * 32 + c])
      }
    }
  }
  if (!wave_active) return;
  const float scale = A.scale;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
    const int d = dt * 32 + c;
    if (d >= hd) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int kr = w * 32 + acc_row(r, h);
      if (kr < Lk) P.dk[((int64_t)b * Lk + kr) * P.ldk + col0 + d] = dk[dt][r] * scale;
    }
  }
}

// Fused lean backward (Lq <= 128, every key valid, Lk % 32 == 0, Lk <= 128): one
// workgroup per (pair, sample, head) computes P and dS ONCE, query on the lane
// (as the dq pass), and produces both gradients from them:
//   dQ = scale dS K   straight from the registers (dS is the MFMA B operand);
//   dK = scale dS^T Q through a transposed dS image in LDS, built in four
//        32-query quarters ([key][32 + 4] floats, ds_write_b32 from the
//        accumulator layout, ds_read_b128 as the A operand of the key-on-lane
//        contraction).
// Against the two passes it saves one S = Q K^T recompute (MFMA), one exp /
// keep-bit pass (VALU), one read of Q, K, LSE and the keep words, and the D
// round trip.  LDS at hd <= 32: K and Q images, 2 x 18 KB (the dS^T quarters
// reuse the K image) -> 4 workgroups per CU, whose load phases hide each other.
// Everything one (pair, sample, head) item of the fused lean backward reads from
// memory, issued at once into registers (one round trip instead of one per
// image / side array): the K and Q head slices, dpbar, LSE, the keep words and
// the sample's modality mask.
template <int HDP, bool PST = false>
struct FusedLoads {
  static constexpr int PER = PKC * (HDP / 4) / NT;   // float4 slots per thread and image
  float4 k[PER], q[PER];
  float gk, lse, msk;
  uint4 kw;
};

template <int HDP, bool PST>
__device__ __forceinline__ void fused_issue_loads(const AttnArgs& A, const AttnPair& P, int b, int head, int c,
                                                  FusedLoads<HDP, PST>& L) {
  constexpr int C4 = HDP / 4;
  const int t = threadIdx.x, w = t >> 6;
  const int hd = A.hd, col0 = head * hd;
  const int Lq = P.Lq, Lk = P.Lk;
  const float* kb = P.k + (int64_t)b * Lk * P.ldk + col0;
  const float* qb = P.q + (int64_t)b * Lq * P.ldq + col0;
  // (32-bit element offsets from the wave-uniform bases: one v_mad per load instead of a
  // 64-bit address computation each)
#pragma unroll
  for (int i = 0; i < FusedLoads<HDP, PST>::PER; ++i) {
    const int idx = t + i * NT;
    const int r = idx / C4, c4 = (idx % C4) * 4;
    L.k[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    L.q[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < Lk && c4 < hd) L.k[i] = *reinterpret_cast<const float4*>(kb + (uint32_t)(r * P.ldk + c4));
    if (r < Lq && c4 < hd) L.q[i] = *reinterpret_cast<const float4*>(qb + (uint32_t)(r * P.ldq + c4));
  }
  const int q = w * 32 + c;
  const int qq = q < Lq ? q : Lq - 1;
  const int64_t bh = (int64_t)b * A.heads + head;
  const int64_t rowidx = bh * Lq + qq;
  const float pdrop = A.drop_p;
  const float inv_keep = pdrop > 0.f && pdrop < 1.f ? 1.f / (1.f - pdrop) : 1.f;
  L.gk = t < Lk ? P.dpbar[bh * Lk + t] * inv_keep / (float)Lq : 0.f;   // PKC <= NT
  L.lse = P.lse[rowidx];
  L.kw = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
  if (P.keep_bits && pdrop > 0.f) L.kw = *reinterpret_cast<const uint4*>(P.keep_bits + rowidx * 4);
  L.msk = P.kmask_mode == 1 ? P.kmask[(int64_t)b * P.kmask_ld] : 1.f;
}

// One (pair, sample, head) item of the fused lean backward from its issued loads;
// Ks / Qs are [PKC][HDP + 4] LDS images (Ks doubles as the dS^T quarter image),
// gk [PKC].  Called by every thread of the workgroup (it holds barriers).
template <int HDP, int BF, bool PST = false>
__device__ __forceinline__ void fused_lean_item(const AttnArgs& A, const AttnPair& P, int b, int head, float* Ks,
                                                float* Qs, float* gk, int h, int c, const FusedLoads<HDP, PST>& LD) {
  constexpr int LS = HDP + 4;
  constexpr int HALF = HDP / 2;
  constexpr int NDT = HDP / 32;
  constexpr int NKT = PKC / 32;
  constexpr int TS = 32 + 4;   // dS^T image row pitch (floats): one wave's 32 queries
  constexpr int C4 = HDP / 4;
  static_assert(PKC * TS <= PKC * LS, "the dS^T quarter image reuses the K image");
  float* const dsT = Ks;
  const int t = threadIdx.x, w = t >> 6;
  const int hd = A.hd, col0 = head * hd;
  const int Lq = P.Lq, Lk = P.Lk, nkt = Lk >> 5;
  const int q = w * 32 + c;
  const bool qvalid = q < Lq;
  const int qq = qvalid ? q : Lq - 1;
  const float pdrop = A.drop_p;
  const float scale = A.scale;
  float* qrow = P.dq + ((int64_t)b * Lq + qq) * P.ldq + col0;
  const int key = w * 32 + c;                 // dK phase: this wave's keys
  const bool kwave = w * 32 < Lk;

  BSTAMP_RT(7)
  BSTAMP(0)
  BSTAMP_ID()
  if (LD.msk == 0.f) {
    // fully masked sample: P = 0 -> dQ = dK = 0
    if (qvalid)
      for (int d = h; d < hd; d += 2) qrow[d] = 0.f;
    if (kwave)
      for (int d = h; d < hd; d += 2) P.dk[((int64_t)b * Lk + key) * P.ldk + col0 + d] = 0.f;
    return;
  }
#pragma unroll
  for (int i = 0; i < FusedLoads<HDP, PST>::PER; ++i) {
    const int idx = t + i * NT;
    const int off = (idx / C4) * LS + (idx % C4) * 4;
    *reinterpret_cast<float4*>(&Ks[off]) = LD.k[i];
    *reinterpret_cast<float4*>(&Qs[off]) = LD.q[i];
  }
  if (t < PKC) gk[t] = LD.gk;
  const float lse2 = (!qvalid || LD.lse == -INFINITY) ? INFINITY : LD.lse * LOG2E;
  // keep words shifted to this lane half once: the per-element tests are constant-offset bit
  // extracts (a variable shift made the compiler keep 16 precomputed masks live)
  uint32_t kwh[4] = {LD.kw.x >> (4 * h), LD.kw.y >> (4 * h), LD.kw.z >> (4 * h), LD.kw.w >> (4 * h)};
  (void)pdrop;
  float pr[NKT][16];
  float4 pld[PST ? 16 : 1];
  if constexpr (PST) {
    // this wave's query tile of the forward's stored P: 16 x 1-KB wave loads, issued once the
    // K / Q image registers are free (before the barrier; the scheduler barrier keeps them there)
    __builtin_amdgcn_sched_barrier(0);
    const float* pst = P.pstore + (((int64_t)b * A.heads + head) * ((Lq + 31) / 32) + w) * 4096 + (t & 63) * 4;
    // (unconditional: the blob reserves 4 key tiles per query tile; tiles past nkt are read
    // and discarded below -- a guarded load per slot made the compiler branch and drain vmcnt)
#pragma unroll
    for (int i = 0; i < 16; ++i) pld[i] = *reinterpret_cast<const float4*>(pst + (i >> 2) * 1024 + (i & 3) * 256);
  }
  __syncthreads();
  BSTAMP(1)

  float D = 0.f;
  if constexpr (PST) {
    // P from the forward (no S recompute); invalid query lanes hold 0
    (void)lse2;
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 pv = pld[kt * 4 + g];
        const float4 gv = *reinterpret_cast<const float4*>(gk + kt * 32 + 8 * g + 4 * h);
        const float pp[4] = {pv.x, pv.y, pv.z, pv.w};
        const float gg[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float p = kt < nkt ? pp[j] : 0.f;
          pr[kt][4 * g + j] = p;
          D += p * keep_sel(kwh[kt], 8 * g + j, gg[j]);
        }
      }
    }
  } else {
    float qf[HALF];
    load_frag_vec<HALF>(qf, Qs + q * LS + h * HALF);
    const float c2 = scale * LOG2E;
    // one accumulator per key tile (tile kt + 1's chain issued before tile kt's exp / D work):
    // a rotating "next" accumulator was copied each tile, and the copy waited (s_nop) for the
    // chain it had just issued to finish
    f32x16 sacc[NKT];
    sacc[0] = dot_rows<HALF, BF>(Ks + c * LS + h * HALF, qf, zero16());
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      if (kt < nkt) {
        if (kt + 1 < NKT && kt + 1 < nkt)
          sacc[kt + 1] = dot_rows<HALF, BF>(Ks + ((kt + 1) * 32 + c) * LS + h * HALF, qf, zero16());
        const f32x16& s = sacc[kt];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 gv = *reinterpret_cast<const float4*>(gk + kt * 32 + 8 * g + 4 * h);
          const float gg[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int r = 4 * g + j;
            const float p = fast_exp2(fmaf(s[r], c2, -lse2));
            pr[kt][r] = p;
            D += p * keep_sel(kwh[kt], 8 * g + j, gg[j]);   // keep ? p * G : 0
          }
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) pr[kt][r] = 0.f;
      }
    }
  }
  D = sum_xor32(D);
  // the dQ chains' K-image reads stay below (hoisted above the D loop they held 64 more
  // registers alive across it and spilled), and the keep tests are redone below rather than
  // kept from the D loop (64 lane masks = 128 SGPRs, spilled); the empty asm makes the
  // compiler treat the words as new values
  if constexpr (PST) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) asm volatile("" : "+v"(kwh[kt]));
  }
  BSTAMP(2)
  BSTAMP(3)
  // dQ = scale dS K (query on the lane; dS is the B operand); dS = P . (G - D) is formed
  // tile by tile, right before its chain, so that VALU work overlaps the previous chain
  {
    f32x16 dq[NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) dq[dt] = zero16();
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
      if (kt < nkt) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float4 gv = *reinterpret_cast<const float4*>(gk + kt * 32 + 8 * g + 4 * h);
          const float gg[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int r = 4 * g + j;
            pr[kt][r] = pr[kt][r] * (keep_sel(kwh[kt], 8 * g + j, gg[j]) - D);
          }
        }
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
MMF_CHAIN16(dq[dt], Ks[(kt * 32 + acc_row(r, h)) * LS + dt * 32 + c], pr[kt][r])
      }
    }
    if (qvalid) {
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d0 = dt * 32 + 8 * g + 4 * h;
          if (d0 + 3 < hd)
            *reinterpret_cast<float4*>(qrow + d0) = make_float4(dq[dt][4 * g] * scale, dq[dt][4 * g + 1] * scale,
                                                                dq[dt][4 * g + 2] * scale, dq[dt][4 * g + 3] * scale);
        }
    }
  }
  BSTAMP(4)
  // dK = scale dS^T Q (key on the lane), over four 32-query quarters of dS^T
  // staged in the K image (K is dead once every wave is past the dQ phase)
  f32x16 dk[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) dk[dt] = zero16();
  for (int qw = 0; qw < 4; ++qw) {
    if (qw * 32 >= Lq) break;   // uniform: no queries left
    __syncthreads();            // K image (qw = 0) / previous quarter no longer read
    if (w == qw) {
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) dsT[(kt * 32 + acc_row(r, h)) * TS + c] = pr[kt][r];
    }
    __syncthreads();
    if (kwave) {
// k-steps (g, j) = query 8g + 4h + j of the quarter; chains of eight over g pairs
#pragma unroll
      for (int gp = 0; gp < 2; ++gp) {
        float av[8], qv[NDT][8];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int g = 2 * gp + u;
          const float4 a4 = *reinterpret_cast<const float4*>(dsT + key * TS + 8 * g + 4 * h);
          av[4 * u + 0] = a4.x; av[4 * u + 1] = a4.y; av[4 * u + 2] = a4.z; av[4 * u + 3] = a4.w;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int qg = qw * 32 + 8 * g + 4 * h + j;
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) qv[dt][4 * u + j] = Qs[qg * LS + dt * 32 + c];
          }
        }
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) dk[dt] = mfma_k16<BF>(av, qv[dt], dk[dt]);
      }
    }
  }
  BSTAMP(5)
  if (!kwave) return;
  // the wave's 32 key rows from a uniform base; per store a 32-bit offset (row multiples of
  // ldk are scalar)
  float* const dkb = P.dk + ((int64_t)b * Lk + w * 32) * P.ldk + col0;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
    const int d = dt * 32 + c;
    if (d >= hd) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r)
      dkb[(uint32_t)(acc_row(r, h) * P.ldk + d)] = dk[dt][r] * scale;
  }
  BSTAMP(6)
  BSTAMP_RT(8)
}

template <int HDP, int BF, bool PST = false>
__global__ __launch_bounds__(NT, 4) void attn_pool_bwd_fused_lean(const AttnArgs A) {
  __shared__ __attribute__((aligned(16))) float Ks[PKC * (HDP + 4)];   // K, then the dS^T quarters
  __shared__ __attribute__((aligned(16))) float Qs[PKC * (HDP + 4)];
  __shared__ __attribute__((aligned(16))) float gk[PKC];
  const int bid = blockIdx.x;
  if (bid >= A.B * A.heads) return;
  const int lane = threadIdx.x & 63;
  const AttnPair& P = A.p[blockIdx.y];
  FusedLoads<HDP, PST> LD;
  fused_issue_loads<HDP, PST>(A, P, bid / A.heads, bid % A.heads, lane & 31, LD);
  fused_lean_item<HDP, BF, PST>(A, P, bid / A.heads, bid % A.heads, Ks, Qs, gk, lane >> 5, lane & 31, LD);
}

// "name<a, b>" -> "name<a, b, ARG>" ("name<>" -> "name<ARG>"): the rocprof name of an
// instantiation (ARG: the precision 0 | 1 | 2, or a trailing bool); stable storage for
// the profiler tags.
const char* with_arg(const char* base, const char* arg) {
  static std::mutex mu;
  static std::map<std::string, std::string> names;
  std::lock_guard<std::mutex> lk(mu);
  std::string key = std::string(base) + "|" + arg;
  auto& slot = names[key];
  if (slot.empty()) {
    std::string b(base);
    const size_t gt = b.rfind('>');
    if (b.size() >= 2 && b.compare(b.size() - 2, 2, "<>") == 0)
      slot = b.substr(0, b.size() - 1) + arg + ">";
    else
      slot = gt == std::string::npos ? b : b.substr(0, gt) + ", " + arg + ">";
  }
  return slot.c_str();
}

enum class Kind { Fwd, Probs, Prep, Dkv, Dq, PoolFwd, PoolDq, PoolDk, PoolFused, PoolLse, PoolColsum, PoolDqLong };

hipError_t launch_generic(Kind kind, const AttnPair* pairs, int npairs, int B, int heads, int hd,
                          float scale, float drop_p, const RngSnap* rng, hipStream_t st, bool words_ready = false) {
  if (hd > 64) return hipErrorInvalidValue;
  const bool small = hd <= 32;
  bool prep_vec = (hd % 4 == 0) && (((hd / 4) & (hd / 4 - 1)) == 0);
  for (int i = 0; i < npairs && prep_vec; ++i)
    prep_vec = (pairs[i].ldo % 4 == 0) && (((uintptr_t)pairs[i].dout & 15) == 0) &&
               (((uintptr_t)pairs[i].o & 15) == 0) && pairs[i].ldo == heads * hd;
  // lean pooled kernels: every pair has all keys valid and float4-able rows
  const bool pooled = kind == Kind::PoolFwd || kind == Kind::PoolDq || kind == Kind::PoolDk || kind == Kind::PoolFused;
  bool lean = pooled && (hd % 4 == 0);
  for (int i = 0; i < npairs && lean; ++i) {
    const AttnPair& P = pairs[i];
    lean = (P.Lk % 32 == 0) && P.Lk <= PKC && P.kmask_mode != 2 && (P.ldq % 4 == 0) && (P.ldk % 4 == 0) &&
           (((uintptr_t)P.q & 15) == 0) && (((uintptr_t)P.k & 15) == 0) &&
           (kind != Kind::PoolDq || (((uintptr_t)P.dq & 15) == 0));
  }
  // lean long-key kernels: whole 32-key tiles and no per-key mask in every pair
  bool long_lean = kind == Kind::PoolLse || kind == Kind::PoolDqLong;
  for (int i = 0; i < npairs && long_lean; ++i) long_lean = (pairs[i].Lk % 32 == 0) && pairs[i].kmask_mode != 2;
  if (kind == Kind::PoolFused) {
    // lean conditions plus a single query block and float4-able dQ rows
    for (int i = 0; i < npairs && lean; ++i)
      lean = pairs[i].Lq <= 128 && (pairs[i].ldq % 4 == 0) && (((uintptr_t)pairs[i].dq & 15) == 0);
    if (!lean) return hipErrorNotSupported;
  }
  // stored probabilities (every pair of the launch has them, or none): the lean forward writes,
  // the fused backward reads P instead of recomputing S
  int npst = 0;
  for (int i = 0; i < npairs; ++i) npst += pairs[i].pstore != nullptr;
  if (npst != 0 && (npst != npairs || !lean || (kind != Kind::PoolFwd && kind != Kind::PoolFused)))
    return hipErrorInvalidValue;
  const bool pst = npst != 0;
  int done = 0;
  while (done < npairs) {
    AttnArgs a;
    memset(&a, 0, sizeof(a));
    int n = 0;
    int64_t maxblk = 0;
    while (done < npairs && n < ATTN_MAX_PAIRS) {
      a.p[n] = pairs[done++];
      const AttnPair& P = a.p[n];
      int64_t nb;
      if (kind == Kind::Prep)
        nb = prep_vec ? ((int64_t)B * P.Lq * (heads * hd / 4) + NT - 1) / NT
                      : ((int64_t)B * P.Lq * heads + NT - 1) / NT;
      else if (kind == Kind::Dkv || kind == Kind::PoolDk || kind == Kind::PoolColsum)
        nb = (int64_t)B * heads * ((P.Lk + 127) / 128);
      else if (kind == Kind::PoolFwd || kind == Kind::PoolFused) nb = (int64_t)B * heads;
      else nb = (int64_t)B * heads * ((P.Lq + 127) / 128);
      // one-chunk pooled kernels hold every key in LDS; the long-key kinds stream them
      if ((kind == Kind::PoolFwd || kind == Kind::PoolDq || kind == Kind::PoolFused) && P.Lk > PKC)
        return hipErrorInvalidValue;
      // long-key keep words: kw_ld words of 32 keys per query row
      if ((kind == Kind::PoolLse || kind == Kind::PoolColsum || kind == Kind::PoolDqLong || kind == Kind::PoolDk) &&
          P.keep_bits != nullptr && P.kw_ld < (P.Lk + 31) / 32)
        return hipErrorInvalidValue;
      if ((kind == Kind::PoolLse || kind == Kind::PoolColsum || kind == Kind::PoolDqLong || kind == Kind::PoolDk) &&
          drop_p > 0.f && P.keep_bits == nullptr)
        return hipErrorInvalidValue;
      if (nb > maxblk) maxblk = nb;
      ++n;
    }
    a.npairs = n;
    a.B = B;
    a.heads = heads;
    a.hd = hd;
    a.scale = scale;
    a.drop_p = drop_p;
    a.rng = rng;
    a.nblk = (int)maxblk;
    if (maxblk <= 0) continue;
    dim3 grid((unsigned)maxblk, n);
    // algorithmic work of this launch (no S recompute counted)
    double fl = 0.0, by = 0.0;
    const double H = (double)heads * hd;
    for (int i = 0; i < n; ++i) {
      const double lq = a.p[i].Lq, lk = a.p[i].Lk, bq = (double)B * lq * H, bk = (double)B * lk * H;
      const double qk = 2.0 * B * lq * lk * H;   // one (B, h, Lq, Lk, hd) contraction
      switch (kind) {
        case Kind::Fwd: fl += 2 * qk; by += 4 * (2 * bq + 2 * bk); break;               // Q K V -> O
        case Kind::Probs: fl += 2 * qk; by += 4 * (2 * bq + 2 * bk + B * heads * lq * lk); break;
        case Kind::Prep: fl += 2.0 * bq; by += 4 * 2 * bq; break;                         // dO, O -> D
        case Kind::Dkv: fl += 3 * qk; by += 4 * (3 * bq + 4 * bk); break;               // Q K V dO -> dK dV
        case Kind::Dq: fl += qk; by += 4 * (3 * bq + 2 * bk); break;                    // Q K V dO -> dQ
        case Kind::PoolFwd: fl += qk; by += 4 * (bq + bk); break;                         // Q K -> lse, pbar
        case Kind::PoolDq: fl += qk; by += 4 * (2 * bq + bk); break;                      // Q K -> dQ
        case Kind::PoolDk: fl += qk; by += 4 * (bq + 2 * bk); break;                      // Q K -> dK
        // (the stored-P plan's P blob is the plan's own intermediate, not the reference algorithm's
        // operand bytes: not counted; PMC traffic shows it)
        case Kind::PoolFused: fl += 2 * qk; by += 4 * (2 * bq + 2 * bk); break;           // Q K -> dQ dK
        case Kind::PoolLse: fl += qk; by += 4 * (bq + bk); break;                         // Q K -> lse
        case Kind::PoolColsum: by += 4 * (bq + bk); break;                                // (S recomputed) -> pbar
        case Kind::PoolDqLong: fl += qk; by += 4 * (2 * bq + bk); break;                  // Q K -> dQ
      }
    }
    static const char* const kNames[12][4] = {
        {"attn_fwd_kernel<32, 0>", "attn_fwd_kernel<64, 0>", "attn_fwd_kernel<32, 0>", "attn_fwd_kernel<64, 0>"},
        {"attn_fwd_kernel<32, 1>", "attn_fwd_kernel<64, 1>", "attn_fwd_kernel<32, 1>", "attn_fwd_kernel<64, 1>"},
        {"attn_bwd_prep_kernel", "attn_bwd_prep_kernel", "attn_bwd_prep_vec_kernel", "attn_bwd_prep_vec_kernel"},
        {"attn_bwd_dkv_kernel<32>", "attn_bwd_dkv_kernel<64>", "attn_bwd_dkv_kernel<32>", "attn_bwd_dkv_kernel<64>"},
        {"attn_bwd_dq_kernel<32>", "attn_bwd_dq_kernel<64>", "attn_bwd_dq_kernel<32>", "attn_bwd_dq_kernel<64>"},
        {"attn_pool_fwd_kernel<32>", "attn_pool_fwd_kernel<64>", "attn_pool_fwd_lean<32>", "attn_pool_fwd_lean<64>"},
        {"attn_pool_bwd_dq_kernel<32>", "attn_pool_bwd_dq_kernel<64>", "attn_pool_bwd_dq_lean<32>",
         "attn_pool_bwd_dq_lean<64>"},
        {"attn_pool_bwd_dk_kernel<32>", "attn_pool_bwd_dk_kernel<64>", "attn_pool_bwd_dk_lean<32>",
         "attn_pool_bwd_dk_lean<64>"},
        {"", "", "attn_pool_bwd_fused_lean<32>", "attn_pool_bwd_fused_lean<64>"},
        {"attn_poolL_lse_kernel<32>", "attn_poolL_lse_kernel<64>", "", ""},
        {"attn_poolL_colsum_kernel<32>", "attn_poolL_colsum_kernel<64>", "", ""},
        {"attn_poolL_dq_kernel<32>", "attn_poolL_dq_kernel<64>", "", ""}};
    const bool alt = kind == Kind::Prep ? prep_vec : (lean && kind <= Kind::PoolFused);
    const int pr = math_mode();
// one launch of the instantiation for the call's precision: PRV names the kernel's
// int precision template argument inside KERNEL
#define MMF_PR_LAUNCH(...)                                                                   \
  switch (pr) {                                                                              \
    case 2: { constexpr int PRV = 2; mmf_launch((__VA_ARGS__), grid, dim3(NT), 0, st, a); } break; \
    case 1: { constexpr int PRV = 1; mmf_launch((__VA_ARGS__), grid, dim3(NT), 0, st, a); } break; \
    default: { constexpr int PRV = 0; mmf_launch((__VA_ARGS__), grid, dim3(NT), 0, st, a); } break; \
  }
    const char* kname = kNames[(int)kind][(alt ? 2 : 0) + (small ? 0 : 1)];
    const char* pname = with_arg(kname, pr == 2 ? "2" : (pr == 1 ? "1" : "0"));
    if (long_lean) pname = with_arg(pname, "true");   // "<hd, pr, true>": the LEAN instantiation
    if (kind == Kind::PoolFwd && lean) pname = with_arg(pname, a.drop_p > 0.f ? "true" : "false");   // DROP
    if (kind == Kind::PoolFwd && lean) pname = with_arg(pname, pst ? "true" : "false");              // PST
    if (kind == Kind::PoolFwd && lean)   // KW (rocprofv3 prints every template argument)
      pname = with_arg(pname, (!pst && a.drop_p > 0.f && words_ready) ? "true" : "false");
    if (kind == Kind::PoolFused) pname = with_arg(pname, pst ? "true" : "false");                    // PST
    ProfLaunch prof_(st, pname, fl, by);
    switch (kind) {
      case Kind::PoolLse:
        if (long_lean) {
          if (small) { MMF_PR_LAUNCH(attn_poolL_lse_kernel<32, PRV, true>) }
          else { MMF_PR_LAUNCH(attn_poolL_lse_kernel<64, PRV, true>) }
        } else {
          if (small) { MMF_PR_LAUNCH(attn_poolL_lse_kernel<32, PRV>) }
          else { MMF_PR_LAUNCH(attn_poolL_lse_kernel<64, PRV>) }
        }
        break;
      case Kind::PoolColsum:
        if (small) { MMF_PR_LAUNCH(attn_poolL_colsum_kernel<32, PRV>) }
        else { MMF_PR_LAUNCH(attn_poolL_colsum_kernel<64, PRV>) }
        break;
      case Kind::PoolDqLong:
        if (long_lean) {
          if (small) { MMF_PR_LAUNCH(attn_poolL_dq_kernel<32, PRV, true>) }
          else { MMF_PR_LAUNCH(attn_poolL_dq_kernel<64, PRV, true>) }
        } else {
          if (small) { MMF_PR_LAUNCH(attn_poolL_dq_kernel<32, PRV>) }
          else { MMF_PR_LAUNCH(attn_poolL_dq_kernel<64, PRV>) }
        }
        break;
      case Kind::Fwd:
        if (small) { MMF_PR_LAUNCH(attn_fwd_kernel<32, 0, PRV>) }
        else { MMF_PR_LAUNCH(attn_fwd_kernel<64, 0, PRV>) }
        break;
      case Kind::Probs:
        if (small) { MMF_PR_LAUNCH(attn_fwd_kernel<32, 1, PRV>) }
        else { MMF_PR_LAUNCH(attn_fwd_kernel<64, 1, PRV>) }
        break;
      case Kind::Prep:
        if (prep_vec) mmf_launch(attn_bwd_prep_vec_kernel, grid, dim3(NT), 0, st, a);
        else mmf_launch(attn_bwd_prep_kernel, grid, dim3(NT), 0, st, a);
        break;
      case Kind::Dkv:
        if (small) { MMF_PR_LAUNCH(attn_bwd_dkv_kernel<32, PRV>) }
        else { MMF_PR_LAUNCH(attn_bwd_dkv_kernel<64, PRV>) }
        break;
      case Kind::Dq:
        if (small) { MMF_PR_LAUNCH(attn_bwd_dq_kernel<32, PRV>) }
        else { MMF_PR_LAUNCH(attn_bwd_dq_kernel<64, PRV>) }
        break;
      case Kind::PoolFwd:
        if (lean && !pst && a.drop_p > 0.f && words_ready) {
          if (small) { MMF_PR_LAUNCH(attn_pool_fwd_lean<32, PRV, true, false, true>) }
          else { MMF_PR_LAUNCH(attn_pool_fwd_lean<64, PRV, true, false, true>) }
        } else if (lean && pst && a.drop_p > 0.f) {
          if (small) { MMF_PR_LAUNCH(attn_pool_fwd_lean<32, PRV, true, true>) }
          else { MMF_PR_LAUNCH(attn_pool_fwd_lean<64, PRV, true, true>) }
        } else if (lean && pst) {
          if (small) { MMF_PR_LAUNCH(attn_pool_fwd_lean<32, PRV, false, true>) }
          else { MMF_PR_LAUNCH(attn_pool_fwd_lean<64, PRV, false, true>) }
        } else if (lean && a.drop_p > 0.f) {
          if (small) { MMF_PR_LAUNCH(attn_pool_fwd_lean<32, PRV, true>) }
          else { MMF_PR_LAUNCH(attn_pool_fwd_lean<64, PRV, true>) }
        } else if (lean) {
          if (small) { MMF_PR_LAUNCH(attn_pool_fwd_lean<32, PRV, false>) }
          else { MMF_PR_LAUNCH(attn_pool_fwd_lean<64, PRV, false>) }
        }
        else if (small) { MMF_PR_LAUNCH(attn_pool_fwd_kernel<32, PRV>) }
        else { MMF_PR_LAUNCH(attn_pool_fwd_kernel<64, PRV>) }
        break;
      case Kind::PoolDq:
        if (lean && small) { MMF_PR_LAUNCH(attn_pool_bwd_dq_lean<32, PRV>) }
        else if (lean) { MMF_PR_LAUNCH(attn_pool_bwd_dq_lean<64, PRV>) }
        else if (small) { MMF_PR_LAUNCH(attn_pool_bwd_dq_kernel<32, PRV>) }
        else { MMF_PR_LAUNCH(attn_pool_bwd_dq_kernel<64, PRV>) }
        break;
      case Kind::PoolFused:
        if (pst) {
          if (small) { MMF_PR_LAUNCH(attn_pool_bwd_fused_lean<32, PRV, true>) }
          else { MMF_PR_LAUNCH(attn_pool_bwd_fused_lean<64, PRV, true>) }
        } else {
          if (small) { MMF_PR_LAUNCH(attn_pool_bwd_fused_lean<32, PRV>) }
          else { MMF_PR_LAUNCH(attn_pool_bwd_fused_lean<64, PRV>) }
        }
        break;
      case Kind::PoolDk:
        if (lean && small) { MMF_PR_LAUNCH(attn_pool_bwd_dk_lean<32, PRV>) }
        else if (lean) { MMF_PR_LAUNCH(attn_pool_bwd_dk_lean<64, PRV>) }
        else if (small) { MMF_PR_LAUNCH(attn_pool_bwd_dk_kernel<32, PRV>) }
        else { MMF_PR_LAUNCH(attn_pool_bwd_dk_kernel<64, PRV>) }
        break;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace

hipError_t launch_attn_fwd(const AttnPair* pairs, int npairs, int B, int heads, int hd, float scale,
                           float drop_p, const RngSnap* rng, hipStream_t st) {
  return launch_generic(Kind::Fwd, pairs, npairs, B, heads, hd, scale, drop_p, rng, st);
}

hipError_t launch_attn_probs(const AttnPair* pairs, int npairs, int B, int heads, int hd,
                             float scale, float drop_p, const RngSnap* rng, hipStream_t st) {
  return launch_generic(Kind::Probs, pairs, npairs, B, heads, hd, scale, drop_p, rng, st);
}

// pairs whose keys fit one LDS chunk (Lk <= PKC) vs the long-key kernels
static void split_by_keys(const AttnPair* pairs, int npairs, std::vector<AttnPair>& shortp,
                          std::vector<AttnPair>& longp) {
  for (int i = 0; i < npairs; ++i) (pairs[i].Lk > PKC ? longp : shortp).push_back(pairs[i]);
}

hipError_t launch_attn_pool_fwd(const AttnPair* pairs, int npairs, int B, int heads, int hd, float scale,
                                float drop_p, const RngSnap* rng, hipStream_t st, bool words_ready) {
  std::vector<AttnPair> sp, lp;
  split_by_keys(pairs, npairs, sp, lp);
  hipError_t e = hipSuccess;
  if (!sp.empty())
    e = launch_generic(Kind::PoolFwd, sp.data(), (int)sp.size(), B, heads, hd, scale, drop_p, rng, st, words_ready);
  if (e == hipSuccess && !lp.empty() && attn_long_fwd_ok(lp.data(), (int)lp.size(), hd, drop_p, rng))
    return launch_attn_long_fused_fwd(lp.data(), (int)lp.size(), B, heads, hd, scale, drop_p, rng, st, words_ready);
  for (const AttnPair& a : lp)   // bf16 Q / K rows only the one-pass kernels read
    if (a.qk_bf16) return hipErrorInvalidValue;
  if (e == hipSuccess && !lp.empty())
    e = launch_generic(Kind::PoolLse, lp.data(), (int)lp.size(), B, heads, hd, scale, drop_p, rng, st);
  if (e == hipSuccess && !lp.empty())
    e = launch_generic(Kind::PoolColsum, lp.data(), (int)lp.size(), B, heads, hd, scale, drop_p, rng, st);
  return e;
}

hipError_t launch_attn_pool_bwd(int stage, const AttnPair* pairs, int npairs, int B, int heads, int hd,
                                float scale, float drop_p, const RngSnap* rng, hipStream_t st) {
  // stage 2: both gradients in one pass when the fused lean kernel applies
  // (hipErrorNotSupported otherwise: run stages 0 and 1)
  std::vector<AttnPair> sp, lp;
  split_by_keys(pairs, npairs, sp, lp);
  if (stage == 2) {
    // every long-key pair on the one-pass bf16 kernel (attn_long.hip), or none: checked before
    // anything launches, so hipErrorNotSupported leaves the caller to run stages 0 and 1
    if (!lp.empty() && !attn_long_fused_ok(lp.data(), (int)lp.size(), hd, drop_p)) return hipErrorNotSupported;
    hipError_t e = hipSuccess;
    if (!sp.empty()) e = launch_generic(Kind::PoolFused, sp.data(), (int)sp.size(), B, heads, hd, scale, drop_p, rng, st);
    if (e == hipSuccess && !lp.empty())
      e = launch_attn_long_fused_bwd(lp.data(), (int)lp.size(), B, heads, hd, scale, drop_p, st);
    return e;
  }
  hipError_t e = hipSuccess;
  if (!sp.empty())
    e = launch_generic(stage == 0 ? Kind::PoolDq : Kind::PoolDk, sp.data(), (int)sp.size(), B, heads, hd, scale,
                       drop_p, rng, st);
  if (e == hipSuccess && !lp.empty())
    e = launch_generic(stage == 0 ? Kind::PoolDqLong : Kind::PoolDk, lp.data(), (int)lp.size(), B, heads, hd,
                       scale, drop_p, rng, st);
  return e;
}

hipError_t launch_attn_bwd_stage(int stage, const AttnPair* pairs, int npairs, int B, int heads, int hd,
                                 float scale, float drop_p, const RngSnap* rng, hipStream_t st) {
  const Kind k = stage == 0 ? Kind::Prep : (stage == 1 ? Kind::Dkv : Kind::Dq);
  return launch_generic(k, pairs, npairs, B, heads, hd, scale, drop_p, rng, st);
}

hipError_t launch_attn_bwd(const AttnPair* pairs, int npairs, int B, int heads, int hd, float scale,
                           float drop_p, const RngSnap* rng, hipStream_t st) {
  hipError_t e = launch_generic(Kind::Prep, pairs, npairs, B, heads, hd, scale, drop_p, rng, st);
  if (e != hipSuccess) return e;
  e = launch_generic(Kind::Dkv, pairs, npairs, B, heads, hd, scale, drop_p, rng, st);
  if (e != hipSuccess) return e;
  return launch_generic(Kind::Dq, pairs, npairs, B, heads, hd, scale, drop_p, rng, st);
}

}  // namespace mmf

// Occupancy the runtime reports for the C2 attention kernels (blocks per CU at 256
// threads): [0] fused backward, [1] pooled forward.  Diagnostic (scripts/attn_stamps.py).
extern "C" int mmf_attn_occupancy(int* out) {
  int a = 0, b = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&a, mmf::attn_pool_bwd_fused_lean<32, 0>, 256, 0) !=
          hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, mmf::attn_pool_fwd_lean<32, 0>, 256, 0) != hipSuccess)
    return 3;
  out[0] = a;
  out[1] = b;
  return 0;
}

#ifdef MMF_STAMPS
extern "C" int mmf_stamps_read(void* out, size_t bytes) {   // fused attention backward
  if (bytes > sizeof(mmf::g_mmf_stamps)) bytes = sizeof(mmf::g_mmf_stamps);
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mmf::g_mmf_stamps), bytes) == hipSuccess ? 0 : 3;
}
extern "C" int mmf_stamps_clear(void) {
  static unsigned long long zero[mmf::STAMP_WG][10];
  return hipMemcpyToSymbol(HIP_SYMBOL(mmf::g_mmf_stamps), zero, sizeof(zero)) == hipSuccess ? 0 : 3;
}
#endif
