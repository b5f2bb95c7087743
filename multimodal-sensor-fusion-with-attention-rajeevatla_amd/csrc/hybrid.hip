// HybridFusion C-ABI entry points (include/mmfusion.h): native orchestration of
// the forward and backward of src/fusion.py::HybridFusion (forward :331-427,
// compute_adaptive_weights :429-479) on the libmmfusion kernels.
//
// Two execution plans compute the same function:
//  * pooled (default; every key modality has L <= 128 and heads <= 8): the
//    attended features are consumed only through their mean over L, so
//    mean_q(P' V) W_o^T + b_o is evaluated as (pbar P_k) W_v^T ... on B rows
//    (attention.hip "Pooled-output attention", pool.hip).  No V / O / attended
//    (B, L, H) tensors exist and the backward needs no dO V^T / dV products.
//  * general (fallback): per-pair Q/K/V projections, flash attention
//    (O = softmax(QK^T) V), out_proj on every row, L-mean in the head.
// Both are exact reformulations (fp32 reassociation only) of the reference.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <unistd.h>

#include "capi_util.h"

using namespace mmf;

namespace {

// The plan switches read from the environment on every call (A/B and diagnostic knobs: they pick
// kernels and so the `saved` / `workspace` layouts).  Their fingerprint is what a caller stores in
// mmf_hybrid_desc.plan_flags when it sizes its buffers; an entry point whose current fingerprint
// differs refuses to run (MMF_EINVAL) instead of laying its buffers out differently from how the
// caller sized them (MMF_PSTORE set after HybridTrainStep allocated `saved`
// overflowed it).  The sum of per-entry FNV-1a hashes of "NAME=VALUE": independent of the order
// of `environ`, and 0 with none of them set.
const char* const kPlanKnobs[] = {
    "MMF_PSTORE", "MMF_NO_LONG_FUSED", "MMF_NO_FUSED_BWD", "MMF_NO_BF16_QK", "MMF_NO_GEMM_B16",
    "MMF_QK_CAT", "MMF_NO_DQK_B16", "MMF_NO_PROJ_B16", "MMF_NO_PCOL", "MMF_NO_POOLE", "MMF_POOLE_FLAT",
    "MMF_NO_L1_LEAN", "MMF_WGRAD_SPLIT_CAP", "MMF_NO_SIDE_STREAM", "MMF_SIDE_STREAM", "MMF_KW_SERIAL",
    "MMF_KW_FUSED", "MMF_NO_KW_FUSED", "MMF_NO_GATE_B16", "MMF_POOL_PER_PAIR", "MMF_TAIL_S"};

uint32_t plan_flags_now() {
  uint32_t sum = 0;
  for (char** e = environ; e && *e; ++e) {
    const char* s = *e;
    if (std::strncmp(s, "MMF_", 4) != 0) continue;
    for (const char* k : kPlanKnobs) {
      const size_t n = std::strlen(k);
      if (std::strncmp(s, k, n) != 0 || s[n] != '=') continue;
      uint32_t h = 2166136261u;
      for (const char* c = s; *c; ++c) h = (h ^ (uint8_t)*c) * 16777619u;
      sum += h | 1u;   // (never 0 for a set knob)
      break;
    }
  }
  return sum;
}

// Before any launch: the plan switches are the ones the caller sized its buffers under, and the
// layout this call computed fits the capacities the caller declared (need_* = the Bump offsets;
// ~0 = that buffer is not used by the call).
int check_buffers(const mmf_hybrid_desc* d, size_t need_saved, size_t need_ws) {
  const uint32_t now = plan_flags_now();
  if (d->plan_flags != now)
    return fail(MMF_EINVAL,
                "the plan switches (MMF_* environment) changed since this descriptor's buffers were sized "
                "(plan_flags %08x, now %08x): size the buffers again and set plan_flags = mmf_hybrid_plan_flags()",
                d->plan_flags, now);
  if (need_saved != ~size_t(0) && need_saved > d->saved_capacity)
    return fail(MMF_EINVAL, "saved buffer too small: this call's layout needs %zu bytes, saved_capacity is %llu",
                need_saved, (unsigned long long)d->saved_capacity);
  if (need_ws != ~size_t(0) && need_ws > d->workspace_capacity)
    return fail(MMF_EINVAL, "workspace too small: this call's layout needs %zu bytes, workspace_capacity is %llu",
                need_ws, (unsigned long long)d->workspace_capacity);
  return MMF_OK;
}

inline int Lm(const mmf_hybrid_desc* d, int m) { return d->seq_len[m] > 0 ? d->seq_len[m] : 1; }
inline bool dropping(const mmf_hybrid_desc* d) { return d->training && d->dropout > 0.f; }
// Pair g attends over ONE key (2-D inputs, the reference's own case, or a 3-D key of
// length 1): softmax over one key is the mask indicator, so the pair has no Q / K /
// QK^T work and its query_proj / key_proj gradients are exactly zero (single_key.hip).
inline bool single_key(const mmf_hybrid_desc* d, int g) { return Lm(d, d->pair_k[g]) == 1; }
// head_dim beyond the fused attention kernels' register budget (MMF_MAX_HEAD_DIM): the pair's
// scores are materialised and contracted by GEMMs (wide.hip)
inline bool wide_pair(const mmf_hybrid_desc* d, int g) {
  return !single_key(d, g) && d->hidden / d->num_heads > MMF_MAX_HEAD_DIM;
}

// Pooled plan (attention.hip "Pooled-output attention"): keys up to 128 run the
// one-chunk kernels, longer keys the streamed long-key kernels; the pooled
// helpers keep heads x Lk query-mean probabilities in LDS (pool.hip POOL_PB_CAP).
bool use_pool(const mmf_hybrid_desc* d) {
  if (d->num_heads > 8) return false;
  for (int g = 0; g < d->num_pairs; ++g)
    if (Lm(d, d->pair_k[g]) * d->num_heads > POOL_PB_CAP) return false;
  return true;
}
inline int kw_ld(int lk) { return lk <= 128 ? 4 : (lk + 31) / 32; }
inline bool long_keys(const mmf_hybrid_desc* d) {
  for (int g = 0; g < d->num_pairs; ++g)
    if (Lm(d, d->pair_k[g]) > 128) return true;
  return false;
}

bool use_tail(const mmf_hybrid_desc* d);

// Training forward keeps the pre-dropout probabilities for the fused backward (no S recompute
// there): the pooled plan with every attention-kernel pair inside the lean fused kernels' shape
// (attn_pstore_ok).  All pairs or none (one launch each way).  Opt-in (MMF_PSTORE=1): measured
// at C2 it costs more than it saves (the 402 MB blob's write and read slow the
// neighbouring kernels more than the skipped recompute gains).
bool pstore_on(const mmf_hybrid_desc* d) {
  if (!d->training || !use_pool(d) || !getenv("MMF_PSTORE")) return false;
  const int hd = d->hidden / d->num_heads;
  int n = 0;
  for (int g = 0; g < d->num_pairs; ++g) {
    if (single_key(d, g) || wide_pair(d, g)) continue;
    if (!attn_pstore_ok(Lm(d, d->pair_q[g]), Lm(d, d->pair_k[g]), 1, hd) || d->hidden % 4 != 0) return false;
    ++n;
  }
  return n > 0;
}

// "medium" long-key pairs on the one-pass kernels (attn_long.hip) keep Q and K in bf16: the
// Q/K GEMM rounds its output once (EPI_BF16) -- exactly the rounding the kernels applied when
// they loaded fp32 rows -- so the GEMM writes and the attention kernels read half the bytes.
// All long pairs or none (the one-pass launches take every long pair); off with
// return_attention (the attention-map kernels read fp32 Q / K) and whenever the streamed
// kernels could run (MMF_NO_LONG_FUSED, MMF_NO_FUSED_BWD; MMF_NO_BF16_QK: fp32 Q / K, A/B).
bool qk_bf16_on(const mmf_hybrid_desc* d) {
  if (math_mode() != 1 || !use_pool(d) || d->return_attention || getenv("MMF_NO_LONG_FUSED") ||
      getenv("MMF_NO_FUSED_BWD") || getenv("MMF_NO_BF16_QK"))
    return false;
  const int hd = d->hidden / d->num_heads;
  if (hd > 64 || hd % 8 != 0 || d->hidden % 8 != 0) return false;
  int n = 0;
  for (int g = 0; g < d->num_pairs; ++g) {
    if (single_key(d, g) || wide_pair(d, g)) continue;
    const int lk = Lm(d, d->pair_k[g]);
    if (lk <= 128) continue;
    if (lk > 512 || lk % 32 != 0) return false;
    ++n;
  }
  return n > 0;
}
bool pair_qk_bf16(const mmf_hybrid_desc* d, int g) {
  return !single_key(d, g) && !wide_pair(d, g) && Lm(d, d->pair_k[g]) > 128 && qk_bf16_on(d);
}

// The Q/K projection GEMM on bf16 copies of both operands ("medium", every Q/K pair stores bf16
// Q / K): the projection GEMM's epilogue also writes P_m as bf16 (EPI_BF16COPY) and the pairs'
// W_q / W_k are converted once per forward; the GEMM (launch_gemm_b16) then streams half the
// operand bytes and feeds its MFMAs without conversions.  MMF_NO_GEMM_B16=1: the fp32-operand form.
bool qk_gemm_b16(const mmf_hybrid_desc* d) {
  if (math_mode() != 1 || getenv("MMF_NO_GEMM_B16") || d->hidden % 8 != 0) return false;
  int n = 0;
  for (int g = 0; g < d->num_pairs; ++g) {
    if (single_key(d, g) || wide_pair(d, g)) continue;
    if (!pair_qk_bf16(d, g)) return false;
    ++n;
  }
  return n > 0 && 2 * n <= CVT_MAX;
}

// The Q / K projections concatenated per modality ("medium", qk_gemm_b16): modality m's Q (pairs
// with query m) and K (pairs with key m) are column blocks of one (B L_m) x (ncat_m H) bf16 matrix,
// written by ONE bf16 GEMM of P_m against the stacked W_q / W_k copies (C5: 6 GEMMs of N = 2 560 in
// place of 60 of N = 256, each P_m row read once); the attention kernels read Q / K (and write dQ /
// dK) through ld = ncat_m H; the dZ GEMM is then one K = ncat_m H source.  Columns in pair order, a
// pair's Q before its K.  Opt-in (MMF_QK_CAT=1): measured at C5 it is slower -- 13.05 / 13.35 ms
// against 12.62 / 12.62 (profiles/r05/c5_qk_cat/): the 2 560-column GEMM on the LDS-DMA kernel
// (1.75 ms) loses to the weight-stationary per-pair GEMMs (1.46 ms), and the attention kernels'
// head-slice rows 5 KB apart instead of 512 B cost them 2-3 %.
bool qk_cat_on(const mmf_hybrid_desc* d) { return qk_gemm_b16(d) && getenv("MMF_QK_CAT"); }
void qk_cols(const mmf_hybrid_desc* d, int* qcol, int* kcol, int* ncat) {
  for (int m = 0; m < d->num_modalities; ++m) ncat[m] = 0;
  for (int g = 0; g < d->num_pairs; ++g) {
    qcol[g] = kcol[g] = -1;
    if (single_key(d, g) || wide_pair(d, g)) continue;
    qcol[g] = ncat[d->pair_q[g]]++;
    kcol[g] = ncat[d->pair_k[g]]++;
  }
}

// The backward on bf16 dQ / dK ("medium", every pair a bf16 Q/K pair of the one-pass kernels):
// attn_poolL_bwd_fused_bf16 stores dQ / dK as bf16 -- the rounding their GEMM consumers' MFMA
// operands get anyway -- and the dZ GEMM (dQ W_q + dK W_k, RK x KR on the forward's W_q / W_k
// copies) and the pairs' weight gradients (dQ^T P_q, dK^T P_k: KR x KR on the P_m copies) run the
// LDS-DMA kernel's bf16-operand forms: half the bytes written by the attention backward and read
// by both GEMMs.  The value-path term E_m is then materialised (pool_e) instead of riding in the
// dZ GEMM as K = heads sources.  MMF_NO_DQK_B16=1: fp32 dQ / dK (A/B).
bool dqk_b16_on(const mmf_hybrid_desc* d) {
  if (!d->training || !qk_gemm_b16(d) || getenv("MMF_NO_DQK_B16")) return false;
  for (int g = 0; g < d->num_pairs; ++g)
    if (!pair_qk_bf16(d, g)) return false;
  return d->num_pairs > 0;
}

// The modality projections on bf16 operands ("medium", dqk_b16_on): the input-mask kernel stores
// X'_m as bf16 (the rounding the fp32-operand GEMM gave its MFMA operands in-kernel) and W_proj is
// converted with the W_q / W_k copies, so the projection GEMM, its weight gradient (dZ^T X') and
// dX = dZ W run the LDS-DMA kernel's bf16 forms (RK x RK, KR x KR, RK x KR); the dZ GEMM stores dZ
// as bf16.  Half the bytes of X' (written once, read twice) and dZ (written once, read twice).
// The projection bias gradient is then the column sum of the bf16 dZ, as the Q / K ones are of
// the bf16 dQ / dK.  MMF_NO_PROJ_B16=1: the fp32-operand forms (A/B).
bool proj_b16_on(const mmf_hybrid_desc* d) {
  if (!dqk_b16_on(d) || qk_cat_on(d) || getenv("MMF_NO_PROJ_B16")) return false;
  int n = 0;
  for (int g = 0; g < d->num_pairs; ++g) n += 2;
  if (d->num_modalities + n > CVT_MAX) return false;
  for (int m = 0; m < d->num_modalities; ++m)
    if (d->in_dim[m] % 8 != 0) return false;
  return d->hidden % 8 == 0;
}

// The head (tail or generic) takes mean_L P_m from per-tile column sums written by the
// projection GEMM's epilogue when every 128-row tile lies inside one sample (pooled plan):
// L / 128 rows per sample instead of L (C5: the generic head read 400 MB with one
// workgroup per sample, 0.35 ms).
bool pcol_in_proj(const mmf_hybrid_desc* d, int m) {
  return d->num_pairs && use_pool(d) && Lm(d, m) % 128 == 0 && !getenv("MMF_NO_PCOL");
}

struct Saved {
  RngSnap* rng;
  float* Xd[MMF_MAX_MODALITIES];   // X_m * mask_m with input dropout (fusion.py:364-373)
  float* P[MMF_MAX_MODALITIES];
  float* Pcol[MMF_MAX_MODALITIES];  // per-128-row column sums of P_m (proj GEMM epilogue; tail plan)
  float *Q[MMF_MAX_PAIRS], *K[MMF_MAX_PAIRS], *lse[MMF_MAX_PAIRS];
  // general plan
  float *V[MMF_MAX_PAIRS], *O[MMF_MAX_PAIRS], *A[MMF_MAX_PAIRS];
  // pooled plan
  float *pbar[MMF_MAX_PAIRS], *U[MMF_MAX_PAIRS], *r[MMF_MAX_PAIRS], *Ob[MMF_MAX_PAIRS], *Ab[MMF_MAX_PAIRS];
  float* pbarT[MMF_MAX_PAIRS];   // (B, Lk, heads): pbar as the RK operand of the dZ GEMM's E_m term
  uint32_t* bits[MMF_MAX_PAIRS];
  float *Pw[MMF_MAX_PAIRS], *Pdw[MMF_MAX_PAIRS];   // wide pairs: probabilities, post-dropout (general)
  float* pst[MMF_MAX_PAIRS];                        // stored probabilities (pstore_on)
  float *pooled, *scores, *weights, *fused, *h1;
  __bf16* Pb[MMF_MAX_MODALITIES];                  // bf16 copies of P_m (qk_gemm_b16)
  __bf16 *Wqb[MMF_MAX_PAIRS], *Wkb[MMF_MAX_PAIRS];  // bf16 copies of W_q / W_k (qk_gemm_b16)
  __bf16* Wpb[MMF_MAX_MODALITIES];                 // bf16 copies of W_proj (proj_b16_on; Xd is then bf16)
  int32_t ldq[MMF_MAX_PAIRS], ldk[MMF_MAX_PAIRS];   // elements between Q (K) rows: H, or ncat H (qk_cat_on)
  // qk_cat_on: per modality the Q / K block matrix, the stacked W copies (Wqb / Wkb point into
  // them), the stacked biases, the column count; per pair its Q / K column slots
  __bf16* QKc[MMF_MAX_MODALITIES];
  __bf16* Wc[MMF_MAX_MODALITIES];
  float* bc[MMF_MAX_MODALITIES];
  int32_t ncat[MMF_MAX_MODALITIES];
  int32_t qcol[MMF_MAX_PAIRS], kcol[MMF_MAX_PAIRS];
};

void layout_saved(const mmf_hybrid_desc* d, Bump& bp, Saved& s) {
  memset(&s, 0, sizeof(s));
  const size_t B = d->batch, H = d->hidden, M = d->num_modalities, nh = d->num_heads;
  const bool pool = use_pool(d);
  const bool cat = qk_cat_on(d);
  if (cat) qk_cols(d, s.qcol, s.kcol, s.ncat);
  for (int g = 0; g < d->num_pairs; ++g) s.ldq[g] = s.ldk[g] = (int32_t)H;
  s.rng = bp.take<RngSnap>(1);
  const bool pb16 = proj_b16_on(d);
  for (int m = 0; m < d->num_modalities; ++m)
    s.Xd[m] = pb16 ? reinterpret_cast<float*>(bp.take<__bf16>(B * Lm(d, m) * d->in_dim[m]))
                   : bp.take<float>(B * Lm(d, m) * d->in_dim[m]);
  for (int m = 0; m < d->num_modalities && pb16; ++m) s.Wpb[m] = bp.take<__bf16>(H * d->in_dim[m]);
  for (int m = 0; m < d->num_modalities; ++m) s.P[m] = bp.take<float>(B * Lm(d, m) * H);
  for (int m = 0; m < d->num_modalities; ++m)
    if (pcol_in_proj(d, m)) s.Pcol[m] = bp.take<float>(B * (Lm(d, m) / 128) * H);
  for (int g = 0; g < d->num_pairs; ++g) {
    const size_t lq = Lm(d, d->pair_q[g]), lk = Lm(d, d->pair_k[g]);
    const bool sk = single_key(d, g), wide = wide_pair(d, g);
    if (!sk) {
      if (!cat) {
        s.Q[g] = bp.take<float>(B * lq * H);
        s.K[g] = bp.take<float>(B * lk * H);
      }
      if (!wide) s.lse[g] = bp.take<float>(B * nh * lq);
    }
    if (wide) {
      s.Pw[g] = bp.take<float>(B * nh * lq * lk);
      if (!pool) s.Pdw[g] = bp.take<float>(B * nh * lq * lk);
    }
    if (pool) {
      s.pbar[g] = bp.take<float>(B * nh * lk);
      s.pbarT[g] = bp.take<float>(B * nh * lk);
      s.U[g] = bp.take<float>(B * nh * H);
      s.r[g] = bp.take<float>(B * nh);
      s.Ob[g] = bp.take<float>(B * H);
      s.Ab[g] = bp.take<float>(B * H);
      if (dropping(d) && !sk && !wide) s.bits[g] = bp.take<uint32_t>(B * nh * lq * kw_ld((int)lk));
      if (!sk && !wide && pstore_on(d)) s.pst[g] = bp.take<float>(B * nh * attn_pstore_floats((int)lq));
    } else {
      s.V[g] = bp.take<float>(B * lk * H);
      s.O[g] = bp.take<float>(B * lq * H);
      s.A[g] = bp.take<float>(B * lq * H);
    }
  }
  s.pooled = bp.take<float>(B * M * H);
  s.scores = bp.take<float>(B * M);
  s.weights = bp.take<float>(B * M);
  s.fused = bp.take<float>(B * H);
  s.h1 = bp.take<float>(B * H);
  if (qk_gemm_b16(d)) {
    bool used[MMF_MAX_MODALITIES] = {};
    for (int g = 0; g < d->num_pairs; ++g)
      if (!single_key(d, g) && !wide_pair(d, g)) {
        used[d->pair_q[g]] = used[d->pair_k[g]] = true;
        if (!cat) {
          s.Wqb[g] = bp.take<__bf16>(H * H);
          s.Wkb[g] = bp.take<__bf16>(H * H);
        }
      }
    for (int m = 0; m < d->num_modalities; ++m)
      if (used[m]) s.Pb[m] = bp.take<__bf16>(B * Lm(d, m) * H);
  }
  if (cat) {
    for (int m = 0; m < d->num_modalities; ++m)
      if (s.ncat[m] > 0) {
        s.QKc[m] = bp.take<__bf16>(B * Lm(d, m) * s.ncat[m] * H);
        s.Wc[m] = bp.take<__bf16>((size_t)s.ncat[m] * H * H);
        s.bc[m] = bp.take<float>((size_t)s.ncat[m] * H);
      }
    for (int g = 0; g < d->num_pairs; ++g) {
      if (s.qcol[g] < 0) continue;
      const int q = d->pair_q[g], k = d->pair_k[g];
      s.Q[g] = reinterpret_cast<float*>(s.QKc[q] + (size_t)s.qcol[g] * H);
      s.K[g] = reinterpret_cast<float*>(s.QKc[k] + (size_t)s.kcol[g] * H);
      s.ldq[g] = s.ncat[q] * (int32_t)H;
      s.ldk[g] = s.ncat[k] * (int32_t)H;
      s.Wqb[g] = s.Wc[q] + (size_t)s.qcol[g] * H * H;
      s.Wkb[g] = s.Wc[k] + (size_t)s.kcol[g] * H * H;
    }
  }
}

struct Ws {
  float *dz1, *dfused, *cvec, *dscore;
  float *dQ[MMF_MAX_PAIRS], *dK[MMF_MAX_PAIRS], *dsum[MMF_MAX_PAIRS];
  float *dO[MMF_MAX_PAIRS], *dV[MMF_MAX_PAIRS];                              // general
  float *dOb[MMF_MAX_PAIRS], *dU[MMF_MAX_PAIRS], *dpbar[MMF_MAX_PAIRS];      // pooled
  float *dS[MMF_MAX_PAIRS], *dPd[MMF_MAX_PAIRS];                             // wide pairs
  float* E[MMF_MAX_MODALITIES];                                              // pooled
  float* dZ[MMF_MAX_MODALITIES];
  // qk_cat_on: per modality the dQ / dK block matrix (the layout of Saved::QKc: fp32-sized, bf16
  // when dqk_b16_on); dQ / dK point into it
  float* dQc[MMF_MAX_MODALITIES];
};

void layout_ws(const mmf_hybrid_desc* d, Bump& bp, Ws& w) {
  memset(&w, 0, sizeof(w));
  const size_t B = d->batch, H = d->hidden, M = d->num_modalities, nh = d->num_heads;
  const bool pool = use_pool(d);
  const bool cat = qk_cat_on(d), b16 = dqk_b16_on(d);
  int qcol[MMF_MAX_PAIRS], kcol[MMF_MAX_PAIRS], ncat[MMF_MAX_MODALITIES];
  if (cat) qk_cols(d, qcol, kcol, ncat);
  w.dz1 = bp.take<float>(B * H);
  w.dfused = bp.take<float>(B * H);
  w.cvec = bp.take<float>(B * M * H);
  w.dscore = bp.take<float>(B * M);
  for (int g = 0; g < d->num_pairs; ++g) {
    const size_t lq = Lm(d, d->pair_q[g]), lk = Lm(d, d->pair_k[g]);
    if (!single_key(d, g)) {
      if (!cat) {
        w.dQ[g] = bp.take<float>(B * lq * H);
        w.dK[g] = bp.take<float>(B * lk * H);
      }
      w.dsum[g] = bp.take<float>(B * nh * lq);
    }
    if (wide_pair(d, g)) {
      w.dS[g] = bp.take<float>(B * nh * lq * lk);
      if (!pool) w.dPd[g] = bp.take<float>(B * nh * lq * lk);
    }
    if (pool) {
      w.dOb[g] = bp.take<float>(B * H);
      w.dU[g] = bp.take<float>(B * nh * H);
      w.dpbar[g] = bp.take<float>(B * nh * lk);
    } else {
      w.dO[g] = bp.take<float>(B * lq * H);
      w.dV[g] = bp.take<float>(B * lk * H);
    }
  }
  for (int m = 0; m < d->num_modalities; ++m) {
    if (pool) w.E[m] = bp.take<float>(B * Lm(d, m) * H);
    w.dZ[m] = bp.take<float>(B * Lm(d, m) * H);
  }
  if (cat) {
    for (int m = 0; m < d->num_modalities; ++m)
      if (ncat[m] > 0) w.dQc[m] = bp.take<float>(B * Lm(d, m) * ncat[m] * H);
    // (element offsets of the column slots: bf16 or fp32 elements, as the attention backward writes)
    auto slot = [&](int m, int col) -> float* {
      return b16 ? reinterpret_cast<float*>(reinterpret_cast<__bf16*>(w.dQc[m]) + (size_t)col * H)
                 : w.dQc[m] + (size_t)col * H;
    };
    for (int g = 0; g < d->num_pairs; ++g) {
      if (qcol[g] < 0) continue;
      w.dQ[g] = slot(d->pair_q[g], qcol[g]);
      w.dK[g] = slot(d->pair_k[g], kcol[g]);
    }
  }
}

int check_hybrid(const mmf_hybrid_desc* d) {
  if (!d) return fail(MMF_EINVAL, "null descriptor");
  if (d->matmul_precision != MMF_PRECISION_HIGHEST && d->matmul_precision != MMF_PRECISION_MEDIUM &&
      d->matmul_precision != MMF_PRECISION_HIGH)
    return fail(MMF_EINVAL, "bad matmul_precision %d", d->matmul_precision);
  if (d->batch < 1) return fail(MMF_EINVAL, "batch must be >= 1 (got %d)", d->batch);
  if (d->num_modalities < 1 || d->num_modalities > MMF_MAX_MODALITIES)
    return fail(MMF_ELIMIT, "num_modalities must be in [1, %d] (got %d)", MMF_MAX_MODALITIES,
                d->num_modalities);
  if (d->num_heads < 1 || d->hidden % d->num_heads != 0)
    return fail(MMF_EINVAL, "hidden_dim (%d) must be divisible by num_heads (%d)", d->hidden,
                d->num_heads);
  if (d->hidden % 4 != 0 || d->hidden > 1024)
    return fail(MMF_ELIMIT, "hidden_dim must be a multiple of 4 and <= 1024 (got %d)", d->hidden);
  if (d->num_classes < 1) return fail(MMF_EINVAL, "num_classes must be >= 1");
  if (d->num_pairs < 0 || d->num_pairs > d->num_modalities * (d->num_modalities - 1))
    return fail(MMF_EINVAL, "bad num_pairs %d", d->num_pairs);
  for (int m = 0; m < d->num_modalities; ++m) {
    if (d->in_dim[m] < 1) return fail(MMF_EINVAL, "in_dim[%d] must be >= 1", m);
    if (d->seq_len[m] < 0) return fail(MMF_EINVAL, "seq_len[%d] must be >= 0", m);
  }
  for (int g = 0; g < d->num_pairs; ++g) {
    const int q = d->pair_q[g], k = d->pair_k[g];
    if (q < 0 || k < 0 || q >= d->num_modalities || k >= d->num_modalities || q == k)
      return fail(MMF_EINVAL, "bad pair %d: (%d, %d)", g, q, k);
  }
  if (!(d->dropout >= 0.f && d->dropout < 1.f))
    return fail(MMF_EINVAL, "dropout must be in [0, 1) (got %g)", (double)d->dropout);
  for (int g = 0; g < d->num_pairs; ++g)
    if (wide_pair(d, g) && !wide_supported(d->batch, d->num_heads, Lm(d, d->pair_q[g]), Lm(d, d->pair_k[g])))
      return fail(MMF_ELIMIT, "head_dim %d: pair %d's (heads x Lq x Lk) score tensor is too large",
                  d->hidden / d->num_heads, g);
  return MMF_OK;
}

// Every weight gradient as a split-K job; the same code sizes the workspace
// (called with null bases) and plans the real launch.
// part (mmf_hybrid_train_step_part): 0 every weight, 1 every weight but the modality projections'
// (known once the attention backward has run), 2 the projections' alone (after dZ); the split
// counts are sized for the launch the part makes.
void plan_wgrads(const mmf_hybrid_desc* d, const float* const* x, const float* mask,
                 const float* dlogits, const Saved& s, const Ws& w, const mmf_hybrid_grads* G,
                 Bump& bw, WgradPlan& wp, int part = 0) {
  const bool want_pairs = part != 2, want_proj = part != 1;
  const int B = d->batch, M = d->num_modalities, H = d->hidden, C = d->num_classes;
  const int nh = d->num_heads, hd = H / nh;
  const bool pool = use_pool(d);
  static const mmf_hybrid_grads kNull = {};
  const mmf_hybrid_grads* g = G ? G : &kNull;
  // Split counts of the long (B*L-row) contractions, sized per launch: launch_gemm packs
  // GEMM_MAX_GROUPS (32) of them per launch (longest slabs first), and a launch should be
  // about one wave of its 3-per-CU workgroups.  Full launches take slots / GEMM_MAX_GROUPS
  // slabs per job; the r jobs of a remainder launch take slots / r (C2: all 15 big jobs fit
  // one launch: 768 / 15 = 51 slabs requested, 49 of 672 rows after rounding to 32).
  const int kBigRows = 4096;
  int nbig = 0;
  for (int p = 0; p < d->num_pairs && want_pairs; ++p) {
    const int lq = Lm(d, d->pair_q[p]), lk = Lm(d, d->pair_k[p]);
    if (!pool) nbig += (B * lq >= kBigRows) + (B * lk >= kBigRows);
    if (!single_key(d, p)) nbig += (B * lq >= kBigRows) + (B * lk >= kBigRows);
  }
  for (int m = 0; m < M && want_proj; ++m) nbig += (B * Lm(d, m) >= kBigRows);
  const int slots = 3 * device_cu_count();
  const int rem = nbig % GEMM_MAX_GROUPS, nfull = nbig - rem;
  int bi = 0;
  auto hint = [&](int rows) {
    if (rows < kBigRows) return 0;
    const int per = bi++ < nfull ? GEMM_MAX_GROUPS : rem;
    int sp = slots / per;
    if (const char* e = getenv("MMF_WGRAD_SPLIT_CAP")) sp = std::min(sp, std::max(1, atoi(e)));
    return std::max(1, std::min(sp, 256));
  };
  if (want_pairs) {
    plan_wgrad(wp, bw, C, H, B, opnd(dlogits, C), opnd(s.h1, H), g->cls2.w, g->cls2.b);
    plan_wgrad(wp, bw, H, H, B, opnd(w.dz1, H), opnd(s.fused, H), g->cls1.w, g->cls1.b);
    // gating_layers[m]: dscore[:, m]^T pooled[:, m, :]
    for (int m = 0; m < M; ++m)
      plan_wgrad(wp, bw, 1, H, B, opnd(w.dscore ? w.dscore + m : nullptr, M),
                 opnd(s.pooled ? s.pooled + (size_t)m * H : nullptr, M * H), g->gate[m].w, g->gate[m].b);
  }
  for (int p = 0; p < d->num_pairs && want_pairs; ++p) {
    const int q = d->pair_q[p], k = d->pair_k[p];
    const int lq = Lm(d, q), lk = Lm(d, k);
    const float* cq = w.cvec ? w.cvec + (size_t)q * H : nullptr;
    if (pool) {
      plan_wgrad(wp, bw, H, H, B, opnd(cq, M * H), opnd(s.Ob[p], H), g->o[p].w, g->o[p].b);
      // value_proj.weight rows of head h = dObar_h^T U_h; bias slice = sum_b r_h[b] dObar_h[b]
      // (Obar_h = U_h W_v,h^T + r_h b_v,h): strided batches over the heads
      Operand dob = opnd(w.dOb[p], H), u = opnd(s.U[p], nh * H), rr = opnd(s.r[p], nh);
      dob.vec = u.vec = (hd % 4 == 0) && (H % 4 == 0);
      rr.vec = 0;
      plan_wgrad_batched(wp, bw, hd, H, B, dob, u, g->v[p].w, nh, hd, H, hd * H);
      plan_wgrad_batched(wp, bw, hd, 1, B, dob, rr, g->v[p].b, nh, hd, 1, hd);
    } else {
      wp.split_hint = hint(B * lq);
      plan_wgrad(wp, bw, H, H, B * lq, opnd(cq, M * H, lq), opnd(s.O[p], H), g->o[p].w, g->o[p].b,
                 1.f / (float)lq);
      wp.split_hint = hint(B * lk);
      plan_wgrad(wp, bw, H, H, B * lk, opnd(w.dV[p], H), opnd(s.P[k], H), g->v[p].w, g->v[p].b);
    }
    if (single_key(d, p)) {
      // softmax over one key: no gradient reaches query_proj / key_proj (exact zeros)
      plan_zero(wp, H, H, g->q[p].w, g->q[p].b);
      plan_zero(wp, H, H, g->k[p].w, g->k[p].b);
      continue;
    }
    const bool b16 = dqk_b16_on(d);
    // (bf16: dQ / dK and the P_m copies as __bf16 addresses, launch_gemm_b16's KR x KR form)
    const float* pq = b16 ? reinterpret_cast<const float*>(s.Pb[q]) : s.P[q];
    const float* pk = b16 ? reinterpret_cast<const float*>(s.Pb[k]) : s.P[k];
    wp.split_hint = hint(B * lq);
    plan_wgrad(wp, bw, H, H, B * lq, opnd(w.dQ[p], s.ldq[p]), opnd(pq, H), g->q[p].w, g->q[p].b);
    if (b16 && !wp.size_only) { wp.jobs_b16.push_back(wp.jobs.back()); wp.jobs.pop_back(); }
    wp.split_hint = hint(B * lk);
    plan_wgrad(wp, bw, H, H, B * lk, opnd(w.dK[p], s.ldk[p]), opnd(pk, H), g->k[p].w, g->k[p].b);
    if (b16 && !wp.size_only) { wp.jobs_b16.push_back(wp.jobs.back()); wp.jobs.pop_back(); }
    wp.split_hint = 0;
  }
  for (int m = 0; m < M && want_proj; ++m) {
    const int L = Lm(d, m), D = d->in_dim[m];
    wp.split_hint = hint(B * L);
    plan_wgrad(wp, bw, H, D, B * L, opnd(w.dZ[m], H), opnd(s.Xd[m], D), g->proj[m].w, g->proj[m].b);
    // (proj_b16_on: dZ and X' are bf16, launch_gemm_b16's KR x KR form)
    if (proj_b16_on(d) && !wp.size_only) { wp.jobs_b16.push_back(wp.jobs.back()); wp.jobs.pop_back(); }
    wp.split_hint = 0;
  }
}

size_t saved_bytes(const mmf_hybrid_desc* d) {
  MathScope math_(d->matmul_precision);   // (the layout depends on the precision: qk_gemm_b16)
  Bump bp(nullptr);
  Saved s{};
  layout_saved(d, bp, s);
  return bp.off + 256;
}

size_t workspace_bytes(const mmf_hybrid_desc* d) {
  MathScope math_(d->matmul_precision);
  Bump bs(nullptr);
  Saved s{};
  layout_saved(d, bs, s);
  Bump bw(nullptr);
  Ws w;
  layout_ws(d, bw, w);
  // the largest slab area of a one-launch backward and of its two parts (their slabs share the
  // area: part 1's reduce has run before part 2's slabs are written)
  size_t top = 0;
  for (int part = 0; part < 3; ++part) {
    Bump b = bw;
    WgradPlan wp;
    wp.size_only = true;
    plan_wgrads(d, nullptr, nullptr, nullptr, s, w, nullptr, b, wp, part);
    top = std::max(top, b.off);
  }
  return top + 256;
}

void fill_head(HeadArgs& ha, const mmf_hybrid_desc* d, const mmf_hybrid_params* W, const float* mask,
               const Saved& s) {
  const bool pool = use_pool(d);
  memset(&ha, 0, sizeof(ha));
  ha.B = d->batch; ha.M = d->num_modalities; ha.H = d->hidden; ha.mask = mask;
  ha.scale_by_mask = 1;
  int cnt[MMF_MAX_MODALITIES];
  for (int m = 0; m < d->num_modalities; ++m) {
    // mean over L of P_m: from the per-128-row column sums when the projection wrote them
    ha.src[ha.nsrc] = s.Pcol[m] ? s.Pcol[m] : s.P[m];
    ha.src_mod[ha.nsrc] = m;
    ha.src_L[ha.nsrc] = s.Pcol[m] ? Lm(d, m) / 128 : Lm(d, m);
    ha.src_scale[ha.nsrc++] = 1.f / (float)Lm(d, m);
    cnt[m] = 1;
    ha.gate_w[m] = W->gate[m].w;
    ha.gate_b[m] = W->gate[m].b;
  }
  for (int g = 0; g < d->num_pairs; ++g) {
    const int q = d->pair_q[g];
    ha.src[ha.nsrc] = pool ? s.Ab[g] : s.A[g];
    ha.src_mod[ha.nsrc] = q;
    ha.src_L[ha.nsrc] = pool ? 1 : Lm(d, q);
    ha.src_scale[ha.nsrc++] = pool ? 1.f : 1.f / (float)Lm(d, q);
    cnt[q]++;
  }
  for (int m = 0; m < d->num_modalities; ++m) ha.inv_cnt[m] = 1.0f / (float)cnt[m];
  ha.pooled = s.pooled; ha.scores = s.scores; ha.weights = s.weights; ha.fused = s.fused;
}

bool use_tail(const mmf_hybrid_desc* d) {
  return use_pool(d) && !long_keys(d) && tail_supported(d->num_modalities, d->hidden, d->num_classes, d->num_heads,
                                       d->hidden / d->num_heads, d->num_pairs);
}

void fill_tail(TailArgs& ta, const mmf_hybrid_desc* d, const mmf_hybrid_params* W, const float* mask,
               const Saved& s) {
  memset(&ta, 0, sizeof(ta));
  const int M = d->num_modalities;
  ta.B = d->batch; ta.M = M; ta.H = d->hidden; ta.C = d->num_classes;
  ta.heads = d->num_heads; ta.hd = d->hidden / d->num_heads; ta.npairs = d->num_pairs;
  ta.mask = mask;
  int cnt[MMF_MAX_MODALITIES];
  for (int m = 0; m < M; ++m) {
    ta.P[m] = s.P[m];
    ta.L[m] = Lm(d, m);
    ta.Pcol[m] = s.Pcol[m];
    ta.ncol[m] = Lm(d, m) / 128;
    ta.gate_w[m] = W->gate[m].w;
    ta.gate_b[m] = W->gate[m].b;
    cnt[m] = 1;
  }
  for (int g = 0; g < d->num_pairs; ++g) {
    TailPair& P = ta.p[g];
    P.pbar = s.pbar[g]; P.Pk = s.P[d->pair_k[g]]; P.Lk = Lm(d, d->pair_k[g]);
    P.U = s.U[g]; P.r = s.r[g];
    P.Wv = W->v[g].w; P.bv = W->v[g].b; P.Wo = W->o[g].w; P.bo = W->o[g].b;
    P.Ob = s.Ob[g]; P.Ab = s.Ab[g];
    P.q = d->pair_q[g];
    P.k = d->pair_k[g];
    cnt[d->pair_q[g]]++;
  }
  for (int m = 0; m < M; ++m) ta.inv_cnt[m] = 1.0f / (float)cnt[m];
  ta.W1 = W->cls1.w; ta.b1 = W->cls1.b; ta.W2 = W->cls2.w; ta.b2 = W->cls2.b;
  ta.pooled = s.pooled; ta.scores = s.scores; ta.weights = s.weights; ta.fused = s.fused; ta.h1 = s.h1;
  ta.drop_p = dropping(d) ? d->dropout : 0.f;
  ta.drop_site = SITE_CLS;
  ta.rng = s.rng;
  ta.gscale = dropping(d) ? 1.f / (1.f - d->dropout) : 1.f;
}

AttnPair make_pair(const mmf_hybrid_desc* d, const Saved& s, const float* mask, int g) {
  AttnPair a;
  memset(&a, 0, sizeof(a));
  const int q = d->pair_q[g], k = d->pair_k[g];
  a.q = s.Q[g]; a.k = s.K[g]; a.v = s.V[g]; a.o = s.O[g]; a.lse = s.lse[g];
  a.kmask = mask + k; a.kmask_mode = 1; a.kmask_ld = d->num_modalities;
  a.Lq = Lm(d, q); a.Lk = Lm(d, k);
  a.ldv = a.ldo = d->hidden;
  a.ldq = s.ldq[g];
  a.ldk = s.ldk[g];
  a.drop_site = SITE_ATTN + g;
  a.pbar = s.pbar[g];
  a.pbarT = s.pbarT[g];
  a.keep_bits = s.bits[g];
  a.kw_ld = kw_ld(a.Lk);
  a.pstore = s.pst[g];
  a.qk_bf16 = pair_qk_bf16(d, g) ? 1 : 0;
  a.dqk_bf16 = a.qk_bf16 && dqk_b16_on(d) ? 1 : 0;
  return a;
}

WidePair make_wide(const mmf_hybrid_desc* d, const Saved& s, const float* mask, int g) {
  WidePair a;
  memset(&a, 0, sizeof(a));
  const int q = d->pair_q[g], k = d->pair_k[g];
  a.q = s.Q[g]; a.k = s.K[g]; a.v = s.V[g];
  a.ldq = a.ldk = a.ldv = a.ldo = d->hidden;
  a.kmask = mask + k; a.kmask_mode = 1; a.kmask_ld = d->num_modalities;
  a.Lq = Lm(d, q); a.Lk = Lm(d, k);
  a.drop_site = SITE_ATTN + g;
  a.P = s.Pw[g]; a.Pd = s.Pdw[g];
  a.pbar = s.pbar[g]; a.pbarT = s.pbarT[g];
  a.o = s.O[g];
  return a;
}

SkPair make_sk(const mmf_hybrid_desc* d, const Saved& s, const float* mask, int g) {
  SkPair a;
  memset(&a, 0, sizeof(a));
  const int q = d->pair_q[g], k = d->pair_k[g];
  a.kmask = mask + k; a.kmask_mode = 1; a.kmask_ld = d->num_modalities;
  a.Lq = Lm(d, q);
  a.drop_site = SITE_ATTN + g;
  a.pbar = s.pbar[g];
  a.pbarT = s.pbarT[g];
  a.v = s.V[g]; a.ldv = d->hidden;
  a.o = s.O[g]; a.ldo = d->hidden;
  return a;
}

// Launch-lean single-key step (l1.hip): every modality 2-D (L = 1, the reference's own
// semantics), every ordered pair present, fp32 ("highest"), H, D_m <= 128 (% 4),
// C <= 16, float4-able inputs and weights.  It writes the single-key pooled plan's Saved / Ws
// slots (Ob = O = P' V, Ab = A, dOb = dV, dU = dP_k|g), so both plans size the buffers alike; the
// choice depends only on the descriptor and the pointers forward and backward both receive.
// MMF_NO_L1_LEAN=1: the general single-key plan (A/B).
// the descriptor half of lean_l1 (the other half: 16-B aligned inputs and weights)
bool lean_l1_desc(const mmf_hybrid_desc* d) {
  const bool off = getenv("MMF_NO_L1_LEAN") != nullptr;
  const int M = d->num_modalities, H = d->hidden;
  if (off || d->matmul_precision != MMF_PRECISION_HIGHEST) return false;
  if (M < 2 || M > L1_MAXM || d->num_pairs != M * (M - 1)) return false;
  if (H % 4 != 0 || H > L1_MAXH || d->num_heads > 8 || d->num_classes > L1_MAXC) return false;
  unsigned seen = 0;
  for (int g = 0; g < d->num_pairs; ++g) seen |= 1u << (d->pair_q[g] * L1_MAXM + d->pair_k[g]);
  if (__builtin_popcount(seen) != d->num_pairs) return false;
  for (int m = 0; m < M; ++m)
    if (Lm(d, m) != 1 || d->in_dim[m] % 4 != 0 || d->in_dim[m] > L1_MAXD) return false;
  return true;
}

bool lean_l1(const mmf_hybrid_desc* d, const mmf_hybrid_params* W, const float* const* x) {
  const int M = d->num_modalities;
  if (!W || !x || !lean_l1_desc(d)) return false;
  for (int m = 0; m < M; ++m) {
    if (!aligned16(x[m]) || !aligned16(W->proj[m].w)) return false;
  }
  for (int g = 0; g < d->num_pairs; ++g)
    if (!aligned16(W->v[g].w) || !aligned16(W->o[g].w)) return false;
  return aligned16(W->cls1.w);
}

// the C2 shape of the L = 1 kernels (l1.hip l1_full): H and every input width 128
bool l1_desc_full(const mmf_hybrid_desc* d) {
  if (d->hidden != 128) return false;
  for (int m = 0; m < d->num_modalities; ++m)
    if (d->in_dim[m] != 128) return false;
  return true;
}

void fill_l1(L1Args& a, const mmf_hybrid_desc* d, const mmf_hybrid_params* W, const float* const* x,
             const float* mask, const Saved& s) {
  memset(&a, 0, sizeof(a));
  const int M = d->num_modalities;
  a.B = d->batch; a.M = M; a.H = d->hidden; a.C = d->num_classes; a.heads = d->num_heads;
  a.npairs = d->num_pairs;
  a.p = dropping(d) ? d->dropout : 0.f;
  a.gscale = dropping(d) ? 1.f / (1.f - d->dropout) : 1.f;
  a.mask = mask;
  int cnt[L1_MAXM];
  for (int m = 0; m < M; ++m) {
    a.D[m] = d->in_dim[m];
    a.x[m] = x[m];
    a.Wp[m] = W->proj[m].w; a.bp[m] = W->proj[m].b;
    a.gw[m] = W->gate[m].w; a.gb[m] = W->gate[m].b;
    a.Xd[m] = s.Xd[m]; a.P[m] = s.P[m];
    a.kdesig[m] = -1;
    cnt[m] = 1;
  }
  for (int g = 0; g < d->num_pairs; ++g) {
    const int q = d->pair_q[g], k = d->pair_k[g];
    a.pq[g] = q; a.pk[g] = k;
    if (a.kdesig[k] < 0) a.kdesig[k] = g;
    a.Wv[g] = W->v[g].w; a.bv[g] = W->v[g].b; a.Wo[g] = W->o[g].w; a.bo[g] = W->o[g].b;
    a.O[g] = s.Ob[g]; a.A[g] = s.Ab[g];
    cnt[q]++;
  }
  for (int m = 0; m < M; ++m) a.inv_cnt[m] = 1.0f / (float)cnt[m];
  a.W1 = W->cls1.w; a.b1 = W->cls1.b; a.W2 = W->cls2.w; a.b2 = W->cls2.b;
  a.pooled = s.pooled; a.scores = s.scores; a.weights = s.weights; a.fused = s.fused; a.h1 = s.h1;
  a.snap = s.rng;
}


// The L = 1 plan's backward arguments: the L1Args of the forward plus the gradient outputs, and
// every weight gradient as a dW = G^T X job over the batch (l1_wgrad_kernel)
void fill_l1_bwd(L1Args& a, L1WgArgs& wa, const mmf_hybrid_desc* d, const mmf_hybrid_params* W,
                 const float* const* x, const float* mask, const Saved& s, const Ws& w, const float* dlogits,
                 const mmf_hybrid_grads* G, float* const* dx) {
  const int B = d->batch, M = d->num_modalities, H = d->hidden, C = d->num_classes;
  fill_l1(a, d, W, x, mask, s);
  a.dlogits = dlogits;
  a.dz1 = w.dz1; a.cvec = w.cvec; a.dscore = w.dscore;
  for (int g = 0; g < d->num_pairs; ++g) {
    a.dV[g] = w.dOb[g];
    a.dPk[g] = w.dU[g];
  }
  for (int m = 0; m < M; ++m) {
    a.dZ[m] = w.dZ[m];
    a.dx[m] = dx ? dx[m] : nullptr;
  }
  memset(&wa, 0, sizeof(wa));
  wa.B = B;
  auto job = [&](const float* Gp, int ldg, const float* Xp, int ldx, int N, int K, float* dW, float* db) {
    if (!dW && !db) return;
    L1WgJob& j = wa.j[wa.njobs++];
    j.G = Gp; j.ldg = ldg; j.X = Xp; j.ldx = ldx; j.N = N; j.K = K; j.dW = dW; j.db = db;
    j.tiles_k = (K + 31) / 32;
    j.tile0 = wa.ntiles;
    wa.ntiles += ((N + 31) / 32) * j.tiles_k;
  };
  auto zero = [&](float* p, int n) {
    if (!p || n <= 0) return;
    wa.z[wa.nz] = p; wa.zn[wa.nz] = n;
    wa.zoff[wa.nz + 1] = wa.zoff[wa.nz] + (n + 4095) / 4096;
    wa.nz++;
  };
  for (int m = 0; m < M; ++m)
    job(w.dZ[m], H, s.Xd[m], d->in_dim[m], H, d->in_dim[m], G->proj[m].w, G->proj[m].b);
  for (int g = 0; g < d->num_pairs; ++g) {
    job(w.dOb[g], H, s.P[d->pair_k[g]], H, H, H, G->v[g].w, G->v[g].b);
    job(w.cvec + (size_t)d->pair_q[g] * H, M * H, s.Ob[g], H, H, H, G->o[g].w, G->o[g].b);
    // softmax over one key: no gradient reaches query_proj / key_proj (exact zeros)
    zero(G->q[g].w, H * H); zero(G->q[g].b, H); zero(G->k[g].w, H * H); zero(G->k[g].b, H);
  }
  job(w.dz1, H, s.fused, H, H, H, G->cls1.w, G->cls1.b);
  job(dlogits, C, s.h1, H, C, H, G->cls2.w, G->cls2.b);
  for (int m = 0; m < M; ++m) job(w.dscore + m, M, s.pooled + (size_t)m * H, M * H, 1, H, G->gate[m].w, G->gate[m].b);
}
}  // namespace

extern "C" {

size_t mmf_hybrid_saved_bytes(const mmf_hybrid_desc* d) {
  if (check_hybrid(d) != MMF_OK) return 0;
  return saved_bytes(d);
}

size_t mmf_hybrid_workspace_bytes(const mmf_hybrid_desc* d) {
  if (check_hybrid(d) != MMF_OK) return 0;
  return workspace_bytes(d);
}

int mmf_hybrid_saved_region(const mmf_hybrid_desc* d, int32_t what, int32_t index, uint64_t* offset,
                            uint64_t* bytes) {
  int rc = check_hybrid(d);
  if (rc) return rc;
  if (!offset || !bytes) return fail(MMF_EINVAL, "saved region: null argument");
  MathScope math_(d->matmul_precision);
  // laid out from a stand-in base (never dereferenced; a null base would give null pointers)
  char* const base = reinterpret_cast<char*>(uintptr_t(1) << 40);
  Bump bp(base);
  Saved s{};
  layout_saved(d, bp, s);
  const size_t B = d->batch, H = d->hidden;
  const float* p = nullptr;
  size_t n = 0;
  if (what == MMF_SAVED_PROJ) {
    if (index < 0 || index >= d->num_modalities)
      return fail(MMF_EINVAL, "saved region: modality %d of %d", index, d->num_modalities);
    p = s.P[index];
    n = B * Lm(d, index) * H;
  } else if (what == MMF_SAVED_CLS_HIDDEN) {
    if (index != 0) return fail(MMF_EINVAL, "saved region: the classifier hidden layer has index 0 (got %d)", index);
    p = s.h1;
    n = B * H;
  } else {
    return fail(MMF_EINVAL, "saved region: unknown region %d", what);
  }
  *offset = (uint64_t)(reinterpret_cast<const char*>(p) - base);
  *bytes = n * sizeof(float);
  return MMF_OK;
}

namespace {

// dZ_m takes its value-path term E_m as extra K = heads sources of the dZ GEMM
// (pbarT against the per-sample dU) when a 128-row tile never straddles two
// samples and the pbarT rows are float4-able; otherwise pool_e materialises E_m.
bool poole_in_dz(const mmf_hybrid_desc* d, int m) {
  if (getenv("MMF_NO_POOLE") || dqk_b16_on(d)) return false;
  return Lm(d, m) % 128 == 0 && d->hidden % 4 == 0 && d->num_heads % 4 == 0;
}

}  // namespace

// A training step's loss inside the tail's head launch (mmf_hybrid_train_step, the pooled tail plan
// with the 16-sample tile head): the loss inputs and outputs, the step's sync word (the head
// launch's tile count) and workspace (dz1, cvec, dscore and the loss rows).  done: the forward's
// head launch ran the loss, dlogits and the head backward (the step skips the cross-entropy
// launch, and the backward its head launch).
struct TailTrain {
  const int64_t* labels;
  float ls_eps, loss_scale;
  float *loss, *dlogits;
  uint32_t* cnt;
  void* workspace;
  bool done;
};

static int hybrid_forward(const mmf_hybrid_desc* d, const mmf_hybrid_params* W, const float* const* x,
                          const float* mask, const uint64_t* rng_state, void* saved, float* logits,
                          float* fusion_weights, float* const* attn_maps, void* stream, TailTrain* tt) {
  int rc = check_hybrid(d);
  if (rc) return rc;
  MathScope math_(d->matmul_precision);
  if (!W || !x || !mask || !saved || !logits) return fail(MMF_EINVAL, "null argument");
  hipStream_t st = (hipStream_t)stream;
  const int B = d->batch, M = d->num_modalities, H = d->hidden, C = d->num_classes;
  const int nh = d->num_heads, hd = H / nh;
  const bool drop = dropping(d);
  const float p = drop ? d->dropout : 0.f;
  const bool pool = use_pool(d);
  if (drop && !rng_state) return fail(MMF_EINVAL, "training with dropout needs rng_state");

  Bump bp(saved);
  Saved s{};
  layout_saved(d, bp, s);
  // (against the capacity the caller declared, under the plan switches it sized `saved` with)
  if ((rc = check_buffers(d, bp.off, ~size_t(0)))) return rc;
  // the rng snapshot {seed, offset} is written by the input-mask kernel (which draws from
  // the live state) and the live offset advanced by the projection GEMM's first launch:
  // no launch of its own
  const RngSnap* rng = rng_state ? s.rng : nullptr;

  if (lean_l1(d, W, x)) {
    L1Args a;
    fill_l1(a, d, W, x, mask, s);
    a.rng_live = rng_state;
    a.rng_advance = const_cast<uint64_t*>(rng_state);
    a.logits = logits;
    a.weights_out = fusion_weights;
    if (d->return_attention && attn_maps)
      for (int g = 0; g < d->num_pairs; ++g) a.maps[g] = attn_maps[g];
    STAGE_TRY("fwd.l1", launch_l1_forward(a, st));
    return MMF_OK;
  }

  // pairs with several keys run the attention kernels; single-key pairs single_key.hip
  std::vector<AttnPair> pairs;
  std::vector<SkPair> skp;
  std::vector<WidePair> wp;
  for (int g = 0; g < d->num_pairs; ++g) {
    float* maps = d->return_attention && attn_maps ? attn_maps[g] : nullptr;
    if (single_key(d, g)) {
      skp.push_back(make_sk(d, s, mask, g));
      skp.back().probs = maps;
    } else if (wide_pair(d, g)) {
      wp.push_back(make_wide(d, s, mask, g));
      wp.back().probs = maps;   // written by the wide softmax itself
    } else {
      pairs.push_back(make_pair(d, s, mask, g));
      pairs.back().probs = maps;
    }
  }
  const int nmp = (int)pairs.size(), nsk = (int)skp.size(), nwp = (int)wp.size();
  // The attention dropout keep words depend only on the rng snapshot: drawn on a side stream
  // (attn_keep_words_kernel) while the projection GEMMs run, so the attention forward reads
  // them instead of drawing inline.  Pooled plan, training, with long-key pairs (C5: the
  // draws are a third of the one-pass forward's VALU work; at C2's 128 keys the concurrent
  // draws slow the fp32 GEMMs more than the lean forward gains, 0.979 -> 0.986 ms); an
  // existing side stream only while st is being captured.  MMF_NO_SIDE_STREAM=1: inline (A/B);
  // MMF_SIDE_STREAM=1: also without long pairs.
  SideStream* side = nullptr;
  // MMF_KW_SERIAL=1 (A/B): the draws on st, ahead of the projection GEMM.  At C2 the lean forward
  // drops 112-116 -> 90 us but the draw kernel takes 26.5 us: 0.968 -> 0.971-0.975 ms
  bool kw_serial = false;
  // Without long-key pairs (and at most 16 pairs) the draws are made by extra workgroups of the
  // input-mask kernel, interleaved with its HBM-bound rows: at C2 the lean forward drops
  // 113 -> 91 us and the mask kernel grows 23 -> 41 us, step 0.969 -> 0.960 ms median
  // (DESIGN §7).  MMF_NO_KW_FUSED=1: off; MMF_KW_FUSED=1: also with long-key pairs.
  bool kw_fused = false;
  bool any_long = false;
  for (const AttnPair& a : pairs) any_long = any_long || a.Lk > 128;
  auto fork_keep_words = [&]() {
    if (!(drop && use_pool(d) && nmp) || getenv("MMF_NO_SIDE_STREAM")) return;
    if (kw_fused) return;
    if (getenv("MMF_KW_SERIAL")) {
      kw_serial = launch_attn_keep_words(pairs.data(), nmp, B, nh, p, rng, st) == hipSuccess;
      return;
    }
    if (!any_long && !getenv("MMF_SIDE_STREAM")) return;
    side = side_stream(!prof_capturing(st));
    if (!side) return;
    if (hipEventRecord(side->fork_ev, st) != hipSuccess || hipStreamWaitEvent(side->s, side->fork_ev, 0) != hipSuccess ||
        launch_attn_keep_words(pairs.data(), nmp, B, nh, p, rng, side->s) != hipSuccess ||
        hipEventRecord(side->join_ev, side->s) != hipSuccess) {
      side = nullptr;   // (a failed fork joins nothing; the kernels draw inline)
    }
  };

  // (1) per-modality projection: P_m = Drop(ReLU(X'_m W_m^T + b_m)), X'_m = Drop(X_m * mask_m)
  //     (fusion.py:364-374); X' is kept for the weight gradient
  const bool pb16 = proj_b16_on(d);
  bool qk_cvt_done = false;
  if (pb16) {
    // bf16 copies of W_proj and (the Q/K branch below then skips its own launch) W_q / W_k
    CvtArgs cv;
    memset(&cv, 0, sizeof(cv));
    for (int m = 0; m < M; ++m) {
      cv.src[cv.count] = W->proj[m].w; cv.dst[cv.count] = s.Wpb[m]; cv.n[cv.count++] = (int64_t)H * d->in_dim[m];
    }
    for (int g = 0; g < d->num_pairs; ++g) {
      if (single_key(d, g) || wide_pair(d, g)) continue;
      cv.src[cv.count] = W->q[g].w; cv.dst[cv.count] = s.Wqb[g]; cv.n[cv.count++] = (int64_t)H * H;
      cv.src[cv.count] = W->k[g].w; cv.dst[cv.count] = s.Wkb[g]; cv.n[cv.count++] = (int64_t)H * H;
    }
    STAGE_TRY("fwd.qk_cvt", launch_cvt_bf16(cv, st));
    qk_cvt_done = true;
  }
  {
    MaskDropArgs ma;
    memset(&ma, 0, sizeof(ma));
    ma.n = M; ma.M = M; ma.mask = mask; ma.p = p; ma.rng = rng;
    ma.rng_live = rng_state; ma.rng_snap = rng_state ? s.rng : nullptr;
    std::vector<GemmJob> jobs;
    for (int m = 0; m < M; ++m) {
      const int L = Lm(d, m), D = d->in_dim[m];
      ma.j[m].x = x[m]; ma.j[m].out = s.Xd[m]; ma.j[m].rows = (int64_t)B * L; ma.j[m].D = D; ma.j[m].L = L;
      ma.j[m].site = SITE_IN + m;
      ma.j[m].outb = pb16 ? 1 : 0;
      GemmJob j = make_job(B * L, H, s.P[m], H,
                           EPI_BIAS | EPI_RELU | (drop ? EPI_DROP : 0) | (s.Pcol[m] ? EPI_COLSUM : 0));
      j.g.bias = W->proj[m].b;
      j.g.colsum = s.Pcol[m];
      j.g.drop_site = SITE_PROJ + m;
      if (s.Pb[m]) {   // (qk_gemm_b16: the Q/K GEMM's bf16 A operand)
        j.g.epi |= EPI_BF16COPY;
        j.g.copy = s.Pb[m];
      }
      add_src(j, opnd(s.Xd[m], D), opnd(W->proj[m].w, D), D);
      jobs.push_back(j);
    }
    if (drop && use_pool(d) && nmp && !getenv("MMF_NO_SIDE_STREAM") && !getenv("MMF_SIDE_STREAM") &&
        !getenv("MMF_KW_SERIAL") && !getenv("MMF_NO_KW_FUSED") && (!any_long || getenv("MMF_KW_FUSED"))) {
      int nkw = 0;
      bool fits = true;
      for (const AttnPair& a : pairs) {
        if (!(a.keep_bits && a.Lk % 32 == 0 && a.Lk > 0 && a.kw_ld >= a.Lk / 32)) continue;
        // at most 16 pairs, each under launch_mask_dropout's 2^31-word bound: otherwise the
        // side-stream / inline draws (never a failed forward)
        const int64_t nw = (int64_t)B * nh * a.Lq * (a.Lk / 32);
        if (nkw == 16 || nw >= ((int64_t)1 << 31)) { fits = false; break; }
        ma.kw[nkw++] = {a.keep_bits, (uint32_t)a.Lq, (uint32_t)a.Lk, (uint32_t)a.kw_ld, a.drop_site};
      }
      ma.nkw = fits ? nkw : 0;
      ma.B = B;
      ma.heads = nh;
      kw_fused = fits;
      static bool warned = false;
      if (!fits && getenv("MMF_KW_FUSED") && !warned) {
        warned = true;
        fprintf(stderr, "mmfusion: MMF_KW_FUSED requested but the keep-word fold does not fit "
                        "(> 16 pairs or > 2^31 words per pair): drawing them on the side stream / inline\n");
      }
    }
    STAGE_TRY("fwd.input_mask", launch_mask_dropout(ma, st));
    fork_keep_words();   // the rng snapshot exists from here on
    if (pb16) {
      for (int m = 0; m < M; ++m) jobs[m].src[0].b.ptr = reinterpret_cast<const float*>(s.Wpb[m]);
      STAGE_TRY("fwd.proj_gemm", launch_gemm_b16(jobs.data(), (int)jobs.size(), st, MODE_RK, MODE_RK, p, rng,
                                                 const_cast<uint64_t*>(rng_state)));
    } else {
      STAGE_TRY("fwd.proj_gemm", launch_gemm(jobs.data(), (int)jobs.size(), MODE_RK, MODE_RK, p, rng, st,
                                             const_cast<uint64_t*>(rng_state)));
    }
  }
  // (2) Q/K (and V for the general plan) projections of every present pair (attention.py:104-106)
  if (d->num_pairs && qk_cat_on(d)) {
    // the stacked bf16 W copies and fp32 biases per modality, then one bf16 GEMM per modality
    // writing every Q / K column block of it (see qk_cat_on)
    std::vector<CvtArgs> cvs(1);
    memset(&cvs[0], 0, sizeof(CvtArgs));
    auto add_cvt = [&](const float* src, __bf16* dst, float* dst32, int64_t n) {
      if (cvs.back().count == CVT_MAX) {
        cvs.emplace_back();
        memset(&cvs.back(), 0, sizeof(CvtArgs));
      }
      CvtArgs& c = cvs.back();
      c.src[c.count] = src; c.dst[c.count] = dst; c.dst32[c.count] = dst32; c.n[c.count++] = n;
    };
    for (int g = 0; g < d->num_pairs; ++g) {
      if (s.qcol[g] < 0) continue;
      const int q = d->pair_q[g], k = d->pair_k[g];
      add_cvt(W->q[g].w, s.Wqb[g], nullptr, (int64_t)H * H);
      add_cvt(W->k[g].w, s.Wkb[g], nullptr, (int64_t)H * H);
      add_cvt(W->q[g].b, nullptr, s.bc[q] + (size_t)s.qcol[g] * H, H);
      add_cvt(W->k[g].b, nullptr, s.bc[k] + (size_t)s.kcol[g] * H, H);
    }
    std::vector<GemmJob> jobs;
    auto bop = [](const __bf16* p, int ld) { return opnd(reinterpret_cast<const float*>(p), ld); };
    for (int m = 0; m < M; ++m) {
      if (s.ncat[m] <= 0) continue;
      const int N = s.ncat[m] * H;
      GemmJob j = make_job(B * Lm(d, m), N, reinterpret_cast<float*>(s.QKc[m]), N, EPI_BIAS | EPI_BF16);
      j.g.bias = s.bc[m];
      add_src(j, bop(s.Pb[m], H), bop(s.Wc[m], H), H);
      jobs.push_back(j);
    }
    for (const CvtArgs& c : cvs) STAGE_TRY("fwd.qk_cvt", launch_cvt_bf16(c, st));
    STAGE_TRY("fwd.qkv_gemm", launch_gemm_b16(jobs.data(), (int)jobs.size(), st));
  } else if (d->num_pairs && qk_gemm_b16(d)) {
    // bf16 copies of W_q / W_k, then one bf16-operand GEMM launch over every Q / K projection
    CvtArgs cv;
    memset(&cv, 0, sizeof(cv));
    std::vector<GemmJob> jobs;
    auto bop = [](const __bf16* p, int ld) { return opnd(reinterpret_cast<const float*>(p), ld); };
    for (int g = 0; g < d->num_pairs; ++g) {
      const int q = d->pair_q[g], k = d->pair_k[g];
      if (single_key(d, g) || wide_pair(d, g)) continue;
      cv.src[cv.count] = W->q[g].w; cv.dst[cv.count] = s.Wqb[g]; cv.n[cv.count++] = (int64_t)H * H;
      cv.src[cv.count] = W->k[g].w; cv.dst[cv.count] = s.Wkb[g]; cv.n[cv.count++] = (int64_t)H * H;
      GemmJob jq = make_job(B * Lm(d, q), H, s.Q[g], H, EPI_BIAS | EPI_BF16);
      jq.g.bias = W->q[g].b;
      add_src(jq, bop(s.Pb[q], H), bop(s.Wqb[g], H), H);
      jobs.push_back(jq);
      GemmJob jk = make_job(B * Lm(d, k), H, s.K[g], H, EPI_BIAS | EPI_BF16);
      jk.g.bias = W->k[g].b;
      add_src(jk, bop(s.Pb[k], H), bop(s.Wkb[g], H), H);
      jobs.push_back(jk);
    }
    if (!qk_cvt_done) STAGE_TRY("fwd.qk_cvt", launch_cvt_bf16(cv, st));
    STAGE_TRY("fwd.qkv_gemm", launch_gemm_b16(jobs.data(), (int)jobs.size(), st));
  } else if (d->num_pairs) {
    std::vector<GemmJob> jobs;
    for (int g = 0; g < d->num_pairs; ++g) {
      const int q = d->pair_q[g], k = d->pair_k[g];
      const int lq = Lm(d, q), lk = Lm(d, k);
      if (!single_key(d, g)) {
        const int qkb = pair_qk_bf16(d, g) ? EPI_BF16 : 0;
        GemmJob jq = make_job(B * lq, H, s.Q[g], H, EPI_BIAS | qkb);
        jq.g.bias = W->q[g].b;
        add_src(jq, opnd(s.P[q], H), opnd(W->q[g].w, H), H);
        jobs.push_back(jq);
        GemmJob jk = make_job(B * lk, H, s.K[g], H, EPI_BIAS | qkb);
        jk.g.bias = W->k[g].b;
        add_src(jk, opnd(s.P[k], H), opnd(W->k[g].w, H), H);
        jobs.push_back(jk);
      }
      if (!pool) {
        GemmJob jv = make_job(B * lk, H, s.V[g], H, EPI_BIAS);
        jv.g.bias = W->v[g].b;
        add_src(jv, opnd(s.P[k], H), opnd(W->v[g].w, H), H);
        jobs.push_back(jv);
      }
    }
    if (!jobs.empty())
      STAGE_TRY("fwd.qkv_gemm", launch_gemm(jobs.data(), (int)jobs.size(), MODE_RK, MODE_RK, 0.f, rng, st));
  }
  const float scale = 1.0f / std::sqrt((float)hd);
  if (side) HIP_TRY(hipStreamWaitEvent(st, side->join_ev, 0));   // join the keep-word draws
  if (d->num_pairs && pool) {
    // (3p) attention -> LSE, pbar = mean_q P'; U = pbar P_k; Obar = U W_v^T + r b_v; Abar = out_proj
    if (nmp)
      STAGE_TRY("fwd.attn", launch_attn_pool_fwd(pairs.data(), nmp, B, nh, hd, scale, p, rng, st, side != nullptr || kw_serial || kw_fused));
    if (nsk) STAGE_TRY("fwd.attn_single_key", launch_sk_fwd(skp.data(), nsk, B, nh, hd, p, rng, st));
    if (nwp) STAGE_TRY("fwd.attn_wide", launch_wide_fwd(wp.data(), nwp, B, nh, hd, scale, p, rng, true, st));
    std::vector<PoolPair> pp(d->num_pairs);
    for (int g = 0; g < d->num_pairs; ++g) {
      memset(&pp[g], 0, sizeof(PoolPair));
      pp[g].pk = s.P[d->pair_k[g]];
      pp[g].Lk = Lm(d, d->pair_k[g]);
      pp[g].pbar = s.pbar[g];
      pp[g].u = s.U[g];
      pp[g].r = s.r[g];
    }
    if (use_tail(d)) {
      // (4p) fused per-sample tail: Obar, Abar, aggregation, weighting, classifier
      TailArgs ta;
      fill_tail(ta, d, W, mask, s);
      ta.weights_out = fusion_weights;
      ta.logits = logits;
      if (tt && seq_head_ok(ta)) {
        // (a training step: the loss, dlogits and the head backward in the head launch)
        Bump bw(tt->workspace);
        Ws w;
        layout_ws(d, bw, w);
        ta.labels = tt->labels; ta.ls_eps = tt->ls_eps; ta.loss_scale = tt->loss_scale;
        ta.loss_rows = w.dfused;   // (B x H floats the tail plan leaves unused)
        ta.loss_mean = tt->loss; ta.loss_cnt = tt->cnt; ta.dlogits_out = tt->dlogits;
        ta.dz1 = w.dz1; ta.cvec = w.cvec; ta.dscore = w.dscore;
        tt->done = true;
      }
      STAGE_TRY("fwd.tail", launch_tail_fwd(ta, st));
    } else {
      STAGE_TRY("fwd.pool_u", launch_pool_u(pp.data(), d->num_pairs, B, nh, hd, H, st));
      std::vector<GemmJob> jobs;
      for (int g = 0; g < d->num_pairs; ++g) {
        // Obar[:, h*hd:(h+1)*hd] = U_h W_v[h*hd:(h+1)*hd, :]^T + r_h b_v,h  (batch over heads)
        GemmJob j = make_job(B, hd, s.Ob[g], H, EPI_BIAS | EPI_BIAS_RS);
        j.g.bias = W->v[g].b;
        j.g.bias_rs = s.r[g];
        j.g.bias_rs_ld = nh;
        j.g.nbatch = nh;
        j.g.bs_a = H; j.g.bs_b = hd * H; j.g.bs_c = hd; j.g.bs_bias = hd; j.g.bs_brs = 1;
        add_src(j, opnd(s.U[g], nh * H), opnd(W->v[g].w, H), H);
        jobs.push_back(j);
      }
      STAGE_TRY("fwd.vbar_gemm", launch_gemm(jobs.data(), (int)jobs.size(), MODE_RK, MODE_RK, 0.f, rng, st));
      jobs.clear();
      for (int g = 0; g < d->num_pairs; ++g) {
        GemmJob j = make_job(B, H, s.Ab[g], H, EPI_BIAS);
        j.g.bias = W->o[g].b;
        add_src(j, opnd(s.Ob[g], H), opnd(W->o[g].w, H), H);
        jobs.push_back(j);
      }
      STAGE_TRY("fwd.out_gemm", launch_gemm(jobs.data(), (int)jobs.size(), MODE_RK, MODE_RK, 0.f, rng, st));
    }
  } else if (d->num_pairs) {
    // (3g) flash attention per pair (key mask = modality mask column k, fusion.py:391-401) + out_proj
    if (nmp) STAGE_TRY("fwd.attn", launch_attn_fwd(pairs.data(), nmp, B, nh, hd, scale, p, rng, st));
    if (nsk) STAGE_TRY("fwd.attn_single_key", launch_sk_out(skp.data(), nsk, B, nh, hd, p, rng, st));
    if (nwp) STAGE_TRY("fwd.attn_wide", launch_wide_fwd(wp.data(), nwp, B, nh, hd, scale, p, rng, false, st));
    std::vector<GemmJob> jobs;
    for (int g = 0; g < d->num_pairs; ++g) {
      const int lq = Lm(d, d->pair_q[g]);
      GemmJob j = make_job(B * lq, H, s.A[g], H, EPI_BIAS);
      j.g.bias = W->o[g].b;
      add_src(j, opnd(s.O[g], H), opnd(W->o[g].w, H), H);
      jobs.push_back(j);
    }
    STAGE_TRY("fwd.out_gemm", launch_gemm(jobs.data(), (int)jobs.size(), MODE_RK, MODE_RK, 0.f, rng, st));
  }
  // (4) aggregation + pooling + gating + adaptive weights + weighted sum (fusion.py:406-418)
  // (5) classifier: Linear -> ReLU -> Dropout -> Linear (fusion.py:323-328)
  if (!(d->num_pairs && use_tail(d))) {
    HeadArgs ha;
    fill_head(ha, d, W, mask, s);
    ha.weights_out = fusion_weights;
    STAGE_TRY("fwd.head", launch_head_fwd(ha, st));
    GemmJob j = make_job(B, H, s.h1, H, EPI_BIAS | EPI_RELU | (drop ? EPI_DROP : 0));
    j.g.bias = W->cls1.b;
    j.g.drop_site = SITE_CLS;
    add_src(j, opnd(s.fused, H), opnd(W->cls1.w, H), H);
    STAGE_TRY("fwd.cls1_gemm", launch_gemm(&j, 1, MODE_RK, MODE_RK, p, rng, st));
    GemmJob j2 = make_job(B, C, logits, C, EPI_BIAS);
    j2.g.bias = W->cls2.b;
    add_src(j2, opnd(s.h1, H), opnd(W->cls2.w, H), H);
    STAGE_TRY("fwd.cls2_gemm", launch_gemm(&j2, 1, MODE_RK, MODE_RK, 0.f, rng, st));
  }
  // (6) optional attention maps (post-dropout, attention.py:130,144-146)
  //     (single-key pairs wrote theirs in sk_fwd; the general plan's sk_out does not)
  if (d->return_attention && attn_maps && d->num_pairs) {
    std::vector<AttnPair> pp;
    for (AttnPair a : pairs)
      if (a.probs) {
        a.pstore = nullptr;   // the stored-probability blob belongs to the pooled kernels only
        pp.push_back(a);
      }
    if (!pp.empty())
      STAGE_TRY("fwd.attn_probs", launch_attn_probs(pp.data(), (int)pp.size(), B, nh, hd, scale, p, rng, st));
    if (!pool) {
      std::vector<SkPair> sp;
      for (SkPair a : skp)
        if (a.probs) {
          a.pbar = a.pbarT = nullptr;
          sp.push_back(a);
        }
      if (!sp.empty())
        STAGE_TRY("fwd.attn_probs_single_key", launch_sk_fwd(sp.data(), (int)sp.size(), B, nh, hd, p, rng, st));
    }
  }
  return MMF_OK;
}

int mmf_hybrid_forward(const mmf_hybrid_desc* d, const mmf_hybrid_params* W, const float* const* x,
                       const float* mask, const uint64_t* rng_state, void* saved, float* logits,
                       float* fusion_weights, float* const* attn_maps, void* stream) {
  return hybrid_forward(d, W, x, mask, rng_state, saved, logits, fusion_weights, attn_maps, stream, nullptr);
}

// head_done: the training step's head launch ran the head backward (TailTrain)
// part: 0 the whole backward; 1 everything up to the attention backward and every weight gradient
// but the modality projections'; 2 dZ, dX and the projections' weight gradients (the L = 1 plan
// runs all of it in part 1)
static int hybrid_backward(const mmf_hybrid_desc* d, const mmf_hybrid_params* W, const float* const* x,
                           const float* mask, const void* saved, const float* dlogits, void* workspace,
                           const mmf_hybrid_grads* G, float* const* dx, void* stream, bool head_done,
                           int part = 0) {
  int rc = check_hybrid(d);
  if (rc) return rc;
  MathScope math_(d->matmul_precision);
  if (!W || !x || !mask || !saved || !dlogits || !workspace || !G)
    return fail(MMF_EINVAL, "null argument");
  hipStream_t st = (hipStream_t)stream;
  const int B = d->batch, M = d->num_modalities, H = d->hidden, C = d->num_classes;
  const int nh = d->num_heads, hd = H / nh;
  const bool drop = dropping(d);
  const float p = drop ? d->dropout : 0.f;
  const float gscale = drop ? 1.f / (1.f - p) : 1.f;
  const bool pool = use_pool(d);

  Bump bs(const_cast<void*>(saved));
  Saved s{};
  layout_saved(d, bs, s);
  const RngSnap* rng = s.rng;
  Bump bw(workspace);
  Ws w;
  layout_ws(d, bw, w);
  if (lean_l1(d, W, x)) {
    if ((rc = check_buffers(d, bs.off, bw.off))) return rc;
    if (part == 2) return MMF_OK;
    L1Args a;
    L1WgArgs wa;
    fill_l1_bwd(a, wa, d, W, x, mask, s, w, dlogits, G, dx);
    STAGE_TRY("bwd.l1", launch_l1_backward(a, wa, st));
    return MMF_OK;
  }
  WgradPlan wp;
  plan_wgrads(d, x, mask, dlogits, s, w, G, bw, wp, part);
  if ((rc = check_buffers(d, bs.off, bw.off))) return rc;

  const bool tail = d->num_pairs && use_tail(d);
  if (part != 2) {
  if (tail) {
    // (1-3p) fused per-sample tail backward: classifier, head, dObar, dU
    TailArgs ta;
    fill_tail(ta, d, W, mask, s);
    ta.dlogits = dlogits; ta.dz1 = w.dz1; ta.cvec = w.cvec; ta.dscore = w.dscore;
    ta.head_done = head_done;
    for (int g = 0; g < d->num_pairs; ++g) {
      ta.p[g].dOb = w.dOb[g];
      ta.p[g].dU = w.dU[g];
      ta.p[g].dpbar = w.dpbar[g];
    }
    STAGE_TRY("bwd.tail", launch_tail_bwd(ta, st));
  } else {
    // (1) classifier backward: dz1 = ReLU'/Dropout' (dlogits W2), dfused = dz1 W1
    {
      GemmJob j = make_job(B, H, w.dz1, H, EPI_GATE);
      j.g.gate = s.h1; j.g.ld_gate = H; j.g.gate_scale = gscale;
      add_src(j, opnd(dlogits, C), opnd(W->cls2.w, H), C);
      STAGE_TRY("bwd.cls_dz1_gemm", launch_gemm(&j, 1, MODE_RK, MODE_KR, 0.f, rng, st));
      GemmJob j2 = make_job(B, H, w.dfused, H, 0);
      add_src(j2, opnd(w.dz1, H), opnd(W->cls1.w, H), H);
      STAGE_TRY("bwd.cls_dfused_gemm", launch_gemm(&j2, 1, MODE_RK, MODE_KR, 0.f, rng, st));
    }
    // (2) head backward: dscore and c_m = dpooled_m * mask_m / n_m
    {
      HeadArgs ha;
      fill_head(ha, d, W, mask, s);
      ha.dfused = w.dfused; ha.cvec = w.cvec; ha.dscore = w.dscore;
      STAGE_TRY("bwd.head", launch_head_bwd(ha, st));
    }
  }
  const float scale = 1.0f / std::sqrt((float)hd);
  std::vector<AttnPair> pairs;
  std::vector<SkPair> skp;
  std::vector<WidePair> wpairs;
  for (int g = 0; g < d->num_pairs; ++g) {
    if (single_key(d, g)) {
      skp.push_back(make_sk(d, s, mask, g));
      skp.back().dout = w.dO[g];
      skp.back().dv = w.dV[g];
      continue;
    }
    if (wide_pair(d, g)) {
      wpairs.push_back(make_wide(d, s, mask, g));
      WidePair& a = wpairs.back();
      a.dpbar = w.dpbar[g]; a.dout = w.dO[g]; a.dPd = w.dPd[g]; a.dS = w.dS[g];
      a.dq = w.dQ[g]; a.dk = w.dK[g]; a.dv = w.dV[g];
      continue;
    }
    pairs.push_back(make_pair(d, s, mask, g));
    AttnPair& a = pairs.back();
    a.dsum = w.dsum[g]; a.dq = w.dQ[g]; a.dk = w.dK[g];
    a.dout = w.dO[g]; a.dv = w.dV[g]; a.dpbar = w.dpbar[g];
  }
  const int nmp = (int)pairs.size(), nsk = (int)skp.size(), nwp = (int)wpairs.size();
  if (d->num_pairs && pool) {
    // (3p) dObar = dAbar W_o (dAbar = c_q); dU_h = dObar_h W_v,h; dpbar; attention dQ/dK; E_m
    if (!tail) {
      std::vector<GemmJob> jobs;
      for (int g = 0; g < d->num_pairs; ++g) {
        GemmJob j = make_job(B, H, w.dOb[g], H, 0);
        add_src(j, opnd(w.cvec + (size_t)d->pair_q[g] * H, M * H), opnd(W->o[g].w, H), H);
        jobs.push_back(j);
      }
      STAGE_TRY("bwd.out_dO_gemm", launch_gemm(jobs.data(), (int)jobs.size(), MODE_RK, MODE_KR, 0.f, rng, st));
      jobs.clear();
      for (int g = 0; g < d->num_pairs; ++g) {
        // dU_h = dObar_h W_v[h*hd:(h+1)*hd, :]  (batch over heads)
        GemmJob j = make_job(B, H, w.dU[g], nh * H, 0);
        j.g.nbatch = nh;
        j.g.bs_a = hd; j.g.bs_b = hd * H; j.g.bs_c = H;
        Operand a = opnd(w.dOb[g], H);
        a.vec = (hd % 4 == 0) && (H % 4 == 0);
        add_src(j, a, opnd(W->v[g].w, H), hd);
        jobs.push_back(j);
      }
      STAGE_TRY("bwd.du_gemm", launch_gemm(jobs.data(), (int)jobs.size(), MODE_RK, MODE_KR, 0.f, rng, st));
    }
    std::vector<PoolPair> pp(d->num_pairs);
    for (int g = 0; g < d->num_pairs; ++g) {
      memset(&pp[g], 0, sizeof(PoolPair));
      pp[g].pk = s.P[d->pair_k[g]];
      pp[g].Lk = Lm(d, d->pair_k[g]);
      pp[g].du = w.dU[g];
      pp[g].dob = w.dOb[g];
      pp[g].bv = W->v[g].b;
      pp[g].dpbar = w.dpbar[g];
    }
    if (!tail) STAGE_TRY("bwd.pool_dpbar", launch_pool_dpbar(pp.data(), d->num_pairs, B, nh, hd, H, st));
    // (single-key pairs: no attention backward, dQ = dK = 0)
    if (nmp) {
      hipError_t fe;
      {
        Stage stage_("bwd.attn", st);
        fe = getenv("MMF_NO_FUSED_BWD") ? hipErrorNotSupported
                                        : launch_attn_pool_bwd(2, pairs.data(), nmp, B, nh, hd, scale, p, rng, st);
      }
      if (fe == hipErrorNotSupported) {
        (void)hipGetLastError();
        for (const AttnPair& a : pairs)
          if (a.qk_bf16) return fail(MMF_EHIP, "bf16 Q / K pair refused by the one-pass backward");
        for (AttnPair& a : pairs) a.pstore = nullptr;   // the two-pass kernels recompute S
        STAGE_TRY("bwd.attn_dq", launch_attn_pool_bwd(0, pairs.data(), nmp, B, nh, hd, scale, p, rng, st));
        STAGE_TRY("bwd.attn_dk", launch_attn_pool_bwd(1, pairs.data(), nmp, B, nh, hd, scale, p, rng, st));
      } else {
        HIP_TRY(fe);
      }
    }
    if (nwp) STAGE_TRY("bwd.attn_wide", launch_wide_bwd(wpairs.data(), nwp, B, nh, hd, scale, p, rng, true, st));
    std::vector<PoolEMod> em;
    for (int m = 0; m < M; ++m) {
      if (poole_in_dz(d, m)) continue;   // E_m is formed in the dZ GEMM's epilogue instead
      em.emplace_back();
      PoolEMod& e = em.back();
      memset(&e, 0, sizeof(PoolEMod));
      e.out = w.E[m];
      e.L = Lm(d, m);
      e.c = w.cvec + (size_t)m * H;
      e.ldc = M * H;
      e.cscale = 1.f / (float)Lm(d, m);
      for (int g = 0; g < d->num_pairs; ++g)
        if (d->pair_k[g] == m) {
          e.pbar[e.nsrc] = s.pbar[g];
          e.du[e.nsrc++] = w.dU[g];
        }
    }
    if (!em.empty()) STAGE_TRY("bwd.pool_e", launch_pool_e(em.data(), (int)em.size(), B, nh, H, st));
  } else if (d->num_pairs) {
    // (3g) dA_g rows = c_q / L_q broadcast: dO = dA W_o; flash attention backward
    std::vector<GemmJob> jobs;
    for (int g = 0; g < d->num_pairs; ++g) {
      const int q = d->pair_q[g], lq = Lm(d, q);
      GemmJob j = make_job(B * lq, H, w.dO[g], H, 0);
      j.g.alpha = 1.f / (float)lq;
      add_src(j, opnd(w.cvec + (size_t)q * H, M * H, lq), opnd(W->o[g].w, H), H);
      jobs.push_back(j);
    }
    STAGE_TRY("bwd.out_dO_gemm", launch_gemm(jobs.data(), (int)jobs.size(), MODE_RK, MODE_KR, 0.f, rng, st));
    if (nmp) {
      STAGE_TRY("bwd.attn_prep", launch_attn_bwd_stage(0, pairs.data(), nmp, B, nh, hd, scale, p, rng, st));
      STAGE_TRY("bwd.attn_dkv", launch_attn_bwd_stage(1, pairs.data(), nmp, B, nh, hd, scale, p, rng, st));
      STAGE_TRY("bwd.attn_dq", launch_attn_bwd_stage(2, pairs.data(), nmp, B, nh, hd, scale, p, rng, st));
    }
    if (nsk) STAGE_TRY("bwd.attn_single_key_dv", launch_sk_dv(skp.data(), nsk, B, nh, hd, p, rng, st));
    if (nwp) STAGE_TRY("bwd.attn_wide", launch_wide_bwd(wpairs.data(), nwp, B, nh, hd, scale, p, rng, false, st));
  }
  }   // part != 2
  if (part == 1) {
    // every weight gradient but the projections': final once these launches complete
    std::stable_sort(wp.jobs.begin(), wp.jobs.end(), [](const GemmJob& a, const GemmJob& b) {
      const int64_t wa = (int64_t)a.g.nsplit * std::max(1, a.g.nbatch) * a.g.M * a.g.N;
      const int64_t wb = (int64_t)b.g.nsplit * std::max(1, b.g.nbatch) * b.g.M * b.g.N;
      return wa > wb;
    });
    STAGE_TRY("bwd.wgrad_gemm", launch_gemm(wp.jobs.data(), (int)wp.jobs.size(), MODE_KR, MODE_KR, p, rng, st));
    if (!wp.jobs_b16.empty())
      STAGE_TRY("bwd.wgrad_gemm", launch_gemm_b16(wp.jobs_b16.data(), (int)wp.jobs_b16.size(), st, MODE_KR, MODE_KR));
    STAGE_TRY("bwd.wgrad_reduce", launch_reduce(wp.reds.data(), (int)wp.reds.size(), st));
    return MMF_OK;
  }
  // (5) dX_m = (dZ_m W_m) * mask * input-dropout' -- built first: with MMF_DX_CHAIN=1 (fp32-operand
  // forms) each rides in its dZ_m job's launch as a chained GEMM (GemmJob::chain: the workgroup that
  // finishes a dZ_m row tile computes that tile's dX_m rows next, dZ_m from L2), otherwise a launch
  // of its own
  std::vector<GemmJob> dxjobs(M);
  std::vector<bool> has_dx(M, false);
  const bool pb16 = proj_b16_on(d);
  for (int m = 0; m < M; ++m) {
    if (!dx || !dx[m]) continue;
    const int L = Lm(d, m), D = d->in_dim[m];
    GemmJob j = make_job(B * L, D, dx[m], D, EPI_ROWSCALE | (drop ? EPI_DROP : 0));
    j.g.rowscale = mask; j.g.rs_div = L; j.g.rs_stride = M; j.g.rs_off = m;
    j.g.drop_site = SITE_IN + m;
    // (proj_b16_on: the bf16 dZ against the forward's W_proj copy, launch_gemm_b16's RK x KR form)
    add_src(j, opnd(w.dZ[m], H), opnd(pb16 ? reinterpret_cast<const float*>(s.Wpb[m]) : W->proj[m].w, D), H);
    dxjobs[m] = j;
    has_dx[m] = true;
  }
  // Opt-in (MMF_DX_CHAIN=1): measured at C2 it saves nothing -- the chained kernel took 192.2 us
  // for what the two launches take in 191.1 (profiles/r06/dx_chain/): every workgroup still runs
  // dZ's epilogue, then dX's prologue, main loop and epilogue in lockstep with all the others, so
  // the chain removes only the launch boundary and dZ's HBM re-read, neither of which bounds it
  const bool chain_dx = !dqk_b16_on(d) && !pb16 && getenv("MMF_DX_CHAIN");
  // (4) dZ_m = gate(P_m) * [direct + sum_q dQ W_q + sum_k dK W_k (+ dV W_v)]
  {
    std::vector<GemmJob> jobs;
    for (int m = 0; m < M; ++m) {
      const int L = Lm(d, m);
      const bool pe = pool && poole_in_dz(d, m);
      GemmJob j = make_job(B * L, H, w.dZ[m], H,
                           EPI_GATE | (pool && !pe ? EPI_ADDMAT : EPI_ROWADD) | (proj_b16_on(d) ? EPI_BF16 : 0));
      if (pool && !pe) {
        j.g.addm = w.E[m];
        j.g.ld_addm = H;
      } else {
        j.g.rowadd = w.cvec + (size_t)m * H;
        j.g.ld_rowadd = M * H;
        j.g.rowadd_div = L;
        j.g.rowadd_scale = 1.f / (float)L;
      }
      j.g.gate = s.P[m];
      j.g.ld_gate = H;
      // (proj_b16_on: the sign of P_m from its bf16 copy -- half the gate bytes; MMF_NO_GATE_B16=1 A/B)
      if (proj_b16_on(d) && s.Pb[m] && !getenv("MMF_NO_GATE_B16")) {
        j.g.gate = reinterpret_cast<const float*>(s.Pb[m]);
        j.g.epi |= EPI_GATE_B16;
      }
      j.g.gate_scale = gscale;
      const bool b16 = dqk_b16_on(d);
      if (b16 && qk_cat_on(d)) {
        // one source: the modality's dQ / dK block matrix against its stacked W copies (K = ncat H,
        // the slots in the order the separate sources had)
        if (s.ncat[m] > 0)
          add_src(j, opnd(w.dQc[m], s.ncat[m] * H), opnd(reinterpret_cast<const float*>(s.Wc[m]), H), s.ncat[m] * H);
      } else {
        for (int g = 0; g < d->num_pairs; ++g) {
          const bool sk = single_key(d, g);
          // (bf16: dQ / dK and the forward's W_q / W_k copies, launch_gemm_b16's RK x KR form)
          const float* wq = b16 ? reinterpret_cast<const float*>(s.Wqb[g]) : W->q[g].w;
          const float* wk = b16 ? reinterpret_cast<const float*>(s.Wkb[g]) : W->k[g].w;
          if (d->pair_q[g] == m && !sk) add_src(j, opnd(w.dQ[g], s.ldq[g]), opnd(wq, H), H);
          if (d->pair_k[g] == m) {
            if (!sk) add_src(j, opnd(w.dK[g], s.ldk[g]), opnd(wk, H), H);
            if (!pool) add_src(j, opnd(w.dV[g], H), opnd(W->v[g].w, H), H);
          }
        }
      }
      if (pe) {
        // E_m = c_m / L (the ROWADD above) + sum over pairs keyed by m of pbar^T dU: per sample a
        // K = heads contraction, rows b*L + l of pbarT (B, L, heads) against dU_b (heads, H)
        j.g.seg_rows = L;
        for (int g = 0; g < d->num_pairs; ++g)
          if (d->pair_k[g] == m && j.nsrc < GEMM_MAX_SRCS) {
            Operand du = opnd(w.dU[g], H);
            du.seg_stride = nh * H;
            add_src(j, opnd(s.pbarT[g], nh), du, nh);
          }
      }
      if (j.nsrc > GEMM_MAX_SRCS) return fail(MMF_ELIMIT, "too many gradient sources");
      if (chain_dx && has_dx[m]) j.chain = &dxjobs[m];
      jobs.push_back(j);
    }
    // (the dX_m of a chained launch take its dropout p: the dZ epilogue has no dropout site)
    if (dqk_b16_on(d)) STAGE_TRY("bwd.dZ_gemm", launch_gemm_b16(jobs.data(), (int)jobs.size(), st, MODE_RK, MODE_KR));
    else STAGE_TRY("bwd.dZ_gemm", launch_gemm(jobs.data(), (int)jobs.size(), MODE_RK, MODE_KR, chain_dx ? p : 0.f, rng, st));
  }
  // (5) dX_m, unless chained above
  if (!chain_dx) {
    std::vector<GemmJob> jobs;
    for (int m = 0; m < M; ++m)
      if (has_dx[m]) jobs.push_back(dxjobs[m]);
    if (!jobs.empty() && pb16)
      STAGE_TRY("bwd.dx_gemm", launch_gemm_b16(jobs.data(), (int)jobs.size(), st, MODE_RK, MODE_KR, p, rng));
    else if (!jobs.empty())
      STAGE_TRY("bwd.dx_gemm", launch_gemm(jobs.data(), (int)jobs.size(), MODE_RK, MODE_KR, p, rng, st));
  }
  // (6) every weight gradient: split-K slabs, then one deterministic reduce
  // biggest jobs first so every launch (<= 8 jobs) is a full grid
  std::stable_sort(wp.jobs.begin(), wp.jobs.end(), [](const GemmJob& a, const GemmJob& b) {
    const int64_t wa = (int64_t)a.g.nsplit * std::max(1, a.g.nbatch) * a.g.M * a.g.N;
    const int64_t wb = (int64_t)b.g.nsplit * std::max(1, b.g.nbatch) * b.g.M * b.g.N;
    return wa > wb;
  });
  STAGE_TRY("bwd.wgrad_gemm", launch_gemm(wp.jobs.data(), (int)wp.jobs.size(), MODE_KR, MODE_KR, p, rng, st));
  if (!wp.jobs_b16.empty())
    STAGE_TRY("bwd.wgrad_gemm", launch_gemm_b16(wp.jobs_b16.data(), (int)wp.jobs_b16.size(), st, MODE_KR, MODE_KR));
  STAGE_TRY("bwd.wgrad_reduce", launch_reduce(wp.reds.data(), (int)wp.reds.size(), st));
  return MMF_OK;
}

int mmf_hybrid_backward(const mmf_hybrid_desc* d, const mmf_hybrid_params* W, const float* const* x,
                        const float* mask, const void* saved, const float* dlogits, void* workspace,
                        const mmf_hybrid_grads* G, float* const* dx, void* stream) {
  return hybrid_backward(d, W, x, mask, saved, dlogits, workspace, G, dx, stream, false);
}

uint32_t mmf_hybrid_plan_flags(void) { return plan_flags_now(); }

int mmf_hybrid_lean_l1(const mmf_hybrid_desc* d) {
  if (check_hybrid(d) != MMF_OK) return 0;
  return lean_l1_desc(d) ? 1 : 0;
}

size_t mmf_hybrid_train_sync_bytes(const mmf_hybrid_desc* d) {
  if (check_hybrid(d) != MMF_OK) return 0;
  // per 16-sample tile: arrivals, head done, done seen, one arrival count per key modality; the
  // error word (l1.hip SyncWords)
  const size_t tiles = ((size_t)d->batch + 15) / 16;
  return std::max<size_t>(256, (4 * (tiles * (3 + L1_MAXM) + 1) + 255) / 256 * 256);
}

int mmf_hybrid_train_status(const mmf_hybrid_desc* d, void* sync, int clear, void* stream) {
  const int rc = check_hybrid(d);
  if (rc) return rc;
  if (!sync) return fail(MMF_EINVAL, "train status: null sync buffer");
  // the error word follows the tile words (l1.hip SyncWords)
  const size_t tiles = ((size_t)d->batch + 15) / 16;
  uint32_t* err = static_cast<uint32_t*>(sync) + tiles * (3 + L1_MAXM);
  hipStream_t st = (hipStream_t)stream;
  uint32_t v = 0;
  if (hipMemcpyAsync(&v, err, sizeof(v), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return fail(MMF_EHIP, "train status: reading the error word failed");
  if (v == 0) return MMF_OK;
  if (clear) {
    static const uint32_t zero = 0;
    if (hipMemcpyAsync(err, &zero, sizeof(zero), hipMemcpyHostToDevice, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return fail(MMF_EHIP, "train status: clearing the error word failed");
  }
  return fail(MMF_ETIMEOUT, "train step: a workgroup of the one-launch L = 1 step gave up waiting for its tile's "
                            "head (the grid was not co-resident); that step's gradients are incomplete (its loss "
                            "is NaN, its update applied a zero gradient); the sync words were reset");
}

int mmf_hybrid_train_step_part(int part, const mmf_hybrid_desc* d, const mmf_hybrid_params* W,
                               const float* const* x, const float* mask, const int64_t* labels,
                               float label_smoothing, float loss_scale, uint64_t* rng_state, void* saved,
                               void* workspace, void* sync, float* logits, float* fusion_weights, float* loss_out,
                               float* dlogits, const mmf_hybrid_grads* G, float* const* dx, float* clip_partial,
                               int64_t* step_dev, const float* grad_flat, int64_t grad_n, void* stream) {
  int rc = check_hybrid(d);
  if (rc) return rc;
  if (part < 0 || part > 2) return fail(MMF_EINVAL, "train step: part must be 0, 1 or 2 (got %d)", part);
  if (!W || !x || !mask || !labels || !saved || !workspace || !logits || !loss_out || !dlogits || !G)
    return fail(MMF_EINVAL, "null argument");
  if (clip_partial && !step_dev) return fail(MMF_EINVAL, "train step: clip partials need the step counter");
  if (clip_partial && part != 0) return fail(MMF_EINVAL, "train step: clip partials need the whole step (part 0)");
  // (the one-launch kernel needs its tiles x pairs workgroups resident at once, one per CU)
  if (sync && lean_l1(d, W, x) &&
      (int64_t)((d->batch + 15) / 16) * d->num_pairs <= l1_train_capacity(l1_desc_full(d))) {
    if (part == 2) return MMF_OK;   // (every gradient came out of part 1's launches)
    MathScope math_(d->matmul_precision);
    hipStream_t st = (hipStream_t)stream;
    Bump bs(saved);
    Saved s{};
    layout_saved(d, bs, s);
    Bump bw(workspace);
    Ws w;
    layout_ws(d, bw, w);
    if ((rc = check_buffers(d, bs.off, bw.off))) return rc;
    L1Args a;
    L1WgArgs wa;
    fill_l1_bwd(a, wa, d, W, x, mask, s, w, dlogits, G, dx);
    a.rng_live = rng_state;
    a.rng_advance = rng_state;
    a.logits = logits;
    a.weights_out = fusion_weights;
    a.tile_cnt = static_cast<uint32_t*>(sync);
    a.labels = labels;
    a.ls_eps = label_smoothing;
    a.loss_scale = loss_scale;
    a.loss_rows = w.dfused;   // (B x H floats the L = 1 plan leaves unused)
    a.dlogits_out = dlogits;
    wa.loss_rows = w.dfused;
    wa.loss = loss_out;
    wa.clip_partial = clip_partial;   // (the weight-gradient launch writes the clip partials itself)
    wa.step_incr = clip_partial ? step_dev : nullptr;
    STAGE_TRY("train.l1", launch_l1_train(a, wa, st));
    return MMF_OK;
  }
  {
    // the whole step's buffers before its first launch (the forward's launches would otherwise
    // run before the backward's workspace check)
    MathScope math_(d->matmul_precision);
    if ((rc = check_buffers(d, saved_bytes(d) - 256, workspace_bytes(d) - 256))) return rc;
  }
  if (part == 2) {
    // the head-done flag of part 1's forward: the same decision, from the same descriptor and
    // pointers (only the backward's tail launch depends on it, and part 2 runs none)
    return hybrid_backward(d, W, x, mask, saved, dlogits, workspace, G, dx, stream, false, 2);
  }
  // (with the sync words: the pooled tail plan runs the loss and the head backward in its head launch)
  TailTrain tt{labels, label_smoothing, loss_scale, loss_out, dlogits, static_cast<uint32_t*>(sync), workspace, false};
  rc = hybrid_forward(d, W, x, mask, rng_state, saved, logits, fusion_weights, nullptr, stream, sync ? &tt : nullptr);
  if (rc) return rc;
  if (!tt.done) {
    rc = mmf_cross_entropy_ls(d->batch, d->num_classes, logits, labels, label_smoothing, loss_scale, loss_out,
                              dlogits, stream);
    if (rc) return rc;
  }
  rc = hybrid_backward(d, W, x, mask, saved, dlogits, workspace, G, dx, stream, tt.done, part);
  if (rc || !clip_partial) return rc;
  if (!grad_flat || grad_n < 0 || (reinterpret_cast<uintptr_t>(grad_flat) & 15))
    return fail(MMF_EINVAL, "train step: clip partials need the 16-byte aligned flat gradient");
  hipStream_t st = (hipStream_t)stream;
  STAGE_TRY("optim.clip_norm", launch_grad_sumsq(grad_n, grad_flat, clip_partial, step_dev, st));
  return MMF_OK;
}

int mmf_hybrid_train_step(const mmf_hybrid_desc* d, const mmf_hybrid_params* W, const float* const* x,
                          const float* mask, const int64_t* labels, float label_smoothing, float loss_scale,
                          uint64_t* rng_state, void* saved, void* workspace, void* sync, float* logits,
                          float* fusion_weights, float* loss_out, float* dlogits, const mmf_hybrid_grads* G,
                          float* const* dx, float* clip_partial, int64_t* step_dev, const float* grad_flat,
                          int64_t grad_n, void* stream) {
  return mmf_hybrid_train_step_part(0, d, W, x, mask, labels, label_smoothing, loss_scale, rng_state, saved,
                                    workspace, sync, logits, fusion_weights, loss_out, dlogits, G, dx, clip_partial,
                                    step_dev, grad_flat, grad_n, stream);
}

}  // extern "C"
