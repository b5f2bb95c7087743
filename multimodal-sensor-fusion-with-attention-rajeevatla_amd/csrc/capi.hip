// C-ABI entry points (include/mmfusion.h) other than HybridFusion (hybrid.hip):
// standalone CrossModalAttention, compute_adaptive_weights, the training-step
// helpers (cross-entropy, AdamW), profiling and error reporting.  Every entry
// point validates first, then only enqueues kernels on the caller's stream.
#include <cmath>
#include <map>

#include "capi_util.h"

namespace mmf {

thread_local std::string g_err;
Prof g_prof;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

}  // namespace mmf

using namespace mmf;

namespace {

// ------------------------------------------------------------ CrossModalAttention
struct CmaSaved { RngSnap* rng; float *Q, *K, *V, *O, *lse, *P, *Pd; };

// Lk == 1 (the reference's 2-D inputs): softmax over one key, no Q / K work
// (single_key.hip); Q, K and the LSE are not kept.
inline bool cma_single_key(const mmf_cma_desc* d) { return d->lk == 1; }
// head_dim > MMF_MAX_HEAD_DIM: materialised scores + GEMMs (wide.hip)
inline bool cma_wide(const mmf_cma_desc* d) {
  return !cma_single_key(d) && d->hidden / d->num_heads > MMF_MAX_HEAD_DIM;
}

void layout_cma(const mmf_cma_desc* d, Bump& bp, CmaSaved& s) {
  const size_t B = d->batch, H = d->hidden;
  const bool sk = cma_single_key(d);
  s.rng = bp.take<RngSnap>(1);
  s.Q = sk ? nullptr : bp.take<float>(B * d->lq * H);
  s.K = sk ? nullptr : bp.take<float>(B * d->lk * H);
  s.V = bp.take<float>(B * d->lk * H);
  s.O = bp.take<float>(B * d->lq * H);
  s.lse = sk ? nullptr : bp.take<float>(B * d->num_heads * d->lq);
  s.P = s.Pd = nullptr;
  if (cma_wide(d)) {
    s.P = bp.take<float>(B * d->num_heads * d->lq * d->lk);
    s.Pd = bp.take<float>(B * d->num_heads * d->lq * d->lk);
  }
}

struct CmaWs { float *dO, *dsum, *dQ, *dK, *dV, *dS, *dPd; };

void layout_cma_ws(const mmf_cma_desc* d, Bump& bp, CmaWs& w) {
  const size_t B = d->batch, H = d->hidden;
  const bool sk = cma_single_key(d);
  w.dO = bp.take<float>(B * d->lq * H);
  w.dsum = sk ? nullptr : bp.take<float>(B * d->num_heads * d->lq);
  w.dQ = sk ? nullptr : bp.take<float>(B * d->lq * H);
  w.dK = sk ? nullptr : bp.take<float>(B * d->lk * H);
  w.dV = bp.take<float>(B * d->lk * H);
  w.dS = w.dPd = nullptr;
  if (cma_wide(d)) {
    w.dS = bp.take<float>(B * d->num_heads * d->lq * d->lk);
    w.dPd = bp.take<float>(B * d->num_heads * d->lq * d->lk);
  }
}

int check_cma(const mmf_cma_desc* d) {
  if (!d) return fail(MMF_EINVAL, "null descriptor");
  if (d->matmul_precision != MMF_PRECISION_HIGHEST && d->matmul_precision != MMF_PRECISION_MEDIUM &&
      d->matmul_precision != MMF_PRECISION_HIGH)
    return fail(MMF_EINVAL, "bad matmul_precision %d", d->matmul_precision);
  if (d->batch < 1 || d->lq < 1 || d->lk < 1 || d->query_dim < 1 || d->key_dim < 1)
    return fail(MMF_EINVAL, "bad CrossModalAttention shape");
  if (d->num_heads < 1 || d->hidden % d->num_heads != 0)
    return fail(MMF_EINVAL, "hidden_dim (%d) must be divisible by num_heads (%d)", d->hidden,
                d->num_heads);
  if (d->mask_mode < 0 || d->mask_mode > 2) return fail(MMF_EINVAL, "bad mask_mode");
  if (d->hidden % 4 != 0) return fail(MMF_ELIMIT, "hidden_dim must be a multiple of 4 (got %d)", d->hidden);
  if (cma_wide(d) && !wide_supported(d->batch, d->num_heads, d->lq, d->lk))
    return fail(MMF_ELIMIT, "head_dim %d: the (heads x Lq x Lk) score tensor is too large",
                d->hidden / d->num_heads);
  if (!(d->dropout >= 0.f && d->dropout < 1.f)) return fail(MMF_EINVAL, "dropout must be in [0, 1)");
  return MMF_OK;
}

size_t cma_partials_bytes(const mmf_cma_desc* d) {
  const int B = d->batch, H = d->hidden;
  return slab_bytes(H, H, B * d->lq) + slab_bytes(H, d->query_dim, B * d->lq) +
         slab_bytes(H, d->key_dim, B * d->lk) * 2;
}

AttnPair cma_pair(const mmf_cma_desc* d, const CmaSaved& s, const float* mask) {
  AttnPair a;
  memset(&a, 0, sizeof(a));
  a.q = s.Q; a.k = s.K; a.v = s.V; a.o = s.O; a.lse = s.lse;
  a.kmask = mask; a.kmask_mode = d->mask_mode; a.kmask_ld = d->mask_mode == 2 ? d->lk : 1;
  a.Lq = d->lq; a.Lk = d->lk;
  a.ldq = a.ldk = a.ldv = a.ldo = d->hidden;
  a.drop_site = SITE_ATTN;
  return a;
}

WidePair cma_wide_pair(const mmf_cma_desc* d, const CmaSaved& s, const float* mask) {
  WidePair a;
  memset(&a, 0, sizeof(a));
  a.q = s.Q; a.k = s.K; a.v = s.V;
  a.ldq = a.ldk = a.ldv = a.ldo = d->hidden;
  a.kmask = mask; a.kmask_mode = d->mask_mode; a.kmask_ld = d->mask_mode == 2 ? d->lk : 1;
  a.Lq = d->lq; a.Lk = d->lk;
  a.drop_site = SITE_ATTN;
  a.P = s.P; a.Pd = s.Pd;
  a.o = s.O;
  return a;
}

SkPair cma_sk(const mmf_cma_desc* d, const CmaSaved& s, const float* mask) {
  SkPair a;
  memset(&a, 0, sizeof(a));
  a.kmask = mask; a.kmask_mode = d->mask_mode; a.kmask_ld = 1;   // (B,) or (B, Lk = 1)
  a.Lq = d->lq;
  a.drop_site = SITE_ATTN;
  a.v = s.V; a.ldv = d->hidden;
  a.o = s.O; a.ldo = d->hidden;
  return a;
}

}  // namespace

namespace mmf {

thread_local ProfArm* g_prof_arm = nullptr;

bool prof_capturing(hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone;
}

SideStream* side_stream(bool create) {
  static thread_local std::map<int, SideStream> streams;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  auto it = streams.find(dev);
  if (it != streams.end()) return &it->second;
  if (!create) return nullptr;
  SideStream ss{};
  if (hipStreamCreateWithFlags(&ss.s, hipStreamNonBlocking) != hipSuccess) return nullptr;
  if (hipEventCreateWithFlags(&ss.fork_ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ss.join_ev, hipEventDisableTiming) != hipSuccess)
    return nullptr;
  return &(streams[dev] = ss);
}

bool prof_arm_begin(ProfArm& arm, hipStream_t st) {
  if (!g_prof.on || prof_capturing(st)) return false;
  arm.a = g_prof.ev();
  arm.b = g_prof.ev();
  arm.launches = 0;
  if (!arm.a || !arm.b) return false;
  g_prof_arm = &arm;
  return true;
}

void prof_arm_end(ProfArm& arm, hipStream_t st, const char* kernel, double flops, double bytes) {
  if (g_prof_arm == &arm) g_prof_arm = nullptr;
  if (!g_prof.on || arm.launches == 0) return;
  hipEvent_t end = arm.b;
  if (arm.launches > 1) {   // several launches: the scope ends after the last one
    end = g_prof.ev();
    if (!end || hipEventRecord(end, st) != hipSuccess) return;
  }
  g_prof.launches.push_back({g_prof.cur_stage, kernel, flops, bytes, arm.a, end});
}

thread_local int g_math_mode = 0;

}  // namespace mmf

extern "C" {

const char* mmf_last_error(void) { return g_err.c_str(); }
const char* mmf_version(void) { return "mmfusion 0.3 (gfx950, fp32 / bf16 MFMA, pooled HybridFusion)"; }

void mmf_profile_begin(void) {
  g_prof.on = true;
  g_prof.cur_stage = "";
  g_prof.recs.clear();
  g_prof.launches.clear();
  g_prof.next = 0;
}

// Ends profiling: waits for the recorded events and writes tab-separated lines
// into out, in launch order:
//   "S <stage> <ms>"                              one per launch group
//   "L <stage> <kernel> <ms> <flops> <bytes>"     one per kernel launch
// (flops / bytes: the launch's algorithmic work, mmf_internal.h ProfLaunch).
// Returns the bytes needed.
size_t mmf_profile_end(char* out, size_t cap) {
  std::string s;
  char line[320];
  for (const ProfRec& r : g_prof.recs) {
    float ms = 0.f;
    if (hipEventSynchronize(r.b) == hipSuccess) (void)hipEventElapsedTime(&ms, r.a, r.b);
    snprintf(line, sizeof(line), "S\t%s\t%.6f\n", r.name, (double)ms);
    s += line;
  }
  for (const LaunchRec& r : g_prof.launches) {
    float ms = 0.f;
    if (hipEventSynchronize(r.b) == hipSuccess) (void)hipEventElapsedTime(&ms, r.a, r.b);
    snprintf(line, sizeof(line), "L\t%s\t%s\t%.6f\t%.6e\t%.6e\n", r.stage, r.kernel, (double)ms, r.flops,
             r.bytes);
    s += line;
  }
  g_prof.on = false;
  g_prof.cur_stage = "";
  g_prof.recs.clear();
  g_prof.launches.clear();
  g_prof.next = 0;
  if (out && cap) {
    const size_t n = s.size() < cap - 1 ? s.size() : cap - 1;
    memcpy(out, s.data(), n);
    out[n] = 0;
  }
  return s.size() + 1;
}

// compute_adaptive_weights workspace: the head-forward scratch (pooled, scores,
// weights, fused) plus the backward's dscore and a cvec (B, M, H) scratch used
// when the caller does not want the feature gradients.
namespace {
struct AdaptiveWs { float *pooled, *scores, *weights, *fused, *dscore, *cvec; };
void layout_adaptive(Bump& bp, int32_t batch, int32_t M, int32_t H, AdaptiveWs& w) {
  w.pooled = bp.take<float>((size_t)batch * M * H);
  w.scores = bp.take<float>((size_t)batch * M);
  w.weights = bp.take<float>((size_t)batch * M);
  w.fused = bp.take<float>((size_t)batch * H);
  w.dscore = bp.take<float>((size_t)batch * M);
  w.cvec = bp.take<float>((size_t)batch * M * H);
}
int check_adaptive(int32_t batch, int32_t M, int32_t H) {
  if (batch < 1 || M < 1 || M > MMF_MAX_MODALITIES || H < 4 || H % 4 != 0 || H > 1024)
    return fail(MMF_ELIMIT, "adaptive weights: unsupported shape B=%d M=%d H=%d", batch, M, H);
  return MMF_OK;
}
// head arguments of src/fusion.py:429-479 alone: one (B, H) source per modality,
// no mask scaling of the features, no list-length divisor
void fill_adaptive(HeadArgs& ha, int32_t batch, int32_t M, int32_t H, const float* const* feats,
                   const float* mask, const mmf_linear* gate, const AdaptiveWs& w) {
  memset(&ha, 0, sizeof(ha));
  ha.B = batch; ha.M = M; ha.H = H; ha.mask = mask;
  ha.scale_by_mask = 0;
  for (int m = 0; m < M; ++m) {
    ha.src[ha.nsrc] = feats[m];
    ha.src_mod[ha.nsrc] = m;
    ha.src_L[ha.nsrc] = 1;
    ha.src_scale[ha.nsrc++] = 1.f;
    ha.inv_cnt[m] = 1.f;
    ha.gate_w[m] = gate[m].w;
    ha.gate_b[m] = gate[m].b;
  }
  ha.pooled = w.pooled; ha.scores = w.scores; ha.weights = w.weights; ha.fused = w.fused;
}
}  // namespace

size_t mmf_adaptive_weights_workspace_bytes(int32_t batch, int32_t M, int32_t H) {
  if (batch < 1 || M < 1 || H < 1) return 0;
  Bump bp(nullptr);
  AdaptiveWs w;
  layout_adaptive(bp, batch, M, H, w);
  return bp.off + 256;
}

int mmf_adaptive_weights(int32_t batch, int32_t M, int32_t H, const float* const* feats,
                         const float* mask, const mmf_linear* gate, float* weights, void* workspace,
                         void* stream) {
  if (int rc = check_adaptive(batch, M, H)) return rc;
  if (!feats || !mask || !gate || !weights || !workspace) return fail(MMF_EINVAL, "null argument");
  hipStream_t st = (hipStream_t)stream;
  Bump bp(workspace);
  AdaptiveWs w;
  layout_adaptive(bp, batch, M, H, w);
  HeadArgs ha;
  fill_adaptive(ha, batch, M, H, feats, mask, gate, w);
  ha.weights_out = weights;
  STAGE_TRY("adaptive_weights", launch_head_fwd(ha, st));
  return MMF_OK;
}

int mmf_adaptive_weights_backward(int32_t batch, int32_t M, int32_t H, const float* const* feats,
                                  const float* mask, const mmf_linear* gate, const float* dweights,
                                  float* dfeats, const mmf_linear_grad* dgate, void* workspace,
                                  void* stream) {
  if (int rc = check_adaptive(batch, M, H)) return rc;
  if (!feats || !mask || !gate || !dweights || !workspace) return fail(MMF_EINVAL, "null argument");
  hipStream_t st = (hipStream_t)stream;
  Bump bp(workspace);
  AdaptiveWs w;
  layout_adaptive(bp, batch, M, H, w);
  HeadArgs ha;
  fill_adaptive(ha, batch, M, H, feats, mask, gate, w);
  // recompute the scores (the backward of the masked softmax re-derives its branch from them)
  STAGE_TRY("adaptive_weights.bwd.recompute", launch_head_fwd(ha, st));
  ha.dfused = nullptr;
  ha.dweights = dweights;
  ha.dscore = w.dscore;
  ha.cvec = dfeats ? dfeats : w.cvec;   // d feat_m = dscore_m * gate_w[m]  (B, M, H)
  STAGE_TRY("adaptive_weights.bwd.head", launch_head_bwd(ha, st));
  if (dgate) {
    float* dgw[MMF_MAX_MODALITIES];
    float* dgb[MMF_MAX_MODALITIES];
    for (int m = 0; m < M; ++m) {
      if (!dgate[m].w || !dgate[m].b) return fail(MMF_EINVAL, "null gate gradient");
      dgw[m] = dgate[m].w;
      dgb[m] = dgate[m].b;
    }
    STAGE_TRY("adaptive_weights.bwd.gate_wgrad", launch_gate_wgrad(batch, M, H, w.dscore, w.pooled, dgw, dgb, st));
  }
  return MMF_OK;
}

size_t mmf_cma_saved_bytes(const mmf_cma_desc* d) {
  if (check_cma(d) != MMF_OK) return 0;
  Bump bp(nullptr);
  CmaSaved s;
  layout_cma(d, bp, s);
  return bp.off + 256;
}

size_t mmf_cma_workspace_bytes(const mmf_cma_desc* d) {
  if (check_cma(d) != MMF_OK) return 0;
  Bump bp(nullptr);
  CmaWs w;
  layout_cma_ws(d, bp, w);
  return bp.off + 256 + cma_partials_bytes(d);
}

int mmf_cma_forward(const mmf_cma_desc* d, const mmf_cma_params* W, const float* query,
                    const float* key, const float* value, const float* mask,
                    const uint64_t* rng_state, void* saved, float* attended, float* attn_weights,
                    void* stream) {
  int rc = check_cma(d);
  if (rc) return rc;
  mmf::MathScope math_(d->matmul_precision);
  if (!W || !query || !key || !value || !saved || !attended) return fail(MMF_EINVAL, "null argument");
  if (d->mask_mode && !mask) return fail(MMF_EINVAL, "mask_mode set but mask is null");
  hipStream_t st = (hipStream_t)stream;
  const int B = d->batch, H = d->hidden, hd = H / d->num_heads;
  const bool drop = d->training && d->dropout > 0.f;
  const float p = drop ? d->dropout : 0.f;
  if (drop && !rng_state) return fail(MMF_EINVAL, "training with dropout needs rng_state");
  Bump bp(saved);
  CmaSaved s;
  layout_cma(d, bp, s);
  if (rng_state) STAGE_TRY("cma.fwd.rng", launch_rng_snapshot(rng_state, s.rng, st));
  const RngSnap* rng = rng_state ? s.rng : nullptr;
  const bool sk = cma_single_key(d);
  GemmJob jobs[3];
  int nj = 0;
  if (!sk) {
    jobs[nj] = make_job(B * d->lq, H, s.Q, H, EPI_BIAS);
    jobs[nj].g.bias = W->q.b;
    add_src(jobs[nj++], opnd(query, d->query_dim), opnd(W->q.w, d->query_dim), d->query_dim);
    jobs[nj] = make_job(B * d->lk, H, s.K, H, EPI_BIAS);
    jobs[nj].g.bias = W->k.b;
    add_src(jobs[nj++], opnd(key, d->key_dim), opnd(W->k.w, d->key_dim), d->key_dim);
  }
  jobs[nj] = make_job(B * d->lk, H, s.V, H, EPI_BIAS);
  jobs[nj].g.bias = W->v.b;
  add_src(jobs[nj++], opnd(value, d->key_dim), opnd(W->v.w, d->key_dim), d->key_dim);
  STAGE_TRY("cma.fwd.qkv_gemm", launch_gemm(jobs, nj, MODE_RK, MODE_RK, 0.f, rng, st));
  if (sk) {
    // softmax over one key (src/attention.py:118-130): P' = mask indicator * dropout keep
    SkPair a = cma_sk(d, s, mask);
    STAGE_TRY("cma.fwd.attn_single_key", launch_sk_out(&a, 1, B, d->num_heads, hd, p, rng, st));
    if (attn_weights) {
      a.probs = attn_weights;
      STAGE_TRY("cma.fwd.attn_probs_single_key", launch_sk_fwd(&a, 1, B, d->num_heads, hd, p, rng, st));
    }
  } else if (cma_wide(d)) {
    WidePair a = cma_wide_pair(d, s, mask);
    a.probs = attn_weights;
    const float scale = 1.0f / std::sqrt((float)hd);
    STAGE_TRY("cma.fwd.attn_wide", launch_wide_fwd(&a, 1, B, d->num_heads, hd, scale, p, rng, false, st));
  } else {
    AttnPair a = cma_pair(d, s, mask);
    a.probs = attn_weights;
    const float scale = 1.0f / std::sqrt((float)hd);
    STAGE_TRY("cma.fwd.attn", launch_attn_fwd(&a, 1, B, d->num_heads, hd, scale, p, rng, st));
    if (attn_weights)
      STAGE_TRY("cma.fwd.attn_probs", launch_attn_probs(&a, 1, B, d->num_heads, hd, scale, p, rng, st));
  }
  GemmJob jo = make_job(B * d->lq, H, attended, H, EPI_BIAS);
  jo.g.bias = W->o.b;
  add_src(jo, opnd(s.O, H), opnd(W->o.w, H), H);
  STAGE_TRY("cma.fwd.out_gemm", launch_gemm(&jo, 1, MODE_RK, MODE_RK, 0.f, rng, st));
  return MMF_OK;
}

int mmf_cma_backward(const mmf_cma_desc* d, const mmf_cma_params* W, const float* query,
                     const float* key, const float* value, const float* mask, const void* saved,
                     const float* dA, void* workspace, const mmf_cma_grads* G, float* dquery,
                     float* dkey, float* dvalue, void* stream) {
  int rc = check_cma(d);
  if (rc) return rc;
  mmf::MathScope math_(d->matmul_precision);
  if (!W || !query || !key || !value || !saved || !dA || !workspace || !G)
    return fail(MMF_EINVAL, "null argument");
  hipStream_t st = (hipStream_t)stream;
  const int B = d->batch, H = d->hidden, hd = H / d->num_heads;
  const bool drop = d->training && d->dropout > 0.f;
  const float p = drop ? d->dropout : 0.f;
  Bump bs(const_cast<void*>(saved));
  CmaSaved s;
  layout_cma(d, bs, s);
  const RngSnap* rng = s.rng;
  Bump bw(workspace);
  CmaWs w;
  layout_cma_ws(d, bw, w);
  const bool sk = cma_single_key(d);
  WgradPlan wp;
  plan_wgrad(wp, bw, H, H, B * d->lq, opnd(dA, H), opnd(s.O, H), G->o.w, G->o.b);
  if (sk) {
    // softmax over one key: query_proj / key_proj get exactly zero gradient
    plan_zero(wp, H, d->query_dim, G->q.w, G->q.b);
    plan_zero(wp, H, d->key_dim, G->k.w, G->k.b);
  } else {
    plan_wgrad(wp, bw, H, d->query_dim, B * d->lq, opnd(w.dQ, H), opnd(query, d->query_dim), G->q.w, G->q.b);
    plan_wgrad(wp, bw, H, d->key_dim, B * d->lk, opnd(w.dK, H), opnd(key, d->key_dim), G->k.w, G->k.b);
  }
  plan_wgrad(wp, bw, H, d->key_dim, B * d->lk, opnd(w.dV, H), opnd(value, d->key_dim), G->v.w, G->v.b);
  if (bw.off > mmf_cma_workspace_bytes(d)) return fail(MMF_EINVAL, "internal: workspace overflow");
  {
    GemmJob j = make_job(B * d->lq, H, w.dO, H, 0);
    add_src(j, opnd(dA, H), opnd(W->o.w, H), H);
    STAGE_TRY("cma.bwd.dO_gemm", launch_gemm(&j, 1, MODE_RK, MODE_KR, 0.f, rng, st));
  }
  std::vector<GemmJob> jobs;
  if (sk) {
    SkPair a = cma_sk(d, s, mask);
    a.dout = w.dO; a.dv = w.dV;
    STAGE_TRY("cma.bwd.attn_single_key_dv", launch_sk_dv(&a, 1, B, d->num_heads, hd, p, rng, st));
    // the query and the key reach the output only through the one-key softmax: zero gradient
    // (a kernel, not hipMemsetAsync: a memset captured into a torch.compile "reduce-overhead"
    // HIP graph left the buffers unwritten on replay)
    float* zp[2] = {dquery, dkey};
    const int64_t zn[2] = {(int64_t)B * d->lq * d->query_dim, (int64_t)B * d->lk * d->key_dim};
    STAGE_TRY("cma.bwd.zero_qk_grads", launch_zero_fill(zp, zn, 2, st));
  } else if (cma_wide(d)) {
    WidePair a = cma_wide_pair(d, s, mask);
    a.dout = w.dO; a.dPd = w.dPd; a.dS = w.dS; a.dq = w.dQ; a.dk = w.dK; a.dv = w.dV;
    const float scale = 1.0f / std::sqrt((float)hd);
    STAGE_TRY("cma.bwd.attn_wide", launch_wide_bwd(&a, 1, B, d->num_heads, hd, scale, p, rng, false, st));
  } else {
    AttnPair a = cma_pair(d, s, mask);
    a.dout = w.dO; a.dsum = w.dsum; a.dq = w.dQ; a.dk = w.dK; a.dv = w.dV;
    const float scale = 1.0f / std::sqrt((float)hd);
    STAGE_TRY("cma.bwd.attn", launch_attn_bwd(&a, 1, B, d->num_heads, hd, scale, p, rng, st));
  }
  if (dquery && !sk) {
    GemmJob j = make_job(B * d->lq, d->query_dim, dquery, d->query_dim, 0);
    add_src(j, opnd(w.dQ, H), opnd(W->q.w, d->query_dim), H);
    jobs.push_back(j);
  }
  if (dkey && !sk) {
    GemmJob j = make_job(B * d->lk, d->key_dim, dkey, d->key_dim, 0);
    add_src(j, opnd(w.dK, H), opnd(W->k.w, d->key_dim), H);
    jobs.push_back(j);
  }
  if (dvalue) {
    GemmJob j = make_job(B * d->lk, d->key_dim, dvalue, d->key_dim, 0);
    add_src(j, opnd(w.dV, H), opnd(W->v.w, d->key_dim), H);
    jobs.push_back(j);
  }
  if (!jobs.empty())
    STAGE_TRY("cma.bwd.dx_gemm", launch_gemm(jobs.data(), (int)jobs.size(), MODE_RK, MODE_KR, 0.f, rng, st));
  STAGE_TRY("cma.bwd.wgrad_gemm", launch_gemm(wp.jobs.data(), (int)wp.jobs.size(), MODE_KR, MODE_KR, 0.f, rng, st));
  STAGE_TRY("cma.bwd.wgrad_reduce", launch_reduce(wp.reds.data(), (int)wp.reds.size(), st));
  return MMF_OK;
}

int mmf_cross_entropy_ls(int32_t batch, int32_t classes, const float* logits, const int64_t* labels,
                         float smoothing, float grad_scale, float* loss_out, float* dlogits,
                         void* stream) {
  if (batch < 1 || classes < 1 || !logits || !labels || !loss_out || !dlogits)
    return fail(MMF_EINVAL, "bad cross-entropy arguments");
  hipStream_t st = (hipStream_t)stream;
  STAGE_TRY("loss.cross_entropy", launch_cross_entropy(batch, classes, logits, labels, smoothing,
                                                       grad_scale, loss_out, dlogits, st));
  return MMF_OK;
}

int mmf_adamw_step(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                   int64_t* step_dev, float lr, float beta1, float beta2, float eps,
                   float weight_decay, float grad_scale, void* stream) {
  if (n < 0 || !param || !grad || !exp_avg || !exp_avg_sq || !step_dev)
    return fail(MMF_EINVAL, "bad AdamW arguments");
  hipStream_t st = (hipStream_t)stream;
  STAGE_TRY("optim.adamw", launch_adamw(n, param, grad, exp_avg, exp_avg_sq, step_dev, lr, beta1, beta2,
                                        eps, weight_decay, grad_scale, st));
  return MMF_OK;
}

size_t mmf_grad_clip_workspace_bytes(void) { return grad_clip_workspace_bytes() + 256; }

int mmf_grad_clip_coef(int64_t n, const float* grad, float grad_scale, float max_norm, float* total_norm,
                       float* clip_coef, void* workspace, void* stream) {
  if (n < 0 || !grad || !clip_coef || !workspace) return fail(MMF_EINVAL, "bad gradient-clip arguments");
  if (reinterpret_cast<uintptr_t>(grad) & 15) return fail(MMF_EINVAL, "gradient-clip: grad must be 16-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  STAGE_TRY("optim.clip_norm", launch_grad_clip_coef(n, grad, grad_scale, max_norm, total_norm, clip_coef,
                                                     (float*)workspace, st));
  return MMF_OK;
}

int mmf_clip_adamw_step_dev(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                            int64_t* step_dev, const float* lr_dev, float max_norm, float* total_norm,
                            float* clip_coef, void* workspace, float beta1, float beta2, float eps,
                            float weight_decay, float grad_scale, void* stream) {
  if (n < 0 || !param || !grad || !exp_avg || !exp_avg_sq || !step_dev || !lr_dev || !workspace)
    return fail(MMF_EINVAL, "bad clip+AdamW arguments");
  if (reinterpret_cast<uintptr_t>(grad) & 15) return fail(MMF_EINVAL, "clip+AdamW: grad must be 16-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  STAGE_TRY("optim.clip_adamw", launch_clip_adamw(n, param, grad, exp_avg, exp_avg_sq, step_dev, lr_dev, beta1,
                                                  beta2, eps, weight_decay, grad_scale, max_norm, total_norm,
                                                  clip_coef, (float*)workspace, st));
  return MMF_OK;
}

int mmf_clip_adamw_apply_dev(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                             int64_t* step_dev, const float* lr_dev, float max_norm, float* total_norm,
                             float* clip_coef, void* workspace, float beta1, float beta2, float eps,
                             float weight_decay, float grad_scale, void* stream) {
  if (n < 0 || !param || !grad || !exp_avg || !exp_avg_sq || !step_dev || !lr_dev || !workspace)
    return fail(MMF_EINVAL, "bad clip+AdamW arguments");
  hipStream_t st = (hipStream_t)stream;
  STAGE_TRY("optim.clip_adamw", launch_clip_adamw_apply(n, param, grad, exp_avg, exp_avg_sq, step_dev, lr_dev, beta1,
                                                        beta2, eps, weight_decay, grad_scale, max_norm, total_norm,
                                                        clip_coef, (const float*)workspace, st));
  return MMF_OK;
}

int mmf_grad_accumulate(int64_t n, const float* src, float* dst, void* stream) {
  if (n < 0 || (n > 0 && (!src || !dst))) return fail(MMF_EINVAL, "bad gradient-accumulate arguments");
  if ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15)
    return fail(MMF_EINVAL, "gradient accumulate: buffers must be 16-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  STAGE_TRY("optim.grad_accum", launch_grad_accum(n, src, dst, st));
  return MMF_OK;
}

size_t mmf_gemm_bf16_workspace_bytes(int32_t M, int32_t N, int32_t K, int32_t nsplit) {
  if (M < 1 || N < 1 || K < 1 || nsplit < 1) return 0;
  int ns = nsplit, kchunk = 0;
  split_rows(K, ns, kchunk, nsplit);
  return ((((size_t)ns * M * N * 4) + 255) & ~size_t(255)) + ((((size_t)ns * M * 4) + 255) & ~size_t(255)) + 256;
}

int mmf_gemm_bf16(int32_t M, int32_t N, int32_t K, const void* A, int32_t lda, int32_t a_kmajor, const void* B,
                  int32_t ldb, int32_t b_kmajor, const float* bias, void* C, int32_t ldc, int32_t c_bf16,
                  void* workspace, int32_t nsplit, float* bias_grad, void* stream) {
  if (M < 1 || N < 1 || K < 1 || !A || !B || !C || ldc < N || nsplit < 1)
    return fail(MMF_EINVAL, "bad bf16 GEMM arguments");
  if (a_kmajor && !b_kmajor) return fail(MMF_EINVAL, "bf16 GEMM: A k-major needs B k-major");
  if ((nsplit > 1 || bias_grad) && (!workspace || !a_kmajor || bias || c_bf16))
    return fail(MMF_EINVAL, "bf16 GEMM: split-K / bias rows need a workspace, a k-major A and an fp32 C");
  const int amode = a_kmajor ? MODE_KR : MODE_RK, bmode = b_kmajor ? MODE_KR : MODE_RK;
  hipStream_t st = (hipStream_t)stream;
  const Operand a = opnd(static_cast<const float*>(A), lda), b = opnd(static_cast<const float*>(B), ldb);
  if (nsplit == 1 && !bias_grad) {
    GemmJob j = make_job(M, N, static_cast<float*>(C), ldc, (bias ? EPI_BIAS : 0) | (c_bf16 ? EPI_BF16 : 0));
    j.g.bias = bias;
    add_src(j, a, b, K);
    if (!gemm_b16_ok(j, amode, bmode)) return fail(MMF_EINVAL, "bf16 GEMM: operand alignment / extents");
    STAGE_TRY("gemm_bf16", launch_gemm_b16(&j, 1, st, amode, bmode));
    return MMF_OK;
  }
  if (ldc != N) return fail(MMF_EINVAL, "bf16 GEMM: split-K writes a dense C (ldc == N)");
  WgradPlan wp;
  wp.split_hint = nsplit;
  Bump bw(workspace);
  plan_wgrad(wp, bw, M, N, K, a, b, static_cast<float*>(C), bias_grad, bias_grad != nullptr);
  if (!gemm_b16_ok(wp.jobs[0], amode, bmode)) return fail(MMF_EINVAL, "bf16 GEMM: operand alignment / extents");
  STAGE_TRY("gemm_bf16", launch_gemm_b16(wp.jobs.data(), 1, st, amode, bmode));
  STAGE_TRY("gemm_bf16_reduce", launch_reduce(wp.reds.data(), 1, st));
  return MMF_OK;
}

int mmf_adamw_step_dev(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                       int64_t* step_dev, const float* lr_dev, const float* grad_coef_dev, float beta1,
                       float beta2, float eps, float weight_decay, float grad_scale, void* stream) {
  if (n < 0 || !param || !grad || !exp_avg || !exp_avg_sq || !step_dev || !lr_dev)
    return fail(MMF_EINVAL, "bad AdamW arguments");
  hipStream_t st = (hipStream_t)stream;
  STAGE_TRY("optim.adamw", launch_adamw(n, param, grad, exp_avg, exp_avg_sq, step_dev, 0.f, beta1, beta2, eps,
                                        weight_decay, grad_scale, st, lr_dev, grad_coef_dev));
  return MMF_OK;
}

}  // extern "C"
