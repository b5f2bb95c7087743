// C-ABI entry points (include/mmfusion.h): the native orchestration of the
// HybridFusion / CrossModalAttention forward and backward.  Every entry point
// validates shapes first (reference error behaviour is raised by the Python
// mirror before we get here; anything that slips through is MMF_EINVAL), then
// only enqueues kernels on the caller's stream: no allocation, no sync.
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "mmf_internal.h"
#include "mmfusion.h"

using namespace mmf;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

// ---------------------------------------------------------------- profiling
// Optional per-stage hipEvent timing (mmf_profile_begin/_end): every launch
// group is bracketed by two events on the caller's stream.  Off by default
// (then a Stage costs one branch).  Not for use under graph capture.
struct ProfRec { const char* name; hipEvent_t a, b; };
struct Prof {
  bool on = false;
  std::vector<ProfRec> recs;
  std::vector<hipEvent_t> pool;
  size_t next = 0;
  hipEvent_t ev() {
    if (next == pool.size()) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return nullptr;
      pool.push_back(e);
    }
    return pool[next++];
  }
};
Prof g_prof;

struct Stage {
  const char* name;
  hipStream_t st;
  hipEvent_t a = nullptr;
  Stage(const char* n, hipStream_t s) : name(n), st(s) {
    if (g_prof.on) {
      a = g_prof.ev();
      if (a) (void)hipEventRecord(a, st);
    }
  }
  ~Stage() {
    if (g_prof.on && a) {
      hipEvent_t b = g_prof.ev();
      if (b) {
        (void)hipEventRecord(b, st);
        g_prof.recs.push_back({name, a, b});
      }
    }
  }
};

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail(MMF_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_));             \
  } while (0)

// Launch group wrapped in a profiling stage.
#define STAGE_TRY(name, expr)                                                           \
  do {                                                                                  \
    Stage stage_(name, st);                                                             \
    HIP_TRY(expr);                                                                      \
  } while (0)

struct Bump {
  char* base;
  size_t off = 0;
  explicit Bump(void* b) : base((char*)b) {}
  template <class T>
  T* take(size_t n) {
    off = (off + 255) & ~size_t(255);
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += n * sizeof(T);
    return p;
  }
};

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

Operand opnd(const float* p, int ld, int row_div = 1) {
  Operand o;
  o.ptr = p;
  o.ld = ld;
  o.row_div = row_div;
  o.vec = (ld % 4 == 0) && aligned16(p);
  o.xf = -1;
  return o;
}

GemmJob make_job(int M, int N, float* C, int ldc, int epi) {
  GemmJob j;
  memset(&j, 0, sizeof(j));
  j.g.M = M;
  j.g.N = N;
  j.g.C = C;
  j.g.ldc = ldc;
  j.g.epi = epi;
  j.g.nsplit = 1;
  j.g.rowadd_div = 1;
  j.g.rs_div = 1;
  j.g.gate_scale = 1.f;
  return j;
}

void add_src(GemmJob& j, Operand a, Operand b, int K) {
  GemmSrc& s = j.src[j.nsrc++];
  s.a = a;
  s.b = b;
  s.K = K;
}

// Split-K (over the B*L rows) weight-gradient job: out(M x N) = A^T B with the
// partial slabs carved from the workspace, plus the reduce job that sums them.
struct WgradPlan {
  std::vector<GemmJob> jobs;
  std::vector<ReduceJob> reds;
};

// Split of a weight-gradient contraction over `rows`: ~1024 rows per slab.
void split_rows(int rows, int& nsplit, int& kchunk) {
  nsplit = rows / 1024;
  if (nsplit < 1) nsplit = 1;
  if (nsplit > 64) nsplit = 64;
  kchunk = (rows + nsplit - 1) / nsplit;
  kchunk = (kchunk + 31) & ~31;
  nsplit = (rows + kchunk - 1) / kchunk;
}

size_t slab_bytes(int M, int N, int rows) {
  int nsplit, kchunk;
  split_rows(rows, nsplit, kchunk);
  return ((((size_t)nsplit * M * N * 4) + 255) & ~size_t(255)) +
         ((((size_t)nsplit * M * 4) + 255) & ~size_t(255)) + 256;
}

void plan_wgrad(WgradPlan& wp, Bump& ws, int M, int N, int rows, Operand a, Operand b,
                float* out_w, float* out_b, bool with_xf_b = false, const Xform* xfb = nullptr) {
  int nsplit, kchunk;
  split_rows(rows, nsplit, kchunk);
  float* part = ws.take<float>((size_t)nsplit * M * N);
  float* part_db = out_b ? ws.take<float>((size_t)nsplit * M) : nullptr;
  GemmJob j = make_job(M, N, part, N, EPI_PARTIAL);
  j.g.nsplit = nsplit;
  j.g.kchunk = kchunk;
  j.g.part_db = part_db;
  add_src(j, a, b, rows);
  if (with_xf_b) {
    j.has_xf_b[0] = 1;
    j.xf_b[0] = *xfb;
  }
  wp.jobs.push_back(j);
  ReduceJob r;
  r.part = part;
  r.part_db = part_db;
  r.out = out_w;
  r.db = out_b;
  r.nsplit = nsplit;
  r.M = M;
  r.N = N;
  wp.reds.push_back(r);
}

// ------------------------------------------------------------ HybridFusion
struct HySaved {
  RngSnap* rng;
  float* P[MMF_MAX_MODALITIES];
  float *Q[MMF_MAX_PAIRS], *K[MMF_MAX_PAIRS], *V[MMF_MAX_PAIRS], *O[MMF_MAX_PAIRS];
  float *lse[MMF_MAX_PAIRS], *A[MMF_MAX_PAIRS];
  float *pooled, *scores, *weights, *fused, *h1;
};

inline int Lm(const mmf_hybrid_desc* d, int m) { return d->seq_len[m] > 0 ? d->seq_len[m] : 1; }

void layout_saved(const mmf_hybrid_desc* d, Bump& bp, HySaved& s) {
  const size_t B = d->batch, H = d->hidden, M = d->num_modalities;
  s.rng = bp.take<RngSnap>(1);
  for (int m = 0; m < d->num_modalities; ++m) s.P[m] = bp.take<float>(B * Lm(d, m) * H);
  for (int g = 0; g < d->num_pairs; ++g) {
    const size_t lq = Lm(d, d->pair_q[g]), lk = Lm(d, d->pair_k[g]);
    s.Q[g] = bp.take<float>(B * lq * H);
    s.K[g] = bp.take<float>(B * lk * H);
    s.V[g] = bp.take<float>(B * lk * H);
    s.O[g] = bp.take<float>(B * lq * H);
    s.lse[g] = bp.take<float>(B * d->num_heads * lq);
    s.A[g] = bp.take<float>(B * lq * H);
  }
  s.pooled = bp.take<float>(B * M * H);
  s.scores = bp.take<float>(B * M);
  s.weights = bp.take<float>(B * M);
  s.fused = bp.take<float>(B * H);
  s.h1 = bp.take<float>(B * H);
}

struct HyWs {
  float *dz1, *dfused, *cvec, *dscore;
  float *dO[MMF_MAX_PAIRS], *dsum[MMF_MAX_PAIRS], *dQ[MMF_MAX_PAIRS], *dK[MMF_MAX_PAIRS],
      *dV[MMF_MAX_PAIRS];
  float* dZ[MMF_MAX_MODALITIES];
};

void layout_ws(const mmf_hybrid_desc* d, Bump& bp, HyWs& w) {
  const size_t B = d->batch, H = d->hidden, M = d->num_modalities;
  w.dz1 = bp.take<float>(B * H);
  w.dfused = bp.take<float>(B * H);
  w.cvec = bp.take<float>(B * M * H);
  w.dscore = bp.take<float>(B * M);
  for (int g = 0; g < d->num_pairs; ++g) {
    const size_t lq = Lm(d, d->pair_q[g]), lk = Lm(d, d->pair_k[g]);
    w.dO[g] = bp.take<float>(B * lq * H);
    w.dsum[g] = bp.take<float>(B * d->num_heads * lq);
    w.dQ[g] = bp.take<float>(B * lq * H);
    w.dK[g] = bp.take<float>(B * lk * H);
    w.dV[g] = bp.take<float>(B * lk * H);
  }
  for (int m = 0; m < d->num_modalities; ++m) w.dZ[m] = bp.take<float>(B * Lm(d, m) * H);
}

int check_hybrid(const mmf_hybrid_desc* d) {
  if (!d) return fail(MMF_EINVAL, "null descriptor");
  if (d->batch < 1) return fail(MMF_EINVAL, "batch must be >= 1 (got %d)", d->batch);
  if (d->num_modalities < 1 || d->num_modalities > MMF_MAX_MODALITIES)
    return fail(MMF_ELIMIT, "num_modalities must be in [1, %d] (got %d)", MMF_MAX_MODALITIES,
                d->num_modalities);
  if (d->num_heads < 1 || d->hidden % d->num_heads != 0)
    return fail(MMF_EINVAL, "hidden_dim (%d) must be divisible by num_heads (%d)", d->hidden,
                d->num_heads);
  if (d->hidden / d->num_heads > MMF_MAX_HEAD_DIM)
    return fail(MMF_ELIMIT, "head_dim %d > %d is not supported by the HIP kernels",
                d->hidden / d->num_heads, MMF_MAX_HEAD_DIM);
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
  return MMF_OK;
}

size_t hybrid_partials_bytes(const mmf_hybrid_desc* d) {
  // Mirror of plan_wgrad's slab sizes for every weight-gradient job.
  auto slab = [](int M, int N, int rows, bool) { return slab_bytes(M, N, rows); };
  const int B = d->batch, H = d->hidden, C = d->num_classes;
  size_t total = slab(C, H, B, true) + slab(H, H, B, true);
  for (int g = 0; g < d->num_pairs; ++g) {
    const int lq = Lm(d, d->pair_q[g]), lk = Lm(d, d->pair_k[g]);
    total += slab(H, H, B * lq, true) * 2 + slab(H, H, B * lk, true) * 2;
  }
  for (int m = 0; m < d->num_modalities; ++m) total += slab(H, d->in_dim[m], B * Lm(d, m), true);
  for (int m = 0; m < d->num_modalities; ++m) total += slab(1, H, B, true);   // gating layers
  return total;
}

}  // namespace

extern "C" {

const char* mmf_last_error(void) { return g_err.c_str(); }

void mmf_profile_begin(void) {
  g_prof.on = true;
  g_prof.recs.clear();
  g_prof.next = 0;
}

// Ends profiling: waits for the recorded events and writes "name ms\n" lines
// (one per launch group, in launch order) into out.  Returns the bytes needed.
size_t mmf_profile_end(char* out, size_t cap) {
  std::string s;
  for (const ProfRec& r : g_prof.recs) {
    float ms = 0.f;
    if (hipEventSynchronize(r.b) == hipSuccess) (void)hipEventElapsedTime(&ms, r.a, r.b);
    char line[160];
    snprintf(line, sizeof(line), "%s %.6f\n", r.name, (double)ms);
    s += line;
  }
  g_prof.on = false;
  g_prof.recs.clear();
  g_prof.next = 0;
  if (out && cap) {
    const size_t n = s.size() < cap - 1 ? s.size() : cap - 1;
    memcpy(out, s.data(), n);
    out[n] = 0;
  }
  return s.size() + 1;
}
const char* mmf_version(void) { return "mmfusion 0.1 (gfx950, fp32 MFMA)"; }

size_t mmf_hybrid_saved_bytes(const mmf_hybrid_desc* d) {
  if (check_hybrid(d) != MMF_OK) return 0;
  Bump bp(nullptr);
  HySaved s;
  layout_saved(d, bp, s);
  return bp.off + 256;
}

size_t mmf_hybrid_workspace_bytes(const mmf_hybrid_desc* d) {
  if (check_hybrid(d) != MMF_OK) return 0;
  Bump bp(nullptr);
  HyWs w;
  layout_ws(d, bp, w);
  return bp.off + 256 + hybrid_partials_bytes(d);
}

int mmf_hybrid_forward(const mmf_hybrid_desc* d, const mmf_hybrid_params* W, const float* const* x,
                       const float* mask, const uint64_t* rng_state, void* saved, float* logits,
                       float* fusion_weights, float* const* attn_maps, void* stream) {
  int rc = check_hybrid(d);
  if (rc) return rc;
  if (!W || !x || !mask || !saved || !logits) return fail(MMF_EINVAL, "null argument");
  hipStream_t st = (hipStream_t)stream;
  const int B = d->batch, M = d->num_modalities, H = d->hidden, C = d->num_classes;
  const int hd = H / d->num_heads;
  const bool drop = d->training && d->dropout > 0.f;
  const float p = drop ? d->dropout : 0.f;
  if (drop && !rng_state) return fail(MMF_EINVAL, "training with dropout needs rng_state");

  Bump bp(saved);
  HySaved s;
  layout_saved(d, bp, s);
  if (rng_state) STAGE_TRY("fwd.rng", launch_rng_snapshot(rng_state, s.rng, st));
  const RngSnap* rng = rng_state ? s.rng : nullptr;

  // (1) per-modality projection: P_m = Drop(ReLU((Drop(X_m*mask)) W_m^T + b_m))
  {
    std::vector<GemmJob> jobs;
    for (int m = 0; m < M; ++m) {
      const int L = Lm(d, m), D = d->in_dim[m];
      GemmJob j = make_job(B * L, H, s.P[m], H, EPI_BIAS | EPI_RELU | (drop ? EPI_DROP : 0));
      j.g.bias = W->proj[m].b;
      j.g.drop_site = SITE_PROJ + m;
      add_src(j, opnd(x[m], D), opnd(W->proj[m].w, D), D);
      j.has_xf_a[0] = 1;
      Xform& xf = j.xf_a[0];
      xf.rowscale = mask;
      xf.rs_div = L;
      xf.rs_stride = M;
      xf.rs_off = m;
      xf.drop_site = drop ? SITE_IN + m : 0;
      xf.ncols = D;
      jobs.push_back(j);
    }
    STAGE_TRY("fwd.proj_gemm", launch_gemm(jobs.data(), (int)jobs.size(), MODE_RK, MODE_RK, p, rng, st));
  }
  // (2) Q/K/V projections of every present pair (src/attention.py:104-106)
  {
    std::vector<GemmJob> jobs;
    for (int g = 0; g < d->num_pairs; ++g) {
      const int q = d->pair_q[g], k = d->pair_k[g];
      const int lq = Lm(d, q), lk = Lm(d, k);
      GemmJob jq = make_job(B * lq, H, s.Q[g], H, EPI_BIAS);
      jq.g.bias = W->q[g].b;
      add_src(jq, opnd(s.P[q], H), opnd(W->q[g].w, H), H);
      GemmJob jk = make_job(B * lk, H, s.K[g], H, EPI_BIAS);
      jk.g.bias = W->k[g].b;
      add_src(jk, opnd(s.P[k], H), opnd(W->k[g].w, H), H);
      GemmJob jv = make_job(B * lk, H, s.V[g], H, EPI_BIAS);
      jv.g.bias = W->v[g].b;
      add_src(jv, opnd(s.P[k], H), opnd(W->v[g].w, H), H);
      jobs.push_back(jq);
      jobs.push_back(jk);
      jobs.push_back(jv);
    }
    if (!jobs.empty()) STAGE_TRY("fwd.qkv_gemm", launch_gemm(jobs.data(), (int)jobs.size(), MODE_RK, MODE_RK, 0.f, rng, st));
  }
  // (3) attention per pair (key mask = modality mask column k, src/fusion.py:391-401)
  std::vector<AttnPair> pairs(d->num_pairs);
  for (int g = 0; g < d->num_pairs; ++g) {
    AttnPair& a = pairs[g];
    memset(&a, 0, sizeof(a));
    const int q = d->pair_q[g], k = d->pair_k[g];
    a.q = s.Q[g]; a.k = s.K[g]; a.v = s.V[g]; a.o = s.O[g]; a.lse = s.lse[g];
    a.kmask = mask + k; a.kmask_mode = 1; a.kmask_ld = M;
    a.Lq = Lm(d, q); a.Lk = Lm(d, k);
    a.ldq = a.ldk = a.ldv = a.ldo = H;
    a.drop_site = SITE_ATTN + g;
    if (attn_maps && d->return_attention) a.probs = attn_maps[g];
  }
  const float scale = 1.0f / std::sqrt((float)hd);
  if (d->num_pairs) {
    STAGE_TRY("fwd.attn", launch_attn_fwd(pairs.data(), d->num_pairs, B, d->num_heads, hd, scale, p, rng, st));
    // (4) out_proj
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
  // (5) aggregation + pooling + gating + adaptive weights + weighted sum
  HeadArgs ha;
  memset(&ha, 0, sizeof(ha));
  ha.B = B; ha.M = M; ha.H = H; ha.mask = mask;
  ha.scale_by_mask = 1;
  int cnt[MMF_MAX_MODALITIES];
  for (int m = 0; m < M; ++m) {
    ha.src[ha.nsrc] = s.P[m];
    ha.src_mod[ha.nsrc++] = m;
    cnt[m] = 1;
    ha.L[m] = Lm(d, m);
    ha.gate_w[m] = W->gate[m].w;
    ha.gate_b[m] = W->gate[m].b;
  }
  for (int g = 0; g < d->num_pairs; ++g) {
    ha.src[ha.nsrc] = s.A[g];
    ha.src_mod[ha.nsrc++] = d->pair_q[g];
    cnt[d->pair_q[g]]++;
  }
  for (int m = 0; m < M; ++m) ha.inv_cnt[m] = 1.0f / ((float)cnt[m] * (float)Lm(d, m));
  ha.pooled = s.pooled; ha.scores = s.scores; ha.weights = s.weights; ha.fused = s.fused;
  ha.weights_out = fusion_weights;
  STAGE_TRY("fwd.head", launch_head_fwd(ha, st));
  // (6) classifier: Linear -> ReLU -> Dropout -> Linear
  {
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
  // (7) optional attention maps (post-dropout, src/attention.py:130,144-146)
  if (d->return_attention && attn_maps && d->num_pairs) {
    std::vector<AttnPair> pp;
    for (int g = 0; g < d->num_pairs; ++g)
      if (pairs[g].probs) pp.push_back(pairs[g]);
    if (!pp.empty())
      STAGE_TRY("fwd.attn_probs", launch_attn_probs(pp.data(), (int)pp.size(), B, d->num_heads, hd, scale, p, rng, st));
  }
  return MMF_OK;
}

int mmf_hybrid_backward(const mmf_hybrid_desc* d, const mmf_hybrid_params* W, const float* const* x,
                        const float* mask, const void* saved, const float* dlogits, void* workspace,
                        const mmf_hybrid_grads* G, float* const* dx, void* stream) {
  int rc = check_hybrid(d);
  if (rc) return rc;
  if (!W || !x || !mask || !saved || !dlogits || !workspace || !G)
    return fail(MMF_EINVAL, "null argument");
  hipStream_t st = (hipStream_t)stream;
  const int B = d->batch, M = d->num_modalities, H = d->hidden, C = d->num_classes;
  const int hd = H / d->num_heads;
  const bool drop = d->training && d->dropout > 0.f;
  const float p = drop ? d->dropout : 0.f;
  const float gscale = drop ? 1.f / (1.f - p) : 1.f;

  Bump bs(const_cast<void*>(saved));
  HySaved s;
  layout_saved(d, bs, s);
  const RngSnap* rng = s.rng;
  Bump bw(workspace);
  HyWs w;
  layout_ws(d, bw, w);
  WgradPlan wp;

  // (1) classifier backward
  {
    GemmJob j = make_job(B, H, w.dz1, H, EPI_GATE);
    j.g.gate = s.h1; j.g.ld_gate = H; j.g.gate_scale = gscale;
    add_src(j, opnd(dlogits, C), opnd(W->cls2.w, H), C);
    STAGE_TRY("bwd.cls_dz1_gemm", launch_gemm(&j, 1, MODE_RK, MODE_KR, 0.f, rng, st));
    GemmJob j2 = make_job(B, H, w.dfused, H, 0);
    add_src(j2, opnd(w.dz1, H), opnd(W->cls1.w, H), H);
    STAGE_TRY("bwd.cls_dfused_gemm", launch_gemm(&j2, 1, MODE_RK, MODE_KR, 0.f, rng, st));
    plan_wgrad(wp, bw, C, H, B, opnd(dlogits, C), opnd(s.h1, H), G->cls2.w, G->cls2.b);
    plan_wgrad(wp, bw, H, H, B, opnd(w.dz1, H), opnd(s.fused, H), G->cls1.w, G->cls1.b);
  }
  // (2) head backward: dscore, per-row grads c_m of every aggregated list entry
  HeadArgs ha;
  memset(&ha, 0, sizeof(ha));
  ha.B = B; ha.M = M; ha.H = H; ha.mask = mask;
  int cnt[MMF_MAX_MODALITIES];
  for (int m = 0; m < M; ++m) {
    cnt[m] = 1;
    ha.L[m] = Lm(d, m);
    ha.gate_w[m] = W->gate[m].w;
    ha.gate_b[m] = W->gate[m].b;
  }
  for (int g = 0; g < d->num_pairs; ++g) cnt[d->pair_q[g]]++;
  for (int m = 0; m < M; ++m) ha.inv_cnt[m] = 1.0f / ((float)cnt[m] * (float)Lm(d, m));
  ha.pooled = s.pooled; ha.scores = s.scores; ha.weights = s.weights;
  ha.dfused = w.dfused; ha.cvec = w.cvec; ha.dscore = w.dscore;
  STAGE_TRY("bwd.head", launch_head_bwd(ha, st));
  // gating_layers[m] grads = dscore[:, m]^T pooled[:, m, :] (+ row sums for the bias):
  // a 1 x H weight-gradient GEMM riding in the split-K batch below.
  for (int m = 0; m < M; ++m)
    plan_wgrad(wp, bw, 1, H, B, opnd(w.dscore + m, M), opnd(s.pooled + (size_t)m * H, M * H),
               G->gate[m].w, G->gate[m].b);
  const float scale = 1.0f / std::sqrt((float)hd);
  if (d->num_pairs) {
    // (3) out_proj backward: dA_g rows are c_{q(g)} broadcast over L_q
    std::vector<GemmJob> jobs;
    for (int g = 0; g < d->num_pairs; ++g) {
      const int q = d->pair_q[g], lq = Lm(d, q);
      GemmJob j = make_job(B * lq, H, w.dO[g], H, 0);
      add_src(j, opnd(w.cvec + (size_t)q * H, M * H, lq), opnd(W->o[g].w, H), H);
      jobs.push_back(j);
      plan_wgrad(wp, bw, H, H, B * lq, opnd(w.cvec + (size_t)q * H, M * H, lq), opnd(s.O[g], H),
                 G->o[g].w, G->o[g].b);
    }
    STAGE_TRY("bwd.out_dO_gemm", launch_gemm(jobs.data(), (int)jobs.size(), MODE_RK, MODE_KR, 0.f, rng, st));
    // (4) attention backward
    std::vector<AttnPair> pairs(d->num_pairs);
    for (int g = 0; g < d->num_pairs; ++g) {
      AttnPair& a = pairs[g];
      memset(&a, 0, sizeof(a));
      const int q = d->pair_q[g], k = d->pair_k[g];
      a.q = s.Q[g]; a.k = s.K[g]; a.v = s.V[g]; a.o = s.O[g]; a.lse = s.lse[g];
      a.kmask = mask + k; a.kmask_mode = 1; a.kmask_ld = M;
      a.Lq = Lm(d, q); a.Lk = Lm(d, k);
      a.ldq = a.ldk = a.ldv = a.ldo = H;
      a.drop_site = SITE_ATTN + g;
      a.dout = w.dO[g]; a.dsum = w.dsum[g]; a.dq = w.dQ[g]; a.dk = w.dK[g]; a.dv = w.dV[g];
    }
    STAGE_TRY("bwd.attn_prep", launch_attn_bwd_stage(0, pairs.data(), d->num_pairs, B, d->num_heads, hd, scale, p, rng, st));
    STAGE_TRY("bwd.attn_dkv", launch_attn_bwd_stage(1, pairs.data(), d->num_pairs, B, d->num_heads, hd, scale, p, rng, st));
    STAGE_TRY("bwd.attn_dq", launch_attn_bwd_stage(2, pairs.data(), d->num_pairs, B, d->num_heads, hd, scale, p, rng, st));
    // (5) Q/K/V weight grads
    for (int g = 0; g < d->num_pairs; ++g) {
      const int q = d->pair_q[g], k = d->pair_k[g];
      const int lq = Lm(d, q), lk = Lm(d, k);
      plan_wgrad(wp, bw, H, H, B * lq, opnd(w.dQ[g], H), opnd(s.P[q], H), G->q[g].w, G->q[g].b);
      plan_wgrad(wp, bw, H, H, B * lk, opnd(w.dK[g], H), opnd(s.P[k], H), G->k[g].w, G->k[g].b);
      plan_wgrad(wp, bw, H, H, B * lk, opnd(w.dV[g], H), opnd(s.P[k], H), G->v[g].w, G->v[g].b);
    }
  }
  // (6) dZ_m = gate(P_m) * [c_m + sum dQ W_q + sum (dK W_k + dV W_v)]
  {
    std::vector<GemmJob> jobs;
    for (int m = 0; m < M; ++m) {
      const int L = Lm(d, m);
      GemmJob j = make_job(B * L, H, w.dZ[m], H, EPI_ROWADD | EPI_GATE);
      j.g.rowadd = w.cvec + (size_t)m * H;
      j.g.ld_rowadd = M * H;
      j.g.rowadd_div = L;
      j.g.gate = s.P[m];
      j.g.ld_gate = H;
      j.g.gate_scale = gscale;
      for (int g = 0; g < d->num_pairs; ++g) {
        if (d->pair_q[g] == m) add_src(j, opnd(w.dQ[g], H), opnd(W->q[g].w, H), H);
        if (d->pair_k[g] == m) {
          add_src(j, opnd(w.dK[g], H), opnd(W->k[g].w, H), H);
          add_src(j, opnd(w.dV[g], H), opnd(W->v[g].w, H), H);
        }
      }
      if (j.nsrc > GEMM_MAX_SRCS) return fail(MMF_ELIMIT, "too many gradient sources");
      jobs.push_back(j);
    }
    STAGE_TRY("bwd.dZ_gemm", launch_gemm(jobs.data(), (int)jobs.size(), MODE_RK, MODE_KR, 0.f, rng, st));
  }
  // (7) projection weight grads (X~ recomputed: mask * input dropout) and dX
  {
    std::vector<GemmJob> jobs;
    for (int m = 0; m < M; ++m) {
      const int L = Lm(d, m), D = d->in_dim[m];
      Xform xf;
      memset(&xf, 0, sizeof(xf));
      xf.rowscale = mask; xf.rs_div = L; xf.rs_stride = M; xf.rs_off = m;
      xf.drop_site = drop ? SITE_IN + m : 0;
      xf.ncols = D;
      plan_wgrad(wp, bw, H, D, B * L, opnd(w.dZ[m], H), opnd(x[m], D), G->proj[m].w, G->proj[m].b,
                 true, &xf);
      if (dx && dx[m]) {
        GemmJob j = make_job(B * L, D, dx[m], D, EPI_ROWSCALE | (drop ? EPI_DROP : 0));
        j.g.rowscale = mask; j.g.rs_div = L; j.g.rs_stride = M; j.g.rs_off = m;
        j.g.drop_site = SITE_IN + m;
        add_src(j, opnd(w.dZ[m], H), opnd(W->proj[m].w, D), H);
        jobs.push_back(j);
      }
    }
    if (!jobs.empty()) STAGE_TRY("bwd.dx_gemm", launch_gemm(jobs.data(), (int)jobs.size(), MODE_RK, MODE_KR, p, rng, st));
  }
  // (8) all weight gradients: split-K slabs (only written here), then one
  // deterministic reduce.
  if (bw.off > mmf_hybrid_workspace_bytes(d))
    return fail(MMF_EINVAL, "internal: workspace overflow");
  STAGE_TRY("bwd.wgrad_gemm", launch_gemm(wp.jobs.data(), (int)wp.jobs.size(), MODE_KR, MODE_KR, p, rng, st));
  STAGE_TRY("bwd.wgrad_reduce", launch_reduce(wp.reds.data(), (int)wp.reds.size(), st));
  return MMF_OK;
}

size_t mmf_adaptive_weights_workspace_bytes(int32_t batch, int32_t M, int32_t H) {
  Bump bp(nullptr);
  bp.take<float>((size_t)batch * M * H);
  bp.take<float>((size_t)batch * M);
  bp.take<float>((size_t)batch * M);
  bp.take<float>((size_t)batch * H);
  return bp.off + 256;
}

int mmf_adaptive_weights(int32_t batch, int32_t M, int32_t H, const float* const* feats,
                         const float* mask, const mmf_linear* gate, float* weights, void* workspace,
                         void* stream) {
  if (batch < 1 || M < 1 || M > MMF_MAX_MODALITIES || H < 4 || H % 4 != 0 || H > 1024)
    return fail(MMF_ELIMIT, "adaptive weights: unsupported shape B=%d M=%d H=%d", batch, M, H);
  if (!feats || !mask || !gate || !weights || !workspace) return fail(MMF_EINVAL, "null argument");
  Bump bp(workspace);
  HeadArgs ha;
  memset(&ha, 0, sizeof(ha));
  ha.B = batch; ha.M = M; ha.H = H; ha.mask = mask;
  ha.scale_by_mask = 0;
  for (int m = 0; m < M; ++m) {
    ha.src[ha.nsrc] = feats[m];
    ha.src_mod[ha.nsrc++] = m;
    ha.L[m] = 1;
    ha.inv_cnt[m] = 1.f;
    ha.gate_w[m] = gate[m].w;
    ha.gate_b[m] = gate[m].b;
  }
  ha.pooled = bp.take<float>((size_t)batch * M * H);
  ha.scores = bp.take<float>((size_t)batch * M);
  ha.weights = bp.take<float>((size_t)batch * M);
  ha.fused = bp.take<float>((size_t)batch * H);
  ha.weights_out = weights;
  HIP_TRY(launch_head_fwd(ha, (hipStream_t)stream));
  return MMF_OK;
}

// ------------------------------------------------------------ CrossModalAttention
}  // extern "C"

namespace {
struct CmaSaved { RngSnap* rng; float *Q, *K, *V, *O, *lse; };
void layout_cma(const mmf_cma_desc* d, Bump& bp, CmaSaved& s) {
  const size_t B = d->batch, H = d->hidden;
  s.rng = bp.take<RngSnap>(1);
  s.Q = bp.take<float>(B * d->lq * H);
  s.K = bp.take<float>(B * d->lk * H);
  s.V = bp.take<float>(B * d->lk * H);
  s.O = bp.take<float>(B * d->lq * H);
  s.lse = bp.take<float>(B * d->num_heads * d->lq);
}
struct CmaWs { float *dO, *dsum, *dQ, *dK, *dV; };
void layout_cma_ws(const mmf_cma_desc* d, Bump& bp, CmaWs& w) {
  const size_t B = d->batch, H = d->hidden;
  w.dO = bp.take<float>(B * d->lq * H);
  w.dsum = bp.take<float>(B * d->num_heads * d->lq);
  w.dQ = bp.take<float>(B * d->lq * H);
  w.dK = bp.take<float>(B * d->lk * H);
  w.dV = bp.take<float>(B * d->lk * H);
}
int check_cma(const mmf_cma_desc* d) {
  if (!d) return fail(MMF_EINVAL, "null descriptor");
  if (d->batch < 1 || d->lq < 1 || d->lk < 1 || d->query_dim < 1 || d->key_dim < 1)
    return fail(MMF_EINVAL, "bad CrossModalAttention shape");
  if (d->num_heads < 1 || d->hidden % d->num_heads != 0)
    return fail(MMF_EINVAL, "hidden_dim (%d) must be divisible by num_heads (%d)", d->hidden,
                d->num_heads);
  if (d->hidden / d->num_heads > MMF_MAX_HEAD_DIM)
    return fail(MMF_ELIMIT, "head_dim %d > %d is not supported by the HIP kernels",
                d->hidden / d->num_heads, MMF_MAX_HEAD_DIM);
  if (d->mask_mode < 0 || d->mask_mode > 2) return fail(MMF_EINVAL, "bad mask_mode");
  if (!(d->dropout >= 0.f && d->dropout < 1.f)) return fail(MMF_EINVAL, "dropout must be in [0, 1)");
  return MMF_OK;
}
size_t cma_partials_bytes(const mmf_cma_desc* d) {
  auto slab = [](int M, int N, int rows) { return slab_bytes(M, N, rows); };
  const int B = d->batch, H = d->hidden;
  return slab(H, H, B * d->lq) + slab(H, d->query_dim, B * d->lq) + slab(H, d->key_dim, B * d->lk) * 2;
}
}  // namespace

extern "C" {

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
  GemmJob jobs[3];
  jobs[0] = make_job(B * d->lq, H, s.Q, H, EPI_BIAS);
  jobs[0].g.bias = W->q.b;
  add_src(jobs[0], opnd(query, d->query_dim), opnd(W->q.w, d->query_dim), d->query_dim);
  jobs[1] = make_job(B * d->lk, H, s.K, H, EPI_BIAS);
  jobs[1].g.bias = W->k.b;
  add_src(jobs[1], opnd(key, d->key_dim), opnd(W->k.w, d->key_dim), d->key_dim);
  jobs[2] = make_job(B * d->lk, H, s.V, H, EPI_BIAS);
  jobs[2].g.bias = W->v.b;
  add_src(jobs[2], opnd(value, d->key_dim), opnd(W->v.w, d->key_dim), d->key_dim);
  STAGE_TRY("cma.fwd.qkv_gemm", launch_gemm(jobs, 3, MODE_RK, MODE_RK, 0.f, rng, st));
  AttnPair a;
  memset(&a, 0, sizeof(a));
  a.q = s.Q; a.k = s.K; a.v = s.V; a.o = s.O; a.lse = s.lse;
  a.kmask = mask; a.kmask_mode = d->mask_mode; a.kmask_ld = d->mask_mode == 2 ? d->lk : 1;
  a.Lq = d->lq; a.Lk = d->lk;
  a.ldq = a.ldk = a.ldv = a.ldo = H;
  a.drop_site = SITE_ATTN;
  a.probs = attn_weights;
  const float scale = 1.0f / std::sqrt((float)hd);
  STAGE_TRY("cma.fwd.attn", launch_attn_fwd(&a, 1, B, d->num_heads, hd, scale, p, rng, st));
  if (attn_weights) STAGE_TRY("cma.fwd.attn_probs", launch_attn_probs(&a, 1, B, d->num_heads, hd, scale, p, rng, st));
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
  WgradPlan wp;
  {
    GemmJob j = make_job(B * d->lq, H, w.dO, H, 0);
    add_src(j, opnd(dA, H), opnd(W->o.w, H), H);
    STAGE_TRY("cma.bwd.dO_gemm", launch_gemm(&j, 1, MODE_RK, MODE_KR, 0.f, rng, st));
    plan_wgrad(wp, bw, H, H, B * d->lq, opnd(dA, H), opnd(s.O, H), G->o.w, G->o.b);
  }
  AttnPair a;
  memset(&a, 0, sizeof(a));
  a.q = s.Q; a.k = s.K; a.v = s.V; a.o = s.O; a.lse = s.lse;
  a.kmask = mask; a.kmask_mode = d->mask_mode; a.kmask_ld = d->mask_mode == 2 ? d->lk : 1;
  a.Lq = d->lq; a.Lk = d->lk;
  a.ldq = a.ldk = a.ldv = a.ldo = H;
  a.drop_site = SITE_ATTN;
  a.dout = w.dO; a.dsum = w.dsum; a.dq = w.dQ; a.dk = w.dK; a.dv = w.dV;
  const float scale = 1.0f / std::sqrt((float)hd);
  STAGE_TRY("cma.bwd.attn", launch_attn_bwd(&a, 1, B, d->num_heads, hd, scale, p, rng, st));
  plan_wgrad(wp, bw, H, d->query_dim, B * d->lq, opnd(w.dQ, H), opnd(query, d->query_dim), G->q.w, G->q.b);
  plan_wgrad(wp, bw, H, d->key_dim, B * d->lk, opnd(w.dK, H), opnd(key, d->key_dim), G->k.w, G->k.b);
  plan_wgrad(wp, bw, H, d->key_dim, B * d->lk, opnd(w.dV, H), opnd(value, d->key_dim), G->v.w, G->v.b);
  std::vector<GemmJob> jobs;
  if (dquery) {
    GemmJob j = make_job(B * d->lq, d->query_dim, dquery, d->query_dim, 0);
    add_src(j, opnd(w.dQ, H), opnd(W->q.w, d->query_dim), H);
    jobs.push_back(j);
  }
  if (dkey) {
    GemmJob j = make_job(B * d->lk, d->key_dim, dkey, d->key_dim, 0);
    add_src(j, opnd(w.dK, H), opnd(W->k.w, d->key_dim), H);
    jobs.push_back(j);
  }
  if (dvalue) {
    GemmJob j = make_job(B * d->lk, d->key_dim, dvalue, d->key_dim, 0);
    add_src(j, opnd(w.dV, H), opnd(W->v.w, d->key_dim), H);
    jobs.push_back(j);
  }
  if (!jobs.empty()) STAGE_TRY("cma.bwd.dx_gemm", launch_gemm(jobs.data(), (int)jobs.size(), MODE_RK, MODE_KR, 0.f, rng, st));
  if (bw.off > mmf_cma_workspace_bytes(d)) return fail(MMF_EINVAL, "internal: workspace overflow");
  STAGE_TRY("cma.bwd.wgrad_gemm", launch_gemm(wp.jobs.data(), (int)wp.jobs.size(), MODE_KR, MODE_KR, 0.f, rng, st));
  STAGE_TRY("cma.bwd.wgrad_reduce", launch_reduce(wp.reds.data(), (int)wp.reds.size(), st));
  return MMF_OK;
}

int mmf_cross_entropy_ls(int32_t batch, int32_t classes, const float* logits, const int64_t* labels,
                         float smoothing, float grad_scale, float* loss_out, float* dlogits,
                         void* stream) {
  if (batch < 1 || classes < 1 || !logits || !labels || !loss_out || !dlogits)
    return fail(MMF_EINVAL, "bad cross-entropy arguments");
  HIP_TRY(launch_cross_entropy(batch, classes, logits, labels, smoothing, grad_scale, loss_out, dlogits,
                               (hipStream_t)stream));
  return MMF_OK;
}

int mmf_adamw_step(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                   int64_t* step_dev, float lr, float beta1, float beta2, float eps,
                   float weight_decay, float grad_scale, void* stream) {
  if (n < 0 || !param || !grad || !exp_avg || !exp_avg_sq || !step_dev)
    return fail(MMF_EINVAL, "bad AdamW arguments");
  HIP_TRY(launch_adamw(n, param, grad, exp_avg, exp_avg_sq, step_dev, lr, beta1, beta2, eps,
                       weight_decay, grad_scale, (hipStream_t)stream));
  return MMF_OK;
}

}  // extern "C"
