// Internal kernel interfaces for libmmfusion (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stddef.h>

namespace mmf {

// ---------------------------------------------------------------------------
// Dropout RNG: Philox4x32-10 keyed by the per-call snapshot {seed, offset};
// counter = (idx>>3 lo, idx>>3 hi, site, offset).  One call yields the keep
// decisions of 8 consecutive elements of one tensor ("site"), 16 bits each.
// ---------------------------------------------------------------------------
struct RngSnap { uint64_t seed; uint64_t offset; };

// ---------------------------------------------------------------------------
// Per-launch profiling (capi.hip).  While mmf_profile_begin() is active, every
// kernel launch of the library is timed by two hipEvents and tagged with the
// kernel's name (as rocprofv3 prints it, minus the namespace) and its
// ALGORITHMIC work: FLOPs of the math it implements (no recompute) and the bytes
// a perfect-reuse kernel would move to/from HBM.  The events ride in the first
// launch's own dispatch packet (hipExtLaunchKernel start / stop events: the
// kernel's start and end, as rocprofv3 sees them); a scope with several launches
// ends at an event recorded after the last.  Inactive, a launch pays one branch.
// `kernel` must point to static storage.
// ---------------------------------------------------------------------------
struct ProfArm {
  hipEvent_t a = nullptr, b = nullptr;
  int launches = 0;
};
extern thread_local ProfArm* g_prof_arm;
// false when profiling is off or `st` is being captured into a graph (events recorded
// inside a capture cannot be timed afterwards: the captured launches run untimed)
bool prof_arm_begin(ProfArm& arm, hipStream_t st);
bool prof_capturing(hipStream_t st);

// A side stream of the calling thread on the current device with two (untimed) events:
// record `fork_ev` on st and make `s` wait on it, enqueue on `s`, record `join_ev` on `s`
// and make st wait on it -- inside a graph capture on st the side work becomes a parallel
// branch of the graph.  create = false: only an existing one (no stream / event creation
// while st is being captured); nullptr when there is none or it cannot be created.
struct SideStream { hipStream_t s; hipEvent_t fork_ev, join_ev; };
SideStream* side_stream(bool create);
void prof_arm_end(ProfArm& arm, hipStream_t st, const char* kernel, double flops, double bytes);
struct ProfLaunch {
  hipStream_t st;
  const char* kernel;
  double flops, bytes;
  ProfArm arm;
  bool armed;
  ProfLaunch(hipStream_t s, const char* k, double f, double b) : st(s), kernel(k), flops(f), bytes(b) {
    armed = prof_arm_begin(arm, st);
  }
  ~ProfLaunch() {
    if (armed) prof_arm_end(arm, st, kernel, flops, bytes);
  }
  ProfLaunch(const ProfLaunch&) = delete;
  ProfLaunch& operator=(const ProfLaunch&) = delete;
};

// Every kernel launch of the library: hipLaunchKernelGGL, or while a ProfLaunch
// scope is armed, its first launch carries the scope's start / stop events.
template <typename F, typename... Args>
inline void mmf_launch(F kernel, const dim3& grid, const dim3& block, uint32_t shmem, hipStream_t st,
                       Args... args) {
  ProfArm* arm = g_prof_arm;
  if (arm && arm->launches++ == 0)
    hipExtLaunchKernelGGL(kernel, grid, block, shmem, st, arm->a, arm->b, 0u, args...);
  else
    hipLaunchKernelGGL(kernel, grid, block, shmem, st, args...);
}

// ---------------------------------------------------------------------------
// Matmul precision of the current C-ABI call (torch.get_float32_matmul_precision
// at the caller): 0 = "highest" (fp32 MFMA), 1 = "medium" (bf16 MFMA operands,
// fp32 accumulate), 2 = "high" (bf16x3: split bf16 operands, three MFMAs).  Set for
// the duration of one entry point by MathScope; the launchers pick the kernel
// instantiation (its int precision template argument) from it (a graph captures
// that choice).
// ---------------------------------------------------------------------------
extern thread_local int g_math_mode;
inline int math_mode() { return g_math_mode; }
struct MathScope {
  int prev;
  explicit MathScope(int mode) : prev(g_math_mode) { g_math_mode = (mode >= 0 && mode <= 2) ? mode : 0; }
  ~MathScope() { g_math_mode = prev; }
  MathScope(const MathScope&) = delete;
  MathScope& operator=(const MathScope&) = delete;
};

enum : uint32_t {
  SITE_IN = 0x100,     // + m : input dropout on X_m*mask  (src/fusion.py:373)
  SITE_PROJ = 0x200,   // + m : projections[m] Dropout     (src/fusion.py:291-298)
  SITE_ATTN = 0x300,   // + p : attention-prob Dropout     (src/attention.py:130)
  SITE_CLS = 0x400,    //       classifier Dropout          (src/fusion.py:326)
};

// ---------------------------------------------------------------------------
// Grouped fp32 GEMM on v_mfma_f32_32x32x2_f32:  C[M,N] = sum_src A_src[M,K] B_src[K,N]
// Operand storage modes (logical A[i][kk], B[kk][j]):
//   A_RK: stored [i][kk] (kk contiguous)      A_KR: stored [kk][i] (i contiguous)
//   B_NK: stored [j][kk] (kk contiguous)      B_KN: stored [kk][j] (j contiguous)
// "stored row" index is divided by row_div (row broadcast, e.g. dA = c[b]).
// ---------------------------------------------------------------------------
enum { MODE_RK = 0, MODE_KR = 1 };  // for B: RK == NK (stored [j][kk]), KR == KN

struct Operand {
  const float* ptr;
  int32_t ld;                // stored row stride (elements)
  int32_t row_div;           // >= 1
  int32_t vec;               // 1 => 16-byte aligned rows, float4 loads allowed
  int32_t seg_stride;        // != 0: + (tile's first row / group seg_rows) * seg_stride elements
                             // (a per-sample operand, e.g. dU (B, heads, H) against rows b*L + l)
};

struct GemmSrc {
  Operand a, b;
  int32_t K;                 // contraction length
  int32_t pad_;
};

enum : int32_t {
  EPI_BIAS = 1, EPI_RELU = 2, EPI_DROP = 4, EPI_ROWADD = 8, EPI_GATE = 16,
  EPI_ROWSCALE = 32, EPI_PARTIAL = 64, EPI_BIAS_RS = 128, EPI_ADDMAT = 256,
  EPI_COLSUM = 512,
  EPI_BF16 = 1024,     // store C as bf16 (round to nearest even; C holds __bf16, ldc in elements; nbatch 1)
  EPI_BF16COPY = 2048,  // also store a bf16 copy of the final C to `copy` (same ldc; nbatch 1, not with EPI_BF16)
  EPI_GATE_B16 = 4096   // with EPI_GATE: `gate` holds a __bf16 matrix (ld_gate in elements; only its sign is read)
};

// Epilogue order: v = alpha*acc; +bias[j] (x bias_rs[i*ld+off] with EPI_BIAS_RS);
// +rowadd_scale*rowadd; +addm[i][j]; relu; gate; rowscale; dropout.
struct GemmGroup {
  int32_t M, N;
  int32_t src_begin, src_count;
  float* C; int32_t ldc;
  int32_t epi;
  float alpha;                                         // scales the accumulator (and part_db)
  const float* bias;                                   // EPI_BIAS
  const float* bias_rs; int32_t bias_rs_ld, bias_rs_off;  // EPI_BIAS_RS: bias[j] * bias_rs[i*ld + off]
  const float* addm; int32_t ld_addm;                  // EPI_ADDMAT: += addm[i*ld + j]
  float rowadd_scale;
  const float* rowadd; int32_t ld_rowadd, rowadd_div;  // EPI_ROWADD: += scale*rowadd[(i/div)*ld + j]
  const float* gate; int32_t ld_gate; float gate_scale;// EPI_GATE: gate[i][j] > 0 ? v*scale : 0
  const float* rowscale; int32_t rs_div, rs_stride;    // EPI_ROWSCALE: v *= rowscale[(i/div)*stride + off]
  int32_t rs_off;
  uint32_t drop_site;                                  // EPI_DROP: idx = i*N + j
  // EPI_PARTIAL (split-K over the contraction): C := part[split][M][N] (ldc = N),
  // part_db[split][M] = row sums of A over the split (bias grad of a TN dW).
  int32_t nsplit, kchunk;
  // EPI_COLSUM (not with EPI_PARTIAL): colsum[(batch*tiles_m + i0/BM)*N + j] = sum over the
  // tile's rows of the final stored value (per-tile column sums, fixed order)
  union { float* part_db; float* colsum; };
  // strided batch: nbatch identical problems, element i offsets every source's A/B
  // by i*bs_a / i*bs_b, C by i*bs_c (partial: i*nsplit*M*N, part_db i*nsplit*M),
  // bias by i*bs_bias and bias_rs_off by i*bs_brs.
  int32_t nbatch;
  int32_t bs_a, bs_b, bs_c, bs_bias, bs_brs;
  int32_t seg_rows;        // rows per segment for operands with seg_stride (a tile never straddles two)
  void* copy;              // EPI_BF16COPY: __bf16 (M, ldc)
  // 1 + the index in GemmArgs::g of a group chained to this one (0: none): its A operand is this
  // group's output, one column tile each, the same rows; the block that finishes a tile of this
  // group runs the chained group's tile of the same rows next (gemm_lds_kernel, fp32 forms).
  // Chained groups own no blocks of the grid (tile_off = the grid size).  Set by launch_gemm.
  int32_t chain;
};

constexpr int GEMM_MAX_GROUPS = 32;   // kernel arguments ~7.8 KB (measured fine on gfx950)
constexpr int GEMM_MAX_SRCS = 32;

struct GemmArgs {
  GemmGroup g[GEMM_MAX_GROUPS];
  GemmSrc s[GEMM_MAX_SRCS];
  int32_t tile_off[GEMM_MAX_GROUPS];   // first block of each group (1-D grid over all groups' tiles)
  int32_t ngroups;
  int32_t amode, bmode;
  float drop_p;              // p of every dropout site in this launch
  const RngSnap* rng;
  uint64_t* rng_advance;     // optional: block 0 advances this live rng state's offset
  int32_t ilv;               // 1: XCD-aware group interleave (every group has tile_off[1] tiles, a multiple of 8)
};

// Host-side description of one output (group) and its sources; launch_gemm
// packs as many jobs per launch as the kernel-argument tables allow.
struct GemmJob {
  GemmGroup g;
  GemmSrc src[GEMM_MAX_SRCS];
  int nsrc;
  // optional: a job whose one source's A operand is this job's output C (ld = ldc, K = N), run by the
  // same workgroups right after this job's tiles (launch_gemm checks the shapes; a pair it cannot
  // chain runs as a launch of its own after this call's)
  const GemmJob* chain;
};

// Launches every job (grouped <= GEMM_MAX_GROUPS per launch).  A launch whose
// operands are all float4-able (16-B aligned, ld % 4 == 0, K % 4 == 0, KR
// extents % 4 == 0) runs the LDS-DMA pipelined kernel; anything else runs the
// register-staged generic kernel.
// rng_advance (optional): a live {seed, offset} rng state whose offset the call's first
// launch advances by one (the hybrid forward's snapshot is written by the input-mask
// kernel, which reads the live state from every block and so cannot advance it itself).
hipError_t launch_gemm(const GemmJob* jobs, int njobs, int amode, int bmode, float drop_p,
                       const RngSnap* rng, hipStream_t st, uint64_t* rng_advance = nullptr);
int device_cu_count();   // CUs of the current device (cached)

// X'_m[r][c] = X_m[r][c] * mask[(r / L_m) * M + m] * (keep(site_m, r*D_m + c) ? 1/(1-p) : 0)
// (the masked, input-dropped modality features of src/fusion.py:364-373,
// materialised once for the projection GEMM and its weight gradient).
// outb: X' stored as bf16 (round to nearest even; `out` holds a __bf16 address): the operand the
// bf16-operand projection GEMM and its weight gradient read (hybrid.hip proj_b16_on)
struct MaskDropJob {
  const float* x; float* out;
  int64_t rows; int32_t D, L;
  uint32_t site; int32_t vec, outb;
};
struct MaskDropArgs {
  MaskDropJob j[8];
  int32_t n, M;
  const float* mask;
  float p;
  const RngSnap* rng;
  // optional: read the draws' {seed, offset} from this live state instead of rng, and
  // write it to rng_snap (block 0) as the call's snapshot; the offset is advanced by
  // a later launch of the call (launch_gemm's rng_advance)
  const uint64_t* rng_live;
  RngSnap* rng_snap;
  // optional: the attention dropout keep words of up to 16 pairs (attn_keep_words_kernel's
  // words, same Philox stream), drawn by extra workgroups interleaved with the mask ones
  struct KeepWordJob { uint32_t* bits; uint32_t Lq, Lk, kw_ld, site; } kw[16];
  int32_t nkw, B, heads;
};
hipError_t launch_mask_dropout(MaskDropArgs a, hipStream_t st);

// Split-K partial-slab reduction: out[e] = sum_s part[s][e]; db[i] = sum_s part_db[s][i].
struct ReduceJob {
  const float* part; const float* part_db;
  float* out; float* db;
  int32_t nsplit, M, N;
  int32_t nbatch, bs_out, bs_db;   // batch i: part += i*nsplit*M*N, out += i*bs_out, db += i*bs_db
};
// "medium" GEMMs whose operands are BOTH bf16 copies in HBM (Operand.ptr holds a __bf16 address,
// ld in elements): RK x RK (Q/K projections), KR x KR (weight gradients, split-K slabs allowed, the
// bias row sums from the bf16 A) or RK x KR (dZ); 16-B aligned rows, K % 8 == 0 along RK rows,
// the output extent % 8 == 0 along KR rows; no batch / segments.  The LDS-DMA kernel's B16 forms
// (DK = 32): half the operand bytes and LDS reads, no conversion; KR tiles read through
// ds_read_b64_tr_b16.
// drop_p / rng / rng_advance: as launch_gemm (EPI_DROP epilogues, the forward's rng advance).
hipError_t launch_gemm_b16(const GemmJob* jobs, int njobs, hipStream_t st, int amode = MODE_RK, int bmode = MODE_RK,
                           float drop_p = 0.f, const RngSnap* rng = nullptr, uint64_t* rng_advance = nullptr);
constexpr int CVT_MAX = 72;
struct CvtArgs {
  // dst[i] (bf16, round to nearest even) or, where dst32[i] is set, an fp32 copy into dst32[i]
  const float* src[CVT_MAX]; __bf16* dst[CVT_MAX]; float* dst32[CVT_MAX]; int64_t n[CVT_MAX]; int32_t count;
};
hipError_t launch_cvt_bf16(const CvtArgs& a, hipStream_t st);
bool gemm_b16_ok(const GemmJob& J, int amode = MODE_RK, int bmode = MODE_RK);
hipError_t launch_reduce(const ReduceJob* jobs, int njobs, hipStream_t st);

// ---------------------------------------------------------------------------
// Attention (per pair, per sample, per head), flash-style, fp32 MFMA.
// Q (B, Lq, ld), K/V (B, Lk, ld), O (B, Lq, ld); head h uses cols [h*hd, h*hd+hd).
// ---------------------------------------------------------------------------
struct AttnPair {
  const float* q; const float* k; const float* v;
  float* o;            // fwd output
  float* lse;          // (B, heads, Lq) fwd output / bwd input
  const float* kmask; int32_t kmask_mode; int32_t kmask_ld;   // 0 none, 1 per-sample, 2 per-key
  int32_t Lq, Lk;
  int32_t ldq, ldk, ldv, ldo;
  uint32_t drop_site;
  // backward
  const float* dout;   // dO (B, Lq, ldo)
  float* dsum;         // D = rowsum(dO*O) (B, heads, Lq)
  float* dq; float* dk; float* dv;   // (B, L, ld*)
  float* probs;        // (B, heads, Lq, Lk) output of attn_probs
  // pooled-output formulation (HybridFusion): only column means of P' are needed
  float* pbar;         // (B, heads, Lk) fwd output: mean over queries of the post-dropout probs
  float* pbarT;        // optional (B, Lk, heads) copy of pbar (an RK GEMM operand for E_m)
  const float* dpbar;  // (B, heads, Lk) bwd input: d loss / d pbar
  uint32_t* keep_bits; // (B, heads, Lq, kw_ld) dropout keep mask written by the pooled forward
                       // (bit k%32 of word k/32), read by its backward
  int32_t kw_ld;       // words per query row: 4 when Lk <= 128, ceil(Lk/32) otherwise
  // optional: the pre-dropout probabilities P written by the lean pooled forward and read by
  // the fused backward instead of recomputing S = QK^T (training, keys and queries <= 128).
  // "Register order": per (sample, head), per 32-query tile qt, key tile kt and register group
  // g, 64 lanes x float4 = P of lane (query c, half h) at regs 4g..4g+3 (attn_pstore_index);
  // attn_pstore_floats(Lq) floats per (sample, head).
  float* pstore;
  // Q and K rows stored as bf16 (ldq / ldk in elements): "medium" long-key pairs on the one-pass
  // kernels (attn_long.hip), whose projections the Q/K GEMM writes in bf16 (EPI_BF16)
  int32_t qk_bf16;
  // dQ and dK written as bf16 (the fused one-pass backward; ldq / ldk in elements): "medium" with
  // every Q/K pair bf16, whose dZ and weight-gradient GEMMs then read bf16 operands (hybrid.hip
  // dqk_b16_on)
  int32_t dqk_bf16;
};

constexpr int ATTN_MAX_PAIRS = 12;
// floats of the stored probabilities per (sample, head) of a pair with Lq queries
inline int64_t attn_pstore_floats(int Lq) { return (int64_t)((Lq + 31) / 32) * 4 * 4 * 64 * 4; }
// the pooled pairs whose probabilities can be stored: the lean fused backward's conditions
// (keys a multiple of 32 and <= 128, queries <= 128, no per-key mask, head_dim <= 64, % 4)
inline bool attn_pstore_ok(int Lq, int Lk, int kmask_mode, int hd) {
  return Lk % 32 == 0 && Lk <= 128 && Lq <= 128 && kmask_mode != 2 && hd <= 64 && hd % 4 == 0;
}

struct AttnArgs {
  AttnPair p[ATTN_MAX_PAIRS];
  int32_t npairs;
  int32_t B, heads, hd;
  float scale, drop_p;
  int32_t nblk;        // blocks along the L axis (max over pairs) for this launch
  const RngSnap* rng;
};

hipError_t launch_attn_fwd(const AttnPair* pairs, int npairs, int B, int heads, int hd, float scale,
                           float drop_p, const RngSnap* rng, hipStream_t st);
hipError_t launch_attn_probs(const AttnPair* pairs, int npairs, int B, int heads, int hd,
                             float scale, float drop_p, const RngSnap* rng, hipStream_t st);
hipError_t launch_attn_bwd(const AttnPair* pairs, int npairs, int B, int heads, int hd, float scale,
                           float drop_p, const RngSnap* rng, hipStream_t st);
// stage 0: D = rowsum(dO*O); 1: dK/dV; 2: dQ
hipError_t launch_attn_bwd_stage(int stage, const AttnPair* pairs, int npairs, int B, int heads, int hd,
                                 float scale, float drop_p, const RngSnap* rng, hipStream_t st);
// Pooled formulation: forward writes LSE and pbar = mean_q P'[q, :];
// backward (stage 0: dQ and D = rowsum(P . dP); stage 1: dK) from dpbar.
// words_ready: the dropout keep words of every pair with Lk % 32 == 0 were drawn beforehand
// (launch_attn_keep_words): the lean and one-pass kernels read them instead of drawing
hipError_t launch_attn_pool_fwd(const AttnPair* pairs, int npairs, int B, int heads, int hd, float scale,
                                float drop_p, const RngSnap* rng, hipStream_t st, bool words_ready = false);
hipError_t launch_attn_pool_bwd(int stage, const AttnPair* pairs, int npairs, int B, int heads, int hd,
                                float scale, float drop_p, const RngSnap* rng, hipStream_t st);
// Long-key pooled backward in one pass (attn_long.hip, bf16 "medium" only): dQ, dK and D of
// pairs with 128 < Lk <= 512 (Lk % 32 == 0, no per-key mask, head_dim <= 64 and % 4).
bool attn_long_fused_ok(const AttnPair* pairs, int npairs, int hd, float drop_p);
// ... and its forward (LSE, keep words, pbar) in one pass
bool attn_long_fwd_ok(const AttnPair* pairs, int npairs, int hd, float drop_p, const RngSnap* rng);
hipError_t launch_attn_long_fused_fwd(const AttnPair* pairs, int npairs, int B, int heads, int hd, float scale,
                                      float drop_p, const RngSnap* rng, hipStream_t st, bool words_ready = false);
// The dropout keep words (B, heads, Lq, kw_ld) of the attention probabilities of the pairs
// with Lk % 32 == 0 and keep_bits (the others are skipped), as the attention kernels draw them
hipError_t launch_attn_keep_words(const AttnPair* pairs, int npairs, int B, int heads, float drop_p,
                                  const RngSnap* rng, hipStream_t st);
hipError_t launch_attn_long_fused_bwd(const AttnPair* pairs, int npairs, int B, int heads, int hd, float scale,
                                      float drop_p, hipStream_t st);

// ---------------------------------------------------------------------------
// Single-key attention (single_key.hip): Lk == 1, the reference's 2-D inputs.
// P'[b, h, q] = [kmask_b != 0] * keep(b, h, q) / (1 - p), independent of Q and K
// (softmax over one key), so no Q / K / QK^T work exists and their gradients are
// exactly zero.  kmask as AttnPair (mode 1 or 2 read element b * kmask_ld).
// ---------------------------------------------------------------------------
struct SkPair {
  const float* kmask; int32_t kmask_mode; int32_t kmask_ld;
  int32_t Lq;
  uint32_t drop_site;
  float* pbar;         // (B, heads) mean_q P'   (sk_fwd; may be null)
  float* pbarT;        // (B, 1, heads) copy     (sk_fwd; may be null)
  float* probs;        // (B, heads, Lq, 1)      (sk_fwd; may be null)
  const float* v; int32_t ldv;   // V (B, 1, ldv)                       (sk_out)
  float* o; int32_t ldo;         // O (B, Lq, ldo) = P' V               (sk_out)
  const float* dout;             // dO (B, Lq, ldo)                     (sk_dv)
  float* dv;                     // dV (B, 1, ldv) = sum_q P' dO        (sk_dv)
};
constexpr int SK_MAX_PAIRS = 16;
struct SkArgs {
  SkPair p[SK_MAX_PAIRS];
  int32_t npairs, B, heads, hd;
  float drop_p;
  const RngSnap* rng;
};
hipError_t launch_sk_fwd(const SkPair* pairs, int npairs, int B, int heads, int hd, float drop_p,
                         const RngSnap* rng, hipStream_t st);
hipError_t launch_sk_out(const SkPair* pairs, int npairs, int B, int heads, int hd, float drop_p,
                         const RngSnap* rng, hipStream_t st);
hipError_t launch_sk_dv(const SkPair* pairs, int npairs, int B, int heads, int hd, float drop_p,
                        const RngSnap* rng, hipStream_t st);
// zero-fills up to 16 buffers of counts[i] 4-byte words (null / empty entries skipped) in one
// kernel launch: a kernel node under stream capture (hipMemsetAsync captured into a torch.compile
// "reduce-overhead" HIP graph was observed to leave its buffer unwritten on replay)
hipError_t launch_zero_fill(float* const* ptrs, const int64_t* counts, int n, hipStream_t st);

// ---------------------------------------------------------------------------
// Attention with head_dim > 64 (wide.hip): materialised scores, grouped strided-batch
// GEMMs for QK^T / P'V / dO V^T / P'^T dO / dS K / dS^T Q and row kernels (softmax,
// query means, softmax backward) between them.  Layout (B, heads, Lq, Lk) for P, P',
// dP', dS.  kmask as AttnPair.
// ---------------------------------------------------------------------------
struct WidePair {
  const float* q; const float* k; const float* v;
  int32_t ldq, ldk, ldv;
  const float* kmask; int32_t kmask_mode; int32_t kmask_ld;
  int32_t Lq, Lk;
  uint32_t drop_site;
  float* P;            // scores, then softmax probabilities in place (fwd; kept for bwd)
  float* Pd;           // post-dropout P' (general plan; kept for bwd)
  float* probs;        // optional attention maps (post-dropout)
  float* pbar; float* pbarT;   // pooled plan: (B, heads, Lk), (B, Lk, heads)
  const float* dpbar;          // pooled plan bwd input
  float* o; int32_t ldo;       // general plan: O (B, Lq, ldo)
  const float* dout;           // general plan bwd: dO (B, Lq, ldo)
  float* dPd;                  // general plan bwd scratch: dP'
  float* dS;                   // bwd scratch
  float* dq; float* dk; float* dv;
};
constexpr int WIDE_MAX_PAIRS = 16;
bool wide_supported(int B, int heads, int Lq, int Lk);
hipError_t launch_wide_fwd(const WidePair* pairs, int npairs, int B, int heads, int hd, float scale, float drop_p,
                           const RngSnap* rng, bool pooled, hipStream_t st);
hipError_t launch_wide_bwd(const WidePair* pairs, int npairs, int B, int heads, int hd, float scale, float drop_p,
                           const RngSnap* rng, bool pooled, hipStream_t st);

// ---------------------------------------------------------------------------
// Pooled-output helpers (pool.hip), per (pair, sample):
//   U[h] = pbar_h P_k      r[h] = sum_j pbar_h[j]            (forward)
//   dpbar_h[j] = P_k[j] . dU[h] + dObar_h . bv_h             (backward)
//   E_m = cscale * c_m (row-broadcast) + sum_{pairs g with key m} pbar_g^T dU_g
// ---------------------------------------------------------------------------
struct PoolPair {
  const float* pk;     // P_k (B, Lk, H)
  int32_t Lk;
  const float* pbar;   // (B, heads, Lk)
  float* u;            // (B, heads, H)
  float* r;            // (B, heads)
  const float* du;     // (B, heads, H)
  const float* dob;    // dObar (B, H)
  const float* bv;     // value_proj.bias (H)
  float* dpbar;        // (B, heads, Lk)
};
constexpr int POOL_MAX_PAIRS = 12;
constexpr int POOL_PB_CAP = 4096;   // heads x Lk query-mean probabilities one pool_u workgroup stages in LDS
struct PoolArgs {
  PoolPair p[POOL_MAX_PAIRS];
  int32_t npairs, B, heads, hd, H;
};
hipError_t launch_pool_u(const PoolPair* pairs, int npairs, int B, int heads, int hd, int H, hipStream_t st);
hipError_t launch_pool_dpbar(const PoolPair* pairs, int npairs, int B, int heads, int hd, int H,
                             hipStream_t st);
constexpr int POOLE_MAX_SRC = 7;
struct PoolEMod {
  float* out;          // (B, L, H)
  int32_t L;
  const float* c; int32_t ldc; float cscale;   // row-broadcast term c[b*ldc + col] * cscale
  int32_t nsrc;
  const float* pbar[POOLE_MAX_SRC];            // (B, heads, L)
  const float* du[POOLE_MAX_SRC];              // (B, heads, H)
};
hipError_t launch_pool_e(const PoolEMod* mods, int nmods, int B, int heads, int H, hipStream_t st);

// ---------------------------------------------------------------------------
// Fusion head: pooling + gating + adaptive weights + weighted sum, and backward.
// ---------------------------------------------------------------------------
constexpr int HEAD_MAX_SRC = 64;
struct HeadArgs {
  int32_t B, M, H;
  const float* mask;                     // (B, M)
  int32_t scale_by_mask;                 // agg *= mask (src/fusion.py:408); 0 for compute_adaptive_weights
  // pooled_m = mask_m * inv_cnt[m] * sum_{sources s of m} src_scale[s] * sum_{rows} src_s
  // (each source is (B, src_L[s], H); src_scale = 1/L for an L-mean)
  const float* src[HEAD_MAX_SRC];
  int32_t src_mod[HEAD_MAX_SRC];
  int32_t src_L[HEAD_MAX_SRC];
  float src_scale[HEAD_MAX_SRC];
  int32_t nsrc;
  float inv_cnt[8];                      // 1 / n_entries_m (the list length, src/fusion.py:406-408)
  const float* gate_w[8]; const float* gate_b[8];
  float* pooled;                         // (B, M, H)
  float* scores;                         // (B, M)
  float* weights;                        // (B, M)
  float* fused;                          // (B, H)
  float* weights_out;                    // optional copy (B, M)
  // backward
  const float* dfused;                   // (B, H); null => dweights gives dL/dw directly
  const float* dweights;                 // (B, M) upstream grad of the weights (when dfused is null)
  float* cvec;                           // (B, M, H) = dpooled_m * mask_m * inv_cnt[m]; a source
                                         // row's grad is cvec * src_scale
  float* dscore;                         // (B, M)
};
hipError_t launch_head_fwd(const HeadArgs& a, hipStream_t st);
hipError_t launch_head_bwd(const HeadArgs& a, hipStream_t st);
// dgw[m][j] = sum_b dscore[b][m] * pooled[b][m][j]; dgb[m] = sum_b dscore[b][m]
hipError_t launch_gate_wgrad(int B, int M, int H, const float* dscore, const float* pooled,
                             float* const* dgw, float* const* dgb, hipStream_t st);

hipError_t launch_rng_snapshot(const uint64_t* state, RngSnap* snap, hipStream_t st);
hipError_t launch_rng_advance(uint64_t* state, hipStream_t st);   // state[1] += 1
hipError_t launch_cross_entropy(int B, int C, const float* logits, const int64_t* labels,
                                float smoothing, float grad_scale, float* loss, float* dlogits,
                                hipStream_t st);
hipError_t launch_grad_accum(int64_t n, const float* src, float* dst, hipStream_t st);   // dst += src
hipError_t launch_adamw(int64_t n, float* p, const float* g, float* m, float* v, int64_t* step,
                        float lr, float b1, float b2, float eps, float wd, float gscale,
                        hipStream_t st, const float* lr_dev = nullptr, const float* coef_dev = nullptr);
size_t grad_clip_workspace_bytes();
hipError_t launch_grad_clip_coef(int64_t n, const float* g, float gscale, float max_norm, float* norm_out,
                                 float* coef_out, float* partial, hipStream_t st);
// grad_sumsq (advancing *step) + one clip-and-AdamW launch (mmf_clip_adamw_step_dev)
hipError_t launch_grad_sumsq(int64_t n, const float* g, float* partial, int64_t* step, hipStream_t st);
hipError_t launch_clip_adamw_apply(int64_t n, float* p, const float* g, float* m, float* v, const int64_t* step,
                                   const float* lr_dev, float b1, float b2, float eps, float wd, float gscale,
                                   float max_norm, float* norm_out, float* coef_out, const float* partial,
                                   hipStream_t st);
constexpr int CLIP_PARTIAL_SLOTS = 1024;   // (head.hip: static_assert(CLIP_SLOTS == CLIP_PARTIAL_SLOTS))
hipError_t launch_clip_adamw(int64_t n, float* p, const float* g, float* m, float* v, int64_t* step,
                             const float* lr_dev, float b1, float b2, float eps, float wd, float gscale,
                             float max_norm, float* norm_out, float* coef_out, float* partial, hipStream_t st);

}  // namespace mmf

namespace mmf {

// ---------------------------------------------------------------------------
// Fused tail of the pooled plan (tail.hip): the B-row work that is otherwise a
// chain of tiny latency-bound launches, as one launch per (pair, sample) and one
// per sample in each direction.
//   forward : U_g = pbar_g P_k; Obar_g = U_g W_v^T (per head) + r_g b_v;  Abar_g = Obar_g W_o^T + b_o;
//             pooled_m = mask_m / n_m * (mean_L P_m + sum_{g: q(g)=m} Abar_g);
//             gating scores, adaptive weights, fused; h1 = Drop(ReLU(fused W1^T + b1));
//             logits = h1 W2^T + b2                                 (src/fusion.py:383-427)
//   backward: dz1 = ReLU'/Drop'(dlogits W2); dfused = dz1 W1; head backward
//             (dscore, cvec); dObar_g = cvec_q(g) W_o; dU_g,h = dObar_g,h W_v,h;
//             dpbar_g,h = P_k dU_g,h + dObar_g,h . b_v,h
// ---------------------------------------------------------------------------
struct TailPair {
  const float* pbar; const float* Pk; int32_t Lk;   // (B, h, Lk) query-mean probs; key features (B, Lk, H)
  int32_t q;                                         // query modality of the pair
  int32_t k;                                         // key modality of the pair
  float* U; float* r;                  // (B, h, H), (B, h) written by the forward
  const float* Wv; const float* bv; const float* Wo; const float* bo;
  float* Ob; float* Ab;                // (B, H) Obar (saved) and Abar
  float* dOb;                          // (B, H)
  float* dU;                           // (B, h, H)
  float* dpbar;                        // (B, h, Lk)
};
constexpr int TAIL_MAX_PAIRS = 12;
constexpr int TAIL_MAX_H = 256;
struct TailArgs {
  int32_t B, M, H, C, heads, hd, npairs;
  const float* mask;                   // (B, M)
  const float* P[8]; int32_t L[8];     // projected features (B, L_m, H)
  const float* Pcol[8]; int32_t ncol[8];  // optional per-128-row column sums of P_m (B, ncol, H)
  float inv_cnt[8];
  const float* gate_w[8]; const float* gate_b[8];
  const float* W1; const float* b1; const float* W2; const float* b2;
  float* pooled; float* scores; float* weights; float* weights_out; float* fused; float* h1; float* logits;
  float drop_p; uint32_t drop_site; const RngSnap* rng;
  // backward
  const float* dlogits; float* dz1; float* cvec; float* dscore; float gscale;
  // a training step's loss in the head launch (the 16-sample tile head, launch_seq_head_fwd):
  // per-sample loss rows, the batch mean by the last tile to count (loss_cnt: zero between
  // calls), dlogits, and the head backward in the same launch (launch_tail_bwd then skips it)
  const int64_t* labels; float ls_eps, loss_scale;
  float* loss_rows; float* loss_mean; uint32_t* loss_cnt; float* dlogits_out;
  int32_t head_done;
  TailPair p[TAIL_MAX_PAIRS];
  // pairs grouped by key modality (launch_tail_*: the P_k-side kernels read P_k[b] once per group)
  int32_t nkg;
  int32_t kg_cnt[8];
  int32_t kg_pair[8][TAIL_MAX_PAIRS];   // (int32: a byte in the kernarg segment is a vector load and a wait)
};
bool tail_supported(int M, int H, int C, int heads, int hd, int npairs);
hipError_t launch_tail_fwd(const TailArgs& a, hipStream_t st);
hipError_t launch_tail_bwd(const TailArgs& a, hipStream_t st);
// The tail's head on 16-sample tiles (l1.hip's head phases, the pooled sources read from the
// projection GEMM's column sums and the pairs' Abar): H <= 128, M <= 4, C <= 16, every modality
// with column sums.  The forward launch also runs the loss and the head backward when a.labels.
bool seq_head_ok(const TailArgs& a);
hipError_t launch_seq_head_fwd(const TailArgs& a, hipStream_t st);
hipError_t launch_seq_head_bwd(const TailArgs& a, hipStream_t st);

// ---------------------------------------------------------------------------
// Launch-lean single-key step (l1.hip): every modality 2-D (L = 1, what src/train.py:261-279
// feeds HybridFusion), every ordered pair present, fp32 ("highest").  Per 16-sample tile:
//   pair fwd  (tile, pair):      X'_k, P_k = Drop(ReLU(X'_k W_k^T + b)), V = P_k W_v^T + b_v,
//                                O = P' V (P' per head), A = O W_o^T + b_o
//   head fwd  (tile):            pooled, gating scores, adaptive weights, fused, h1, logits
//   head bwd  (tile):            dz1, dfused = dz1 W1, dscore, cvec
//   pair bwd  (tile, pair):      dO = cvec_q W_o, dV = P' dO, dP_k|g = dV W_v
//   modality bwd (tile, m):      dZ_m = gate(cvec_m + sum_g dP_k|g), dX_m = (dZ_m W_m) mask keep
//   wgrad     (32x32 tiles):     every weight / bias gradient, K = B split over 4 waves, fixed
//                                order; query / key projection gradients written as zeros
// ---------------------------------------------------------------------------
constexpr int L1_MAXM = 4, L1_MAXP = 12, L1_MAXH = 128, L1_MAXD = 128, L1_MAXC = 16;
struct L1Args {
  int32_t B, M, H, C, heads, npairs;
  int32_t D[L1_MAXM];
  int32_t pq[L1_MAXP], pk[L1_MAXP];
  int32_t kdesig[L1_MAXM];           // the pair that stores X'_k and P_k (first pair keyed by k)
  float p, gscale;                    // dropout p (0: no dropout) and 1 / (1 - p) (1 without)
  float inv_cnt[L1_MAXM];
  const float* mask;                  // (B, M)
  const float* x[L1_MAXM];            // (B, D_m)
  const uint64_t* rng_live;           // forward: the caller's live {seed, offset} (null: eval)
  uint64_t* rng_advance;              // forward: offset advanced by the head kernel
  RngSnap* snap;                      // the call's snapshot (saved)
  const float *Wp[L1_MAXM], *bp[L1_MAXM];
  const float *Wv[L1_MAXP], *bv[L1_MAXP], *Wo[L1_MAXP], *bo[L1_MAXP];
  const float *gw[L1_MAXM], *gb[L1_MAXM];
  const float *W1, *b1, *W2, *b2;
  float *Xd[L1_MAXM], *P[L1_MAXM], *O[L1_MAXP], *A[L1_MAXP];
  float *pooled, *scores, *weights, *fused, *h1;
  float *logits, *weights_out;
  float* maps[L1_MAXP];               // optional attention maps (B, heads, 1, 1)
  const float* dlogits;
  float *dz1, *cvec, *dscore;
  float *dV[L1_MAXP], *dPk[L1_MAXP], *dZ[L1_MAXM], *dx[L1_MAXM];
  // the one-launch forward + loss + head backward of a training step (launch_l1_train)
  uint32_t* tile_cnt;                 // the one-launch step's sync words (zero between calls):
                                      // tiles x (arrivals, head done, seen, L1_MAXM key arrivals), error
  uint32_t poll_bound;                // polls of the head's done word before a waiter gives up (timeout)
  const int64_t* labels;
  float ls_eps, loss_scale;           // label smoothing; dlogits scale (1 / accumulation steps)
  float* loss_rows;                   // (B) per-sample loss
  float* dlogits_out;                 // (B, C)
  // the sequence tail's head (launch_seq_head_*): P[m] holds the projection GEMM's per-128-row
  // column sums of P_m (B, ncol, H), scaled by inv_L; A[g] the pair's Abar (B, H)
  int32_t ncol[L1_MAXM];
  float inv_L[L1_MAXM];
  float* loss_mean; uint32_t* loss_cnt;   // optional: the batch-mean loss by the last tile to count
};
constexpr int L1_MAXJOBS = 40, L1_MAXZ = 48;
struct L1WgJob {                      // dW (N x K) = G^T X over B rows; db = column sums of G
  const float* G; const float* X; float* dW; float* db;
  int32_t ldg, ldx, N, K, tiles_k, tile0;
};
struct L1WgArgs {
  L1WgJob j[L1_MAXJOBS];
  int32_t njobs, B, ntiles;
  float* z[L1_MAXZ]; int32_t zn[L1_MAXZ]; int32_t zoff[L1_MAXZ + 1]; int32_t nz;
  const float* loss_rows; float* loss;   // optional: loss = mean of loss_rows (one extra workgroup)
  float* clip_partial;                   // optional: squared-norm partial per output tile (CLIP_PARTIAL_SLOTS)
  int64_t* step_incr;                    // optional: the optimizer step counter, advanced once
  uint64_t* rng_advance;                 // optional: the live dropout state's offset, advanced once
  // optional (launch_l1_train): the one-launch step's sync words.  The extra workgroup reads the
  // error word the forward launch may have set (a waiter's poll timed out); if set it returns the
  // sync_words tile words to 0 (the next call starts clean), writes loss = NaN and one +inf clip
  // partial (the update then applies a zero gradient), and leaves the error word for the host
  // (mmf_hybrid_train_status)
  uint32_t* sync; int32_t sync_words;
};
hipError_t launch_l1_forward(const L1Args& a, hipStream_t st);
hipError_t launch_l1_backward(const L1Args& a, const L1WgArgs& w, hipStream_t st);
// forward + cross-entropy + backward of a training step: three launches
hipError_t launch_l1_train(const L1Args& a, const L1WgArgs& w, hipStream_t st);
// workgroups of the one-launch step's forward kernel the device holds at once (occupancy x CUs)
int l1_train_capacity(bool full_h128);

}  // namespace mmf
