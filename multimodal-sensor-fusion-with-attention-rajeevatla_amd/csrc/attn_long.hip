// Long-key pooled attention backward in one pass, bf16 operands ("medium").
//
// The pooled formulation's backward (src/attention.py:118-139 under the pooled output of
// src/fusion.py:406-408) needs, per (pair, sample, head):
//   P[q, k]  = exp(s[q, k] - lse[q]),  s = scale q.k
//   D[q]     = sum_k keep[q, k] P[q, k] g[k],          g[k] = dpbar[k] / ((1 - p) Lq)
//   dS[q, k] = P[q, k] (keep[q, k] g[k] - D[q])
//   dQ = scale dS K,  dK = scale dS^T Q.
// The two-kernel path (attn_poolL_dq_kernel: a D pass and a dS pass over the keys, then
// attn_pool_bwd_dk_kernel) recomputes S and exp three times per score; at C5's Lk = 512
// those kernels are bound by the vector ALU, not the matrix cores or HBM.  Here one
// workgroup (8 waves) owns every key of one (pair, sample, head):
//   * the key image (Lk x 64 bf16) is staged in LDS once;
//   * wave w owns key tiles w and w + 8 (32 keys each) and walks the queries in blocks of
//     32: S^T = K Q^T on the matrix cores (query on the lane), P and its partial D in
//     registers, the partial D's of the 8 waves summed through LDS (fixed order), then dS
//     from the registers -- one exp per score;
//   * dQ = dS K takes dS straight from the accumulator registers and K through transposed
//     LDS reads (ds_read_b64_tr_b16); the 8 waves' partial dQ tiles are summed through LDS
//     in a fixed order (deterministic) and stored;
//   * dK += dS^T Q stays in registers for the whole pass: dS goes through a per-wave LDS
//     tile and comes back transposed (ds_read_b64_tr_b16), Q likewise from its block image.
// Images: 128-B rows with the 16-B chunk c of row r at c ^ swk(r) (conflict-free row reads
// of the 32x32x16 operands and 4-row transposed reads); the dS tile: 64-B rows, chunk
// g at g ^ ((q >> 1) & 3), 8-B halves flipped by q bit 3 (ds_off4); the dQ partials: [d][q] fp32,
// 16-B chunk j at j ^ f(d).
// Conditions (attn_long_fused_ok): 128 < Lk <= 512, Lk % 32 == 0, no per-key mask,
// head_dim <= 64 and % 4, float4-able Q / K rows; dropout through the forward's keep words.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mmf_device.h"

namespace mmf {

namespace {

constexpr int LF_NT = 512;                 // 8 waves: two per SIMD
constexpr int LF_MAXK = 512;
constexpr int LF_QB = 32;                  // queries per block
constexpr float LF_LOG2E = 1.4426950408889634f;

constexpr int OFF_K = 0;                               // [LF_MAXK][64] bf16
constexpr int OFF_Q = OFF_K + LF_MAXK * 128;           // [2][32][64] bf16
constexpr int OFF_S = OFF_Q + 2 * LF_QB * 128;         // [8][32 q][32 keys] bf16
constexpr int OFF_R = OFF_S + 8 * LF_QB * 64;          // [8][64 d][32 q] fp32
constexpr int OFF_D = OFF_R + 8 * 64 * LF_QB * 4;      // [2][8][32] fp32
constexpr int OFF_G = OFF_D + 2 * 8 * LF_QB * 4;       // [LF_MAXK] fp32
constexpr int OFF_L = OFF_G + LF_MAXK * 4;             // [2][32] fp32
constexpr int LF_LDS = OFF_L + 2 * LF_QB * 4;          // 160,000 bytes
static_assert(LF_LDS <= 160 * 1024, "one workgroup per CU");

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

__device__ __forceinline__ int swk(int row) { return (((row >> 1) & 1) << 2) | ((row >> 2) & 3); }
// byte offset of 16-B chunk c (columns 8c .. 8c+7) of row `row` of a 128-B-row bf16 image
__device__ __forceinline__ int img_off(int row, int c) { return row * 128 + 16 * (c ^ swk(row)); }
// byte offset of the 4 columns d0 .. d0+3 (d0 % 4 == 0) of row `row`
__device__ __forceinline__ int img_off4(int row, int d0) { return img_off(row, d0 >> 3) + 2 * (d0 & 7); }
// the dS tile: 64-B rows (32 keys), 16-B chunk g (keys 8g .. 8g+7) at g ^ ((q >> 1) & 3), and
// within it the 8-B half of keys key0 .. key0+3 (key0 % 4 == 0) flipped by query bit 3: the
// register-order stores (ds_write_b64, 16 consecutive lanes = queries q .. q+15 of one 4-key
// group) then cover 16 distinct 8-B bank pairs (queries q and q + 8 shared one before: the 2-way
// conflict both one-pass kernels showed, 18.95 M cycles each at C5 "medium",
// profiles/r05/close3/pmc_sq_c5_medium.json); the transposed reads (8 B per lane, a 4-key group
// of rows q0 .. q0+3 with q0 % 16 < 4 or in 8 .. 11) stay a bijection onto the 256-B bank row.
__device__ __forceinline__ int ds_off4(int q, int key0) {
  return q * 64 + 16 * ((key0 >> 3) ^ ((q >> 1) & 3)) + 8 * (((key0 >> 2) & 1) ^ ((q >> 3) & 1));
}
// the dQ partials: [d][32 q] fp32, 16-B chunk j (queries 4j .. 4j+3) at j ^ f(d)
__device__ __forceinline__ int red_off(int d, int j) {
  return d * 32 + 4 * (j ^ ((d & 7) ^ ((d >> 4) & 1)));
}

__device__ __forceinline__ bf16x4 tr_read(const char* lds, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(lds + off));
}
__device__ __forceinline__ bf16x8 cat8(bf16x4 lo, bf16x4 hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ bf16x8 to_bf16x8(float4 a, float4 b) {
  bf16x8 v;
  v[0] = (__bf16)a.x; v[1] = (__bf16)a.y; v[2] = (__bf16)a.z; v[3] = (__bf16)a.w;
  v[4] = (__bf16)b.x; v[5] = (__bf16)b.y; v[6] = (__bf16)b.z; v[7] = (__bf16)b.w;
  return v;
}
__device__ __forceinline__ f32x16 mfma_bf16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
// MMF_LONG_PK=0 (A/B build, Makefile `nopk`): the exp arguments and the pair trees below as
// scalar v_fma / v_add_f32 in the same association (bit-identical results) instead of
// v_pk_fma_f32 / v_pk_add_f32
#ifndef MMF_LONG_PK
#define MMF_LONG_PK 1
#endif
// sum of N (a power of two) packed pairs as a tree
template <int N>
__device__ __forceinline__ float tree_sum(f32x2* p) {
#if MMF_LONG_PK
#pragma unroll
  for (int n = N / 2; n >= 1; n /= 2)
#pragma unroll
    for (int i = 0; i < n; ++i) p[i] = p[i] + p[i + n];
  return p[0].x + p[0].y;
#else
  float a[N], b[N];
#pragma unroll
  for (int i = 0; i < N; ++i) { a[i] = p[i].x; b[i] = p[i].y; }
#pragma unroll
  for (int n = N / 2; n >= 1; n /= 2)
#pragma unroll
    for (int i = 0; i < n; ++i) { a[i] = a[i] + a[i + n]; b[i] = b[i] + b[i + n]; }
  return a[0] + b[0];
#endif
}
// (x0, x1) = (s0, s1) * c - o, one v_pk_fma_f32 or two v_fma_f32
__device__ __forceinline__ void exp_args2(float s0, float s1, float c, float o, float& x0, float& x1) {
#if MMF_LONG_PK
  const f32x2 x = f32x2{s0, s1} * f32x2{c, c} - f32x2{o, o};
  x0 = x[0];
  x1 = x[1];
#else
  x0 = __builtin_fmaf(s0, c, -o);
  x1 = __builtin_fmaf(s1, c, -o);
#endif
}

__device__ __forceinline__ f32x16 zero16f() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// 8 columns [d0, d0 + 8) of a row (zero past hd; hd % 4 == 0, 16-B aligned rows)
__device__ __forceinline__ void load8(const float* row, int d0, int hd, bool valid, float4& a, float4& b) {
  a = make_float4(0.f, 0.f, 0.f, 0.f);
  b = a;
  if (valid && d0 < hd) a = *reinterpret_cast<const float4*>(row + d0);
  if (valid && d0 + 4 < hd) b = *reinterpret_cast<const float4*>(row + d0 + 4);
}

// Columns [8c, 8c + 8) of element row `off` (element offset of the row's head slice) of a Q
// or K tensor as bf16: fp32 storage converted (round to nearest even), bf16 storage
// (AttnPair::qk_bf16, hd % 8 == 0) copied; zero past hd and for an invalid row
__device__ __forceinline__ bf16x8 row_chunk(const float* base, bool bf, int64_t off, int c, int hd, bool valid) {
  if (bf) {
    bf16x8 z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = (__bf16)0.f;
    if (valid && 8 * c < hd) z = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const __bf16*>(base) + off + 8 * c);
    return z;
  }
  float4 a, b;
  load8(base + off, 8 * c, hd, valid, a, b);
  return to_bf16x8(a, b);
}

#ifdef MMF_STAMPS
// Diagnostic build only (make stampsl): per-phase s_memtime sums over the query blocks of wave 0
// (slots 0..4) and of the first wave of the younger half (slots 5..8), and the workgroup's
// s_memrealtime lifetime (slot 9, 100 MHz); read by mmf_long_stamps_read (scripts/attn_stamps.py
// long / longf).  Never in the product library.
__device__ __forceinline__ unsigned long long ls_now() {
  unsigned long long t_;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t_;
}
__device__ __forceinline__ unsigned long long ls_rt() {
  unsigned long long t_;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t_;
}
#define LS_DECL                                       \
  unsigned long long ls_acc[5] = {0, 0, 0, 0, 0};     \
  const unsigned long long ls_rt0 = ls_rt();          \
  unsigned long long ls_prev = ls_now();
#define LS_MARK(k)                                    \
  {                                                   \
    const unsigned long long t_ = ls_now();           \
    ls_acc[k] += t_ - ls_prev;                        \
    ls_prev = t_;                                     \
  }
#define LS_STORE(w, wy)                                                                        \
  {                                                                                            \
    const unsigned long long rt_ = ls_rt();                                                    \
    const int sid_ = blockIdx.y * gridDim.x + blockIdx.x;                                      \
    if ((threadIdx.x & 63) == 0 && sid_ < STAMP_WG) {                                          \
      if ((w) == 0) {                                                                          \
        for (int k_ = 0; k_ < 5; ++k_) g_mmf_stamps[sid_][k_] = ls_acc[k_];                   \
        g_mmf_stamps[sid_][9] = rt_ - ls_rt0;                                                  \
      } else if ((w) == (wy)) {                                                                \
        for (int k_ = 0; k_ < 4; ++k_) g_mmf_stamps[sid_][5 + k_] = ls_acc[k_];               \
      }                                                                                        \
    }                                                                                          \
  }
#else
#define LS_DECL
#define LS_MARK(k)
#define LS_STORE(w, wy)
#endif

// Prefetches that stay in flight: ONE unconditional load at a clamped, in-bounds address and no
// use of the loaded register until the consumer (the image store a phase later, or the next
// block).  A guarded load (a per-lane zero fill) or a shift / conversion right behind the load
// is a use: the compiler waits for it there (s_waitcnt vmcnt(0) behind every prefetch: three
// global round trips exposed in every query block of both kernels).  Validity is applied where
// the value is consumed (chunk_keep).  fp32 Q / K storage converts at the load (row_chunk: its
// wait stays; not the bf16 path the "medium" plan runs).
// The prefetches go through buffer loads: a wave-uniform resource (base, size) in SGPRs, a
// lane offset fixed for the whole kernel and a per-block scalar offset, so the loop builds no
// 64-bit VGPR addresses (a rebuilt address register that had been a load's destination was
// another wait, for every store in flight).  Reads past the size return zeros.
// a wave-uniform pointer the compiler computed in VGPRs (64-bit offset arithmetic goes to the
// VALU) back into SGPRs: a VGPR buffer resource turns each load into a waterfall loop
template <class T>
__device__ __forceinline__ T* sgpr_ptr(T* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<T*>(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, bytes, 0x00020000);
}
__device__ __forceinline__ bf16x8 buf_b128(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ uint32_t buf_b32(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0);
}
__device__ __forceinline__ bf16x8 chunk_keep(bf16x8 v, bool valid) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  u32x4 u = __builtin_bit_cast(u32x4, v);
#pragma unroll
  for (int j = 0; j < 4; ++j) u[j] = valid ? u[j] : 0u;
  return __builtin_bit_cast(bf16x8, u);
}

// FULL: Lk == LF_MAXK, every wave's two key tiles exist (no per-tile guards, whose skip
// paths made the compiler zero-fill the tiles' registers every query block)
template <bool BITS, bool FULL>
__global__ __launch_bounds__(LF_NT, 1) void attn_poolL_bwd_fused_bf16(const AttnArgs A) {
  __shared__ __attribute__((aligned(16))) char lds[LF_LDS];
  const AttnPair& P = A.p[blockIdx.y];
  if ((int)blockIdx.x >= A.B * A.heads) return;
  const int head = blockIdx.x % A.heads, b = blockIdx.x / A.heads;
  // (w through readfirstlane: the compiler then knows it is wave-uniform, so the `w < 4` guards
  // around the prefetches are scalar branches and their buffer resources stay in SGPRs)
  const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6), hh = lane >> 5, r = lane & 31;
  // transposed-read addressing: lane 4 qp + pp of each 16-lane group g16 names row qp,
  // columns 4 pp .. 4 pp + 3 of the group's 16 columns (16 (g16 & 1) ..)
  const int g16 = lane >> 4, qp = (lane & 15) >> 2, pp = lane & 3;
  const int hd = A.hd, col0 = head * hd;
  const int Lq = P.Lq, Lk = P.Lk, nkt = Lk >> 5, nqb = (Lq + LF_QB - 1) / LF_QB, kwl = P.kw_ld;
  const int64_t bh = (int64_t)b * A.heads + head;
  const float scale = A.scale, pdrop = A.drop_p;
  const float inv_keep = pdrop > 0.f ? (pdrop < 1.f ? 1.f / (1.f - pdrop) : 0.f) : 1.f;
  const float sl2 = scale * LF_LOG2E;
  const bool qkb = P.qk_bf16 != 0;
  const int64_t q_off = (int64_t)b * Lq * P.ldq + col0, k_off = (int64_t)b * Lk * P.ldk + col0;   // elements
  float* dQg = P.dq + (int64_t)b * Lq * P.ldq + col0;
  float* dKg = P.dk + (int64_t)b * Lk * P.ldk + col0;
  // bf16 dQ / dK (AttnPair::dqk_bf16): the same element offsets, 2-byte elements
  const bool dqb = P.dqk_bf16 != 0;
  __bf16* dQh = reinterpret_cast<__bf16*>(P.dq) + (int64_t)b * Lq * P.ldq + col0;
  __bf16* dKh = reinterpret_cast<__bf16*>(P.dk) + (int64_t)b * Lk * P.ldk + col0;

  if (P.kmask_mode == 1 && P.kmask[(int64_t)b * P.kmask_ld] == 0.f) {
    // masked key modality: every probability is 0 (src/attention.py:127-129), so are dQ, dK, D
    for (int i = t; i < Lq * hd; i += LF_NT) {
      const int64_t o = (int64_t)(i / hd) * P.ldq + i % hd;
      if (dqb) dQh[o] = (__bf16)0.f;
      else dQg[o] = 0.f;
    }
    for (int i = t; i < Lk * hd; i += LF_NT) {
      const int64_t o = (int64_t)(i / hd) * P.ldk + i % hd;
      if (dqb) dKh[o] = (__bf16)0.f;
      else dKg[o] = 0.f;
    }
    for (int i = t; i < Lq; i += LF_NT) P.dsum[bh * Lq + i] = 0.f;
    return;
  }

  float* gs = reinterpret_cast<float*>(lds + OFF_G);
  float* lse_s = reinterpret_cast<float*>(lds + OFF_L);
  float* Dpart = reinterpret_cast<float*>(lds + OFF_D);

  // ---- prologue: the key image, g, and query block 0
  {
    const int nch = Lk * 8;   // 16-B chunks of the image
    for (int i0 = 0; i0 < nch; i0 += LF_NT * 4) {
      bf16x8 kv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int idx = i0 + t + j * LF_NT;
        const int key = idx >> 3, c = idx & 7;
        kv[j] = row_chunk(P.k, qkb, k_off + (int64_t)(idx < nch ? key : 0) * P.ldk, c, hd, idx < nch);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int idx = i0 + t + j * LF_NT;
        if (idx < nch) *reinterpret_cast<bf16x8*>(lds + OFF_K + img_off(idx >> 3, idx & 7)) = kv[j];
      }
    }
    const float gsc = inv_keep / (float)Lq;   // dP'[q, k] = dpbar[k] / Lq, through the dropout scale
    for (int k = t; k < Lk; k += LF_NT) gs[k] = P.dpbar[bh * Lk + k] * gsc;
  }
  // query block images: the younger half (waves 4-7, thread tq = t - 256: row tq >> 3, chunk tq & 7)
  // stages the Q chunks, lanes 0-31 of wave 0 the LSE -- the older half is the pole at both
  // barriers once the younger issues at priority 1, so the extra work goes to the younger
  // (raw prefetches, wave-uniform guards; the resources are rebuilt at each use from the
  // wave-uniform bases: held across the loop, they were kept in VGPRs and every load became a
  // waterfall loop)
  constexpr int QW0 = 4, LW = 0;
  const int tq = t - 64 * QW0;
  const bool qstage = w >= QW0 && w < QW0 + 4;
  const uint32_t q_voff = (uint32_t)((((tq >> 3) & 31) * P.ldq + 8 * (tq & 7)) * 2);
  const __bf16* q_u = sgpr_ptr(reinterpret_cast<const __bf16*>(P.q) + q_off);
  const float* lse_u = sgpr_ptr(P.lse + bh * Lq);
  const uint32_t q_bytes = (uint32_t)(((int64_t)(Lq - 1) * P.ldq + hd) * 2);
  auto q_load = [&](int qb, bf16x8& v, float& l) {
    const int row = (tq >> 3) & 31, q = qb * LF_QB + row;
    if (qstage) {
      if (qkb) v = buf_b128(buf_rsrc(q_u, q_bytes), q_voff, (uint32_t)(qb * LF_QB * P.ldq * 2));
      else v = row_chunk(P.q, false, q_off + (int64_t)(q < Lq ? q : 0) * P.ldq, tq & 7, hd, q < Lq);
    }
    if (w == LW) l = __uint_as_float(buf_b32(buf_rsrc(lse_u, (uint32_t)Lq * 4u), (uint32_t)(t & 31) * 4u, (uint32_t)(qb * LF_QB * 4)));
  };
  auto q_store = [&](int qb, int buf, const bf16x8& v, float l) {
    const int q = qb * LF_QB + ((tq >> 3) & 31);
    if (qstage)
      *reinterpret_cast<bf16x8*>(lds + OFF_Q + buf * 4096 + img_off((tq >> 3) & 31, tq & 7)) =
          chunk_keep(v, q < Lq && 8 * (tq & 7) < hd);
    // log2 units; +inf for an invalid or fully masked query: every p = exp2(s - inf) = 0
    const int ql = qb * LF_QB + (t & 31);
    if (w == LW && lane < LF_QB)
      lse_s[buf * LF_QB + lane] = (ql >= Lq || l == -INFINITY) ? INFINITY : l * LF_LOG2E;
  };
  {
    bf16x8 v;
    float l;
    q_load(0, v, l);
    q_store(0, 0, v, l);
  }
  __syncthreads();

  f32x16 dk[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) dk[i][dt] = zero16f();
  char* Sw = lds + OFF_S + w * 2048;
  float* redw = reinterpret_cast<float*>(lds + OFF_R) + w * 2048;
  // the keep words of a query block as loaded (raw prefetch; the half shift and the validity
  // applied by the block that uses them)
  // (words of missing tiles, kt >= nkt, are read from wherever they land and never used)
  const uint32_t kw_voff = (uint32_t)((r * kwl + w) * 4);
  const uint32_t* kw_u = sgpr_ptr(P.keep_bits + bh * Lq * kwl);
  auto kw_fetch = [&](int qb, uint32_t (&raw)[2]) {
    const __amdgpu_buffer_rsrc_t rk = buf_rsrc(kw_u, (uint32_t)((int64_t)Lq * kwl * 4));
#pragma unroll
    for (int i = 0; i < 2; ++i) raw[i] = buf_b32(rk, kw_voff + 32u * i, (uint32_t)(qb * LF_QB * kwl * 4));
  };
  // keep words of the next block, shifted to this lane's half and validated at the END of the
  // block that loaded them (a loop-carried raw register would be copied at the loop head, a use
  // that waits for the load issued just before it)
  auto kw_finish = [&](int qb, const uint32_t (&raw)[2], uint32_t (&wd)[2]) {
    const bool ok = qb * LF_QB + r < Lq;
#pragma unroll
    for (int i = 0; i < 2; ++i) wd[i] = ((FULL || w + 8 * i < nkt) && ok) ? raw[i] >> (4 * hh) : 0xFFFFFFFFu;
  };
  uint32_t nwords[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};
  if (BITS) {
    uint32_t raw[2];
    kw_fetch(0, raw);
    kw_finish(0, raw, nwords);
  }

  // the younger half (waves 4-7: the arbitration losers, the pole at both barriers) issues at
  // priority 1 (MI355X_MICROARCH "two waves per SIMD" item 4; C5 4.20 -> 4.13 ms of this kernel
  // per step; MMF_LONG_NO_PRIO builds the A/B arm)
#ifndef MMF_LONG_NO_PRIO
  if (w >= 4) __builtin_amdgcn_s_setprio(1);
#endif
  LS_DECL
  for (int qb = 0; qb < nqb; ++qb) {
    const int buf = qb & 1, qbase = qb * LF_QB;
    const bool has_next = qb + 1 < nqb;
    bf16x8 nv;
    float nl;   // (no initial value: a register write here waited for every store in flight)
    if (has_next) q_load(qb + 1, nv, nl);   // in flight during this block
    const char* Qi = lds + OFF_Q + buf * 4096;
    const int q = qbase + r;
    const bool qvalid = q < Lq;
    // this block's keep words (loaded during the previous block), the next block's in flight
    const uint32_t words[2] = {nwords[0], nwords[1]};
    uint32_t nraw[2];
    if (BITS && has_next) kw_fetch(qb + 1, nraw);
    bf16x8 qf[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(Qi + img_off(r, 2 * s + hh));
    const float lse2 = lse_s[buf * LF_QB + r];

    // S^T = K Q^T per own key tile (key in the registers, query on the lane); P, keep * P * g, D
    float pv[2][16], pk[2][16];
    f32x2 dpp[16];   // keep * P * g pairs, summed as a packed tree
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int kt = w + 8 * i;
      if (!FULL && kt >= nkt) {
#pragma unroll
        for (int e = 0; e < 16; ++e) pv[i][e] = pk[i][e] = 0.f;
        continue;
      }
      f32x16 s = zero16f();
      const int krow = kt * 32 + r;
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
        s = mfma_bf16(*reinterpret_cast<const bf16x8*>(lds + OFF_K + img_off(krow, 2 * s4 + hh)), qf[s4], s);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 g4 = *reinterpret_cast<const float4*>(gs + kt * 32 + 8 * g + 4 * hh);
        const float gv[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
        for (int j = 0; j < 4; j += 2) {
          const int e = 4 * g + j;
          // (the exp arguments as packed FMAs: 16 v_pk_fma_f32 for the 32 scores)
          float x0, x1;
          exp_args2(s[e], s[e + 1], sl2, lse2, x0, x1);
          const float p0 = __builtin_amdgcn_exp2f(x0), p1 = __builtin_amdgcn_exp2f(x1);
          pv[i][e] = p0;
          pv[i][e + 1] = p1;
          pk[i][e] = p0 * keep_sel(words[i], j + 8 * g, gv[j]);
          pk[i][e + 1] = p1 * keep_sel(words[i], j + 1 + 8 * g, gv[j + 1]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 8; ++e) dpp[8 * i + e] = f32x2{pk[i][2 * e], pk[i][2 * e + 1]};
    const float Dp = sum_xor32(tree_sum<16>(dpp));
    if (hh == 0) Dpart[buf * 256 + w * 32 + r] = Dp;
    LS_MARK(0)
    __syncthreads();   // (A) partial D's
    LS_MARK(1)

    float D = 0.f;
#pragma unroll
    for (int ww = 0; ww < 8; ++ww) D += Dpart[buf * 256 + ww * 32 + r];
    if (w == 7 && hh == 0 && qvalid) P.dsum[bh * Lq + q] = D;   // (a younger wave: see q_load)

    // dS = P (keep g - D) of both tiles first (the bf16 A operands of dQ = dS K, register
    // e = 8 s2 + j): P and keep * P * g die here, before the matrix-core phase
    bf16x8 da[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int e = 8 * s2 + j;
          da[i][s2][j] = (__bf16)__builtin_fmaf(-pv[i][e], D, pk[i][e]);
        }
    f32x16 dq[2] = {zero16f(), zero16f()};
    // dQ[q][d] += sum_key dS[q][key] K[key][d]: K rows 32 kt + 16 s2 + 4 hh + {0..3, 8..11}
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int kt = w + 8 * i;
      if (!FULL && kt >= nkt) continue;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int d0 = 32 * dt + 16 * (g16 & 1) + 4 * pp;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int k0 = kt * 32 + 16 * s2 + 4 * hh + qp;
          const bf16x8 kb = cat8(tr_read(lds, OFF_K + img_off4(k0, d0)), tr_read(lds, OFF_K + img_off4(k0 + 8, d0)));
          dq[dt] = mfma_bf16(da[i][s2], kb, dq[dt]);
        }
      }
    }
    // dK[key][d] += sum_q dS[q][key] Q[q][d]: queries 16 s + 8 hh + {0..7}; the Q operands
    // (shared by both tiles) read once
    bf16x8 qb8[2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const int q0 = 16 * s + 8 * hh + qp, d0 = 32 * dt + 16 * (g16 & 1) + 4 * pp;
        qb8[s][dt] = cat8(tr_read(Qi, img_off4(q0, d0)), tr_read(Qi, img_off4(q0 + 4, d0)));
      }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int kt = w + 8 * i;
      if (!FULL && kt >= nkt) continue;
      // the dS tile [q][key] (registers 4g .. 4g+3 = keys 8g + 4hh + 0..3 of query r)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = da[i][g >> 1][4 * (g & 1) + j];
        *reinterpret_cast<bf16x4*>(Sw + ds_off4(r, 8 * g + 4 * hh)) = v;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int q0 = 16 * s + 8 * hh + qp;
        const int key0 = 16 * (g16 & 1) + 4 * pp;
        const bf16x8 sa = cat8(tr_read(Sw, ds_off4(q0, key0)), tr_read(Sw, ds_off4(q0 + 4, key0)));
#pragma unroll
        for (int dt = 0; dt < 2; ++dt) dk[i][dt] = mfma_bf16(sa, qb8[s][dt], dk[i][dt]);
      }
    }
    // this wave's partial dQ tile: lane = d, registers 4g .. 4g+3 = queries 8g + 4hh + 0..3
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      const int d = 32 * dt + r;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(redw + red_off(d, 2 * g + hh)) =
            make_float4(dq[dt][4 * g], dq[dt][4 * g + 1], dq[dt][4 * g + 2], dq[dt][4 * g + 3]);
    }
    // the next query block's images: its loads (issued at the top of this block) have had
    // phases 1 and 2 to land; buffer buf ^ 1 was last read in the previous block's phase 2
    if (has_next) q_store(qb + 1, buf ^ 1, nv, nl);
    // (here, not after this block's dQ stores: vmcnt counts stores, so a wait there is for them)
    if (BITS && has_next) kw_finish(qb + 1, nraw, nwords);
    LS_MARK(2)
    __syncthreads();   // (B) partial dQ's, next query block
    LS_MARK(3)

    {
      const int d = t & 63, j = t >> 6;   // queries 4j .. 4j+3 of column d
      const float* red = reinterpret_cast<const float*>(lds + OFF_R);
#if MMF_LONG_PK
      f32x2 a01, a23;   // packed adds
      {
        const float4 v = *reinterpret_cast<const float4*>(red + red_off(d, j));
        a01 = f32x2{v.x, v.y};
        a23 = f32x2{v.z, v.w};
      }
#pragma unroll
      for (int ww = 1; ww < 8; ++ww) {
        const float4 v = *reinterpret_cast<const float4*>(red + ww * 2048 + red_off(d, j));
        a01 += f32x2{v.x, v.y};
        a23 += f32x2{v.z, v.w};
      }
      const float av[4] = {a01.x, a01.y, a23.x, a23.y};
#else
      float av[4];
      {
        const float4 v = *reinterpret_cast<const float4*>(red + red_off(d, j));
        av[0] = v.x; av[1] = v.y; av[2] = v.z; av[3] = v.w;
      }
#pragma unroll
      for (int ww = 1; ww < 8; ++ww) {
        const float4 v = *reinterpret_cast<const float4*>(red + ww * 2048 + red_off(d, j));
        av[0] += v.x; av[1] += v.y; av[2] += v.z; av[3] += v.w;
      }
#endif
      if (d < hd) {
        // one 64-bit row offset per block, the 4 rows by 32-bit steps (per-element 64-bit
        // products were 24 integer multiplies per block)
        const int q0 = qbase + 4 * j, ld = P.ldq;
        const int64_t o0 = (int64_t)q0 * ld + d;
        if (dqb) {
          __bf16* dst = dQh + o0;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (q0 + e < Lq) dst[e * ld] = (__bf16)(av[e] * scale);
        } else {
          float* dst = dQg + o0;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (q0 + e < Lq) dst[e * ld] = av[e] * scale;
        }
      }
    }
    LS_MARK(4)
  }
  LS_STORE(w, 4)

  // dK: lane = d, registers = keys 32 kt + acc_row(e, hh)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int kt = w + 8 * i;
    if (!FULL && kt >= nkt) continue;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      const int d = 32 * dt + r;
      if (d >= hd) continue;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t o = (int64_t)(kt * 32 + acc_row(e, hh)) * P.ldk + d;
        if (dqb) dKh[o] = (__bf16)(dk[i][dt][e] * scale);
        else dKg[o] = dk[i][dt][e] * scale;
      }
    }
  }
}


// ---------------------------------------------------------------------------
// Dropout keep words of the attention probabilities, (B, heads, Lq, kw_ld) u32: bit j of
// word kt of row (b, head, q) keeps element ((b heads + head) Lq + q) Lk + 32 kt + j of the
// pair's Philox stream (site drop_site) -- the same words the streamed forward
// (attn_poolL_lse_kernel) draws inline and every backward reads.  One thread per word
// (4 Philox blocks of 8 elements; Lk % 32 == 0 keeps them aligned): the draws run at full
// occupancy here instead of inside the one-pass forward's exp phase.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void attn_keep_words_kernel(const AttnArgs A) {
  const AttnPair& P = A.p[blockIdx.y];
  const uint32_t nkt = (uint32_t)P.Lk >> 5;
  // 32-bit word index (the launcher checks B heads Lq nkt < 2^31): no 64-bit division
  const uint32_t nwords = (uint32_t)A.B * (uint32_t)A.heads * (uint32_t)P.Lq * nkt;
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= nwords) return;
  const uint32_t row = (nkt & (nkt - 1)) == 0 ? i >> (31 - __builtin_clz(nkt)) : i / nkt;
  const uint32_t kt = i - row * nkt;
  const RngSnap rs = *A.rng;
  const uint32_t thr = p16(A.drop_p);
  const uint64_t blk0 = ((uint64_t)row * P.Lk + 32 * kt) >> 3;
  uint32_t bits = 0;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const uint4 rr = philox_block(rs, P.drop_site, blk0 + g);
    const uint32_t wv[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      // element 2k: the low 16 bits of word k, element 2k + 1: the high 16 bits (keep_from)
      bits |= ((wv[k] & 0xFFFFu) >= thr ? 1u : 0u) << (8 * g + 2 * k);
      bits |= ((wv[k] >> 16) >= thr ? 1u : 0u) << (8 * g + 2 * k + 1);
    }
  }
  P.keep_bits[(uint64_t)row * P.kw_ld + kt] = bits;
}

// ---------------------------------------------------------------------------
// Forward in one pass (same conditions; "medium"): LSE, the dropout keep words and
// pbar = mean_q P' for every key of one (pair, sample, head).  Per 32-query block each
// wave forms S^T for its two key tiles, the 8 waves' row maxima and sums meet in LDS
// (fixed order), and P' = keep * exp2(s - m) * (1-p)^-1 / (l Lq) -- one exp per score,
// where the two-kernel path (attn_poolL_lse_kernel + attn_poolL_colsum_kernel) recomputes
// S and exp in a second pass.  The column sums over the queries (the lanes) go through a
// per-wave transposed P' tile (bf16, as the reference's P'.V operand at "medium") into an
// all-ones MFMA whose accumulator carries pbar across the query blocks.
// ---------------------------------------------------------------------------
// NW waves per workgroup (16: four per SIMD, one key tile each at Lk = 512; 8: two tiles each)
template <int NW>
struct FwdLds {
  static constexpr int Q = 0;                                // [2][32][64] bf16
  static constexpr int P = Q + 2 * LF_QB * 128;              // [NW][32 q][32 keys] bf16
  static constexpr int M = P + NW * LF_QB * 64;              // [2][NW][32] fp32 row maxima
  static constexpr int S = M + 2 * NW * LF_QB * 4;           // [2][NW][32] fp32 row sums
  static constexpr int BYTES = S + 2 * NW * LF_QB * 4;       // 28 KB (8 waves) / 48 KB (16)
};

template <bool DROP, int NW = 16>
__global__ __launch_bounds__(NW * 64, 1) void attn_poolL_fwd_fused_bf16(const AttnArgs A) {
  constexpr int NTW = NW * 64, TPW = 16 / NW;   // threads; key tiles per wave (Lk <= 512)
  using L_ = FwdLds<NW>;
  constexpr int FOFF_Q = L_::Q, FOFF_P = L_::P, FOFF_M = L_::M, FOFF_S = L_::S;
  __shared__ __attribute__((aligned(16))) char lds[L_::BYTES];
  const AttnPair& P = A.p[blockIdx.y];
  if ((int)blockIdx.x >= A.B * A.heads) return;
  const int head = blockIdx.x % A.heads, b = blockIdx.x / A.heads;
  // (w through readfirstlane: the compiler then knows it is wave-uniform, so the `w < 4` guards
  // around the prefetches are scalar branches and their buffer resources stay in SGPRs)
  const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6), hh = lane >> 5, r = lane & 31;
  const int g16 = lane >> 4, qp = (lane & 15) >> 2, pp = lane & 3;
  const int hd = A.hd, col0 = head * hd;
  const int Lq = P.Lq, Lk = P.Lk, nkt = Lk >> 5, nqb = (Lq + LF_QB - 1) / LF_QB, kwl = P.kw_ld;
  const int64_t bh = (int64_t)b * A.heads + head;
  const float pdrop = A.drop_p;
  const float inv_keep = pdrop > 0.f ? (pdrop < 1.f ? 1.f / (1.f - pdrop) : 0.f) : 1.f;
  const float sl2 = A.scale * LF_LOG2E;
  const bool qkb = P.qk_bf16 != 0;
  const int64_t q_off = (int64_t)b * Lq * P.ldq + col0, k_off = (int64_t)b * Lk * P.ldk + col0;   // elements

  if (P.kmask_mode == 1 && P.kmask[(int64_t)b * P.kmask_ld] == 0.f) {
    // masked key modality: every probability is 0 (src/attention.py:127-129); the keep words
    // are never read when LSE = -inf
    for (int i = t; i < Lq; i += NTW) P.lse[bh * Lq + i] = -INFINITY;
    for (int k = t; k < Lk; k += NTW) {
      P.pbar[bh * Lk + k] = 0.f;
      if (P.pbarT) P.pbarT[((int64_t)b * Lk + k) * A.heads + head] = 0.f;
    }
    return;
  }
  float* Mpart = reinterpret_cast<float*>(lds + FOFF_M);
  float* Spart = reinterpret_cast<float*>(lds + FOFF_S);

  // each wave's key tiles stay in registers for every query block (the MFMA A operand:
  // lane (r, hh) holds columns [16 s4 + 8 hh, +8) of key row 32 kt + r)
  bf16x8 kf[TPW][4];
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int krow = (w + NW * i) * 32 + r;
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4)
      kf[i][s4] = row_chunk(P.k, qkb, k_off + (int64_t)(krow < Lk ? krow : 0) * P.ldk, 2 * s4 + hh, hd, krow < Lk);
  }
  // (raw prefetches through buffer loads: waves 0-3 stage the Q chunks)
  // (the younger half's first 4 waves stage the Q images, as the backward)
  constexpr int QW0 = NW / 2;
  const int tq = t - 64 * QW0;
  const bool qstage = w >= QW0 && w < QW0 + 4;
  const uint32_t q_voff = (uint32_t)((((tq >> 3) & 31) * P.ldq + 8 * (tq & 7)) * 2);
  const __bf16* q_u = sgpr_ptr(reinterpret_cast<const __bf16*>(P.q) + q_off);
  const uint32_t q_bytes = (uint32_t)(((int64_t)(Lq - 1) * P.ldq + hd) * 2);
  auto q_load = [&](int qb, bf16x8& v) {
    const int q = qb * LF_QB + ((tq >> 3) & 31);
    if (qstage) {
      if (qkb) v = buf_b128(buf_rsrc(q_u, q_bytes), q_voff, (uint32_t)(qb * LF_QB * P.ldq * 2));
      else v = row_chunk(P.q, false, q_off + (int64_t)(q < Lq ? q : 0) * P.ldq, tq & 7, hd, q < Lq);
    }
  };
  auto q_store = [&](int qb, int buf, const bf16x8& v) {
    const int q = qb * LF_QB + ((tq >> 3) & 31);
    if (qstage)
      *reinterpret_cast<bf16x8*>(lds + FOFF_Q + buf * 4096 + img_off((tq >> 3) & 31, tq & 7)) =
          chunk_keep(v, q < Lq && 8 * (tq & 7) < hd);
  };
  {
    bf16x8 v;
    q_load(0, v);
    q_store(0, 0, v);
  }
  __syncthreads();

  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;
  f32x16 cs[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) cs[i] = zero16f();   // every row of C = the column sums of P'
  char* Pw = lds + FOFF_P + w * 2048;
  // S = K Q^T of the own tiles for query block `qb` (raw scores; the scale folds into the
  // exp's FMA).  Block qb + 1's products are issued right after barrier A of block qb, so
  // the matrix cores run them under that block's exp / sum phase.
  auto scores = [&](int qbuf, f32x16 (&sc)[TPW]) {
    const char* Qi = lds + FOFF_Q + qbuf * 4096;
    bf16x8 qf[4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) qf[s4] = *reinterpret_cast<const bf16x8*>(Qi + img_off(r, 2 * s4 + hh));
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      if (w + NW * i >= nkt) continue;   // (not read for a missing tile)
      sc[i] = zero16f();
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) sc[i] = mfma_bf16(kf[i][s4], qf[s4], sc[i]);
    }
  };
  f32x16 sn[TPW];
  scores(0, sn);
  // Loads run two query blocks ahead of their LDS store: the images of block qb + 1 are stored
  // before barrier A of block qb (block qb + 1's products are issued right after it), so their
  // loads are issued at the top of block qb - 1 (one whole block of latency cover; issued at
  // the top of block qb, phase 1 alone -- a few hundred cycles -- had to cover them).  The keep
  // words of block qb + 1 likewise load during block qb.
  bf16x8 nv;
  if (nqb > 1) q_load(1, nv);
  // raw keep words (the half shift and validity applied by the block that uses them)
  const uint32_t* kw_u = sgpr_ptr(P.keep_bits + bh * Lq * kwl);
  const uint32_t kw_voff = (uint32_t)((r * kwl + w) * 4);
  auto kw_load = [&](int qb, uint32_t (&kw)[TPW]) {
    const __amdgpu_buffer_rsrc_t rk = buf_rsrc(kw_u, (uint32_t)((int64_t)Lq * kwl * 4));
#pragma unroll
    for (int i = 0; i < TPW; ++i) kw[i] = buf_b32(rk, kw_voff + 4u * NW * i, (uint32_t)(qb * LF_QB * kwl * 4));
  };
  // shifted to this lane's half and validated at the end of the block that loaded them (see the
  // backward's kw_finish)
  auto kw_finish = [&](int qb, const uint32_t (&raw)[TPW], uint32_t (&wd)[TPW]) {
    const bool ok = qb * LF_QB + r < Lq;
#pragma unroll
    for (int i = 0; i < TPW; ++i) wd[i] = (ok && w + NW * i < nkt) ? raw[i] >> (4 * hh) : 0xFFFFFFFFu;
  };
  uint32_t kwn[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) kwn[i] = 0xFFFFFFFFu;
  if (DROP) {
    uint32_t raw[TPW];
    kw_load(0, raw);
    kw_finish(0, raw, kwn);
  }

#ifndef MMF_LONG_NO_PRIO
  if (w >= NW / 2) __builtin_amdgcn_s_setprio(1);   // (the younger half, as the backward)
#endif
  LS_DECL
  for (int qb = 0; qb < nqb; ++qb) {
    const int buf = qb & 1, qbase = qb * LF_QB;
    const bool has_next = qb + 1 < nqb;
    bf16x8 nv2;
    if (qb + 2 < nqb) q_load(qb + 2, nv2);
    const int q = qbase + r;
    const bool qvalid = q < Lq;
    // the keep words of the own tiles (attn_keep_words_kernel), consumed after barrier B
    uint32_t kw[TPW], kraw[TPW];
#pragma unroll
    for (int i = 0; i < TPW; ++i) kw[i] = kwn[i];
    if (DROP && has_next) kw_load(qb + 1, kraw);
    float x[TPW][16];
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      if (w + NW * i >= nkt) continue;   // (x[i] is not read for a missing tile)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        x[i][e] = sn[i][e];
        mx = fmaxf(mx, x[i][e]);
      }
    }
    mx = max_xor32(mx) * sl2;   // log2 units (max(s) * c == max(s * c) for c > 0)
    if (hh == 0) Mpart[buf * NW * 32 + w * 32 + r] = mx;
    if (has_next) q_store(qb + 1, buf ^ 1, nv);
    LS_MARK(0)
    __syncthreads();   // (A) row maxima, next query block
    LS_MARK(1)
    if (has_next) scores(buf ^ 1, sn);
    float m = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < NW; ++ww) m = fmaxf(m, Mpart[buf * NW * 32 + ww * 32 + r]);
    const float mref = m == -INFINITY ? 0.f : m;
    // row sums as packed trees (v_pk_add_f32, two adds per instruction, no serial chain)
    float ls = 0.f;
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      if (w + NW * i >= nkt) continue;   // wave-uniform
      f32x2 pr[8];
#pragma unroll
      for (int e = 0; e < 16; e += 2) {
        float y0, y1;
        exp_args2(x[i][e], x[i][e + 1], sl2, mref, y0, y1);   // (v_pk_fma_f32)
        x[i][e] = __builtin_amdgcn_exp2f(y0);
        x[i][e + 1] = __builtin_amdgcn_exp2f(y1);
        pr[e >> 1] = f32x2{x[i][e], x[i][e + 1]};
      }
      ls += tree_sum<8>(pr);
    }
    ls = sum_xor32(ls);
    if (hh == 0) Spart[buf * NW * 32 + w * 32 + r] = ls;
    LS_MARK(2)
    __syncthreads();   // (B) row sums
    LS_MARK(3)
    // the loads issued at the top of this block have had phases 1 and 2 (and nothing stored
    // since: vmcnt counts stores too)
    nv = nv2;
    if (DROP && has_next) kw_finish(qb + 1, kraw, kwn);
    float l;
    {
      float sp[NW];   // (scalar tree: packed adds would need the ds_read2 pairs re-registered)
#pragma unroll
      for (int ww = 0; ww < NW; ++ww) sp[ww] = Spart[buf * NW * 32 + ww * 32 + r];
#pragma unroll
      for (int n = NW / 2; n >= 1; n /= 2)
#pragma unroll
        for (int i = 0; i < n; ++i) sp[i] += sp[i + n];
      l = sp[0];
    }
    if (w == NW - 1 && hh == 0 && qvalid) P.lse[bh * Lq + q] = l > 0.f ? (m + __log2f(l)) * (1.f / LF_LOG2E) : -INFINITY;
    // P' / Lq of this lane's query (0 for a query past Lq)
    const float cq = (qvalid && l > 0.f) ? inv_keep * __builtin_amdgcn_rcpf(l * (float)Lq) : 0.f;
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int kt = w + NW * i;
      if (kt >= nkt) continue;
      // the P' tile [q][key], registers 4g .. 4g+3 = keys 8g + 4hh + 0..3
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int e = 4 * g + j;
          v[j] = (__bf16)keep_sel(kw[i], j + 8 * g, x[i][e] * cq);
        }
        *reinterpret_cast<bf16x4*>(Pw + ds_off4(r, 8 * g + 4 * hh)) = v;
      }
      // C[.][key] += sum_q 1 * P'[q][key]
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int q0 = 16 * s + 8 * hh + qp;
        const int key0 = 16 * (g16 & 1) + 4 * pp;
        const bf16x8 pb = cat8(tr_read(Pw, ds_off4(q0, key0)), tr_read(Pw, ds_off4(q0 + 4, key0)));
        cs[i] = mfma_bf16(ones, pb, cs[i]);
      }
    }
    LS_MARK(4)
  }
  LS_STORE(w, NW / 2)
  // pbar: lane = key, every register the same column sum
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int kt = w + NW * i;
    if (kt >= nkt || hh != 0) continue;
    const int key = kt * 32 + r;
    P.pbar[bh * Lk + key] = cs[i][0];
    if (P.pbarT) P.pbarT[((int64_t)b * Lk + key) * A.heads + head] = cs[i][0];
  }
}

}  // namespace

bool attn_long_fused_ok(const AttnPair* pairs, int npairs, int hd, float drop_p) {
  if (getenv("MMF_NO_LONG_FUSED")) return false;
  if (math_mode() != 1 || hd > 64 || hd % 4 != 0 || npairs <= 0) return false;
  for (int i = 0; i < npairs; ++i) {
    const AttnPair& P = pairs[i];
    if (P.Lk <= 128 || P.Lk > LF_MAXK || P.Lk % 32 != 0 || P.Lq < 1 || P.kmask_mode == 2) return false;
    if (P.ldq % 4 != 0 || P.ldk % 4 != 0 || ((uintptr_t)P.q & 15) != 0 || ((uintptr_t)P.k & 15) != 0) return false;
    if (P.qk_bf16 && (hd % 8 != 0 || P.ldq % 8 != 0 || P.ldk % 8 != 0)) return false;
    if (P.dqk_bf16 && !P.qk_bf16) return false;
    if (!P.dq || !P.dk || !P.dsum || !P.dpbar || !P.lse) return false;
    if (drop_p > 0.f && (!P.keep_bits || P.kw_ld < P.Lk / 32)) return false;
  }
  return true;
}

bool attn_long_fwd_ok(const AttnPair* pairs, int npairs, int hd, float drop_p, const RngSnap* rng) {
  if (getenv("MMF_NO_LONG_FUSED")) return false;
  if (math_mode() != 1 || hd > 64 || hd % 4 != 0 || npairs <= 0) return false;
  if (drop_p > 0.f && !rng) return false;
  for (int i = 0; i < npairs; ++i) {
    const AttnPair& P = pairs[i];
    if (P.Lk <= 128 || P.Lk > LF_MAXK || P.Lk % 32 != 0 || P.Lq < 1 || P.kmask_mode == 2) return false;
    if (P.ldq % 4 != 0 || P.ldk % 4 != 0 || ((uintptr_t)P.q & 15) != 0 || ((uintptr_t)P.k & 15) != 0) return false;
    if (P.qk_bf16 && (hd % 8 != 0 || P.ldq % 8 != 0 || P.ldk % 8 != 0)) return false;
    if (!P.lse || !P.pbar) return false;
    if (drop_p > 0.f && (!P.keep_bits || P.kw_ld < P.Lk / 32)) return false;
  }
  return true;
}

hipError_t launch_attn_keep_words(const AttnPair* pairs, int npairs, int B, int heads, float drop_p,
                                  const RngSnap* rng, hipStream_t st) {
  if (!(drop_p > 0.f) || !rng) return hipSuccess;
  std::vector<AttnPair> ps;
  for (int i = 0; i < npairs; ++i)
    if (pairs[i].keep_bits && pairs[i].Lk % 32 == 0 && pairs[i].Lk > 0 && pairs[i].kw_ld >= pairs[i].Lk / 32) {
      if ((int64_t)B * heads * pairs[i].Lq * (pairs[i].Lk / 32) >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
      ps.push_back(pairs[i]);
    }
  for (size_t done = 0; done < ps.size();) {
    AttnArgs a;
    memset(&a, 0, sizeof(a));
    int n = 0;
    int64_t maxw = 0;
    double wb = 0.0;
    while (done < ps.size() && n < ATTN_MAX_PAIRS) {
      a.p[n] = ps[done++];
      const int64_t nw = (int64_t)B * heads * a.p[n].Lq * (a.p[n].Lk / 32);
      maxw = std::max(maxw, nw);
      wb += 4.0 * nw;
      ++n;
    }
    a.npairs = n;
    a.B = B;
    a.heads = heads;
    a.drop_p = drop_p;
    a.rng = rng;
    ProfLaunch prof_(st, "attn_keep_words_kernel", 0.0, wb);
    mmf_launch(attn_keep_words_kernel, dim3((unsigned)((maxw + 255) / 256), (unsigned)n), dim3(256), 0, st, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_attn_long_fused_fwd(const AttnPair* pairs, int npairs, int B, int heads, int hd, float scale,
                                      float drop_p, const RngSnap* rng, hipStream_t st, bool words_ready) {
  if (!attn_long_fwd_ok(pairs, npairs, hd, drop_p, rng)) return hipErrorNotSupported;
  const bool drop = drop_p > 0.f;
  for (int done = 0; done < npairs;) {
    AttnArgs a;
    memset(&a, 0, sizeof(a));
    int n = 0;
    double fl = 0.0, by = 0.0;
    while (done < npairs && n < ATTN_MAX_PAIRS) {
      a.p[n] = pairs[done++];
      const double lq = a.p[n].Lq, lk = a.p[n].Lk, H = (double)heads * hd;
      const double esz = a.p[n].qk_bf16 ? 2.0 : 4.0;   // Q / K as stored (bf16 at "medium", §4.4)
      // S = QK^T and the column-sum contraction (the pooled P'V's share, as PoolFwd)
      fl += 2.0 * B * lq * lk * H;
      // Q, K in; the dropout keep words (B, h, Lq, Lk / 32) read or written; lse, pbar out
      by += esz * (B * lq * H + B * lk * H) + (drop ? 4.0 * B * heads * lq * (lk / 32) : 0.0) +
            4.0 * B * heads * (lq + lk);
      ++n;
    }
    a.npairs = n;
    a.B = B;
    a.heads = heads;
    a.hd = hd;
    a.scale = scale;
    a.drop_p = drop_p;
    a.rng = rng;
    a.nblk = B * heads;
    if (drop && !words_ready) {
      int64_t maxw = 0;
      double wb = 0.0;
      for (int i = 0; i < n; ++i) {
        const int64_t nw = (int64_t)B * heads * a.p[i].Lq * (a.p[i].Lk / 32);
        maxw = std::max(maxw, nw);
        wb += 4.0 * nw;
      }
      ProfLaunch prof_(st, "attn_keep_words_kernel", 0.0, wb);
      mmf_launch(attn_keep_words_kernel, dim3((unsigned)((maxw + 255) / 256), (unsigned)n), dim3(256), 0, st, a);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    const dim3 grid((unsigned)(B * heads), (unsigned)n);
    // 16 waves (one key tile each at Lk = 512); MMF_LONG_FWD_W8=1: the 8-wave form (A/B)
    static const bool w8 = getenv("MMF_LONG_FWD_W8") != nullptr;
    const char* kn = w8 ? (drop ? "attn_poolL_fwd_fused_bf16<true, 8>" : "attn_poolL_fwd_fused_bf16<false, 8>")
                        : (drop ? "attn_poolL_fwd_fused_bf16<true, 16>" : "attn_poolL_fwd_fused_bf16<false, 16>");
    ProfLaunch prof_(st, kn, fl, by);
    if (w8) {
      if (drop) mmf_launch(attn_poolL_fwd_fused_bf16<true, 8>, grid, dim3(8 * 64), 0, st, a);
      else mmf_launch(attn_poolL_fwd_fused_bf16<false, 8>, grid, dim3(8 * 64), 0, st, a);
    } else {
      if (drop) mmf_launch(attn_poolL_fwd_fused_bf16<true, 16>, grid, dim3(16 * 64), 0, st, a);
      else mmf_launch(attn_poolL_fwd_fused_bf16<false, 16>, grid, dim3(16 * 64), 0, st, a);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_attn_long_fused_bwd(const AttnPair* pairs, int npairs, int B, int heads, int hd, float scale,
                                      float drop_p, hipStream_t st) {
  if (!attn_long_fused_ok(pairs, npairs, hd, drop_p)) return hipErrorNotSupported;
  const bool bits = drop_p > 0.f;
  // pairs with Lk == LF_MAXK take the guard-free FULL instantiation, in launches of their own
  for (int full = 1; full >= 0; --full) {
    std::vector<AttnPair> ps;
    for (int i = 0; i < npairs; ++i)
      if ((pairs[i].Lk == LF_MAXK) == (full != 0)) ps.push_back(pairs[i]);
    for (size_t done = 0; done < ps.size();) {
      AttnArgs a;
      memset(&a, 0, sizeof(a));
      int n = 0;
      double fl = 0.0, by = 0.0;
      while (done < ps.size() && n < ATTN_MAX_PAIRS) {
        a.p[n] = ps[done++];
        const double lq = a.p[n].Lq, lk = a.p[n].Lk, H = (double)heads * hd;
        const double esz = a.p[n].qk_bf16 ? 2.0 : 4.0;   // Q / K as stored (bf16 at "medium", §4.4)
        const double gsz = a.p[n].dqk_bf16 ? 2.0 : 4.0;  // dQ / dK as stored
        fl += 2.0 * (2.0 * B * lq * lk * H);          // dQ and dK contractions (S recompute not counted)
        // Q, K in (as stored); dQ, dK out (as stored); the keep words in; lse, dpbar, D sums in (small)
        by += esz * (B * lq * H + B * lk * H) + gsz * (B * lq * H + B * lk * H) +
              (bits ? 4.0 * B * heads * lq * (lk / 32) : 0.0) + 4.0 * B * heads * (2.0 * lq + lk);
        ++n;
      }
      a.npairs = n;
      a.B = B;
      a.heads = heads;
      a.hd = hd;
      a.scale = scale;
      a.drop_p = drop_p;
      a.nblk = B * heads;
      const dim3 grid((unsigned)(B * heads), (unsigned)n);
      static const char* const kName[4] = {"attn_poolL_bwd_fused_bf16<false, false>", "attn_poolL_bwd_fused_bf16<false, true>",
                                           "attn_poolL_bwd_fused_bf16<true, false>", "attn_poolL_bwd_fused_bf16<true, true>"};
      ProfLaunch prof_(st, kName[2 * bits + full], fl, by);
      if (bits && full) mmf_launch((attn_poolL_bwd_fused_bf16<true, true>), grid, dim3(LF_NT), 0, st, a);
      else if (bits) mmf_launch((attn_poolL_bwd_fused_bf16<true, false>), grid, dim3(LF_NT), 0, st, a);
      else if (full) mmf_launch((attn_poolL_bwd_fused_bf16<false, true>), grid, dim3(LF_NT), 0, st, a);
      else mmf_launch((attn_poolL_bwd_fused_bf16<false, false>), grid, dim3(LF_NT), 0, st, a);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

}  // namespace mmf

#ifdef MMF_STAMPS
extern "C" int mmf_long_stamps_read(void* out, size_t bytes) {   // attn_long.hip phase stamps
  if (bytes > sizeof(mmf::g_mmf_stamps)) bytes = sizeof(mmf::g_mmf_stamps);
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mmf::g_mmf_stamps), bytes) == hipSuccess ? 0 : 3;
}
#endif
