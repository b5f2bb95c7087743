// Launch-lean single-key HybridFusion step (every modality 2-D: L = 1).
//
// src/train.py:261-279 feeds HybridFusion the pooled encoder outputs (B, D_m), so every
// CrossModalAttention of the reference attends over ONE key (src/attention.py:92-146): the
// post-dropout probability of (b, head) is [mask_k != 0] keep / (1 - p), independent of Q and K
// (single_key.hip), and the whole forward / backward is a chain of (B x 128) x (128 x 128)
// products: 0.4 GFLOP per C2 step, 2.6 us of fp32 MFMA on the chip.  The general plan runs it as
// ~17 launches of 5-30 us (the GEMM library's fixed cost, per-sample GEMV tails).  Here each
// stage is ONE launch over 16-sample tiles (v_mfma_f32_16x16x4_f32, 16 rows = 16 samples),
// every weight a wave needs loaded into registers at kernel start beside the activations (one
// memory round trip per kernel), the intermediates of a tile kept in LDS between the chained
// products of one launch:
//   l1_pair_fwd   (tile, pair)     X'_k = Drop(X_k mask_k), P_k = Drop(ReLU(X'_k W_k^T + b_k))
//                                  (recomputed by both pairs keyed by k: cheaper than a launch),
//                                  V = P_k W_v^T + b_v, O = P' V, A = O W_o^T + b_o
//                                  (src/fusion.py:364-404, src/attention.py:104-140)
//   l1_head_fwd   (tile)           pooled, gating, adaptive weights, fused, classifier
//                                  (src/fusion.py:406-427, :429-479)
//   l1_head_bwd   (tile)           dz1, dfused = dz1 W1, dscore, cvec = dpooled mask / n
//   l1_pair_bwd   (tile, pair)     dO = cvec_q W_o, dV = P' dO, dP_k|g = dV W_v
//   l1_mod_bwd    (tile, m)        dZ_m = gate(cvec_m + sum_g dP_k|g), dX_m = (dZ_m W_m) mask keep
//   l1_wgrad      (32 x 32 tiles)  every weight / bias gradient as G^T X over the batch
//                                  (K = B split over 4 waves, summed in a fixed order: deterministic)
//                                  + the exactly-zero query / key projection gradients
// Dropout draws are the library's Philox streams (same sites and element indices as the
// general plan: tests/_philox.py replays them for the oracle).
#include <cstdlib>
#include <cstring>

#include "mmf_device.h"

namespace mmf {
namespace {

#ifdef MMF_STAMPS
// Diagnostic build only (make stampsl1): s_memtime at phase boundaries (slots 0..7) and
// s_memrealtime (100 MHz, one clock for the whole chip) at the start / end (slots 8 / 9) of
// thread 0 of every workgroup, per kernel k (0 pair fwd, 1 head fwd, 2 head bwd, 3 key bwd,
// 4 wgrad); read by mmf_l1_stamps_read (scripts/l1_stamps.py).  Never in the product library.
constexpr int L1_STAMP_WG = 1024;
__device__ unsigned long long g_l1_stamps[5][L1_STAMP_WG][10];
// (the counter moves to VGPRs inside the asm: an SGPR result kept live to a store that the
// compiler sinks past later code failed in instruction selection, "illegal VGPR to SGPR copy")
#define L1_TS(k, i, ins)                                                                     \
  {                                                                                        \
    unsigned lo_, hi_;                                                                     \
    __builtin_amdgcn_sched_barrier(0);                                                     \
    asm volatile(ins " s[92:93]\n\ts_waitcnt lgkmcnt(0)\n\tv_mov_b32 %0, s92\n\tv_mov_b32 %1, s93" \
                 : "=v"(lo_), "=v"(hi_)::"s92", "s93", "memory");                          \
    __builtin_amdgcn_sched_barrier(0);                                                     \
    const int sid_ = blockIdx.y * gridDim.x + blockIdx.x;                                  \
    if (threadIdx.x == 0 && sid_ < L1_STAMP_WG)                                            \
      g_l1_stamps[k][sid_][i] = ((unsigned long long)hi_ << 32) | lo_;                     \
  }
#define L1_ST(k, i) L1_TS(k, i, "s_memtime")
#define L1_RT(k, i) L1_TS(k, i, "s_memrealtime")
#else
#define L1_ST(k, i)
#define L1_RT(k, i)
#endif


typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int NT = 256;          // 4 waves
constexpr int S = 16;            // samples per tile (the 16 rows of a 16x16x4 MFMA)
constexpr int KG = L1_MAXD / 16; // 16-deep k groups (K <= 128)
constexpr int NTL = 2;           // 16-column tiles per wave (N <= 128: tiles wave, wave + 4)
constexpr int LD = 128 + 4;      // LDS row stride (floats) of a 16 x 128 activation tile

// v_mfma_f32_16x16x4_f32: lane l supplies A[i = l & 15][k = l >> 4], B[k = l >> 4][j = l & 15];
// the 16x16 result: lane l, reg r holds row 4 (l >> 4) + r, column l & 15.  The contraction runs
// in 16-deep groups with lane quarter kq feeding k = 16 g + 4 kq + s at step s (one float4 per
// lane and group for row-contiguous operands; the same permutation on A and B).
__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// The one-launch step hands P_k and A tiles from the pair workgroups to the last pair workgroup of
// a tile (l1_fwd_loss_kernel) without fences: every handed-off element is stored write-through
// (sc1, an agent-scope relaxed atomic store: the line leaves the producer's XCD L2), every storing
// wave drains its stores (s_waitcnt vmcnt(0)) before the workgroup barrier behind which one lane
// counts the tile's arrivals (agent-scope relaxed add), and every load of those bytes in the
// consumer is a 16-B sc1 buffer load (L1 bypassed, served coherently): MI355X_MICROARCH.md
// "Workgroup dispatch, XCD placement & inter-workgroup visibility", hand-off table row 1.  (An
// agent-scope release + acquire per workgroup instead cost ~13 us per step: scripts/l1_stamps.py.)
typedef __attribute__((address_space(1))) float gfloat;
typedef __attribute__((address_space(1))) unsigned gu32;
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store((gfloat*)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-B sc1 store at byte offset `off` of a (wave-uniform) tensor base of `bytes` bytes
__device__ __forceinline__ void st_wt4(float* base, uint32_t bytes, uint32_t off, float4 v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, bytes, 0x00020000);
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 x = {__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
  __builtin_amdgcn_raw_buffer_store_b128(x, r, off, 0, 16);   // aux 16: sc1
}
// 16-B load at byte offset `off` of a (wave-uniform) tensor base of `bytes` bytes (zeros past it)
__device__ __forceinline__ float4 ld_rb4(const float* base, uint32_t bytes, uint32_t off) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, bytes, 0x00020000);
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
  return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}
// 16-B sc1 load at byte offset `off` of a (wave-uniform) tensor base of `bytes` bytes
__device__ __forceinline__ float4 ld_wt4(const float* base, uint32_t bytes, uint32_t off) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, bytes, 0x00020000);
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16);   // aux 16: sc1
  return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
}

__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load((gfloat*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// (tile, pair) of this workgroup (one place, so a different layout of the grid changes one
// function).  Workgroups are dealt to the 8 XCDs round-robin in dispatch order (x fastest), so with
// the plain (tile, pair) = (blockIdx.x, blockIdx.y) and a tile count that is a multiple of 8 all the
// pair workgroups of one tile sit on ONE XCD (the tile's hand-off stays in that XCD's L2), and every
// XCD fetches every pair's W_k / W_v / W_o into its own L2: 8 copies of ~1.1 MB of weights per
// launch at C2 (profiles/pmc_traffic_c2_l1_highest.json: 18.1 vs 9.25 MB algorithmic).
// MMF_L1_XCD_IDS (`make l1xcd`) deals work item w = (l % 8) (N / 8) + l / 8 to dispatch index l
// instead -- the tiles of one or two pairs on one XCD, so each XCD fetches at most two pairs'
// weights: 13.3 MB instead of 18.1 MB per fused-step launch, but 43.9 / 44.1 us instead of 42.2 /
// 42.0 us (round 5, profiles/r05/l1_xcd_ab/): the hand-offs then cross XCDs.  The plain layout stays.
__device__ __forceinline__ void l1_ids(int& tile, int& pair) {
#ifdef MMF_L1_XCD_IDS
  const unsigned T = gridDim.x, N = gridDim.x * gridDim.y;
  if (gridDim.y > 1 && (N & 7u) == 0) {
    const unsigned l = blockIdx.x + T * blockIdx.y;
    const unsigned w = (l & 7u) * (N >> 3) + (l >> 3);
    pair = (int)(w / T);
    tile = (int)(w - (unsigned)pair * T);
    return;
  }
#endif
  tile = blockIdx.x;
  pair = blockIdx.y;
}
__device__ __forceinline__ int l1_tile() {
  int t, p;
  l1_ids(t, p);
  return t;
}

// The rng state / snapshot of the call, read through the constant address space: nothing in the
// reading launch writes it (the live offset advances in a later launch), so the load is a scalar
// one whose wait does not drain the vector loads issued beside it.
typedef __attribute__((address_space(4))) const uint64_t cu64;
__device__ __forceinline__ RngSnap load_rng(const void* p) {
  cu64* q = (cu64*)p;
  return RngSnap{q[0], q[1]};
}

struct WTile {
  float4 w[NTL][KG];
};


// Weight loads are unconditional (clamped indices, out-of-range values zeroed after the load): a
// guarded load becomes a branch, and the compiler's wait counts cannot see through the branches
// (it then drains every load in flight at the first use of any of them).
__device__ __forceinline__ float4 zero_if(bool z, float4 v) {
  return z ? make_float4(0.f, 0.f, 0.f, 0.f) : v;
}

// y = x W^T with W (N x K) row-major (nn.Linear): B[k][j] = W[n0 + j][k]
__device__ __forceinline__ void wload_nt(const float* __restrict__ W, int N, int K, int wave, int lane, WTile& t) {
  const int r = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int u = 0; u < NTL; ++u) {
    const int n = 16 * (wave + 4 * u) + r;
#pragma unroll
    for (int g = 0; g < KG; ++g) {
      const int k = 16 * g + 4 * kq;
      const float4 v = *reinterpret_cast<const float4*>(W + (int64_t)min(n, N - 1) * K + min(k, K - 4));
      t.w[u][g] = zero_if(n >= N || k >= K, v);
    }
  }
}

// y = x W with W (K x N) row-major: B[k][j] = W[k][n0 + j] (four rows per lane and group)
__device__ __forceinline__ void wload_nn(const float* __restrict__ W, int N, int K, int wave, int lane, WTile& t) {
  const int r = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int u = 0; u < NTL; ++u) {
    const int n = 16 * (wave + 4 * u) + r;
#pragma unroll
    for (int g = 0; g < KG; ++g) {
      const int k = 16 * g + 4 * kq;
      const float* p = W + (int64_t)min(k, K - 4) * N + min(n, N - 1);
      t.w[u][g] = zero_if(n >= N || k >= K, make_float4(p[0], p[N], p[2 * N], p[3 * N]));
    }
  }
}

// acc[u] (this wave's 16-column tiles of a 16 x N product) = xs (16 x 128, LDS, row stride LD) * B:
// every k group and both tiles unconditionally (no branches in the MFMA chain: columns past K
// of xs are zero-padded, weights past K / N zero), so the chain is one straight sequence
__device__ __forceinline__ void mma(const float* xs, const WTile& t, f32x4 (&acc)[NTL], int lane) {
  const int r = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int u = 0; u < NTL; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int g = 0; g < KG; ++g) {
    const float4 a = *reinterpret_cast<const float4*>(xs + r * LD + 16 * g + 4 * kq);
#pragma unroll
    for (int u = 0; u < NTL; ++u) {
      acc[u] = mfma16(a.x, t.w[u][g].x, acc[u]);
      acc[u] = mfma16(a.y, t.w[u][g].y, acc[u]);
      acc[u] = mfma16(a.z, t.w[u][g].z, acc[u]);
      acc[u] = mfma16(a.w, t.w[u][g].w, acc[u]);
    }
  }
}

// 8 keep decisions (bit e: element 8 blk + e kept) of one Philox block
__device__ __forceinline__ uint32_t keep8(const RngSnap& rs, uint32_t site, uint64_t blk, uint32_t thr) {
  const uint4 r = philox_block(rs, site, blk);
  uint32_t bits = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) bits |= keep_from(r, e, thr) ? (1u << e) : 0u;
  return bits;
}

// keep bits of a tile's rows b0 .. b0 + 15 of a (B, N) tensor of site `site` (element (b) N + j,
// a contiguous range: one Philox block per 8 elements), byte c = block (b0 N) / 8 + c
constexpr int KB_BYTES = S * 128 / 8 + 8;
__device__ __forceinline__ void keep_tile(const RngSnap& rs, uint32_t site, int b0, int N, float p, uint8_t* kb) {
  const uint32_t thr = p16(p);
  const uint64_t lo = (uint64_t)b0 * N, hi = (uint64_t)(b0 + S) * N;
  const int nblk = (int)(((hi + 7) >> 3) - (lo >> 3));
  for (int e = threadIdx.x; e < nblk; e += NT) kb[e] = (uint8_t)keep8(rs, site, (lo >> 3) + e, thr);
}

__device__ __forceinline__ bool kept(const uint8_t* kb, int b0, int N, int i, int j) {
  const uint32_t e = (uint32_t)(((uint64_t)(b0 + i) * N + j) - (((uint64_t)b0 * N) & ~7ull));
  return (kb[e >> 3] >> (e & 7)) & 1;
}

// columns [n, 128) of a 16-row LDS tile := 0 (the zero-padded tail of a contraction)
__device__ __forceinline__ void zero_pad(float* tile, int n) {
  const int w = 128 - n;
  for (int e = threadIdx.x; e < S * w; e += NT) tile[(e / w) * LD + n + e % w] = 0.f;
}

// P'[i][h] of pair g: [mask_k != 0] keep(b h) / (1 - p) (src/attention.py:118-130 at one key)
__device__ __forceinline__ void pprime_tile(const L1Args& a, const RngSnap& rs, int g, int b0, float* pp) {
  const int k = a.pk[g];
  for (int e = threadIdx.x; e < S * a.heads; e += NT) {
    const int i = e / a.heads, h = e - i * a.heads, b = b0 + i;
    float v = 0.f;
    if (b < a.B && a.mask[(int64_t)b * a.M + k] != 0.f) {
      v = 1.f;
      if (a.p > 0.f) v = keep1(rs, SITE_ATTN + g, (uint64_t)b * a.heads + h, a.p) ? a.gscale : 0.f;
    }
    pp[e] = v;
  }
}

// 16 x N activation tile rows b0.. of a (B, ld) tensor into LDS (zeros past B); float4 loads from
// clamped rows (unconditional: see wload_nt)
__device__ __forceinline__ void load_tile(const float* __restrict__ src, int ld, int B, int b0, int N, float* dst) {
  // (N <= 128: at most two float4 per thread, both loads issued before either LDS write -- a
  // runtime-trip loop waited for each load in turn)
  const int n4 = N / 4;
  float4 v[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int e = threadIdx.x + u * NT, i = min(e / n4, S - 1), c = e - (e / n4) * n4;
    v[u] = *reinterpret_cast<const float4*>(src + (int64_t)min(b0 + i, B - 1) * ld + 4 * c);
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int e = threadIdx.x + u * NT, i = e / n4, c = e - i * n4;
    if (i < S) *reinterpret_cast<float4*>(dst + i * LD + 4 * c) = b0 + i < B ? v[u] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// sum over the 16 lanes of a lane row (l & ~15 .. +15); every lane of the row gets it
__device__ __forceinline__ float sum16(float v) {
  v += dpp<DPP_ROR8>(v);
  return sum8(v);
}

// out[i][c] = xs[i] . W[c] + bias[c] for i < 16, c < N (16 lanes per dot), rows < B written
template <typename F>
__device__ __forceinline__ void rowdots(const float* xs, const float* W, int ldw, int K, int nout, F&& emit) {
  const int t = threadIdx.x, grp = t >> 4, l16 = t & 15;
  for (int d = grp; d < S * nout; d += NT / 16) {
    const int i = d / nout, c = d - i * nout;
    float s = 0.f;
    for (int k = l16; k < K; k += 16) s += xs[i * LD + k] * W[(int64_t)c * ldw + k];
    s = sum16(s);
    if (l16 == 0) emit(i, c, s);
  }
}

// adaptive weights of one sample (src/fusion.py:462-478; head.hip adaptive_fwd arithmetic).  The
// loops run over the compile-time L1_MAXM with m < M guards, so sm / w stay in registers (with a
// runtime trip count the private arrays went to scratch memory: 4.5 K cycles for three weights in
// the round-4 stamps, scripts/l1_stamps.py); the padding terms add exact zeros.
__device__ __forceinline__ float adaptive(int M, const float* score, const float* mask, float (&sm)[L1_MAXM],
                                          float (&w)[L1_MAXM]) {
  float mx = -INFINITY;
#pragma unroll
  for (int m = 0; m < L1_MAXM; ++m)
    if (m < M && mask[m] > 0.f) mx = fmaxf(mx, score[m]);
  float z = 0.f;
#pragma unroll
  for (int m = 0; m < L1_MAXM; ++m) {
    sm[m] = (m < M && mask[m] > 0.f) ? __expf(score[m] - mx) : 0.f;
    z += sm[m];
  }
  float sw = 0.f, ms = 0.f;
#pragma unroll
  for (int m = 0; m < L1_MAXM; ++m) {
    const float mk = m < M ? mask[m] : 0.f;
    sm[m] = (mx == -INFINITY || m >= M) ? 0.f : sm[m] / z;
    w[m] = sm[m] * mk;
    sw += w[m];
    ms += mk;
  }
  if (sw > 0.f) {
    const float den = sw + 1e-8f;
#pragma unroll
    for (int m = 0; m < L1_MAXM; ++m) w[m] = w[m] / den;
  } else {
#pragma unroll
    for (int m = 0; m < L1_MAXM; ++m) w[m] = m < M ? (ms > 0.f ? mask[m] / (ms + 1e-8f) : 1.f / (float)M) : 0.f;
  }
  return sw;
}

// ------------------------------------------------------------------------------ forward
struct PairLds {
  float xs[S * LD], ps[S * LD], os[S * LD];
  uint8_t kin[KB_BYTES], kpr[KB_BYTES];
  float pp[S * 8];
  float msk[S];
};

// One (tile, pair) of the forward: X'_k, P_k, V, O, A for the 16 samples of the
// workgroup's (tile, pair), l1_ids (stamps: kernel 0)
template <int FH>
__device__ __forceinline__ RngSnap pair_fwd_tile(const L1Args& a, PairLds& L) {
  float* xs = L.xs;
  float* ps = L.ps;
  float* os = L.os;
  uint8_t* kin = L.kin;
  uint8_t* kpr = L.kpr;
  float* pp = L.pp;
  float* msk = L.msk;
  int tile_, g;
  l1_ids(tile_, g);
  const int b0 = tile_ * S;
  const int k = a.pk[g], D = FH ? FH : a.D[k], H = FH ? FH : a.H, B = a.B;
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6) & 3;
  const bool desig = a.kdesig[k] == g;
  // every global operand first, those needed first issued first (the input rows, the mask and the
  // rng state, then the three weights of this wave's columns: the waits before the keep draws and
  // X' leave the weight loads in flight)
  RngSnap rs{0, 0};
  if (a.rng_live) rs = load_rng(a.rng_live);
  const int d4 = D / 4;
  float4 xr[2];
  int xi[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int e = t + u * NT;
    const int i = e / d4;
    xi[u] = (i < S && b0 + i < B) ? e : -1;
    // unconditional loads from clamped rows (a guarded load becomes a branch whose wait the
    // compiler places right behind it, ahead of the weight loads)
    const int row = min(b0 + min(i, S - 1), B - 1);
    xr[u] = *reinterpret_cast<const float4*>(a.x[k] + (int64_t)row * D + 4 * (e - i * d4));
  }
  const float mk = a.mask[(int64_t)min(b0 + (t & (S - 1)), B - 1) * a.M + k];
  const int ih = t / a.heads;
  const float mkh = a.mask[(int64_t)min(b0 + min(ih, S - 1), B - 1) * a.M + k];
  L1_RT(0, 8);
  L1_ST(0, 0);
  __builtin_amdgcn_sched_barrier(0);   // (these loads issue before the weights')
  // (W_v / W_o issue behind the first barrier: 96 workgroups issuing all three weights at once
  // held the keep / P' phase for 13.7 K cycles, 0.0721 -> 0.0700 ms with the split, scripts/gpu_l1ab.sh)
  WTile wk, wv, wo;
  wload_nt(a.Wp[k], H, D, wave, lane, wk);
  float bpk[NTL], bvv[NTL], bov[NTL];
#pragma unroll
  for (int u = 0; u < NTL; ++u) {
    const int j = 16 * (wave + 4 * u) + (lane & 15), jc = min(j, H - 1);
    const bool on = j < H;
    bpk[u] = a.bp[k][jc];
    bvv[u] = a.bv[g][jc];
    bov[u] = a.bo[g][jc];
    if (!on) bpk[u] = bvv[u] = bov[u] = 0.f;
  }
  if (t < S) msk[t] = b0 + t < B ? mk : 0.f;
  if (a.p > 0.f) {
    keep_tile(rs, SITE_IN + k, b0, D, a.p, kin);
    keep_tile(rs, SITE_PROJ + k, b0, H, a.p, kpr);
  }
  // P'[i][h] = [mask_k != 0] keep(b h) / (1 - p) (src/attention.py:118-130 at one key)
  if (t < S * a.heads) {
    float v = 0.f;
    if (b0 + ih < B && mkh != 0.f) {
      v = 1.f;
      if (a.p > 0.f) v = keep1(rs, SITE_ATTN + g, (uint64_t)(b0 + ih) * a.heads + (t - ih * a.heads), a.p) ? a.gscale : 0.f;
    }
    pp[t] = v;
  }
  if (a.snap && tile_ == 0 && g == 0 && t == 0 && a.rng_live) *a.snap = rs;
  __syncthreads();
  L1_ST(0, 1);
  wload_nt(a.Wv[g], H, H, wave, lane, wv);
  wload_nt(a.Wo[g], H, H, wave, lane, wo);
  // X' = X mask (input dropout), src/fusion.py:373
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int e = xi[u] >= 0 ? xi[u] : t + u * NT;
    const int i = e / d4, c = 4 * (e - i * d4);
    if (i >= S) continue;
    if (xi[u] < 0) xr[u] = make_float4(0.f, 0.f, 0.f, 0.f);   // a row past B: zeros
    float v[4] = {xr[u].x, xr[u].y, xr[u].z, xr[u].w};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      v[s] *= msk[i];
      if (a.p > 0.f) v[s] = kept(kin, b0, D, i, c + s) ? v[s] * a.gscale : 0.f;
    }
    const float4 o = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(xs + i * LD + c) = o;
    if (desig && b0 + i < B) *reinterpret_cast<float4*>(a.Xd[k] + (int64_t)(b0 + i) * D + c) = o;
  }
  zero_pad(xs, D);
  if (a.maps[g])
    for (int e = t; e < S * a.heads; e += NT)
      if (b0 + e / a.heads < B) a.maps[g][(int64_t)b0 * a.heads + e] = pp[e];
  __syncthreads();
  L1_ST(0, 2);
  const int kq = lane >> 4, jl = lane & 15;
  f32x4 acc[NTL];
  // P_k = Drop(ReLU(X' W_k^T + b_k))  (projections[k], src/fusion.py:291-298)
  mma(xs, wk, acc, lane);
#pragma unroll
  for (int u = 0; u < NTL; ++u) {
    const int j = 16 * (wave + 4 * u) + jl;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 4 * kq + r;
      float v = fmaxf(acc[u][r] + bpk[u], 0.f);
      if (j >= H) v = 0.f;
      else if (a.p > 0.f) v = kept(kpr, b0, H, i, j) ? v * a.gscale : 0.f;
      ps[i * LD + j] = v;
      if (desig && b0 + i < B && j < H) st_wt(a.P[k] + (int64_t)(b0 + i) * H + j, v);   // (handed off)
    }
  }
  __syncthreads();
  L1_ST(0, 3);
  // V = P_k W_v^T + b_v;  O = P' V per head (one key: attn @ v, src/attention.py:132)
  mma(ps, wv, acc, lane);
  const int hd = H / a.heads;
#pragma unroll
  for (int u = 0; u < NTL; ++u) {
    const int j = 16 * (wave + 4 * u) + jl;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 4 * kq + r;
      const float v = j < H ? (acc[u][r] + bvv[u]) * pp[i * a.heads + j / hd] : 0.f;
      os[i * LD + j] = v;
      if (b0 + i < B && j < H) a.O[g][(int64_t)(b0 + i) * H + j] = v;
    }
  }
  __syncthreads();
  L1_ST(0, 4);
  // A = O W_o^T + b_o  (out_proj, src/attention.py:140)
  mma(os, wo, acc, lane);
#pragma unroll
  for (int u = 0; u < NTL; ++u) {
    const int j = 16 * (wave + 4 * u) + jl;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 4 * kq + r;
      if (b0 + i < B && j < H) st_wt(a.A[g] + (int64_t)(b0 + i) * H + j, acc[u][r] + bov[u]);   // (handed off)
    }
  }
  L1_ST(0, 5);
  L1_RT(0, 9);
  return rs;
}

template <int FH>
__global__ __launch_bounds__(NT) void l1_pair_fwd_kernel(const L1Args a) {
  __shared__ __attribute__((aligned(16))) PairLds L;
  pair_fwd_tile<FH>(a, L);
}

// the small head operands (gating rows, classifier output rows, biases) staged in LDS at kernel
// start beside the activation loads: no global load inside a dot-product loop
struct HeadSmall {
  float gw[L1_MAXM * L1_MAXH];
  float w2[L1_MAXC * L1_MAXH];
  float gb[L1_MAXM], b2[L1_MAXC];
};
__device__ __forceinline__ void stage_small(const L1Args& a, HeadSmall& hs) {
  // every load issued before the first LDS write (unrolled over the compile-time maxima: a loop
  // with a runtime trip count, or a per-lane pointer-table index, waited for each load in turn)
  // (unconditional loads from clamped indices, the guards as selects after them: a guarded load
  // compiles to a branch, and the wait counts do not see through branches; the gating biases by
  // uniform pointers -- a per-lane index into the pointer table is a vector load of the pointer
  // and a wait for every load in flight before the load through it)
  const int t = threadIdx.x, M = a.M, H = a.H, C = a.C;
  float gv[L1_MAXM], wv[(L1_MAXC * L1_MAXH + NT - 1) / NT];
#pragma unroll
  for (int m = 0; m < L1_MAXM; ++m) gv[m] = a.gw[min(m, M - 1)][min(t, H - 1)];
#pragma unroll
  for (int r = 0; r < (L1_MAXC * L1_MAXH + NT - 1) / NT; ++r) wv[r] = a.W2[min(t + r * NT, C * H - 1)];
  float gbv = 0.f;
#pragma unroll
  for (int m = 0; m < L1_MAXM; ++m) {
    const float v = a.gb[min(m, M - 1)][0];
    if (t == m) gbv = v;
  }
  const float b2v = a.b2[min(max(t - 64, 0), C - 1)];
#pragma unroll
  for (int m = 0; m < L1_MAXM; ++m)
    if (m < M && t < H) hs.gw[m * H + t] = gv[m];
#pragma unroll
  for (int r = 0; r < (L1_MAXC * L1_MAXH + NT - 1) / NT; ++r)
    if (t + r * NT < C * H) hs.w2[t + r * NT] = wv[r];
  if (t < M) hs.gb[t] = gbv;
  if (t >= 64 && t < 64 + C) hs.b2[t - 64] = b2v;
}

// LDS of the head phases of one 16-sample tile: the forward, the loss, the backward
struct HeadLds {
  float pl[L1_MAXM * S * LD];     // pooled_m rows (forward output, backward operand)
  float fs[S * LD];               // fused (forward) -> dz1 (backward)
  float hs[S * LD];               // h1 (forward) -> dfused (backward)
  HeadSmall sm;
  uint8_t kcl[KB_BYTES];
  float msk[S * L1_MAXM], sc[S * L1_MAXM];   // mask, gating score rows
  float dl[S * L1_MAXC];                       // dlogits rows (the standalone head backward)
};

// Row group of the head's per-sample phases: the 16 lanes t / 16 == i own sample i of the tile
// (NT / 16 == S groups), lane l16 its float4 columns l16 and l16 + 16 (H <= 128).  A 16-lane sum
// (sum16) leaves a dot product in every lane of the group, so a chain of per-sample steps (scores
// -> adaptive weights -> fused, logits -> loss -> dz1, d weights -> adaptive backward -> cvec)
// runs with no barrier between its steps.
struct RowGroup {
  int i, l16;
  __device__ RowGroup() : i(threadIdx.x >> 4), l16(threadIdx.x & 15) {}
};
static_assert(NT / 16 == S, "one 16-lane group per sample of the tile");

// CrossEntropyLoss(label_smoothing) of sample b (src/train.py:185-186, 310) with the arithmetic of
// head.hip's cross_entropy_kernel, in every lane of its row group: the per-sample loss into
// loss_rows (the batch mean is taken in the wgrad launch, in the standalone kernel's order), dlogits
// = (softmax - target) / B * loss_scale into dl and the caller's buffer (zeros past B)
__device__ __forceinline__ void loss_rows(const L1Args& a, const RowGroup& rg, int b, int y, const float (&z)[L1_MAXC],
                                          float (&dl)[L1_MAXC]) {
  const int C = a.C, B = a.B;
  const float eps = a.ls_eps;
  float mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < L1_MAXC; ++c)
    if (c < C) mx = fmaxf(mx, z[c]);
  float se = 0.f, sz = 0.f, zy = 0.f;
#pragma unroll
  for (int c = 0; c < L1_MAXC; ++c) {
    if (c >= C) break;
    se += __expf(z[c] - mx);
    sz += z[c];
    if (c == y) zy = z[c];
  }
  const float lse = mx + __logf(se);
  // (a label outside [0, C) -- torch raises, ignore_index included: the fused step's mean is over
  // all B rows -- makes the row's loss NaN, so the step's loss reads NaN)
  const bool bad = (unsigned)y >= (unsigned)C;
  if (b < B && rg.l16 == 0)
    st_wt(a.loss_rows + b, bad ? NAN : __builtin_fmaf(1.f - eps, lse - zy, eps * (lse - sz / (float)C)));
#pragma unroll
  for (int c = 0; c < L1_MAXC; ++c) {
    dl[c] = 0.f;
    if (c >= C) continue;
    const float pc = __expf(z[c] - lse);
    const float tgt = (c == y ? (1.f - eps) : 0.f) + eps / (float)C;
    dl[c] = b < B ? (pc - tgt) / (float)B * a.loss_scale : 0.f;
    if (b < B && rg.l16 == c) a.dlogits_out[(int64_t)b * C + c] = dl[c];
  }
}

// dz1 = ReLU' Drop' (dlogits W2) of the row group's sample (its float4 columns; hv: its h1 columns,
// post-dropout, so h1 > 0 marks kept, active units) into L.fs and the saved dz1
template <int FH>
__device__ __forceinline__ void dz1_rows(const L1Args& a, HeadLds& L, const RowGroup& rg, const float4 (&hv)[2],
                                         const float (&dl)[L1_MAXC]) {
  const int H = FH ? FH : a.H, h4 = H / 4, C = a.C, b = l1_tile() * S + rg.i;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int c4 = rg.l16 + 16 * q;
    if (c4 >= h4) continue;
    const float hvv[4] = {hv[q].x, hv[q].y, hv[q].z, hv[q].w};
    // (the classes unrolled over L1_MAXC: one float4 W2 read per class, the same summation order)
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int cc = 0; cc < L1_MAXC; ++cc) {
      if (cc >= C) break;
      const float4 w2 = *reinterpret_cast<const float4*>(L.sm.w2 + cc * H + 4 * c4);
      acc[0] += dl[cc] * w2.x; acc[1] += dl[cc] * w2.y; acc[2] += dl[cc] * w2.z; acc[3] += dl[cc] * w2.w;
    }
    float z[4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) z[s4] = (b < a.B && hvv[s4] > 0.f) ? acc[s4] * a.gscale : 0.f;
    const float4 zv = make_float4(z[0], z[1], z[2], z[3]);
    *reinterpret_cast<float4*>(L.fs + rg.i * LD + 4 * c4) = zv;
    if (b < a.B) *reinterpret_cast<float4*>(a.dz1 + (int64_t)b * H + 4 * c4) = zv;
  }
}


// Head forward of tile l1_tile() (src/fusion.py:406-427, :429-479): pooled, gating scores,
// adaptive weights, fused, h1 = Drop(ReLU(fused W1^T + b1)), logits.  Leaves pooled (pl), the
// mask / score / weight rows, h1 (hs) and the logits (lg) in L.  rs: the call's rng snapshot.
template <int FH, bool LOSS, bool SEQ = false>
__device__ __forceinline__ void head_fwd_tile(const L1Args& a, HeadLds& L, const RngSnap& rs, int kstamp, WTile* w1n) {
  float* pl = L.pl;
  float* fs = L.fs;
  float* hs = L.hs;
  HeadSmall& sm_ = L.sm;
  uint8_t* kcl = L.kcl;
  float *msk = L.msk, *sc = L.sc;
  const int b0 = l1_tile() * S;
  const int M = a.M, H = FH ? FH : a.H, B = a.B, C = a.C;
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6) & 3;
  // loads, first-needed first: the mask rows, the attended and projected rows, the small
  // operands, then W1
  // (the row guard applied where msk is written: a select right after the load became a branch whose
  // other side waited for the load before zeroing its register)
  const float mrow = a.mask[min((int64_t)b0 * M + min(t, S * M - 1), (int64_t)B * M - 1)];   // (S M <= NT)
  int ylab = 0;   // (the loss's label of this lane's row group, loaded with the first operands)
  if constexpr (LOSS) ylab = (int)a.labels[min(b0 + (t >> 4), B - 1)];
  // pooled_m = mean(P_m, A_g for every pair with query m) * mask_m (src/fusion.py:406-408): each
  // thread sums its float4 of every list entry in registers.  Every pooled-source load is issued
  // first, then the small operands' loads and LDS writes (whose waits then cover one round trip for
  // both), then the adds.  Unconditional buffer loads: an absent modality / pair reads a zero-size
  // range, which returns zeros (a guarded load is a branch the wait counts do not see through).
  const int h4 = H / 4;
  float4 pv[2][L1_MAXM], xa[2][L1_MAXP];
  int pe[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int e = t + u * NT, i = e / h4;
    pe[u] = (i < S) ? e : -1;
    const int bb = min(b0 + min(i, S - 1), B - 1), col = 4 * (e - i * h4);
    const uint32_t hb = (uint32_t)B * (uint32_t)H * 4u, ho = (uint32_t)(((int64_t)bb * H + col) * 4);
    if constexpr (SEQ) {
      // mean_L P_m from the projection GEMM's per-128-row column sums, then the pairs' attended
      // means Abar (earlier launches); column-sum rows past the first (L_m > 128) after the adds
#pragma unroll
      for (int m = 0; m < L1_MAXM; ++m) {
        const int nc = m < M ? a.ncol[m] : 0;
        pv[u][m] = ld_rb4(m < M ? a.P[m] : a.mask, (uint32_t)nc * hb, (uint32_t)(((int64_t)bb * nc * H + col) * 4));
      }
#pragma unroll
      for (int g = 0; g < L1_MAXP; ++g) xa[u][g] = ld_rb4(g < a.npairs ? a.A[g] : a.mask, g < a.npairs ? hb : 0u, ho);
    } else {
      // (the P_k / A tiles of the other pair workgroups: sc1 loads, see st_wt)
#pragma unroll
      for (int m = 0; m < L1_MAXM; ++m) pv[u][m] = ld_wt4(m < M ? a.P[m] : a.mask, m < M ? hb : 0u, ho);
#pragma unroll
      for (int g = 0; g < L1_MAXP; ++g) xa[u][g] = ld_wt4(g < a.npairs ? a.A[g] : a.mask, g < a.npairs ? hb : 0u, ho);
    }
  }
  stage_small(a, sm_);
  if (t < S * M) msk[t] = b0 + t / M < B ? mrow : 0.f;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if constexpr (SEQ) {
      const int e = t + u * NT, i = e / h4;
      const int bb = min(b0 + min(i, S - 1), B - 1), col = 4 * (e - i * h4);
#pragma unroll
      for (int m = 0; m < L1_MAXM; ++m) {
        if (m >= M) break;
        const float* pc = a.P[m] + (int64_t)bb * a.ncol[m] * H + col;
        for (int c = 1; c < a.ncol[m]; ++c) {
          const float4 v = *reinterpret_cast<const float4*>(pc + (int64_t)c * H);
          pv[u][m].x += v.x; pv[u][m].y += v.y; pv[u][m].z += v.z; pv[u][m].w += v.w;
        }
        const float il = a.inv_L[m];
        pv[u][m] = make_float4(pv[u][m].x * il, pv[u][m].y * il, pv[u][m].z * il, pv[u][m].w * il);
      }
    }
#pragma unroll
    for (int g = 0; g < L1_MAXP; ++g) {
      const int q = g < a.npairs ? a.pq[g] : -1;   // (a guard, not a break: the loop stays unrolled)
#pragma unroll
      for (int m = 0; m < L1_MAXM; ++m)
        if (m == q) { pv[u][m].x += xa[u][g].x; pv[u][m].y += xa[u][g].y; pv[u][m].z += xa[u][g].z; pv[u][m].w += xa[u][g].w; }
    }
  }
  if (kstamp) {
    L1_RT(1, 8);
    L1_ST(1, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
  WTile w1;
  wload_nt(a.W1, H, H, wave, lane, w1);
  float b1v[NTL];
#pragma unroll
  for (int u = 0; u < NTL; ++u) {
    const int j = 16 * (wave + 4 * u) + (lane & 15);
    b1v[u] = a.b1[min(j, H - 1)];
    if (j >= H) b1v[u] = 0.f;
  }
  if (a.p > 0.f) keep_tile(rs, SITE_CLS, b0, H, a.p, kcl);
  __syncthreads();
  if (kstamp) L1_ST(1, 1);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int e = pe[u];
    if (e < 0) continue;
    const int i = e / h4, c = 4 * (e - i * h4);
    const bool in = b0 + i < B;
#pragma unroll
    for (int m = 0; m < L1_MAXM; ++m) {
      if (m >= M) break;
      const float f = in ? a.inv_cnt[m] * msk[i * M + m] : 0.f;
      const float4 o = make_float4(pv[u][m].x * f, pv[u][m].y * f, pv[u][m].z * f, pv[u][m].w * f);
      *reinterpret_cast<float4*>(pl + (m * S + i) * LD + c) = o;
      if (in) *reinterpret_cast<float4*>(a.pooled + ((int64_t)(b0 + i) * M + m) * H + c) = o;
    }
  }
  __syncthreads();
  if (kstamp) L1_ST(1, 2);
  // gating scores (nn.Linear(H, 1), src/fusion.py:452-461), the adaptive weights (:462-478) and
  // fused = sum_m w_m pooled_m (:413-418) of sample i by the 16 lanes of row group i (RowGroup):
  // the 16-lane sums leave the M scores in every lane of the group, so the three need no barrier
  {
    const RowGroup rg;
    const bool in = b0 + rg.i < B;
    float4 pr[2][L1_MAXM];
    float s[L1_MAXM], mr[L1_MAXM];
#pragma unroll
    for (int m = 0; m < L1_MAXM; ++m) {
      float d = 0.f;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int c4 = rg.l16 + 16 * q;
        pr[q][m] = (m < M && c4 < h4) ? *reinterpret_cast<const float4*>(pl + (m * S + rg.i) * LD + 4 * c4)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 gv = (m < M && c4 < h4) ? *reinterpret_cast<const float4*>(sm_.gw + m * H + 4 * c4)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
        d += pr[q][m].x * gv.x + pr[q][m].y * gv.y + pr[q][m].z * gv.z + pr[q][m].w * gv.w;
      }
      d = sum16(d);
      s[m] = m < M ? d + sm_.gb[m] : 0.f;
      mr[m] = m < M ? msk[rg.i * M + m] : 0.f;
    }
    float smx[L1_MAXM], w[L1_MAXM];
    adaptive(M, s, mr, smx, w);
#pragma unroll
    for (int m = 0; m < L1_MAXM; ++m) {
      if (m < M && rg.l16 == m) {
        sc[rg.i * M + m] = s[m];
        if (in) {
          a.scores[(int64_t)(b0 + rg.i) * M + m] = s[m];
          a.weights[(int64_t)(b0 + rg.i) * M + m] = w[m];
          if (a.weights_out) a.weights_out[(int64_t)(b0 + rg.i) * M + m] = w[m];
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c4 = rg.l16 + 16 * q;
      if (c4 >= h4) continue;
      float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int m = 0; m < L1_MAXM; ++m) {
        if (m >= M) break;
        f.x += pr[q][m].x * w[m]; f.y += pr[q][m].y * w[m]; f.z += pr[q][m].z * w[m]; f.w += pr[q][m].w * w[m];
      }
      *reinterpret_cast<float4*>(fs + rg.i * LD + 4 * c4) = f;
      if (in) *reinterpret_cast<float4*>(a.fused + (int64_t)(b0 + rg.i) * H + 4 * c4) = f;
    }
  }
  zero_pad(fs, H);
  __syncthreads();
  if (kstamp) L1_ST(1, 3);
  // h1 = Drop(ReLU(fused W1^T + b1)) (classifier[0..2], src/fusion.py:323-328)
  f32x4 acc[NTL];
  mma(fs, w1, acc, lane);
  // (the backward's W1 columns, in flight through the loss; issued with the forward's W1 instead,
  // they lengthened the head's load phase 2.2 -> 6.4 K cycles and the loss phase kept its 6.7 K:
  // 0.0684 / 0.0677 vs 0.0659 / 0.0673 ms, profiles/r04/l1/ab_w1n/)
  if constexpr (LOSS) wload_nn(a.W1, H, H, wave, lane, *w1n);
  const int kq = lane >> 4, jl = lane & 15;
#pragma unroll
  for (int u = 0; u < NTL; ++u) {
    const int j = 16 * (wave + 4 * u) + jl;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 4 * kq + r;
      float v = fmaxf(acc[u][r] + b1v[u], 0.f);
      if (j >= H) v = 0.f;
      else if (a.p > 0.f) v = kept(kcl, b0, H, i, j) ? v * a.gscale : 0.f;
      hs[i * LD + j] = v;
      if (b0 + i < B && j < H) a.h1[(int64_t)(b0 + i) * H + j] = v;
    }
  }
  __syncthreads();
  if (kstamp) L1_ST(1, 4);
  // logits = h1 W2^T + b2 (classifier[3]) of sample i by row group i; with LOSS the group goes on
  // with the sample's cross-entropy and dz1 (loss_dz1_rows), no barrier between
  {
    const RowGroup rg;
    const int b = b0 + rg.i;
    int y = 0;
    if constexpr (LOSS) y = b < B ? ylab : 0;
    float4 hv[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c4 = rg.l16 + 16 * q;
      hv[q] = c4 < h4 ? *reinterpret_cast<const float4*>(hs + rg.i * LD + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float z[L1_MAXC];
#pragma unroll
    for (int cc = 0; cc < L1_MAXC; ++cc) {
      if (cc >= C) break;
      float d = 0.f;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int c4 = rg.l16 + 16 * q;
        const float4 w2 = c4 < h4 ? *reinterpret_cast<const float4*>(sm_.w2 + cc * H + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
        d += hv[q].x * w2.x + hv[q].y * w2.y + hv[q].z * w2.z + hv[q].w * w2.w;
      }
      z[cc] = sum16(d) + sm_.b2[cc];
      if (rg.l16 == cc && b < B) a.logits[(int64_t)b * C + cc] = z[cc];
    }
    if constexpr (LOSS) {
      float dlv[L1_MAXC];
      loss_rows(a, rg, b, y, z, dlv);
      dz1_rows<FH>(a, L, rg, hv, dlv);
    }
  }
  if (kstamp) {
    L1_ST(1, 5);
    L1_RT(1, 9);
  }
}

// Head backward of tile l1_tile() from dz1 (L.fs, zero-padded past H; dz1_rows wrote it):
// dfused = dz1 W1, d weights, compute_adaptive_weights backward, cvec_m (the gradient of every
// entry of m's aggregation list).  Reads pl, msk / sc and sm from L (the forward left them there,
// or the standalone kernel staged them); w1n: this wave's W1 columns in y = x W form.
template <int FH>
__device__ __forceinline__ void head_bwd_tile(const L1Args& a, HeadLds& L, const WTile& w1n, int kstamp) {
  float* pl = L.pl;
  float* zs = L.fs;
  float* dfs = L.hs;   // (h1 until dz1_rows has read it)
  HeadSmall& sm_ = L.sm;
  float *msk = L.msk, *sc = L.sc;
  const int b0 = l1_tile() * S;
  const int M = a.M, H = FH ? FH : a.H, B = a.B;
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6) & 3;
  const int h4 = H / 4;
  // dfused = dz1 W1
  f32x4 acc[NTL];
  mma(zs, w1n, acc, lane);
  const int kq = lane >> 4, jl = lane & 15;
#pragma unroll
  for (int u = 0; u < NTL; ++u) {
    const int j = 16 * (wave + 4 * u) + jl;
#pragma unroll
    for (int r = 0; r < 4; ++r) dfs[(4 * kq + r) * LD + j] = acc[u][r];
  }
  __syncthreads();
  if (kstamp) L1_ST(2, 1);
  // d weights_m = dfused . pooled_m, the compute_adaptive_weights backward (renormalisation and the
  // masked softmax) and cvec_m = (w_m dfused + dscore_m gate_w_m) mask_m / n_m of sample i by row
  // group i (the 16-lane sums leave every d weight in every lane of the group: no barrier)
  {
    const RowGroup rg;
    const int b = b0 + rg.i;
    float4 dv[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c4 = rg.l16 + 16 * q;
      dv[q] = c4 < h4 ? *reinterpret_cast<const float4*>(dfs + rg.i * LD + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float dwv[L1_MAXM], mk[L1_MAXM], scv[L1_MAXM];
#pragma unroll
    for (int m = 0; m < L1_MAXM; ++m) {
      float d = 0.f;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int c4 = rg.l16 + 16 * q;
        const float4 pv = (m < M && c4 < h4) ? *reinterpret_cast<const float4*>(pl + (m * S + rg.i) * LD + 4 * c4)
                                             : make_float4(0.f, 0.f, 0.f, 0.f);
        d += dv[q].x * pv.x + dv[q].y * pv.y + dv[q].z * pv.z + dv[q].w * pv.w;
      }
      dwv[m] = m < M ? sum16(d) : 0.f;
      mk[m] = m < M ? msk[rg.i * M + m] : 0.f;
      scv[m] = m < M ? sc[rg.i * M + m] : 0.f;
    }
    float smx[L1_MAXM], w[L1_MAXM], ds[L1_MAXM], dsm[L1_MAXM];
    const float sw = adaptive(M, scv, mk, smx, w);
#pragma unroll
    for (int m = 0; m < L1_MAXM; ++m) ds[m] = 0.f;
    if (sw > 0.f) {
      const float Sd = sw + 1e-8f;
      float dot = 0.f;
#pragma unroll
      for (int m = 0; m < L1_MAXM; ++m)
        if (m < M) dot += dwv[m] * smx[m] * mk[m];
      float sdot = 0.f;
#pragma unroll
      for (int m = 0; m < L1_MAXM; ++m) {
        dsm[m] = (dwv[m] / Sd - dot / (Sd * Sd)) * mk[m];
        if (m < M) sdot += smx[m] * dsm[m];
      }
#pragma unroll
      for (int m = 0; m < L1_MAXM; ++m) ds[m] = mk[m] > 0.f ? smx[m] * (dsm[m] - sdot) : 0.f;
    }
    if (b < B) {
#pragma unroll
      for (int m = 0; m < L1_MAXM; ++m) {
        if (m >= M) break;
        if (rg.l16 == m) a.dscore[(int64_t)b * M + m] = ds[m];
        const float f = mk[m] * a.inv_cnt[m];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int c4 = rg.l16 + 16 * q;
          if (c4 >= h4) continue;
          const float4 gv = *reinterpret_cast<const float4*>(sm_.gw + m * H + 4 * c4);
          const float4 v = make_float4((w[m] * dv[q].x + ds[m] * gv.x) * f, (w[m] * dv[q].y + ds[m] * gv.y) * f,
                                       (w[m] * dv[q].z + ds[m] * gv.z) * f, (w[m] * dv[q].w + ds[m] * gv.w) * f);
          // (sc1: the pair workgroups of the one-launch step read cvec in the same launch)
          st_wt4(a.cvec, (uint32_t)B * (uint32_t)M * (uint32_t)H * 4u, (uint32_t)((((int64_t)b * M + m) * H + 4 * c4) * 4), v);
        }
      }
    }
  }
  if (kstamp) {
    L1_ST(2, 2);
    L1_RT(2, 9);
  }
}

template <int FH>
__global__ __launch_bounds__(NT) void l1_head_fwd_kernel(const L1Args a) {
  __shared__ __attribute__((aligned(16))) HeadLds L;
  RngSnap rs{0, 0};
  if (a.p > 0.f) rs = load_rng(a.snap);
  head_fwd_tile<FH, false>(a, L, rs, 1, nullptr);
  // the live stream advances once per call (the pair kernel read it; the snapshot is saved)
  if (a.rng_advance && blockIdx.x == 0 && threadIdx.x == 0) a.rng_advance[1] += 1;
}

// ------------------------------------------------------------------------------ backward
template <int FH>
__global__ __launch_bounds__(NT) void l1_head_bwd_kernel(const L1Args a) {
  __shared__ __attribute__((aligned(16))) HeadLds L;
  const int b0 = blockIdx.x * S;
  const int M = a.M, H = FH ? FH : a.H, B = a.B, C = a.C;
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6) & 3;
  // what the fused forward leaves in LDS, from the saved tensors
  for (int e = t; e < S * C; e += NT) L.dl[e] = b0 + e / C < B ? a.dlogits[(int64_t)b0 * C + e] : 0.f;
  for (int e = t; e < S * M; e += NT) {
    const bool in = b0 + e / M < B;
    L.msk[e] = in ? a.mask[(int64_t)b0 * M + e] : 0.f;
    L.sc[e] = in ? a.scores[(int64_t)b0 * M + e] : 0.f;
  }
  stage_small(a, L.sm);
  load_tile(a.h1, H, B, b0, H, L.hs);
  const int h4 = H / 4;
  for (int e = t; e < M * S * h4; e += NT) {
    const int mi = e / h4, c = 4 * (e - mi * h4), m = mi / S, i = mi - m * S;
    const float4 v = *reinterpret_cast<const float4*>(a.pooled + ((int64_t)min(b0 + i, B - 1) * M + m) * H + c);
    *reinterpret_cast<float4*>(L.pl + mi * LD + c) = b0 + i < B ? v : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __builtin_amdgcn_sched_barrier(0);
  WTile w1;
  wload_nn(a.W1, H, H, wave, lane, w1);
  __syncthreads();
  // dz1 from the upstream dlogits (the one-launch step forms it beside the loss, the same dz1_rows)
  {
    const RowGroup rg;
    float4 hv[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int c4 = rg.l16 + 16 * q;
      hv[q] = c4 < h4 ? *reinterpret_cast<const float4*>(L.hs + rg.i * LD + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float dlv[L1_MAXC];
#pragma unroll
    for (int cc = 0; cc < L1_MAXC; ++cc) dlv[cc] = cc < C ? L.dl[rg.i * C + cc] : 0.f;
    dz1_rows<FH>(a, L, rg, hv, dlv);
  }
  zero_pad(L.fs, H);
  __syncthreads();
  head_bwd_tile<FH>(a, L, w1, 0);
}

// ---- the sequence tail's head on 16-sample tiles ----
// The pooled plan's head (tail.hip launch_tail_fwd / _bwd) with the phases above: pooled_m from the
// projection GEMM's column sums and the pairs' Abar, then the row-group / MFMA head of the L = 1
// step.  With LOSS (a training step): the cross-entropy, dz1 and the head backward in the same
// launch (the forward's tiles still in LDS), and the batch-mean loss by the last tile to count
// (loss rows stored sc1, drained before the count; cross_entropy_kernel's summation order).
template <int FH, bool LOSS>
__global__ __launch_bounds__(NT) void seq_head_kernel(const L1Args a) {
  __shared__ __attribute__((aligned(16))) HeadLds L;
  RngSnap rs{0, 0};
  if (a.p > 0.f) rs = load_rng(a.snap);
  if constexpr (!LOSS) {
    head_fwd_tile<FH, false, true>(a, L, rs, 0, nullptr);
  } else {
    WTile w1n;
    head_fwd_tile<FH, true, true>(a, L, rs, 0, &w1n);
    zero_pad(L.fs, FH ? FH : a.H);
    __syncthreads();
    head_bwd_tile<FH>(a, L, w1n, 0);
    if (!a.loss_mean) return;
    __shared__ int last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's loss rows (sc1) drained
    __syncthreads();
    const int t = threadIdx.x;
    if (t == 0)
      last = __hip_atomic_fetch_add((gu32*)a.loss_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
             gridDim.x - 1;
    __syncthreads();
    if (!last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (t == 0) __hip_atomic_store((gu32*)a.loss_cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float* red = L.hs;   // (the head is done with its LDS)
    float acc = 0.f;
    for (int i = t; i < a.B; i += NT) acc += ld_wt(a.loss_rows + i);
    red[t] = acc;
    __syncthreads();
    for (int s = NT / 2; s > 0; s >>= 1) {
      if (t < s) red[t] += red[t + s];
      __syncthreads();
    }
    if (t == 0) a.loss_mean[0] = red[0] / (float)a.B;
  }
}

// ---- the key-modality backward inside the one-launch step (round 4) ----
// After a tile's head (the last pair workgroup of the tile) has written cvec (sc1 stores) and set
// the tile's done word, every pair workgroup g = (q, k) of the tile runs its share of what
// l1_key_bwd_kernel does per key modality: dO = cvec_q W_o, dV = P' dO (stored for dW_v), and
// dP_k|g = dV W_v (stored sc1); the last of the pairs keyed by k to count (per (tile, k) arrival
// count) forms dZ_k = gate(cvec_k + sum_g dP_k|g) in pair order (the same sums, bit for bit, as the
// separate launch) and dX_k = (dZ_k W_k) mask_k input-dropout'.  The waiting workgroups poll the
// done word relaxed (one lane, s_sleep between polls, bounded: a timeout sets the error word and
// leaves the tile's outputs unwritten, never a hang); every load of a handed-off byte (cvec, dP,
// P_k) is an sc1 load.  The grid (tiles x pairs <= 16 x 12 at B = 256) is resident at one
// workgroup per CU, so every poll ends.
struct SyncWords {
  gu32 *cnt, *done, *seen, *mcnt, *err;
};
__device__ __forceinline__ SyncWords sync_words(const L1Args& a) {
  const int tiles = (a.B + S - 1) / S;
  gu32* base = (gu32*)a.tile_cnt;
  return SyncWords{base, base + tiles, base + 2 * tiles, base + 3 * tiles, base + (3 + L1_MAXM) * tiles};
}
__device__ __forceinline__ bool poll_eq(gu32* w, unsigned want, unsigned bound) {
  for (unsigned i = 0; i < bound; ++i) {
    if (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == want) return true;
    __builtin_amdgcn_s_sleep(2);
  }
  return false;
}

template <int FH>
__device__ __forceinline__ void pair_key_bwd(const L1Args& a, PairLds& L, const RngSnap& rs, int* flag,
                                             const WTile& wo, const WTile& wv) {
  int tile, g;
  l1_ids(tile, g);
  const int b0 = tile * S;
  const int q = a.pq[g], k = a.pk[g];
  const int H = FH ? FH : a.H, D = FH ? FH : a.D[k], B = a.B, M = a.M;
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6) & 3;
  float* cs = L.xs;
  float* vs = L.ps;
  float* zs = L.os;
  float* pp = L.pp;
  uint8_t* kin = L.kin;
  float* msk = L.msk;
  L1_RT(3, 8);
  L1_ST(3, 0);
  // cvec_q rows of the tile (sc1: the head wrote them in this launch), P' of the pair (W_o / W_v:
  // the caller loaded them, a waiting workgroup before its poll)
  {
    // the mask entry of P' first (an unconditional load: a guarded one waited for every load in
    // flight), the cvec rows, then P' (Philox) while the cvec rows are in flight
    const int ih = min(t / a.heads, S - 1);
    const float mkh = a.mask[(int64_t)min(b0 + ih, B - 1) * M + k];
    const int h4 = H / 4;
    const uint32_t nbytes = (uint32_t)B * (uint32_t)M * (uint32_t)H * 4u;
    float4 v[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = t + u * NT, i = min(e / h4, S - 1), c = e - (e / h4) * h4;
      v[u] = ld_wt4(a.cvec, nbytes, (uint32_t)((((int64_t)min(b0 + i, B - 1) * M + q) * H + 4 * c) * 4));
    }
    // P'[i][h] = [mask_k != 0] keep(b h) / (1 - p) (pprime_tile's arithmetic)
    if (t < S * a.heads) {
      const int hh = t - ih * a.heads;
      float pv = 0.f;
      if (b0 + ih < B && mkh != 0.f) {
        pv = 1.f;
        if (a.p > 0.f) pv = keep1(rs, SITE_ATTN + g, (uint64_t)(b0 + ih) * a.heads + hh, a.p) ? a.gscale : 0.f;
      }
      pp[t] = pv;
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = t + u * NT, i = e / h4, c = e - i * h4;
      if (i < S) *reinterpret_cast<float4*>(cs + i * LD + 4 * c) = b0 + i < B ? v[u] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  zero_pad(cs, H);
  __syncthreads();
  const int kq = lane >> 4, jl = lane & 15, hd = H / a.heads;
  f32x4 acc[NTL];
  mma(cs, wo, acc, lane);
#pragma unroll
  for (int u = 0; u < NTL; ++u) {
    const int j = 16 * (wave + 4 * u) + jl;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ii = 4 * kq + r;
      const float v = j < H ? acc[u][r] * pp[ii * a.heads + j / hd] : 0.f;
      vs[ii * LD + j] = v;
      if (b0 + ii < B && j < H) a.dV[g][(int64_t)(b0 + ii) * H + j] = v;
    }
  }
  __syncthreads();
  mma(vs, wv, acc, lane);
#pragma unroll
  for (int u = 0; u < NTL; ++u) {
    const int j = 16 * (wave + 4 * u) + jl;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ii = 4 * kq + r;
      if (b0 + ii < B && j < H) st_wt(a.dPk[g] + (int64_t)(b0 + ii) * H + j, acc[u][r]);   // (handed off)
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const SyncWords sw = sync_words(a);
  const int npk = a.npairs / M;   // pairs keyed by each modality (every ordered pair present)
  if (t == 0) {
    gu32* mc = sw.mcnt + tile * L1_MAXM + k;
    const bool lastk = __hip_atomic_fetch_add(mc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(npk - 1);
    if (lastk) __hip_atomic_store(mc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = lastk;
  }
  __syncthreads();
  L1_ST(3, 1);
  L1_RT(3, 9);
  if (!*flag) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // the last of k's pairs: dZ_k = ReLU' Drop' (cvec_k + sum_g dP_k|g) (P_k post-dropout: > 0 marks
  // kept, active units; the dP in pair order, as l1_key_bwd_kernel sums them), then dX_k.  dZ in
  // row-major float4 chunks, two per thread: every handed-off operand (cvec, P_k, the dP of k's
  // pairs) one 16-B sc1 load, all issued before the first add (a per-element load loop waited
  // for each load in turn: 11 us of the launch in the round-4 stamps)
  const bool want_dx = a.dx[k] != nullptr;
  WTile wp;
  if (want_dx) wload_nn(a.Wp[k], D, H, wave, lane, wp);
  const float mk_ = a.mask[(int64_t)min(b0 + (t & (S - 1)), B - 1) * M + k];   // (unconditional: see above)
  if (a.p > 0.f && want_dx) keep_tile(rs, SITE_IN + k, b0, D, a.p, kin);
  {
    constexpr int MK = L1_MAXM - 1;   // pairs keyed by one modality (every ordered pair present)
    int kg[MK], nk = 0;
#pragma unroll
    for (int q = 0; q < MK; ++q) kg[q] = -1;
#pragma unroll
    for (int gg = 0; gg < L1_MAXP; ++gg)
      if (gg < a.npairs && a.pk[gg] == k) {
#pragma unroll
        for (int q = 0; q < MK; ++q)
          if (nk == q) kg[q] = gg;
        ++nk;
      }
    const int h4 = H / 4;
    const uint32_t nbh = (uint32_t)B * (uint32_t)H * 4u, nbc = (uint32_t)B * (uint32_t)M * (uint32_t)H * 4u;
    float4 cv[2], pv[2], dv[2][MK];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = t + u * NT, i = e / h4, c = 4 * (e - i * h4);
      const int bb = min(b0 + min(i, S - 1), B - 1);
      const uint32_t off = (uint32_t)(((int64_t)bb * H + c) * 4);
      cv[u] = ld_wt4(a.cvec, nbc, (uint32_t)((((int64_t)bb * M + k) * H + c) * 4));
      pv[u] = ld_wt4(a.P[k], nbh, off);
#pragma unroll
      for (int q = 0; q < MK; ++q)
        dv[u][q] = ld_wt4(kg[q] >= 0 ? a.dPk[kg[q]] : a.cvec, kg[q] >= 0 ? nbh : 0u, off);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = t + u * NT, i = e / h4, c = 4 * (e - i * h4);
      if (i >= S) continue;
      float4 dp = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int q = 0; q < MK; ++q)
        if (q < nk) { dp.x += dv[u][q].x; dp.y += dv[u][q].y; dp.z += dv[u][q].z; dp.w += dv[u][q].w; }
      const bool in = b0 + i < B;
      float4 z;
      z.x = (in && pv[u].x > 0.f) ? (cv[u].x + dp.x) * a.gscale : 0.f;
      z.y = (in && pv[u].y > 0.f) ? (cv[u].y + dp.y) * a.gscale : 0.f;
      z.z = (in && pv[u].z > 0.f) ? (cv[u].z + dp.z) * a.gscale : 0.f;
      z.w = (in && pv[u].w > 0.f) ? (cv[u].w + dp.w) * a.gscale : 0.f;
      *reinterpret_cast<float4*>(zs + i * LD + c) = z;
      if (in) *reinterpret_cast<float4*>(a.dZ[k] + (int64_t)(b0 + i) * H + c) = z;
    }
    zero_pad(zs, H);
  }
  if (t < S) msk[t] = b0 + t < B ? mk_ : 0.f;
  if (!want_dx) return;
  __syncthreads();
  mma(zs, wp, acc, lane);
#pragma unroll
  for (int u = 0; u < NTL; ++u) {
    const int j = 16 * (wave + 4 * u) + jl;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ii = 4 * kq + r;
      if (b0 + ii >= B || j >= D) continue;
      float v = acc[u][r] * msk[ii];
      if (a.p > 0.f) v = kept(kin, b0, D, ii, j) ? v * a.gscale : 0.f;
      a.dx[k][(int64_t)(b0 + ii) * D + j] = v;
    }
  }
  L1_RT(3, 9);   // (the dZ / dX workgroup's end)
}

// The forward, the loss and the head backward of a training step in one launch over (tile,
// pair): every workgroup runs its pair's forward (pair_fwd_tile); the last of a tile's pair
// workgroups to finish (a per-tile arrival count; every workgroup's stores released before it
// counts, the last one's loads acquired after) runs the tile's head forward, the cross-entropy
// and the head backward, with the forward's intermediates still in LDS.  The count returns to 0
// (the caller zeroes it once: mmf_hybrid_train_sync_bytes).  Replaces the pair / head-forward /
// cross-entropy / head-backward launches of the split path (scripts/l1_stamps.py: 7.4 and 9 us
// between them).
template <int FH>
__global__ __launch_bounds__(NT) void l1_fwd_loss_kernel(const L1Args a) {
  // (LDS over 80 KB: one workgroup per CU, the residency the hand-off protocol was measured at)
  __shared__ __attribute__((aligned(16))) union Lds { PairLds p; HeadLds h; char pad[82 * 1024]; } L;
  __shared__ int last, flag;
  int tile, g;
  l1_ids(tile, g);
  const int H = FH ? FH : a.H;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) & 3;
  WTile wo, wv;
  const RngSnap rs = pair_fwd_tile<FH>(a, L.p);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its sc1 stores
  __syncthreads();
  L1_ST(0, 6);
  const SyncWords sw = sync_words(a);
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(sw.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
           (unsigned)(a.npairs - 1);
  __syncthreads();
  L1_ST(0, 7);
  if (last) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // (keeps the sc1 loads behind the count)
    if (threadIdx.x == 0)   // every pair workgroup of this tile has counted: back to 0 for the next call
      __hip_atomic_store(sw.cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    WTile w1n;   // (the backward's W1 columns, loaded behind the forward's h1 product)
    head_fwd_tile<FH, true>(a, L.h, rs, 1, &w1n);   // (through the loss and dz1)
    zero_pad(L.h.fs, FH ? FH : a.H);
    __syncthreads();
    L1_RT(2, 8);
    L1_ST(2, 0);
    head_bwd_tile<FH>(a, L.h, w1n, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // cvec (sc1) drained by every wave
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(sw.done + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    wload_nn(a.Wo[g], H, H, wave, lane, wo);   // (after the done word: not behind the drain)
    wload_nn(a.Wv[g], H, H, wave, lane, wv);
  } else {
    // this pair's backward weights in flight while the head runs
    wload_nn(a.Wo[g], H, H, wave, lane, wo);
    wload_nn(a.Wv[g], H, H, wave, lane, wv);
    if (threadIdx.x == 0) {
      const bool ok = poll_eq(sw.done + tile, 1u, a.poll_bound);
      if (ok) {
        // the last of the tile's waiting workgroups to see the head done returns the words to 0
        if (__hip_atomic_fetch_add(sw.seen + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            (unsigned)(a.npairs - 2)) {
          __hip_atomic_store(sw.seen + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(sw.done + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      } else {
        __hip_atomic_store(sw.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      flag = ok;
    }
    __syncthreads();
    if (!flag) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  __syncthreads();   // (the head's LDS becomes the pair backward's)
  pair_key_bwd<FH>(a, L.p, rs, &flag, wo, wv);
}

// Backward of everything keyed by one modality m, per 16-sample tile (tile, m): for every pair
// g = (q, m) in order, dO = cvec_q W_o (dA = cvec_q), dV = P' dO per head (stored for dW_v),
// dP_m += dV W_v; then dZ_m = ReLU' Drop' (cvec_m + dP_m) (P_m is post-dropout: P_m > 0 marks
// kept, active units) and dX_m = (dZ_m W_m) mask_m input-dropout'.  Every weight of the launch is
// loaded at kernel start; dP_m accumulates in the registers across the pairs.
template <int FH, int NPK>
__global__ __launch_bounds__(NT) void l1_key_bwd_kernel(const L1Args a) {
  __shared__ __attribute__((aligned(16))) float cs[NPK][S * LD];
  __shared__ __attribute__((aligned(16))) float vs[S * LD];
  __shared__ __attribute__((aligned(16))) float zs[S * LD];
  __shared__ float pp[NPK][S * 8];
  __shared__ uint8_t kin[KB_BYTES];
  __shared__ float msk[S];
  const int m = blockIdx.y, b0 = blockIdx.x * S;
  const int H = FH ? FH : a.H, D = FH ? FH : a.D[m], B = a.B, M = a.M;
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6) & 3;
  const bool want_dx = a.dx[m] != nullptr;
  // the pairs keyed by m, in pair order
  int gl[NPK];
  {
    int n = 0;
    for (int g = 0; g < a.npairs; ++g)
      if (a.pk[g] == m && n < NPK) gl[n++] = g;
  }
  RngSnap rs{0, 0};
  if (a.p > 0.f) rs = load_rng(a.snap);
#pragma unroll
  for (int i = 0; i < NPK; ++i) load_tile(a.cvec + (int64_t)a.pq[gl[i]] * H, M * H, B, b0, H, cs[i]);
  if (t < S) msk[t] = b0 + t < B ? a.mask[(int64_t)min(b0 + t, B - 1) * M + m] : 0.f;
  L1_RT(3, 8);
  L1_ST(3, 0);
  __builtin_amdgcn_sched_barrier(0);
  WTile wo[NPK], wv[NPK];
#pragma unroll
  for (int i = 0; i < NPK; ++i) {
    wload_nn(a.Wo[gl[i]], H, H, wave, lane, wo[i]);
    wload_nn(a.Wv[gl[i]], H, H, wave, lane, wv[i]);
  }
#pragma unroll
  for (int i = 0; i < NPK; ++i) {
    pprime_tile(a, rs, gl[i], b0, pp[i]);
    zero_pad(cs[i], H);
  }
  if (a.p > 0.f && want_dx) keep_tile(rs, SITE_IN + m, b0, D, a.p, kin);
  __syncthreads();
  L1_ST(3, 1);
  const int kq = lane >> 4, jl = lane & 15, hd = H / a.heads;
  f32x4 dp[NTL], acc[NTL];
#pragma unroll
  for (int u = 0; u < NTL; ++u) dp[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < NPK; ++i) {
    const int g = gl[i];
    mma(cs[i], wo[i], acc, lane);
#pragma unroll
    for (int u = 0; u < NTL; ++u) {
      const int j = 16 * (wave + 4 * u) + jl;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ii = 4 * kq + r;
        const float v = j < H ? acc[u][r] * pp[i][ii * a.heads + j / hd] : 0.f;
        vs[ii * LD + j] = v;
        if (b0 + ii < B && j < H) a.dV[g][(int64_t)(b0 + ii) * H + j] = v;
      }
    }
    __syncthreads();
    mma(vs, wv[i], acc, lane);
#pragma unroll
    for (int u = 0; u < NTL; ++u) dp[u] += acc[u];
    if (i + 1 < NPK) __syncthreads();   // (vs is rewritten by the next pair)
  }
  L1_ST(3, 2);
  // dZ_m, from the accumulator layout: lane (jl, kq), reg r = row 4 kq + r, column 16 (wave + 4u) + jl
  WTile wp;
  if (want_dx) wload_nn(a.Wp[m], D, H, wave, lane, wp);
#pragma unroll
  for (int u = 0; u < NTL; ++u) {
    const int j = 16 * (wave + 4 * u) + jl;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ii = 4 * kq + r;
      float z = 0.f;
      if (b0 + ii < B && j < H) {
        const int64_t row = (int64_t)(b0 + ii) * H + j;
        const float c = a.cvec[((int64_t)(b0 + ii) * M + m) * H + j];
        z = a.P[m][row] > 0.f ? (c + dp[u][r]) * a.gscale : 0.f;
        a.dZ[m][row] = z;
      }
      zs[ii * LD + j] = z;
    }
  }
  // (launch_l1_train: the live stream advances here, after every forward workgroup has read it)
  if (a.rng_advance && blockIdx.x == 0 && blockIdx.y == 0 && t == 0) a.rng_advance[1] += 1;
  if (!want_dx) return;
  __syncthreads();
  L1_ST(3, 3);
  // dX_m = (dZ_m W_m) mask_m input-dropout'
  mma(zs, wp, acc, lane);
#pragma unroll
  for (int u = 0; u < NTL; ++u) {
    const int j = 16 * (wave + 4 * u) + jl;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int ii = 4 * kq + r;
      if (b0 + ii >= B || j >= D) continue;
      float v = acc[u][r] * msk[ii];
      if (a.p > 0.f) v = kept(kin, b0, D, ii, j) ? v * a.gscale : 0.f;
      a.dx[m][(int64_t)(b0 + ii) * D + j] = v;
    }
  }
  L1_ST(3, 4);
  L1_RT(3, 9);
}

// One 32 x 32 tile of dW = G^T X (rows of G: the batch) per workgroup; wave w takes batch rows
// [w R, (w + 1) R) of each 4R-row chunk, the four partial tiles summed in order through LDS.
// Workgroups past the tiles zero-fill 4096-float chunks of the zero list.
constexpr int WG_ROWS = 64;   // batch rows per wave per chunk (32 MFMA steps)
__global__ __launch_bounds__(NT) void l1_wgrad_kernel(const L1WgArgs w) {
  __shared__ float red[4][16][64];
  __shared__ float bred[4][32];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  int tile = blockIdx.x;
  if ((w.loss || w.clip_partial || w.rng_advance) && tile == gridDim.x - 1) {
    // the extra workgroup: the batch-mean loss in cross_entropy_kernel's order (per-thread strided
    // sums, then a tree); the clip partial slots no tile fills zeroed; the step counter advanced
    // a poll of the forward launch timed out (sync words: the error word after the tile words):
    // the step's outputs are incomplete.  The tile words go back to 0 so the next call starts
    // clean, the loss reads NaN and one clip partial +inf (norm inf, clip coefficient 0: the update
    // applies a zero gradient); the error word stays for the host (mmf_hybrid_train_status)
    const bool failed = w.sync && __hip_atomic_load(w.sync + w.sync_words, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT) != 0u;
    if (failed)
      for (int s = t; s < w.sync_words; s += NT) w.sync[s] = 0u;
    if (w.clip_partial)
      for (int s = w.ntiles + t; s < CLIP_PARTIAL_SLOTS; s += NT)
        w.clip_partial[s] = (failed && s == w.ntiles) ? INFINITY : 0.f;
    if (w.step_incr && t == 0) w.step_incr[0] += 1;
    if (w.rng_advance && t == 0) w.rng_advance[1] += 1;   // (launch_l1_train: every forward workgroup has read it)
    if (!w.loss) return;
    __shared__ float lred[NT];
    float acc = 0.f;
    for (int i = t; i < w.B; i += NT) acc += w.loss_rows[i];
    lred[t] = acc;
    __syncthreads();
    for (int s = NT / 2; s > 0; s >>= 1) {
      if (t < s) lred[t] += lred[t + s];
      __syncthreads();
    }
    if (t == 0) w.loss[0] = failed ? NAN : lred[0] / (float)w.B;
    return;
  }
  if (tile >= w.ntiles) {
    const int zb = tile - w.ntiles;
    int i = 0;   // (unrolled: every offset's scalar load in flight at once, not one per step)
#pragma unroll
    for (int z = 1; z <= L1_MAXZ; ++z)
      if (z <= w.nz && w.zoff[z] <= zb) i = z;
    if (i >= w.nz) return;
    const int64_t lo = (int64_t)(zb - w.zoff[i]) * 4096, hi = min((int64_t)w.zn[i], lo + 4096);
    for (int64_t e = lo + t; e < hi; e += NT) w.z[i][e] = 0.f;
    return;
  }
  // the job of this tile: unrolled over L1_MAXJOBS, every tile0 scalar load in flight at once (a
  // while loop waited for one kernarg load per job: up to 40 round trips before the first load)
  int ji = 0;
#pragma unroll
  for (int i = 1; i < L1_MAXJOBS; ++i)
    if (i < w.njobs && w.j[i].tile0 <= tile) ji = i;
  const L1WgJob J = w.j[ji];
  const int lt = tile - J.tile0, n0 = 32 * (lt / J.tiles_k), k0 = 32 * (lt % J.tiles_k);
  L1_RT(4, 8);
  L1_ST(4, 0);
  const int col = lane & 31, hf = lane >> 5;
  const int n = n0 + col, kk = k0 + col;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float bsum = 0.f;
  for (int c0 = 0; c0 < w.B; c0 += 4 * WG_ROWS) {
    const int rb = c0 + wave * WG_ROWS + hf;
    float ga[WG_ROWS / 2], xb[WG_ROWS / 2];
#pragma unroll
    for (int s = 0; s < WG_ROWS / 2; ++s) {
      const int bc = min(rb + 2 * s, w.B - 1);
      ga[s] = J.G[(int64_t)bc * J.ldg + min(n, J.N - 1)];
      xb[s] = J.X[(int64_t)bc * J.ldx + min(kk, J.K - 1)];
    }
    // (every load above issued before the first select and MFMA: left to itself the scheduler
    // interleaved them two or three at a time with the dependent MFMA chain, one round trip per
    // few steps)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < WG_ROWS / 2; ++s) {
      const bool in = rb + 2 * s < w.B;
      ga[s] = (in && n < J.N) ? ga[s] : 0.f;
      xb[s] = (in && kk < J.K) ? xb[s] : 0.f;
    }
#pragma unroll
    for (int s = 0; s < WG_ROWS / 2; ++s) {
      acc = mfma32(ga[s], xb[s], acc);
      bsum += ga[s];
    }
  }
  L1_ST(4, 1);
#pragma unroll
  for (int r = 0; r < 16; ++r) red[wave][r][lane] = acc[r];
  const bool do_db = J.db && k0 == 0;
  if (do_db) {
    const float v = sum_xor32(bsum);   // both lane halves: column n's sum over this wave's rows
    if (hf == 0) bred[wave][col] = v;
  }
  __syncthreads();
  float sq = 0.f;   // this tile's share of the gradient's squared norm (clip_partial)
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int v = t + u * NT;          // (reg r, lane l) of the 32 x 32 tile
    const int r = v >> 6, l = v & 63;
    const float s = ((red[0][r][l] + red[1][r][l]) + red[2][r][l]) + red[3][r][l];
    const int i = n0 + acc_row(r, l >> 5), j = k0 + (l & 31);
    if (i < J.N && j < J.K) {
      J.dW[(int64_t)i * J.K + j] = s;
      sq += s * s;
    }
  }
  if (do_db && t < 32 && n0 + t < J.N) {
    const float s = ((bred[0][t] + bred[1][t]) + bred[2][t]) + bred[3][t];
    J.db[n0 + t] = s;
    sq += s * s;
  }
  if (w.clip_partial) {   // fixed-order block sum: xor butterfly per wave, then the four waves
    __shared__ float sqr[4];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) sq += __shfl_xor(sq, off);
    if (lane == 0) sqr[wave] = sq;
    __syncthreads();
    if (t == 0) w.clip_partial[tile] = (sqr[0] + sqr[1]) + (sqr[2] + sqr[3]);
  }
  L1_ST(4, 2);
  L1_RT(4, 9);
}

// the C2 shape: every hidden and input width 128 (compile-time tile guards)
// polls of the head's done word before a waiting workgroup gives up: 2^22 (about 0.3 s with the
// s_sleep between polls); MMF_L1_POLL_BOUND overrides it (the timeout test sets 0: every waiter
// times out at once)
unsigned l1_poll_bound() {
  const char* e = getenv("MMF_L1_POLL_BOUND");
  return e ? (unsigned)strtoul(e, nullptr, 0) : (1u << 22);
}

bool l1_full(const L1Args& a) {
  if (a.H != 128) return false;
  for (int m = 0; m < a.M; ++m)
    if (a.D[m] != 128) return false;
  return true;
}

}  // namespace

// workgroups of l1_fwd_loss_kernel the device holds at once: the occupancy the runtime reports
// for the kernel at its block size and LDS, times the compute units (cached per instantiation)
int l1_train_capacity(bool full) {
  static int cap[2] = {-1, -1};
  int& c = cap[full ? 1 : 0];
  if (c < 0) {
    int per_cu = 0;
    hipError_t e = full ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, l1_fwd_loss_kernel<128>, NT, 0)
                        : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, l1_fwd_loss_kernel<0>, NT, 0);
    c = (e == hipSuccess && per_cu > 0) ? per_cu * device_cu_count() : 0;
  }
  return c;
}

hipError_t launch_l1_forward(const L1Args& a, hipStream_t st) {
  if (a.M > L1_MAXM || a.npairs > L1_MAXP || a.H > L1_MAXH || a.H % 4 != 0 || a.C > L1_MAXC || a.heads > 8)
    return hipErrorInvalidValue;
  for (int m = 0; m < a.M; ++m)
    if (a.D[m] > L1_MAXD || a.D[m] % 4 != 0) return hipErrorInvalidValue;
  const unsigned tiles = (unsigned)((a.B + S - 1) / S);
  const double B = a.B, H = a.H;
  {
    double fl = 0.0, by = 0.0;
    for (int g = 0; g < a.npairs; ++g) {
      const double D = a.D[a.pk[g]];
      fl += 2.0 * B * H * (D + 2.0 * H);
      by += 4.0 * (B * (D + 2.0 * H) + H * (D + 2.0 * H));
    }
    ProfLaunch prof_(st, l1_full(a) ? "l1_pair_fwd_kernel<128>" : "l1_pair_fwd_kernel<0>", fl, by);
    if (l1_full(a)) mmf_launch(l1_pair_fwd_kernel<128>, dim3(tiles, a.npairs), dim3(NT), 0, st, a);
    else mmf_launch(l1_pair_fwd_kernel<0>, dim3(tiles, a.npairs), dim3(NT), 0, st, a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  ProfLaunch prof_(st, l1_full(a) ? "l1_head_fwd_kernel<128>" : "l1_head_fwd_kernel<0>", 2.0 * B * H * (H + a.C) + 4.0 * a.M * B * H,
                   4.0 * (B * ((a.M + a.npairs) * H + a.M * H + 2 * H + a.C) + H * (H + a.C)));
  if (l1_full(a)) mmf_launch(l1_head_fwd_kernel<128>, dim3(tiles), dim3(NT), 0, st, a);
  else mmf_launch(l1_head_fwd_kernel<0>, dim3(tiles), dim3(NT), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_l1_backward(const L1Args& a, const L1WgArgs& w, hipStream_t st) {
  if (a.npairs != a.M * (a.M - 1) || a.M < 2) return hipErrorInvalidValue;
  const unsigned tiles = (unsigned)((a.B + S - 1) / S);
  const double B = a.B, H = a.H;
  hipError_t e;
  {
    ProfLaunch prof_(st, l1_full(a) ? "l1_head_bwd_kernel<128>" : "l1_head_bwd_kernel<0>", 2.0 * B * H * (H + a.C) + 4.0 * a.M * B * H,
                     4.0 * (B * (a.C + 2 * H + 2 * a.M * H) + H * (H + a.C)));
    if (l1_full(a)) mmf_launch(l1_head_bwd_kernel<128>, dim3(tiles), dim3(NT), 0, st, a);
    else mmf_launch(l1_head_bwd_kernel<0>, dim3(tiles), dim3(NT), 0, st, a);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  {
    double fl = 0.0, by = 0.0;
    for (int m = 0; m < a.M; ++m) {
      fl += a.dx[m] ? 2.0 * B * H * a.D[m] : 0.0;
      by += 4.0 * (B * H * 2 + (a.dx[m] ? B * a.D[m] + H * a.D[m] : 0.0));
    }
    fl += 4.0 * B * H * H * a.npairs;
    by += 4.0 * a.npairs * (2.0 * B * H + 2.0 * H * H);
    const bool full = l1_full(a);
    const int npk = a.npairs / a.M;
    ProfLaunch prof_(st, full ? "l1_key_bwd_kernel<128>" : "l1_key_bwd_kernel<0>", fl, by);
    const dim3 grid(tiles, a.M);
#define L1_KEY(FH)                                                                     \
    switch (npk) {                                                                     \
      case 1: mmf_launch(l1_key_bwd_kernel<FH, 1>, grid, dim3(NT), 0, st, a); break;   \
      case 2: mmf_launch(l1_key_bwd_kernel<FH, 2>, grid, dim3(NT), 0, st, a); break;   \
      default: mmf_launch(l1_key_bwd_kernel<FH, 3>, grid, dim3(NT), 0, st, a); break;  \
    }
    if (full) { L1_KEY(128) } else { L1_KEY(0) }
#undef L1_KEY
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  double fl = 0.0, by = 0.0;
  for (int i = 0; i < w.njobs; ++i) {
    const L1WgJob& J = w.j[i];
    fl += 2.0 * B * J.N * J.K;
    by += 4.0 * (B * (J.N + J.K) + (double)J.N * J.K);
  }
  int zblocks = w.nz ? w.zoff[w.nz] : 0;
  for (int i = 0; i < w.nz; ++i) by += 4.0 * w.zn[i];
  ProfLaunch prof_(st, "l1_wgrad_kernel", fl, by);
  mmf_launch(l1_wgrad_kernel, dim3((unsigned)(w.ntiles + zblocks)), dim3(NT), 0, st, w);
  return hipGetLastError();
}

hipError_t launch_l1_train(const L1Args& a, const L1WgArgs& w_in, hipStream_t st) {
  if (a.M > L1_MAXM || a.npairs > L1_MAXP || a.H > L1_MAXH || a.H % 4 != 0 || a.C > L1_MAXC || a.heads > 8)
    return hipErrorInvalidValue;
  if (a.npairs != a.M * (a.M - 1) || a.M < 2 || !a.tile_cnt || !a.labels || !a.loss_rows || !a.dlogits_out)
    return hipErrorInvalidValue;
  for (int m = 0; m < a.M; ++m)
    if (a.D[m] > L1_MAXD || a.D[m] % 4 != 0) return hipErrorInvalidValue;
  const unsigned tiles = (unsigned)((a.B + S - 1) / S);
  const bool full = l1_full(a);
  // every workgroup of the one-launch kernel resident at once, by the occupancy the device reports
  // for this kernel (one per CU: its LDS); a grid that does not fit is refused before launch.  The
  // polls are bounded all the same (another stream or process may hold CUs): a timeout is reported
  // through the error word and the weight-gradient launch resets the sync words
  if (tiles * (unsigned)a.npairs > (unsigned)l1_train_capacity(full)) return hipErrorInvalidValue;
  const double B = a.B, H = a.H;
  hipError_t e;
  {
    double fl = 2.0 * B * H * (H + a.C) + 4.0 * a.M * B * H + 2.0 * B * H * (H + a.C);
    double by = 4.0 * (B * ((a.M + a.npairs) * H + a.M * H + 2 * H + a.C) + 2.0 * H * (H + a.C));
    for (int g = 0; g < a.npairs; ++g) {
      const double D = a.D[a.pk[g]];
      fl += 2.0 * B * H * (D + 2.0 * H);
      by += 4.0 * (B * (D + 2.0 * H) + H * (D + 2.0 * H));
    }
    // the key-modality backward (in the same launch)
    for (int m = 0; m < a.M; ++m) {
      fl += a.dx[m] ? 2.0 * B * H * a.D[m] : 0.0;
      by += 4.0 * (B * H * 2 + (a.dx[m] ? B * a.D[m] + H * a.D[m] : 0.0));
    }
    fl += 4.0 * B * H * H * a.npairs;
    by += 4.0 * a.npairs * (2.0 * B * H + 2.0 * H * H);
    L1Args af = a;
    af.rng_advance = nullptr;   // (advanced by the weight-gradient launch)
    af.poll_bound = l1_poll_bound();
    ProfLaunch prof_(st, full ? "l1_fwd_loss_kernel<128>" : "l1_fwd_loss_kernel<0>", fl, by);
    if (full) mmf_launch(l1_fwd_loss_kernel<128>, dim3(tiles, a.npairs), dim3(NT), 0, st, af);
    else mmf_launch(l1_fwd_loss_kernel<0>, dim3(tiles, a.npairs), dim3(NT), 0, st, af);
  }
  if ((e = hipGetLastError()) != hipSuccess) return e;
  L1WgArgs w = w_in;
  w.rng_advance = a.rng_advance;
  w.sync = a.tile_cnt;
  w.sync_words = (int32_t)(tiles * (3 + L1_MAXM));   // (SyncWords: the error word follows them)
  double fl = 0.0, by = 0.0;
  for (int i = 0; i < w.njobs; ++i) {
    const L1WgJob& J = w.j[i];
    fl += 2.0 * B * J.N * J.K;
    by += 4.0 * (B * (J.N + J.K) + (double)J.N * J.K);
  }
  const int zblocks = w.nz ? w.zoff[w.nz] : 0;
  for (int i = 0; i < w.nz; ++i) by += 4.0 * w.zn[i];
  ProfLaunch prof_(st, "l1_wgrad_kernel", fl, by);
  if (w.clip_partial && w.ntiles > CLIP_PARTIAL_SLOTS) return hipErrorInvalidValue;
  const bool extra = w.loss || w.clip_partial || w.rng_advance;
  mmf_launch(l1_wgrad_kernel, dim3((unsigned)(w.ntiles + zblocks + (extra ? 1 : 0))), dim3(NT), 0, st, w);
  return hipGetLastError();
}

bool seq_head_ok(const TailArgs& t) {
  const bool off = getenv("MMF_TAIL_HEAD_GEMV") != nullptr;   // (the per-sample kernels, for A/B)
  if (off || t.H > L1_MAXH || t.H % 4 != 0 || t.M < 1 || t.M > L1_MAXM || t.npairs > L1_MAXP || t.C > L1_MAXC ||
      t.C < 1)
    return false;
  for (int m = 0; m < t.M; ++m)
    if (!t.Pcol[m] || t.ncol[m] < 1) return false;
  return true;
}

static L1Args seq_head_args(const TailArgs& t) {
  L1Args a;
  memset(&a, 0, sizeof(a));
  a.B = t.B; a.M = t.M; a.H = t.H; a.C = t.C; a.heads = t.heads; a.npairs = t.npairs;
  const bool drop = t.drop_p > 0.f && t.rng != nullptr;
  a.p = drop ? t.drop_p : 0.f;
  a.gscale = t.gscale;
  a.snap = const_cast<RngSnap*>(t.rng);
  a.mask = t.mask;
  for (int m = 0; m < t.M; ++m) {
    a.inv_cnt[m] = t.inv_cnt[m];
    a.P[m] = const_cast<float*>(t.Pcol[m]);
    a.ncol[m] = t.ncol[m];
    a.inv_L[m] = 1.f / (float)t.L[m];
    a.gw[m] = t.gate_w[m];
    a.gb[m] = t.gate_b[m];
  }
  for (int g = 0; g < t.npairs; ++g) {
    a.pq[g] = t.p[g].q;
    a.pk[g] = t.p[g].k;
    a.A[g] = const_cast<float*>(t.p[g].Ab);
  }
  a.W1 = t.W1; a.b1 = t.b1; a.W2 = t.W2; a.b2 = t.b2;
  a.pooled = t.pooled; a.scores = t.scores; a.weights = t.weights; a.fused = t.fused; a.h1 = t.h1;
  a.logits = t.logits; a.weights_out = t.weights_out;
  a.dlogits = t.dlogits; a.dz1 = t.dz1; a.cvec = t.cvec; a.dscore = t.dscore;
  a.labels = t.labels; a.ls_eps = t.ls_eps; a.loss_scale = t.loss_scale;
  a.loss_rows = t.loss_rows; a.dlogits_out = t.dlogits_out;
  a.loss_mean = t.loss_mean; a.loss_cnt = t.loss_cnt;
  return a;
}

hipError_t launch_seq_head_fwd(const TailArgs& t, hipStream_t st) {
  if (!seq_head_ok(t)) return hipErrorInvalidValue;
  const L1Args a = seq_head_args(t);
  const bool loss = t.labels != nullptr;
  if (loss && (!t.loss_rows || !t.dlogits_out || !t.dz1 || !t.cvec || !t.dscore || (t.loss_mean && !t.loss_cnt)))
    return hipErrorInvalidValue;
  const unsigned tiles = (unsigned)((t.B + S - 1) / S);
  const double B = t.B, H = t.H, M = t.M, C = t.C;
  double ncs = 0.0;
  for (int m = 0; m < t.M; ++m) ncs += t.ncol[m];
  const bool full = t.H == 128;
  // forward: W1 / W2 once per tile, the column sums, Abar, mask in; pooled, fused, h1, logits,
  // scores / weights out.  With the loss: + dlogits, dz1, dscore, cvec out, W1 again
  double fl = 2.0 * B * H * (H + C) + 4.0 * M * B * H;
  double by = 4.0 * (tiles * (H * H + C * H) + B * (ncs * H + t.npairs * H + M) +
                     B * (M * H + 2 * H + C + 2 * M));
  if (loss) {
    fl += 2.0 * B * H * (H + C) + 4.0 * M * B * H;
    by += 4.0 * (tiles * H * H + B * (2 * C + H + M + M * H));
  }
  const char* nm = loss ? (full ? "seq_head_kernel<128, 1>" : "seq_head_kernel<0, 1>")
                        : (full ? "seq_head_kernel<128, 0>" : "seq_head_kernel<0, 0>");
  ProfLaunch prof_(st, nm, fl, by);
  if (loss) {
    if (full) mmf_launch(seq_head_kernel<128, true>, dim3(tiles), dim3(NT), 0, st, a);
    else mmf_launch(seq_head_kernel<0, true>, dim3(tiles), dim3(NT), 0, st, a);
  } else {
    if (full) mmf_launch(seq_head_kernel<128, false>, dim3(tiles), dim3(NT), 0, st, a);
    else mmf_launch(seq_head_kernel<0, false>, dim3(tiles), dim3(NT), 0, st, a);
  }
  return hipGetLastError();
}

hipError_t launch_seq_head_bwd(const TailArgs& t, hipStream_t st) {
  if (!seq_head_ok(t) || !t.dlogits || !t.dz1 || !t.cvec || !t.dscore) return hipErrorInvalidValue;
  const L1Args a = seq_head_args(t);
  const unsigned tiles = (unsigned)((t.B + S - 1) / S);
  const double B = t.B, H = t.H, M = t.M, C = t.C;
  const bool full = t.H == 128;
  ProfLaunch prof_(st, full ? "l1_head_bwd_kernel<128>" : "l1_head_bwd_kernel<0>",
                   2.0 * B * H * (H + C) + 4.0 * M * B * H,
                   4.0 * (tiles * (H * H + C * H) + B * (C + 2 * M + H + M * H) + B * (H + M + M * H)));
  if (full) mmf_launch(l1_head_bwd_kernel<128>, dim3(tiles), dim3(NT), 0, st, a);
  else mmf_launch(l1_head_bwd_kernel<0>, dim3(tiles), dim3(NT), 0, st, a);
  return hipGetLastError();
}

#ifdef MMF_STAMPS
extern "C" int mmf_l1_stamps_read(void* out, size_t bytes) {   // l1 kernels' phase stamps
  if (bytes > sizeof(mmf::g_l1_stamps)) bytes = sizeof(mmf::g_l1_stamps);
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mmf::g_l1_stamps), bytes) == hipSuccess ? 0 : 3;
}
#endif

}  // namespace mmf

