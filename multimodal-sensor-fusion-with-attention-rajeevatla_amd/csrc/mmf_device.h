// Device helpers shared by the libmmfusion kernels (gfx950 / CDNA4).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mmf_internal.h"

namespace mmf {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4v __attribute__((ext_vector_type(4)));   // (a native 4-vector: one b128 LDS store)

// v_mfma_f32_32x32x2_f32: lane l supplies A[i=l&31][k=l>>5] and B[k=l>>5][j=l&31];
// the 32x32 result sits in 16 regs: col j = l&31, row i = (r&3) + 8*(r>>2) + 4*(l>>5).
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int acc_row(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

// ---------------------------------------------------------------- bf16 math mode
// torch.set_float32_matmul_precision("medium") (config/base.yaml:80 via
// src/train.py:53-68,448) lets fp32 matmuls run with bf16 operands and fp32
// accumulation.  Operands stay fp32 in HBM and LDS; a kernel's MFMA issue
// switches from eight v_mfma_f32_32x32x2_f32 k-steps to one
// v_mfma_f32_32x32x16_bf16 over the same 16 products.  Lane half h of the
// fp32 form feeds k-pair element h at step j (j = 0..7); the bf16 form takes
// element j of lane half h as k = 8h + j.  Applied to A and B alike this is a
// permutation of the contraction, so a chain of eight fp32 k-steps into one
// accumulator maps 1:1 onto one bf16 MFMA with a[j], b[j] = step j's operands.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

//
// "high" (PR = 2, torch.set_float32_matmul_precision("high")): torch defines it as fp32
// matmuls on TF32 operands or with "each float32 number as the sum of two bfloat16
// numbers"; gfx950 has no TF32, so the bf16x3 form: x = hi + lo with hi = bf16(x) (round
// to nearest even) and lo = bf16(x - hi) (x - hi is exact in fp32), and
// a.b = lo_a.hi_b + hi_a.lo_b + hi_a.hi_b (the lo.lo term, < 2^-16 relative, dropped),
// smallest terms first, all three into the fp32 accumulator: 3 bf16 MFMAs (96 cycles)
// instead of 8 fp32 ones (512 cycles) per 16 products, ~16 significant bits per operand.
template <int PR>
__device__ __forceinline__ f32x16 mfma_k16(const float (&a)[8], const float (&b)[8], f32x16 c) {
  if constexpr (PR == 2) {
    bf16x8 ah, al, bh, bl;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      ah[j] = (__bf16)a[j];
      bh[j] = (__bf16)b[j];
      al[j] = (__bf16)(a[j] - (float)ah[j]);
      bl[j] = (__bf16)(b[j] - (float)bh[j]);
    }
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, c, 0, 0, 0);
  } else if constexpr (PR == 1) {
    bf16x8 av, bv;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      av[j] = (__bf16)a[j];   // v_cvt_pk_bf16_f32: round to nearest even, NaN kept
      bv[j] = (__bf16)b[j];
    }
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, c, 0, 0, 0);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) c = mfma32(a[j], b[j], c);
    return c;
  }
}

// ---------------------------------------------------------------- cross-lane without LDS
// gfx950 v_permlane{16,32}_swap and DPP moves instead of ds_bpermute (__shfl_xor):
// no LDS round trip, and the DPP move folds into the consuming VALU op.
// permlane16_swap(x, y): x' = [x.r0, y.r0, x.r2, y.r2], y' = [x.r1, y.r1, x.r3, y.r3]
// (rows of 16 lanes); permlane32_swap(x, y): x' = [x.lo, y.lo], y' = [x.hi, y.hi]
// (measured, scripts/micro/lane_micro.cpp).
__device__ __forceinline__ void swap16(float& x, float& y) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(y), false, false);
  x = __uint_as_float(r[0]);
  y = __uint_as_float(r[1]);
}
__device__ __forceinline__ void swap32(float& x, float& y) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(y), false, false);
  x = __uint_as_float(r[0]);
  y = __uint_as_float(r[1]);
}
__device__ __forceinline__ uint32_t swap32u_partner(uint32_t x, bool upper) {   // x of lane ^ 32
  const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return upper ? r[0] : r[1];
}
// max / sum of a value over the lane pair (l, l ^ 32); every lane gets the result
__device__ __forceinline__ float max_xor32(float v) {
  float a = v, b = v;
  swap32(a, b);
  return fmaxf(a, b);
}
__device__ __forceinline__ float sum_xor32(float v) {
  float a = v, b = v;
  swap32(a, b);
  return a + b;
}
__device__ __forceinline__ uint32_t or_xor32(uint32_t v) {
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return r[0] | r[1];
}
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
constexpr int DPP_ROR8 = 0x128, DPP_HALF_MIRROR = 0x141, DPP_XOR2 = 0x4E, DPP_XOR1 = 0xB1;

// all-reduce sums without LDS.  Pairings: lane ^ 16 (permlane16_swap), ^ 8 (row_ror:8),
// the 8-lane mirror (lane ^ 7: disjoint from the pairs before it), ^ 2, ^ 1; every
// lane ends with the same bits.
__device__ __forceinline__ float sum8(float v) {   // over lanes (l & ~7) .. +7
  v += dpp<DPP_XOR1>(v);
  v += dpp<DPP_XOR2>(v);
  return v + dpp<DPP_HALF_MIRROR>(v);
}
__device__ __forceinline__ float sum32(float v) {  // over the lane's half (32 lanes)
  float a = v, b = v;
  swap16(a, b);
  v = a + b;
  v += dpp<DPP_ROR8>(v);
  return sum8(v);
}
__device__ __forceinline__ float sum64(float v) { return sum32(sum_xor32(v)); }

// x where bit `bit` of `word` is set, else +0: one v_bfe_i32 (0 / all ones) and one v_and.
// (Written as asm: from the builtin the compiler forms v_and + v_cmp + v_cndmask, three
// VALU instructions per element.)
__device__ __forceinline__ float keep_sel(uint32_t word, int bit, float x) {
  uint32_t m;
  asm("v_bfe_i32 %0, %1, %2, 1" : "=v"(m) : "v"(word), "i"(bit));
  return __uint_as_float(__float_as_uint(x) & m);
}

// ---------------------------------------------------------------- Philox4x32-10
__device__ __forceinline__ uint4 philox10(uint4 c, uint32_t k0, uint32_t k1) {
  // the key schedule is rebuilt per call (2 SALU per round): hoisted, its 20 words
  // stay live in SGPRs across whole loops and spill in the register-tight kernels
  asm volatile("" : "+s"(k0), "+s"(k1));
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    // one v_mad_u64_u32 per 32x32->64 product (hi and lo together)
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    // three-input XORs as one v_bitop3_b32 each (gfx950): -25% per Philox call, same bits
    c = make_uint4(__builtin_amdgcn_bitop3_b32(hi1, c.y, k0, 0x96), lo1,
                   __builtin_amdgcn_bitop3_b32(hi0, c.w, k1, 0x96), lo0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ uint4 philox_block(const RngSnap& s, uint32_t site, uint64_t blk) {
  return philox10(make_uint4((uint32_t)blk, (uint32_t)(blk >> 32), site, (uint32_t)s.offset),
                  (uint32_t)s.seed, (uint32_t)(s.seed >> 32));
}

// One Philox call = 128 random bits = 8 keep decisions of 16 bits each:
// element idx uses block idx>>3, word (idx>>1)&3, half idx&1, and is kept iff
// u16 * 2^-16 >= p (p is quantised to 2^-16, |error| < 1.6e-5).
__device__ __forceinline__ uint32_t pick(const uint4& r, int j) {
  return j == 0 ? r.x : (j == 1 ? r.y : (j == 2 ? r.z : r.w));
}
__device__ __forceinline__ uint32_t p16(float p) {
  return (uint32_t)ceilf(p * 65536.0f);   // keep iff u16 >= p16
}
__device__ __forceinline__ bool keep_from(const uint4& r, int e, uint32_t thr) {
  const uint32_t w = pick(r, (e >> 1) & 3);
  return ((w >> (16 * (e & 1))) & 0xFFFFu) >= thr;
}

// keep decision for element idx of tensor `site` (drop with probability p)
__device__ __forceinline__ bool keep1(const RngSnap& s, uint32_t site, uint64_t idx, float p) {
  const uint4 r = philox_block(s, site, idx >> 3);
  return keep_from(r, (int)(idx & 7), p16(p));
}

// keep decisions for idx .. idx+3 (bit j set => element idx+j kept)
__device__ __forceinline__ uint32_t keep4(const RngSnap& s, uint32_t site, uint64_t idx, float p) {
  const uint64_t b0 = idx >> 3;
  const int o = (int)(idx & 7);
  const uint32_t thr = p16(p);
  const uint4 r0 = philox_block(s, site, b0);
  uint32_t bits = 0;
  if (o <= 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j) bits |= keep_from(r0, o + j, thr) ? (1u << j) : 0u;
    return bits;
  }
  const uint4 r1 = philox_block(s, site, b0 + 1);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int t = o + j;
    bits |= (t < 8 ? keep_from(r0, t, thr) : keep_from(r1, t - 8, thr)) ? (1u << j) : 0u;
  }
  return bits;
}

// Keep mask for one lane's 16 accumulator registers of a 32-key MFMA tile whose
// first element index is `base` (a row of a (.., Lk) probability tensor): reg r
// holds key 8*(r>>2) + 4*half + (r&3).  The two lane halves split the four
// 8-key Philox blocks (2 calls per lane instead of 4) and swap the decisions
// that belong to the other half with one xor-32 shuffle.  Bit r set => kept.
// Every lane of the wave must call it (it shuffles); `aligned` (base % 8 == 0 in
// every lane, e.g. Lk % 8 == 0) must be wave-uniform.
__device__ __forceinline__ uint32_t keep_tile16(const RngSnap& s, uint32_t site, uint64_t base, float p,
                                                int half, bool active, bool aligned) {
  uint32_t mine = 0, other = 0;
  if (aligned) {
    const uint32_t thr = p16(p);
    if (active) {
#pragma unroll
      for (int gi = 0; gi < 2; ++gi) {
        const int g = 2 * half + gi;
        const uint4 r = philox_block(s, site, (base >> 3) + g);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          mine |= keep_from(r, 4 * half + j, thr) ? (1u << (4 * g + j)) : 0u;
          other |= keep_from(r, 4 * (1 - half) + j, thr) ? (1u << (4 * g + j)) : 0u;
        }
      }
    }
    return mine | swap32u_partner(other, half != 0);
  }
  if (active) {
#pragma unroll
    for (int g = 0; g < 4; ++g) mine |= keep4(s, site, base + 8 * g + 4 * half, p) << (4 * g);
  }
  return mine;
}

#ifdef MMF_STAMPS
// Diagnostic build only (make stamps): s_memtime at phase boundaries, wave 0 of each
// workgroup, into a per-translation-unit buffer (no relocatable device code) that
// the TU's own reader copies out (mmf_stamps_read: attention.hip, mmf_tail_stamps_read:
// tail.hip).  Never in the product library.
namespace {
constexpr int STAMP_WG = 8192;
__device__ unsigned long long g_mmf_stamps[STAMP_WG][10];
}  // namespace
#define MMF_STAMP(i)                                                                       \
  {                                                                                        \
    unsigned long long t_;                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                                     \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");            \
    __builtin_amdgcn_sched_barrier(0);                                                     \
    const int sid_ = blockIdx.y * gridDim.x + blockIdx.x;                                  \
    if ((threadIdx.x & 63) == 0 && (threadIdx.x >> 6) == 0 && sid_ < STAMP_WG) g_mmf_stamps[sid_][i] = t_; \
  }
// s_memrealtime (constant 100 MHz) into slot i: with two s_memtime stamps it gives the
// shader clock the workgroup ran at (MI355X_MICROARCH.md, DVFS item 6)
#define MMF_STAMP_RT(i)                                                                    \
  {                                                                                        \
    unsigned long long t_;                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                                     \
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");        \
    __builtin_amdgcn_sched_barrier(0);                                                     \
    const int sid_ = blockIdx.y * gridDim.x + blockIdx.x;                                  \
    if ((threadIdx.x & 63) == 0 && (threadIdx.x >> 6) == 0 && sid_ < STAMP_WG) g_mmf_stamps[sid_][i] = t_; \
  }
#define MMF_STAMP_ID()                                                                     \
  {                                                                                        \
    const unsigned hw_ = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));             \
    const unsigned xcc_ = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (31 << 11));           \
    const int sid_ = blockIdx.y * gridDim.x + blockIdx.x;                                  \
    if ((threadIdx.x & 63) == 0 && (threadIdx.x >> 6) == 0 && sid_ < STAMP_WG)             \
      g_mmf_stamps[sid_][9] = ((unsigned long long)xcc_ << 32) | hw_;                      \
  }
#else
#define MMF_STAMP(i)
#define MMF_STAMP_RT(i)
#define MMF_STAMP_ID()
#endif

}  // namespace mmf
