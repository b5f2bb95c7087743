// Device helpers shared by the libmmfusion kernels (gfx950 / CDNA4).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mmf_internal.h"

namespace mmf {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// v_mfma_f32_32x32x2_f32: lane l supplies A[i=l&31][k=l>>5] and B[k=l>>5][j=l&31];
// the 32x32 result sits in 16 regs: col j = l&31, row i = (r&3) + 8*(r>>2) + 4*(l>>5).
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int acc_row(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

// ---------------------------------------------------------------- Philox4x32-10
__device__ __forceinline__ uint4 philox10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ uint4 philox_block(const RngSnap& s, uint32_t site, uint64_t blk) {
  return philox10(make_uint4((uint32_t)blk, (uint32_t)(blk >> 32), site, (uint32_t)s.offset),
                  (uint32_t)s.seed, (uint32_t)(s.seed >> 32));
}

__device__ __forceinline__ float u01(uint32_t w) { return (float)(w >> 8) * (1.0f / 16777216.0f); }

__device__ __forceinline__ uint32_t pick(const uint4& r, int j) {
  return j == 0 ? r.x : (j == 1 ? r.y : (j == 2 ? r.z : r.w));
}

// keep decision for element idx of tensor `site` (drop with probability p)
__device__ __forceinline__ bool keep1(const RngSnap& s, uint32_t site, uint64_t idx, float p) {
  const uint4 r = philox_block(s, site, idx >> 2);
  return u01(pick(r, (int)(idx & 3))) >= p;
}

// keep decisions for idx .. idx+3 (bit j set => element idx+j kept)
__device__ __forceinline__ uint32_t keep4(const RngSnap& s, uint32_t site, uint64_t idx, float p) {
  const uint64_t b0 = idx >> 2;
  const int o = (int)(idx & 3);
  const uint4 r0 = philox_block(s, site, b0);
  uint32_t bits = 0;
  if (o == 0) {
    bits |= (u01(r0.x) >= p) ? 1u : 0u;
    bits |= (u01(r0.y) >= p) ? 2u : 0u;
    bits |= (u01(r0.z) >= p) ? 4u : 0u;
    bits |= (u01(r0.w) >= p) ? 8u : 0u;
    return bits;
  }
  const uint4 r1 = philox_block(s, site, b0 + 1);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int t = o + j;
    const uint32_t w = t < 4 ? pick(r0, t) : pick(r1, t - 4);
    bits |= (u01(w) >= p) ? (1u << j) : 0u;
  }
  return bits;
}

}  // namespace mmf
