// Pooled-output helpers for HybridFusion (see attention.hip, "Pooled-output
// attention").  Per (pair g = q->k, sample b), with P_k the key modality's
// projected features (Lk x H):
//   forward   U_h = pbar_h P_k,  r_h = sum_j pbar_h[j]
//             (then Obar_h = U_h W_v,h^T + r_h b_v,h, an ordinary small GEMM)
//   backward  dpbar_h[j] = P_k[j] . dU_h + dObar_h . b_v,h
//             E_m = c_m/L_m (row broadcast) + sum_{g: key(g)=m} sum_h pbar_{g,h}^T dU_{g,h}
// E_m is the part of dP_m that flows through value_proj (and the direct
// aggregation term); the Q/K parts come from the dZ GEMM that adds E_m.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "mmf_device.h"

namespace mmf {

namespace {

constexpr int NT = 256;
constexpr int MAXH = 8;           // heads supported by the pooled helpers
__global__ __launch_bounds__(NT) void pool_u_kernel(const PoolArgs a) {
  __shared__ float pb[POOL_PB_CAP];
  __shared__ float4 red[NT];
  const PoolPair& P = a.p[blockIdx.y];
  const int b = blockIdx.x, t = threadIdx.x;
  const int H = a.H, heads = a.heads, Lk = P.Lk;
  const float* pbar = P.pbar + (int64_t)b * heads * Lk;
  for (int i = t; i < heads * Lk; i += NT) pb[i] = pbar[i];
  __syncthreads();
  if (t < heads) {
    float s = 0.f;
    for (int j = 0; j < Lk; ++j) s += pb[t * Lk + j];
    P.r[(int64_t)b * heads + t] = s;
  }
  const int H4 = H / 4;
  const int ncol = heads * H4;
  const float* pk = P.pk + (int64_t)b * Lk * H;
  for (int task0 = 0; task0 < ncol; task0 += NT) {
    const int nact = min(NT, ncol - task0);
    const int RG = NT / nact;
    const int task = task0 + t % nact, rg = t / nact;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (rg < RG) {
      const int hh = task / H4, c4 = task % H4;
      float4 acc2 = acc;
      int j = rg;
#pragma unroll 4
      for (; j + RG < Lk; j += 2 * RG) {
        const float4 v = *reinterpret_cast<const float4*>(pk + (int64_t)j * H + 4 * c4);
        const float4 u = *reinterpret_cast<const float4*>(pk + (int64_t)(j + RG) * H + 4 * c4);
        const float w = pb[hh * Lk + j], w2 = pb[hh * Lk + j + RG];
        acc.x += w * v.x; acc.y += w * v.y; acc.z += w * v.z; acc.w += w * v.w;
        acc2.x += w2 * u.x; acc2.y += w2 * u.y; acc2.z += w2 * u.z; acc2.w += w2 * u.w;
      }
      if (j < Lk) {
        const float4 v = *reinterpret_cast<const float4*>(pk + (int64_t)j * H + 4 * c4);
        const float w = pb[hh * Lk + j];
        acc.x += w * v.x; acc.y += w * v.y; acc.z += w * v.z; acc.w += w * v.w;
      }
      acc.x += acc2.x; acc.y += acc2.y; acc.z += acc2.z; acc.w += acc2.w;
    }
    __syncthreads();
    red[t] = acc;
    __syncthreads();
    if (t < nact) {
      float4 s = red[t];
      for (int g = 1; g < RG; ++g) {
        const float4 v = red[g * nact + t];
        s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
      }
      const int task_t = task0 + t;
      const int hh = task_t / H4, c4 = task_t % H4;
      *reinterpret_cast<float4*>(P.u + ((int64_t)b * heads + hh) * H + 4 * c4) = s;
    }
  }
}

__global__ __launch_bounds__(NT) void pool_dpbar_kernel(const PoolArgs a) {
  extern __shared__ __attribute__((aligned(16))) float du_s[];   // heads * H
  __shared__ float dr_s[MAXH];
  const PoolPair& P = a.p[blockIdx.y];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int H = a.H, heads = a.heads, hd = a.hd, Lk = P.Lk;
  const float* du = P.du + (int64_t)b * heads * H;
  for (int i = t; i < heads * H; i += NT) du_s[i] = du[i];
  // dr_h = dObar_h . b_v,h  (d/d r_h of r_h * b_v,h)
  for (int hh = wave; hh < heads; hh += 4) {
    float s = 0.f;
    for (int d = lane; d < hd; d += 64) s += P.dob[(int64_t)b * H + hh * hd + d] * P.bv[hh * hd + d];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
    if (lane == 0) dr_s[hh] = s;
  }
  __syncthreads();
  const float* pk = P.pk + (int64_t)b * Lk * H;
  const int half = lane >> 5, l32 = lane & 31;
#pragma unroll 2
  for (int j0 = 2 * wave; j0 < Lk; j0 += 8) {
    const int j = j0 + half;
    float acc[MAXH];
#pragma unroll
    for (int hh = 0; hh < MAXH; ++hh) acc[hh] = 0.f;
    if (j < Lk) {
      for (int c4 = l32; c4 < H / 4; c4 += 32) {
        const float4 v = *reinterpret_cast<const float4*>(pk + (int64_t)j * H + 4 * c4);
#pragma unroll
        for (int hh = 0; hh < MAXH; ++hh) {
          if (hh < heads) {
            const float4 u = *reinterpret_cast<const float4*>(&du_s[hh * H + 4 * c4]);
            acc[hh] += v.x * u.x + v.y * u.y + v.z * u.z + v.w * u.w;
          }
        }
      }
    }
#pragma unroll
    for (int hh = 0; hh < MAXH; ++hh) {
      if (hh < heads) {
        float s = acc[hh];
#pragma unroll
        for (int o = 16; o >= 1; o >>= 1) s += __shfl_xor(s, o);
        if (l32 == 0 && j < Lk) P.dpbar[((int64_t)b * heads + hh) * Lk + j] = s + dr_s[hh];
      }
    }
  }
}

struct PoolEArgs {
  PoolEMod m[8];
  int32_t B, heads, H;
  int32_t blocks_per_b[8];
};

__global__ __launch_bounds__(NT) void pool_e_kernel(const PoolEArgs a) {
  const PoolEMod& E = a.m[blockIdx.y];
  const int H = a.H, H4 = H / 4, heads = a.heads, L = E.L;
  const int bpb = a.blocks_per_b[blockIdx.y];
  const int b = blockIdx.x / bpb;
  if (b >= a.B) return;
  const int64_t e = (int64_t)(blockIdx.x % bpb) * NT + threadIdx.x;   // (j, c4) inside sample b
  if (e >= (int64_t)L * H4) return;
  const int j = (int)(e / H4), c4 = (int)(e % H4);
  const float4 cv = *reinterpret_cast<const float4*>(E.c + (int64_t)b * E.ldc + 4 * c4);
  float4 acc = make_float4(cv.x * E.cscale, cv.y * E.cscale, cv.z * E.cscale, cv.w * E.cscale);
#pragma unroll 2
  for (int s = 0; s < E.nsrc; ++s) {
    const float* pb = E.pbar[s] + (int64_t)b * heads * L;
    const float* du = E.du[s] + (int64_t)b * heads * H;
#pragma unroll 4
    for (int hh = 0; hh < heads; ++hh) {
      const float w = pb[hh * L + j];
      const float4 u = *reinterpret_cast<const float4*>(du + hh * H + 4 * c4);
      acc.x += w * u.x; acc.y += w * u.y; acc.z += w * u.z; acc.w += w * u.w;
    }
  }
  *reinterpret_cast<float4*>(E.out + ((int64_t)b * L + j) * H + 4 * c4) = acc;
}

// Key-modality groups: every pair whose key modality is m reads the same P_m[b]; one
// workgroup per (sample, group) reads it once for all of them (a 5-pair group at C5 reads
// 1/5 of the bytes the per-pair kernels do).  R = pairs x heads rows (<= POOL_GRP_ROWS).
constexpr int POOL_GRP_MAX = 32;      // pairs per launch
constexpr int POOL_GRP_ROWS = 32;     // (pair, head) rows per group
struct PoolGrpArgs {
  PoolPair p[POOL_GRP_MAX];
  int32_t gbeg[POOL_GRP_MAX], gcnt[POOL_GRP_MAX];
  int32_t ngroups, B, heads, hd, H;
};

// U_row = pbar_row P_k[b] and r_row = sum_j pbar_row[j] for the group's rows: thread
// (c4 = t & 63, row group t >> 6) accumulates 4 columns of up to 8 rows over the keys
__global__ __launch_bounds__(NT) void pool_u_grp_kernel(const PoolGrpArgs a) {
  extern __shared__ __attribute__((aligned(16))) float pbg[];   // [R][Lk]
  const int b = blockIdx.x, gi = blockIdx.y, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int beg = a.gbeg[gi], heads = a.heads, H = a.H, H4 = H / 4;
  const int R = a.gcnt[gi] * heads, Lk = a.p[beg].Lk;
  for (int i = t; i < R * Lk; i += NT) {
    const int row = i / Lk, j = i - row * Lk;
    const PoolPair& P = a.p[beg + row / heads];
    pbg[i] = P.pbar[((int64_t)b * heads + row % heads) * Lk + j];
  }
  __syncthreads();
  for (int row = wave; row < R; row += NT / 64) {
    float s = 0.f;
    for (int j = lane; j < Lk; j += 64) s += pbg[row * Lk + j];
    s = sum64(s);
    if (lane == 0) a.p[beg + row / heads].r[(int64_t)b * heads + row % heads] = s;
  }
  const int c4 = lane, rg = wave;
  if (c4 >= H4) return;
  float4 acc[POOL_GRP_ROWS / 4];
#pragma unroll
  for (int i = 0; i < POOL_GRP_ROWS / 4; ++i) acc[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  const float* pk = a.p[beg].pk + (int64_t)b * Lk * H + 4 * c4;
  int j = 0;
  for (; j + 2 <= Lk; j += 2) {
    const float4 v0 = *reinterpret_cast<const float4*>(pk + (int64_t)j * H);
    const float4 v1 = *reinterpret_cast<const float4*>(pk + (int64_t)(j + 1) * H);
#pragma unroll
    for (int i = 0; i < POOL_GRP_ROWS / 4; ++i) {
      const int row = rg + 4 * i;
      if (row < R) {
        const float w0 = pbg[row * Lk + j], w1 = pbg[row * Lk + j + 1];
        acc[i].x += w0 * v0.x + w1 * v1.x; acc[i].y += w0 * v0.y + w1 * v1.y;
        acc[i].z += w0 * v0.z + w1 * v1.z; acc[i].w += w0 * v0.w + w1 * v1.w;
      }
    }
  }
  if (j < Lk) {
    const float4 v0 = *reinterpret_cast<const float4*>(pk + (int64_t)j * H);
#pragma unroll
    for (int i = 0; i < POOL_GRP_ROWS / 4; ++i) {
      const int row = rg + 4 * i;
      if (row < R) {
        const float w0 = pbg[row * Lk + j];
        acc[i].x += w0 * v0.x; acc[i].y += w0 * v0.y; acc[i].z += w0 * v0.z; acc[i].w += w0 * v0.w;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < POOL_GRP_ROWS / 4; ++i) {
    const int row = rg + 4 * i;
    if (row < R)
      *reinterpret_cast<float4*>(a.p[beg + row / heads].u + ((int64_t)b * heads + row % heads) * H + 4 * c4) = acc[i];
  }
}

// dpbar_row[j] = P_k[b][j] . dU_row + dObar_row . b_v,row: half a wave per key, lanes over the
// columns, every row's dot summed over the 32 lanes (permlane / DPP)
__global__ __launch_bounds__(NT) void pool_dpbar_grp_kernel(const PoolGrpArgs a) {
  extern __shared__ __attribute__((aligned(16))) float dug[];   // [R][H]
  __shared__ float dr_s[POOL_GRP_ROWS];
  const int b = blockIdx.x, gi = blockIdx.y, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int beg = a.gbeg[gi], heads = a.heads, H = a.H, hd = a.hd, H4 = H / 4;
  const int R = a.gcnt[gi] * heads, Lk = a.p[beg].Lk;
  for (int i = t; i < R * H; i += NT) {
    const int row = i / H, c = i - row * H;
    dug[i] = a.p[beg + row / heads].du[((int64_t)b * heads + row % heads) * H + c];
  }
  for (int row = wave; row < R; row += NT / 64) {
    const PoolPair& P = a.p[beg + row / heads];
    const int hh = row % heads;
    float s = 0.f;
    for (int d = lane; d < hd; d += 64) s += P.dob[(int64_t)b * H + hh * hd + d] * P.bv[hh * hd + d];
    s = sum64(s);
    if (lane == 0) dr_s[row] = s;
  }
  __syncthreads();
  const float* pk = a.p[beg].pk + (int64_t)b * Lk * H;
  const int half = lane >> 5, l32 = lane & 31;
  for (int j0 = 2 * wave; j0 < Lk; j0 += 2 * (NT / 64)) {
    const int j = j0 + half;   // both halves step together (sum32 needs the whole wave)
    float acc[POOL_GRP_ROWS];
#pragma unroll
    for (int row = 0; row < POOL_GRP_ROWS; ++row) acc[row] = 0.f;
    if (j < Lk) {
      for (int c4 = l32; c4 < H4; c4 += 32) {
        const float4 v = *reinterpret_cast<const float4*>(pk + (int64_t)j * H + 4 * c4);
#pragma unroll
        for (int row = 0; row < POOL_GRP_ROWS; ++row) {
          if (row < R) {
            // (indexed as float4: with a float pointer and a runtime H the compiler could not prove
            // 16-B alignment and split the read into ds_read2_b32 pairs, 4-way bank conflicts:
            // SQ conflict ratio 9.2 in round 3)
            const float4 u = reinterpret_cast<const float4*>(dug)[row * H4 + c4];
            acc[row] += v.x * u.x + v.y * u.y + v.z * u.z + v.w * u.w;
          }
        }
      }
    }
#pragma unroll
    for (int row = 0; row < POOL_GRP_ROWS; ++row) {
      if (row < R) {
        const float s = sum32(acc[row]);
        if (l32 == 0 && j < Lk)
          a.p[beg + row / heads].dpbar[((int64_t)b * heads + row % heads) * Lk + j] = s + dr_s[row];
      }
    }
  }
}

// ---- the grouped pools on the fp32 matrix cores (round 5) ----
// Both are small-side GEMMs per (sample, group): U = pbar P_k (M = R <= 32 rows, N = H, K = Lk) and
// dpbar^T = P_k dU^T (M = Lk, N = R, K = H).  The VALU forms above spent their time on the dot
// products and, for dpbar, on a 32-lane reduction per (row, key): 0.37 / 0.25 ms per C5 step for
// 0.40 GB of P_k each.  32x32x2 f32 MFMAs, fp32 products and sums as before (other order).  The
// P_k operand streams from HBM as float4 per lane (each element is used once per workgroup) by
// permuting the MFMA's K or N index: dpbar -- lane half h takes columns c0 + 4h .. +3 and MFMA i
// of a quad contracts column c0 + 4h + i on both operands; U -- lane n' holds columns 4n' .. 4n'+3
// of a key row and MFMA i produces the interleaved column tile {4n' + i}.
constexpr int POOL_MFMA_HMAX = 256;
__device__ __forceinline__ f32x16 mfma_f32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// dpbar_row[j] = P_k[b][j] . dU_row + dObar_row . b_v,row; wave w takes key tiles w, w + 4, ...
__global__ __launch_bounds__(NT) void pool_dpbar_mfma_kernel(const PoolGrpArgs a) {
  constexpr int LDU = POOL_MFMA_HMAX + 4;   // (+4 floats: the 32 rows' float4 reads spread over the banks)
  __shared__ __attribute__((aligned(16))) float dus[POOL_GRP_ROWS * LDU];   // dU, rows >= R zero
  __shared__ float dr_s[POOL_GRP_ROWS];
  const int b = blockIdx.x, gi = blockIdx.y, t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int beg = a.gbeg[gi], heads = a.heads, H = a.H, hd = a.hd;
  const int R = a.gcnt[gi] * heads, Lk = a.p[beg].Lk;
  for (int i = t; i < POOL_GRP_ROWS * H; i += NT) {
    const int row = i / H, c = i - row * H;
    dus[row * LDU + c] = row < R ? a.p[beg + row / heads].du[((int64_t)b * heads + row % heads) * H + c] : 0.f;
  }
  for (int row = w; row < R; row += NT / 64) {
    const PoolPair& P = a.p[beg + row / heads];
    const int hh = row % heads;
    float s = 0.f;
    for (int d = lane; d < hd; d += 64) s += P.dob[(int64_t)b * H + hh * hd + d] * P.bv[hh * hd + d];
    s = sum64(s);
    if (lane == 0) dr_s[row] = s;
  }
  __syncthreads();
  const int n = lane & 31, h = lane >> 5;
  const float* pk = a.p[beg].pk + (int64_t)b * Lk * H;
  const float* du_row = dus + n * LDU + 4 * h;
  for (int jt = w; jt < Lk / 32; jt += NT / 64) {
    const float* arow = pk + (int64_t)(jt * 32 + n) * H + 4 * h;
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    // the row's float4s in chunks of 8 (32 registers), the next chunk issued before this one's MFMAs
    float4 av[2][8];
#pragma unroll
    for (int k = 0; k < 8; ++k) av[0][k] = k * 8 < H ? *reinterpret_cast<const float4*>(arow + 8 * k) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int ch = 0; ch < POOL_MFMA_HMAX / 64; ++ch) {
      const int cur = ch & 1;
      if (ch + 1 < POOL_MFMA_HMAX / 64 && (ch + 1) * 64 < H) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int c0 = (ch + 1) * 64 + 8 * k;
          av[cur ^ 1][k] = c0 < H ? *reinterpret_cast<const float4*>(arow + c0) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
      if (ch * 64 >= H) break;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c0 = ch * 64 + 8 * k;
        if (c0 >= H) break;
        const float4 bv = *reinterpret_cast<const float4*>(du_row + c0);
        const float4 x = av[cur][k];
        acc = mfma_f32(x.x, bv.x, acc);
        acc = mfma_f32(x.y, bv.y, acc);
        acc = mfma_f32(x.z, bv.z, acc);
        acc = mfma_f32(x.w, bv.w, acc);
      }
    }
    // C[j][r]: lane (r = n) holds keys jt * 32 + 8 g + 4 h + 0..3 in registers 4 g .. 4 g + 3
    if (n < R) {
      float* dst = a.p[beg + n / heads].dpbar + ((int64_t)b * heads + n % heads) * Lk + jt * 32 + 4 * h;
      const float dr = dr_s[n];
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(dst + 8 * g) =
            make_float4(acc[4 * g] + dr, acc[4 * g + 1] + dr, acc[4 * g + 2] + dr, acc[4 * g + 3] + dr);
    }
  }
}

// U_row = pbar_row P_k[b] and r_row = sum_j pbar_row[j].  Waves (cb, kh): column block cb of 128
// (lane n' holds columns 4n' .. 4n'+3, MFMA i the interleaved tile {4n' + i}) over key half kh;
// the two key halves of a column block are summed through LDS (fixed order).  pbar rows at a
// stride of Lk + 2 floats (the A reads -- 32 rows, one float each -- hit distinct banks; at Lk
// they were 32-way conflicts); the partials reuse that area once the products are done, so two
// workgroups fit a CU.
__global__ __launch_bounds__(NT, 2) void pool_u_mfma_kernel(const PoolGrpArgs a) {
  extern __shared__ __attribute__((aligned(16))) float pbg[];   // [32][Lk + 2] (rows >= R zero)
  const int b = blockIdx.x, gi = blockIdx.y, t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int beg = a.gbeg[gi], heads = a.heads, H = a.H;
  const int R = a.gcnt[gi] * heads, Lk = a.p[beg].Lk, LDP = Lk + 2;
  // staging: wave w the rows w, w + 4, ...; float4 loads (Lk % 4 == 0), scalar LDS stores
  for (int row = w; row < POOL_GRP_ROWS; row += NT / 64) {
    const float* src = row < R ? a.p[beg + row / heads].pbar + ((int64_t)b * heads + row % heads) * Lk : nullptr;
    for (int c4 = lane; c4 < Lk / 4; c4 += 64) {
      const float4 v = src ? *reinterpret_cast<const float4*>(src + 4 * c4) : make_float4(0.f, 0.f, 0.f, 0.f);
      float* d = pbg + row * LDP + 4 * c4;
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    }
  }
  __syncthreads();
  for (int row = w; row < R; row += NT / 64) {
    float s = 0.f;
    for (int j = lane; j < Lk; j += 64) s += pbg[row * LDP + j];
    s = sum64(s);
    if (lane == 0) a.p[beg + row / heads].r[(int64_t)b * heads + row % heads] = s;
  }
  const int n = lane & 31, h = lane >> 5;
  const int cb = w & 1, kh = w >> 1, ncb = H / 128;
  const int half = Lk / 2, j_beg = kh * half;   // (Lk even)
  for (int cbb = cb; cbb < 2 * ((ncb + 1) / 2); cbb += 2) {   // (H = 256: one pass; H = 128: wave cb 1 idles)
    const bool on = cbb < ncb;
    f32x16 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    if (on) {
      const float* bcol = a.p[beg].pk + ((int64_t)b * Lk + j_beg + h) * H + 128 * cbb + 4 * n;
      const float* arow = pbg + n * LDP + j_beg + h;
      // 8 key pairs per chunk: the P_k float4s of the next chunk issued before this one's MFMAs
      float4 bvv[2][8];
#pragma unroll
      for (int k = 0; k < 8; ++k)
        bvv[0][k] = 2 * k < half ? *reinterpret_cast<const float4*>(bcol + (int64_t)2 * k * H) : make_float4(0.f, 0.f, 0.f, 0.f);
      for (int k0 = 0; k0 < half; k0 += 32) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int jj = k0 + 16 + 2 * k;
          if (jj < half) bvv[1][k] = *reinterpret_cast<const float4*>(bcol + (int64_t)jj * H);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int jj = k0 + 2 * k;
          if (jj < half) {
            const float av = arow[jj];
            const float4 x = bvv[0][k];
            acc[0] = mfma_f32(av, x.x, acc[0]);
            acc[1] = mfma_f32(av, x.y, acc[1]);
            acc[2] = mfma_f32(av, x.z, acc[2]);
            acc[3] = mfma_f32(av, x.w, acc[3]);
          }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int jj = k0 + 32 + 2 * k;
          if (jj < half) bvv[0][k] = *reinterpret_cast<const float4*>(bcol + (int64_t)jj * H);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int jj = k0 + 16 + 2 * k;
          if (jj < half) {
            const float av = arow[jj];
            const float4 x = bvv[1][k];
            acc[0] = mfma_f32(av, x.x, acc[0]);
            acc[1] = mfma_f32(av, x.y, acc[1]);
            acc[2] = mfma_f32(av, x.z, acc[2]);
            acc[3] = mfma_f32(av, x.w, acc[3]);
          }
        }
      }
    }
    __syncthreads();   // (every wave's A reads done: the partials reuse the pbar area)
    float* part = pbg;   // [2 col blocks][32 rows][128]
    // key half 1 parks its partial in LDS, key half 0 adds it and stores (rows acc_row(e, h),
    // column 128 cbb + 4 n + i of tile i)
    if (kh == 1 && on) {
#pragma unroll
      for (int e = 0; e < 16; ++e)
        *reinterpret_cast<float4*>(part + (cb * 32 + acc_row(e, h)) * 128 + 4 * n) =
            make_float4(acc[0][e], acc[1][e], acc[2][e], acc[3][e]);
    }
    __syncthreads();
    if (kh == 0 && on) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = acc_row(e, h);
        if (row >= R) continue;
        const float4 o = *reinterpret_cast<const float4*>(part + (cb * 32 + row) * 128 + 4 * n);
        *reinterpret_cast<float4*>(a.p[beg + row / heads].u + ((int64_t)b * heads + row % heads) * H + 128 * cbb + 4 * n) =
            make_float4(acc[0][e] + o.x, acc[1][e] + o.y, acc[2][e] + o.z, acc[3][e] + o.w);
      }
    }
    if (cbb + 2 < 2 * ((ncb + 1) / 2)) {   // (another pass re-stages nothing: H > 256 is refused)
      __syncthreads();
    }
  }
}

// Group the pairs by key modality (same P_k) and launch the grouped kernels; false when the
// shapes do not fit them (the caller runs the per-pair kernels)
bool launch_pool_grouped(bool fwd, const PoolPair* pairs, int npairs, int B, int heads, int hd, int H,
                         hipStream_t st, hipError_t& err) {
  err = hipSuccess;
  if (getenv("MMF_POOL_PER_PAIR") || H % 4 != 0 || H > 256 || npairs < 2) return false;
  // the fp32-MFMA forms (MMF_POOL_VALU=1: the VALU forms, A/B)
  static const bool valu = getenv("MMF_POOL_VALU") != nullptr;
  std::vector<std::vector<int>> groups;
  std::vector<const float*> keyp;
  for (int g = 0; g < npairs; ++g) {
    size_t i = 0;
    while (i < keyp.size() && (keyp[i] != pairs[g].pk || pairs[groups[i][0]].Lk != pairs[g].Lk)) ++i;
    if (i == keyp.size()) { keyp.push_back(pairs[g].pk); groups.emplace_back(); }
    groups[i].push_back(g);
  }
  if (groups.size() == (size_t)npairs) return false;   // nothing shared
  bool mfma = !valu;
  for (auto& gr : groups) {
    const int R = (int)gr.size() * heads, Lk = pairs[gr[0]].Lk;
    if (R > POOL_GRP_ROWS || (size_t)R * (fwd ? Lk : H) * sizeof(float) > 64 * 1024) return false;
    // dpbar: H % 8 (the float4 quads), Lk % 32 (key tiles); U: H % 128 (column blocks), Lk even and
    // the pbar rows + partials in LDS; 16-B aligned P_k rows
    if (fwd ? (H % 128 != 0 || H > 256 || Lk % 4 != 0 ||
               (size_t)std::max(POOL_GRP_ROWS * (Lk + 2), 2 * 32 * 128) * 4 > 80 * 1024)
            : (H % 8 != 0 || Lk % 32 != 0))
      mfma = false;
    for (int g : gr)
      if (((uintptr_t)pairs[g].pk & 15) != 0 || (fwd && ((uintptr_t)pairs[g].pbar & 15) != 0)) mfma = false;
  }
  size_t gi = 0;
  while (gi < groups.size()) {
    PoolGrpArgs a;
    memset(&a, 0, sizeof(a));
    int np = 0, ng = 0;
    size_t shm = 0;
    double fl = 0.0, by = 0.0;
    while (gi < groups.size() && np + (int)groups[gi].size() <= POOL_GRP_MAX) {
      a.gbeg[ng] = np;
      a.gcnt[ng] = (int)groups[gi].size();
      const int Lk = pairs[groups[gi][0]].Lk, R = a.gcnt[ng] * heads;
      for (int g : groups[gi]) a.p[np++] = pairs[g];
      shm = std::max(shm, mfma ? (fwd ? (size_t)std::max(POOL_GRP_ROWS * (Lk + 2), 2 * 32 * 128) * 4 : 0)
                               : (size_t)R * (fwd ? Lk : H) * sizeof(float));
      fl += 2.0 * B * R * Lk * H;
      by += 4.0 * B * ((double)Lk * H + R * (Lk + H));   // P_k once per group
      ++ng;
      ++gi;
    }
    a.ngroups = ng;
    a.B = B; a.heads = heads; a.hd = hd; a.H = H;
    if (mfma) {
      ProfLaunch prof_(st, fwd ? "pool_u_mfma_kernel" : "pool_dpbar_mfma_kernel", fl, by);
      if (fwd) {
        static bool attr = false;
        if (!attr && shm > 64 * 1024) {
          (void)hipFuncSetAttribute((const void*)pool_u_mfma_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
          attr = true;
        }
        mmf_launch(pool_u_mfma_kernel, dim3(B, ng), dim3(NT), (uint32_t)shm, st, a);
      } else {
        mmf_launch(pool_dpbar_mfma_kernel, dim3(B, ng), dim3(NT), 0, st, a);
      }
    } else {
      ProfLaunch prof_(st, fwd ? "pool_u_grp_kernel" : "pool_dpbar_grp_kernel", fl, by);
      if (fwd) mmf_launch(pool_u_grp_kernel, dim3(B, ng), dim3(NT), (uint32_t)shm, st, a);
      else mmf_launch(pool_dpbar_grp_kernel, dim3(B, ng), dim3(NT), (uint32_t)shm, st, a);
    }
    err = hipGetLastError();
    if (err != hipSuccess) return true;
  }
  return true;
}

hipError_t launch_pool(bool fwd, const PoolPair* pairs, int npairs, int B, int heads, int hd, int H,
                       hipStream_t st) {
  if (heads > MAXH || H % 4 != 0) return hipErrorInvalidValue;
  hipError_t gerr;
  if (launch_pool_grouped(fwd, pairs, npairs, B, heads, hd, H, st, gerr)) return gerr;
  int done = 0;
  while (done < npairs) {
    PoolArgs a;
    memset(&a, 0, sizeof(a));
    int n = 0;
    while (done < npairs && n < POOL_MAX_PAIRS) {
      if (pairs[done].Lk * heads > POOL_PB_CAP || heads > MAXH) return hipErrorInvalidValue;
      a.p[n++] = pairs[done++];
    }
    a.npairs = n;
    a.B = B; a.heads = heads; a.hd = hd; a.H = H;
    double fl = 0.0, by = 0.0;   // U_h = pbar_h P_k  /  dpbar = P_k . dU_h: one pass over P_k
    for (int i = 0; i < n; ++i) {
      fl += 2.0 * B * heads * a.p[i].Lk * H;
      by += 4.0 * B * ((double)a.p[i].Lk * H + heads * (a.p[i].Lk + H));
    }
    ProfLaunch prof_(st, fwd ? "pool_u_kernel" : "pool_dpbar_kernel", fl, by);
    if (fwd) {
      mmf_launch(pool_u_kernel, dim3(B, n), dim3(NT), 0, st, a);
    } else {
      const size_t shm = (size_t)heads * H * sizeof(float);
      mmf_launch(pool_dpbar_kernel, dim3(B, n), dim3(NT), shm, st, a);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace

hipError_t launch_pool_u(const PoolPair* pairs, int npairs, int B, int heads, int hd, int H, hipStream_t st) {
  return launch_pool(true, pairs, npairs, B, heads, hd, H, st);
}

hipError_t launch_pool_dpbar(const PoolPair* pairs, int npairs, int B, int heads, int hd, int H,
                             hipStream_t st) {
  return launch_pool(false, pairs, npairs, B, heads, hd, H, st);
}

// E_m as a rank-(nsrc x heads) update of 32-row blocks, for H <= 256 and nsrc x heads <= 24 (C5:
// 5 x 4): a workgroup takes 32 rows j of one sample, its 64 float4 columns x 4 row groups; each
// thread keeps its column's dU vectors (one per (source, head)) in registers and the block's
// pbar weights come from LDS, so per output float4 the loads are LDS broadcasts only (pool_e_kernel
// re-loaded every dU vector per output: 40 loads per 16 B written, 0.39 ms at C5).
constexpr int POOLE_RB = 32, POOLE_NSH = 24;
__global__ __launch_bounds__(NT) void pool_e_blk_kernel(const PoolEArgs a) {
  __shared__ float w_s[POOLE_RB][POOLE_NSH];
  const PoolEMod& E = a.m[blockIdx.y];
  const int H = a.H, H4 = H / 4, heads = a.heads, L = E.L, nsh = E.nsrc * heads;
  const int nblk = (L + POOLE_RB - 1) / POOLE_RB;
  const int b = blockIdx.x / nblk, j0 = (blockIdx.x % nblk) * POOLE_RB;
  if (b >= a.B) return;
  const int t = threadIdx.x;
  for (int i = t; i < POOLE_RB * nsh; i += NT) {
    const int r = i / nsh, q = i % nsh, sidx = q / heads, hh = q % heads;
    const int j = min(j0 + r, L - 1);
    w_s[r][q] = E.pbar[sidx][((int64_t)b * heads + hh) * L + j];
  }
  const int c4 = t & 63, rg = t >> 6;
  const bool col_ok = c4 < H4;
  float4 u[POOLE_NSH];
#pragma unroll
  for (int q = 0; q < POOLE_NSH; ++q) {
    u[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (q < nsh && col_ok) {
      const int sidx = q / heads, hh = q % heads;
      u[q] = *reinterpret_cast<const float4*>(E.du[sidx] + ((int64_t)b * heads + hh) * H + 4 * c4);
    }
  }
  float4 cv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (col_ok) {
    cv = *reinterpret_cast<const float4*>(E.c + (int64_t)b * E.ldc + 4 * c4);
    cv = make_float4(cv.x * E.cscale, cv.y * E.cscale, cv.z * E.cscale, cv.w * E.cscale);
  }
  __syncthreads();
  for (int r = rg; r < POOLE_RB; r += NT / 64) {
    const int j = j0 + r;
    if (j >= L || !col_ok) continue;
    float4 acc = cv;
#pragma unroll
    for (int q = 0; q < POOLE_NSH; ++q) {
      if (q < nsh) {
        const float w = w_s[r][q];
        acc.x += w * u[q].x; acc.y += w * u[q].y; acc.z += w * u[q].z; acc.w += w * u[q].w;
      }
    }
    *reinterpret_cast<float4*>(E.out + ((int64_t)b * L + j) * H + 4 * c4) = acc;
  }
}

// The same update on the fp32 matrix cores: a 64-row block of one sample per workgroup, wave w
// the 32-row tile w >> 1 and the 128-column block w & 1 (lane n' holds columns 4n' .. 4n'+3, MFMA
// i the interleaved tile {4n' + i}, so the row stores are float4); K = sources x heads (padded to
// even) from LDS, 32x32x2 f32 MFMAs.  The VALU form is bound by its 80 FMAs per float4 stored.
constexpr int POOLE_MROWS = 64;
__global__ __launch_bounds__(NT) void pool_e_mfma_kernel(const PoolEArgs a) {
  __shared__ __attribute__((aligned(16))) float w_s[POOLE_MROWS][POOLE_NSH];
  __shared__ __attribute__((aligned(16))) float du_s[POOLE_NSH][POOL_MFMA_HMAX];
  const PoolEMod& E = a.m[blockIdx.y];
  const int H = a.H, heads = a.heads, L = E.L, nsh = E.nsrc * heads;
  const int nblk = (L + POOLE_MROWS - 1) / POOLE_MROWS;
  const int b = blockIdx.x / nblk, j0 = (blockIdx.x % nblk) * POOLE_MROWS;
  if (b >= a.B) return;
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  for (int i = t; i < POOLE_MROWS * POOLE_NSH; i += NT) {
    const int r = i / POOLE_NSH, q = i % POOLE_NSH, j = min(j0 + r, L - 1);
    w_s[r][q] = q < nsh ? E.pbar[q / heads][((int64_t)b * heads + q % heads) * L + j] : 0.f;
  }
  for (int i = t; i < POOLE_NSH * (H / 4); i += NT) {
    const int q = i / (H / 4), c4 = i % (H / 4);
    const float4 v = q < nsh ? *reinterpret_cast<const float4*>(E.du[q / heads] + ((int64_t)b * heads + q % heads) * H + 4 * c4)
                             : make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(&du_s[q][4 * c4]) = v;
  }
  __syncthreads();
  const int rt = w >> 1, cb = w & 1, n = lane & 31, h = lane >> 5;
  if (128 * cb >= H) return;
  f32x16 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
  const int ksteps = (nsh + 1) / 2;
#pragma unroll
  for (int s2 = 0; s2 < POOLE_NSH / 2; ++s2) {
    if (s2 < ksteps) {   // (wave-uniform; a guard, not a break: the loop stays unrolled)
      const float av = w_s[rt * 32 + n][2 * s2 + h];
      const float4 x = *reinterpret_cast<const float4*>(&du_s[2 * s2 + h][128 * cb + 4 * n]);
      acc[0] = mfma_f32(av, x.x, acc[0]);
      acc[1] = mfma_f32(av, x.y, acc[1]);
      acc[2] = mfma_f32(av, x.z, acc[2]);
      acc[3] = mfma_f32(av, x.w, acc[3]);
    }
  }
  const int col = 128 * cb + 4 * n;
  float4 cv = *reinterpret_cast<const float4*>(E.c + (int64_t)b * E.ldc + col);
  cv = make_float4(cv.x * E.cscale, cv.y * E.cscale, cv.z * E.cscale, cv.w * E.cscale);
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int j = j0 + rt * 32 + acc_row(e, h);
    if (j < L)
      *reinterpret_cast<float4*>(E.out + ((int64_t)b * L + j) * H + col) =
          make_float4(cv.x + acc[0][e], cv.y + acc[1][e], cv.z + acc[2][e], cv.w + acc[3][e]);
  }
}

hipError_t launch_pool_e(const PoolEMod* mods, int nmods, int B, int heads, int H, hipStream_t st) {
  if (nmods > 8 || H % 4 != 0) return hipErrorInvalidValue;
  bool blk = H <= 256 && !getenv("MMF_POOLE_FLAT");
  for (int i = 0; i < nmods && blk; ++i) blk = mods[i].nsrc * heads <= POOLE_NSH;
  // the MFMA form: H % 128 (column blocks), 16-B aligned rows (MMF_POOL_VALU=1: the VALU form)
  static const bool valu = getenv("MMF_POOL_VALU") != nullptr;
  bool mf = blk && !valu && H % 128 == 0;
  for (int i = 0; i < nmods && mf; ++i)
    mf = ((uintptr_t)mods[i].out & 15) == 0 && ((uintptr_t)mods[i].c & 15) == 0 && mods[i].ldc % 4 == 0;
  if (mf) {
    PoolEArgs a;
    memset(&a, 0, sizeof(a));
    a.B = B; a.heads = heads; a.H = H;
    int maxb = 0;
    double fl = 0.0, by = 0.0;
    for (int i = 0; i < nmods; ++i) {
      if (mods[i].nsrc > POOLE_MAX_SRC) return hipErrorInvalidValue;
      for (int sidx = 0; sidx < mods[i].nsrc; ++sidx)
        if (((uintptr_t)mods[i].du[sidx] & 15) != 0) return hipErrorInvalidValue;
      a.m[i] = mods[i];
      maxb = std::max(maxb, B * ((mods[i].L + POOLE_MROWS - 1) / POOLE_MROWS));
      fl += 2.0 * B * mods[i].nsrc * heads * mods[i].L * H;
      by += 4.0 * B * ((double)mods[i].L * H + mods[i].nsrc * heads * (mods[i].L + H) + H);
    }
    ProfLaunch prof_(st, "pool_e_mfma_kernel", fl, by);
    mmf_launch(pool_e_mfma_kernel, dim3(maxb, nmods), dim3(NT), 0, st, a);
    return hipGetLastError();
  }
  if (blk) {
    PoolEArgs a;
    memset(&a, 0, sizeof(a));
    a.B = B; a.heads = heads; a.H = H;
    int maxb = 0;
    double fl = 0.0, by = 0.0;
    for (int i = 0; i < nmods; ++i) {
      if (mods[i].nsrc > POOLE_MAX_SRC) return hipErrorInvalidValue;
      a.m[i] = mods[i];
      maxb = std::max(maxb, B * ((mods[i].L + POOLE_RB - 1) / POOLE_RB));
      fl += 2.0 * B * mods[i].nsrc * heads * mods[i].L * H;
      by += 4.0 * B * ((double)mods[i].L * H + mods[i].nsrc * heads * (mods[i].L + H) + H);
    }
    ProfLaunch prof_(st, "pool_e_blk_kernel", fl, by);
    mmf_launch(pool_e_blk_kernel, dim3(maxb, nmods), dim3(NT), 0, st, a);
    return hipGetLastError();
  }
  PoolEArgs a;
  memset(&a, 0, sizeof(a));
  a.B = B; a.heads = heads; a.H = H;
  int maxb = 0;
  for (int i = 0; i < nmods; ++i) {
    if (mods[i].nsrc > POOLE_MAX_SRC) return hipErrorInvalidValue;
    a.m[i] = mods[i];
    const int64_t per_b = (int64_t)mods[i].L * (H / 4);
    a.blocks_per_b[i] = (int)((per_b + NT - 1) / NT);
    const int nb = a.blocks_per_b[i] * B;
    if (nb > maxb) maxb = nb;
  }
  double fl = 0.0, by = 0.0;   // E_m = c/L + sum_s pbar_s^T dU_s, written once
  for (int i = 0; i < nmods; ++i) {
    fl += 2.0 * B * mods[i].nsrc * heads * mods[i].L * H;
    by += 4.0 * B * ((double)mods[i].L * H + mods[i].nsrc * heads * (mods[i].L + H) + H);
  }
  ProfLaunch prof_(st, "pool_e_kernel", fl, by);
  mmf_launch(pool_e_kernel, dim3(maxb, nmods), dim3(NT), 0, st, a);
  return hipGetLastError();
}

}  // namespace mmf
