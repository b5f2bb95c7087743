// Grouped, multi-source fp32 GEMM on CDNA4 matrix cores (v_mfma_f32_32x32x2_f32).
//
// One launch covers several independent outputs ("groups": e.g. the Q/K
// projections of every modality pair, src/attention.py:104-106, or the
// per-modality projections, src/fusion.py:291-298).  A group may sum several
// (A, B) sources into one output tile (the backward of a tensor that feeds
// several Linears, e.g. dP_m = sum over pairs of dQ W_q + dK W_k), and may
// split its contraction into slabs (dW = dY^T X over B*L rows) that a
// deterministic reduce kernel sums.
//
// Tile: 128x128 outputs per 256-thread workgroup = 4 waves as 2x2, each wave
// 64x64 = 2x2 MFMA 32x32 accumulators.  Two kernels share that tiling and the
// epilogue:
//  * gemm_lds_kernel (the fast path): operand tiles (128 x 32 fp32) go
//    global -> LDS by LDS-DMA (global_load_lds_dwordx4, no VGPR round trip),
//    double-buffered so tile t+1 streams in while tile t feeds the MFMAs; one
//    barrier per k-tile.  k-contiguous tiles are stored [e][k] with an XOR
//    swizzle on the 16-B slot (applied on the global source address, the LDS
//    image stays lane-linear) so each ds_read_b128 fragment read (4 k-steps of
//    one lane) is bank-conflict free; k-strided tiles are stored [k][e] and
//    read with conflict-free ds_read_b32.
//  * gemm_generic_kernel: register-staged, element-guarded; for operands that
//    are not float4-able (odd leading dims, K % 4 != 0).
// MFMA k-order: within each 8-deep k chunk j, lane half h feeds k = 8j+4h+s at
// step s (the same permutation on A and B, so the contraction is unchanged).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

#include "mmf_device.h"

namespace mmf {

namespace {

constexpr int BM = 128, BN = 128, BK = 32, NT = 256;
#ifndef MMF_GEMM_DK
#define MMF_GEMM_DK 16   // k-tile depth of the LDS-DMA kernel
#endif
#ifndef MMF_GEMM_NS
#define MMF_GEMM_NS 3    // LDS ring stages
#endif
constexpr int LDS_STRIDE = BM + 4;      // generic kernel, KR image
constexpr int LDS_STRIDE_T = BM + 1;    // generic kernel, RK image (transposing writes)

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct TileCtx {
  int i0, j0, batch, split, nsplit;
  float* Cb;
  float* part_db;
  const float* biasb;
  int brs_off;
};

// XCD-aware group interleave (see group_of_block): 0 off, 1 launches without split-K groups
// (the default: C5 projections 2.58 -> 2.47 ms/step; the split-K weight gradients were
// slower interleaved, 2.00 -> 2.27 ms), 2 every launch.  MMF_GEMM_ILV overrides.
int gemm_interleave_mode() {
  const char* e = getenv("MMF_GEMM_ILV");
  if (!e || !e[0]) return 1;
  return e[0] == '0' ? 0 : (e[0] == '2' ? 2 : 1);
}

// The grid is 1-D over the tiles of every group of the launch, in group order
// (launch_gemm puts the longest contractions first).  With args.ilv the groups
// are interleaved instead: workgroups are dealt round-robin to the 8 XCDs, so
// block b runs on XCD b % 8; its (b / 8)-th block there takes group (b/8) % ng
// at local tile 8 * ((b/8) / ng) + b % 8.  Every group's copy of one local tile
// then runs back to back on the same XCD, and groups that share an operand
// (the projections of one modality read the same P_m rows; the weight
// gradients of one modality the same P_m k-chunk) hit that XCD's L2 for it.
__device__ __forceinline__ int group_of_block(const GemmArgs& args, int& local) {
  const int b = blockIdx.x;
  if (args.ilv) {
    const int idx = b >> 3, ng = args.ngroups;
    const int k = idx / ng;
    local = k * 8 + (b & 7);
    return idx - k * ng;
  }
  int g = 0;
#pragma unroll
  for (int i = 1; i < GEMM_MAX_GROUPS; ++i)
    if (i < args.ngroups && b >= args.tile_off[i]) g = i;
  local = b - args.tile_off[g];
  return g;
}

// XCD-aware tile order: a group's workgroups `local` and `local + 8` run on the same XCD (the
// dispatcher deals workgroups round-robin to the 8 XCDs, in both group layouts), and each XCD has
// its own L2.  The tiles that share an operand -- the column tiles of one row block (they read the
// same A rows), or the output tiles of one split-K slab (the same A and B k-chunk) -- are dealt to
// one XCD back to back: with n_in such tiles per set, local = 8 r + x takes set 8 (r / n_in) + x,
// member r % n_in.  Where the sets do not come in multiples of 8 the plain order stays.  (C5 dZ,
// two column tiles: the A rows were fetched once per column tile, 5.4 GB per step for 3.2 GB of
// operands.)
__device__ __forceinline__ bool tile_ctx(const GemmGroup& G, int local, TileCtx& t, int bn = BN) {
  const int tiles_n = (G.N + bn - 1) / bn;
  const int tiles_m = (G.M + BM - 1) / BM;
  t.nsplit = (G.epi & EPI_PARTIAL) ? G.nsplit : 1;
  const int per_batch = tiles_m * tiles_n * t.nsplit;
  t.batch = local / per_batch;
  if (t.batch >= G.nbatch) return false;
  int tile = local - t.batch * per_batch;
  const int n_in = t.nsplit > 1 ? tiles_m * tiles_n : tiles_n;   // tiles per operand-sharing set
  const int n_out = t.nsplit > 1 ? t.nsplit : tiles_m;           // sets
  if (n_in > 1 && (n_out & 7) == 0) {
    const int x = tile & 7, r = tile >> 3;
    const int set = (r / n_in) * 8 + x, mem = r % n_in;
    if (t.nsplit > 1) {
      t.split = set;
      t.i0 = (mem / tiles_n) * BM;
      t.j0 = (mem % tiles_n) * bn;
    } else {
      t.split = 0;
      t.i0 = set * BM;
      t.j0 = mem * bn;
    }
  } else {
    t.split = tile % t.nsplit;
    tile /= t.nsplit;
    t.i0 = (tile / tiles_n) * BM;
    t.j0 = (tile % tiles_n) * bn;
  }
  t.Cb = (G.epi & EPI_PARTIAL) ? G.C + (int64_t)t.batch * t.nsplit * G.M * G.N
                               : G.C + (int64_t)t.batch * G.bs_c;
  t.part_db = G.part_db ? G.part_db + (int64_t)t.batch * t.nsplit * G.M : nullptr;
  t.biasb = G.bias ? G.bias + (int64_t)t.batch * G.bs_bias : nullptr;
  t.brs_off = G.bias_rs_off + t.batch * G.bs_brs;
  return true;
}

// ------------------------------------------------------------------ epilogue
// The accumulators go through LDS (two passes of 64 rows, [64][BN+4] image)
// so the epilogue runs row-major: each thread finishes 8 consecutive columns
// of a row at a time (float4 loads/stores, one Philox call per 8 dropout
// decisions), and the code stays small (the kernels are I-cache sensitive at
// small grids).  Order: v = alpha*acc; +bias[j] (x bias_rs[i]); +rowadd;
// +addm; relu; gate; rowscale; dropout (keep(site, i*N + j)).
constexpr int CS = BN + 4;
// Register budget: gemm_lds_kernel sits at ~163 VGPRs; past 168 it drops from 3
// to 2 waves/SIMD, which measured ~30% slower on every GEMM.  Keep epilogue
// state out of registers that live across the passes (EPI_COLSUM reuses the image).

// 8 consecutive floats of a side operand row (vec: two 16-B loads)
__device__ __forceinline__ void load8(float (&d)[8], const float* p, int nv, bool vec) {
  if (vec) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(p);
    const f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
    d[0] = a[0]; d[1] = a[1]; d[2] = a[2]; d[3] = a[3];
    d[4] = b[0]; d[5] = b[1]; d[6] = b[2]; d[7] = b[3];
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) d[e] = e < nv ? p[e] : 0.f;
  }
}

template <int PR = 64>   // rows per LDS pass (64 or 32)
__device__ __forceinline__ void epilogue(const GemmGroup& G, const TileCtx& T, f32x16 (&acc)[2][2], float* cs,
                                         const RngSnap& rs, float p, float inv_keep, int wm, int wn, int h,
                                         int c) {
  const int t = threadIdx.x;
  const int epi = G.epi;
  const bool partial = (epi & EPI_PARTIAL) != 0;
  const bool drop = !partial && (epi & EPI_DROP) && p > 0.f;
  const bool coop = drop && (G.N % 8) == 0;
  const uint32_t thr = p16(p);
  float* const out = partial ? T.Cb + (int64_t)T.split * G.M * G.N : T.Cb;
  const int ldc = partial ? G.N : G.ldc;
  const bool vst = (ldc % 4) == 0 && ((uintptr_t)out & 15) == 0;
  const bool vstb = (ldc % 8) == 0 && ((uintptr_t)T.Cb & 15) == 0;   // EPI_BF16: 16-B rows of 8
  // a thread always finishes the same 8 columns (rows t>>4 + 16*it of each 64-row pass)
  const int cg = (t & 15) * 8, j0 = T.j0 + cg;
  const int nv = min(8, G.N - j0);
  // side operands (rowadd / addm / gate) row-vectorisable: 16-B aligned rows, 8 columns present
  const bool vside = nv == 8 && (j0 % 4) == 0 &&
                     (!(epi & EPI_ROWADD) || ((G.ld_rowadd % 4) == 0 && ((uintptr_t)G.rowadd & 15) == 0)) &&
                     (!(epi & EPI_ADDMAT) || ((G.ld_addm % 4) == 0 && ((uintptr_t)G.addm & 15) == 0)) &&
                     (!(epi & EPI_GATE) ||
                      ((G.ld_gate % ((epi & EPI_GATE_B16) ? 8 : 4)) == 0 && ((uintptr_t)G.gate & 15) == 0));
  float bias[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bias[e] = (!partial && (epi & EPI_BIAS) && e < nv) ? T.biasb[j0 + e] : 0.f;
  float csum = 0.f;   // EPI_COLSUM: thread t < BN owns column T.j0 + t (rows in fixed order)
  for (int pass = 0; pass < BM / PR; ++pass) {
    __syncthreads();
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int rb = wm * 64 + a * 32 - pass * PR;    // this accumulator's first row in the pass
      if (rb >= 0 && rb < PR) {
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int r = 0; r < 16; ++r) cs[(rb + acc_row(r, h)) * CS + wn * 64 + b * 32 + c] = acc[a][b][r];
      }
    }
    __syncthreads();
    // (threads whose 8 columns lie past N skip the rows, not the pass: every thread
    // reaches the EPI_COLSUM barrier below)
#pragma unroll
    for (int it = 0; it < PR / 16; ++it) {
      const int lr = (t >> 4) + 16 * it;
      const int i = T.i0 + pass * PR + lr;
      if (i >= G.M || nv <= 0) continue;
      const f32x4 lo = *reinterpret_cast<const f32x4*>(cs + lr * CS + cg);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(cs + lr * CS + cg + 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if (partial) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= G.alpha;
      } else {
        uint4 rr = make_uint4(0, 0, 0, 0);
        if (coop) rr = philox_block(rs, G.drop_site, ((uint64_t)i * (uint64_t)G.N + (uint64_t)j0) >> 3);
        const float brs = (epi & EPI_BIAS_RS) ? G.bias_rs[(int64_t)i * G.bias_rs_ld + T.brs_off] : 1.f;
        const float rsc = (epi & EPI_ROWSCALE) ? G.rowscale[(int64_t)(i / G.rs_div) * G.rs_stride + G.rs_off] : 1.f;
        // the row's side operands as two 16-B loads each (issued together, before the math)
        float ad[8], gt[8];
        if (epi & EPI_ROWADD) {
          load8(ad, G.rowadd + (int64_t)(i / G.rowadd_div) * G.ld_rowadd + j0, nv, vside);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = v[e] * G.alpha + G.rowadd_scale * ad[e];
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] *= G.alpha;
        }
        if (epi & EPI_ADDMAT) {
          load8(ad, G.addm + (int64_t)i * G.ld_addm + j0, nv, vside);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += ad[e];
        }
        if ((epi & EPI_GATE) && (epi & EPI_GATE_B16)) {
          // (the bf16 copy of P: 8 signs in one 16-B load)
          const __bf16* gb = reinterpret_cast<const __bf16*>(G.gate) + (int64_t)i * G.ld_gate + j0;
          if (vside) {
            const bf16x8 q = *reinterpret_cast<const bf16x8*>(gb);
#pragma unroll
            for (int e = 0; e < 8; ++e) gt[e] = (float)q[e];
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) gt[e] = e < nv ? (float)gb[e] : 0.f;
          }
        } else if (epi & EPI_GATE) {
          load8(gt, G.gate + (int64_t)i * G.ld_gate + j0, nv, vside);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (e >= nv) break;
          const int j = j0 + e;
          float x = v[e] + bias[e] * brs;
          if (epi & EPI_RELU) x = fmaxf(x, 0.f);
          if (epi & EPI_GATE) x = gt[e] > 0.f ? x * G.gate_scale : 0.f;
          x *= rsc;
          if (drop) {
            const bool keep = coop ? keep_from(rr, e, thr)
                                   : keep1(rs, G.drop_site, (uint64_t)i * (uint64_t)G.N + (uint64_t)j, p);
            x = keep ? x * inv_keep : 0.f;
          }
          v[e] = x;
        }
      }
      if (epi & EPI_COLSUM) {
        // the final values back into the image for the column sums.  ds_write_b128 banks are
        // (a / 4) mod 32 over groups of 8 consecutive lanes, whose 8-column slices lie 32 B apart:
        // lanes with bit 2 set store their upper half first, so each store instruction covers
        // all 32 banks once (the plain lo-then-hi order was 2-way conflicted: 43 % of the
        // projection GEMM's LDS cycles, profiles/r05/close3/pmc_sq_c2.json)
        const bool sw = (t & 4) != 0;
        const f32x4 lo = f32x4{v[0], v[1], v[2], v[3]}, hi = f32x4{v[4], v[5], v[6], v[7]};
        float* row = cs + lr * CS + cg;
        *reinterpret_cast<f32x4*>(row + (sw ? 4 : 0)) = sw ? hi : lo;
        *reinterpret_cast<f32x4*>(row + (sw ? 0 : 4)) = sw ? lo : hi;
      }
      if (epi & EPI_BF16COPY) {   // (never with EPI_PARTIAL / EPI_BF16; nbatch 1)
        __bf16* ob = reinterpret_cast<__bf16*>(G.copy) + (int64_t)i * ldc + j0;
        if (vstb && nv == 8 && ((uintptr_t)G.copy & 15) == 0) {
          bf16x8 pk;
#pragma unroll
          for (int e = 0; e < 8; ++e) pk[e] = (__bf16)v[e];
          *reinterpret_cast<bf16x8*>(ob) = pk;
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (e < nv) ob[e] = (__bf16)v[e];
        }
      }
      if (epi & EPI_BF16) {   // (never with EPI_PARTIAL; nbatch 1)
        __bf16* ob = reinterpret_cast<__bf16*>(T.Cb) + (int64_t)i * ldc + j0;
        if (vstb && nv == 8) {
          bf16x8 pk;
#pragma unroll
          for (int e = 0; e < 8; ++e) pk[e] = (__bf16)v[e];
          *reinterpret_cast<bf16x8*>(ob) = pk;
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (e < nv) ob[e] = (__bf16)v[e];
        }
        continue;
      }
      float* o = out + (int64_t)i * ldc + j0;
      if (vst && nv == 8) {
        *reinterpret_cast<f32x4*>(o) = f32x4{v[0], v[1], v[2], v[3]};
        *reinterpret_cast<f32x4*>(o + 4) = f32x4{v[4], v[5], v[6], v[7]};
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (e < nv) o[e] = v[e];
      }
    }
    if (epi & EPI_COLSUM) {
      __syncthreads();
      const int nr = min(PR, G.M - T.i0 - pass * PR);
      if (t < BN)
        for (int r = 0; r < nr; ++r) csum += cs[r * CS + t];
    }
  }
  if ((epi & EPI_COLSUM) && t < BN && T.j0 + t < G.N) {
    const int tiles_m = (G.M + BM - 1) / BM;
    G.colsum[((int64_t)T.batch * tiles_m + T.i0 / BM) * G.N + T.j0 + t] = csum;
  }
}

// ------------------------------------------------------------------ LDS-DMA kernel
// k-tiles of DK = 16 in a 3-deep LDS ring: tile t+2 is issued while tile t
// feeds the MFMAs and tile t+1 is in flight (2 tiles = 32 KB in flight per
// workgroup, 3 workgroups per CU).  A 128 x 16 operand tile is 8 KB = 8
// wave-instructions of 1 KB (wave w issues 2).  Rows past `eext` and k past
// `kend` are clamped to valid addresses; the k tail is zeroed afterwards
// (zero_tail), the row tail only feeds outputs that are never stored.
// RK image [e][DK], 4*DK-byte rows; 16-B slots XOR-swizzled by the row's
// position in its 256-B bank row so ds_read_b128 fragment reads are conflict
// free.  KR image [DK][128], 512-B k-rows.  A wave-instruction moves 1 KB.
template <int DK>
__device__ __forceinline__ int swz(int row) {
  constexpr int S = DK / 4;              // slots per row
  constexpr int RB = 64 / DK;            // rows per 256-B bank row
  return (row / RB) & (S - 1);
}

template <int MODE, int DK>
__device__ __forceinline__ void stage_tile(float* lds, const Operand& op, int64_t boff, int e0, int eext, int k0,
                                           int kend, int wave, int lane) {
  constexpr int PER_WAVE = BM * DK / 256 / 4;   // 1-KB instructions per wave
  constexpr int S = DK / 4;
#pragma unroll
  for (int u = 0; u < PER_WAVE; ++u) {
    const int ins = wave * PER_WAVE + u;
    const float* src;
    // (row_div is wave-uniform and 1 on every hot launch: the division stays off that path)
    if (MODE == MODE_RK) {
      const int row = ins * (64 / S) + lane / S;
      const int slot = (lane % S) ^ swz<DK>(row);
      const int e = min(e0 + row, eext - 1);
      const int k = min(k0 + 4 * slot, kend - 4);
      const int er = op.row_div == 1 ? e : e / op.row_div;
      src = op.ptr + boff + (int64_t)er * op.ld + k;
    } else {
      const int kr = min(k0 + ins * 2 + (lane >> 5), kend - 1);
      const int e = min(e0 + 4 * (lane & 31), eext - 4);
      const int krr = op.row_div == 1 ? kr : kr / op.row_div;
      src = op.ptr + boff + (int64_t)krr * op.ld + e;
    }
    __builtin_amdgcn_global_load_lds((const void*)src,
                                     (__attribute__((address_space(3))) void*)(lds + ins * 256), 16, 0, 0);
  }
}

// Zero the k >= kv part of a staged tile (last tile of a contraction; kv % 4 == 0 for RK).
template <int MODE, int DK>
__device__ __forceinline__ void zero_tail(float* lds, int kv) {
  const int t = threadIdx.x;
  if (MODE == MODE_RK) {
    constexpr int S = DK / 4;
    for (int idx = t; idx < BM * S; idx += NT) {
      const int row = idx / S, slot = idx % S;
      if (4 * slot >= kv)
        *reinterpret_cast<f32x4*>(lds + row * DK + ((slot ^ swz<DK>(row)) << 2)) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  } else {
    for (int idx = t; idx < DK * BM / 4; idx += NT) {
      if (idx / (BM / 4) >= kv) *reinterpret_cast<f32x4*>(lds + idx * 4) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
}

// Fragment of 4 consecutive MFMA k-steps (chunk j) for tile row/col e.
template <int MODE, int DK>
__device__ __forceinline__ f32x4 frag(const float* lds, int e, int j, int h) {
  if (MODE == MODE_RK) {
    const int slot = (2 * j + h) ^ swz<DK>(e);
    return *reinterpret_cast<const f32x4*>(lds + e * DK + (slot << 2));
  } else {
    const float* p = lds + (8 * j + 4 * h) * BM + e;
    return f32x4{p[0], p[BM], p[2 * BM], p[3 * BM]};
  }
}

// bf16 operand tiles (gemm_lds_kernel<..., B16 = 1>, "medium" with bf16 copies of both operands in
// HBM, RK mode, DK = 32 bf16 k per tile): [e][32] bf16 = 64-B rows, the fp32 DK = 16 image's row
// size, 16-B slots (8 k each) XOR-swizzled the same way (swz<16>), so the LDS-DMA pieces, the ring
// footprint and the conflict-free fragment reads carry over; a fragment (lane half h of k-chunk u:
// k = 16 u + 8 h .. + 7) is ONE ds_read_b128 with no conversion, half the LDS bytes per MFMA of the
// fp32-operand form.
__device__ __forceinline__ void stage_tile_b16(float* lds, const Operand& op, int64_t boff, int e0, int eext, int k0,
                                               int kend, int wave, int lane) {
  constexpr int PER_WAVE = BM * 32 * 2 / 1024 / 4;   // 1-KB pieces per wave (2)
#pragma unroll
  for (int u = 0; u < PER_WAVE; ++u) {
    const int ins = wave * PER_WAVE + u;
    const int row = ins * 16 + lane / 4;
    const int slot = (lane & 3) ^ swz<16>(row);
    const int e = min(e0 + row, eext - 1);
    const int k = min(k0 + 8 * slot, kend - 8);
    const __bf16* src = reinterpret_cast<const __bf16*>(op.ptr) + boff + (int64_t)e * op.ld + k;
    __builtin_amdgcn_global_load_lds((const void*)src,
                                     (__attribute__((address_space(3))) void*)(lds + ins * 256), 16, 0, 0);
  }
}
// the same tile staged by NWV waves (8 / NWV pieces each)
template <int NWV>
__device__ __forceinline__ void stage_tile_b16_nw(float* lds, const Operand& op, int64_t boff, int e0, int eext, int k0,
                                                  int kend, int wave, int lane) {
  constexpr int PER_WAVE = BM * 32 * 2 / 1024 / NWV;
  static_assert(PER_WAVE >= 1, "at most 8 staging waves");
#pragma unroll
  for (int u = 0; u < PER_WAVE; ++u) {
    const int ins = wave * PER_WAVE + u;
    const int row = ins * 16 + lane / 4;
    const int slot = (lane & 3) ^ swz<16>(row);
    const int e = min(e0 + row, eext - 1);
    const int k = min(k0 + 8 * slot, kend - 8);
    const __bf16* src = reinterpret_cast<const __bf16*>(op.ptr) + boff + (int64_t)e * op.ld + k;
    __builtin_amdgcn_global_load_lds((const void*)src,
                                     (__attribute__((address_space(3))) void*)(lds + ins * 256), 16, 0, 0);
  }
}
__device__ __forceinline__ void zero_tail_b16(float* lds, int kv) {
  for (int idx = threadIdx.x; idx < BM * 4; idx += NT) {
    const int row = idx / 4, slot = idx % 4;
    if (8 * slot >= kv)
      *reinterpret_cast<f32x4*>(lds + row * 16 + ((slot ^ swz<16>(row)) << 2)) = f32x4{0.f, 0.f, 0.f, 0.f};
  }
}
__device__ __forceinline__ bf16x8 frag_b16(const float* lds, int e, int u, int h) {
  const int slot = (2 * u + h) ^ swz<16>(e);
  return *reinterpret_cast<const bf16x8*>(lds + e * 16 + (slot << 2));
}

// k-strided bf16 tiles (B16 = 2 / 3: an operand stored [k][e], e contiguous -- the dQ / dK /
// P_m rows of a weight gradient, the W_q / W_k rows of dZ): a [32 k][128 e] image of 256-B rows,
// 16-B chunk ch (e = 8 ch .. 8 ch + 7) of row r at slot ch ^ xkr(r) -- the layout on which both the
// LDS-DMA fill and the transposed fragment reads are conflict-free (cdna_hip_programming.md T10,
// image (b)).  One 1-KB DMA piece = 4 k rows: lane L fills slot L & 15 of row 4 ins + L / 16 by
// choosing its source chunk.  The MFMA fragment (lane r = l & 31 of half h: e row r, k = 8 h + j)
// is two ds_read_b64_tr_b16, each a 4 (k) x 16 (e) block delivered column-major.
__device__ __forceinline__ int xkr(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ void stage_tile_b16_kr(float* lds, const Operand& op, int64_t boff, int e0, int eext,
                                                  int k0, int kend, int wave, int lane) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int ins = wave * 2 + u;
    const int row = 4 * ins + (lane >> 4);
    const int ch = (lane & 15) ^ xkr(row);
    const int k = min(k0 + row, kend - 1);
    const int e = min(e0 + 8 * ch, eext - 8);
    const __bf16* src = reinterpret_cast<const __bf16*>(op.ptr) + boff + (int64_t)k * op.ld + e;
    __builtin_amdgcn_global_load_lds((const void*)src,
                                     (__attribute__((address_space(3))) void*)(lds + ins * 256), 16, 0, 0);
  }
}
__device__ __forceinline__ void zero_tail_b16_kr(float* lds, int kv) {
  for (int idx = threadIdx.x; idx < 32 * 16; idx += NT)
    if ((idx >> 4) >= kv) *reinterpret_cast<f32x4*>(lds + idx * 4) = f32x4{0.f, 0.f, 0.f, 0.f};
}
typedef __bf16 bf16x4g __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4g lds_bf16x4g;
__device__ __forceinline__ int kr_off(int row, int e) { return 256 * row + 16 * ((e >> 3) ^ xkr(row)) + 2 * (e & 7); }
// fragment of k-step u (16 k) for e rows e_base .. e_base + 31
__device__ __forceinline__ bf16x8 frag_b16_kr(const float* lds, int e_base, int u, int lane) {
  const char* img = reinterpret_cast<const char*>(lds);
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int e = e_base + 16 * (g & 1) + 4 * p;
  const int k0 = 16 * u + 8 * (g >> 1) + q;
  const bf16x4g lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4g*)(img + kr_off(k0, e)));
  const bf16x4g hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4g*)(img + kr_off(k0 + 4, e)));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// (source, k0) cursor over one tile's contraction
struct KCursor { int si, k0, kend; };

// B16: both operands bf16 in HBM (BF = 1, DK = 32 bf16 k per tile): 1 RK / RK (stage_tile_b16),
// 2 KR / KR (stage_tile_b16_kr: weight gradients), 3 RK / KR (dZ = dQ W_q).
// WIDE (B16 forms 2 / 3, N % 256 == 0): 128 x 256 output tiles -- a stage holds A and TWO B
// tiles, wave (wm, wn) the 64 rows wm and the columns wn * 64 + {0, 32} of each 128-column half
// (acc[a][b], b >> 1 = half), and the epilogue runs once per half.  With N = 256 (dZ: every
// modality's H; the weight gradients' H x H) a tile covers every column, so its A rows are read
// once instead of once per 128-column tile (the second read relied on L2 timing: 1.6 x the
// operand bytes from HBM at C5).
template <int AMODE, int BMODE, int DK, int NSTAGE, int BF, int B16, int WIDE, int CHAIN>
__device__ __forceinline__ void gemm_lds_body(const GemmArgs& args) {
  static_assert(!B16 || (BF == 1 && DK == 32 && AMODE == (B16 == 2 ? MODE_KR : MODE_RK) &&
                         BMODE == (B16 == 1 ? MODE_RK : MODE_KR)),
                "bf16-operand form");
  static_assert(!WIDE || B16 >= 2, "WIDE: bf16 forms 2 / 3");
  constexpr int NB = WIDE ? 2 : 1;                      // B tiles per stage
  constexpr int DTILE = B16 ? BM * DK / 2 : BM * DK;   // floats per operand tile
  constexpr int DMA_PER_TILE = B16 ? (1 + NB) * (BM * DK / 2048) : 2 * (BM * DK / 1024);  // glds per wave per stage
  int local;
  int gi = group_of_block(args, local);

  // one LDS object: NSTAGE x [A | B (| B)] tiles (also the epilogue image) + 128 floats for the row-sum combine
  constexpr int SSTRIDE = (1 + NB) * DTILE;   // floats per stage
  __shared__ __attribute__((aligned(16))) float lds[NSTAGE * SSTRIDE + BM];
  constexpr int PR = NSTAGE * SSTRIDE >= 64 * CS ? 64 : 32;   // epilogue rows per LDS pass
  static_assert(NSTAGE * SSTRIDE >= PR * CS, "epilogue image does not fit");

  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int wm = wave >> 1, wn = wave & 1;

  RngSnap rs{0, 0};
  const float p = args.drop_p;
  const float inv_keep = p < 1.f ? 1.f / (1.f - p) : 0.f;
  if (p > 0.f && args.rng) rs = *args.rng;
  if (args.rng_advance && blockIdx.x == 0 && threadIdx.x == 0) args.rng_advance[1] += 1;   // see launch_gemm

  // The tile of the block's group, then of each group chained to it (GemmGroup::chain: a GEMM
  // whose A operand is this tile's output rows -- dX_m = dZ_m W_m after dZ_m -- run by the same
  // workgroup on the same rows once the first tile's stores have landed: no launch of its own and
  // its A rows from L2, not HBM)
  for (;;) {
  const GemmGroup& G = args.g[gi];
  TileCtx T;
  if (!tile_ctx(G, local, T, NB * BN)) return;
  const int64_t offA = (int64_t)T.batch * G.bs_a, offB = (int64_t)T.batch * G.bs_b;

  f32x16 acc[2][2 * NB];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2 * NB; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const bool partial = (G.epi & EPI_PARTIAL) != 0;
  const bool want_db = partial && T.part_db != nullptr && T.j0 == 0;
  float dbsum = 0.f;

  auto first_from = [&](int si) {
    KCursor k;
    for (k.si = si; k.si < G.src_count; ++k.si) {
      const GemmSrc& S = args.s[G.src_begin + k.si];
      k.k0 = partial ? T.split * G.kchunk : 0;
      k.kend = partial ? min(S.K, k.k0 + G.kchunk) : S.K;
      if (k.k0 < k.kend) break;
    }
    return k;
  };
  auto advance = [&](KCursor k) {
    if (k.si >= G.src_count) return k;
    k.k0 += DK;
    if (k.k0 < k.kend) return k;
    return first_from(k.si + 1);
  };
  // the staged source's operands, re-read from the kernel arguments only when
  // the cursor moves to another source
  Operand opA = args.s[G.src_begin].a, opB = args.s[G.src_begin].b;
  int op_si = 0;
  // per-segment operands (seg_stride != 0): offset by the segment of the tile's first row
  const int64_t seg = G.seg_rows > 0 ? T.i0 / G.seg_rows : 0;
  auto stage = [&](int buf, const KCursor& k) {
    if (k.si != op_si) {
      opA = args.s[G.src_begin + k.si].a;
      opB = args.s[G.src_begin + k.si].b;
      op_si = k.si;
    }
    float* At = lds + buf * SSTRIDE;
    if constexpr (B16) {
      if constexpr (AMODE == MODE_KR)
        stage_tile_b16_kr(At, opA, offA + seg * opA.seg_stride, T.i0, G.M, k.k0, k.kend, wave, lane);
      else
        stage_tile_b16(At, opA, offA + seg * opA.seg_stride, T.i0, G.M, k.k0, k.kend, wave, lane);
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) {
        if constexpr (BMODE == MODE_KR)
          stage_tile_b16_kr(At + (1 + nb) * DTILE, opB, offB + seg * opB.seg_stride, T.j0 + nb * BN, G.N, k.k0, k.kend,
                            wave, lane);
        else
          stage_tile_b16(At + (1 + nb) * DTILE, opB, offB + seg * opB.seg_stride, T.j0 + nb * BN, G.N, k.k0, k.kend,
                         wave, lane);
      }
    } else {
      stage_tile<AMODE, DK>(At, opA, offA + seg * opA.seg_stride, T.i0, G.M, k.k0, k.kend, wave, lane);
      stage_tile<BMODE, DK>(At + DTILE, opB, offB + seg * opB.seg_stride, T.j0, G.N, k.k0, k.kend, wave, lane);
    }
  };
  // wait until at most `ahead` tiles' DMAs are outstanding (vmcnt needs an immediate)
  auto wait_tiles = [&](int ahead) {
    if (ahead <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DMA_PER_TILE) : "memory");
    else if (ahead == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * DMA_PER_TILE) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * DMA_PER_TILE) : "memory");
  };
  static_assert(NSTAGE >= 2 && NSTAGE <= 5, "ring depth");

  KCursor cur = first_from(0);
  if (cur.si < G.src_count) {
    // prologue: NSTAGE-1 tiles in flight; tile n always lives in buffer n % NSTAGE
    KCursor iss = cur;
    int nissued = 0;
    for (int q = 0; q < NSTAGE - 1 && iss.si < G.src_count; ++q) {
      stage(q, iss);
      iss = advance(iss);
      ++nissued;
    }
    int tile = 0, buf = 0;
    for (;;) {
      // tile `tile` has landed once only the later tiles' DMAs are outstanding;
      // the barrier also means every wave is done with the buffer restaged below
      wait_tiles(nissued - tile - 1);
      lds_barrier();
      float* At = lds + buf * SSTRIDE;
      float* Bt = At + DTILE;
      const int kv = cur.kend - cur.k0;
      if (kv < DK) {
        if constexpr (B16) {
          if constexpr (AMODE == MODE_KR) zero_tail_b16_kr(At, kv);
          else zero_tail_b16(At, kv);
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) {
            if constexpr (BMODE == MODE_KR) zero_tail_b16_kr(Bt + nb * DTILE, kv);
            else zero_tail_b16(Bt + nb * DTILE, kv);
          }
        } else {
          zero_tail<AMODE, DK>(At, kv);
          zero_tail<BMODE, DK>(Bt, kv);
        }
        lds_barrier();
      }
      if (iss.si < G.src_count) {
        stage(nissued % NSTAGE, iss);
        iss = advance(iss);
        ++nissued;
      }
      if (B16 && AMODE == MODE_KR && want_db) {
        // bias grad of a TN dW from the bf16 A image (thread: row t&127, k half t>>7)
        const int row = t & (BM - 1), kh = t >> 7;
        const char* img = reinterpret_cast<const char*>(At);
#pragma unroll
        for (int q = 0; q < 16; ++q) dbsum += (float)*reinterpret_cast<const __bf16*>(img + kr_off(kh * 16 + q, row));
      }
      if (!B16 && want_db) {
        // bias grad of a TN dW: row sums of A over this k-tile (thread: row t&127, k half t>>7)
        const int row = t & (BM - 1), kh = t >> 7;
#pragma unroll
        for (int q = 0; q < DK / 2; ++q) {
          const int kk = kh * (DK / 2) + q;
          dbsum += AMODE == MODE_KR ? At[kk * BM + row]
                                    : At[row * DK + ((((kk >> 2) ^ swz<DK>(row))) << 2) + (kk & 3)];
        }
      }
if constexpr (B16) {
#pragma unroll
        for (int u = 0; u < DK / 16; ++u) {
          bf16x8 av[2], bv[2 * NB];
#pragma unroll
          for (int a = 0; a < 2; ++a)
            av[a] = AMODE == MODE_KR ? frag_b16_kr(At, wm * 64 + a * 32, u, lane) : frag_b16(At, wm * 64 + a * 32 + c, u, h);
#pragma unroll
          for (int b = 0; b < 2 * NB; ++b) {
            const float* Bh = Bt + (b >> 1) * DTILE;   // (the 128-column half)
            bv[b] = BMODE == MODE_KR ? frag_b16_kr(Bh, wn * 64 + (b & 1) * 32, u, lane)
                                     : frag_b16(Bh, wn * 64 + (b & 1) * 32 + c, u, h);
          }
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2 * NB; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[a], bv[b], acc[a][b], 0, 0, 0);
        }
      } else if constexpr (BF != 0) {
        // chunks 2u, 2u+1 (16 k) -> one bf16 MFMA per accumulator
#pragma unroll
        for (int u = 0; u < DK / 16; ++u) {
          float av[2][8], bv[2][8];
#pragma unroll
          for (int jj = 0; jj < 2; ++jj) {
#pragma unroll
            for (int a = 0; a < 2; ++a) {
              const f32x4 f = frag<AMODE, DK>(At, wm * 64 + a * 32 + c, 2 * u + jj, h);
#pragma unroll
              for (int s = 0; s < 4; ++s) av[a][4 * jj + s] = f[s];
            }
#pragma unroll
            for (int b = 0; b < 2; ++b) {
              const f32x4 f = frag<BMODE, DK>(Bt, wn * 64 + b * 32 + c, 2 * u + jj, h);
#pragma unroll
              for (int s = 0; s < 4; ++s) bv[b][4 * jj + s] = f[s];
            }
          }
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) acc[a][b] = mfma_k16<BF>(av[a], bv[b], acc[a][b]);
        }
      } else {
#pragma unroll
      for (int j = 0; j < DK / 8; ++j) {
        f32x4 af[2], bf[2];
#pragma unroll
        for (int a = 0; a < 2; ++a) af[a] = frag<AMODE, DK>(At, wm * 64 + a * 32 + c, j, h);
#pragma unroll
        for (int b = 0; b < 2; ++b) bf[b] = frag<BMODE, DK>(Bt, wn * 64 + b * 32 + c, j, h);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) acc[a][b] = mfma32(af[a][s], bf[b][s], acc[a][b]);
      }
      }
      const KCursor nx = advance(cur);
      if (nx.si >= G.src_count) break;
      cur = nx;
      ++tile;
      buf = buf == NSTAGE - 1 ? 0 : buf + 1;
    }
  }

  if (want_db) {
    float* red = lds + NSTAGE * SSTRIDE;
    __syncthreads();
    if (t >= BM) red[t - BM] = dbsum;
    __syncthreads();
    if (t < BM && T.i0 + t < G.M)
      T.part_db[(int64_t)T.split * G.M + T.i0 + t] = (dbsum + red[t]) * G.alpha;
  }
  if constexpr (WIDE) {
    // one epilogue per 128-column half (each re-syncs before it reuses the LDS image)
    f32x16 lo[2][2] = {{acc[0][0], acc[0][1]}, {acc[1][0], acc[1][1]}};
    epilogue<PR>(G, T, lo, lds, rs, p, inv_keep, wm, wn, h, c);
    TileCtx T2 = T;
    T2.j0 += BN;
    f32x16 hi[2][2] = {{acc[0][2], acc[0][3]}, {acc[1][2], acc[1][3]}};
    epilogue<PR>(G, T2, hi, lds, rs, p, inv_keep, wm, wn, h, c);
  } else {
    epilogue<PR>(G, T, acc, lds, rs, p, inv_keep, wm, wn, h, c);
  }
  if constexpr (!CHAIN) break;
  if (!G.chain) break;
  gi = G.chain - 1;
  // every wave's stores of this tile complete (vmcnt counts stores), every wave past the epilogue's
  // reads of the LDS image, and the L1 invalidated (agent-scope acquire) before the chained tile's
  // DMA reads those rows back
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
}

template <int AMODE, int BMODE, int DK, int NSTAGE, int BF = 0, int B16 = 0, int WIDE = 0>
__global__ __launch_bounds__(NT, (NSTAGE * (B16 ? DK / 2 : DK) <= 32 ? 4 : 2)) void gemm_lds_kernel(const GemmArgs args) {
  gemm_lds_body<AMODE, BMODE, DK, NSTAGE, BF, B16, WIDE, 0>(args);
}
// The same with chained groups (GemmGroup::chain: dX_m after dZ_m), held to 3 waves per SIMD like
// the plain kernel (168 VGPRs: the chain's loop-carried state must not cost a wave)
template <int AMODE, int BMODE, int DK, int NSTAGE, int BF = 0>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(3)))
void gemm_lds_chain_kernel(const GemmArgs args) {
  gemm_lds_body<AMODE, BMODE, DK, NSTAGE, BF, 0, 0, 1>(args);
}

// ------------------------------------------------------------------ weight-stationary kernel
// Y (rows x N) = X (rows x K) W^T (+bias, relu) for N <= 128, K <= 128 (16 | K):
// the projection shape of the fused modalities (Q/K projections of every pair,
// src/attention.py:104-105).  At K = 128 a 128 x 128 tile is 4.2 MFLOP against
// 128 KB of operands, so staging BOTH operands through LDS per tile makes the
// LDS-DMA fill (~6 TB/s chip-wide) the co-bottleneck with the fp32 MFMA.  Here
// each wave loads its 64 columns of W^T once into registers (128 VGPRs at K =
// 128, in the MFMA k-order of the A fragments) and keeps them while the
// workgroup walks a contiguous run of row tiles; only X streams through a
// 6-deep LDS-DMA ring of 128 x 16 k-tiles, which runs ahead across tile
// boundaries.  The epilogue stores straight from the accumulators (each store
// instruction writes two 128-B row segments), so the ring keeps filling while
// a tile is written out.  Persistent grid: 2 workgroups per CU.
constexpr int WSR_DK = 16, WSR_NS = 6, WSR_NKC = 16;   // k-tile, ring depth, max 8-deep k chunks (K <= 128)

// EXT: the extended epilogue (row scale, dropout, column sums) and B stored [k][n] (the modality
// projections and dX at C2); without it the round-5 kernel (Q / K projections: bias, ReLU)
template <int BF, bool EXT>
__global__ __launch_bounds__(NT, 2) void gemm_wsr_kernel(const GemmArgs args, int total_items, int K) {
  constexpr int DTILE = BM * WSR_DK;
  __shared__ __attribute__((aligned(16))) float ring[WSR_NS * DTILE];
  __shared__ float csx[BN];   // EPI_COLSUM: the lower-half waves' (wm = 1) 64-row column sums
  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int wm = wave >> 1, wn = wave & 1;
  const int nkt = K / WSR_DK, nkc = K / 8;

  RngSnap rs{0, 0};
  const float p = args.drop_p;
  const float inv_keep = p < 1.f ? 1.f / (1.f - p) : 0.f;
  const uint32_t thr = p16(p);
  if (p > 0.f && args.rng) rs = *args.rng;
  if (args.rng_advance && blockIdx.x == 0 && threadIdx.x == 0) args.rng_advance[1] += 1;   // see launch_gemm
  const int nwg = gridDim.x;
  const int item0 = (int)(((int64_t)blockIdx.x * total_items) / nwg);
  const int item1 = (int)(((int64_t)(blockIdx.x + 1) * total_items) / nwg);
  if (item0 >= item1) return;

  // flat DMA cursor over (item, k-tile)
  const int nflat = (item1 - item0) * nkt;
  auto item_group = [&](int item, int& rowtile) {
    int g = 0;
#pragma unroll
    for (int i = 1; i < GEMM_MAX_GROUPS; ++i)
      if (i < args.ngroups && item >= args.tile_off[i]) g = i;
    rowtile = item - args.tile_off[g];
    return g;
  };
  // DMA cursor: (item, k-tile) advance monotonically, so the group is tracked
  // incrementally (a 32-way tile_off search per issue held all 32 offsets in
  // SGPRs and spilled them)
  int di = item0, dk = 0, drt = 0;
  int dg = item_group(item0, drt);
  const int g_first = dg, rt_first = drt;
  auto issue = [&](int f) {
    const int slot = f % WSR_NS;
    const GemmSrc& S = args.s[args.g[dg].src_begin];
    stage_tile<MODE_RK, WSR_DK>(ring + slot * DTILE, S.a, 0, drt * BM, args.g[dg].M, dk * WSR_DK, K, wave, lane);
    if (++dk == nkt) {
      dk = 0;
      ++di;
      ++drt;
      while (dg + 1 < args.ngroups && di >= args.tile_off[dg + 1]) { ++dg; drt = di - args.tile_off[dg]; }
    }
  };
  // Wait for k-tile f: every later k-tile (2 LDS-DMAs per wave each) and the
  // epilogue stores issued after it (16 per wave per tile, exact: WSR tiles are
  // never partial) may stay in flight -- vmcnt counts loads, stores and DMAs
  // together, in issue order.
  auto wait_ahead = [&](int ahead, bool stores_younger) {
    if (stores_younger) {
      switch (ahead) {
        case 0: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(22)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
      }
    } else {
      switch (ahead) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
      }
    }
  };
  static_assert(WSR_NS - 2 <= 4, "wait_ahead covers 4 tiles ahead");

  int nissued = 0;
  for (; nissued < WSR_NS - 1 && nissued < nflat; ++nissued) issue(nissued);

  f32x4 breg[2][WSR_NKC];
  float bias[2];
  int cur_g = -1;
  int f = 0;
  int epi_mark = 0;   // k-tiles issued before the latest epilogue's stores
  int g = g_first, rt = rt_first;   // compute cursor (the same walk as the DMA cursor, behind it)
  for (int item = item0; item < item1; ++item, ++rt) {
    while (g + 1 < args.ngroups && item >= args.tile_off[g + 1]) { ++g; rt = item - args.tile_off[g]; }
    const GemmGroup& G = args.g[g];
    if (g != cur_g) {
      // this group's W^T slice for the wave's 64 columns, in the A fragments' k-order:
      // breg[b][m] = W[col][8m + 4h .. 8m + 4h + 3], col = wn*64 + b*32 + c
      cur_g = g;
      const GemmSrc& S = args.s[G.src_begin];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int col = wn * 64 + b * 32 + c;
        const bool ok = col < G.N;
        if (EXT && args.bmode == MODE_KR) {
          // B stored [k][n] (dX = dZ W_proj): the same fragments gathered down column `col`
          const float* wcol = S.b.ptr + (ok ? col : 0) + (int64_t)(4 * h) * S.b.ld;
#pragma unroll
          for (int m = 0; m < WSR_NKC; ++m)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              breg[b][m][e] = (ok && m < nkc) ? wcol[(int64_t)(8 * m + e) * S.b.ld] : 0.f;
        } else {
          const float* wrow = S.b.ptr + (int64_t)(ok ? col : 0) * S.b.ld + 4 * h;
#pragma unroll
          for (int m = 0; m < WSR_NKC; ++m)
            breg[b][m] = (ok && m < nkc) ? *reinterpret_cast<const f32x4*>(wrow + 8 * m) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        bias[b] = (ok && (G.epi & EPI_BIAS)) ? G.bias[col] : 0.f;
      }
      // Retire these loads here with a wait the compiler can see (the builtin,
      // not inline asm: vmcnt(0), lgkmcnt/expcnt untouched).  Otherwise it
      // cannot tell them apart from the LDS-DMAs issued after them and drains
      // the whole ring (vmcnt(0)) before every k-tile that uses them.
      __builtin_amdgcn_s_waitcnt(0x0F70);
    }
    f32x16 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

#pragma unroll
    for (int kt = 0; kt < WSR_NKC / 2; ++kt) {
      if (kt < nkt) {
        wait_ahead(nissued - f - 1, f < epi_mark);
        lds_barrier();   // tile f landed for every wave; every wave is done with slot (f-1) % NS
        if (nissued < nflat) issue(nissued++);
        const float* At = ring + (f % WSR_NS) * DTILE;
if constexpr (BF != 0) {
          float av[2][8], bv[2][8];
#pragma unroll
          for (int j = 0; j < 2; ++j) {
#pragma unroll
            for (int a = 0; a < 2; ++a) {
              const f32x4 fa = frag<MODE_RK, WSR_DK>(At, wm * 64 + a * 32 + c, j, h);
#pragma unroll
              for (int s = 0; s < 4; ++s) av[a][4 * j + s] = fa[s];
            }
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
              for (int s = 0; s < 4; ++s) bv[b][4 * j + s] = breg[b][2 * kt + j][s];
          }
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) acc[a][b] = mfma_k16<BF>(av[a], bv[b], acc[a][b]);
        } else {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x4 af[2];
#pragma unroll
          for (int a = 0; a < 2; ++a) af[a] = frag<MODE_RK, WSR_DK>(At, wm * 64 + a * 32 + c, j, h);
#pragma unroll
          for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
              for (int b = 0; b < 2; ++b) acc[a][b] = mfma32(af[a][s], breg[b][2 * kt + j][s], acc[a][b]);
        }
        }
        ++f;
      }
    }
    // Epilogue straight from the accumulators: v = alpha*acc + bias[j]; relu; rowscale; dropout
    // (the LDS-DMA kernel's order and keep(site, i*N + j) decisions).
    // Lane (c, h) holds rows 8q+4h+{0..3} of column c; a 4x4 transpose across
    // the lane quad (xor 2, then xor 1) leaves it 4 consecutive columns of one
    // row, stored as one 16-B store (8 rows x 128 B per wave instruction).
    const int x = c & 3;
    const int i0 = rt * BM + wm * 64;
    const int epi = EXT ? G.epi : 0;
    const bool drop = (epi & EPI_DROP) && p > 0.f;
    // EPI_ROWSCALE: one scale per row tile (job_wsr: rs_div % BM == 0), a scalar load
    float rsc = 1.f;
    if (epi & EPI_ROWSCALE)
      rsc = ((const __attribute__((address_space(4))) float*)G.rowscale)[(rt * BM / G.rs_div) * G.rs_stride + G.rs_off];
    float csum[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};   // EPI_COLSUM
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v[e] = acc[a][b][4 * q + e] * G.alpha + bias[b];
            if (G.epi & EPI_RELU) v[e] = fmaxf(v[e], 0.f);
          }
          // v[r] = M[r][x]; step 1 swaps the off-diagonal 2x2 blocks (partner x^2)
          {
            const bool up = (x & 2) != 0;
            const float s0 = dpp<DPP_XOR2>(up ? v[0] : v[2]);
            const float s1 = dpp<DPP_XOR2>(up ? v[1] : v[3]);
            if (up) { v[0] = s0; v[1] = s1; } else { v[2] = s0; v[3] = s1; }
          }
          // now lane x holds M[x&2 .. +1][x&1 + (0|2)]; step 2 swaps within 2x2 (partner x^1)
          {
            const bool odd = (x & 1) != 0;
            const float s0 = dpp<DPP_XOR1>(odd ? v[0] : v[1]);
            const float s1 = dpp<DPP_XOR1>(odd ? v[2] : v[3]);
            if (odd) { v[0] = s0; v[2] = s1; } else { v[1] = s0; v[3] = s1; }
          }
          const int row = i0 + a * 32 + 8 * q + 4 * h + x;
          const int col = wn * 64 + b * 32 + (c & ~3);
          if (epi & EPI_ROWSCALE) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] *= rsc;
          }
          if (drop) {
            // the Philox block of columns (col & ~7) .. +7 of this row (shared with lane c ^ 4),
            // this lane's four of its eight decisions
            const uint4 rr = philox_block(rs, G.drop_site, ((uint64_t)row * (uint64_t)G.N + (uint64_t)(col & ~7)) >> 3);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = keep_from(rr, (col & 4) + e, thr) ? v[e] * inv_keep : 0.f;
          }
          if (epi & EPI_COLSUM) {
#pragma unroll
            for (int e = 0; e < 4; ++e) csum[b][e] += v[e];
          }
          *reinterpret_cast<f32x4*>(G.C + (int64_t)row * G.ldc + col) = f32x4{v[0], v[1], v[2], v[3]};
        }
      }
    if (epi & EPI_COLSUM) {
      // per-tile column sums of the stored values (GemmGroup::colsum): each lane's 8 rows (a, q),
      // then the quad (rows x, xor 1 / 2) and the halves (rows h, xor 32) -- every lane of quad
      // c & ~3 then holds the wave's 64-row sums of columns (c & ~3) + e; lane (c, h) keeps column
      // wn*64 + 32 h + c; the wm = 1 waves hand theirs to the wm = 0 waves through LDS (rows 0-63
      // + rows 64-127, fixed order)
      float mine = 0.f;
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float sv = csum[b][e];
          sv += dpp<DPP_XOR1>(sv);
          sv += dpp<DPP_XOR2>(sv);
          sv = sum_xor32(sv);
          if (b == h && e == x) mine = sv;
        }
      const int colx = wn * 64 + 32 * h + c;
      if (wm == 1) csx[colx] = mine;
      lds_barrier();
      if (wm == 0 && colx < G.N) G.colsum[(int64_t)rt * G.N + colx] = mine + csx[colx];
    }
    epi_mark = nissued;
  }
}

// ------------------------------------------------------------------ weight-stationary bf16 kernel
// Y (rows x N <= 128, bf16) = X (rows x K, bf16) W^T (+ bias) for 32 <= K <= 256 (32 | K): the "medium"
// Q / K projections of the long-key pairs (src/attention.py:104-105 at C5: 60 GEMMs of
// 65536 x 256 x 256, each split into two 128-column groups).  The LDS-DMA kernel's 128 x 128 tile
// restages W's 64 KB k-strip from L2 for every tile and its 8 k-tiles leave prologue and epilogue
// exposed (0.11 of the bf16 peak at C5); here each wave loads its 64 columns of W^T once into
// registers (128 VGPRs at K = 256, the B fragments of v_mfma_f32_32x32x16_bf16) and keeps them
// while the workgroup walks a contiguous run of row tiles; X streams through a 6-deep LDS-DMA ring
// of the RK bf16 tiles (stage_tile_b16: [128 rows][32 k], 8 KB), which runs ahead across tile
// boundaries; the epilogue stores 4 bf16 per lane straight from the accumulators.  Persistent
// grid, 2 workgroups per CU; the two column groups of one GEMM are adjacent, so their workgroups
// (16 apart in dispatch order at C5: the same XCD) read the same X rows at about the same time.
constexpr int WSR16_NKS = 16;   // max 16-deep k-steps (K <= 256)
typedef __bf16 bf16x4s __attribute__((ext_vector_type(4)));

// WSR16_NS: the ring depth (tiles of 8 KB; WSR16_NS - 1 in flight ahead of the one being consumed).
// NWV = 8 (one 512-thread workgroup per CU): 256-column groups, wave (wm, wn) the 64 rows wm and
// the 64 columns wn of 4 -- both 128-column halves of a GEMM read each staged X tile, so X streams
// once per 256 columns instead of once per 128 (C5: 10 instead of 20 passes per modality).
template <int WSR16_NS, int NWV = 4>
__global__ __launch_bounds__(64 * NWV, NWV == 8 ? 1 : 2) void gemm_wsr_b16_kernel(const GemmArgs args, int total_items, int K) {
  constexpr int DTILE = BM * 32 / 2;   // floats per bf16 tile
  constexpr int PW = BM * 32 * 2 / 1024 / NWV;   // LDS-DMA pieces per wave per tile
  __shared__ __attribute__((aligned(16))) float ring[WSR16_NS * DTILE];
  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int wm = NWV == 8 ? wave >> 2 : wave >> 1, wn = NWV == 8 ? wave & 3 : wave & 1;
  const int nkt = K / 32, nks = K / 16;

  const int nwg = gridDim.x;
  const int item0 = (int)(((int64_t)blockIdx.x * total_items) / nwg);
  const int item1 = (int)(((int64_t)(blockIdx.x + 1) * total_items) / nwg);
  if (item0 >= item1) return;

  const int nflat = (item1 - item0) * nkt;
  auto item_group = [&](int item, int& rowtile) {
    int g = 0;
#pragma unroll
    for (int i = 1; i < GEMM_MAX_GROUPS; ++i)
      if (i < args.ngroups && item >= args.tile_off[i]) g = i;
    rowtile = item - args.tile_off[g];
    return g;
  };
  int di = item0, dk = 0, drt = 0;
  int dg = item_group(item0, drt);
  const int g_first = dg, rt_first = drt;
  auto issue = [&](int f) {
    const int slot = f % WSR16_NS;
    const GemmSrc& S = args.s[args.g[dg].src_begin];
    stage_tile_b16_nw<NWV>(ring + slot * DTILE, S.a, 0, drt * BM, args.g[dg].M, dk * 32, K, wave, lane);
    if (++dk == nkt) {
      dk = 0;
      ++di;
      ++drt;
      while (dg + 1 < args.ngroups && di >= args.tile_off[dg + 1]) { ++dg; drt = di - args.tile_off[dg]; }
    }
  };
  // as gemm_wsr_kernel: PW LDS-DMAs per wave per k-tile, 16 epilogue stores per wave per row tile
  // (vmcnt counts both, in issue order; the counter holds up to 63)
  auto wait_ahead = [&](int ahead, bool stores_younger) {
    const int n = PW * ahead + (stores_younger ? 16 : 0);
    switch (n) {
#define MMF_WC(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
      MMF_WC(0) MMF_WC(1) MMF_WC(2) MMF_WC(3) MMF_WC(4) MMF_WC(5) MMF_WC(6) MMF_WC(7) MMF_WC(8)
      MMF_WC(9) MMF_WC(10) MMF_WC(11) MMF_WC(12) MMF_WC(13) MMF_WC(14) MMF_WC(15) MMF_WC(16) MMF_WC(17)
      MMF_WC(18) MMF_WC(19) MMF_WC(20) MMF_WC(21) MMF_WC(22) MMF_WC(23) MMF_WC(24) MMF_WC(25) MMF_WC(26)
      MMF_WC(27) MMF_WC(28) MMF_WC(29) MMF_WC(30) MMF_WC(31) MMF_WC(32) MMF_WC(33) MMF_WC(34) MMF_WC(35)
      MMF_WC(36) MMF_WC(37) MMF_WC(38) MMF_WC(39) MMF_WC(40) MMF_WC(41) MMF_WC(42)
#undef MMF_WC
      default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
  };
  static_assert(PW * (WSR16_NS - 2) + 16 <= 42, "wait_ahead's table");

  int nissued = 0;
  for (; nissued < WSR16_NS - 1 && nissued < nflat; ++nissued) issue(nissued);

  bf16x8 breg[2][WSR16_NKS];
  float bias[2];
  int cur_g = -1;
  int f = 0;
  int epi_mark = 0;
  int g = g_first, rt = rt_first;
  for (int item = item0; item < item1; ++item, ++rt) {
    while (g + 1 < args.ngroups && item >= args.tile_off[g + 1]) { ++g; rt = item - args.tile_off[g]; }
    const GemmGroup& G = args.g[g];
    if (g != cur_g) {
      // this group's W^T slice for the wave's 64 columns: breg[b][s] = W[col][16 s + 8 h .. + 7]
      cur_g = g;
      const GemmSrc& S = args.s[G.src_begin];
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int col = wn * 64 + b * 32 + c;
        const bool ok = col < G.N;
        const __bf16* wrow = reinterpret_cast<const __bf16*>(S.b.ptr) + (int64_t)(ok ? col : 0) * S.b.ld + 8 * h;
#pragma unroll
        for (int m = 0; m < WSR16_NKS; ++m) {
          bf16x8 z;
#pragma unroll
          for (int e = 0; e < 8; ++e) z[e] = (__bf16)0.f;
          breg[b][m] = (ok && m < nks) ? *reinterpret_cast<const bf16x8*>(wrow + 16 * m) : z;
        }
        bias[b] = (ok && (G.epi & EPI_BIAS)) ? G.bias[col] : 0.f;
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);   // (see gemm_wsr_kernel: retire these loads visibly)
    }
    f32x16 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

#pragma unroll
    for (int kt = 0; kt < WSR16_NKS / 2; ++kt) {
      if (kt < nkt) {
        wait_ahead(nissued - f - 1, f < epi_mark);
        lds_barrier();
        if (nissued < nflat) issue(nissued++);
        const float* At = ring + (f % WSR16_NS) * DTILE;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          bf16x8 av[2];
#pragma unroll
          for (int a = 0; a < 2; ++a) av[a] = frag_b16(At, wm * 64 + a * 32 + c, u, h);
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
              acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[a], breg[b][2 * kt + u], acc[a][b], 0, 0, 0);
        }
        ++f;
      }
    }
    // epilogue: v = alpha*acc + bias[j], 4x4 transpose across the lane quad, 4 bf16 per store
    const int x = c & 3;
    const int i0 = rt * BM + wm * 64;
    __bf16* Cb = reinterpret_cast<__bf16*>(G.C);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[a][b][4 * q + e] * G.alpha + bias[b];
          {
            const bool up = (x & 2) != 0;
            const float s0 = dpp<DPP_XOR2>(up ? v[0] : v[2]);
            const float s1 = dpp<DPP_XOR2>(up ? v[1] : v[3]);
            if (up) { v[0] = s0; v[1] = s1; } else { v[2] = s0; v[3] = s1; }
          }
          {
            const bool odd = (x & 1) != 0;
            const float s0 = dpp<DPP_XOR1>(odd ? v[0] : v[1]);
            const float s1 = dpp<DPP_XOR1>(odd ? v[2] : v[3]);
            if (odd) { v[0] = s0; v[2] = s1; } else { v[1] = s0; v[3] = s1; }
          }
          const int row = i0 + a * 32 + 8 * q + 4 * h + x;
          const int col = wn * 64 + b * 32 + (c & ~3);
          if (col < G.N) {
            bf16x4s o;
            o[0] = (__bf16)v[0]; o[1] = (__bf16)v[1]; o[2] = (__bf16)v[2]; o[3] = (__bf16)v[3];
            *reinterpret_cast<bf16x4s*>(Cb + (int64_t)row * G.ldc + col) = o;
          }
        }
      }
    epi_mark = nissued;
  }
}

// ------------------------------------------------------------------ generic kernel
struct TileRegs { float4 v[4]; };

// Load one 128 x 32 tile of an operand into registers (element-guarded).
//  MODE_RK: stored [e][kk] (kk contiguous): thread t covers e = t/8 + 32u, kk = 4*(t%8)..+3
//  MODE_KR: stored [kk][e] (e contiguous):  thread t covers kk = t/32 + 8u, e = 4*(t%32)..+3
template <int MODE>
__device__ __forceinline__ void load_tile(TileRegs& R, const Operand& op, int64_t boff, int e0, int eext, int k0,
                                          int kend) {
  const int t = threadIdx.x;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    int e, kk;
    if (MODE == MODE_RK) { e = e0 + (t >> 3) + 32 * u; kk = k0 + 4 * (t & 7); }
    else                 { kk = k0 + (t >> 5) + 8 * u; e = e0 + 4 * (t & 31); }
    float x[4] = {0.f, 0.f, 0.f, 0.f};
    if (MODE == MODE_RK) {
      if (e < eext) {
        const float* rowp = op.ptr + boff + (int64_t)(e / op.row_div) * op.ld;
        if (op.vec && kk + 3 < kend) {
          const float4 f = *reinterpret_cast<const float4*>(rowp + kk);
          x[0] = f.x; x[1] = f.y; x[2] = f.z; x[3] = f.w;
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) if (kk + q < kend) x[q] = rowp[kk + q];
        }
      }
    } else {
      if (kk < kend) {
        const float* rowp = op.ptr + boff + (int64_t)(kk / op.row_div) * op.ld;
        if (op.vec && e + 3 < eext) {
          const float4 f = *reinterpret_cast<const float4*>(rowp + e);
          x[0] = f.x; x[1] = f.y; x[2] = f.z; x[3] = f.w;
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) if (e + q < eext) x[q] = rowp[e + q];
        }
      }
    }
    R.v[u] = make_float4(x[0], x[1], x[2], x[3]);
  }
}

template <int MODE>
__device__ __forceinline__ void store_tile(const TileRegs& R, float* S) {
  const int t = threadIdx.x;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    if (MODE == MODE_RK) {
      const int e = (t >> 3) + 32 * u, kk = 4 * (t & 7);
      S[(kk + 0) * LDS_STRIDE_T + e] = R.v[u].x;
      S[(kk + 1) * LDS_STRIDE_T + e] = R.v[u].y;
      S[(kk + 2) * LDS_STRIDE_T + e] = R.v[u].z;
      S[(kk + 3) * LDS_STRIDE_T + e] = R.v[u].w;
    } else {
      const int kk = (t >> 5) + 8 * u, e = 4 * (t & 31);
      *reinterpret_cast<float4*>(&S[kk * LDS_STRIDE + e]) = R.v[u];
    }
  }
}

template <int AMODE, int BMODE>
__global__ __launch_bounds__(NT) void gemm_generic_kernel(const GemmArgs args) {
  int local;
  const GemmGroup& G = args.g[group_of_block(args, local)];
  TileCtx T;
  if (!tile_ctx(G, local, T)) return;
  const int64_t offA = (int64_t)T.batch * G.bs_a, offB = (int64_t)T.batch * G.bs_b;
  const int64_t seg = G.seg_rows > 0 ? T.i0 / G.seg_rows : 0;

  // one LDS object: A and B tiles, reused as the [64][CS] epilogue image
  __shared__ __attribute__((aligned(16))) float sm[2 * BK * LDS_STRIDE];
  static_assert(2 * BK * LDS_STRIDE >= 64 * CS, "epilogue image does not fit");
  float* const As = sm;
  float* const Bs = sm + BK * LDS_STRIDE;
  constexpr int SA = AMODE == MODE_RK ? LDS_STRIDE_T : LDS_STRIDE;
  constexpr int SB = BMODE == MODE_RK ? LDS_STRIDE_T : LDS_STRIDE;

  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int wm = wave >> 1, wn = wave & 1;

  RngSnap rs{0, 0};
  const float p = args.drop_p;
  const float inv_keep = p < 1.f ? 1.f / (1.f - p) : 0.f;
  if (p > 0.f && args.rng) rs = *args.rng;
  if (args.rng_advance && blockIdx.x == 0 && threadIdx.x == 0) args.rng_advance[1] += 1;   // see launch_gemm

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const bool want_db = (G.epi & EPI_PARTIAL) && T.part_db != nullptr && T.j0 == 0;
  float dbsum = 0.f;

  for (int si = 0; si < G.src_count; ++si) {
    const GemmSrc& S = args.s[G.src_begin + si];
    int kbeg = 0, kend = S.K;
    if (G.epi & EPI_PARTIAL) {
      kbeg = T.split * G.kchunk;
      kend = min(S.K, kbeg + G.kchunk);
    }
    if (kbeg >= kend) continue;
    const int ntk = (kend - kbeg + BK - 1) / BK;
    TileRegs ra, rb;
    load_tile<AMODE>(ra, S.a, offA + seg * S.a.seg_stride, T.i0, G.M, kbeg, kend);
    load_tile<BMODE>(rb, S.b, offB + seg * S.b.seg_stride, T.j0, G.N, kbeg, kend);
    for (int kt = 0; kt < ntk; ++kt) {
      __syncthreads();
      store_tile<AMODE>(ra, As);
      store_tile<BMODE>(rb, Bs);
      __syncthreads();
      if (kt + 1 < ntk) {
        const int kn = kbeg + (kt + 1) * BK;
        load_tile<AMODE>(ra, S.a, offA + seg * S.a.seg_stride, T.i0, G.M, kn, kend);
        load_tile<BMODE>(rb, S.b, offB + seg * S.b.seg_stride, T.j0, G.N, kn, kend);
      }
      if (want_db && t < BM) {
#pragma unroll 8
        for (int kk = 0; kk < BK; ++kk) dbsum += As[kk * SA + t];
      }
      const float* ap = As + (16 * h) * SA + wm * 64 + c;
      const float* bp = Bs + (16 * h) * SB + wn * 64 + c;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const float a0 = ap[s * SA], a1 = ap[s * SA + 32];
        const float b0 = bp[s * SB], b1 = bp[s * SB + 32];
        acc[0][0] = mfma32(a0, b0, acc[0][0]);
        acc[0][1] = mfma32(a0, b1, acc[0][1]);
        acc[1][0] = mfma32(a1, b0, acc[1][0]);
        acc[1][1] = mfma32(a1, b1, acc[1][1]);
      }
    }
  }
  if (want_db && t < BM && T.i0 + t < G.M) T.part_db[(int64_t)T.split * G.M + T.i0 + t] = dbsum * G.alpha;
  epilogue(G, T, acc, sm, rs, p, inv_keep, wm, wn, h, c);
}

// ------------------------------------------------------------------ small split-K slabs
// The weight gradients of the B-row tail layers that are not LDS-DMA-able (C x H
// classifier output, 1 x H gates, per-head value biases: odd or unaligned
// extents) are a few thousand outputs of <= 64-row dot products.  As 128 x 128
// generic tiles they cost a tile's whole prologue / epilogue chain each (18 us
// for ~0.1 MFLOP at C2); here one thread computes one slab element
// C[split][i][j] = alpha sum_{k in split} A(i, k) B(k, j) (A, B stored [k][e]),
// j == N standing for the bias-row slab part_db[split][i] = alpha sum_k A(i, k),
// with its rows' loads 8 at a time in flight.  Same fixed summation order per
// slab every call (deterministic); the split-K reduce then sums the slabs.
struct SmallSlabArgs {
  GemmGroup g[GEMM_MAX_GROUPS];
  GemmSrc s[GEMM_MAX_GROUPS];
  int32_t off[GEMM_MAX_GROUPS + 1];   // first thread of each group (1-D grid)
  int32_t ngroups;
};

// 8 lanes per slab element: lane q of the group takes rows k0 + q, k0 + q + 8, ... (all
// its loads in flight at once), the 8 partial sums are combined by xor shuffles in a
// fixed order.
__global__ __launch_bounds__(256) void small_slab_kernel(const SmallSlabArgs a) {
  const int gtid = blockIdx.x * 256 + threadIdx.x;
  const int tid = gtid >> 3, q = gtid & 7;
  const bool live = tid < a.off[a.ngroups];
  int gi = 0;
  for (int i = 1; i < a.ngroups; ++i)
    if (tid >= a.off[i]) gi = i;
  const GemmGroup& G = a.g[gi];
  const GemmSrc& S = a.s[gi];
  const int ncol = G.N + (G.part_db ? 1 : 0);
  int r = live ? tid - a.off[gi] : 0;
  const int j = r % ncol; r /= ncol;
  const int i = r % G.M; r /= G.M;
  const int split = r % G.nsplit;
  const int batch = r / G.nsplit;
  const int k0 = split * G.kchunk, k1 = min(S.K, k0 + G.kchunk);
  const bool bias = j == G.N;
  const float* ap = S.a.ptr + (int64_t)batch * G.bs_a + i;
  const float* bp = S.b.ptr + (int64_t)batch * G.bs_b + min(j, G.N - 1);   // (the bias column reads column N - 1, unused)
  constexpr int MAXR = 256 / 8;   // kchunk <= 256 (job_small_slab)
  // Unconditional loads from clamped rows, eight per step, the row guards applied in the sum (a
  // guarded load compiled to a branch that waited for each load in turn)
  float av[MAXR], bv[MAXR];
#pragma unroll
  for (int u0 = 0; u0 < MAXR; u0 += 8) {
    if (k0 + 8 * u0 >= k1) break;   // (uniform per group of 8 lanes: a bound, not a branch on data)
#pragma unroll
    for (int u = u0; u < u0 + 8; ++u) {
      const int kk = min(k0 + q + 8 * u, k1 - 1);
      const int ka = S.a.row_div == 1 ? kk : kk / S.a.row_div;
      const int kb = S.b.row_div == 1 ? kk : kk / S.b.row_div;
      av[u] = ap[(int64_t)ka * S.a.ld];
      bv[u] = bp[(int64_t)kb * S.b.ld];
    }
  }
  float acc = 0.f;
#pragma unroll
  for (int u = 0; u < MAXR; ++u) {
    if (k0 + 8 * u >= k1) break;
    const bool in = live && k0 + q + 8 * u < k1;
    acc = fmaf(in ? av[u] : 0.f, in ? (bias ? 1.f : bv[u]) : 0.f, acc);
  }
  acc = sum8(acc);
  if (!live || q != 0) return;
  if (bias)
    G.part_db[((int64_t)batch * G.nsplit + split) * G.M + i] = acc * G.alpha;
  else
    G.C[(((int64_t)batch * G.nsplit + split) * G.M + i) * G.N + j] = acc * G.alpha;
}

bool job_small_slab(const GemmJob& J, int amode, int bmode) {
  const GemmGroup& g = J.g;
  if (amode != MODE_KR || bmode != MODE_KR || J.nsrc != 1 || !(g.epi & EPI_PARTIAL)) return false;
  if (g.seg_rows > 0 || J.src[0].a.seg_stride || J.src[0].b.seg_stride) return false;
  const int64_t n = (int64_t)(g.nbatch < 1 ? 1 : g.nbatch) * g.nsplit * g.M * (g.N + 1);
  return n <= (1 << 20) && g.kchunk <= 256;
}

// ------------------------------------------------------------------ split-K reduce
struct ReduceArgs {
  ReduceJob j[48];
  int32_t njobs;
};

// Block: 64 float4 columns (256 outputs) x 4 split-groups; a thread sums the
// splits sg, sg+4, ... with 4 loads in flight, then the 4 group sums are
// combined in a fixed order (deterministic).
__global__ __launch_bounds__(256) void partial_reduce_kernel(const ReduceArgs a) {
  ReduceJob J = a.j[blockIdx.y];
  const int64_t MN = (int64_t)J.M * J.N;
  const int batch = blockIdx.z;
  if (batch >= J.nbatch) return;
  J.part += (int64_t)batch * J.nsplit * MN;
  if (J.part_db) J.part_db += (int64_t)batch * J.nsplit * J.M;
  J.out += (int64_t)batch * J.bs_out;
  if (J.db) J.db += (int64_t)batch * J.bs_db;
  __shared__ f32x4 red[4][64];
  const int el = threadIdx.x & 63, sg = threadIdx.x >> 6;
  const bool v4 = (MN % 4) == 0 && ((uintptr_t)J.part & 15) == 0;
  const int64_t n4 = v4 ? MN / 4 : MN;        // vector (or scalar) columns
  const bool out_al = ((uintptr_t)J.out & 15) == 0;
  for (int64_t c0 = (int64_t)blockIdx.x * 64; c0 < n4; c0 += (int64_t)gridDim.x * 64) {
    const int64_t col = c0 + el;
    f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, s2 = s0, s3 = s0;
    if (col < n4) {
      if (v4) {
        const f32x4* base = reinterpret_cast<const f32x4*>(J.part) + col;
        const int64_t st = MN / 4;
        int k = sg;
#pragma unroll 4
        for (; k + 12 < J.nsplit; k += 16) {
          s0 += base[(int64_t)k * st];
          s1 += base[(int64_t)(k + 4) * st];
          s2 += base[(int64_t)(k + 8) * st];
          s3 += base[(int64_t)(k + 12) * st];
        }
        for (; k < J.nsplit; k += 4) s0 += base[(int64_t)k * st];
      } else {
        for (int k = sg; k < J.nsplit; k += 4) s0[0] += J.part[(int64_t)k * MN + col];
      }
    }
    __syncthreads();
    red[sg][el] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    if (sg == 0 && col < n4) {
      const f32x4 r = (red[0][el] + red[1][el]) + (red[2][el] + red[3][el]);
      if (!v4) J.out[col] = r[0];
      else if (out_al) reinterpret_cast<f32x4*>(J.out)[col] = r;
      else {
        float* o = J.out + col * 4;
        o[0] = r[0]; o[1] = r[1]; o[2] = r[2]; o[3] = r[3];
      }
    }
  }
  // bias gradient: row sums of the slabs' part_db, on the dedicated last block
  // (launch_reduce adds it past the column blocks).  Same split-group layout as
  // the columns: 64 rows x 4 groups, 4 partial sums per thread (16 loads in
  // flight), combined in a fixed order => deterministic.
  // (nsplit == 0: a gradient that is exactly zero, e.g. query_proj / key_proj at Lk = 1,
  // single_key.hip; the column blocks above wrote zeros, this block zeroes the bias)
  if (J.db && (J.part_db || J.nsplit == 0) && blockIdx.x == gridDim.x - 1) {
    __shared__ float redb[4][64];
    for (int i0 = 0; i0 < J.M; i0 += 64) {
      const int i = i0 + el;
      float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
      if (i < J.M) {
        int k = sg;
#pragma unroll 4
        for (; k + 12 < J.nsplit; k += 16) {
          s0 += J.part_db[(int64_t)k * J.M + i];
          s1 += J.part_db[(int64_t)(k + 4) * J.M + i];
          s2 += J.part_db[(int64_t)(k + 8) * J.M + i];
          s3 += J.part_db[(int64_t)(k + 12) * J.M + i];
        }
        for (; k < J.nsplit; k += 4) s0 += J.part_db[(int64_t)k * J.M + i];
      }
      __syncthreads();
      redb[sg][el] = (s0 + s1) + (s2 + s3);
      __syncthreads();
      if (sg == 0 && i < J.M) J.db[i] = (redb[0][el] + redb[1][el]) + (redb[2][el] + redb[3][el]);
    }
  }
}

// ------------------------------------------------------------------ input mask + dropout
// X'_m = X_m * mask[:, m] * keep / (1-p) for every modality in one launch
// (blockIdx.x = modality, blockIdx.y = chunk of 256 Philox blocks); a thread handles the 8
// elements of one Philox block.  Workgroups blockIdx.x >= n draw the attention keep words of
// pair blockIdx.x - n instead (a.kw): VALU work interleaved with the HBM-bound mask rows.
__global__ __launch_bounds__(256) void mask_dropout_rows_kernel(const MaskDropArgs a) {
  const int m = blockIdx.x;
  const bool drop = a.p > 0.f && (a.rng != nullptr || a.rng_live != nullptr);
  RngSnap rs{0, 0};
  {
    // live state (the hybrid forward) or a snapshot: a uniform pointer either way
    const uint64_t* src = a.rng_live ? a.rng_live : (drop ? reinterpret_cast<const uint64_t*>(a.rng) : nullptr);
    if (src) {
      rs.seed = src[0];
      rs.offset = src[1];
    }
  }
  const uint32_t thr = p16(a.p);
  if (m >= a.n) {
    // keep words, as attn_keep_words_kernel: bit j of word kt of row (b, head, q) keeps element
    // row Lk + 32 kt + j of the pair's stream
    const MaskDropArgs::KeepWordJob& K = a.kw[m - a.n];
    const uint32_t nkt = K.Lk >> 5;
    const uint32_t nwords = (uint32_t)a.B * (uint32_t)a.heads * K.Lq * nkt;
    for (uint32_t i = blockIdx.y * 256u + threadIdx.x; i < nwords; i += gridDim.y * 256u) {
      const uint32_t row = (nkt & (nkt - 1)) == 0 ? i >> (31 - __builtin_clz(nkt)) : i / nkt;
      const uint32_t kt = i - row * nkt;
      const uint64_t blk0 = ((uint64_t)row * K.Lk + 32 * kt) >> 3;
      uint32_t bits = 0;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const uint4 rr = philox_block(rs, K.site, blk0 + g);
        const uint32_t wv[4] = {rr.x, rr.y, rr.z, rr.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          bits |= ((wv[k] & 0xFFFFu) >= thr ? 1u : 0u) << (8 * g + 2 * k);
          bits |= ((wv[k] >> 16) >= thr ? 1u : 0u) << (8 * g + 2 * k + 1);
        }
      }
      K.bits[(uint64_t)row * K.kw_ld + kt] = bits;
    }
    return;
  }
  const MaskDropJob& J = a.j[m];
  const int64_t n = J.rows * J.D;
  const float inv_keep = a.p < 1.f ? 1.f / (1.f - a.p) : 0.f;
  const int D = J.D, L = J.L, M = a.M;
  for (int64_t blk = (int64_t)blockIdx.y * blockDim.x + threadIdx.x; blk * 8 < n;
       blk += (int64_t)gridDim.y * blockDim.x) {
    uint4 r = make_uint4(0, 0, 0, 0);
    if (drop) r = philox_block(rs, J.site, (uint64_t)blk);
    const int64_t base = blk * 8;
    if (J.vec && base + 8 <= n) {
      const float sc = a.mask[(base / D / L) * M + m];
      const float4 v0 = *reinterpret_cast<const float4*>(J.x + base);
      const float4 v1 = *reinterpret_cast<const float4*>(J.x + base + 4);
      float o[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float v = o[e] * sc;
        if (drop) v = keep_from(r, e, thr) ? v * inv_keep : 0.f;
        o[e] = v;
      }
      if (J.outb) {
        bf16x8 pk;
#pragma unroll
        for (int e = 0; e < 8; ++e) pk[e] = (__bf16)o[e];
        *reinterpret_cast<bf16x8*>(reinterpret_cast<__bf16*>(J.out) + base) = pk;
      } else {
        *reinterpret_cast<float4*>(J.out + base) = make_float4(o[0], o[1], o[2], o[3]);
        *reinterpret_cast<float4*>(J.out + base + 4) = make_float4(o[4], o[5], o[6], o[7]);
      }
    } else {
      for (int e = 0; e < 8 && base + e < n; ++e) {
        const int64_t idx = base + e;
        float v = J.x[idx] * a.mask[(idx / D / L) * M + m];
        if (drop) v = keep_from(r, e, thr) ? v * inv_keep : 0.f;
        if (J.outb) reinterpret_cast<__bf16*>(J.out)[idx] = (__bf16)v;
        else J.out[idx] = v;
      }
    }
  }
  // the call's rng snapshot (after the loop: a store ahead of the Philox key's SGPR
  // constraint made the backend fail to keep the key uniform)
  if (a.rng_snap && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) *a.rng_snap = rs;
}

// LDS-DMA eligibility of one operand: 16-B aligned rows (and batch strides),
// plus an extent % 4 == 0 along the contiguous axis for KR operands.
bool dma_ok(const Operand& op, int mode, int eext, int bstride, int nbatch) {
  if (!op.vec || op.row_div < 1) return false;
  if (nbatch > 1 && (bstride % 4) != 0) return false;
  if (mode == MODE_KR && (eext % 4) != 0) return false;
  return true;
}

bool job_fast(const GemmJob& J, int amode, int bmode) {
  const GemmGroup& g = J.g;
  const int nb = g.nbatch < 1 ? 1 : g.nbatch;
  if ((g.epi & EPI_PARTIAL) && (g.kchunk % 32) != 0) return false;
  for (int s = 0; s < J.nsrc; ++s) {
    const GemmSrc& src = J.src[s];
    if ((src.K % 4) != 0 || !dma_ok(src.a, amode, g.M, g.bs_a, nb) || !dma_ok(src.b, bmode, g.N, g.bs_b, nb))
      return false;
  }
  return true;
}

}  // namespace

namespace {

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

bool job_wsr(const GemmJob& J, int amode, int bmode) {
  const GemmGroup& g = J.g;
  if (amode != MODE_RK || (bmode != MODE_RK && bmode != MODE_KR) || J.nsrc != 1 || g.nbatch > 1) return false;
  if (g.epi & ~(EPI_BIAS | EPI_RELU | EPI_DROP | EPI_COLSUM | EPI_ROWSCALE)) return false;
  // The extended forms (row scale, dropout, column sums, B stored [k][n]) are opt-in
  // (MMF_WSR_EPI=1): at C2 they would take the modality projections and dX, 768 row tiles each,
  // which the LDS-DMA kernel runs as one lockstep wave of 3 workgroups per CU in 62 / 59 us; the
  // persistent weight-stationary grid (2 workgroups per CU, 1-2 tiles each: ~24 us per tile per
  // workgroup, its register-resident W^T loaded per workgroup) took 75 / 75 us and the step
  // 0.959-0.972 -> 0.984-0.998 ms (profiles/r06/wsr_epi/).  It pays with many tiles per
  // workgroup (the Q / K projections: 3072 tiles), not here.
  static const bool ext_on = getenv("MMF_WSR_EPI") != nullptr;
  if (!ext_on && (bmode != MODE_RK || (g.epi & ~(EPI_BIAS | EPI_RELU)))) return false;
  // one row scale per 128-row tile (a scalar load); column sums per tile into colsum
  if ((g.epi & EPI_ROWSCALE) && (g.rs_div <= 0 || g.rs_div % BM != 0 || !g.rowscale)) return false;
  if ((g.epi & EPI_COLSUM) && !g.colsum) return false;
  const GemmSrc& s = J.src[0];
  const bool b_ok = bmode == MODE_RK ? (s.b.ld % 4 == 0 && aligned16(s.b.ptr)) : s.b.ld >= g.N;
  return g.N == BN && g.M % BM == 0 && s.K % WSR_DK == 0 && s.K >= WSR_DK && s.K <= 8 * WSR_NKC &&
         s.a.row_div == 1 && s.b.row_div == 1 && s.a.ld % 4 == 0 && aligned16(s.a.ptr) && b_ok &&
         s.a.seg_stride == 0 && s.b.seg_stride == 0 && g.ldc % 4 == 0 && aligned16(g.C);
}

int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

// Every job weight-stationary-eligible with one common K: persistent launches
// of up to GEMM_MAX_GROUPS groups.
hipError_t launch_wsr(const GemmJob* jobs, int njobs, hipStream_t st, uint64_t* rng_advance, int bmode, float drop_p,
                      const RngSnap* rng) {
  for (int done = 0; done < njobs;) {
    GemmArgs args;
    memset(&args, 0, sizeof(args));
    args.amode = MODE_RK;
    args.bmode = bmode;
    args.drop_p = drop_p;
    args.rng = rng;
    args.rng_advance = rng_advance;
    rng_advance = nullptr;
    int ng = 0, items = 0;
    double fl = 0.0, by = 0.0;
    while (done < njobs && ng < GEMM_MAX_GROUPS) {
      GemmGroup g = jobs[done].g;
      g.nbatch = 1;
      g.src_begin = ng;
      g.src_count = 1;
      args.s[ng] = jobs[done].src[0];
      args.tile_off[ng] = items;
      args.g[ng++] = g;
      items += g.M / BM;
      fl += 2.0 * g.M * g.N * jobs[done].src[0].K;
      by += 4.0 * ((double)g.M + g.N) * jobs[done].src[0].K + 4.0 * g.M * g.N;
      ++done;
    }
    args.ngroups = ng;
    const int K = args.s[0].K;
    const int grid = std::min(items, 2 * cu_count());
    const int pr = math_mode();
    bool ext = bmode != MODE_RK;
    for (int i = 0; i < ng; ++i) ext = ext || (args.g[i].epi & ~(EPI_BIAS | EPI_RELU)) != 0;
#define MMF_WSR_LAUNCH(BFV, EXTV, NAME)                                             \
  {                                                                                 \
    ProfLaunch prof_(st, NAME, fl, by);                                             \
    mmf_launch((gemm_wsr_kernel<BFV, EXTV>), dim3(grid), dim3(NT), 0, st, args, items, K); \
  }
    if (ext) {
      if (pr == 2) MMF_WSR_LAUNCH(2, true, "gemm_wsr_kernel<2, true>")
      else if (pr == 1) MMF_WSR_LAUNCH(1, true, "gemm_wsr_kernel<1, true>")
      else MMF_WSR_LAUNCH(0, true, "gemm_wsr_kernel<0, true>")
    } else {
      if (pr == 2) MMF_WSR_LAUNCH(2, false, "gemm_wsr_kernel<2>")
      else if (pr == 1) MMF_WSR_LAUNCH(1, false, "gemm_wsr_kernel<1>")
      else MMF_WSR_LAUNCH(0, false, "gemm_wsr_kernel<0>")
    }
#undef MMF_WSR_LAUNCH
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace

int device_cu_count() { return cu_count(); }

hipError_t launch_gemm(const GemmJob* jobs_in, int njobs, int amode, int bmode, float drop_p,
                       const RngSnap* rng, hipStream_t st, uint64_t* rng_advance) {
  // bf16 outputs: only the LDS-DMA kernel's epilogue writes them (one batch, no split-K)
  for (int i = 0; i < njobs; ++i)
    if ((jobs_in[i].g.epi & EPI_BF16) &&
        (!job_fast(jobs_in[i], amode, bmode) || jobs_in[i].g.nbatch > 1 || (jobs_in[i].g.epi & EPI_PARTIAL)))
      return hipErrorInvalidValue;
  {
    bool wsr = njobs > 0;
    for (int i = 0; i < njobs && wsr; ++i)
      wsr = job_wsr(jobs_in[i], amode, bmode) && jobs_in[i].src[0].K == jobs_in[0].src[0].K && !jobs_in[i].chain;
    if (wsr && getenv("MMF_NO_WSR") == nullptr) return launch_wsr(jobs_in, njobs, st, rng_advance, bmode, drop_p, rng);
  }
  // the tiled launches below take the rng advance on their first launch; a call that
  // ends in small slabs only advances with a launch of its own
  struct AdvanceLeft {
    uint64_t*& adv;
    hipStream_t st;
    hipError_t finish(hipError_t e) { return (e == hipSuccess && adv) ? launch_rng_advance(adv, st) : e; }
  } left{rng_advance, st};
  // Small, non-DMA-able split-K slabs: one thread per slab element, all in one launch
  // (the remaining jobs go through the tiled kernels below).
  std::vector<GemmJob> rest;
  {
    SmallSlabArgs sa;
    memset(&sa, 0, sizeof(sa));
    int total = 0;
    double fl = 0.0, by = 0.0;
    auto flush = [&]() -> hipError_t {
      if (sa.ngroups == 0) return hipSuccess;
      sa.off[sa.ngroups] = total;
      ProfLaunch prof_(st, "small_slab_kernel", fl, by);
      mmf_launch(small_slab_kernel, dim3((8 * total + 255) / 256), dim3(256), 0, st, sa);
      memset(&sa, 0, sizeof(sa));
      total = 0; fl = by = 0.0;
      return hipGetLastError();
    };
    for (int i = 0; i < njobs; ++i) {
      const GemmJob& J = jobs_in[i];
      if (job_fast(J, amode, bmode) || !job_small_slab(J, amode, bmode) || J.chain) {
        rest.push_back(J);
        continue;
      }
      GemmGroup g = J.g;
      if (g.nbatch < 1) g.nbatch = 1;
      sa.g[sa.ngroups] = g;
      sa.s[sa.ngroups] = J.src[0];
      sa.off[sa.ngroups] = total;
      total += g.nbatch * g.nsplit * g.M * (g.N + (g.part_db ? 1 : 0));
      fl += 2.0 * g.nbatch * g.M * g.N * J.src[0].K;
      by += 4.0 * g.nbatch * ((double)g.M + g.N) * J.src[0].K + 4.0 * g.nbatch * g.nsplit * g.M * g.N;
      if (++sa.ngroups == GEMM_MAX_GROUPS)
        if (hipError_t e = flush()) return e;
    }
    if (hipError_t e = flush()) return e;
    if (rest.empty()) return left.finish(hipSuccess);
    jobs_in = rest.data();
    njobs = (int)rest.size();
  }
  // Chained jobs (GemmJob::chain) ride in their parent's launch when the shapes allow (the same
  // rows, one column tile each, the parent's fp32 output as the chained job's RK A operand, both on
  // the LDS-DMA kernel); any other chained job runs as a launch of its own after this call's.
  auto chain_ok = [&](const GemmJob& J) {
    const GemmJob* C = J.chain;
    if (!C || amode != MODE_RK) return false;
    const GemmGroup &a = J.g, &b = C->g;
    if (!job_fast(J, amode, bmode) || !job_fast(*C, amode, bmode)) return false;
    if ((a.epi & (EPI_PARTIAL | EPI_BF16)) || (b.epi & EPI_PARTIAL) || a.nbatch > 1 || b.nbatch > 1) return false;
    if (a.N > BN || b.N > BN || b.M != a.M || C->nsrc != 1) return false;
    const GemmSrc& x = C->src[0];
    return x.a.ptr == a.C && x.a.ld == a.ldc && x.K == a.N && x.a.row_div == 1 && x.a.seg_stride == 0;
  };
  std::vector<GemmJob> later;
  for (int i = 0; i < njobs; ++i)
    if (jobs_in[i].chain && !chain_ok(jobs_in[i])) {
      later.push_back(*jobs_in[i].chain);
      later.back().chain = nullptr;
    }
  // The jobs of one call are independent outputs, so they may be launched in
  // any order: longest contraction per tile first (the first-dispatched blocks
  // carry the most work), fast-path jobs packed together.
  std::vector<int> order(njobs);
  std::vector<double> work(njobs);
  for (int i = 0; i < njobs; ++i) {
    order[i] = i;
    const GemmGroup& g = jobs_in[i].g;
    const bool partial = (g.epi & EPI_PARTIAL) != 0;
    double kk = 0.0;
    for (int s = 0; s < jobs_in[i].nsrc; ++s) kk += jobs_in[i].src[s].K;
    work[i] = partial ? (double)g.kchunk : kk;
  }
  // With the interleave on, jobs of equal work are further clustered by their
  // most-shared operand (the pointer that the most jobs of this call read), so
  // one launch holds the groups that can share it in L2.
  const int ilv_mode = gemm_interleave_mode();
  bool any_partial = false;
  for (int i = 0; i < njobs; ++i) any_partial |= (jobs_in[i].g.epi & EPI_PARTIAL) != 0;
  const bool ilv_on = ilv_mode == 2 || (ilv_mode == 1 && !any_partial);
  std::vector<uintptr_t> share(njobs, 0);
  if (ilv_on) {
    std::map<uintptr_t, int> uses;
    for (int i = 0; i < njobs; ++i) {
      ++uses[(uintptr_t)jobs_in[i].src[0].a.ptr];
      ++uses[(uintptr_t)jobs_in[i].src[0].b.ptr];
    }
    for (int i = 0; i < njobs; ++i) {
      const uintptr_t a = (uintptr_t)jobs_in[i].src[0].a.ptr, b = (uintptr_t)jobs_in[i].src[0].b.ptr;
      share[i] = uses[b] > uses[a] ? b : a;
    }
  }
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
    const bool fx = job_fast(jobs_in[x], amode, bmode), fy = job_fast(jobs_in[y], amode, bmode);
    if (fx != fy) return fx;
    if (work[x] != work[y]) return work[x] > work[y];
    return share[x] < share[y];
  });
  int done = 0;
  while (done < njobs) {
    GemmArgs args;
    memset(&args, 0, sizeof(args));
    args.amode = amode;
    args.bmode = bmode;
    args.drop_p = drop_p;
    args.rng = rng;
    args.rng_advance = rng_advance;
    rng_advance = nullptr;
    int ng = 0, ns = 0, max_blocks = 0;
    // chained groups go after the launch's own groups (they own no blocks)
    int nch = 0, nch_src = 0, ch_parent[GEMM_MAX_GROUPS];
    const GemmJob* ch_job[GEMM_MAX_GROUPS];
    // one launch = consecutive jobs of the same kernel flavour
    const bool fast = job_fast(jobs_in[order[done]], amode, bmode);
    while (done < njobs && ng + nch < GEMM_MAX_GROUPS) {
      const GemmJob& J = jobs_in[order[done]];
      if (J.nsrc > GEMM_MAX_SRCS) return hipErrorInvalidValue;
      const bool ch = J.chain && chain_ok(J);
      if (ng + nch + (ch ? 2 : 1) > GEMM_MAX_GROUPS) break;
      if (ns + nch_src + J.nsrc + (ch ? J.chain->nsrc : 0) > GEMM_MAX_SRCS) break;
      if (job_fast(J, amode, bmode) != fast) break;
      GemmGroup g = J.g;
      if (g.nbatch < 1) g.nbatch = 1;
      g.src_begin = ns;
      g.src_count = J.nsrc;
      g.chain = 0;
      const bool partial = (g.epi & EPI_PARTIAL) != 0;
      for (int s = 0; s < J.nsrc; ++s) args.s[ns++] = J.src[s];
      const int tiles = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN) * (partial ? g.nsplit : 1) * g.nbatch;
      if (ch) {
        ch_parent[nch] = ng;
        ch_job[nch++] = J.chain;
        nch_src += J.chain->nsrc;
      }
      args.tile_off[ng] = max_blocks;
      args.g[ng++] = g;
      max_blocks += tiles;
      ++done;
    }
    if (ng == 0) return hipErrorInvalidValue;
    for (int k = 0; k < nch; ++k) {
      GemmGroup g = ch_job[k]->g;
      g.nbatch = 1;
      g.src_begin = ns;
      g.src_count = ch_job[k]->nsrc;
      g.chain = 0;
      for (int s = 0; s < ch_job[k]->nsrc; ++s) args.s[ns++] = ch_job[k]->src[s];
      args.tile_off[ng + k] = max_blocks;   // (no block maps to a chained group)
      args.g[ng + k] = g;
      args.g[ch_parent[k]].chain = ng + k + 1;
    }
    args.ngroups = ng + nch;
    if (ilv_on && ng > 1 && nch == 0) {
      const int T = args.tile_off[1];
      bool even = T > 0 && T % 8 == 0;
      for (int gi = 1; gi < ng && even; ++gi)
        even = (gi + 1 < ng ? args.tile_off[gi + 1] : max_blocks) - args.tile_off[gi] == T;
      args.ilv = even ? 1 : 0;
    }
    if (max_blocks > 0) {
      dim3 grid(max_blocks, 1);
      double fl = 0.0, by = 0.0;
      for (int gi = 0; gi < args.ngroups; ++gi) {
        const GemmGroup& g = args.g[gi];
        for (int si = g.src_begin; si < g.src_begin + g.src_count; ++si) {
          fl += 2.0 * g.M * g.N * args.s[si].K * g.nbatch;
          by += 4.0 * ((double)g.M + g.N) * args.s[si].K * g.nbatch;
        }
        by += 4.0 * g.M * g.N * g.nbatch;
      }
      static const char* const kLdsName[12] = {
          "gemm_lds_kernel<0, 0, 16, 3, 0>", "gemm_lds_kernel<0, 1, 16, 3, 0>",
          "gemm_lds_kernel<1, 0, 16, 3, 0>", "gemm_lds_kernel<1, 1, 16, 3, 0>",
          "gemm_lds_kernel<0, 0, 16, 3, 1>", "gemm_lds_kernel<0, 1, 16, 3, 1>",
          "gemm_lds_kernel<1, 0, 16, 3, 1>", "gemm_lds_kernel<1, 1, 16, 3, 1>",
          "gemm_lds_kernel<0, 0, 16, 3, 2>", "gemm_lds_kernel<0, 1, 16, 3, 2>",
          "gemm_lds_kernel<1, 0, 16, 3, 2>", "gemm_lds_kernel<1, 1, 16, 3, 2>"};
      const int pr = math_mode();
      static const char* const kGenName[4] = {"gemm_generic_kernel<0, 0>", "gemm_generic_kernel<0, 1>",
                                              "gemm_generic_kernel<1, 0>", "gemm_generic_kernel<1, 1>"};
      const int flavour = (amode == MODE_KR ? 2 : 0) + (bmode == MODE_KR ? 1 : 0);
      static const char* const kChainName[6] = {
          "gemm_lds_chain_kernel<0, 0, 16, 3, 0>", "gemm_lds_chain_kernel<0, 1, 16, 3, 0>",
          "gemm_lds_chain_kernel<0, 0, 16, 3, 1>", "gemm_lds_chain_kernel<0, 1, 16, 3, 1>",
          "gemm_lds_chain_kernel<0, 0, 16, 3, 2>", "gemm_lds_chain_kernel<0, 1, 16, 3, 2>"};
      ProfLaunch prof_(st, nch ? kChainName[(bmode == MODE_KR ? 1 : 0) + 2 * pr]
                               : fast ? kLdsName[flavour + 4 * pr] : kGenName[flavour], fl, by);
#define MMF_LAUNCH_CFG2(DKV, NSV, BFV)                                                              \
      if (amode == MODE_RK && bmode == MODE_RK)                                                     \
        mmf_launch((gemm_lds_kernel<MODE_RK, MODE_RK, DKV, NSV, BFV>), grid, dim3(NT), 0, st, args); \
      else if (amode == MODE_RK && bmode == MODE_KR)                                                \
        mmf_launch((gemm_lds_kernel<MODE_RK, MODE_KR, DKV, NSV, BFV>), grid, dim3(NT), 0, st, args); \
      else if (amode == MODE_KR && bmode == MODE_KR)                                                \
        mmf_launch((gemm_lds_kernel<MODE_KR, MODE_KR, DKV, NSV, BFV>), grid, dim3(NT), 0, st, args); \
      else                                                                                          \
        mmf_launch((gemm_lds_kernel<MODE_KR, MODE_RK, DKV, NSV, BFV>), grid, dim3(NT), 0, st, args);
#define MMF_LAUNCH_CFG(DKV, NSV)                                                                    \
      if (pr == 2) { MMF_LAUNCH_CFG2(DKV, NSV, 2) } else if (pr == 1) { MMF_LAUNCH_CFG2(DKV, NSV, 1) } \
      else { MMF_LAUNCH_CFG2(DKV, NSV, 0) }
#define MMF_LAUNCH(KERNEL)                                                                 \
      if (amode == MODE_RK && bmode == MODE_RK)                                            \
        mmf_launch((KERNEL<MODE_RK, MODE_RK>), grid, dim3(NT), 0, st, args);       \
      else if (amode == MODE_RK && bmode == MODE_KR)                                       \
        mmf_launch((KERNEL<MODE_RK, MODE_KR>), grid, dim3(NT), 0, st, args);       \
      else if (amode == MODE_KR && bmode == MODE_KR)                                       \
        mmf_launch((KERNEL<MODE_KR, MODE_KR>), grid, dim3(NT), 0, st, args);       \
      else                                                                                 \
        mmf_launch((KERNEL<MODE_KR, MODE_RK>), grid, dim3(NT), 0, st, args);
      if (nch) {
        // (chain_ok: the LDS-DMA kernel, A row-major)
        if (bmode == MODE_KR) {
          if (pr == 2) mmf_launch((gemm_lds_chain_kernel<MODE_RK, MODE_KR, 16, 3, 2>), grid, dim3(NT), 0, st, args);
          else if (pr == 1) mmf_launch((gemm_lds_chain_kernel<MODE_RK, MODE_KR, 16, 3, 1>), grid, dim3(NT), 0, st, args);
          else mmf_launch((gemm_lds_chain_kernel<MODE_RK, MODE_KR, 16, 3, 0>), grid, dim3(NT), 0, st, args);
        } else {
          if (pr == 2) mmf_launch((gemm_lds_chain_kernel<MODE_RK, MODE_RK, 16, 3, 2>), grid, dim3(NT), 0, st, args);
          else if (pr == 1) mmf_launch((gemm_lds_chain_kernel<MODE_RK, MODE_RK, 16, 3, 1>), grid, dim3(NT), 0, st, args);
          else mmf_launch((gemm_lds_chain_kernel<MODE_RK, MODE_RK, 16, 3, 0>), grid, dim3(NT), 0, st, args);
        }
      } else if (fast) {
        // (DK, ring depth) = (16, 3): measured best of (16|32) x (2|3|4) at C2
        // (profiles/tune_gemm_cfg.sh)
        MMF_LAUNCH_CFG(MMF_GEMM_DK, MMF_GEMM_NS)
      } else {
        MMF_LAUNCH(gemm_generic_kernel)
      }
#undef MMF_LAUNCH
#undef MMF_LAUNCH_CFG
#undef MMF_LAUNCH_CFG2
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    } else if (args.rng_advance) {
      rng_advance = args.rng_advance;   // nothing launched: the next launch (or finish) takes it
    }
  }
  if (!later.empty())
    if (hipError_t e = launch_gemm(later.data(), (int)later.size(), amode, bmode, drop_p, rng, st, nullptr))
      return e;
  return left.finish(hipSuccess);
}

// fp32 -> bf16 copies of small tensors (the weights of a bf16-operand GEMM), round to nearest
// even: blockIdx.y = tensor, float4 -> 4 bf16 per thread step
__global__ __launch_bounds__(256) void cvt_bf16_kernel(const CvtArgs a) {
  const int q = blockIdx.y;
  const float* s = a.src[q];
  __bf16* d = a.dst[q];
  const int64_t n = a.n[q];
  if (float* d32 = a.dst32[q]) {   // (fp32 copy: the concatenated Q/K bias vectors)
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) d32[i] = s[i];
    return;
  }
  for (int64_t i = 4 * ((int64_t)blockIdx.x * 256 + threadIdx.x); i < n; i += 4 * (int64_t)gridDim.x * 256) {
    if (i + 4 <= n) {
      const float4 v = *reinterpret_cast<const float4*>(s + i);
      d[i] = (__bf16)v.x; d[i + 1] = (__bf16)v.y; d[i + 2] = (__bf16)v.z; d[i + 3] = (__bf16)v.w;
    } else {
      for (int64_t e = i; e < n; ++e) d[e] = (__bf16)s[e];
    }
  }
}

hipError_t launch_cvt_bf16(const CvtArgs& a, hipStream_t st) {
  if (a.count <= 0) return hipSuccess;
  if (a.count > CVT_MAX) return hipErrorInvalidValue;
  int64_t mx = 0;
  double by = 0.0;
  for (int i = 0; i < a.count; ++i) {
    if (!a.dst32[i] && ((uintptr_t)a.src[i] & 15) != 0) return hipErrorInvalidValue;
    mx = std::max<int64_t>(mx, a.dst32[i] ? a.n[i] : a.n[i] / 4);   // elements (copy) / float4s per thread pass
    by += (a.dst32[i] ? 8.0 : 6.0) * a.n[i];
  }
  const int gx = (int)std::min<int64_t>((mx + 255) / 256, 64);
  ProfLaunch prof_(st, "cvt_bf16_kernel", 0.0, by);
  mmf_launch(cvt_bf16_kernel, dim3(std::max(gx, 1), a.count), dim3(256), 0, st, a);
  return hipGetLastError();
}

// bf16 operands in HBM: 16-B aligned rows (ld % 8), k a multiple of 8 along an RK operand's rows,
// the e extent a multiple of 8 along a KR operand's rows; split-K slabs of whole 32-k tiles
bool gemm_b16_ok(const GemmJob& J, int amode, int bmode) {
  const GemmGroup& g = J.g;
  if (g.nbatch > 1 || g.seg_rows > 0) return false;
  if ((g.epi & EPI_PARTIAL) && (g.kchunk % 32 != 0 || g.nsplit < 1)) return false;
  if ((g.epi & EPI_PARTIAL) && g.part_db && amode != MODE_KR) return false;   // (part_db shares colsum's slot)
  for (int s = 0; s < J.nsrc; ++s) {
    const GemmSrc& x = J.src[s];
    const Operand* ops[2] = {&x.a, &x.b};
    const int modes[2] = {amode, bmode}, ext[2] = {g.M, g.N};
    for (int i = 0; i < 2; ++i) {
      const Operand* o = ops[i];
      if (o->row_div != 1 || o->seg_stride != 0 || o->ld % 8 != 0 || ((uintptr_t)o->ptr & 15) != 0) return false;
      if (modes[i] == MODE_KR ? (ext[i] % 8 != 0 || ext[i] < 8) : (x.K % 8 != 0 || x.K < 8)) return false;
    }
  }
  return true;
}

// gemm_wsr_b16_kernel's jobs: one source, bf16 output (+ bias), whole 128-row tiles and 128-column
// groups (the wait counts assume every store is issued), 32 | K <= 256
bool job_wsr_b16(const GemmJob& J) {
  const GemmGroup& g = J.g;
  if (J.nsrc != 1 || g.nbatch > 1 || g.seg_rows > 0 || !(g.epi & EPI_BF16) || (g.epi & ~(EPI_BIAS | EPI_BF16))) return false;
  const GemmSrc& s = J.src[0];
  // (N <= 256: wider outputs -- the concatenated Q / K blocks -- would re-read X per 128-column group;
  // the LDS-DMA kernel's XCD-aware tile order reads it once)
  return g.M % BM == 0 && g.N % BN == 0 && g.N <= 2 * BN && s.K % 32 == 0 && s.K >= 32 && s.K <= 16 * WSR16_NKS &&
         s.a.row_div == 1 &&
         s.b.row_div == 1 && s.a.seg_stride == 0 && s.a.ld % 8 == 0 && s.b.ld % 8 == 0 && aligned16(s.a.ptr) &&
         aligned16(s.b.ptr) && g.ldc % 4 == 0 && ((uintptr_t)g.C & 7) == 0;
}

hipError_t launch_wsr_b16(const GemmJob* jobs, int njobs, hipStream_t st) {
  // 8-wave workgroups over 256-column groups when every job is 256 wide (MMF_WSR16_W4=1: 4 waves
  // over 128-column groups, A/B)
  static const bool w4 = getenv("MMF_WSR16_W4") != nullptr;
  bool w8 = !w4;
  for (int i = 0; i < njobs && w8; ++i) w8 = jobs[i].g.N % (2 * BN) == 0;
  const int cw = w8 ? 2 * BN : BN;
  // every job split into its column groups, adjacent (see the kernel)
  std::vector<GemmJob> parts;
  std::vector<int> first;   // the job's first column group (its X rows counted once)
  for (int i = 0; i < njobs; ++i)
    for (int c0 = 0; c0 < jobs[i].g.N; c0 += cw) {
      first.push_back(c0 == 0);
      GemmJob p = jobs[i];
      p.g.N = cw;
      p.g.C = reinterpret_cast<float*>(reinterpret_cast<__bf16*>(jobs[i].g.C) + c0);
      if (p.g.bias) p.g.bias = jobs[i].g.bias + c0;
      p.src[0].b.ptr = reinterpret_cast<const float*>(reinterpret_cast<const __bf16*>(jobs[i].src[0].b.ptr) +
                                                      (int64_t)c0 * jobs[i].src[0].b.ld);
      parts.push_back(p);
    }
  for (size_t done = 0; done < parts.size();) {
    GemmArgs args;
    memset(&args, 0, sizeof(args));
    args.amode = MODE_RK;
    args.bmode = MODE_RK;
    int ng = 0, items = 0;
    double fl = 0.0, by = 0.0;
    const int K = parts[done].src[0].K;
    while (done < parts.size() && ng < GEMM_MAX_GROUPS && parts[done].src[0].K == K) {
      GemmGroup g = parts[done].g;
      g.nbatch = 1;
      g.src_begin = ng;
      g.src_count = 1;
      args.s[ng] = parts[done].src[0];
      args.tile_off[ng] = items;
      args.g[ng++] = g;
      items += g.M / BM;
      fl += 2.0 * g.M * g.N * K;
      // X rows once per GEMM (the two column groups share them through L2), W, Y in bf16
      by += 2.0 * (first[done] ? (double)g.M * K : 0.0) + 2.0 * g.N * K + 2.0 * g.M * g.N;
      ++done;
    }
    args.ngroups = ng;
    if (w8) {
      // one 8-wave workgroup per CU, a 12-deep ring (96 KB)
      const int grid = std::min(items, cu_count());
      ProfLaunch prof_(st, "gemm_wsr_b16_kernel<12, 8>", fl, by);
      mmf_launch((gemm_wsr_b16_kernel<12, 8>), dim3(grid), dim3(8 * 64), 0, st, args, items, K);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
      continue;
    }
    const int grid = std::min(items, 2 * cu_count());
    // ring depth: 9 tiles (72 KB: two workgroups per CU), MMF_WSR16_NS=6 the first form (A/B)
    const char* ns = getenv("MMF_WSR16_NS");
    if (ns && ns[0] == '6') {
      ProfLaunch prof_(st, "gemm_wsr_b16_kernel<6>", fl, by);
      mmf_launch(gemm_wsr_b16_kernel<6>, dim3(grid), dim3(NT), 0, st, args, items, K);
    } else {
      ProfLaunch prof_(st, "gemm_wsr_b16_kernel<9>", fl, by);
      mmf_launch(gemm_wsr_b16_kernel<9>, dim3(grid), dim3(NT), 0, st, args, items, K);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_gemm_b16(const GemmJob* jobs_in, int njobs, hipStream_t st, int amode, int bmode, float drop_p,
                           const RngSnap* rng, uint64_t* rng_advance) {
  if (njobs <= 0) return rng_advance ? launch_rng_advance(rng_advance, st) : hipSuccess;
  if (amode == MODE_RK && bmode == MODE_RK && !getenv("MMF_NO_WSR16")) {
    bool wsr = true;
    for (int i = 0; i < njobs && wsr; ++i) wsr = job_wsr_b16(jobs_in[i]);
    if (wsr) {
      const hipError_t e = launch_wsr_b16(jobs_in, njobs, st);
      return (e == hipSuccess && rng_advance) ? launch_rng_advance(rng_advance, st) : e;
    }
  }
  const int form = amode == MODE_RK && bmode == MODE_RK ? 1 : amode == MODE_KR && bmode == MODE_KR ? 2
                 : amode == MODE_RK && bmode == MODE_KR ? 3 : 0;
  if (form == 0) return hipErrorInvalidValue;
  for (int i = 0; i < njobs; ++i)
    if (!gemm_b16_ok(jobs_in[i], amode, bmode) || jobs_in[i].nsrc > GEMM_MAX_SRCS) {
      const GemmJob& J = jobs_in[i];
      fprintf(stderr, "mmfusion: launch_gemm_b16 form (%d, %d) refused job %d: M %d N %d nsrc %d K %d lda %d ldb %d "
                      "a %p b %p epi 0x%x nbatch %d seg_rows %d\n", amode, bmode, i, J.g.M, J.g.N, J.nsrc,
              J.nsrc ? J.src[0].K : 0, J.nsrc ? J.src[0].a.ld : 0, J.nsrc ? J.src[0].b.ld : 0,
              J.nsrc ? (const void*)J.src[0].a.ptr : nullptr, J.nsrc ? (const void*)J.src[0].b.ptr : nullptr, J.g.epi,
              J.g.nbatch, J.g.seg_rows);
      return hipErrorInvalidValue;
    }
  // longest contraction first, then clustered by the most-shared operand (launch_gemm's order)
  std::vector<int> order(njobs);
  std::vector<double> work(njobs);
  std::map<uintptr_t, int> uses;
  bool any_partial = false;
  for (int i = 0; i < njobs; ++i) {
    order[i] = i;
    const GemmGroup& g = jobs_in[i].g;
    const bool partial = (g.epi & EPI_PARTIAL) != 0;
    any_partial |= partial;
    double kk = 0.0;
    for (int s = 0; s < jobs_in[i].nsrc; ++s) kk += jobs_in[i].src[s].K;
    work[i] = partial ? (double)g.kchunk : kk;
    ++uses[(uintptr_t)jobs_in[i].src[0].a.ptr];
    ++uses[(uintptr_t)jobs_in[i].src[0].b.ptr];
  }
  const int ilv_mode = gemm_interleave_mode();
  const bool ilv_on = ilv_mode == 2 || (ilv_mode == 1 && !any_partial);
  // 128 x 256 tiles (WIDE) for the weight gradients (form 2) when every job's N is a multiple of
  // 256: C5 0.89 -> 0.85 ms per step.  dZ (form 3) measured 0.99 -> 1.01 ms with them (its second
  // column tile already found the A rows in L2: 1.62 -> 1.51 GB read per launch), so it keeps
  // 128 x 128 unless MMF_GEMM_WIDE_DZ=1; MMF_GEMM_NO_WIDE=1: 128 x 128 everywhere (A/B,
  // profiles/r05/c5_gemm_wide/)
  // Round 5, with dZ on bf16 output and gate: RK x KR calls whose every contraction is >= 1 024
  // (dZ: K = 10 H at C5) take them too -- dZ 0.96 -> 0.92 ms, while dX (K = H) measured 0.21 -> 0.23
  // with them and keeps 128 x 128 (profiles/r05/c5_wide_dz_long/)
  static const bool no_wide = getenv("MMF_GEMM_NO_WIDE") != nullptr;
  static const bool wide_dz = getenv("MMF_GEMM_WIDE_DZ") != nullptr;
  double kmin = 1e30;
  for (int i = 0; i < njobs; ++i) kmin = std::min(kmin, work[i]);
  bool wide = !no_wide && (form == 2 || (form == 3 && (wide_dz || (!any_partial && kmin >= 1024.0))));
  for (int i = 0; i < njobs && wide; ++i) wide = jobs_in[i].g.N % (2 * BN) == 0;
  const int bn = wide ? 2 * BN : BN;
  std::vector<uintptr_t> share(njobs, 0);
  for (int i = 0; i < njobs; ++i) {
    const uintptr_t a = (uintptr_t)jobs_in[i].src[0].a.ptr, b = (uintptr_t)jobs_in[i].src[0].b.ptr;
    share[i] = uses[b] > uses[a] ? b : a;
  }
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) {
    if (work[x] != work[y]) return work[x] > work[y];
    return share[x] < share[y];
  });
  int done = 0;
  while (done < njobs) {
    GemmArgs args;
    memset(&args, 0, sizeof(args));
    args.amode = amode;
    args.bmode = bmode;
    args.drop_p = drop_p;
    args.rng = rng;
    args.rng_advance = rng_advance;   // (the first launch)
    rng_advance = nullptr;
    int ng = 0, ns = 0, max_blocks = 0;
    while (done < njobs && ng < GEMM_MAX_GROUPS) {
      const GemmJob& J = jobs_in[order[done]];
      if (ns + J.nsrc > GEMM_MAX_SRCS) break;
      GemmGroup g = J.g;
      g.nbatch = 1;
      g.src_begin = ns;
      g.src_count = J.nsrc;
      for (int s = 0; s < J.nsrc; ++s) args.s[ns++] = J.src[s];
      const bool partial = (g.epi & EPI_PARTIAL) != 0;
      args.tile_off[ng] = max_blocks;
      args.g[ng++] = g;
      max_blocks += ((g.M + BM - 1) / BM) * ((g.N + bn - 1) / bn) * (partial ? g.nsplit : 1);
      ++done;
    }
    args.ngroups = ng;
    if (ilv_on && ng > 1) {
      const int T = args.tile_off[1];
      bool even = T > 0 && T % 8 == 0;
      for (int gi = 1; gi < ng && even; ++gi)
        even = (gi + 1 < ng ? args.tile_off[gi + 1] : max_blocks) - args.tile_off[gi] == T;
      args.ilv = even ? 1 : 0;
    }
    double fl = 0.0, by = 0.0;
    for (int gi = 0; gi < ng; ++gi) {
      const GemmGroup& g = args.g[gi];
      const bool partial = (g.epi & EPI_PARTIAL) != 0;
      for (int si = g.src_begin; si < g.src_begin + g.src_count; ++si) {
        fl += 2.0 * g.M * g.N * args.s[si].K;
        by += 2.0 * ((double)g.M + g.N) * args.s[si].K;   // bf16 operands
      }
      by += partial ? 4.0 * g.nsplit * g.M * g.N
                    : ((g.epi & EPI_BF16) ? 2.0 : 4.0) * g.M * g.N + ((g.epi & EPI_BF16COPY) ? 2.0 * g.M * g.N : 0.0);
    }
    static const char* const kName[4] = {"", "gemm_lds_kernel<0, 0, 32, 3, 1, 1>", "gemm_lds_kernel<1, 1, 32, 3, 1, 2>",
                                         "gemm_lds_kernel<0, 1, 32, 3, 1, 3>"};
    static const char* const kNameW[4] = {"", "", "gemm_lds_kernel<1, 1, 32, 3, 1, 2, 1>",
                                          "gemm_lds_kernel<0, 1, 32, 3, 1, 3, 1>"};
    ProfLaunch prof_(st, wide ? kNameW[form] : kName[form], fl, by);
    if (form == 1) mmf_launch((gemm_lds_kernel<MODE_RK, MODE_RK, 32, 3, 1, 1>), dim3(max_blocks, 1), dim3(NT), 0, st, args);
    else if (form == 2 && wide) mmf_launch((gemm_lds_kernel<MODE_KR, MODE_KR, 32, 3, 1, 2, 1>), dim3(max_blocks, 1), dim3(NT), 0, st, args);
    else if (form == 2) mmf_launch((gemm_lds_kernel<MODE_KR, MODE_KR, 32, 3, 1, 2>), dim3(max_blocks, 1), dim3(NT), 0, st, args);
    else if (wide) mmf_launch((gemm_lds_kernel<MODE_RK, MODE_KR, 32, 3, 1, 3, 1>), dim3(max_blocks, 1), dim3(NT), 0, st, args);
    else mmf_launch((gemm_lds_kernel<MODE_RK, MODE_KR, 32, 3, 1, 3>), dim3(max_blocks, 1), dim3(NT), 0, st, args);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_reduce(const ReduceJob* jobs, int njobs, hipStream_t st) {
  int done = 0;
  while (done < njobs) {
    ReduceArgs a;
    memset(&a, 0, sizeof(a));
    int n = 0;
    int64_t maxmn = 0;
    int maxbatch = 1;
    while (done < njobs && n < 48) {
      a.j[n] = jobs[done++];
      if (a.j[n].nbatch < 1) a.j[n].nbatch = 1;
      if (a.j[n].nbatch > maxbatch) maxbatch = a.j[n].nbatch;
      const int64_t mn = (int64_t)a.j[n].M * a.j[n].N;
      if (mn > maxmn) maxmn = mn;
      ++n;
    }
    a.njobs = n;
    int blocks = (int)((maxmn / 4 + 63) / 64);
    if (blocks < 1) blocks = 1;
    if (blocks > 4096) blocks = 4096;
    for (int i = 0; i < n; ++i)
      if (a.j[i].db && (a.j[i].part_db || a.j[i].nsplit == 0)) { ++blocks; break; }   // dedicated bias-row block
    double by = 0.0;   // slabs (+ bias-row slabs) read once, sums written once
    for (int i = 0; i < n; ++i) {
      const ReduceJob& r = a.j[i];
      by += 4.0 * r.nbatch * ((double)r.nsplit + 1) * r.M * ((double)r.N + (r.part_db ? 1 : 0));
    }
    ProfLaunch prof_(st, "partial_reduce_kernel", 0.0, by);
    mmf_launch(partial_reduce_kernel, dim3(blocks, n, maxbatch), dim3(256), 0, st, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_mask_dropout(MaskDropArgs a, hipStream_t st) {
  if (a.n < 1 || a.n > 8 || a.nkw < 0 || a.nkw > 16) return hipErrorInvalidValue;
  int64_t maxblk = 1;
  for (int m = 0; m < a.n; ++m) {
    MaskDropJob& J = a.j[m];
    J.vec = (J.D % 8) == 0 && ((uintptr_t)J.x & 15) == 0 && ((uintptr_t)J.out & 15) == 0;
    maxblk = std::max<int64_t>(maxblk, (J.rows * J.D + 7) / 8);
  }
  double by = 0.0;
  for (int m = 0; m < a.n; ++m) by += (a.j[m].outb ? 6.0 : 8.0) * a.j[m].rows * a.j[m].D;   // read x, write x'
  for (int i = 0; i < a.nkw; ++i) {
    const int64_t nw = (int64_t)a.B * a.heads * a.kw[i].Lq * (a.kw[i].Lk / 32);
    if (a.kw[i].Lk % 32 != 0 || nw >= ((int64_t)1 << 31)) return hipErrorInvalidValue;
    maxblk = std::max<int64_t>(maxblk, nw);   // one thread per word
    by += 4.0 * nw;
  }
  const int grid = (int)std::min<int64_t>((maxblk + 255) / 256, 2048);
  ProfLaunch prof_(st, "mask_dropout_rows_kernel", 0.0, by);
  mmf_launch(mask_dropout_rows_kernel, dim3(a.n + a.nkw, grid), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace mmf
