// Grouped, multi-source fp32 GEMM on CDNA4 matrix cores (v_mfma_f32_32x32x2_f32).
//
// One launch covers several independent outputs ("groups": e.g. the Q/K/V
// projections of every modality pair, src/attention.py:104-106, or the
// per-modality projections, src/fusion.py:291-298).  A group may sum several
// (A, B) sources into one output tile (the backward of a tensor that feeds
// several Linears, e.g. dP_m = sum over pairs of dQ W_q + dK W_k + dV W_v),
// and may split its contraction into slabs (dW = dY^T X over B*L rows) that a
// deterministic reduce kernel sums.
//
// Tile: 128x128x32, 256 threads = 4 waves as 2x2, each wave 64x64 = 2x2
// MFMA 32x32 accumulators (64 acc VGPRs).  Tiles are staged global -> regs ->
// LDS with the next tile's global loads in flight during the MFMAs.  The LDS
// image is contraction-major ([kk][i]) so every MFMA operand is one
// conflict-free ds_read_b32 (lanes 0-31 read 32 consecutive dwords).
#include <cstring>

#include "mmf_device.h"

namespace mmf {

namespace {

constexpr int BM = 128, BN = 128, BK = 32, NT = 256;
constexpr int LDS_STRIDE = BM + 4;      // KR image (float4 writes need 16-B rows)
constexpr int LDS_STRIDE_T = BM + 1;    // RK image (transposing scalar writes, conflict-free)

struct TileRegs { float4 v[4]; };

__device__ __forceinline__ float apply_xf(float v, const Xform& xf, int64_t srow, int64_t col,
                                          const RngSnap& rs, float p, float inv_keep) {
  if (xf.rowscale) v *= xf.rowscale[(srow / xf.rs_div) * xf.rs_stride + xf.rs_off];
  if (xf.drop_site && p > 0.f) {
    v = keep1(rs, xf.drop_site, (uint64_t)srow * (uint64_t)xf.ncols + (uint64_t)col, p) ? v * inv_keep
                                                                                           : 0.f;
  }
  return v;
}

// Load one 128 x 32 tile of an operand into registers.
//  MODE_RK: stored [e][kk] (kk contiguous): thread t covers e = t/8 + 32u, kk = 4*(t%8)..+3
//  MODE_KR: stored [kk][e] (e contiguous):  thread t covers kk = t/32 + 8u, e = 4*(t%32)..+3
template <int MODE>
__device__ __forceinline__ void load_tile(TileRegs& R, const Operand& op, int64_t boff, const Xform* xft, int e0,
                                          int eext, int k0, int kend, const RngSnap& rs, float p,
                                          float inv_keep) {
  const int t = threadIdx.x;
  const bool has_xf = op.xf >= 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    int e, kk;
    if (MODE == MODE_RK) { e = e0 + (t >> 3) + 32 * u; kk = k0 + 4 * (t & 7); }
    else                 { kk = k0 + (t >> 5) + 8 * u; e = e0 + 4 * (t & 31); }
    float x[4] = {0.f, 0.f, 0.f, 0.f};
    if (MODE == MODE_RK) {
      if (e < eext) {
        const int64_t srow = e / op.row_div;
        const float* rowp = op.ptr + boff + srow * (int64_t)op.ld;
        if (op.vec && kk + 3 < kend) {
          const float4 f = *reinterpret_cast<const float4*>(rowp + kk);
          x[0] = f.x; x[1] = f.y; x[2] = f.z; x[3] = f.w;
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c) if (kk + c < kend) x[c] = rowp[kk + c];
        }
        if (has_xf) {
#pragma unroll
          for (int c = 0; c < 4; ++c) x[c] = apply_xf(x[c], xft[op.xf], srow, kk + c, rs, p, inv_keep);
        }
      }
    } else {
      if (kk < kend) {
        const int64_t srow = kk / op.row_div;
        const float* rowp = op.ptr + boff + srow * (int64_t)op.ld;
        if (op.vec && e + 3 < eext) {
          const float4 f = *reinterpret_cast<const float4*>(rowp + e);
          x[0] = f.x; x[1] = f.y; x[2] = f.z; x[3] = f.w;
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c) if (e + c < eext) x[c] = rowp[e + c];
        }
        if (has_xf) {
#pragma unroll
          for (int c = 0; c < 4; ++c) x[c] = apply_xf(x[c], xft[op.xf], srow, e + c, rs, p, inv_keep);
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
__global__ __launch_bounds__(NT) void gemm_kernel(const GemmArgs args) {
  const GemmGroup& G = args.g[blockIdx.y];
  const int tiles_n = (G.N + BN - 1) / BN;
  const int tiles_m = (G.M + BM - 1) / BM;
  const int nsplit = (G.epi & EPI_PARTIAL) ? G.nsplit : 1;
  const int per_batch = tiles_m * tiles_n * nsplit;
  const int batch = blockIdx.x / per_batch;
  if (batch >= G.nbatch) return;
  int tile = blockIdx.x - batch * per_batch;
  const int split = tile % nsplit;
  tile /= nsplit;
  const int tm = tile / tiles_n, tn = tile % tiles_n;
  const int i0 = tm * BM, j0 = tn * BN;
  // strided-batch element: shift every pointer of this problem
  const int64_t offA = (int64_t)batch * G.bs_a, offB = (int64_t)batch * G.bs_b;
  float* const Cb = (G.epi & EPI_PARTIAL) ? G.C + (int64_t)batch * nsplit * G.M * G.N
                                          : G.C + (int64_t)batch * G.bs_c;
  float* const part_db = G.part_db ? G.part_db + (int64_t)batch * nsplit * G.M : nullptr;
  const float* const biasb = G.bias ? G.bias + (int64_t)batch * G.bs_bias : nullptr;
  const int brs_off = G.bias_rs_off + batch * G.bs_brs;

  __shared__ __attribute__((aligned(16))) float As[BK * LDS_STRIDE];
  __shared__ __attribute__((aligned(16))) float Bs[BK * LDS_STRIDE];
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

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const bool want_db = (G.epi & EPI_PARTIAL) && part_db != nullptr && tn == 0;
  float dbsum = 0.f;

  for (int si = 0; si < G.src_count; ++si) {
    const GemmSrc& S = args.s[G.src_begin + si];
    int kbeg = 0, kend = S.K;
    if (G.epi & EPI_PARTIAL) {
      kbeg = split * G.kchunk;
      kend = min(S.K, kbeg + G.kchunk);
    }
    if (kbeg >= kend) continue;
    const int ntk = (kend - kbeg + BK - 1) / BK;
    TileRegs ra, rb;
    load_tile<AMODE>(ra, S.a, offA, args.xf, i0, G.M, kbeg, kend, rs, p, inv_keep);
    load_tile<BMODE>(rb, S.b, offB, args.xf, j0, G.N, kbeg, kend, rs, p, inv_keep);
    for (int kt = 0; kt < ntk; ++kt) {
      __syncthreads();
      store_tile<AMODE>(ra, As);
      store_tile<BMODE>(rb, Bs);
      __syncthreads();
      if (kt + 1 < ntk) {
        const int kn = kbeg + (kt + 1) * BK;
        load_tile<AMODE>(ra, S.a, offA, args.xf, i0, G.M, kn, kend, rs, p, inv_keep);
        load_tile<BMODE>(rb, S.b, offB, args.xf, j0, G.N, kn, kend, rs, p, inv_keep);
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

  // ------------------------------------------------------------- epilogue
  if (G.epi & EPI_PARTIAL) {
    float* out = Cb + (int64_t)split * G.M * G.N;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int j = j0 + wn * 64 + b * 32 + c;
        if (j >= G.N) continue;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int i = i0 + wm * 64 + a * 32 + acc_row(r, h);
          if (i < G.M) out[(int64_t)i * G.N + j] = acc[a][b][r] * G.alpha;
        }
      }
    if (want_db && t < BM && i0 + t < G.M) part_db[(int64_t)split * G.M + i0 + t] = dbsum * G.alpha;
    return;
  }
  const int epi = G.epi;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int j = j0 + wn * 64 + b * 32 + c;
      if (j >= G.N) continue;
      const float bj = (epi & EPI_BIAS) ? biasb[j] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int i = i0 + wm * 64 + a * 32 + acc_row(r, h);
        if (i >= G.M) continue;
        float v = acc[a][b][r] * G.alpha;
        if (epi & EPI_BIAS_RS) v += bj * G.bias_rs[(int64_t)i * G.bias_rs_ld + brs_off];
        else v += bj;
        if (epi & EPI_ROWADD)
          v += G.rowadd_scale * G.rowadd[(int64_t)(i / G.rowadd_div) * G.ld_rowadd + j];
        if (epi & EPI_ADDMAT) v += G.addm[(int64_t)i * G.ld_addm + j];
        if (epi & EPI_RELU) v = fmaxf(v, 0.f);
        if (epi & EPI_GATE) v = G.gate[(int64_t)i * G.ld_gate + j] > 0.f ? v * G.gate_scale : 0.f;
        if (epi & EPI_ROWSCALE) v *= G.rowscale[(int64_t)(i / G.rs_div) * G.rs_stride + G.rs_off];
        if ((epi & EPI_DROP) && p > 0.f)
          v = keep1(rs, G.drop_site, (uint64_t)i * (uint64_t)G.N + (uint64_t)j, p) ? v * inv_keep : 0.f;
        Cb[(int64_t)i * G.ldc + j] = v;
      }
    }
}

struct ReduceArgs {
  ReduceJob j[16];
  int32_t njobs;
};

__global__ __launch_bounds__(256) void partial_reduce_kernel(const ReduceArgs a) {
  ReduceJob J = a.j[blockIdx.y];
  const int64_t MN = (int64_t)J.M * J.N;
  const int batch = blockIdx.z;
  if (batch >= J.nbatch) return;
  J.part += (int64_t)batch * J.nsplit * MN;
  if (J.part_db) J.part_db += (int64_t)batch * J.nsplit * J.M;
  J.out += (int64_t)batch * J.bs_out;
  if (J.db) J.db += (int64_t)batch * J.bs_db;
  // 64 outputs x 4 split-groups per block; the 4 partial sums are combined in a
  // fixed order, so the result is deterministic.
  __shared__ float red[4][64];
  const int el = threadIdx.x & 63, sg = threadIdx.x >> 6;
  const int64_t gstride = (int64_t)gridDim.x * 64;
  for (int64_t e0 = (int64_t)blockIdx.x * 64; e0 < MN; e0 += gstride) {
    const int64_t e = e0 + el;
    float s0 = 0.f, s1 = 0.f;
    if (e < MN) {
      int k = sg;
      for (; k + 4 < J.nsplit; k += 8) {
        s0 += J.part[(int64_t)k * MN + e];
        s1 += J.part[(int64_t)(k + 4) * MN + e];
      }
      for (; k < J.nsplit; k += 4) s0 += J.part[(int64_t)k * MN + e];
    }
    __syncthreads();
    red[sg][el] = s0 + s1;
    __syncthreads();
    if (sg == 0 && e < MN) J.out[e] = (red[0][el] + red[1][el]) + (red[2][el] + red[3][el]);
  }
  if (J.db && J.part_db && blockIdx.x == 0) {
    for (int i = threadIdx.x; i < J.M; i += blockDim.x) {
      float s = 0.f;
      for (int k = 0; k < J.nsplit; ++k) s += J.part_db[(int64_t)k * J.M + i];
      J.db[i] = s;
    }
  }
}

}  // namespace

hipError_t launch_gemm(const GemmJob* jobs, int njobs, int amode, int bmode, float drop_p,
                       const RngSnap* rng, hipStream_t st) {
  int done = 0;
  while (done < njobs) {
    GemmArgs args;
    memset(&args, 0, sizeof(args));
    args.amode = amode;
    args.bmode = bmode;
    args.drop_p = drop_p;
    args.rng = rng;
    int ng = 0, ns = 0, nx = 0, max_blocks = 0;
    while (done < njobs && ng < GEMM_MAX_GROUPS) {
      const GemmJob& J = jobs[done];
      int need_x = 0;
      for (int s = 0; s < J.nsrc; ++s) need_x += J.has_xf_a[s] + J.has_xf_b[s];
      if (J.nsrc > GEMM_MAX_SRCS) return hipErrorInvalidValue;
      if (ns + J.nsrc > GEMM_MAX_SRCS || nx + need_x > GEMM_MAX_XF) break;
      GemmGroup g = J.g;
      if (g.nbatch < 1) g.nbatch = 1;
      g.src_begin = ns;
      g.src_count = J.nsrc;
      for (int s = 0; s < J.nsrc; ++s) {
        GemmSrc src = J.src[s];
        src.a.xf = J.has_xf_a[s] ? nx : -1;
        if (J.has_xf_a[s]) args.xf[nx++] = J.xf_a[s];
        src.b.xf = J.has_xf_b[s] ? nx : -1;
        if (J.has_xf_b[s]) args.xf[nx++] = J.xf_b[s];
        args.s[ns++] = src;
      }
      args.g[ng++] = g;
      const int tiles = ((g.M + BM - 1) / BM) * ((g.N + BN - 1) / BN) *
                        ((g.epi & EPI_PARTIAL) ? g.nsplit : 1) * g.nbatch;
      if (tiles > max_blocks) max_blocks = tiles;
      ++done;
    }
    if (ng == 0) return hipErrorInvalidValue;
    args.ngroups = ng;
    if (max_blocks > 0) {
      dim3 grid(max_blocks, ng);
      if (amode == MODE_RK && bmode == MODE_RK)
        hipLaunchKernelGGL((gemm_kernel<MODE_RK, MODE_RK>), grid, dim3(NT), 0, st, args);
      else if (amode == MODE_RK && bmode == MODE_KR)
        hipLaunchKernelGGL((gemm_kernel<MODE_RK, MODE_KR>), grid, dim3(NT), 0, st, args);
      else if (amode == MODE_KR && bmode == MODE_KR)
        hipLaunchKernelGGL((gemm_kernel<MODE_KR, MODE_KR>), grid, dim3(NT), 0, st, args);
      else
        hipLaunchKernelGGL((gemm_kernel<MODE_KR, MODE_RK>), grid, dim3(NT), 0, st, args);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
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
    while (done < njobs && n < 16) {
      a.j[n] = jobs[done++];
      if (a.j[n].nbatch < 1) a.j[n].nbatch = 1;
      if (a.j[n].nbatch > maxbatch) maxbatch = a.j[n].nbatch;
      const int64_t mn = (int64_t)a.j[n].M * a.j[n].N;
      if (mn > maxmn) maxmn = mn;
      ++n;
    }
    a.njobs = n;
    int blocks = (int)((maxmn + 63) / 64);
    if (blocks < 1) blocks = 1;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(partial_reduce_kernel, dim3(blocks, n, maxbatch), dim3(256), 0, st, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace mmf
