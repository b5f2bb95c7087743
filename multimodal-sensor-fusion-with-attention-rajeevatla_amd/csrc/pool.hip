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

// Group the pairs by key modality (same P_k) and launch the grouped kernels; false when the
// shapes do not fit them (the caller runs the per-pair kernels)
bool launch_pool_grouped(bool fwd, const PoolPair* pairs, int npairs, int B, int heads, int hd, int H,
                         hipStream_t st, hipError_t& err) {
  err = hipSuccess;
  if (getenv("MMF_POOL_PER_PAIR") || H % 4 != 0 || H > 256 || npairs < 2) return false;
  std::vector<std::vector<int>> groups;
  std::vector<const float*> keyp;
  for (int g = 0; g < npairs; ++g) {
    size_t i = 0;
    while (i < keyp.size() && (keyp[i] != pairs[g].pk || pairs[groups[i][0]].Lk != pairs[g].Lk)) ++i;
    if (i == keyp.size()) { keyp.push_back(pairs[g].pk); groups.emplace_back(); }
    groups[i].push_back(g);
  }
  if (groups.size() == (size_t)npairs) return false;   // nothing shared
  for (auto& gr : groups) {
    const int R = (int)gr.size() * heads, Lk = pairs[gr[0]].Lk;
    if (R > POOL_GRP_ROWS || (size_t)R * (fwd ? Lk : H) * sizeof(float) > 64 * 1024) return false;
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
      shm = std::max(shm, (size_t)R * (fwd ? Lk : H) * sizeof(float));
      fl += 2.0 * B * R * Lk * H;
      by += 4.0 * B * ((double)Lk * H + R * (Lk + H));   // P_k once per group
      ++ng;
      ++gi;
    }
    a.ngroups = ng;
    a.B = B; a.heads = heads; a.hd = hd; a.H = H;
    ProfLaunch prof_(st, fwd ? "pool_u_grp_kernel" : "pool_dpbar_grp_kernel", fl, by);
    if (fwd) mmf_launch(pool_u_grp_kernel, dim3(B, ng), dim3(NT), (uint32_t)shm, st, a);
    else mmf_launch(pool_dpbar_grp_kernel, dim3(B, ng), dim3(NT), (uint32_t)shm, st, a);
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

hipError_t launch_pool_e(const PoolEMod* mods, int nmods, int B, int heads, int H, hipStream_t st) {
  if (nmods > 8 || H % 4 != 0) return hipErrorInvalidValue;
  bool blk = H <= 256 && !getenv("MMF_POOLE_FLAT");
  for (int i = 0; i < nmods && blk; ++i) blk = mods[i].nsrc * heads <= POOLE_NSH;
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
