// Persistent LSTM recurrence (SequenceEncoder, src/encoders.py:67-75,
// 135-166; PyTorch nn.LSTM semantics, gate order i, f, g, o):
//   pre_t = xproj_t + W_hh h_{t-1}          (xproj = x W_ih^T + b_ih + b_hh, precomputed)
//   c_t = sigmoid(f) c_{t-1} + sigmoid(i) tanh(g);  h_t = sigmoid(o) tanh(c_t)
// C3 spent 98 % of a step in MIOpen's LSTM: 1024 sequential
// steps of a 1024 x 256 recurrent matvec.  Here one launch runs the whole
// recurrence: G = H / 64 workgroups of 1024 threads per (LSTM, <= 4 batch rows)
// instance each keep their 64 hidden units' 4 x 64 rows of W_hh in VGPRs (64
// floats per thread, loaded once) and exchange h_t every step through tagged
// 8-byte granules {epoch, value} (agent-scope relaxed atomic stores and polls,
// double-buffered by step parity: the data is its own flag -- CDNA guide §6
// Guideline 16, R2).  Nothing is ordered by dispatch or placement; every spin is
// bounded: a wait that gives up sets the call's timeout word and poisons the
// missing values with NaN, so the results can never be silently wrong.  The backward runs the same way in reverse:
// each workgroup publishes its partial W_hh^T dgates for every hidden unit, each
// unit's owner sums the G partials (fixed order).  The time-parallel GEMMs
// (input projection, weight gradients) are left to the caller.
//
// Per step and workgroup: one barrier; the matvec runs as packed FMAs on
// register-resident weights against LDS-broadcast operands (16 lanes share a
// 4 x 16 weight block per row so each lane reads 16 operands, not 64: the LDS
// read rate, not the FMA rate, bounded the first version), partial sums are
// transpose-reduced across the 16 lanes with DPP moves (no LDS round trip), and
// one wave per batch row polls the granules (MI355X_MICROARCH.md handoff-1to1:
// the price of a hand-off sits in the consumer CU's memory queue).
#include <cmath>

#include "capi_util.h"

namespace mmf {

namespace {

typedef __attribute__((address_space(1))) unsigned long long gu64;
constexpr int LNT = 1024;          // threads per workgroup
constexpr int LU = 64;             // hidden units per workgroup
constexpr int LMAX_B = 4;          // batch rows per instance (one workgroup group)
constexpr int LMAX_H = 256;
constexpr int LMAX_N = 8;          // LSTMs per launch (one per modality)
constexpr int LMAX_I = 32;         // instances per launch: (LSTM, <= 4 batch rows) pairs
constexpr unsigned SPIN_LIMIT = 1u << 20;   // ~1 s of polling

struct LstmArgs {
  int T, H, G, ninst;
  int8_t lstm_of[LMAX_I];          // instance -> LSTM
  int16_t b0[LMAX_I];              // instance -> first batch row
  int8_t nb[LMAX_I];               // instance -> batch rows (<= 4)
  const float* xproj[LMAX_N];      // (B, T, 4H)
  const float* w_hh[LMAX_N];       // (4H, H)
  float* h[LMAX_N];                // (B, T, H)
  float* c[LMAX_N];                // (B, T, H)
  float* gates[LMAX_N];            // (B, T, 4H) activated i, f, g, o
  // backward
  const float* dh[LMAX_N];         // (B, T, H) upstream gradient of every h_t (may be null)
  float* dgates[LMAX_N];           // (B, T, 4H) gradient of the PRE-activation gates
  gu64* gran[LMAX_N];              // 2 x G x B x H granules (the forward uses 2 x B x H)
  unsigned* timeout;
};


// fast activations for the recurrences: v_exp_f32 + v_rcp_f32 (a few ulp; parity is 1e-3 relative)
__device__ __forceinline__ float fsigm(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float ftanh(float x) { return 2.f * __builtin_amdgcn_rcpf(1.f + __expf(-2.f * x)) - 1.f; }

// DPP lane moves (no LDS round trip): quad_perm xor 1 / xor 2, row_newbcast:n (lane n of each 16-lane row)
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float quad_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  return v + dpp<0x4E>(v);   // quad_perm [2,3,0,1]
}

typedef float f2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void put(gu64* g, unsigned epoch, float v) {
  __hip_atomic_store(g, ((unsigned long long)epoch << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool timed_out(unsigned spins, unsigned* tmo) {
  return (spins & 255) == 255 && tmo &&
         (spins > SPIN_LIMIT || __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// lane l (of a 16-lane row) holds partials P0..P3 of four outputs; returns, in lane l, the
// row-wide total of output (l >> 2) & 3
__device__ __forceinline__ float transpose_reduce4(float P0, float P1, float P2, float P3, int l) {
  const bool b3 = (l >> 3) & 1, b2 = (l >> 2) & 1;
  const float r0 = (b3 ? P2 : P0) + dpp<0x128>(b3 ? P0 : P2);   // row_ror:8 (lane l ^ 8)
  const float r1 = (b3 ? P3 : P1) + dpp<0x128>(b3 ? P1 : P3);
  const float snd = b2 ? r0 : r1;
  const float from_lo = dpp<0x124>(snd), from_hi = dpp<0x12C>(snd);   // row_ror:4 / :12 (lanes l - 4, l + 4)
  return quad_sum((b2 ? r1 : r0) + (b2 ? from_lo : from_hi));
}

// Backward: lane u of wave b polls the G partials of dh[b][unit u] with
// independent loads and runs the cell backward directly (no barrier in between);
// dg_s is double-buffered, so one barrier per step remains.
__global__ __launch_bounds__(LNT) void lstm_bwd_kernel(const LstmArgs a) {
  __shared__ __attribute__((aligned(16))) float dg_s[2][LMAX_B][4 * LU];
  const int inst = blockIdx.x / a.G, j = blockIdx.x - inst * a.G;
  if (inst >= a.ninst) return;
  const int li = a.lstm_of[inst], b0 = a.b0[inst];
  const int t0 = threadIdx.x;
  const int H = a.H, B = a.nb[inst], G = a.G, H4X = 4 * H;
  const float* cin = a.c[li] + (int64_t)b0 * a.T * H;
  const float* gin = a.gates[li] + (int64_t)b0 * a.T * H4X;
  const float* dhin = a.dh[li] ? a.dh[li] + (int64_t)b0 * a.T * H : nullptr;
  float* dgout = a.dgates[li] + (int64_t)b0 * a.T * H4X;
  gu64* gr = a.gran[li] + (int64_t)2 * G * b0 * H;
  // matvec lanes: wave w, lane l -> local rows (l & 15) * 16 .. + 16 (row = gate * 64 + unit),
  // hidden columns kc .. kc + 3 with kc = 4 (4 w + (l >> 4)); the butterfly leaves column
  // kc + ((l >> 2) & 3) in lane l
  const int l = t0 & 63, rp = l & 15;
  const int kc = ((t0 >> 6) * 4 + (l >> 4)) * 4;
  const int k = kc + ((l >> 2) & 3);
  const bool kthread = kc < H;
  f2v w[4][8];   // w[c][i / 2] = W_hh[grow(rp * 16 + i)][kc + c]
#pragma unroll
  for (int i = 0; i < 16; i += 2) {
    float4 v0 = {0.f, 0.f, 0.f, 0.f}, v1 = v0;
    if (kthread) {
      const int r0 = rp * 16 + i, r1 = r0 + 1;
      v0 = *reinterpret_cast<const float4*>(a.w_hh[li] + (int64_t)((r0 >> 6) * H + j * LU + (r0 & 63)) * H + kc);
      v1 = *reinterpret_cast<const float4*>(a.w_hh[li] + (int64_t)((r1 >> 6) * H + j * LU + (r1 & 63)) * H + kc);
    }
    w[0][i / 2] = f2v{v0.x, v1.x};
    w[1][i / 2] = f2v{v0.y, v1.y};
    w[2][i / 2] = f2v{v0.z, v1.z};
    w[3][i / 2] = f2v{v0.w, v1.w};
  }
  const int ub = t0 / LU, lu = t0 - ub * LU;
  const bool unit_thread = ub < B;
  const int unit = j * LU + lu;
  float dc = 0.f;
  const int64_t par = (int64_t)G * B * H;
  for (int s = 0; s < a.T; ++s) {
    const int t = a.T - 1 - s;
    float (*db)[4 * LU] = dg_s[s & 1];
    if (unit_thread) {
      const int64_t bt = (int64_t)ub * a.T + t;
      const float* gp = gin + bt * H4X;
      const float ig = gp[unit], fg = gp[H + unit], gg = gp[2 * H + unit], og = gp[3 * H + unit];
      const float ct = cin[bt * H + unit];
      const float cp = t > 0 ? cin[(bt - 1) * H + unit] : 0.f;
      float dh = dhin ? dhin[bt * H + unit] : 0.f;
      if (s > 0) {
        gu64* g0 = gr + (s & 1) * par + (int64_t)ub * H + unit;
        float v[LMAX_H / LU];
        unsigned ready = 0, spins = 0;
        const unsigned all = (1u << G) - 1;
        while (ready != all) {
#pragma unroll
          for (int q = 0; q < LMAX_H / LU; ++q) {
            if (q < G && !(ready >> q & 1)) {
              const unsigned long long x =
                  __hip_atomic_load(g0 + (int64_t)q * B * H, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              if ((unsigned)(x >> 32) == (unsigned)s) { v[q] = __uint_as_float((unsigned)x); ready |= 1u << q; }
            }
          }
          if (ready == all) break;
          if (timed_out(++spins, a.timeout)) {
            atomicOr(a.timeout, 1u);
            // poison what never arrived: the gradients become NaN, never silently wrong
            for (int q = 0; q < LMAX_H / LU; ++q) if (!(ready >> q & 1)) v[q] = __builtin_nanf("");
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
#pragma unroll
        for (int q = 0; q < LMAX_H / LU; ++q) if (q < G) dh += v[q];
      }
      const float tc = ftanh(ct);
      dc += dh * og * (1.f - tc * tc);
      const float d_o = dh * tc * og * (1.f - og);
      const float d_i = dc * gg * ig * (1.f - ig);
      const float d_g = dc * ig * (1.f - gg * gg);
      const float d_f = dc * cp * fg * (1.f - fg);
      dc *= fg;
      float* dp = dgout + bt * H4X;
      dp[unit] = d_i;
      dp[H + unit] = d_f;
      dp[2 * H + unit] = d_g;
      dp[3 * H + unit] = d_o;
      db[ub][lu] = d_i;
      db[ub][LU + lu] = d_f;
      db[ub][2 * LU + lu] = d_g;
      db[ub][3 * LU + lu] = d_o;
    }
    __syncthreads();
    if (t > 0) {
#pragma unroll
      for (int b = 0; b < LMAX_B; ++b) {
        if (b >= B) break;
        const float4* dr = reinterpret_cast<const float4*>(&db[b][rp * 16]);
        f2v acc[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = f2v{0.f, 0.f};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float4 d4 = dr[i];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            acc[c] = __builtin_elementwise_fma(w[c][2 * i], f2v{d4.x, d4.y}, acc[c]);
            acc[c] = __builtin_elementwise_fma(w[c][2 * i + 1], f2v{d4.z, d4.w}, acc[c]);
          }
        }
        const float acc1 = transpose_reduce4(acc[0].x + acc[0].y, acc[1].x + acc[1].y, acc[2].x + acc[2].y,
                                             acc[3].x + acc[3].y, l);
        if ((l & 3) == 0 && k < H)
          put(gr + ((s + 1) & 1) * par + ((int64_t)j * B + b) * H + k, (unsigned)(s + 1), acc1);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Forward: wave b (< B) sweeps batch row b's H granules of h_{t-1} (H / 64 loads
// per lane in flight at once, then re-polls only the missing ones) into LDS;
// lane l of wave w owns unit 4 w + (l >> 4) and the k slice (l & 15) * H / 16 of
// its 4 gate rows; after the transpose-reduce lane l holds gate (l >> 2) & 3,
// row_newbcast gathers the unit's 4 activations, lane b updates row b's cell.
// ---------------------------------------------------------------------------
constexpr int SWEEP_MAX = LMAX_H / 64;   // granules per lane


#ifdef MMF_LSTM_PROBE
__device__ unsigned long long g_lstm_probe[2][8];
#define PROBE_DECL unsigned long long pr_acc[6] = {0, 0, 0, 0, 0, 0}; unsigned long long pr_t = __builtin_amdgcn_s_memtime();
#define PROBE(i) { const unsigned long long n_ = __builtin_amdgcn_s_memtime(); pr_acc[i] += n_ - pr_t; pr_t = n_; }
#define PROBE_END                                                                         \
  if (blockIdx.x == 0 && (t0 == 0 || t0 == LNT - 64))                                     \
    for (int i = 0; i < 6; ++i) g_lstm_probe[t0 == 0 ? 0 : 1][i] = pr_acc[i];
#else
#define PROBE_DECL
#define PROBE(i)
#define PROBE_END
#endif

template <int HH>
__global__ __launch_bounds__(LNT) void lstm_fwd_kernel(const LstmArgs a) {
  __shared__ __attribute__((aligned(16))) float h_s[2][LMAX_B * LMAX_H];
  const int inst = blockIdx.x / a.G, j = blockIdx.x - inst * a.G;
  if (inst >= a.ninst) return;
  const int li = a.lstm_of[inst], b0 = a.b0[inst];
  const int t0 = threadIdx.x;
  constexpr int H = HH, H4X = 4 * H;
  const int B = a.nb[inst];
  const float* xproj = a.xproj[li] + (int64_t)b0 * a.T * H4X;
  float* hout = a.h[li] + (int64_t)b0 * a.T * H;
  float* cout = a.c[li] + (int64_t)b0 * a.T * H;
  float* gout = a.gates[li] + (int64_t)b0 * a.T * H4X;
  gu64* gr = a.gran[li] + (int64_t)2 * a.G * b0 * H;
  const int l = t0 & 63;
  const int pb = t0 >> 6;   // poller wave of batch row pb
  const bool poller = pb < B;
  const int unit = j * LU + (t0 >> 6) * 4 + (l >> 4);
  // lane l of wave w: unit 4 w + (l >> 4); k slice (l & 15) * KP .. + KP of all 4 gate rows
  const int kp = l & 15, gate = (l >> 2) & 3, mb = l & 15;
  constexpr int KP = H / 16;
  const int grow = gate * H + unit;   // the gate row this lane finishes (after the butterfly)
  const int nbh = B * H;
  f2v w[4][KP / 2];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4* wr = reinterpret_cast<const float4*>(a.w_hh[li] + (int64_t)(g * H + unit) * H + kp * KP);
#pragma unroll
    for (int i = 0; i < KP / 4; ++i) {
      const float4 v = wr[i];
      w[g][2 * i] = f2v{v.x, v.y};
      w[g][2 * i + 1] = f2v{v.z, v.w};
    }
  }
  float c = 0.f;
  PROBE_DECL
  for (int t = 0; t < a.T; ++t) {
    float xv[LMAX_B];
#pragma unroll
    for (int b = 0; b < LMAX_B; ++b) xv[b] = b < B ? xproj[((int64_t)b * a.T + t) * H4X + grow] : 0.f;
    float* hb = h_s[t & 1];   // [b * H + k]
    PROBE(0)
    if (poller) {
      float* dst = hb + pb * H;
      if (t == 0) {
        for (int k = l; k < H; k += 64) dst[k] = 0.f;
      } else {
        const gu64* src = gr + (int64_t)(t & 1) * nbh + pb * H;
        unsigned long long x[SWEEP_MAX];
        unsigned pending = 0;
#pragma unroll
        for (int p = 0; p < SWEEP_MAX; ++p)
          if (64 * p < H) {  // compile-time
            x[p] = __hip_atomic_load(src + l + 64 * p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            pending |= 1u << p;
          }
        for (unsigned spins = 0;; ++spins) {
#pragma unroll
          for (int p = 0; p < SWEEP_MAX; ++p)
            if ((pending >> p & 1) && (unsigned)(x[p] >> 32) == (unsigned)t) {
              dst[l + 64 * p] = __uint_as_float((unsigned)x[p]);
              pending &= ~(1u << p);
            }
          if (!pending) break;
          if (timed_out(spins, a.timeout)) {
            atomicOr(a.timeout, 1u);
#pragma unroll
            for (int p = 0; p < SWEEP_MAX; ++p)
              if (pending >> p & 1) dst[l + 64 * p] = __builtin_nanf("");   // poison: outputs become NaN
            break;
          }
          __builtin_amdgcn_s_sleep(1);
#pragma unroll
          for (int p = 0; p < SWEEP_MAX; ++p)
            if (pending >> p & 1)
              x[p] = __hip_atomic_load(src + l + 64 * p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    PROBE(1)
    __syncthreads();
    PROBE(2)
    float ig = 0.f, fg = 0.f, gg = 0.f, og = 0.f;
#pragma unroll
    for (int b = 0; b < LMAX_B; ++b) {
      if (b >= B) break;
      const float4* hr = reinterpret_cast<const float4*>(hb + b * H + kp * KP);
      f2v acc[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[g] = f2v{0.f, 0.f};
#pragma unroll
      for (int i = 0; i < KP / 4; ++i) {
        const float4 h4 = hr[i];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          acc[g] = __builtin_elementwise_fma(w[g][2 * i], f2v{h4.x, h4.y}, acc[g]);
          acc[g] = __builtin_elementwise_fma(w[g][2 * i + 1], f2v{h4.z, h4.w}, acc[g]);
        }
      }
      // lane l ends with the total of gate (l >> 2) & 3
      const float acc1 = transpose_reduce4(acc[0].x + acc[0].y, acc[1].x + acc[1].y, acc[2].x + acc[2].y,
                                           acc[3].x + acc[3].y, l);
      const float pre = acc1 + xv[b];
      const float act = gate == 2 ? ftanh(pre) : fsigm(pre);
      if ((l & 3) == 0) gout[((int64_t)b * a.T + t) * H4X + grow] = act;
      const float vi = dpp<0x150>(act), vf = dpp<0x154>(act);
      const float vg = dpp<0x158>(act), vo = dpp<0x15C>(act);
      if (mb == b) { ig = vi; fg = vf; gg = vg; og = vo; }
    }
    PROBE(3)
    if (mb < B) {
      c = fg * c + ig * gg;
      const float hv = og * ftanh(c);
      const int64_t bt = (int64_t)mb * a.T + t;
      hout[bt * H + unit] = hv;
      cout[bt * H + unit] = c;
      put(gr + (int64_t)((t + 1) & 1) * nbh + mb * H + unit, (unsigned)(t + 1), hv);
    }
    PROBE(4)
  }
  PROBE_END
}

// The recurrence needs every workgroup of the grid resident at once (they wait on
// each other's granules).  Refuse a grid the device cannot hold even when idle;
// residency under concurrent kernels (e.g. RCCL under DDP) is not guaranteed, which
// the bounded spins + NaN poisoning + per-call timeout word make loud, not silent.
template <typename K>
int check_coresident(K kernel, int grid, const char* what) {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, LNT, 0) != hipSuccess)
    return fail(MMF_EHIP, "%s: occupancy query failed", what);
  if ((int64_t)per_cu * cus < grid)
    return fail(MMF_ELIMIT, "%s: %d workgroups of %d threads cannot be co-resident (%d per CU x %d CUs)", what,
                grid, LNT, per_cu, cus);
  return MMF_OK;
}

// split every LSTM's batch into instances of <= LMAX_B rows
int lstm_plan(LstmArgs& a, int num_lstm, int batch, int steps, int hidden, unsigned* timeout) {
  if (num_lstm < 1 || num_lstm > LMAX_N || batch < 1 || steps < 1 || hidden < LU || hidden > LMAX_H ||
      hidden % LU != 0)
    return fail(MMF_ELIMIT, "lstm: 1..%d LSTMs, hidden a multiple of %d up to %d (got n=%d B=%d T=%d H=%d)",
                LMAX_N, LU, LMAX_H, num_lstm, batch, steps, hidden);
  const int per = (batch + LMAX_B - 1) / LMAX_B;
  if (per * num_lstm > LMAX_I)
    return fail(MMF_ELIMIT, "lstm: num_lstm x ceil(batch / %d) = %d instances (max %d)", LMAX_B,
                per * num_lstm, LMAX_I);
  if (!timeout) return fail(MMF_EINVAL, "lstm: a device timeout word is required");
  memset(&a, 0, sizeof(a));
  a.T = steps; a.H = hidden; a.G = hidden / LU; a.timeout = timeout;
  for (int i = 0; i < num_lstm; ++i)
    for (int b = 0; b < batch; b += LMAX_B) {
      a.lstm_of[a.ninst] = (int8_t)i;
      a.b0[a.ninst] = (int16_t)b;
      a.nb[a.ninst] = (int8_t)(batch - b < LMAX_B ? batch - b : LMAX_B);
      ++a.ninst;
    }
  return MMF_OK;
}

}  // namespace

}  // namespace mmf

using namespace mmf;

namespace {
// the sync granules of every LSTM and the timeout word, zeroed by one kernel
int zero_sync(int num_lstm, int batch, int hidden, void* const* sync, uint32_t* timeout, hipStream_t st) {
  float* ptrs[LMAX_N + 1];
  int64_t counts[LMAX_N + 1];
  int n = 0;
  for (int i = 0; i < num_lstm; ++i) {
    ptrs[n] = (float*)sync[i];
    counts[n++] = (int64_t)(mmf_lstm_sync_bytes(batch, hidden) / 4);
  }
  ptrs[n] = (float*)timeout;
  counts[n++] = 1;
  HIP_TRY(launch_zero_fill(ptrs, counts, n, st));
  return MMF_OK;
}
}  // namespace

extern "C" {

size_t mmf_lstm_sync_bytes(int32_t batch, int32_t hidden) {
  // 2 parities x G x B x H granules (the backward's partial sums; >= the forward's 2 x B x H)
  if (batch < 1 || hidden < 1) return 0;
  const size_t G = (size_t)(hidden + LU - 1) / LU;
  return 2 * G * (size_t)batch * hidden * sizeof(unsigned long long);
}

int mmf_lstm_forward(int32_t num_lstm, int32_t batch, int32_t steps, int32_t hidden, const float* const* xproj,
                     const float* const* w_hh, float* const* h, float* const* c, float* const* gates,
                     void* const* sync, uint32_t* timeout, void* stream) {
  LstmArgs a;
  if (int rc = lstm_plan(a, num_lstm, batch, steps, hidden, timeout)) return rc;
  hipStream_t st = (hipStream_t)stream;
  for (int i = 0; i < num_lstm; ++i)
    if (reinterpret_cast<uintptr_t>(w_hh[i]) & 15) return fail(MMF_EINVAL, "lstm: w_hh must be 16-byte aligned");
  for (int i = 0; i < num_lstm; ++i) {
    a.xproj[i] = xproj[i]; a.w_hh[i] = w_hh[i]; a.h[i] = h[i]; a.c[i] = c[i]; a.gates[i] = gates[i];
    a.gran[i] = (gu64*)sync[i];
  }
  // every polled word is zeroed before the launch (epochs start at 1); the timeout word per
  // call (a stale flag never aborts waits); one zero-fill kernel (graph-capturable)
  if (int rc = zero_sync(num_lstm, batch, hidden, sync, timeout, st)) return rc;
  const int grid = a.G * a.ninst;
  void (*kern)(const LstmArgs) = hidden == 64    ? lstm_fwd_kernel<64>
                                 : hidden == 128 ? lstm_fwd_kernel<128>
                                 : hidden == 192 ? lstm_fwd_kernel<192>
                                                 : lstm_fwd_kernel<256>;
  if (int rc = check_coresident(kern, grid, "lstm forward")) return rc;
  ProfLaunch prof_(st, "lstm_fwd_kernel", 8.0 * num_lstm * batch * steps * hidden * hidden,
                   4.0 * num_lstm * ((double)4 * hidden * hidden + (double)batch * steps * 10 * hidden));
  mmf_launch(kern, dim3(grid), dim3(LNT), 0, st, a);
  HIP_TRY(hipGetLastError());
  return MMF_OK;
}

int mmf_lstm_backward(int32_t num_lstm, int32_t batch, int32_t steps, int32_t hidden,
                      const float* const* w_hh, const float* const* c, const float* const* gates,
                      const float* const* dh, float* const* dgates, void* const* sync, uint32_t* timeout,
                      void* stream) {
  LstmArgs a;
  if (int rc = lstm_plan(a, num_lstm, batch, steps, hidden, timeout)) return rc;
  hipStream_t st = (hipStream_t)stream;
  for (int i = 0; i < num_lstm; ++i)
    if (reinterpret_cast<uintptr_t>(w_hh[i]) & 15) return fail(MMF_EINVAL, "lstm: w_hh must be 16-byte aligned");
  for (int i = 0; i < num_lstm; ++i) {
    a.w_hh[i] = w_hh[i]; a.c[i] = (float*)c[i]; a.gates[i] = (float*)gates[i]; a.dh[i] = dh[i];
    a.dgates[i] = dgates[i]; a.gran[i] = (gu64*)sync[i];
  }
  if (int rc = zero_sync(num_lstm, batch, hidden, sync, timeout, st)) return rc;
  if (int rc = check_coresident(lstm_bwd_kernel, a.G * a.ninst, "lstm backward")) return rc;
  ProfLaunch prof_(st, "lstm_bwd_kernel", 8.0 * num_lstm * batch * steps * hidden * hidden,
                   4.0 * num_lstm * ((double)4 * hidden * hidden + (double)batch * steps * 14 * hidden));
  mmf_launch(lstm_bwd_kernel, dim3(a.G * a.ninst), dim3(LNT), 0, st, a);
  HIP_TRY(hipGetLastError());
  return MMF_OK;
}

#ifdef MMF_LSTM_PROBE
int mmf_lstm_probe_read(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lstm_probe), sizeof(g_lstm_probe)) == hipSuccess ? 0 : 3;
}
#endif

}  // extern "C"
