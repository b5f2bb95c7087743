// Persistent LSTM recurrence (SequenceEncoder, src/encoders.py:67-75,
// 135-166; PyTorch nn.LSTM semantics, gate order i, f, g, o):
//   pre_t = xproj_t + W_hh h_{t-1}          (xproj = x W_ih^T + b_ih + b_hh, precomputed)
//   c_t = sigmoid(f) c_{t-1} + sigmoid(i) tanh(g);  h_t = sigmoid(o) tanh(c_t)
// C3 spends 98 % of a step in MIOpen's LSTM: 1024 sequential
// steps of a 1024 x 256 recurrent matvec.  Here one launch runs the whole
// recurrence: G = H / 64 workgroups of 1024 threads per LSTM each keep their 64
// hidden units' 4 x 64 rows of W_hh in VGPRs (64 floats per thread, loaded once)
// and exchange h_t every step through tagged 8-byte granules {epoch, value}
// (agent-scope relaxed atomic stores and polls, double-buffered by step parity:
// the data is its own flag -- CDNA guide §6 Guideline 16, R2).  Nothing is
// ordered by dispatch or placement; every spin is bounded and reports a timeout.
// The backward runs the same way in reverse: each workgroup publishes its
// partial W_hh^T dgates for every hidden unit, each unit's owner sums the G
// partials (fixed order).  The time-parallel GEMMs (input projection, weight
// gradients) are left to the caller.
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

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

__device__ __forceinline__ void put(gu64* g, unsigned epoch, float v) {
  __hip_atomic_store(g, ((unsigned long long)epoch << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// poll one granule until it carries `epoch`; false (and the timeout word set) on give-up.
// Once any wait has given up, every later wait of the launch gives up within 256 spins.
__device__ __forceinline__ bool take(gu64* g, unsigned epoch, float& v, unsigned* tmo) {
  for (unsigned spins = 0;; ++spins) {
    const unsigned long long x = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((unsigned)(x >> 32) == epoch) {
      v = __uint_as_float((unsigned)x);
      return true;
    }
    if ((spins & 255) == 255 && tmo &&
        (spins > SPIN_LIMIT || __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
      atomicOr(tmo, 1u);
      v = 0.f;
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// thread t: local row lr = t >> 2 (gate = lr >> 6, unit = lr & 63), k quarter kq = t & 3
__global__ __launch_bounds__(LNT) void lstm_fwd_kernel(const LstmArgs a) {
  __shared__ float h_s[LMAX_B][LMAX_H];
  __shared__ float g_s[LMAX_B][4 * LU];
  const int inst = blockIdx.x / a.G, j = blockIdx.x - inst * a.G;
  if (inst >= a.ninst) return;
  const int li = a.lstm_of[inst], b0 = a.b0[inst];
  const int t0 = threadIdx.x;
  const int H = a.H, B = a.nb[inst], H4 = H >> 2, H4X = 4 * H;
  const float* xproj = a.xproj[li] + (int64_t)b0 * a.T * H4X;
  float* hout = a.h[li] + (int64_t)b0 * a.T * H;
  float* cout = a.c[li] + (int64_t)b0 * a.T * H;
  float* gout = a.gates[li] + (int64_t)b0 * a.T * H4X;
  gu64* gr = a.gran[li] + (int64_t)2 * a.G * b0 * H;
  const int lr = t0 >> 2, kq = t0 & 3;
  const int grow = (lr >> 6) * H + j * LU + (lr & 63);     // row of W_hh / gate column
  float w[LMAX_H / 4];
  {
    const float* wr = a.w_hh[li] + (int64_t)grow * H + kq * H4;
#pragma unroll
    for (int i = 0; i < LMAX_H / 4; ++i) w[i] = i < H4 ? wr[i] : 0.f;
  }
  const int ub = t0 / LU, lu = t0 - ub * LU;                // unit thread: (batch row, unit)
  const bool unit_thread = ub < B;
  const int unit = j * LU + lu;
  float c = 0.f;
  for (int t = 0; t < a.T; ++t) {
    // this step's input projections, issued before the wait so their latency hides behind it
    float xv[LMAX_B];
#pragma unroll
    for (int b = 0; b < LMAX_B; ++b)
      xv[b] = (kq == 0 && b < B) ? xproj[((int64_t)b * a.T + t) * H4X + grow] : 0.f;
    // h_{t-1}: granules of epoch t in buffer t & 1 (h_{-1} = 0)
    for (int idx = t0; idx < B * H; idx += LNT) {
      float v = 0.f;
      if (t > 0) take(gr + (int64_t)(t & 1) * B * H + idx, (unsigned)t, v, a.timeout);
      h_s[idx / H][idx % H] = v;
    }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < LMAX_B; ++b) {
      if (b >= B) break;
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < LMAX_H / 4; ++i)
        if (i < H4) acc = fmaf(w[i], h_s[b][kq * H4 + i], acc);
      acc += __shfl_xor(acc, 1);
      acc += __shfl_xor(acc, 2);
      if (kq == 0) g_s[b][lr] = acc + xv[b];
    }
    __syncthreads();
    if (unit_thread) {
      const float ig = sigm(g_s[ub][lu]), fg = sigm(g_s[ub][LU + lu]);
      const float gg = tanhf(g_s[ub][2 * LU + lu]), og = sigm(g_s[ub][3 * LU + lu]);
      c = fg * c + ig * gg;
      const float hv = og * tanhf(c);
      const int64_t bt = (int64_t)ub * a.T + t;
      hout[bt * H + unit] = hv;
      cout[bt * H + unit] = c;
      float* gp = gout + bt * H4X;
      gp[unit] = ig;
      gp[H + unit] = fg;
      gp[2 * H + unit] = gg;
      gp[3 * H + unit] = og;
      put(gr + (int64_t)((t + 1) & 1) * B * H + ub * H + unit, (unsigned)(t + 1), hv);
    }
  }
}

// thread t: hidden column k = t >> 2, local row quarter rq = t & 3 (rows 64 rq .. 64 rq + 63)
__global__ __launch_bounds__(LNT) void lstm_bwd_kernel(const LstmArgs a) {
  __shared__ float dg_s[LMAX_B][4 * LU];
  __shared__ float dh_s[LMAX_B][LU];
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
  const int k = t0 >> 2, rq = t0 & 3;
  const bool kthread = k < H;
  float w[LU];   // W_hh[grow(64 rq + i)][k]
#pragma unroll
  for (int i = 0; i < LU; ++i) {
    const int lr = rq * LU + i;
    const int grow = (lr >> 6) * H + j * LU + (lr & 63);
    w[i] = kthread ? a.w_hh[li][(int64_t)grow * H + k] : 0.f;
  }
  const int ub = t0 / LU, lu = t0 - ub * LU;
  const bool unit_thread = ub < B;
  const int unit = j * LU + lu;
  float dc = 0.f;
  const int64_t par = (int64_t)G * B * H;   // granules per parity buffer
  for (int s = 0; s < a.T; ++s) {
    const int t = a.T - 1 - s;
    // this step's saved state, issued before the wait
    float ig = 0.f, fg = 0.f, gg = 0.f, og = 0.f, ct = 0.f, cp = 0.f, dho = 0.f;
    if (unit_thread) {
      const int64_t bt = (int64_t)ub * a.T + t;
      const float* gp = gin + bt * H4X;
      ig = gp[unit]; fg = gp[H + unit]; gg = gp[2 * H + unit]; og = gp[3 * H + unit];
      ct = cin[bt * H + unit];
      cp = t > 0 ? cin[(bt - 1) * H + unit] : 0.f;
      if (dhin) dho = dhin[bt * H + unit];
    }
    // dh_t from the recurrence: sum over the G workgroups' partials (epoch s, buffer s & 1)
    for (int idx = t0; idx < B * LU; idx += LNT) {
      const int b = idx / LU, u = idx - b * LU;
      float sum = 0.f;
      if (s > 0)
        for (int q = 0; q < G; ++q) {
          float v;
          take(gr + (s & 1) * par + ((int64_t)q * B + b) * H + j * LU + u, (unsigned)s, v, a.timeout);
          sum += v;
        }
      dh_s[b][u] = sum;
    }
    __syncthreads();
    if (unit_thread) {
      const int64_t bt = (int64_t)ub * a.T + t;
      const float dh = dh_s[ub][lu] + dho;
      const float tc = tanhf(ct);
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
      dg_s[ub][lu] = d_i;
      dg_s[ub][LU + lu] = d_f;
      dg_s[ub][2 * LU + lu] = d_g;
      dg_s[ub][3 * LU + lu] = d_o;
    }
    __syncthreads();
    if (t > 0) {
      // partial dh_{t-1}[k] over this workgroup's rows, published for every k (epoch s + 1)
#pragma unroll
      for (int b = 0; b < LMAX_B; ++b) {
        if (b >= B) break;
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < LU; ++i) acc = fmaf(w[i], dg_s[b][rq * LU + i], acc);
        acc += __shfl_xor(acc, 1);
        acc += __shfl_xor(acc, 2);
        if (rq == 0 && kthread)
          put(gr + ((s + 1) & 1) * par + ((int64_t)j * B + b) * H + k, (unsigned)(s + 1), acc);
      }
    }
    __syncthreads();   // dg_s / dh_s are rewritten next step
  }
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
  for (int i = 0; i < num_lstm; ++i) {
    a.xproj[i] = xproj[i]; a.w_hh[i] = w_hh[i]; a.h[i] = h[i]; a.c[i] = c[i]; a.gates[i] = gates[i];
    a.gran[i] = (gu64*)sync[i];
    // every polled word is zeroed before the launch (epochs start at 1)
    HIP_TRY(hipMemsetAsync(sync[i], 0, mmf_lstm_sync_bytes(batch, hidden), st));
  }
  ProfLaunch prof_(st, "lstm_fwd_kernel", 8.0 * num_lstm * batch * steps * hidden * hidden,
                   4.0 * num_lstm * ((double)4 * hidden * hidden + (double)batch * steps * 10 * hidden));
  hipLaunchKernelGGL(lstm_fwd_kernel, dim3(a.G * a.ninst), dim3(LNT), 0, st, a);
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
  for (int i = 0; i < num_lstm; ++i) {
    a.w_hh[i] = w_hh[i]; a.c[i] = (float*)c[i]; a.gates[i] = (float*)gates[i]; a.dh[i] = dh[i];
    a.dgates[i] = dgates[i]; a.gran[i] = (gu64*)sync[i];
    HIP_TRY(hipMemsetAsync(sync[i], 0, mmf_lstm_sync_bytes(batch, hidden), st));
  }
  ProfLaunch prof_(st, "lstm_bwd_kernel", 8.0 * num_lstm * batch * steps * hidden * hidden,
                   4.0 * num_lstm * ((double)4 * hidden * hidden + (double)batch * steps * 14 * hidden));
  hipLaunchKernelGGL(lstm_bwd_kernel, dim3(a.G * a.ninst), dim3(LNT), 0, st, a);
  HIP_TRY(hipGetLastError());
  return MMF_OK;
}

}  // extern "C"
