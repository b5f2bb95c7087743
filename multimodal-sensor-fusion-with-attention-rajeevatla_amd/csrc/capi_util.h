// Host-side helpers shared by the C-ABI translation units (capi.hip, hybrid.hip):
// error reporting, optional per-stage hipEvent profiling, workspace carving and
// GEMM job builders.  Nothing here allocates device memory or synchronises.
#pragma once

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "mmf_internal.h"
#include "mmfusion.h"

namespace mmf {

int fail(int code, const char* fmt, ...);

// ---------------------------------------------------------------- profiling
struct ProfRec { const char* name; hipEvent_t a, b; };
struct LaunchRec { const char* stage; const char* kernel; double flops, bytes; hipEvent_t a, b; };
struct Prof {
  bool on = false;
  const char* cur_stage = "";
  std::vector<ProfRec> recs;
  std::vector<LaunchRec> launches;
  std::vector<hipEvent_t> pool;
  size_t next = 0;
  hipEvent_t ev() {
    if (next == pool.size()) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return nullptr;
      pool.push_back(e);
    }
    return pool[next++];
  }
};
extern Prof g_prof;

// Brackets one launch group with two events on its stream while profiling is on.
struct Stage {
  const char* name;
  hipStream_t st;
  hipEvent_t a = nullptr;
  const char* outer = nullptr;
  Stage(const char* n, hipStream_t s) : name(n), st(s) {
    if (g_prof.on && !prof_capturing(s)) {
      outer = g_prof.cur_stage;
      g_prof.cur_stage = n;
      a = g_prof.ev();
      if (a) (void)hipEventRecord(a, st);
    }
  }
  ~Stage() {
    if (outer) g_prof.cur_stage = outer;
    if (g_prof.on && a) {
      hipEvent_t b = g_prof.ev();
      if (b) {
        (void)hipEventRecord(b, st);
        g_prof.recs.push_back({name, a, b});
      }
    }
  }
};

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return ::mmf::fail(MMF_EHIP, "%s failed: %s", #expr, hipGetErrorString(e_));      \
  } while (0)

#define STAGE_TRY(name, expr)                                                           \
  do {                                                                                  \
    ::mmf::Stage stage_(name, st);                                                      \
    HIP_TRY(expr);                                                                      \
  } while (0)

// ---------------------------------------------------------------- carving
struct Bump {
  char* base;
  size_t off = 0;
  explicit Bump(void* b) : base((char*)b) {}
  template <class T>
  T* take(size_t n) {
    off = (off + 255) & ~size_t(255);
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += n * sizeof(T);
    return p;
  }
};

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

inline Operand opnd(const float* p, int ld, int row_div = 1) {
  Operand o;
  o.ptr = p;
  o.ld = ld;
  o.row_div = row_div;
  o.vec = (ld % 4 == 0) && aligned16(p);
  o.seg_stride = 0;
  return o;
}

inline GemmJob make_job(int M, int N, float* C, int ldc, int epi) {
  GemmJob j;
  memset(&j, 0, sizeof(j));
  j.g.M = M;
  j.g.N = N;
  j.g.C = C;
  j.g.ldc = ldc;
  j.g.epi = epi;
  j.g.alpha = 1.f;
  j.g.nsplit = 1;
  j.g.rowadd_div = 1;
  j.g.rowadd_scale = 1.f;
  j.g.rs_div = 1;
  j.g.gate_scale = 1.f;
  return j;
}

inline void add_src(GemmJob& j, Operand a, Operand b, int K) {
  GemmSrc& s = j.src[j.nsrc++];
  s.a = a;
  s.b = b;
  s.K = K;
}

// Split of a weight-gradient contraction over `rows`: slabs of 512 rows for
// long contractions (a launch of 8 128x128-output jobs at B*L = 32768 rows is
// 512 workgroups, 2 per CU; the slabs of all 15 such jobs are 63 MB) and of
// >= 64 rows for short ones (B = 256 rows -> 4 slabs: a short serial chain).
inline void split_rows(int rows, int& nsplit, int& kchunk, int hint = 0) {
  if (hint > 0) {
    // a chosen split count (launch-level wave sizing, plan_wgrads): slabs of >= 32 rows
    kchunk = (rows + hint - 1) / hint;
    kchunk = (kchunk + 31) & ~31;
    nsplit = (rows + kchunk - 1) / kchunk;
    return;
  }
  int chunk = rows / 4;
  if (chunk > 512) chunk = 512;
  if (chunk < 64) chunk = 64;
  nsplit = (rows + chunk - 1) / chunk;
  if (nsplit < 1) nsplit = 1;
  if (nsplit > 64) nsplit = 64;
  kchunk = (rows + nsplit - 1) / nsplit;
  kchunk = (kchunk + 31) & ~31;
  nsplit = (rows + kchunk - 1) / kchunk;
}

inline size_t slab_bytes(int M, int N, int rows) {
  int nsplit, kchunk;
  split_rows(rows, nsplit, kchunk);
  return ((((size_t)nsplit * M * N * 4) + 255) & ~size_t(255)) +
         ((((size_t)nsplit * M * 4) + 255) & ~size_t(255)) + 256;
}

// Weight gradients out(M x N) = alpha * A^T B over `rows` as split-K slabs
// (deterministic: a reduce kernel sums the slabs in order) + their row sums
// (the bias gradient) when out_b is given.
struct WgradPlan {
  std::vector<GemmJob> jobs;
  std::vector<ReduceJob> reds;
  int split_hint = 0;   // > 0: split count of the next plan_wgrad (set per job by the caller)
  std::vector<GemmJob> jobs_b16;   // bf16-operand KR x KR jobs (launch_gemm_b16), reduced with the rest
  bool size_only = false;          // a workspace-sizing pass: take the slabs, keep no jobs
};

// has_db: the layer has a bias whose gradient (row sums) is produced too.  It is
// explicit (not out_b != nullptr) so a sizing pass with null grads reserves the
// same workspace as the real call.
inline void plan_wgrad(WgradPlan& wp, Bump& ws, int M, int N, int rows, Operand a, Operand b,
                       float* out_w, float* out_b, bool has_db, float alpha = 1.f) {
  int nsplit, kchunk;
  split_rows(rows, nsplit, kchunk, wp.split_hint);
  float* part = ws.take<float>((size_t)nsplit * M * N);
  float* part_db = has_db ? ws.take<float>((size_t)nsplit * M) : nullptr;
  GemmJob j = make_job(M, N, part, N, EPI_PARTIAL);
  j.g.alpha = alpha;
  j.g.nsplit = nsplit;
  j.g.kchunk = kchunk;
  j.g.part_db = part_db;
  if (wp.size_only) return;
  add_src(j, a, b, rows);
  wp.jobs.push_back(j);
  ReduceJob r;
  memset(&r, 0, sizeof(r));
  r.nbatch = 1;
  r.part = part;
  r.part_db = part_db;
  r.out = out_w;
  r.db = out_b;
  r.nsplit = nsplit;
  r.M = M;
  r.N = N;
  wp.reds.push_back(r);
}

// Strided batch of `nbatch` weight-gradient problems without bias: problem i
// reads A + i*bs_a, B + i*bs_b and writes out_w + i*bs_out (e.g. the per-head
// row blocks of value_proj.weight in the pooled plan).
inline void plan_wgrad_batched(WgradPlan& wp, Bump& ws, int M, int N, int rows, Operand a, Operand b,
                               float* out_w, int nbatch, int bs_a, int bs_b, int bs_out) {
  int nsplit, kchunk;
  split_rows(rows, nsplit, kchunk);
  float* part = ws.take<float>((size_t)nbatch * nsplit * M * N);
  GemmJob j = make_job(M, N, part, N, EPI_PARTIAL);
  j.g.nsplit = nsplit;
  j.g.kchunk = kchunk;
  j.g.nbatch = nbatch;
  j.g.bs_a = bs_a;
  j.g.bs_b = bs_b;
  if (wp.size_only) return;
  add_src(j, a, b, rows);
  wp.jobs.push_back(j);
  ReduceJob r;
  memset(&r, 0, sizeof(r));
  r.part = part;
  r.out = out_w;
  r.nsplit = nsplit;
  r.M = M;
  r.N = N;
  r.nbatch = nbatch;
  r.bs_out = bs_out;
  wp.reds.push_back(r);
}

// A weight (and bias) gradient that is exactly zero: a reduce job over no slabs, so the
// split-K reduce launch writes the zeros (no launch of its own).
inline void plan_zero(WgradPlan& wp, int M, int N, float* out_w, float* out_b) {
  if (wp.size_only) return;
  ReduceJob r;
  memset(&r, 0, sizeof(r));
  r.nbatch = 1;
  r.out = out_w;
  r.db = out_b;
  r.nsplit = 0;
  r.M = M;
  r.N = N;
  if (out_w) wp.reds.push_back(r);
}

// Linear layer with bias (the common case).
inline void plan_wgrad(WgradPlan& wp, Bump& ws, int M, int N, int rows, Operand a, Operand b,
                       float* out_w, float* out_b, float alpha = 1.f) {
  plan_wgrad(wp, ws, M, N, rows, a, b, out_w, out_b, true, alpha);
}

}  // namespace mmf
