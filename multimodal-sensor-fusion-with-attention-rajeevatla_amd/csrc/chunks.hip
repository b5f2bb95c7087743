// GPU-resident manifest data path: the PAMAP2 shard rows
// of a split live in HBM as one (rows, ncols) fp32 table; a batch of chunk
// windows (src/data.py:199-214 `_build_chunks`, :275-298 `__getitem__`) is
// gathered into per-modality (B, T, c_m) tensors in one launch:
//   out_m[b][t][j] = nan_to_num(table[(row0[b] + t) * ncols + col_m[j]])  for t < len[b], else 0,
// and the chunk label is the activity_id of its first row; rows whose
// activity_id differs from it are counted (the reference raises
// "Activity id varies within shard chunk.", src/data.py:283-284).
// Pure byte movement: one thread per (b, t) row reads the row's selected
// columns (the 54 floats of a row are one 216-B segment) and writes them.
#include <cmath>

#include "capi_util.h"

namespace mmf {

namespace {

constexpr int NT = 256;
constexpr int CH_MAX_MOD = 8;

struct GatherArgs {
  const float* table;
  int64_t rows;
  int32_t ncols;
  const int64_t* row0;     // (B) first table row of each chunk
  const int32_t* len;      // (B) rows in each chunk (<= T)
  int32_t B, T;
  int32_t nmod;
  const int32_t* cols;     // concatenated selected columns of every modality
  int32_t col_off[CH_MAX_MOD + 1];
  float* out[CH_MAX_MOD];  // (B, T, c_m)
  int32_t label_col;
  int64_t* labels;         // (B)
  int32_t* mismatch;       // rows whose activity_id differs from the chunk's first row (summed)
};

__device__ __forceinline__ float sanitize(float v) { return isfinite(v) ? v : 0.f; }

__global__ __launch_bounds__(NT) void gather_chunks_kernel(const GatherArgs a) {
  const int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;   // (b, t)
  if (i >= (int64_t)a.B * a.T) return;
  const int b = (int)(i / a.T), t = (int)(i - (int64_t)b * a.T);
  const int n = a.len[b];
  const bool valid = t < n;
  const int64_t r = a.row0[b] + t;
  const float* row = a.table + (valid ? r : 0) * a.ncols;
  for (int m = 0; m < a.nmod; ++m) {
    const int c0 = a.col_off[m], c1 = a.col_off[m + 1], cm = c1 - c0;
    float* o = a.out[m] + ((int64_t)b * a.T + t) * cm;
    for (int j = 0; j < cm; ++j) o[j] = valid ? sanitize(row[a.cols[c0 + j]]) : 0.f;
  }
  if (a.labels && valid) {
    const float first = a.table[a.row0[b] * a.ncols + a.label_col];
    if (t == 0) a.labels[b] = (int64_t)first;
    if (row[a.label_col] != first) atomicAdd(a.mismatch, 1);
  }
}

}  // namespace

}  // namespace mmf

using namespace mmf;

extern "C" {

int mmf_gather_chunks(const float* table, int64_t rows, int32_t ncols, const int64_t* chunk_row0,
                      const int32_t* chunk_len, int32_t batch, int32_t T, int32_t num_modalities,
                      const int32_t* cols, const int32_t* col_offsets, float* const* out, int32_t label_col,
                      int64_t* labels, int32_t* mismatch, void* stream) {
  if (batch < 0 || T < 1 || ncols < 1 || rows < 0) return fail(MMF_EINVAL, "gather_chunks: bad shape");
  if (num_modalities < 1 || num_modalities > CH_MAX_MOD)
    return fail(MMF_ELIMIT, "gather_chunks: %d modalities (max %d)", num_modalities, CH_MAX_MOD);
  if (labels && (label_col < 0 || label_col >= ncols || !mismatch))
    return fail(MMF_EINVAL, "gather_chunks: bad label column");
  if (batch == 0) return MMF_OK;
  GatherArgs a;
  memset(&a, 0, sizeof(a));
  a.table = table; a.rows = rows; a.ncols = ncols; a.row0 = chunk_row0; a.len = chunk_len;
  a.B = batch; a.T = T; a.nmod = num_modalities; a.cols = cols;
  int total = 0;
  for (int m = 0; m <= num_modalities; ++m) {
    a.col_off[m] = col_offsets[m];
    if (m && col_offsets[m] < col_offsets[m - 1]) return fail(MMF_EINVAL, "gather_chunks: column offsets");
  }
  total = col_offsets[num_modalities] - col_offsets[0];
  for (int m = 0; m < num_modalities; ++m) a.out[m] = out[m];
  a.label_col = label_col; a.labels = labels; a.mismatch = mismatch;
  hipStream_t st = (hipStream_t)stream;
  const int64_t n = (int64_t)batch * T;
  ProfLaunch prof_(st, "gather_chunks_kernel", 0.0, 8.0 * n * total);
  mmf_launch(gather_chunks_kernel, dim3((unsigned)((n + NT - 1) / NT)), dim3(NT), 0, st, a);
  HIP_TRY(hipGetLastError());
  return MMF_OK;
}

}  // extern "C"
