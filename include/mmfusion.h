/*
 * mmfusion — MI355X-native cross-modal attention fusion (C-ABI boundary).
 *
 * This is the drop-in boundary for the reference's hot path:
 *   src/fusion.py::HybridFusion          (forward src/fusion.py:331-427,
 *                                          compute_adaptive_weights :429-479)
 *   src/attention.py::CrossModalAttention (forward src/attention.py:68-146)
 * The reference is Python; its "FFI" for this path is the nn.Module forward()
 * plus autograd.  The host mirror (package fusion.py / attention.py) binds the
 * entry points below through ctypes.
 *
 * Conventions
 *  - All tensors are fp32, contiguous, row-major, resident in device (HBM)
 *    memory; pointers are plain device pointers.  No torch types appear here.
 *  - Linear weights use PyTorch nn.Linear layout: w (out,in), b (out);
 *    y = x w^T + b.
 *  - `stream` is a hipStream_t (passed as void*).  Entry points only enqueue
 *    work on it: no allocation, no host synchronisation, no host->device
 *    copies, so they are safe inside hipGraph / torch.cuda.graph capture.
 *  - Caller-owned buffers: `saved` (forward -> backward activations, size
 *    mmf_*_saved_bytes) and `workspace` (backward scratch, size
 *    mmf_*_workspace_bytes), 256-byte aligned.
 *  - Dropout RNG: `rng_state` is a device array {uint64 seed, uint64 offset}.
 *    Each forward snapshots it into `saved` and advances offset by 1 on the
 *    device (graph-replay safe); backward replays the same Philox4x32-10
 *    streams from the snapshot.
 *  - Return value: 0 on success, otherwise an MMF_E* code with a message in
 *    mmf_last_error().  Shape/limit checks run before any launch.
 */
#ifndef MMFUSION_H_
#define MMFUSION_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MMF_MAX_MODALITIES 8
#define MMF_MAX_PAIRS (MMF_MAX_MODALITIES * (MMF_MAX_MODALITIES - 1))
/* head_dim (hidden / num_heads) the fused attention kernels hold in registers; beyond it
 * (up to hidden) a pair's scores are materialised and contracted by MFMA GEMMs (csrc/wide.hip).
 * Pairs with ONE key (2-D inputs) have no Q / K work at all and any head_dim. */
#define MMF_MAX_HEAD_DIM 64

enum {
  MMF_PRECISION_HIGHEST = 0, /* "highest": fp32 operands */
  MMF_PRECISION_MEDIUM = 1,  /* "medium": bf16 operands, fp32 accumulate */
  MMF_PRECISION_HIGH = 2     /* "high": every fp32 operand split into bf16 hi + lo, three bf16 MFMAs
                                (lo*hi + hi*lo + hi*hi), fp32 accumulate -- torch's "sum of two bfloat16
                                numbers" form of "high" (gfx950 has no TF32) */
};

enum {
  MMF_OK = 0,
  MMF_EINVAL = 1,   /* bad shape / argument (reference would raise) */
  MMF_ELIMIT = 2,   /* outside the kernel limits (e.g. head_dim > 64) */
  MMF_EHIP = 3,     /* HIP runtime error while enqueueing */
  MMF_ETIMEOUT = 4  /* a bounded inter-workgroup wait of a training step gave up (mmf_hybrid_train_status) */
};

/* nn.Linear parameters (and their gradients). */
typedef struct mmf_linear { const float* w; const float* b; } mmf_linear;
typedef struct mmf_linear_grad { float* w; float* b; } mmf_linear_grad;

/* ---------------------------------------------------------------------
 * HybridFusion (src/fusion.py:248-479)
 * Modalities are in HybridFusion.modality_names order.  seq_len[m] == 0 means a
 * 2-D (B, D_m) input (reference semantics: L = 1 attention); > 0 means a 3-D
 * (B, L_m, D_m) input (sequence mode: agg mean-pooled over L_m).
 * pair_q/pair_k list the PRESENT attention modules "{q}_to_{k}" in the
 * reference's iteration order (src/fusion.py:383-404); deleted pairs are
 * simply absent.
 * ------------------------------------------------------------------- */
typedef struct mmf_hybrid_desc {
  int32_t batch;
  int32_t num_modalities;
  int32_t hidden;
  int32_t num_heads;
  int32_t num_classes;
  int32_t seq_len[MMF_MAX_MODALITIES];
  int32_t in_dim[MMF_MAX_MODALITIES];
  int32_t num_pairs;
  int32_t pair_q[MMF_MAX_PAIRS];
  int32_t pair_k[MMF_MAX_PAIRS];
  float dropout;            /* nn.Dropout p shared by every dropout site */
  int32_t training;         /* module.training */
  int32_t return_attention; /* write attention maps */
  /* torch.get_float32_matmul_precision() of the caller (config/base.yaml:80
   * training.matmul_precision, applied at src/train.py:53-68,448):
   * MMF_PRECISION_HIGHEST = fp32 MFMA; MMF_PRECISION_HIGH = bf16x3 (each fp32
   * operand split into bf16 hi + lo, three bf16 MFMAs, fp32 accumulate);
   * MMF_PRECISION_MEDIUM = bf16 MFMA operands with fp32 accumulation (storage,
   * softmax and reductions stay fp32 in every mode). */
  int32_t matmul_precision;
  /* Buffer contract, checked by every entry point below that takes `saved` / `workspace` before
   * its first launch (MMF_EINVAL otherwise):
   *  plan_flags: mmf_hybrid_plan_flags() when the caller sized its buffers -- the fingerprint of
   *    the MMF_* plan switches in the environment, which select kernels and so the buffer layouts
   *    (0 when none is set); a call made under different switches is refused rather than laying the
   *    buffers out differently from how they were sized;
   *  saved_capacity / workspace_capacity: the bytes the caller allocated for `saved` / `workspace`
   *    (mmf_hybrid_saved_bytes / mmf_hybrid_workspace_bytes of this descriptor); a layout that
   *    needs more is refused.  The size queries ignore these three fields. */
  uint32_t plan_flags;
  uint64_t saved_capacity;
  uint64_t workspace_capacity;
} mmf_hybrid_desc;

typedef struct mmf_hybrid_params {
  mmf_linear proj[MMF_MAX_MODALITIES];   /* projections.{m}.0 */
  mmf_linear q[MMF_MAX_PAIRS];           /* attention_modules.{q}_to_{k}.query_proj */
  mmf_linear k[MMF_MAX_PAIRS];           /*   .key_proj   */
  mmf_linear v[MMF_MAX_PAIRS];           /*   .value_proj */
  mmf_linear o[MMF_MAX_PAIRS];           /*   .out_proj   */
  mmf_linear gate[MMF_MAX_MODALITIES];   /* gating_layers.{m} (1 x H) */
  mmf_linear cls1;                       /* classifier.0 (H x H) */
  mmf_linear cls2;                       /* classifier.3 (C x H) */
} mmf_hybrid_params;

typedef struct mmf_hybrid_grads {
  mmf_linear_grad proj[MMF_MAX_MODALITIES];
  mmf_linear_grad q[MMF_MAX_PAIRS];
  mmf_linear_grad k[MMF_MAX_PAIRS];
  mmf_linear_grad v[MMF_MAX_PAIRS];
  mmf_linear_grad o[MMF_MAX_PAIRS];
  mmf_linear_grad gate[MMF_MAX_MODALITIES];
  mmf_linear_grad cls1;
  mmf_linear_grad cls2;
} mmf_hybrid_grads;

size_t mmf_hybrid_saved_bytes(const mmf_hybrid_desc* d);
size_t mmf_hybrid_workspace_bytes(const mmf_hybrid_desc* d);
/* The current plan-switch fingerprint (mmf_hybrid_desc.plan_flags). */
uint32_t mmf_hybrid_plan_flags(void);
/* Inspection (tests, debuggers): where an activation of the last forward lives in `saved`.
 * what = MMF_SAVED_PROJ, index = modality m: P_m = dropout(ReLU(X'_m W_m^T + b_m)), fp32
 * (B, L_m, H) row-major (src/fusion.py:364-374); what = MMF_SAVED_CLS_HIDDEN, index 0: the
 * classifier's hidden layer after its ReLU and dropout, fp32 (B, H) (src/fusion.py:413-419).
 * The backward takes ReLU'(z) as (value > 0) from these.  Writes the byte offset from the start
 * of `saved` and the region's size; MMF_EINVAL for an unknown region or index. */
enum { MMF_SAVED_PROJ = 0, MMF_SAVED_CLS_HIDDEN = 1 };
int mmf_hybrid_saved_region(const mmf_hybrid_desc* d, int32_t what, int32_t index, uint64_t* offset,
                            uint64_t* bytes);

/* Forward.  x[m]: (B, L_m, D_m); mask: (B, M) float (fractional values scale
 * features, src/fusion.py:361-373).  Writes logits (B, C), fusion_weights
 * (B, M) and, when d->return_attention, attn_maps[p] (B, h, Lq, Lk) post-
 * dropout for each present pair p (NULL entries skipped). */
int mmf_hybrid_forward(const mmf_hybrid_desc* d, const mmf_hybrid_params* params,
                       const float* const* x, const float* mask, const uint64_t* rng_state,
                       void* saved, float* logits, float* fusion_weights,
                       float* const* attn_maps, void* stream);

/* Backward of sum(logits * dlogits).  Parameter gradients are WRITTEN (not
 * accumulated) to `grads`; dx[m] (may be NULL) receives d/dx[m]. */
int mmf_hybrid_backward(const mmf_hybrid_desc* d, const mmf_hybrid_params* params,
                        const float* const* x, const float* mask, const void* saved,
                        const float* dlogits, void* workspace, const mmf_hybrid_grads* grads,
                        float* const* dx, void* stream);

/* Public HybridFusion.compute_adaptive_weights (src/fusion.py:429-479):
 * feats[m] (B, H) per modality -> weights (B, M).  workspace: see
 * mmf_adaptive_weights_workspace_bytes. */
size_t mmf_adaptive_weights_workspace_bytes(int32_t batch, int32_t num_modalities, int32_t hidden);
int mmf_adaptive_weights(int32_t batch, int32_t num_modalities, int32_t hidden,
                         const float* const* feats, const float* mask,
                         const mmf_linear* gate /* [M] */, float* weights, void* workspace,
                         void* stream);
/* Backward of sum(weights * dweights) through compute_adaptive_weights (the
 * reference's result is differentiable, src/fusion.py:452-479): dfeats (B, M, H)
 * stacked per modality (may be NULL), dgate[m] = gradients of gating_layers.{m}
 * (WRITTEN, batch-reduced in a fixed order; may be NULL).  The masked positions
 * and the fallback branch get zero score gradients, as in autograd through
 * masked_fill / torch.where.  Same workspace as the forward. */
int mmf_adaptive_weights_backward(int32_t batch, int32_t num_modalities, int32_t hidden,
                                  const float* const* feats, const float* mask,
                                  const mmf_linear* gate /* [M] */, const float* dweights,
                                  float* dfeats, const mmf_linear_grad* dgate /* [M] */,
                                  void* workspace, void* stream);

/* ---------------------------------------------------------------------
 * CrossModalAttention (src/attention.py:16-146), standalone.
 * lq/lk: sequence lengths (use 1 for the reference's 2-D inputs; lk == 1 runs the
 * single-key plan: no Q / K work, exact-zero query / key gradients).
 * mask_mode: 0 none, 1 per-sample (B,) (src/attention.py:120-121),
 *            2 per-key (B, Lk).
 * ------------------------------------------------------------------- */
typedef struct mmf_cma_desc {
  int32_t batch, lq, lk, query_dim, key_dim, hidden, num_heads;
  int32_t mask_mode;
  float dropout;
  int32_t training;
  int32_t matmul_precision; /* as mmf_hybrid_desc.matmul_precision */
} mmf_cma_desc;

typedef struct mmf_cma_params { mmf_linear q, k, v, o; } mmf_cma_params;
typedef struct mmf_cma_grads { mmf_linear_grad q, k, v, o; } mmf_cma_grads;

size_t mmf_cma_saved_bytes(const mmf_cma_desc* d);
size_t mmf_cma_workspace_bytes(const mmf_cma_desc* d);

/* attended: (B, Lq, H); attn_weights: (B, h, Lq, Lk) post-dropout. */
int mmf_cma_forward(const mmf_cma_desc* d, const mmf_cma_params* params, const float* query,
                    const float* key, const float* value, const float* mask,
                    const uint64_t* rng_state, void* saved, float* attended,
                    float* attn_weights, void* stream);

/* Backward of sum(attended * d_attended).  dquery/dkey/dvalue may be NULL. */
int mmf_cma_backward(const mmf_cma_desc* d, const mmf_cma_params* params, const float* query,
                     const float* key, const float* value, const float* mask, const void* saved,
                     const float* d_attended, void* workspace, const mmf_cma_grads* grads,
                     float* dquery, float* dkey, float* dvalue, void* stream);

/* ---------------------------------------------------------------------
 * FrameEncoder.attention_pool (src/encoders.py:313-336): learned-score
 * softmax pooling over frames.  x (B, T, D); score_w (D) / score_b (1) are
 * FrameEncoder.attention (nn.Linear(D, 1)); mask (B, T) or NULL (frames with
 * mask == 0 are excluded; an all-masked row gives weights 0 and pooled 0, the
 * reference's nan_to_num).  Outputs pooled (B, D) and weights (B, T), which
 * the backward reads.  T <= 8192.
 * ------------------------------------------------------------------- */
size_t mmf_attention_pool_workspace_bytes(int32_t batch, int32_t dim);
int mmf_attention_pool_forward(int32_t batch, int32_t frames, int32_t dim, const float* x,
                               const float* score_w, const float* score_b, const float* mask,
                               float* pooled, float* weights, void* stream);
/* Backward of sum(pooled * dpooled): dx (B, T, D), dscore_w (D), dscore_b (1)
 * (overwritten, batch-reduced in a fixed order). */
int mmf_attention_pool_backward(int32_t batch, int32_t frames, int32_t dim, const float* x,
                                const float* score_w, const float* weights, const float* dpooled,
                                float* dx, float* dscore_w, float* dscore_b, void* workspace,
                                void* stream);

/* ---------------------------------------------------------------------
 * LateFusion weighting (src/fusion.py:228-245): logits (B, M, C) stacked
 * per-modality classifier outputs, weight_logits (M), mask (B, M) or NULL.
 * fused (B, C) = sum_m w[b, m] logits[b, m, :] with w = softmax(weight_logits)
 * * mask renormalised by (sum + 1e-8), or 1/M where the masked sum is 0.
 * weights (B, M) is written for the backward.  M <= 64.
 * ------------------------------------------------------------------- */
size_t mmf_late_fusion_workspace_bytes(int32_t batch, int32_t num_modalities);
int mmf_late_fusion_forward(int32_t batch, int32_t num_modalities, int32_t num_classes,
                            const float* logits, const float* weight_logits, const float* mask,
                            float* fused, float* weights, void* stream);
/* Backward of sum(fused * dfused): dlogits (B, M, C), dweight_logits (M). */
int mmf_late_fusion_backward(int32_t batch, int32_t num_modalities, int32_t num_classes,
                             const float* logits, const float* weight_logits, const float* mask,
                             const float* weights, const float* dfused, float* dlogits,
                             float* dweight_logits, void* workspace, void* stream);

/* ---------------------------------------------------------------------
 * Manifest data path (src/data.py:110-343, MultimodalDataset over .pt shards
 * {columns, data (rows, ncols)}): gather a batch of chunk windows from the
 * HBM-resident shard table into per-modality tensors.
 *   table (rows, ncols) fp32 device; chunk_row0 (B) int64 / chunk_len (B)
 *   int32 device (first table row and length <= T of each chunk); cols: device
 *   int32, the selected columns of every modality concatenated; col_offsets:
 *   HOST int32[num_modalities + 1] (modality m = cols[off[m] .. off[m+1]));
 *   out: HOST array of num_modalities device pointers, out[m] (B, T, c_m).
 * Values are nan_to_num'd (NaN / +-inf -> 0, src/data.py:289-291); rows t >=
 * chunk_len[b] are zero.  With labels != NULL: labels[b] = activity_id of the
 * chunk's first row, and *mismatch (device int32, caller-zeroed) counts rows
 * whose activity_id differs (the reference raises, src/data.py:283-284).
 * ------------------------------------------------------------------- */
int mmf_gather_chunks(const float* table, int64_t rows, int32_t ncols, const int64_t* chunk_row0,
                      const int32_t* chunk_len, int32_t batch, int32_t T, int32_t num_modalities,
                      const int32_t* cols, const int32_t* col_offsets, float* const* out,
                      int32_t label_col, int64_t* labels, int32_t* mismatch, void* stream);

/* ---------------------------------------------------------------------
 * LSTM recurrence (SequenceEncoder's nn.LSTM, src/encoders.py:67-75 / 135-166;
 * torch.nn.LSTM semantics, gate order i, f, g, o, zero initial state).
 * One persistent launch runs all `steps` time steps of up to 4 independent
 * LSTMs (one per modality); the input projection xproj = x W_ih^T + b_ih +
 * b_hh and the weight gradients are time-parallel GEMMs left to the caller.
 * Each LSTM's batch is split into instances of <= 4 rows that run side by
 * side (G = hidden / 64 workgroups of 1024 threads each, all co-resident).
 * Limits: hidden a multiple of 64 up to 256, num_lstm <= 8,
 * num_lstm * ceil(batch / 4) <= 32.
 * Arrays are HOST arrays of num_lstm device pointers:
 *   xproj (B, T, 4H), w_hh (4H, H), h / c (B, T, H), gates (B, T, 4H) =
 *   activated (i, f, g, o) saved for the backward;
 *   dh (B, T, H) upstream gradient of every h_t (entries may be NULL = 0),
 *   dgates (B, T, 4H) = gradient of the pre-activation gates (= d xproj;
 *   dW_hh = sum_t dgates_t^T h_{t-1}).
 * sync[i]: device scratch of mmf_lstm_sync_bytes(batch, hidden) bytes per
 * LSTM (re-zeroed on the stream by every call).  timeout: device uint32, zeroed
 * on the stream by every call, that the kernel ORs 1 into if an inter-workgroup
 * wait gives up; the values that never arrived are then NaN, so the call's
 * outputs (h, c, gates / dgates) carry NaN rather than silently wrong numbers.
 * A grid the device cannot hold co-resident returns MMF_ELIMIT before launch.
 * ------------------------------------------------------------------- */
size_t mmf_lstm_sync_bytes(int32_t batch, int32_t hidden);
int mmf_lstm_forward(int32_t num_lstm, int32_t batch, int32_t steps, int32_t hidden, const float* const* xproj,
                     const float* const* w_hh, float* const* h, float* const* c, float* const* gates,
                     void* const* sync, uint32_t* timeout, void* stream);
int mmf_lstm_backward(int32_t num_lstm, int32_t batch, int32_t steps, int32_t hidden,
                      const float* const* w_hh, const float* const* c, const float* const* gates,
                      const float* const* dh, float* const* dgates, void* const* sync, uint32_t* timeout,
                      void* stream);

/* ---------------------------------------------------------------------
 * Training-step helpers used by the data-parallel step (not part of the
 * reference interface; the reference uses torch.optim.AdamW via Lightning,
 * src/train.py:374-414).
 * ------------------------------------------------------------------- */
/* Fused CrossEntropyLoss(label_smoothing) forward+backward on (B, C) logits:
 * loss_out[0] = mean loss, dlogits = d(loss)/d(logits) * grad_scale. */
int mmf_cross_entropy_ls(int32_t batch, int32_t classes, const float* logits,
                         const int64_t* labels, float smoothing, float grad_scale,
                         float* loss_out, float* dlogits, void* stream);

/* AdamW over a flat fp32 buffer (torch.optim.AdamW semantics, decoupled decay).
 * step_dev: device int64 step counter, incremented by this call. */
int mmf_adamw_step(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                   int64_t* step_dev, float lr, float beta1, float beta2, float eps,
                   float weight_decay, float grad_scale, void* stream);

/* One training step's forward, CrossEntropyLoss(label_smoothing) and backward of the
 * reference's training_step (src/train.py:185-186, 303-313 over src/fusion.py:331-479): the
 * results of mmf_hybrid_forward -> mmf_cross_entropy_ls(grad_scale = loss_scale) ->
 * mmf_hybrid_backward(dlogits) in one call (logits, fusion_weights, loss_out[0] = mean loss,
 * dlogits, every parameter gradient WRITTEN to grads, dx[m] when non-NULL), the dropout state
 * advanced once.  The launch-lean L = 1 plan runs it in three launches (forward + loss + head
 * backward in one); other plans issue the three calls.  sync: mmf_hybrid_train_sync_bytes(d)
 * bytes, zeroed by the caller before the first call; every call leaves it zero.
 * clip_partial (optional, mmf_grad_clip_workspace_bytes()): also write the squared-norm partials of
 * the gradient just written -- grad_flat (16-byte aligned, grad_n floats) is the buffer `grads`
 * points into -- and advance *step_dev, for mmf_clip_adamw_apply_dev (the L = 1 plan fills them in
 * its weight-gradient launch; others run the reduction pass of mmf_clip_adamw_step_dev here). */
size_t mmf_hybrid_train_sync_bytes(const mmf_hybrid_desc* d);
/* 1 when the launch-lean L = 1 plan serves this descriptor (2-D inputs, fp32 "highest", every
 * ordered pair present, H <= 128, ...; given 16-byte aligned inputs and weights, as torch
 * allocates them): its training step is three short launches, so a caller may prefer eager
 * dispatch to a graph replay, whose boundary costs more on this stack (bench.py --workload c2_l1). */
int mmf_hybrid_lean_l1(const mmf_hybrid_desc* d);
/* Status of the train steps issued on `sync` so far: reads the sync buffer's error word on `stream`
 * (a 4-byte device-to-host copy, then a stream synchronize).  The launch-lean L = 1 step's waiting
 * workgroups poll for their tile's head a bounded number of times (co-residency is checked against
 * the device's reported occupancy before launch, but another stream or process may hold CUs); a
 * wait that gives up leaves that tile's gradients unwritten, sets the error word, and the step's
 * weight-gradient launch then returns every other sync word to 0, writes loss_out[0] = NaN and one
 * +inf clip partial (clip coefficient 0: mmf_clip_adamw_apply_dev applies a zero gradient).  Returns
 * MMF_OK, or MMF_ETIMEOUT when the error word is set (cleared first when `clear`); the next call
 * after a timeout starts from clean sync words. */
int mmf_hybrid_train_status(const mmf_hybrid_desc* d, void* sync, int clear, void* stream);
int mmf_hybrid_train_step(const mmf_hybrid_desc* d, const mmf_hybrid_params* params, const float* const* x,
                          const float* mask, const int64_t* labels, float label_smoothing, float loss_scale,
                          uint64_t* rng_state, void* saved, void* workspace, void* sync, float* logits,
                          float* fusion_weights, float* loss_out, float* dlogits, const mmf_hybrid_grads* grads,
                          float* const* dx, float* clip_partial, int64_t* step_dev, const float* grad_flat,
                          int64_t grad_n, void* stream);

/* mmf_hybrid_train_step in two parts, for a data-parallel caller that overlaps its gradient
 * exchange with the rest of the backward: part 1 = the forward, the loss and the backward up to
 * every parameter gradient except the modality projections' (projections.{m}.0.*: all written
 * when part 1's launches complete); part 2 = dZ, dX and the projections' weight gradients (the
 * launch-lean L = 1 plan writes every gradient in part 1, its part 2 is empty).  part 0 = both
 * (mmf_hybrid_train_step).  Parts 1 and 2 are called in that order with the same arguments;
 * clip_partial needs part 0. */
int mmf_hybrid_train_step_part(int part, const mmf_hybrid_desc* d, const mmf_hybrid_params* params,
                               const float* const* x, const float* mask, const int64_t* labels,
                               float label_smoothing, float loss_scale, uint64_t* rng_state, void* saved,
                               void* workspace, void* sync, float* logits, float* fusion_weights, float* loss_out,
                               float* dlogits, const mmf_hybrid_grads* grads, float* const* dx, float* clip_partial,
                               int64_t* step_dev, const float* grad_flat, int64_t grad_n, void* stream);

/* AdamW with the learning rate and an extra gradient factor read from device
 * scalars (lr_dev[0]; grad_coef_dev[0], may be NULL = 1), so a captured hipGraph
 * step follows an LR scheduler (CosineAnnealingLR, src/train.py:394-402) and
 * gradient clipping without re-capture.  Effective gradient =
 * grad * grad_scale * grad_coef_dev[0]. */
int mmf_adamw_step_dev(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                       int64_t* step_dev, const float* lr_dev, const float* grad_coef_dev, float beta1,
                       float beta2, float eps, float weight_decay, float grad_scale, void* stream);

/* The update half of mmf_clip_adamw_step_dev: clip + AdamW from squared-norm partials already in
 * `workspace` (written by mmf_hybrid_train_step's clip_partial), *step_dev already advanced. */
int mmf_clip_adamw_apply_dev(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                             int64_t* step_dev, const float* lr_dev, float max_norm, float* total_norm,
                             float* clip_coef, void* workspace, float beta1, float beta2, float eps,
                             float weight_decay, float grad_scale, void* stream);

/* dst += src over n floats (both 16-byte aligned): the gradient of one micro-batch added into
 * the accumulated one (Lightning's accumulate_grad_batches, config/base.yaml:75
 * gradient_accumulation; the caller scales each micro-batch loss by 1 / accumulate, as
 * mmf_cross_entropy_ls's grad_scale does). */
int mmf_grad_accumulate(int64_t n, const float* src, float* dst, void* stream);

/* The bf16-operand GEMM forms of the "medium" plans, for tests and diagnostics:
 * C (M x N, ldc) = sum over k of A(m, k) B(n, k) (+ bias[n]), with A stored [m][k] (a_kmajor = 0,
 * lda) or [k][m] (a_kmajor = 1), B likewise; bf16 (__bf16) operands, 16-byte aligned, lda / ldb
 * multiples of 8; fp32 accumulation; C fp32, or bf16 with c_bf16 = 1 (rounded to nearest even).
 * Forms: (0, 0), (1, 1) and (0, 1) -- the Q/K projections (bf16 C with bias: the weight-stationary
 * kernel when M and N are multiples of 128 and 32 | K <= 256), the weight gradients, dZ.
 * nsplit > 1 (k-major A, fp32 C): split-K slabs in `workspace` (mmf_gemm_bf16_workspace_bytes)
 * reduced in a fixed order; bias_grad (k-major A, may be NULL): also write the row sums of A over k
 * (a weight gradient's bias gradient). */
size_t mmf_gemm_bf16_workspace_bytes(int32_t M, int32_t N, int32_t K, int32_t nsplit);
int mmf_gemm_bf16(int32_t M, int32_t N, int32_t K, const void* A, int32_t lda, int32_t a_kmajor, const void* B,
                  int32_t ldb, int32_t b_kmajor, const float* bias, void* C, int32_t ldc, int32_t c_bf16,
                  void* workspace, int32_t nsplit, float* bias_grad, void* stream);

/* Global-norm gradient clipping (torch.nn.utils.clip_grad_norm_(max_norm,
 * norm_type=2) as Lightning applies gradient_clip_val, src/train.py:416-430,
 * config/base.yaml:74 gradient_clip_norm): over the flat gradient scaled by
 * grad_scale, total_norm[0] (may be NULL) = ||grad * grad_scale||_2 and
 * clip_coef[0] = min(1, max_norm / (total_norm + 1e-6)) (1 when max_norm <= 0; 0 when total_norm is not
 * finite, clipping on or off: a step that gave up waiting (mmf_hybrid_train_status) applies a zero gradient),
 * both device floats; feed clip_coef to mmf_adamw_step_dev.  Deterministic
 * fixed-order reduction.  grad 16-byte aligned. */
size_t mmf_grad_clip_workspace_bytes(void);
int mmf_grad_clip_coef(int64_t n, const float* grad, float grad_scale, float max_norm, float* total_norm,
                       float* clip_coef, void* workspace, void* stream);

/* mmf_grad_clip_coef followed by mmf_adamw_step_dev in two launches instead of
 * four (sum-of-squares partials; then every AdamW block re-reduces them itself):
 * the same total_norm / clip_coef outputs (either may be NULL) and the same
 * update, step_dev advanced by one.  workspace: mmf_grad_clip_workspace_bytes().
 * Replaces the clip_grad_norm_ + AdamW pair of src/train.py:374-430. */
int mmf_clip_adamw_step_dev(int64_t n, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                            int64_t* step_dev, const float* lr_dev, float max_norm, float* total_norm,
                            float* clip_coef, void* workspace, float beta1, float beta2, float eps,
                            float weight_decay, float grad_scale, void* stream);

/* Timing for the benchmark: between begin and end every launch group AND
 * every kernel launch of the entry points above is bracketed by hipEvents on
 * its stream.  end() synchronises those events and writes tab-separated lines
 * into out (truncated to cap), returning the bytes needed:
 *   "S <stage> <ms>"                            per launch group
 *   "L <stage> <kernel> <ms> <flops> <bytes>"   per kernel launch, with the
 *                                               launch's algorithmic FLOPs and
 *                                               HBM bytes (no recompute).
 * Kernel names are rocprofv3's minus the "mmf::(anonymous namespace)::" prefix.
 * Eager use only (not under graph capture). */
void mmf_profile_begin(void);
size_t mmf_profile_end(char* out, size_t cap);

const char* mmf_last_error(void);
const char* mmf_version(void);

#ifdef __cplusplus
}
#endif
#endif /* MMFUSION_H_ */
