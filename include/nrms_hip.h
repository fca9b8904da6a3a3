/*
 * nrms_hip.h — C ABI of the MI355X (gfx950) NRMS scoring library
 * (libnrms_hip.so, built from newsrecommendationsystem_amd/csrc/).
 *
 * Drop-in boundary for the NRMS scoring path of Maguire1999/
 * NewsRecommendationSystem (paths below are relative to that repo). The
 * reference is PyTorch only and has no FFI of its own; each entry point here
 * replaces the ATen op sequence of one reference method, cited per function.
 * The Python host mirror (newsrecommendationsystem_amd/nrms.py) binds these
 * through ctypes behind the reference's own NRMS module interface.
 *
 * Conventions
 *   - All tensor arguments are caller-allocated DEVICE pointers, borrowed for
 *     the call (except nrms_adam_step_multi's descriptor array, a HOST array
 *     read during the call). The library never allocates or frees device
 *     memory and never synchronises the stream; any host thread may call it
 *     on any stream, and every call is capturable into a hipGraph. It keeps
 *     no per-call state. Process-wide state is limited to: the GEMM
 *     arithmetic, title-dedupe and token-compaction switches (atomics read at
 *     enqueue time; each can be overridden per host thread), the last HIP
 *     error (thread-local), and a mutex-guarded record of which (device,
 *     kernel) pairs have had their dynamic-LDS limit raised.
 *   - fp32 row-major everywhere; ids are int64 (the reference's LongTensor).
 *   - Every function returns NRMS_OK (0) or an nrms_status_t error code; a
 *     launch failure returns NRMS_ERR_HIP and the HIP error is kept for
 *     nrms_last_hip_error().
 *   - Kernels assume ids are in [0, V); callers validate (the Python glue does,
 *     mirroring nn.Embedding's IndexError). An out-of-range id never reads out
 *     of bounds: its row is produced as NaN.
 *   - Eval-mode semantics (dropout = identity, src/model/NRMS/news_encoder.py:
 *     38-40,43-45) for the scoring path; the training kernels at the end of
 *     this header provide the train-mode forward pieces and the backward.
 */
#ifndef NRMS_HIP_H
#define NRMS_HIP_H

#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: nrms_user_encode takes batch / row strides; nrms_adam_step_multi takes a
 *    host descriptor array (no device table, no total_blocks); q|k|v buffers
 *    carry a row stride (nrms_qkv_row_stride). */
/* 3: nrms_forward_timed / nrms_forward_stage_name; nrms_forward's workspace
 *    holds the UserEncoder row list (nrms_forward_workspace_size grew). */
/* 4: nrms_qkv_project_ws; the encode / forward workspaces hold the split
 *    Q|K|V weight (their *_workspace_size functions grew). */
/* 5: nrms_set_token_compaction; title-level padding dedupe; the encode /
 *    forward workspaces hold the title buckets (*_workspace_size grew). */
/* 6: nrms_set_thread_gemm_arith / _title_dedupe / _token_compaction
 *    (per-thread overrides of the process-wide switches). */
/* 7: host-side readers of the eval split files (nrms_behaviors_scan /
 *    nrms_behaviors_parse / nrms_news_parse); nrms_forward's workspace holds
 *    the UserEncoder dispatch order (nrms_forward_workspace_size grew). */
#define NRMS_ABI_VERSION 8

typedef enum {
  NRMS_OK = 0,
  NRMS_ERR_INVALID_ARG = 1,   /* null pointer, negative size, misalignment   */
  NRMS_ERR_UNSUPPORTED = 2,   /* shape outside the compiled kernel set       */
  NRMS_ERR_WORKSPACE = 3,     /* workspace missing or too small              */
  NRMS_ERR_HIP = 4            /* a HIP launch/API call failed                */
} nrms_status_t;

/* One encoder's parameters (device pointers), nn.Linear layout [out, in].
 * Mirrors MultiHeadSelfAttention (src/model/general/attention/
 * multihead_self.py:27-44) + AdditiveAttention (src/model/general/attention/
 * additive.py:13-20). */
typedef struct {
  const float* w_q; const float* b_q;   /* [D, D], [D] */
  const float* w_k; const float* b_k;   /* [D, D], [D] */
  const float* w_v; const float* b_v;   /* [D, D], [D] */
  const float* w_add; const float* b_add; /* additive linear [Q, D], [Q] */
  const float* q_add;                   /* attention_query_vector [Q]  */
  int32_t d_model;                      /* D  (300)                    */
  int32_t n_heads;                      /* H  (15); D / H must be 20   */
  int32_t query_dim;                    /* Q  (200); must be <= 208    */
} nrms_encoder_weights_t;

/* News-encoder projection strategy. FOLDED projects the whole vocabulary once
 * (qkv_table[V, 3D] = E W^T + b) and gathers projected rows per token; DIRECT
 * gathers embedding rows and projects every token. Both give the same result
 * (each projected row depends only on its token id); AUTO picks FOLDED when
 * the batch has more tokens than the vocabulary. */
typedef enum { NRMS_PROJ_AUTO = 0, NRMS_PROJ_DIRECT = 1, NRMS_PROJ_FOLDED = 2 } nrms_proj_mode_t;

/* Arithmetic of the matrix-core GEMMs (Q|K|V projections and the news
 * encoder's additive projection; attention contractions are always f32 MFMA).
 * SPLIT_BF16X6: each fp32 operand is split exactly into three bf16 planes
 * (hi + mid + lo, 8 significand bits each) and the six plane products with
 * i + j <= 2 are accumulated in fp32 on v_mfma_f32_16x16x32_bf16; every bf16
 * product is exact and the dropped terms are below 2^-25 |a||b|, so the result
 * has fp32-GEMM accuracy (measured: normwise error vs fp64 at or below the F32
 * mode's) at 6/16 of the f32-MFMA cycles.
 * SPLIT_F16X3 (default): the news encoder's additive projection splits each
 * operand into two fp16 planes, a = hi + 2^-11 lo (22 significand bits), and
 * accumulates lo·hi + hi·lo + hi·(2^11 hi) in one fp32 accumulator on
 * v_mfma_f32_16x16x32_f16 (3 products instead of 6); the dropped terms are
 * ~2^-22 |a||b|, normwise error vs fp64 still below a plain fp32 GEMM's. An
 * operand outside fp16's range (|a| >= 65,520) turns its outputs into NaN,
 * and those title groups are recomputed by the SPLIT_BF16X6 / reference-exp
 * recheck pass, so results never depend on the range. The encoders' Q|K|V
 * projections (nrms_qkv_project_ws, nrms_forward, the encode entry points)
 * scale every input row and every weight row by a power of two into fp16's
 * range (exact, any magnitude), split the input exactly into three fp16
 * pieces and the weights into two (22 bits), and accumulate three products
 * (four when some weight column fits in 11 bits; NRMS_PROJ_PRODUCTS=4 forces
 * four): fp32-GEMM accuracy, and products as exact as fp32's for weights
 * that fit in 11 bits. The fused UserEncoder's additive GEMM scales each context row
 * the same way and accumulates three fp16 products (22-bit operands). The
 * staged nrms_qkv_project and the stage kernels run SPLIT_BF16X6 in this mode.
 * F32: v_mfma_f32_16x16x4_f32, each product an exact fp32 FMA.
 * Process-wide; the initial value comes from the environment (NRMS_GEMM=f32
 * selects F32, NRMS_GEMM=x6 SPLIT_BF16X6). Returns the previous mode, or
 * -NRMS_ERR_INVALID_ARG for an unknown mode. Not synchronised with launches
 * in flight: set it before enqueuing work. */
typedef enum {
  NRMS_GEMM_SPLIT_BF16X6 = 0,
  NRMS_GEMM_F32 = 1,
  NRMS_GEMM_SPLIT_F16X3 = 2
} nrms_gemm_arith_t;
int32_t nrms_set_gemm_arith(int32_t mode);
int32_t nrms_get_gemm_arith(void);

/* All-padding titles (20 zero ids: the left-padding of short histories,
 * src/dataset.py:79-83, ~45 % of the clicked slots at BASELINE config 3) all
 * have the same news vector. With dedupe on (default), the fused news tail
 * encodes one of them per call and copies its vector to the others; every
 * output is bitwise the same as encoding each title (a title's vector depends
 * on its own ids only, never on where in the launch it is encoded). Applies
 * where ids are passed (16-B aligned id rows). Process-wide, read at enqueue
 * time; returns the previous setting. NRMS_DEDUPE=0 in the environment starts
 * with it off. */
int32_t nrms_set_title_dedupe(int32_t on);

/* Token compaction in the fused news tail (default on): the id-0 tokens of a
 * title (its right-padding, src/data_preprocess.py:115,132-139) share one
 * q|k|v row, so a title with c real tokens is encoded on c + 1 distinct rows,
 * the padding row carrying its multiplicity 20 - c in the raw-exp sums, the
 * attention context and the additive softmax / pooling (news_fused.hip). For
 * right-padded titles (all id-0 tokens after the real ones) the raw-exp row
 * sums are bitwise the uncompacted ones (the padding row's exp is added
 * 20 - c times, in the reference's key order). An id-0 token in the middle
 * of a title (an out-of-vocabulary word, src/data_preprocess.py:134-135) is
 * summed after the real keys instead, so its row sums agree only to fp32
 * rounding. The context and pooling replace 20 - c equal additions by one
 * product: results agree with the uncompacted computation to fp32 rounding. Process-wide, read at enqueue
 * time; returns the previous setting. NRMS_COMPACT=0 in the environment
 * starts with it off. */
int32_t nrms_set_token_compaction(int32_t on);

/* Per-thread overrides of the three process-wide switches above (ABI 6): a
 * value >= 0 applies to the work the CALLING host thread enqueues, in place
 * of the process-wide setting, so host threads driving different arithmetics
 * (or dedupe / compaction settings) on different streams do not race; -1
 * clears the thread's override. Each returns the thread's previous override
 * (-1: none), or -NRMS_ERR_INVALID_ARG. nrms_get_gemm_arith reports the
 * calling thread's effective mode. */
int32_t nrms_set_thread_gemm_arith(int32_t mode);
int32_t nrms_set_thread_title_dedupe(int32_t on);
int32_t nrms_set_thread_token_compaction(int32_t on);

int32_t nrms_abi_version(void);
const char* nrms_status_string(int32_t status);
int32_t nrms_last_hip_error(void);

/* nn.Embedding forward (src/model/NRMS/news_encoder.py:38): out[t,:] =
 * table[ids[t],:] for t < n_tok, bit-exact copy; id 0 is gathered like any id. */
int32_t nrms_embedding_gather(const int64_t* ids, int64_t n_tok, const float* table,
                              int64_t V, int32_t D, float* out, hipStream_t stream);

/* Row stride (floats) of the q|k|v rows the fused kernels prefer: 3D (900 for
 * D = 300; rows padded to whole 128-B lines, 928, measured 5 % slower per
 * step: DESIGN.md). Any stride >= 3D that is a multiple of 4 is accepted. */
int32_t nrms_qkv_row_stride(int32_t D);

/* Q|K|V projection (multihead_self.py:53-58): qkv[m * ld_qkv + 0:3D] =
 * x[row(m)] [W_Q;W_K;W_V]^T + [b_Q;b_K;b_V], row(m) = row_ids ? row_ids[m] : m
 * (row_ids index x's rows, n_rows_x bounds them); ld_qkv = 0 means 3D.
 * MFMA GEMM (arithmetic: nrms_set_gemm_arith). */
int32_t nrms_qkv_project(const float* x, int64_t n_rows_x, const int64_t* row_ids, int64_t M,
                         const nrms_encoder_weights_t* w, float* qkv, int64_t ld_qkv,
                         hipStream_t stream);

/* The same projection through the workspace — the one the encode / forward
 * entry points use. For the NRMS shape (D = 300, split arithmetic) the weight
 * is split once per call into MFMA fragments (workspace) and one persistent
 * workgroup per CU keeps a 64-row tile of x resident in LDS while it streams
 * the fragments from L2. Bitwise equal to nrms_qkv_project under
 * NRMS_GEMM_SPLIT_BF16X6 (same x6 products in the same order) and under
 * NRMS_GEMM_F32 (both run the f32 GEMM). Under NRMS_GEMM_SPLIT_F16X3 (the
 * default) it runs the scaled split-f16 arithmetic instead — each x row and
 * each weight row scaled by a power of two into fp16's range, x split exactly
 * into three fp16 pieces, the weight into two (22 bits), three products
 * summed in fp32 (four when some weight column fits in 11 bits): within
 * ~2^-22 |x||w| per product of the exact result (fp32-GEMM accuracy; exact
 * products for weights that fit in 11 bits) — so only within
 * rounding of nrms_qkv_project's x6 rows, not bitwise. Other shapes: as
 * nrms_qkv_project. */
size_t nrms_qkv_project_workspace_size(int32_t D);
int32_t nrms_qkv_project_ws(const float* x, int64_t n_rows_x, const int64_t* row_ids, int64_t M,
                            const nrms_encoder_weights_t* w, float* qkv, int64_t ld_qkv,
                            void* workspace, size_t workspace_bytes, hipStream_t stream);

/* Multi-head raw-exp self-attention over sequences of length L
 * (ScaledDotProductAttention, multihead_self.py:15-23, heads concatenated
 * :74-75) over packed q|k|v rows (stride 3D): for sequence s, token i reads qkv row r(s,i) = tok_ids ?
 * tok_ids[s*L+i] : s*L+i (tok_ids index qkv's n_rows_qkv rows). Sequences
 * s >= n_seq_a take their ids from tok_ids_b + (s-n_seq_a)*L (NULL: same
 * array). ctx[s*L+i, :] is the [D] context row. L <= 4096 (beyond 64 the
 * K|V rows are read through L2 instead of LDS). */
int32_t nrms_self_attention(const float* qkv, int64_t n_rows_qkv, const int64_t* tok_ids,
                            int64_t n_seq_a, const int64_t* tok_ids_b, int64_t n_seq,
                            int32_t L, const nrms_encoder_weights_t* w, float* ctx,
                            hipStream_t stream);

/* AdditiveAttention (additive.py:27-53) over x[n_seq, L, D]:
 * out[s] = sum_l softmax_l(tanh(x W^T + b) . q) x[s,l]. scores_ws: device
 * scratch of n_seq*L floats. */
int32_t nrms_additive_attention(const float* x, int64_t n_seq, int32_t L,
                                const nrms_encoder_weights_t* w, float* scores_ws,
                                float* out, hipStream_t stream);

/* The two halves of nrms_additive_attention, for callers that time or fuse
 * them separately: per-token scores[m] = tanh(x[m] W^T + b) . q for m <
 * n_rows (additive.py:35-38; the [n_rows, Q] tile stays in registers), and
 * the pooling out[s] = sum_l softmax_l(scores[s, :]) x[s, l] (:39,51-52). */
int32_t nrms_additive_scores(const float* x, int64_t n_rows, const nrms_encoder_weights_t* w,
                             float* scores, hipStream_t stream);
int32_t nrms_additive_pool(const float* x, const float* scores, int64_t n_seq, int32_t L,
                           int32_t D, float* out, hipStream_t stream);

/* Fused NewsEncoder tail (news_encoder.py:42-47): raw-exp MHSA over projected
 * rows + additive attention + pooling, 4 titles per workgroup per step, all
 * contractions on the matrix cores, the context kept in LDS for the additive
 * GEMM and the pooling (workspace: only a packed copy of W_add). Row
 * addressing as
 * nrms_self_attention. Compiled for the reference geometry (L = 20, D = 300,
 * H = 15, Q = 200); other shapes return NRMS_ERR_UNSUPPORTED (use the stage
 * entry points). Used by nrms_news_encode* and nrms_forward when it applies. */
size_t nrms_news_attention_pool_workspace_size(int64_t n_titles, int32_t L, int32_t D);
int32_t nrms_news_attention_pool(const float* qkv, int64_t ld_qkv, int64_t n_rows_qkv,
                                 const int64_t* tok_ids, int64_t n_seq_a, const int64_t* tok_ids_b,
                                 int64_t n_titles, int32_t L, const nrms_encoder_weights_t* w,
                                 float* out, void* workspace, size_t workspace_bytes,
                                 hipStream_t stream);

/* NewsEncoder.forward (src/model/NRMS/news_encoder.py:27-48), eval mode:
 * ids[n_titles, L] -> out[n_titles, D]. */
size_t nrms_news_encode_workspace_size(int64_t n_titles, int32_t L, int64_t V, int32_t D,
                                       int32_t proj_mode);
int32_t nrms_news_encode(const int64_t* ids, int64_t n_titles, int32_t L, const float* table,
                         int64_t V, const nrms_encoder_weights_t* w, int32_t proj_mode,
                         float* out, void* workspace, size_t workspace_bytes,
                         hipStream_t stream);

/* Same, from a caller-held folded table qkv_table[V] (rows at stride ld_qkv,
 * nrms_qkv_project of the whole embedding table; 0 = 3D): lets an eval loop
 * reuse one projection across calls while the weights are unchanged. */
size_t nrms_news_encode_folded_workspace_size(int64_t n_titles, int32_t L, int32_t D);
int32_t nrms_news_encode_folded(const int64_t* ids, int64_t n_titles, int32_t L,
                                const float* qkv_table, int64_t ld_qkv, int64_t V,
                                const nrms_encoder_weights_t* w, float* out,
                                void* workspace, size_t workspace_bytes, hipStream_t stream);

/* UserEncoder.forward (src/model/NRMS/user_encoder.py:15-26), also
 * NRMS.get_user_vector (src/model/NRMS/__init__.py:63-71): clicked is a
 * [B, N, D] view, element (b, n, d) at clicked[b*stride_b + n*stride_n + d]
 * (strides in floats, multiples of 4; the innermost stride is 1) -> out[B, D].
 * Contiguous input: stride_b = N*D, stride_n = D. The reference caller's
 * torch.stack(..., dim=0).transpose(0, 1) view (src/evaluate.py:220-224) is
 * stride_b = D, stride_n = B*D and is read in place, without a copy. */
size_t nrms_user_encode_workspace_size(int64_t B, int32_t N, int32_t D);
int32_t nrms_user_encode(const float* clicked, int64_t B, int32_t N, int64_t stride_b,
                         int64_t stride_n, const nrms_encoder_weights_t* w, float* out,
                         void* workspace, size_t workspace_bytes, hipStream_t stream);

/* Fused UserEncoder tail (user_encoder.py:15-26 after the projection): raw-exp
 * MHSA over qkv rows b*N + i (stride ld_qkv, 0 = 3D) + additive attention + pooling, one
 * workgroup per user, the context kept in LDS; out[B, D]. N <= 64, reference
 * geometry (D = 300, H = 15, Q = 200). Used by nrms_user_encode and
 * nrms_forward when it applies. Workspace: a packed copy of W_add. */
size_t nrms_user_attention_pool_workspace_size(int64_t B, int32_t N, int32_t D);
int32_t nrms_user_attention_pool(const float* qkv, int64_t ld_qkv, int64_t B, int32_t N,
                                 const nrms_encoder_weights_t* w, float* out, void* workspace,
                                 size_t workspace_bytes, hipStream_t stream);
/* The same with pad_flags[B * N] (uint8, non-zero: position b*N + i holds an
 * all-padding title, src/dataset.py:79-83 -- all such positions carry one
 * news vector, so their qkv rows are equal). With token compaction on
 * (nrms_set_token_compaction) each user is encoded on its distinct rows: the
 * padding positions collapse into one row, counted once per position in the
 * raw-exp sums (bitwise the uncompacted sums for left padding), the context
 * and the softmax / pooling (fp32-rounding-level difference); nrms_forward
 * does the same. Off: as nrms_user_attention_pool. */
int32_t nrms_user_attention_pool_padded(const float* qkv, int64_t ld_qkv, int64_t B, int32_t N,
                                        const uint8_t* pad_flags, const nrms_encoder_weights_t* w, float* out,
                                        void* workspace, size_t workspace_bytes, hipStream_t stream);

/* DotProductClickPredictor.forward (src/model/general/click_predictor/
 * dot_product.py:8-19): out[b, c] = <news[b*stride_b + c*stride_c, :], user[b*stride_u, :]>,
 * strides in floats. Also NRMS.get_prediction (src/model/NRMS/__init__.py:73-84)
 * with B = 1. */
int32_t nrms_score(const float* news, int64_t B, int32_t C, int64_t stride_b,
                   int64_t stride_c, const float* user, int64_t stride_u, int32_t D,
                   float* out, hipStream_t stream);

/* Eval-semantics scoring (src/evaluate.py:245-260): out[k] = <news[news_idx[k]],
 * user[user_idx[k]]> for k < n_pairs — all candidates of all impressions of a
 * split in one launch (each impression's get_prediction, __init__.py:73-84,
 * becomes a contiguous run of pairs). Indices out of range give NaN. */
int32_t nrms_score_pairs(const float* news, int64_t n_news, const float* user, int64_t n_users,
                         const int64_t* news_idx, const int64_t* user_idx, int64_t n_pairs,
                         int32_t D, float* out, hipStream_t stream);

/* Per-impression ranking metrics (src/evaluate.py:24-42,160-168) over ragged
 * impressions: impression i owns scores/labels [offsets[i], offsets[i+1]).
 * out[i*4 + {0,1,2,3}] = AUC, MRR, nDCG@5, nDCG@10 in fp64. A non-finite
 * score or an empty impression: all four NaN (roc_auc_score raises, the
 * reference's ValueError branch). One class only: AUC NaN (scikit-learn >= 1.3
 * warns instead of raising) and MRR / nDCG as numpy computes them (all
 * negative: NaN; all positive: MRR = mean(1/rank), nDCG = 1). Ranking order = np.argsort(score)[::-1]: descending,
 * equal scores by larger index first. */
int32_t nrms_impression_metrics(const float* scores, const int32_t* labels,
                                const int64_t* offsets, int64_t n_imp, double* out,
                                hipStream_t stream);

/* NRMS.forward (src/model/NRMS/__init__.py:19-48), eval mode:
 * cand_ids[B, C, L], clicked_ids[B, N, L] -> logits[B, C]. Every one of the
 * B*(C+N) titles gets its news vector (forward semantics), then the user
 * vector and the scores. With title dedupe (nrms_set_title_dedupe, default)
 * all-padding history titles are encoded once per batch and copied, and the
 * UserEncoder projects their q|k|v rows once as well; the logits are bitwise
 * those of encoding and projecting every title. */
size_t nrms_forward_workspace_size(int64_t B, int32_t C, int32_t N, int32_t L, int64_t V,
                                   int32_t D, int32_t proj_mode);
int32_t nrms_forward(const int64_t* cand_ids, const int64_t* clicked_ids, int64_t B, int32_t C,
                     int32_t N, int32_t L, const float* table, int64_t V,
                     const nrms_encoder_weights_t* news_w, const nrms_encoder_weights_t* user_w,
                     int32_t proj_mode, float* logits, void* workspace, size_t workspace_bytes,
                     hipStream_t stream);

/* nrms_forward with per-stage timing: stage_events[i] (n_events =
 * NRMS_FORWARD_STAGES + 1 caller-created HIP events, or n_events = 0 for none)
 * is recorded on the stream before stage i and the last one after the final
 * stage. Stages: nrms_forward_stage_name(0 .. NRMS_FORWARD_STAGES - 1) =
 * qkv_news (Q|K|V projection), news_fused (news attention + additive pooling,
 * incl. the padding-group and recheck launches), qkv_user, user_fused, score. */
#define NRMS_FORWARD_STAGES 5
int32_t nrms_forward_timed(const int64_t* cand_ids, const int64_t* clicked_ids, int64_t B, int32_t C,
                           int32_t N, int32_t L, const float* table, int64_t V,
                           const nrms_encoder_weights_t* news_w, const nrms_encoder_weights_t* user_w,
                           int32_t proj_mode, float* logits, void* workspace, size_t workspace_bytes,
                           hipStream_t stream, hipEvent_t* stage_events, int32_t n_events);
const char* nrms_forward_stage_name(int32_t stage);

/* ---------------------------------------------------------------------------
 * Training kernels: the train-mode forward pieces and the backward of the path
 * above, as src/train.py:202-236 needs them (loss.backward(), Adam step). The
 * Python glue (newsrecommendationsystem_amd/train_hip.py) chains them in a
 * torch.autograd.Function. Gradient outputs named d_* are ACCUMULATED into
 * (callers zero them), dx / dqkv / dnews outputs are overwritten. fp32; the
 * GEMMs of the backward use f32 MFMA whatever nrms_set_gemm_arith says. */

/* F.dropout(x, p, training=True) (news_encoder.py:38-40,43-45): y[i] = x[i] /
 * (1-p) if u(seed, i) >= p else 0, u a counter-based uniform (splitmix64 of
 * seed and i), so the same call on the gradient is the backward. 0 <= p < 1;
 * x == y allowed. */
int32_t nrms_dropout(const float* x, float* y, int64_t n, float p, uint64_t seed,
                     hipStream_t stream);

/* AdditiveAttention.forward (additive.py:27-53) keeping what the backward
 * needs: y_tanh[n_seq*L, Q] = tanh(x W^T + b), scores[n_seq*L] = y . q,
 * out[n_seq, D] = sum_l softmax_l(scores) x_l. */
int32_t nrms_additive_forward_train(const float* x, int64_t n_seq, int32_t L,
                                    const nrms_encoder_weights_t* w, float* y_tanh, float* scores,
                                    float* out, hipStream_t stream);

/* Its backward: dx[n_seq*L, D] (written) from dout[n_seq, D]; d_w_add [Q, D],
 * d_b_add [Q], d_q_add [Q] accumulated. Workspace:
 * nrms_additive_backward_workspace_size bytes. */
size_t nrms_additive_backward_workspace_size(int64_t n_seq, int32_t L, int32_t D, int32_t Q);
int32_t nrms_additive_backward(const float* x, int64_t n_seq, int32_t L,
                               const nrms_encoder_weights_t* w, const float* y_tanh,
                               const float* scores, const float* dout, float* dx, float* d_w_add,
                               float* d_b_add, float* d_q_add, void* workspace,
                               size_t workspace_bytes, hipStream_t stream);

/* Backward of nrms_self_attention over per-token rows (row s*L + i of
 * qkv[n_seq*L, 3D]): dqkv[n_seq*L, 3D] (written) from dctx[n_seq*L, D],
 * recomputing the raw-exp attention (multihead_self.py:15-23). L <= 64. */
int32_t nrms_self_attention_backward(const float* qkv, const float* dctx, int64_t n_seq,
                                     int32_t L, const nrms_encoder_weights_t* w, float* dqkv,
                                     hipStream_t stream);

/* Backward of nrms_qkv_project (identity rows): dx[rows, D] = dqkv [W_Q; W_K;
 * W_V] (written; NULL skips it), d_w_qkv[3D, D] += dqkv^T x, d_b_qkv[3D] +=
 * column sums of dqkv. Workspace: nrms_qkv_project_backward_workspace_size. */
size_t nrms_qkv_project_backward_workspace_size(int32_t D);
int32_t nrms_qkv_project_backward(const float* x, int64_t rows, const nrms_encoder_weights_t* w,
                                  const float* dqkv, float* dx, float* d_w_qkv, float* d_b_qkv,
                                  void* workspace, size_t workspace_bytes, hipStream_t stream);

/* Backward of nrms_score (dot_product.py:8-19): dnews[B, C, D] (contiguous,
 * written) = dlogits[b, c] user[b]; duser[B, D] (written) = sum_c dlogits[b, c]
 * news[b, c]. Strides as nrms_score. */
int32_t nrms_score_backward(const float* news, int64_t B, int32_t C, int64_t stride_b,
                            int64_t stride_c, const float* user, int64_t stride_u, int32_t D,
                            const float* dlogits, float* dnews, float* duser, hipStream_t stream);

/* Backward of nrms_embedding_gather as nn.Embedding(padding_idx) computes it:
 * dtable[ids[t]] += dx[t] for every t with ids[t] != padding_idx (dense
 * [V, D] gradient, accumulated). Float atomics: the additions to one row land
 * in arrival order, so results may differ by rounding from run to run; the _ws
 * form below is deterministic. */
int32_t nrms_embedding_backward(const int64_t* ids, int64_t n_tok, const float* dx, int64_t V,
                                int32_t D, int64_t padding_idx, float* dtable,
                                hipStream_t stream);

/* (ABI 8) The same gradient, deterministic: the tokens are sorted by id (a
 * stable radix sort) and each row's contributions added in a fixed order --
 * token order for an id with at most 256 tokens (the CPU reference's
 * index_add order, bitwise), and for a longer run sums of 64-token segments
 * (each in token order) added in segment order (round 6: parallel; within
 * fp32 rounding of index_add). Bitwise reproducible. Workspace:
 * nrms_embedding_backward_workspace_size(n_tok, V) bytes; n_tok, V < 2^31. */
size_t nrms_embedding_backward_workspace_size(int64_t n_tok, int64_t V);
int32_t nrms_embedding_backward_ws(const int64_t* ids, int64_t n_tok, const float* dx, int64_t V,
                                   int32_t D, int64_t padding_idx, float* dtable, void* workspace,
                                   size_t workspace_bytes, hipStream_t stream);

/* torch.optim.Adam step (src/train.py:127; amsgrad off, no weight decay) on
 * one parameter, in torch's operation order; `step` counts from 1. */
int32_t nrms_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                       int64_t n, float lr, float beta1, float beta2, float eps, int64_t step,
                       hipStream_t stream);

/* The same Adam step over many parameters: `tensors` is a HOST array of n
 * descriptors, read during the call; up to 32 of them go to the device by
 * value in the kernel arguments of one launch (ceil(n / 32) launches). All
 * tensors share lr / betas / eps / step. Replaces one nrms_adam_step launch
 * per parameter (torch.optim.Adam's foreach path). `first_block` is ignored
 * (kept for layout stability). */
typedef struct {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t numel;
  int64_t first_block;
} nrms_adam_tensor_t;

int32_t nrms_adam_step_multi(const nrms_adam_tensor_t* tensors, int32_t n, float lr, float beta1,
                             float beta2, float eps, int64_t step, hipStream_t stream);

/* ---------------------------------------------------------------------------
 * Host-side readers of the eval split (csrc/tsv_io.hip). HOST pointers, no
 * stream: they replace the Python line loop of the reference's readers
 * (src/evaluate.py:55-71 news_parsed.tsv, :133-157 behaviors.tsv) for the
 * MIND id form ("N<digits>" without leading zeros). Any other form -- a '\r',
 * a non-ASCII byte, a cell outside the plain form below -- returns
 * NRMS_ERR_UNSUPPORTED and the caller reads the file on its general path
 * (newsrecommendationsystem_amd/data.py), which also raises the reference's
 * errors. Values equal the general path's wherever these accept the input.
 *
 * behaviors.tsv: non-empty lines of at least five tab-separated columns
 * (impression id, user, time, history, impressions); impressions cell
 * "N<id>-<label>" tokens separated by single spaces (labels <= 9 digits);
 * history cell blank or "N<id>" tokens separated by single spaces (outer
 * spaces ignored, as str.strip). nrms_behaviors_scan checks the bytes and
 * writes upper bounds of the lines, candidate tokens and history ids into
 * counts[3]; nrms_behaviors_parse takes those (or any) capacities[3] and
 * fills, per line k: fields[10 k + 2 c], [.. + 1] = byte span of column c;
 * the candidates' numeric ids and labels and their count per line; the
 * history ids and their count; and hist_user[k] = the index of line k's
 * history string among the distinct history strings in first-seen order (an
 * empty field counts as " ", as the reference's fillna(' ')); counts[4] =
 * lines, candidates, history ids, distinct histories. NRMS_ERR_WORKSPACE
 * when a capacity is short. */
int32_t nrms_behaviors_scan(const char* buf, int64_t len, int64_t* counts);
int32_t nrms_behaviors_parse(const char* buf, int64_t len, const int64_t* capacity, int64_t* counts,
                             int64_t* fields, int64_t* cand_num, int32_t* labels, int64_t* cand_count,
                             int64_t* hist_num, int64_t* hist_count, int64_t* hist_user);
/* news_parsed.tsv: a header naming "id" and "title" columns, then rows whose
 * id is N<digits> and whose title is a list literal of exactly L ints
 * ("[12, 7, 0, ...]"). Writes *n_rows, and for the first `capacity` rows the
 * numeric id, the id's byte span [2] and the title [L]; NRMS_ERR_WORKSPACE
 * when there are more rows than `capacity` (*n_rows says how many). */
int32_t nrms_news_parse(const char* buf, int64_t len, int32_t L, int64_t* n_rows, int64_t* ids,
                        int64_t* id_spans, int64_t* titles, int64_t capacity);

#ifdef __cplusplus
}
#endif
#endif /* NRMS_HIP_H */
