// Shared device helpers and launch plumbing for libnrms_hip.so (gfx950 only).
#pragma once
#include <cstdio>
#include <cstdlib>

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nrms_hip.h"

namespace nrms {
namespace tl {
struct ClassifyJob;
struct TailJobs;
}  // namespace tl

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;  // CDNA wavefront

// Remember the last HIP failure per host thread (nrms_last_hip_error()).
void set_last_hip_error(hipError_t e);

inline int32_t launch_status() {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_last_hip_error(e);
    return NRMS_ERR_HIP;
  }
  return NRMS_OK;
}

__device__ __forceinline__ float qnan() { return __builtin_nanf(""); }

__device__ __forceinline__ float4 nan4() {
  const float n = qnan();
  return make_float4(n, n, n, n);
}

// Longest title / history the inference kernels take (K|V of a sequence of
// more than 64 rows are read through L2 instead of LDS).
constexpr int kMaxSeqLen = 4096;

// Raw-exp attention weights (ScaledDotProductAttention, multihead_self.py:
// 16-20): the reference computes e = exp(fl(d / sqrt(d_k))) in fp32 with NO max
// subtraction, then e / (sum e + 1e-8). The kernels take a fast path, one
// v_exp_f32 of d * log2(e) / sqrt(d_k) (a few ulp from expf), which can differ
// from the reference only where a row comes within ulps of fp32 overflow:
// e = inf there gives NaN weights, sum = inf gives zero weights. A row whose
// fast sum reaches kExpRecheck (2^120: a score of at least ~80, never seen in
// practice) or is not finite is recomputed with the reference's own arithmetic
// (ref_exp: correctly rounded division, ~1-ulp expf), so those boundaries fall
// where torch's do (tests/test_gpu_flow.py, overflow fixture at +-2 steps).
constexpr float kExpRecheck = 0x1p120f;
__device__ __forceinline__ bool exp_row_needs_recheck(float fast_sum) {
  return !(fast_sum < kExpRecheck);
}
__device__ __forceinline__ float ref_exp(float d, float sqrt_dk) { return expf(d / sqrt_dk); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// max that propagates NaN (torch.max semantics): any NaN lane -> NaN.
__device__ __forceinline__ float nan_max(float a, float b) {
  return (a != a || b != b) ? qnan() : fmaxf(a, b);
}

__device__ __forceinline__ float wave_max_nan(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = nan_max(v, __shfl_xor(v, o));
  return v;
}

// Exact three-way bf16 split of two floats at once: x = hi + mid + lo with
// each part the round-to-nearest bf16 of what the previous parts leave. The
// paired conversion (one v_cvt_pk_bf16_f32 per plane per pair) and v_pk_add_f32
// residuals take 4.5 VALU per element where converting one float at a time
// takes about 8; the packed words come out as [x0 | x1 << 16] per plane.
typedef __bf16 nrms_bf16x2 __attribute__((ext_vector_type(2)));
typedef float nrms_f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split3x2(float x0, float x1, uint32_t& hi, uint32_t& mid,
                                         uint32_t& lo) {
  hi = __builtin_bit_cast(uint32_t, __builtin_convertvector((nrms_f32x2){x0, x1}, nrms_bf16x2));
  const float r0 = x0 - __builtin_bit_cast(float, hi << 16);
  const float r1 = x1 - __builtin_bit_cast(float, hi & 0xffff0000u);
  mid = __builtin_bit_cast(uint32_t, __builtin_convertvector((nrms_f32x2){r0, r1}, nrms_bf16x2));
  const float s0 = r0 - __builtin_bit_cast(float, mid << 16);
  const float s1 = r1 - __builtin_bit_cast(float, mid & 0xffff0000u);
  lo = __builtin_bit_cast(uint32_t, __builtin_convertvector((nrms_f32x2){s0, s1}, nrms_bf16x2));
}

// Split-f16 x3 operands (NRMS_GEMM_SPLIT_F16X3): x = hi + 2^-11 lo with
// hi = fp16(x), lo = fp16((x - hi) 2^11) — 11 + 11 significand bits, relative
// error ~2^-22 for |x| >= ~1.2e-4 and at most ~1.5e-11 absolute below it. The
// residual scaled by 2^11 never overflows where hi does not; an x at or past
// 65,520 gives hi = inf, lo = -inf, and every product sum it enters becomes
// NaN. The weight side also keeps hi' = 2^11 hi (NaN where that overflows,
// |w| >= 32), so lo·hi + hi·lo + hi·hi' = 2^11 x·w in one accumulator.
// Used for the additive projections (news and UserEncoder): their outputs
// feed tanh and a max-subtracted softmax, so ulp-level operand rounding has no
// boundary effects there. The Q|K|V projections do not use this two-plane
// form: under SPLIT_F16X3 they scale rows into fp16's range and split the
// input exactly into three pieces (proj_x6.hip), so single-term products --
// and with them the raw-exp overflow boundary of the attention scores -- stay
// bit-exact with the reference.
constexpr float kF16LoScale = 2048.0f, kF16LoUnscale = 1.0f / 2048.0f;
typedef _Float16 nrms_f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 nrms_f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 nrms_f16x8 __attribute__((ext_vector_type(8)));
// packed [x0 | x1 << 16] words of hi and lo (one v_cvt_pk_f16_f32 per plane)
__device__ __forceinline__ void split2x2h(float x0, float x1, uint32_t& hi, uint32_t& lo) {
  const nrms_f16x2 h = __builtin_convertvector((nrms_f32x2){x0, x1}, nrms_f16x2);
  const nrms_f32x2 r = ((nrms_f32x2){x0, x1} - __builtin_convertvector(h, nrms_f32x2)) * kF16LoScale;
  hi = __builtin_bit_cast(uint32_t, h);
  lo = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, nrms_f16x2));
}
// Bijective XCD-aware block remap (cdna_hip_programming.md §5, "XCD swizzle
// must be bijective"): blocks dealt round-robin over 8 XCDs get contiguous
// logical ids per XCD, so tiles that share operands share an L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// Row segments of a stacked weight W[N, K] = [W_0; W_1; W_2] with biases
// (the Q|K|V projection is three nn.Linear weights used as one N = 3D GEMM).
struct WeightRows {
  const float* w[3];
  const float* b[3];   // may be null: no bias
  int seg_rows;
  int nseg;
  int accumulate = 0;  // store GEMMs: Y += X W^T (+ b)
};

// Run-time knobs read from the environment (the A/B switches of the launch
// folding and the compaction, measurement and test hooks): each is read once,
// and one that is set is announced on stderr, so a stray variable in a
// user's environment cannot change a layout or a dispatch silently.
inline const char* env_knob(const char* name) {
  const char* e = getenv(name);
  if (e) fprintf(stderr, "[nrms] environment knob %s=%s is active (non-default layout / dispatch)\n", name, e);
  return e;
}

// Row stride (floats) of the q|k|v rows the hot path writes and the fused
// kernels read: 3D, unpadded. Rows padded to whole 128-B lines (928 for
// D = 300) were measured slower end to end (0.911 vs 0.869 ms per bench step,
// same box, 2 reps each; 912 / 960: 0.877 / 0.906): the fused kernels' gathers
// read the same 16-B slice offset from every row, and with every row on a
// line boundary those slices all fall at one offset within the line.
// NRMS_QKV_STRIDE (measurement only, profiles/r5): a larger stride spreads
// the same rows over a larger address range (e.g. past the 256 MB Infinity
// Cache) without changing the bytes any kernel reads or writes.
inline int64_t qkv_row_stride(int D) {
  static const int64_t extra = [] {
    const char* e = env_knob("NRMS_QKV_STRIDE");
    return e ? (int64_t)atoll(e) - 900 : (int64_t)0;
  }();
  const int64_t s = (int64_t)3 * D;
  return (extra > 0 && s == 900 && (s + extra) % 4 == 0) ? s + extra : s;
}

// Process-wide GEMM arithmetic (nrms_set_gemm_arith; defined in capi.hip).
int gemm_arith();

// hipFuncAttributeMaxDynamicSharedMemorySize for `fn` on the calling thread's
// current device, set once per (device, kernel, size); thread-safe (capi.hip).
void ensure_dynamic_lds(const void* fn, int bytes);

// Addressing of a GEMM's A rows: logical row r (after the optional id
// indirection) lives at X + (r / per_batch) * stride_batch + (r % per_batch) *
// stride_row floats. The plain contiguous case is per_batch = INT64_MAX,
// stride_row = K; a [B, N, K] view with strides (sb, sn, 1) is per_batch = N.
struct ARows {
  int64_t per_batch;
  int64_t stride_batch;
  int64_t stride_row;
  __host__ __device__ __forceinline__ int64_t offset(int64_t r) const {
    return per_batch == INT64_MAX ? r * stride_row
                                  : (r / per_batch) * stride_batch + (r % per_batch) * stride_row;
  }
};
inline ARows contiguous_rows(int K) { return ARows{INT64_MAX, 0, K}; }

// Host-side launchers (defined in the .hip files).
int32_t launch_gather(const int64_t* ids, int64_t n_tok, const float* table, int64_t V, int D,
                      float* out, hipStream_t s);
int32_t launch_gemm_store(const float* X, int64_t n_rows_x, const int64_t* row_ids, int64_t M,
                          int K, const WeightRows& w, int N, float* Y, int64_t ldy,
                          hipStream_t s);
// Row-list GEMM (split arithmetic only): Y[rows[m]] = X[rows[m]] W^T + b for
// m < *count_dev (device memory); the grid covers max_rows.
int32_t launch_gemm_store_list(const float* X, int64_t n_rows_x, const int64_t* rows,
                               const int32_t* count_dev, int64_t max_rows, int K, const WeightRows& w,
                               int N, float* Y, int64_t ldy, hipStream_t s);
// Same, A rows addressed through `ar` (strided [B, N, K] input views).
int32_t launch_gemm_store_rows(const float* X, int64_t n_rows_x, ARows ar, const int64_t* row_ids,
                               int64_t M, int K, const WeightRows& w, int N, float* Y,
                               int64_t ldy, hipStream_t s);
// Q|K|V projection with W split once per call (proj_x6.hip): K = 300, N = 900,
// split arithmetic, no accumulate. The pack (proj_x6_pack_floats() floats,
// 16-B aligned) is written by launch_proj_x6_pack for one or two weight sets
// and read by launch_proj_x6 with the same h3. h3 = false: split-bf16 x6,
// bitwise the result of launch_gemm_store_rows / launch_gemm_store_list;
// h3 = true: scaled split-f16 x3 (proj_x6.hip). m_dev non-null: row-list mode
// (row_ids lists the rows, *m_dev their count; outputs written in place).
size_t proj_x6_pack_floats();
bool proj_x6_supported(int K, int N, const WeightRows& w);
int32_t launch_proj_x6_pack(const WeightRows& w0, float* d0, const WeightRows* w1, float* d1, bool h3,
                            hipStream_t s);
// tail (optional): work every workgroup runs after its items (titles.hpp).
int32_t launch_proj_x6(const float* X, int64_t n_rows_x, ARows ar, const int64_t* row_ids, int64_t M,
                       const float* packed, float* Y, int64_t ldy, const int32_t* m_dev, bool h3, hipStream_t s,
                       const tl::TailJobs* tail = nullptr);
// nrms_forward's weight packings in one launch (split arithmetic): both
// encoders' Q|K|V (launch_proj_x6_pack layout, h3 = f16), the news W_add into
// the fused news workspace (f16 planes too when f16) with its counters reset,
// and the UserEncoder W_add (x6 layout) into its workspace. cls (optional):
// the first half of the news titles' classification in the same launch
// (titles.hpp).
int32_t launch_forward_pack(const WeightRows& wn, float* pn, const WeightRows& wu, float* pu,
                            const float* news_wadd, float* news_ws, bool f16, const float* user_wadd,
                            float* user_ws, hipStream_t s, const tl::ClassifyJob* cls = nullptr);
int32_t launch_gemm_additive_score(const float* X, int64_t M, int K, const float* W,
                                   const float* b, const float* q, int N, float* score,
                                   hipStream_t s);
// ld: q|k|v row stride in floats (>= 3 H DK, a multiple of 4: the padded
// folded table of nrms_qkv_row_stride works as well as packed 3D rows)
int32_t launch_mhsa(const float* qkv, int64_t ld, int64_t n_rows, const int64_t* ids_a, int64_t n_seq_a,
                    const int64_t* ids_b, int64_t n_seq, int L, int H, int DK, float* ctx,
                    hipStream_t s);
int32_t launch_additive_pool(const float* x, const float* score, int64_t n_seq, int L, int D,
                             float* out, hipStream_t s);
// f32-MFMA store GEMM regardless of the process-wide arithmetic (training path).
int32_t launch_gemm_store_f32(const float* X, int64_t M, int K, const WeightRows& w, int N, float* Y,
                              int64_t ldy, hipStream_t s);
// Additive projection GEMM that also stores y = tanh(X W^T + b) [M, N] (training forward).
int32_t launch_gemm_additive_score_y(const float* X, int64_t M, int K, const float* W,
                                     const float* b, const float* q, int N, float* score,
                                     float* y_out, hipStream_t s);
// training kernels (train.hip)
int32_t launch_dropout(const float* x, float* y, int64_t n, float p, uint64_t seed, hipStream_t s);
int32_t launch_score_backward(const float* news, int64_t B, int C, int64_t sb, int64_t sc,
                              const float* user, int64_t su, int D, const float* dl, float* dnews,
                              float* duser, hipStream_t s);
// (deterministic: per-sequence dq / db partials in `part` [2][n_seq][Q], then a
// fixed-order reduction into dq, db)
int32_t launch_additive_backward_rows(const float* x, const float* y, const float* score,
                                      const float* q, const float* dout, int64_t n_seq, int L,
                                      int D, int Q, float* dx, float* dz, float* dq, float* db,
                                      float* part, hipStream_t s);
size_t additive_backward_part_floats(int64_t n_seq, int Q);
int32_t launch_mhsa_backward(const float* qkv, const float* dctx, int64_t n_seq, int L, int D,
                             int H, float* dqkv, hipStream_t s);
// dW += dY^T X (+ db += column sums of dY), deterministic: row-slice partials
// in `part` (gemm_tn_part_floats(N, K) floats), summed in slice order.
int32_t launch_gemm_tn(const float* dY, int64_t R, int N, const float* X, int K, float* dW,
                       float* db, float* part, hipStream_t s);
size_t gemm_tn_part_floats(int N, int K);
int32_t launch_transpose(const float* const* src, int nseg, int seg_rows, int cols, float* dst,
                         hipStream_t s);
int32_t launch_embedding_backward(const int64_t* ids, int64_t n_tok, const float* dx, int64_t V,
                                  int D, int64_t padding_idx, float* dtable, hipStream_t s);
// The same, deterministic: tokens sorted by id (stable radix sort: token order
// within an id), one wave per id summing its rows in token order.
size_t embedding_backward_sorted_bytes(int64_t n_tok, int64_t V);
int32_t launch_embedding_backward_sorted(const int64_t* ids, int64_t n_tok, const float* dx, int64_t V,
                                         int D, int64_t padding_idx, float* dtable, void* ws,
                                         size_t ws_bytes, hipStream_t s);
int32_t launch_adam_multi(const nrms_adam_tensor_t* ts, int n, float lr, float b1, float b2,
                          float eps, int64_t step, hipStream_t s);
int32_t launch_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr, float b1,
                    float b2, float eps, int64_t step, hipStream_t s);

// Device-side padding classification a deduplicating fused-news launch left
// in its workspace: pad_title[t] = 1 for all-padding titles (20 zero ids), and
// every such title t != *rep carries a copy of title *rep's vector (computed
// once; the computation of a title does not depend on where it is encoded).
// user_count: the launch's (zeroed) slot for launch_user_row_list's count.
struct PaddingGroups {
  const uint8_t* pad_title;
  const int32_t* rep;
  int32_t* user_count;
};
size_t fused_user_packed_b_floats();
bool fused_user_supported(int L, int D, int H, int Q);
// pg (optional): the clicked titles' padding flags. copied: rows m = b L + i
// of copied padding titles (see PaddingGroups) were not projected and are read
// from row *rep. compact (L <= 64): each user is encoded on its distinct rows,
// its padding positions collapsed into one row with their count
// (user_fused.hip). order (optional, B int32 of workspace, with compact):
// the users are dispatched longest compacted length first (NRMS_USER_LPT=0
// in the environment: in user order).
// nrms_forward's click scores folded into the UserEncoder launch: logits[b C
// + c] = news[b C + c] · user[b] in the score kernel's lane order and
// reduction (score.hip: bitwise its logits), computed by the user's workgroup
// once its vector is pooled.
struct ScoreFold {
  const float* news;   // [B C][D] candidate vectors, 16-B aligned (nullptr: no scores)
  float* logits;       // [B C]
  PaddingGroups pg;    // optional: a copied all-padding candidate reads rep's vector
  int64_t title0;      // title index of candidate 0 (pg)
  int C;
};
int32_t launch_fused_user(const float* qkv, int64_t ldq, int64_t B, int L, const float* w_add,
                          const float* b_add, const float* q_add, float* wap, float* out,
                          hipStream_t s, const PaddingGroups* pg = nullptr, bool prepacked = false,
                          bool copied = false, bool compact = false, int32_t* order = nullptr,
                          bool order_ready = false, const ScoreFold* score = nullptr);
// the longest-first user dispatch order is on (NRMS_USER_LPT, default 1)
bool user_lpt();
// Process-wide switch (news_fused.hip): encode one all-padding title per
// batch and broadcast its vector (nrms_set_title_dedupe; NRMS_DEDUPE=0 in the
// environment turns it off).
int title_dedupe();
int set_title_dedupe(int on);
// Process-wide switch (news_fused.hip): token compaction -- the id-0 tokens of
// a title share one q|k|v row, so the news tail encodes each distinct padding
// row once with its multiplicity (nrms_set_token_compaction; NRMS_COMPACT=0
// turns it off).
int token_compaction();
int set_token_compaction(int on);
// per-thread overrides of the two switches above (-1 clears; return the previous override)
int set_thread_title_dedupe(int on);
int set_thread_token_compaction(int on);

// workspace of launch_fused_news: packed W_add, special rows, recheck list
size_t fused_news_workspace_floats(int64_t n_titles);
bool fused_news_supported(int L, int D, int H, int Q);
// dedupe_setting / compact_setting: -1 = the process-wide setting
// (nrms_set_title_dedupe / nrms_set_token_compaction), else 0 / 1; *deduped
// (optional) tells whether the launch deduplicated the all-padding titles;
// *classified (optional) whether it classified them at all (the pad_title
// flags of fused_news_padding_groups are then valid until the workspace is
// reused).
// broadcast_from: the copies of the rep title's vector are written for titles
// >= broadcast_from only. user_list (optional): when the launch deduplicates,
// the main pass also builds launch_user_row_list's list of titles
// 0 .. user_rows - 1 (count in the PaddingGroups user_count). prepacked: ws
// already holds the packed W_add and reset counters (launch_forward_pack).
// preclassified: the titles were classified by the forward's split
// classification (fused_news_classify_split, titles.hpp) -- no classification
// launch here.
// direct_rows: the q|k|v rows are per token (row s L + i, the per-token
// projection); the ids (if any) only classify the tokens.
int32_t launch_fused_news(const float* qkv, int64_t ldq, int64_t n_rows, const int64_t* ids_a,
                          int64_t n_seq_a, const int64_t* ids_b, int64_t n_titles,
                          const float* w_add, const float* b_add, const float* q_add, float* ws,
                          float* out, hipStream_t s, int dedupe_setting = -1, bool* deduped = nullptr,
                          int64_t broadcast_from = 0, int64_t* user_list = nullptr, int64_t user_rows = 0,
                          bool prepacked = false, bool direct_rows = false, int compact_setting = -1,
                          bool* classified = nullptr, bool preclassified = false);
PaddingGroups fused_news_padding_groups(float* ws, int64_t n_titles);
// The rows m < n_rows of titles not copied from rep (the UserEncoder's rows to
// project), appended to list in any order; their count in *pg.user_count.
int32_t launch_user_row_list(const PaddingGroups& pg, int64_t n_rows, int64_t* list, hipStream_t s);
int32_t launch_score_pairs(const float* news, int64_t n_news, const float* user, int64_t n_users,
                           const int64_t* news_idx, const int64_t* user_idx, int64_t n_pairs,
                           int D, float* out, hipStream_t s);
int32_t launch_impression_metrics(const float* scores, const int32_t* labels,
                                  const int64_t* offsets, int64_t n_imp, double* out,
                                  hipStream_t s);
// pg (optional): candidates that are copied all-padding titles read the rep
// title's vector; the candidates are titles title0 + b C + c of a contiguous array
// (news points at title0's row).
int32_t launch_score(const float* news, int64_t B, int C, int64_t sb, int64_t sc,
                     const float* user, int64_t su, int D, float* out, hipStream_t s,
                     const PaddingGroups* pg = nullptr, int64_t title0 = 0);

}  // namespace nrms
