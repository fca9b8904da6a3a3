// C ABI (include/nrms_hip.h): argument validation, workspace carving and the
// stage order of the NRMS encoders. Every call only enqueues work on the
// caller's stream (no allocation, no synchronisation); the only globals are the
// process-wide GEMM arithmetic and the once-per-(device, kernel) LDS attribute.
#include "nrms_common.hpp"
#include "titles.hpp"

#include <atomic>
#include <cstdlib>
#include <mutex>
#include <set>
#include <tuple>

namespace nrms {

static thread_local int32_t g_last_hip = 0;
void set_last_hip_error(hipError_t e) { g_last_hip = (int32_t)e; }

static int initial_gemm_arith() {
  const char* e = env_knob("NRMS_GEMM");
  if (e && (e[0] == 'f' || e[0] == 'F')) return NRMS_GEMM_F32;
  if (e && (e[0] == 'x' || e[0] == 'X')) return NRMS_GEMM_SPLIT_BF16X6;
  return NRMS_GEMM_SPLIT_F16X3;
}
static std::atomic<int> g_gemm_arith{initial_gemm_arith()};
// A/B switches of nrms_forward's launch folding (default on; "0" turns off):
// NRMS_SPLIT_CLASSIFY -- the titles' classification in the pack launch and the
// vocabulary projection's tail (titles.hpp) instead of a launch of its own
// (the user dispatch order moves with it); NRMS_SCORE_FOLD -- the click scores
// in the UserEncoder launch instead of the score kernel.
static bool env_on(const char* name) {
  const char* e = env_knob(name);
  return !(e && e[0] == '0');
}
static const bool g_split_classify = env_on("NRMS_SPLIT_CLASSIFY");
// test only (tests/test_gpu_parity.py): classification half A in the pack
// launch but no tail jobs in the projection, so the news launch classifies
// again itself -- the fallback nrms_forward takes when the projection leaves
// its fragment path after the pack
static const bool g_skip_classify_tail = [] {
  const char* e = env_knob("NRMS_TEST_SKIP_CLASSIFY_TAIL");
  return e && e[0] == '1';
}();
static const bool g_score_fold = env_on("NRMS_SCORE_FOLD");
static thread_local int32_t t_gemm_arith = -1;   // nrms_set_thread_gemm_arith (-1: none)
int gemm_arith() {
  const int32_t t = t_gemm_arith;
  return t >= 0 ? t : g_gemm_arith.load(std::memory_order_relaxed);
}

void ensure_dynamic_lds(const void* fn, int bytes) {
  static std::mutex mu;
  static std::set<std::tuple<int, const void*, int>> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return;
  std::lock_guard<std::mutex> lock(mu);
  if (done.insert(std::make_tuple(dev, fn, bytes)).second)
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

namespace {

constexpr int kDK = 20;   // d_k = D / H supported by the attention kernel
constexpr int kQMax = 208;

size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

// Bump allocator over the caller's workspace.
struct Carve {
  char* base;
  size_t cap, off = 0;
  bool ok = true;
  float* floats(size_t n) {
    const size_t need = align_up(n * sizeof(float));
    if (off + need > cap) { ok = false; return nullptr; }
    float* p = reinterpret_cast<float*>(base + off);
    off += need;
    return p;
  }
};

bool weights_ok(const nrms_encoder_weights_t* w) {
  if (!w) return false;
  if (!w->w_q || !w->b_q || !w->w_k || !w->b_k || !w->w_v || !w->b_v || !w->w_add ||
      !w->b_add || !w->q_add)
    return false;
  return w->d_model > 0 && w->n_heads > 0 && w->query_dim > 0;
}

int32_t shape_ok(const nrms_encoder_weights_t* w) {
  if (!weights_ok(w)) return NRMS_ERR_INVALID_ARG;
  if (w->d_model % w->n_heads != 0) return NRMS_ERR_INVALID_ARG;  // multihead_self.py:31
  if (w->d_model / w->n_heads != kDK || w->n_heads != 15) return NRMS_ERR_UNSUPPORTED;
  if (w->query_dim > kQMax || w->d_model % 4 != 0) return NRMS_ERR_UNSUPPORTED;
  return NRMS_OK;
}

WeightRows qkv_rows(const nrms_encoder_weights_t* w) {
  WeightRows r{};
  r.w[0] = w->w_q; r.w[1] = w->w_k; r.w[2] = w->w_v;
  r.b[0] = w->b_q; r.b[1] = w->b_k; r.b[2] = w->b_v;
  r.seg_rows = w->d_model;
  r.nseg = 3;
  return r;
}

// q|k|v row stride of the hot path (nrms_qkv_row_stride; 3D since round 3)
int64_t news_ld(const nrms_encoder_weights_t* w, int32_t L) {
  return fused_news_supported(L, w->d_model, w->n_heads, w->query_dim) ? qkv_row_stride(w->d_model)
                                                                         : 3 * (int64_t)w->d_model;
}
int64_t user_ld(const nrms_encoder_weights_t* w, int32_t N) {
  return fused_user_supported(N, w->d_model, w->n_heads, w->query_dim) ? qkv_row_stride(w->d_model)
                                                                        : 3 * (int64_t)w->d_model;
}

bool use_folded(int32_t mode, int64_t n_tok, int64_t V) {
  if (mode == NRMS_PROJ_FOLDED) return true;
  if (mode == NRMS_PROJ_DIRECT) return false;
  return n_tok > V;
}

// Per-stage sizes (floats).
struct NewsSizes {
  size_t qkv, ctx, scores, wap, pack;
};
NewsSizes news_sizes(int64_t n_titles, int32_t L, int64_t V, int32_t D, bool folded) {
  const size_t ntok = (size_t)n_titles * (size_t)L;
  return {(folded ? (size_t)V : ntok) * (size_t)qkv_row_stride(D), ntok * (size_t)D, ntok,
          fused_news_workspace_floats(n_titles), proj_x6_pack_floats()};
}
size_t news_bytes(const NewsSizes& z) {
  return align_up(z.qkv * 4) + align_up(z.ctx * 4) + align_up(z.scores * 4) + align_up(z.wap * 4) +
         align_up(z.pack * 4);
}

// Q|K|V projection of the encoders: the pre-split-W kernel (proj_x6.hip) when
// the shape and arithmetic allow, packing w into `pack` first unless the
// caller already did (packed = true, with the same arith); the staged GEMM
// otherwise (x6: bitwise the same rows; f16x3: the kernel's scaled split-f16
// arithmetic, the staged GEMM's x6 rows only within rounding). list_count
// non-null: row-list mode (launch_gemm_store_list). arith < 0: the current mode.
int32_t project_qkv(const float* X, int64_t n_rows_x, ARows ar, const int64_t* row_ids, int64_t M,
                    const nrms_encoder_weights_t* w, float* pack, bool packed, float* Y, int64_t ld,
                    hipStream_t s, const int32_t* list_count = nullptr, int arith = -1,
                    const tl::TailJobs* tail = nullptr, bool* tail_done = nullptr) {
  const int D = w->d_model;
  const WeightRows wr = qkv_rows(w);
  if (arith < 0) arith = gemm_arith();
  const bool h3 = arith == NRMS_GEMM_SPLIT_F16X3;
  if (tail_done) *tail_done = false;
  if (pack && arith != NRMS_GEMM_F32 && proj_x6_supported(D, 3 * D, wr) && ((uintptr_t)Y % 16) == 0 &&
      ld % 4 == 0) {
    if (!packed)
      if (int32_t st = launch_proj_x6_pack(wr, pack, nullptr, nullptr, h3, s)) return st;
    const int32_t st = launch_proj_x6(X, n_rows_x, ar, row_ids, M, pack, Y, ld, list_count, h3, s, tail);
    if (tail_done) *tail_done = st == NRMS_OK && tail != nullptr;
    return st;
  }
  if (list_count) return launch_gemm_store_list(X, n_rows_x, row_ids, list_count, M, D, wr, 3 * D, Y, ld, s);
  return launch_gemm_store_rows(X, n_rows_x, ar, row_ids, M, D, wr, 3 * D, Y, ld, s);
}

// attention + additive pooling from projected rows (shared by news and user
// paths). `wap` non-null: use the fused news kernel when the geometry allows.
int32_t encode_from_qkv(const float* qkv, int64_t ldq, int64_t n_rows, const int64_t* ids_a,
                        int64_t n_seq_a, const int64_t* ids_b, int64_t n_seq, int32_t L,
                        const nrms_encoder_weights_t* w, float* ctx, float* scores, float* out,
                        hipStream_t s, float* wap = nullptr, bool* deduped = nullptr,
                        int64_t broadcast_from = 0, int64_t* user_list = nullptr, int64_t user_rows = 0,
                        bool prepacked = false, bool direct_rows = false, bool* classified = nullptr,
                        bool preclassified = false) {
  const int D = w->d_model;
  if (deduped) *deduped = false;
  if (classified) *classified = false;
  if (wap && fused_news_supported(L, D, w->n_heads, w->query_dim))
    return launch_fused_news(qkv, ldq, n_rows, ids_a, n_seq_a, ids_b, n_seq, w->w_add, w->b_add,
                             w->q_add, wap, out, s, -1, deduped, broadcast_from, user_list, user_rows,
                             prepacked, direct_rows, -1, classified, preclassified);
  if (preclassified) return NRMS_ERR_INVALID_ARG;
  if (direct_rows) ids_a = ids_b = nullptr;   // per-token rows: the ids only classify (fused kernel)
  // stage kernels: any row stride >= 3D (packed rows, or the folded table's
  // rows of nrms_qkv_row_stride)
  int32_t st = launch_mhsa(qkv, ldq, n_rows, ids_a, n_seq_a, ids_b, n_seq, L, w->n_heads, kDK, ctx, s);
  if (st) return st;
  st = launch_gemm_additive_score(ctx, n_seq * L, D, w->w_add, w->b_add, w->q_add, w->query_dim,
                                  scores, s);
  if (st) return st;
  return launch_additive_pool(ctx, scores, n_seq, L, D, out, s);
}

}  // namespace
}  // namespace nrms

using namespace nrms;

extern "C" {

int32_t nrms_abi_version(void) { return NRMS_ABI_VERSION; }

int32_t nrms_set_gemm_arith(int32_t mode) {
  if (mode != NRMS_GEMM_SPLIT_BF16X6 && mode != NRMS_GEMM_F32 && mode != NRMS_GEMM_SPLIT_F16X3)
    return -NRMS_ERR_INVALID_ARG;
  return g_gemm_arith.exchange(mode);
}

int32_t nrms_get_gemm_arith(void) { return gemm_arith(); }

int32_t nrms_set_title_dedupe(int32_t on) { return set_title_dedupe(on); }

int32_t nrms_set_token_compaction(int32_t on) { return set_token_compaction(on); }

int32_t nrms_set_thread_gemm_arith(int32_t mode) {
  if (mode != -1 && mode != NRMS_GEMM_SPLIT_BF16X6 && mode != NRMS_GEMM_F32 && mode != NRMS_GEMM_SPLIT_F16X3)
    return -NRMS_ERR_INVALID_ARG;
  const int32_t prev = t_gemm_arith;
  t_gemm_arith = mode;
  return prev;
}

int32_t nrms_set_thread_title_dedupe(int32_t on) {
  if (on < -1) return -NRMS_ERR_INVALID_ARG;
  return set_thread_title_dedupe(on);
}

int32_t nrms_set_thread_token_compaction(int32_t on) {
  if (on < -1) return -NRMS_ERR_INVALID_ARG;
  return set_thread_token_compaction(on);
}

const char* nrms_status_string(int32_t st) {
  switch (st) {
    case NRMS_OK: return "ok";
    case NRMS_ERR_INVALID_ARG: return "invalid argument";
    case NRMS_ERR_UNSUPPORTED: return "unsupported shape or alignment";
    case NRMS_ERR_WORKSPACE: return "workspace missing or too small";
    case NRMS_ERR_HIP: return "HIP launch failed";
    default: return "unknown status";
  }
}

int32_t nrms_last_hip_error(void) { return g_last_hip; }

int32_t nrms_embedding_gather(const int64_t* ids, int64_t n_tok, const float* table, int64_t V,
                              int32_t D, float* out, hipStream_t stream) {
  if (n_tok < 0 || V < 0 || D <= 0) return NRMS_ERR_INVALID_ARG;
  if (n_tok > 0 && (!ids || !table || !out)) return NRMS_ERR_INVALID_ARG;
  return launch_gather(ids, n_tok, table, V, D, out, stream);
}

int32_t nrms_qkv_row_stride(int32_t D) { return D > 0 ? (int32_t)qkv_row_stride(D) : 0; }

int32_t nrms_qkv_project(const float* x, int64_t n_rows_x, const int64_t* row_ids, int64_t M,
                         const nrms_encoder_weights_t* w, float* qkv, int64_t ld_qkv,
                         hipStream_t stream) {
  if (M < 0 || n_rows_x < 0) return NRMS_ERR_INVALID_ARG;
  if (int32_t st = shape_ok(w)) return st;
  if (M > 0 && (!x || !qkv)) return NRMS_ERR_INVALID_ARG;
  const int D = w->d_model;
  if (ld_qkv == 0) ld_qkv = 3 * D;
  if (ld_qkv < 3 * D) return NRMS_ERR_INVALID_ARG;
  return launch_gemm_store(x, n_rows_x, row_ids, M, D, qkv_rows(w), 3 * D, qkv, ld_qkv, stream);
}

size_t nrms_qkv_project_workspace_size(int32_t D) {
  return D > 0 ? align_up(proj_x6_pack_floats() * 4) : 0;
}

int32_t nrms_qkv_project_ws(const float* x, int64_t n_rows_x, const int64_t* row_ids, int64_t M,
                            const nrms_encoder_weights_t* w, float* qkv, int64_t ld_qkv, void* workspace,
                            size_t workspace_bytes, hipStream_t stream) {
  if (M < 0 || n_rows_x < 0) return NRMS_ERR_INVALID_ARG;
  if (int32_t st = shape_ok(w)) return st;
  if (M > 0 && (!x || !qkv)) return NRMS_ERR_INVALID_ARG;
  const int D = w->d_model;
  if (ld_qkv == 0) ld_qkv = 3 * D;
  if (ld_qkv < 3 * D) return NRMS_ERR_INVALID_ARG;
  if (M == 0) return NRMS_OK;
  Carve cv{static_cast<char*>(workspace), workspace ? workspace_bytes : 0};
  float* pack = cv.floats(proj_x6_pack_floats());
  if (!cv.ok) return NRMS_ERR_WORKSPACE;
  return project_qkv(x, n_rows_x, contiguous_rows(D), row_ids, M, w, pack, false, qkv, ld_qkv, stream);
}

int32_t nrms_self_attention(const float* qkv, int64_t n_rows_qkv, const int64_t* tok_ids,
                            int64_t n_seq_a, const int64_t* tok_ids_b, int64_t n_seq, int32_t L,
                            const nrms_encoder_weights_t* w, float* ctx, hipStream_t stream) {
  if (n_seq < 0 || n_seq_a < 0 || L <= 0) return NRMS_ERR_INVALID_ARG;
  if (int32_t st = shape_ok(w)) return st;
  if (n_seq > 0 && (!qkv || !ctx)) return NRMS_ERR_INVALID_ARG;
  return launch_mhsa(qkv, 3 * (int64_t)w->d_model, n_rows_qkv, tok_ids, n_seq_a, tok_ids_b, n_seq, L, w->n_heads, kDK, ctx,
                     stream);
}

int32_t nrms_additive_attention(const float* x, int64_t n_seq, int32_t L,
                                const nrms_encoder_weights_t* w, float* scores_ws, float* out,
                                hipStream_t stream) {
  if (n_seq < 0 || L <= 0) return NRMS_ERR_INVALID_ARG;
  if (int32_t st = shape_ok(w)) return st;
  if (n_seq > 0 && (!x || !scores_ws || !out)) return NRMS_ERR_INVALID_ARG;
  const int D = w->d_model;
  int32_t st = launch_gemm_additive_score(x, n_seq * L, D, w->w_add, w->b_add, w->q_add,
                                          w->query_dim, scores_ws, stream);
  if (st) return st;
  return launch_additive_pool(x, scores_ws, n_seq, L, D, out, stream);
}

int32_t nrms_additive_scores(const float* x, int64_t n_rows, const nrms_encoder_weights_t* w,
                             float* scores, hipStream_t stream) {
  if (n_rows < 0) return NRMS_ERR_INVALID_ARG;
  if (int32_t st = shape_ok(w)) return st;
  if (n_rows > 0 && (!x || !scores)) return NRMS_ERR_INVALID_ARG;
  return launch_gemm_additive_score(x, n_rows, w->d_model, w->w_add, w->b_add, w->q_add,
                                    w->query_dim, scores, stream);
}

int32_t nrms_additive_pool(const float* x, const float* scores, int64_t n_seq, int32_t L,
                           int32_t D, float* out, hipStream_t stream) {
  if (n_seq < 0 || L <= 0 || D <= 0) return NRMS_ERR_INVALID_ARG;
  if (n_seq > 0 && (!x || !scores || !out)) return NRMS_ERR_INVALID_ARG;
  return launch_additive_pool(x, scores, n_seq, L, D, out, stream);
}

size_t nrms_news_attention_pool_workspace_size(int64_t n_titles, int32_t L, int32_t D) {
  if (n_titles < 0 || L <= 0 || D <= 0) return 0;
  return align_up(fused_news_workspace_floats(n_titles) * 4);   // the context stays on chip
}

int32_t nrms_news_attention_pool(const float* qkv, int64_t ld_qkv, int64_t n_rows_qkv,
                                 const int64_t* tok_ids, int64_t n_seq_a, const int64_t* tok_ids_b,
                                 int64_t n_titles, int32_t L, const nrms_encoder_weights_t* w,
                                 float* out, void* workspace, size_t workspace_bytes,
                                 hipStream_t stream) {
  if (n_titles < 0 || n_seq_a < 0 || L <= 0) return NRMS_ERR_INVALID_ARG;
  if (int32_t st = shape_ok(w)) return st;
  if (!fused_news_supported(L, w->d_model, w->n_heads, w->query_dim)) return NRMS_ERR_UNSUPPORTED;
  if (n_titles == 0) return NRMS_OK;
  if (!qkv || !out) return NRMS_ERR_INVALID_ARG;
  Carve cv{static_cast<char*>(workspace), workspace ? workspace_bytes : 0};
  float* wap = cv.floats(fused_news_workspace_floats(n_titles));
  if (!cv.ok) return NRMS_ERR_WORKSPACE;
  if (ld_qkv == 0) ld_qkv = 3 * (int64_t)w->d_model;
  return launch_fused_news(qkv, ld_qkv, n_rows_qkv, tok_ids, n_seq_a, tok_ids_b, n_titles, w->w_add,
                           w->b_add, w->q_add, wap, out, stream);
}

size_t nrms_news_encode_workspace_size(int64_t n_titles, int32_t L, int64_t V, int32_t D,
                                       int32_t proj_mode) {
  if (n_titles < 0 || L <= 0 || V < 0 || D <= 0) return 0;
  const bool folded = use_folded(proj_mode, n_titles * L, V);
  return news_bytes(news_sizes(n_titles, L, V, D, folded));
}

int32_t nrms_news_encode(const int64_t* ids, int64_t n_titles, int32_t L, const float* table,
                         int64_t V, const nrms_encoder_weights_t* w, int32_t proj_mode, float* out,
                         void* workspace, size_t workspace_bytes, hipStream_t stream) {
  if (n_titles < 0 || L <= 0 || V <= 0) return NRMS_ERR_INVALID_ARG;
  if (int32_t st = shape_ok(w)) return st;
  if (n_titles == 0) return NRMS_OK;
  if (!ids || !table || !out) return NRMS_ERR_INVALID_ARG;
  const int D = w->d_model;
  const bool folded = use_folded(proj_mode, n_titles * L, V);
  const NewsSizes z = news_sizes(n_titles, L, V, D, folded);
  const int64_t ld = news_ld(w, L);
  Carve cv{static_cast<char*>(workspace), workspace ? workspace_bytes : 0};
  float* qkv = cv.floats(z.qkv);
  float* ctx = cv.floats(z.ctx);
  float* scores = cv.floats(z.scores);
  float* wap = cv.floats(z.wap);
  float* pack = cv.floats(z.pack);
  if (!cv.ok) return NRMS_ERR_WORKSPACE;
  int32_t st;
  if (folded) {
    // Vocabulary-level projection: one GEMM over the table, then rows gathered by id.
    st = project_qkv(table, V, contiguous_rows(D), nullptr, V, w, pack, false, qkv, ld, stream);
    if (st) return st;
    return encode_from_qkv(qkv, ld, V, ids, n_titles, nullptr, n_titles, L, w, ctx, scores, out,
                           stream, wap);
  }
  // Per-token projection with the embedding gather fused into the A-operand load.
  st = project_qkv(table, V, contiguous_rows(D), ids, n_titles * L, w, pack, false, qkv, ld, stream);
  if (st) return st;
  return encode_from_qkv(qkv, ld, n_titles * L, ids, n_titles, nullptr, n_titles, L, w, ctx,
                         scores, out, stream, wap, nullptr, 0, nullptr, 0, false, /*direct_rows=*/true);
}

size_t nrms_news_encode_folded_workspace_size(int64_t n_titles, int32_t L, int32_t D) {
  if (n_titles < 0 || L <= 0 || D <= 0) return 0;
  const size_t ntok = (size_t)n_titles * L;
  return align_up(ntok * D * 4) + align_up(ntok * 4) +
         align_up(fused_news_workspace_floats(n_titles) * 4);
}

int32_t nrms_news_encode_folded(const int64_t* ids, int64_t n_titles, int32_t L,
                                const float* qkv_table, int64_t ld_qkv, int64_t V,
                                const nrms_encoder_weights_t* w, float* out, void* workspace,
                                size_t workspace_bytes, hipStream_t stream) {
  if (n_titles < 0 || L <= 0 || V <= 0) return NRMS_ERR_INVALID_ARG;
  if (int32_t st = shape_ok(w)) return st;
  if (n_titles == 0) return NRMS_OK;
  if (!ids || !qkv_table || !out) return NRMS_ERR_INVALID_ARG;
  const size_t ntok = (size_t)n_titles * L;
  Carve cv{static_cast<char*>(workspace), workspace ? workspace_bytes : 0};
  float* ctx = cv.floats(ntok * w->d_model);
  float* scores = cv.floats(ntok);
  float* wap = cv.floats(fused_news_workspace_floats(n_titles));
  if (!cv.ok) return NRMS_ERR_WORKSPACE;
  if (ld_qkv == 0) ld_qkv = 3 * (int64_t)w->d_model;
  return encode_from_qkv(qkv_table, ld_qkv, V, ids, n_titles, nullptr, n_titles, L, w, ctx, scores,
                         out, stream, wap);
}

size_t nrms_user_encode_workspace_size(int64_t B, int32_t N, int32_t D) {
  if (B < 0 || N <= 0 || D <= 0) return 0;
  const size_t rows = (size_t)B * N;
  return align_up(rows * (size_t)qkv_row_stride(D) * 4) + align_up(rows * D * 4) + align_up(rows * 4) +
         align_up(fused_user_packed_b_floats() * 4) + align_up(proj_x6_pack_floats() * 4);
}

size_t nrms_user_attention_pool_workspace_size(int64_t B, int32_t N, int32_t D) {
  if (B < 0 || N <= 0 || D <= 0) return 0;
  return align_up(fused_user_packed_b_floats() * 4);
}

int32_t nrms_user_attention_pool(const float* qkv, int64_t ld_qkv, int64_t B, int32_t N,
                                 const nrms_encoder_weights_t* w, float* out, void* workspace,
                                 size_t workspace_bytes, hipStream_t stream) {
  if (B < 0 || N <= 0) return NRMS_ERR_INVALID_ARG;
  if (int32_t st = shape_ok(w)) return st;
  if (!fused_user_supported(N, w->d_model, w->n_heads, w->query_dim)) return NRMS_ERR_UNSUPPORTED;
  if (B == 0) return NRMS_OK;
  if (!qkv || !out) return NRMS_ERR_INVALID_ARG;
  Carve cv{static_cast<char*>(workspace), workspace ? workspace_bytes : 0};
  float* wap = cv.floats(fused_user_packed_b_floats());
  if (!cv.ok) return NRMS_ERR_WORKSPACE;
  if (ld_qkv == 0) ld_qkv = 3 * (int64_t)w->d_model;
  return launch_fused_user(qkv, ld_qkv, B, N, w->w_add, w->b_add, w->q_add, wap, out, stream);
}

int32_t nrms_user_attention_pool_padded(const float* qkv, int64_t ld_qkv, int64_t B, int32_t N,
                                        const uint8_t* pad_flags, const nrms_encoder_weights_t* w, float* out,
                                        void* workspace, size_t workspace_bytes, hipStream_t stream) {
  if (B < 0 || N <= 0) return NRMS_ERR_INVALID_ARG;
  if (int32_t st = shape_ok(w)) return st;
  if (!fused_user_supported(N, w->d_model, w->n_heads, w->query_dim)) return NRMS_ERR_UNSUPPORTED;
  if (B == 0) return NRMS_OK;
  if (!qkv || !out || !pad_flags) return NRMS_ERR_INVALID_ARG;
  Carve cv{static_cast<char*>(workspace), workspace ? workspace_bytes : 0};
  float* wap = cv.floats(fused_user_packed_b_floats());
  if (!cv.ok) return NRMS_ERR_WORKSPACE;
  if (ld_qkv == 0) ld_qkv = 3 * (int64_t)w->d_model;
  const bool compact = token_compaction() && N <= 64;
  const PaddingGroups pg{pad_flags, nullptr, nullptr};   // (no rep: every flagged row was projected)
  return launch_fused_user(qkv, ld_qkv, B, N, w->w_add, w->b_add, w->q_add, wap, out, stream,
                           compact ? &pg : nullptr, false, false, compact);
}

int32_t nrms_user_encode(const float* clicked, int64_t B, int32_t N, int64_t stride_b,
                         int64_t stride_n, const nrms_encoder_weights_t* w, float* out,
                         void* workspace, size_t workspace_bytes, hipStream_t stream) {
  if (B < 0 || N <= 0 || stride_b < 0 || stride_n < 0) return NRMS_ERR_INVALID_ARG;
  if (int32_t st = shape_ok(w)) return st;
  if (B == 0) return NRMS_OK;
  if (!clicked || !out) return NRMS_ERR_INVALID_ARG;
  const int D = w->d_model;
  const int64_t rows = B * N;
  Carve cv{static_cast<char*>(workspace), workspace ? workspace_bytes : 0};
  const int64_t ld = user_ld(w, N);
  float* qkv = cv.floats((size_t)rows * (size_t)ld);
  float* ctx = cv.floats((size_t)rows * D);
  float* scores = cv.floats((size_t)rows);
  float* wap = cv.floats(fused_user_packed_b_floats());
  float* pack = cv.floats(proj_x6_pack_floats());
  if (!cv.ok) return NRMS_ERR_WORKSPACE;
  // the [B, N, D] view is read in place (e.g. the transpose(0, 1) of
  // src/evaluate.py:220-224: stride_b = D, stride_n = B * D)
  const ARows ar = (stride_b == (int64_t)N * D && stride_n == D) ? contiguous_rows(D)
                                                                 : ARows{N, stride_b, stride_n};
  int32_t st = project_qkv(clicked, rows, ar, nullptr, rows, w, pack, false, qkv, ld, stream);
  if (st) return st;
  if (fused_user_supported(N, D, w->n_heads, w->query_dim) && ((uintptr_t)out % 16) == 0)
    return launch_fused_user(qkv, ld, B, N, w->w_add, w->b_add, w->q_add, wap, out, stream);
  return encode_from_qkv(qkv, ld, rows, nullptr, B, nullptr, B, N, w, ctx, scores, out, stream);
}

int32_t nrms_score(const float* news, int64_t B, int32_t C, int64_t stride_b, int64_t stride_c,
                   const float* user, int64_t stride_u, int32_t D, float* out,
                   hipStream_t stream) {
  if (B < 0 || C < 0 || D <= 0) return NRMS_ERR_INVALID_ARG;
  if (B * C > 0 && (!news || !user || !out)) return NRMS_ERR_INVALID_ARG;
  return launch_score(news, B, C, stride_b, stride_c, user, stride_u, D, out, stream);
}

int32_t nrms_score_pairs(const float* news, int64_t n_news, const float* user, int64_t n_users,
                         const int64_t* news_idx, const int64_t* user_idx, int64_t n_pairs,
                         int32_t D, float* out, hipStream_t stream) {
  if (n_pairs < 0 || n_news < 0 || n_users < 0 || D <= 0) return NRMS_ERR_INVALID_ARG;
  if (n_pairs > 0 && (!news || !user || !news_idx || !user_idx || !out)) return NRMS_ERR_INVALID_ARG;
  return launch_score_pairs(news, n_news, user, n_users, news_idx, user_idx, n_pairs, D, out, stream);
}

int32_t nrms_impression_metrics(const float* scores, const int32_t* labels,
                                const int64_t* offsets, int64_t n_imp, double* out,
                                hipStream_t stream) {
  if (n_imp < 0) return NRMS_ERR_INVALID_ARG;
  if (n_imp > 0 && (!scores || !labels || !offsets || !out)) return NRMS_ERR_INVALID_ARG;
  return launch_impression_metrics(scores, labels, offsets, n_imp, out, stream);
}

size_t nrms_forward_workspace_size(int64_t B, int32_t C, int32_t N, int32_t L, int64_t V,
                                   int32_t D, int32_t proj_mode) {
  if (B < 0 || C < 0 || N <= 0 || L <= 0 || V < 0 || D <= 0) return 0;
  const int64_t n_all = B * (C + N);
  return nrms_news_encode_workspace_size(n_all, L, V, D, proj_mode) +
         align_up((size_t)n_all * D * 4) + align_up((size_t)B * D * 4) +
         nrms_user_encode_workspace_size(B, N, D) + align_up((size_t)B * N * 8) + align_up((size_t)B * 4);
}

namespace {

// nrms_forward / nrms_forward_timed. ev (optional, NRMS_FORWARD_STAGES + 1
// events): recorded on the stream before each stage and after the last.
int32_t forward_impl(const int64_t* cand_ids, const int64_t* clicked_ids, int64_t B, int32_t C,
                     int32_t N, int32_t L, const float* table, int64_t V,
                     const nrms_encoder_weights_t* news_w, const nrms_encoder_weights_t* user_w,
                     int32_t proj_mode, float* logits, void* workspace, size_t workspace_bytes,
                     hipStream_t stream, hipEvent_t* ev) {
  if (B < 0 || C < 0 || N <= 0 || L <= 0 || V <= 0) return NRMS_ERR_INVALID_ARG;
  if (int32_t st = shape_ok(news_w)) return st;
  if (int32_t st = shape_ok(user_w)) return st;
  if (news_w->d_model != user_w->d_model) return NRMS_ERR_INVALID_ARG;
  if (B == 0) return NRMS_OK;
  if (!cand_ids || !clicked_ids || !table || !logits) return NRMS_ERR_INVALID_ARG;
  const int D = news_w->d_model;
  const int64_t n_clk = B * N, n_all = B * (C + N);
  const bool folded = use_folded(proj_mode, n_all * L, V);
  const NewsSizes z = news_sizes(n_all, L, V, D, folded);
  const int64_t ld = news_ld(news_w, L);
  const int64_t uld = user_ld(user_w, N);
  Carve cv{static_cast<char*>(workspace), workspace ? workspace_bytes : 0};
  float* qkv = cv.floats(z.qkv);
  float* ctx = cv.floats(z.ctx);
  float* scores = cv.floats(z.scores);
  float* wap = cv.floats(z.wap);
  float* pack = cv.floats(z.pack);
  float* news = cv.floats((size_t)n_all * D);   // [clicked B*N | candidates B*C] x D
  float* user = cv.floats((size_t)B * D);
  float* uqkv = cv.floats((size_t)n_clk * (size_t)uld);
  float* uctx = cv.floats((size_t)n_clk * D);
  float* uscores = cv.floats((size_t)n_clk);
  float* uwap = cv.floats(fused_user_packed_b_floats());
  float* upack = cv.floats(proj_x6_pack_floats());
  int64_t* ulist = reinterpret_cast<int64_t*>(cv.floats((size_t)n_clk * 2));
  int32_t* uorder = reinterpret_cast<int32_t*>(cv.floats((size_t)B));   // user dispatch order
  if (!cv.ok) return NRMS_ERR_WORKSPACE;
  auto rec = [&](int i) -> int32_t {
    if (ev && hipEventRecord(ev[i], stream) != hipSuccess) return launch_status();
    return NRMS_OK;
  };

  int32_t st;
  bool deduped = false, classified = false;
  const int arith = gemm_arith();
  const bool user_fused = fused_user_supported(N, D, user_w->n_heads, user_w->query_dim) &&
                          ((uintptr_t)user % 16) == 0;
  // with the UserEncoder's row-list projection the clicked padding titles'
  // vectors are never read, and the scorer reads a copied candidate from the
  // rep group: no copies are written
  const int64_t bcast_from = (user_fused && arith != NRMS_GEMM_F32) ? n_all : 0;
  // ... and the news kernel lists the UserEncoder's rows in its prologue
  const bool user_rows_here = user_fused && arith != NRMS_GEMM_F32;
  if ((st = rec(0))) return st;
  // every weight split / packing of the step in one launch: both encoders'
  // Q|K|V, and (fused tails) both W_add
  const WeightRows nwr = qkv_rows(news_w), uwr = qkv_rows(user_w);
  const bool packed = arith != NRMS_GEMM_F32 && proj_x6_supported(D, 3 * D, nwr);
  const bool h3 = arith == NRMS_GEMM_SPLIT_F16X3;
  const bool all_packed = packed && folded && user_fused;   // (the fused news tail takes folded + L = 20)
  const bool news_fused_ok = fused_news_supported(L, D, news_w->n_heads, news_w->query_dim);
  const bool prepacked = all_packed && news_fused_ok;
  // the titles' classification without a launch of its own (titles.hpp): the
  // first half in the pack launch, the second in the vocabulary projection's tail
  tl::ClassifyJob cjob{};
  tl::TailJobs ntail{};
  const bool split_cls =
      g_split_classify && prepacked && fused_news_classify_split(wap, clicked_ids, n_clk, cand_ids, n_all, V, &cjob, &ntail.sc);
  if (prepacked) {
    if ((st = launch_forward_pack(nwr, pack, uwr, upack, news_w->w_add, wap, h3, user_w->w_add, uwap, stream,
                                  split_cls ? &cjob : nullptr)))
      return st;
  } else if (packed && (st = launch_proj_x6_pack(nwr, pack, &uwr, upack, h3, stream))) {
    return st;
  }
  if (folded) {
    bool tail_done = false;
    st = project_qkv(table, V, contiguous_rows(D), nullptr, V, news_w, pack, packed, qkv, ld, stream, nullptr,
                     arith, (split_cls && !g_skip_classify_tail) ? &ntail : nullptr, &tail_done);
    if (st) return st;
    if ((st = rec(1))) return st;
    // (without the tail the news launch classifies the titles itself)
    st = encode_from_qkv(qkv, ld, V, clicked_ids, n_clk, cand_ids, n_all, L, news_w, ctx, scores,
                         news, stream, wap, &deduped, bcast_from, user_rows_here ? ulist : nullptr, n_clk,
                         prepacked, false, &classified, split_cls && tail_done);
  } else {
    st = project_qkv(table, V, contiguous_rows(D), clicked_ids, n_clk * L, news_w, pack, packed, qkv, ld,
                     stream, nullptr, arith);
    if (st) return st;
    st = project_qkv(table, V, contiguous_rows(D), cand_ids, B * C * L, news_w, pack, packed,
                     qkv + (size_t)n_clk * L * ld, ld, stream, nullptr, arith);
    if (st) return st;
    if ((st = rec(1))) return st;
    // (the ids only classify the tokens: the rows are per token; the all-padding
    // titles' copies are written for every title, so the UserEncoder and the
    // scorer read plain rows)
    st = encode_from_qkv(qkv, ld, n_all * L, clicked_ids, n_clk, cand_ids, n_all, L, news_w, ctx,
                         scores, news, stream, wap, nullptr, 0, nullptr, 0, false, /*direct_rows=*/true,
                         &classified);
  }
  if (st) return st;
  if ((st = rec(2))) return st;
  // UserEncoder (src/model/NRMS/user_encoder.py:15-26) over the clicked news
  // vectors. After a deduplicating news launch, the clicked titles of copied
  // all-padding groups have the rep group's vectors (bitwise; not written out
  // here, see bcast_from), so their q|k|v rows are the rep rows': only the
  // other rows are projected (row-list GEMM) and the fused tail reads copied
  // positions from the rep rows. Bitwise the same logits as projecting every row.
  const bool user_dedupe = deduped && user_fused && arith != NRMS_GEMM_F32;
  // UserEncoder token compaction (user_fused.hip): a user's padding positions
  // (one news vector) collapse into one row carrying their count
  const bool user_compact = user_fused && classified && token_compaction() && N <= 64;
  PaddingGroups pg{nullptr, nullptr, nullptr};
  const PaddingGroups pg_all = deduped ? fused_news_padding_groups(wap, n_all) : pg;
  const PaddingGroups pg_flags = classified ? fused_news_padding_groups(wap, n_all) : pg;
  // the users' longest-first dispatch order in the projection's tail (titles.hpp)
  tl::TailJobs utail{};
  const bool order_tail = g_split_classify && user_compact && user_lpt() && B * N <= INT32_MAX;
  if (order_tail) utail.uo = tl::UserOrder{pg_flags.pad_title, uorder, B, N};
  bool order_ready = false;
  if (user_dedupe) {
    pg = fused_news_padding_groups(wap, n_all);
    // (listed by the news kernel's prologue in the folded mode; the direct mode
    // has no ids to deduplicate by, so user_dedupe is false there)
    st = project_qkv(news, n_clk, contiguous_rows(D), ulist, n_clk, user_w, upack, packed, uqkv, uld, stream,
                     pg.user_count, arith, order_tail ? &utail : nullptr, &order_ready);
  } else {
    st = project_qkv(news, n_clk, contiguous_rows(D), nullptr, n_clk, user_w, upack, packed, uqkv, uld, stream,
                     nullptr, arith, order_tail ? &utail : nullptr, &order_ready);
  }
  if (st) return st;
  if ((st = rec(3))) return st;
  // the click scores in the fused UserEncoder launch (bitwise the score
  // kernel's; its stage is then empty)
  const float* cand_news = news + (size_t)n_clk * D;
  const PaddingGroups* cand_pg = bcast_from == n_all && deduped ? &pg_all : nullptr;
  const bool score_fold = g_score_fold && user_fused && C > 0 && ((uintptr_t)cand_news % 16) == 0;
  const ScoreFold sfold{cand_news, logits, cand_pg ? *cand_pg : PaddingGroups{nullptr, nullptr, nullptr}, n_clk, C};
  if (user_fused)
    st = launch_fused_user(uqkv, uld, B, N, user_w->w_add, user_w->b_add, user_w->q_add, uwap, user,
                           stream, (user_dedupe || user_compact) ? &pg_flags : nullptr, prepacked, user_dedupe,
                           user_compact, uorder, order_ready, score_fold ? &sfold : nullptr);
  else
    st = encode_from_qkv(uqkv, uld, n_clk, nullptr, B, nullptr, B, N, user_w, uctx, uscores, user,
                         stream);
  if (st) return st;
  if ((st = rec(4))) return st;
  if (!score_fold) {
    st = launch_score(cand_news, B, C, (int64_t)C * D, D, user, D, D, logits, stream, cand_pg, n_clk);
    if (st) return st;
  }
  return rec(5);
}

}  // namespace

int32_t nrms_forward(const int64_t* cand_ids, const int64_t* clicked_ids, int64_t B, int32_t C,
                     int32_t N, int32_t L, const float* table, int64_t V,
                     const nrms_encoder_weights_t* news_w, const nrms_encoder_weights_t* user_w,
                     int32_t proj_mode, float* logits, void* workspace, size_t workspace_bytes,
                     hipStream_t stream) {
  return forward_impl(cand_ids, clicked_ids, B, C, N, L, table, V, news_w, user_w, proj_mode, logits,
                      workspace, workspace_bytes, stream, nullptr);
}

int32_t nrms_forward_timed(const int64_t* cand_ids, const int64_t* clicked_ids, int64_t B, int32_t C,
                           int32_t N, int32_t L, const float* table, int64_t V,
                           const nrms_encoder_weights_t* news_w, const nrms_encoder_weights_t* user_w,
                           int32_t proj_mode, float* logits, void* workspace, size_t workspace_bytes,
                           hipStream_t stream, hipEvent_t* stage_events, int32_t n_events) {
  if (n_events != 0 && (n_events != NRMS_FORWARD_STAGES + 1 || !stage_events))
    return NRMS_ERR_INVALID_ARG;
  return forward_impl(cand_ids, clicked_ids, B, C, N, L, table, V, news_w, user_w, proj_mode, logits,
                      workspace, workspace_bytes, stream, n_events ? stage_events : nullptr);
}

const char* nrms_forward_stage_name(int32_t i) {
  static const char* names[NRMS_FORWARD_STAGES] = {"qkv_news", "news_fused", "qkv_user", "user_fused",
                                                   "score"};
  return (i >= 0 && i < NRMS_FORWARD_STAGES) ? names[i] : nullptr;
}


// ---------------------------------------------------------------------------
// Training kernels (train-mode forward pieces, backward, optimizer step).

int32_t nrms_dropout(const float* x, float* y, int64_t n, float p, uint64_t seed,
                     hipStream_t stream) {
  if (n < 0 || !(p >= 0.f && p < 1.f)) return NRMS_ERR_INVALID_ARG;
  if (n > 0 && (!x || !y)) return NRMS_ERR_INVALID_ARG;
  return launch_dropout(x, y, n, p, seed, stream);
}

int32_t nrms_additive_forward_train(const float* x, int64_t n_seq, int32_t L,
                                    const nrms_encoder_weights_t* w, float* y_tanh, float* scores,
                                    float* out, hipStream_t stream) {
  if (n_seq < 0 || L <= 0) return NRMS_ERR_INVALID_ARG;
  if (!weights_ok(w)) return NRMS_ERR_INVALID_ARG;
  if (n_seq == 0) return NRMS_OK;
  if (!x || !y_tanh || !scores || !out) return NRMS_ERR_INVALID_ARG;
  int32_t st = launch_gemm_additive_score_y(x, n_seq * L, w->d_model, w->w_add, w->b_add, w->q_add,
                                            w->query_dim, scores, y_tanh, stream);
  if (st) return st;
  return launch_additive_pool(x, scores, n_seq, L, w->d_model, out, stream);
}

size_t nrms_additive_backward_workspace_size(int64_t n_seq, int32_t L, int32_t D, int32_t Q) {
  if (n_seq < 0 || L <= 0 || D <= 0 || Q <= 0) return 0;
  return align_up((size_t)n_seq * L * Q * 4) + align_up((size_t)D * Q * 4) +
         align_up(additive_backward_part_floats(n_seq, Q) * 4) + align_up(gemm_tn_part_floats(Q, D) * 4);
}

int32_t nrms_additive_backward(const float* x, int64_t n_seq, int32_t L,
                               const nrms_encoder_weights_t* w, const float* y_tanh,
                               const float* scores, const float* dout, float* dx, float* d_w_add,
                               float* d_b_add, float* d_q_add, void* workspace,
                               size_t workspace_bytes, hipStream_t stream) {
  if (n_seq < 0 || L <= 0) return NRMS_ERR_INVALID_ARG;
  if (!weights_ok(w)) return NRMS_ERR_INVALID_ARG;
  if (n_seq == 0) return NRMS_OK;
  if (!x || !y_tanh || !scores || !dout || !dx || !d_w_add || !d_b_add || !d_q_add)
    return NRMS_ERR_INVALID_ARG;
  const int D = w->d_model, Q = w->query_dim;
  if (D % 4 != 0 || Q % 4 != 0) return NRMS_ERR_UNSUPPORTED;
  Carve cv{static_cast<char*>(workspace), workspace ? workspace_bytes : 0};
  float* dz = cv.floats((size_t)n_seq * L * Q);
  float* waT = cv.floats((size_t)D * Q);
  float* part_rows = cv.floats(additive_backward_part_floats(n_seq, Q));
  float* part_tn = cv.floats(gemm_tn_part_floats(Q, D));
  if (!cv.ok) return NRMS_ERR_WORKSPACE;
  int32_t st = launch_additive_backward_rows(x, y_tanh, scores, w->q_add, dout, n_seq, L, D, Q, dx,
                                             dz, d_q_add, d_b_add, part_rows, stream);
  if (st) return st;
  const float* wa[1] = {w->w_add};
  st = launch_transpose(wa, 1, Q, D, waT, stream);   // [Q, D] -> [D, Q]
  if (st) return st;
  WeightRows r{};
  r.w[0] = waT;
  r.b[0] = nullptr;
  r.seg_rows = D;
  r.nseg = 1;
  r.accumulate = 1;
  st = launch_gemm_store_f32(dz, n_seq * L, Q, r, D, dx, D, stream);   // dx += dz W_add
  if (st) return st;
  return launch_gemm_tn(dz, n_seq * L, Q, x, D, d_w_add, nullptr, part_tn, stream);   // dW += dz^T x
}

int32_t nrms_self_attention_backward(const float* qkv, const float* dctx, int64_t n_seq,
                                     int32_t L, const nrms_encoder_weights_t* w, float* dqkv,
                                     hipStream_t stream) {
  if (n_seq < 0 || L <= 0) return NRMS_ERR_INVALID_ARG;
  if (int32_t st = shape_ok(w)) return st;
  if (n_seq == 0) return NRMS_OK;
  if (!qkv || !dctx || !dqkv) return NRMS_ERR_INVALID_ARG;
  return launch_mhsa_backward(qkv, dctx, n_seq, L, w->d_model, w->n_heads, dqkv, stream);
}

size_t nrms_qkv_project_backward_workspace_size(int32_t D) {
  if (D <= 0) return 0;
  return align_up((size_t)3 * D * D * 4) + align_up(gemm_tn_part_floats(3 * D, D) * 4);
}

int32_t nrms_qkv_project_backward(const float* x, int64_t rows, const nrms_encoder_weights_t* w,
                                  const float* dqkv, float* dx, float* d_w_qkv, float* d_b_qkv,
                                  void* workspace, size_t workspace_bytes, hipStream_t stream) {
  if (rows < 0) return NRMS_ERR_INVALID_ARG;
  if (!weights_ok(w)) return NRMS_ERR_INVALID_ARG;
  if (rows == 0) return NRMS_OK;
  if (!x || !dqkv || !d_w_qkv || !d_b_qkv) return NRMS_ERR_INVALID_ARG;
  const int D = w->d_model;
  int32_t st;
  Carve cv{static_cast<char*>(workspace), workspace ? workspace_bytes : 0};
  float* wT = cv.floats((size_t)3 * D * D);
  float* part_tn = cv.floats(gemm_tn_part_floats(3 * D, D));
  if (!cv.ok) return NRMS_ERR_WORKSPACE;
  if (dx) {
    const float* ws3[3] = {w->w_q, w->w_k, w->w_v};
    st = launch_transpose(ws3, 3, D, D, wT, stream);   // [3D, D] -> [D, 3D]
    if (st) return st;
    WeightRows r{};
    r.w[0] = wT;
    r.b[0] = nullptr;
    r.seg_rows = D;
    r.nseg = 1;
    st = launch_gemm_store_f32(dqkv, rows, 3 * D, r, D, dx, D, stream);   // dx = dqkv [Wq; Wk; Wv]
    if (st) return st;
  }
  return launch_gemm_tn(dqkv, rows, 3 * D, x, D, d_w_qkv, d_b_qkv, part_tn, stream);
}

int32_t nrms_score_backward(const float* news, int64_t B, int32_t C, int64_t stride_b,
                            int64_t stride_c, const float* user, int64_t stride_u, int32_t D,
                            const float* dlogits, float* dnews, float* duser, hipStream_t stream) {
  if (B < 0 || C < 0 || D <= 0) return NRMS_ERR_INVALID_ARG;
  if (B * C > 0 && (!news || !user || !dlogits || !dnews || !duser)) return NRMS_ERR_INVALID_ARG;
  return launch_score_backward(news, B, C, stride_b, stride_c, user, stride_u, D, dlogits, dnews,
                               duser, stream);
}

int32_t nrms_embedding_backward(const int64_t* ids, int64_t n_tok, const float* dx, int64_t V,
                                int32_t D, int64_t padding_idx, float* dtable,
                                hipStream_t stream) {
  if (n_tok < 0 || V <= 0 || D <= 0) return NRMS_ERR_INVALID_ARG;
  if (n_tok > 0 && (!ids || !dx || !dtable)) return NRMS_ERR_INVALID_ARG;
  return launch_embedding_backward(ids, n_tok, dx, V, D, padding_idx, dtable, stream);
}

size_t nrms_embedding_backward_workspace_size(int64_t n_tok, int64_t V) {
  if (n_tok < 0 || V <= 0) return 0;
  return embedding_backward_sorted_bytes(n_tok, V);
}

int32_t nrms_embedding_backward_ws(const int64_t* ids, int64_t n_tok, const float* dx, int64_t V, int32_t D,
                                   int64_t padding_idx, float* dtable, void* workspace, size_t workspace_bytes,
                                   hipStream_t stream) {
  if (n_tok < 0 || V <= 0 || D <= 0) return NRMS_ERR_INVALID_ARG;
  if (n_tok > 0 && (!ids || !dx || !dtable)) return NRMS_ERR_INVALID_ARG;
  return launch_embedding_backward_sorted(ids, n_tok, dx, V, D, padding_idx, dtable, workspace, workspace_bytes,
                                          stream);
}

int32_t nrms_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                       int64_t n, float lr, float beta1, float beta2, float eps, int64_t step,
                       hipStream_t stream) {
  if (n < 0 || step < 1) return NRMS_ERR_INVALID_ARG;
  if (n > 0 && (!param || !grad || !exp_avg || !exp_avg_sq)) return NRMS_ERR_INVALID_ARG;
  return launch_adam(param, grad, exp_avg, exp_avg_sq, n, lr, beta1, beta2, eps, step, stream);
}

int32_t nrms_adam_step_multi(const nrms_adam_tensor_t* tensors, int32_t n, float lr, float beta1,
                             float beta2, float eps, int64_t step, hipStream_t stream) {
  if (n < 0 || step < 1) return NRMS_ERR_INVALID_ARG;
  if (n > 0 && !tensors) return NRMS_ERR_INVALID_ARG;
  for (int32_t i = 0; i < n; ++i) {
    const nrms_adam_tensor_t& t = tensors[i];
    if (t.numel < 0) return NRMS_ERR_INVALID_ARG;
    if (t.numel > 0 && (!t.param || !t.grad || !t.exp_avg || !t.exp_avg_sq))
      return NRMS_ERR_INVALID_ARG;
  }
  return launch_adam_multi(tensors, n, lr, beta1, beta2, eps, step, stream);
}

}  // extern "C"
