// Fused NewsEncoder tail: raw-exp MHSA -> additive projection -> tanh·q
// scores -> softmax over tokens -> pooled news vector, one persistent launch
// (src/model/NRMS/news_encoder.py:42-47, multihead_self.py:15-23,74-75,
// additive.py:35-52). Everything that is a contraction runs on the matrix
// cores in exact fp32; the context never leaves the CU.
//
// One workgroup (4 waves, one per SIMD, up to 512 registers each) per CU walks
// title groups of 4 titles (80 token rows). Per title group:
//
//   A  attention, wave w = heads 4w..4w+3 (wave 3: 12..14) with
//      v_mfma_f32_4x4x1_16b_f32: its 16 blocks are the 16 (title, head) pairs
//      of the wave, so the block-diagonal 20x20 attention products run at the
//      full f32 matrix rate (no padding). Lane (block b, x) holds the Q and K
//      slices of tokens {x, x+4, .., x+16} and dims 5x..5x+4 of all 20 V
//      rows, loaded straight from the projected rows into registers.
//        S^T = K·Q^T (25 4x4 tiles x 20 dims): lane x ends up holding the
//        scores of queries {x, x+4, ..} against all 20 keys, so exp (v_exp_f32
//        of the pre-scaled score, no max subtraction, as the reference), the
//        row sums and the division by (sum + 1e-8) are lane-local;
//        ctx^T = V^T·P^T (25 tiles x 20 keys): P is already in the B-operand
//        layout; lane x ends up with all 20 dims of its 5 query rows, stored
//        to the LDS context tile ctx[80][300] (+4 zero columns).
//   B  additive GEMM Y[80 x 208] = ctx · Wa^T with v_mfma_f32_16x16x4_f32,
//      A fragments ds_read_b128 from the context tile (row stride 328 floats:
//      conflict-free), B fragments from a pre-packed L2-resident copy of Wa
//      (one global_load_dwordx4 per lane per 16-deep k-group and N tile);
//      epilogue: per-row partials of sum_n q[n]·tanh(Y + b[n]) -> LDS.
//   C  softmax over the 20 tokens (max-subtracted, as F.softmax) and pooling
//      out[t] = sum_i w_i ctx[20t + i] from the attention's own O registers:
//      the 4 lanes of a block hold all 20 rows of one (title, head), so both
//      reduce inside the lane quad (DPP); the LDS tile is not read again.
//
// Two workgroup barriers per title group (after A and after B); the next
// group's q|k slices are loaded in the B epilogue, its V slices at the end
// of C.
// Output tile ownership in B (13 N-tiles x 5 M-tiles of 16x16): wave w owns
// N-tiles 3w..3w+2 for all 5 M-tiles plus (M-tile w, N-tile 12); wave 0 also
// (M-tile 4, N-tile 12).
#include "nrms_common.hpp"
#include "packs.hpp"
#include "titles.hpp"

#include <atomic>
#include <cstdlib>
#include <type_traits>

namespace nrms {
namespace {

constexpr int FT = 4;                // titles per group
constexpr int FL = 20;               // tokens per title (config.num_words_title)
constexpr int FROWS = FT * FL;       // 80 token rows
constexpr int FD = 300, FH = 15, FDK = 20, FQ = 200;
constexpr int FKG = 19;              // k-groups of 16 (K = 300 padded to 304)
constexpr int FNT = 13;              // N tiles of 16 (208 >= Q)
constexpr int SC = 328;              // context row stride in floats (== 8 mod 32)
constexpr int NTHR = 256;
constexpr int WAP_FLOATS = FKG * FNT * 64 * 4;             // packed Wa
constexpr int ROW = (3 * FD + 31) / 32 * 32;               // zero / NaN row slots (928 floats: room for any q|k|v offset)
constexpr int SPECIAL_FLOATS = 2 * ROW;                    // zero row + NaN row
// after the context tile: row partials [80][PART_STRIDE] (the four waves' N-tile
// sums + the N-tile-12 sum), row pointers [RPB][80] (u64), title meta [RPB][8]
// and the group schedule [16] (int32). RPB buffers: a group's row pointers are
// written two groups ahead (its Q slices load during the previous group's
// attention), and a buffer is rewritten only after a barrier past its readers.
constexpr int PART_STRIDE = 8;
constexpr int RPB = 4;
constexpr int TAIL_FLOATS = PART_STRIDE * FROWS + 2 * RPB * FROWS + 8 * RPB + 16;
constexpr int LDS_FLOATS = FROWS * SC + TAIL_FLOATS;   // ctx, partials, rowptr, meta
constexpr size_t LDS_BYTES = LDS_FLOATS * sizeof(float);

// Split-bf16 GEMM variant (X6): the context is stored as three bf16 planes
// hi | mid | lo with hi + mid + lo == ctx exactly (8 + 8 + 8 significand
// bits, each residual exact in fp32), and Wa likewise; the additive GEMM sums
// the six products with i + j <= 2 on v_mfma_f32_16x16x32_bf16 (exact bf16
// products, fp32 accumulation). The dropped terms are < 2^-25 |a||b|, below
// one fp32 rounding: the result is as accurate as an fp32 GEMM (tested against
// the fp64 oracle) at 6/16 of the f32-MFMA time.
constexpr int XKS = 10;                   // k-steps of 32 (K = 300 padded to 320)
constexpr int XKP = XKS * 32;             // 320
// Row stride in bf16: 976 (1,952 B = 488 dwords, = 8 mod 32 and 40 mod 64).
// Conflict-free both ways: the A-fragment ds_read_b128 lane groups (16 rows x
// 4 kq, bank = dword mod 64) cover all 64 banks once, and the attention's
// ds_write_b64 plane stores (16-lane groups: 4 rows x 4 heads, bank = dword
// mod 32) hit 16 distinct bank pairs. (968 = 484 dwords, = 4 mod 32, was
// read-conflict-free but 2-way on the stores: 57 M conflict cycles/launch.)
#ifndef NRMS_XRB_PAD
#define NRMS_XRB_PAD 16
#endif
constexpr int XRB = 3 * XKP + NRMS_XRB_PAD;
constexpr int WAP3_FLOATS = XKS * FNT * 3 * 64 * 4;   // [ks][nt][plane][lane][8 bf16]
constexpr int WAP_MAX = WAP3_FLOATS > WAP_FLOATS ? WAP3_FLOATS : WAP_FLOATS;
constexpr size_t LDS_BYTES_X6 = (size_t)FROWS * XRB * 2 + TAIL_FLOATS * sizeof(float);
static_assert(LDS_BYTES_X6 <= 160 * 1024, "LDS (x6)");
static_assert((FROWS * XRB * 2) % 16 == 0 && (XRB * 2) % 16 == 0, "x6 row stride");
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

// Split-f16 x3 variant (F16X3, main pass only): the context and Wa are split
// into two fp16 planes, a = hi + 2^-11 lo (hi = fp16(a), lo = fp16((a - hi)
// 2^11): 11 + 11 significand bits; the scaled residual stays normal down to
// |a| ~ 6e-5 and never overflows where hi does not). Wa's third operand,
// hi' = 2^11 hi (exact), is formed in registers from the hi plane (the pack
// also stores it; the kernel loads two planes), so the three products lo·hi,
// hi·lo, hi·hi' all carry the factor 2^11 and sum in ONE fp32 accumulator on
// v_mfma_f32_16x16x32_f16 (exact fp16 products): Y = 2^-11 acc. The dropped
// lo·lo term and the operand residuals are ~2^-22 |a||b| — normwise error
// below a plain fp32 GEMM's at half the x6 MFMA count.
// fp16's range is the price. A context value at or beyond 65,520 becomes inf
// in hi and -inf in lo, so lo·hi + hi·hi' is inf - inf = NaN in every output
// column of its row; a weight with |hi'| past fp16 has NaN packed in hi. Either
// way the row's score is NaN, and the score check in C routes the group to
// the recheck pass (x6 + reference exp), as it does for NaN inputs.
// Row stride 720 halves = 360 dwords (= 40 mod 64, 8 mod 32): the same bank
// pattern as the x6 stride, conflict-free for the fragment reads and the
// plane stores.
constexpr int XRH = 2 * XKP + 80;
constexpr int WAP2_FLOATS = XKS * FNT * 3 * 64 * 4;   // [ks][nt][plane hi' | lo | hi][lane][8 f16]
constexpr size_t LDS_BYTES_H = (size_t)FROWS * XRH * 2 + TAIL_FLOATS * sizeof(float);
static_assert(LDS_BYTES_H <= 160 * 1024 && (XRH / 2) % 64 == 40, "f16x3 row stride");
constexpr float kLoUnscale = kF16LoUnscale;
typedef nrms_f16x8 f16x8;

__device__ __forceinline__ void split3(float x, __bf16& hi, __bf16& mid, __bf16& lo) {
  hi = (__bf16)x;
  const float r = x - (float)hi;
  mid = (__bf16)r;
  lo = (__bf16)(r - (float)mid);
}

static_assert(FD == FH * FDK && FDK == 20 && FL == 20, "geometry");
static_assert(FKG * 16 >= FD && SC >= FKG * 16, "K padding");
static_assert(LDS_BYTES <= 160 * 1024, "LDS");

// WaP[c][nt][lane][4]: the B fragments of k-group c for lane (n = lane & 15,
// kq = lane >> 4): Wa[16 nt + n][16 c + 4 kq + t], t = 0..3 (0 past Q or D).
// After it: a zero q|k|v row (padding titles) and a NaN row (invalid ids).
__global__ __launch_bounds__(256) void pack_additive_b_kernel(const float* __restrict__ Wa,
                                                              float* __restrict__ WaP,
                                                              int32_t* __restrict__ recheck_count) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx < pk::NEWS_NCOUNT)   // [recheck count, bucket counts x5, rep, user row-list count, group claims, spare]
    recheck_count[idx] = idx == pk::NEWS_CNT_REP ? INT32_MAX : 0;
  if (idx >= WAP_FLOATS + SPECIAL_FLOATS) return;
  if (idx >= WAP_FLOATS) {
    const int sidx = idx - WAP_FLOATS;
    WaP[WAP_MAX + sidx] = sidx < ROW ? 0.f : qnan();
    return;
  }
  const int t = idx & 3;
  const int lane = (idx >> 2) & 63;
  const int nt = (idx >> 8) % FNT;
  const int c = (idx >> 8) / FNT;
  const int n = 16 * nt + (lane & 15);
  const int k = 16 * c + 4 * (lane >> 4) + t;
  WaP[idx] = (n < FQ && k < FD) ? Wa[n * FD + k] : 0.f;
}

// X6: WaP3[ks][nt][plane][lane][8] bf16 = plane of Wa[16 nt + (lane & 15)][32 ks + 8 (lane >> 4) + i]
// (the B-operand fragments of v_mfma_f32_16x16x32_bf16), zero past Q or D.
// F16: also the fp16 planes WaP2[ks][nt][plane][lane][8] (2^11 hi, the
// 2^11-scaled residual, hi) after the special rows, for the F16X3 main pass.
template <bool F16>
__global__ __launch_bounds__(256) void pack_additive_b3_kernel(const float* __restrict__ Wa,
                                                               float* __restrict__ WaP,
                                                               int32_t* __restrict__ recheck_count) {
  pk::pack_news_additive<F16>(blockIdx.x * 256 + threadIdx.x, Wa, WaP, recheck_count);
}
static_assert(pk::NEWS_WAP_MAX == WAP_MAX && pk::NEWS_SPECIAL == SPECIAL_FLOATS && pk::KS == XKS &&
                  pk::NT == FNT && pk::Q == FQ && pk::D == FD && pk::NEWS_X6_ELEMS == XKS * FNT * 64 * 8,
              "packs.hpp layout");
static_assert(pk::NEWS_COUNTERS == WAP_MAX + SPECIAL_FLOATS + WAP2_FLOATS, "packs.hpp counters");


// ------------------------------------------------------------------ titles and rows
//
// Token compaction. Every id-0 token of a title (the right-padding of titles
// shorter than 20 words, src/data_preprocess.py:115,132-139) has the same
// q|k|v row, so it gives the same attention scores against every key and the
// same context row as a query. A title with c real tokens (ids != 0) and
// n_pad = 20 - c padding tokens is therefore encoded on Le = c + (n_pad > 0)
// distinct rows: its real tokens in order, then ONE padding row (the "rep")
// that carries the multiplicity n_pad:
//   raw-exp sums  sum_k e_k: the real keys, the rep, then n_pad - 1 more
//                 additions of the rep's e, in that order (the reference's key
//                 order for right padding: the sum, and with it the overflow /
//                 NaN behaviour of multihead_self.py:16-20, is bitwise the
//                 uncompacted one when all padding is trailing; an interior
//                 id-0 token -- an OOV word, src/data_preprocess.py:134-135 --
//                 moves to the end of the sum, fp32-rounding-level); the
//                 main pass (fast exp, already within rounding of the
//                 reference's) adds the n_pad - 1 copies as one fma, the
//                 recheck pass (rows near overflow) one at a time;
//   context       ctx = sum_k P_k v_k with the rep's P scaled by n_pad;
//   softmax/pool  the rep's score and context row weighted by n_pad
//                 (additive.py:37-52).
// Only the summation of n_pad equal terms changes (one product instead of
// n_pad additions): results agree with the uncompacted computation to fp32
// rounding. Titles are bucketed by NB = ceil(Le / 4) (blocks of 4 rows, the
// 4x4x1 MFMA attention's granule) and encoded in groups of 4 titles of one
// bucket: 16 NB rows, NB M-tiles, NB^2 of the 25 attention tile pairs.
// Without compaction every title is one 20-row slot (NB = 5).
constexpr int NBK = tl::NBK;                             // buckets NB = 1..5
constexpr int NCNT = pk::NEWS_NCOUNT;                    // int32 counters of a launch
constexpr int CNT_RECHECK = 0, CNT_BUCKET = tl::CNT_BUCKET, CNT_REP = pk::NEWS_CNT_REP, CNT_USER = 7, CNT_CLAIM = 8;
static_assert(CNT_BUCKET + NBK == CNT_REP && CNT_CLAIM < NCNT && NCNT % 4 == 0 && tl::FL == FL, "counter layout");

using tl::RowMap;   // q|k|v row of token i of title s
using tl::Titles;   // the classification's output
using tl::CLS_T;

// Classification as a launch of its own (titles.hpp: classify_block; list
// entries through one atomicAdd per bucket and one atomicMin per block).
__global__ __launch_bounds__(CLS_T) void classify_titles_kernel(RowMap rm, Titles tt, int dedupe, int compact) {
  tl::classify_block<false>(blockIdx.x, threadIdx.x, rm, tt, dedupe, compact, tl::TitleSlots{nullptr, nullptr});
}

// out[s] = out[rep] for every other all-padding title s >= s0.
__global__ __launch_bounds__(256) void broadcast_padding_kernel(const uint8_t* __restrict__ pad_title,
                                                                const int32_t* __restrict__ rep, int64_t s0,
                                                                int64_t n_titles, float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;   // (title - s0, float4 column)
  const int64_t s = s0 + t / (FD / 4);
  if (s >= n_titles || !pad_title[s]) return;
  const int64_t r = *rep;
  if (s == r || r == INT32_MAX) return;
  const int c = (int)(t - (s - s0) * (FD / 4));
  reinterpret_cast<float4*>(out + s * FD)[c] = reinterpret_cast<const float4*>(out + r * FD)[c];
}

// The clicked rows m < n_rows (titles 0 .. n_rows - 1 of the launch) whose
// q|k|v the UserEncoder needs: all but the copied all-padding titles, whose
// news vectors are rep's (the UserEncoder reads those rows from row rep).
// Appended in any order (vector atomics, one per wave); the count must start
// at 0. One 256-thread block lists rows m0 .. m0 + URL_ROWS - 1 (four 256-row
// chunks), with one atomic (per-wave atomics on the one counter serialised:
// 11 us; one per 256 rows: ~200 at config 3).
constexpr int URL_ROWS = 1024, URL_C = URL_ROWS / 256;
__device__ __forceinline__ void user_row_list_block(const uint8_t* __restrict__ pad_title,
                                                    const int32_t* __restrict__ rep, int64_t n_rows,
                                                    int64_t* __restrict__ list, int32_t* __restrict__ count,
                                                    int64_t m0) {
  __shared__ int wcount[URL_C * 4], wbase[URL_C * 4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t r = (int64_t)*rep;
  bool keep[URL_C];
  uint64_t ballot[URL_C];
#pragma unroll
  for (int c = 0; c < URL_C; ++c) {
    const int64_t m = m0 + 256 * c + threadIdx.x;
    keep[c] = m < n_rows && !(pad_title[m] && m != r);
    ballot[c] = __ballot(keep[c]);
    if (lane == 0) wcount[4 * c + w] = __popcll(ballot[c]);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
    for (int i = 0; i < URL_C * 4; ++i) tot += wcount[i];
    int b = tot ? atomicAdd(count, tot) : 0;
    for (int i = 0; i < URL_C * 4; ++i) { wbase[i] = b; b += wcount[i]; }
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < URL_C; ++c)
    if (keep[c]) list[wbase[4 * c + w] + __popcll(ballot[c] & ((1ull << lane) - 1))] = m0 + 256 * c + threadIdx.x;
}

__global__ __launch_bounds__(256) void user_row_list_kernel(const uint8_t* __restrict__ pad_title,
                                                            const int32_t* __restrict__ rep,
                                                            int64_t n_rows, int64_t* __restrict__ list,
                                                            int32_t* __restrict__ count) {
  user_row_list_block(pad_title, rep, n_rows, list, count, (int64_t)blockIdx.x * URL_ROWS);
}

// The UserEncoder's row list, built by the deduplicating main pass itself
// (nrms_forward): its workgroups list the rows before their first group.
struct UserRows {
  int64_t* list;   // null: not built here
  int64_t n_rows;
  const uint8_t* pad_title;
  const int32_t* rep;
  int32_t* count;
};

// Titles near fp32 overflow (nrms_common.hpp, kExpRecheck). The main pass
// (EXACT = false) takes the fast exp everywhere and appends (group << 4 |
// title mask) for the titles that need the reference's exp (one entry per
// flagging wave; duplicates are harmless: the recomputation is idempotent). A
// second launch of the same kernel (EXACT = true) recomputes those groups with
// the reference's exp in every row and overwrites the flagged titles' outputs
// only (a title's result never depends on its group). With no such rows (all
// real inputs), the second launch reads the zero count and exits.
struct RecheckList {
  int32_t* count;
  int32_t* list;   // capacity 4 * (groups)
};

// The bucket lists as the main kernel reads them; list == null: no
// classification (every title one 20-row slot, group k = titles 4k .. 4k + 3,
// rows from the RowMap).
struct TitleSet {
  const int32_t* crow;
  const uint8_t* cnt;
  const int32_t* list;
  const int32_t* counters;
  int64_t stride;
  int rep_bucket;   // the bucket rep is appended to (0 with compaction: Le = 1)
};

// Float offsets, within one q|k|v row, of what lane (head slot hl, x) of wave
// (head group) g loads: q / k dims 4c..4c+3 of head h = 4g + hl, and v dims
// 5x..5x+3 and 5x+4.
#ifdef NRMS_QKV_PERM
// (probe) chunk-major q / k sections: chunk c of the 4 heads of group g contiguous
struct QkvOffsets {
  __device__ static int qk(int g, int hl, int c) { return g < 3 ? 80 * g + 16 * c + 4 * hl : 240 + 12 * c + 4 * hl; }
  __device__ static int q(int g, int hl, int c) { return qk(g, hl, c); }
  __device__ static int k(int g, int hl, int c) { return 304 + qk(g, hl, c); }
  __device__ static int v4(int g, int hl, int x) { return 608 + FDK * (4 * g + hl) + 5 * x; }
  __device__ static int v1(int g, int hl, int x) { return 608 + FDK * (4 * g + hl) + 5 * x + 4; }
};
#else
struct QkvOffsets {
  __device__ static int q(int g, int hl, int c) { return FDK * (4 * g + hl) + 4 * c; }
  __device__ static int k(int g, int hl, int c) { return FD + FDK * (4 * g + hl) + 4 * c; }
  __device__ static int v4(int g, int hl, int x) { return 2 * FD + FDK * (4 * g + hl) + 5 * x; }
  __device__ static int v1(int g, int hl, int x) { return 2 * FD + FDK * (4 * g + hl) + 5 * x + 4; }
};
#endif

// 4 floats from a 4-byte-aligned address (V slices start at 5x floats).
typedef float float4_a4 __attribute__((ext_vector_type(4), aligned(4)));
// Row pointers come back from LDS as generic pointers; loads through them are
// issued as global (not flat) loads so that they count in vmcnt only.
#define NRMS_GLOBAL __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ const NRMS_GLOBAL T* gptr(const float* p) {
  return reinterpret_cast<const NRMS_GLOBAL T*>(reinterpret_cast<uintptr_t>(p));
}

// Phase timing (profiles/probes/news_variants.hip builds with NRMS_FUSED_TIMING):
// shader-cycle stamps accumulated per wave into dbg[wave][8].
#ifdef NRMS_FUSED_TIMING
#define NRMS_TIMING_PARAM , unsigned long long* __restrict__ dbg
#define NRMS_STAMP(k)                                                 \
  {                                                                   \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();     \
    tacc[k] += now_ - tprev;                                          \
    tprev = now_;                                                     \
  }
#else
#define NRMS_TIMING_PARAM
#define NRMS_STAMP(k)
#endif

// Sum over the 16 lanes of a DPP row (all 16 get the total): quad butterflies,
// then half-row and row mirrors. VALU only, no LDS crossbar round trips.
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));  // quad_perm [1,0,3,2]
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));  // quad_perm [2,3,0,1]
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false)); // row_half_mirror
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false)); // row_mirror
  return v;
}

// Four independent DPP row sums, stage by stage: each stage's four adds fill
// the DPP read-after-write wait states the single-value form pads with s_nop.
__device__ __forceinline__ void row16_sum4(float (&v)[4]) {
#define NRMS_DPP4(CTRL)                                                                                   \
  _Pragma("unroll") for (int r = 0; r < 4; ++r) v[r] += __builtin_bit_cast(                              \
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v[r]), CTRL, 0xF, 0xF, false));
  NRMS_DPP4(0xB1) NRMS_DPP4(0x4E) NRMS_DPP4(0x141) NRMS_DPP4(0x140)
#undef NRMS_DPP4
}

// value of lane ^ 1 / lane ^ 2 within the quad (DPP quad_perm)
__device__ __forceinline__ float quad_xor1(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float quad_xor2(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
}

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
}

// MODE 0: f32 MFMA additive GEMM, fp32 context tile. MODE 1: split-bf16 x6,
// context stored as bf16 planes. MODE 2: split-f16 x3 (main pass only; its
// recheck pass runs MODE 1), context stored as fp16 planes.
// A group of bucket NB holds 4 titles of LR = 4 NB rows each: title t's
// compacted row p is tile row LR t + p (M = 16 NB rows, NB M-tiles).
// CLS: the titles come classified (bucket lists and compacted rows: ts.list
// and ts.crow set, nrms_forward's path); else every title is one 20-row slot
// read through the RowMap. A template flag, so the per-group row staging
// keeps no run-time branch on it (SGPRs the loop would otherwise spill).
template <int MODE, bool EXACT, bool CLS>
__global__ __launch_bounds__(NTHR, 1) void fused_news_kernel(
    const float* __restrict__ qkv, int64_t ldq, RowMap rmap, TitleSet ts,
    const float* __restrict__ WaP,
    const float* __restrict__ b_add, const float* __restrict__ q_add, float* __restrict__ out,
    RecheckList rl, UserRows ur NRMS_TIMING_PARAM) {
  using Off = QkvOffsets;
  constexpr bool X6 = MODE == 1;
  constexpr bool H3 = MODE == 2;
  static_assert(!(H3 && EXACT), "the F16X3 main pass is rechecked by the x6 kernel");
  if constexpr (EXACT) {
    // nothing flagged (every real input): leave before the prologue
    if (__builtin_amdgcn_readfirstlane(*rl.count) == 0) return;
  }
  if constexpr (!EXACT) {
    // (workgroup-uniform; the padding classification ran in an earlier launch).
    // Chunks go to the LAST workgroups first: the title groups below are dealt
    // from block 0, so those blocks are the ones short of a group in the final
    // round (r5zk: news_fused -1.1 %, faster 3/3 same-box).
    if (ur.list)
      for (int64_t m0 = (int64_t)(gridDim.x - 1 - blockIdx.x) * URL_ROWS; m0 < ur.n_rows;
           m0 += (int64_t)gridDim.x * URL_ROWS) {
        user_row_list_block(ur.pad_title, ur.rep, ur.n_rows, ur.list, ur.count, m0);
        __syncthreads();   // (the block's LDS counters are reused)
      }
  }
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* ctxL = lds;                                   // f32: [80][SC]
  __bf16* ctxB = reinterpret_cast<__bf16*>(lds);       // x6:  [80][XRB] = hi | mid | lo planes
  _Float16* ctxH = reinterpret_cast<_Float16*>(lds);   // f16x3: [80][XRH] = hi | lo planes
  float* part = X6 ? lds + FROWS * XRB / 2 : (H3 ? lds + FROWS * XRH / 2 : ctxL + FROWS * SC);   // [80][8] row partials
  const float** rowptr = reinterpret_cast<const float**>(part + PART_STRIDE * FROWS);   // [RPB][4 titles][20 slots]
  int32_t* tmeta = reinterpret_cast<int32_t*>(rowptr + RPB * FROWS);   // [RPB][title index x4 | count x4]
  int32_t* sched = tmeta + 8 * RPB;   // [gend x NBK | bucket counts x NBK | rep | groups | claim] (see below)

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const float* zero_row = WaP + WAP_MAX;
  const float* nan_row = zero_row + ROW;

  // K padding: context columns 300..303 (x6: 300..319 of every plane) stay zero for the whole launch.
  if (tid < FROWS) {
    if constexpr (X6) {
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
#pragma unroll
        for (int c = 0; c < (XKP - FD) / 4; ++c)
          *reinterpret_cast<uint2*>(ctxB + tid * XRB + pl * XKP + FD + 4 * c) = make_uint2(0u, 0u);
    } else if constexpr (H3) {
#pragma unroll
      for (int pl = 0; pl < 2; ++pl)
#pragma unroll
        for (int c = 0; c < (XKP - FD) / 4; ++c)
          *reinterpret_cast<uint2*>(ctxH + tid * XRH + pl * XKP + FD + 4 * c) = make_uint2(0u, 0u);
    } else {
      *reinterpret_cast<float4*>(ctxL + tid * SC + FD) = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }

  // ---- group schedule (workgroup-uniform, kept in LDS: as registers the
  // five-bucket state spilled). Buckets NB = 5 .. 1 in turn (longest titles
  // first, for the persistent loop's balance); gend[b] = one past the
  // bucket's last group in that order.
  const int64_t n_titles = rmap.n_titles;
  if (tid == 0) {
    int32_t n_groups = (int32_t)((n_titles + FT - 1) / FT);   // (groups < 2^27, checked at launch)
    int32_t rep = INT32_MAX;
    if constexpr (CLS) {
      rep = ts.counters[CNT_REP];
      int32_t acc = 0;
      for (int b = NBK - 1; b >= 0; --b) {
        const int32_t cb = ts.counters[CNT_BUCKET + b];
        const int32_t c = cb + ((b == ts.rep_bucket && rep != INT32_MAX) ? 1 : 0);
        acc += (c + FT - 1) / FT;
        sched[b] = acc;
        sched[NBK + b] = cb;
      }
      n_groups = acc;
    } else {
      for (int b = 0; b < NBK; ++b) { sched[b] = n_groups; sched[NBK + b] = 0; }
    }
    sched[2 * NBK] = rep;
    sched[2 * NBK + 1] = n_groups;
  }
  __syncthreads();
  const int32_t n_groups = __builtin_amdgcn_readfirstlane(sched[2 * NBK + 1]);
  // group k -> bucket (-1 past the end) and the group's index g within it
  // (group indices and keys are int32: groups < 2^27, checked at launch)
  auto bucket_of = [&](int32_t k, int32_t& g) -> int {
    int bsel = -1;
    int32_t start = 0, prev = 0;
#pragma unroll
    for (int b = NBK - 1; b >= 0; --b) {
      const int32_t ge = sched[b];
      if (bsel < 0 && k < ge) { bsel = b; start = prev; }
      prev = ge;
    }
    g = k - __builtin_amdgcn_readfirstlane(start);
    return __builtin_amdgcn_readfirstlane(bsel);
  };
  // iteration idx: the group key k and (recheck pass) the mask of titles to write
  const int32_t n_iter = EXACT ? *rl.count : n_groups;
  auto key_at = [&](int32_t idx, int& tmask) -> int32_t {
    tmask = 0xF;
    if constexpr (EXACT) {
      if (idx >= n_iter) return n_groups;
      const int32_t e = rl.list[idx];
      tmask = e & 0xF;
      return e >> 4;
    }
    return idx;
  };

  // Row pointers of a group: slot (t = tid / 20, p = tid % 20) of threads
  // tid < 80, in three stages so that the dependent loads (bucket list ->
  // compacted row id) hide behind other work: the title index, then its row
  // id and count, then the pointer and the title's (index, count) into LDS.
  // Each stage issues its loads unconditionally, from a safe address where
  // there is nothing to load, and the raw values are resolved by the next
  // stage: a load inside a divergent branch makes the waitcnt pass wait for
  // every older load (the prefetched gathers) where the branch rejoins.
  const int tslot = tid / FL, pslot = tid - tslot * FL;
  struct S1 {
    int32_t raw;    // list entry (or the title itself without classification)
    int32_t mode;   // 0: raw, 1: the rep title, 2: no title
  };
  auto stage1 = [&](int b, int32_t g) -> S1 {
    const int32_t c = FT * g + tslot;
    const bool ok = tid < FROWS && b >= 0;
    S1 x;
    if constexpr (!CLS) {
      x.raw = c;
      x.mode = (ok && c < n_titles) ? 0 : 2;   // (n_titles <= INT32_MAX, checked at launch)
      return x;
    }
    const int bb = b >= 0 ? b : 0;
    const int32_t cbb = sched[NBK + bb], rep = sched[2 * NBK];
    const bool listed = ok && c < cbb;
    x.raw = ts.list[listed ? (int64_t)bb * ts.stride + c : 0];
    x.mode = listed ? 0 : ((ok && b == ts.rep_bucket && c == cbb && rep != INT32_MAX) ? 1 : 2);
    return x;
  };
  auto resolve1 = [&](const S1& x) -> int32_t { return x.mode == 0 ? x.raw : (x.mode == 1 ? sched[2 * NBK] : -1); };
  struct S2 {
    int32_t s;       // title (-1: none)
    int32_t rawc;    // its real-token count (classified)
    int32_t rawr;    // its compacted row id (classified; widened in stage 3, after the load)
    int64_t rawid;   // without classification: its token id (RowMap)
  };
  auto stage2 = [&](int32_t s) -> S2 {
    S2 y;
    y.s = s;
    const int32_t ss = s < 0 ? 0 : s;   // (title 0 exists: n_titles > 0)
    y.rawc = FL;
    y.rawr = 0;
    y.rawid = 0;
    if constexpr (CLS) {
      y.rawc = ts.cnt[ss];
      y.rawr = ts.crow[(int64_t)ss * FL + pslot];
    } else if (!rmap.direct && rmap.ids_a) {
      y.rawid = rmap.ids_of(ss)[pslot];
    }
    return y;
  };
  auto stage3 = [&](const S2& y, int buf) {
    int c = 0;
    int64_t r = -2;
    if (y.s >= 0) {
      c = y.rawc;
      if constexpr (CLS) r = (int64_t)y.rawr;
      else if (rmap.direct || !rmap.ids_a) r = (int64_t)y.s * FL + pslot;
      else r = (uint64_t)y.rawid < (uint64_t)rmap.n_rows ? y.rawid : -1;
    }
    if (tid < FROWS) {
      rowptr[buf * FROWS + tid] = r == -2 ? zero_row : (r < 0 ? nan_row : qkv + r * ldq);
      if (pslot == 0) {
        tmeta[8 * buf + tslot] = y.s;
        tmeta[8 * buf + 4 + tslot] = c;
      }
    }
  };

  // attention roles: block b = (title t, head slot hl), lane x within the block
  const int blk = lane >> 2, x = lane & 3;
  const int at = blk >> 2, hl = blk & 3;
  const int h = 4 * w + hl;
  const bool hval = h < FH;
  const int hls = hval ? hl : 0;   // the idle 16th head slot of wave 3 reads head 12
  // exp(d / sqrt(d_k)) as v_exp_f32(d * log2(e) / sqrt(d_k)): same overflow
  // (-> inf -> NaN) and underflow (-> 0) behaviour as the reference's exp.
  const float c_exp = 1.4426950408889634f / sqrtf((float)FDK);
  const float sqrt_dk = sqrtf((float)FDK);

  // GEMM roles
  const int lm = lane & 15, kq = lane >> 4;
  float qv[3], bv[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int col = 16 * (3 * w + j) + lm;
    qv[j] = q_add[col];
    bv[j] = b_add[col];
  }
  const int colx = 192 + lm;
  const bool xok = colx < FQ;
  const float qx = xok ? q_add[colx] : 0.f, bx = xok ? b_add[colx] : 0.f;
  // B epilogue: q tanh(y + b) = q - 2q / (e^(2(y + b)) + 1), so a lane's
  // partial over its N-tiles starts at sum_j q_j and adds -2 q_j r_j with
  // r_j = rcp(exp2(fma(acc, 2 log2(e) s, 2 log2(e) b_j)) + 1); s = 2^-11 undoes
  // the split-f16 accumulator scaling (exact) -- five VALU per element
  // (v_exp_f32 + v_rcp_f32: absolute error ~1e-7 over the whole range -- the
  // scores are sums of q_n tanh(.) with |q_n| <= 0.1, so absolute error is what
  // matters; saturates to +-1 and propagates NaN)
  constexpr float kC2 = 2.8853900817779268f;   // 2 log2(e)
  const float ysc = H3 ? kC2 * kLoUnscale : kC2;
  float cbv[3], m2q[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    cbv[j] = kC2 * bv[j];
    m2q[j] = -2.0f * qv[j];
  }
  const float qsum = (qv[0] + qv[1]) + qv[2];
  const float cbx = kC2 * bx, m2qx = -2.0f * qx;
  auto tq = [&](float a, float cb) __attribute__((always_inline)) {
    return __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(fmaf(a, ysc, cb)) + 1.0f);
  };
  const float4* Bp = reinterpret_cast<const float4*>(WaP) + lane;
  const float* Aw = ctxL + lm * SC + 4 * kq;

  // q|k|v slices of one title group, lane (block (t, hl), x): Q / K of tokens
  // x + 4j, V dims 5x..5x+4 of tokens k < 4 NB. Loaded for the NEXT group: Q / K
  // at the start of the B epilogue (in flight behind the tanh work, a barrier
  // and the pooling), V at the end of C (behind the next S^T phase).
  float qf[5][FDK], kf[5][FDK], vf[FL][5];
  // token x + 4j of the lane's title: its Q slice (loaded in the previous
  // group's attention as query column j retires) and K slice (B epilogue)
  auto prefetch_q_tok = [&](int buf, int j) {
    const float* rp = rowptr[buf * FROWS + FL * at + x + 4 * j];
#pragma unroll
    for (int c = 0; c < FDK / 4; ++c) {
      const floatx4 a = *gptr<floatx4>(rp + Off::q(w, hls, c));
      qf[j][4 * c] = a.x; qf[j][4 * c + 1] = a.y; qf[j][4 * c + 2] = a.z; qf[j][4 * c + 3] = a.w;
    }
  };
  auto prefetch_k_tok = [&](int buf, int j) {
    const float* rp = rowptr[buf * FROWS + FL * at + x + 4 * j];
#pragma unroll
    for (int c = 0; c < FDK / 4; ++c) {
      const floatx4 b = *gptr<floatx4>(rp + Off::k(w, hls, c));
      kf[j][4 * c] = b.x; kf[j][4 * c + 1] = b.y; kf[j][4 * c + 2] = b.z; kf[j][4 * c + 3] = b.w;
    }
  };
  auto prefetch_qk_tok = [&](int buf, int j) {
    prefetch_q_tok(buf, j);
    prefetch_k_tok(buf, j);
  };
  // slices past the next group's rows are zeroed, not left alone: a register
  // the next group might read is live across the GEMM otherwise (spills)
  auto zero_qk_tok = [&](int j) {
#pragma unroll
    for (int d = 0; d < FDK; ++d) { qf[j][d] = 0.f; kf[j][d] = 0.f; }
  };
  auto prefetch_qk = [&](int buf, int nbq) {
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      if (j < nbq) prefetch_qk_tok(buf, j);
      else zero_qk_tok(j);
    }
  };
  // (50 + 40 loads in two batches: at most 63 may be outstanding per wave)
  auto prefetch_v_tok = [&](int buf, int k) {
    const float* vr = rowptr[buf * FROWS + FL * at + k];
    const float4_a4 a = *gptr<float4_a4>(vr + Off::v4(w, hls, x));
    vf[k][0] = a.x; vf[k][1] = a.y; vf[k][2] = a.z; vf[k][3] = a.w;
    vf[k][4] = *gptr<float>(vr + Off::v1(w, hls, x));
  };
  auto prefetch_v = [&](int buf, int nbq) {
#pragma unroll
    for (int kb = 0; kb < 5; ++kb) {
      if (kb < nbq) {
#pragma unroll
        for (int r = 0; r < 4; ++r) prefetch_v_tok(buf, 4 * kb + r);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int m = 0; m < 5; ++m) vf[4 * kb + r][m] = 0.f;
      }
    }
  };

  // the row pointers of the first two groups (buffers 0 and 1), the title
  // indices of the third (s_carry), then the first group's slices
  S1 s_carry;
  {
    int b0 = -1;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      int tm0;
      int32_t g0 = 0;
      const int32_t i0 = (int32_t)blockIdx.x + p * (int32_t)gridDim.x;
      const int b = i0 < n_iter ? bucket_of(key_at(i0, tm0), g0) : -1;
      if (p == 0) b0 = b;
      stage3(stage2(resolve1(stage1(b, g0))), p);
    }
    {
      int tm2;
      int32_t g2 = 0;
      const int32_t i2 = (int32_t)blockIdx.x + 2 * (int32_t)gridDim.x;
      s_carry = stage1(i2 < n_iter ? bucket_of(key_at(i2, tm2), g2) : -1, g2);
    }
    __syncthreads();
    if (b0 >= 0) {
      prefetch_qk(0, b0 + 1);
      prefetch_v(0, b0 + 1);
    }
  }
#ifdef NRMS_FUSED_TIMING
  unsigned long long tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tprev = __builtin_amdgcn_s_memtime();
#endif

  int it = 0;
  // main pass: the launch's group-claim counter (reset by the pack kernel)
  // and the last claim, read back by every wave
  const __amdgpu_buffer_rsrc_t crs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<int32_t*>(ts.counters + CNT_CLAIM), 0, 4, 0x00020000);
  int32_t q_claim = 0;
  // H3: the first k-step's W_add fragments are loaded at the end of phase A,
  // before the A -> B barrier: the barrier wait covers their L2 latency
  const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(WaP + WAP_MAX + SPECIAL_FLOATS), 0, WAP2_FLOATS * 4, 0x00020000);
  int wvoff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) wvoff[j] = lane * 16 + (j < 3 ? 3 * w + j : 12) * 3 * 1024;
  f16x8 wb0[4][3];
  // one iteration: group key_at(idx), of bucket NB - 1
  // iterate(idx, idx_n, idx_n3): this group, the next, and the one three
  // ahead (its title indices are read at this group's end)
  auto iterate = [&](int32_t idx, int32_t idx_n, int32_t idx_n3, auto nbc) {
    constexpr int NB = decltype(nbc)::value;
    int tmask, tmask_n;
    const int32_t k = key_at(idx, tmask);
    int32_t g, gn = 0;
    bucket_of(k, g);
    const int32_t kn = key_at(idx_n, tmask_n);
    const int bn = (idx_n < n_iter) ? bucket_of(kn, gn) : -1;
    const int nb_next = bn + 1;   // 0: no next group
    // the group after next has its row pointers staged during this attention
    // (its title indices were read at the end of the previous group: s_carry);
    // the group after that has its title indices read at the end of this one
    int tmask_n3;
    int32_t gn3 = 0;
    const int32_t kn3 = key_at(idx_n3, tmask_n3);
    const int bn3 = (idx_n3 < n_iter) ? bucket_of(kn3, gn3) : -1;
    // main pass: claim the group four ahead (wave 0 lane 0's offset is the
    // only one in range: no branch around the atomic, whose return the
    // waitcnt pass would otherwise wait for at the branch's join)
    [[maybe_unused]] int32_t claim_v = 0;
    if constexpr (!EXACT) claim_v = __builtin_amdgcn_raw_ptr_buffer_atomic_add_i32(1, crs, tid == 0 ? 0 : 64, 0, 0);
    // row-pointer buffers: this group's, the next group's, the one after's
    const int buf = it & (RPB - 1), nbuf = (it + 1) & (RPB - 1), nbuf2 = (it + 2) & (RPB - 1);
    {
      // this lane's title's real-token count (its index is read in C)
      const int my_c = tmeta[8 * buf + 4 + at];
      constexpr int LR = 4 * NB;             // tile rows per title
      constexpr int XMAX = 23 - 4 * NB;      // most extra additions of the rep's exp (n_pad - 1)
      // compacted length Le = c + (c < 20) in [LR - 3, LR]; the rep (row c,
      // multiplicity n_pad = 20 - c) sits in the last key block, register rrep
      const int le = my_c + (my_c < FL ? 1 : 0);
      const int npad = FL - my_c;
      const int rrep = my_c - 4 * (NB - 1);
      // (no barrier here: the context tile's last readers, the previous group's
      // B mainloop, finished before its B -> C barrier; C reads registers + part)
#ifdef NRMS_FUSED_TIMING
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // probe only: time the wait for this group's q|k|v
#endif
      NRMS_STAMP(0)
      floatx4 O[5][NB];   // this wave's context rows, live until the pooling in C
      uint64_t recheck = 0;   // lanes whose row needs the recheck pass (RecheckList)

      // ---------------- A: attention (4x4x1 MFMA, 16 (title, head) blocks) --------------
      {
        // the slot rows of the group after next: stage 1 (the title index) came
        // from the end of the previous group, so its load has landed; stage 2's
        // dependent row-id loads go out after the first query column and are
        // done long before stage 3 at this phase's end
        S2 r_next;
        // S^T tiles: rows = keys 4j + r (A = K), cols = queries 4i + x (B = Q)
        floatx4 S[NB][NB];
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
          for (int i = 0; i < NB; ++i) S[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};
        // One query column i at a time (S^T, exp, ctx^T, split + store), so a
        // column's S registers die before the next column's are written: short
        // live ranges, no spills.
        auto s_mfma = [&](int i) {
#pragma unroll
          for (int d = 0; d < FDK; ++d)
#pragma unroll
            for (int j = 0; j < NB; ++j) S[j][i] = mfma4(kf[j][d], qf[i][d], S[j][i]);
        };
        // P = exp(S / sqrt(dk)) / (sum_keys + 1e-8): query 4i + x, key 4j + r.
        // Keys past Le (unused slots) are 0; the rep's other n_pad - 1 copies
        // are added after the rep (recheck pass: one at a time, the
        // uncompacted sum bitwise; main pass: one fma, below).
        auto s_exp = [&](int i) {
          float sum = 0.f;
#pragma unroll
          for (int j = 0; j < NB; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float e = EXACT ? ref_exp(S[j][i][r], sqrt_dk) : __builtin_amdgcn_exp2f(S[j][i][r] * c_exp);
              if (j == NB - 1) e = (4 * j + r < le) ? e : 0.f;
              S[j][i][r] = e;
              sum += e;
            }
          float erep = 0.f;
#pragma unroll
          for (int r = 0; r < 4; ++r) erep = r == rrep ? S[NB - 1][i][r] : erep;
          if constexpr (!EXACT) {
            // main pass: the rep's other n_pad - 1 copies in one fma (fp32
            // rounding; the recheck pass adds them one at a time, as the
            // uncompacted sum: profiles/r5/r5zj_news_variants_maxilp_ab.txt)
            sum = fmaf((float)(npad > 1 ? npad - 1 : 0), erep, sum);
          } else {
#pragma unroll
            for (int c = 0; c < XMAX; ++c) sum += (c + 1 < npad) ? erep : 0.f;
          }
          // rows near fp32 overflow (or non-finite): flagged (no branch here),
          // recomputed by the EXACT pass (RecheckList)
          if constexpr (!EXACT) recheck |= __builtin_amdgcn_ballot_w64(exp_row_needs_recheck(sum));
          // (main pass: v_rcp_f32, 1 ulp; the recheck pass divides as the reference)
          const float inv = EXACT ? 1.0f / (sum + 1e-8f) : __builtin_amdgcn_rcpf(sum + 1e-8f);
#pragma unroll
          for (int j = 0; j < NB; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) S[j][i][r] *= inv;
          // the rep key's weight carries its multiplicity into ctx = sum_k P_k v_k
          const float fpad = (float)npad;
#pragma unroll
          for (int r = 0; r < 4; ++r)
            S[NB - 1][i][r] = (r == rrep && npad > 1) ? S[NB - 1][i][r] * fpad : S[NB - 1][i][r];
        };
        // ctx^T tiles: rows = dims 5r' + m (A = V^T), cols = queries 4i + x (B = P^T);
        // lane x holds ctx[query 4i + x][dim 5r' + m] = O[m][i][r']
        auto o_mfma = [&](int i) {
#pragma unroll
          for (int m = 0; m < 5; ++m) O[m][i] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kk = 0; kk < LR; ++kk)
#pragma unroll
            for (int m = 0; m < 5; ++m) O[m][i] = mfma4(vf[kk][m], S[kk >> 2][i][kk & 3], O[m][i]);
        };
        // (a branch-free form, with the idle head slot storing its bit-identical
        // copy of head 12, measured 9 % slower: the compiler then interleaves the
        // stores into the next column's MFMAs and spills)
        auto o_store = [&](int i) {
          if (!hval) return;
          const int row = LR * at + 4 * i + x;
          if constexpr (H3) {
            _Float16* dst = ctxH + row * XRH + FDK * h;
#pragma unroll
            for (int c = 0; c < FDK / 4; ++c) {
              uint32_t hw[2], lw[2];
#pragma unroll
              for (int e = 0; e < 2; ++e) {
                const int d = 4 * c + 2 * e;
                split2x2h(O[d % 5][i][d / 5], O[(d + 1) % 5][i][(d + 1) / 5], hw[e], lw[e]);
              }
              *reinterpret_cast<uint2*>(dst + 4 * c) = make_uint2(hw[0], hw[1]);
              *reinterpret_cast<uint2*>(dst + XKP + 4 * c) = make_uint2(lw[0], lw[1]);
            }
          } else if constexpr (X6) {
            __bf16* dst = ctxB + row * XRB + FDK * h;
#pragma unroll
            for (int c = 0; c < FDK / 4; ++c) {
              uint32_t hh[2], m[2], l[2];
#pragma unroll
              for (int e = 0; e < 2; ++e) {
                const int d = 4 * c + 2 * e;
                split3x2(O[d % 5][i][d / 5], O[(d + 1) % 5][i][(d + 1) / 5], hh[e], m[e], l[e]);
              }
              *reinterpret_cast<uint2*>(dst + 4 * c) = make_uint2(hh[0], hh[1]);
              *reinterpret_cast<uint2*>(dst + XKP + 4 * c) = make_uint2(m[0], m[1]);
              *reinterpret_cast<uint2*>(dst + 2 * XKP + 4 * c) = make_uint2(l[0], l[1]);
            }
          } else {
            float4* dst = reinterpret_cast<float4*>(ctxL + row * SC + FDK * h);
#pragma unroll
            for (int c = 0; c < FDK / 4; ++c) {
              const int d0 = 4 * c;
              dst[c] = make_float4(O[d0 % 5][i][d0 / 5], O[(d0 + 1) % 5][i][(d0 + 1) / 5],
                                   O[(d0 + 2) % 5][i][(d0 + 2) / 5], O[(d0 + 3) % 5][i][(d0 + 3) / 5]);
            }
          }
        };
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          s_mfma(i);
          // query column i's Q slices are dead: the next group's go into them
          // (main pass: the next group is of this bucket or a smaller one, so
          // its queries are tokens < 4 NB; slots past its rows read the zero row)
#ifndef NRMS_PROBE_NO_QLOAD   // (probe builds: the phase without its gather loads)
          if constexpr (!EXACT) prefetch_q_tok(nbuf, i);
#endif
          s_exp(i);
          o_mfma(i);
          o_store(i);
          if (i == 0) r_next = stage2(resolve1(s_carry));
        }
        stage3(r_next, nbuf2);
        if constexpr (H3) {
#pragma unroll
          for (int pl = 2; pl >= 1; --pl)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              wb0[j][pl] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(wrs, wvoff[j], pl * 1024, 0));
        }
      }
      NRMS_STAMP(1)
      __syncthreads();   // context tile complete
      NRMS_STAMP(2)

      // ---------------- B: additive GEMM + tanh·q row partials ----------------
      // Wave w: N-tiles 3w..3w+2 of every M-tile, and N-tile 12 (the last, half
      // past Q) of M-tile w (w < NB) and, for wave 0, of M-tile 4 (NB = 5). Each
      // row's score sums its partials in one order, (((p0 + p1) + p2) + p3) + p12,
      // whichever wave holds N-tile 12 for it: a title's result does not depend
      // on its slot.
      {
        floatx4 acc[NB][3], accX = floatx4{0.f, 0.f, 0.f, 0.f}, accX2 = floatx4{0.f, 0.f, 0.f, 0.f};
        // N-tile 12: this wave's M-tile xm (waves past NB compute an unused tile
        // on M-tile 0), and M-tile 4 for wave 0 when NB = 5
        const int xm = w < NB ? w : 0;
        const bool extra = NB == 5 && w == 0;
#pragma unroll
        for (int mt = 0; mt < NB; ++mt)
#pragma unroll
          for (int j = 0; j < 3; ++j) acc[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};
        if constexpr (X6) {
          // A fragments (16x16x32): lane holds A[row lm][32 ks + 8 kq .. + 7] of each plane
          const __bf16* Ab = ctxB + lm * XRB + 8 * kq;
          const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
              const_cast<float*>(WaP), 0, WAP3_FLOATS * 4, 0x00020000);
          int bvoff[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) bvoff[j] = lane * 16 + (j < 3 ? 3 * w + j : 12) * 3 * 1024;
          // plane-major: the hi planes (first product's B) arrive first
          auto load_b = [&](int ks, bf16x8 (&dst)[4][3]) {
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
#pragma unroll
              for (int j = 0; j < 4; ++j)
                dst[j][pl] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                    brs, bvoff[j], (ks * FNT * 3 + pl) * 1024, 0));
          };
          // one 32-deep k-step, the same code for every wave (one copy per NB:
          // wave-specialised copies made the kernel ~4x larger than the
          // instruction cache); the N-tile-12 rows (M-tile xm) are read as
          // their own fragments; A planes loaded lo first, the order the
          // products consume them
          auto kstep = [&](int ks, const bf16x8 (&bb)[4][3]) {
            bf16x8 a[NB][3], ax[3];
#pragma unroll
            for (int pl = 2; pl >= 0; --pl) {
#pragma unroll
              for (int mt = 0; mt < NB; ++mt)
                a[mt][pl] = *reinterpret_cast<const bf16x8*>(Ab + 16 * mt * XRB + pl * XKP + 32 * ks);
              ax[pl] = *reinterpret_cast<const bf16x8*>(Ab + 16 * xm * XRB + pl * XKP + 32 * ks);
            }
            // the six products with i + j <= 2, smallest first
#define NRMS_X6STEP(PA, PB)                                                                              \
  _Pragma("unroll") for (int mt = 0; mt < NB; ++mt)                                                      \
  _Pragma("unroll") for (int j = 0; j < 3; ++j)                                                          \
      acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt][PA], bb[j][PB], acc[mt][j], 0, 0, 0);   \
  accX = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax[PA], bb[3][PB], accX, 0, 0, 0);                      \
  if (extra) accX2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[NB - 1][PA], bb[3][PB], accX2, 0, 0, 0);
            NRMS_X6STEP(2, 0) NRMS_X6STEP(1, 1) NRMS_X6STEP(0, 2) NRMS_X6STEP(1, 0) NRMS_X6STEP(0, 1)
            NRMS_X6STEP(0, 0)
#undef NRMS_X6STEP
          };
          // two B buffers in turn (XKS is even): no register copies between k-steps
          bf16x8 b0[4][3], b1[4][3];
          load_b(0, b0);
#pragma unroll
          for (int ks = 0; ks < XKS; ks += 2) {
            // (each k-step's loads pinned ahead of the other buffer's MFMAs: left
            // to the scheduler they sank among them and the next k-step waited
            // for them -- with fewer M-tiles the k-step no longer covered the
            // L2 latency)
            load_b(ks + 1, b1);
            __builtin_amdgcn_sched_barrier(0);
            kstep(ks, b0);
            __builtin_amdgcn_sched_barrier(0);
            if (ks + 2 < XKS) load_b(ks + 2, b0);
            __builtin_amdgcn_sched_barrier(0);
            kstep(ks + 1, b1);
            __builtin_amdgcn_sched_barrier(0);
          }
          static_assert(XKS % 2 == 0, "k-steps in pairs");
        } else if constexpr (H3) {
          // products lo·hi, hi·lo, hi·hi' (each 2^11 x the true product) into acc
          const _Float16* Ah = ctxH + lm * XRH + 8 * kq;
          // B fragments through a buffer resource: one VGPR offset (the lane), the
          // fragment offset in an SGPR (no per-load address registers when unrolled)
          const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
              const_cast<float*>(WaP + WAP_MAX + SPECIAL_FLOATS), 0, WAP2_FLOATS * 4, 0x00020000);
          int bvoff[4];   // lane + N-tile in the VGPR offset; k-step in soffset; plane immediate
#pragma unroll
          for (int j = 0; j < 4; ++j) bvoff[j] = lane * 16 + (j < 3 ? 3 * w + j : 12) * 3 * 1024;
          // B plane pb: 0 = hi' (formed in registers from hi: 2,048 hi is exact,
          // and the pack stores NaN in hi where it would pass fp16's range; the
          // packed hi' plane is not read), 1 = lo, 2 = hi; loaded in consumption order
          auto load_b = [&](int ks, f16x8 (&dst)[4][3]) {
#pragma unroll
            for (int pl = 2; pl >= 1; --pl)
#pragma unroll
              for (int j = 0; j < 4; ++j)
                dst[j][pl] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(
                    brs, bvoff[j], (ks * FNT * 3 + pl) * 1024, 0));
          };
          // products lo·hi, hi·lo, hi·hi' of one k-step (one copy of the k-step
          // for every wave, as the x6 path)
#define NRMS_H3STEP2(PA, PB)                                                                           \
  _Pragma("unroll") for (int mt = 0; mt < NB; ++mt)                                                    \
  _Pragma("unroll") for (int j = 0; j < 3; ++j)                                                        \
      acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[mt][PA], bb[j][PB], acc[mt][j], 0, 0, 0);  \
  accX = __builtin_amdgcn_mfma_f32_16x16x32_f16(ax[PA], bb[3][PB], accX, 0, 0, 0);                     \
  if (extra) accX2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[NB - 1][PA], bb[3][PB], accX2, 0, 0, 0);
          // fully unrolled, each k-step's loads and MFMAs fenced in place
          // (without the fences the scheduler hoists every load: 1,100 spills);
          // a rolled loop permuted the accumulators at its back-edge (~170
          // AGPR moves per iteration): 1.41 -> 1.33 ms. The first k-step's W
          // fragments were loaded before the A -> B barrier (wb0).
          f16x8 b0[4][3], b1[4][3];
#pragma unroll
          for (int j = 0; j < 4; ++j) { b0[j][1] = wb0[j][1]; b0[j][2] = wb0[j][2]; }
          // A fragments one k-step ahead without extra registers: product 1 is
          // the only reader of the lo plane (A lo x W hi), so the next k-step's
          // lo fragments are read from LDS into the same registers right after
          // it, under products 2 and 3; the next hi fragments after product 3,
          // under the next k-step's product 1. The LDS latency leaves the k-step.
          auto ld_a = [&](int ks, int pl, f16x8 (&a)[NB][2], f16x8 (&ax)[2]) {
#pragma unroll
            for (int mt = 0; mt < NB; ++mt)
              a[mt][pl] = *reinterpret_cast<const f16x8*>(Ah + 16 * mt * XRH + pl * XKP + 32 * ks);
            ax[pl] = *reinterpret_cast<const f16x8*>(Ah + 16 * xm * XRH + pl * XKP + 32 * ks);
          };
          f16x8 ar[NB][2], arx[2];
          ld_a(0, 1, ar, arx);
          ld_a(0, 0, ar, arx);
          auto kstep_rot = [&](int ks, f16x8 (&bb)[4][3]) {
            const f16x8 (&a)[NB][2] = ar;
            const f16x8 (&ax)[2] = arx;
#pragma unroll
            for (int j = 0; j < 4; ++j) bb[j][0] = bb[j][2] * (_Float16)kF16LoScale;
            NRMS_H3STEP2(1, 2)
            __builtin_amdgcn_sched_barrier(0);
            if (ks + 1 < XKS) ld_a(ks + 1, 1, ar, arx);
            __builtin_amdgcn_sched_barrier(0);
            NRMS_H3STEP2(0, 1) NRMS_H3STEP2(0, 0)
            __builtin_amdgcn_sched_barrier(0);
            if (ks + 1 < XKS) ld_a(ks + 1, 0, ar, arx);
          };
#undef NRMS_H3STEP2
#pragma unroll
          for (int ks = 0; ks < XKS; ks += 2) {
            load_b(ks + 1, b1);
            __builtin_amdgcn_sched_barrier(0);
            kstep_rot(ks, b0);
            __builtin_amdgcn_sched_barrier(0);
            if (ks + 2 < XKS) load_b(ks + 2, b0);
            __builtin_amdgcn_sched_barrier(0);
            kstep_rot(ks + 1, b1);
            __builtin_amdgcn_sched_barrier(0);
          }
          // (the 2^-11 unscale is folded into the epilogue's exp argument)
        } else {
          float4 bb[4], bn4[4];
#pragma unroll
          for (int j = 0; j < 3; ++j) bb[j] = Bp[(3 * w + j) * 64];
          bb[3] = Bp[12 * 64];
          for (int c = 0; c < FKG; ++c) {
            if (c + 1 < FKG) {
#pragma unroll
              for (int j = 0; j < 3; ++j) bn4[j] = Bp[((c + 1) * FNT + 3 * w + j) * 64];
              bn4[3] = Bp[((c + 1) * FNT + 12) * 64];
            }
            float4 a[NB];
#pragma unroll
            for (int mt = 0; mt < NB; ++mt) a[mt] = *reinterpret_cast<const float4*>(Aw + 16 * mt * SC + 16 * c);
            const float4 ax = *reinterpret_cast<const float4*>(Aw + 16 * (w < NB ? w : 0) * SC + 16 * c);
#define NRMS_KSTEP(F)                                                                             \
  _Pragma("unroll") for (int mt = 0; mt < NB; ++mt)                                               \
  _Pragma("unroll") for (int j = 0; j < 3; ++j)                                                   \
      acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt].F, bb[j].F, acc[mt][j], 0, 0, 0);   \
  if (w < NB) accX = __builtin_amdgcn_mfma_f32_16x16x4f32(ax.F, bb[3].F, accX, 0, 0, 0);           \
  if (NB == 5 && w == 0) accX2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[NB - 1].F, bb[3].F, accX2, 0, 0, 0);
            NRMS_KSTEP(x) NRMS_KSTEP(y) NRMS_KSTEP(z) NRMS_KSTEP(w)
#undef NRMS_KSTEP
            if (c + 1 < FKG) {
#pragma unroll
              for (int j = 0; j < 4; ++j) bb[j] = bn4[j];
            }
          }
        }
        NRMS_STAMP(3)
        // C/D layout of 16x16 MFMA: col = lane & 15, row = (lane >> 4) * 4 + reg.
        // The next group's Q|K slices go out one token per M-tile, between the
        // tanh blocks (pinned by sched_barrier): issued all at once ahead of the
        // tanh work, the in-order issue stalls the VALU behind the gather's
        // address/TA queue.
        // Main pass: the next group is of this bucket or a smaller one (buckets
        // run NB = 5 .. 1), so its slices are tokens < 4 NB: loaded
        // unconditionally (slots past its rows, or no next group, read the zero
        // row), no zero fill. The recheck pass walks groups of any bucket.
#pragma unroll
        for (int mt = 0; mt < NB; ++mt) {
#ifndef NRMS_PROBE_NO_KLOAD
          if constexpr (!EXACT) prefetch_k_tok(nbuf, mt);
#else
          if constexpr (!EXACT) {}
#endif
          else if (mt < nb_next) prefetch_qk_tok(nbuf, mt);
          else zero_qk_tok(mt);
          __builtin_amdgcn_sched_barrier(0);
          float p[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            p[r] = qsum;
#pragma unroll
            for (int j = 0; j < 3; ++j) p[r] = fmaf(m2q[j], tq(acc[mt][j][r], cbv[j]), p[r]);
          }
          row16_sum4(p);
          if (lm == 0)
#pragma unroll
            for (int r = 0; r < 4; ++r) part[PART_STRIDE * (16 * mt + 4 * kq + r) + w] = p[r];
          const bool own_x = (mt == w && w < NB) || (NB == 5 && w == 0 && mt == 4);
          if (own_x) {
            float px[4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
              px[r] = fmaf(m2qx, tq((NB == 5 && mt == 4) ? accX2[r] : accX[r], cbx), qx);
            row16_sum4(px);
            if (lm == 0)
#pragma unroll
              for (int r = 0; r < 4; ++r) part[PART_STRIDE * (16 * mt + 4 * kq + r) + 4] = px[r];
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (EXACT) {
#pragma unroll
          for (int j = NB; j < 5; ++j) {
            if (j < nb_next) prefetch_qk_tok(nbuf, j);
            else zero_qk_tok(j);
          }
        }
      }
      NRMS_STAMP(4)
      if constexpr (!EXACT)
        if (tid == 0) sched[2 * NBK + 2] = claim_v;   // (read after the barrier; rewritten after the next A -> B barrier)
      __syncthreads();   // row partials complete
      NRMS_STAMP(5)

      // ---------------- C: softmax over tokens + pooling from the O registers ----------------
      // Lane (block (at, hl), x) holds rows 4i + x (i < NB) of title at, head h:
      // the 4 lanes of a block see all its rows, so the softmax (max-subtracted,
      // as F.softmax) and the pooling out[20h + d] = sum_l w_l ctx[l][20h + d]
      // reduce within the lane quad (DPP); the LDS tile is not read. Row 4i + x
      // counts 1 (a real token), n_pad (the rep) or 0 (an unused slot).
      {
        float sc[NB], mult[NB];
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          const int row = LR * at + 4 * i + x;
          const float4 pv = *reinterpret_cast<const float4*>(part + PART_STRIDE * row);
          sc[i] = (((pv.x + pv.y) + pv.z) + pv.w) + part[PART_STRIDE * row + 4];
          const int q = 4 * i + x;
          mult[i] = q < my_c ? 1.f : ((q == my_c && npad > 0) ? (float)npad : 0.f);
        }
        // the softmax maximum over the counted rows (v_max_f32 skips a NaN) and
        // nz = 0, or NaN when a counted score is NaN (scores are finite or NaN:
        // sums of q tanh(.)); the quad's NaN is added to the maximum below, so
        // a NaN score makes every weight of its title NaN, as F.softmax
        float mx = -INFINITY, nz = 0.f;
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          mx = mult[i] > 0.f ? fmaxf(mx, sc[i]) : mx;
          nz = mult[i] > 0.f ? nz + (sc[i] - sc[i]) : nz;
        }
        if constexpr (H3) {
          // a NaN score: an operand beyond fp16's range (or NaN inputs) -> recheck pass
          recheck |= __builtin_amdgcn_ballot_w64(nz != nz);
        }
        if constexpr (!EXACT) {
          // titles of the flagged lanes (title at = lanes 16 at .. 16 at + 15)
          int tm = 0;
#pragma unroll
          for (int t = 0; t < FT; ++t) tm |= ((recheck >> (16 * t)) & 0xFFFFull) ? (1 << t) : 0;
          if (tm != 0 && lane == 0) rl.list[atomicAdd(rl.count, 1)] = (int32_t)((k << 4) | tm);
        }
        mx = fmaxf(mx, quad_xor1(mx));
        nz += quad_xor1(nz);
        mx = fmaxf(mx, quad_xor2(mx));
        nz += quad_xor2(nz);
        mx += nz;
        // exp on v_exp_f32 (arguments <= 0: no overflow; NaN propagates) and one
        // reciprocal per title instead of a division per row (fp32 rounding)
        float ex[NB], sum = 0.f;
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          ex[i] = mult[i] > 0.f ? __builtin_amdgcn_exp2f((sc[i] - mx) * 1.4426950408889634f) * mult[i] : 0.f;
          sum += ex[i];
        }
        sum += quad_xor1(sum);
        sum += quad_xor2(sum);
        const float rsum = __builtin_amdgcn_rcpf(sum);
        float wt[NB];
#pragma unroll
        for (int i = 0; i < NB; ++i) wt[i] = ex[i] * rsum;
        // pz[m][r'] = dim 5r' + m of head h, summed over this lane's rows, then
        // the quad; unused slots (last row block only) are skipped, not
        // weighted by 0 (their context may be non-finite)
        float pz[5][4];
#pragma unroll
        for (int m = 0; m < 5; ++m)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float a = 0.f;
#pragma unroll
            for (int i = 0; i < NB; ++i)
              a = (i < NB - 1 || mult[i] > 0.f) ? fmaf(wt[i], O[m][i][r], a) : a;
            a += quad_xor1(a);
            pz[m][r] = a + quad_xor2(a);
          }
        const int32_t my_s = tmeta[8 * buf + at];   // this lane's title (-1: none)
        const bool write = hval && my_s >= 0 && (!EXACT || ((tmask >> at) & 1));
        if (write) {
          // lane x stores dims 5x .. 5x + 4 of head h
          float v[5];
#pragma unroll
          for (int m = 0; m < 5; ++m)
            v[m] = x == 0 ? pz[m][0] : (x == 1 ? pz[m][1] : (x == 2 ? pz[m][2] : pz[m][3]));
          float* dst = out + (int64_t)my_s * FD + FDK * h + 5 * x;
          float4_a4 v4;
          v4.x = v[0]; v4.y = v[1]; v4.z = v[2]; v4.w = v[3];
          *reinterpret_cast<float4_a4*>(dst) = v4;
          dst[4] = v[4];
        }
        // V slices of the next group: issued here, after O is dead (holding both
        // through the B epilogue spills); the S^T phase of the next group covers
        // most of their latency
        s_carry = stage1(bn3, gn3);   // (issued ahead of the V slices)
        if constexpr (EXACT) {
          prefetch_v(nbuf, nb_next);
        } else {
#ifndef NRMS_PROBE_NO_VLOAD
#pragma unroll
          for (int kk = 0; kk < LR; ++kk) prefetch_v_tok(nbuf, kk);   // (as the Q|K slices above)
#endif
        }
      }
      NRMS_STAMP(6)
    }
    if constexpr (!EXACT) q_claim = __builtin_amdgcn_readfirstlane(sched[2 * NBK + 2]);
    ++it;
  };
  if constexpr (EXACT) {
    // flagged groups in list order, any bucket
    for (int32_t idx = blockIdx.x; idx < n_iter; idx += gridDim.x) {
      int tm;
      int32_t g;
      const int32_t i1 = idx + (int32_t)gridDim.x, i3 = idx + 3 * (int32_t)gridDim.x;
      switch (bucket_of(key_at(idx, tm), g)) {
        case 0: iterate(idx, i1, i3, std::integral_constant<int, 1>{}); break;
        case 1: iterate(idx, i1, i3, std::integral_constant<int, 2>{}); break;
        case 2: iterate(idx, i1, i3, std::integral_constant<int, 3>{}); break;
        case 3: iterate(idx, i1, i3, std::integral_constant<int, 4>{}); break;
        default: iterate(idx, i1, i3, std::integral_constant<int, 5>{}); break;
      }
    }
  } else {
    // The main pass walks the groups in order (buckets NB = 5 .. 1, one loop
    // per NB: a single loop switching between the five bodies spilled ~600
    // registers). A workgroup's first four groups are blockIdx.x + p grid
    // (p < 4, the prologue's); each iteration then claims the group four
    // ahead from a launch counter (4 grid + claims so far), so the
    // workgroups that drew lighter groups take more of them: with the static
    // stride the slowest workgroup ran 1.9 % past the mean
    // (profiles/r6/r6s_news_balance.txt). Claims are increasing per workgroup,
    // so the next group is of this bucket or a smaller one, as before.
    const int32_t grid = gridDim.x;
    int32_t q0 = (int32_t)blockIdx.x, q1 = q0 + grid, q2 = q1 + grid, q3 = q2 + grid;
    auto run_bucket = [&](auto nbc) {
      constexpr int NB = decltype(nbc)::value;
      const int32_t end = __builtin_amdgcn_readfirstlane(sched[NB - 1]);
      while (q0 < end) {
        iterate(q0, q1, q3, nbc);
        q0 = q1;
        q1 = q2;
        q2 = q3;
        q3 = 4 * grid + q_claim;
      }
    };
    run_bucket(std::integral_constant<int, 5>{});
    run_bucket(std::integral_constant<int, 4>{});
    run_bucket(std::integral_constant<int, 3>{});
    run_bucket(std::integral_constant<int, 2>{});
    run_bucket(std::integral_constant<int, 1>{});
  }
#ifdef NRMS_FUSED_TIMING
  if (!EXACT && lane == 0)
    for (int k = 0; k < 8; ++k) dbg[(blockIdx.x * 4 + w) * 8 + k] = tacc[k];
#endif
}

}  // namespace

// Workspace after the packed W_add, special rows and f16 planes: int32
// counters [NCNT] (reset by the pack kernel of every launch), the recheck list
// (4 per group), the bucket lists [NBK][n], the compacted rows [n][20], the
// split classification's slot codes [n] and block counts [nblk][8] (16-B
// aligned), then bytes: counts [n] and all-padding flags [n].
static size_t fused_news_list_offset() { return (size_t)WAP_MAX + SPECIAL_FLOATS + WAP2_FLOATS; }
static int64_t max_groups(int64_t n_titles) { return (n_titles + FT - 1) / FT + NBK; }
size_t fused_news_workspace_floats(int64_t n_titles) {
  return fused_news_list_offset() + NCNT + 4 * (size_t)max_groups(n_titles) + (size_t)NBK * n_titles + 4 +
         (size_t)FL * n_titles + (size_t)n_titles + 4 + (size_t)tl::BLK_INTS * tl::classify_blocks(n_titles) +
         ((size_t)2 * n_titles + 3) / 4;
}
namespace {
struct NewsWs {
  int32_t* counters;
  int32_t* recheck;
  int32_t* list;
  int32_t* crow;
  int32_t* slot;
  int32_t* blkcnt;
  uint8_t* cnt;
  uint8_t* pad_title;
};
NewsWs news_ws(float* ws, int64_t n_titles) {
  NewsWs z;
  z.counters = reinterpret_cast<int32_t*>(ws + fused_news_list_offset());
  z.recheck = z.counters + NCNT;
  z.list = z.recheck + 4 * max_groups(n_titles);
  // (16-B aligned: the classification writes each title's 80-B row as 16-B stores)
  z.crow = reinterpret_cast<int32_t*>((reinterpret_cast<uintptr_t>(z.list + NBK * n_titles) + 15) & ~uintptr_t(15));
  z.slot = z.crow + FL * n_titles;
  z.blkcnt = reinterpret_cast<int32_t*>((reinterpret_cast<uintptr_t>(z.slot + n_titles) + 15) & ~uintptr_t(15));
  z.cnt = reinterpret_cast<uint8_t*>(z.blkcnt + tl::BLK_INTS * tl::classify_blocks(n_titles));
  z.pad_title = z.cnt + n_titles;
  return z;
}
}  // namespace

static std::atomic<int> g_title_dedupe{[] {
  const char* e = env_knob("NRMS_DEDUPE");
  return (e && e[0] == '0') ? 0 : 1;
}()};
static std::atomic<int> g_token_compaction{[] {
  const char* e = env_knob("NRMS_COMPACT");
  return (e && e[0] == '0') ? 0 : 1;
}()};
// per-thread overrides (nrms_set_thread_*; -1: none)
static thread_local int t_title_dedupe = -1, t_token_compaction = -1;
int title_dedupe() { return t_title_dedupe >= 0 ? t_title_dedupe : g_title_dedupe.load(std::memory_order_relaxed); }
int set_title_dedupe(int on) { return g_title_dedupe.exchange(on ? 1 : 0); }
int token_compaction() {
  return t_token_compaction >= 0 ? t_token_compaction : g_token_compaction.load(std::memory_order_relaxed);
}
int set_token_compaction(int on) { return g_token_compaction.exchange(on ? 1 : 0); }
int set_thread_title_dedupe(int on) {
  const int prev = t_title_dedupe;
  t_title_dedupe = on < 0 ? -1 : (on ? 1 : 0);
  return prev;
}
int set_thread_token_compaction(int on) {
  const int prev = t_token_compaction;
  t_token_compaction = on < 0 ? -1 : (on ? 1 : 0);
  return prev;
}

bool fused_news_supported(int L, int D, int H, int Q) {
  return L == FL && D == FD && H == FH && Q == FQ;
}

#ifdef NRMS_FUSED_TIMING
unsigned long long* g_fused_dbg = nullptr;   // set by profiles/probes/news_variants.hip
#define NRMS_TIMING_ARG , g_fused_dbg
#else
#define NRMS_TIMING_ARG
#endif

namespace {
struct ClassifyDecision {
  bool classify, dedupe, compact;
};
// classification (title dedupe and / or token compaction) needs the token ids
// as 16-B aligned rows, and row ids / title indices that fit int32
ClassifyDecision classify_decision(const int64_t* ids_a, const int64_t* ids_b, int64_t n_titles, int64_t n_rows,
                                   bool direct_rows, int dedupe_setting, int compact_setting) {
  const int dedupe_on = dedupe_setting < 0 ? title_dedupe() : dedupe_setting;
  const int compact_on = compact_setting < 0 ? token_compaction() : compact_setting;
  const int64_t row_span = direct_rows ? n_titles * FL : n_rows;
  const bool classify = ids_a != nullptr && (dedupe_on || compact_on) &&
                        (((uintptr_t)ids_a | (uintptr_t)(ids_b ? ids_b : ids_a)) % 16) == 0 &&
                        row_span <= INT32_MAX && n_titles <= INT32_MAX;
  return {classify, classify && dedupe_on != 0, classify && compact_on != 0};
}
}  // namespace

bool fused_news_classify_split(float* ws, const int64_t* ids_a, int64_t n_seq_a, const int64_t* ids_b,
                               int64_t n_titles, int64_t n_rows, tl::ClassifyJob* job, tl::TitleScatter* sc) {
  const ClassifyDecision d = classify_decision(ids_a, ids_b, n_titles, n_rows, false, -1, -1);
  if (!d.classify || n_titles == 0 || ((uintptr_t)ws % 16)) return false;
  const NewsWs z = news_ws(ws, n_titles);
  const int64_t nblk = tl::classify_blocks(n_titles);
  job->rm = RowMap{ids_a, ids_b, n_seq_a, n_titles, n_rows, false};
  job->tt = Titles{z.crow, z.cnt, z.pad_title, z.list, z.counters, n_titles};
  job->sl = tl::TitleSlots{z.slot, z.blkcnt};
  job->dedupe = d.dedupe ? 1 : 0;
  job->compact = d.compact ? 1 : 0;
  job->nblk = nblk;
  *sc = tl::TitleScatter{z.slot, z.blkcnt, z.list, z.counters, n_titles, n_titles, nblk};
  return true;
}

int32_t launch_fused_news(const float* qkv, int64_t ldq, int64_t n_rows, const int64_t* ids_a,
                          int64_t n_seq_a, const int64_t* ids_b, int64_t n_titles,
                          const float* w_add, const float* b_add, const float* q_add, float* ws,
                          float* out, hipStream_t s, int dedupe_setting, bool* deduped,
                          int64_t broadcast_from, int64_t* user_list, int64_t user_rows, bool prepacked,
                          bool direct_rows, int compact_setting, bool* classified, bool preclassified) {
  if (deduped) *deduped = false;
  if (classified) *classified = false;
  if (n_titles == 0) return NRMS_OK;
  if (((uintptr_t)qkv | (uintptr_t)out | (uintptr_t)ws) % 16) return NRMS_ERR_UNSUPPORTED;
  if (ldq < 3 * FD || ldq % 4) return NRMS_ERR_UNSUPPORTED;   // float4 q / k slices
  if (max_groups(n_titles) >= (1ll << 27)) return NRMS_ERR_UNSUPPORTED;   // recheck entries: group << 4 | mask
  // F16X3: f16x3 main pass, x6 recheck pass
  const int arith = gemm_arith();
  const bool h3 = arith == NRMS_GEMM_SPLIT_F16X3;
  const bool x6 = arith != NRMS_GEMM_F32;
  const NewsWs z = news_ws(ws, n_titles);
  const RecheckList rl{z.counters + CNT_RECHECK, z.recheck};
  const ClassifyDecision cd =
      classify_decision(ids_a, ids_b, n_titles, n_rows, direct_rows, dedupe_setting, compact_setting);
  const bool classify = cd.classify, dedupe = cd.dedupe, compact = cd.compact;
  auto kern = classify ? (h3 ? &fused_news_kernel<2, false, true>
                             : (x6 ? &fused_news_kernel<1, false, true> : &fused_news_kernel<0, false, true>))
                       : (h3 ? &fused_news_kernel<2, false, false>
                             : (x6 ? &fused_news_kernel<1, false, false> : &fused_news_kernel<0, false, false>));
  auto kern_exact = classify ? (x6 ? &fused_news_kernel<1, true, true> : &fused_news_kernel<0, true, true>)
                             : (x6 ? &fused_news_kernel<1, true, false> : &fused_news_kernel<0, true, false>);
  const size_t lds_bytes = h3 ? LDS_BYTES_H : (x6 ? LDS_BYTES_X6 : LDS_BYTES);
  const size_t lds_bytes_exact = x6 ? LDS_BYTES_X6 : LDS_BYTES;
  ensure_dynamic_lds(reinterpret_cast<const void*>(kern), (int)lds_bytes);
  ensure_dynamic_lds(reinterpret_cast<const void*>(kern_exact), (int)lds_bytes_exact);
  if (preclassified && (!classify || direct_rows || !prepacked)) return NRMS_ERR_INVALID_ARG;
  const TitleSet ts{classify ? z.crow : nullptr, z.cnt, classify ? z.list : nullptr, z.counters, n_titles,
                    compact ? 0 : NBK - 1};
  // the UserEncoder's row list (nrms_forward) in the main pass's prologue
  const UserRows ur{dedupe && user_list && user_rows > 0 ? user_list : nullptr, user_rows, z.pad_title,
                    z.counters + CNT_REP, z.counters + CNT_USER};
  if (prepacked) {
    // (forward_pack_kernel packed W_add and reset the counters)
  } else if (x6) {
    const int npk = XKS * FNT * 64 * 8 + SPECIAL_FLOATS;
    if (h3)
      hipLaunchKernelGGL(pack_additive_b3_kernel<true>, dim3((npk + 255) / 256), dim3(256), 0, s, w_add, ws,
                         z.counters);
    else
      hipLaunchKernelGGL(pack_additive_b3_kernel<false>, dim3((npk + 255) / 256), dim3(256), 0, s, w_add, ws,
                         z.counters);
  } else {
    const int npk = WAP_FLOATS + SPECIAL_FLOATS;
    hipLaunchKernelGGL(pack_additive_b_kernel, dim3((npk + 255) / 256), dim3(256), 0, s, w_add, ws,
                       z.counters);
  }
  if (int32_t st = launch_status()) return st;
  int dev = 0, n_cu = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      n_cu = v;
  }
  const int64_t groups = classify ? max_groups(n_titles) : (n_titles + FT - 1) / FT;
  const int64_t blocks = groups < n_cu ? groups : n_cu;   // persistent: one workgroup per CU
  const RowMap rm{ids_a, ids_b, n_seq_a, n_titles, n_rows, direct_rows};
  if (classify && !preclassified) {
    const Titles tt{z.crow, z.cnt, z.pad_title, z.list, z.counters, n_titles};
    hipLaunchKernelGGL(classify_titles_kernel, dim3((unsigned)((n_titles + CLS_T - 1) / CLS_T)), dim3(CLS_T), 0, s,
                       rm, tt, dedupe ? 1 : 0, compact ? 1 : 0);
    if (int32_t st = launch_status()) return st;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(NTHR), lds_bytes, s, qkv, ldq, rm, ts, ws,
                     b_add, q_add, out, rl, ur NRMS_TIMING_ARG);
  if (int32_t st = launch_status()) return st;
  // the recheck pass: reads the count the main pass left; exits at once when 0
  const int64_t blocks_x = blocks < 16 ? blocks : 16;   // (flagged groups are rare; a smaller grid launches faster)
  hipLaunchKernelGGL(kern_exact, dim3((unsigned)blocks_x), dim3(NTHR), lds_bytes_exact, s, qkv, ldq, rm, ts,
                     ws, b_add, q_add, out, rl, UserRows{nullptr, 0, nullptr, nullptr, nullptr} NRMS_TIMING_ARG);
  if (int32_t st = launch_status()) return st;
  // (titles below broadcast_from are not copied: nrms_forward's UserEncoder
  // reads the clicked padding titles from the rep title's rows)
  const int64_t b0 = broadcast_from < 0 ? 0 : broadcast_from;
  if (dedupe && b0 < n_titles) {
    const int64_t nt4 = (n_titles - b0) * (FD / 4);
    hipLaunchKernelGGL(broadcast_padding_kernel, dim3((unsigned)((nt4 + 255) / 256)), dim3(256), 0, s,
                       z.pad_title, z.counters + CNT_REP, b0, n_titles, out);
  }
  const int32_t st = launch_status();
  if (st == NRMS_OK && deduped) *deduped = dedupe;
  if (st == NRMS_OK && classified) *classified = classify;
  return st;
}

PaddingGroups fused_news_padding_groups(float* ws, int64_t n_titles) {
  const NewsWs z = news_ws(ws, n_titles);
  return PaddingGroups{z.pad_title, z.counters + CNT_REP, z.counters + CNT_USER};
}

int32_t launch_user_row_list(const PaddingGroups& pg, int64_t n_rows, int64_t* list, hipStream_t s) {
  if (n_rows == 0) return NRMS_OK;
  hipLaunchKernelGGL(user_row_list_kernel, dim3((unsigned)((n_rows + URL_ROWS - 1) / URL_ROWS)), dim3(256), 0, s,
                     pg.pad_title, pg.rep, n_rows, list, pg.user_count);
  return launch_status();
}

}  // namespace nrms
