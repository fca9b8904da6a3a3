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
constexpr int FMT = FROWS / 16;      // 5 M tiles
constexpr int SC = 328;              // context row stride in floats (== 8 mod 32)
constexpr int NTHR = 256;
constexpr int WAP_FLOATS = FKG * FNT * 64 * 4;             // packed Wa
constexpr int ROW = 3 * FD;                                // q|k|v row: [q 300 | k 300 | v 300]
constexpr int SPECIAL_FLOATS = 2 * ROW;                    // zero row + NaN row
constexpr int LDS_FLOATS = FROWS * SC + 4 * FROWS + 2 * 2 * FROWS;   // ctx, partials, rowptr[2] (u64)
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
constexpr size_t LDS_BYTES_X6 = (size_t)FROWS * XRB * 2 + (4 * FROWS + 2 * 2 * FROWS) * sizeof(float);
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
constexpr size_t LDS_BYTES_H = (size_t)FROWS * XRH * 2 + (4 * FROWS + 2 * 2 * FROWS) * sizeof(float);
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
  if (idx < 4)   // [recheck count, group-list count, rep, user row-list count]
    recheck_count[idx] = idx == 2 ? INT32_MAX : 0;
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


struct RowMap {
  const int64_t* ids_a;
  const int64_t* ids_b;
  int64_t n_seq_a, n_titles, n_rows;
  // q|k|v row of token i of title s: >= 0 row, -1 invalid id (NaN row), -2 padding title
  __device__ __forceinline__ int64_t operator()(int64_t s, int i) const {
    if (s >= n_titles) return -2;
    if (!ids_a) return s * FL + i;
    const int64_t* ids = (s < n_seq_a || ids_b == nullptr) ? ids_a + s * FL : ids_b + (s - n_seq_a) * FL;
    const int64_t id = ids[i];
    return ((uint64_t)id < (uint64_t)n_rows) ? id : -1;
  }
  __device__ __forceinline__ const int64_t* ids_of(int64_t s) const {
    return (s < n_seq_a || ids_b == nullptr) ? ids_a + s * FL : ids_b + (s - n_seq_a) * FL;
  }
};

// Groups the main pass encodes. Every all-padding title (20 zero ids: the
// left-padding of short histories, src/dataset.py:79-83) has the same news
// vector in a given slot of its 4-title group, and padding runs are contiguous
// (histories are left-padded), so whole groups are padding. With a list, the
// main pass encodes only the groups holding a real title, plus one
// all-padding group (rep, the lowest); broadcast_padding_kernel then copies
// rep's vector of slot s % 4 to every title s of the other all-padding groups.
// Groups keep their titles and slots, so every output is bitwise the one the
// undeduplicated launch computes (a row's additive score sums its N-tile
// partials in an order set by its slot); the list order (atomics) only
// decides which workgroup encodes which group. Without a list group k is k.
struct GroupList {
  const int32_t* list;
  const int32_t* count;
  const int32_t* rep;   // INT32_MAX: no all-padding group
};

// One thread per title (10 x 16-B id loads), the 4 lanes of a group combined
// by a ballot: classify each group (all 80 ids zero; slots past n_titles count
// as padding) and append the others to the list; one atomicAdd and one
// atomicMin per 1,024-title block (device-scope atomics on one address
// serialise: 256-title blocks took 8.8 us at config 3).
constexpr int CLS_T = 1024, CLS_W = CLS_T / 64;
__global__ __launch_bounds__(CLS_T) void classify_groups_kernel(RowMap rm, int64_t n_groups,
                                                                int32_t* __restrict__ list,
                                                                int32_t* __restrict__ count,
                                                                int32_t* __restrict__ rep,
                                                                uint8_t* __restrict__ pad_group) {
  __shared__ int wcount[CLS_W], wbase[CLS_W], wrep[CLS_W];
  const int64_t s = (int64_t)blockIdx.x * CLS_T + threadIdx.x;   // title
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t any = 0;
  if (s < rm.n_titles) {
    const int64_t* ids = rm.ids_of(s);
#pragma unroll
    for (int i = 0; i < FL; i += 2) {
      const int4 v = *reinterpret_cast<const int4*>(ids + i);   // 16-B aligned id rows (checked)
      any |= (int64_t)(v.x | v.y | v.z | v.w);
    }
  }
  const uint64_t real = __ballot(any != 0);
  const int64_t g = s >> 2;
  const bool lead = (lane & 3) == 0 && g < n_groups;
  const bool pad = ((real >> (lane & ~3)) & 0xFull) == 0;
  if (lead) pad_group[g] = pad ? 1 : 0;
  const uint64_t keep = __ballot(lead && !pad);
  const uint64_t pads = __ballot(lead && pad);
  if (lane == 0) {
    wcount[w] = __popcll(keep);
    wrep[w] = pads ? (int32_t)((s >> 2) + ((__ffsll((long long)pads) - 1) >> 2)) : INT32_MAX;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int r = INT32_MAX, tot = 0;
    for (int i = 0; i < CLS_W; ++i) {
      r = min(r, wrep[i]);
      tot += wcount[i];
    }
    if (r != INT32_MAX) atomicMin(rep, r);
    int b = tot ? atomicAdd(count, tot) : 0;
    for (int i = 0; i < CLS_W; ++i) { wbase[i] = b; b += wcount[i]; }
  }
  __syncthreads();
  if (lead && !pad) list[wbase[w] + __popcll(keep & ((1ull << lane) - 1))] = (int32_t)g;
}

// out[s] = out[4 rep + s % 4] for every title s >= s0 of the other all-padding groups.
__global__ __launch_bounds__(256) void broadcast_padding_kernel(const uint8_t* __restrict__ pad_group,
                                                                const int32_t* __restrict__ rep, int64_t s0,
                                                                int64_t n_titles, float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;   // (title - s0, float4 column)
  const int64_t s = s0 + t / (FD / 4);
  if (s >= n_titles || !pad_group[s / FT]) return;
  const int64_t r = *rep;
  if (s / FT == r) return;
  const int c = (int)(t - (s - s0) * (FD / 4));
  reinterpret_cast<float4*>(out + s * FD)[c] =
      reinterpret_cast<const float4*>(out + (r * FT + (s % FT)) * FD)[c];
}

// The clicked rows m < n_rows (titles 0 .. n_rows - 1 of the launch) whose
// q|k|v the UserEncoder needs: all but the rows of all-padding groups other
// than rep, whose news vectors are copies of rep's slot m % 4 (the UserEncoder
// reads those rows from 4 rep + m % 4 instead). Appended in any order (vector
// atomics, one per wave); the count must start at 0.
// One 256-thread block lists rows m0 .. m0 + URL_ROWS - 1 (four 256-row
// chunks), with one atomic (per-wave atomics on the one counter serialised:
// 11 us; one per 256 rows: ~200 at config 3).
constexpr int URL_ROWS = 1024, URL_C = URL_ROWS / 256;
__device__ __forceinline__ void user_row_list_block(const uint8_t* __restrict__ pad_group,
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
    const int64_t m = m0 + 256 * c + threadIdx.x, g = m >> 2;
    keep[c] = m < n_rows && !(pad_group[g] && g != r);
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

__global__ __launch_bounds__(256) void user_row_list_kernel(const uint8_t* __restrict__ pad_group,
                                                            const int32_t* __restrict__ rep,
                                                            int64_t n_rows, int64_t* __restrict__ list,
                                                            int32_t* __restrict__ count) {
  user_row_list_block(pad_group, rep, n_rows, list, count, (int64_t)blockIdx.x * URL_ROWS);
}

// The UserEncoder's row list, built by the deduplicating main pass itself
// (nrms_forward): its workgroups list the rows before their first group.
struct UserRows {
  int64_t* list;   // null: not built here
  int64_t n_rows;
  const uint8_t* pad_group;
  const int32_t* rep;
  int32_t* count;
};

// Rows near fp32 overflow (nrms_common.hpp, kExpRecheck). The main pass
// (EXACT = false) takes the fast exp everywhere and appends the title groups
// that need the reference's exp to `list` (one entry per flagging wave;
// duplicates are harmless: the recomputation is idempotent). A second launch
// of the same kernel (EXACT = true) walks that list with the reference's exp
// in every row and overwrites those groups' outputs. With no such rows (all
// real inputs), the second launch reads the zero count and exits.
struct RecheckList {
  int32_t* count;
  int32_t* list;   // capacity 4 * n_groups
};

// Float offsets, within one q|k|v row, of what lane (head slot hl, x) of wave
// (head group) g loads: q / k dims 4c..4c+3 of head h = 4g + hl, and v dims
// 5x..5x+3 and 5x+4.
struct QkvOffsets {
  __device__ static int q(int g, int hl, int c) { return FDK * (4 * g + hl) + 4 * c; }
  __device__ static int k(int g, int hl, int c) { return FD + FDK * (4 * g + hl) + 4 * c; }
  __device__ static int v4(int g, int hl, int x) { return 2 * FD + FDK * (4 * g + hl) + 5 * x; }
  __device__ static int v1(int g, int hl, int x) { return 2 * FD + FDK * (4 * g + hl) + 5 * x + 4; }
};

// 4 floats from a 4-byte-aligned address (V slices start at 5x floats).
typedef float float4_a4 __attribute__((ext_vector_type(4), aligned(4)));
// Row pointers come back from LDS as generic pointers; loads through them are
// issued as global (not flat) loads so that they count in vmcnt only.
#define NRMS_GLOBAL __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ const NRMS_GLOBAL T* gptr(const float* p) {
  return reinterpret_cast<const NRMS_GLOBAL T*>(reinterpret_cast<uintptr_t>(p));
}

// Phase timing (profiles/probes/fused_timing.hip builds with NRMS_FUSED_TIMING):
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

// tanh(x) = 1 - 2 / (e^2x + 1): v_exp_f32 + v_rcp_f32, absolute error ~1e-7
// over the whole range (the additive scores are sums of q_n tanh(.) with
// |q_n| <= 0.1, so absolute error is what matters); saturates to +-1 and
// propagates NaN.
__device__ __forceinline__ float tanh_fast(float x) {
  const float e = __builtin_amdgcn_exp2f(2.8853900817779268f * x);   // e^(2x)
  return fmaf(-2.0f, __builtin_amdgcn_rcpf(e + 1.0f), 1.0f);
}

// Sum over the 16 lanes of a DPP row (all 16 get the total): quad butterflies,
// then half-row and row mirrors. VALU only, no LDS crossbar round trips.
__device__ __forceinline__ float row16_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));  // quad_perm [1,0,3,2]
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));  // quad_perm [2,3,0,1]
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false)); // row_half_mirror
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false)); // row_mirror
  return v;
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
template <int MODE, bool EXACT>
__global__ __launch_bounds__(NTHR, 1) void fused_news_kernel(
    const float* __restrict__ qkv, int64_t ldq, RowMap rmap, GroupList gl,
    const float* __restrict__ WaP,
    const float* __restrict__ b_add, const float* __restrict__ q_add, float* __restrict__ out,
    RecheckList rl, UserRows ur NRMS_TIMING_PARAM) {
  using Off = QkvOffsets;
  constexpr bool X6 = MODE == 1;
  constexpr bool H3 = MODE == 2;
  static_assert(!(H3 && EXACT), "the F16X3 main pass is rechecked by the x6 kernel");
  if constexpr (!EXACT) {
    if (ur.list)   // (workgroup-uniform; the padding classification ran in an earlier launch)
      for (int64_t m0 = (int64_t)blockIdx.x * URL_ROWS; m0 < ur.n_rows; m0 += (int64_t)gridDim.x * URL_ROWS) {
        user_row_list_block(ur.pad_group, ur.rep, ur.n_rows, ur.list, ur.count, m0);
        __syncthreads();   // (the block's LDS counters are reused)
      }
  }
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* ctxL = lds;                                   // f32: [80][SC]
  __bf16* ctxB = reinterpret_cast<__bf16*>(lds);       // x6:  [80][XRB] = hi | mid | lo planes
  _Float16* ctxH = reinterpret_cast<_Float16*>(lds);   // f16x3: [80][XRH] = hi | lo planes
  float* part = X6 ? lds + FROWS * XRB / 2 : (H3 ? lds + FROWS * XRH / 2 : ctxL + FROWS * SC);   // [80][4] per-wave row partials
  const float** rowptr = reinterpret_cast<const float**>(part + 4 * FROWS);   // [2][80]

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

  // row pointers of title group tg -> rowptr[buf]: the token id is loaded by
  // row_of (threads < 80), the pointer stored later by store_row, so the id
  // load's latency hides behind the work in between.
  const int64_t n_groups = (rmap.n_titles + FT - 1) / FT;
  // row_of issues the id load unconditionally (a safe address where there is
  // no id) and returns the raw value; store_row, at the end of phase A,
  // recomputes the title / token from tg and maps it (out of range: NaN row,
  // past the titles: zero row) — a use or a branch right after the load made
  // the wait for it land at the start of the phase
  auto tok = [&](int64_t tg, int64_t& s_, int& i_) __attribute__((always_inline)) -> bool {
    int tl = tid;
    asm volatile("" : "+v"(tl));   // (recomputed: a hoisted 64-bit token index spilled)
    const int t = tl / FL;
    i_ = tl - t * FL;
    s_ = tg * FT + t;
    return tl < FROWS && s_ < rmap.n_titles;
  };
  auto row_of = [&](int64_t tg) -> int64_t {
    int64_t s_;
    int i_;
    const bool ok = tok(tg, s_, i_) && rmap.ids_a;
    const int64_t* ip = ok ? rmap.ids_of(s_) + i_ : reinterpret_cast<const int64_t*>(WaP);
    return *ip;
  };
  auto store_row = [&](int64_t raw, int64_t tg, int buf) {
    int64_t s_;
    int i_;
    const bool ok = tok(tg, s_, i_);
    const int64_t r = rmap.ids_a ? raw : s_ * FL + i_;
    if (tid < FROWS)
      rowptr[buf * FROWS + tid] = !ok ? zero_row : ((uint64_t)r < (uint64_t)rmap.n_rows ? qkv + r * ldq : nan_row);
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
  const float4* Bp = reinterpret_cast<const float4*>(WaP) + lane;
  const float* Aw = ctxL + lm * SC + 4 * kq;

  // q|k|v slices of one title group, lane (block (t, hl), x): Q / K of tokens
  // x + 4j, V dims 5x..5x+4 of all 20 tokens. Loaded for the NEXT group: Q / K
  // at the start of the B epilogue (in flight behind the tanh work, a barrier
  // and the pooling), V at the end of C (behind the next S^T phase).
  float qf[5][FDK], kf[5][FDK], vf[FL][5];
  auto prefetch_qk_tok = [&](int buf, int j) {   // token x + 4j of the lane's title
    const float* rp = rowptr[buf * FROWS + FL * at + x + 4 * j];
#pragma unroll
    for (int c = 0; c < FDK / 4; ++c) {
      const floatx4 a = *gptr<floatx4>(rp + Off::q(w, hls, c));
      const floatx4 b = *gptr<floatx4>(rp + Off::k(w, hls, c));
      qf[j][4 * c] = a.x; qf[j][4 * c + 1] = a.y; qf[j][4 * c + 2] = a.z; qf[j][4 * c + 3] = a.w;
      kf[j][4 * c] = b.x; kf[j][4 * c + 1] = b.y; kf[j][4 * c + 2] = b.z; kf[j][4 * c + 3] = b.w;
    }
  };
  auto prefetch_qk = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 5; ++j) prefetch_qk_tok(buf, j);
  };
  // (50 + 40 loads in two batches: at most 63 may be outstanding per wave)
  auto prefetch_v_tok = [&](int buf, int k) {
    const float* vr = rowptr[buf * FROWS + FL * at + k];
    const float4_a4 a = *gptr<float4_a4>(vr + Off::v4(w, hls, x));
    vf[k][0] = a.x; vf[k][1] = a.y; vf[k][2] = a.z; vf[k][3] = a.w;
    vf[k][4] = *gptr<float>(vr + Off::v1(w, hls, x));
  };
  auto prefetch_v = [&](int buf) {
#pragma unroll
    for (int k = 0; k < FL; ++k) prefetch_v_tok(buf, k);
  };

  // iteration k of this workgroup handles title group group_at(k): k itself in
  // the main pass, the k-th flagged group in the EXACT pass (past the end: a
  // group of padding titles, so the prefetch of "the next group" stays valid)
  // (main pass with a group list: the listed groups, then rep)
  const int64_t n_list = gl.list ? (int64_t)*gl.count : n_groups;
  const int32_t rep = gl.list ? *gl.rep : INT32_MAX;
  const int64_t n_iter = EXACT ? (int64_t)*rl.count : n_list + (rep != INT32_MAX ? 1 : 0);
  auto group_at = [&](int64_t k) -> int64_t {
    if constexpr (EXACT) return k < n_iter ? (int64_t)rl.list[k] : n_groups;
    if (gl.list) return k < n_list ? (int64_t)gl.list[k] : (k == n_list && rep != INT32_MAX ? (int64_t)rep : n_groups);
    else return k;
  };
  if (blockIdx.x < n_iter) store_row(row_of(group_at(blockIdx.x)), group_at(blockIdx.x), 0);
  __syncthreads();
  if (blockIdx.x < n_iter) {
    prefetch_qk(0);
    prefetch_v(0);
  }
#ifdef NRMS_FUSED_TIMING
  unsigned long long tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tprev = __builtin_amdgcn_s_memtime();
#endif

  int it = 0;
  for (int64_t k = blockIdx.x; k < n_iter; k += gridDim.x, ++it) {
    const int64_t tg = group_at(k);
    const int nbuf = (it + 1) & 1;
    // (no barrier here: the context tile's last readers, the previous group's
    // B mainloop, finished before its B -> C barrier; C reads registers + part)
#ifdef NRMS_FUSED_TIMING
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // probe only: time the wait for this group's q|k|v
#endif
    NRMS_STAMP(0)
    floatx4 O[5][5];   // this wave's context rows, live until the pooling in C
    uint64_t recheck = 0;   // lanes whose row needs the recheck pass (RecheckList)

    // ---------------- A: attention (4x4x1 MFMA, 16 (title, head) blocks) --------------
    {
      // row pointers of the next group, for the prefetch in this group's B
      // epilogue (past the last group: zero rows, so the prefetch is
      // unconditional and its registers are dead during the GEMM); stored at
      // the end of this phase
      const int64_t next_tg = group_at(k + gridDim.x);
      const int64_t next_row = row_of(next_tg);
      // S^T tiles: rows = keys 4j + r (A = K), cols = queries 4i + x (B = Q)
      floatx4 S[5][5];
#pragma unroll
      for (int j = 0; j < 5; ++j)
#pragma unroll
        for (int i = 0; i < 5; ++i) S[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};
      // One query column i at a time (S^T, exp, ctx^T, split + store), so a
      // column's S registers die before the next column's are written: short
      // live ranges, no spills (all S^T first, then all ctx^T: 2 % slower;
      // column i's split interleaved with column i + 1's MFMAs through
      // sched_group_barrier: no better).
      auto s_mfma = [&](int i) {
#pragma unroll
        for (int d = 0; d < FDK; ++d)
#pragma unroll
          for (int j = 0; j < 5; ++j) S[j][i] = mfma4(kf[j][d], qf[i][d], S[j][i]);
      };
      // P = exp(S / sqrt(dk)) / (sum_keys + 1e-8): query 4i + x, key 4j + r
      auto s_exp = [&](int i) {
        float sum = 0.f;
#pragma unroll
        for (int j = 0; j < 5; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float e = EXACT ? ref_exp(S[j][i][r], sqrt_dk)
                                  : __builtin_amdgcn_exp2f(S[j][i][r] * c_exp);
            S[j][i][r] = e;
            sum += e;
          }
        // rows near fp32 overflow (or non-finite): flagged (no branch here),
        // recomputed by the EXACT pass (RecheckList)
        if constexpr (!EXACT) recheck |= __builtin_amdgcn_ballot_w64(exp_row_needs_recheck(sum));
        const float inv = 1.0f / (sum + 1e-8f);
#pragma unroll
        for (int j = 0; j < 5; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) S[j][i][r] *= inv;
      };
      // ctx^T tiles: rows = dims 5r' + m (A = V^T), cols = queries 4i + x (B = P^T);
      // lane x holds ctx[query 4i + x][dim 5r' + m] = O[m][i][r']
      auto o_mfma = [&](int i) {
#pragma unroll
        for (int m = 0; m < 5; ++m) O[m][i] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < FL; ++k)
#pragma unroll
          for (int m = 0; m < 5; ++m) O[m][i] = mfma4(vf[k][m], S[k >> 2][i][k & 3], O[m][i]);
      };
      // (a branch-free form, with the idle head slot storing its bit-identical
      // copy of head 12, measured 9 % slower: the compiler then interleaves the
      // stores into the next column's MFMAs and spills)
      auto o_store = [&](int i) {
        if (!hval) return;
        if constexpr (H3) {
          _Float16* dst = ctxH + (FL * at + 4 * i + x) * XRH + FDK * h;
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
          __bf16* dst = ctxB + (FL * at + 4 * i + x) * XRB + FDK * h;
#pragma unroll
          for (int c = 0; c < FDK / 4; ++c) {
            uint32_t h[2], m[2], l[2];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              const int d = 4 * c + 2 * e;
              split3x2(O[d % 5][i][d / 5], O[(d + 1) % 5][i][(d + 1) / 5], h[e], m[e], l[e]);
            }
            *reinterpret_cast<uint2*>(dst + 4 * c) = make_uint2(h[0], h[1]);
            *reinterpret_cast<uint2*>(dst + XKP + 4 * c) = make_uint2(m[0], m[1]);
            *reinterpret_cast<uint2*>(dst + 2 * XKP + 4 * c) = make_uint2(l[0], l[1]);
          }
        } else {
          float4* dst = reinterpret_cast<float4*>(ctxL + (FL * at + 4 * i + x) * SC + FDK * h);
#pragma unroll
          for (int c = 0; c < FDK / 4; ++c) {
            const int d0 = 4 * c;
            dst[c] = make_float4(O[d0 % 5][i][d0 / 5], O[(d0 + 1) % 5][i][(d0 + 1) / 5],
                                 O[(d0 + 2) % 5][i][(d0 + 2) / 5], O[(d0 + 3) % 5][i][(d0 + 3) / 5]);
          }
        }
      };
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        s_mfma(i);
        s_exp(i);
        o_mfma(i);
        o_store(i);
      }
      store_row(next_row, next_tg, nbuf);
    }
    NRMS_STAMP(1)
    __syncthreads();   // context tile complete
    NRMS_STAMP(2)

    // ---------------- B: additive GEMM + tanh·q row partials ----------------
    {
      floatx4 acc[FMT][3], accX = floatx4{0.f, 0.f, 0.f, 0.f}, accX2 = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int mt = 0; mt < FMT; ++mt)
#pragma unroll
        for (int j = 0; j < 3; ++j) acc[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};
      if constexpr (X6) {
        // A fragments (16x16x32): lane holds A[row lm][32 ks + 8 kq .. + 7] of each plane
        const __bf16* Ab = ctxB + lm * XRB + 8 * kq;
        // B fragments through a buffer resource (as the F16X3 path below)
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
        // one 32-deep k-step; EXTRA: wave 0 also owns (M-tile 4, N-tile 12)
        // the wave index is a template constant (the X tile's A rows = M-tile
        // W: no second read of them); A planes loaded lo first, the order the
        // products consume them
        auto kstep = [&](int ks, const bf16x8 (&bb)[4][3], auto wc) {
          constexpr int W = decltype(wc)::value;
          constexpr bool EXTRA = W == 0;
          bf16x8 a[FMT][3];
#pragma unroll
          for (int pl = 2; pl >= 0; --pl)
#pragma unroll
            for (int mt = 0; mt < FMT; ++mt)
              a[mt][pl] = *reinterpret_cast<const bf16x8*>(Ab + 16 * mt * XRB + pl * XKP + 32 * ks);
          const bf16x8 (&ax)[3] = a[W];
          // the six products with i + j <= 2, smallest first
#define NRMS_X6STEP(PA, PB)                                                                              \
  _Pragma("unroll") for (int mt = 0; mt < FMT; ++mt)                                                     \
  _Pragma("unroll") for (int j = 0; j < 3; ++j)                                                          \
      acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt][PA], bb[j][PB], acc[mt][j], 0, 0, 0);   \
  accX = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax[PA], bb[3][PB], accX, 0, 0, 0);                      \
  if constexpr (EXTRA) accX2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[FMT - 1][PA], bb[3][PB], accX2, 0, 0, 0);
          NRMS_X6STEP(2, 0) NRMS_X6STEP(1, 1) NRMS_X6STEP(0, 2) NRMS_X6STEP(1, 0) NRMS_X6STEP(0, 1)
          NRMS_X6STEP(0, 0)
#undef NRMS_X6STEP
        };
        // two B buffers in turn (XKS is even): no register copies between k-steps
        auto mainloop = [&](auto extra) {
          bf16x8 b0[4][3], b1[4][3];
          load_b(0, b0);
#pragma unroll
          for (int ks = 0; ks < XKS; ks += 2) {
            load_b(ks + 1, b1);
            kstep(ks, b0, extra);
            __builtin_amdgcn_sched_barrier(0);
            if (ks + 2 < XKS) load_b(ks + 2, b0);
            kstep(ks + 1, b1, extra);
            __builtin_amdgcn_sched_barrier(0);
          }
        };
        static_assert(XKS % 2 == 0, "k-steps in pairs");
        switch (w) {
          case 0: mainloop(std::integral_constant<int, 0>{}); break;
          case 1: mainloop(std::integral_constant<int, 1>{}); break;
          case 2: mainloop(std::integral_constant<int, 2>{}); break;
          default: mainloop(std::integral_constant<int, 3>{}); break;
        }
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
        // packed hi' plane is not read — 2/3 of the fragment loads: news_fused
        // -2 %), 1 = lo, 2 = hi; loaded in consumption order
        auto load_b = [&](int ks, f16x8 (&dst)[4][3]) {
#pragma unroll
          for (int pl = 2; pl >= 1; --pl)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              dst[j][pl] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(
                  brs, bvoff[j], (ks * FNT * 3 + pl) * 1024, 0));
        };
        auto kstep = [&](int ks, f16x8 (&bb)[4][3], auto wc) {
          constexpr int W = decltype(wc)::value;
          constexpr bool EXTRA = W == 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) bb[j][0] = bb[j][2] * (_Float16)kF16LoScale;
          f16x8 a[FMT][2];
#pragma unroll
          for (int pl = 1; pl >= 0; --pl)
#pragma unroll
            for (int mt = 0; mt < FMT; ++mt)
              a[mt][pl] = *reinterpret_cast<const f16x8*>(Ah + 16 * mt * XRH + pl * XKP + 32 * ks);
          const f16x8 (&ax)[2] = a[W];
#define NRMS_H3STEP(PA, PB)                                                                            \
  _Pragma("unroll") for (int mt = 0; mt < FMT; ++mt)                                                   \
  _Pragma("unroll") for (int j = 0; j < 3; ++j)                                                        \
      acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[mt][PA], bb[j][PB], acc[mt][j], 0, 0, 0);  \
  accX = __builtin_amdgcn_mfma_f32_16x16x32_f16(ax[PA], bb[3][PB], accX, 0, 0, 0);                     \
  if constexpr (EXTRA) accX2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[FMT - 1][PA], bb[3][PB], accX2, 0, 0, 0);
          NRMS_H3STEP(1, 2) NRMS_H3STEP(0, 1) NRMS_H3STEP(0, 0)
#undef NRMS_H3STEP
        };
        auto mainloop = [&](auto extra) {
          f16x8 b0[4][3], b1[4][3];
          load_b(0, b0);
          // fully unrolled, each k-step's loads and MFMAs fenced in place
          // (without the fences the scheduler hoists every load: 1,100 spills);
          // a rolled loop permuted the accumulators at its back-edge (~170
          // AGPR moves per iteration): 1.41 -> 1.33 ms
#pragma unroll
          for (int ks = 0; ks < XKS; ks += 2) {
            load_b(ks + 1, b1);
            kstep(ks, b0, extra);
            __builtin_amdgcn_sched_barrier(0);
            if (ks + 2 < XKS) load_b(ks + 2, b0);
            kstep(ks + 1, b1, extra);
            __builtin_amdgcn_sched_barrier(0);
          }
        };
        switch (w) {
          case 0: mainloop(std::integral_constant<int, 0>{}); break;
          case 1: mainloop(std::integral_constant<int, 1>{}); break;
          case 2: mainloop(std::integral_constant<int, 2>{}); break;
          default: mainloop(std::integral_constant<int, 3>{}); break;
        }
#pragma unroll
        for (int mt = 0; mt < FMT; ++mt)
#pragma unroll
          for (int j = 0; j < 3; ++j) acc[mt][j] *= kLoUnscale;
        accX *= kLoUnscale;
        accX2 *= kLoUnscale;
      } else {
      float4 bb[4], bn[4];
#pragma unroll
      for (int j = 0; j < 3; ++j) bb[j] = Bp[(3 * w + j) * 64];
      bb[3] = Bp[12 * 64];
      for (int c = 0; c < FKG; ++c) {
        if (c + 1 < FKG) {
#pragma unroll
          for (int j = 0; j < 3; ++j) bn[j] = Bp[((c + 1) * FNT + 3 * w + j) * 64];
          bn[3] = Bp[((c + 1) * FNT + 12) * 64];
        }
        float4 a[FMT];
#pragma unroll
        for (int mt = 0; mt < FMT; ++mt) a[mt] = *reinterpret_cast<const float4*>(Aw + 16 * mt * SC + 16 * c);
        const float4 ax = *reinterpret_cast<const float4*>(Aw + 16 * w * SC + 16 * c);
#define NRMS_KSTEP(F)                                                                             \
  _Pragma("unroll") for (int mt = 0; mt < FMT; ++mt)                                              \
  _Pragma("unroll") for (int j = 0; j < 3; ++j)                                                   \
      acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt].F, bb[j].F, acc[mt][j], 0, 0, 0);   \
  accX = __builtin_amdgcn_mfma_f32_16x16x4f32(ax.F, bb[3].F, accX, 0, 0, 0);                      \
  if (w == 0) accX2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[FMT - 1].F, bb[3].F, accX2, 0, 0, 0);
        NRMS_KSTEP(x) NRMS_KSTEP(y) NRMS_KSTEP(z) NRMS_KSTEP(w)
#undef NRMS_KSTEP
        if (c + 1 < FKG) {
#pragma unroll
          for (int j = 0; j < 4; ++j) bb[j] = bn[j];
        }
      }
      }
      NRMS_STAMP(3)
      // C/D layout of 16x16 MFMA: col = lane & 15, row = (lane >> 4) * 4 + reg.
      // The next group's Q|K slices go out one token per M-tile, between the
      // tanh blocks (pinned by sched_barrier): issued all at once ahead of the
      // tanh work, the in-order issue stalls the VALU behind the gather's
      // address/TA queue (measured 3 % slower for the whole kernel).
#pragma unroll
      for (int mt = 0; mt < FMT; ++mt) {
        prefetch_qk_tok(nbuf, mt);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float p = 0.f;
#pragma unroll
          for (int j = 0; j < 3; ++j) p = fmaf(qv[j], tanh_fast(acc[mt][j][r] + bv[j]), p);
          if (xok && mt == w) p = fmaf(qx, tanh_fast(accX[r] + bx), p);
          if (xok && w == 0 && mt == FMT - 1) p = fmaf(qx, tanh_fast(accX2[r] + bx), p);
          p = row16_sum(p);
          if (lm == 0) part[4 * (16 * mt + 4 * kq + r) + w] = p;   // [row][wave]
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    NRMS_STAMP(4)
    __syncthreads();   // row partials complete
    NRMS_STAMP(5)

    // ---------------- C: softmax over tokens + pooling from the O registers ----------------
    // Lane (block (at, hl), x) holds rows 4i + x (i < 5) of title at, head h:
    // the 4 lanes of a block see all 20 tokens, so the softmax (max-subtracted,
    // as F.softmax) and the pooling out[20h + d] = sum_l w_l ctx[l][20h + d]
    // reduce within the lane quad (DPP); the LDS tile is not read.
    {
      float sc[5];
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        const float4 pv = *reinterpret_cast<const float4*>(part + 4 * (FL * at + 4 * i + x));
        sc[i] = ((pv.x + pv.y) + pv.z) + pv.w;
      }
      if constexpr (H3) {
        // a NaN score: an operand beyond fp16's range (or NaN inputs) -> recheck pass
        bool bad = false;
#pragma unroll
        for (int i = 0; i < 5; ++i) bad |= sc[i] != sc[i];
        recheck |= __builtin_amdgcn_ballot_w64(bad);
      }
      if constexpr (!EXACT) {
        if (recheck != 0 && lane == 0) rl.list[atomicAdd(rl.count, 1)] = (int32_t)tg;
      }
      float mx = sc[0];
#pragma unroll
      for (int i = 1; i < 5; ++i) mx = nan_max(mx, sc[i]);
      mx = nan_max(mx, quad_xor1(mx));
      mx = nan_max(mx, quad_xor2(mx));
      float ex[5], sum = 0.f;
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        ex[i] = expf(sc[i] - mx);
        sum += ex[i];
      }
      sum += quad_xor1(sum);
      sum += quad_xor2(sum);
      float wt[5];
#pragma unroll
      for (int i = 0; i < 5; ++i) wt[i] = ex[i] / sum;
      // pz[m][r'] = dim 5r' + m of head h, summed over this lane's 5 queries, then the quad
      float pz[5][4];
#pragma unroll
      for (int m = 0; m < 5; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float a = 0.f;
#pragma unroll
          for (int i = 0; i < 5; ++i) a = fmaf(wt[i], O[m][i][r], a);
          a += quad_xor1(a);
          pz[m][r] = a + quad_xor2(a);
        }
      const int64_t s = tg * FT + at;
      if (hval && s < rmap.n_titles) {
        // lane x stores dims 5x .. 5x + 4 of head h
        float v[5];
#pragma unroll
        for (int m = 0; m < 5; ++m)
          v[m] = x == 0 ? pz[m][0] : (x == 1 ? pz[m][1] : (x == 2 ? pz[m][2] : pz[m][3]));
        float* dst = out + s * FD + FDK * h + 5 * x;
        float4_a4 v4;
        v4.x = v[0]; v4.y = v[1]; v4.z = v[2]; v4.w = v[3];
        *reinterpret_cast<float4_a4*>(dst) = v4;
        dst[4] = v[4];
      }
      // V slices of the next group: issued here, after O is dead (holding both
      // through the B epilogue spills); the S^T phase of the next group covers
      // most of their latency (measured wait ~1.3k cycles per group)
      prefetch_v(nbuf);
    }
    NRMS_STAMP(6)
  }
#ifdef NRMS_FUSED_TIMING
  if (!EXACT && lane == 0)
    for (int k = 0; k < 8; ++k) dbg[(blockIdx.x * 4 + w) * 8 + k] = tacc[k];
#endif
}

}  // namespace

// packed W_add + special rows, then int32 [recheck count, group-list count,
// rep, user row-list count] (zeroed / rep = INT32_MAX by the pack kernel of
// every launch), the recheck list (4 per group), the group list, pad_group
// bytes
static size_t fused_news_list_offset() { return (size_t)WAP_MAX + SPECIAL_FLOATS + WAP2_FLOATS; }
size_t fused_news_workspace_floats(int64_t n_titles) {
  const int64_t n_groups = (n_titles + FT - 1) / FT;
  return fused_news_list_offset() + 4 + 4 * (size_t)n_groups + (size_t)n_groups +
         ((size_t)n_groups + 3) / 4;
}

static std::atomic<int> g_title_dedupe{[] {
  const char* e = getenv("NRMS_DEDUPE");
  return (e && e[0] == '0') ? 0 : 1;
}()};
int title_dedupe() { return g_title_dedupe.load(std::memory_order_relaxed); }
static bool dedupe_applies(int dedupe, const int64_t* ids_a, const int64_t* ids_b) {
  return dedupe && ids_a != nullptr && (((uintptr_t)ids_a | (uintptr_t)(ids_b ? ids_b : ids_a)) % 16) == 0;
}
int set_title_dedupe(int on) { return g_title_dedupe.exchange(on ? 1 : 0); }

bool fused_news_supported(int L, int D, int H, int Q) {
  return L == FL && D == FD && H == FH && Q == FQ;
}

#ifdef NRMS_FUSED_TIMING
unsigned long long* g_fused_dbg = nullptr;   // set by profiles/probes/news_variants.hip
#define NRMS_TIMING_ARG , g_fused_dbg
#else
#define NRMS_TIMING_ARG
#endif

int32_t launch_fused_news(const float* qkv, int64_t ldq, int64_t n_rows, const int64_t* ids_a,
                          int64_t n_seq_a, const int64_t* ids_b, int64_t n_titles,
                          const float* w_add, const float* b_add, const float* q_add, float* ws,
                          float* out, hipStream_t s, int dedupe_setting, bool* deduped,
                          int64_t broadcast_from, int64_t* user_list, int64_t user_rows, bool prepacked) {
  if (deduped) *deduped = false;
  if (n_titles == 0) return NRMS_OK;
  if (((uintptr_t)qkv | (uintptr_t)out | (uintptr_t)ws) % 16) return NRMS_ERR_UNSUPPORTED;
  if (ldq < ROW || ldq % 4) return NRMS_ERR_UNSUPPORTED;   // float4 q / k slices
  const int64_t n_groups = (n_titles + FT - 1) / FT;
  if (4 * n_groups > INT32_MAX) return NRMS_ERR_UNSUPPORTED;
  // F16X3: f16x3 main pass, x6 recheck pass
  const int arith = gemm_arith();
  const bool h3 = arith == NRMS_GEMM_SPLIT_F16X3;
  const bool x6 = arith != NRMS_GEMM_F32;
  auto kern = h3 ? &fused_news_kernel<2, false> : (x6 ? &fused_news_kernel<1, false> : &fused_news_kernel<0, false>);
  auto kern_exact = x6 ? &fused_news_kernel<1, true> : &fused_news_kernel<0, true>;
  const size_t lds_bytes = h3 ? LDS_BYTES_H : (x6 ? LDS_BYTES_X6 : LDS_BYTES);
  const size_t lds_bytes_exact = x6 ? LDS_BYTES_X6 : LDS_BYTES;
  ensure_dynamic_lds(reinterpret_cast<const void*>(kern), (int)lds_bytes);
  ensure_dynamic_lds(reinterpret_cast<const void*>(kern_exact), (int)lds_bytes_exact);
  int32_t* rcount = reinterpret_cast<int32_t*>(ws + fused_news_list_offset());
  const RecheckList rl{rcount, rcount + 4};
  int32_t* glist = rcount + 4 + 4 * n_groups;
  uint8_t* pad_group = reinterpret_cast<uint8_t*>(glist + n_groups);
  // padding-group dedupe needs the token ids (gathered rows), 16-B aligned id rows
  const bool dedupe = dedupe_applies(dedupe_setting < 0 ? title_dedupe() : dedupe_setting, ids_a, ids_b);
  const GroupList gl{dedupe ? glist : nullptr, rcount + 1, rcount + 2};
  // the UserEncoder's row list (nrms_forward) in the main pass's prologue
  const UserRows ur{dedupe && user_list && user_rows > 0 ? user_list : nullptr, user_rows, pad_group, rcount + 2,
                    rcount + 3};
  if (prepacked) {
    // (forward_pack_kernel packed W_add and reset the counters)
  } else if (x6) {
    const int npk = XKS * FNT * 64 * 8 + SPECIAL_FLOATS;
    if (h3)
      hipLaunchKernelGGL(pack_additive_b3_kernel<true>, dim3((npk + 255) / 256), dim3(256), 0, s, w_add, ws,
                         rcount);
    else
      hipLaunchKernelGGL(pack_additive_b3_kernel<false>, dim3((npk + 255) / 256), dim3(256), 0, s, w_add, ws,
                         rcount);
  } else {
    const int npk = WAP_FLOATS + SPECIAL_FLOATS;
    hipLaunchKernelGGL(pack_additive_b_kernel, dim3((npk + 255) / 256), dim3(256), 0, s, w_add, ws,
                       rcount);
  }
  if (int32_t st = launch_status()) return st;
  int dev = 0, n_cu = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      n_cu = v;
  }
  const int64_t blocks = n_groups < n_cu ? n_groups : n_cu;   // persistent: one workgroup per CU
  RowMap rm{ids_a, ids_b, n_seq_a, n_titles, n_rows};
  if (dedupe) {
    hipLaunchKernelGGL(classify_groups_kernel, dim3((unsigned)((4 * n_groups + CLS_T - 1) / CLS_T)), dim3(CLS_T),
                       0, s, rm, n_groups, glist, rcount + 1, rcount + 2, pad_group);
    if (int32_t st = launch_status()) return st;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(NTHR), lds_bytes, s, qkv, ldq, rm, gl, ws,
                     b_add, q_add, out, rl, ur NRMS_TIMING_ARG);
  if (int32_t st = launch_status()) return st;
  // the recheck pass: reads the count the main pass left; exits at once when 0
  const int64_t blocks_x = blocks < 64 ? blocks : 64;
  hipLaunchKernelGGL(kern_exact, dim3((unsigned)blocks_x), dim3(NTHR), lds_bytes_exact, s, qkv, ldq, rm, gl,
                     ws, b_add, q_add, out, rl, UserRows{nullptr, 0, nullptr, nullptr, nullptr} NRMS_TIMING_ARG);
  if (int32_t st = launch_status()) return st;
  // (titles below broadcast_from are not copied: nrms_forward's UserEncoder
  // reads the clicked padding titles from the rep group's rows)
  const int64_t b0 = broadcast_from < 0 ? 0 : (broadcast_from / FT) * FT;
  if (dedupe && b0 < n_titles) {
    const int64_t nt4 = (n_titles - b0) * (FD / 4);
    hipLaunchKernelGGL(broadcast_padding_kernel, dim3((unsigned)((nt4 + 255) / 256)), dim3(256), 0, s,
                       pad_group, rcount + 2, b0, n_titles, out);
  }
  const int32_t st = launch_status();
  if (st == NRMS_OK && deduped) *deduped = dedupe;
  return st;
}

PaddingGroups fused_news_padding_groups(float* ws, int64_t n_titles) {
  const int64_t n_groups = (n_titles + FT - 1) / FT;
  int32_t* rcount = reinterpret_cast<int32_t*>(ws + fused_news_list_offset());
  int32_t* glist = rcount + 4 + 4 * n_groups;
  return PaddingGroups{reinterpret_cast<const uint8_t*>(glist + n_groups), rcount + 2, rcount + 3};
}

int32_t launch_user_row_list(const PaddingGroups& pg, int64_t n_rows, int64_t* list, hipStream_t s) {
  if (n_rows == 0) return NRMS_OK;
  int32_t* count = pg.user_count;
  hipLaunchKernelGGL(user_row_list_kernel, dim3((unsigned)((n_rows + URL_ROWS - 1) / URL_ROWS)), dim3(256), 0, s,
                     pg.pad_group, pg.rep, n_rows, list, count);
  return launch_status();
}

}  // namespace nrms
