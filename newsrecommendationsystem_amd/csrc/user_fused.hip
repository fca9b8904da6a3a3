// Fused UserEncoder tail (src/model/NRMS/user_encoder.py:15-26): raw-exp
// MHSA over the clicked-news Q|K|V rows (multihead_self.py:15-23,74-75), the
// additive projection tanh(ctx W^T + b)·q (additive.py:35-38), the softmax over
// the N clicked positions and the pooling (:39,51-52) in one launch, one
// workgroup per user. Replaces the mhsa / additive-score / pool stage kernels
// and their two HBM round trips of the [B*N, 300] context.
//
// LDS holds one [LMAX][600] fp32 tile (153.6 KB at LMAX = 64):
//   0. the user's K|V rows (qkv columns 300..899) are staged in it;
//   1. every (head, query) pair is one thread (15 N <= blockDim): q slice in
//      registers, the N raw exps in registers (no max subtraction, as the
//      reference), / (sum + 1e-8), context slice accumulated in registers;
//      after a barrier the context rows are written over the K|V tile, with
//      columns 300..319 zeroed (K padding):
//      MODE 1 writes the context as its exact three-way bf16 split (three
//      planes of 320 per row, k in MFMA fragment order), MODE 0 as fp32;
//   2. additive GEMM [N x 320] x [320 x 208]: split-bf16 x6 on
//      v_mfma_f32_16x16x32_bf16 (MODE 1; lane (lm, kq) reads k = 32ks + 4kq +
//      0..3 and 32ks + 16 + 4kq + 0..3 of each plane in one ds_read_b128,
//      conflict-free at row stride 600 floats), W_add pre-split into bf16
//      planes packed in the same K order; or exact f32 MFMA 16x16x4 (MODE 0). Wave w owns N-tiles w, w + NW, ...
//      for all M-tiles (rows >= N read row N-1 and are dropped). Epilogue:
//      per-row partials of q_n tanh(y + b_n) (v_exp + v_rcp form), one LDS row per N-tile;
//   3. softmax over the N rows (max-subtracted, F.softmax) and the pooling
//      (up to eight lanes per float4 column, combined by lane shuffles).
// MODE 2 (split-f16, the default arithmetic): each context row is scaled by
// a power of two, 2^-ea (its max |value| into [2^3, 2^4): each (head,
// query) thread leaves its max in an LDS slot, read by the row's 15 threads
// after the barrier — an LDS atomic kept the row index live across the
// attention and spilled), and stored as three fp16
// planes, 2^11 a' = 2^11 hi + lo + r (exact for every value within 2^-15 of
// the row max; the pooling rebuilds the context from them); W_add comes split
// per output column (packs.hpp pack_user_additive_h3). The GEMM reads two
// planes and accumulates a_hi·w_lo + a_lo·w_hi + (2^11 a_hi)·w_hi on
// v_mfma_f32_16x16x32_f16 (three products instead of six, 22-bit operands as
// the news kernel's additive GEMM), y = ldexp(acc, ea + ew - 11). No range
// fallback is needed: the scaling keeps every operand inside fp16.
#include "nrms_common.hpp"
#include "packs.hpp"

#include <atomic>
#include <cstdlib>
#include <type_traits>

namespace nrms {
namespace {

constexpr int UD = 300, UH = 15, UDK = 20, UQ = 200;
constexpr int UKS = 10;                    // bf16 k-steps of 32 (K 300 -> 320)
constexpr int UKG = 19;                    // f32 k-groups of 16 (K 300 -> 304)
constexpr int UNT = 13;                    // N tiles (208 >= 200)
constexpr int UWAP3 = UKS * UNT * 3 * 64 * 4;   // floats: [ks][nt][plane][lane][8 bf16]
constexpr int UWAP1 = UKG * UNT * 64 * 4;       // floats: [kg][nt][lane][4]
constexpr int UWAP_MAX = UWAP3 > UWAP1 ? UWAP3 : UWAP1;
#ifdef NRMS_USER_TIMING
constexpr int USTAMP_FLOATS = 4096 * 8 * 2;     // probe: 8 u64 per user (B <= 4096)
#else
constexpr int USTAMP_FLOATS = 0;
#endif
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 uf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 uf16x4 __attribute__((ext_vector_type(4)));


// W_add -> B fragments. x6: element i of lane (n = lane & 15, kq = lane >> 4)
// is k = 32 ks + 4 kq + (i & 3) + 16 (i >> 2), three bf16 planes. f32: the
// 16x16x4 layout of the news kernel, k = 16 kg + 4 kq + t.
__global__ __launch_bounds__(256) void pack_user_b_kernel(const float* __restrict__ Wa,
                                                          float* __restrict__ WaP, int mode) {
  if (mode == 2) pk::pack_user_additive_h3(blockIdx.x, threadIdx.x, Wa, WaP);
  else pk::pack_user_additive(blockIdx.x * 256 + threadIdx.x, Wa, WaP, mode);
}
static_assert(pk::KS == UKS && pk::NT == UNT && pk::KG == UKG && pk::Q == UQ && pk::D == UD &&
                  pk::USER_F32_ELEMS == UWAP1,
              "packs.hpp layout");
static_assert(pk::USER_H3_EXP + pk::NT * 16 <= UWAP_MAX, "split-f16 W_add pack fits the workspace");

constexpr int URS = 2 * UD;                // LDS row stride: K|V, then context (conflict-free)
constexpr int UKP = 320;                   // bf16 context plane width (K padded)

// Position of context column k in a bf16 plane: within each 32-column block,
// lane kq's eight fragment elements (k = 4kq + 0..3 and 16 + 4kq + 0..3) are
// contiguous, so one ds_read_b128 per plane fetches them.
__device__ __forceinline__ int ukpos(int k) {
  return (k & ~31) + 8 * ((k & 15) >> 2) + 4 * ((k & 31) >> 4) + (k & 3);
}

// Token compaction (uflags & UF_COMPACT, nrms_forward): the clicked positions
// of a user whose titles are all padding (the left-padding of short
// histories, src/dataset.py:79-83) have one news vector, so wave 0 lists the
// user's Le = real + 1 distinct rows -- the padding row first, the real
// positions in order -- and the whole tail runs on Le rows, the padding row
// counted n_pad times: its exp added n_pad times first in every raw-exp sum
// (the reference's key order for left padding: the sums are bitwise the
// uncompacted ones), its attention weight and its softmax weight scaled by
// n_pad. UF_COPIED: the copied padding titles' rows were not projected (the
// row-list projection after dedupe); the padding row is then rep's, else the
// user's own first padding position's.
constexpr int UF_COPIED = 1, UF_COMPACT = 2;
// UF_TASK_SPLIT: the chunked instance's two passes split by task index (the
// round-5 form) even where the head split adds no wave (NRMS_USER_HSPLIT=0:
// the test that the head split changes no bit)
constexpr int UF_TASK_SPLIT = 4;
// UF_NO_PAIR: the chunked instance's long users (more tasks than threads) in
// two passes (split by head or task index) instead of two queries per thread
// in one pass (NRMS_USER_PAIR=0: the test that the pairing changes no bit)
constexpr int UF_NO_PAIR = 8;
#ifndef NRMS_USER_WDEPTH
#define NRMS_USER_WDEPTH 4
#endif

// Dispatch order of the users (with compaction): longest compacted length Le
// first, so that the last workgroups dispatched are the short users (LPT:
// one workgroup per user and per CU, 23 k to 61 k cycles per user by Le --
// dispatched in user order, the makespan was set by long users started
// last). One block per 1,024 users: an LDS histogram over Le and a
// descending scan; users of equal Le in any order (a user's result does not
// depend on when its workgroup runs).
constexpr int UORD_T = 1024;
__global__ __launch_bounds__(UORD_T) void user_order_kernel(const uint8_t* __restrict__ pad, int64_t B,
                                                            int L_all, int32_t* __restrict__ order) {
  __shared__ int cnt[65], base[65];
  const int64_t u = (int64_t)blockIdx.x * UORD_T + threadIdx.x;
  if (threadIdx.x < 65) cnt[threadIdx.x] = 0;
  __syncthreads();
  int le = -1;
  if (u < B) {
    const uint8_t* p = pad + u * L_all;
    int npad = 0;
    for (int i = 0; i < L_all; ++i) npad += p[i] ? 1 : 0;
    le = L_all - npad + (npad > 0 ? 1 : 0);
    atomicAdd(&cnt[le], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int l = 64; l >= 0; --l) {
      base[l] = acc;
      acc += cnt[l];
    }
  }
  __syncthreads();
  if (u < B) order[(int64_t)blockIdx.x * UORD_T + atomicAdd(&base[le], 1)] = (int32_t)u;
}

template <int MODE, int LMAX, int NT, int KVR = LMAX>
#ifndef NRMS_USER_CHUNK_MINWAVES
#define NRMS_USER_CHUNK_MINWAVES 4
#endif
__global__ __launch_bounds__(NT, (KVR < LMAX) ? NRMS_USER_CHUNK_MINWAVES : 1) void fused_user_kernel(
    const float* __restrict__ qkv, int64_t ldq, int L_all, const float* __restrict__ WaP,
    const float* __restrict__ b_add, const float* __restrict__ q_add, float* __restrict__ out,
    PaddingGroups pg, int uflags, const int32_t* __restrict__ order, ScoreFold sf) {
  constexpr bool CHUNKED = KVR < LMAX;   // (see the attention below)
  static_assert(CHUNKED || NT >= UH * LMAX, "one (head, query) task per thread");
  static_assert(!CHUNKED || MODE == 2, "the chunked instance is split-f16 only");
  constexpr int NW = NT / 64;
  constexpr int NTPW = (UNT + NW - 1) / NW;            // N-tiles per wave
  constexpr int MT = (LMAX + 15) / 16;                 // M-tiles
  extern __shared__ __attribute__((aligned(16))) float ulds[];
  // Wave priority: 2, except 0 in the additive GEMM (below). Two workgroups
  // share a CU; a GEMM wave waits on its W fragments from L2 between MFMA
  // groups and gives the issue slots to the other workgroup's staging /
  // attention / pooling waves (user_fused -1.3 %, faster 6/6 same-box;
  // priority to the GEMM instead: -1.7 %, 3/3; over the attention alone:
  // -1.0 %; over the softmax / pooling / scores alone: nothing;
  // profiles/r5/r5zm_setprio_ab.txt, r5zn_user_setprio_ab.txt)
  __builtin_amdgcn_s_setprio(2);
#ifdef NRMS_USER_TIMING   // probe build (profiles/probes/user_phases.py): phase cycles of wave 0
  unsigned long long ut[8] = {0, 0, 0, 0, 0, 0, 0, 0}, uprev = __builtin_amdgcn_s_memtime();
#define NRMS_U_STAMP(k)                                           \
  {                                                               \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    ut[k] = now_ - uprev;                                         \
    uprev = now_;                                                 \
  }
#else
#define NRMS_U_STAMP(k)
#endif
  float* tile = ulds;                                  // [KVR][URS]
  float* part = tile + KVR * URS;                      // [UNT][64]
  float* wts = part + UNT * 64;                        // [64]
  // MODE 2: part | wts | [64] hold one max |ctx| per (head, query) thread
  // until the split; then [64] row exponents ea
  int32_t* rexp = reinterpret_cast<int32_t*>(wts + 128);
  const int64_t s = order ? (int64_t)order[blockIdx.x] : (int64_t)blockIdx.x;   // (user_order_kernel)
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // q|k|v row of position i (stride ldq floats); with pg, a position holding a
  // copied padding title reads the row of the title it copies
  const int32_t rep = (pg.pad_title && pg.rep) ? *pg.rep : 0;   // (no rep: the padded stage entry)
  const bool compact = (uflags & UF_COMPACT) != 0;
  __shared__ int32_t urow[LMAX + 1];   // compacted rows, then n_pad
  int L = L_all, m0 = 1;               // rows of this user; times row 0 counts
  if (compact) {
    static_assert(LMAX <= 64, "one lane per history position");
    if (w == 0) {
      const int64_t base = s * L_all;
      const bool padp = lane < L_all && pg.pad_title[base + lane];
      const uint64_t pm = __ballot(padp);
      const uint64_t real = __ballot(lane < L_all && !padp);
      const int npad = __popcll(pm);
      const int lead = npad > 0 ? 1 : 0;
      if (lane < L_all && !padp) urow[lead + __popcll(real & ((1ull << lane) - 1))] = (int32_t)(base + lane);
      if (lane == 0) {
        if (npad) urow[0] = (uflags & UF_COPIED) ? rep : (int32_t)(base + __ffsll((long long)pm) - 1);
        urow[LMAX] = npad;
      }
    }
    __syncthreads();
    const int npad = urow[LMAX];
    L = L_all - npad + (npad > 0 ? 1 : 0);
    m0 = npad > 1 ? npad : 1;
  }
  L = __builtin_amdgcn_readfirstlane(L);   // (workgroup-uniform: scalar loop bounds below)
  auto row = [&](int i) -> const float* {
    if (compact) return qkv + (int64_t)urow[i] * ldq;
    int64_t m = s * L + i;
    if (pg.pad_title && pg.pad_title[m] && m != rep) m = rep;
    return qkv + m * ldq;
  };

  // ---------------- 0. stage K|V (all loads in flight at once), q slices ----------------
  // LDS-DMA (global_load_lds_dwordx4): the tile's rows are the K|V rows back
  // to back (2,400 B each), so wave-instruction p fills bytes 1,024 p .. +
  // 1,023 of it, each lane from its own row; lanes past the last row reload
  // its last 16 B into the LDS after the staged rows (unused rows, or part:
  // free until the attention's end). (Register staging: user_fused 2.1 us
  // slower, profiles/r4m_user_staging_gemm_ab.txt)
  auto stage = [&](int r0, int nr) __attribute__((always_inline)) {
    const int nbytes = nr * URS * 4;
    const int npieces = (nbytes + 1023) >> 10;
    for (int p = w; p < npieces; p += NT / 64) {
      int o = (p << 10) + 16 * lane;
      o = o < nbytes ? o : nbytes - 16;
      const int i = o / (URS * 4), wb = o - i * (URS * 4);
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(row(r0 + i) + UD + (wb >> 2)),
                                       (__attribute__((address_space(3))) void*)(tile + (p << 8)), 16, 0, 0);
    }
  };
  // CHUNKED (the 512-thread, 80-KB instance for histories of 33..50 titles,
  // two workgroups per CU): a user whose (head, query) tasks fit the threads
  // (33, 34 titles) stages its K|V rows KVR at a time (the keys in order, each
  // chunk behind a barrier); a user with more tasks than threads (35..50
  // titles) runs them in two passes split by HEAD (round 6): heads 0 .. hs-1,
  // then hs .. 14, each pass staging the K|V columns of its heads for all L
  // keys (rows of 40 hs floats), so every K|V byte is staged once (the
  // round-5 passes split by task index re-staged both key chunks in the
  // second pass: traffic 1.44x its floor) and the first pass's context is
  // kept in registers. hs = 8, 9 or 10, the first that leaves no more partly
  // filled waves than the task-index split (e.g. 50 titles: 10 + 5 heads, 8 + 4
  // waves; 8 + 7 heads would be 7 + 6); none does at 46 titles, which keeps
  // the task-index split. A 10-head tile (80,000 B at 50 keys) runs into the
  // part / wts / rexp slots after the 76.8-KB tile, which are free until the
  // attention's end. Either way each task runs the whole-tile instances'
  // arithmetic over the keys in the same order: bitwise their results.
#ifndef NRMS_USER_HS_MAX
#define NRMS_USER_HS_MAX 10
#endif
  constexpr int HS_MAX = NRMS_USER_HS_MAX;     // most heads of the first pass
  static_assert(!CHUNKED || (HS_MAX * LMAX <= NT && (UH - 8) * LMAX <= NT), "one pass per head group");
  // (the last wave-instruction of a staging fills a whole 1-KB block)
  static_assert(!CHUNKED || ((LMAX * 40 * HS_MAX / 4 + 63) / 64) * 1024 <=
                                (KVR * URS + UNT * 64 + 64 + 2 * 64) * 4, "a head group's K|V fits the LDS");
  const int ntask = UH * L;
  const int npass = CHUNKED ? (ntask + NT - 1) / NT : 1;    // (workgroup-uniform)
  // two queries of one head per thread, one pass over two key chunks (round
  // 6, see the attention below): 15 ceil(L / 2) <= 375 tasks
#ifndef NRMS_USER_PAIR_MIN
#define NRMS_USER_PAIR_MIN 35
#endif
#ifndef NRMS_USER_NO_PAIR_CODE
  const bool pairmode = CHUNKED && (npass > 1 || L >= NRMS_USER_PAIR_MIN) && !(uflags & UF_NO_PAIR);
#else
  const bool pairmode = false;   // (probe builds without the paired path)
#endif
  int hs = 0;                                               // heads of the first pass (0: no head split)
  if (CHUNKED && npass > 1 && !pairmode && !(uflags & UF_TASK_SPLIT)) {
    const int waves_task = NT / 64 + (ntask - NT + 63) / 64;
    for (int c = HS_MAX; c >= 8; --c)
#ifdef NRMS_USER_HS_SKIP9
      if (c != 9)
#endif
      if (c * L <= NT && (c * L + 63) / 64 + ((UH - c) * L + 63) / 64 <= waves_task) hs = c;
  }
  hs = __builtin_amdgcn_readfirstlane(hs);
  const bool hsplit = hs > 0;
  const int nchunk = CHUNKED && !hsplit ? (L + KVR - 1) / KVR : 1;
  const int npair = (L + 1) / 2;                            // (pairmode) query pairs per head
  const int tb = hsplit ? hs * L : NT;                      // the second pass's first task
  // K|V columns of heads hb .. hb + nh - 1 of rows 0 .. nr - 1 (head split):
  // 10 nh 16-B pieces per row (stride 40 nh floats), K's then V's
  auto stage_heads = [&](int hb, int nh, int nr) __attribute__((always_inline)) {
    const int pps = nh * (UDK / 4), ppr = 2 * pps;   // pieces per section / per row
    const int np = nr * ppr;
    for (int p = w; p < (np + 63) >> 6; p += NT / 64) {
      int g = (p << 6) + lane;
      g = g < np ? g : np - 1;
      const int i = g / ppr, c = g - i * ppr;
      const int sec = c >= pps ? 1 : 0, cc = c - sec * pps;
      const float* src = row(i) + (1 + sec) * UD + UDK * hb + 4 * cc;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src),
                                       (__attribute__((address_space(3))) void*)(tile + (p << 8)), 16, 0, 0);
    }
  };
  static_assert(!CHUNKED || UH * LMAX <= 2 * NT, "at most two task passes");
  static_assert(MODE != 2 || UNT * 64 + 64 + 64 >= UH * LMAX, "per-thread max slots before rexp");
  // exp(d / sqrt(d_k)) as v_exp_f32(d · log2(e) / sqrt(d_k)), as the news kernel
  const float rs = 1.4426950408889634f / sqrtf((float)UDK);
  const float sqrt_dk = sqrtf((float)UDK);
  typedef float f2 __attribute__((ext_vector_type(2)));
  float acc[UDK], q[UDK];
  [[maybe_unused]] float acc0[UDK];   // CHUNKED, two passes: the first pass's context
  float mrow = 0.f, mrow0 = 0.f;      // MODE 2: max |ctx| of this thread's task (per pass)
  // ---- pairmode (CHUNKED, 35..50 rows): thread = (head h, queries 2p, 2p + 1)
  // The attention of the long users was bound by the LDS returns of its
  // broadcast K|V reads (160 B per key per (head, query) task at 256 B/clk/CU
  // against ~half that time of VALU work); with two queries per thread each
  // K|V slice read serves both, so the bytes halve, the 15 ceil(L / 2) <= 375
  // tasks fit one pass and the keys are staged once, in two chunks. Each
  // query runs exactly the single-query arithmetic (the same dot product,
  // exp, key order of the sums, four-key groups with weight-0 padding, and
  // recheck path): bitwise the two-pass forms' results.
  [[maybe_unused]] float q1[UDK];
  [[maybe_unused]] float mrow1 = 0.f;
  [[maybe_unused]] const bool phas = pairmode && tid < UH * npair;
  [[maybe_unused]] const int ph = phas ? tid / npair : 0, pq = phas ? 2 * (tid - ph * npair) : 0;
  [[maybe_unused]] const bool phas1 = phas && pq + 1 < L;
  if constexpr (CHUNKED) {
#ifndef NRMS_USER_NO_PAIR_CODE
    if (pairmode) {
      auto loadq = [&](float (&qq)[UDK], int qi) __attribute__((always_inline)) {
        const float4* qp = reinterpret_cast<const float4*>(row(qi) + UDK * ph);
#pragma unroll
        for (int t = 0; t < UDK / 4; ++t) {
          const float4 v = qp[t];
          qq[4 * t] = v.x; qq[4 * t + 1] = v.y; qq[4 * t + 2] = v.z; qq[4 * t + 3] = v.w;
        }
      };
      loadq(q, pq);
      loadq(q1, phas1 ? pq + 1 : pq);
      // both queries' dot products with one K slice read (the single-query
      // form's even / odd partial sums), and both context updates with one V
      auto dot2 = [&](const float* kp, float& da, float& db) __attribute__((always_inline)) {
        const float4* kr = reinterpret_cast<const float4*>(kp);
        f2 a = f2{0.f, 0.f}, b = f2{0.f, 0.f};
#pragma unroll
        for (int t = 0; t < UDK / 4; ++t) {
          const float4 k4 = kr[t];
          a = __builtin_elementwise_fma(f2{q[4 * t], q[4 * t + 1]}, f2{k4.x, k4.y}, a);
          a = __builtin_elementwise_fma(f2{q[4 * t + 2], q[4 * t + 3]}, f2{k4.z, k4.w}, a);
          b = __builtin_elementwise_fma(f2{q1[4 * t], q1[4 * t + 1]}, f2{k4.x, k4.y}, b);
          b = __builtin_elementwise_fma(f2{q1[4 * t + 2], q1[4 * t + 3]}, f2{k4.z, k4.w}, b);
        }
        da = a.x + a.y;
        db = b.x + b.y;
      };
      auto axpy2 = [&](float ea, float eb, const float* vp) __attribute__((always_inline)) {
        const float4* vr = reinterpret_cast<const float4*>(vp);
        const f2 a2 = f2{ea, ea}, b2 = f2{eb, eb};
#pragma unroll
        for (int t = 0; t < UDK / 4; ++t) {
          const float4 v4 = vr[t];
          const f2 lo = __builtin_elementwise_fma(a2, f2{v4.x, v4.y}, f2{acc[4 * t], acc[4 * t + 1]});
          const f2 hi = __builtin_elementwise_fma(a2, f2{v4.z, v4.w}, f2{acc[4 * t + 2], acc[4 * t + 3]});
          acc[4 * t] = lo.x; acc[4 * t + 1] = lo.y; acc[4 * t + 2] = hi.x; acc[4 * t + 3] = hi.y;
          const f2 lo1 = __builtin_elementwise_fma(b2, f2{v4.x, v4.y}, f2{acc0[4 * t], acc0[4 * t + 1]});
          const f2 hi1 = __builtin_elementwise_fma(b2, f2{v4.z, v4.w}, f2{acc0[4 * t + 2], acc0[4 * t + 3]});
          acc0[4 * t] = lo1.x; acc0[4 * t + 1] = lo1.y; acc0[4 * t + 2] = hi1.x; acc0[4 * t + 3] = hi1.y;
        }
      };
#pragma unroll
      for (int t = 0; t < UDK; ++t) { acc[t] = 0.f; acc0[t] = 0.f; }
      float sa = 0.f, sb = 0.f;
      for (int c = 0; c < nchunk; ++c) {
        const int kb = c * KVR, ke = L < kb + KVR ? L : kb + KVR;
        if (c > 0) __syncthreads();   // the previous chunk's readers are done
        stage(kb, ke - kb);
        __syncthreads();
        if (c == 0) { NRMS_U_STAMP(0) }   // K|V staged
        if (phas) {
          const float* kt = tile - (int64_t)kb * URS + UDK * ph;   // key j's K slice: kt + j URS
          // one key per iteration, rolled (the four-key unrolled form of the
          // single-query loop, with weight-0 padding keys: 56 KB of code, 128
          // VGPRs + scratch, user_fused 0.0700 against 0.0676 ms,
          // profiles/r6/r6l_user_pair_ab.txt). Without the padding keys the
          // sums and context updates are the same operations on the same
          // values: a padding key adds 0 to the sum and 0·v to a context that
          // starts at +0 (never -0), and a non-finite v makes the real key's
          // update non-finite too (recheck path) -- bitwise the padded forms.
#pragma unroll 1
          for (int j = kb; j < ke; ++j) {
            float da, db;
            dot2(kt + j * URS, da, db);
            float ea = __builtin_amdgcn_exp2f(da * rs), eb = __builtin_amdgcn_exp2f(db * rs);
            if (j == 0) {
              for (int cc = 0; cc < m0; ++cc) { sa += ea; sb += eb; }   // (row 0's multiplicity)
              ea *= (float)m0;
              eb *= (float)m0;
            } else {
              sa += ea;
              sb += eb;
            }
            axpy2(ea, eb, kt + j * URS + UD);
          }
        }
      }
      if (phas) {
        // normalisation, or (rare) the reference-order recheck, per query
        auto finish = [&](const float (&qq)[UDK], float (&aa)[UDK], float sum) __attribute__((always_inline)) {
          bool finite = true;
#pragma unroll
          for (int t = 0; t < UDK; ++t) finite &= __builtin_isfinite(aa[t]);
          if (!exp_row_needs_recheck(sum) && finite) {
            const float inv = 1.0f / (sum + 1e-8f);
#pragma unroll
            for (int t = 0; t < UDK; ++t) aa[t] *= inv;
          } else {
            auto dotq = [&](const float* kp) __attribute__((always_inline)) {
              const float4* kr = reinterpret_cast<const float4*>(kp);
              f2 d = f2{0.f, 0.f};
#pragma unroll
              for (int t = 0; t < UDK / 4; ++t) {
                const float4 k4 = kr[t];
                d = __builtin_elementwise_fma(f2{qq[4 * t], qq[4 * t + 1]}, f2{k4.x, k4.y}, d);
                d = __builtin_elementwise_fma(f2{qq[4 * t + 2], qq[4 * t + 3]}, f2{k4.z, k4.w}, d);
              }
              return d.x + d.y;
            };
            float s2 = 0.f;
            for (int j = 0; j < L; ++j) {
              const float x = ref_exp(dotq(row(j) + UD + UDK * ph), sqrt_dk);
              if (j == 0)
                for (int cc = 0; cc < m0; ++cc) s2 += x;
              else
                s2 += x;
            }
            const float inv = 1.0f / (s2 + 1e-8f);
#pragma unroll
            for (int t = 0; t < UDK; ++t) aa[t] = 0.f;
            for (int j = 0; j < L; ++j) {
              float a = ref_exp(dotq(row(j) + UD + UDK * ph), sqrt_dk) * inv;
              if (j == 0 && m0 > 1) a *= (float)m0;
              const float4* vr = reinterpret_cast<const float4*>(row(j) + 2 * UD + UDK * ph);
              const f2 a2 = f2{a, a};
#pragma unroll
              for (int t = 0; t < UDK / 4; ++t) {
                const float4 v4 = vr[t];
                const f2 lo = __builtin_elementwise_fma(a2, f2{v4.x, v4.y}, f2{aa[4 * t], aa[4 * t + 1]});
                const f2 hi = __builtin_elementwise_fma(a2, f2{v4.z, v4.w}, f2{aa[4 * t + 2], aa[4 * t + 3]});
                aa[4 * t] = lo.x; aa[4 * t + 1] = lo.y; aa[4 * t + 2] = hi.x; aa[4 * t + 3] = hi.y;
              }
            }
          }
          float m = 0.f;
#pragma unroll
          for (int t = 0; t < UDK; ++t) m = fmaxf(m, fabsf(aa[t]));
          return m;
        };
        mrow = finish(q, acc, sa);
        mrow1 = finish(q1, acc0, sb);
      }
    }
#endif
  }
  for (int pass = 0; pass < (pairmode ? 0 : npass); ++pass) {
    const int task = tb * pass + tid;
    const bool has = task < ntask && (!hsplit || pass > 0 || tid < tb);
    const int h = has ? task / L : 0, qi = has ? task - h * L : 0;
    // head h's K and V slices within a staged row (stride krs floats)
    // (head split: this pass's heads h0 .. h0 + nh - 1, rows of 40 nh floats)
    const int h0 = hs * pass, nh = pass == 0 ? hs : UH - hs;
    const int krs = hsplit ? 2 * UDK * nh : URS;
    const int kofs = hsplit ? UDK * (h - h0) : UDK * h;
    const int vofs = hsplit ? UDK * nh + UDK * (h - h0) : UD + UDK * h;
    {
      const float4* qp = reinterpret_cast<const float4*>(row(qi) + UDK * h);
#pragma unroll
      for (int t = 0; t < UDK / 4; ++t) {
        const float4 v = qp[t];
        q[4 * t] = v.x; q[4 * t + 1] = v.y; q[4 * t + 2] = v.z; q[4 * t + 3] = v.w;
      }
    }
    // packed FP32 (v_pk_fma_f32, two FMAs per lane per instruction): the dot
    // product as even / odd partial sums added at the end, the context update
    // elementwise (the same FMAs as the scalar form): user_fused -1.3 us
    // (profiles/r4o_user_pk_fma_ab.txt). kp / vp: head h's K / V slice of a key.
    auto dot = [&](const float* kp) __attribute__((always_inline)) {
      const float4* kr = reinterpret_cast<const float4*>(kp);
      f2 d = f2{0.f, 0.f};
#pragma unroll
      for (int t = 0; t < UDK / 4; ++t) {
        const float4 k4 = kr[t];
        d = __builtin_elementwise_fma(f2{q[4 * t], q[4 * t + 1]}, f2{k4.x, k4.y}, d);
        d = __builtin_elementwise_fma(f2{q[4 * t + 2], q[4 * t + 3]}, f2{k4.z, k4.w}, d);
      }
      return d.x + d.y;
    };
    auto axpy = [&](float a, const float* vp) __attribute__((always_inline)) {
      const float4* vr = reinterpret_cast<const float4*>(vp);
      const f2 a2 = f2{a, a};
#pragma unroll
      for (int t = 0; t < UDK / 4; ++t) {
        const float4 v4 = vr[t];
        const f2 lo = __builtin_elementwise_fma(a2, f2{v4.x, v4.y}, f2{acc[4 * t], acc[4 * t + 1]});
        const f2 hi = __builtin_elementwise_fma(a2, f2{v4.z, v4.w}, f2{acc[4 * t + 2], acc[4 * t + 3]});
        acc[4 * t] = lo.x; acc[4 * t + 1] = lo.y; acc[4 * t + 2] = hi.x; acc[4 * t + 3] = hi.y;
      }
    };
#pragma unroll
    for (int t = 0; t < UDK; ++t) acc[t] = 0.f;
    // Fast path, one pass over the user's L keys (a rolled loop, four keys per
    // iteration: their dot products interleave; keys past the staged rows in
    // the last iteration read the last one with weight 0): sum = the raw exps
    // in the reference's key order (row 0 counted m0 times, one addition at a
    // time), acc = sum_j e_j v_j, ctx = acc / (sum + 1e-8). Only the
    // normalisation moves (after the sum instead of per weight: fp32
    // rounding). No exp is kept, so the work is ~L, not LMAX, keys per query.
    float sum = 0.f;
    for (int c = 0; c < nchunk; ++c) {
      const int kb = c * KVR, ke = CHUNKED && !hsplit ? (L < kb + KVR ? L : kb + KVR) : L;
      if (CHUNKED && (pass > 0 || c > 0)) __syncthreads();   // the previous chunk's readers are done
      if (hsplit) stage_heads(h0, nh, L);
      else stage(kb, ke - kb);
      __syncthreads();
      if (c == 0 && pass == 0) { NRMS_U_STAMP(0) }   // K|V staged
      if (has) {
        const float* kt = tile - (int64_t)kb * krs;   // key j's staged row: kt + j krs
        for (int j0 = kb; j0 < ke; j0 += 4) {
          float e[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int j = j0 + u;
            e[u] = j < ke ? __builtin_amdgcn_exp2f(dot(kt + (j < ke ? j : ke - 1) * krs + kofs) * rs) : 0.f;
          }
          if (j0 == 0) {
            for (int cc = 0; cc < m0; ++cc) sum += e[0];   // (row 0's multiplicity)
            e[0] *= (float)m0;
          } else {
            sum += e[0];
          }
          sum += e[1];
          sum += e[2];
          sum += e[3];
#pragma unroll
          for (int u = 0; u < 4; ++u) axpy(e[u], kt + (j0 + u < ke ? j0 + u : ke - 1) * krs + vofs);
        }
      }
    }
    if (has) {
      bool finite = true;
#pragma unroll
      for (int t = 0; t < UDK; ++t) finite &= __builtin_isfinite(acc[t]);
      if (!exp_row_needs_recheck(sum) && finite) {
        const float inv = 1.0f / (sum + 1e-8f);
#pragma unroll
        for (int t = 0; t < UDK; ++t) acc[t] *= inv;
      } else {
        // rare (rows near fp32 overflow, non-finite inputs, or a context past
        // fp32 before the normalisation): the reference's own arithmetic and
        // order -- ref_exp weights, e_j / (sum + 1e-8) per key, then sum_j P_j v_j
        // (kExpRecheck); the exps are recomputed in the second pass. The K|V
        // rows from the tile, or (CHUNKED: only the last chunk is staged) from
        // the projected rows themselves.
        auto kvr = [&](int j) -> const float* { return CHUNKED ? row(j) + UD : tile + j * URS; };
        sum = 0.f;
        for (int j = 0; j < L; ++j) {
          const float x = ref_exp(dot(kvr(j) + UDK * h), sqrt_dk);
          if (j == 0)
            for (int cc = 0; cc < m0; ++cc) sum += x;
          else
            sum += x;
        }
        const float inv = 1.0f / (sum + 1e-8f);
#pragma unroll
        for (int t = 0; t < UDK; ++t) acc[t] = 0.f;
        for (int j = 0; j < L; ++j) {
          float a = ref_exp(dot(kvr(j) + UDK * h), sqrt_dk) * inv;
          if (j == 0 && m0 > 1) a *= (float)m0;
          axpy(a, kvr(j) + UD + UDK * h);
        }
      }
      if constexpr (MODE == 2) {
        float m = 0.f;
#pragma unroll
        for (int t = 0; t < UDK; ++t) m = fmaxf(m, fabsf(acc[t]));
        mrow = m;
        // (one slot per (head, query) task in part | wts | rmax; the row max
        // after the barrier; CHUNKED: written after the last chunk's readers,
        // as a later chunk's staging may run past the tile into part)
        if constexpr (!CHUNKED) part[task] = m;
      }
    }
    if constexpr (CHUNKED) {
      if (pass == 0 && npass > 1) {
#pragma unroll
        for (int t = 0; t < UDK; ++t) acc0[t] = acc[t];
        mrow0 = mrow;
      }
    }
  }
  __syncthreads();   // every K|V read done: the tile becomes the context
  NRMS_U_STAMP(1)   // attention
  // the context's row stride in halves (and its planes): the whole-tile
  // instances keep each row at its K|V row (2,400 B, three planes);
  // CHUNKED packs them (1,952 B, three planes; past 39 rows 1,312 B and two
  // planes, hi | lo: the pooling then rebuilds the context from those two,
  // 22 bits, as the GEMM reads it). Both strides conflict-free for the GEMM's
  // fragment reads.
  const bool three = !CHUNKED || L * 1952 <= KVR * URS * 4;
  const int cs = !CHUNKED ? 2 * URS : (three ? 976 : 656);
  const int npl = three ? 3 : 2;
  const int h = tid < ntask ? tid / L : 0, qi = tid < ntask ? tid - h * L : 0;   // (the first pass's task)
  const bool has = tid < ntask;
  if constexpr (MODE == 2) {
    // (CHUNKED: the first pass's tasks are 0 .. tb - 1, the second pass's tb ..)
    [[maybe_unused]] const bool has0 = hsplit ? tid < tb : tid < ntask;
    [[maybe_unused]] const bool has1 = npass > 1 && tb + tid < ntask;
    if constexpr (CHUNKED) {
      if (pairmode) {
        if (phas) part[ph * L + pq] = mrow;
        if (phas1) part[ph * L + pq + 1] = mrow1;
      } else {
        if (has0) part[tid] = npass > 1 ? mrow0 : mrow;
        if (has1) part[tb + tid] = mrow;
      }
      __syncthreads();
    }
    // three fp16 planes per row (hi | lo | r), in the MODE 1 positions
    _Float16* t16 = reinterpret_cast<_Float16*>(tile);
    auto write_ctx = [&](int task, const float (&a)[UDK]) __attribute__((always_inline)) {
      const int th = task / L, tq = task - th * L;
      float mx = 0.f;
      for (int hh = 0; hh < UH; ++hh) mx = fmaxf(mx, part[hh * L + tq]);   // the row's 15 head tasks
      const int ea = pk::exp_field(mx) - 3;
      if (th == 0) rexp[tq] = ea;
#pragma unroll
      for (int g = 0; g < UDK / 4; ++g) {
        _Float16 hv[3][4];
#pragma unroll
        for (int x = 0; x < 4; ++x) {
          const float v = ldexpf(a[4 * g + x], -ea);
          hv[0][x] = (_Float16)v;
          const float r1 = (v - (float)hv[0][x]) * kF16LoScale;   // exact
          hv[1][x] = (_Float16)r1;
          hv[2][x] = (_Float16)(r1 - (float)hv[1][x]);
        }
        const int pos = tq * cs + ukpos(UDK * th + 4 * g);
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          if (pl < npl) *reinterpret_cast<uf16x4*>(t16 + pos + UKP * pl) = uf16x4{hv[pl][0], hv[pl][1], hv[pl][2], hv[pl][3]};
      }
    };
    if constexpr (CHUNKED) {
      if (pairmode) {
        if (phas) write_ctx(ph * L + pq, acc);
        if (phas1) write_ctx(ph * L + pq + 1, acc0);
      } else if (npass > 1) {
        if (has0) write_ctx(tid, acc0);
        if (has1) write_ctx(tb + tid, acc);
      } else if (has) {
        write_ctx(tid, acc);
      }
    } else if (has) {
      write_ctx(tid, acc);
    }
    uint16_t* z16 = reinterpret_cast<uint16_t*>(tile);
    for (int e = tid; e < L * 15; e += NT) {   // K padding 300..319, each plane
      const int i = e / 15, g = (e % 15) % 5, pl = (e % 15) / 5;
      if (pl < npl) *reinterpret_cast<uint2*>(z16 + i * cs + UKP * pl + ukpos(UD + 4 * g)) = make_uint2(0u, 0u);
    }
  } else if constexpr (MODE == 1) {
    // three bf16 planes per row (plane p at bf16 offset 320 p), k permuted to
    // the MFMA fragment order: lane (lm, kq) of k-step ks reads 16 contiguous
    // bytes per plane (see ukpos)
    uint16_t* t16 = reinterpret_cast<uint16_t*>(tile);
    if (has) {
#pragma unroll
      for (int g = 0; g < UDK / 4; ++g) {
        uint32_t hv[3][2];
#pragma unroll
        for (int x = 0; x < 2; ++x)
          split3x2(acc[4 * g + 2 * x], acc[4 * g + 2 * x + 1], hv[0][x], hv[1][x], hv[2][x]);
        const int pos = qi * (2 * URS) + ukpos(UDK * h + 4 * g);
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          *reinterpret_cast<uint2*>(t16 + pos + UKP * pl) = make_uint2(hv[pl][0], hv[pl][1]);
      }
    }
    for (int e = tid; e < L * 15; e += NT) {   // K padding 300..319, each plane
      const int i = e / 15, g = (e % 15) % 5, pl = (e % 15) / 5;
      *reinterpret_cast<uint2*>(t16 + i * (2 * URS) + UKP * pl + ukpos(UD + 4 * g)) = make_uint2(0u, 0u);
    }
  } else {
    if (has) {
      float4* dst = reinterpret_cast<float4*>(tile + qi * URS + UDK * h);
#pragma unroll
      for (int t = 0; t < UDK / 4; ++t)
        dst[t] = make_float4(acc[4 * t], acc[4 * t + 1], acc[4 * t + 2], acc[4 * t + 3]);
    }
    for (int e = tid; e < L * 5; e += NT)   // K padding 300..319
      *reinterpret_cast<float4*>(tile + (e / 5) * URS + UD + 4 * (e % 5)) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  NRMS_U_STAMP(2)   // context split + stores

  // ---------------- 2. additive GEMM + tanh·q row partials ----------------
  // M-tiles past row L - 1 are skipped: one copy of the GEMM per live M-tile
  // count MTE = ceil(L / 16) (rows L.. of the last tile read row L - 1 and are dropped)
  auto gemm = [&](auto mtc) {
    constexpr int MT = decltype(mtc)::value;
    const int lm = lane & 15, kq = lane >> 4;
    float qv[NTPW], bv[NTPW];
    [[maybe_unused]] int ewv[NTPW];   // MODE 2: column exponents
#pragma unroll
    for (int j = 0; j < NTPW; ++j) {
      const int nt = w + NW * j;
      const int col = 16 * nt + lm;
      const bool ok = nt < UNT && col < UQ;
      qv[j] = ok ? q_add[col] : 0.f;
      bv[j] = ok ? b_add[col] : 0.f;
      if constexpr (MODE == 2) ewv[j] = nt < UNT ? reinterpret_cast<const int32_t*>(WaP)[pk::USER_H3_EXP + col] : 0;
    }
    int arow[MT], arow16[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int r = 16 * mt + lm;
      arow[mt] = (r < L ? r : L - 1) * URS;
      arow16[mt] = (r < L ? r : L - 1) * cs;   // (MODE 2: the context's stride in halves)
    }
    floatx4 c[MT][NTPW];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < NTPW; ++j) c[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};

    if constexpr (MODE == 2) {
      const uf16x8* Bq = reinterpret_cast<const uf16x8*>(WaP) + lane;
      const _Float16* t16 = reinterpret_cast<const _Float16*>(tile);
      // W fragments PD k-steps in flight (an L2 round trip per k-step was the
      // phase's latency: 6.7 k cycles even for one M-tile; one k-step ahead
      // covers one group of MFMAs, so the fewer M-tiles, the deeper: PD = 4
      // up to two M-tiles, in the registers the larger tiles' accumulators
      // and A fragments take)
      // (profiles/r5/r5zf_user_wdepth_ab.txt: user_fused -0.7 us; three k-steps
      // for three or four M-tiles took 142 VGPRs, past two workgroups per CU)
      constexpr int PD = MT <= 2 ? NRMS_USER_WDEPTH : 2;
      uf16x8 bq[PD][NTPW][2];
      auto load_bk = [&](int ks, uf16x8 (&dst)[NTPW][2]) __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < NTPW; ++j) {
          const int nt = w + NW * j < UNT ? w + NW * j : UNT - 1;   // (tiles past N: not used)
#pragma unroll
          for (int pl = 0; pl < 2; ++pl) dst[j][pl] = Bq[((ks * UNT + nt) * 2 + pl) * 64];
        }
      };
#pragma unroll
      for (int p = 0; p < PD - 1; ++p) load_bk(p, bq[p]);
#pragma unroll
      for (int ks = 0; ks < UKS; ++ks) {
        if (ks + PD - 1 < UKS) load_bk(ks + PD - 1, bq[(ks + PD - 1) % PD]);
        const uf16x8 (&bc)[NTPW][2] = bq[ks % PD];
        uf16x8 a[MT][2];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int pl = 0; pl < 2; ++pl)
            a[mt][pl] = *reinterpret_cast<const uf16x8*>(t16 + arow16[mt] + UKP * pl + 32 * ks + 8 * kq);
#pragma unroll
        for (int j = 0; j < NTPW; ++j) {
          const int nt = w + NW * j;
          if (nt >= UNT) break;
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
            c[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[mt][0], bc[j][1], c[mt][j], 0, 0, 0);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
            c[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[mt][1], bc[j][0], c[mt][j], 0, 0, 0);
#pragma unroll
          for (int mt = 0; mt < MT; ++mt)
            c[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[mt][0] * (_Float16)kF16LoScale, bc[j][0], c[mt][j],
                                                                0, 0, 0);
        }
      }
    } else if constexpr (MODE == 1) {
      const bf16x8* Bq = reinterpret_cast<const bf16x8*>(WaP) + lane;
      const uint16_t* t16 = reinterpret_cast<const uint16_t*>(tile);
      for (int ks = 0; ks < UKS; ++ks) {
        bf16x8 a[MT][3];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int pl = 0; pl < 3; ++pl)
            a[mt][pl] = *reinterpret_cast<const bf16x8*>(t16 + 2 * arow[mt] + UKP * pl + 32 * ks + 8 * kq);
#pragma unroll
        for (int j = 0; j < NTPW; ++j) {
          const int nt = w + NW * j;
          if (nt >= UNT) break;
          bf16x8 b[3];
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) b[pl] = Bq[((ks * UNT + nt) * 3 + pl) * 64];
#define NRMS_UX6(PA, PB)                                                                            \
  _Pragma("unroll") for (int mt = 0; mt < MT; ++mt)                                                 \
      c[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt][PA], b[PB], c[mt][j], 0, 0, 0);
          NRMS_UX6(2, 0) NRMS_UX6(1, 1) NRMS_UX6(0, 2) NRMS_UX6(1, 0) NRMS_UX6(0, 1) NRMS_UX6(0, 0)
#undef NRMS_UX6
        }
      }
    } else {
      const float4* Bp = reinterpret_cast<const float4*>(WaP) + lane;
      for (int cg = 0; cg < UKG; ++cg) {
        float4 a[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
          a[mt] = *reinterpret_cast<const float4*>(tile + arow[mt] + 16 * cg + 4 * kq);
#pragma unroll
        for (int j = 0; j < NTPW; ++j) {
          const int nt = w + NW * j;
          if (nt >= UNT) break;
          const float4 b = Bp[(cg * UNT + nt) * 64];
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            c[mt][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt].x, b.x, c[mt][j], 0, 0, 0);
            c[mt][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt].y, b.y, c[mt][j], 0, 0, 0);
            c[mt][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt].z, b.z, c[mt][j], 0, 0, 0);
            c[mt][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt].w, b.w, c[mt][j], 0, 0, 0);
          }
        }
      }
    }
    // C/D layout: col = lane & 15, row = 4 (lane >> 4) + reg; one partial row per N-tile
#pragma unroll
    for (int j = 0; j < NTPW; ++j) {
      const int nt = w + NW * j;
      if (nt >= UNT) break;
      // q tanh(y + b) = q - 2q / (e^(2(y + b)) + 1): v_exp_f32 + v_rcp_f32
      // (absolute error ~1e-7, as the news kernel's epilogue; saturates,
      // propagates NaN); the four rows' DPP sums stage by stage
      constexpr float kC2 = 2.8853900817779268f;   // 2 log2(e)
      const float cb = kC2 * bv[j], m2q = -2.0f * qv[j];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        float p[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float y = c[mt][j][r];
          if constexpr (MODE == 2) {
            const int row = 16 * mt + 4 * kq + r;
            y = ldexpf(y, rexp[row < L ? row : L - 1] + ewv[j] - 11);
          }
          p[r] = fmaf(m2q, __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(fmaf(y, kC2, cb)) + 1.0f), qv[j]);
        }
#define NRMS_UDPP4(CTRL)                                                                                  \
  _Pragma("unroll") for (int r = 0; r < 4; ++r) p[r] += __builtin_bit_cast(                              \
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, p[r]), CTRL, 0xF, 0xF, false));
        NRMS_UDPP4(0xB1) NRMS_UDPP4(0x4E) NRMS_UDPP4(0x141) NRMS_UDPP4(0x140)
#undef NRMS_UDPP4
        if (lm == 0)
#pragma unroll
          for (int r = 0; r < 4; ++r) part[nt * 64 + 16 * mt + 4 * kq + r] = p[r];
      }
    }
  };
  __builtin_amdgcn_s_setprio(0);
  if (w < UNT) {
    const int mte = (L + 15) / 16;
    if (mte <= 1) gemm(std::integral_constant<int, 1>{});
    else if (mte == 2) gemm(std::integral_constant<int, 2 < MT ? 2 : MT>{});
    else if (mte == 3) gemm(std::integral_constant<int, 3 < MT ? 3 : MT>{});
    else gemm(std::integral_constant<int, MT>{});
  }
  __builtin_amdgcn_s_setprio(2);
  __syncthreads();
  NRMS_U_STAMP(3)   // additive GEMM + tanh·q

  // ---------------- 3. softmax over the L rows + pooling ----------------
  if (w == 0) {
    float v = -INFINITY;
    if (lane < L) {
      v = part[lane];
#pragma unroll
      for (int nt = 1; nt < UNT; ++nt) v += part[nt * 64 + lane];
    }
    const float mx = wave_max_nan(v);
    float ex = lane < L ? expf(v - mx) : 0.f;
    if (lane == 0 && m0 > 1) ex *= (float)m0;
    wts[lane] = ex / wave_sum(ex);
  }
  __syncthreads();
  NRMS_U_STAMP(4)   // softmax
  // click scores (ScoreFold): wave c < C loads candidate c's vector now, under
  // the pooling (lane i holds float4 columns i and i + 64, the score kernel's)
  const bool scoring = sf.news != nullptr;
  auto cand_vec = [&](int c) -> const float4* {
    const int64_t pair = s * sf.C + c;
    const float* nv = sf.news + pair * UD;
    if (sf.pg.pad_title) {
      const int64_t t = sf.title0 + pair, r = *sf.pg.rep;
      if (sf.pg.pad_title[t] && t != r) nv = sf.news + (r - sf.title0) * UD;
    }
    return reinterpret_cast<const float4*>(nv);
  };
  float4 cn[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
  if (scoring && w < sf.C) {
    const float4* n4 = cand_vec(w);
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (lane + 64 * k < UD / 4) cn[k] = n4[lane + 64 * k];
  }
  // PP lanes per float4 column (rows i = par mod PP each), combined by lane
  // shuffles: 8 per column (600 lanes) when the workgroup has them
  constexpr int PP = NT >= 8 * (UD / 4) ? 8 : (NT >= 4 * (UD / 4) ? 4 : 2);
  constexpr int PT = (PP * (UD / 4) + 63) / 64 * 64;
  if (tid < PT) {
    const int u = tid / PP, par = tid % PP;
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    if (u < UD / 4) {
      for (int i = par; i < L; i += PP) {
        const float wi = wts[i];
        float4 cv;
        if constexpr (MODE == 2) {   // ldexp(hi + 2^-11 (lo + r), ea): the fp32 context (see MODE 2)
          const _Float16* t16 = reinterpret_cast<const _Float16*>(tile) + i * cs + ukpos(4 * u);
          const uf16x4 p0 = *reinterpret_cast<const uf16x4*>(t16);
          const uf16x4 p1 = *reinterpret_cast<const uf16x4*>(t16 + UKP);
          const uf16x4 p2 = three ? *reinterpret_cast<const uf16x4*>(t16 + 2 * UKP) : uf16x4{0, 0, 0, 0};
          const int ea = rexp[i];
          cv.x = ldexpf((float)p0[0] + ((float)p1[0] + (float)p2[0]) * kF16LoUnscale, ea);
          cv.y = ldexpf((float)p0[1] + ((float)p1[1] + (float)p2[1]) * kF16LoUnscale, ea);
          cv.z = ldexpf((float)p0[2] + ((float)p1[2] + (float)p2[2]) * kF16LoUnscale, ea);
          cv.w = ldexpf((float)p0[3] + ((float)p1[3] + (float)p2[3]) * kF16LoUnscale, ea);
        } else if constexpr (MODE == 1) {   // hi + mid + lo == the fp32 context exactly
          const uint16_t* t16 = reinterpret_cast<const uint16_t*>(tile) + i * (2 * URS) + ukpos(4 * u);
          const uint2 p0 = *reinterpret_cast<const uint2*>(t16);
          const uint2 p1 = *reinterpret_cast<const uint2*>(t16 + UKP);
          const uint2 p2 = *reinterpret_cast<const uint2*>(t16 + 2 * UKP);
          auto f = [](uint32_t wd, int hi) { return __uint_as_float(hi ? (wd & 0xffff0000u) : (wd << 16)); };
          cv.x = (f(p0.x, 0) + f(p1.x, 0)) + f(p2.x, 0);
          cv.y = (f(p0.x, 1) + f(p1.x, 1)) + f(p2.x, 1);
          cv.z = (f(p0.y, 0) + f(p1.y, 0)) + f(p2.y, 0);
          cv.w = (f(p0.y, 1) + f(p1.y, 1)) + f(p2.y, 1);
        } else {
          cv = *reinterpret_cast<const float4*>(tile + i * URS + 4 * u);
        }
        o.x = fmaf(wi, cv.x, o.x);
        o.y = fmaf(wi, cv.y, o.y);
        o.z = fmaf(wi, cv.z, o.z);
        o.w = fmaf(wi, cv.w, o.w);
      }
    }
#pragma unroll
    for (int m = 1; m < PP; m <<= 1) {
      o.x += __shfl_xor(o.x, m);
      o.y += __shfl_xor(o.y, m);
      o.z += __shfl_xor(o.z, m);
      o.w += __shfl_xor(o.w, m);
    }
    if (u < UD / 4 && par == 0) {
      reinterpret_cast<float4*>(out + s * UD)[u] = o;
      if (scoring) reinterpret_cast<float4*>(part)[u] = o;   // (part is free after the softmax)
    }
  }
  if (scoring) {
    __syncthreads();
    const float4* u4 = reinterpret_cast<const float4*>(part);
    for (int c = w; c < sf.C; c += NW) {   // (uniform per wave)
      if (c != w) {
        const float4* n4 = cand_vec(c);
#pragma unroll
        for (int k = 0; k < 2; ++k)
          if (lane + 64 * k < UD / 4) cn[k] = n4[lane + 64 * k];
      }
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if (lane + 64 * k < UD / 4) {
          const float4 a = cn[k], uu = u4[lane + 64 * k];
          acc = fmaf(a.x, uu.x, acc);
          acc = fmaf(a.y, uu.y, acc);
          acc = fmaf(a.z, uu.z, acc);
          acc = fmaf(a.w, uu.w, acc);
        }
      }
      acc = wave_sum(acc);
      if (lane == 0) sf.logits[s * sf.C + c] = acc;
    }
  }
#ifdef NRMS_USER_TIMING
  NRMS_U_STAMP(5)   // pooling
  if (tid == 0) {
    unsigned long long* dbg = reinterpret_cast<unsigned long long*>(const_cast<float*>(WaP) + UWAP_MAX);
    for (int k = 0; k < 8; ++k) dbg[s * 8 + k] = ut[k];
  }
#endif
}

template <int MODE, int LMAX, int NT, int KVR = LMAX>
int32_t launch_user_inst(const float* qkv, int64_t ldq, int64_t B, int L, const float* wap,
                         const float* b_add, const float* q_add, float* out, hipStream_t s,
                         PaddingGroups pg, int uflags, const int32_t* order, const ScoreFold& sf) {
  const size_t lds = ((size_t)KVR * URS + UNT * 64 + 64 + 2 * 64) * 4;
  ensure_dynamic_lds(reinterpret_cast<const void*>(&fused_user_kernel<MODE, LMAX, NT, KVR>), (int)lds);
  hipLaunchKernelGGL((fused_user_kernel<MODE, LMAX, NT, KVR>), dim3((unsigned)B), dim3(NT), lds, s, qkv,
                     ldq, L, wap, b_add, q_add, out, pg, uflags, order, sf);
  return launch_status();
}

static std::atomic<int> g_user_chunk{[] {
  const char* e = env_knob("NRMS_USER_CHUNK");
  return (e && e[0] == '0') ? 0 : 1;
}()};

// (measurement only) NRMS_USER_LMAX=n: take the instance of the smallest LMAX >= max(L, n)
static const int g_user_lmax_min = [] {
  const char* e = env_knob("NRMS_USER_LMAX");
  return e ? atoi(e) : 0;
}();

template <int MODE>
int32_t launch_user_mode(const float* qkv, int64_t ldq, int64_t B, int L, const float* wap,
                         const float* b_add, const float* q_add, float* out, hipStream_t s,
                         PaddingGroups pg, int uflags, const int32_t* order, const ScoreFold& sf) {
  const int Li = L > g_user_lmax_min ? L : g_user_lmax_min;
  // 33..50-title histories, split-f16: 512 threads and 80 KB of LDS (K|V
  // staged 32 rows at a time), so two workgroups share a CU
  // (NRMS_USER_CHUNK=0: the 832-thread whole-tile instance)
  if constexpr (MODE == 2)
    if (Li > 32 && Li <= 50 && g_user_chunk.load(std::memory_order_relaxed))
      return launch_user_inst<MODE, 50, 512, 32>(qkv, ldq, B, L, wap, b_add, q_add, out, s, pg, uflags, order, sf);
  if (Li <= 16) return launch_user_inst<MODE, 16, 256>(qkv, ldq, B, L, wap, b_add, q_add, out, s, pg, uflags, order, sf);
  if (Li <= 32) return launch_user_inst<MODE, 32, 512>(qkv, ldq, B, L, wap, b_add, q_add, out, s, pg, uflags, order, sf);
  if (Li <= 50) return launch_user_inst<MODE, 50, 832>(qkv, ldq, B, L, wap, b_add, q_add, out, s, pg, uflags, order, sf);
  return launch_user_inst<MODE, 64, 1024>(qkv, ldq, B, L, wap, b_add, q_add, out, s, pg, uflags, order, sf);
}

}  // namespace

size_t fused_user_packed_b_floats() { return (size_t)UWAP_MAX + USTAMP_FLOATS; }

static std::atomic<int> g_user_pair{[] {
  const char* e = env_knob("NRMS_USER_PAIR");
  return (e && e[0] == '0') ? 0 : 1;
}()};

static std::atomic<int> g_user_hsplit{[] {
  const char* e = env_knob("NRMS_USER_HSPLIT");
  return (e && e[0] == '0') ? 0 : 1;
}()};

static std::atomic<int> g_user_lpt{[] {
  const char* e = env_knob("NRMS_USER_LPT");
  return (e && e[0] == '0') ? 0 : 1;
}()};
bool user_lpt() { return g_user_lpt.load(std::memory_order_relaxed) != 0; }

bool fused_user_supported(int L, int D, int H, int Q) {
  return L >= 1 && L <= 64 && D == UD && H == UH && Q == UQ;
}

int32_t launch_fused_user(const float* qkv, int64_t ldq, int64_t B, int L, const float* w_add,
                          const float* b_add, const float* q_add, float* wap, float* out,
                          hipStream_t s, const PaddingGroups* pgp, bool prepacked, bool copied, bool compact,
                          int32_t* order, bool order_ready, const ScoreFold* score) {
  const PaddingGroups pg = pgp ? *pgp : PaddingGroups{nullptr, nullptr, nullptr};
  if (compact && (!pgp || L > 64 || B * L > INT32_MAX)) return NRMS_ERR_UNSUPPORTED;
  if (copied && !pgp) return NRMS_ERR_INVALID_ARG;
  const int uflags = (copied ? UF_COPIED : 0) | (compact ? UF_COMPACT : 0) |
                     (g_user_hsplit.load(std::memory_order_relaxed) ? 0 : UF_TASK_SPLIT) |
                     (g_user_pair.load(std::memory_order_relaxed) ? 0 : UF_NO_PAIR);
  if (B == 0) return NRMS_OK;
  if (!fused_user_supported(L, UD, UH, UQ) || B > INT32_MAX) return NRMS_ERR_UNSUPPORTED;
  if (((uintptr_t)qkv | (uintptr_t)out | (uintptr_t)wap) % 16 || ldq < 3 * UD || ldq % 4)
    return NRMS_ERR_UNSUPPORTED;
  ScoreFold sf{};
  if (score && score->C > 0) {
    if (!score->news || !score->logits || ((uintptr_t)score->news % 16)) return NRMS_ERR_INVALID_ARG;
    if (score->pg.pad_title && !score->pg.rep) return NRMS_ERR_INVALID_ARG;
    sf = *score;
  }
  const int ar = gemm_arith();
  const int mode = ar == NRMS_GEMM_F32 ? 0 : (ar == NRMS_GEMM_SPLIT_F16X3 ? 2 : 1);
  if (!prepacked) {
    const int blocks = mode == 2 ? pk::USER_H3_BLOCKS : ((mode ? UKS * UNT * 64 * 8 : UWAP1) + 255) / 256;
    hipLaunchKernelGGL(pack_user_b_kernel, dim3(blocks), dim3(256), 0, s, w_add, wap, mode);
    if (int32_t st = launch_status()) return st;
  }
  // longest users first (compaction only: Le comes from the padding flags)
  const int32_t* ord = nullptr;
  if (compact && order && order_ready) {
    ord = order;   // (computed by the UserEncoder projection's tail, titles.hpp)
  } else if (compact && order && g_user_lpt.load(std::memory_order_relaxed)) {
    hipLaunchKernelGGL(user_order_kernel, dim3((unsigned)((B + UORD_T - 1) / UORD_T)), dim3(UORD_T), 0, s,
                       pg.pad_title, B, L, order);
    if (int32_t st = launch_status()) return st;
    ord = order;
  }
  if (mode == 2) return launch_user_mode<2>(qkv, ldq, B, L, wap, b_add, q_add, out, s, pg, uflags, ord, sf);
  if (mode == 1) return launch_user_mode<1>(qkv, ldq, B, L, wap, b_add, q_add, out, s, pg, uflags, ord, sf);
  return launch_user_mode<0>(qkv, ldq, B, L, wap, b_add, q_add, out, s, pg, uflags, ord, sf);
}

}  // namespace nrms
