// Title classification of the fused news pass (token compaction and title
// dedupe, news_fused.hip) and the UserEncoder's dispatch order
// (user_fused.hip), shared so that nrms_forward runs them inside launches it
// makes anyway instead of launches of their own.
//
// Every small launch of the forward costs 4.6 us or more on a graph replay
// (kernel-trace durations, start to end, back to back: the dispatch and the
// cache release at each kernel boundary), and the classification kernel
// serialised one device-scope atomic per bucket and per 256-title block on one
// cache line (13.2 us at config 3). In nrms_forward the work is split in two
// halves without atomics:
//   A (forward_pack_kernel, proj_x6.hip: extra blocks next to the weight
//     packing) -- each block of CLS_T titles classifies its titles, writes the
//     compacted rows, counts and flags as before, and instead of list entries
//     a slot code per title (bucket << 16 | rank among the block's titles of
//     that bucket) and the block's bucket counts and lowest all-padding title;
//   B (the "tail jobs" of the vocabulary projection, proj_qkv_kernel: every
//     workgroup, under the loads of its first A tile) -- each workgroup takes a contiguous
//     range of classification blocks, sums the counts of the blocks before
//     its range, and writes its titles into the bucket lists; workgroup 0
//     writes the bucket totals and the rep title into the counters; the
//     UserEncoder's dispatch order is computed in the tail of the UserEncoder's
//     projection.
// The list order is then fixed (block order, ranks within blocks): a title's
// result does not depend on the group or slot it is encoded in, so the
// outputs are the atomic version's.
#pragma once

#include "nrms_common.hpp"
#include "packs.hpp"

namespace nrms {
namespace tl {

constexpr int FL = 20;                          // tokens per title (config.num_words_title)
constexpr int NBK = 5;                          // buckets NB = ceil(Le / 4) = 1 .. 5
constexpr int CLS_T = 256, CLS_W = CLS_T / 64;  // titles per classification block
constexpr int CNT_BUCKET = 1, CNT_REP = pk::NEWS_CNT_REP;
constexpr int BLK_INTS = 8;                     // per block: 5 bucket counts, lowest all-padding title, 2 unused

struct RowMap {
  const int64_t* ids_a;
  const int64_t* ids_b;
  int64_t n_seq_a, n_titles, n_rows;
  bool direct;   // per-token rows s * FL + i (the per-token projection); ids only classify
  // q|k|v row of token i of title s: >= 0 row, -1 invalid id (NaN row), -2 no title (zero row)
  __device__ __forceinline__ int64_t operator()(int64_t s, int i) const {
    if (s < 0 || s >= n_titles) return -2;
    if (direct || !ids_a) return s * FL + i;
    const int64_t id = ids_of(s)[i];
    return ((uint64_t)id < (uint64_t)n_rows) ? id : -1;
  }
  __device__ __forceinline__ const int64_t* ids_of(int64_t s) const {
    return (s < n_seq_a || ids_b == nullptr) ? ids_a + s * FL : ids_b + (s - n_seq_a) * FL;
  }
};

// Classification output (workspace): compacted row ids per title slot, the
// real-token count, the all-padding flag, per-bucket title lists and counters.
struct Titles {
  int32_t* crow;        // [n_titles][FL]: >= 0 row, -1 NaN row (invalid id), -2 zero row (unused slot)
  uint8_t* cnt;         // [n_titles] c (FL without compaction)
  uint8_t* pad_title;   // [n_titles] all 20 ids zero
  int32_t* list;        // [NBK][stride]
  int32_t* counters;    // [pk::NEWS_NCOUNT]
  int64_t stride;
};

// Split mode (half A): slot code per title (-1: not listed) and per-block counts.
struct TitleSlots {
  int32_t* slot;     // [n_titles]
  int32_t* blkcnt;   // [nblk][BLK_INTS] (16-B aligned)
};

__host__ __device__ constexpr int64_t classify_blocks(int64_t n_titles) { return (n_titles + CLS_T - 1) / CLS_T; }

// One thread per title (10 x 16-B id loads) of block blk. Lists every title in
// the bucket of its compacted length, except (dedupe) the all-padding titles:
// those are one vector, encoded once for the lowest of them (rep, appended to
// its bucket by the main pass) and copied. SPLIT: slot codes and block counts
// (half A above); else one atomicAdd per bucket and one atomicMin per block
// into the counters and the list entries directly.
// LDS_ROWS: the compacted row ids through an LDS row per thread (the pack
// launch's half A: 20 KB of static LDS there; -1 µs on qkv_news,
// profiles/r5/r5zc_rowlist_clslds_ab.txt) instead of the register form.
template <bool SPLIT, bool LDS_ROWS = false>
__device__ __forceinline__ void classify_block(int64_t blk, int tid, const RowMap& rm, const Titles& tt, int dedupe,
                                               int compact, TitleSlots sl) {
  __shared__ int wcnt[NBK][CLS_W], wbase[NBK][CLS_W], wrep[CLS_W];
  __shared__ __attribute__((aligned(16))) int32_t cls_rows[LDS_ROWS ? CLS_T : 1][FL];   // (this thread's row ids)
  const int64_t s = blk * CLS_T + tid;
  const int lane = tid & 63, w = tid >> 6;
  int bucket = -1;
  bool allpad = false;
  if (s < rm.n_titles) {
    const int4* ids4 = reinterpret_cast<const int4*>(rm.ids_of(s));   // 16-B aligned id rows (checked)
    int64_t id[FL];
#pragma unroll
    for (int i = 0; i < FL / 2; ++i) {
      const int4 v = ids4[i];
      id[2 * i] = (int64_t)(((uint64_t)(uint32_t)v.y << 32) | (uint32_t)v.x);
      id[2 * i + 1] = (int64_t)(((uint64_t)(uint32_t)v.w << 32) | (uint32_t)v.z);
    }
    auto row = [&](int i) -> int32_t {
      if (rm.direct) return (int32_t)(s * FL + i);
      return ((uint64_t)id[i] < (uint64_t)rm.n_rows) ? (int32_t)id[i] : -1;
    };
    // the 20 compacted row ids, stored as five 16-B writes
    int32_t out[FL];
    uint32_t nz = 0;
#pragma unroll
    for (int i = 0; i < FL; ++i) nz |= (id[i] != 0 ? 1u : 0u) << i;
    int c = __popc(nz);
    if (compact) {
      // the rep's row: id 0's (folded) or the first padding token's (per token)
      const int first_pad = __ffs(~nz & ((1u << FL) - 1)) - 1;   // (-1: no padding)
      const int32_t rep_row = rm.direct ? (int32_t)(s * FL + (first_pad < 0 ? 0 : first_pad))
                                        : (rm.n_rows > 0 ? 0 : -1);
      if constexpr (LDS_ROWS) {
        // through this thread's LDS row: real token i goes to position
        // popc(nz below i) (a dynamic index; in registers it would spill, and the
        // static form is 210 selects per title)
        int4* mine = reinterpret_cast<int4*>(cls_rows[tid]);
#pragma unroll
        for (int k = 0; k < FL / 4; ++k) {
          const int q = 4 * k;
          mine[k] = make_int4(q == c ? rep_row : -2, q + 1 == c ? rep_row : -2, q + 2 == c ? rep_row : -2,
                              q + 3 == c ? rep_row : -2);
        }
#pragma unroll
        for (int i = 0; i < FL; ++i)
          if ((nz >> i) & 1) cls_rows[tid][__popc(nz & ((1u << i) - 1))] = row(i);
#pragma unroll
        for (int k = 0; k < FL / 4; ++k) {
          const int4 v = mine[k];
          out[4 * k] = v.x; out[4 * k + 1] = v.y; out[4 * k + 2] = v.z; out[4 * k + 3] = v.w;
        }
      } else {
        // (static indices only: a running output index spilled the array and
        // turned the stores into 20 scattered 4-B writes per title)
#pragma unroll
        for (int q = 0; q < FL; ++q) out[q] = q == c ? rep_row : -2;
#pragma unroll
        for (int i = 0; i < FL; ++i) {
          const int d = __popc(nz & ((1u << i) - 1));   // real token i's compacted position (<= i)
          const bool real = (nz >> i) & 1;
          const int32_t r = row(i);
#pragma unroll
          for (int q = 0; q <= i; ++q) out[q] = (real && d == q) ? r : out[q];
        }
      }
      const int le = c + (c < FL ? 1 : 0);
      bucket = (le + 3) / 4 - 1;
    } else {
#pragma unroll
      for (int i = 0; i < FL; ++i) out[i] = row(i);
      bucket = NBK - 1;
    }
    int4* cr4 = reinterpret_cast<int4*>(tt.crow + s * FL);   // (80-B rows, 16-B aligned: workspace)
#pragma unroll
    for (int k = 0; k < FL / 4; ++k) cr4[k] = make_int4(out[4 * k], out[4 * k + 1], out[4 * k + 2], out[4 * k + 3]);
    allpad = c == 0;
    tt.cnt[s] = (uint8_t)(compact ? c : FL);
    tt.pad_title[s] = allpad ? 1 : 0;
    if (dedupe && allpad) bucket = -1;
  }
  const uint64_t pads = __ballot(dedupe && allpad);
  uint64_t bal[NBK];
#pragma unroll
  for (int b = 0; b < NBK; ++b) {
    bal[b] = __ballot(bucket == b);
    if (lane == 0) wcnt[b][w] = __popcll(bal[b]);
  }
  if (lane == 0) wrep[w] = pads ? (int32_t)(blk * CLS_T + 64 * w + __ffsll((long long)pads) - 1) : INT32_MAX;
  __syncthreads();
  if (tid < NBK) {
    const int b = tid;
    int tot = 0;
    for (int i = 0; i < CLS_W; ++i) tot += wcnt[b][i];
    int base = 0;
    if constexpr (SPLIT) sl.blkcnt[blk * BLK_INTS + b] = tot;
    else base = tot ? atomicAdd(&tt.counters[CNT_BUCKET + b], tot) : 0;
    for (int i = 0; i < CLS_W; ++i) { wbase[b][i] = base; base += wcnt[b][i]; }
  } else if (tid == NBK) {
    int r = INT32_MAX;
    for (int i = 0; i < CLS_W; ++i) r = min(r, wrep[i]);
    if constexpr (SPLIT) sl.blkcnt[blk * BLK_INTS + NBK] = r;
    else if (r != INT32_MAX) atomicMin(&tt.counters[CNT_REP], r);
  }
  __syncthreads();
  uint64_t mine = 0;
  int base = 0;
#pragma unroll
  for (int b = 0; b < NBK; ++b)
    if (bucket == b) { mine = bal[b]; base = wbase[b][w]; }
  const int rank = base + __popcll(mine & ((1ull << lane) - 1));
  if constexpr (SPLIT) {
    if (s < rm.n_titles) sl.slot[s] = bucket >= 0 ? (bucket << 16 | rank) : -1;
  } else {
    if (bucket >= 0) tt.list[bucket * tt.stride + rank] = (int32_t)s;
  }
}

// Half B: the bucket lists from the slot codes and block counts.
struct TitleScatter {
  const int32_t* slot;     // nullptr: no scatter
  const int32_t* blkcnt;
  int32_t* list;
  int32_t* counters;
  int64_t stride, n_titles, nblk;
};

// The UserEncoder's dispatch order (user_fused.hip): longest compacted length
// Le first, per block of UORD_U users (LDS histogram over Le, descending
// offsets); users of equal Le in any order.
constexpr int UORD_U = 1024, UORD_LMAX = 64;
struct UserOrder {
  const uint8_t* pad;   // nullptr: no order; [B][L] all-padding flags of the clicked titles
  int32_t* order;       // [B]
  int64_t B;
  int L;
};

struct TailJobs {
  TitleScatter sc;
  UserOrder uo;
};

template <int NTH>
__device__ __forceinline__ int wg_sum(int v, int* red, int tid) {
  // (callers: every thread; red: NTH / 64 ints; ends with the sum visible to all)
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  int t = 0;
#pragma unroll
  for (int i = 0; i < NTH / 64; ++i) t += red[i];
  __syncthreads();
  return t;
}

template <int NTH>
__device__ __forceinline__ int wg_min(int v, int* red, int tid) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v = min(v, __shfl_xor(v, d));
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  int t = INT32_MAX;
#pragma unroll
  for (int i = 0; i < NTH / 64; ++i) t = min(t, red[i]);
  __syncthreads();
  return t;
}

// Every thread of the workgroup calls this (it synchronises the workgroup).
template <int NTH>
__device__ __forceinline__ void run_tail_jobs(const TailJobs& tj, int tid) {
  __shared__ int red[NTH / 64];
  const TitleScatter& sc = tj.sc;
  if (sc.slot) {
    const int64_t g = blockIdx.x, G = gridDim.x;
    const int64_t c0 = g * sc.nblk / G, c1 = (g + 1) * sc.nblk / G;
    const bool totals = g == 0;
    if (c0 < c1 || totals) {
      // bucket offsets of block c0 (sum over the blocks before it), and the
      // totals and the rep (workgroup 0: over every block)
      int pre[NBK], tot[NBK], rep = INT32_MAX;
#pragma unroll
      for (int b = 0; b < NBK; ++b) pre[b] = tot[b] = 0;
      const int64_t jend = totals ? sc.nblk : c0;
      for (int64_t j = tid; j < jend; j += NTH) {
        const int4 x = *reinterpret_cast<const int4*>(sc.blkcnt + j * BLK_INTS);
        const int4 y = *reinterpret_cast<const int4*>(sc.blkcnt + j * BLK_INTS + 4);
        const int v[NBK] = {x.x, x.y, x.z, x.w, y.x};
#pragma unroll
        for (int b = 0; b < NBK; ++b) {
          pre[b] += j < c0 ? v[b] : 0;
          tot[b] += v[b];
        }
        rep = min(rep, y.y);
      }
#pragma unroll
      for (int b = 0; b < NBK; ++b) pre[b] = wg_sum<NTH>(pre[b], red, tid);
      if (totals) {
#pragma unroll
        for (int b = 0; b < NBK; ++b) tot[b] = wg_sum<NTH>(tot[b], red, tid);
        rep = wg_min<NTH>(rep, red, tid);
        if (tid < NBK) {
          int t = 0;
#pragma unroll
          for (int b = 0; b < NBK; ++b) t = tid == b ? tot[b] : t;
          sc.counters[CNT_BUCKET + tid] = t;
        } else if (tid == NBK) {
          sc.counters[CNT_REP] = rep;
        }
      }
      for (int64_t blk = c0; blk < c1; ++blk) {
        for (int t = tid; t < CLS_T; t += NTH) {
          const int64_t s = blk * CLS_T + t;
          const int32_t code = s < sc.n_titles ? sc.slot[s] : -1;
          if (code >= 0) {
            const int b = code >> 16;
            int base = 0;
#pragma unroll
            for (int q = 0; q < NBK; ++q) base = b == q ? pre[q] : base;
            sc.list[b * sc.stride + base + (code & 0xffff)] = (int32_t)s;
          }
        }
        const int4 x = *reinterpret_cast<const int4*>(sc.blkcnt + blk * BLK_INTS);
        const int y = sc.blkcnt[blk * BLK_INTS + 4];
        pre[0] += x.x; pre[1] += x.y; pre[2] += x.z; pre[3] += x.w; pre[4] += y;
      }
    }
  }
  const UserOrder& uo = tj.uo;
  if (uo.pad) {
    __shared__ int cnt[UORD_LMAX + 1], base[UORD_LMAX + 1];
    constexpr int UPT = (UORD_U + NTH - 1) / NTH;   // users per thread
    const int64_t nub = (uo.B + UORD_U - 1) / UORD_U;
    // (user blocks from the last workgroup down: workgroup 0 has the totals)
    for (int64_t ub = (int64_t)gridDim.x - 1 - blockIdx.x; ub < nub; ub += gridDim.x) {
      const int64_t u0 = ub * UORD_U;
      if (tid <= UORD_LMAX) cnt[tid] = 0;
      __syncthreads();
      int le[UPT];
#pragma unroll
      for (int k = 0; k < UPT; ++k) {
        const int64_t u = u0 + tid + (int64_t)k * NTH;
        le[k] = -1;
        if (tid + k * NTH < UORD_U && u < uo.B) {
          const uint8_t* p = uo.pad + u * uo.L;
          int npad = 0;
          for (int i = 0; i < uo.L; ++i) npad += p[i] ? 1 : 0;
          le[k] = uo.L - npad + (npad > 0 ? 1 : 0);
          atomicAdd(&cnt[le[k]], 1);
        }
      }
      __syncthreads();
      if (tid <= UORD_LMAX) {   // base[l] = sum of cnt[m], m > l
        int acc = 0;
        for (int m = tid + 1; m <= UORD_LMAX; ++m) acc += cnt[m];
        base[tid] = acc;
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < UPT; ++k)
        if (le[k] >= 0) uo.order[u0 + atomicAdd(&base[le[k]], 1)] = (int32_t)(u0 + tid + (int64_t)k * NTH);
      __syncthreads();
    }
  }
}

// Half A's arguments (forward_pack_kernel's classification blocks).
struct ClassifyJob {
  RowMap rm;
  Titles tt;
  TitleSlots sl;
  int dedupe, compact;
  int64_t nblk;
};

}  // namespace tl

// The forward's split classification of the titles of a folded-row fused news
// launch on workspace ws (news_fused.hip): false when launch_fused_news would
// not classify them; else both halves' arguments. The news launch then takes
// preclassified = true (and prepacked: the pack's counter reset comes first).
bool fused_news_classify_split(float* ws, const int64_t* ids_a, int64_t n_seq_a, const int64_t* ids_b,
                               int64_t n_titles, int64_t n_rows, tl::ClassifyJob* job, tl::TitleScatter* sc);

}  // namespace nrms
