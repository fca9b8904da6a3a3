// Q|K|V projection Y = X[row(m)] · [Wq; Wk; Wv]^T + [bq; bk; bv] for the
// NRMS shape (K = D = 300, N = 3D = 900; multihead_self.py:53-58) on the
// split-bf16 x6 arithmetic, with the weight split once per call.
//
// gemm_x6_kernel (gemm_f32.hip) stages A and W chunks through LDS and splits
// both while staging: for a 64 x 192 tile the 192 W rows are split again for
// every 64 rows of A, three times the splitting the A tile itself needs, and
// that VALU work is what bounds it (4-5 VALU per MFMA, PMC). Here:
//   * proj_x6_pack_kernel splits W once per call into MFMA B fragments,
//     [k-step][N tile][plane][lane][8 bf16] (1.75 MB, stays in every XCD's
//     L2), plus the bias row;
//   * one persistent workgroup per CU keeps a 64-row A tile resident in LDS as
//     three bf16 planes (split once, 125 KB) and computes its outputs in three
//     20-tile column ranges (items), each wave 5 N tiles x 4 M tiles, streaming
//     the B fragments from L2 through a buffer resource (lane / N tile in one
//     VGPR offset, k-step / plane in the SGPR offset: no per-load address
//     registers in the unrolled 10-k-step mainloop);
//   * the next row tile's A rows are loaded into registers during the last
//     k-step of the tile's last item, split into LDS behind one barrier pair.
// x6: each output tile accumulates exactly the MFMA sequence of
// gemm_x6_kernel — the same k-steps, fragment K order and product order
// (lo·hi, mid·mid, hi·lo, mid·hi, hi·mid, hi·hi), then (0 + acc) + bias — so
// the two kernels agree bitwise (tests/test_gpu_parity.py compares them).
//
// H3 (the default arithmetic, NRMS_GEMM_SPLIT_F16X3): split-f16 with
// power-of-two scaling, three or four products instead of six. Every A row and every
// W row (output column) is scaled by its own power of two, 2^-ea (row max
// into [2^3, 2^4)) and 2^-ew (into [2^14, 2^15)), which is exact and puts both
// in fp16's range whatever their magnitude. A is split into three fp16
// pieces, 2^11 a = 2^11 hi + lo + r exactly (hi = fp16(a), lo = fp16 of the
// 2^11-scaled residual, r the bits lo misses); W into two, w = hi + 2^-11 lo
// (22 bits). The products w_hi·r, w_lo·a_hi, w_hi·a_lo and w_hi·(2^11 a_hi)
// (formed in registers) all carry 2^11 and sum in one fp32 accumulator on
// v_mfma_f32_16x16x32_f16 (fp16 products are exact in fp32), and
// y = ldexp(acc, ea + ew - 11) + bias. The dropped terms (w_lo·(lo + r),
// W's residual) are ~2^-22 of each column's largest |w|: the rows stay within
// fp32 GEMM rounding (tests bound them against an fp64 oracle), and a W that
// fits in 11 bits (e.g. the overflow-boundary fixtures' one-hot W_Q) gives
// products as exact as fp32's — the reference's raw-exp overflow boundary is
// reproduced. That exactness is all the fourth product, w_hi·r (A's bits past
// 22), adds: where a column's w_lo is non-zero, the dropped w_lo·(lo + r) is
// of its size. So the kernel runs three products (w_lo·a_hi, w_hi·a_lo,
// w_hi·(2^11 a_hi); no r plane staged) unless some column of the weight set
// fits in 11 bits (the pack's column flags; NRMS_PROJ_PRODUCTS=4 forces four).
// W streams as two fp16 planes instead of three bf16 planes. A NaN stays NaN;
// an infinite input gives NaN in its row (column), as x6.

#include "nrms_common.hpp"
#include "packs.hpp"
#include "titles.hpp"

#include <type_traits>

namespace nrms {
namespace {

constexpr int PK = 300, PN = 900;
constexpr int PKS = 10;                          // k-steps of 32 (K padded to 320)
constexpr int PKP = PKS * 32;                    // 320
constexpr int PNT = (PN + 15) / 16;              // 57 N tiles (the last: 4 live columns)
#ifndef NRMS_PX_PM   // (probe: other tile heights; profiles/r6/r6w_proj_tile_height_ab.txt)
#define NRMS_PX_PM 64
#endif
constexpr int PM = NRMS_PX_PM;                   // A rows per tile
constexpr int PMT = PM / 16;                     // 4 M tiles
constexpr int PTW = 5;                           // N tiles per wave per item
constexpr int PRANGE = 4 * PTW;                  // N tiles per item
constexpr int PNR = (PNT + PRANGE - 1) / PRANGE; // items per row tile (3)
static_assert(PNT > (PNR - 1) * PRANGE, "item ranges");
// LDS row: [hi 320 | mid 320 | lo 320 | pad 16] bf16 = 1,952 B = 488 dwords
// (= 40 mod 64): the 16-row x 4-kq fragment reads cover all 64 banks once.
constexpr int PRB = 3 * PKP + 16;
constexpr size_t P_LDS = (size_t)PM * PRB * 2 + PM * (sizeof(int64_t) + sizeof(int32_t));
static_assert(P_LDS <= 160 * 1024, "LDS");
constexpr int PACK_BF16 = PKS * PNT * 3 * 512;   // B fragments
constexpr int PTRASH = 16 * PNT;                 // floats: target of the stores of rows past M
static_assert(PN % 4 == 0, "16-B output pieces");
// + bias row (0 past N), zero row, NaN row, trash line
#ifdef NRMS_PX_TIMING
// probe build (profiles/probes/px_phases.py): per-wave phase cycles after the pack
constexpr int PSTAMP_FLOATS = 256 * 8 * 8 * 2;
#else
constexpr int PSTAMP_FLOATS = 0;
#endif
// [fragments (x6: 3 bf16 planes, H3: 2 fp16 planes)][bias][zero row][NaN row][trash][H3 column exponents]
// [H3 column flags: 1 = no fourth product (W has bits past 11, or the column is past N)][stamps]
constexpr int OFF_BIAS = PACK_BF16 / 2, OFF_ZERO = OFF_BIAS + PNT * 16, OFF_NAN = OFF_ZERO + PKP;
constexpr int OFF_TRASH = OFF_NAN + PKP, OFF_EXP = OFF_TRASH + PTRASH, OFF_WRES = OFF_EXP + PNT * 16;
constexpr int OFF_STAMP = OFF_WRES + PNT * 16;
constexpr int PACK_FLOATS = OFF_STAMP + PSTAMP_FLOATS;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
constexpr float kTwo11 = 2048.0f;

// unbiased exponent field of |x| (0 -> -127; inf / NaN -> 128)
using pk::exp_field;

__device__ __forceinline__ void split3(float x, __bf16& hi, __bf16& mid, __bf16& lo) {
  hi = (__bf16)x;
  const float r = x - (float)hi;
  mid = (__bf16)r;
  lo = (__bf16)(r - (float)mid);
}

// [ks][nt][plane][lane][8]: plane of W[16 nt + (lane & 15)][32 ks + 8 (lane >> 4) + i]
// (0 past N or K), then bias[16 PNT], a zero row and a NaN row (the A rows of
// rows past M / of invalid ids). blockIdx.y selects the weight set.
constexpr int PACK_ELEMS = PKS * PNT * 512 + PNT * 16 + 2 * PKP;   // threads of one weight set's packing

__device__ __forceinline__ void pack_proj(int idx, const WeightRows& w, float* __restrict__ dst) {
  constexpr int NE = PKS * PNT * 512;
  if (idx < NE) {
    const int i = idx & 7, lane = (idx >> 3) & 63, t = idx >> 9;
    const int nt = t % PNT, ks = t / PNT;
    const int n = 16 * nt + (lane & 15), k = 32 * ks + 8 * (lane >> 4) + i;
    float v = 0.f;
    if (n < PN && k < PK) {
      const int seg = n / w.seg_rows;
      v = w.w[seg][(int64_t)(n - seg * w.seg_rows) * PK + k];
    }
    __bf16 hi, mid, lo;
    split3(v, hi, mid, lo);
    __bf16* o = reinterpret_cast<__bf16*>(dst) + (int64_t)t * 3 * 512 + lane * 8 + i;
    o[0] = hi;
    o[512] = mid;
    o[1024] = lo;
  } else if (idx < NE + PNT * 16) {
    const int c = idx - NE;
    float b = 0.f;
    if (c < PN) {
      const int seg = c / w.seg_rows;
      b = w.b[seg] ? w.b[seg][c - seg * w.seg_rows] : 0.f;
    }
    dst[PACK_BF16 / 2 + c] = b;
  } else if (idx < NE + PNT * 16 + 2 * PKP) {
    const int c = idx - NE - PNT * 16;
    dst[PACK_BF16 / 2 + PNT * 16 + c] = c < PKP ? 0.f : qnan();
  }
}

// H3: one wave per W row n < 16 PNT (rows past N: zeros), lane k = lane + 64 i
// (i < 5 covers the K padding to 320): the row's max |w| (wave reduction)
// gives its exponent ew; [ks][nt][plane hi | 2^-11 lo][lane][8 f16] as the x6
// fragments; lane 0 writes the bias, ew and whether the column can do
// without the projection's fourth product (an element of the row has bits
// past hi, so lo != 0; columns past N: yes). Block
// PACK_ROWS_H3 / 4 writes the zero and NaN rows.
constexpr int PACK_BLOCKS_H3 = PNT * 16 / 4 + 1;
__device__ __forceinline__ void pack_proj_h3(int b, int t, const WeightRows& w, float* __restrict__ dst) {
  if (b == PACK_BLOCKS_H3 - 1) {
    for (int c = t; c < 2 * PKP; c += 256) dst[OFF_ZERO + c] = c < PKP ? 0.f : qnan();
    return;
  }
  const int lane = t & 63, n = 4 * b + (t >> 6);
  const int seg = n < PN ? n / w.seg_rows : 0;
  const float* wr = w.w[seg] + (int64_t)(n - seg * w.seg_rows) * PK;
  float v[5], mx = 0.f;
  bool inexact = false;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int k = lane + 64 * i;
    v[i] = (n < PN && k < PK) ? wr[k] : 0.f;
    mx = fmaxf(mx, fabsf(v[i]));
  }
#pragma unroll
  for (int o = 32; o; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  const int ew = exp_field(mx) - 14;
  _Float16* o = reinterpret_cast<_Float16*>(dst);
  const int nt = n >> 4, r = n & 15;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int k = lane + 64 * i, ks = k >> 5, kq = (k >> 3) & 3;
    const float x = ldexpf(v[i], -ew);
    const _Float16 hi = (_Float16)x;
    // lo plane at 2^-11 of the split's: it multiplies the staged 2^11 a_hi
    // (a fp16 subnormal below 2^-14: bits lost only where the element is
    // under 2^-18 of its column's largest)
    const _Float16 lo = (_Float16)(x - (float)hi);
    inexact |= !(x == (float)hi);                 // bits past 11 (NaN: inexact)
    const int e = ((ks * PNT + nt) * 2) * 512 + (r + 16 * kq) * 8 + (k & 7);
    o[e] = hi;
    o[e + 512] = lo;
  }
  const bool row_inexact = __ballot(inexact) != 0;
  if (lane == 0) {
    dst[OFF_BIAS + n] = (n < PN && w.b[seg]) ? w.b[seg][n - seg * w.seg_rows] : 0.f;
    reinterpret_cast<int32_t*>(dst)[OFF_EXP + n] = ew;
    reinterpret_cast<int32_t*>(dst)[OFF_WRES + n] = (row_inexact || n >= PN) ? 1 : 0;
  }
}

__global__ __launch_bounds__(256) void proj_x6_pack_kernel(WeightRows w0, WeightRows w1, float* __restrict__ d0,
                                                           float* __restrict__ d1, int h3) {
  if (h3) pack_proj_h3(blockIdx.x, threadIdx.x, blockIdx.y ? w1 : w0, blockIdx.y ? d1 : d0);
  else pack_proj(blockIdx.x * 256 + threadIdx.x, blockIdx.y ? w1 : w0, blockIdx.y ? d1 : d0);
}

// nrms_forward's four packings in one launch: blocks [0, P) news Q|K|V,
// [P, 2P) user Q|K|V (P = PACK_BLOCKS, or PACK_BLOCKS_H3 when f16), then the
// news W_add (x6 planes, f16 planes if f16, the special rows, the counters),
// then the UserEncoder W_add (x6 layout, or split-f16 when f16); before all of
// them (cj.nblk > 0) the first half of the news titles' classification
// (titles.hpp).
constexpr int PACK_BLOCKS = (PACK_ELEMS + 255) / 256;
constexpr int NEWS_ADD_BLOCKS = (pk::NEWS_X6_ELEMS + pk::NEWS_SPECIAL + 255) / 256;
constexpr int USER_ADD_BLOCKS = (pk::USER_X6_ELEMS + 255) / 256;
__global__ __launch_bounds__(256) void forward_pack_kernel(WeightRows wn, float* __restrict__ pn, WeightRows wu,
                                                           float* __restrict__ pu, const float* __restrict__ nwa,
                                                           float* __restrict__ nws, int nf16,
                                                           const float* __restrict__ uwa, float* __restrict__ uws,
                                                           tl::ClassifyJob cj) {
  int b = blockIdx.x;
  const int t = threadIdx.x;
  // the classification blocks first (their id loads are the launch's long
  // pole; dispatched last they set its end)
  if (b < cj.nblk) return tl::classify_block<true, true>(b, t, cj.rm, cj.tt, cj.dedupe, cj.compact, cj.sl);
  b -= (int)cj.nblk;
  if (nf16) {
    if (b < PACK_BLOCKS_H3) return pack_proj_h3(b, t, wn, pn);
    b -= PACK_BLOCKS_H3;
    if (b < PACK_BLOCKS_H3) return pack_proj_h3(b, t, wu, pu);
    b -= PACK_BLOCKS_H3;
  } else {
    if (b < PACK_BLOCKS) return pack_proj(b * 256 + t, wn, pn);
    b -= PACK_BLOCKS;
    if (b < PACK_BLOCKS) return pack_proj(b * 256 + t, wu, pu);
    b -= PACK_BLOCKS;
  }
  if (b < NEWS_ADD_BLOCKS) {
    int32_t* counters = reinterpret_cast<int32_t*>(nws + pk::NEWS_COUNTERS);
    if (nf16) pk::pack_news_additive<true>(b * 256 + t, nwa, nws, counters);
    else pk::pack_news_additive<false>(b * 256 + t, nwa, nws, counters);
    return;
  }
  b -= NEWS_ADD_BLOCKS;
  if (nf16) pk::pack_user_additive_h3(b, t, uwa, uws);
  else pk::pack_user_additive(b * 256 + t, uwa, uws, 1);
  static_assert(tl::CLS_T == 256, "classification blocks of the pack launch");
}

// SCATTER: output row m goes to Y row row_ids[m] (row-list mode; the count is
// *m_dev, written by an earlier launch). Otherwise row_ids (optional) only
// gathers the A rows (the fused embedding gather of the per-token mode).
// NW waves: 4 (one per SIMD, five N tiles each) or 8 (two per SIMD: waves
// w < 4 three tiles, w >= 4 two, so each SIMD still owns five tiles of an
// item and one wave's waits / stores run under its partner's MFMAs).
// H3: the split-f16 arithmetic above (A planes 2^11 hi | lo | r in LDS, W
// planes hi | 2^-11 lo), else x6.
template <bool SCATTER, int NW, bool H3>
__global__ __launch_bounds__(64 * NW, 1) void proj_qkv_kernel(const float* __restrict__ X, int64_t n_rows_x, ARows ar,
                                                            const int64_t* __restrict__ row_ids, int64_t M,
                                                            const float* __restrict__ packed, float* __restrict__ Y,
                                                            int64_t ldy, const int32_t* __restrict__ m_dev,
                                                            tl::TailJobs tj, int force4) {
  static_assert(NW == 4 || NW == 8, "waves per workgroup");
  constexpr int NTH = 64 * NW;
  constexpr int TPR = NTH / PM;                      // threads per A row (4 or 8)
  constexpr int AP = (PK / 4 + TPR - 1) / TPR;       // float4 pieces per thread (19 or 10)
  constexpr int NPL = H3 ? 2 : 3;                    // W planes
  using frag = std::conditional_t<H3, f16x8, bf16x8>;
  extern __shared__ __attribute__((aligned(16))) float lds_f[];
  __bf16* As = reinterpret_cast<__bf16*>(lds_f);
  int64_t* orow = reinterpret_cast<int64_t*>(As + PM * PRB);   // output row offset (-1: no row)
  int32_t* erow = reinterpret_cast<int32_t*>(orow + PM);       // H3: row exponent ea - 11

#ifdef NRMS_PX_SC1
  // (probe) the output rows through a buffer resource with sc1 stores (the
  // line leaves the XCD's L2 once written: the W planes are not evicted by
  // the 263-MB output stream); rows past M, columns past N and (SCATTER) ids
  // past the capacity M get an out-of-range offset (dropped by the hardware)
  const uint64_t y_bytes = (uint64_t)M * (uint64_t)ldy * 4;
  const bool sc1 = y_bytes + 64 < 0xFFFFFF00ull;   // (workgroup-uniform)
  const int64_t m_cap = M;
  const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(Y, 0, sc1 ? (int)y_bytes : 0, 0x00020000);
#endif
  if constexpr (SCATTER) {
    const int64_t mc = *m_dev;
    M = mc < M ? mc : M;
  }
  const int64_t n_items = (M + PM - 1) / PM * PNR;
#ifdef NRMS_PX_XCD
  // (probe) XCD-major workgroup order: workgroups b, b + 8, .. (one XCD) take
  // consecutive item ranges, so a row tile split between two workgroups is
  // staged twice within one L2
  const int64_t lb = (gridDim.x % 8 == 0) ? (int64_t)(blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8
                                          : (int64_t)blockIdx.x;
  const int64_t i0 = lb * n_items / gridDim.x;
  const int64_t i1 = (lb + 1) * n_items / gridDim.x;
#else
  const int64_t i0 = (int64_t)blockIdx.x * n_items / gridDim.x;
  const int64_t i1 = ((int64_t)blockIdx.x + 1) * n_items / gridDim.x;
#endif
  const bool tail = tj.sc.slot || tj.uo.pad;
  if (i0 >= i1) {
    if (tail) tl::run_tail_jobs<NTH>(tj, threadIdx.x);
    return;
  }

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lm = lane & 15, kq = lane >> 4;
#ifdef NRMS_PX_STAGGER   // probe: odd workgroups start ~NRMS_PX_STAGGER x 8k cycles late
  if (blockIdx.x & 1)
    for (int i = 0; i < NRMS_PX_STAGGER; ++i) __builtin_amdgcn_s_sleep(127);
#endif

  // K padding: columns 300..319 of every plane stay zero for the whole launch
  for (int e = tid; e < PM * 3 * ((PKP - PK) / 4); e += NTH) {
    const int r = e / (3 * ((PKP - PK) / 4)), rem = e - r * (3 * ((PKP - PK) / 4));
    const int pl = rem / ((PKP - PK) / 4), c = rem - pl * ((PKP - PK) / 4);
    *reinterpret_cast<uint2*>(As + r * PRB + pl * PKP + PK + 4 * c) = make_uint2(0u, 0u);
  }

  // A tile staging: thread (row ar_ = tid / TPR, q = tid % TPR) moves the
  // float4 pieces q, q + TPR, .. of one row, from one source pointer per row
  // tile: the row itself, the pack's zero row (past M) or its NaN row
  // (invalid id: the row becomes NaN, as gemm_x6_kernel)
  const int ar_ = tid / TPR, aq = tid % TPR;
  const float* zero_row = packed + OFF_ZERO;
  const float* nan_row = packed + OFF_NAN;
  struct ASrc {
    const float* p;
    int64_t o;   // output row offset (-1: no row)
  };
  // The row id of the next tile's row is loaded unconditionally (a safe
  // index past M) and resolved only where the row is loaded, after the
  // mainloop: consumed at once, its load made the waitcnt pass wait for every
  // older memory operation -- the previous item's output stores included.
  auto a_id = [&](int64_t rt) __attribute__((always_inline)) -> int64_t {
    const int64_t m = rt * PM + ar_;
    return row_ids ? row_ids[m < M ? m : 0] : m;
  };
  auto a_resolve = [&](int64_t rt, int64_t id) __attribute__((always_inline)) -> ASrc {
    const int64_t m = rt * PM + ar_;
    if (m >= M) return ASrc{zero_row, -1};
    const int64_t o = (SCATTER ? id : m) * ldy;
    return ASrc{(uint64_t)id < (uint64_t)n_rows_x ? X + ar.offset(id) : nan_row, o};
  };
  auto a_src = [&](int64_t rt) __attribute__((always_inline)) -> ASrc { return a_resolve(rt, a_id(rt)); };
  float4 ra[AP];
  auto load_a = [&](const float* src) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < AP; ++j) {
      const int c4 = aq + TPR * j < PK / 4 ? aq + TPR * j : PK / 4 - 1;   // (pieces past the row: unused)
#ifdef NRMS_PX_NT_A   // probe: A rows as streaming loads (keep the W planes in L2)
      const floatx4 v = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(src + 4 * c4));
      ra[j] = make_float4(v[0], v[1], v[2], v[3]);
#else
      ra[j] = *reinterpret_cast<const float4*>(src + 4 * c4);
#endif
    }
  };
  // H3 on three products unless some W column fits in 11 bits (the pack's
  // column flags, read by every workgroup; header comment).
  bool p4 = true;
  int p3_cols = 1;
  if constexpr (H3) {
    const int32_t* wres0 = reinterpret_cast<const int32_t*>(packed) + OFF_WRES;
    for (int c = threadIdx.x; c < PNT * 16; c += NTH) p3_cols &= wres0[c];
  }
  auto store_a = [&](int64_t o) __attribute__((always_inline)) {
    if constexpr (H3) {
      // the row's max |a| over its TPR threads (consecutive lanes; pieces past
      // the row repeat piece 74) -> ea, then a' = 2^-ea a in [2^3, 2^4) at most
      float mx = 0.f;
#pragma unroll
      for (int j = 0; j < AP; ++j)
        mx = fmaxf(mx, fmaxf(fmaxf(fabsf(ra[j].x), fabsf(ra[j].y)), fmaxf(fabsf(ra[j].z), fabsf(ra[j].w))));
#pragma unroll
      for (int d = 1; d < TPR; d <<= 1) mx = fmaxf(mx, __shfl_xor(mx, d));
      const int ea = exp_field(mx) - 3;
#pragma unroll
      for (int j = 0; j < AP; ++j) {
        const int c4 = aq + TPR * j;
        if (c4 < PK / 4) {
          _Float16 h[4], l[4], r[4];
          const float xs[4] = {ra[j].x, ra[j].y, ra[j].z, ra[j].w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float x = ldexpf(xs[e], -ea);
            h[e] = (_Float16)x;
            const float r1 = (x - (float)h[e]) * kTwo11;   // exact
            l[e] = (_Float16)r1;
            r[e] = (_Float16)(r1 - (float)l[e]);           // exact (the bits lo misses)
          }
          _Float16* d = reinterpret_cast<_Float16*>(As) + ar_ * PRB + 4 * c4;
          typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
          // plane 0 holds 2^11 hi (exact: |hi| <= 16)
          *reinterpret_cast<f16x4*>(d) = f16x4{h[0], h[1], h[2], h[3]} * (_Float16)kTwo11;
          *reinterpret_cast<f16x4*>(d + PKP) = f16x4{l[0], l[1], l[2], l[3]};
          if (p4) *reinterpret_cast<f16x4*>(d + 2 * PKP) = f16x4{r[0], r[1], r[2], r[3]};
        }
      }
      if (aq == 0) {
        orow[ar_] = o;
        erow[ar_] = ea - 11;
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < AP; ++j) {
      const int c4 = aq + TPR * j;
      if (c4 < PK / 4) {
        uint32_t h0, m0, l0, h1, m1, l1;
        split3x2(ra[j].x, ra[j].y, h0, m0, l0);
        split3x2(ra[j].z, ra[j].w, h1, m1, l1);
        __bf16* d = As + ar_ * PRB + 4 * c4;
        *reinterpret_cast<uint2*>(d) = make_uint2(h0, h1);
        *reinterpret_cast<uint2*>(d + PKP) = make_uint2(m0, m1);
        *reinterpret_cast<uint2*>(d + 2 * PKP) = make_uint2(l0, l1);
      }
    }
    if (aq == 0) orow[ar_] = o;
  };

  {
    const ASrc a0 = a_src(i0 / PNR);
    load_a(a0.p);
    // the tail jobs (titles.hpp) under the first A tile's loads: after the
    // last item they added their dependent loads to the kernel's end
    if (tail) tl::run_tail_jobs<NTH>(tj, tid);
    if constexpr (H3) p4 = force4 || !__syncthreads_and(p3_cols);
    store_a(a0.o);
  }
  __syncthreads();

  const __amdgpu_buffer_rsrc_t brs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(packed), 0, PACK_BF16 * 2, 0x00020000);
  const float* bias = packed + OFF_BIAS;
  const int32_t* wexp = reinterpret_cast<const int32_t*>(packed) + OFF_EXP;   // H3 column exponents
  float* trash = const_cast<float*>(packed) + OFF_TRASH;   // stores of rows past M
#ifdef NRMS_PX_TIMING
  unsigned long long tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tprev = __builtin_amdgcn_s_memtime();
#define NRMS_PX_STAMP(k)                                          \
  {                                                               \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    tacc[k] += now_ - tprev;                                      \
    tprev = now_;                                                 \
  }
#else
#define NRMS_PX_STAMP(k)
#endif
  // A fragments (16x16x32): lane holds A[row lm + 16 mt][32 ks + 8 kq .. + 7] of each plane
  const __bf16* Ab = As + lm * PRB + 8 * kq;

  // The wave's N tiles of item (row tile rt, range rg): t0 = 20 rg + off ..
  // t0 + C - 1; tiles past N (the last range has 17) are computed on a clamped
  // copy and not stored — those waves would otherwise wait at the next restage
  // barrier for the waves with live tiles.
  const int off_w = NW == 4 ? PTW * w : (w < 4 ? 3 * w : 12 + 2 * (w - 4));
  // p4c: H3 on four products, or three (below)
  auto run = [&](auto cc, auto p4c) __attribute__((always_inline)) {
    constexpr int C = decltype(cc)::value;
    auto tile_of = [&](int64_t item, int j) __attribute__((always_inline)) -> int {
      const int t = (int)(item % PNR) * PRANGE + off_w + j;
      return t < PNT ? t : PNT - 1;
    };
    // plane-major: x6, the hi planes (first product's B) arrive first; H3,
    // lo (first product's B) then hi
    auto load_b = [&](int ks, const int (&bvo)[C], frag (&dst)[C][NPL]) __attribute__((always_inline)) {
#pragma unroll
      for (int q = 0; q < NPL; ++q) {
        const int pl = H3 ? 1 - q : q;
#pragma unroll
        for (int j = 0; j < C; ++j)
          dst[j][pl] = __builtin_bit_cast(
              frag, __builtin_amdgcn_raw_buffer_load_b128(brs, bvo[j], (ks * PNT * NPL + pl) * 1024, 0));
      }
    };
    // A fragments of one k-step in the order the products use them (x6: lo
    // planes first; H3: 2^11 hi, lo, r)
    auto load_afrag = [&](int ks, frag (&a)[PMT][3], auto p4c) __attribute__((always_inline)) {
      constexpr int NAP = (H3 && !decltype(p4c)::value) ? 2 : 3;   // A planes read
#pragma unroll
      for (int q = 0; q < NAP; ++q) {
        const int pl = H3 ? q : 2 - q;
#pragma unroll
        for (int mt = 0; mt < PMT; ++mt)
          a[mt][pl] = *reinterpret_cast<const frag*>(Ab + 16 * mt * PRB + pl * PKP + 32 * ks);
      }
    };
    floatx4 acc[PMT][C];
    // one product (A plane PA, W plane PB) of M tile mt, N tile j
    auto mfma = [&](const frag (&a)[PMT][3], const frag (&bb)[C][NPL], int mt, int j, int PA, int PB)
        __attribute__((always_inline)) {
      if constexpr (H3)
        acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bb[j][PB], a[mt][PA], acc[mt][j], 0, 0, 0);
      else
        acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb[j][PB], a[mt][PA], acc[mt][j], 0, 0, 0);
    };
    // H3: 2^11 a = 2^11 hi + lo + r exactly; with w = hi + 2^-11 lo the
    // products w_hi·r (P4), w_lo·a_hi, w_hi·a_lo, w_hi·(2^11 a_hi) accumulate
    // 2^11 w·a. The A planes in LDS are [2^11 hi | lo | r] and the W lo plane
    // is packed at 2^-11, so w_lo·a_hi = (2^-11 w_lo)·(2^11 hi): every product
    // is one plane pair, no operand formed in registers.
    auto mfma_h = [&](const frag& b, const frag& a, int mt, int j) __attribute__((always_inline)) {
      acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(b, a, acc[mt][j], 0, 0, 0);
    };
    // product p: (W plane, A plane) = (hi, r), (lo, 2^11 hi), (hi, lo), (hi, 2^11 hi)
    auto pw = [](int p) constexpr { return p == 1 ? 1 : 0; };
    auto pa = [](int p) constexpr { return p == 0 ? 2 : p == 2 ? 1 : 0; };
    auto kstep = [&](const frag (&a)[PMT][3], const frag (&bb)[C][NPL], auto p4c) __attribute__((always_inline)) {
      if constexpr (H3) {
#pragma unroll
        for (int p = decltype(p4c)::value ? 0 : 1; p < 4; ++p)
#pragma unroll
          for (int j = 0; j < C; ++j)
#pragma unroll
            for (int mt = 0; mt < PMT; ++mt) mfma_h(bb[j][pw(p)], a[mt][pa(p)], mt, j);
      } else {
        constexpr int pa_[6] = {2, 1, 0, 1, 0, 0}, pb_[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
        for (int p = 0; p < 6; ++p)
#pragma unroll
          for (int j = 0; j < C; ++j)
#pragma unroll
            for (int mt = 0; mt < PMT; ++mt) mfma(a, bb, mt, j, pa_[p], pb_[p]);
      }
    };

    int bvoff[C];
#pragma unroll
    for (int j = 0; j < C; ++j) bvoff[j] = lane * 16 + tile_of(i0, j) * NPL * 1024;
    frag b0[C][NPL], b1[C][NPL];
    load_b(0, bvoff, b0);   // each item's first k-step is loaded by the previous item

    for (int64_t it = i0; it < i1; ++it) {
      NRMS_PX_STAMP(0)   // (loop overhead, restage of the previous item)
      const int64_t rt = it / PNR;
      const bool restage = it + 1 < i1 && (it + 1) / PNR != rt;   // workgroup-uniform
      const int64_t an_id = restage ? a_id(rt + 1) : 0;   // (its load completes behind the mainloop)
      const int t0 = (int)(it % PNR) * PRANGE + off_w;
      float4 bj[C];
      int4 ej[C];   // H3: column exponents
      int bnext[C];
#pragma unroll
      for (int j = 0; j < C; ++j) {
        bj[j] = *reinterpret_cast<const float4*>(bias + 16 * tile_of(it, j) + 4 * kq);   // (0 past N)
        if constexpr (H3) ej[j] = *reinterpret_cast<const int4*>(wexp + 16 * tile_of(it, j) + 4 * kq);
        bnext[j] = lane * 16 + tile_of(it + 1 < i1 ? it + 1 : it, j) * NPL * 1024;
      }
#pragma unroll
      for (int mt = 0; mt < PMT; ++mt)
#pragma unroll
        for (int j = 0; j < C; ++j) acc[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};
      // two B buffers (and, at one wave per SIMD, two A-fragment buffers) in
      // turn; each k-step's loads fenced where they are issued (left free, the
      // scheduler sinks them to their first use); the last k-step pair loads
      // the next item's first B
      // The products run with W as the MFMA's A operand, so the 16x16 C/D
      // layout (col = lane & 15, row = 4 kq + reg) is transposed: lane (lm, kq)
      // holds output row 16 mt + lm, columns 16 t + 4 kq .. + 3 — one 16-B store
      // per (M tile, N tile). (Swapping the operands of a product changes no
      // bit of it; tests compare with gemm_x6_kernel.) One base address per
      // output row (rows past M write the pack's trash line), the N tiles at
      // immediate offsets; tiles past N skipped, columns past N of the last masked.
      float* base[PMT];
      int ea[PMT];   // H3: row exponent - 11
#ifdef NRMS_PX_SC1
      uint32_t yoff[PMT];   // byte offsets into Y (0xFFFFFFF0: dropped)
#endif
#pragma unroll
      for (int mt = 0; mt < PMT; ++mt) {
        const int64_t o = orow[16 * mt + lm];
        base[mt] = (o >= 0 ? Y + o : trash) + 16 * t0 + 4 * kq;
#ifdef NRMS_PX_SC1
        yoff[mt] = (o >= 0 && o < m_cap * ldy) ? (uint32_t)((o + 16 * t0 + 4 * kq) * 4) : 0xFFFFFFF0u;
#endif
        if constexpr (H3) ea[mt] = erow[16 * mt + lm];
      }
      auto store_tile = [&](int j) __attribute__((always_inline)) {
        if (t0 + j >= PNT) return;                        // wave-uniform
        const bool full = 16 * (t0 + j) + 16 <= PN;       // wave-uniform
#pragma unroll
        for (int mt = 0; mt < PMT; ++mt) {
          float4 v;
          if constexpr (H3) {
            v.x = ldexpf(acc[mt][j][0], ea[mt] + ej[j].x) + bj[j].x;
            v.y = ldexpf(acc[mt][j][1], ea[mt] + ej[j].y) + bj[j].y;
            v.z = ldexpf(acc[mt][j][2], ea[mt] + ej[j].z) + bj[j].z;
            v.w = ldexpf(acc[mt][j][3], ea[mt] + ej[j].w) + bj[j].w;
          } else {
            v.x = (0.f + acc[mt][j][0]) + bj[j].x;
            v.y = (0.f + acc[mt][j][1]) + bj[j].y;
            v.z = (0.f + acc[mt][j][2]) + bj[j].z;
            v.w = (0.f + acc[mt][j][3]) + bj[j].w;
          }
#ifdef NRMS_PX_NOSTORE   // probe: the epilogue without its stores
          if (v.x == 12345.f) *reinterpret_cast<float4*>(base[mt] + 16 * j) = v;
#elif defined(NRMS_PX_SC1)
          if (sc1) {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            const uint32_t off =
                (yoff[mt] != 0xFFFFFFF0u && (full || 16 * (t0 + j) + 4 * kq < PN)) ? yoff[mt] + 64u * j : 0xFFFFFFF0u;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), yrs, off, 0, 16 /* sc1 */);
          } else if (full || 16 * (t0 + j) + 4 * kq < PN) {
            *reinterpret_cast<float4*>(base[mt] + 16 * j) = v;
          }
#else
          // (non-temporal stores: qkv_news 0.26 vs 0.16 ms, profiles/r4q_proj_store_waves_ab.txt)
          if (full || 16 * (t0 + j) + 4 * kq < PN) *reinterpret_cast<float4*>(base[mt] + 16 * j) = v;
#endif
        }
      };
      // the last k-step tile by tile, each tile's stores issued behind the next
      // tile's MFMAs (the store bursts of all CUs at an item's end cost ~17 % of
      // the kernel; here they run under the MFMAs)
      auto kstep_final = [&](const frag (&a)[PMT][3], const frag (&bb)[C][NPL], auto p4c)
          __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < C; ++j) {
          if constexpr (H3) {
#pragma unroll
            for (int p = decltype(p4c)::value ? 0 : 1; p < 4; ++p)
#pragma unroll
              for (int mt = 0; mt < PMT; ++mt)
                mfma_h(bb[j][pw(p)], a[mt][pa(p)], mt, j);
          } else {
            constexpr int pa_[6] = {2, 1, 0, 1, 0, 0}, pb_[6] = {0, 1, 2, 0, 1, 0};
#pragma unroll
            for (int p = 0; p < 6; ++p)
#pragma unroll
              for (int mt = 0; mt < PMT; ++mt) mfma(a, bb, mt, j, pa_[p], pb_[p]);
          }
          if (j > 0) store_tile(j - 1);
          __builtin_amdgcn_sched_barrier(0);
        }
        store_tile(C - 1);
      };
      constexpr bool A2 = NW == 4;
      {
        frag a0[PMT][3], a1[PMT][3];
        if constexpr (A2) load_afrag(0, a0, p4c);
#pragma unroll
        for (int ks = 0; ks < PKS; ks += 2) {
          load_b(ks + 1, bvoff, b1);
          if constexpr (A2) load_afrag(ks + 1, a1, p4c);
          else load_afrag(ks, a0, p4c);
          __builtin_amdgcn_sched_barrier(0);
          kstep(a0, b0, p4c);
          __builtin_amdgcn_sched_barrier(0);
          if (ks == 0) { NRMS_PX_STAMP(1) }   // item setup + first k-step (B(0) / A fragment waits)
          if (ks + 2 < PKS) {
            load_b(ks + 2, bvoff, b0);
            if constexpr (A2) load_afrag(ks + 2, a0, p4c);
          } else {
            // unconditional (the last item reloads its own first k-step): behind a
            // branch, the waitcnt pass merged both paths into vmcnt(0) waits in
            // the last k-step, i.e. waited for these loads there
            load_b(0, bnext, b0);
          }
          if constexpr (!A2) load_afrag(ks + 1, a0, p4c);
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (A2) {
            if (ks + 2 < PKS) kstep(a1, b1, p4c);
            else kstep_final(a1, b1, p4c);
          } else {
            if (ks + 2 < PKS) kstep(a0, b1, p4c);
            else kstep_final(a0, b1, p4c);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int j = 0; j < C; ++j) bvoff[j] = bnext[j];
      NRMS_PX_STAMP(2)   // k-steps 1..9
      // the next row tile's A: loads in flight until the restage below
      ASrc an{zero_row, -1};
      if (restage) {
        an = a_resolve(rt + 1, an_id);
        load_a(an.p);
      }
      NRMS_PX_STAMP(3)   // epilogue stores issued
      if (restage) {
        __syncthreads();   // every wave is done with this A tile
        NRMS_PX_STAMP(4)   // barrier wait
        store_a(an.o);
        NRMS_PX_STAMP(5)   // A loads landed + split + LDS stores
        __syncthreads();
        NRMS_PX_STAMP(6)   // second barrier
      }
    }
  };
  auto run_w = [&](auto p4c) __attribute__((always_inline)) {
    if constexpr (NW == 4) run(std::integral_constant<int, PTW>{}, p4c);
    else if (w < 4) run(std::integral_constant<int, 3>{}, p4c);
    else run(std::integral_constant<int, 2>{}, p4c);
  };
  if (!H3 || p4) run_w(std::true_type{});
  else run_w(std::false_type{});
#ifdef NRMS_PX_TIMING
  if (lane == 0) {
    unsigned long long* dbg = reinterpret_cast<unsigned long long*>(const_cast<float*>(packed) + OFF_STAMP);
    for (int k = 0; k < 8; ++k) dbg[(blockIdx.x * NW + w) * 8 + k] = tacc[k];
  }
#endif
}

}  // namespace

size_t proj_x6_pack_floats() { return PACK_FLOATS; }

bool proj_x6_supported(int K, int N, const WeightRows& w) {
  return K == PK && N == PN && w.accumulate == 0 && gemm_arith() != NRMS_GEMM_F32;
}

int32_t launch_proj_x6_pack(const WeightRows& w0, float* d0, const WeightRows* w1, float* d1, bool h3,
                            hipStream_t s) {
  if (((uintptr_t)d0 % 16) || (d1 && ((uintptr_t)d1 % 16))) return NRMS_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(proj_x6_pack_kernel, dim3(h3 ? PACK_BLOCKS_H3 : PACK_BLOCKS, w1 ? 2 : 1), dim3(256), 0, s, w0,
                     w1 ? *w1 : w0, d0, d1 ? d1 : d0, h3 ? 1 : 0);
  return launch_status();
}

int32_t launch_forward_pack(const WeightRows& wn, float* pn, const WeightRows& wu, float* pu,
                            const float* news_wadd, float* news_ws, bool f16, const float* user_wadd,
                            float* user_ws, hipStream_t s, const tl::ClassifyJob* cls) {
  if (((uintptr_t)pn | (uintptr_t)pu) % 16) return NRMS_ERR_UNSUPPORTED;
  tl::ClassifyJob cj{};
  if (cls) cj = *cls;
  const int64_t blocks = 2 * (f16 ? PACK_BLOCKS_H3 : PACK_BLOCKS) + NEWS_ADD_BLOCKS +
                         (f16 ? pk::USER_H3_BLOCKS : USER_ADD_BLOCKS) + (cls ? cj.nblk : 0);
  if (blocks > INT32_MAX) return NRMS_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(forward_pack_kernel, dim3((unsigned)blocks), dim3(256), 0, s, wn, pn, wu, pu, news_wadd,
                     news_ws, f16 ? 1 : 0, user_wadd, user_ws, cj);
  return launch_status();
}

namespace {
// NRMS_PROJ_PRODUCTS=4: the split-f16 projection on four products for every
// column (A/B and the bitwise comparisons of tests/test_gpu_parity.py)
int proj_force4() {
  static const int v = [] {
    const char* e = env_knob("NRMS_PROJ_PRODUCTS");
    return (e && e[0] == '4') ? 1 : 0;
  }();
  return v;
}

template <bool SCATTER, bool H3>
void launch_proj_kernel(int64_t grid, const float* X, int64_t n_rows_x, ARows ar, const int64_t* row_ids, int64_t M,
                        const float* packed, float* Y, int64_t ldy, const int32_t* m_dev, const tl::TailJobs& tj,
                        hipStream_t s) {
#ifndef NRMS_PX_WAVES
#define NRMS_PX_WAVES 8
#endif
  constexpr int NW = NRMS_PX_WAVES;
  ensure_dynamic_lds(reinterpret_cast<const void*>(&proj_qkv_kernel<SCATTER, NW, H3>), (int)P_LDS);
  hipLaunchKernelGGL((proj_qkv_kernel<SCATTER, NW, H3>), dim3((unsigned)grid), dim3(64 * NW), P_LDS, s, X, n_rows_x,
                     ar, row_ids, M, packed, Y, ldy, m_dev, tj, proj_force4());
}
}  // namespace

int32_t launch_proj_x6(const float* X, int64_t n_rows_x, ARows ar, const int64_t* row_ids, int64_t M,
                       const float* packed, float* Y, int64_t ldy, const int32_t* m_dev, bool h3, hipStream_t s,
                       const tl::TailJobs* tail) {
  if (M == 0 && !tail) return NRMS_OK;
  if (((uintptr_t)X % 16) || ((uintptr_t)packed % 16) || ar.stride_row % 4 ||
      (ar.per_batch != INT64_MAX && ar.stride_batch % 4) || ldy < PN || ((uintptr_t)Y % 16) || ldy % 4)
    return NRMS_ERR_UNSUPPORTED;
  if (m_dev && !row_ids) return NRMS_ERR_INVALID_ARG;
  int dev = 0, n_cu = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) n_cu = v;
  }
  const int64_t items = (M + PM - 1) / PM * PNR;
  // persistent: one workgroup per CU (every CU with tail jobs: they are spread
  // over the grid)
  const int64_t grid = tail ? n_cu : (items < n_cu ? items : n_cu);
  const tl::TailJobs tj = tail ? *tail : tl::TailJobs{};
  if (m_dev) {
    if (h3) launch_proj_kernel<true, true>(grid, X, n_rows_x, ar, row_ids, M, packed, Y, ldy, m_dev, tj, s);
    else launch_proj_kernel<true, false>(grid, X, n_rows_x, ar, row_ids, M, packed, Y, ldy, m_dev, tj, s);
  } else {
    if (h3) launch_proj_kernel<false, true>(grid, X, n_rows_x, ar, row_ids, M, packed, Y, ldy, nullptr, tj, s);
    else launch_proj_kernel<false, false>(grid, X, n_rows_x, ar, row_ids, M, packed, Y, ldy, nullptr, tj, s);
  }
  return launch_status();
}

}  // namespace nrms
