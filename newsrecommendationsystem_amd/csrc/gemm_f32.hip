// fp32 MFMA GEMM Y = X[row(m)] · W^T + b for the NRMS projections:
//   * Q|K|V projection (multihead_self.py:53-58), N = 3D = 900, optional row
//     indirection so the A operand can be gathered straight from the
//     embedding table (DIRECT mode) or be the whole table (FOLDED mode);
//   * additive-attention projection (additive.py:35-38), N = Q = 200, with the
//     tanh(.)·q row reduction fused into the epilogue: the [rows, 200] tile
//     never leaves registers, only one score per row is written.
//
// gfx950 specifics: v_mfma_f32_16x16x4_f32 (exact fp32, 256 FLOP/clk/CU);
// 4 waves x (32 rows x 16·TN cols) per 128-row block; K staged through LDS in
// 32-deep chunks with register prefetch of the next chunk; each lane reads
// its A/B fragments with conflict-free ds_read_b128 (row stride 40 floats);
// XCD-aware block order so the column tiles of one row tile share an L2.
#include "nrms_common.hpp"

namespace nrms {
namespace {

constexpr int BM = 128;
constexpr int BK = 32;
constexpr int LDS_LD = 40;  // floats: ds_read_b128 fragment reads conflict-free, rows 16-B aligned
constexpr int kThreads = 256;

// K-permutation: MFMA step (c, t) gives lane group kq (= lane >> 4) the K index
// 16c + 4kq + t, so each lane fetches its four consecutive K values with one
// ds_read_b128; A and B use the same map, so every K term is summed once.
// One 128 x (16 TN) output tile at (m0, n0); As / Bs are the workgroup's LDS
// tiles (declared once by the kernel so both tile widths share them).
template <int TN, bool ADDITIVE>
__device__ __forceinline__ void gemm_tile(
    const float* __restrict__ X, int64_t n_rows_x, ARows ar, const int64_t* __restrict__ row_ids,
    int64_t M, int K, const WeightRows& wr, int N, float* __restrict__ Y, int64_t ldy,
    const float* __restrict__ qvec, float* __restrict__ score, int64_t m0, int n0,
    float* __restrict__ As, float* __restrict__ Bs) {
  constexpr int BN = 16 * TN;
  constexpr int A_PASSES = BM * BK / 4 / kThreads;              // 4
  constexpr int B_PASSES = (BN * BK / 4 + kThreads - 1) / kThreads;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lrow = tid >> 3, lc4 = tid & 7;

  // Staging sources: one A row and one W row per pass per thread.
  const float* a_src[A_PASSES];
  bool a_bad[A_PASSES];
#pragma unroll
  for (int p = 0; p < A_PASSES; ++p) {
    const int64_t m = m0 + lrow + 32 * p;
    a_src[p] = nullptr;
    a_bad[p] = false;
    if (m < M) {
      const int64_t r = row_ids ? row_ids[m] : m;
      if ((uint64_t)r < (uint64_t)n_rows_x) a_src[p] = X + ar.offset(r);
      else a_bad[p] = true;  // invalid id: the row becomes NaN
    }
  }
  const float* b_src[B_PASSES];
#pragma unroll
  for (int p = 0; p < B_PASSES; ++p) {
    const int n = n0 + lrow + 32 * p;
    b_src[p] = nullptr;
    if (lrow + 32 * p < BN && n < N) {
      const int seg = n / wr.seg_rows;
      b_src[p] = wr.w[seg] + (int64_t)(n - seg * wr.seg_rows) * K;
    }
  }

  float4 ra[A_PASSES], rb[B_PASSES];
  auto gload = [&](int kc) {
    const int k = kc * BK + lc4 * 4;
    const bool kin = k < K;
#pragma unroll
    for (int p = 0; p < A_PASSES; ++p)
      ra[p] = (a_src[p] && kin) ? *reinterpret_cast<const float4*>(a_src[p] + k)
                                : (a_bad[p] ? nan4() : make_float4(0.f, 0.f, 0.f, 0.f));
#pragma unroll
    for (int p = 0; p < B_PASSES; ++p)
      rb[p] = (b_src[p] && kin) ? *reinterpret_cast<const float4*>(b_src[p] + k)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto lstore = [&]() {
#pragma unroll
    for (int p = 0; p < A_PASSES; ++p)
      *reinterpret_cast<float4*>(&As[(lrow + 32 * p) * LDS_LD + lc4 * 4]) = ra[p];
#pragma unroll
    for (int p = 0; p < B_PASSES; ++p)
      if (lrow + 32 * p < BN)
        *reinterpret_cast<float4*>(&Bs[(lrow + 32 * p) * LDS_LD + lc4 * 4]) = rb[p];
  };

  floatx4 acc[2][TN];
#pragma unroll
  for (int ms = 0; ms < 2; ++ms)
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) acc[ms][tn] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int lm = lane & 15, kq = lane >> 4;
  const float* Aw = As + (wave * 32 + lm) * LDS_LD + 4 * kq;
  const float* Bw = Bs + lm * LDS_LD + 4 * kq;

  const int nk = (K + BK - 1) / BK;
  gload(0);
  lstore();
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    if (kc + 1 < nk) gload(kc + 1);
#pragma unroll
    for (int c = 0; c < BK / 16; ++c) {
      if (kc * BK + 16 * c >= K) break;   // K tail: the zero-padded half chunk (K = 300)
      const float4 a0 = *reinterpret_cast<const float4*>(Aw + 16 * c);
      const float4 a1 = *reinterpret_cast<const float4*>(Aw + 16 * LDS_LD + 16 * c);
      // B fragments two column tiles at a time: 4 independent accumulators per
      // k-step keep the MFMA pipe busy without holding all TN fragments live.
#pragma unroll
      for (int tn = 0; tn < TN; tn += 2) {
        const float4 b0 = *reinterpret_cast<const float4*>(Bw + tn * 16 * LDS_LD + 16 * c);
        if (tn + 1 < TN) {
          const float4 b1 = *reinterpret_cast<const float4*>(Bw + (tn + 1) * 16 * LDS_LD + 16 * c);
#define NRMS_MFMA4(F)                                                                             \
  acc[0][tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.F, b0.F, acc[0][tn], 0, 0, 0);             \
  acc[1][tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.F, b0.F, acc[1][tn], 0, 0, 0);             \
  acc[0][tn + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.F, b1.F, acc[0][tn + 1], 0, 0, 0);     \
  acc[1][tn + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.F, b1.F, acc[1][tn + 1], 0, 0, 0);
          NRMS_MFMA4(x) NRMS_MFMA4(y) NRMS_MFMA4(z) NRMS_MFMA4(w)
#undef NRMS_MFMA4
        } else {
#define NRMS_MFMA2(F)                                                                             \
  acc[0][tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.F, b0.F, acc[0][tn], 0, 0, 0);             \
  acc[1][tn] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.F, b0.F, acc[1][tn], 0, 0, 0);
          NRMS_MFMA2(x) NRMS_MFMA2(y) NRMS_MFMA2(z) NRMS_MFMA2(w)
#undef NRMS_MFMA2
        }
      }
    }
    __syncthreads();
    if (kc + 1 < nk) {
      lstore();
      __syncthreads();
    }
  }

  // C/D layout of 16x16 MFMA: col = lane & 15, row = (lane >> 4) * 4 + reg.
  const int64_t row_base = m0 + wave * 32 + kq * 4;
  if constexpr (!ADDITIVE) {
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int col = n0 + tn * 16 + lm;
      if (col >= N) continue;
      const int seg = col / wr.seg_rows;
      const float bias = wr.b[seg] ? wr.b[seg][col - seg * wr.seg_rows] : 0.f;
#pragma unroll
      for (int ms = 0; ms < 2; ++ms)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = row_base + ms * 16 + r;
          if (row < M) {
            float* yp = Y + row * ldy + col;
            *yp = (wr.accumulate ? *yp : 0.f) + acc[ms][tn][r] + bias;
          }
        }
    }
  } else {
    float qv[TN], bv[TN];
#pragma unroll
    for (int tn = 0; tn < TN; ++tn) {
      const int col = tn * 16 + lm;
      qv[tn] = col < N ? qvec[col] : 0.f;
      bv[tn] = col < N ? wr.b[0][col] : 0.f;
    }
#pragma unroll
    for (int ms = 0; ms < 2; ++ms)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float part = 0.f;
        const int64_t yrow = row_base + ms * 16 + r;
#pragma unroll
        for (int tn = 0; tn < TN; ++tn)
          if (tn * 16 + lm < N) {
            const float t = tanhf(acc[ms][tn][r] + bv[tn]);
            if (Y && yrow < M) Y[yrow * N + tn * 16 + lm] = t;   // training forward keeps y
            part = fmaf(qv[tn], t, part);
          }
        part += __shfl_xor(part, 1);
        part += __shfl_xor(part, 2);
        part += __shfl_xor(part, 4);
        part += __shfl_xor(part, 8);
        const int64_t row = row_base + ms * 16 + r;
        if (lm == 0 && row < M) score[row] = part;
      }
  }
}

// Column tiles of width 16 TN; when N is not a multiple of 16 TN the last
// column tile is TNT tiles wide (N = 900: 4 x 192 + 1 x 144), so no MFMA is
// spent on all-padding columns.
template <int TN, int TNT, bool ADDITIVE>
__global__ __launch_bounds__(kThreads, 2) void gemm_xwt_f32_kernel(
    const float* __restrict__ X, int64_t n_rows_x, ARows ar, const int64_t* __restrict__ row_ids,
    int64_t M, int K, WeightRows wr, int N, float* __restrict__ Y, int64_t ldy,
    const float* __restrict__ qvec, float* __restrict__ score, int n_col_tiles) {
  __shared__ __attribute__((aligned(16))) float As[BM * LDS_LD];
  __shared__ __attribute__((aligned(16))) float Bs[16 * TN * LDS_LD];
  const int wg = xcd_remap(blockIdx.x, gridDim.x);
  const int ct = wg % n_col_tiles;
  const int64_t m0 = (int64_t)(wg / n_col_tiles) * BM;
  const int n0 = ct * 16 * TN;
  if (TNT == TN || n0 + 16 * TN <= N)
    gemm_tile<TN, ADDITIVE>(X, n_rows_x, ar, row_ids, M, K, wr, N, Y, ldy, qvec, score, m0, n0, As, Bs);
  else
    gemm_tile<TNT, ADDITIVE>(X, n_rows_x, ar, row_ids, M, K, wr, N, Y, ldy, qvec, score, m0, n0, As, Bs);
}

// ---------------------------------------------------------------------------
// Split-bf16 (x6) variant of the store GEMM: every fp32 operand is split into
// hi + mid + lo bf16 planes (exact: 8 + 8 + 8 significand bits) while it is
// staged into LDS, and each 16x16 output tile accumulates the six products
// with plane indices i + j <= 2 on v_mfma_f32_16x16x32_bf16 (exact bf16
// products, fp32 accumulation). Dropped terms are < 2^-25 |a||b| per product:
// fp32-GEMM accuracy (tests compare against the fp64 oracle) at 6/16 of the
// f32-MFMA cycles.
// Block tile 64 x 192, K staged 32 deep (one bf16 k-step) with register
// prefetch of the next chunk; 4 waves as 2 (rows) x 2 (cols), wave tile
// 32 x (16 TNW); 148 VGPRs and 49 KB of LDS, so three workgroups share a CU
// and stage while the others compute (the 128-row tile at 236 VGPRs, two per
// CU, ran 3.5 % slower; 64 x 96 at four per CU no faster: its A tile is split
// ten times per row instead of five).
constexpr int XBM = 64;
constexpr int XBK = 32;
constexpr int XLD = 32;   // bf16 per LDS row (64 B, unpadded)
// The 16-B chunk kq of row r sits at chunk kq ^ xsw(r): with 64-B rows this
// makes every ds_read_b128 lane group of the 16x16x32 fragment reads hit 16
// distinct 16-B bank slots (groups {0-3,12-15,20-27}, ...: MI355X_MICROARCH.md
// §LDS), and each 16-lane ds_write_b64 group of the staging stores covers two
// whole rows = one 128-B bank window.
__device__ __forceinline__ int xsw(int r) { return ((r >> 3) & 1) << 1; }
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split4(const float4 v, bf16x4& h, bf16x4& m, bf16x4& l) {
  uint32_t h0, m0, l0, h1, m1, l1;
  split3x2(v.x, v.y, h0, m0, l0);
  split3x2(v.z, v.w, h1, m1, l1);
  h = __builtin_bit_cast(bf16x4, make_uint2(h0, h1));
  m = __builtin_bit_cast(bf16x4, make_uint2(m0, m1));
  l = __builtin_bit_cast(bf16x4, make_uint2(l0, l1));
}

// SCATTER: output row m goes to Y row row_ids[m] (row-list GEMM: the rows to
// project are listed, each written back in place).
template <int TNW, int BMT, bool SCATTER>
__device__ __forceinline__ void gemm_x6_tile(
    const float* __restrict__ X, int64_t n_rows_x, ARows ar, const int64_t* __restrict__ row_ids,
    int64_t M, int K, const WeightRows& wr, int N, float* __restrict__ Y, int64_t ldy,
    int64_t m0, int n0, __bf16* __restrict__ As, __bf16* __restrict__ Bs) {
  constexpr int BN = 32 * TNW;
  constexpr int A_PASSES = BMT * XBK / 4 / kThreads;              // 4 (BMT 128), 2 (64)
  constexpr int MT = BMT / 32;                                   // 16-row tiles per wave
  constexpr int B_PASSES = (BN * XBK / 4 + kThreads - 1) / kThreads;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int lrow = tid >> 3, lc4 = tid & 7;

  const float* a_src[A_PASSES];
  bool a_bad[A_PASSES];
#pragma unroll
  for (int p = 0; p < A_PASSES; ++p) {
    const int64_t m = m0 + lrow + 32 * p;
    a_src[p] = nullptr;
    a_bad[p] = false;
    if (m < M) {
      const int64_t r = row_ids ? row_ids[m] : m;
      if ((uint64_t)r < (uint64_t)n_rows_x) a_src[p] = X + ar.offset(r);
      else a_bad[p] = true;  // invalid id: the row becomes NaN
    }
  }
  const float* b_src[B_PASSES];
#pragma unroll
  for (int p = 0; p < B_PASSES; ++p) {
    const int n = n0 + lrow + 32 * p;
    b_src[p] = nullptr;
    if (lrow + 32 * p < BN && n < N) {
      const int seg = n / wr.seg_rows;
      b_src[p] = wr.w[seg] + (int64_t)(n - seg * wr.seg_rows) * K;
    }
  }

  float4 ra[A_PASSES], rb[B_PASSES];
  auto gload = [&](int kc) {
    const int k = kc * XBK + lc4 * 4;
    const bool kin = k < K;
#pragma unroll
    for (int p = 0; p < A_PASSES; ++p)
      ra[p] = (a_src[p] && kin) ? *reinterpret_cast<const float4*>(a_src[p] + k)
                                : (a_bad[p] ? nan4() : make_float4(0.f, 0.f, 0.f, 0.f));
#pragma unroll
    for (int p = 0; p < B_PASSES; ++p)
      rb[p] = (b_src[p] && kin) ? *reinterpret_cast<const float4*>(b_src[p] + k)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
  };
  auto lstore = [&]() {
#pragma unroll
    for (int p = 0; p < A_PASSES; ++p) {
      bf16x4 h, m, l;
      split4(ra[p], h, m, l);
      const int r = lrow + 32 * p;
      __bf16* d = As + r * XLD + (((lc4 >> 1) ^ xsw(r)) << 3) + (lc4 & 1) * 4;
      *reinterpret_cast<bf16x4*>(d) = h;
      *reinterpret_cast<bf16x4*>(d + BMT * XLD) = m;
      *reinterpret_cast<bf16x4*>(d + 2 * BMT * XLD) = l;
    }
#pragma unroll
    for (int p = 0; p < B_PASSES; ++p)
      if (lrow + 32 * p < BN) {
        bf16x4 h, m, l;
        split4(rb[p], h, m, l);
        const int r = lrow + 32 * p;
        __bf16* d = Bs + r * XLD + (((lc4 >> 1) ^ xsw(r)) << 3) + (lc4 & 1) * 4;
        *reinterpret_cast<bf16x4*>(d) = h;
        *reinterpret_cast<bf16x4*>(d + BN * XLD) = m;
        *reinterpret_cast<bf16x4*>(d + 2 * BN * XLD) = l;
      }
  };

  floatx4 acc[MT][TNW];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < TNW; ++nt) acc[mt][nt] = floatx4{0.f, 0.f, 0.f, 0.f};
  // N tiles of this wave past N hold no output: skip their MFMAs (wave-uniform)
  int nt_live = TNW;
  {
    const int first = n0 + 16 * TNW * wn;
    const int live = (N - first + 15) / 16;
    nt_live = live < 0 ? 0 : (live < TNW ? live : TNW);
  }

  const int lm = lane & 15, kq = lane >> 4;
  // rows 64 wm + 16 mt + lm and 16 TNW wn + 16 nt + lm all have xsw == xsw(lm)
  const __bf16* Aw = As + ((BMT / 2) * wm + lm) * XLD + ((kq ^ xsw(lm)) << 3);
  const __bf16* Bw = Bs + (16 * TNW * wn + lm) * XLD + ((kq ^ xsw(lm)) << 3);

  const int nk = (K + XBK - 1) / XBK;
  gload(0);
  lstore();
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    if (kc + 1 < nk) gload(kc + 1);
    bf16x8 a[MT][3];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        a[mt][pl] = *reinterpret_cast<const bf16x8*>(Aw + pl * BMT * XLD + 16 * mt * XLD);
#pragma unroll
    for (int nt = 0; nt < TNW; ++nt) {
      if (nt >= nt_live) break;
      bf16x8 b[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        b[pl] = *reinterpret_cast<const bf16x8*>(Bw + pl * BN * XLD + 16 * nt * XLD);
      // the six products with i + j <= 2, smallest first
#define NRMS_X6(PA, PB)                                                                             \
  _Pragma("unroll") for (int mt = 0; mt < MT; ++mt)                                                  \
      acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt][PA], b[PB], acc[mt][nt], 0, 0, 0);
      NRMS_X6(2, 0) NRMS_X6(1, 1) NRMS_X6(0, 2) NRMS_X6(1, 0) NRMS_X6(0, 1) NRMS_X6(0, 0)
#undef NRMS_X6
    }
    __syncthreads();
    if (kc + 1 < nk) {
      lstore();
      __syncthreads();
    }
  }

  // C/D layout of 16x16 MFMA: col = lane & 15, row = (lane >> 4) * 4 + reg.
  const int64_t row_base = m0 + (BMT / 2) * wm + kq * 4;
#pragma unroll
  for (int nt = 0; nt < TNW; ++nt) {
    const int col = n0 + 16 * TNW * wn + 16 * nt + lm;
    if (col >= N) continue;
    const int seg = col / wr.seg_rows;
    const float bias = wr.b[seg] ? wr.b[seg][col - seg * wr.seg_rows] : 0.f;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t row = row_base + 16 * mt + r;
        if (row < M) {
          float* yp = Y + (SCATTER ? row_ids[row] : row) * ldy + col;
          *yp = (wr.accumulate ? *yp : 0.f) + acc[mt][nt][r] + bias;
        }
      }
  }
}

// 192-wide column tiles; a last partial tile of <= 160 columns (N = 900:
// 4 x 192 + 132) runs the 160-wide instantiation so its two wave columns
// stay balanced (5 + 4 live N tiles instead of 6 + 3).
// Row-list mode (SCATTER): row_ids lists the rows to project, m_dev their
// count (device memory, written by an earlier launch; the grid is sized for
// M rows and the blocks past the count exit at once).
template <bool SCATTER>
__global__ __launch_bounds__(kThreads, 3) void gemm_x6_kernel(
    const float* __restrict__ X, int64_t n_rows_x, ARows ar, const int64_t* __restrict__ row_ids,
    int64_t M, int K, WeightRows wr, int N, float* __restrict__ Y, int64_t ldy, int n_col_tiles,
    const int32_t* __restrict__ m_dev) {
  __shared__ __attribute__((aligned(16))) __bf16 As[3 * XBM * XLD];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[3 * 192 * XLD];
  // list mode: only the first ceil(count / 64) row tiles are live; the blocks
  // past them exit, and the XCD remap runs over the live range only (over the
  // whole grid it would pack every live tile onto the first XCDs)
  int nwg = gridDim.x;
  if constexpr (SCATTER) {
    const int64_t mc = *m_dev;
    M = mc < M ? mc : M;
    nwg = (int)((M + XBM - 1) / XBM) * n_col_tiles;
    if ((int)blockIdx.x >= nwg) return;
  }
  const int wg = xcd_remap(blockIdx.x, nwg);
  const int ct = wg % n_col_tiles;
  const int64_t m0 = (int64_t)(wg / n_col_tiles) * XBM;
  const int n0 = ct * 192;
  if (N - n0 > 160)
    gemm_x6_tile<6, XBM, SCATTER>(X, n_rows_x, ar, row_ids, M, K, wr, N, Y, ldy, m0, n0, As, Bs);
  else
    gemm_x6_tile<5, XBM, SCATTER>(X, n_rows_x, ar, row_ids, M, K, wr, N, Y, ldy, m0, n0, As, Bs);
}

constexpr int TN_STORE = 12;     // BN = 192: N = 900 -> 4 column tiles of 192 + one of 144
constexpr int TN_STORE_TAIL = 9;
constexpr int TN_ADDITIVE = 13;  // BN = 208 >= Q = 200: one column tile

}  // namespace

int32_t launch_gemm_store(const float* X, int64_t n_rows_x, const int64_t* row_ids, int64_t M,
                          int K, const WeightRows& w, int N, float* Y, int64_t ldy,
                          hipStream_t s) {
  return launch_gemm_store_rows(X, n_rows_x, contiguous_rows(K), row_ids, M, K, w, N, Y, ldy, s);
}

int32_t launch_gemm_store_rows(const float* X, int64_t n_rows_x, ARows ar, const int64_t* row_ids,
                               int64_t M, int K, const WeightRows& w, int N, float* Y,
                               int64_t ldy, hipStream_t s) {
  if (M == 0) return NRMS_OK;
  // float4 A loads: every row start must stay 16-B aligned
  if (K % 4 != 0 || ((uintptr_t)X % 16) != 0 || ar.stride_row % 4 != 0 ||
      (ar.per_batch != INT64_MAX && ar.stride_batch % 4 != 0))
    return NRMS_ERR_UNSUPPORTED;
  for (int i = 0; i < w.nseg; ++i)
    if (((uintptr_t)w.w[i] % 16) != 0) return NRMS_ERR_UNSUPPORTED;
  if (gemm_arith() != NRMS_GEMM_F32) {
    // 192-wide column tiles; a last partial tile of <= 160 columns runs the
    // TNW = 5 instantiation (N = 900: 4 x 192 + 132)
    const int nct = (N + 191) / 192;
    const int64_t nrt = (M + XBM - 1) / XBM;
    const int64_t blocks = nrt * nct;
    if (blocks > INT32_MAX) return NRMS_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(gemm_x6_kernel<false>, dim3((unsigned)blocks), dim3(kThreads), 0, s, X, n_rows_x,
                       ar, row_ids, M, K, w, N, Y, ldy, nct, (const int32_t*)nullptr);
    return launch_status();
  }
  const int nct = (N + 16 * TN_STORE - 1) / (16 * TN_STORE);
  const int64_t nrt = (M + BM - 1) / BM;
  const int64_t blocks = nrt * nct;
  if (blocks > INT32_MAX) return NRMS_ERR_UNSUPPORTED;
  // the narrow last tile covers N = 900's remainder (132 columns); for other N
  // fall back to full-width tiles
  const int rem = N % (16 * TN_STORE);
  if (rem > 0 && rem <= 16 * TN_STORE_TAIL)
    hipLaunchKernelGGL((gemm_xwt_f32_kernel<TN_STORE, TN_STORE_TAIL, false>), dim3((unsigned)blocks),
                       dim3(kThreads), 0, s, X, n_rows_x, ar, row_ids, M, K, w, N, Y, ldy,
                       (const float*)nullptr, (float*)nullptr, nct);
  else
    hipLaunchKernelGGL((gemm_xwt_f32_kernel<TN_STORE, TN_STORE, false>), dim3((unsigned)blocks),
                       dim3(kThreads), 0, s, X, n_rows_x, ar, row_ids, M, K, w, N, Y, ldy,
                       (const float*)nullptr, (float*)nullptr, nct);
  return launch_status();
}

int32_t launch_gemm_store_list(const float* X, int64_t n_rows_x, const int64_t* rows,
                               const int32_t* count_dev, int64_t max_rows, int K, const WeightRows& w,
                               int N, float* Y, int64_t ldy, hipStream_t s) {
  if (max_rows == 0) return NRMS_OK;
  if (K % 4 != 0 || ((uintptr_t)X % 16) != 0 || !rows || !count_dev) return NRMS_ERR_UNSUPPORTED;
  for (int i = 0; i < w.nseg; ++i)
    if (((uintptr_t)w.w[i] % 16) != 0) return NRMS_ERR_UNSUPPORTED;
  if (gemm_arith() == NRMS_GEMM_F32) return NRMS_ERR_UNSUPPORTED;   // callers project every row instead
  const int nct = (N + 191) / 192;
  const int64_t blocks = (max_rows + XBM - 1) / XBM * nct;
  if (blocks > INT32_MAX) return NRMS_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(gemm_x6_kernel<true>, dim3((unsigned)blocks), dim3(kThreads), 0, s, X, n_rows_x,
                     contiguous_rows(K), rows, max_rows, K, w, N, Y, ldy, nct, count_dev);
  return launch_status();
}

int32_t launch_gemm_store_f32(const float* X, int64_t M, int K, const WeightRows& w, int N, float* Y,
                              int64_t ldy, hipStream_t s) {
  if (M == 0) return NRMS_OK;
  // the training dX GEMMs: split-bf16 x6 like the forward projections unless
  // exact f32 MFMA is selected (NRMS_GEMM=f32)
  if (gemm_arith() != NRMS_GEMM_F32) return launch_gemm_store(X, M, nullptr, M, K, w, N, Y, ldy, s);
  if (K % 4 != 0 || ((uintptr_t)X % 16) != 0) return NRMS_ERR_UNSUPPORTED;
  for (int i = 0; i < w.nseg; ++i)
    if (((uintptr_t)w.w[i] % 16) != 0) return NRMS_ERR_UNSUPPORTED;
  const int nct = (N + 16 * TN_STORE - 1) / (16 * TN_STORE);
  const int64_t blocks = (M + BM - 1) / BM * nct;
  if (blocks > INT32_MAX) return NRMS_ERR_UNSUPPORTED;
  hipLaunchKernelGGL((gemm_xwt_f32_kernel<TN_STORE, TN_STORE, false>), dim3((unsigned)blocks),
                     dim3(kThreads), 0, s, X, M, contiguous_rows(K), (const int64_t*)nullptr, M, K,
                     w, N, Y, ldy, (const float*)nullptr, (float*)nullptr, nct);
  return launch_status();
}

int32_t launch_gemm_additive_score(const float* X, int64_t M, int K, const float* W,
                                   const float* b, const float* q, int N, float* score,
                                   hipStream_t s) {
  return launch_gemm_additive_score_y(X, M, K, W, b, q, N, score, nullptr, s);
}

int32_t launch_gemm_additive_score_y(const float* X, int64_t M, int K, const float* W,
                                     const float* b, const float* q, int N, float* score,
                                     float* y_out, hipStream_t s) {
  if (M == 0) return NRMS_OK;
  if (N > 16 * TN_ADDITIVE) return NRMS_ERR_UNSUPPORTED;
  if (K % 4 != 0 || ((uintptr_t)X % 16) != 0 || ((uintptr_t)W % 16) != 0)
    return NRMS_ERR_UNSUPPORTED;
  WeightRows w{};
  w.w[0] = W;
  w.b[0] = b;
  w.seg_rows = N;
  w.nseg = 1;
  const int64_t blocks = (M + BM - 1) / BM;
  if (blocks > INT32_MAX) return NRMS_ERR_UNSUPPORTED;
  hipLaunchKernelGGL((gemm_xwt_f32_kernel<TN_ADDITIVE, TN_ADDITIVE, true>), dim3((unsigned)blocks),
                     dim3(kThreads), 0, s, X, M, contiguous_rows(K), (const int64_t*)nullptr, M,
                     K, w, N, y_out, (int64_t)N, q, score, 1);
  return launch_status();
}

}  // namespace nrms
