// Fused NewsEncoder tail: raw-exp MHSA -> additive projection -> tanh·q
// scores -> softmax over tokens -> pooled news vector, for 4 titles per
// workgroup, in one launch (src/model/NRMS/news_encoder.py:42-47,
// multihead_self.py:15-23,74-75, additive.py:35-52).
//
// Why fused: the separate path writes the [titles·20, 300] context to HBM
// and reads it back twice (GEMM A operand, pooling). Here the additive GEMM
// consumes the context head-group by head-group straight from LDS:
//
//   for g in 5 head groups (3 heads = 60 context columns = 15 MFMA k-steps):
//     stage K|V slices of the group for the block's 80 token rows (LDS)
//     attention: one (row, head) task per lane -> 20 context values,
//                written to the LDS A-buffer [80][62] (and to the context
//                scratch in HBM, needed once more by the pooling below)
//     MFMA: acc[80 x 208] += A[80 x 60] · Wa[:, 60g:60g+60]^T
//           (v_mfma_f32_16x16x4_f32, K-permutation: lane group kq owns
//           columns 15kq..15kq+14 of the group, B fragments pre-packed so
//           every lane loads 4 x dwordx4)
//   epilogue: scores[row] = sum_n q[n] tanh(acc[row][n] + b[n]) (the 80 x 200
//             tile never leaves registers), softmax per title, pooling from
//             the block's own just-written context rows (L2-resident).
//
// 4 waves, ~59 KB LDS -> 2 workgroups per CU, so one block's attention
// (VALU/LDS) overlaps the other block's MFMA phase.
//
// Output tile ownership (13 N-tiles x 5 M-tiles = 65 16x16 tiles): wave w
// owns N-tiles 3w..3w+2 for all 5 M-tiles, plus N-tile 12 (columns 192..207,
// 8 valid) for M-tile w; wave 0 also takes (M-tile 4, N-tile 12): 17/16/16/16.
#include "nrms_common.hpp"

namespace nrms {
namespace {

constexpr int FT = 4;                // titles per workgroup
constexpr int FL = 20;               // tokens per title (config.num_words_title)
constexpr int FROWS = FT * FL;       // 80 token rows
constexpr int FD = 300, FH = 15, FDK = 20, FQ = 200;
constexpr int FG = 3;                // heads per group
constexpr int FNG = FH / FG;         // 5 groups
constexpr int FGK = FG * FDK;        // 60 context columns per group
constexpr int FKS = FGK / 4;         // 15 MFMA k-steps per group
constexpr int FNT = 13;              // N tiles of 16 (208 >= Q)
constexpr int FMT = FROWS / 16;      // 5 M tiles
constexpr int SA = 62;               // A-buffer row stride: b32 fragment reads conflict-free
constexpr int KVW = FG * 2 * FDK;    // 120 floats of K|V per row per group
constexpr int NTHR = 256;
constexpr int LDS_FLOATS = FROWS * SA + FROWS * KVW + 4 * FROWS + FROWS;
constexpr size_t LDS_BYTES = LDS_FLOATS * sizeof(float) + FROWS * sizeof(int64_t);

static_assert(FD == FH * FDK && FH % FG == 0 && FGK % 4 == 0, "geometry");

// WaP[g][nt][lane][16]: the B fragment of k-step s for lane (n = lane & 15,
// kq = lane >> 4) = Wa[16 nt + n][60 g + 15 kq + s] (0 beyond Q or s = 15).
__global__ __launch_bounds__(256) void pack_additive_b_kernel(const float* __restrict__ Wa,
                                                              float* __restrict__ WaP) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= FNG * FNT * 64 * 16) return;
  const int s = idx & 15;
  const int lane = (idx >> 4) & 63;
  const int nt = (idx >> 10) % FNT;
  const int g = (idx >> 10) / FNT;
  const int n = 16 * nt + (lane & 15);
  const int k = FGK * g + 15 * (lane >> 4) + s;
  WaP[idx] = (s < FKS && n < FQ) ? Wa[n * FD + k] : 0.f;
}

__global__ __launch_bounds__(NTHR, 2) void fused_news_kernel(
    const float* __restrict__ qkv, int64_t n_rows, const int64_t* __restrict__ ids_a,
    int64_t n_seq_a, const int64_t* __restrict__ ids_b, int64_t n_titles,
    const float* __restrict__ WaP, const float* __restrict__ b_add,
    const float* __restrict__ q_add, float* __restrict__ ctx_g, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* A = lds;                          // [80][SA]
  float* KV = A + FROWS * SA;              // [80][3][K20|V20]
  float* part = KV + FROWS * KVW;          // [4][80]
  float* wsm = part + 4 * FROWS;           // [80] scores, then softmax weights
  int64_t* rowidx = reinterpret_cast<int64_t*>(wsm + FROWS);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t title0 = (int64_t)blockIdx.x * FT;

  if (tid < FROWS) {
    const int t = tid / FL, i = tid - t * FL;
    const int64_t s = title0 + t;
    int64_t r = -2;  // padding title beyond n_titles
    if (s < n_titles) {
      if (ids_a) {
        const int64_t* ids = (s < n_seq_a || ids_b == nullptr) ? ids_a + s * FL : ids_b + (s - n_seq_a) * FL;
        const int64_t id = ids[i];
        r = ((uint64_t)id < (uint64_t)n_rows) ? id : -1;
      } else {
        r = s * FL + i;
      }
    }
    rowidx[tid] = r;
  }

  floatx4 accA[FMT][3], accX[2];
#pragma unroll
  for (int mt = 0; mt < FMT; ++mt)
#pragma unroll
    for (int j = 0; j < 3; ++j) accA[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};
  accX[0] = accX[1] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int lm = lane & 15, kq = lane >> 4;
  const float rs = 1.0f / sqrtf((float)FDK);
  __syncthreads();

  for (int g = 0; g < FNG; ++g) {
    // ---- stage K|V slices of this head group: 80 rows x 3 heads x 10 float4
    for (int e = tid; e < FROWS * FG * 10; e += NTHR) {
      const int r = e / (FG * 10);
      const int rem = e - r * (FG * 10);
      const int hl = rem / 10, c = rem - hl * 10;
      const int h = FG * g + hl;
      const int64_t row = rowidx[r];
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row >= 0) {
        const int col = (c < 5 ? FD + FDK * h + 4 * c : 2 * FD + FDK * h + 4 * (c - 5));
        v = *reinterpret_cast<const float4*>(qkv + row * (3 * FD) + col);
      } else if (row == -1) {
        v = nan4();
      }
      *reinterpret_cast<float4*>(KV + (r * FG + hl) * 40 + 4 * c) = v;
    }
    // ---- B fragments of this group for the wave's N tiles (global, L2-resident)
    float bA[3][16], bX[16];
    {
      const float* base = WaP + (size_t)g * FNT * 64 * 16;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const float4* p = reinterpret_cast<const float4*>(base + ((3 * wave + j) * 64 + lane) * 16);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float4 v = p[c];
          bA[j][4 * c] = v.x; bA[j][4 * c + 1] = v.y; bA[j][4 * c + 2] = v.z; bA[j][4 * c + 3] = v.w;
        }
      }
      const float4* p = reinterpret_cast<const float4*>(base + (12 * 64 + lane) * 16);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float4 v = p[c];
        bX[4 * c] = v.x; bX[4 * c + 1] = v.y; bX[4 * c + 2] = v.z; bX[4 * c + 3] = v.w;
      }
    }
    __syncthreads();

    // ---- attention: task (head hl, row r); 240 of 256 lanes busy
    if (tid < FG * FROWS) {
      const int hl = tid / FROWS, r = tid - hl * FROWS;
      const int t = r / FL, i = r - t * FL;
      const int h = FG * g + hl;
      const int64_t row = rowidx[r];
      float ctxv[FDK];
      if (row == -2) {
#pragma unroll
        for (int d = 0; d < FDK; ++d) ctxv[d] = 0.f;
      } else {
        float q[FDK];
        if (row >= 0) {
          const float4* qp = reinterpret_cast<const float4*>(qkv + row * (3 * FD) + FDK * h);
#pragma unroll
          for (int c = 0; c < FDK / 4; ++c) {
            const float4 v = qp[c];
            q[4 * c] = v.x; q[4 * c + 1] = v.y; q[4 * c + 2] = v.z; q[4 * c + 3] = v.w;
          }
        } else {
#pragma unroll
          for (int d = 0; d < FDK; ++d) q[d] = qnan();
        }
        const float* kvt = KV + (FL * t * FG + hl) * 40;   // row j of title t: + j * KVW
        float e[FL];
        float sum = 0.f;
#pragma unroll
        for (int j = 0; j < FL; ++j) {
          const float4* kr = reinterpret_cast<const float4*>(kvt + j * KVW);
          float d = 0.f;
#pragma unroll
          for (int c = 0; c < FDK / 4; ++c) {
            const float4 k4 = kr[c];
            d = fmaf(q[4 * c], k4.x, d);
            d = fmaf(q[4 * c + 1], k4.y, d);
            d = fmaf(q[4 * c + 2], k4.z, d);
            d = fmaf(q[4 * c + 3], k4.w, d);
          }
          e[j] = expf(d * rs);
          sum += e[j];
        }
        const float inv = 1.0f / (sum + 1e-8f);
#pragma unroll
        for (int d = 0; d < FDK; ++d) ctxv[d] = 0.f;
#pragma unroll
        for (int j = 0; j < FL; ++j) {
          const float a = e[j] * inv;
          const float4* vr = reinterpret_cast<const float4*>(kvt + j * KVW + FDK);
#pragma unroll
          for (int c = 0; c < FDK / 4; ++c) {
            const float4 v4 = vr[c];
            ctxv[4 * c] = fmaf(a, v4.x, ctxv[4 * c]);
            ctxv[4 * c + 1] = fmaf(a, v4.y, ctxv[4 * c + 1]);
            ctxv[4 * c + 2] = fmaf(a, v4.z, ctxv[4 * c + 2]);
            ctxv[4 * c + 3] = fmaf(a, v4.w, ctxv[4 * c + 3]);
          }
        }
        float4* cg = reinterpret_cast<float4*>(ctx_g + ((title0 + t) * FL + i) * FD + FDK * h);
#pragma unroll
        for (int c = 0; c < FDK / 4; ++c)
          cg[c] = make_float4(ctxv[4 * c], ctxv[4 * c + 1], ctxv[4 * c + 2], ctxv[4 * c + 3]);
      }
      float2* ap = reinterpret_cast<float2*>(A + r * SA + FDK * hl);
#pragma unroll
      for (int c = 0; c < FDK / 2; ++c) ap[c] = make_float2(ctxv[2 * c], ctxv[2 * c + 1]);
    }
    __syncthreads();

    // ---- MFMA over the group's 60 context columns
    const float* Aw = A + lm * SA + 15 * kq;
#pragma unroll
    for (int s = 0; s < FKS; ++s) {
      float a[FMT];
#pragma unroll
      for (int mt = 0; mt < FMT; ++mt) a[mt] = Aw[16 * mt * SA + s];
      const float ax0 = Aw[16 * wave * SA + s];
#pragma unroll
      for (int mt = 0; mt < FMT; ++mt)
#pragma unroll
        for (int j = 0; j < 3; ++j)
          accA[mt][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt], bA[j][s], accA[mt][j], 0, 0, 0);
      accX[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(ax0, bX[s], accX[0], 0, 0, 0);
      if (wave == 0)
        accX[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[FMT - 1], bX[s], accX[1], 0, 0, 0);
    }
    __syncthreads();  // A / KV are restaged by the next group
  }

  // ---- epilogue: per-row partial scores over the wave's columns
  float qv[3], bv[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int col = 16 * (3 * wave + j) + lm;
    qv[j] = q_add[col];
    bv[j] = b_add[col];
  }
  const int colx = 192 + lm;
  const bool xok = colx < FQ;
  const float qx = xok ? q_add[colx] : 0.f, bx = xok ? b_add[colx] : 0.f;
#pragma unroll
  for (int mt = 0; mt < FMT; ++mt) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float p = 0.f;
#pragma unroll
      for (int j = 0; j < 3; ++j) p = fmaf(qv[j], tanhf(accA[mt][j][r] + bv[j]), p);
      if (xok && mt == wave) p = fmaf(qx, tanhf(accX[0][r] + bx), p);
      if (xok && wave == 0 && mt == FMT - 1) p = fmaf(qx, tanhf(accX[1][r] + bx), p);
      p += __shfl_xor(p, 1);
      p += __shfl_xor(p, 2);
      p += __shfl_xor(p, 4);
      p += __shfl_xor(p, 8);
      if (lm == 0) part[wave * FROWS + 16 * mt + 4 * kq + r] = p;
    }
  }
  __syncthreads();
  if (tid < FROWS) wsm[tid] = part[tid] + part[FROWS + tid] + part[2 * FROWS + tid] + part[3 * FROWS + tid];
  __syncthreads();
  {
    // softmax over each title's 20 scores (additive.py:37-39): wave t <-> title t
    const int t = wave;
    const float v = lane < FL ? wsm[FL * t + lane] : -INFINITY;
    const float m = wave_max_nan(v);
    const float e = lane < FL ? expf(v - m) : 0.f;
    const float sum = wave_sum(e);
    __syncthreads();
    if (lane < FL) wsm[FL * t + lane] = e / sum;
  }
  __syncthreads();
  // ---- pooling (additive.py:51-52) from this block's context rows
  for (int idx = tid; idx < FT * (FD / 4); idx += NTHR) {
    const int t = idx / (FD / 4), c = idx - t * (FD / 4);
    const int64_t s = title0 + t;
    if (s >= n_titles) continue;
    const float4* xr = reinterpret_cast<const float4*>(ctx_g + s * FL * FD) + c;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int i = 0; i < FL; ++i) {
      const float w = wsm[FL * t + i];
      const float4 x = xr[i * (FD / 4)];
      acc.x = fmaf(w, x.x, acc.x);
      acc.y = fmaf(w, x.y, acc.y);
      acc.z = fmaf(w, x.z, acc.z);
      acc.w = fmaf(w, x.w, acc.w);
    }
    reinterpret_cast<float4*>(out + s * FD)[c] = acc;
  }
}

}  // namespace

size_t fused_news_packed_b_floats() { return (size_t)FNG * FNT * 64 * 16; }

bool fused_news_supported(int L, int D, int H, int Q) {
  return L == FL && D == FD && H == FH && Q == FQ;
}

int32_t launch_fused_news(const float* qkv, int64_t n_rows, const int64_t* ids_a, int64_t n_seq_a,
                          const int64_t* ids_b, int64_t n_titles, const float* w_add,
                          const float* b_add, const float* q_add, float* wap, float* ctx,
                          float* out, hipStream_t s) {
  if (n_titles == 0) return NRMS_OK;
  if (((uintptr_t)qkv | (uintptr_t)ctx | (uintptr_t)out | (uintptr_t)wap) % 16) return NRMS_ERR_UNSUPPORTED;
  const int npk = FNG * FNT * 64 * 16;
  hipLaunchKernelGGL(pack_additive_b_kernel, dim3((npk + 255) / 256), dim3(256), 0, s, w_add, wap);
  if (int32_t st = launch_status()) return st;
  const int64_t blocks = (n_titles + FT - 1) / FT;
  if (blocks > INT32_MAX) return NRMS_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(fused_news_kernel, dim3((unsigned)blocks), dim3(NTHR), LDS_BYTES, s, qkv,
                     n_rows, ids_a, n_seq_a, ids_b, n_titles, wap, b_add, q_add, ctx, out);
  return launch_status();
}

}  // namespace nrms
