// Fused NewsEncoder tail: raw-exp MHSA -> additive projection -> tanh·q
// scores -> softmax over tokens -> pooled news vector, in one persistent
// launch (src/model/NRMS/news_encoder.py:42-47, multihead_self.py:15-23,74-75,
// additive.py:35-52).
//
// Work item = (title group of 4 titles = 80 token rows, head group g of 3
// heads = 60 context columns). Each workgroup (8 waves, one per CU) walks its
// title groups; per title group it runs the 5 head groups through a
// two-stage software pipeline with role-specialised waves:
//
//   producer waves 4-7 (VALU + LDS): first issue the LDS-DMA gather
//       (global_load_lds_dwordx4, no registers) of the Q|K|V slices of item
//       s+1 into QKV[(s+1) % 2]; then attention for item s from QKV[s % 2] —
//       one (row, head) task per lane: 20 raw exps (v_exp_f32 of the
//       pre-scaled score, no max subtraction, as the reference) kept in
//       registers, then the context slice -> LDS A-buffer[s % 2] (and the
//       context scratch in HBM, read once more for pooling). The DMA lands
//       behind the attention and is retired by the step's barrier.
//   consumer waves 0-3 (MFMA): acc[80 x 208] += A[(s-1) % 2][80 x 60] ·
//       Wa[:, 60g:60g+60]^T with v_mfma_f32_16x16x4_f32; after the last head
//       group, tanh(acc + b)·q row partials -> LDS, and one step later the
//       per-title softmax and the pooling (wave t <-> title t).
//
// One workgroup barrier per step. Every SIMD hosts one producer and one
// consumer wave, so the VALU/LDS attention of item s overlaps the MFMA work of
// item s-1 (MI355X_MICROARCH.md "Two waves per SIMD"). The [80 x 200] additive
// tile never leaves registers; the context never makes an HBM round trip
// before the additive GEMM.
//
// Output tile ownership (13 N-tiles x 5 M-tiles of 16x16): consumer wave w
// owns N-tiles 3w..3w+2 for all 5 M-tiles plus (M-tile w, N-tile 12); wave 0
// also (M-tile 4, N-tile 12): 17/16/16/16 tiles.
#include "nrms_common.hpp"

#include <cstdlib>

namespace nrms {
namespace {

constexpr int FT = 4;                // titles per group
constexpr int FL = 20;               // tokens per title (config.num_words_title)
constexpr int FROWS = FT * FL;       // 80 token rows
constexpr int FD = 300, FH = 15, FDK = 20, FQ = 200;
constexpr int FG = 3;                // heads per head group
constexpr int FNG = FH / FG;         // 5 head groups
constexpr int FGK = FG * FDK;        // 60 context columns per head group
constexpr int FKS = FGK / 4;         // 15 MFMA k-steps per head group
constexpr int FNT = 13;              // N tiles of 16 (208 >= Q)
constexpr int FMT = FROWS / 16;      // 5 M tiles
constexpr int SA = 62;               // A-buffer row stride: b32 fragment reads conflict-free
constexpr int HW = 3 * FDK;          // 60 floats: q|k|v of one (row, head)
constexpr int RW = FG * HW;          // 180 floats of Q|K|V per row per head group
constexpr int NTHR = 512;
constexpr int A_FL = FROWS * SA;     // 4960
constexpr int KV_FL = FROWS * RW;    // 14400 (57.6 KB)
constexpr int KV_F4 = KV_FL / 4;     // 3600 float4 = 56.25 LDS-DMA wave instructions
constexpr int LDS_FLOATS = 2 * A_FL + 2 * KV_FL + 4 * FROWS + 2 * 2 * FROWS + 2 * FROWS;  // + rowptr[2][80] (u64) + wsm[2][80]
constexpr int SPECIAL_FLOATS = 2 * 3 * FD;   // a zero row and a NaN row (q|k|v width)
constexpr size_t LDS_BYTES = LDS_FLOATS * sizeof(float);

static_assert(FD == FH * FDK && FH % FG == 0 && FGK % 4 == 0, "geometry");
static_assert(LDS_BYTES <= 160 * 1024, "LDS");

// WaP[g][nt][lane][16]: the B fragment of k-step s for lane (n = lane & 15,
// kq = lane >> 4) = Wa[16 nt + n][60 g + 15 kq + s] (0 beyond Q or s = 15).
__global__ __launch_bounds__(256) void pack_additive_b_kernel(const float* __restrict__ Wa,
                                                              float* __restrict__ WaP) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  constexpr int NPK = FNG * FNT * 64 * 16;
  if (idx >= NPK + SPECIAL_FLOATS) return;
  if (idx >= NPK) {  // special q|k|v rows for padding titles (0) and invalid ids (NaN)
    WaP[idx] = (idx - NPK) < 3 * FD ? 0.f : qnan();
    return;
  }
  const int s = idx & 15;
  const int lane = (idx >> 4) & 63;
  const int nt = (idx >> 10) % FNT;
  const int g = (idx >> 10) / FNT;
  const int n = 16 * nt + (lane & 15);
  const int k = FGK * g + 15 * (lane >> 4) + s;
  WaP[idx] = (s < FKS && n < FQ) ? Wa[n * FD + k] : 0.f;
}

typedef __attribute__((address_space(3))) void lds_void;

// One global_load_lds_dwordx4: lane i's 16 source bytes land at LDS byte
// address lds_byte + 16 i. Written in asm so that hipcc does not order its own
// LDS reads of the OTHER staging buffer behind it (as a builtin it emits a
// vmcnt(0) before the next ds_read); completion is waited explicitly by the
// issuing waves before the step's barrier (MI355X guide §5.7 recipe).
__device__ __forceinline__ void dma16(const void* gsrc, unsigned lds_byte) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_byte)
      : "memory");
}

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
};

// ABL (diagnostic ablation, -DNRMS_FUSED_ABLATION build + NRMS_FUSED_ABLATE env):
// 0 full; 1 producer skips the
// attention arithmetic; 2 consumer skips the MFMAs; 3 producer skips the DMA;
// 4 producer idle; 5 both idle (loop + barrier + pool skeleton); 6 consumer
// idle + producer DMA only; 7 consumer idle + producer attention only.
template <int ABL>
__global__ __launch_bounds__(NTHR, 1) void fused_news_kernel(
    const float* __restrict__ qkv, RowMap rmap, int64_t n_groups, const float* __restrict__ WaP,
    const float* __restrict__ b_add, const float* __restrict__ q_add, float* __restrict__ ctx_g,
    float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* Abuf = lds;                       // [2][80][SA]
  float* KVbuf = Abuf + 2 * A_FL;          // [2][80][3][q20|k20|v20]
  float* part = KVbuf + 2 * KV_FL;         // [4][80] per-consumer-wave row partials
  // [2][80] source row pointer of every token row of a title group (by group parity)
  const float** rowptr = reinterpret_cast<const float**>(part + 4 * FROWS);
  float* wsm = part + 4 * FROWS + 4 * FROWS;   // [2][80] softmax weights by title-group parity

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool producer = wave >= 4;
  const int ptid = tid - 256;              // producer thread index 0..255

  // title groups of this workgroup: blockIdx.x, +gridDim.x, ...
  const int64_t my_groups = n_groups > blockIdx.x ? (n_groups - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  const int64_t items = my_groups * FNG;
  auto group_of = [&](int64_t it) { return (int64_t)blockIdx.x + (it / FNG) * (int64_t)gridDim.x; };

  // producer: row pointers of title group `tg` -> rowptr[tg & 1] (written two
  // steps before its first DMA; padding / invalid rows point at the zero /
  // NaN row that the pack kernel wrote after WaP).
  const float* zero_row = WaP + FNG * FNT * 64 * 16;
  const float* nan_row = zero_row + 3 * FD;
  auto load_rows = [&](int64_t tg_local) {
    if (ptid < FROWS) {
      const int t = ptid / FL;
      const int64_t s = (int64_t)blockIdx.x + tg_local * gridDim.x;
      const int64_t row = rmap(s * FT + t, ptid - t * FL);
      rowptr[(tg_local & 1) * FROWS + ptid] =
          row >= 0 ? qkv + row * (3 * FD) : (row == -1 ? nan_row : zero_row);
    }
  };
  // producer: LDS-DMA gather of the Q|K|V slices of item `it` into buffer
  // `buf`, laid out [row r][head hl][q20|k20|v20] (15 float4 per (r, hl)).
  // One global_load_lds_dwordx4 writes 64 consecutive float4 of that layout;
  // each lane's source is its row's slice.
  auto stage = [&](int64_t it, int buf) {
    const int g = (int)(it % FNG);
    const float* const* rp = rowptr + ((it / FNG) & 1) * FROWS;
    float* KV = KVbuf + buf * KV_FL;

    for (int base = (wave - 4) * 64; base < KV_F4; base += 256) {
      const int e = base + lane;
      if (e < KV_F4) {
        const int r = e / (FG * 15);
        const int rem = e - r * (FG * 15);
        const int hl = rem / 15, c = rem - hl * 15;
        const int part3 = c / 5, cc = c - part3 * 5;
        const float* src = rp[r] + (part3 * FD + FDK * (FG * g + hl) + 4 * cc);
        const unsigned dst = __builtin_amdgcn_readfirstlane(
            (unsigned)(uintptr_t)(lds_void*)(KV + 4 * base));
        dma16(src, dst);
      }
    }
  };

  // exp(d / sqrt(d_k)) as v_exp_f32(d * log2(e) / sqrt(d_k)): same overflow
  // (-> inf -> NaN) and underflow (-> 0) behaviour as the reference's exp.
  const float c_exp = 1.4426950408889634f / sqrtf((float)FDK);

  floatx4 accA[FMT][3], accX[2];
  const int lm = lane & 15, kq = lane >> 4;

  // consumer: B fragments of head group g for the wave's N tiles (L2-resident
  // WaP). Loaded at the end of the previous step, so the load latency hides
  // behind the step barrier instead of stalling the first MFMA.
  float bA[3][16], bX[16];
  auto load_b = [&](int g) {
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
  };
  if (!producer) load_b(0);

  if (producer && items > 0) load_rows(0);
  __syncthreads();
  if (producer && items > 0) stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // Role-split loops (same barrier count in both) so the compiler allocates
  // registers per role: producer temporaries and consumer accumulators are
  // never live at the same time.
  if (producer) {
    for (int64_t step = 0; step < items + 7; ++step) {
        // next title group's row pointers, two steps before its first DMA
        // (before this step's DMA so that its id-load wait does not drain it)
        if (step % FNG == FNG - 2 && step + 2 < items) load_rows(step / FNG + 1);
        // pooling (additive.py:51-52) of title group tgp, chunk k, from the
        // softmax weights the consumers wrote two steps after its last MFMA:
        // loads issued now, consumed after the attention below.
        const int64_t pstep = step - 7;
        const int64_t tgp = pstep >= 0 ? pstep / FNG : -1;
        const int pk = pstep >= 0 ? (int)(pstep % FNG) : 0;
        const bool pool_on = pstep >= 0 && tgp < my_groups && ptid < 60;
        int64_t pool_title = 0;
        int pool_c = 0, pool_t = 0;
        float4 px[FL];
        if (pool_on) {
          const int o = pk * 60 + ptid;          // 300 float4 outputs per title group
          pool_t = o / (FD / 4);
          pool_c = o - pool_t * (FD / 4);
          pool_title = ((int64_t)blockIdx.x + tgp * gridDim.x) * FT + pool_t;
          if (pool_title < rmap.n_titles) {
            const float4* xr = reinterpret_cast<const float4*>(ctx_g + pool_title * FL * FD) + pool_c;
#pragma unroll
            for (int i = 0; i < FL; ++i) px[i] = xr[i * (FD / 4)];
          }
        }
        if (ABL != 3 && ABL != 4 && ABL != 5 && ABL != 7 && step + 1 < items) stage(step + 1, (int)((step + 1) & 1));
        if (step < items) {
          // ---- attention for item `step`: task (head hl, row r); 240 of 256 lanes
          const int64_t it = step;
          const int g = (int)(it % FNG);
          const int64_t title0 = group_of(it) * FT;
          const float* KV = KVbuf + (it & 1) * KV_FL;
          float* A = Abuf + (it & 1) * A_FL;
          if (ptid < FG * FROWS) {
            const int hl = ptid / FROWS, r = ptid - hl * FROWS;
            const int t = r / FL, i = r - t * FL;
            const int h = FG * g + hl;
            float ctxv[FDK];
  #pragma unroll
            for (int d = 0; d < FDK; ++d) ctxv[d] = 0.f;
            if (ABL != 1 && ABL != 4 && ABL != 5 && ABL != 6 && title0 + t < rmap.n_titles) {
              float q[FDK];
              const float4* qp = reinterpret_cast<const float4*>(KV + (r * FG + hl) * HW);
  #pragma unroll
              for (int c = 0; c < FDK / 4; ++c) {
                const float4 v = qp[c];
                q[4 * c] = v.x; q[4 * c + 1] = v.y; q[4 * c + 2] = v.z; q[4 * c + 3] = v.w;
              }
              const float* kvt = KV + (FL * t * FG + hl) * HW;   // token j: + j * RW
              float e[FL];
              float sum = 0.f;
              // Tokens are processed 4 at a time: the 20 ds_read_b128 of a block
            // are issued together (one LDS latency per 4 tokens) and the 4 dot
            // products run as independent FMA chains.
            constexpr int JB = 4;
#pragma unroll
            for (int j0 = 0; j0 < FL; j0 += JB) {
              float4 kr[JB][FDK / 4];
#pragma unroll
              for (int u = 0; u < JB; ++u)
#pragma unroll
                for (int c = 0; c < FDK / 4; ++c)
                  kr[u][c] = reinterpret_cast<const float4*>(kvt + (j0 + u) * RW + FDK)[c];
              float d[JB];
#pragma unroll
              for (int u = 0; u < JB; ++u) d[u] = 0.f;
#pragma unroll
              for (int c = 0; c < FDK / 4; ++c)
#pragma unroll
                for (int u = 0; u < JB; ++u) {
                  d[u] = fmaf(q[4 * c], kr[u][c].x, d[u]);
                  d[u] = fmaf(q[4 * c + 1], kr[u][c].y, d[u]);
                  d[u] = fmaf(q[4 * c + 2], kr[u][c].z, d[u]);
                  d[u] = fmaf(q[4 * c + 3], kr[u][c].w, d[u]);
                }
#pragma unroll
              for (int u = 0; u < JB; ++u) {
                e[j0 + u] = __builtin_amdgcn_exp2f(d[u] * c_exp);
                sum += e[j0 + u];
              }
            }
            const float inv = 1.0f / (sum + 1e-8f);
#pragma unroll
            for (int j0 = 0; j0 < FL; j0 += JB) {
              float4 vr[JB][FDK / 4];
#pragma unroll
              for (int u = 0; u < JB; ++u)
#pragma unroll
                for (int c = 0; c < FDK / 4; ++c)
                  vr[u][c] = reinterpret_cast<const float4*>(kvt + (j0 + u) * RW + 2 * FDK)[c];
#pragma unroll
              for (int u = 0; u < JB; ++u) {
                const float a = e[j0 + u] * inv;
#pragma unroll
                for (int c = 0; c < FDK / 4; ++c) {
                  ctxv[4 * c] = fmaf(a, vr[u][c].x, ctxv[4 * c]);
                  ctxv[4 * c + 1] = fmaf(a, vr[u][c].y, ctxv[4 * c + 1]);
                  ctxv[4 * c + 2] = fmaf(a, vr[u][c].z, ctxv[4 * c + 2]);
                  ctxv[4 * c + 3] = fmaf(a, vr[u][c].w, ctxv[4 * c + 3]);
                }
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
        }
        if (pool_on && pool_title < rmap.n_titles) {
          const float* wv = wsm + (tgp & 1) * FROWS + FL * pool_t;
          float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int i = 0; i < FL; ++i) {
            const float wi = wv[i];
            acc.x = fmaf(wi, px[i].x, acc.x);
            acc.y = fmaf(wi, px[i].y, acc.y);
            acc.z = fmaf(wi, px[i].z, acc.z);
            acc.w = fmaf(wi, px[i].w, acc.w);
          }
          reinterpret_cast<float4*>(out + pool_title * FD)[pool_c] = acc;
        }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // retire this step's DMA
      __syncthreads();
    }
  } else {
    for (int64_t step = 0; step < items + 7; ++step) {
        // ---- consumer: (a) softmax of the title group whose MFMA finished last step
        const int64_t done = step - 2;   // item whose MFMA finished in step-1
        if (done >= 0 && done % FNG == FNG - 1) {
          const int t = wave;
          const int64_t s = group_of(done) * FT + t;
          const float v = lane < FL ? part[t * FL + lane] + part[FROWS + t * FL + lane] +
                                          part[2 * FROWS + t * FL + lane] + part[3 * FROWS + t * FL + lane]
                                    : -INFINITY;
          const float m = wave_max_nan(v);
          const float ex = lane < FL ? expf(v - m) : 0.f;
          const float sum = wave_sum(ex);
          const float w = ex / sum;
          // pooling is done by the producer waves over the next 5 steps
          if (lane < FL) wsm[((done / FNG) & 1) * FROWS + FL * t + lane] = w;
          (void)s;
        }
        // ---- (b) MFMA for item step-1
        const int64_t it = step - 1;
        if (ABL != 2 && ABL != 5 && ABL != 6 && ABL != 7 && it >= 0 && it < items) {
          const int g = (int)(it % FNG);
          if (g == 0) {
  #pragma unroll
            for (int mt = 0; mt < FMT; ++mt)
  #pragma unroll
              for (int j = 0; j < 3; ++j) accA[mt][j] = floatx4{0.f, 0.f, 0.f, 0.f};
            accX[0] = accX[1] = floatx4{0.f, 0.f, 0.f, 0.f};
          }
          const float* Aw = Abuf + (it & 1) * A_FL + lm * SA + 15 * kq;
          // A fragments one k-step ahead of the MFMAs that consume them
          float a[FMT], ax0, an[FMT], axn = 0.f;
  #pragma unroll
          for (int mt = 0; mt < FMT; ++mt) a[mt] = Aw[16 * mt * SA];
          ax0 = Aw[16 * wave * SA];
  #pragma unroll
          for (int s = 0; s < FKS; ++s) {
            if (s + 1 < FKS) {
  #pragma unroll
              for (int mt = 0; mt < FMT; ++mt) an[mt] = Aw[16 * mt * SA + s + 1];
              axn = Aw[16 * wave * SA + s + 1];
            }
  #pragma unroll
            for (int mt = 0; mt < FMT; ++mt)
  #pragma unroll
              for (int j = 0; j < 3; ++j)
                accA[mt][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[mt], bA[j][s], accA[mt][j], 0, 0, 0);
            accX[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(ax0, bX[s], accX[0], 0, 0, 0);
            if (wave == 0)
              accX[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[FMT - 1], bX[s], accX[1], 0, 0, 0);
            if (s + 1 < FKS) {
  #pragma unroll
              for (int mt = 0; mt < FMT; ++mt) a[mt] = an[mt];
              ax0 = axn;
            }
          }
            if (g == FNG - 1) {
            // scores: per-row partials of sum_n q[n] tanh(acc + b[n]) over the wave's columns
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
          }
        }
          if (it + 1 < items) load_b((int)((it + 1) % FNG));
      // Raw barrier: LDS traffic retired, but the B-fragment loads just issued
      // stay in flight across it (a __syncthreads() would wait vmcnt(0) here);
      // hipcc waits for them at their first use in the next step.
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  }
}

}  // namespace

size_t fused_news_packed_b_floats() { return (size_t)FNG * FNT * 64 * 16 + SPECIAL_FLOATS; }

bool fused_news_supported(int L, int D, int H, int Q) {
  return L == FL && D == FD && H == FH && Q == FQ;
}

int32_t launch_fused_news(const float* qkv, int64_t n_rows, const int64_t* ids_a, int64_t n_seq_a,
                          const int64_t* ids_b, int64_t n_titles, const float* w_add,
                          const float* b_add, const float* q_add, float* wap, float* ctx,
                          float* out, hipStream_t s) {
  if (n_titles == 0) return NRMS_OK;
  if (((uintptr_t)qkv | (uintptr_t)ctx | (uintptr_t)out | (uintptr_t)wap) % 16) return NRMS_ERR_UNSUPPORTED;
  // Diagnostic ablations (see fused_news_kernel) exist only in builds with
  // -DNRMS_FUSED_ABLATION; the product build instantiates the full kernel.
#ifdef NRMS_FUSED_ABLATION
  static int abl = -1;
  if (abl < 0) {
    const char* e = getenv("NRMS_FUSED_ABLATE");
    abl = e ? atoi(e) : 0;
  }
  static const void* kerns[8] = {
      (const void*)&fused_news_kernel<0>, (const void*)&fused_news_kernel<1>,
      (const void*)&fused_news_kernel<2>, (const void*)&fused_news_kernel<3>,
      (const void*)&fused_news_kernel<4>, (const void*)&fused_news_kernel<5>,
      (const void*)&fused_news_kernel<6>, (const void*)&fused_news_kernel<7>};
  auto kern = (decltype(&fused_news_kernel<0>))kerns[abl & 7];
#else
  auto kern = &fused_news_kernel<0>;
#endif
  static bool attr_done = false;
  if (!attr_done) {
#ifdef NRMS_FUSED_ABLATION
    for (auto k : kerns)
      (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_BYTES);
#else
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_BYTES);
#endif
    attr_done = true;
  }
  const int npk = FNG * FNT * 64 * 16 + SPECIAL_FLOATS;
  hipLaunchKernelGGL(pack_additive_b_kernel, dim3((npk + 255) / 256), dim3(256), 0, s, w_add, wap);
  if (int32_t st = launch_status()) return st;
  const int64_t n_groups = (n_titles + FT - 1) / FT;
  int dev = 0, n_cu = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      n_cu = v;
  }
  const int64_t blocks = n_groups < n_cu ? n_groups : n_cu;   // persistent: one workgroup per CU
  RowMap rm{ids_a, ids_b, n_seq_a, n_titles, n_rows};
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(NTHR), LDS_BYTES, s, qkv, rm, n_groups, wap,
                     b_add, q_add, ctx, out);
  return launch_status();
}

}  // namespace nrms
