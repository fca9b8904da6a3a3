// Training (train-mode forward + backward + Adam) kernels of the NRMS path:
// the autograd of src/model/NRMS (news_encoder.py:27-48, user_encoder.py:15-26,
// multihead_self.py:15-75, additive.py:27-53, dot_product.py:8-19) and the
// optimizer step of src/train.py:127,205-236, restated as explicit backward
// kernels. fp32 results; the weight-gradient GEMM runs on split-bf16 x6
// (exact f32 MFMA under NRMS_GEMM=f32).
//
//   dropout            counter-based: keep(i) = hash(seed, i) >= p, so the
//                      backward regenerates the mask instead of storing it
//   score_backward     d news = dlogit * user, d user = sum_c dlogit * news
//   additive_backward  softmax / tanh·q chain per sequence; dz = ds q (1 - y^2)
//   mhsa_backward      raw-exp attention per (sequence, head): A = E / (Z + 1e-8),
//                      dS = A (dA - rowsum(dA A)), dQ = dS K / sqrt(dk), ...
//   gemm_tn            dW[n][k] += sum_r dY[r][n] X[r][k] (split over row slices; the
//                      slices' partials summed in slice order: deterministic)
//   embedding_backward dtable[id] += dx (rows with id == padding_idx skipped);
//                      deterministic form: tokens sorted by id (embed_sort.hip)
// Every training kernel is deterministic (no float atomics): two runs of a step
// give bitwise the same gradients (tests/test_gpu_train.py).
//   adam               torch.optim.Adam's update, same operation order
#include "nrms_common.hpp"

namespace nrms {
namespace {

// splitmix64 finaliser of (seed, index): uniform in [0, 1) with 24 bits.
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t i) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ULL * (i + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

__global__ __launch_bounds__(256) void dropout_kernel(const float* __restrict__ x,
                                                      float* __restrict__ y, int64_t n, float p,
                                                      float scale, uint64_t seed) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  y[i] = uniform01(seed, (uint64_t)i) >= p ? x[i] * scale : 0.f;
}

// One wave per (impression b): duser[b] = sum_c dl[b,c] news[b,c,:];
// dnews[b,c,:] = dl[b,c] user[b,:] (dnews contiguous [B, C, D]).
__global__ __launch_bounds__(256) void score_backward_kernel(
    const float* __restrict__ news, int64_t B, int C, int64_t sb, int64_t sc,
    const float* __restrict__ user, int64_t su, int D, const float* __restrict__ dl,
    float* __restrict__ dnews, float* __restrict__ duser) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (b >= B) return;
  for (int d = lane; d < D; d += 64) {
    const float u = user[b * su + d];
    float acc = 0.f;
    for (int c = 0; c < C; ++c) {
      const float g = dl[b * C + c];
      acc = fmaf(g, news[b * sb + c * sc + d], acc);
      dnews[(b * C + c) * D + d] = g * u;
    }
    duser[b * D + d] = acc;
  }
}

// Additive attention backward, per sequence s (one workgroup of 256 threads):
//   w = softmax_l(score), out = sum_l w_l x_l
//   dx_l   = w_l dout                    (written; the dz·Wa term is added by a GEMM)
//   dw_l   = x_l · dout
//   ds_l   = w_l (dw_l - sum_l' w_l' dw_l')
//   dz_lq  = ds_l q_q (1 - y_lq^2)       (written, [rows, Q])
//   dq    += sum_l ds_l y_l ;  db += sum_l dz_l   (per-sequence partials pq / pb
//            [n_seq][Q], summed over the sequences in a fixed order by reduce_rows_add)
__global__ __launch_bounds__(256) void additive_backward_rows_kernel(
    const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ score,
    const float* __restrict__ q, const float* __restrict__ dout, int L, int D, int Q,
    float* __restrict__ dx, float* __restrict__ dz, float* __restrict__ pq,
    float* __restrict__ pb) {
  __shared__ float sw[64], sds[64], sdw[64];
  const int64_t s = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const float* xs = x + s * L * D;
  const float* os = dout + s * D;
  // dw_l = x_l . dout: wave wv takes rows wv, wv+4, ...
  for (int l = wv; l < L; l += 4) {
    float a = 0.f;
    for (int d = lane; d < D; d += 64) a = fmaf(xs[l * D + d], os[d], a);
    a = wave_sum(a);
    if (lane == 0) sdw[l] = a;
  }
  __syncthreads();
  if (wv == 0) {
    const float v = lane < L ? score[s * L + lane] : -INFINITY;
    const float m = wave_max_nan(v);
    const float e = lane < L ? expf(v - m) : 0.f;
    const float w = e / wave_sum(e);
    const float dwv = lane < L ? sdw[lane] : 0.f;
    const float dot = wave_sum(lane < L ? w * dwv : 0.f);
    if (lane < L) {
      sw[lane] = w;
      sds[lane] = w * (dwv - dot);
    }
  }
  __syncthreads();
  for (int e = tid; e < L * D; e += 256) {
    const int l = e / D, d = e - l * D;
    dx[(s * L + l) * D + d] = sw[l] * os[d];
  }
  for (int qq = tid; qq < Q; qq += 256) {
    const float qv = q[qq];
    float aq = 0.f, ab = 0.f;
    for (int l = 0; l < L; ++l) {
      const float yv = y[(s * L + l) * Q + qq];
      const float g = sds[l] * qv * (1.f - yv * yv);
      dz[(s * L + l) * Q + qq] = g;
      aq = fmaf(sds[l], yv, aq);
      ab += g;
    }
    pq[s * Q + qq] = aq;
    pb[s * Q + qq] = ab;
  }
}

// Column sums of part [rows][cols] in a fixed order (deterministic): thread
// (column c, chunk blockIdx.y) sums rows [chunk y, chunk (y + 1)) in order
// (loads eight rows ahead); with one chunk the sum is added to out[c],
// otherwise stored to out[y][c] for a second pass.
__global__ __launch_bounds__(256) void reduce_rows_kernel(const float* __restrict__ part, int64_t rows,
                                                          int64_t cols, int64_t chunk, float* __restrict__ out,
                                                          int accumulate) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  const int64_t r0 = (int64_t)blockIdx.y * chunk, r1 = r0 + chunk < rows ? r0 + chunk : rows;
  float a = 0.f;
  int64_t r = r0;
  for (; r + 8 <= r1; r += 8) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = part[(r + i) * cols + c];
#pragma unroll
    for (int i = 0; i < 8; ++i) a += v[i];
  }
  for (; r < r1; ++r) a += part[r * cols + c];
  if (accumulate) out[c] += a;
  else out[(int64_t)blockIdx.y * cols + c] = a;
}

constexpr int64_t RED_CHUNK = 64;
// floats of the second-pass buffer reduce_rows_add needs for `rows` rows
inline size_t reduce_scratch_floats(int64_t rows, int64_t cols) {
  return rows > RED_CHUNK ? (size_t)((rows + RED_CHUNK - 1) / RED_CHUNK) * cols : 0;
}
// whether reduce_rows_add takes `rows` rows (its chunk count is a grid y
// extent); callers check it before writing any output, so an UNSUPPORTED
// return leaves every output untouched
inline bool reduce_rows_supported(int64_t rows) { return (rows + RED_CHUNK - 1) / RED_CHUNK <= 65535; }
// out[c] += sum_r part[r][c]: one pass for at most RED_CHUNK rows, else chunks
// of RED_CHUNK rows into `scratch` and a second pass over the chunk sums
int32_t reduce_rows_add(const float* part, int64_t rows, int64_t cols, float* out, float* scratch, hipStream_t s) {
  const unsigned gx = (unsigned)((cols + 255) / 256);
  if (rows <= RED_CHUNK) {
    hipLaunchKernelGGL(reduce_rows_kernel, dim3(gx), dim3(256), 0, s, part, rows, cols, rows, out, 1);
    return launch_status();
  }
  const int64_t nch = (rows + RED_CHUNK - 1) / RED_CHUNK;
  if (nch > 65535) return NRMS_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(reduce_rows_kernel, dim3(gx, (unsigned)nch), dim3(256), 0, s, part, rows, cols, RED_CHUNK,
                     scratch, 0);
  if (int32_t st = launch_status()) return st;
  hipLaunchKernelGGL(reduce_rows_kernel, dim3(gx), dim3(256), 0, s, scratch, nch, cols, nch, out, 1);
  return launch_status();
}

// Raw-exp multi-head attention backward, one workgroup per (sequence, head).
// qkv rows of the sequence: s*L + i (per-token projection layout, ld = 3D);
// dctx [rows, D]; writes dqkv [rows, 3D] slices of this head.
template <int LMAX>
__global__ __launch_bounds__(256) void mhsa_backward_kernel(const float* __restrict__ qkv,
                                                            const float* __restrict__ dctx, int L,
                                                            int D, int H,
                                                            float* __restrict__ dqkv) {
  constexpr int DK = 20;
  __shared__ float sq[LMAX][DK], sk[LMAX][DK], sv[LMAX][DK], so[LMAX][DK];
  __shared__ float sa[LMAX][LMAX + 1], sda[LMAX][LMAX + 1];
  __shared__ float srow[LMAX];
  const int64_t s = blockIdx.x / H;
  const int h = blockIdx.x - (int)(s * H);
  const int tid = threadIdx.x;
  const int ld = 3 * D;
  const float rs = 1.0f / sqrtf((float)DK);
  for (int e = tid; e < L * DK; e += 256) {
    const int i = e / DK, t = e - i * DK;
    const float* row = qkv + (s * L + i) * ld + h * DK + t;
    sq[i][t] = row[0];
    sk[i][t] = row[D];
    sv[i][t] = row[2 * D];
    so[i][t] = dctx[(s * L + i) * D + h * DK + t];
  }
  __syncthreads();
  // E_ij = exp(q_i k_j / sqrt(dk)) (no max subtraction, as the forward); dA_ij = dO_i . V_j
  for (int e = tid; e < L * L; e += 256) {
    const int i = e / L, j = e - i * L;
    float d = 0.f, g = 0.f;
#pragma unroll
    for (int t = 0; t < DK; ++t) {
      d = fmaf(sq[i][t], sk[j][t], d);
      g = fmaf(so[i][t], sv[j][t], g);
    }
    sa[i][j] = expf(d * rs);
    sda[i][j] = g;
  }
  __syncthreads();
  // A = E / (Z + 1e-8); rowdot_i = sum_j dA_ij A_ij
  if (tid < L) {
    const int i = tid;
    float z = 0.f;
    for (int j = 0; j < L; ++j) z += sa[i][j];
    const float inv = 1.0f / (z + 1e-8f);
    float rd = 0.f;
    for (int j = 0; j < L; ++j) {
      const float a = sa[i][j] * inv;
      sa[i][j] = a;
      rd = fmaf(sda[i][j], a, rd);
    }
    srow[i] = rd;
  }
  __syncthreads();
  // dV_j = sum_i A_ij dO_i
  for (int e = tid; e < L * DK; e += 256) {
    const int j = e / DK, t = e - j * DK;
    float acc = 0.f;
    for (int i = 0; i < L; ++i) acc = fmaf(sa[i][j], so[i][t], acc);
    dqkv[(s * L + j) * ld + 2 * D + h * DK + t] = acc;
  }
  __syncthreads();
  // dS_ij = A_ij (dA_ij - rowdot_i), scaled by 1/sqrt(dk) for dQ / dK
  for (int e = tid; e < L * L; e += 256) {
    const int i = e / L, j = e - i * L;
    sda[i][j] = sa[i][j] * (sda[i][j] - srow[i]) * rs;
  }
  __syncthreads();
  for (int e = tid; e < L * DK; e += 256) {
    const int i = e / DK, t = e - i * DK;
    float gq = 0.f, gk = 0.f;
    for (int j = 0; j < L; ++j) {
      gq = fmaf(sda[i][j], sk[j][t], gq);
      gk = fmaf(sda[j][i], sq[j][t], gk);
    }
    dqkv[(s * L + i) * ld + h * DK + t] = gq;
    dqkv[(s * L + i) * ld + D + h * DK + t] = gk;
  }
}

// The same for titles (L <= 20) with one WAVE per (sequence, head): four
// independent tasks per workgroup, each on its own LDS slice, phases
// separated by wave-level LDS fences instead of workgroup barriers (the
// workgroup version spends most of its time in five barriers around
// 400-element loops).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ __launch_bounds__(256) void mhsa_backward_wave_kernel(const float* __restrict__ qkv,
                                                                 const float* __restrict__ dctx,
                                                                 int64_t n_tasks, int L, int D,
                                                                 int H, float* __restrict__ dqkv) {
  constexpr int DK = 20, LM = 20;
  struct Slice {
    float q[LM][DK], k[LM][DK], v[LM][DK], o[LM][DK];
    float a[LM][LM + 1], da[LM][LM + 1], row[LM];
  };
  __shared__ Slice ws[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t task = (int64_t)blockIdx.x * 4 + wv;
  if (task >= n_tasks) return;   // no workgroup barrier below: a finished wave may leave
  const int64_t s = task / H;
  const int h = (int)(task - s * H);
  Slice& W = ws[wv];
  const int ld = 3 * D;
  const float rs = 1.0f / sqrtf((float)DK);
  for (int e = lane; e < L * DK; e += 64) {
    const int i = e / DK, t = e - i * DK;
    const float* row = qkv + (s * L + i) * ld + h * DK + t;
    W.q[i][t] = row[0];
    W.k[i][t] = row[D];
    W.v[i][t] = row[2 * D];
    W.o[i][t] = dctx[(s * L + i) * D + h * DK + t];
  }
  wave_lds_sync();
  for (int e = lane; e < L * L; e += 64) {
    const int i = e / L, j = e - i * L;
    float d = 0.f, g = 0.f;
#pragma unroll
    for (int t = 0; t < DK; ++t) {
      d = fmaf(W.q[i][t], W.k[j][t], d);
      g = fmaf(W.o[i][t], W.v[j][t], g);
    }
    W.a[i][j] = expf(d * rs);
    W.da[i][j] = g;
  }
  wave_lds_sync();
  if (lane < L) {
    const int i = lane;
    float z = 0.f;
    for (int j = 0; j < L; ++j) z += W.a[i][j];
    const float inv = 1.0f / (z + 1e-8f);
    float rd = 0.f;
    for (int j = 0; j < L; ++j) {
      const float a = W.a[i][j] * inv;
      W.a[i][j] = a;
      rd = fmaf(W.da[i][j], a, rd);
    }
    W.row[i] = rd;
  }
  wave_lds_sync();
  for (int e = lane; e < L * DK; e += 64) {
    const int j = e / DK, t = e - j * DK;
    float acc = 0.f;
    for (int i = 0; i < L; ++i) acc = fmaf(W.a[i][j], W.o[i][t], acc);
    dqkv[(s * L + j) * ld + 2 * D + h * DK + t] = acc;
  }
  wave_lds_sync();
  for (int e = lane; e < L * L; e += 64) {
    const int i = e / L, j = e - i * L;
    W.da[i][j] = W.a[i][j] * (W.da[i][j] - W.row[i]) * rs;
  }
  wave_lds_sync();
  for (int e = lane; e < L * DK; e += 64) {
    const int i = e / DK, t = e - i * DK;
    float gq = 0.f, gk = 0.f;
    for (int j = 0; j < L; ++j) {
      gq = fmaf(W.da[i][j], W.k[j][t], gq);
      gk = fmaf(W.da[j][i], W.q[j][t], gk);
    }
    dqkv[(s * L + i) * ld + h * DK + t] = gq;
    dqkv[(s * L + i) * ld + D + h * DK + t] = gk;
  }
}

// part[z][n][k] = sum_{r in slice z} dY[r][n] X[r][k] (+ part_b[z][n] = the
// slice's column sums of dY, from the column tile 0 blocks). f32 MFMA 16x16x4;
// block = 64 (n) x 64 (k) tile over a row slice of `slice` rows (a multiple
// of 32), 4 waves each a 16-row (n) strip x 64 cols; LDS tiles of 32 rows.
// The slices' partials are summed in slice order (reduce_rows_add).
constexpr int TN_TILE = 64, TN_BK = 32;
#ifndef NRMS_TN_BLOCKS
#define NRMS_TN_BLOCKS 4096
#endif
#ifndef NRMS_TN_MAX_SLICES
#define NRMS_TN_MAX_SLICES 64
#endif
constexpr int TN_BLOCKS = NRMS_TN_BLOCKS;    // aim: (n tiles) x (k tiles) x slices >= this many blocks
constexpr int TN_MAX_SLICES = NRMS_TN_MAX_SLICES;
__global__ __launch_bounds__(256) void gemm_tn_kernel(const float* __restrict__ dY, int64_t R,
                                                      int N, const float* __restrict__ X, int K,
                                                      int64_t slice, float* __restrict__ part,
                                                      float* __restrict__ part_b) {
  __shared__ float sy[TN_BK][TN_TILE + 1], sx[TN_BK][TN_TILE + 1];
  const int n0 = blockIdx.x * TN_TILE, k0 = blockIdx.y * TN_TILE;
  const int64_t r0 = (int64_t)blockIdx.z * slice;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lm = lane & 15, kq = lane >> 4;
  floatx4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;   // db: thread tid < 64 sums column n0 + tid
  for (int64_t rb = 0; rb < slice && r0 + rb < R; rb += TN_BK) {
    for (int e = tid; e < TN_BK * TN_TILE; e += 256) {
      const int rr = e / TN_TILE, c = e - rr * TN_TILE;
      const int64_t r = r0 + rb + rr;
      const bool rin = r < R;
      sy[rr][c] = (rin && n0 + c < N) ? dY[r * N + n0 + c] : 0.f;
      sx[rr][c] = (rin && k0 + c < K) ? X[r * K + k0 + c] : 0.f;
    }
    __syncthreads();
    if (part_b && blockIdx.y == 0 && tid < TN_TILE)
      for (int rr = 0; rr < TN_BK; ++rr) bsum += sy[rr][tid];
#pragma unroll
    for (int kk = 0; kk < TN_BK; kk += 4) {
      // A[i = n][k = r] = dY[r][n], B[k = r][j = col] = X[r][col]
      const float a = sy[kk + kq][16 * w + lm];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float b = sx[kk + kq][16 * j + lm];
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  // C/D: col = lane & 15, row = 4 (lane >> 4) + reg
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + 16 * w + 4 * kq + r, k = k0 + 16 * j + lm;
      if (n < N && k < K) part[((int64_t)blockIdx.z * N + n) * K + k] = acc[j][r];
    }
  if (part_b && blockIdx.y == 0 && tid < TN_TILE && n0 + tid < N) part_b[(int64_t)blockIdx.z * N + n0 + tid] = bsum;
}

// The same dW += dY^T X on split-bf16 x6 (v_mfma_f32_16x16x32_bf16, the
// forward GEMMs' arithmetic): per 32-row chunk each thread loads a 4 (rows) x
// 4 (columns) block of dY (threads 0..127) or X (128..255), transposes it in
// registers and stores each column's 4 rows as three bf16 planes, so LDS holds
// [plane][n or k][32 rows] and every MFMA fragment (8 consecutive rows of one
// column) is one conflict-free ds_read_b128 (64-B rows, chunk kq at kq ^ xsw).
// db sums stay exact fp32, from the loaded registers.
typedef __bf16 tn_bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ int tn_xsw(int row) { return ((row >> 3) & 1) << 1; }

__global__ __launch_bounds__(256) void gemm_tn_x6_kernel(const float* __restrict__ dY, int64_t R,
                                                         int N, const float* __restrict__ X, int K,
                                                         int64_t slice, float* __restrict__ part,
                                                         float* __restrict__ part_b) {
  constexpr int RK = 32, PL = TN_TILE * RK;   // rows per chunk, bf16 per plane
  __shared__ __attribute__((aligned(16))) __bf16 sa[3 * PL], sb[3 * PL];
  const int n0 = blockIdx.x * TN_TILE, k0 = blockIdx.y * TN_TILE;
  const int64_t r0 = (int64_t)blockIdx.z * slice;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lm = lane & 15, kq = lane >> 4;
  // staging role: a 4 x 4 block (rows 4 rb.., columns 4 cb..) of dY or X
  const bool isa = tid < 128;
  const int t = tid & 127, rb = t >> 4, cb = t & 15;
  const float* src = isa ? dY : X;
  const int ld = isa ? N : K;
  const int c0 = (isa ? n0 : k0) + 4 * cb;
  const bool cin = c0 < ld;   // ld % 4 == 0: a float4 is all in or all out
  __bf16* dst = isa ? sa : sb;
  float4 v[4];
  auto gload = [&](int64_t rbase) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t r = rbase + 4 * rb + i;
      v[i] = (cin && r < R) ? *reinterpret_cast<const float4*>(src + r * ld + c0)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  float bs[4] = {0.f, 0.f, 0.f, 0.f};   // db partials of columns c0..c0+3
  auto stage = [&]() {
    const float col[4][4] = {{v[0].x, v[1].x, v[2].x, v[3].x}, {v[0].y, v[1].y, v[2].y, v[3].y},
                             {v[0].z, v[1].z, v[2].z, v[3].z}, {v[0].w, v[1].w, v[2].w, v[3].w}};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (isa) bs[c] += ((col[c][0] + col[c][1]) + col[c][2]) + col[c][3];
      uint32_t h0, m0, l0, h1, m1, l1;
      split3x2(col[c][0], col[c][1], h0, m0, l0);
      split3x2(col[c][2], col[c][3], h1, m1, l1);
      const int row = 4 * cb + c;
      __bf16* d = dst + row * RK + (((rb >> 1) ^ tn_xsw(row)) << 3) + (rb & 1) * 4;
      *reinterpret_cast<uint2*>(d) = make_uint2(h0, h1);
      *reinterpret_cast<uint2*>(d + PL) = make_uint2(m0, m1);
      *reinterpret_cast<uint2*>(d + 2 * PL) = make_uint2(l0, l1);
    }
  };
  floatx4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int arow = 16 * w + lm;
  const __bf16* Af = sa + arow * RK + ((kq ^ tn_xsw(arow)) << 3);
  const __bf16* Bf = sb + lm * RK + ((kq ^ tn_xsw(lm)) << 3);   // + 16 j rows: same swizzle

  gload(r0);
  stage();
  __syncthreads();
  for (int64_t rc = 0; rc < slice; rc += RK) {
    const bool more = rc + RK < slice && r0 + rc + RK < R;
    if (more) gload(r0 + rc + RK);
    tn_bf16x8 a[3];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) a[pl] = *reinterpret_cast<const tn_bf16x8*>(Af + pl * PL);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      tn_bf16x8 b[3];
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        b[pl] = *reinterpret_cast<const tn_bf16x8*>(Bf + pl * PL + 16 * j * RK);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc[j], 0, 0, 0);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc[j], 0, 0, 0);
    }
    if (!more) break;
    __syncthreads();
    stage();
    __syncthreads();
  }
  // C/D: col = lane & 15 (k), row = 4 (lane >> 4) + reg (n)
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + 16 * w + 4 * kq + r, k = k0 + 16 * j + lm;
      if (n < N && k < K) part[((int64_t)blockIdx.z * N + n) * K + k] = acc[j][r];
    }
  if (part_b && blockIdx.y == 0) {
    // the slice's rows are spread over the 8 rb threads of a column block:
    // combine their partials through LDS (the staging tiles are free now)
    __syncthreads();
    float* red = reinterpret_cast<float*>(sb);   // [8 rb][64 columns]
    if (isa)
#pragma unroll
      for (int c = 0; c < 4; ++c) red[rb * TN_TILE + 4 * cb + c] = bs[c];
    __syncthreads();
    if (tid < TN_TILE && n0 + tid < N) {
      float sum = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) sum += red[q * TN_TILE + tid];
      part_b[(int64_t)blockIdx.z * N + n0 + tid] = sum;
    }
  }
}

// dtable[ids[t]] += dx[t] for ids[t] != padding_idx (nn.Embedding(padding_idx=0)
// leaves that row's gradient zero). One wave per token row, 4 columns per lane.
__global__ __launch_bounds__(256) void embedding_backward_kernel(
    const int64_t* __restrict__ ids, int64_t n_tok, const float* __restrict__ dx, int64_t V,
    int D, int64_t padding_idx, float* __restrict__ dtable) {
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= n_tok) return;
  const int64_t id = ids[t];
  if (id == padding_idx || (uint64_t)id >= (uint64_t)V) return;
  for (int d = lane; d < D; d += 64) atomicAdd(dtable + id * D + d, dx[t * D + d]);
}

// torch.optim.Adam (default, amsgrad = False, weight_decay = 0), in its
// single-tensor operation order: m = lerp(m, g, 1 - b1); v = b2 v + (1 - b2) g^2;
// denom = sqrt(v) / sqrt(1 - b2^t) + eps; p -= (lr / (1 - b1^t)) m / denom.
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p,
                                                   const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   int64_t n, float lr, float b1, float b2,
                                                   float eps, float bc1, float bc2_sqrt) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float gi = g[i];
  const float mi = m[i] + (1.0f - b1) * (gi - m[i]);
  const float vi = v[i] * b2 + (1.0f - b2) * gi * gi;
  m[i] = mi;
  v[i] = vi;
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  p[i] -= (lr / bc1) * (mi / denom);
}

// Multi-tensor Adam: up to kAdamChunk descriptors travel BY VALUE in the
// kernel arguments (48 B each, 1.5 KB of the 4 KB kernarg segment), so no
// device-side table has to outlive the launch or follow the caller's stream.
// Block b belongs to the tensor whose [first_block, next first_block) range
// holds it (n is small: a linear scan over SGPR-uniform data).
constexpr int kAdamChunk = 32;
struct AdamChunk {
  nrms_adam_tensor_t t[kAdamChunk];
  int64_t first_block[kAdamChunk];
};
__global__ __launch_bounds__(256) void adam_multi_kernel(const AdamChunk c, int n, float lr,
                                                         float b1, float b2, float eps, float bc1,
                                                         float bc2_sqrt) {
  const int64_t b = blockIdx.x;
  int t = 0;
  while (t + 1 < n && c.first_block[t + 1] <= b) ++t;
  const nrms_adam_tensor_t d = c.t[t];
  const int64_t i = (b - c.first_block[t]) * 256 + threadIdx.x;
  if (i >= d.numel) return;
  const float gi = d.grad[i];
  const float mi = d.exp_avg[i] + (1.0f - b1) * (gi - d.exp_avg[i]);
  const float vi = d.exp_avg_sq[i] * b2 + (1.0f - b2) * gi * gi;
  d.exp_avg[i] = mi;
  d.exp_avg_sq[i] = vi;
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  d.param[i] -= (lr / bc1) * (mi / denom);
}

// dst[c][r] = W[r][c] for the stacked segments W = [src_0; src_1; ...]
// (seg_rows rows each, `cols` columns): the [in, out] copy of nn.Linear
// weights that turns dX = dY W into the X W^T form of the store GEMM.
__global__ __launch_bounds__(256) void transpose_kernel(const float* s0, const float* s1,
                                                        const float* s2, int seg_rows, int rows,
                                                        int cols, float* __restrict__ dst) {
  __shared__ float t[32][33];
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
  for (int k = ty; k < 32; k += 8) {
    const int r = r0 + k, c = c0 + tx;
    if (r < rows && c < cols) {
      const int seg = r / seg_rows;
      const float* src = seg == 0 ? s0 : (seg == 1 ? s1 : s2);
      t[k][tx] = src[(int64_t)(r - seg * seg_rows) * cols + c];
    }
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int c = c0 + k, r = r0 + tx;
    if (r < rows && c < cols) dst[(int64_t)c * rows + r] = t[tx][k];
  }
}

inline unsigned grid256(int64_t n) { return (unsigned)((n + 255) / 256); }

}  // namespace

int32_t launch_dropout(const float* x, float* y, int64_t n, float p, uint64_t seed, hipStream_t s) {
  if (n == 0) return NRMS_OK;
  const float scale = p < 1.f ? 1.0f / (1.0f - p) : 0.f;
  hipLaunchKernelGGL(dropout_kernel, dim3(grid256(n)), dim3(256), 0, s, x, y, n, p, scale, seed);
  return launch_status();
}

int32_t launch_score_backward(const float* news, int64_t B, int C, int64_t sb, int64_t sc,
                              const float* user, int64_t su, int D, const float* dl, float* dnews,
                              float* duser, hipStream_t s) {
  if (B == 0) return NRMS_OK;
  hipLaunchKernelGGL(score_backward_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, s, news, B,
                     C, sb, sc, user, su, D, dl, dnews, duser);
  return launch_status();
}

size_t additive_backward_part_floats(int64_t n_seq, int Q) {
  return (size_t)2 * n_seq * Q + 2 * reduce_scratch_floats(n_seq, Q);
}

int32_t launch_additive_backward_rows(const float* x, const float* y, const float* score,
                                      const float* q, const float* dout, int64_t n_seq, int L,
                                      int D, int Q, float* dx, float* dz, float* dq, float* db,
                                      float* part, hipStream_t s) {
  if (n_seq == 0) return NRMS_OK;
  if (L < 1 || L > 64) return NRMS_ERR_UNSUPPORTED;
  if (n_seq > INT32_MAX || !reduce_rows_supported(n_seq)) return NRMS_ERR_UNSUPPORTED;
  float* pq = part;
  float* pb = part + n_seq * Q;
  hipLaunchKernelGGL(additive_backward_rows_kernel, dim3((unsigned)n_seq), dim3(256), 0, s, x, y,
                     score, q, dout, L, D, Q, dx, dz, pq, pb);
  if (int32_t st = launch_status()) return st;
  float* scratch = pb + n_seq * Q;
  if (int32_t st = reduce_rows_add(pq, n_seq, Q, dq, scratch, s)) return st;
  return reduce_rows_add(pb, n_seq, Q, db, scratch + reduce_scratch_floats(n_seq, Q), s);
}

int32_t launch_mhsa_backward(const float* qkv, const float* dctx, int64_t n_seq, int L, int D,
                             int H, float* dqkv, hipStream_t s) {
  if (n_seq == 0) return NRMS_OK;
  if (D != 20 * H || L < 1 || L > 64) return NRMS_ERR_UNSUPPORTED;
  const int64_t blocks = n_seq * H;
  if (blocks > INT32_MAX) return NRMS_ERR_UNSUPPORTED;
  if (L <= 20)   // titles: one wave per (title, head); 297 -> 311 training steps/s
    hipLaunchKernelGGL(mhsa_backward_wave_kernel, dim3((unsigned)((blocks + 3) / 4)), dim3(256), 0,
                       s, qkv, dctx, blocks, L, D, H, dqkv);
  else
    hipLaunchKernelGGL(mhsa_backward_kernel<64>, dim3((unsigned)blocks), dim3(256), 0, s, qkv, dctx,
                       L, D, H, dqkv);
  return launch_status();
}

// row slices of dW += dY^T X: enough blocks to fill the chip, at most
// TN_MAX_SLICES (the partials' workspace does not grow with R)
static int64_t gemm_tn_slices(int N, int K) {
  const int64_t tiles = (int64_t)((N + TN_TILE - 1) / TN_TILE) * ((K + TN_TILE - 1) / TN_TILE);
  const int64_t z = (TN_BLOCKS + tiles - 1) / tiles;
  return z < 1 ? 1 : (z > TN_MAX_SLICES ? TN_MAX_SLICES : z);
}
size_t gemm_tn_part_floats(int N, int K) {
  const int64_t z = gemm_tn_slices(N, K), nk = (int64_t)N * K;
  return (size_t)z * (nk + N) + reduce_scratch_floats(z, nk) + reduce_scratch_floats(z, N);
}

int32_t launch_gemm_tn(const float* dY, int64_t R, int N, const float* X, int K, float* dW,
                       float* db, float* part, hipStream_t s) {
  if (R == 0) return NRMS_OK;
  if (!part) return NRMS_ERR_WORKSPACE;
  // slices of a multiple of 32 rows; zs <= gemm_tn_slices(N, K)
  int64_t slice = (R + gemm_tn_slices(N, K) - 1) / gemm_tn_slices(N, K);
  slice = (slice + TN_BK - 1) / TN_BK * TN_BK;
  const int64_t zs = (R + slice - 1) / slice;
  dim3 grid((N + TN_TILE - 1) / TN_TILE, (K + TN_TILE - 1) / TN_TILE, (unsigned)zs);
  float* part_b = db ? part + zs * (int64_t)N * K : nullptr;
  const bool x6 = gemm_arith() != NRMS_GEMM_F32 && N % 4 == 0 && K % 4 == 0 &&
                  ((uintptr_t)dY | (uintptr_t)X) % 16 == 0;
  if (x6)
    hipLaunchKernelGGL(gemm_tn_x6_kernel, grid, dim3(256), 0, s, dY, R, N, X, K, slice, part, part_b);
  else
    hipLaunchKernelGGL(gemm_tn_kernel, grid, dim3(256), 0, s, dY, R, N, X, K, slice, part, part_b);
  if (int32_t st = launch_status()) return st;
  const int64_t zmax = gemm_tn_slices(N, K), nk = (int64_t)N * K;
  float* scratch = part + zmax * (nk + N);   // (second-pass buffers, zs > RED_CHUNK only)
  if (int32_t st = reduce_rows_add(part, zs, nk, dW, scratch, s)) return st;
  return db ? reduce_rows_add(part_b, zs, N, db, scratch + reduce_scratch_floats(zmax, nk), s) : NRMS_OK;
}

int32_t launch_transpose(const float* const* src, int nseg, int seg_rows, int cols, float* dst,
                         hipStream_t s) {
  const int rows = nseg * seg_rows;
  if (rows == 0 || cols == 0) return NRMS_OK;
  dim3 grid((cols + 31) / 32, (rows + 31) / 32);
  hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, s, src[0], nseg > 1 ? src[1] : src[0],
                     nseg > 2 ? src[2] : src[0], seg_rows, rows, cols, dst);
  return launch_status();
}

int32_t launch_embedding_backward(const int64_t* ids, int64_t n_tok, const float* dx, int64_t V,
                                  int D, int64_t padding_idx, float* dtable, hipStream_t s) {
  if (n_tok == 0) return NRMS_OK;
  hipLaunchKernelGGL(embedding_backward_kernel, dim3((unsigned)((n_tok + 3) / 4)), dim3(256), 0, s,
                     ids, n_tok, dx, V, D, padding_idx, dtable);
  return launch_status();
}

int32_t launch_adam_multi(const nrms_adam_tensor_t* ts, int n, float lr, float b1, float b2,
                          float eps, int64_t step, hipStream_t s) {
  const float bc1 = (float)(1.0 - pow((double)b1, (double)step));
  const float bc2_sqrt = (float)sqrt(1.0 - pow((double)b2, (double)step));
  for (int base = 0; base < n; base += kAdamChunk) {
    AdamChunk c{};
    const int k = n - base < kAdamChunk ? n - base : kAdamChunk;
    int64_t blocks = 0;
    for (int i = 0; i < k; ++i) {
      c.t[i] = ts[base + i];
      c.first_block[i] = blocks;
      blocks += (ts[base + i].numel + 255) / 256;
    }
    if (blocks == 0) continue;
    if (blocks > INT32_MAX) return NRMS_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(adam_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, s, c, k, lr, b1, b2,
                       eps, bc1, bc2_sqrt);
    if (int32_t st = launch_status()) return st;
  }
  return NRMS_OK;
}

int32_t launch_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr, float b1,
                    float b2, float eps, int64_t step, hipStream_t s) {
  if (n == 0) return NRMS_OK;
  // bias corrections in double then rounded, as torch computes them on the host
  const float bc1 = (float)(1.0 - pow((double)b1, (double)step));
  const float bc2_sqrt = (float)sqrt(1.0 - pow((double)b2, (double)step));
  hipLaunchKernelGGL(adam_kernel, dim3(grid256(n)), dim3(256), 0, s, p, g, m, v, n, lr, b1, b2, eps,
                     bc1, bc2_sqrt);
  return launch_status();
}

}  // namespace nrms
