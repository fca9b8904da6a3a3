// Multi-head raw-exp self-attention and additive-attention pooling.
//
// mhsa_rawexp_kernel restates ScaledDotProductAttention
// (src/model/general/attention/multihead_self.py:15-23) exactly as the
// reference normalises: e = exp(QK^T / sqrt(d_k)) with NO max subtraction,
// attn = e / (sum(e) + 1e-8), ctx = attn · V, heads concatenated in head
// order (:74-75). Overflow therefore yields inf/inf = NaN and all-underflow
// yields a zero context, as in the reference.
//
// One workgroup per sequence (a title, L = 20, or a user history, L = 50).
// K|V of the whole sequence (L x 2D floats) are staged once in LDS; each lane
// owns one (query token, head) task: its q slice lives in registers, the L raw
// exps stay in registers between the two passes, and K/V rows are read with
// ds_read_b128 (lanes of one head read the same address: broadcast).
//
// additive_pool_kernel restates the second half of AdditiveAttention
// (src/model/general/attention/additive.py:37-52): a standard max-subtracted
// softmax over the per-token scores (produced by the fused GEMM epilogue) and
// the weighted sum of the token rows. One wave per sequence.
#include "nrms_common.hpp"


namespace nrms {
namespace {

template <int LMAX, int DK, int H, int NT>
__global__ __launch_bounds__(NT) void mhsa_rawexp_kernel(
    const float* __restrict__ qkv, int64_t ld, int64_t n_rows, const int64_t* __restrict__ ids_a,
    int64_t n_seq_a, const int64_t* __restrict__ ids_b, int L, float* __restrict__ ctx) {
  extern __shared__ __attribute__((aligned(16))) float kv[];  // [L][2D] then row ids
  constexpr int D = H * DK;
  const int64_t s = blockIdx.x;
  const int tid = threadIdx.x;

  const int64_t* ids = nullptr;
  if (ids_a) ids = (s < n_seq_a || ids_b == nullptr) ? ids_a + s * L : ids_b + (s - n_seq_a) * L;
  int64_t* rowidx = reinterpret_cast<int64_t*>(kv + (size_t)L * 2 * D);
  for (int i = tid; i < L; i += NT) {
    const int64_t r = ids ? ids[i] : s * L + i;
    rowidx[i] = ((uint64_t)r < (uint64_t)n_rows) ? r : -1;
  }
  __syncthreads();

  constexpr int d2q = (2 * D) / 4;  // float4 per K|V row
  for (int e = tid; e < L * d2q; e += NT) {
    const int i = e / d2q;
    const int c = e - i * d2q;
    const int64_t r = rowidx[i];
    const float4 v = r >= 0 ? *reinterpret_cast<const float4*>(qkv + r * ld + D + 4 * c) : nan4();
    *reinterpret_cast<float4*>(kv + (size_t)i * 2 * D + 4 * c) = v;
  }
  __syncthreads();

  // fast path exp2(d * log2(e) / sqrt(d_k)); exact path for rows near overflow
  const float c_exp = 1.4426950408889634f / sqrtf((float)DK);
  const float sqrt_dk = sqrtf((float)DK);
  for (int task = tid; task < L * H; task += NT) {
    const int h = task / L;
    const int i = task - h * L;
    const int64_t r = rowidx[i];

    float q[DK];
    if (r >= 0) {
      const float4* qp = reinterpret_cast<const float4*>(qkv + r * ld + h * DK);
#pragma unroll
      for (int t = 0; t < DK / 4; ++t) {
        const float4 v = qp[t];
        q[4 * t] = v.x; q[4 * t + 1] = v.y; q[4 * t + 2] = v.z; q[4 * t + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int t = 0; t < DK; ++t) q[t] = qnan();
    }

    auto dot = [&](int j) {
      const float4* kr = reinterpret_cast<const float4*>(kv + (size_t)j * 2 * D + h * DK);
      float d = 0.f;
#pragma unroll
      for (int t = 0; t < DK / 4; ++t) {
        const float4 k4 = kr[t];
        d = fmaf(q[4 * t], k4.x, d);
        d = fmaf(q[4 * t + 1], k4.y, d);
        d = fmaf(q[4 * t + 2], k4.z, d);
        d = fmaf(q[4 * t + 3], k4.w, d);
      }
      return d;
    };
    float e[LMAX];
    float sum = 0.f;
#pragma unroll
    for (int j = 0; j < LMAX; ++j) {
      e[j] = j < L ? __builtin_amdgcn_exp2f(dot(j) * c_exp) : 0.f;
      sum += e[j];
    }
    if (exp_row_needs_recheck(sum)) {   // rare: rows near fp32 overflow (nrms_common.hpp)
      sum = 0.f;
#pragma unroll
      for (int j = 0; j < LMAX; ++j) {
        e[j] = j < L ? ref_exp(dot(j), sqrt_dk) : 0.f;
        sum += e[j];
      }
    }
    const float inv = 1.0f / (sum + 1e-8f);

    float acc[DK];
#pragma unroll
    for (int t = 0; t < DK; ++t) acc[t] = 0.f;
#pragma unroll
    for (int j = 0; j < LMAX; ++j) {
      if (j < L) {
        const float a = e[j] * inv;
        const float4* vr = reinterpret_cast<const float4*>(kv + (size_t)j * 2 * D + D + h * DK);
#pragma unroll
        for (int t = 0; t < DK / 4; ++t) {
          const float4 v4 = vr[t];
          acc[4 * t] = fmaf(a, v4.x, acc[4 * t]);
          acc[4 * t + 1] = fmaf(a, v4.y, acc[4 * t + 1]);
          acc[4 * t + 2] = fmaf(a, v4.z, acc[4 * t + 2]);
          acc[4 * t + 3] = fmaf(a, v4.w, acc[4 * t + 3]);
        }
      }
    }
    float4* op = reinterpret_cast<float4*>(ctx + (s * L + i) * D + h * DK);
#pragma unroll
    for (int t = 0; t < DK / 4; ++t)
      op[t] = make_float4(acc[4 * t], acc[4 * t + 1], acc[4 * t + 2], acc[4 * t + 3]);
  }
}

// Histories longer than 64 (K|V no longer fit LDS next to the exps in
// registers): K|V rows read through L2, the raw exps computed twice (a sum
// pass, then an accumulate pass; expf is deterministic, so the weights equal a
// single-pass evaluation). Same arithmetic order per (query, head) as above.
constexpr int kLongThreads = 256;

__global__ __launch_bounds__(kLongThreads) void mhsa_rawexp_long_kernel(
    const float* __restrict__ qkv, int64_t ld, int64_t n_rows, const int64_t* __restrict__ ids_a,
    int64_t n_seq_a, const int64_t* __restrict__ ids_b, int L, float* __restrict__ ctx) {
  constexpr int DK = 20, H = 15, D = H * DK;
  extern __shared__ __attribute__((aligned(16))) int64_t lrow[];   // [L] row ids
  const int64_t s = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t* ids = nullptr;
  if (ids_a) ids = (s < n_seq_a || ids_b == nullptr) ? ids_a + s * L : ids_b + (s - n_seq_a) * L;
  for (int i = tid; i < L; i += kLongThreads) {
    const int64_t r = ids ? ids[i] : s * L + i;
    lrow[i] = ((uint64_t)r < (uint64_t)n_rows) ? r : -1;
  }
  __syncthreads();
  const float c_exp = 1.4426950408889634f / sqrtf((float)DK);
  const float sqrt_dk = sqrtf((float)DK);
  for (int task = tid; task < L * H; task += kLongThreads) {
    const int h = task / L;
    const int i = task - h * L;
    const int64_t r = lrow[i];
    float q[DK];
#pragma unroll
    for (int t = 0; t < DK / 4; ++t) {
      const float4 v = r >= 0 ? reinterpret_cast<const float4*>(qkv + r * ld + h * DK)[t] : nan4();
      q[4 * t] = v.x; q[4 * t + 1] = v.y; q[4 * t + 2] = v.z; q[4 * t + 3] = v.w;
    }
    bool exact = false;   // the row takes the reference's exp (kExpRecheck)
    auto raw = [&](int j) {
      const int64_t rj = lrow[j];
      float d = 0.f;
#pragma unroll
      for (int t = 0; t < DK / 4; ++t) {
        const float4 k4 = rj >= 0 ? reinterpret_cast<const float4*>(qkv + rj * ld + D + h * DK)[t]
                                  : nan4();
        d = fmaf(q[4 * t], k4.x, d);
        d = fmaf(q[4 * t + 1], k4.y, d);
        d = fmaf(q[4 * t + 2], k4.z, d);
        d = fmaf(q[4 * t + 3], k4.w, d);
      }
      return exact ? ref_exp(d, sqrt_dk) : __builtin_amdgcn_exp2f(d * c_exp);
    };
    float sum = 0.f;
    for (int j = 0; j < L; ++j) sum += raw(j);
    if (exp_row_needs_recheck(sum)) {
      exact = true;
      sum = 0.f;
      for (int j = 0; j < L; ++j) sum += raw(j);
    }
    const float inv = 1.0f / (sum + 1e-8f);
    float acc[DK];
#pragma unroll
    for (int t = 0; t < DK; ++t) acc[t] = 0.f;
    for (int j = 0; j < L; ++j) {
      const float a = raw(j) * inv;
      const int64_t rj = lrow[j];
#pragma unroll
      for (int t = 0; t < DK / 4; ++t) {
        const float4 v4 = rj >= 0
            ? reinterpret_cast<const float4*>(qkv + rj * ld + 2 * D + h * DK)[t] : nan4();
        acc[4 * t] = fmaf(a, v4.x, acc[4 * t]);
        acc[4 * t + 1] = fmaf(a, v4.y, acc[4 * t + 1]);
        acc[4 * t + 2] = fmaf(a, v4.z, acc[4 * t + 2]);
        acc[4 * t + 3] = fmaf(a, v4.w, acc[4 * t + 3]);
      }
    }
    float4* op = reinterpret_cast<float4*>(ctx + (s * L + i) * D + h * DK);
#pragma unroll
    for (int t = 0; t < DK / 4; ++t)
      op[t] = make_float4(acc[4 * t], acc[4 * t + 1], acc[4 * t + 2], acc[4 * t + 3]);
  }
}

constexpr int kPoolThreads = 256;

__global__ __launch_bounds__(kPoolThreads) void additive_pool_kernel(
    const float* __restrict__ x, const float* __restrict__ score, int64_t n_seq, int L, int D,
    float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t s = (int64_t)blockIdx.x * (kPoolThreads / kWave) + (threadIdx.x >> 6);
  if (s >= n_seq) return;
  const float* sc = score + s * L;
  const int d4 = D / 4;
  const float4* xs = reinterpret_cast<const float4*>(x + s * L * D);
  float4* os = reinterpret_cast<float4*>(out + s * D);
  if (L > kWave) {   // long sequence: strided max / sum, weights recomputed per row
    float m = -INFINITY;
    for (int l = lane; l < L; l += kWave) m = nan_max(m, sc[l]);
    m = wave_max_nan(m);
    float se = 0.f;
    for (int l = lane; l < L; l += kWave) se += expf(sc[l] - m);
    const float sum = wave_sum(se);
    for (int c = lane; c < d4; c += kWave) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int l = 0; l < L; ++l) {
        const float wl = expf(sc[l] - m) / sum;
        const float4 xv = xs[(int64_t)l * d4 + c];
        acc.x = fmaf(wl, xv.x, acc.x);
        acc.y = fmaf(wl, xv.y, acc.y);
        acc.z = fmaf(wl, xv.z, acc.z);
        acc.w = fmaf(wl, xv.w, acc.w);
      }
      os[c] = acc;
    }
    return;
  }
  const float v = lane < L ? sc[lane] : -INFINITY;
  const float m = wave_max_nan(v);
  const float e = lane < L ? expf(v - m) : 0.f;
  const float sum = wave_sum(e);
  const float w = e / sum;
  // The shuffle must run with every lane active (a bpermute from an inactive
  // lane reads garbage), so the column guard sits inside the l-loop.
  for (int c0 = 0; c0 < d4; c0 += kWave) {
    const int c = c0 + lane;
    const bool live = c < d4;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int l = 0; l < L; ++l) {
      const float wl = __shfl(w, l);
      if (live) {
        const float4 xv = xs[l * d4 + c];
        acc.x = fmaf(wl, xv.x, acc.x);
        acc.y = fmaf(wl, xv.y, acc.y);
        acc.z = fmaf(wl, xv.z, acc.z);
        acc.w = fmaf(wl, xv.w, acc.w);
      }
    }
    if (live) os[c] = acc;
  }
}

template <int LMAX, int NT>
int32_t launch_mhsa_inst(const float* qkv, int64_t ld, int64_t n_rows, const int64_t* ids_a, int64_t n_seq_a,
                         const int64_t* ids_b, int64_t n_seq, int L, float* ctx, hipStream_t s) {
  constexpr int DK = 20, H = 15;
  constexpr int D = H * DK;
  const size_t lds = (size_t)L * 2 * D * sizeof(float) + (size_t)L * sizeof(int64_t);
  if (lds > 160 * 1024) return NRMS_ERR_UNSUPPORTED;
  ensure_dynamic_lds(reinterpret_cast<const void*>(&mhsa_rawexp_kernel<LMAX, DK, H, NT>),
                     160 * 1024);
  hipLaunchKernelGGL((mhsa_rawexp_kernel<LMAX, DK, H, NT>), dim3((unsigned)n_seq), dim3(NT), lds,
                     s, qkv, ld, n_rows, ids_a, n_seq_a, ids_b, L, ctx);
  return launch_status();
}

}  // namespace

int32_t launch_mhsa(const float* qkv, int64_t ld, int64_t n_rows, const int64_t* ids_a, int64_t n_seq_a,
                    const int64_t* ids_b, int64_t n_seq, int L, int H, int DK, float* ctx,
                    hipStream_t s) {
  if (n_seq == 0) return NRMS_OK;
  // Compiled for the reference configuration: d_k = 20, 15 heads (config.py:34,45).
  if (DK != 20 || H != 15 || L < 1 || L > kMaxSeqLen) return NRMS_ERR_UNSUPPORTED;
  // q|k|v rows: [q D | k D | v D] at any row stride that keeps the float4 slices aligned
  if (ld < 3 * (int64_t)H * DK || ld % 4 != 0) return NRMS_ERR_UNSUPPORTED;
  if (((uintptr_t)qkv % 16) != 0 || ((uintptr_t)ctx % 16) != 0) return NRMS_ERR_UNSUPPORTED;
  if (n_seq > INT32_MAX) return NRMS_ERR_UNSUPPORTED;
  if (L > 64) {
    hipLaunchKernelGGL(mhsa_rawexp_long_kernel, dim3((unsigned)n_seq), dim3(kLongThreads),
                       (size_t)L * sizeof(int64_t), s, qkv, ld, n_rows, ids_a, n_seq_a, ids_b, L, ctx);
    return launch_status();
  }
  if (L <= 20) return launch_mhsa_inst<20, 320>(qkv, ld, n_rows, ids_a, n_seq_a, ids_b, n_seq, L, ctx, s);
  if (L <= 32) return launch_mhsa_inst<32, 512>(qkv, ld, n_rows, ids_a, n_seq_a, ids_b, n_seq, L, ctx, s);
  if (L <= 50) return launch_mhsa_inst<50, 768>(qkv, ld, n_rows, ids_a, n_seq_a, ids_b, n_seq, L, ctx, s);
  return launch_mhsa_inst<64, 1024>(qkv, ld, n_rows, ids_a, n_seq_a, ids_b, n_seq, L, ctx, s);
}

int32_t launch_additive_pool(const float* x, const float* score, int64_t n_seq, int L, int D,
                             float* out, hipStream_t s) {
  if (n_seq == 0) return NRMS_OK;
  if (L < 1 || L > kMaxSeqLen || D % 4 != 0) return NRMS_ERR_UNSUPPORTED;
  if (((uintptr_t)x % 16) != 0 || ((uintptr_t)out % 16) != 0) return NRMS_ERR_UNSUPPORTED;
  const int per = kPoolThreads / kWave;
  const int64_t blocks = (n_seq + per - 1) / per;
  hipLaunchKernelGGL(additive_pool_kernel, dim3((unsigned)blocks), dim3(kPoolThreads), 0, s, x,
                     score, n_seq, L, D, out);
  return launch_status();
}

}  // namespace nrms
