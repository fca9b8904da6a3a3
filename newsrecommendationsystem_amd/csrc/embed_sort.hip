// Deterministic embedding backward (nn.Embedding(padding_idx) backward,
// src/model/NRMS/news_encoder.py:14-20,38): dtable[id] += dx[t] for every
// token t with ids[t] != padding_idx, summed per id in a fixed order, so two
// runs give bitwise the same gradient (the atomic form in train.hip adds in
// arrival order).
//
//   keys:  key[t] = ids[t], or V for padding / out-of-range ids (sorted last)
//   sort:  (key, t) pairs by key, stable LSD radix sort (rocprim::radix_sort_pairs):
//          within one id the tokens stay in ascending t
//   sum:   one wave per sorted position that starts a run of equal keys finds
//          the run's end; a run of at most EMB_LONG tokens is summed by that
//          wave, acc = dtable[id]; acc += dx[t] in token order -- the CPU
//          reference's index_add order, bitwise; a longer run (stopwords and
//          punctuation of real tokenized titles: ~10^3 tokens of one id in a
//          training batch) is listed for embed_long_run_kernel, which sums it
//          in segments of EMB_SEG tokens in parallel (each segment in token
//          order) and adds the segment sums to dtable[id] in segment order:
//          fixed, so bitwise reproducible, and within fp32 rounding of the
//          sequential order.
#include "nrms_common.hpp"

#include <rocprim/device/device_radix_sort.hpp>

namespace nrms {
namespace {

constexpr int EMB_COLS = 5;      // 5 x 64 = 320 columns per pass (D = 300: one pass)
constexpr int EMB_UNROLL = 8;    // tokens whose loads are in flight together
constexpr int EMB_LONG = 256;    // runs past this many tokens are summed in segments
constexpr int EMB_SEG = 64;      // tokens per segment
constexpr int EMB_SW = 16;       // waves (segments in flight) per long run

__global__ __launch_bounds__(256) void embed_keys_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t V,
                                                         int64_t padding_idx, int32_t* __restrict__ key,
                                                         int32_t* __restrict__ tok, int32_t* __restrict__ n_long) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t == 0) *n_long = 0;
  if (t >= n) return;
  const int64_t id = ids[t];
  key[t] = (id == padding_idx || (uint64_t)id >= (uint64_t)V) ? (int32_t)V : (int32_t)id;
  tok[t] = (int32_t)t;
}

// acc[j] (columns d0 + lane + 64 j) += dx[tok[p]] for p in [p0, p1), in order:
// the tok / dx loads of EMB_UNROLL tokens issued ahead of their adds (the loop
// bound is not a load), one add chain per column
__device__ __forceinline__ void sum_tokens(float (&acc)[EMB_COLS], const int32_t* __restrict__ tok, int64_t p0,
                                           int64_t p1, const float* __restrict__ dx, int D, int d0, int lane) {
  int64_t p = p0;
  for (; p + EMB_UNROLL <= p1; p += EMB_UNROLL) {
    // the block's token indices: lanes 0..7 load one each, broadcast
    const int32_t my_t = tok[p + (lane & (EMB_UNROLL - 1))];
    float v[EMB_UNROLL][EMB_COLS];
#pragma unroll
    for (int u = 0; u < EMB_UNROLL; ++u) {
      const float* src = dx + (int64_t)__shfl(my_t, u) * D;
#pragma unroll
      for (int j = 0; j < EMB_COLS; ++j) {
        const int d = d0 + lane + 64 * j;
        v[u][j] = d < D ? src[d] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < EMB_UNROLL; ++u)
#pragma unroll
      for (int j = 0; j < EMB_COLS; ++j) acc[j] += v[u][j];
  }
  for (; p < p1; ++p) {
    const float* src = dx + (int64_t)tok[p] * D;
#pragma unroll
    for (int j = 0; j < EMB_COLS; ++j) {
      const int d = d0 + lane + 64 * j;
      if (d < D) acc[j] += src[d];
    }
  }
}

// one wave per sorted position i; only the first position of each run of
// equal keys works (the others exit at once). The run's end is found first by
// a coalesced scan of the keys (64 per step, a ballot for the first other
// key), so the token loop has a bound that is not a load (it used
// to be key[p], a dependent load per token). Runs of at most EMB_LONG tokens
// are summed here, all of D in one pass (lane l adds columns l + 64 j); longer
// ones go to the long-run list.
__global__ __launch_bounds__(256) void embed_run_sum_kernel(const int32_t* __restrict__ key,
                                                            const int32_t* __restrict__ tok, int64_t n,
                                                            int64_t V, const float* __restrict__ dx, int D,
                                                            float* __restrict__ dtable, int32_t* __restrict__ longs,
                                                            int32_t* __restrict__ n_long) {
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const int32_t k = key[i];
  if (k >= V || (i > 0 && key[i - 1] == k)) return;
  // run end: the first position after i holding another key (or n)
  int64_t end = n;
  for (int64_t p = i + 1; p < n; p += 64) {
    const int64_t q = p + lane;
    const bool other = q >= n || key[q] != k;
    const uint64_t m = __ballot(other);
    if (m) {
      end = p + __builtin_ctzll(m);
      break;
    }
  }
  if (end > n) end = n;
  if (end - i > EMB_LONG) {
    // (list order is arrival order: each run's sum does not depend on it)
    if (lane == 0) {
      const int32_t slot = atomicAdd(n_long, 1);
      longs[2 * slot] = (int32_t)i;
      longs[2 * slot + 1] = (int32_t)end;
    }
    return;
  }
  float* row = dtable + (int64_t)k * D;
  for (int d0 = 0; d0 < D; d0 += 64 * EMB_COLS) {
    float acc[EMB_COLS];
#pragma unroll
    for (int j = 0; j < EMB_COLS; ++j) {
      const int d = d0 + lane + 64 * j;
      acc[j] = d < D ? row[d] : 0.f;
    }
    sum_tokens(acc, tok, i, end, dx, D, d0, lane);
#pragma unroll
    for (int j = 0; j < EMB_COLS; ++j) {
      const int d = d0 + lane + 64 * j;
      if (d < D) row[d] = acc[j];
    }
  }
}

// One workgroup per listed long run (blocks past the list's count exit): its
// EMB_SW waves sum EMB_SW consecutive segments of EMB_SEG tokens at a time,
// each in token order from 0, into LDS; then the row's columns add those
// segment sums in segment order to the running acc (= dtable[id] first).
__global__ __launch_bounds__(64 * EMB_SW) void embed_long_run_kernel(const int32_t* __restrict__ key,
                                                                     const int32_t* __restrict__ tok,
                                                                     const float* __restrict__ dx, int D,
                                                                     float* __restrict__ dtable,
                                                                     const int32_t* __restrict__ longs,
                                                                     const int32_t* __restrict__ n_long) {
  constexpr int W = 64 * EMB_COLS;   // columns per pass
  __shared__ float seg[EMB_SW][W];
  if ((int32_t)blockIdx.x >= *n_long) return;
  const int64_t start = longs[2 * blockIdx.x], end = longs[2 * blockIdx.x + 1];
  const int32_t k = key[start];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int nseg = (int)((end - start + EMB_SEG - 1) / EMB_SEG);
  float* row = dtable + (int64_t)k * D;
  for (int d0 = 0; d0 < D; d0 += W) {
    float acc = (t < W && d0 + t < D) ? row[d0 + t] : 0.f;   // thread t < W: column d0 + t
    for (int s0 = 0; s0 < nseg; s0 += EMB_SW) {
      const int s = s0 + w;
      if (s < nseg) {
        float part[EMB_COLS];
#pragma unroll
        for (int j = 0; j < EMB_COLS; ++j) part[j] = 0.f;
        const int64_t p0 = start + (int64_t)s * EMB_SEG;
        const int64_t p1 = p0 + EMB_SEG < end ? p0 + EMB_SEG : end;
        sum_tokens(part, tok, p0, p1, dx, D, d0, lane);
#pragma unroll
        for (int j = 0; j < EMB_COLS; ++j) seg[w][lane + 64 * j] = part[j];
      }
      __syncthreads();
      if (t < W)
        for (int q = 0; q < EMB_SW && s0 + q < nseg; ++q) acc += seg[q][t];
      __syncthreads();
    }
    if (t < W && d0 + t < D) row[d0 + t] = acc;
  }
}

int end_bit_of(int64_t V) {
  int b = 1;
  while (b < 31 && ((int64_t)1 << b) <= V) ++b;   // keys 0..V fit in b bits
  return b;
}

size_t sort_temp_bytes(int64_t n, int64_t V) {
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs(nullptr, bytes, (const int32_t*)nullptr, (int32_t*)nullptr,
                                  (const int32_t*)nullptr, (int32_t*)nullptr, (size_t)n, 0u,
                                  (unsigned)end_bit_of(V), (hipStream_t)0);
  return bytes;
}

constexpr size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }
// most runs longer than EMB_LONG among n tokens
inline int64_t max_long_runs(int64_t n) { return n / (EMB_LONG + 1) + 1; }

}  // namespace

// [key in | tok in | key out | tok out] (n int32 each), the long-run list
// (count + 2 int32 per run), then the sort's temporary storage
size_t embedding_backward_sorted_bytes(int64_t n_tok, int64_t V) {
  if (n_tok <= 0 || n_tok > INT32_MAX || V <= 0 || V >= INT32_MAX) return 0;
  return 4 * align256((size_t)n_tok * 4) + align256((size_t)(1 + 2 * max_long_runs(n_tok)) * 4) +
         align256(sort_temp_bytes(n_tok, V));
}

int32_t launch_embedding_backward_sorted(const int64_t* ids, int64_t n_tok, const float* dx, int64_t V, int D,
                                         int64_t padding_idx, float* dtable, void* ws, size_t ws_bytes,
                                         hipStream_t s) {
  if (n_tok == 0) return NRMS_OK;
  if (n_tok > INT32_MAX || V >= INT32_MAX) return NRMS_ERR_UNSUPPORTED;
  if (!ws || ws_bytes < embedding_backward_sorted_bytes(n_tok, V)) return NRMS_ERR_WORKSPACE;
  char* p = static_cast<char*>(ws);
  const size_t a = align256((size_t)n_tok * 4);
  const size_t la = align256((size_t)(1 + 2 * max_long_runs(n_tok)) * 4);
  int32_t* key_in = reinterpret_cast<int32_t*>(p);
  int32_t* tok_in = reinterpret_cast<int32_t*>(p + a);
  int32_t* key_out = reinterpret_cast<int32_t*>(p + 2 * a);
  int32_t* tok_out = reinterpret_cast<int32_t*>(p + 3 * a);
  int32_t* n_long = reinterpret_cast<int32_t*>(p + 4 * a);
  int32_t* longs = n_long + 1;
  void* temp = p + 4 * a + la;
  size_t temp_bytes = ws_bytes - 4 * a - la;
  hipLaunchKernelGGL(embed_keys_kernel, dim3((unsigned)((n_tok + 255) / 256)), dim3(256), 0, s, ids, n_tok, V,
                     padding_idx, key_in, tok_in, n_long);
  if (int32_t st = launch_status()) return st;
  const hipError_t e = rocprim::radix_sort_pairs(temp, temp_bytes, key_in, key_out, tok_in, tok_out,
                                                 (size_t)n_tok, 0u, (unsigned)end_bit_of(V), s);
  if (e != hipSuccess) {
    set_last_hip_error(e);
    return NRMS_ERR_HIP;
  }
  hipLaunchKernelGGL(embed_run_sum_kernel, dim3((unsigned)((n_tok + 3) / 4)), dim3(256), 0, s, key_out, tok_out,
                     n_tok, V, dx, D, dtable, longs, n_long);
  if (int32_t st = launch_status()) return st;
  hipLaunchKernelGGL(embed_long_run_kernel, dim3((unsigned)max_long_runs(n_tok)), dim3(64 * EMB_SW), 0, s,
                     key_out, tok_out, dx, D, dtable, longs, n_long);
  return launch_status();
}

}  // namespace nrms
