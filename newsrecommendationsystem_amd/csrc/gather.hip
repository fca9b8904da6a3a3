// Embedding row gather (nn.Embedding forward, src/model/NRMS/news_encoder.py:38).
// HBM-bound: 16-B lanes, each 1200-B row read by consecutive lanes, output
// written fully contiguous. Bit-exact copy; id 0 is an ordinary row.
#include "nrms_common.hpp"

namespace nrms {
namespace {

constexpr int kGatherThreads = 256;
constexpr int kRowsPerBlock = 64;
constexpr int kUnroll = 4;

// D4 = row length in float4 units (75 for D = 300); compile-time so that the
// row/column split of the flat index is a multiply-shift, not a division.
template <int D4>
__global__ __launch_bounds__(kGatherThreads) void gather_rows_kernel(
    const int64_t* __restrict__ ids, int64_t n_tok, const float4* __restrict__ table, int64_t V,
    float4* __restrict__ out) {
  const int64_t r0 = (int64_t)blockIdx.x * kRowsPerBlock;
  const int rows = (int)min<int64_t>(kRowsPerBlock, n_tok - r0);
  const int total = rows * D4;
  const int64_t* id_blk = ids + r0;
  float4* out_blk = out + r0 * D4;
  for (int base = threadIdx.x; base < total; base += kGatherThreads * kUnroll) {
    float4 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int i = base + u * kGatherThreads;
      if (i < total) {
        const int r = i / D4;
        const int c = i - r * D4;
        const int64_t id = id_blk[r];
        v[u] = ((uint64_t)id < (uint64_t)V) ? table[id * D4 + c] : nan4();
      }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int i = base + u * kGatherThreads;
      if (i < total) out_blk[i] = v[u];
    }
  }
}

// Generic D (any D, scalar lanes).
__global__ __launch_bounds__(kGatherThreads) void gather_rows_scalar_kernel(
    const int64_t* __restrict__ ids, int64_t n_tok, const float* __restrict__ table, int64_t V,
    int D, float* __restrict__ out) {
  const int64_t t = blockIdx.x;
  const int64_t id = ids[t];
  const bool ok = (uint64_t)id < (uint64_t)V;
  for (int c = threadIdx.x; c < D; c += kGatherThreads)
    out[t * D + c] = ok ? table[id * D + c] : qnan();
}

}  // namespace

int32_t launch_gather(const int64_t* ids, int64_t n_tok, const float* table, int64_t V, int D,
                      float* out, hipStream_t s) {
  if (n_tok == 0) return NRMS_OK;
  const bool aligned = ((uintptr_t)table % 16 == 0) && ((uintptr_t)out % 16 == 0) && (D % 4 == 0);
  if (aligned && D == 300) {
    const int64_t blocks = (n_tok + kRowsPerBlock - 1) / kRowsPerBlock;
    hipLaunchKernelGGL(gather_rows_kernel<75>, dim3((unsigned)blocks), dim3(kGatherThreads), 0, s,
                       ids, n_tok, reinterpret_cast<const float4*>(table), V,
                       reinterpret_cast<float4*>(out));
  } else {
    hipLaunchKernelGGL(gather_rows_scalar_kernel, dim3((unsigned)n_tok), dim3(kGatherThreads), 0, s,
                       ids, n_tok, table, V, D, out);
  }
  return launch_status();
}

}  // namespace nrms
