// Two waves on one SIMD: does one wave's MFMA stream overlap the other wave's
// VALU (or MFMA) stream? Workgroup of 8 waves (wave w and w + 4 share SIMD
// w % 4); waves 0-3 run stream X, waves 4-7 stream Y, each ITERS iterations;
// cycles per iteration of the slower team (s_memtime) and kernel wall time.
//   hipcc -O3 --offload-arch=gfx950 simd_share_probe.hip -o /tmp/simd_share && /tmp/simd_share
// Streams: 0 idle, 1 = 8 x v_mfma_f32_4x4x1_16b_f32 (8 accumulators),
// 2 = 64 v_fma_f32 (8 chains), 3 = 8 x v_mfma_f32_16x16x32_f16 (8 accumulators),
// 4 = 16 v_exp_f32 (8 chains), 5 = 8 x v_mfma_f32_4x4x4_16b_f16.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef _Float16 halfx4 __attribute__((ext_vector_type(4)));
typedef _Float16 halfx8 __attribute__((ext_vector_type(8)));

template <int KIND>
__device__ __forceinline__ void stream(int iters, float a, float b, float* out) {
  floatx4 acc[8];
  float v[8];
  for (int i = 0; i < 8; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < 8; ++c) v[c] = a + c;
  const halfx4 h4 = {(_Float16)a, (_Float16)b, (_Float16)a, (_Float16)b};
  const halfx8 h8 = {(_Float16)a, (_Float16)b, (_Float16)a, (_Float16)b, (_Float16)a, (_Float16)b, (_Float16)a, (_Float16)b};
  for (int it = 0; it < iters; ++it) {
    if constexpr (KIND == 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[i], 0, 0, 0);
    } else if constexpr (KIND == 2) {
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = fmaf(v[c], b, a);
      asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]));
    } else if constexpr (KIND == 3) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(h8, h8, acc[i], 0, 0, 0);
    } else if constexpr (KIND == 4) {
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = __builtin_amdgcn_exp2f(v[c] * b);
      asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]));
    } else if constexpr (KIND == 5) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f32_4x4x4f16(h4, h4, acc[i], 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  for (int c = 0; c < 8; ++c) s += v[c];
  if (s == 1234.5f) out[threadIdx.x] = s;
}

template <int X, int Y>
__global__ __launch_bounds__(512) void probe(float* out, long long* cyc, int iters) {
  const int w = threadIdx.x >> 6;
  const float a = threadIdx.x * 1e-3f, b = 1.0f - threadIdx.x * 1e-4f;
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  if (w < 4) stream<X>(iters, a, b, out);
  else stream<Y>(iters, a, b, out);
  const long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}

static const char* NAMES[] = {"idle", "4x4x1_f32 x8", "64 fma", "16x16x32_f16 x8", "16 exp", "4x4x4_f16 x8"};

template <int X, int Y>
void run(float* out, long long* cyc, int iters, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((probe<X, Y>), dim3(blocks), dim3(512), 0, 0, out, cyc, iters);
  hipEventRecord(e0);
  hipLaunchKernelGGL((probe<X, Y>), dim3(blocks), dim3(512), 0, 0, out, cyc, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  long long h[8 * 256];
  hipMemcpy(h, cyc, sizeof(long long) * 8 * blocks, hipMemcpyDeviceToHost);
  double cx = 0, cy = 0;
  for (int b = 0; b < blocks; ++b)
    for (int w = 0; w < 8; ++w) (w < 4 ? cx : cy) += (double)h[b * 8 + w];
  cx /= 4.0 * blocks * iters;
  cy /= 4.0 * blocks * iters;
  printf("X=%-16s Y=%-16s  cycles/iter: X %7.2f  Y %7.2f   wall %.3f ms\n", NAMES[X], NAMES[Y], cx, cy, ms);
}

int main() {
  float* out;
  long long* cyc;
  hipMalloc(&out, 4096 * 4);
  hipMalloc(&cyc, 8 * 256 * 8);
  const int iters = 20000, blocks = 256;
#define R(X, Y) run<X, Y>(out, cyc, iters, blocks);
  R(1, 0) R(0, 2) R(1, 2) R(2, 2)
  R(3, 0) R(3, 2) R(3, 4) R(0, 4) R(1, 4)
  R(3, 1) R(1, 1) R(3, 3)
  R(5, 0) R(5, 2) R(5, 4)
  return 0;
}
