// Issue rate of the small (4x4, 16-block) MFMA forms on gfx950 and whether
// independent VALU work co-issues with them (one wave per SIMD):
//   hipcc -O3 --offload-arch=gfx950 mfma_coissue_probe.hip -o /tmp/mfma_coissue && /tmp/mfma_coissue
// Each kernel runs ITERS iterations of {NACC MFMAs on independent
// accumulators, NV independent fma per VALU chain over 8 chains}; cycles per
// iteration from s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef _Float16 halfx4 __attribute__((ext_vector_type(4)));
typedef short shortx4 __attribute__((ext_vector_type(4)));

template <int KIND, int NACC, int NV>
__global__ void probe_kernel(float* out, long long* cyc, int iters) {
  floatx4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
  const float a = threadIdx.x * 1e-3f, b = 1.0f - threadIdx.x * 1e-4f;
  const halfx4 ah = {(_Float16)a, (_Float16)b, (_Float16)a, (_Float16)b};
  const shortx4 as = {(short)threadIdx.x, 3, 5, 7};
  float v[8];
  for (int c = 0; c < 8; ++c) v[c] = a + c;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
      if constexpr (KIND == 0) acc[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[i], 0, 0, 0);
      if constexpr (KIND == 1) acc[i] = __builtin_amdgcn_mfma_f32_4x4x4f16(ah, ah, acc[i], 0, 0, 0);
      if constexpr (KIND == 2) acc[i] = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(as, as, acc[i], 0, 0, 0);
      if constexpr (KIND == 3) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
#pragma unroll
      for (int k = 0; k < NV; ++k)
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = fmaf(v[c], b, a);
    }
  }
  const long long t1 = clock64();
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  for (int c = 0; c < 8; ++c) s += v[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND, int NACC, int NV>
void run(const char* name, float* dout, long long* dcyc) {
  const int iters = 2048;
  hipLaunchKernelGGL((probe_kernel<KIND, NACC, NV>), dim3(1), dim3(256), 0, 0, dout, dcyc, iters);
  hipDeviceSynchronize();
  long long hc = 0;
  hipMemcpy(&hc, dcyc, 8, hipMemcpyDeviceToHost);
  const double per = (double)hc / (iters * (double)NACC);
  printf("%-14s NACC %2d, %2d VALU fma per MFMA: %7.2f cycles per MFMA (+VALU)\n", name, NACC, 8 * NV, per);
}

int main() {
  float* dout;
  long long* dcyc;
  hipMalloc(&dout, 1 << 20);
  hipMalloc(&dcyc, 4096 * 8);
  run<0, 8, 0>("4x4x1 f32", dout, dcyc);
  run<0, 8, 1>("4x4x1 f32", dout, dcyc);
  run<0, 8, 2>("4x4x1 f32", dout, dcyc);
  run<1, 8, 0>("4x4x4 f16", dout, dcyc);
  run<1, 8, 1>("4x4x4 f16", dout, dcyc);
  run<1, 8, 2>("4x4x4 f16", dout, dcyc);
  run<2, 8, 0>("4x4x4 bf16", dout, dcyc);
  run<2, 8, 1>("4x4x4 bf16", dout, dcyc);
  run<3, 8, 0>("16x16x4 f32", dout, dcyc);
  run<3, 8, 1>("16x16x4 f32", dout, dcyc);
  run<3, 8, 2>("16x16x4 f32", dout, dcyc);
  run<9, 8, 1>("VALU only", dout, dcyc);
  run<9, 8, 2>("VALU only", dout, dcyc);
  return 0;
}
