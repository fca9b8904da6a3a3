// Probe of v_mfma_f32_4x4x1_16b_f32 on gfx950: operand/result lane layout and
// issue rate (one wave per SIMD, independent accumulators).
//   hipcc -O3 --offload-arch=gfx950 mfma4x4_probe.hip -o /tmp/mfma4x4_probe && /tmp/mfma4x4_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx4 __attribute__((ext_vector_type(4)));

__global__ void layout_kernel(float* outA, float* outB) {
  const int l = threadIdx.x;
  floatx4 z = {0.f, 0.f, 0.f, 0.f};
  // run 1: B = 1 -> D = A value of the contributing lane
  floatx4 d1 = __builtin_amdgcn_mfma_f32_4x4x1f32((float)l, 1.0f, z, 0, 0, 0);
  // run 2: A = 1 -> D = B value of the contributing lane
  floatx4 d2 = __builtin_amdgcn_mfma_f32_4x4x1f32(1.0f, (float)l, z, 0, 0, 0);
  for (int r = 0; r < 4; ++r) {
    outA[l * 4 + r] = d1[r];
    outB[l * 4 + r] = d2[r];
  }
}

template <int NACC>
__global__ void rate_kernel(float* out, long long* cyc, int iters) {
  floatx4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
  float a = threadIdx.x * 1e-3f, b = 1.0f - threadIdx.x * 1e-4f;
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[i], 0, 0, 0);
  }
  long long t1 = clock64();
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NACC>
__global__ void rate16_kernel(float* out, long long* cyc, int iters) {
  floatx4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = floatx4{0.f, 0.f, 0.f, 0.f};
  float a = threadIdx.x * 1e-3f, b = 1.0f - threadIdx.x * 1e-4f;
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  long long t1 = clock64();
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float *dA, *dB, *dout;
  long long* dcyc;
  hipMalloc(&dA, 256 * 4);
  hipMalloc(&dB, 256 * 4);
  hipMalloc(&dout, 1 << 20);
  hipMalloc(&dcyc, 4096 * 8);
  hipLaunchKernelGGL(layout_kernel, dim3(1), dim3(64), 0, 0, dA, dB);
  float hA[256], hB[256];
  hipMemcpy(hA, dA, 1024, hipMemcpyDeviceToHost);
  hipMemcpy(hB, dB, 1024, hipMemcpyDeviceToHost);
  printf("lane: vgpr0..3 = (A-lane, B-lane)\n");
  for (int l = 0; l < 64; ++l) {
    printf("%2d:", l);
    for (int r = 0; r < 4; ++r) printf(" (%2d,%2d)", (int)hA[l * 4 + r], (int)hB[l * 4 + r]);
    printf("\n");
  }
  const int iters = 4096;
  long long hc[4];
  hipLaunchKernelGGL(rate_kernel<8>, dim3(1), dim3(64), 0, 0, dout, dcyc, iters);
  hipDeviceSynchronize();
  hipMemcpy(hc, dcyc, 8, hipMemcpyDeviceToHost);
  printf("4x4x1_16b: %.2f cycles per MFMA (8 independent acc, 1 wave)\n", (double)hc[0] / (iters * 8.0));
  hipLaunchKernelGGL(rate_kernel<16>, dim3(1), dim3(64), 0, 0, dout, dcyc, iters);
  hipDeviceSynchronize();
  hipMemcpy(hc, dcyc, 8, hipMemcpyDeviceToHost);
  printf("4x4x1_16b: %.2f cycles per MFMA (16 independent acc, 1 wave)\n", (double)hc[0] / (iters * 16.0));
  hipLaunchKernelGGL(rate_kernel<2>, dim3(1), dim3(64), 0, 0, dout, dcyc, iters);
  hipDeviceSynchronize();
  hipMemcpy(hc, dcyc, 8, hipMemcpyDeviceToHost);
  printf("4x4x1_16b: %.2f cycles per MFMA (2 independent acc, 1 wave)\n", (double)hc[0] / (iters * 2.0));
  hipLaunchKernelGGL(rate16_kernel<8>, dim3(1), dim3(64), 0, 0, dout, dcyc, iters);
  hipDeviceSynchronize();
  hipMemcpy(hc, dcyc, 8, hipMemcpyDeviceToHost);
  printf("16x16x4:   %.2f cycles per MFMA (8 independent acc, 1 wave)\n", (double)hc[0] / (iters * 8.0));
  return 0;
}
