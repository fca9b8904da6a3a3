// Phase-A attention of the news kernel (S = K Q^T and ctx = V^T P^T for the
// 16 (title, head) pairs of one wave and one title group of NB key blocks) in
// its two candidate MFMA forms, operands already in registers (the best case
// for the 16-bit form: no extra loads, no layout moves):
//   f32   : v_mfma_f32_4x4x1_16b_f32, 20 NB^2 + 20 NB^2 instructions (round 1..6);
//   f16x3 : v_mfma_f32_4x4x4_16b_f16 with split operands, q = qh + 2^-11 ql
//           (the same for k, v and p): three products per 4 K elements, 15 NB^2
//           + 15 NB^2 instructions, plus the splits of q, k, v (per group) and
//           of p (per group), the 2^-11 recombination of S, on the VALU.
// One wave per SIMD (256-thread blocks, one per CU), cycles per group from
// clock64 around ITERS groups, median over the waves. The exp / softmax work
// both forms share is left out.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 attn_forms_probe.hip -o /tmp/attn_forms && /tmp/attn_forms
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));

constexpr int ITERS = 64;

// every element of a register array opaque to the compiler (no instruction)
__device__ __forceinline__ void opaque(float& x) { asm volatile("" : "+v"(x)); }
template <typename T, int N>
__device__ __forceinline__ void opaque(T (&x)[N]);
template <int N>
__device__ __forceinline__ void opaque(float (&x)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) opaque(x[i]);
}
template <typename T, int N>
__device__ __forceinline__ void opaque(T (&x)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) opaque(x[i]);
}
constexpr float kLo = 2048.f;

template <int NB>
__global__ __launch_bounds__(256, 1) void f32_form(const float* __restrict__ in, float* __restrict__ out,
                                                   long long* __restrict__ cyc) {
  const int l = threadIdx.x;
  float qf[NB][20], kf[NB][20], vf[4 * NB][5];
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int d = 0; d < 20; ++d) {
      qf[i][d] = in[(l + 7 * i + d) & 1023];
      kf[i][d] = in[(l + 11 * i + 3 * d) & 1023];
    }
#pragma unroll
  for (int k = 0; k < 4 * NB; ++k)
#pragma unroll
    for (int m = 0; m < 5; ++m) vf[k][m] = in[(l + 5 * k + m) & 1023];
  float sink = 0.f;
  const long long t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    opaque(qf); opaque(kf); opaque(vf);   // (a new group's rows: nothing hoisted)
    floatx4 S[NB][NB];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int i = 0; i < NB; ++i) S[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int d = 0; d < 20; ++d)
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int i = 0; i < NB; ++i) S[j][i] = __builtin_amdgcn_mfma_f32_4x4x1f32(kf[j][d], qf[i][d], S[j][i], 0, 0, 0);
    floatx4 O[5][NB];
#pragma unroll
    for (int m = 0; m < 5; ++m)
#pragma unroll
      for (int i = 0; i < NB; ++i) O[m][i] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 4 * NB; ++kk)
#pragma unroll
      for (int m = 0; m < 5; ++m)
#pragma unroll
        for (int i = 0; i < NB; ++i)
          O[m][i] = __builtin_amdgcn_mfma_f32_4x4x1f32(vf[kk][m], S[kk >> 2][i][kk & 3], O[m][i], 0, 0, 0);
#pragma unroll
    for (int m = 0; m < 5; ++m)
#pragma unroll
      for (int i = 0; i < NB; ++i) sink += O[m][i][0] + O[m][i][3];
  }
  const long long t1 = clock64();
  out[blockIdx.x * 256 + l] = sink;
  if (l % 64 == 0) cyc[blockIdx.x * 4 + l / 64] = t1 - t0;
}

__device__ __forceinline__ void split4(const float* x, half4& h, half4& lo) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const _Float16 hh = (_Float16)x[e];
    h[e] = hh;
    lo[e] = (_Float16)((x[e] - (float)hh) * kLo);
  }
}

template <int NB>
__global__ __launch_bounds__(256, 1) void f16x3_form(const float* __restrict__ in, float* __restrict__ out,
                                                     long long* __restrict__ cyc) {
  const int l = threadIdx.x;
  float qf[NB][20], kf[NB][20], vf[NB][5][4];   // v: 4 keys of each of 5 dims per key block
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int d = 0; d < 20; ++d) {
      qf[i][d] = in[(l + 7 * i + d) & 1023];
      kf[i][d] = in[(l + 11 * i + 3 * d) & 1023];
    }
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int m = 0; m < 5; ++m)
#pragma unroll
      for (int e = 0; e < 4; ++e) vf[j][m][e] = in[(l + 5 * j + 4 * m + e) & 1023];
  float sink = 0.f;
  const long long t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    opaque(qf); opaque(kf); opaque(vf);   // (a new group's rows: nothing hoisted)
    // the group's operands split (the real kernel loads fp32 q|k|v rows)
    half4 qh[NB][5], ql[NB][5], kh[NB][5], kl[NB][5], vh[NB][5], vl[NB][5];
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int c = 0; c < 5; ++c) {
        split4(&qf[i][4 * c], qh[i][c], ql[i][c]);
        split4(&kf[i][4 * c], kh[i][c], kl[i][c]);
        split4(vf[i][c], vh[i][c], vl[i][c]);
      }
    floatx4 S[NB][NB];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        floatx4 a = floatx4{0.f, 0.f, 0.f, 0.f}, b = a;
#pragma unroll
        for (int c = 0; c < 5; ++c) {
          a = __builtin_amdgcn_mfma_f32_4x4x4f16(kh[j][c], qh[i][c], a, 0, 0, 0);
          b = __builtin_amdgcn_mfma_f32_4x4x4f16(kh[j][c], ql[i][c], b, 0, 0, 0);
          b = __builtin_amdgcn_mfma_f32_4x4x4f16(kl[j][c], qh[i][c], b, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) S[j][i][r] = __builtin_fmaf(b[r], 1.f / kLo, a[r]);
      }
    // p = S (the real kernel: exp and scale first), split per key block
    half4 ph[NB][NB], pl[NB][NB];
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        float s4[4] = {S[j][i][0], S[j][i][1], S[j][i][2], S[j][i][3]};
        split4(s4, ph[j][i], pl[j][i]);
      }
    floatx4 O[5][NB];
#pragma unroll
    for (int m = 0; m < 5; ++m)
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        floatx4 a = floatx4{0.f, 0.f, 0.f, 0.f}, b = a;
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          a = __builtin_amdgcn_mfma_f32_4x4x4f16(vh[j][m], ph[j][i], a, 0, 0, 0);
          b = __builtin_amdgcn_mfma_f32_4x4x4f16(vh[j][m], pl[j][i], b, 0, 0, 0);
          b = __builtin_amdgcn_mfma_f32_4x4x4f16(vl[j][m], ph[j][i], b, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) O[m][i][r] = __builtin_fmaf(b[r], 1.f / kLo, a[r]);
      }
#pragma unroll
    for (int m = 0; m < 5; ++m)
#pragma unroll
      for (int i = 0; i < NB; ++i) sink += O[m][i][0] + O[m][i][3];
  }
  const long long t1 = clock64();
  out[blockIdx.x * 256 + l] = sink;
  if (l % 64 == 0) cyc[blockIdx.x * 4 + l / 64] = t1 - t0;
}

template <int NB>
void run(float* in, float* out, long long* cyc, int n_cu) {
  std::vector<long long> h(n_cu * 4);
  double med[2];
  for (int f = 0; f < 2; ++f) {
    for (int rep = 0; rep < 2; ++rep) {   // (the first launch warms up)
      if (f == 0) hipLaunchKernelGGL(f32_form<NB>, dim3(n_cu), dim3(256), 0, 0, in, out, cyc);
      else hipLaunchKernelGGL(f16x3_form<NB>, dim3(n_cu), dim3(256), 0, 0, in, out, cyc);
      (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
    std::sort(h.begin(), h.end());
    med[f] = (double)h[h.size() / 2] / ITERS;
  }
  printf("NB=%d  f32 4x4x1: %7.0f cycles/group (%d MFMA)   f16x3 4x4x4 + splits: %7.0f cycles/group (%d MFMA)   ratio %.2f\n",
         NB, med[0], 40 * NB * NB, med[1], 30 * NB * NB, med[1] / med[0]);
}

int main() {
  int n_cu = 256;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
  float *in, *out;
  long long* cyc;
  (void)hipMalloc(&in, 1024 * 4);
  (void)hipMalloc(&out, (size_t)n_cu * 256 * 4);
  (void)hipMalloc(&cyc, (size_t)n_cu * 4 * 8);
  std::vector<float> h(1024);
  for (int i = 0; i < 1024; ++i) h[i] = 0.01f * (float)((i * 37) % 101) - 0.5f;
  (void)hipMemcpy(in, h.data(), 4096, hipMemcpyHostToDevice);
  run<2>(in, out, cyc, n_cu);
  run<3>(in, out, cyc, n_cu);
  run<4>(in, out, cyc, n_cu);
  run<5>(in, out, cyc, n_cu);
  return 0;
}
