// Q|K|V projection GEMM alone on the qkv_news shape (M = 70,976, K = 300,
// N = 900): kernel time per launch in the current arithmetic
// (split-bf16 x6 unless -DPROBE_F32). Measured with diagnostic hooks in
// gemm_f32.hip (since removed; DESIGN.md lists the numbers): the store of the
// 255-MB output costs ~0.1 ms of the 0.36 ms (no-store build 0.25 ms),
// skipping the W split saves 3 %, non-temporal or LDS-staged row-contiguous
// stores do not help.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include [-D...] \
//     profiles/probes/gemm_probe.hip -o profiles/probes/gemm_probe
#include "../../newsrecommendationsystem_amd/csrc/gemm_f32.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

namespace nrms {
void set_last_hip_error(hipError_t) {}
#ifdef PROBE_F32
int gemm_arith() { return NRMS_GEMM_F32; }
#else
int gemm_arith() { return NRMS_GEMM_SPLIT_BF16X6; }
#endif
}

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                        \
    }                                                                  \
  } while (0)

int main(int argc, char** argv) {
  const int64_t M = argc > 1 ? atoll(argv[1]) : 70976;
  const int K = 300, N = 900;
  std::vector<float> hx((size_t)M * K), hw((size_t)N * K), hb(N);
  uint64_t st = 7;
  auto rnd = [&]() { st = st * 6364136223846793005ULL + 1442695040888963407ULL; return (float)((st >> 40) & 0xFFFFFF) / 16777216.f - 0.5f; };
  for (auto& v : hx) v = rnd();
  for (auto& v : hw) v = 0.1f * rnd();
  for (auto& v : hb) v = rnd();
  float *x, *w, *b, *y;
  CK(hipMalloc(&x, hx.size() * 4));
  CK(hipMalloc(&w, hw.size() * 4));
  CK(hipMalloc(&b, N * 4));
  CK(hipMalloc(&y, (size_t)M * N * 4));
  CK(hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(b, hb.data(), N * 4, hipMemcpyHostToDevice));
  nrms::WeightRows wr{};
  wr.w[0] = w; wr.b[0] = b; wr.seg_rows = N; wr.nseg = 1;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int it = 0; it < 3; ++it)
    if (nrms::launch_gemm_store(x, M, nullptr, M, K, wr, N, y, N, 0)) return 2;
  const int reps = 20;
  CK(hipEventRecord(e0, 0));
  for (int it = 0; it < reps; ++it)
    if (nrms::launch_gemm_store(x, M, nullptr, M, K, wr, N, y, N, 0)) return 2;
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("M=%lld GEMM %.4f ms (%.1f TF fp32-equivalent)\n", (long long)M, ms / reps,
         2.0 * M * N * K / (ms / reps * 1e-3) / 1e12);
  return 0;
}
