// Phase breakdown of the fused news kernel (shader cycles per wave, from
// s_memtime stamps compiled in with NRMS_FUSED_TIMING) on the bench shape:
// 56,320 titles (1024 impressions x 55), folded q|k|v table of V = 70,976 rows.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include \
//     profiles/probes/fused_timing.hip -o profiles/probes/fused_timing
#define NRMS_FUSED_TIMING 1
#include "../../newsrecommendationsystem_amd/csrc/news_fused.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

namespace nrms {
void set_last_hip_error(hipError_t) {}
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);     \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main(int argc, char** argv) {
  const int64_t V = 70976, n_titles = argc > 1 ? atoll(argv[1]) : 56320;
  const int64_t id_range = argc > 2 ? atoll(argv[2]) : V - 2;   // small: table slice stays in L2
  std::vector<float> h_qkv((size_t)V * 900), h_wa(200 * 300), h_b(200), h_q(200);
  std::vector<int64_t> h_ids((size_t)n_titles * 20);
  uint64_t st = 12345;
  auto rnd = [&]() { st = st * 6364136223846793005ULL + 1442695040888963407ULL; return (float)((st >> 40) & 0xFFFFFF) / 16777216.f; };
  for (auto& v : h_qkv) v = (rnd() - 0.5f) * 1.5f;
  for (auto& v : h_wa) v = (rnd() - 0.5f) * 0.1f;
  for (auto& v : h_b) v = (rnd() - 0.5f) * 0.1f;
  for (auto& v : h_q) v = (rnd() - 0.5f) * 0.2f;
  for (auto& v : h_ids) v = 1 + (int64_t)(rnd() * id_range);
  float *qkv, *wa, *b, *q, *wap, *out;
  int64_t* ids;
  unsigned long long* dbg;
  CK(hipMalloc(&qkv, h_qkv.size() * 4));
  CK(hipMalloc(&wa, h_wa.size() * 4));
  CK(hipMalloc(&b, 800));
  CK(hipMalloc(&q, 800));
  CK(hipMalloc(&wap, nrms::fused_news_packed_b_floats() * 4));
  CK(hipMalloc(&out, (size_t)n_titles * 300 * 4));
  CK(hipMalloc(&ids, h_ids.size() * 8));
  CK(hipMalloc(&dbg, 256 * 4 * 8 * 8));
  CK(hipMemcpy(qkv, h_qkv.data(), h_qkv.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(wa, h_wa.data(), h_wa.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(b, h_b.data(), 800, hipMemcpyHostToDevice));
  CK(hipMemcpy(q, h_q.data(), 800, hipMemcpyHostToDevice));
  CK(hipMemcpy(ids, h_ids.data(), h_ids.size() * 8, hipMemcpyHostToDevice));
  nrms::g_fused_dbg = dbg;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int it = 0; it < 3; ++it)
    if (nrms::launch_fused_news(qkv, V, ids, n_titles, nullptr, n_titles, wa, b, q, wap, out, 0)) return 2;
  CK(hipEventRecord(e0, 0));
  const int reps = 5;
  for (int it = 0; it < reps; ++it)
    if (nrms::launch_fused_news(qkv, V, ids, n_titles, nullptr, n_titles, wa, b, q, wap, out, 0)) return 2;
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> h_dbg(256 * 4 * 8);
  CK(hipMemcpy(h_dbg.data(), dbg, h_dbg.size() * 8, hipMemcpyDeviceToHost));
  const char* names[7] = {"barrier0 (+C tail)", "A attention", "barrier1", "B mainloop", "B epilogue", "barrier2", "C softmax+pool"};
  printf("kernel avg %.4f ms (pack + fused), %lld titles, ids in [1, %lld]\n", ms / reps,
         (long long)n_titles, (long long)id_range);
  for (int w = 0; w < 4; ++w) {
    printf("wave %d:", w);
    double tot = 0;
    for (int k = 0; k < 7; ++k) {
      double s = 0;
      for (int blk = 0; blk < 256; ++blk) s += h_dbg[(blk * 4 + w) * 8 + k];
      s /= 256;
      tot += s;
      printf(" %s=%.0f", names[k], s);
    }
    printf(" | total=%.0f cycles\n", tot);
  }
  return 0;
}
