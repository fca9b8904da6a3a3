// Fused news kernel, the three additive-GEMM variants (split-f16 x3,
// split-bf16 x6 and exact f32 MFMA) on the bench shape (56,320 titles, folded q|k|v table of V = 70,976
// rows): wall time per launch (HIP events), output agreement between the
// variants, and the per-phase shader-cycle breakdown (s_memtime stamps
// compiled in with NRMS_FUSED_TIMING; a diagnostic build, the stamps cost time).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include \
//     profiles/probes/news_variants.hip -o profiles/probes/news_variants
//   ./news_variants [n_titles] [reps] [id_range]
#ifndef NRMS_NO_STAMPS
#define NRMS_FUSED_TIMING 1
#endif
#include "../../newsrecommendationsystem_amd/csrc/news_fused.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace nrms {
void set_last_hip_error(hipError_t) {}
int g_arith = NRMS_GEMM_SPLIT_BF16X6;
int gemm_arith() { return g_arith; }
void ensure_dynamic_lds(const void* fn, int bytes) {
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}
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
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  const int64_t id_range = argc > 3 ? atoll(argv[3]) : V - 2;   // small: the table slice stays in L2
  const int64_t LDQ = getenv("NV_LDQ") ? atoll(getenv("NV_LDQ")) : 928;
  std::vector<float> h_qkv((size_t)V * LDQ), h_wa(200 * 300), h_b(200), h_q(200);
  std::vector<int64_t> h_ids((size_t)n_titles * 20);
  uint64_t st = 12345;
  auto rnd = [&]() { st = st * 6364136223846793005ULL + 1442695040888963407ULL; return (float)((st >> 40) & 0xFFFFFF) / 16777216.f; };
  for (auto& v : h_qkv) v = (rnd() - 0.5f) * 1.5f;
  for (auto& v : h_wa) v = (rnd() - 0.5f) * 0.1f;
  for (auto& v : h_b) v = (rnd() - 0.5f) * 0.1f;
  for (auto& v : h_q) v = (rnd() - 0.5f) * 0.2f;
  // titles of the bench's stream: length U{5..20}, right-padded with id 0
  const int fixed_len = getenv("NV_LEN") ? atoi(getenv("NV_LEN")) : 0;   // every title this long
  for (int64_t s = 0; s < n_titles; ++s) {
    const int len = fixed_len ? fixed_len : 5 + (int)(rnd() * 16);
    for (int t = 0; t < 20; ++t) h_ids[s * 20 + t] = t < len ? 1 + (int64_t)(rnd() * id_range) : 0;
  }
  for (int t = 0; t < 20; ++t) h_ids[7 * 20 + t] = 0;   // an all-padding title
  float *qkv, *wa, *b, *q, *wap, *out0, *out1, *out2;
  int64_t* ids;
  unsigned long long* dbg;
  CK(hipMalloc(&qkv, h_qkv.size() * 4));
  CK(hipMalloc(&wa, h_wa.size() * 4));
  CK(hipMalloc(&b, 800));
  CK(hipMalloc(&q, 800));
  CK(hipMalloc(&wap, nrms::fused_news_workspace_floats(n_titles) * 4));
  CK(hipMalloc(&out0, (size_t)n_titles * 300 * 4));
  CK(hipMalloc(&out1, (size_t)n_titles * 300 * 4));
  CK(hipMalloc(&out2, (size_t)n_titles * 300 * 4));
  CK(hipMalloc(&ids, h_ids.size() * 8));
  CK(hipMalloc(&dbg, 256 * 8 * 8 * 8));
  CK(hipMemcpy(qkv, h_qkv.data(), h_qkv.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(wa, h_wa.data(), h_wa.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(b, h_b.data(), 800, hipMemcpyHostToDevice));
  CK(hipMemcpy(q, h_q.data(), 800, hipMemcpyHostToDevice));
  CK(hipMemcpy(ids, h_ids.data(), h_ids.size() * 8, hipMemcpyHostToDevice));
#ifdef NRMS_FUSED_TIMING
  nrms::g_fused_dbg = dbg;
#endif
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* vname[3] = {"exact f32 MFMA", "split-bf16 x6", "split-f16 x3"};
  const int nwaves[3] = {4, 4, 4};
  const int arith[3] = {NRMS_GEMM_F32, NRMS_GEMM_SPLIT_BF16X6, NRMS_GEMM_SPLIT_F16X3};
  float* outs[3] = {out0, out1, out2};
  const int compact_runs = getenv("NV_BOTH") ? 2 : 1;
  for (int cr = 0; cr < compact_runs; ++cr)
  for (int var = 2; var >= 0; --var) {
    if (getenv("NV_ONLY_H3") && var != 2) continue;
    nrms::set_token_compaction(cr == 0 ? 1 : 0);
    printf("token compaction %s\n", cr == 0 ? "on" : "off");
    nrms::g_arith = arith[var];
    float* out = outs[var];
    for (int it = 0; it < 2; ++it)
      if (nrms::launch_fused_news(qkv, LDQ, V, ids, n_titles, nullptr, n_titles, wa, b, q, wap, out, 0)) return 2;
    CK(hipDeviceSynchronize());
    CK(hipMemset(dbg, 0, 256 * 8 * 8 * 8));
    CK(hipEventRecord(e0, 0));
    for (int it = 0; it < reps; ++it)
      if (nrms::launch_fused_news(qkv, LDQ, V, ids, n_titles, nullptr, n_titles, wa, b, q, wap, out, 0)) return 2;
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("%s: kernel avg %.4f ms (pack + fused), %lld titles\n", vname[var], ms / reps, (long long)n_titles);
#ifdef NRMS_FUSED_TIMING
    std::vector<unsigned long long> h_dbg(256 * 8 * 8);
    CK(hipMemcpy(h_dbg.data(), dbg, h_dbg.size() * 8, hipMemcpyDeviceToHost));
    const char* names[7] = {"wait qk", "A", "barrier1", "B main", "B epi", "barrier2", "C"};
    const int nk = 7;
    for (int w = 0; w < nwaves[var]; ++w) {
      printf("  wave %d:", w);
      double tot = 0;
      for (int k = 0; k < nk; ++k) {
        double s = 0;
        // the last launch only (dbg is overwritten per launch)
        for (int blk = 0; blk < 256; ++blk) s += h_dbg[(blk * nwaves[var] + w) * 8 + k];
        s /= 256;
        tot += s;
        printf(" %s=%.0f", names[k], s);
      }
      printf(" | total=%.0f\n", tot);
    }
    {
      // per-workgroup busy cycles (wave 0, all phases): the persistent grid's
      // balance -- max over mean is the tail the static group stride leaves
      std::vector<double> tb(256, 0.0);
      for (int blk = 0; blk < 256; ++blk)
        for (int k = 0; k < nk; ++k) tb[blk] += (double)h_dbg[(blk * nwaves[var]) * 8 + k];
      std::vector<double> srt = tb;
      std::sort(srt.begin(), srt.end());
      double mean = 0;
      for (double v : tb) mean += v / 256;
      printf("  workgroup totals: min %.0f p10 %.0f median %.0f p90 %.0f max %.0f mean %.0f (max/mean %.4f)\n",
             srt[0], srt[25], srt[128], srt[230], srt[255], mean, srt[255] / mean);
    }
#endif
  }
  std::vector<float> a((size_t)n_titles * 300), c((size_t)n_titles * 300);
  CK(hipMemcpy(c.data(), out0, c.size() * 4, hipMemcpyDeviceToHost));
  double worst_all = 0;
  size_t nan_all = 0;
  for (int var = 1; var <= 2; ++var) {
    CK(hipMemcpy(a.data(), outs[var], a.size() * 4, hipMemcpyDeviceToHost));
    double worst = 0, num = 0, den = 0;
    size_t nan_mismatch = 0;
    for (int64_t t = 0; t < n_titles; ++t) {
      double n2 = 0, d2 = 0;
      for (int d = 0; d < 300; ++d) {
        const float x = a[t * 300 + d], y = c[t * 300 + d];
        if (std::isnan(x) != std::isnan(y)) ++nan_mismatch;
        if (std::isnan(x) || std::isnan(y)) continue;
        n2 += (double)(x - y) * (x - y);
        d2 += (double)y * y;
      }
      num += n2; den += d2;
      const double r = d2 > 0 ? std::sqrt(n2 / d2) : std::sqrt(n2);
      if (r > worst) worst = r;
    }
    printf("%s vs f32: max normwise rel err %.3e, overall %.3e, NaN mismatches %zu\n", vname[var], worst,
           std::sqrt(num / den), nan_mismatch);
    worst_all = worst > worst_all ? worst : worst_all;
    nan_all += nan_mismatch;
  }
  const double worst = worst_all;
  const size_t nan_mismatch = nan_all;
  return (worst < 2e-6 && nan_mismatch == 0) ? 0 : 3;
}
