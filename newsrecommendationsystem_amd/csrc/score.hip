// Batched dot-product click predictor (DotProductClickPredictor.forward,
// src/model/general/click_predictor/dot_product.py:8-19): one wave per
// (impression, candidate), float4 lanes, shuffle reduction.
#include "nrms_common.hpp"

namespace nrms {
namespace {

constexpr int kScoreThreads = 256;

// pg (optional, nrms_forward after padding-title dedupe): the candidates are
// titles title0 + b C + c of a contiguous [titles, D] array (news = its row
// title0); a copied all-padding candidate reads the rep title's vector
// instead (PaddingGroups), so no copies need to be written.
__global__ __launch_bounds__(kScoreThreads) void score_kernel(
    const float* __restrict__ news, int64_t B, int C, int64_t sb, int64_t sc,
    const float* __restrict__ user, int64_t su, int D, float* __restrict__ out, PaddingGroups pg,
    int64_t title0) {
  const int lane = threadIdx.x & 63;
  const int64_t pair = (int64_t)blockIdx.x * (kScoreThreads / kWave) + (threadIdx.x >> 6);
  if (pair >= B * C) return;
  const int64_t b = pair / C;
  const int c = (int)(pair - b * C);
  const float* nv = news + b * sb + (int64_t)c * sc;
  if (pg.pad_title) {
    const int64_t t = title0 + pair, r = *pg.rep;
    if (pg.pad_title[t] && t != r) nv = news + (r - title0) * D;
  }
  const float* uv = user + b * su;
  float acc = 0.f;
  if ((((uintptr_t)nv | (uintptr_t)uv) & 15) == 0 && (D & 3) == 0) {
    const float4* n4 = reinterpret_cast<const float4*>(nv);
    const float4* u4 = reinterpret_cast<const float4*>(uv);
    for (int i = lane; i < D / 4; i += kWave) {
      const float4 a = n4[i], u = u4[i];
      acc = fmaf(a.x, u.x, acc);
      acc = fmaf(a.y, u.y, acc);
      acc = fmaf(a.z, u.z, acc);
      acc = fmaf(a.w, u.w, acc);
    }
  } else {
    for (int i = lane; i < D; i += kWave) acc = fmaf(nv[i], uv[i], acc);
  }
  acc = wave_sum(acc);
  if (lane == 0) out[pair] = acc;
}

}  // namespace

int32_t launch_score(const float* news, int64_t B, int C, int64_t sb, int64_t sc,
                     const float* user, int64_t su, int D, float* out, hipStream_t s,
                     const PaddingGroups* pg, int64_t title0) {
  if (pg && (sb != (int64_t)C * D || sc != D)) return NRMS_ERR_UNSUPPORTED;
  if (B == 0 || C == 0) return NRMS_OK;
  const int per = kScoreThreads / kWave;
  const int64_t blocks = (B * C + per - 1) / per;
  if (blocks > INT32_MAX) return NRMS_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(score_kernel, dim3((unsigned)blocks), dim3(kScoreThreads), 0, s, news, B, C,
                     sb, sc, user, su, D, out, pg ? *pg : PaddingGroups{nullptr, nullptr, nullptr}, title0);
  return launch_status();
}

}  // namespace nrms
