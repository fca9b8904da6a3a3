// Eval-semantics scoring (src/evaluate.py:171-272) on the GPU:
//  * pair scorer: logits of ragged impressions from cached news / user
//    vectors (evaluate.py:251-260: get_prediction per impression), one wave
//    per (candidate, user) pair — every impression of a split in one launch
//    instead of a Python loop with a device->host sync per impression;
//  * per-impression ranking metrics (evaluate.py:24-42,160-168): AUC (the
//    Mann-Whitney statistic with ties counted 1/2, which is what
//    sklearn.metrics.roc_auc_score computes for binary labels), MRR, nDCG@5,
//    nDCG@10, one wave per impression, fp64 accumulation. Edge cases follow
//    the reference as it runs against scikit-learn 1.7 (pinned by
//    tests/golden/nrms_flow_golden.npz): a non-finite score makes
//    roc_auc_score raise, so all four are NaN (the ValueError branch,
//    evaluate.py:167-168); a single-class impression gets AUC = NaN (sklearn
//    warns instead of raising) while MRR / nDCG keep numpy's arithmetic:
//    all-negative -> 0/0 = NaN, all-positive -> MRR = mean(1/rank), nDCG = 1.
#include "nrms_common.hpp"

namespace nrms {
namespace {

constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void score_pairs_kernel(
    const float* __restrict__ news, int64_t n_news, const float* __restrict__ user,
    int64_t n_users, const int64_t* __restrict__ news_idx, const int64_t* __restrict__ user_idx,
    int64_t n_pairs, int D, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t k = (int64_t)blockIdx.x * (kThreads / kWave) + (threadIdx.x >> 6);
  if (k >= n_pairs) return;
  const int64_t a = news_idx[k], b = user_idx[k];
  if ((uint64_t)a >= (uint64_t)n_news || (uint64_t)b >= (uint64_t)n_users) {
    if (lane == 0) out[k] = qnan();
    return;
  }
  const float* nv = news + a * D;
  const float* uv = user + b * D;
  float acc = 0.f;
  if ((D & 3) == 0) {
    const float4* n4 = reinterpret_cast<const float4*>(nv);
    const float4* u4 = reinterpret_cast<const float4*>(uv);
    for (int i = lane; i < D / 4; i += kWave) {
      const float4 x = n4[i], y = u4[i];
      acc = fmaf(x.x, y.x, acc);
      acc = fmaf(x.y, y.y, acc);
      acc = fmaf(x.z, y.z, acc);
      acc = fmaf(x.w, y.w, acc);
    }
  } else {
    for (int i = lane; i < D; i += kWave) acc = fmaf(nv[i], uv[i], acc);
  }
  acc = wave_sum(acc);
  if (lane == 0) out[k] = acc;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Rank of candidate c under the reference's order: np.argsort(y_score)[::-1]
// (descending score; among equal scores the larger index comes first, i.e. a
// stable ascending sort reversed). rank = 1 + #{j : s_j > s_c or (s_j == s_c and j > c)}.
__global__ __launch_bounds__(kThreads) void impression_metrics_kernel(
    const float* __restrict__ scores, const int32_t* __restrict__ labels,
    const int64_t* __restrict__ offsets, int64_t n_imp, double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t imp = (int64_t)blockIdx.x * (kThreads / kWave) + (threadIdx.x >> 6);
  if (imp >= n_imp) return;
  const int64_t b = offsets[imp], e = offsets[imp + 1];
  const int n = (int)(e - b);
  const float* s = scores + b;
  const int32_t* y = labels + b;

  // class counts and non-finite check (sklearn's check_array rejects NaN / inf)
  double npos = 0.0, nbad = 0.0;
  for (int c = lane; c < n; c += kWave) {
    npos += (y[c] == 1) ? 1.0 : 0.0;
    nbad += __builtin_isfinite(s[c]) ? 0.0 : 1.0;
  }
  npos = wave_sum_d(npos);
  nbad = wave_sum_d(nbad);
  const double nneg = (double)n - npos;
  double* o = out + imp * 4;
  if (n == 0 || npos == 0.0 || nbad > 0.0) {   // all-negative: every metric is 0/0
    if (lane < 4) o[lane] = __builtin_nan("");
    return;
  }
  double auc_num = 0.0, rr = 0.0, dcg5 = 0.0, dcg10 = 0.0;
  for (int c = lane; c < n; c += kWave) {
    if (y[c] != 1) continue;
    const float sc = s[c];
    int higher = 0;
    double wins = 0.0;
    for (int j = 0; j < n; ++j) {
      const float sj = s[j];
      higher += (sj > sc || (sj == sc && j > c)) ? 1 : 0;
      if (y[j] != 1) wins += (sc > sj) ? 1.0 : (sc == sj ? 0.5 : 0.0);
    }
    const int rank = higher + 1;
    auc_num += wins;
    rr += 1.0 / rank;
    const double disc = 1.0 / log2((double)rank + 1.0);
    if (rank <= 5) dcg5 += disc;
    if (rank <= 10) dcg10 += disc;
  }
  auc_num = wave_sum_d(auc_num);
  rr = wave_sum_d(rr);
  dcg5 = wave_sum_d(dcg5);
  dcg10 = wave_sum_d(dcg10);
  // ideal DCG: the positives occupy ranks 1..npos (evaluate.py:32-35)
  double idcg5 = 0.0, idcg10 = 0.0;
  const int np_i = (int)npos;
  for (int r = 1; r <= np_i && r <= 10; ++r) {
    const double d = 1.0 / log2((double)r + 1.0);
    if (r <= 5) idcg5 += d;
    idcg10 += d;
  }
  if (lane == 0) {
    const bool one_class = nneg == 0.0;   // all positive: identical DCG arrays, ratio 1
    o[0] = one_class ? __builtin_nan("") : auc_num / (npos * nneg);
    o[1] = rr / npos;
    o[2] = one_class ? 1.0 : dcg5 / idcg5;
    o[3] = one_class ? 1.0 : dcg10 / idcg10;
  }
}

}  // namespace

int32_t launch_score_pairs(const float* news, int64_t n_news, const float* user, int64_t n_users,
                           const int64_t* news_idx, const int64_t* user_idx, int64_t n_pairs,
                           int D, float* out, hipStream_t s) {
  if (n_pairs == 0) return NRMS_OK;
  const int per = kThreads / kWave;
  const int64_t blocks = (n_pairs + per - 1) / per;
  if (blocks > INT32_MAX) return NRMS_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(score_pairs_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, s, news,
                     n_news, user, n_users, news_idx, user_idx, n_pairs, D, out);
  return launch_status();
}

int32_t launch_impression_metrics(const float* scores, const int32_t* labels,
                                  const int64_t* offsets, int64_t n_imp, double* out,
                                  hipStream_t s) {
  if (n_imp == 0) return NRMS_OK;
  const int per = kThreads / kWave;
  const int64_t blocks = (n_imp + per - 1) / per;
  if (blocks > INT32_MAX) return NRMS_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(impression_metrics_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, s,
                     scores, labels, offsets, n_imp, out);
  return launch_status();
}

}  // namespace nrms
