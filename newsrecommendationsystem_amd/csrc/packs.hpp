// Per-element bodies of the W_add packings of the fused news and UserEncoder
// kernels (layouts documented in news_fused.hip / user_fused.hip), shared so
// that nrms_forward can pack all of its weights in one launch
// (proj_x6.hip: forward_pack_kernel). The owning files check that their
// constants equal these.
#pragma once

#include "nrms_common.hpp"

namespace nrms {
namespace pk {

constexpr int D = 300, Q = 200;
constexpr int KS = 10;                          // bf16 / f16 k-steps of 32 (K 300 -> 320)
constexpr int NT = 13;                          // N tiles of 16 (208 >= Q)
constexpr int KG = 19;                          // f32 k-groups of 16 (K 300 -> 304)
constexpr int ROW = (3 * D + 31) / 32 * 32;     // q|k|v row slot of the zero / NaN rows (qkv_row_stride)
// news: [x6 planes | f32 fragments] (max), zero + NaN q|k|v rows, f16 planes
constexpr int NEWS_WAP_F32 = KG * NT * 64 * 4;
constexpr int NEWS_WAP_X6 = KS * NT * 3 * 64 * 4;
constexpr int NEWS_WAP_MAX = NEWS_WAP_X6 > NEWS_WAP_F32 ? NEWS_WAP_X6 : NEWS_WAP_F32;
constexpr int NEWS_SPECIAL = 2 * ROW;
constexpr int NEWS_COUNTERS = NEWS_WAP_MAX + NEWS_SPECIAL + NEWS_WAP_X6;   // int32 [NEWS_NCOUNT] after the f16 planes
// the news launch's counters: [recheck count, title-bucket counts 0..4, rep
// title (INT32_MAX: none), user row-list count]
constexpr int NEWS_NCOUNT = 12, NEWS_CNT_REP = 6;   // (a multiple of 4: the arrays after them stay 16-B aligned)
constexpr int NEWS_X6_ELEMS = KS * NT * 64 * 8;   // threads of the x6 / f16 packing
constexpr int USER_X6_ELEMS = KS * NT * 64 * 8;
constexpr int USER_F32_ELEMS = KG * NT * 64 * 4;
constexpr float kLoScale = kF16LoScale;

__device__ __forceinline__ void split3(float x, __bf16& hi, __bf16& mid, __bf16& lo) {
  hi = (__bf16)x;
  const float r = x - (float)hi;
  mid = (__bf16)r;
  lo = (__bf16)(r - (float)mid);
}

// News W_add, split arithmetic: element idx < NEWS_X6_ELEMS + NEWS_SPECIAL.
// x6 planes [ks][nt][plane][lane][8] (bf16 hi | mid | lo of Wa[16 nt + (lane
// & 15)][32 ks + 8 (lane >> 4) + i], 0 past Q or D); F16: also the fp16 planes
// (2^11 hi, 2^11-scaled residual, hi) after the special rows; then the zero
// and NaN q|k|v rows; idx < NEWS_NCOUNT resets the launch's counters.
template <bool F16>
__device__ __forceinline__ void pack_news_additive(int idx, const float* __restrict__ Wa, float* __restrict__ WaP,
                                                   int32_t* __restrict__ counters) {
  if (idx < NEWS_NCOUNT) counters[idx] = idx == NEWS_CNT_REP ? INT32_MAX : 0;
  if (idx >= NEWS_X6_ELEMS + NEWS_SPECIAL) return;
  if (idx >= NEWS_X6_ELEMS) {
    const int sidx = idx - NEWS_X6_ELEMS;
    WaP[NEWS_WAP_MAX + sidx] = sidx < ROW ? 0.f : qnan();
    return;
  }
  const int i = idx & 7, lane = (idx >> 3) & 63, nt = (idx >> 9) % NT, ks = (idx >> 9) / NT;
  const int n = 16 * nt + (lane & 15), k = 32 * ks + 8 * (lane >> 4) + i;
  const float v = (n < Q && k < D) ? Wa[n * D + k] : 0.f;
  __bf16 hi, mid, lo;
  split3(v, hi, mid, lo);
  __bf16* o = reinterpret_cast<__bf16*>(WaP) + (((ks * NT + nt) * 3) * 64 + lane) * 8 + i;
  o[0] = hi;
  o[64 * 8] = mid;
  o[2 * 64 * 8] = lo;
  if constexpr (F16) {
    const _Float16 h = (_Float16)v;
    _Float16* o2 = reinterpret_cast<_Float16*>(WaP + NEWS_WAP_MAX + NEWS_SPECIAL) +
                   (((ks * NT + nt) * 3) * 64 + lane) * 8 + i;
    const float hs = (float)h * kLoScale;   // exact unless it overflows fp16: NaN then (-> recheck)
    o2[0] = fabsf(hs) < 65504.f ? (_Float16)hs : (_Float16)qnan();
    o2[64 * 8] = (_Float16)((v - (float)h) * kLoScale);
    o2[2 * 64 * 8] = fabsf(hs) < 65504.f ? h : (_Float16)qnan();   // (NaN too: hi' may be formed from it)
  }
}

// UserEncoder W_add. x6: element idx < USER_X6_ELEMS, element i of lane (n =
// lane & 15, kq = lane >> 4) is k = 32 ks + 4 kq + (i & 3) + 16 (i >> 2), three
// bf16 planes. f32: idx < USER_F32_ELEMS, the 16x16x4 layout k = 16 kg + 4 kq + t.
__device__ __forceinline__ void pack_user_additive(int idx, const float* __restrict__ Wa, float* __restrict__ WaP,
                                                   int x6) {
  if (x6) {
    if (idx >= USER_X6_ELEMS) return;
    const int i = idx & 7, lane = (idx >> 3) & 63, nt = (idx >> 9) % NT, ks = (idx >> 9) / NT;
    const int n = 16 * nt + (lane & 15);
    const int k = 32 * ks + 4 * (lane >> 4) + (i & 3) + 16 * (i >> 2);
    const float v = (n < Q && k < D) ? Wa[n * D + k] : 0.f;
    __bf16 hi, mid, lo;
    split3(v, hi, mid, lo);
    __bf16* o = reinterpret_cast<__bf16*>(WaP) + (((ks * NT + nt) * 3) * 64 + lane) * 8 + i;
    o[0] = hi;
    o[64 * 8] = mid;
    o[2 * 64 * 8] = lo;
  } else {
    if (idx >= USER_F32_ELEMS) return;
    const int t = idx & 3, lane = (idx >> 2) & 63, nt = (idx >> 8) % NT, c = (idx >> 8) / NT;
    const int n = 16 * nt + (lane & 15), k = 16 * c + 4 * (lane >> 4) + t;
    WaP[idx] = (n < Q && k < D) ? Wa[n * D + k] : 0.f;
  }
}

// UserEncoder W_add, split-f16 (user_fused.hip MODE 2): one wave per W row
// n < 16 NT (block b holds rows 4b..4b+3; rows past Q are zeros), lane k =
// lane + 64 i (i < 5 covers the K padding to 320). The row's max |w| gives its
// exponent ew (into [2^14, 2^15)); planes hi | lo (w' = hi + 2^-11 lo) in the
// x6 fragment layout [ks][nt][plane][lane][8] with two planes, k of element i
// of lane (n & 15) + 16 kq = 32 ks + 4 kq + (i & 3) + 16 (i >> 2); ew as int32
// at float offset USER_H3_EXP.
constexpr int USER_H3_BLOCKS = NT * 16 / 4;
constexpr int USER_H3_EXP = KS * NT * 2 * 64 * 4;
__device__ __forceinline__ int exp_field(float ax) { return (int)((__float_as_uint(ax) >> 23) & 255u) - 127; }
__device__ __forceinline__ void pack_user_additive_h3(int b, int t, const float* __restrict__ Wa,
                                                      float* __restrict__ WaP) {
  const int lane = t & 63, n = 4 * b + (t >> 6);
  float v[5], mx = 0.f;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int k = lane + 64 * i;
    v[i] = (n < Q && k < D) ? Wa[n * D + k] : 0.f;
    mx = fmaxf(mx, fabsf(v[i]));
  }
#pragma unroll
  for (int o = 32; o; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  const int ew = exp_field(mx) - 14;
  _Float16* o = reinterpret_cast<_Float16*>(WaP);
  const int nt = n >> 4;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int k = lane + 64 * i, ks = k >> 5, wi = k & 31, rem = wi & 15;
    const int kq = rem >> 2, e = 4 * (wi >> 4) + (rem & 3);
    const float x = ldexpf(v[i], -ew);
    const _Float16 hi = (_Float16)x;
    const _Float16 lo = (_Float16)((x - (float)hi) * kF16LoScale);
    const int off = ((ks * NT + nt) * 2) * 512 + ((n & 15) + 16 * kq) * 8 + e;
    o[off] = hi;
    o[off + 512] = lo;
  }
  if (lane == 0) reinterpret_cast<int32_t*>(WaP)[USER_H3_EXP + n] = ew;
}

}  // namespace pk
}  // namespace nrms
