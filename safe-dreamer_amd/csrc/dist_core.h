// Shared device math of the one-hot straight-through sampler (OneHotDist + F.gumbel_softmax(hard=True),
// distributions.py:16-33): used by the standalone sampler kernels (dist.hip) and by the fused RSSM scan (scan.hip).
#pragma once
#include "common.h"

namespace {

// ---------------------------------------------------------------- one-hot ST sampler
// Lanes [0, K) of a team of T lanes hold one categorical. Returns normalised unimix logits (nl) and p = softmax(l).
template <int T>
SD_DEV void unimix_forward(float l, bool act, int K, float unimix, float& p, float& pp, float& nl) {
  const float NEG = -INFINITY;
  float m = group_max<T>(act ? l : NEG);
  float e = act ? expf(l - m) : 0.f;
  float s = group_sum<T>(e);
  p = e / s;
  const float uni = unimix / (float)K;
  pp = p * (1.f - unimix) + uni;
  float lg = act ? logf(pp) : NEG;
  float m2 = group_max<T>(lg);
  float e2 = act ? expf(lg - m2) : 0.f;
  float s2 = group_sum<T>(e2);
  nl = act ? lg - (m2 + logf(s2)) : NEG;
}

// gradient of nl = log_softmax(log(p(1-u) + u/K)), p = softmax(l), w.r.t. l, given d_nl
template <int T>
SD_DEV float unimix_backward(float d_nl, float p, float pp, float nl, bool act, float unimix) {
  const float q = act ? expf(nl) : 0.f;  // softmax(lg)
  const float sd = group_sum<T>(act ? d_nl : 0.f);
  const float d_lg = d_nl - q * sd;
  const float d_p = act ? d_lg / pp * (1.f - unimix) : 0.f;
  const float sp = group_sum<T>(d_p * p);
  return act ? p * (d_p - sp) : 0.f;
}

template <int T>
SD_DEV void st_soft(float nl, float g, bool act, float& ys, int& idx, int lane_in_team) {
  const float y = act ? nl + g : -INFINITY;
  const float m = group_max<T>(y);
  const float e = act ? expf(y - m) : 0.f;
  const float s = group_sum<T>(e);
  ys = e / s;
  // first index of the maximum soft value (torch max(dim) tie-break)
  float best = act ? ys : -1.f;
  int bi = act ? lane_in_team : 0x7fffffff;
#pragma unroll
  for (int o = T / 2; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  idx = bi;
}

}  // namespace
