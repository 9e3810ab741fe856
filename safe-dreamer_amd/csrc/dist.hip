// Distribution heads, latent sampling, KL and the GRU-style gate of the RSSM.
//
//  * one-hot straight-through sampler with unimix (OneHotDist.__init__/rsample, distributions.py:16-33 +
//    torch F.gumbel_softmax(hard=True)): one team of K lanes per categorical, noise generated in-kernel (philox.h);
//    backward recomputes everything from the logits (no saved soft samples);
//  * categorical KL on raw logits, summed over the S latents and clipped at free nats (rssm.py:222-230,
//    distributions.py:266-271); unimix entropy for the dyn/rep entropy metrics (dreamer.py:575-576);
//  * symexp two-hot: mode (distributions.py:78-98) and log_prob (100-129) fwd/bwd, one wave per 255-bin row;
//  * bounded normal (distributions.py:217-222): sample, log_prob, entropy fwd/bwd; discrete-actor log_prob/entropy;
//  * Bernoulli continue head (torchd.Bernoulli(logits)): log_prob fwd/bwd;
//  * Deter gates (rssm.py:65-75): r = sigmoid, c = tanh(r*c), u = sigmoid(u-1), h' = u*c + (1-u)*h, fwd/bwd.
#include "common.h"
#include "philox.h"
#include "sdhip.h"
#include "dist_core.h"

namespace {

template <int T>
__global__ void onehot_sample_fwd(const float* __restrict__ logits, float* __restrict__ out, int* __restrict__ index,
                                  float* __restrict__ entropy, long groups, int K, float unimix, uint64_t seed,
                                  uint32_t stream, uint32_t step, long group_offset, const uint64_t* seed_ptr) {
  if (seed_ptr) seed += *seed_ptr;
  const int lt = threadIdx.x % T;
  const long g = ((long)blockIdx.x * blockDim.x + threadIdx.x) / T;
  if (g >= groups) return;  // whole teams exit together (groups are team-aligned)
  const bool act = lt < K;
  const float l = act ? logits[g * K + lt] : 0.f;
  float p, pp, nl;
  unimix_forward<T>(l, act, K, unimix, p, pp, nl);
  if (entropy) {
    const float h = group_sum<T>(act ? -expf(nl) * nl : 0.f);
    if (lt == 0) entropy[g] = h;
  }
  if (!out) return;
  const float gn = act ? sd_gumbel(seed, stream, step, (uint64_t)(g + group_offset) * K + lt) : 0.f;
  float ys;
  int idx;
  st_soft<T>(nl, gn, act, ys, idx, lt);
  if (act) {
    const float hard = lt == idx ? 1.f : 0.f;
    out[g * K + lt] = (hard - ys) + ys;
  }
  if (index && lt == 0) index[g] = idx;
}

template <int T>
__global__ void onehot_sample_bwd(const float* __restrict__ logits, const float* __restrict__ dout,
                                  float* __restrict__ dlogits, long groups, int K, float unimix, uint64_t seed,
                                  uint32_t stream, uint32_t step, long group_offset, int accumulate,
                                  const uint64_t* seed_ptr) {
  if (seed_ptr) seed += *seed_ptr;
  const int lt = threadIdx.x % T;
  const long g = ((long)blockIdx.x * blockDim.x + threadIdx.x) / T;
  if (g >= groups) return;
  const bool act = lt < K;
  const float l = act ? logits[g * K + lt] : 0.f;
  float p, pp, nl;
  unimix_forward<T>(l, act, K, unimix, p, pp, nl);
  const float gn = act ? sd_gumbel(seed, stream, step, (uint64_t)(g + group_offset) * K + lt) : 0.f;
  float ys;
  int idx;
  st_soft<T>(nl, gn, act, ys, idx, lt);
  const float d = act ? dout[g * K + lt] : 0.f;
  const float sd = group_sum<T>(d * ys);
  const float dnl = act ? ys * (d - sd) : 0.f;
  const float dl = unimix_backward<T>(dnl, p, pp, nl, act, unimix);
  if (act) dlogits[g * K + lt] = accumulate ? dlogits[g * K + lt] + dl : dl;
}

// discrete actor: logp(a) = nl[argmax a], entropy = -sum exp(nl) nl  (OneHotCategorical.log_prob / entropy)
template <int T>
__global__ void onehot_logp_ent_fwd(const float* __restrict__ logits, const float* __restrict__ action,
                                    float* __restrict__ logp, float* __restrict__ ent, long rows, int K, float unimix) {
  const int lt = threadIdx.x % T;
  const long g = ((long)blockIdx.x * blockDim.x + threadIdx.x) / T;
  if (g >= rows) return;
  const bool act = lt < K;
  const float l = act ? logits[g * K + lt] : 0.f;
  float p, pp, nl;
  unimix_forward<T>(l, act, K, unimix, p, pp, nl);
  // argmax of the action one-hot (value.max(-1)[1]: first max)
  float best = act ? action[g * K + lt] : -INFINITY;
  int bi = act ? lt : 0x7fffffff;
#pragma unroll
  for (int o = T / 2; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  const float sel = group_sum<T>(lt == bi ? nl : 0.f);
  const float h = group_sum<T>(act ? -expf(nl) * nl : 0.f);
  if (lt == 0) { logp[g] = sel; ent[g] = h; }
}

template <int T>
__global__ void onehot_logp_ent_bwd(const float* __restrict__ logits, const float* __restrict__ action,
                                    const float* __restrict__ glogp, const float* __restrict__ gent,
                                    float* __restrict__ dlogits, long rows, int K, float unimix) {
  const int lt = threadIdx.x % T;
  const long g = ((long)blockIdx.x * blockDim.x + threadIdx.x) / T;
  if (g >= rows) return;
  const bool act = lt < K;
  const float l = act ? logits[g * K + lt] : 0.f;
  float p, pp, nl;
  unimix_forward<T>(l, act, K, unimix, p, pp, nl);
  float best = act ? action[g * K + lt] : -INFINITY;
  int bi = act ? lt : 0x7fffffff;
#pragma unroll
  for (int o = T / 2; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  const float s = act ? expf(nl) : 0.f;
  const float h = group_sum<T>(act ? -s * nl : 0.f);
  const float gl = glogp ? glogp[g] : 0.f, ge = gent ? gent[g] : 0.f;
  // d logp / d nl = onehot(bi);  d H / d nl_k = -s_k (1 + nl_k + H)   (probs = softmax(nl))
  const float dnl = act ? (lt == bi ? gl : 0.f) + ge * (-s * (1.f + nl + h)) : 0.f;
  const float dl = unimix_backward<T>(dnl, p, pp, nl, act, unimix);
  if (act) dlogits[g * K + lt] = dl;
}

// ---------------------------------------------------------------- KL (raw logits) summed over S, per row
template <int T>
__global__ void kl_fwd(const float* __restrict__ post, const float* __restrict__ prior, float* __restrict__ kl_row,
                       float* __restrict__ dyn, float* __restrict__ rep, float free_nats, int rows, int S, int K) {
  __shared__ float red[4];
  const int teams = 256 / T;
  const int team = threadIdx.x / T, lt = threadIdx.x % T;
  const bool act = lt < K;
  for (int r = blockIdx.x; r < rows; r += gridDim.x) {
    float acc = 0.f;
    for (int s = team; s < S; s += teams) {
      const long o = ((long)r * S + s) * K + lt;
      const float a = act ? post[o] : -INFINITY, b = act ? prior[o] : -INFINITY;
      const float ma = group_max<T>(a), mb = group_max<T>(b);
      const float ea = act ? expf(a - ma) : 0.f, eb = act ? expf(b - mb) : 0.f;
      const float sa = group_sum<T>(ea), sb = group_sum<T>(eb);
      const float lpa = a - ma - logf(sa), lpb = b - mb - logf(sb);
      const float pa = ea / sa;
      const float kg = group_sum<T>(act ? pa * (lpa - lpb) : 0.f);
      if (lt == 0) acc += kg;
    }
    const float tot = block_sum<256>(acc, red);
    if (threadIdx.x == 0) {
      kl_row[r] = tot;
      const float cl = tot < free_nats ? free_nats : tot;  // torch.clamp(min=free): NaN stays NaN
      if (dyn) dyn[r] = cl;
      if (rep) rep[r] = cl;
    }
    __syncthreads();
  }
}

// d rep / d post = g_rep[r] * 1[kl_r >= free] * pa (lpa - lpb - kl_s) ;  d dyn / d prior = g_dyn[r] * 1[..] * (pb - pa)
template <int T>
__global__ void kl_bwd(const float* __restrict__ post, const float* __restrict__ prior, const float* __restrict__ kl_row,
                       const float* __restrict__ g_rep, const float* __restrict__ g_dyn, float free_nats,
                       float* __restrict__ d_post, float* __restrict__ d_prior, int rows, int S, int K, int acc_post,
                       int acc_prior) {
  const long g = ((long)blockIdx.x * blockDim.x + threadIdx.x) / T;
  const int lt = threadIdx.x % T;
  if (g >= (long)rows * S) return;
  const int r = (int)(g / S);
  const bool act = lt < K;
  const long o = g * K + lt;
  const float a = act ? post[o] : -INFINITY, b = act ? prior[o] : -INFINITY;
  const float ma = group_max<T>(a), mb = group_max<T>(b);
  const float ea = act ? expf(a - ma) : 0.f, eb = act ? expf(b - mb) : 0.f;
  const float sa = group_sum<T>(ea), sb = group_sum<T>(eb);
  const float lpa = a - ma - logf(sa), lpb = b - mb - logf(sb);
  const float pa = ea / sa, pb = eb / sb;
  const float kg = group_sum<T>(act ? pa * (lpa - lpb) : 0.f);
  const bool pass = kl_row[r] >= free_nats;  // torch.clip(min=free) passes the gradient where x >= min
  if (!act) return;
  if (d_post) {
    const float v = pass && g_rep ? g_rep[r] * pa * (lpa - lpb - kg) : 0.f;
    d_post[o] = acc_post ? d_post[o] + v : v;
  }
  if (d_prior) {
    const float v = pass && g_dyn ? g_dyn[r] * (pb - pa) : 0.f;
    d_prior[o] = acc_prior ? d_prior[o] + v : v;
  }
}

// ---------------------------------------------------------------- symexp two-hot (one wave per row)
SD_DEV void row_softmax64(const float* l, int NB, float (&p)[4], float& lse, int lane) {
  float v[4];
  float m = -INFINITY;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = lane + 64 * j;
    v[j] = c < NB ? l[c] : -INFINITY;
    m = fmaxf(m, v[j]);
  }
  m = wave_max(m);
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = lane + 64 * j;
    p[j] = c < NB ? expf(v[j] - m) : 0.f;
    s += p[j];
  }
  s = wave_sum(s);
#pragma unroll
  for (int j = 0; j < 4; ++j) p[j] /= s;
  lse = m + logf(s);
}

// mode = p[c] b[c] + sum_i (p[c-1-i] b[c-1-i] + p[c+1+i] b[c+1+i]),  c = (NB-1)/2  (NB odd)
__global__ void twohot_mode_kernel(const float* __restrict__ logits, const float* __restrict__ bins,
                                   float* __restrict__ out, long rows, int NB) {
  __shared__ float sp[4][256];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + wave;
  if (r >= rows) return;
  float p[4], lse;
  row_softmax64(logits + r * NB, NB, p, lse, lane);
#pragma unroll
  for (int j = 0; j < 4; ++j) sp[wave][lane + 64 * j] = p[j];
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  const int c = (NB - 1) / 2;
  float acc = 0.f;
  for (int i = lane; i < c; i += 64) {
    const float lo = sp[wave][c - 1 - i] * bins[c - 1 - i];
    const float hi = sp[wave][c + 1 + i] * bins[c + 1 + i];
    acc += lo + hi;
  }
  acc = wave_sum(acc);
  if (lane == 0) out[r] = sp[wave][c] * bins[c] + acc;
}

SD_DEV void twohot_target(const float* bins, int NB, float t, int& below, int& above, float& wb, float& wa, int lane) {
  // below = #(bins <= t) - 1, above = NB - #(bins > t), clamped (distributions.py:106-109)
  int cle = 0, cgt = 0;
  for (int c = lane; c < NB; c += 64) {
    const float b = bins[c];
    cle += b <= t ? 1 : 0;
    cgt += b > t ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cle += __shfl_xor(cle, o, 64);
    cgt += __shfl_xor(cgt, o, 64);
  }
  below = min(max(cle - 1, 0), NB - 1);
  above = min(max(NB - cgt, 0), NB - 1);
  const bool eq = below == above;
  const float db = eq ? 1.f : fabsf(bins[below] - t);
  const float da = eq ? 1.f : fabsf(bins[above] - t);
  const float tot = db + da;
  wb = da / tot;
  wa = db / tot;
}

__global__ void twohot_logp_fwd(const float* __restrict__ logits, const float* __restrict__ bins,
                                const float* __restrict__ target, float* __restrict__ logp, long rows, int NB) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + wave;
  if (r >= rows) return;
  const float* l = logits + r * NB;
  float p[4], lse;
  row_softmax64(l, NB, p, lse, lane);
  int below, above;
  float wb, wa;
  twohot_target(bins, NB, target[r], below, above, wb, wa, lane);
  if (lane == 0) {
    float v = wb * (l[below] - lse);
    v += wa * (l[above] - lse);
    logp[r] = v;
  }
}

__global__ void twohot_logp_bwd(const float* __restrict__ logits, const float* __restrict__ bins,
                                const float* __restrict__ target, const float* __restrict__ glogp,
                                float* __restrict__ dlogits, long rows, int NB, int accumulate) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + wave;
  if (r >= rows) return;
  const float* l = logits + r * NB;
  float p[4], lse;
  row_softmax64(l, NB, p, lse, lane);
  int below, above;
  float wb, wa;
  twohot_target(bins, NB, target[r], below, above, wb, wa, lane);
  const float gsc = glogp[r];
  const float tsum = wb + wa;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = lane + 64 * j;
    if (c < NB) {
      const float td = (c == below ? wb : 0.f) + (c == above ? wa : 0.f);
      const float v = gsc * (td - p[j] * tsum);
      float* d = dlogits + r * NB + c;
      *d = accumulate ? *d + v : v;
    }
  }
}

// Replay-value loss (dreamer.py:652-658): row r's term w[r] * (-logp(ret[r]) - logp(slow[r])) under the TwoHot head
// logits (distributions.py:100-129), and its logits gradient for a given d loss / d term (one wave per row). The
// backward is the sum of the two twohot_logp_bwd terms in one pass: g (td_ret + td_slow - p (tsum_ret + tsum_slow)),
// g = -w[r] * gscale[0] * inv_n (gscale: device scalar, d total / d mean).
// replay-value rows (dreamer.py:638-658): loss row r = (b, t < Tr) reads logits / slow / last row b * Tl + t (the value
// head ran on all Tl posterior steps; Tr = Tl - 1 of them have a return) and ret[r]; weight = 1 - last.
__global__ void repval_fwd_kernel(const float* __restrict__ logits, const float* __restrict__ bins,
                                  const float* __restrict__ ret, const float* __restrict__ slow,
                                  const float* __restrict__ last, float* __restrict__ row_loss, long rows, int Tl,
                                  int Tr, int NB) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + wave;
  if (r >= rows) return;
  const long lr_ = (r / Tr) * Tl + r % Tr;
  const float* l = logits + lr_ * NB;
  float p[4], lse;
  row_softmax64(l, NB, p, lse, lane);
  int b1, a1, b2, a2;
  float wb1, wa1, wb2, wa2;
  twohot_target(bins, NB, ret[r], b1, a1, wb1, wa1, lane);
  twohot_target(bins, NB, slow[lr_], b2, a2, wb2, wa2, lane);
  if (lane == 0) {
    float lr = wb1 * (l[b1] - lse);
    lr += wa1 * (l[a1] - lse);
    float ls = wb2 * (l[b2] - lse);
    ls += wa2 * (l[a2] - lse);
    row_loss[r] = (1.f - last[lr_]) * (-lr - ls);
  }
}

// d logits of the mean of the rows above, for all B * Tl logits rows (zero on the rows without a return)
__global__ void repval_bwd_kernel(const float* __restrict__ logits, const float* __restrict__ bins,
                                  const float* __restrict__ ret, const float* __restrict__ slow,
                                  const float* __restrict__ last, const float* __restrict__ gscale, float inv_n,
                                  float* __restrict__ dlogits, long lrows, int Tl, int Tr, int NB) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long lr_ = (long)blockIdx.x * 4 + wave;
  if (lr_ >= lrows) return;
  const int t = (int)(lr_ % Tl);
  if (t >= Tr) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (lane + 64 * j < NB) dlogits[lr_ * NB + lane + 64 * j] = 0.f;
    return;
  }
  const long r = (lr_ / Tl) * Tr + t;
  const float* l = logits + lr_ * NB;
  float p[4], lse;
  row_softmax64(l, NB, p, lse, lane);
  int b1, a1, b2, a2;
  float wb1, wa1, wb2, wa2;
  twohot_target(bins, NB, ret[r], b1, a1, wb1, wa1, lane);
  twohot_target(bins, NB, slow[lr_], b2, a2, wb2, wa2, lane);
  const float g = -(1.f - last[lr_]) * (gscale[0] * inv_n);
  const float t1 = wb1 + wa1, t2 = wb2 + wa2;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = lane + 64 * j;
    if (c < NB) {
      const float td1 = (c == b1 ? wb1 : 0.f) + (c == a1 ? wa1 : 0.f);
      const float td2 = (c == b2 ? wb2 : 0.f) + (c == a2 ? wa2 : 0.f);
      dlogits[lr_ * NB + c] = g * (td1 - p[j] * t1) + g * (td2 - p[j] * t2);
    }
  }
}

// imagined actor-critic losses (dreamer.py:623-636, 653-671) on H * N time-major rows r = t * N + n, the returns /
// weights batch-major (n, t), the values time-major (t, n): adv = (ret[n, t] - val[t, n]) / scale[0] (metrics),
// value row  = w[n, t] * (-logp(vl[r], ret[n, t]) - logp(vl[r], slow[r]))   (TwoHot, distributions.py:100-129),
// policy row = w[n, t] * -(logpi[r] * adv + coef * ent[r]).  One wave per row.
__global__ void imag_ac_fwd_kernel(const float* __restrict__ vl, const float* __restrict__ bins,
                                   const float* __restrict__ ret, const float* __restrict__ slow,
                                   const float* __restrict__ w, const float* __restrict__ val,
                                   const float* __restrict__ scale, const float* __restrict__ logpi,
                                   const float* __restrict__ ent, float coef, long N, int H, int H1, int NB,
                                   float* __restrict__ rows_v, float* __restrict__ rows_p, float* __restrict__ adv) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + wave;
  if (r >= N * H) return;
  const long n = r % N;
  const int t = (int)(r / N);
  const float* l = vl + r * NB;
  const float rt = ret[n * H + t];
  float p[4], lse;
  row_softmax64(l, NB, p, lse, lane);
  int b1, a1, b2, a2;
  float wb1, wa1, wb2, wa2;
  twohot_target(bins, NB, rt, b1, a1, wb1, wa1, lane);
  twohot_target(bins, NB, slow[r], b2, a2, wb2, wa2, lane);
  if (lane == 0) {
    float lr = wb1 * (l[b1] - lse);
    lr += wa1 * (l[a1] - lse);
    float ls = wb2 * (l[b2] - lse);
    ls += wa2 * (l[a2] - lse);
    const float wt = w[n * H1 + t];
    const float a = (rt - val[(long)t * N + n]) / scale[0];
    rows_v[r] = wt * (-lr - ls);
    rows_p[r] = wt * -(logpi[r] * a + coef * ent[r]);
    adv[n * H + t] = a;
  }
}
// d vl (value loss, both log-prob terms), d logpi and d ent (policy loss); g = (policy, value) upstream gradients
__global__ void imag_ac_bwd_kernel(const float* __restrict__ vl, const float* __restrict__ bins,
                                   const float* __restrict__ ret, const float* __restrict__ slow,
                                   const float* __restrict__ w, const float* __restrict__ adv,
                                   const float* __restrict__ gp, const float* __restrict__ gv, float sp, float sv,
                                   float coef, float inv_n, long N, int H, int H1, int NB, float* __restrict__ dvl,
                                   float* __restrict__ dlogpi, float* __restrict__ dent) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + wave;
  if (r >= N * H) return;
  const long n = r % N;
  const int t = (int)(r / N);
  const float* l = vl + r * NB;
  float p[4], lse;
  row_softmax64(l, NB, p, lse, lane);
  int b1, a1, b2, a2;
  float wb1, wa1, wb2, wa2;
  twohot_target(bins, NB, ret[n * H + t], b1, a1, wb1, wa1, lane);
  twohot_target(bins, NB, slow[r], b2, a2, wb2, wa2, lane);
  const float wt = w[n * H1 + t];
  const float g = -wt * ((gv ? gv[0] * sv : 0.f) * inv_n);
  const float t1 = wb1 + wa1, t2 = wb2 + wa2;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = lane + 64 * j;
    if (c < NB) {
      const float td1 = (c == b1 ? wb1 : 0.f) + (c == a1 ? wa1 : 0.f);
      const float td2 = (c == b2 ? wb2 : 0.f) + (c == a2 ? wa2 : 0.f);
      dvl[r * NB + c] = g * (td1 - p[j] * t1) + g * (td2 - p[j] * t2);
    }
  }
  if (lane == 0) {
    const float gg = -wt * ((gp ? gp[0] * sp : 0.f) * inv_n);
    dlogpi[r] = gg * adv[n * H + t];
    dent[r] = gg * coef;
  }
}

// ---------------------------------------------------------------- bounded normal actor
__global__ void bnormal_sample(const float* __restrict__ x, float* __restrict__ action, long rows, int A, float min_std,
                               float max_std, uint64_t seed, uint32_t stream, uint32_t step, long row_offset,
                               const uint64_t* seed_ptr) {
  if (seed_ptr) seed += *seed_ptr;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * A) return;
  const long r = t / A;
  const int j = (int)(t % A);
  const float loc = tanhf(x[r * 2 * A + j]);
  const float sc = (max_std - min_std) * sigmoidf_(x[r * 2 * A + A + j] + 2.f) + min_std;
  const float eps = sd_normal(seed, stream, step, (uint64_t)(r + row_offset) * A + j);
  action[t] = loc + eps * sc;
}

__global__ void bnormal_logp_ent_fwd(const float* __restrict__ x, const float* __restrict__ action,
                                     float* __restrict__ logp, float* __restrict__ ent, long rows, int A, float min_std,
                                     float max_std) {
  const long r = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const float c0 = 0.91893853320467274178f;  // log(sqrt(2*pi))
  float lp = 0.f, h = 0.f;
  for (int j = 0; j < A; ++j) {
    const float loc = tanhf(x[r * 2 * A + j]);
    const float sc = (max_std - min_std) * sigmoidf_(x[r * 2 * A + A + j] + 2.f) + min_std;
    const float d = action[r * A + j] - loc;
    lp += -(d * d) / (2.f * sc * sc) - logf(sc) - c0;
    h += 0.5f + c0 + logf(sc);
  }
  logp[r] = lp;
  ent[r] = h;
}

__global__ void bnormal_logp_ent_bwd(const float* __restrict__ x, const float* __restrict__ action,
                                     const float* __restrict__ glogp, const float* __restrict__ gent,
                                     float* __restrict__ dx, long rows, int A, float min_std, float max_std) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= rows * A) return;
  const long r = t / A;
  const int j = (int)(t % A);
  const float loc = tanhf(x[r * 2 * A + j]);
  const float sg = sigmoidf_(x[r * 2 * A + A + j] + 2.f);
  const float sc = (max_std - min_std) * sg + min_std;
  const float d = action[r * A + j] - loc;
  const float gl = glogp ? glogp[r] : 0.f, ge = gent ? gent[r] : 0.f;
  const float d_loc = gl * d / (sc * sc);
  const float d_sc = gl * (d * d / (sc * sc * sc) - 1.f / sc) + ge / sc;
  dx[r * 2 * A + j] = d_loc * (1.f - loc * loc);
  dx[r * 2 * A + A + j] = d_sc * (max_std - min_std) * sg * (1.f - sg);
}

// ---------------------------------------------------------------- Bernoulli(logits) continue head, 1 logit/row
__global__ void bernoulli_fwd(const float* __restrict__ logit, const float* __restrict__ value, float* __restrict__ logp,
                              float* __restrict__ mean, long rows) {
  const long r = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const float x = logit[r];
  if (mean) mean[r] = sigmoidf_(x);
  if (logp) {
    const float y = value[r];
    const float mx = fmaxf(-x, 0.f);  // torch binary_cross_entropy_with_logits
    const float loss = (1.f - y) * x + mx + logf(expf(-mx) + expf(-x - mx));
    logp[r] = -loss;
  }
}

__global__ void bernoulli_bwd(const float* __restrict__ logit, const float* __restrict__ value,
                              const float* __restrict__ glogp, float* __restrict__ dlogit, long rows) {
  const long r = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  dlogit[r] = glogp[r] * (value[r] - sigmoidf_(logit[r]));
}

// ---------------------------------------------------------------- Deter GRU-style gates (rssm.py:65-75)
// gates: (M, G, 3, Dg) = the dyn_gru BlockLinear output; h: (M, G*Dg)
__global__ void gru_fwd(const float* __restrict__ gates, const float* __restrict__ h, float* __restrict__ out, long M,
                        int G, int Dg) {
  const long D = (long)G * Dg;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= M * D) return;
  const long m = t / D;
  const int gd = (int)(t % D), g = gd / Dg, j = gd % Dg;
  const float* gr = gates + m * 3 * D + (long)g * 3 * Dg;
  const float rs = sigmoidf_(gr[j]);
  const float c = tanhf(rs * gr[Dg + j]);
  const float u = sigmoidf_(gr[2 * Dg + j] - 1.f);
  out[t] = u * c + (1.f - u) * h[t];
}

__global__ void gru_bwd(const float* __restrict__ gates, const float* __restrict__ h, const float* __restrict__ dout,
                        float* __restrict__ dgates, float* __restrict__ dh, long M, int G, int Dg, int accumulate_dh) {
  const long D = (long)G * Dg;
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= M * D) return;
  const long m = t / D;
  const int gd = (int)(t % D), g = gd / Dg, j = gd % Dg;
  const long base = m * 3 * D + (long)g * 3 * Dg;
  const float ra = gates[base + j], ca = gates[base + Dg + j], ua = gates[base + 2 * Dg + j];
  const float rs = sigmoidf_(ra);
  const float c = tanhf(rs * ca);
  const float u = sigmoidf_(ua - 1.f);
  const float d = dout[t];
  const float hv = h[t];
  const float du = d * (c - hv) * u * (1.f - u);
  const float dtc = d * u * (1.f - c * c);
  const float dc = dtc * rs;
  const float dr = dtc * ca * rs * (1.f - rs);
  dgates[base + j] = dr;
  dgates[base + Dg + j] = dc;
  dgates[base + 2 * Dg + j] = du;
  const float v = d * (1.f - u);
  dh[t] = accumulate_dh ? dh[t] + v : v;
}

int team_pow2(int K) { return K <= 8 ? 8 : K <= 16 ? 16 : K <= 32 ? 32 : 64; }
int blocks_for(long n, int per) { long b = (n + per - 1) / per; return (int)b; }

}  // namespace

#define SD_TEAM_SWITCH(T, ...)                      \
  switch (T) {                                      \
    case 8: { constexpr int TT = 8; __VA_ARGS__; } break;   \
    case 16: { constexpr int TT = 16; __VA_ARGS__; } break; \
    case 32: { constexpr int TT = 32; __VA_ARGS__; } break; \
    default: { constexpr int TT = 64; __VA_ARGS__; } break; \
  }

extern "C" int sd_onehot_sample_fwd(const float* logits, float* out, int* index, float* entropy, long groups, int K,
                                    float unimix, uint64_t seed, int stream_id, int step, long group_offset,
                                    const uint64_t* seed_ptr, sd_stream s) {
  if (groups <= 0) return SD_OK;
  if (K < 1 || K > 64) return SD_ESHAPE;
  const int T = team_pow2(K);
  const int grid = blocks_for(groups * T, 256);
  SD_TEAM_SWITCH(T, onehot_sample_fwd<TT><<<grid, 256, 0, (hipStream_t)s>>>(logits, out, index, entropy, groups, K,
                                                                          unimix, seed, stream_id, step, group_offset, seed_ptr))
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_onehot_sample_bwd(const float* logits, const float* dout, float* dlogits, long groups, int K,
                                    float unimix, uint64_t seed, int stream_id, int step, long group_offset,
                                    int accumulate, const uint64_t* seed_ptr, sd_stream s) {
  if (groups <= 0) return SD_OK;
  if (K < 1 || K > 64) return SD_ESHAPE;
  const int T = team_pow2(K);
  const int grid = blocks_for(groups * T, 256);
  SD_TEAM_SWITCH(T, onehot_sample_bwd<TT><<<grid, 256, 0, (hipStream_t)s>>>(logits, dout, dlogits, groups, K, unimix,
                                                                          seed, stream_id, step, group_offset,
                                                                          accumulate, seed_ptr))
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_onehot_logp_ent_fwd(const float* logits, const float* action, float* logp, float* ent, long rows,
                                      int K, float unimix, sd_stream s) {
  if (rows <= 0) return SD_OK;
  if (K < 1 || K > 64) return SD_ESHAPE;
  const int T = team_pow2(K);
  const int grid = blocks_for(rows * T, 256);
  SD_TEAM_SWITCH(T, onehot_logp_ent_fwd<TT><<<grid, 256, 0, (hipStream_t)s>>>(logits, action, logp, ent, rows, K,
                                                                            unimix))
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_onehot_logp_ent_bwd(const float* logits, const float* action, const float* glogp, const float* gent,
                                      float* dlogits, long rows, int K, float unimix, sd_stream s) {
  if (rows <= 0) return SD_OK;
  if (K < 1 || K > 64) return SD_ESHAPE;
  const int T = team_pow2(K);
  const int grid = blocks_for(rows * T, 256);
  SD_TEAM_SWITCH(T, onehot_logp_ent_bwd<TT><<<grid, 256, 0, (hipStream_t)s>>>(logits, action, glogp, gent, dlogits,
                                                                            rows, K, unimix))
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_kl_fwd(const float* post, const float* prior, float* kl_row, float* dyn, float* rep, float free_nats,
                         int rows, int S, int K, sd_stream s) {
  if (rows <= 0) return SD_OK;
  if (K < 1 || K > 64) return SD_ESHAPE;
  const int T = team_pow2(K);
  const int grid = rows < 4096 ? rows : 4096;
  SD_TEAM_SWITCH(T, kl_fwd<TT><<<grid, 256, 0, (hipStream_t)s>>>(post, prior, kl_row, dyn, rep, free_nats, rows, S, K))
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_kl_bwd(const float* post, const float* prior, const float* kl_row, const float* g_rep,
                         const float* g_dyn, float free_nats, float* d_post, float* d_prior, int rows, int S, int K,
                         int acc_post, int acc_prior, sd_stream s) {
  if (rows <= 0) return SD_OK;
  if (K < 1 || K > 64) return SD_ESHAPE;
  const int T = team_pow2(K);
  const int grid = blocks_for((long)rows * S * T, 256);
  SD_TEAM_SWITCH(T, kl_bwd<TT><<<grid, 256, 0, (hipStream_t)s>>>(post, prior, kl_row, g_rep, g_dyn, free_nats, d_post,
                                                               d_prior, rows, S, K, acc_post, acc_prior))
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_twohot_mode(const float* logits, const float* bins, float* out, long rows, int NB, sd_stream s) {
  if (rows <= 0) return SD_OK;
  if (NB > 256 || NB % 2 == 0) return SD_ESHAPE;
  twohot_mode_kernel<<<blocks_for(rows, 4), 256, 0, (hipStream_t)s>>>(logits, bins, out, rows, NB);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_twohot_logp_fwd(const float* logits, const float* bins, const float* target, float* logp, long rows,
                                  int NB, sd_stream s) {
  if (rows <= 0) return SD_OK;
  if (NB > 256) return SD_ESHAPE;
  twohot_logp_fwd<<<blocks_for(rows, 4), 256, 0, (hipStream_t)s>>>(logits, bins, target, logp, rows, NB);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_twohot_logp_bwd(const float* logits, const float* bins, const float* target, const float* glogp,
                                  float* dlogits, long rows, int NB, int accumulate, sd_stream s) {
  if (rows <= 0) return SD_OK;
  if (NB > 256) return SD_ESHAPE;
  twohot_logp_bwd<<<blocks_for(rows, 4), 256, 0, (hipStream_t)s>>>(logits, bins, target, glogp, dlogits, rows, NB,
                                                                    accumulate);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_repval_loss_fwd(const float* logits, const float* bins, const float* ret, const float* slow,
                                  const float* last, float* row_loss, int B, int Tl, int Tr, int NB, sd_stream s) {
  if (B <= 0 || Tr <= 0) return SD_OK;
  if (NB > 256 || Tr > Tl) return SD_ESHAPE;
  const long rows = (long)B * Tr;
  repval_fwd_kernel<<<blocks_for(rows, 4), 256, 0, (hipStream_t)s>>>(logits, bins, ret, slow, last, row_loss, rows, Tl,
                                                                      Tr, NB);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_repval_loss_bwd(const float* logits, const float* bins, const float* ret, const float* slow,
                                  const float* last, const float* gscale, float inv_n, float* dlogits, int B, int Tl,
                                  int Tr, int NB, sd_stream s) {
  if (B <= 0) return SD_OK;
  if (NB > 256 || !gscale || Tr > Tl) return SD_ESHAPE;
  const long lrows = (long)B * Tl;
  repval_bwd_kernel<<<blocks_for(lrows, 4), 256, 0, (hipStream_t)s>>>(logits, bins, ret, slow, last, gscale, inv_n,
                                                                       dlogits, lrows, Tl, Tr, NB);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_imag_ac_loss_fwd(const float* vl, const float* bins, const float* ret, const float* slow,
                                   const float* w, const float* val, const float* scale, const float* logpi,
                                   const float* ent, float coef, long N, int H, int H1, int NB, float* rows_v,
                                   float* rows_p, float* adv, sd_stream s) {
  if (N <= 0 || H <= 0) return SD_OK;
  if (NB > 256 || H1 <= H) return SD_ESHAPE;
  imag_ac_fwd_kernel<<<blocks_for(N * H, 4), 256, 0, (hipStream_t)s>>>(vl, bins, ret, slow, w, val, scale, logpi, ent,
                                                                       coef, N, H, H1, NB, rows_v, rows_p, adv);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_imag_ac_loss_bwd(const float* vl, const float* bins, const float* ret, const float* slow,
                                   const float* w, const float* adv, const float* gpolicy, const float* gvalue,
                                   float spolicy, float svalue, float coef, long N, int H, int H1, int NB, float* dvl,
                                   float* dlogpi, float* dent, sd_stream s) {
  if (N <= 0 || H <= 0) return SD_OK;
  if (NB > 256 || H1 <= H) return SD_ESHAPE;
  imag_ac_bwd_kernel<<<blocks_for(N * H, 4), 256, 0, (hipStream_t)s>>>(vl, bins, ret, slow, w, adv, gpolicy, gvalue,
                                                                       spolicy, svalue, coef, 1.f / (float)(N * H), N,
                                                                       H, H1, NB, dvl, dlogpi, dent);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_bnormal_sample(const float* x, float* action, long rows, int A, float min_std, float max_std,
                                 uint64_t seed, int stream_id, int step, long row_offset, const uint64_t* seed_ptr,
                                 sd_stream s) {
  if (rows <= 0) return SD_OK;
  bnormal_sample<<<blocks_for(rows * A, 256), 256, 0, (hipStream_t)s>>>(x, action, rows, A, min_std, max_std, seed,
                                                                        stream_id, step, row_offset, seed_ptr);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_bnormal_logp_ent_fwd(const float* x, const float* action, float* logp, float* ent, long rows, int A,
                                       float min_std, float max_std, sd_stream s) {
  if (rows <= 0) return SD_OK;
  bnormal_logp_ent_fwd<<<blocks_for(rows, 256), 256, 0, (hipStream_t)s>>>(x, action, logp, ent, rows, A, min_std,
                                                                          max_std);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_bnormal_logp_ent_bwd(const float* x, const float* action, const float* glogp, const float* gent,
                                       float* dx, long rows, int A, float min_std, float max_std, sd_stream s) {
  if (rows <= 0) return SD_OK;
  bnormal_logp_ent_bwd<<<blocks_for(rows * A, 256), 256, 0, (hipStream_t)s>>>(x, action, glogp, gent, dx, rows, A,
                                                                              min_std, max_std);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_bernoulli_fwd(const float* logit, const float* value, float* logp, float* mean, long rows,
                                sd_stream s) {
  if (rows <= 0) return SD_OK;
  bernoulli_fwd<<<blocks_for(rows, 256), 256, 0, (hipStream_t)s>>>(logit, value, logp, mean, rows);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_bernoulli_bwd(const float* logit, const float* value, const float* glogp, float* dlogit, long rows,
                                sd_stream s) {
  if (rows <= 0) return SD_OK;
  bernoulli_bwd<<<blocks_for(rows, 256), 256, 0, (hipStream_t)s>>>(logit, value, glogp, dlogit, rows);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_gru_fwd(const float* gates, const float* h, float* out, long M, int G, int Dg, sd_stream s) {
  if (M <= 0) return SD_OK;
  gru_fwd<<<blocks_for(M * G * Dg, 256), 256, 0, (hipStream_t)s>>>(gates, h, out, M, G, Dg);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_gru_bwd(const float* gates, const float* h, const float* dout, float* dgates, float* dh, long M, int G,
                          int Dg, int accumulate_dh, sd_stream s) {
  if (M <= 0) return SD_OK;
  gru_bwd<<<blocks_for(M * G * Dg, 256), 256, 0, (hipStream_t)s>>>(gates, h, dout, dgates, dh, M, G, Dg, accumulate_dh);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
