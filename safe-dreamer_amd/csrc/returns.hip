// λ-returns, imagination weights and the ReturnEMA quantile tracker.
//
//  * sd_lambda_return: Dreamer._lambda_return (dreamer.py:694-707), one lane per row, reverse recurrence in
//    registers; also emits the imagination continue probabilities and cumprod weights (dreamer.py:590-598)
//    when given continue logits (term = 1 - sigmoid(logit), last = 0).
//  * sd_return_ema: ReturnEMA.__call__ (networks.py:416-422): torch.quantile(x, [0.05, 0.95]) (linear
//    interpolation, torch's lerp) via an exact 4-pass 8-bit radix select for the 4 order statistics, then the
//    EMA update and (offset, scale). One 1024-thread workgroup; no host synchronisation (scalars stay on device).
#include "common.h"
#include "sdhip.h"

namespace {

// reward (row r, step t) at reward[r * rs.rew_r + t * rs.rew_t], the continue logit likewise (the imagined heads'
// outputs are time-major); term / last / the outputs are (N, T) row-major
struct LrStrides {
  long rew_r, rew_t, cont_r, cont_t, boot_r, boot_t;
};

__global__ void lambda_return_kernel(const float* __restrict__ reward, const float* __restrict__ term_in,
                                     const float* __restrict__ cont_logit, const float* __restrict__ last_in,
                                     const float* __restrict__ boot, LrStrides rs,
                                     float* __restrict__ ret, float* __restrict__ cont_out, float* __restrict__ weight,
                                     int N, int T, float disc, float lamb) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= N) return;
  const long base = (long)r * T;
  const long boot_row_stride = rs.boot_r, boot_t_stride = rs.boot_t;
  if (cont_logit && (cont_out || weight)) {
    float w = 1.f;
    for (int t = 0; t < T; ++t) {
      const float c = sigmoidf_(cont_logit[r * rs.cont_r + t * rs.cont_t]);
      if (cont_out) cont_out[base + t] = c;
      w = w * (c * disc);  // torch.cumprod(imag_cont * disc)
      if (weight) weight[base + t] = w;
    }
  }
  float out = boot[(long)r * boot_row_stride + (long)(T - 1) * boot_t_stride];
  for (int t = T - 2; t >= 0; --t) {
    const int i = t + 1;
    float term;
    if (term_in) term = term_in[base + i];
    else term = 1.f - sigmoidf_(cont_logit[r * rs.cont_r + i * rs.cont_t]);  // term = 1 - imag_cont (dreamer.py:599)
    const float last = last_in ? last_in[base + i] : 0.f;
    const float live = (1.f - term) * disc;
    const float cnt = (1.f - last) * lamb;
    const float interm = reward[r * rs.rew_r + i * rs.rew_t] +
                         (1.f - cnt) * live * boot[(long)r * boot_row_stride + (long)i * boot_t_stride];
    out = interm + live * cnt * out;
    ret[(long)r * (T - 1) + t] = out;
  }
}

// The same recursion with the inputs staged first: a workgroup stages LR_RB rows x T of reward, term (or continue
// logit), last and boot into LDS with all its threads (independent loads, one round trip), then one thread per row
// runs the serial T-step recursion from LDS. The per-thread version above issues its loads inside the serial loop,
// one dependent memory round trip per step (the replay return at B = 16, T = 64 took 17 us). Same arithmetic, same
// order: bit-identical.
constexpr int LR_RB = 16;
__global__ __launch_bounds__(256) void lambda_return_staged(const float* __restrict__ reward,
                                                            const float* __restrict__ term_in,
                                                            const float* __restrict__ cont_logit,
                                                            const float* __restrict__ last_in,
                                                            const float* __restrict__ boot, LrStrides rs,
                                                            float* __restrict__ ret,
                                                            float* __restrict__ cont_out, float* __restrict__ weight,
                                                            int N, int T, float disc, float lamb) {
  extern __shared__ float sm[];
  float* s_rew = sm;
  float* s_tc = sm + LR_RB * T;
  float* s_last = sm + 2 * LR_RB * T;
  float* s_boot = sm + 3 * LR_RB * T;
  const int r0 = blockIdx.x * LR_RB;
  for (int i = threadIdx.x; i < LR_RB * T; i += blockDim.x) {
    const int row = i / T, t = i % T, r = r0 + row;
    float rw = 0.f, tc = 0.f, ls = 0.f, bt = 0.f;
    if (r < N) {
      const long gi = (long)r * T + t;
      rw = reward[r * rs.rew_r + t * rs.rew_t];
      tc = term_in ? term_in[gi] : cont_logit[r * rs.cont_r + t * rs.cont_t];
      ls = last_in ? last_in[gi] : 0.f;
      bt = boot[(long)r * rs.boot_r + (long)t * rs.boot_t];
    }
    s_rew[i] = rw;
    s_tc[i] = tc;
    s_last[i] = ls;
    s_boot[i] = bt;
  }
  __syncthreads();
  const int row = threadIdx.x, r = r0 + row;
  if (row >= LR_RB || r >= N) return;
  const long base = (long)r * T;
  const float* rw = s_rew + row * T;
  const float* tc = s_tc + row * T;
  const float* ls = s_last + row * T;
  const float* bt = s_boot + row * T;
  if (!term_in && (cont_out || weight)) {
    float w = 1.f;
    for (int t = 0; t < T; ++t) {
      const float c = sigmoidf_(tc[t]);
      if (cont_out) cont_out[base + t] = c;
      w = w * (c * disc);  // torch.cumprod(imag_cont * disc)
      if (weight) weight[base + t] = w;
    }
  }
  float out = bt[T - 1];
  for (int t = T - 2; t >= 0; --t) {
    const int i = t + 1;
    const float term = term_in ? tc[i] : 1.f - sigmoidf_(tc[i]);  // term = 1 - imag_cont (dreamer.py:599)
    const float last = ls[i];
    const float live = (1.f - term) * disc;
    const float cnt = (1.f - last) * lamb;
    const float interm = rw[i] + (1.f - cnt) * live * bt[i];
    out = interm + live * cnt * out;
    ret[(long)r * (T - 1) + t] = out;
  }
}

SD_DEV uint32_t fkey(float f) {
  const uint32_t b = __float_as_uint(f);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
SD_DEV float funkey(uint32_t k) {
  const uint32_t b = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(b);
}

// x: n floats. ema[2] updated in place; os[0] = offset, os[1] = scale, qout[2] = raw quantiles (optional)
constexpr int RE_KPT = 16;  // keys kept in registers per thread (n <= 16,384: one global read of x in all 4 passes)
__global__ __launch_bounds__(1024) void return_ema_kernel(const float* __restrict__ x, int n, float* ema, float* os,
                                                          float* qout, float alpha, float q0, float q1) {
  __shared__ unsigned hist[4][256];
  __shared__ uint32_t prefix[4];
  __shared__ int rank[4];
  __shared__ float val[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // ranks = q * (n - 1) in float32 (torch.quantile), below = floor, above = ceil
  const float nm1 = (float)(n - 1);
  const float r0 = q0 * nm1, r1 = q1 * nm1;
  if (tid < 4) {
    const float rr = tid < 2 ? r0 : r1;
    const int lo = (int)floorf(rr);
    const int hi = (int)ceilf(rr);
    rank[tid] = (tid & 1) ? hi : lo;
    prefix[tid] = 0;
  }
  const bool in_regs = n <= 1024 * RE_KPT;
  uint32_t kr[RE_KPT];
#pragma unroll
  for (int j = 0; j < RE_KPT; ++j) {
    const int i = tid + 1024 * j;
    kr[j] = (in_regs && i < n) ? fkey(x[i]) : 0u;
  }
  __syncthreads();
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    (&hist[0][0])[tid] = 0;
    __syncthreads();
    const uint32_t hmask = pass == 0 ? 0u : (0xFFFFFFFFu << (32 - 8 * pass));
    const uint32_t p0 = prefix[0], p1 = prefix[1], p2 = prefix[2], p3 = prefix[3];
    auto add = [&](uint32_t k) {
      const uint32_t d = (k >> shift) & 0xFFu, h = k & hmask;
      if (h == p0) atomicAdd(&hist[0][d], 1u);
      if (h == p1) atomicAdd(&hist[1][d], 1u);
      if (h == p2) atomicAdd(&hist[2][d], 1u);
      if (h == p3) atomicAdd(&hist[3][d], 1u);
    };
    if (in_regs) {
#pragma unroll
      for (int j = 0; j < RE_KPT; ++j)
        if (tid + 1024 * j < n) add(kr[j]);
    } else {
      for (int i = tid; i < n; i += 1024) add(fkey(x[i]));
    }
    __syncthreads();
    if (wave < 4) {  // wave q finds quantile q's digit: lane l holds bins 4l..4l+3, wave-wide inclusive prefix sum
      const int rem = rank[wave];
      const unsigned c0 = hist[wave][4 * lane], c1 = hist[wave][4 * lane + 1], c2 = hist[wave][4 * lane + 2],
                     c3 = hist[wave][4 * lane + 3];
      const unsigned own = c0 + c1 + c2 + c3;
      unsigned inc = own;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
      }
      const unsigned exc = inc - own;
      // the lane whose [exc, inc) holds rem: its first bin with rem < running count
      const bool mine = (unsigned)rem >= exc && (unsigned)rem < inc;
      if (mine) {
        unsigned r = (unsigned)rem - exc;
        int b = 4 * lane;
        if (r >= c0) { r -= c0; ++b;
          if (r >= c1) { r -= c1; ++b;
            if (r >= c2) { r -= c2; ++b; } } }
        prefix[wave] |= ((uint32_t)b << shift);
        rank[wave] = (int)r;
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    for (int q = 0; q < 4; ++q) val[q] = funkey(prefix[q]);
    float qv[2];
    for (int j = 0; j < 2; ++j) {
      const float rr = j == 0 ? r0 : r1;
      const float w = rr - floorf(rr);
      const float a = val[2 * j], b = val[2 * j + 1];
      qv[j] = w < 0.5f ? a + w * (b - a) : b - (b - a) * (1.f - w);  // torch.lerp
    }
    if (qout) { qout[0] = qv[0]; qout[1] = qv[1]; }
    const float e0 = alpha * qv[0] + (1.f - alpha) * ema[0];
    const float e1 = alpha * qv[1] + (1.f - alpha) * ema[1];
    ema[0] = e0;
    ema[1] = e1;
    os[0] = e0;
    os[1] = fmaxf(e1 - e0, 1.f);
  }
}

}  // namespace

extern "C" int sd_lambda_return_strided(const float* reward, long rew_row_stride, long rew_t_stride, const float* term,
                                        const float* cont_logit, long cont_row_stride, long cont_t_stride,
                                        const float* last, const float* boot, long boot_row_stride, long boot_t_stride,
                                        float* ret, float* cont, float* weight, int N, int T, float disc, float lamb,
                                        sd_stream s) {
  if (N <= 0 || T <= 0) return SD_OK;
  if (!term && !cont_logit) return SD_EARG;
  const LrStrides rs{rew_row_stride, rew_t_stride, cont_row_stride, cont_t_stride, boot_row_stride, boot_t_stride};
  if (T <= 255 && !(term && cont_logit))  // 4 staged (LR_RB, T) planes fit the default 64 KB of dynamic LDS
    lambda_return_staged<<<(N + LR_RB - 1) / LR_RB, 256, 4 * LR_RB * T * sizeof(float), (hipStream_t)s>>>(
        reward, term, cont_logit, last, boot, rs, ret, cont, weight, N, T, disc, lamb);
  else
    lambda_return_kernel<<<(N + 255) / 256, 256, 0, (hipStream_t)s>>>(reward, term, cont_logit, last, boot, rs, ret,
                                                                     cont, weight, N, T, disc, lamb);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_lambda_return(const float* reward, const float* term, const float* cont_logit, const float* last,
                                const float* boot, long boot_row_stride, long boot_t_stride, float* ret, float* cont,
                                float* weight, int N, int T, float disc, float lamb, sd_stream s) {
  return sd_lambda_return_strided(reward, T, 1, term, cont_logit, T, 1, last, boot, boot_row_stride, boot_t_stride, ret,
                                  cont, weight, N, T, disc, lamb, s);
}

extern "C" int sd_return_ema(const float* x, int n, float* ema, float* offset_scale, float* quantiles, float alpha,
                             float q0, float q1, sd_stream s) {
  if (n <= 0) return SD_EARG;
  return_ema_kernel<<<1, 1024, 0, (hipStream_t)s>>>(x, n, ema, offset_scale, quantiles, alpha, q0, q1);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
