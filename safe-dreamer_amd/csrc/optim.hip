// Fused multi-tensor optimiser step over one flat fp32 parameter arena:
//   clip_grad_agc_ (utils/optim/agc.py:15-53, foreach path) -> LaProp.step (utils/optim/laprop.py:46-118)
// with LambdaLR warm-up (dreamer.py:214-225), plus the slow-critic Polyak update (dreamer.py:242-249).
//
// Parameters, gradients and both LaProp moments live in flat arenas; a static chunk table (built once on the
// host) maps each 256-thread block to a contiguous slice of one tensor, so per-tensor norms are fixed-order
// partial sums (deterministic) and the elementwise update is a single streaming pass (HBM-bound: 5 reads +
// 3 writes of 4 B per parameter). The scalar LaProp state (step, lr EMAs; Python floats in the reference) is
// kept in float64 on the device and advanced in-kernel, so a captured graph replays correct warm-up steps.
#include "common.h"
#include "sdhip.h"

namespace {

struct OptScalars {  // device-resident, float64 like the reference's Python floats
  double step;        // optimizer steps taken (LambdaLR last_epoch)
  double lr_ema1, lr_ema2;
  double lr;          // lr used by the most recent step
};

__global__ void norms_kernel(const float* __restrict__ p, const float* __restrict__ g, const long* __restrict__ chunk_beg,
                             const long* __restrict__ chunk_end, float* __restrict__ pn2, float* __restrict__ gn2) {
  __shared__ float red[4];
  const int c = blockIdx.x;
  const long b = chunk_beg[c], e = chunk_end[c];
  float sp = 0.f, sg = 0.f;
  for (long i = b + threadIdx.x; i < e; i += 256) {
    const float pv = p[i], gv = g[i];
    sp += pv * pv;
    sg += gv * gv;
  }
  sp = block_sum<256>(sp, red);
  sg = block_sum<256>(sg, red);
  if (threadIdx.x == 0) { pn2[c] = sp; gn2[c] = sg; }
}

__global__ void scales_kernel(const float* __restrict__ pn2, const float* __restrict__ gn2,
                              const int* __restrict__ tensor_chunk0, int ntensors, float clip, float pmin,
                              float* __restrict__ scale, float* __restrict__ gnorm_out, OptScalars* st, double lr0,
                              double warmup, double beta1, double beta2) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < ntensors) {
    float sp = 0.f, sg = 0.f;
    for (int c = tensor_chunk0[t]; c < tensor_chunk0[t + 1]; ++c) { sp += pn2[c]; sg += gn2[c]; }
    const float pn = sqrtf(sp), gn = sqrtf(sg);
    const float upper = fmaxf(pn, pmin) * clip;
    scale[t] = 1.f / fmaxf(gn / upper, 1.f);
    if (gnorm_out) gnorm_out[t] = gn;
  }
  if (t == 0) {
    const double lr = warmup > 0 ? lr0 * fmin(1.0, (st->step + 1.0) / warmup) : lr0;
    st->lr = lr;
    st->lr_ema1 = st->lr_ema1 * beta1 + (1.0 - beta1) * lr;
    st->lr_ema2 = st->lr_ema2 * beta2 + (1.0 - beta2);
  }
}

__global__ void laprop_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                              float* __restrict__ v, const long* __restrict__ chunk_beg, const long* __restrict__ chunk_end,
                              const int* __restrict__ chunk_tensor, const float* __restrict__ scale,
                              const OptScalars* __restrict__ st, float beta1, float beta2, float one_m_beta2, float eps) {
  const int c = blockIdx.x;
  const long b = chunk_beg[c], e = chunk_end[c];
  const float sc = scale[chunk_tensor[c]];
  const double lr = st->lr;
  const float bc2 = (float)st->lr_ema2;
  const float a1 = (float)((1.0 - (double)beta1) * lr);
  const double bc1 = lr != 0.0 ? st->lr_ema1 / lr : 1.0;
  const float neg_step = (float)(-(1.0 / bc1));
  for (long i = b + threadIdx.x; i < e; i += 256) {
    const float gv = g[i] * sc;                     // AGC (agc.py:52-56)
    float vv = v[i] * beta2;                        // exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
    vv = vv + one_m_beta2 * gv * gv;
    v[i] = vv;
    const float denom = sqrtf(vv / bc2) + eps;      // denom = (v / bc2).sqrt() + eps
    float mv = m[i] * beta1;                        // exp_avg.mul_(b1).add_(g/denom, alpha=(1-b1)*lr)
    mv = mv + a1 * (gv / denom);
    m[i] = mv;
    p[i] = p[i] + neg_step * mv;                    // p.add_(exp_avg, alpha=-1/bc1)
  }
}

__global__ void step_inc(OptScalars* st) { st->step += 1.0; }

__global__ void polyak_kernel(const float* __restrict__ src, float* __restrict__ dst, long n, float mix, float keep) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = mix * src[i] + keep * dst[i];
}

}  // namespace

extern "C" int sd_opt_scalars_bytes(void) { return (int)sizeof(OptScalars); }

extern "C" int sd_agc_laprop_step(float* params, float* grads, float* exp_avg, float* exp_avg_sq, const long* chunk_beg,
                                  const long* chunk_end, const int* chunk_tensor, const int* tensor_chunk0, int nchunks,
                                  int ntensors, float* workspace, void* scalars, float* grad_norms, float clip,
                                  float pmin, double lr0, double warmup, double beta1, double beta2, double eps,
                                  sd_stream stream_) {
  hipStream_t s = (hipStream_t)stream_;
  if (nchunks <= 0) return SD_OK;
  float* pn2 = workspace;
  float* gn2 = workspace + nchunks;
  float* scale = workspace + 2 * nchunks;
  OptScalars* st = (OptScalars*)scalars;
  norms_kernel<<<nchunks, 256, 0, s>>>(params, grads, chunk_beg, chunk_end, pn2, gn2);
  SD_LAUNCH_CHECK();
  scales_kernel<<<(ntensors + 255) / 256, 256, 0, s>>>(pn2, gn2, tensor_chunk0, ntensors, clip, pmin, scale, grad_norms,
                                                        st, lr0, warmup, beta1, beta2);
  SD_LAUNCH_CHECK();
  laprop_kernel<<<nchunks, 256, 0, s>>>(params, grads, exp_avg, exp_avg_sq, chunk_beg, chunk_end, chunk_tensor, scale,
                                         st, (float)beta1, (float)beta2, (float)(1.0 - beta2), (float)eps);
  SD_LAUNCH_CHECK();
  step_inc<<<1, 1, 0, s>>>(st);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_polyak(const float* src, float* dst, long n, float mix, sd_stream s) {
  if (n <= 0) return SD_OK;
  polyak_kernel<<<(int)((n + 255) / 256), 256, 0, (hipStream_t)s>>>(src, dst, n, mix, (float)(1.0 - (double)mix));
  SD_LAUNCH_CHECK();
  return SD_OK;
}
