// Fused multi-tensor optimiser step over one flat fp32 parameter arena:
//   clip_grad_agc_ (utils/optim/agc.py:15-53, foreach path) -> LaProp.step (utils/optim/laprop.py:46-118)
// with LambdaLR warm-up (dreamer.py:214-225), plus the slow-critic Polyak update (dreamer.py:242-249).
//
// Parameters, gradients and both LaProp moments live in flat arenas; a static chunk table (built once on the
// host) maps each 256-thread block to a contiguous slice of one tensor, so per-tensor norms are fixed-order
// partial sums (deterministic) and the elementwise update is a single streaming pass (HBM-bound: 2 reads for
// the norms, then 4 reads + 3 writes of 4 B per parameter). The scalar LaProp state (step, lr EMAs; Python floats in the reference) is
// kept in float64 on the device and advanced in-kernel, so a captured graph replays correct warm-up steps.
#include "common.h"
#include "sdhip.h"

namespace {

struct OptScalars {  // device-resident, float64 like the reference's Python floats
  double step;        // optimizer steps taken (LambdaLR last_epoch)
  double lr_ema1, lr_ema2;
  double lr;          // lr used by the most recent step
};

// Per-chunk sums of squares of parameters and gradients (float4 streams: chunks start 16-B aligned and a chunk's
// float4 tail runs into the zero padding of the arena, optim.py FlatArena). Block 0 also advances the scalar state
// (LambdaLR warm-up lr from the step count before this step, the lr EMAs, the step count): laprop_kernel reads it
// after this launch, and nothing else in this launch does.
__global__ void norms_kernel(const float* __restrict__ p, const float* __restrict__ g, const long* __restrict__ chunk_beg,
                             const long* __restrict__ chunk_end, float* __restrict__ pn2, float* __restrict__ gn2,
                             OptScalars* st, double lr0, double warmup, double beta1, double beta2, float gscale,
                             const int* __restrict__ chunk_tensor, int gate_tensor, const float* __restrict__ gate) {
  __shared__ float red[4];
  const int c = blockIdx.x;
  if (c == 0 && threadIdx.x == 0) {
    const double lr = warmup > 0 ? lr0 * fmin(1.0, (st->step + 1.0) / warmup) : lr0;
    st->lr = lr;
    st->lr_ema1 = st->lr_ema1 * beta1 + (1.0 - beta1) * lr;
    st->lr_ema2 = st->lr_ema2 * beta2 + (1.0 - beta2);
    st->step += 1.0;
  }
  const long b = chunk_beg[c], e4 = (chunk_end[c] + 3) & ~3L;
  const float gs = chunk_tensor[c] == gate_tensor ? gscale * gate[0] : gscale;
  float sp = 0.f, sg = 0.f;
  for (long i = b + 4 * threadIdx.x; i < e4; i += 1024) {
    const f32x4 pv = *reinterpret_cast<const f32x4*>(p + i), gv = gs * *reinterpret_cast<const f32x4*>(g + i);
    sp += pv[0] * pv[0] + pv[1] * pv[1] + pv[2] * pv[2] + pv[3] * pv[3];
    sg += gv[0] * gv[0] + gv[1] * gv[1] + gv[2] * gv[2] + gv[3] * gv[3];
  }
  sp = block_sum<256>(sp, red);
  sg = block_sum<256>(sg, red);
  if (threadIdx.x == 0) { pn2[c] = sp; gn2[c] = sg; }
}

// AGC scale of the block's tensor from its chunks' sums (every block of a tensor sums them in the same order), then
// the LaProp update of the chunk, float4-wide (elementwise: the same per-element arithmetic as the scalar form; the
// arena padding stays 0 through it). The block of a tensor's first chunk writes the tensor's gradient norm.
__global__ void laprop_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                              float* __restrict__ v, const long* __restrict__ chunk_beg, const long* __restrict__ chunk_end,
                              const int* __restrict__ chunk_tensor, const int* __restrict__ tensor_chunk0,
                              const float* __restrict__ pn2, const float* __restrict__ gn2, float* __restrict__ gnorm_out,
                              const OptScalars* __restrict__ st, float clip, float pmin, float beta1, float beta2,
                              float one_m_beta2, float eps, float gscale, int gate_tensor,
                              const float* __restrict__ gate, int zero_grads) {
  __shared__ float red[4];
  const int c = blockIdx.x, t = chunk_tensor[c], c0 = tensor_chunk0[t], c1 = tensor_chunk0[t + 1];
  float sp = 0.f, sg = 0.f;
  for (int k = c0 + threadIdx.x; k < c1; k += 256) { sp += pn2[k]; sg += gn2[k]; }
  sp = block_sum<256>(sp, red);
  sg = block_sum<256>(sg, red);
  const float pn = sqrtf(sp), gn = sqrtf(sg);
  const float sc = 1.f / fmaxf(gn / (fmaxf(pn, pmin) * clip), 1.f);  // agc.py:40-56
  const float gs = t == gate_tensor ? gscale * gate[0] : gscale;
  if (gnorm_out && c == c0 && threadIdx.x == 0) gnorm_out[t] = gn;
  const double lr = st->lr;
  const float bc2 = (float)st->lr_ema2;
  const float a1 = (float)((1.0 - (double)beta1) * lr);
  const double bc1 = lr != 0.0 ? st->lr_ema1 / lr : 1.0;
  const float neg_step = (float)(-(1.0 / bc1));
  const long b = chunk_beg[c], e4 = (chunk_end[c] + 3) & ~3L;
  for (long i = b + 4 * threadIdx.x; i < e4; i += 1024) {
    const f32x4 gq = *reinterpret_cast<const f32x4*>(g + i);
    if (zero_grads) *reinterpret_cast<f32x4*>(g + i) = f32x4{0.f, 0.f, 0.f, 0.f};  // the next update's zero_grad
    f32x4 vq = *reinterpret_cast<const f32x4*>(v + i), mq = *reinterpret_cast<const f32x4*>(m + i),
          pq = *reinterpret_cast<const f32x4*>(p + i);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gv = (gs * gq[j]) * sc;           // (data-parallel mean, gate) then AGC (agc.py:52-56)
      float vv = vq[j] * beta2;                     // exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
      vv = vv + one_m_beta2 * gv * gv;
      vq[j] = vv;
      const float denom = sqrtf(vv / bc2) + eps;    // denom = (v / bc2).sqrt() + eps
      float mv = mq[j] * beta1;                     // exp_avg.mul_(b1).add_(g/denom, alpha=(1-b1)*lr)
      mv = mv + a1 * (gv / denom);
      mq[j] = mv;
      pq[j] = pq[j] + neg_step * mv;                // p.add_(exp_avg, alpha=-1/bc1)
    }
    *reinterpret_cast<f32x4*>(v + i) = vq;
    *reinterpret_cast<f32x4*>(m + i) = mq;
    *reinterpret_cast<f32x4*>(p + i) = pq;
  }
}

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
                                  float grad_scale, int gate_tensor, const float* gate, int zero_grads,
                                  sd_stream stream_) {
  hipStream_t s = (hipStream_t)stream_;
  if (nchunks <= 0) return SD_OK;
  if (gate_tensor >= ntensors || (gate_tensor >= 0 && !gate)) return SD_EARG;
  float* pn2 = workspace;
  float* gn2 = workspace + nchunks;
  OptScalars* st = (OptScalars*)scalars;
  // two launches: per-chunk norms (+ the scalar state), then per-tensor AGC scale + LaProp per chunk
  norms_kernel<<<nchunks, 256, 0, s>>>(params, grads, chunk_beg, chunk_end, pn2, gn2, st, lr0, warmup, beta1, beta2,
                                       grad_scale, chunk_tensor, gate_tensor, gate);
  SD_LAUNCH_CHECK();
  laprop_kernel<<<nchunks, 256, 0, s>>>(params, grads, exp_avg, exp_avg_sq, chunk_beg, chunk_end, chunk_tensor,
                                         tensor_chunk0, pn2, gn2, grad_norms, st, clip, pmin, (float)beta1, (float)beta2,
                                         (float)(1.0 - beta2), (float)eps, grad_scale, gate_tensor, gate,
                                         zero_grads);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_polyak(const float* src, float* dst, long n, float mix, sd_stream s) {
  if (n <= 0) return SD_OK;
  polyak_kernel<<<(int)((n + 255) / 256), 256, 0, (hipStream_t)s>>>(src, dst, n, mix, (float)(1.0 - (double)mix));
  SD_LAUNCH_CHECK();
  return SD_OK;
}
