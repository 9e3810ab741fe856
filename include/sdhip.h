/* sdhip.h — C ABI of the MI355X-native Dreamer world-model / imagination hot path (libsdhip.so, gfx950).
 *
 * The reference (sharmaabhijith/safe-dreamer) has no FFI: its hot path is the Python call chain
 * Dreamer.update -> _cal_grad -> {encoder, RSSM.observe, RSSM.prior, kl_loss, heads, _imagine,
 * _lambda_return, ReturnEMA, losses} -> backward -> clip_grad_agc_ -> LaProp.step
 * (world_model/dreamer.py:402-707, world_model/rssm.py:36-230, world_model/networks.py:24-422,
 *  world_model/distributions.py:16-271, utils/optim/agc.py:15-53, utils/optim/laprop.py:46-118).
 * Each entry point below replaces one step of that chain; the comment names the reference code it stands in for.
 *
 * Conventions:
 *  - plain device pointers + sizes; fp32 data, int32 indices; row-major unless stated;
 *  - every call enqueues on `stream` and never synchronises, allocates or frees (graph-capturable);
 *  - the caller owns all memory, including workspaces;
 *  - return 0 on success, a positive hipError_t on launch failure, negative SD_E* on bad arguments.
 */
#ifndef SDHIP_H
#define SDHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* a hipStream_t passed as an opaque handle (0 = the null stream) */
typedef void* sd_stream;

#define SDHIP_ABI_VERSION 1
int sd_abi_version(void);

/* ---------------------------------------------------------------- dense contractions (MFMA fp32)
 * C[b] = alpha * A[b].B[b] (+ bias[b][n]) (+ beta * C[b]);  A: M x K, B: K x N, C: M x N (ldc).
 * a_kcontig: A(m,k) at A + m*lda + k   (else A + k*lda + m);
 * b_kcontig: B(k,n) at B + n*ldb + k   (else B + k*ldb + n).
 * Replaces nn.Linear fwd/bwd (networks.py:325,348-362; rssm.py:16-32,106-130), BlockLinear.forward's
 * einsum (networks.py:52) as a batch over blocks, Projector (networks.py:380-387) and torch.mm in the
 * Barlow loss (dreamer.py:528). ksplit > 1 needs workspace >= ksplit*batch*M*N floats (deterministic reduce).
 * tile: -1 auto, 0: 128x128, 1: 64x64, 2: 32x128, 3: 128x64. */
typedef struct sd_gemm_desc {
  const float* A;
  const float* B;
  float* C;
  const float* bias;
  long lda, ldb, ldc;
  long strideA, strideB, strideC, strideBias;
  int M, N, K, batch;
  int a_kcontig, b_kcontig;
  int ksplit, tile;
  float alpha, beta;
} sd_gemm_desc;
int sd_gemm_f32(const sd_gemm_desc* d, float* workspace, long workspace_floats, sd_stream stream);
/* Same contract on the split-bf16 path (csrc/gemm3_core.h): a = hi + lo (bf16 each), a*b = hi*hi + hi*lo + lo*hi on
 * v_mfma_f32_16x16x32_bf16 with f32 accumulation, ~1e-5 relative to the typical |term| * sqrt(K), 5.3x the f32 MFMA
 * rate. For gradient contractions and frozen heads (no sampled index depends on them). M, N or K < 64 -> f32 path. */
int sd_gemm_bf16x3(const sd_gemm_desc* d, float* workspace, long workspace_floats, sd_stream stream);
/* Weight gradient with its bias gradient (nn.Linear backward): the sd_gemm_bf16x3 contraction C = A . B for
 * rows-contiguous A (A = dy^T, a_kcontig 0, batch 1) that also forms rowsum[m] = alpha * sum_k A[m, k] (the bias
 * gradient, dy's column sums), added to rowsum when accumulate. With split-K the workspace needs ksplit * M floats
 * after the ksplit * M * N partial slabs. SD_ESHAPE for shapes the split-bf16 kernel does not take (M, N or K < 64). */
int sd_gemm_bf16x3_wgrad(const sd_gemm_desc* d, float* workspace, long workspace_floats, float* rowsum, int accumulate,
                         sd_stream stream);
/* The same for two layers' weight gradients over one input (dW = [dy_a | dy_b]^T x, C rows [0, rs_split) the first
 * layer's, the rest the second's, ldc apart — e.g. the imagined actor's and value head's first layers, whose weights
 * the arena places back to back, dreamer.py:607,613): the bias gradients of rows >= rs_split go to
 * rowsum2[m - rs_split]. 0 < rs_split < M. */
int sd_gemm_bf16x3_wgrad2(const sd_gemm_desc* d, float* workspace, long workspace_floats, float* rowsum,
                          float* rowsum2, int rs_split, int accumulate, sd_stream stream);
/* One MLP layer (networks.py:313-336 Linear -> RMSNorm -> SiLU chains) on the split-bf16 core, batched like the GEMM:
 * C[b] = act(rms(A[b]) * norm_w[b]) . B[b] + bias[b] with k-contiguous A (M, K) and B = W^T (W (N, K) row-major),
 * K a multiple of 32, beta 0, no split-K. norm_w null: A used as is. Otherwise rstd(row m) = 1 / sqrt(sum_q
 * part_in[b][q][m] / K + eps) from the producer's npart_in partial sums of squares per row, act 1 = SiLU (0: none).
 * part_out (N % 64 == 0) receives this layer's partials, (N / 64, M) per batch entry: part_out[b][n / 64][m] =
 * sum of C[b][m][n'] ^ 2 over the 64 columns n' of block n / 64. Returns SD_ESHAPE outside these shapes.
 * Per-entry operands (batch <= SD_MLP_MAXB): a non-null w_ptr[b] / bias_ptr[b] / norm_w_ptr[b] replaces
 * B + b * strideB / bias + b * strideBias / norm_w + b * stride_norm_w (each weight (w_rows[b], K) row-major with row
 * stride ldb), and w_rows[b] > 0 limits entry b's weight to that many rows: its columns n >= w_rows[b] of C get 0
 * (+ no bias). So several heads' layers run as one launch without stacking (or zero-padding) their weights. */
#define SD_MLP_MAXB 4
typedef struct sd_mlp_ext {
  const float* norm_w;
  long stride_norm_w;
  const float* part_in;
  long stride_part_in;
  int npart_in, act;
  float eps;
  float* part_out;
  long stride_part_out;
  const float* w_ptr[SD_MLP_MAXB];
  const float* bias_ptr[SD_MLP_MAXB];
  const float* norm_w_ptr[SD_MLP_MAXB];
  int w_rows[SD_MLP_MAXB];
} sd_mlp_ext;
int sd_gemm_bf16x3_mlp(const sd_gemm_desc* d, const sd_mlp_ext* x, sd_stream stream);

/* ---------------------------------------------------------------- row norms
 * y = act(x * rsqrt(mean(x^2) + eps) * w) per row; act 0 = none, 1 = SiLU. rstd (M) saved for backward.
 * Replaces nn.RMSNorm(eps=1e-4) + nn.SiLU in every MLP/RSSM layer (rssm.py:16-31,106-130; networks.py:326-327)
 * and RMSNorm2D on channels-last conv activations (networks.py:88-96). N <= 4096. */
int sd_rmsnorm_fwd(const float* x, const float* w, float* y, float* rstd, int M, int N, float eps, int act,
                   sd_stream stream);
/* same with an output row stride ldy (writes straight into a column slice of a wider activation) */
int sd_rmsnorm_fwd_ld(const float* x, const float* w, float* y, long ldy, float* rstd, int M, int N, float eps,
                      int act, sd_stream stream);
/* number of dw partial rows sd_rmsnorm_bwd writes (size dw_partial >= blocks * N) */
int sd_rmsnorm_bwd_blocks(int M, int N);
int sd_rmsnorm_bwd(const float* x, const float* w, const float* rstd, const float* dy, float* dx, float* dw,
                   float* dw_partial, int M, int N, int act, int accumulate_dx, int accumulate_dw, sd_stream stream);
/* the same with dy rows of stride ldy (a column block of a wider gradient read in place) */
int sd_rmsnorm_bwd_ld(const float* x, const float* w, const float* rstd, const float* dy, long ldy, float* dx,
                      float* dw, float* dw_partial, int M, int N, int act, int accumulate_dx, int accumulate_dw,
                      sd_stream stream);
/* the same with dx rows of stride ldx as well (writes into a column block of a wider gradient: two MLP heads' first
 * layers on the same input, whose weight gradients are then one sd_gemm_bf16x3_wgrad2 over the joint dy) */
int sd_rmsnorm_bwd_ldx(const float* x, const float* w, const float* rstd, const float* dy, long ldy, float* dx,
                       long ldx, float* dw, float* dw_partial, int M, int N, int act, int accumulate_dx,
                       int accumulate_dw, sd_stream stream);
/* out[n] (+)= sum_r in[r*ld + n] (fixed-order column sums; bias gradients) */
int sd_colsum(const float* in, float* out, int R, int N, long ld, int accumulate, sd_stream stream);
/* two-pass variant for long columns: workspace >= sd_colsum_chunks(R) * N floats */
int sd_colsum_chunks(int R);
int sd_colsum_ws(const float* in, float* out, int R, int N, long ld, int accumulate, float* workspace,
                 sd_stream stream);

/* ---------------------------------------------------------------- categorical latents
 * Straight-through one-hot sample of unimix categoricals (OneHotDist.__init__/rsample, distributions.py:16-33;
 * RSSM.get_dist(...).rsample(), rssm.py:177,194,219-220). groups = rows*S categoricals of K logits each.
 * Gumbel noise = Philox(seed, stream_id, step, (group + group_offset)*K + k) (see oracle/noise.py); when seed_ptr
 * is non-NULL the effective seed is seed + *seed_ptr (device-resident: a captured HIP graph replays fresh noise).
 * out = onehot(argmax) - y_soft + y_soft; index (groups) optional; entropy (groups) optional (metrics). */
int sd_onehot_sample_fwd(const float* logits, float* out, int* index, float* entropy, long groups, int K,
                         float unimix, uint64_t seed, int stream_id, int step, long group_offset,
                         const uint64_t* seed_ptr, sd_stream stream);
/* straight-through gradient: d logits (+)= d/dlogits <dout, y_soft> (recomputes y_soft from logits+noise) */
int sd_onehot_sample_bwd(const float* logits, const float* dout, float* dlogits, long groups, int K, float unimix,
                         uint64_t seed, int stream_id, int step, long group_offset, int accumulate,
                         const uint64_t* seed_ptr, sd_stream stream);
/* discrete actor: log_prob(action one-hot) and entropy of the unimix categorical (OneHotDist, distributions.py:16-36) */
int sd_onehot_logp_ent_fwd(const float* logits, const float* action, float* logp, float* ent, long rows, int K,
                           float unimix, sd_stream stream);
int sd_onehot_logp_ent_bwd(const float* logits, const float* action, const float* glogp, const float* gent,
                           float* dlogits, long rows, int K, float unimix, sd_stream stream);
/* KL(post || prior) on raw logits summed over S per row (dists.kl + RSSM.kl_loss sum, rssm.py:222-230) */
int sd_kl_fwd(const float* post, const float* prior, float* kl_row, float* dyn, float* rep, float free_nats, int rows,
              int S, int K, sd_stream stream);
/* gradients of clip(kl_row, min=free): d_post <- g_rep * pa (lpa - lpb - kl_s), d_prior <- g_dyn * (pb - pa) */
int sd_kl_bwd(const float* post, const float* prior, const float* kl_row, const float* g_rep, const float* g_dyn,
              float free_nats, float* d_post, float* d_prior, int rows, int S, int K, int acc_post, int acc_prior,
              sd_stream stream);

/* ---------------------------------------------------------------- heads
 * symexp two-hot (TwoHot, distributions.py:67-129; symexp_twohot bins 242-251): mode, log_prob fwd/bwd. NB odd <= 255 */
int sd_twohot_mode(const float* logits, const float* bins, float* out, long rows, int NB, sd_stream stream);
int sd_twohot_logp_fwd(const float* logits, const float* bins, const float* target, float* logp, long rows, int NB,
                       sd_stream stream);
int sd_twohot_logp_bwd(const float* logits, const float* bins, const float* target, const float* glogp,
                       float* dlogits, long rows, int NB, int accumulate, sd_stream stream);
/* Replay-value loss (dreamer.py:652-658; replaces the two TwoHot.log_prob calls, distributions.py:100-129, and the
 * weighted mean's elementwise ops). The value head ran on all Tl posterior steps of B rows: logits (B, Tl, NB),
 * slow / last (B, Tl); the Tr = Tl - 1 steps with a replay return ret (B, Tr) are the loss rows:
 * row_loss[b, t] = (1 - last[b, t]) * (-logp(ret[b, t]) - logp(slow[b, t])). The backward writes the gradient of
 * mean(row_loss) * gscale[0] (device scalar; inv_n = 1 / (B Tr)) for every (B, Tl) logits row (zero for t >= Tr).
 * NB <= 256. */
int sd_repval_loss_fwd(const float* logits, const float* bins, const float* ret, const float* slow, const float* last,
                       float* row_loss, int B, int Tl, int Tr, int NB, sd_stream s);
int sd_repval_loss_bwd(const float* logits, const float* bins, const float* ret, const float* slow, const float* last,
                       const float* gscale, float inv_n, float* dlogits, int B, int Tl, int Tr, int NB, sd_stream s);
/* Imagined actor-critic losses (dreamer.py:623-636, 653-671) over H * N time-major rows r = t * N + n: value logits
 * vl (H * N, NB), logpi / ent (H * N) of the imagined actions, slow (H * N) slow-value targets; batch-major
 * ret (N, H), w = weight (N, H1), val = imagined value (H1, N) time-major; scale: device scalar (ReturnEMA scale).
 * fwd writes adv (N, H) = (ret - val[:, :H]) / scale and the row terms rows_v = w (-logp(ret) - logp(slow)),
 * rows_p = w -(logpi adv + coef ent) (H * N each; the losses are their means). bwd: d vl, d logpi, d ent from the
 * upstream gradients of the two means: device scalars gpolicy / gvalue (null = 0) times spolicy / svalue (the loss
 * scales, so both can point at the gradient of the weighted total). */
int sd_imag_ac_loss_fwd(const float* vl, const float* bins, const float* ret, const float* slow, const float* w,
                        const float* val, const float* scale, const float* logpi, const float* ent, float coef, long N,
                        int H, int H1, int NB, float* rows_v, float* rows_p, float* adv, sd_stream s);
int sd_imag_ac_loss_bwd(const float* vl, const float* bins, const float* ret, const float* slow, const float* w,
                        const float* adv, const float* gpolicy, const float* gvalue, float spolicy, float svalue,
                        float coef, long N, int H, int H1, int NB, float* dvl, float* dlogpi, float* dent, sd_stream s);
/* bounded normal actor (bounded_normal, distributions.py:217-222): x (rows, 2A) = [mean | std-logit] */
int sd_bnormal_sample(const float* x, float* action, long rows, int A, float min_std, float max_std, uint64_t seed,
                      int stream_id, int step, long row_offset, const uint64_t* seed_ptr, sd_stream stream);
int sd_bnormal_logp_ent_fwd(const float* x, const float* action, float* logp, float* ent, long rows, int A,
                            float min_std, float max_std, sd_stream stream);
int sd_bnormal_logp_ent_bwd(const float* x, const float* action, const float* glogp, const float* gent, float* dx,
                            long rows, int A, float min_std, float max_std, sd_stream stream);
/* Bernoulli(logits) continue head (binary, distributions.py:238): logp, mean = sigmoid */
int sd_bernoulli_fwd(const float* logit, const float* value, float* logp, float* mean, long rows, sd_stream stream);
int sd_bernoulli_bwd(const float* logit, const float* value, const float* glogp, float* dlogit, long rows,
                     sd_stream stream);

/* ---------------------------------------------------------------- RSSM deterministic transition
 * GRU-style gates of Deter.forward (rssm.py:65-75) on the dyn_gru BlockLinear output gates (M, G, 3, Dg). */
int sd_gru_fwd(const float* gates, const float* h, float* out, long M, int G, int Dg, sd_stream stream);
int sd_gru_bwd(const float* gates, const float* h, const float* dout, float* dgates, float* dh, long M, int G, int Dg,
               int accumulate_dh, sd_stream stream);
/* a / max(|a|, 1) (rssm.py:44) */
int sd_action_norm(const float* a, float* y, long n, sd_stream stream);
/* y[r,:] = mask[r*mask_stride] ? 0 : x[r,:]   (reset of the posterior state, rssm.py:161-165) */
int sd_mask_rows(const float* x, const uint8_t* mask, long mask_stride, float* y, long rows, int width,
                 sd_stream stream);

/* ---------------------------------------------------------------- returns
 * Dreamer._lambda_return (dreamer.py:694-707): ret (N, T-1). term/last may be NULL (term = 1 - sigmoid(cont_logit),
 * last = 0: the imagination case, dreamer.py:597-602). With cont_logit also emits cont = sigmoid and
 * weight = cumprod(cont * disc). boot(r, t) = boot[r*boot_row_stride + t*boot_t_stride]. */
int sd_lambda_return(const float* reward, const float* term, const float* cont_logit, const float* last,
                     const float* boot, long boot_row_stride, long boot_t_stride, float* ret, float* cont,
                     float* weight, int N, int T, float disc, float lamb, sd_stream stream);
/* The same with reward(r, t) = reward[r*rew_row_stride + t*rew_t_stride] and the continue logit likewise (the
 * imagined heads' time-major outputs read in place, dreamer.py:598-602); term / last / ret / cont / weight stay
 * (N, T) row-major. sd_lambda_return is this with strides (T, 1). */
int sd_lambda_return_strided(const float* reward, long rew_row_stride, long rew_t_stride, const float* term,
                             const float* cont_logit, long cont_row_stride, long cont_t_stride, const float* last,
                             const float* boot, long boot_row_stride, long boot_t_stride, float* ret, float* cont,
                             float* weight, int N, int T, float disc, float lamb, sd_stream stream);
/* ReturnEMA (networks.py:406-422): torch.quantile(x, [q0, q1]) (exact radix select + lerp), ema <- alpha q +
 * (1-alpha) ema, offset_scale = (ema[0], max(ema[1]-ema[0], 1)). quantiles (2) optional. */
int sd_return_ema(const float* x, int n, float* ema, float* offset_scale, float* quantiles, float alpha, float q0,
                  float q1, sd_stream stream);

/* ---------------------------------------------------------------- convolution (NHWC, implicit GEMM on MFMA)
 * Conv2dSamePad, stride 1 (networks.py:59-85): out (Nb, Hs<<ups, Ws<<ups, Co); w (Co, kh, kw, Ci); ups = 1 reads
 * the input through nn.Upsample(2, nearest) (ConvDecoder, networks.py:259-265). */
int sd_conv2d_fwd(const float* in, const float* w, const float* bias, float* out, int Nb, int Hs, int Ws, int Ci,
                  int Co, int kh, int kw, int pad, int ups, sd_stream stream);
/* Optional accumulation target of the bwd-weight entry points below: when acc is non-null the [dW | db] result is
 * ADDED into the parameter gradients (dw (Co, kh, kw, ci_w), ci_w <= Ci: the input's padded channels dropped; db
 * (Co)) by the launch's final reduction instead of being written to dw_db (which is then scratch for the paths
 * without a reduction) — no separate add launches. */
typedef struct sd_wgrad_acc {
  float* dw;
  float* db;
  int ci_w;
} sd_wgrad_acc;
/* dw_db (Co, kh*kw*Ci + 1) = [dW | d bias]; ksplit > 1 needs workspace >= ksplit*Co*(kh*kw*Ci+1) floats */
int sd_conv2d_wgrad(const float* in, const float* dout, float* dw_db, float* workspace, long ws_floats, int ksplit,
                    int Nb, int Hs, int Ws, int Ci, int Co, int kh, int kw, int pad, int ups, const sd_wgrad_acc* acc,
                    sd_stream stream);
/* partial-slab count sd_conv2d_wgrad uses for this request (workspace >= slabs * Co * (kh*kw*Ci + 1) floats when
 * slabs > 1): stride-1 convs with Co % 16 == 0 take a direct kernel (dy rows + input patch staged in LDS, no im2col
 * re-reads) whose split is fixed by the library; others use `ksplit` over the im2col implicit GEMM. */
int sd_conv2d_wgrad_slabs(int Nb, int Hs, int Ws, int Ci, int Co, int kh, int kw, int ups, int ksplit);
/* bwd-weight of a pooled ConvEncoder stage from (dpool, argmax) of sd_pool_rms_bwd_compact (the conv gradient is
 * expanded inside the direct kernel while staging). _slabs: workspace slabs (each Co x (kh*kw*Ci+1) floats), 0 when
 * the shape is outside the direct kernel (then sd_conv2d_wgrad_pool returns SD_ESHAPE). Alignment: in and dpool
 * 16 B, amax 4 B (read as uint32 words), else SD_EARG. */
int sd_conv2d_wgrad_pool_slabs(int Nb, int H, int W, int Ci, int Co, int kh, int kw);
int sd_conv2d_wgrad_pool(const float* in, const float* dpool, const uint8_t* amax, float* dw_db, float* workspace,
                         long ws_floats, int Nb, int H, int W, int Ci, int Co, int kh, int kw, int pad,
                         const sd_wgrad_acc* acc, sd_stream stream);
/* Split-bf16 (bf16x3, ~1e-5 relative) backward convolutions (csrc/conv.hip, gemm3_core.h). SD_ESHAPE when the
 * shape is outside the kernels (the caller then takes the f32 path). dgrad: same arguments as sd_conv2d_fwd with
 * in = dOut (Ci channels), w = the flipped weight (sd_conv_flip_weight), out = dIn (Co channels), ups = 0.
 * wgrad: [dW | db] as sd_conv2d_wgrad (ups = 0, Ci % 4 == 0, Ci >= 16, Co <= 64, power-of-two W >= 8);
 * workspace >= slabs * Co * (kh*kw*Ci + 1) floats, slabs from sd_conv2d_wgrad_bf16x3_slabs (SD_ESHAPE: not
 * eligible). Replace the backward of Conv2dSamePad (networks.py:59-85). */
int sd_conv2d_dgrad_bf16x3(const float* dout, const float* wflip, float* din, int Nb, int Hs, int Ws, int Ci, int Co,
                           int kh, int kw, int pad, sd_stream stream);
int sd_conv2d_wgrad_bf16x3_slabs(int Nb, int Hs, int Ws, int Ci, int Co, int kh, int kw, int ups);
int sd_conv2d_wgrad_bf16x3(const float* in, const float* dout, float* dw_db, float* workspace, long ws_floats,
                           int Nb, int Hs, int Ws, int Ci, int Co, int kh, int kw, int pad, const sd_wgrad_acc* acc,
                           sd_stream stream);
/* sd_conv2d_wgrad_pool (the pooled first stage's bwd-weight from sd_pool_rms_bwd_compact's gradient + argmax) on the
 * split-bf16 direct kernel (conv_wgrad3_direct, the 32-pixel steps dealt to the 8 waves, the pooled gradient routed
 * through the argmax while staged). Same arguments; _slabs: workspace slabs (each Co x (kh*kw*Ci+1) floats), 0 when
 * the shape is outside it (J + 1 <= 112, W a power of two dividing 256 into an even row count; then SD_ESHAPE). */
int sd_conv2d_wgrad_pool_bf16x3_slabs(int Nb, int H, int W, int Ci, int Co, int kh, int kw);
int sd_conv2d_wgrad_pool_bf16x3(const float* in, const float* dpool, const uint8_t* amax, float* dw_db,
                                float* workspace, long ws_floats, int Nb, int H, int W, int Ci, int Co, int kh, int kw,
                                int pad, const sd_wgrad_acc* acc, sd_stream stream);
/* The same bwd-data as a direct convolution (csrc/conv.hip conv_dgrad3_direct: each workgroup stages its dOut patch
 * once, split to bf16 planes; same products and order per k as sd_conv2d_dgrad_bf16x3, k summed in the same order).
 * wsplit = sd_conv_split_weight(wflip, rows = Co, K = kh*kw*Ci). Instantiated for the 5x5 pad-2 stages of the
 * BASELINE encoders' two large bwd-data stages (dOut -> dIn channels 48->32 at 32x32, 64->48 at 16x16);
 * SD_ESHAPE otherwise (the caller then takes sd_conv2d_dgrad_bf16x3). Replaces conv_dgrad's role in the backward of
 * Conv2dSamePad (networks.py:59-85). */
int sd_conv2d_dgrad_direct(const float* dout, const void* wsplit, float* din, int Nb, int Hs, int Ws, int Ci, int Co,
                           int kh, int kw, int pad, sd_stream stream);
/* sd_conv2d_fwd_pool on the fp32-accurate three-way split-bf16 path (csrc/conv.hip conv_fwd6_direct_pool, gemm6_core.h
 * "bf16x6": six bf16 MFMAs per product, <= 2^-26 |ab| dropped per product, fp32-level error): a direct convolution from
 * the tile's input patch staged once in LDS as three bf16 planes. wsplit3 = sd_conv_split3_weight(w, rows = Co,
 * K = kh*kw*Ci). Instantiated for the 5x5 pad-2 stages 32->48 at 32x32 and 48->64 at 16x16 (SD_ESHAPE otherwise:
 * the caller takes sd_conv2d_fwd_pool). Replaces ConvEncoder's Conv2dSamePad -> MaxPool2d -> RMSNorm2D -> SiLU stage
 * (networks.py:201-216). */
int sd_conv2d_fwd_pool6(const float* in, const void* wsplit3, const float* bias, const float* nw, float* pooled,
                        uint8_t* amax, float* y, float* rstd, int Nb, int Hs, int Ws, int Ci, int Co, int kh, int kw,
                        int pad, float eps, int nchw_flat, sd_stream stream);
/* wsplit3 = [plane][rows][KP] bf16 three-way split (a0 = bf16(w), a1 = bf16(w - a0), a2 = bf16(w - a0 - a1)) of a
 * (rows, K) fp32 matrix, KP = K rounded up to 32, zero past K: 6 * rows * KP bytes */
int sd_conv_split3_weight(const float* w, void* wsplit, int rows, int K, sd_stream stream);
/* wsplit = [plane][rows][KP] bf16 (hi = bf16(w), lo = bf16(w - hi), KP = K rounded up to 32, zero past K) of a
 * (rows, K) fp32 matrix: 4 * rows * KP bytes */
int sd_conv_split_weight(const float* w, void* wsplit, int rows, int K, sd_stream stream);
/* Wf[ci][ky][kx][co] = W[co][kh-1-ky][kw-1-kx][ci]  (input-gradient conv weights) */
int sd_conv_flip_weight(const float* w, float* wf, int Co, int kh, int kw, int Ci, sd_stream stream);
/* backward of nearest 2x upsample: din (Nb,H,W,C) = 2x2 sums of du (Nb,2H,2W,C) */
int sd_sumpool2(const float* du, float* din, int Nb, int H, int W, int C, sd_stream stream);
/* ConvEncoder layer tail: y = SiLU(RMSNorm2D(MaxPool2d(2)(x))) (networks.py:211-214); pooled/amax/rstd saved.
 * nchw_flat: write y in the reference's NCHW flatten order (networks.py:232). C <= 128. */
/* ConvEncoder stage fused (networks.py:201-216): conv -> MaxPool2d(2) -> RMSNorm2D(nw) -> SiLU in one launch, writing
 * only the pooled outputs (pooled pre-norm values, 2x2 argmax, rstd: the inputs of sd_pool_rms_bwd). Returns
 * SD_ESHAPE (nothing launched) outside its instantiations: Co in {16,32,48,64}, Ci % 4 == 0, W a power of two <= 64,
 * H even, Nb*H*W % 128 == 0 — the caller then runs sd_conv2d_fwd + sd_pool_rms_fwd. */
int sd_conv2d_fwd_pool(const float* in, const float* w, const float* bias, const float* nw, float* pooled,
                       uint8_t* amax, float* y, float* rstd, int Nb, int Hs, int Ws, int Ci, int Co, int kh, int kw,
                       int pad, float eps, int nchw_flat, sd_stream stream);
int sd_pool_rms_fwd(const float* x, const float* w, float* pooled, uint8_t* amax, float* y, float* rstd, int Nb,
                    int H, int W, int C, float eps, int nchw_flat, sd_stream stream);
/* dw_partial >= (sd_pool_rms_bwd_blocks + sd_colsum_chunks(sd_pool_rms_bwd_blocks)) * C floats */
int sd_pool_rms_bwd_blocks(int Nb, int H, int W);
int sd_pool_rms_bwd(const float* pooled, const uint8_t* amax, const float* w, const float* rstd, const float* dy,
                    float* dx, float* dw, float* dw_partial, int Nb, int H, int W, int C, int nchw_flat,
                    int accumulate_dw, sd_stream stream);
/* Same backward, writing the pooled-resolution gradient dpool (Nb, H/2, W/2, C) instead of scattering it into the
 * full-resolution (3/4 zero) conv gradient; consumed by sd_conv2d_wgrad_pool together with the forward's argmax. */
int sd_pool_rms_bwd_compact(const float* pooled, const uint8_t* amax, const float* w, const float* rstd,
                            const float* dy, float* dpool, float* dw, float* dw_partial, int Nb, int H, int W, int C,
                            int nchw_flat, int accumulate_dw, sd_stream stream);

/* ---------------------------------------------------------------- optimiser (flat parameter arena)
 * clip_grad_agc_ (agc.py:15-53) + LaProp.step (laprop.py:46-118) + LambdaLR warm-up (dreamer.py:214-225), fused.
 * chunk tables are device arrays built once by the caller; scalars = sd_opt_scalars_bytes() zeroed bytes of device
 * memory (float64 step / lr EMAs); workspace >= 3*nchunks floats; grad_norms (ntensors) optional. Every gradient is
 * read as grad_scale * g (data parallel: 1 / world after the sum all-reduce), tensor gate_tensor's (>= 0) also times
 * the device scalar *gate (DreamerPro's prototype freeze, dreamer.py:424-425); -1 = no gated tensor. zero_grads: every
 * gradient element the step reads is set to 0 after the read (the next update's optimizer.zero_grad(), dreamer.py:423,
 * folded into this pass; the arena padding between tensors stays 0 anyway). */
int sd_opt_scalars_bytes(void);
int sd_agc_laprop_step(float* params, float* grads, float* exp_avg, float* exp_avg_sq, const long* chunk_beg,
                       const long* chunk_end, const int* chunk_tensor, const int* tensor_chunk0, int nchunks,
                       int ntensors, float* workspace, void* scalars, float* grad_norms, float clip, float pmin,
                       double lr0, double warmup, double beta1, double beta2, double eps, float grad_scale,
                       int gate_tensor, const float* gate, int zero_grads, sd_stream stream);
/* slow critic: dst = mix*src + (1-mix)*dst (Dreamer._update_slow_target, dreamer.py:242-249) */
int sd_polyak(const float* src, float* dst, long n, float mix, sd_stream stream);

/* ---------------------------------------------------------------- metrics
 * The update's metric vector in two launches (tools.tensorstats, tools.py:275-281, and the scalar losses / means of
 * dreamer.py:566-671): out[b] = sum over requests r with r.out == b (in order) of r.scale * stat(r.x[0:r.n]),
 * stat = mean (SD_STAT_MEAN, a scalar is its own mean), unbiased std, min or max. Request q covers chunks
 * [chunk0, chunk0 + ceil(n / SD_STAT_CHUNK)) (consecutive from 0); workspace >= 5 floats per chunk. */
#define SD_STAT_CHUNK 4096
#define SD_STAT_MEAN 0
#define SD_STAT_STD 1
#define SD_STAT_MIN 2
#define SD_STAT_MAX 3
#define SD_MAX_STATS 96
typedef struct sd_stat_req {
  const float* x;
  long n;
  int kind, out;
  float scale;
  int chunk0;
  const float* sub; /* nullable device scalars: the stat becomes (stat - sub[0]) / div[0] before the scale */
  const float* div;
} sd_stat_req;
typedef struct sd_stats {
  sd_stat_req r[SD_MAX_STATS];
  int nreq;
} sd_stats;
int sd_multi_stats(const sd_stats* s, float* workspace, float* out, int nout, sd_stream stream);

/* World-model loss total (dreamer.py:571-576, `sum(v * self._scales[k] for k, v in losses.items())`): term i is
 * coef_i * mean(x_i[0:n_i]) (coef = -1 for the log-prob losses), total = sum_i scale_i * term_i in term order;
 * means (n terms, nullable) and total (1) on device. Backward: g_i[j] = (g_total * scale_i + g_means[i]) * coef_i / n_i
 * into each term's g (nullable = no gradient; g_total / g_means nullable = 0). One launch each way. */
#define SD_MAX_LOSS_TERMS 8
typedef struct sd_loss_term {
  const float* x;
  float* g;
  long n;
  float coef, scale;
} sd_loss_term;
typedef struct sd_loss_terms {
  sd_loss_term t[SD_MAX_LOSS_TERMS];
  int n;
} sd_loss_terms;
int sd_loss_terms_fwd(const sd_loss_terms* terms, float* means, float* total, sd_stream stream);
int sd_loss_terms_bwd(const sd_loss_terms* terms, const float* g_total, const float* g_means, sd_stream stream);

/* Layout copies in one launch (the scan backward's W^T images, rssm.py:36-75 contractions transposed; the first
 * conv layer's channel pad; get_feat's concatenation into a strided slot): mode 0 transposes src (batch, rows, cols;
 * row stride sr, batch stride sb) into dst (batch, cols, rows) contiguous; mode 1 copies it into dst rows
 * (batch * rows of stride dld, 0 = dcols) of dcols values, zero-filling columns >= cols. */
#define SD_MAX_LAYOUT_COPIES 12
typedef struct sd_layout_copy {
  const float* src;
  float* dst;
  long sb, sr, dld;
  int batch, rows, cols, dcols, mode;
} sd_layout_copy;
typedef struct sd_layout_copies {
  sd_layout_copy e[SD_MAX_LAYOUT_COPIES];
  int n;
} sd_layout_copies;
int sd_layout_copies_run(const sd_layout_copies* copies, sd_stream stream);
/* is_last / is_terminal bytes (n) -> f32 last, term, cont = 1 - term (the losses' episode-boundary operands) */
int sd_episode_flags(const uint8_t* is_last, const uint8_t* is_term, long n, float* last, float* term, float* cont,
                     sd_stream stream);

/* ---------------------------------------------------------------- misc
 * Measurement aid: one empty dispatch (kernel k_trace_mark, `tag` workgroups, 1 <= tag <= 64) that a rocprofv3 kernel
 * trace can find; bench.py brackets its timed steps with tags 1 and 2 (tools/kernel_table.py). */
int sd_trace_mark(int tag, sd_stream stream);
/* Measurement aid: shader clock under an f32-MFMA load. nwg workgroups run `iters` MFMA chains each; stamps
 * (2 * nwg int64) receive per workgroup (shader cycles, 100 MHz ticks) around the loop: clock = cycles / ticks * 0.1 GHz.
 * sink (nwg floats) is never written in practice. */
int sd_clock_probe(long long* stamps, float* sink, int nwg, int iters, sd_stream stream);
/* Scheduling aid: a stream whose workgroups run only on CUs [first_cu, first_cu + ncu) (hipExtStreamCreateWithCUMask),
 * for the update's filler phases, so they leave the rest of the chip to the latency-bound chain beside them
 * (SDREAMER_FILL_CUS, dreamer.py). sd_stream_destroy releases it. */
int sd_stream_create_cumask(int first_cu, int ncu, sd_stream* out);
int sd_stream_destroy(sd_stream stream);
/* Scheduling aid: dynamic LDS (bytes, 0..65536) reserved by every split-bf16 / f32 GEMM launch issued after this
 * call (the kernels do not use it), so fewer of their workgroups fit on a CU beside the latency-bound chain of the
 * other stream; graph-captured per phase (SDREAMER_FILL_LDS, dreamer.py). Returns the previous value. */
int sd_set_lds_pad(int bytes);
/* number of launches that ran without the requested pad because the runtime refused the kernel's dynamic-LDS limit
 * (each refused kernel is also named once on stderr) */
int sd_lds_pad_failures(void);
/* Dreamer.preprocess + ConvEncoder's "-0.5": out = in/255 - shift (dreamer.py:710-713, networks.py:224) */
int sd_u8_to_f32(const uint8_t* in, float* out, long n, float shift, sd_stream stream);
/* NHWC channel pad + shift: out[p][c] = in[p][c] - shift (c < C), 0 (C <= c < Cp). The ConvEncoder input
 * (obs - 0.5, networks.py:224) padded 3 -> 4 channels so the first conv takes the float4 / direct-wgrad paths. */
int sd_pad_channels(const float* in, float* out, long pixels, int C, int Cp, float shift, sd_stream stream);
/* Both float forms of a uint8 NHWC image in one launch: img = in / 255 (Dreamer.preprocess, nullable when nothing
 * reads it) and enc = in / 255 - shift zero-padded to Cp channels (the ConvEncoder input, networks.py:224). */
int sd_u8_image_inputs(const uint8_t* in, float* img, float* enc, long pixels, int C, int Cp, float shift,
                       sd_stream stream);
/* symlog (distributions.py:8-9) for MLP-encoder inputs (networks.py:333-334) */
int sd_symlog(const float* x, float* y, long n, sd_stream stream);
int sd_fill_gumbel(float* out, long n, uint64_t seed, int stream_id, int step, long offset, sd_stream stream);
int sd_fill_normal(float* out, long n, uint64_t seed, int stream_id, int step, long offset, sd_stream stream);
/* Barlow-twins loss pieces (dreamer.py:525-532): column mean / unbiased std, standardise fwd/bwd,
 * loss = sum (c_ii-1)^2 + lambd sum_{i!=j} c_ij^2 (partial >= 2*nblocks floats), dc = g * dloss/dc */
int sd_colstats(const float* x, int R, int C, float* mean, float* stdv, sd_stream stream);
int sd_standardize(const float* x, const float* mean, const float* stdv, float* y, long R, int C, float eps,
                   sd_stream stream);
int sd_standardize_bwd(const float* x, const float* mean, const float* stdv, const float* dn, float* dx, int R,
                       int C, float eps, sd_stream stream);
int sd_barlow_loss(const float* c, int E, float lambd, float* partial, int nblocks, float* loss, sd_stream stream);
int sd_barlow_dc(const float* c, const float* g, float* dc, int E, float lambd, sd_stream stream);
/* Data-parallel Barlow (sdreamer/parallel.py barlow_dist; dreamer.py:525-532 over the global batch of Nt rows, R of
 * them on this rank, E = embed width). sums (2, E): the all-reduced column sums of x1 and x2.
 * center: d1 = x1 - sums[0] / Nt, d2 = x2 - sums[1] / Nt (R, E), q (2, E) = this rank's column sums of d^2.
 * finish: from stats = [q (2, E) | d1^T d2 (E, E)] all-reduced: stdv (2, E) = sqrt(q / (Nt - 1)), sc = stdv + 1e-8,
 *   c (E, E) = (d1^T d2)_ij / (sc1_i sc2_j) / Nt, n2 (R, E) = d2 / sc2, z2 (E) = (sums[1] - Nt (sums[1] / Nt)) / sc2.
 * rowstats: s0_j = (dc z2)_j / Nt, A_j = (stdv1_j + 1e-8) sum_k dc_jk c_jk.
 * dist_dx: dx1 = world ((dn1 - s0 / Nt) / sc1 - (x1 - sums[0] / Nt) A / (sc1^2 (Nt - 1) stdv1)), dn1 = n2 dc^T / Nt. */
int sd_barlow_center(const float* x1, const float* x2, const float* sums, float Nt, int R, int E, float* d1, float* d2,
                     float* q, sd_stream stream);
int sd_barlow_finish(const float* stats, const float* sums, float Nt, int E, const float* d2, int R, float* c,
                     float* stdv, float* n2, float* z2, sd_stream stream);
int sd_barlow_rowstats(const float* dc, const float* c, const float* z2, const float* stdv1, float Nt, int E, float* s0,
                       float* A, sd_stream stream);
int sd_barlow_dist_dx(const float* x1, const float* dn1, const float* sums, const float* stdv1, const float* s0,
                      const float* A, float Nt, float world, long R, int E, float* dx1, sd_stream stream);

/* ---------------------------------------------------------------- fused RSSM posterior scan (ObserveScan)
 * RSSM.observe's recurrence (rssm.py:140-178 + Deter.forward rssm.py:36-75) for B <= 16 rows per step, as
 * 5 fused launches per step forward and 6 per step backward (instead of ~15 / ~20 separate kernels): every launch is
 * an M=16 MFMA contraction whose A panel is built in LDS by a fused prologue (split-K slab reduction, RMSNorm+SiLU,
 * straight-through sampler backward, RMSNorm backward) and whose epilogue fuses bias, the GRU gate fwd/bwd, the
 * unimix sampler and the reset masks. Recurrence-free work (action branch, embed half of obs_net_0, all weight
 * gradients) stays outside as (T*B)-row GEMMs. Weight operands are k-contiguous (row n of a [N][K] matrix);
 * the backward uses transposed copies the caller prepares once per update. Time-major (T,B,.) activations.
 * Requirements: B <= 16; D % G == 0; U, D/G, S*Kd multiples of 64; Kd in {16, 32, 64}. */
typedef struct sd_rssm_scan {
  int B, T, D, U, SK, Kd, G;
  int ks_d, ks_s;              /* K splits of the D-wide and SK-wide step GEMMs (slabs summed by the consumer) */
  float eps, unimix;
  uint64_t seed;
  const uint64_t* seed_ptr;    /* optional device seed offset (graph replay) */
  int stream_id;
  long group_offset;           /* global categorical index of row 0 (data-parallel row offset * S) */
  /* parameters */
  const float *W0, *b0, *n0;   /* _dyn_in0: (U,D) (U) (U) */
  const float *W1, *b1, *n1;   /* _dyn_in1: (U,SK) */
  const float *Wh, *bh, *nh;   /* _dyn_hid: (G, D/G, D/G+3U) (D) (D) */
  const float *Wg, *bg;        /* _dyn_gru: (G, 3D/G, D/G) (3D) */
  const float *WoD, *no;       /* obs_net_0 weight[:, :D] as a contiguous (U,D); obs_net_n_0 (U) */
  const float *Wl, *bl;        /* obs_net_logit: (SK,U) (SK) */
  const float *W0T, *W1T, *WshT, *WbdT, *WgT, *WoDT, *WlT;  /* backward: (D,U) (SK,U) (3U,D) (G,Dg,Dg) (G,Dg,3Dg) (D,U) (U,SK) */
  /* inputs */
  const unsigned char* reset;  /* (T,B), or (B,T) with reset_bm */
  const float *stoch0, *deter0;/* (B,SK) (B,D) */
  const float *x2, *eproj;     /* (T,B,U): action branch output; embed half of obs_net_0 + bias */
  /* saved activations (written by fwd, read by bwd) */
  float *s_in, *h_in, *x0p, *x1p, *r0, *r1, *xcat, *hp, *hh, *rh, *gates, *deter, *op, *oo, *ro, *logit, *stoch;
  /* backward */
  const float *d_stoch, *d_deter, *d_logit;  /* (T,B,SK) (T,B,D) (T,B,SK) incoming grads (bm_grads: (B,T,.)); each
                                                may be NULL */
  float* dl;                       /* out (T,B,SK): total d logit (incl. the straight-through sample gradient) */
  float *d_o, *d_op, *d_gates, *d_hh, *d_hp, *d_xcat, *d_x0p, *d_x1p;  /* (T,B,.) */
  float* work;                     /* >= sd_rssm_scan_work_floats(d) floats */
  /* optional forward layout (0 / NULL: the layouts above) */
  int bm_inputs;                   /* x2 / eproj batch-major (B,T,U), computed on the caller's batch-major rows */
  long ld_wod;                     /* row stride of WoD: the full obs_net_0 weight (U, D+E) read in place; 0 = D */
  float *post_stoch, *post_deter, *post_logit;  /* (B,T,.) batch-major copies of stoch / deter / logit (RSSM.observe's
                                                   outputs, rssm.py:140-156); stoch may then be NULL */
  /* optional backward layout: bm_grads = d_stoch / d_deter / d_logit batch-major (B,T,.), plus second summands
     d_stoch2 / d_deter2 (batch-major rows b*T + t with row stride ld_g2, e.g. the two halves of a (B,T,SK+D) feat
     gradient; each may be NULL): the posterior gradient d_stoch + d_stoch2 is formed where it is read */
  int bm_grads;
  const float *d_stoch2, *d_deter2;
  long ld_g2;
  /* rows per workgroup tile (1..16; 0 = 16): every step kernel runs ceil(B / row_tile) row tiles side by side in its
     grid (rows are independent sequences, rssm.py:146-151), so B > 16 is one scan and B = 16 with row_tile 8 uses
     twice the workgroups */
  int row_tile;
  /* measurement aid (a build with -DSD_SCAN_TRACE only; NULL otherwise): per launch slot and workgroup 4 timestamps
     (s_memrealtime, 100 MHz): entry, operands staged, contraction reduced, exit. Slot = t * 8 + phase (forward) or
     (T + t) * 8 + phase (backward); trace_slot is set per launch by the library */
  uint64_t* trace;
  int trace_slot;
  int reset_bm; /* 1: reset is (B, T) batch-major (the replay batch's is_first, read in place); 0: (T, B) */
  float* d_op_bm; /* optional backward output: a batch-major (B, T, U) copy of d_op (the embed gradient's operand) */
  float* d_x2_bm; /* optional backward output: a batch-major (B, T, U) copy of d_xcat's x2 block (action branch) */
} sd_rssm_scan;
int sd_rssm_scan_work_floats(const sd_rssm_scan* d);
int sd_rssm_scan_fwd(const sd_rssm_scan* d, sd_stream stream);
int sd_rssm_scan_bwd(const sd_rssm_scan* d, sd_stream stream);
/* Measurement aid (bench.py): one launch of forward step t's phase `which` as sd_rssm_scan_fwd issues it, after a run
 * on the same descriptor: 0 = x1p slab (k_slab), 1 = _dyn_hid (k_hid), 2 = _dyn_gru + GRU (k_gate), 3 = obs_net_0 deter
 * half + next _dyn_in0 (k_slab), 4 = obs_net logits + sampler (k_logit). Only t = T - 1 rewrites the values the run
 * wrote. */
int sd_rssm_scan_step_kernel(const sd_rssm_scan* d, int which, int t, sd_stream stream);

/* ---------------------------------------------------------------- fused imagination (Dreamer._imagine)
 * Dreamer._imagine (dreamer.py:673-692) over N start states for H1 actor steps: per step the actor MLP
 * (networks.py:313-377) + action sample (bounded normal / one-hot, distributions.py:217-222 / 16-33), then
 * RSSM.img_step (rssm.py:180-187: Deter.forward + prior logits + one-hot sample) — 9 launches per step. Every launch
 * is a row-tiled MFMA contraction whose A loader applies the previous layer's RMSNorm+SiLU on the fly (row rstd from
 * per-tile partial sums written by the producer's epilogue) and whose epilogue fuses bias, the GRU gate, the
 * samplers and the action branch (action_norm -> _dyn_in2 -> RMSNorm -> SiLU). Requirements: N % 64 == 0,
 * U == 256, D/G in {256, 512}, S*Kd % 64 == 0, Kd in {16, 32}, 2A <= 32 (A <= 16 discrete), 1..4 actor layers,
 * 1..4 img layers. feats (H1, N, S*Kd + D): row block t = 0 holds the start state on entry. */
typedef struct sd_imagine {
  int N, H1, D, U, SK, Kd, G, A, act_discrete, actor_layers, img_layers;
  float eps, unimix, act_unimix, min_std, max_std;
  uint64_t seed;
  const uint64_t* seed_ptr;
  int stream_img, stream_act;
  long row_offset;
  const float* Wa[4]; const float* ba[4]; const float* na[4];  /* actor layer i: (U, in_i) (U) (U) */
  const float *Wao, *bao;                  /* actor output: (2A or A, U) rows */
  const float *W0, *b0, *n0, *W1, *b1, *n1, *W2, *b2, *n2;       /* _dyn_in0/1/2 */
  const float *Wh, *bh, *nh, *Wg, *bg;                           /* _dyn_hid (G,Dg,Dg+3U), _dyn_gru (G,3Dg,Dg) */
  const float* Wi[4]; const float* bi[4]; const float* ni[4];    /* img_net layer i */
  const float *Wl, *bl;                                          /* img_net_logit (SK, U) */
  float* feats;
  float* actions;                                                /* (H1, N, A) */
  float* work;
  int t_begin, t_end; /* run steps [t_begin, t_end) (t_end <= 0: H1); chunks share `work` and run in order (the
                         t_begin == 0 chunk also writes the pre-split images of _dyn_hid / _dyn_gru into `work`) */
  float* actor_h0;    /* optional (H1, N, U): actor layer 0's pre-norm output of every step, feat . Wa0^T + ba0 in
                         fp32 (null: kept in `work` only); the policy loss's actor forward starts from it */
  const float* noise_img; /* optional (H1 - 1, N, SK): the prior samples' Gumbel noise, drawn ahead by
                             sd_imagine_noise (null: drawn inside the sampler); the same values either way */
  const float* noise_act; /* optional (H1, N, A): the action samples' noise (N(0,1) for a bounded-normal actor, Gumbel
                             for one-hot; stream stream_act, step t), drawn ahead by sd_imagine_noise */
  uint64_t* trace;        /* measurement aid, -DSD_SCAN_TRACE builds only (NULL otherwise): per launch slot
                             (t * 16 + launch of the step) and workgroup, entry / staged / contracted / exit timestamps */
  int prepped;            /* 1: sd_imagine_prep already wrote the weight images into `work` (the t_begin == 0 chunk
                             skips them) */
} sd_imagine;
int sd_imagine_work_floats(const sd_imagine* d);
int sd_imagine_run(const sd_imagine* d, sd_stream stream);
/* The weight-only part of the t_begin == 0 chunk — the pre-split bf16 images of _dyn_hid, _dyn_gru, img_net_0,
 * _dyn_in0 and actor layer 0's deter columns, the transposed one-hot weights — into `work`, ahead of the run (e.g. on
 * another stream beside the work that produces the start state); the run then sets `prepped`. */
int sd_imagine_prep(const sd_imagine* d, sd_stream stream);
/* noise (H1 - 1, N, SK) = the Gumbel noise of every imagined prior sample (Philox stream d->stream_img, step t, element
 * (row + row_offset) * SK + k; the effective seed read on the device as sd_imagine_run reads it), and when noise_act
 * is non-null (H1, N, A) the action samples' noise (stream d->stream_act, element (row + row_offset) * A + j): one
 * full-chip launch instead of the per-step sampler epilogues computing them (the f64 transforms leave the chain). */
int sd_imagine_noise(const sd_imagine* d, float* noise, float* noise_act, sd_stream stream);
/* Measurement aid (bench.py roofline): one launch of step t's largest contractions exactly as sd_imagine_run issues
 * them, after a run on the same descriptor/workspace: which = 0: img_net_0 + _dyn_in0 + actor layer 0's deter part
 * (three (N, D) x (D, U) GEMMs, k_lin), 1: _dyn_hid (k_hid), 2: _dyn_gru + GRU (k_gate). 0 <= t < H1 - 1. Launches 0
 * and 1 rewrite workspace values only; launch 2 reads the workspace's last _dyn_hid output and writes feats(t + 1)'s
 * deter, so only t = H1 - 2 reproduces the run's values (other t overwrite the trajectory: time it, keep no output). */
int sd_imagine_step_kernel(const sd_imagine* d, int which, int t, sd_stream stream);

/* InfoNCE representation loss (dreamer.py:533-542): cross_entropy(logits - rowmax(logits), arange) on an (n, ncol)
 * row-major logits block (ld floats between rows), row r labelled with column r + label_off (data parallel: local
 * rows against the gathered x2 of every rank). fwd writes per-row losses, the row log-sum-exp (saved for bwd) and the
 * mean loss (1 float); bwd writes dlogits (n, ncol) = g[0] * scale * (softmax - onehot), g a device scalar. */
int sd_infonce_fwd(const float* logits, long ld, int n, int ncol, long label_off, float* row_loss, float* lse,
                   float* loss, sd_stream stream);
int sd_infonce_bwd(const float* logits, long ld, int n, int ncol, long label_off, const float* lse, const float* g,
                   float scale, float* dlogits, sd_stream stream);

/* Replay slices (utils/buffer.py:27-53): storage keys laid out (cap, E, row_bytes) in HBM. Slice b starts at
 * (t0, e) = starts[2 * pick[b]], starts[2 * pick[b] + 1]; key k moves steps j < steps of time (t0 + shift + j) % cap
 * between storage and batch (B, steps, row_bytes): gather (scatter = 0; also writes the data rows' indices
 * t_idx / e_idx (B, L) when non-null, time = (t0 + 1 + j) % cap), or the latent write-back (scatter = 1). One launch
 * for every key. */
#define SD_MAX_SLICE_KEYS 16
typedef struct sd_slice_key {
  void* storage;
  void* batch;
  long row_bytes;
  int steps, shift;
} sd_slice_key;
typedef struct sd_slice_keys {
  sd_slice_key k[SD_MAX_SLICE_KEYS];
  int n;
} sd_slice_keys;
/* Replay slice picks (utils/buffer.py:27-42's random slice choice): pick[b] = uniform integer in [0, nstarts) from the
 * counter-based Philox stream (seed, stream 8, step = draw, index b) — the buffer's sampling without a host RNG or a
 * torch generator kernel; `draw` counts the buffer's sample calls. */
int sd_replay_pick(uint64_t seed, uint32_t draw, long nstarts, int B, int64_t* pick, sd_stream stream);
int sd_replay_slices(const sd_slice_keys* keys, const int64_t* starts, const int64_t* pick, int B, int L, long cap,
                     int E, int64_t* t_idx, int64_t* e_idx, int scatter, sd_stream stream);

/* r2dreamer augmentation (dreamer.py:716-729,845-880): (B*T, H, W, C) f32 images replicate-padded by `pad` and
 * shifted by Philox integer shifts in [0, 2 pad] (stream 6, per slice row if same_across_time else per image);
 * bilinear = the reference's aug.bilinear: 0 = grid_sample nearest (the exact integer gather), 1 = grid_sample
 * bilinear's f32 arithmetic (neighbour weights of float-rounding size, bit-exact with torch's CPU kernel). */
int sd_random_translate(const float* in, float* out, int B, int T, int H, int W, int C, int pad, uint64_t seed,
                        const uint64_t* seed_ptr, long row_offset, int same_across_time, int bilinear,
                        sd_stream stream);

/* Profiling aid: store the device wall clock (constant rate, sd_wall_clock_khz) into buf[idx] when `stream` reaches
 * this point; capturable into a HIP graph. Not part of the reference interface. */
int sd_mark(uint64_t* buf, int idx, sd_stream stream);
int sd_wall_clock_khz(int device);

#ifdef __cplusplus
}
#endif
#endif
