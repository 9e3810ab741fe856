// Channels-last (NHWC) convolution as implicit GEMM on the shared MFMA core, plus the fused pooling/norm epilogue
// kernels of the conv encoder/decoder.
//
// Reference: Conv2dSamePad (networks.py:59-85; stride 1, TF-SAME padding), ConvEncoder layers
// [conv -> MaxPool2d(2) -> RMSNorm2D -> SiLU] (networks.py:192-234), ConvDecoder layers
// [Upsample(2, nearest) -> conv -> RMSNorm2D -> SiLU] (networks.py:237-310).
// Layout: activations NHWC (the reference image is already (B,T,H,W,C); RMSNorm2D normalises channels, which
// is a contiguous row in NHWC). Weights are kept as (Co, kh, kw, Ci) so W is a K-contiguous GEMM operand.
//   fwd:        out[m=(n,y,x)][co]      = sum_k im2col(m, k=(ky,kx,ci)) W[co][k] (+ bias)
//   bwd-data:   the same kernel on dOut with the flipped/transposed weight Wf[ci][ky][kx][co], pad' = k-1-pad
//   bwd-weight: dW[co][k]  = sum_m dOut[m][co] im2col(m, k)   (+ a ones column -> d bias), split-K over pixels
// `ups = 1` reads the input through a nearest 2x upsample (decoder) without materialising it.
#include "gemm_core.h"
#include "sdhip.h"

extern "C" int sd_colsum(const float* in, float* out, int R, int N, long ld, int accumulate, sd_stream s);

namespace {
using namespace sdg;

struct Geom {
  const float* in;
  int Nb, Hs, Ws, C;  // stored input
  int Hg, Wg;         // conv grid (= Hs<<ups, Ws<<ups)
  int kh, kw, pad, ups;
};

SD_DEV bool tap(const Geom& G, int n, int y, int x, int k, long& off) {
  const int t = k / G.C, c = k - t * G.C;
  const int ky = t / G.kw, kx = t - ky * G.kw;
  const int yy = y + ky - G.pad, xx = x + kx - G.pad;
  if (yy < 0 || yy >= G.Hg || xx < 0 || xx >= G.Wg) return false;
  off = (((long)n * G.Hs + (yy >> G.ups)) * G.Ws + (xx >> G.ups)) * G.C + c;
  return true;
}

// A operand of fwd / bwd-data: rows = output pixels, k = (ky, kx, ci) contiguous in ci.
template <int ROWS, bool VEC>
struct Im2colRows {
  static constexpr int NV = ROWS * BK / 4 / 256 > 0 ? ROWS * BK / 4 / 256 : 1;
  Geom G;
  int pn[NV], py[NV], px[NV];
  f32x4 r[NV];
  TileLoader<ROWS, true, false> st;  // only for store()
  SD_DEV Im2colRows(const Geom& g, int M, int row0) : G(g) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + v * 256;
      const int m = row0 + i / (BK / 4);
      pn[v] = -1;
      if (i < ROWS * BK / 4 && m < M) {
        const int hw = G.Hg * G.Wg;
        pn[v] = m / hw;
        const int rem = m - pn[v] * hw;
        py[v] = rem / G.Wg;
        px[v] = rem - py[v] * G.Wg;
      }
    }
  }
  SD_DEV void load(int k0, int kend) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + v * 256;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      const int gk = k0 + 4 * (i % (BK / 4));
      if (pn[v] >= 0) {
        if (VEC) {  // C % 16 == 0: the 4 k's share one (ky, kx)
          long off;
          if (gk < kend && tap(G, pn[v], py[v], px[v], gk, off)) x = *reinterpret_cast<const f32x4*>(G.in + off);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            long off;
            if (gk + j < kend && tap(G, pn[v], py[v], px[v], gk + j, off)) x[j] = G.in[off];
          }
        }
      }
      st.r[v] = x;
    }
  }
  SD_DEV void store(float* lds) const { st.store(lds); }
};

// B operand of bwd-weight: rows = j = (ky, kx, ci) (+ one ones-row at j == J for the bias), k = pixel.
template <int ROWS, bool VEC>
struct Im2colCols {
  static constexpr int NV = ROWS * BK / 4 / 256 > 0 ? ROWS * BK / 4 / 256 : 1;
  Geom G;
  int J, row0;
  TileLoader<ROWS, false, false> st;
  SD_DEV Im2colCols(const Geom& g, int J_, int row0_) : G(g), J(J_), row0(row0_) {}
  SD_DEV void load(int k0, int kend) {
    const int hw = G.Hg * G.Wg;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + v * 256;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      const int m = k0 + i % BK;
      const int j0 = row0 + 4 * (i / BK);
      if (i < ROWS * BK / 4 && m < kend) {
        const int n = m / hw, rem = m - n * hw;
        const int y = rem / G.Wg, xq = rem - y * G.Wg;
        if (VEC && j0 + 3 < J) {
          long off;
          if (tap(G, n, y, xq, j0, off)) x = *reinterpret_cast<const f32x4*>(G.in + off);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int jj = j0 + j;
            long off;
            if (jj < J) {
              if (tap(G, n, y, xq, jj, off)) x[j] = G.in[off];
            } else if (jj == J) {
              x[j] = 1.f;
            }
          }
        }
      }
      st.r[v] = x;
    }
  }
  SD_DEV void store(float* lds) const { st.store(lds); }
};

template <int BM, int BN, int WM, int WN, bool VA, bool VB>
__global__ __launch_bounds__(256) void conv_fwd_kernel(GemmArgs g, Geom G) {
  const int bn0 = blockIdx.x * BN, bm0 = blockIdx.y * BM;
  Im2colRows<BM, VA> la(G, g.M, bm0);
  DenseOperand<BN, true, VB> lb(g.B, g.ldb, g.N, bn0);
  gemm_block<BM, BN, WM, WN>(g, la, lb, bm0, bn0, 0, 0, 0, g.K);
}

template <int BM, int BN, int WM, int WN, bool VA, bool VB>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(GemmArgs g, Geom G, int J) {
  const int bn0 = blockIdx.x * BN, bm0 = blockIdx.y * BM;
  const int split = blockIdx.z;
  const int kbeg = split * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  DenseOperand<BM, false, VA> la(g.A, g.lda, g.M, bm0);
  Im2colCols<BN, VB> lb(G, J, bn0);
  gemm_block<BM, BN, WM, WN>(g, la, lb, bm0, bn0, 0, split, kbeg, kend);
}

// ---------------------------------------------------------------- pooling / norm epilogues
// y = silu(rms(maxpool2(x))) per output pixel (team of T lanes, VPT channels each); keeps pooled + argmax.
template <int T, int VPT>
__global__ void pool_rms_fwd(const float* __restrict__ x, const float* __restrict__ w, float* __restrict__ pooled,
                             uint8_t* __restrict__ amax, float* __restrict__ y, float* __restrict__ rstd, int Nb, int H,
                             int W, int C, float eps, int nchw_flat) {
  const int Ho = H / 2, Wo = W / 2;
  const long P = (long)Nb * Ho * Wo;
  const long pix = ((long)blockIdx.x * blockDim.x + threadIdx.x) / T;
  const int t = threadIdx.x % T;
  if (pix >= P) return;
  const int n = (int)(pix / (Ho * Wo));
  const int rem = (int)(pix % (Ho * Wo));
  const int yo = rem / Wo, xo = rem % Wo;
  float v[VPT];
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int c = t + j * T;
    v[j] = 0.f;
    if (c < C) {
      float best = -INFINITY;
      int bi = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int yy = 2 * yo + (q >> 1), xx = 2 * xo + (q & 1);
        const float val = x[(((long)n * H + yy) * W + xx) * C + c];
        if (val > best || isnan(val)) { best = val; bi = q; }
      }
      v[j] = best;
      pooled[pix * C + c] = best;
      amax[pix * C + c] = (uint8_t)bi;
    }
    ss += v[j] * v[j];
  }
  ss = group_sum<T>(ss);
  const float r = rsqrtf(ss / (float)C + eps);
  if (t == 0) rstd[pix] = r;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int c = t + j * T;
    if (c < C) {
      const float z = v[j] * r * w[c];
      const long o = nchw_flat ? (long)n * C * Ho * Wo + (long)c * Ho * Wo + rem : pix * C + c;
      y[o] = siluf_(z);
    }
  }
}

template <int T, int VPT>
__global__ void pool_rms_bwd(const float* __restrict__ pooled, const uint8_t* __restrict__ amax,
                             const float* __restrict__ w, const float* __restrict__ rstd, const float* __restrict__ dy,
                             float* __restrict__ dx, float* __restrict__ dw_part, int Nb, int H, int W, int C,
                             int nchw_flat) {
  const int Ho = H / 2, Wo = W / 2;
  const long P = (long)Nb * Ho * Wo;
  const int t = threadIdx.x % T;
  const int team = threadIdx.x / T;
  constexpr int TPB = 256 / T;
  float dwacc[VPT];
#pragma unroll
  for (int j = 0; j < VPT; ++j) dwacc[j] = 0.f;
  for (long pix = (long)blockIdx.x * TPB + team; pix < P; pix += (long)gridDim.x * TPB) {
    const int n = (int)(pix / (Ho * Wo));
    const int rem = (int)(pix % (Ho * Wo));
    const int yo = rem / Wo, xo = rem % Wo;
    const float r = rstd[pix];
    float xh[VPT], g[VPT];
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int c = t + j * T;
      xh[j] = g[j] = 0.f;
      if (c < C) {
        const float xv = pooled[pix * C + c] * r;
        const float wv = w[c];
        const float z = xv * wv;
        const float s = sigmoidf_(z);
        const long o = nchw_flat ? (long)n * C * Ho * Wo + (long)c * Ho * Wo + rem : pix * C + c;
        const float dz = dy[o] * s * (1.f + z * (1.f - s));
        xh[j] = xv;
        g[j] = dz * wv;
        dwacc[j] += dz * xv;
        dot += g[j] * xv;
      }
    }
    dot = group_sum<T>(dot) / (float)C;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int c = t + j * T;
      if (c < C) {
        const float dp = r * (g[j] - xh[j] * dot);
        const int bi = amax[pix * C + c];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int yy = 2 * yo + (q >> 1), xx = 2 * xo + (q & 1);
          dx[(((long)n * H + yy) * W + xx) * C + c] = q == bi ? dp : 0.f;
        }
      }
    }
  }
  // per-block dw partials
  __shared__ float wp[TPB * T * VPT];
#pragma unroll
  for (int j = 0; j < VPT; ++j) wp[(team * VPT + j) * T + t] = dwacc[j];
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    const int j = c / T, tt = c % T;
    float s = 0.f;
    for (int tm = 0; tm < TPB; ++tm) s += wp[(tm * VPT + j) * T + tt];
    dw_part[(long)blockIdx.x * C + c] = s;
  }
}

// Wf[ci][ky][kx][co] = W[co][kh-1-ky][kw-1-kx][ci]
__global__ void flip_weight(const float* __restrict__ w, float* __restrict__ wf, int Co, int kh, int kw, int Ci) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)Co * kh * kw * Ci;
  if (t >= total) return;
  const int co = (int)(t % Co);
  long r = t / Co;
  const int kx = (int)(r % kw);
  r /= kw;
  const int ky = (int)(r % kh);
  const int ci = (int)(r / kh);
  wf[t] = w[(((long)co * kh + (kh - 1 - ky)) * kw + (kw - 1 - kx)) * Ci + ci];
}

// dIn[n,Y,X,c] = sum_{dy,dx} dU[n,2Y+dy,2X+dx,c]   (backward of nearest 2x upsample)
__global__ void sumpool2(const float* __restrict__ du, float* __restrict__ din, int Nb, int H, int W, int C) {
  const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)Nb * H * W * C;
  if (t >= total) return;
  const int c = (int)(t % C);
  long r = t / C;
  const int X = (int)(r % W);
  r /= W;
  const int Y = (int)(r % H);
  const int n = (int)(r / H);
  const int W2 = 2 * W, H2 = 2 * H;
  const float* b = du + (((long)n * H2 + 2 * Y) * W2 + 2 * X) * C + c;
  din[t] = (b[0] + b[C]) + (b[(long)W2 * C] + b[(long)W2 * C + C]);
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

template <int BM, int BN, int WM, int WN>
void fwd_tile(GemmArgs& g, Geom& G, bool va, bool vb, hipStream_t s) {
  dim3 grid(sd_cdiv(g.N, BN), sd_cdiv(g.M, BM), 1);
  if (va && vb) conv_fwd_kernel<BM, BN, WM, WN, true, true><<<grid, 256, 0, s>>>(g, G);
  else if (vb) conv_fwd_kernel<BM, BN, WM, WN, false, true><<<grid, 256, 0, s>>>(g, G);
  else conv_fwd_kernel<BM, BN, WM, WN, false, false><<<grid, 256, 0, s>>>(g, G);
}

template <int BM, int BN, int WM, int WN>
void wgrad_tile(GemmArgs& g, Geom& G, int J, bool va, bool vb, hipStream_t s) {
  dim3 grid(sd_cdiv(g.N, BN), sd_cdiv(g.M, BM), g.ksplit);
  if (va && vb) conv_wgrad_kernel<BM, BN, WM, WN, true, true><<<grid, 256, 0, s>>>(g, G, J);
  else if (va) conv_wgrad_kernel<BM, BN, WM, WN, true, false><<<grid, 256, 0, s>>>(g, G, J);
  else if (vb) conv_wgrad_kernel<BM, BN, WM, WN, false, true><<<grid, 256, 0, s>>>(g, G, J);
  else conv_wgrad_kernel<BM, BN, WM, WN, false, false><<<grid, 256, 0, s>>>(g, G, J);
}

int vpt_for(int C, int T) { int v = (C + T - 1) / T; return v <= 1 ? 1 : v <= 2 ? 2 : v <= 4 ? 4 : 8; }

}  // namespace

// out (Nb, Hg, Wg, Co) = conv_same(in (Nb, Hs, Ws, Ci) [upsampled x2 if ups], w (Co, kh, kw, Ci)) + bias
extern "C" int sd_conv2d_fwd(const float* in, const float* w, const float* bias, float* out, int Nb, int Hs, int Ws,
                             int Ci, int Co, int kh, int kw, int pad, int ups, sd_stream stream_) {
  hipStream_t s = (hipStream_t)stream_;
  if (Nb <= 0) return SD_OK;
  Geom G{in, Nb, Hs, Ws, Ci, Hs << ups, Ws << ups, kh, kw, pad, ups};
  GemmArgs g{};
  g.B = w; g.C = out; g.bias = bias; g.ldb = (long)kh * kw * Ci; g.ldc = Co;
  g.M = Nb * G.Hg * G.Wg; g.N = Co; g.K = kh * kw * Ci; g.batch = 1; g.ksplit = 1; g.kchunk = g.K;
  g.alpha = 1.f; g.beta = 0.f;
  const bool vb = (((long)kh * kw * Ci) % 4 == 0) && al16(w);
  const bool va = (Ci % 16 == 0) && al16(in) && vb;
  if (Co <= 32) fwd_tile<128, 32, 32, 32>(g, G, va, vb, s);
  else fwd_tile<128, 64, 64, 32>(g, G, va, vb, s);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

// dw_db (Co, kh*kw*Ci + 1) = [dW | d bias] = sum over pixels of dout (Nb,Hg,Wg,Co) x im2col(in)
extern "C" int sd_conv2d_wgrad(const float* in, const float* dout, float* dw_db, float* workspace, long ws_floats,
                               int ksplit, int Nb, int Hs, int Ws, int Ci, int Co, int kh, int kw, int pad, int ups,
                               sd_stream stream_) {
  hipStream_t s = (hipStream_t)stream_;
  if (Nb <= 0) return SD_OK;
  Geom G{in, Nb, Hs, Ws, Ci, Hs << ups, Ws << ups, kh, kw, pad, ups};
  const int J = kh * kw * Ci;
  GemmArgs g{};
  g.A = dout; g.lda = Co; g.C = dw_db; g.ldc = J + 1; g.ws = workspace;
  g.M = Co; g.N = J + 1; g.K = Nb * G.Hg * G.Wg; g.batch = 1;
  int ks = ksplit < 1 ? 1 : ksplit;
  if (ks > 1 && (!workspace || ws_floats < (long)ks * g.M * g.N)) return SD_EARG;
  g.ksplit = ks;
  long kc = ((long)g.K + ks - 1) / ks;
  g.kchunk = (int)((kc + BK - 1) / BK * BK);
  g.alpha = 1.f; g.beta = 0.f;
  const bool va = al16(dout) && Co % 4 == 0;
  const bool vb = (Ci % 4 == 0) && al16(in);
  if (Co <= 32) wgrad_tile<32, 128, 32, 32>(g, G, J, va, vb, s);
  else wgrad_tile<64, 64, 32, 32>(g, G, J, va, vb, s);
  SD_LAUNCH_CHECK();
  if (ks > 1) {
    long total = (long)g.M * g.N;
    int blocks = (int)((total + 255) / 256);
    gemm_reduce_kernel<<<blocks, 256, 0, s>>>(g);
    SD_LAUNCH_CHECK();
  }
  return SD_OK;
}

extern "C" int sd_conv_flip_weight(const float* w, float* wf, int Co, int kh, int kw, int Ci, sd_stream s) {
  const long total = (long)Co * kh * kw * Ci;
  flip_weight<<<(int)((total + 255) / 256), 256, 0, (hipStream_t)s>>>(w, wf, Co, kh, kw, Ci);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_sumpool2(const float* du, float* din, int Nb, int H, int W, int C, sd_stream s) {
  const long total = (long)Nb * H * W * C;
  if (total <= 0) return SD_OK;
  sumpool2<<<(int)((total + 255) / 256), 256, 0, (hipStream_t)s>>>(du, din, Nb, H, W, C);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

#define SD_POOL_SWITCH(KERNEL, GRID, ...)                                                  \
  switch (vpt_for(C, 16)) {                                                                 \
    case 1: KERNEL<16, 1><<<GRID, 256, 0, s>>>(__VA_ARGS__); break;                          \
    case 2: KERNEL<16, 2><<<GRID, 256, 0, s>>>(__VA_ARGS__); break;                          \
    case 4: KERNEL<16, 4><<<GRID, 256, 0, s>>>(__VA_ARGS__); break;                          \
    default: KERNEL<16, 8><<<GRID, 256, 0, s>>>(__VA_ARGS__); break;                         \
  }

extern "C" int sd_pool_rms_fwd(const float* x, const float* w, float* pooled, uint8_t* amax, float* y, float* rstd,
                               int Nb, int H, int W, int C, float eps, int nchw_flat, sd_stream stream_) {
  hipStream_t s = (hipStream_t)stream_;
  if (C > 128) return SD_ESHAPE;
  const long P = (long)Nb * (H / 2) * (W / 2);
  if (P <= 0) return SD_OK;
  const int grid = (int)((P * 16 + 255) / 256);
  SD_POOL_SWITCH(pool_rms_fwd, grid, x, w, pooled, amax, y, rstd, Nb, H, W, C, eps, nchw_flat)
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_pool_rms_bwd_blocks(int Nb, int H, int W) {
  const long P = (long)Nb * (H / 2) * (W / 2);
  long b = (P + 15) / 16;
  return (int)(b < 2048 ? (b > 0 ? b : 1) : 2048);
}

extern "C" int sd_pool_rms_bwd(const float* pooled, const uint8_t* amax, const float* w, const float* rstd,
                               const float* dy, float* dx, float* dw, float* dw_partial, int Nb, int H, int W, int C,
                               int nchw_flat, int accumulate_dw, sd_stream stream_) {
  hipStream_t s = (hipStream_t)stream_;
  if (C > 128) return SD_ESHAPE;
  const int grid = sd_pool_rms_bwd_blocks(Nb, H, W);
  SD_POOL_SWITCH(pool_rms_bwd, grid, pooled, amax, w, rstd, dy, dx, dw_partial, Nb, H, W, C, nchw_flat)
  SD_LAUNCH_CHECK();
  return sd_colsum(dw_partial, dw, grid, C, C, accumulate_dw, stream_);
}
