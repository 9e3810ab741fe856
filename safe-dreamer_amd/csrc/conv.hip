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
#include <stdlib.h>

#include "gemm3_core.h"
#include "gemm6_core.h"
#include "gemm_core.h"
#include "sdhip.h"

extern "C" int sd_colsum(const float* in, float* out, int R, int N, long ld, int accumulate, sd_stream s);
extern "C" int sd_colsum_ws(const float* in, float* out, int R, int N, long ld, int accumulate, float* workspace,
                            sd_stream s);

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
  static constexpr int NV = (ROWS * BK / 4 + 255) / 256;
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
  static constexpr int NV = (ROWS * BK / 4 + 255) / 256;
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

// ---------------------------------------------------------------- tap-table loaders (C % 4 == 0, pow2 grid)
// The k -> (ky, kx, ci) decode of the implicit-GEMM A operand is table-driven: each workgroup writes one packed
// int per 4 k's into LDS (ci | ky << 16 | kx << 24) before its first tile, so a float4 of the im2col row costs an
// LDS read, two compares and an address instead of two runtime integer divisions.
constexpr int MAX_TAPQ = 512;  // K <= 2048
constexpr int NW_D = 8;        // waves of the direct bwd-weight kernel

SD_DEV void build_taps(int* tab, const Geom& G, int K) {
  for (int kq = threadIdx.x; kq < K / 4; kq += blockDim.x) {
    const int k = 4 * kq, t = k / G.C, c = k - t * G.C;
    const int ky = t / G.kw, kx = t - ky * G.kw;
    tab[kq] = c | (ky << 16) | (kx << 24);
  }
  __syncthreads();
}

template <int ROWS>
struct Im2colRowsT {
  static constexpr int NV = (ROWS * BK / 4 + 255) / 256;
  Geom G;
  const int* tab;
  int py[NV], px[NV];
  long pbase[NV];  // n * Hs (row index base) or -1
  TileLoader<ROWS, true, false> st;
  SD_DEV Im2colRowsT(const Geom& g, const int* tab_, int M, int row0, int lw, int lhw) : G(g), tab(tab_) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + v * 256;
      const int m = row0 + i / (BK / 4);
      pbase[v] = -1;
      if (i < ROWS * BK / 4 && m < M) {
        const int n = m >> lhw, rem = m & ((1 << lhw) - 1);
        py[v] = rem >> lw;
        px[v] = rem & ((1 << lw) - 1);
        pbase[v] = (long)n * G.Hs;
      }
    }
  }
  SD_DEV void load(int k0, int kend) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + v * 256;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      const int gk = k0 + 4 * (i % (BK / 4));
      if (pbase[v] >= 0 && gk < kend) {
        const int e = tab[gk >> 2];
        const int yy = py[v] + ((e >> 16) & 0xff) - G.pad, xx = px[v] + (e >> 24) - G.pad;
        if (yy >= 0 && yy < G.Hg && xx >= 0 && xx < G.Wg)
          x = *reinterpret_cast<const f32x4*>(G.in + ((pbase[v] + (yy >> G.ups)) * G.Ws + (xx >> G.ups)) * G.C +
                                              (e & 0xffff));
      }
      st.r[v] = x;
    }
  }
  SD_DEV void store(float* lds) const { st.store(lds); }
};

// Branch-free variant of Im2colRowsT on buffer loads (out-of-image taps and the K tail read 0 through the
// descriptor's range check), for gemm16_mainloop_es. Input must be < 2 GiB (checked by the launcher).
template <int ROWS>
struct Im2colRowsB {
  static constexpr int NV = (ROWS * BK / 4 + 255) / 256;
  Geom G;
  const int* tab;
  sd_rsrc rs;
  int py[NV], px[NV], pb[NV];  // pb: n * Hs, or a large negative value for rows past M
  TileLoader<ROWS, true, false> st;
  SD_DEV Im2colRowsB(const Geom& g, const int* tab_, int M, int row0, int lw, int lhw) : G(g), tab(tab_) {
    rs = sd_make_rsrc(g.in, (long)g.Nb * g.Hs * g.Ws * g.C * 4);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + v * 256;
      const int m = row0 + i / (BK / 4);
      const int n = m >> lhw, rem = m & ((1 << lhw) - 1);
      py[v] = rem >> lw;
      px[v] = rem & ((1 << lw) - 1);
      pb[v] = (i < ROWS * BK / 4 && m < M) ? n * G.Hs : -(1 << 28);
    }
  }
  SD_DEV void load(int k0, int kend) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + v * 256;
      const int gk = k0 + 4 * (i % (BK / 4));
      const int e = tab[min(gk >> 2, MAX_TAPQ - 1)];
      const int yy = py[v] + ((e >> 16) & 0xff) - G.pad, xx = px[v] + (e >> 24) - G.pad;
      const bool ok = pb[v] >= 0 && gk < kend && (unsigned)yy < (unsigned)G.Hg && (unsigned)xx < (unsigned)G.Wg;
      const uint32_t off = (uint32_t)((((pb[v] + (yy >> G.ups)) * G.Ws + (xx >> G.ups)) * G.C + (e & 0xffff)) * 4);
      st.r[v] = sd_bload4(rs, ok ? off : SD_OOB);
    }
  }
  SD_DEV void store(float* lds) const { st.store(lds); }
};

// Branch-free dense operand, k contiguous, ROWS x BK tiles of a (nrows x K) matrix with K % 4 == 0 (buffer loads)
template <int ROWS>
struct DenseKCB {
  static constexpr int NV = (ROWS * BK / 4 + 255) / 256;
  sd_rsrc rs;
  long ld;
  int nrows, row0;
  TileLoader<ROWS, true, false> st;
  SD_DEV DenseKCB(const float* base, long ld_, int nrows_, int row0_) : ld(ld_), nrows(nrows_), row0(row0_) {
    rs = sd_make_rsrc(base, (long)nrows_ * ld_ * 4);
  }
  SD_DEV void load(int k0, int kend) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + v * 256;
      const int row = row0 + i / (BK / 4), gk = k0 + 4 * (i % (BK / 4));
      const bool ok = i < ROWS * BK / 4 && row < nrows && gk < kend;
      st.r[v] = sd_bload4(rs, ok ? (uint32_t)((row * ld + gk) * 4) : SD_OOB);
    }
  }
  SD_DEV void store(float* lds) const { st.store(lds); }
};

// bwd-weight B operand, k-major: rows j = (ky, kx, ci) fixed per thread (decoded once), k = pixel (pow2 grid:
// shifts). Consecutive lanes take consecutive 4-channel groups of one pixel -> coalesced 16-B loads.
template <int ROWS>
struct Im2colColsKM : KMajor<ROWS> {
  using KMajor<ROWS>::r;
  using KMajor<ROWS>::NV;
  Geom G;
  int J, lw, lhw;
  int jc[NV], jy[NV], jx[NV], j0v[NV];  // jc < 0: the group straddles J (scalar path incl. the ones column)
  SD_DEV Im2colColsKM(const Geom& g, int J_, int row0, int lw_, int lhw_) : G(g), J(J_), lw(lw_), lhw(lhw_) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + v * 256;
      const int j0 = row0 + 4 * this->rq(i);
      j0v[v] = j0;
      jc[v] = -1;
      jy[v] = jx[v] = 0;
      if (j0 + 3 < J) {
        const int t = j0 / G.C;
        jc[v] = j0 - t * G.C;
        jy[v] = t / G.kw - G.pad;
        jx[v] = t - (t / G.kw) * G.kw - G.pad;
      }
    }
  }
  SD_DEV void load(int k0, int kend) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + v * 256;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      const int m = k0 + this->kk(i);
      if (i < ROWS * BK / 4 && m < kend && j0v[v] <= J) {
        const int n = m >> lhw, rem = m & ((1 << lhw) - 1);
        const int y = rem >> lw, xq = rem & ((1 << lw) - 1);
        if (jc[v] >= 0) {
          const int yy = y + jy[v], xx = xq + jx[v];
          if (yy >= 0 && yy < G.Hg && xx >= 0 && xx < G.Wg)
            x = *reinterpret_cast<const f32x4*>(
                G.in + (((long)n * G.Hs + (yy >> G.ups)) * G.Ws + (xx >> G.ups)) * G.C + jc[v]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int jj = j0v[v] + j;
            long off;
            if (jj < J) {
              if (tap(G, n, y, xq, jj, off)) x[j] = G.in[off];
            } else if (jj == J) {
              x[j] = 1.f;
            }
          }
        }
      }
      r[v] = x;
    }
  }
};

// fwd / bwd-data: M = pixels, N = Co (tile = all output channels), 16x16x4 MFMA, 4 waves along M
template <int BN, bool ES>
__global__ __launch_bounds__(256) void conv_fwd16(GemmArgs g, Geom G, int lw, int lhw) {
  __shared__ int tab[MAX_TAPQ];
  build_taps(tab, G, g.K);
  constexpr int BM = 128;
  const int bm0 = blockIdx.x * BM;
  if constexpr (ES) {
    Im2colRowsB<BM> la(G, tab, g.M, bm0, lw, lhw);
    DenseKCB<BN> lb(g.B, g.ldb, g.N, 0);
    gemm_block16<BM, BN, 32, BN, true>(g, la, lb, bm0, 0, 0, 0, 0, g.K);
  } else {
    Im2colRowsT<BM> la(G, tab, g.M, bm0, lw, lhw);
    DenseOperand<BN, true, true> lb(g.B, g.ldb, g.N, 0);
    gemm_block16<BM, BN, 32, BN>(g, la, lb, bm0, 0, 0, 0, 0, g.K);
  }
}

// Stage epilogue shared by the fused forward kernels: the 128-pixel conv tile (+ bias) is staged in LDS at C, 2x2
// max-pooled (argmax kept for the backward), RMS-normalised over the BN channels (8 threads per pooled pixel) and
// SiLU'd; only the pooled outputs are written (pooled pre-norm values, argmax, rstd; y NHWC or NCHW-flat).
// pre (optional): the caller's registers holding this lane's bias values (BN / 16: column 16 j + l16) and norm
// weights (BN / 8: channel t8 + 8 k), loaded once per workgroup — in a kernel with loads in flight at the epilogue
// (a prefetched next patch) the per-tile loads here would each wait for them too (vmcnt counts in issue order).
template <int BN>
struct EpiPre {
  float bias[BN / 16];
  float nw[BN / 8];
};
template <int BN, int WM>
SD_DEV void pool_epilogue(const f32x4 (&acc)[WM / 16][BN / 16], float* C, const GemmArgs& g, const Geom& G, int lw,
                          int lhw, int bm0, const float* nw, float* pooled, uint8_t* amax, float* y, float* rstd,
                          float eps, int nchw_flat, const EpiPre<BN>* pre = nullptr) {
  constexpr int LDC = BN + 1;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, q = lane >> 4;
#pragma unroll
  for (int i = 0; i < WM / 16; ++i)
#pragma unroll
    for (int j = 0; j < BN / 16; ++j) {
      const int col = 16 * j + l16;
      const float bv = pre ? pre->bias[j] : g.bias ? g.bias[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) C[(wave * WM + 16 * i + 4 * q + r) * LDC + col] = acc[i][j][r] + bv;
    }
  __syncthreads();
  constexpr int NK = BN / 8;
  // WM / 32 passes of (threads / 8) pooled pixels x 8 threads (a wave's WM pixels hold WM / 4 pooled ones)
#pragma unroll
  for (int ps = 0; ps < WM / 32; ++ps) {
  const int tid = threadIdx.x, pp = (tid >> 3) + ps * (int)(blockDim.x >> 3), t8 = tid & 7;
  const int W = G.Wg, Wo = W >> 1, lwo = lw - 1;
  const int yo = pp >> lwo, xo = pp & (Wo - 1);
  const int l0 = (2 * yo) * W + 2 * xo;                     // local pixel of the window's top-left
  const int gp = bm0 + l0;                                    // global conv pixel
  const int n = gp >> lhw, rem = gp & ((1 << lhw) - 1), yy = rem >> lw, xx = rem & (W - 1);
  const int Ho = G.Hg >> 1;
  const long gpp = ((long)n * Ho + (yy >> 1)) * Wo + (xx >> 1);  // global pooled pixel
  const bool valid = gp < g.M;
  float v[NK];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c = t8 + 8 * k;
    float best = -INFINITY;
    int bi = 0;
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) {
      const float val = C[(l0 + (qd >> 1) * W + (qd & 1)) * LDC + c];
      if (val > best || isnan(val)) { best = val; bi = qd; }
    }
    v[k] = best;
    ss += best * best;
    if (valid) {
      pooled[gpp * BN + c] = best;
      amax[gpp * BN + c] = (uint8_t)bi;
    }
  }
  ss = group_sum<8>(ss);
  const float r = rsqrtf(ss / (float)BN + eps);
  if (valid && t8 == 0) rstd[gpp] = r;
  const long prem = gpp - (long)n * Ho * Wo;
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c = t8 + 8 * k;
    const float z = v[k] * r * (pre ? pre->nw[k] : nw[c]);
    const long o = nchw_flat ? (long)n * BN * Ho * Wo + (long)c * Ho * Wo + prem : gpp * BN + c;
    if (valid) y[o] = siluf_(z);
  }
  }
}


// ConvEncoder stage fused: conv (fwd16 main loop) -> MaxPool2d(2) -> RMSNorm2D -> SiLU (networks.py:201-216).
// A 128-pixel M tile holds whole 2x2 windows (128 % 2W == 0, image rows come in pairs), so the epilogue stages the
// conv tile in the main loop's LDS area, pools it, normalises over the Co channels (8 threads per pooled pixel) and
// writes only the pooled outputs (pooled pre-norm values, argmax, rstd for the backward; y NHWC or NCHW-flat).
template <int BN, bool ES>
__global__ __launch_bounds__(256) void conv_fwd16_pool(GemmArgs g, Geom G, int lw, int lhw, const float* nw,
                                                       float* pooled, uint8_t* amax, float* y, float* rstd, float eps,
                                                       int nchw_flat) {
  __shared__ int tab[MAX_TAPQ];
  build_taps(tab, G, g.K);
  constexpr int BM = 128, WM = 32;
  const int bm0 = blockIdx.x * BM;
  EpiPre<BN> pre;  // epilogue operands issued ahead of the main loop (no loads behind the epilogue's own stores)
#pragma unroll
  for (int j = 0; j < BN / 16; ++j) pre.bias[j] = g.bias ? g.bias[16 * j + (threadIdx.x & 15)] : 0.f;
#pragma unroll
  for (int k = 0; k < BN / 8; ++k) pre.nw[k] = nw[(threadIdx.x & 7) + 8 * k];
  f32x4 acc[WM / 16][BN / 16];
  if constexpr (ES) {
    Im2colRowsB<BM> la(G, tab, g.M, bm0, lw, lhw);
    DenseKCB<BN> lb(g.B, g.ldb, g.N, 0);
    gemm16_mainloop_es<BM, BN, WM, BN>(la, lb, 0, g.K, acc);
  } else {
    Im2colRowsT<BM> la(G, tab, g.M, bm0, lw, lhw);
    DenseOperand<BN, true, true> lb(g.B, g.ldb, g.N, 0);
    gemm16_mainloop<BM, BN, WM, BN>(la, lb, 0, g.K, acc);
  }
  __syncthreads();  // every wave is done reading the staging area
  float* C = sd_smem<gemm16_smem_floats<BM, BN>()>();
  static_assert(BM * (BN + 1) <= gemm16_smem_floats<BM, BN>(), "tile fits the staging area");
  pool_epilogue<BN, WM>(acc, C, g, G, lw, lhw, bm0, nw, pooled, amax, y, rstd, eps, nchw_flat, &pre);
}

// Direct ConvEncoder stage forward (stride 1, same padding, no upsample): the 128-pixel tile is R = 128 / W whole
// output rows of one image, so its receptive field is one (R + KS - 1) x (W + KS - 1) x CI input patch. The patch
// is staged in LDS once (pixel stride CI + 4 floats: conflict-free ds_read_b128 fragments) and every tap's A
// fragments are read from it at the tap's offset — the 25x im2col expansion is never re-read from L2. The weights
// stream through a double-buffered early-store B stage, one (tap, 32-channel) k tile per iteration; the epilogue
// (pool + RMSNorm + SiLU) is conv_fwd16_pool's, staged in the patch area. Wave w owns tile pixels 32w..32w+31
// (TM = 2) x all BN channels. A workgroup runs TPW vertically adjacent tiles (XCD-aware order: an XCD's workgroups
// cover a contiguous tile range, so the KS - 1 halo rows adjacent tiles share are L2 hits), loading the next tile's
// patch into registers under the current tile's MFMAs.
template <int BN, int CI, int LW, int KS, int TPW>
__global__ __launch_bounds__(256) void conv_fwd_direct_pool(GemmArgs g, Geom G, int lhw, const float* nw,
                                                            float* pooled, uint8_t* amax, float* y, float* rstd,
                                                            float eps, int nchw_flat) {
  constexpr int BM = 128, WM = 32, TM = WM / 16, TN = BN / 16, W = 1 << LW, R = BM / W;
  constexpr int PH = R + KS - 1, PW = W + KS - 1, CSI = CI + 4, PAD = KS / 2;
  constexpr int PATCH = PH * PW * CSI, SB = BN * LDS_ROW;
  constexpr int NQ = PH * PW * (CI / 4), NQT = (NQ + 255) / 256;
  constexpr int NK = KS * KS * (CI / BK);
  static_assert(CI % 32 == 0 && (CSI / 4) % 2 == 1, "32-channel k tiles, odd float4 pixel stride");
  static_assert(BM * (BN + 1) <= PATCH, "epilogue tile fits the patch area");
  float* smem = sd_smem<PATCH + 2 * SB>();
  float* patch = smem;
  float* bst = smem + PATCH;
  const int nwg = gridDim.x, ntiles = g.M / BM;
  const int wg = (nwg & 7) ? blockIdx.x : (blockIdx.x & 7) * (nwg >> 3) + (blockIdx.x >> 3);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, q = lane >> 4;
  const sd_rsrc rs = sd_make_rsrc(G.in, (long)G.Nb * G.Hs * G.Ws * CI * 4);
  f32x4 v[NQT];
  auto load_patch = [&](int tile) {  // zero outside the image (range-checked buffer loads)
    const int bm0 = tile * BM, n = bm0 >> lhw, y0 = (bm0 & ((1 << lhw) - 1)) >> LW;
#pragma unroll
    for (int u = 0; u < NQT; ++u) {
      const int i = threadIdx.x + 256 * u;
      const int pix = i / (CI / 4), c4 = i % (CI / 4);
      const int py = pix / PW, px = pix % PW;
      const int yy = y0 + py - PAD, xx = px - PAD;
      const bool ok = i < NQ && tile < ntiles && (unsigned)yy < (unsigned)G.Hs && (unsigned)xx < (unsigned)W;
      v[u] = sd_bload4(rs, ok ? (uint32_t)((((n * G.Hs + yy) * W + xx) * CI + 4 * c4) * 4) : SD_OOB);
    }
  };
  // fragment base of tile pixel p = 32w + 16i + l16 (row p >> LW, column p & (W - 1)) at tap (0, 0)
  int abase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int p = wave * WM + 16 * i + l16;
    abase[i] = ((p >> LW) * PW + (p & (W - 1))) * CSI + 8 * q;
  }
  DenseKCB<BN> lb(g.B, g.ldb, g.N, 0);
  load_patch(wg * TPW);
  for (int it = 0; it < TPW; ++it) {
    const int tile = wg * TPW + it;
    if (tile >= ntiles) break;  // uniform over the workgroup
    if (it > 0) __syncthreads();  // the previous tile's epilogue is done with the patch area
    lb.load(0, g.K);
#pragma unroll
    for (int u = 0; u < NQT; ++u) {
      const int i = threadIdx.x + 256 * u;
      if ((u + 1) * 256 <= NQ || i < NQ)
        *reinterpret_cast<f32x4*>(patch + (i / (CI / 4)) * CSI + 4 * (i % (CI / 4))) = v[u];
    }
    lb.store(bst);
    lb.load(BK, g.K);
    __syncthreads();
    if (it + 1 < TPW) load_patch(tile + 1);
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < NK; ++kt) {
      const float* cur = bst + (kt & 1) * SB;
      float* nxt = bst + ((kt & 1) ^ 1) * SB;
      const int tap = kt / (CI / BK), ci0 = (kt % (CI / BK)) * BK;
      const int toff = ((tap / KS) * PW + tap % KS) * CSI + ci0;
      float af[TM][8], bf[TN][8];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const float* pa = patch + abase[i] + toff;
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(pa), x1 = *reinterpret_cast<const f32x4*>(pa + 4);
#pragma unroll
        for (int s = 0; s < 4; ++s) { af[i][s] = x0[s]; af[i][4 + s] = x1[s]; }
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const float* pb = cur + (16 * j + l16) * LDS_ROW + 8 * q;
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(pb), x1 = *reinterpret_cast<const f32x4*>(pb + 4);
#pragma unroll
        for (int s = 0; s < 4; ++s) { bf[j][s] = x0[s]; bf[j][4 + s] = x1[s]; }
      }
      lb.store(nxt);
      lb.load((kt + 2 < NK ? kt + 2 : NK - 1) * BK, g.K);
#pragma unroll
      for (int s = 0; s < 8; ++s)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
      __syncthreads();
    }
    pool_epilogue<BN, WM>(acc, patch, g, G, LW, lhw, tile * BM, nw, pooled, amax, y, rstd, eps, nchw_flat);
  }
}

// conv_fwd_direct_pool on the fp32-accurate three-way split-bf16 path (gemm6_core.h: a = a0 + a1 + a2, six
// v_mfma_f32_16x16x32_bf16 per 32-deep k chunk, smallest terms first, <= 2^-26 |ab| dropped per product; 2.67x the
// f32 MFMA rate). The 128-pixel tile's input patch is staged once, split into three bf16 planes (pixel stride CI + 8
// bf16: conflict-free ds_read_b128 fragments), and every tap reads its shifted window from there; the weight comes
// pre-split ([plane][BN][KP] bf16, sd_conv_split3_weight) straight from L2, one k chunk ahead. A lane's 8 k values of
// a chunk are 8 consecutive channels of one tap (CI % 8 == 0), so CI need not be a multiple of 32. Wave w owns tile
// pixels 32w..32w+31 (two 16-pixel tiles) x all BN channels; the epilogue (pool + RMSNorm + SiLU) is
// conv_fwd16_pool's, staged in the patch area.
template <int BN, int CI, int LW, int KS>
__global__ __launch_bounds__(256, 2) void conv_fwd6_direct_pool(GemmArgs g, Geom G, int lhw,
                                                                 const __bf16* __restrict__ wsp, const float* nw,
                                                                 float* pooled, uint8_t* amax, float* y, float* rstd,
                                                                 float eps, int nchw_flat) {
  constexpr int W = 1 << LW, R = 128 / W, PH = R + KS - 1, PW = W + KS - 1, CP = CI + 8, PAD = KS / 2;
  constexpr int PLANE = PH * PW * CP, K = KS * KS * CI, NKC = (K + 31) / 32, KP = NKC * 32, TN = BN / 16;
  constexpr int CI4 = CI / 4, NEL = PH * PW * CI4, NE = (NEL + 255) / 256;
  static_assert(CI % 8 == 0 && 128 % W == 0 && BN % 16 == 0, "geometry");
  static_assert(128 * (BN + 1) * 4 <= 3 * PLANE * 2, "epilogue tile fits the patch area");
  typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
  extern __shared__ __attribute__((aligned(16))) __bf16 patch6[];  // [plane][PH][PW][CP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l16 = lane & 15, q = lane >> 4;
  const int bm0 = blockIdx.x * 128, n = bm0 >> lhw, y0 = (bm0 & ((1 << lhw) - 1)) >> LW;
  {
    f32x4 v[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const int i = tid + 256 * e, c4 = i % CI4, pix = i / CI4, pc = pix % PW, pr = pix / PW;
      const int yy = y0 + pr - PAD, xx = pc - PAD;
      v[e] = (i < NEL && (unsigned)yy < (unsigned)G.Hs && (unsigned)xx < (unsigned)W)
                 ? *reinterpret_cast<const f32x4*>(G.in + (((long)n * G.Hs + yy) * W + xx) * CI + 4 * c4)
                 : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const int i = tid + 256 * e;
      if (i < NEL) {
        const int c4 = i % CI4, pix = i / CI4;
        float h0, h1, h2, h3, m0, m1, m2, m3;
        const u32x2 h{bf16_pair(v[e][0], v[e][1], h0, h1), bf16_pair(v[e][2], v[e][3], h2, h3)};
        const float r0 = v[e][0] - h0, r1 = v[e][1] - h1, r2 = v[e][2] - h2, r3 = v[e][3] - h3;
        const u32x2 m{bf16_pair(r0, r1, m0, m1), bf16_pair(r2, r3, m2, m3)};
        const f32x4 l{r0 - m0, r1 - m1, r2 - m2, r3 - m3};
        __bf16* dst = patch6 + pix * CP + 4 * c4;
        *reinterpret_cast<u32x2*>(dst) = h;
        *reinterpret_cast<u32x2*>(dst + PLANE) = m;
        *reinterpret_cast<bf16x4*>(dst + 2 * PLANE) = __builtin_convertvector(l, bf16x4);
      }
    }
  }
  int pbase[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int p = 32 * wave + 16 * mt + l16;
    pbase[mt] = ((p >> LW) * PW + (p & (W - 1))) * CP;
  }
  const __bf16* wl = wsp + (long)l16 * KP + 8 * q;
  bf16x8 b[2][TN][3];
  auto bload = [&](int kc, int s) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        b[s][j][pl] = *reinterpret_cast<const bf16x8*>(wl + ((long)pl * BN + 16 * j) * KP + 32 * kc);
  };
  f32x4 acc[2][TN];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bload(0, 0);
  __syncthreads();
  auto chunk = [&](int kc, int s) {
    if (kc + 1 < NKC) bload(kc + 1, s ^ 1);
    int k0 = 32 * kc + 8 * q;
    k0 = k0 < K ? k0 : K - 8;  // past K: any in-patch address (the weight is zero there)
    const int tap = k0 / CI, c0 = k0 - tap * CI, ky = tap / KS, kx = tap - ky * KS;
    const int off = (ky * PW + kx) * CP + c0;
    bf16x8 a[2][3];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) a[mt][pl] = *reinterpret_cast<const bf16x8*>(patch6 + pl * PLANE + pbase[mt] + off);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x4 c = acc[mt][j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt][2], b[s][j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt][1], b[s][j][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt][0], b[s][j][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt][1], b[s][j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt][0], b[s][j][1], c, 0, 0, 0);
        acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt][0], b[s][j][0], c, 0, 0, 0);
      }
  };
  int kc = 0;
  for (; kc + 2 <= NKC; kc += 2) {
    chunk(kc, 0);
    chunk(kc + 1, 1);
  }
  if (kc < NKC) chunk(kc, 0);
  __syncthreads();  // every wave is done reading the patch
  pool_epilogue<BN, 32>(acc, reinterpret_cast<float*>(patch6), g, G, LW, lhw, bm0, nw, pooled, amax, y, rstd, eps,
                        nchw_flat);
}

// conv_fwd6_direct_pool with the weight through LDS (round 6): 256-pixel tiles on 512-thread workgroups, the input
// patch staged once as three bf16 planes (as there), and the pre-split weight staged per 32-deep k chunk into a
// double-buffered LDS ring shared by the 8 waves (conv_dgrad3_direct's ring, three planes) instead of every lane loading
// its own fragments from L2 (0.9 MB of weight per 128-pixel tile: the L2 -> CU path bound the kernel, MFMA busy 0.37).
// Same products in the same k order: bit-identical to conv_fwd6_direct_pool.
// CG: the patch planes channel-group-major ([plane][CI / 8][PH * PW][8] bf16) instead of pixel-major with a pad: the 16
// lanes of a fragment read 16 consecutive pixels' 16-B pieces (conflict-free with no pad), so the 48 -> 64 stage's
// whole-image 256-pixel tile (20 x 20 x 48 patch) fits beside the ring (146 KB; pixel-major with its pad is 165 KB).
// PIPE: the fragments of chunk kc + 1 are read from LDS into a second register set under chunk kc's MFMAs (the ring
// stage chunk kc + 2 goes to is the one every wave finished reading before the previous barrier), so the LDS read
// latency is no longer exposed once per chunk; one barrier per chunk either way, same products in the same order.
// TPW: a workgroup runs TPW consecutive tiles (XCD-contiguous ranges, so the halo rows adjacent tiles share are L2
// hits), the next tile's patch loaded into registers under this tile's MFMAs and the ring's first chunk under its
// epilogue: with one workgroup per CU the prologue's HBM round trip was otherwise exposed once per tile.
// MT: 16-pixel m tiles per wave (2: 256-pixel tiles; 4: 512-pixel tiles, each wave 64 pixels x BN channels — 21
// fragment reads per 72 MFMAs instead of 15 per 36: less LDS traffic per product). BROW: the ring's row stride in bf16
// (40 = 32 + a pad; 32 = packed, the 64-B rows of a fragment read are still 1 KB contiguous).
// NTH: threads (the 48 -> 64 stage's whole image as four 64-pixel waves on 256 threads measured slower than eight
// 32-pixel waves, 213.7 vs 180.5 us, profiles/r06m3: one wave per SIMD).
template <int BN, int CI, int LW, int KS, bool CG, bool PIPE, int TPW, int MT = 2, int BROW = 40, int NTH = 512>
__global__ __launch_bounds__(NTH, 1) void conv_fwd6r_direct_pool(GemmArgs g, Geom G, int lhw,
                                                                  const __bf16* __restrict__ wsp, const float* nw,
                                                                  float* pooled, uint8_t* amax, float* y, float* rstd,
                                                                  float eps, int nchw_flat) {
  constexpr int TP = 16 * MT * (NTH / 64);
  static_assert(!PIPE || MT == 2, "the fragment pipeline is built for two m tiles");
  constexpr int W = 1 << LW, R = TP / W, PH = R + KS - 1, PW = W + KS - 1, CP = CG ? CI : CI + 8, PAD = KS / 2;
  constexpr int NPIX = PH * PW, PLANE = NPIX * CP, K = KS * KS * CI, NKC = (K + 31) / 32, KP = NKC * 32, TN = BN / 16;
  constexpr int CI4 = CI / 4, NEL = PH * PW * CI4, NE = (NEL + NTH - 1) / NTH;
  constexpr int SB = 3 * BN * BROW, NPC = 3 * BN * 4, NPT = (NPC + NTH - 1) / NTH;  // ring: [plane][n][BROW]
  // element offset of (pixel, channel c, c % 4 == 0) in a plane
  auto poff = [](int pix, int c) { return CG ? ((c >> 3) * NPIX + pix) * 8 + (c & 7) : pix * CP + c; };
  static_assert(CI % 8 == 0 && TP % W == 0 && BN % 16 == 0, "geometry");
  static_assert(TP * (BN + 1) * 4 <= 3 * PLANE * 2, "epilogue tile fits the patch area");
  typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
  extern __shared__ __attribute__((aligned(16))) __bf16 patch6r[];  // [plane][PH][PW][CP], then the ring [2][SB]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l16 = lane & 15, q = lane >> 4;
  const int nwg = gridDim.x, ntiles = g.M / TP;
  const int wg = (nwg & 7) ? blockIdx.x : (blockIdx.x & 7) * (nwg >> 3) + (blockIdx.x >> 3);
  __bf16* bst = patch6r + 3 * PLANE;
  bf16x8 br[NPT];
  auto bload = [&](int kc) {  // piece i: plane i / (4 BN), row (i / 4) % BN, 16-B piece i % 4 of the chunk
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int i = tid + NTH * u;
      if (i < NPC) br[u] = *reinterpret_cast<const bf16x8*>(wsp + (long)(i >> 2) * KP + 32 * kc + 8 * (i & 3));
    }
  };
  auto bstore = [&](int st) {
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int i = tid + NTH * u;
      if (i < NPC) *reinterpret_cast<bf16x8*>(bst + st * SB + (i >> 2) * BROW + 8 * (i & 3)) = br[u];
    }
  };
  f32x4 v[NE];
  auto load_patch = [&](int tile) {
    const int bm0 = tile * TP, n = bm0 >> lhw, y0 = (bm0 & ((1 << lhw) - 1)) >> LW;
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const int i = tid + NTH * e, c4 = i % CI4, pix = i / CI4, pc = pix % PW, pr = pix / PW;
      const int yy = y0 + pr - PAD, xx = pc - PAD;
      v[e] = (i < NEL && tile < ntiles && (unsigned)yy < (unsigned)G.Hs && (unsigned)xx < (unsigned)W)
                 ? *reinterpret_cast<const f32x4*>(G.in + (((long)n * G.Hs + yy) * W + xx) * CI + 4 * c4)
                 : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto store_patch = [&]() {
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const int i = tid + NTH * e;
      if (i < NEL) {
        const int c4 = i % CI4, pix = i / CI4;
        float h0, h1, h2, h3, m0, m1, m2, m3;
        const u32x2 h{bf16_pair(v[e][0], v[e][1], h0, h1), bf16_pair(v[e][2], v[e][3], h2, h3)};
        const float r0 = v[e][0] - h0, r1 = v[e][1] - h1, r2 = v[e][2] - h2, r3 = v[e][3] - h3;
        const u32x2 m{bf16_pair(r0, r1, m0, m1), bf16_pair(r2, r3, m2, m3)};
        const f32x4 l{r0 - m0, r1 - m1, r2 - m2, r3 - m3};
        __bf16* dst = patch6r + poff(pix, 4 * c4);
        *reinterpret_cast<u32x2*>(dst) = h;
        *reinterpret_cast<u32x2*>(dst + PLANE) = m;
        *reinterpret_cast<bf16x4*>(dst + 2 * PLANE) = __builtin_convertvector(l, bf16x4);
      }
    }
  };
  int pbase[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int p = 16 * MT * wave + 16 * mt + l16;
    pbase[mt] = (p >> LW) * PW + (p & (W - 1));  // pixel index at tap (0, 0)
  }
  bload(0);
  load_patch(wg * TPW);
  for (int it = 0; it < TPW; ++it) {
  const int tile = wg * TPW + it;
  if (tile >= ntiles) break;  // uniform over the workgroup
  if (it > 0) __syncthreads();  // the previous tile's epilogue is done with the patch area
  store_patch();
  bstore(0);
  if (NKC > 1) bload(1);
  f32x4 acc[MT][TN];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  if (it + 1 < TPW) load_patch(tile + 1);
  if constexpr (PIPE) {
    bf16x8 a[2][2][3], b[2][TN][3];
    auto frag = [&](int kc, int s) {  // chunk kc's fragments (ring stage kc & 1, the patch) into register set s
      const __bf16* bs = bst + (kc & 1) * SB + l16 * BROW + 8 * q;
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          b[s][j][pl] = *reinterpret_cast<const bf16x8*>(bs + (pl * BN + 16 * j) * BROW);
      int k0 = 32 * kc + 8 * q;
      k0 = k0 < K ? k0 : K - 8;  // past K: any in-patch address (the weight is zero there)
      const int tap = k0 / CI, c0 = k0 - tap * CI, ky = tap / KS, kx = tap - ky * KS;
      const int toff = ky * PW + kx;
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
          a[s][mt][pl] = *reinterpret_cast<const bf16x8*>(patch6r + pl * PLANE + poff(pbase[mt] + toff, c0));
    };
    frag(0, 0);
    if (NKC > 1) bstore(1);  // chunk 1 (in br) into stage 1
    if (NKC > 2) bload(2);
    __syncthreads();  // chunk 1 visible; every wave's chunk-0 reads are done
    auto step = [&](int kc, int s) {  // register set s holds chunk kc; stage (kc + 1) & 1 holds chunk kc + 1
      if (kc + 1 < NKC) frag(kc + 1, s ^ 1);
      if (kc + 2 < NKC) bstore(kc & 1);  // chunk kc + 2 (in br) over chunk kc, read before the last barrier
      if (kc + 3 < NKC) bload(kc + 3);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          f32x4 c = acc[mt][j];
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s][mt][2], b[s][j][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s][mt][1], b[s][j][1], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s][mt][0], b[s][j][2], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s][mt][1], b[s][j][0], c, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s][mt][0], b[s][j][1], c, 0, 0, 0);
          acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s][mt][0], b[s][j][0], c, 0, 0, 0);
        }
      __syncthreads();
    };
    int kc = 0;
    for (; kc + 2 <= NKC; kc += 2) {
      step(kc, 0);
      step(kc + 1, 1);
    }
    if (kc < NKC) step(kc, 0);
  } else
  for (int kc = 0; kc < NKC; ++kc) {
    const __bf16* bs = bst + (kc & 1) * SB + l16 * BROW + 8 * q;
    bf16x8 b[TN][3];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl) b[j][pl] = *reinterpret_cast<const bf16x8*>(bs + (pl * BN + 16 * j) * BROW);
    int k0 = 32 * kc + 8 * q;
    k0 = k0 < K ? k0 : K - 8;  // past K: any in-patch address (the weight is zero there)
    const int tap = k0 / CI, c0 = k0 - tap * CI, ky = tap / KS, kx = tap - ky * KS;
    const int toff = ky * PW + kx;
    bf16x8 a[MT][3];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int pl = 0; pl < 3; ++pl)
        a[mt][pl] = *reinterpret_cast<const bf16x8*>(patch6r + pl * PLANE + poff(pbase[mt] + toff, c0));
    if (kc + 1 < NKC) bstore((kc + 1) & 1);  // chunk kc + 1 (loaded one iteration ago) into the other stage
    if (kc + 2 < NKC) bload(kc + 2);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x4 c = acc[mt][j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt][2], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt][1], b[j][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt][0], b[j][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt][1], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt][0], b[j][1], c, 0, 0, 0);
        acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt][0], b[j][0], c, 0, 0, 0);
      }
    __syncthreads();
  }
  if (it + 1 < TPW) bload(0);  // the next tile's first weight chunk (the same weights) under the epilogue
  pool_epilogue<BN, 16 * MT>(acc, reinterpret_cast<float*>(patch6r), g, G, LW, lhw, tile * TP, nw, pooled, amax, y,
                             rstd, eps, nchw_flat);
  }
}

// [plane][n][KP] three-way split-bf16 image (gemm6_core.h split) of a (rows, K) fp32 matrix, zero past K
__global__ __launch_bounds__(256) void split3_weight(const float* __restrict__ w, __bf16* __restrict__ out, int rows,
                                                     int K, int KP) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)rows * KP) return;
  const int r = (int)(i / KP), k = (int)(i % KP);
  const float v = k < K ? w[(long)r * K + k] : 0.f;
  const __bf16 a0 = (__bf16)v;
  const float r1 = v - (float)a0;
  const __bf16 a1 = (__bf16)r1;
  const long pl = (long)rows * KP;
  out[i] = a0;
  out[pl + i] = a1;
  out[2 * pl + i] = (__bf16)(r1 - (float)a1);
}

// Direct forward for the 4-channel (padded RGB) first stage: K = 25 taps x 4 channels, so one
// v_mfma_f32_16x16x4_f32 step is exactly one tap (lane (l16, q) supplies channel q of pixel l16's tap sample) and
// nothing is padded to a 32-wide k tile. The whole weight (BN x 100 floats) lives in registers (each lane keeps its
// 25 x TN fragments, loaded once per workgroup), the (R + KS - 1) x (W + KS - 1) x 4 input patch in LDS (one
// float4 per pixel: the b32 fragment reads of 64 lanes hit 64 distinct banks). A workgroup runs TPW vertically
// adjacent tiles (XCD-aware: an XCD's workgroups cover a contiguous tile range), prefetching the next tile's patch
// into registers under the current tile's MFMAs; the epilogue is conv_fwd16_pool's, in its own LDS area.
// tpw (runtime) tiles per workgroup: the launcher sizes the grid to one round of resident workgroups (OCC per CU),
// so no partial last round of long workgroups idles part of the chip.
template <int BN, int LW, int KS, int OCC>
__global__ __launch_bounds__(256, OCC) void conv_fwd_direct_pool_c4(GemmArgs g, Geom G, int lhw, int TPW,
                                                                    const float* nw, float* pooled, uint8_t* amax,
                                                                    float* y, float* rstd, float eps, int nchw_flat) {
  constexpr int BM = 128, WM = 32, TM = WM / 16, TN = BN / 16, W = 1 << LW, R = BM / W;
  constexpr int PH = R + KS - 1, PW = W + KS - 1, PAD = KS / 2, NT = KS * KS;
  constexpr int NQ = PH * PW, NQT = (NQ + 255) / 256;
  // the patch area is padded to NQT * 256 pixels, so every thread's staging store is unconditional (a store under a
  // branch left the compiler a path on which the loop-invariant weight loads looked outstanding: it then waited for
  // the next tile's prefetch, vmcnt(0), before the first MFMA of every tile)
  float* smem = sd_smem<NQT * 256 * 4 + BM * (BN + 1)>();
  float* patch = smem;
  float* C = smem + NQT * 256 * 4;
  const int nwg = gridDim.x, ntiles = g.M / BM;
  const int wg = (nwg & 7) ? blockIdx.x : (blockIdx.x & 7) * (nwg >> 3) + (blockIdx.x >> 3);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l16 = lane & 15, q = lane >> 4;
  float bw[NT][TN];
  {
    const sd_rsrc rb = sd_make_rsrc(g.B, (long)g.N * g.ldb * 4);
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int j = 0; j < TN; ++j) bw[t][j] = sd_bload1(rb, (uint32_t)(((16 * j + l16) * g.ldb + 4 * t + q) * 4));
  }
  EpiPre<BN> pre;
#pragma unroll
  for (int j = 0; j < TN; ++j) pre.bias[j] = g.bias ? g.bias[16 * j + l16] : 0.f;
#pragma unroll
  for (int k = 0; k < BN / 8; ++k) pre.nw[k] = nw[(threadIdx.x & 7) + 8 * k];
  const sd_rsrc rs = sd_make_rsrc(G.in, (long)G.Nb * G.Hs * G.Ws * 16);
  f32x4 v[NQT];
  auto load_patch = [&](int tile) {
    const int bm0 = tile * BM, n = bm0 >> lhw, y0 = (bm0 & ((1 << lhw) - 1)) >> LW;
#pragma unroll
    for (int u = 0; u < NQT; ++u) {
      const int i = threadIdx.x + 256 * u;
      const int py = i / PW, px = i % PW;
      const int yy = y0 + py - PAD, xx = px - PAD;
      const bool ok = i < NQ && tile < ntiles && (unsigned)yy < (unsigned)G.Hs && (unsigned)xx < (unsigned)W;
      v[u] = sd_bload4(rs, ok ? (uint32_t)(((n * G.Hs + yy) * W + xx) * 16) : SD_OOB);
    }
  };
  int abase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int p = wave * WM + 16 * i + l16;
    abase[i] = ((p >> LW) * PW + (p & (W - 1))) * 4 + q;
  }
  load_patch(wg * TPW);
  for (int it = 0; it < TPW; ++it) {
    const int tile = wg * TPW + it;
    if (tile >= ntiles) break;  // uniform over the workgroup
#pragma unroll
    for (int u = 0; u < NQT; ++u) *reinterpret_cast<f32x4*>(patch + 4 * (threadIdx.x + 256 * u)) = v[u];
    __syncthreads();  // patch staged (and the previous tile's epilogue is past its C reads)
    if (it + 1 < TPW) load_patch(tile + 1);
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int toff = ((t / KS) * PW + t % KS) * 4;
      float a[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = patch[abase[i] + toff];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], bw[t][j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();  // every wave is done reading the patch before the next tile's is stored
    pool_epilogue<BN, WM>(acc, C, g, G, LW, lhw, tile * BM, nw, pooled, amax, y, rstd, eps, nchw_flat, &pre);
  }
}

// SDHIP_CONV_DIRECT_FWD (benchmarking knob): 1 (default) = conv_fwd_direct_pool where it applies, 0 = implicit GEMM.
// (A variant streaming each lane's weight fragments into registers — no LDS stage, no barriers, 3 workgroups per
// CU — measured slower: 679 vs 660 us on encoder stage 2 at 1024 images.)
bool conv_direct_fwd() {
  static int a = -1;
  if (a < 0) {
    const char* e = getenv("SDHIP_CONV_DIRECT_FWD");
    a = e ? atoi(e) : 1;
  }
  return a != 0;
}

// bwd-weight: M = Co (one tile), N = kh*kw*Ci + 1, K = pixels (split-K slabs), 4 waves along N
template <int BM>
__global__ __launch_bounds__(256) void conv_wgrad16(GemmArgs g, Geom G, int J, int lw, int lhw) {
  constexpr int BN = 128;
  const int bn0 = blockIdx.x * BN;
  const int split = blockIdx.z;
  const int kbeg = split * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  DenseKM<BM, true> la(g.A, g.lda, g.M, 0);
  Im2colColsKM<BN> lb(G, J, bn0, lw, lhw);
  gemm_block16<BM, BN, BM, 32>(g, la, lb, 0, bn0, 0, split, kbeg, kend);
}

// ---------------------------------------------------------------- direct bwd-weight (stride 1, no upsample)
// dW[co][j = (ky,kx,ci)] (+ d bias at j = J) = sum over pixels of dy[p][co] * x[p + (ky,kx) - pad][ci].
// A 512-thread workgroup stages one block of R image rows in LDS — the dy rows (R*W x Co) and the input patch with
// its halo ((R+kh-1) x (W+kw-1) x Ci, zero padded) — and runs every (co, j) product of that block from LDS, so the
// 25x im2col expansion is never read from memory (one patch read per row block instead of one per tap).
// Wave w owns NBW 16-column blocks of j, all TM 16-row blocks of co: acc = TM*NBW 16x16 fp32 tiles in registers,
// accumulated over the row blocks blockIdx.y, +gridDim.y, ...; the gridDim.y partial slabs are summed by
// gemm_reduce_kernel. MFMA 16x16x4: lane (l16, q) supplies dy[p = 4s+q][co = l16] and x-patch[p = 4s+q][j = l16].
// LDS row strides are padded to 16 (mod 64) floats so the 4 lane groups hit distinct banks.
struct DirectW {
  const float* x;
  const float* dy;      // (Nb, H, W, Co) conv-output gradient, or (PL) the pooled-resolution gradient (Nb, H/2, W/2, Co)
  const uint8_t* amax;  // PL: the 2x2 max-pool argmax per pooled element (dy is routed to that window position)
  float* ws;
  int Nb, H, W, Ci, Co, kh, kw, pad, R, lw;  // lw = log2(W)
  int J, PW, PH, SA, CP, blocks;
};

SD_DEV int pad16(int c) { return c % 32 == 0 ? c + 16 : c; }

constexpr int WD_VA = 4, WD_VP = 6;  // max float4 per thread of a staged dy block / input patch

// WS (wave split): for narrow j ranges every wave covers all j blocks over every 8th k step and writes its own slab
// PL: dy is the max-pool backward's input (pooled resolution + argmax), expanded while it is fetched — the
// full-resolution conv gradient (3/4 zeros) is never written to or read from HBM.
template <int TM, int NBW, bool WS, bool PL = false>
__global__ __launch_bounds__(512) void conv_wgrad_direct(DirectW d) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, q = lane >> 4;
  const int P = d.R * d.W;
  float* dyl = lds;                 // [P][SA]
  float* xp = lds + P * d.SA;       // [PH][PW][CP]; channel Ci holds 1.0 (bias column), Ci+1 holds 0.0
  // per-lane column decode of this wave's j blocks (j == J -> the ones channel, j > J -> the zero channel)
  int off[NBW];
#pragma unroll
  for (int b = 0; b < NBW; ++b) {
    const int j = 16 * (WS ? b : (blockIdx.x * NW_D + wave) * NBW + b) + l16;
    if (j < d.J) {
      const int t = j / d.Ci, ci = j - t * d.Ci, ky = t / d.kw, kx = t - ky * d.kw;
      off[b] = (ky * d.PW + kx) * d.CP + ci;
    } else {
      off[b] = d.Ci + (j == d.J ? 0 : 1);
    }
  }
  f32x4 acc[TM][NBW];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int b = 0; b < NBW; ++b) acc[i][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int rows_per_img = d.H / d.R, cq = d.Ci / 4, nA = P * d.Co / 4, nP = d.PH * d.PW * cq;
  f32x4 ra[WD_VA], rp[WD_VP];
  uint32_t aa[PL ? WD_VA : 1];
  // global -> registers for row block rb (all loads issued together)
  auto fetch = [&](int rb) {
    const int n = rb / rows_per_img, y0 = (rb - n * rows_per_img) * d.R;
    const float* dsrc = d.dy + ((long)n * d.H + y0) * d.W * d.Co;
#pragma unroll
    for (int v = 0; v < WD_VA; ++v) {
      const int i = tid + 512 * v;
      if constexpr (PL) {  // item i = (pooled pixel of the block, 4-channel group): raw gradient + argmax bytes
        ra[v] = f32x4{0.f, 0.f, 0.f, 0.f};
        aa[v] = 0xffffffffu;
        if (i < nA / 4) {
          const long pp = (((long)n * (d.H >> 1) + (y0 >> 1)) * (d.W >> 1)) * d.Co + 4 * i;
          ra[v] = *reinterpret_cast<const f32x4*>(d.dy + pp);
          aa[v] = *reinterpret_cast<const uint32_t*>(d.amax + pp);
        }
      } else {
        ra[v] = i < nA ? *reinterpret_cast<const f32x4*>(dsrc + 4 * i) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int v = 0; v < WD_VP; ++v) {
      const int i = tid + 512 * v;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      if (i < nP) {
        const int pix = i / cq, c = 4 * (i - pix * cq);
        const int py = pix / d.PW, px = pix - py * d.PW;
        const int iy = y0 - d.pad + py, ix = px - d.pad;
        if (iy >= 0 && iy < d.H && ix >= 0 && ix < d.W)
          x = *reinterpret_cast<const f32x4*>(d.x + (((long)n * d.H + iy) * d.W + ix) * d.Ci + c);
      }
      rp[v] = x;
    }
  };
  auto stage = [&]() {
#pragma unroll
    for (int v = 0; v < WD_VA; ++v) {
      const int i = tid + 512 * v;
      if constexpr (PL) {  // route the pooled gradient to its argmax position of the 2x2 window, zeros elsewhere
        if (i < nA / 4) {
          const int e = 4 * i, pl = e / d.Co, c = e - pl * d.Co;
          const int hw = d.W >> 1, pr = pl / hw, pc = pl - pr * hw;
#pragma unroll
          for (int qd = 0; qd < 4; ++qd) {
            const int p = (2 * pr + (qd >> 1)) * d.W + 2 * pc + (qd & 1);
            f32x4 val;
#pragma unroll
            for (int k = 0; k < 4; ++k) val[k] = ((aa[v] >> (8 * k)) & 0xffu) == (uint32_t)qd ? ra[v][k] : 0.f;
            *reinterpret_cast<f32x4*>(dyl + p * d.SA + c) = val;
          }
        }
      } else if (i < nA) {
        const int e = 4 * i, p = e / d.Co, c = e - p * d.Co;
        *reinterpret_cast<f32x4*>(dyl + p * d.SA + c) = ra[v];
      }
    }
#pragma unroll
    for (int v = 0; v < WD_VP; ++v) {
      const int i = tid + 512 * v;
      if (i < nP) {
        const int pix = i / cq, c = 4 * (i - pix * cq);
        *reinterpret_cast<f32x4*>(xp + pix * d.CP + c) = rp[v];
      }
    }
  };
  // the constant channels never change: write them once
  for (int pix = tid; pix < d.PH * d.PW; pix += 512) {
    xp[pix * d.CP + d.Ci] = 1.f;
    xp[pix * d.CP + d.Ci + 1] = 0.f;
  }
  int rb = blockIdx.y;
  if (rb < d.blocks) fetch(rb);
  for (; rb < d.blocks; rb += gridDim.y) {
    __syncthreads();  // previous block's LDS reads are done
    stage();
    __syncthreads();
    if (rb + (int)gridDim.y < d.blocks) fetch(rb + gridDim.y);  // next block's loads overlap this block's MFMAs
    for (int s = WS ? wave : 0; s < P / 4; s += WS ? NW_D : 1) {
      const int p = 4 * s + q, py = p >> d.lw, px = p & (d.W - 1);
      float a[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = dyl[p * d.SA + 16 * i + l16];
      const float* xb = xp + (py * d.PW + px) * d.CP;
      float bv[NBW];
#pragma unroll
      for (int b = 0; b < NBW; ++b) bv[b] = xb[off[b]];
#pragma unroll
      for (int b = 0; b < NBW; ++b)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[i][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], bv[b], acc[i][b], 0, 0, 0);
    }
  }
  // partial slab blockIdx.y: ws[split][co][J+1]
  float* out = d.ws + (long)blockIdx.y * d.Co * (d.J + 1);
  if (WS) {  // sum the 8 waves' tiles through LDS (the staging area is free now), one 16x16 tile at a time
#pragma unroll
    for (int b = 0; b < NBW; ++b)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 4; ++r) lds[(wave * 4 + r) * 64 + lane] = acc[i][b][r];
        __syncthreads();
        if (tid < 256) {
          const int r = tid >> 6, ln = tid & 63;
          float v = 0.f;
#pragma unroll
          for (int w = 0; w < NW_D; ++w) v += lds[(w * 4 + r) * 64 + ln];
          const int j = 16 * b + (ln & 15), co = 16 * i + 4 * (ln >> 4) + r;
          if (j <= d.J && co < d.Co) out[(long)co * (d.J + 1) + j] = v;
        }
      }
    return;
  }
#pragma unroll
  for (int b = 0; b < NBW; ++b) {
    const int j = 16 * ((blockIdx.x * NW_D + wave) * NBW + b) + l16;
    if (j <= d.J) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = 16 * i + 4 * q + r;
          if (co < d.Co) out[(long)co * (d.J + 1) + j] = acc[i][b][r];
        }
    }
  }
}

// ---------------------------------------------------------------- split-bf16 backward (gemm3_core.h)
// The two backward contractions of a convolution on the bf16x3 MFMA path (~1e-5 relative, 5.3x the f32 rate):
// only gradients flow through them, no sampled latent depends on them.

// A KC-layout f32 loader (st.r[v]: thread i = tid + 256 v holds row i / 8, k 4 * (i % 8) .. +3) staged as split bf16
template <class L, int ROWS>
struct KCSplit {
  L& l;
  SD_DEV explicit KCSplit(L& l_) : l(l_) {}
  SD_DEV void load(int k0, int kend) { l.load(k0, kend); }
  SD_DEV void store(__bf16* lds) const {
#pragma unroll
    for (int v = 0; v < L::NV; ++v) {
      const int i = threadIdx.x + v * 256;
      if ((v + 1) * 256 <= ROWS * BK / 4 || i < ROWS * BK / 4)
        sdb::split_store(lds + (i / (BK / 4)) * sdb::LROW + 4 * (i % (BK / 4)), l.st.r[v]);
    }
  }
};

// bwd-data: dIn = conv_same(dOut, flipped W) as implicit GEMM, M = pixels (128 per workgroup), N = the input's
// channels (one tile), K = kh*kw*C(dOut); 4 waves along M.
template <int BN>
__global__ __launch_bounds__(256, 2) void conv_dgrad3(GemmArgs g, Geom G, int lw, int lhw) {
  __shared__ int tab[MAX_TAPQ];
  build_taps(tab, G, g.K);
  constexpr int BM = 128;
  const int bm0 = blockIdx.x * BM;
  Im2colRowsB<BM> la0(G, tab, g.M, bm0, lw, lhw);
  DenseKCB<BN> lb0(g.B, g.ldb, g.N, 0);
  KCSplit<Im2colRowsB<BM>, BM> la(la0);
  KCSplit<DenseKCB<BN>, BN> lb(lb0);
  f32x4 acc[2][BN / 16];
  sdb::gemm3_mainloop<BM, BN, 32, BN>(la, lb, 0, g.K, acc);
  sdb::gemm3_epilogue<BM, BN, 32, BN>(g, acc, bm0, 0, 0, 0);
}

// bwd-data as a DIRECT convolution on split-bf16 MFMAs: conv_dgrad3's contraction (dIn = conv_same(dOut, flipped W),
// K = (ky, kx, c) with c contiguous), but each workgroup stages its dOut patch (R image rows + the kh-1 / kw-1 halo,
// zero outside the image) ONCE in LDS, split to (hi, lo) bf16 planes on the way in, and every tap reads its shifted
// window from there: each dOut element is loaded and split once per workgroup instead of once per tap it feeds
// (conv_dgrad3's im2col staging re-split it up to kh*kw times: VALU-bound, 0.2 of the bf16x3 peak). The B operand
// comes pre-split ([plane][n][KP] bf16, sd_conv_split_weight) straight from global memory (L2-resident, 16 B per lane
// per plane), one k chunk ahead. M = R*W output pixels per workgroup (128), 4 waves x 2 16-pixel tiles, NT 16-channel
// tiles of dIn; per 32-deep k chunk a lane's 8 k values are 8 consecutive channels of one tap (CIN % 8 == 0), one
// ds_read_b128 per plane. Products: lo_a*hi_b + hi_a*lo_b + hi_a*hi_b (gemm3_mainloop's order), f32 accumulation.
// MT / CG / NTHR (round 6): MT 16-pixel m tiles per wave over NTHR threads (the tile is 16 MT NTHR / 64 pixels), the
// patch channel-group-major when CG ([plane][CIN / 8][pixel][8]: no pad, conflict-free), as conv_fwd6r_direct_pool's
// 64-pixel waves: 12 fragment reads per 24 MFMAs instead of 8 per 12. Same products in the same k order.
template <int CIN, int NT, int LW, int KS, int MT = 2, bool CG = false, int NTHR = 256>
__global__ __launch_bounds__(NTHR, 2) void conv_dgrad3_direct(const float* __restrict__ dout,
                                                               const __bf16* __restrict__ wsp, float* __restrict__ din,
                                                               int Nb, int H, int pad) {
  constexpr int TP = 16 * MT * (NTHR / 64);
  constexpr int W = 1 << LW, R = TP / W, PH = R + KS - 1, PW = W + KS - 1, CP = CG ? CIN : CIN + 8, NPIX = PH * PW;
  constexpr int PLANE = PH * PW * CP, K = KS * KS * CIN, NKC = (K + 31) / 32, KP = NKC * 32, NOUT = 16 * NT;
  constexpr int CIN4 = CIN / 4, NEL = PH * PW * CIN4, NE = (NEL + NTHR - 1) / NTHR;
  static_assert(CIN % 8 == 0 && R >= 1 && TP % W == 0, "geometry");
  // element offset of (pixel, channel c, c % 4 == 0) in a plane
  auto poff = [](int pix, int c) { return CG ? ((c >> 3) * NPIX + pix) * 8 + (c & 7) : pix * CP + c; };
  extern __shared__ __attribute__((aligned(16))) __bf16 patch[];  // [plane][PH][PW][CP]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l16 = lane & 15, q = lane >> 4;
  const int rows_per_img = H / R, n = blockIdx.x / rows_per_img, y0 = (blockIdx.x % rows_per_img) * R;
  // stage the patch: every load first, then split + store
  {
    f32x4 v[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const int i = tid + NTHR * e, c4 = i % CIN4, pix = i / CIN4, pc = pix % PW, pr = pix / PW;
      const int y = y0 + pr - pad, x = pc - pad;
      v[e] = (i < NEL && y >= 0 && y < H && x >= 0 && x < W)
                 ? *reinterpret_cast<const f32x4*>(dout + (((long)n * H + y) * W + x) * CIN + 4 * c4)
                 : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const int i = tid + NTHR * e;
      if (i < NEL) {
        const int c4 = i % CIN4, pix = i / CIN4;
        sdb::bf16x4 hi, lo;
        sdb::split2(v[e], hi, lo);
        *reinterpret_cast<sdb::bf16x4*>(patch + poff(pix, 4 * c4)) = hi;
        *reinterpret_cast<sdb::bf16x4*>(patch + PLANE + poff(pix, 4 * c4)) = lo;
      }
    }
  }
  // this lane's MT pixel tiles: pixel p = 16 MT wave + 16 mt + l16 -> patch-local pixel index (row, x)
  int pbase[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int p = 16 * MT * wave + 16 * mt + l16;
    pbase[mt] = (p >> LW) * PW + (p & (W - 1));
  }
  // B: one k chunk of the pre-split weight ([plane][NOUT][32] bf16, 16-B pieces) per LDS stage, double-buffered and
  // shared by the 4 waves (each wave reading its fragments from global memory itself made the L1 path the bound)
  typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
  constexpr int BROW = 40, SB = 2 * NOUT * BROW, NPC = 8 * NOUT, NPT = (NPC + NTHR - 1) / NTHR;
  __bf16* bst = patch + 2 * PLANE;
  bf16x8 br[NPT];
  auto bload = [&](int kc) {
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int i = tid + NTHR * u;
      if (i < NPC) br[u] = *reinterpret_cast<const bf16x8*>(wsp + (long)(i >> 2) * KP + 32 * kc + 8 * (i & 3));
    }
  };
  auto bstore = [&](int stage) {
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
      const int i = tid + NTHR * u;
      if (i < NPC) *reinterpret_cast<bf16x8*>(bst + stage * SB + (i >> 2) * BROW + 8 * (i & 3)) = br[u];
    }
  };
  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bload(0);
  bstore(0);
  if (NKC > 1) bload(1);
  __syncthreads();
  for (int kc = 0; kc < NKC; ++kc) {
    const __bf16* bs = bst + (kc & 1) * SB + l16 * BROW + 8 * q;
    bf16x8 bh[NT], bl[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      bh[j] = *reinterpret_cast<const bf16x8*>(bs + 16 * j * BROW);
      bl[j] = *reinterpret_cast<const bf16x8*>(bs + (NOUT + 16 * j) * BROW);
    }
    int k0 = 32 * kc + 8 * q;
    k0 = k0 < K ? k0 : K - 8;  // past K: any in-patch address (B is zero there)
    const int tap = k0 / CIN, c0 = k0 - tap * CIN, ky = tap / KS, kx = tap - ky * KS;
    const int toff = ky * PW + kx;
    bf16x8 ah[MT], al[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      ah[mt] = *reinterpret_cast<const bf16x8*>(patch + poff(pbase[mt] + toff, c0));
      al[mt] = *reinterpret_cast<const bf16x8*>(patch + PLANE + poff(pbase[mt] + toff, c0));
    }
    if (kc + 1 < NKC) bstore((kc + 1) & 1);  // chunk kc+1 (loaded one iteration ago) into the other stage
    if (kc + 2 < NKC) bload(kc + 2);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[mt], bh[j], acc[mt][j], 0, 0, 0);
        acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[mt], bl[j], acc[mt][j], 0, 0, 0);
        acc[mt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[mt], bh[j], acc[mt][j], 0, 0, 0);
      }
    __syncthreads();
  }
  // acc[mt][j][r]: pixel 16 MT wave + 16 mt + 4 q + r, channel 16 j + l16
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int p = 16 * MT * wave + 16 * mt + 4 * q + r, y = y0 + (p >> LW), x = p & (W - 1);
      float* o = din + (((long)n * H + y) * W + x) * NOUT + l16;
#pragma unroll
      for (int j = 0; j < NT; ++j) o[16 * j] = acc[mt][j][r];
    }
}

// [plane][n][KP] bf16 split image of a (rows, K) fp32 matrix, KP = K rounded up to 32, zero past K
__global__ __launch_bounds__(256) void split_weight(const float* __restrict__ w, __bf16* __restrict__ out, int rows,
                                                    int K, int KP) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)rows * KP) return;
  const int r = (int)(i / KP), k = (int)(i % KP);
  const float v = k < K ? w[(long)r * K + k] : 0.f;
  const __bf16 hi = (__bf16)v;
  out[i] = hi;
  out[(long)rows * KP + i] = (__bf16)(v - (float)hi);
}

// out[e] = sum_s ws[s * n + e] in a fixed order; 64 outputs per workgroup (one per lane), the 4 waves take every
// 4th slab and are summed through LDS.
// acc.dw set: out is not written; the sums are added into the parameter gradients (element e = (co, j) of the
// (Co, J + 1) [dW | db] layout, J = taps * cx channels; channels >= acc.ci_w dropped)
__global__ __launch_bounds__(256) void slab_reduce(const float* __restrict__ ws, int slabs, long n,
                                                   float* __restrict__ out, sd_wgrad_acc acc, int J, int cx) {
  __shared__ float part[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long e = (long)blockIdx.x * 64 + lane;
  float v = 0.f;
  if (e < n) {
    int s = wave;
    for (; s + 12 < slabs; s += 16) {
      const float a0 = ws[(long)s * n + e], a1 = ws[(long)(s + 4) * n + e];
      const float a2 = ws[(long)(s + 8) * n + e], a3 = ws[(long)(s + 12) * n + e];
      v += (a0 + a1) + (a2 + a3);
    }
    for (; s < slabs; s += 4) v += ws[(long)s * n + e];
  }
  part[wave][lane] = v;
  __syncthreads();
  if (wave == 0 && e < n) {
    const float r = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
    if (!acc.dw) {
      out[e] = r;
    } else {
      const long co = e / (J + 1);
      const int j = (int)(e - co * (J + 1));
      if (j == J) {
        acc.db[co] += r;
      } else {
        const int tap = j / cx, c = j - tap * cx;
        if (c < acc.ci_w) acc.dw[(co * (J / cx) + tap) * acc.ci_w + c] += r;
      }
    }
  }
}

// ---------------------------------------------------------------- direct split-bf16 bwd-weight
// conv_wgrad_direct's structure (one block of R image rows per step: the input patch with its halo staged in LDS
// once, every (co, j) product of the block taken from LDS, partial slabs per blockIdx.y) on v_mfma_f32_16x16x32_bf16.
// k = pixels, 32 per MFMA step: lane group q supplies pixels 4i + q (i = 0..7) of the step, so the 4 lane groups read
// neighbouring pixels of the patch (CP floats apart: conflict-free) and each lane's 8 B-values are 8 ds_read_b32 at
// precomputed pixel offsets + its column's tap offset, split to (hi, lo) in registers. dy of the block is staged
// transposed and pre-split, [co][pos] per plane with pos = 8 (p % 4) + (p / 4) % 8 inside each 32-pixel step, so a
// lane's 8 A-values (the same pixels) are one ds_read_b128 per plane. Wave w owns NBW 16-column blocks of j and all
// TM 16-row blocks of co (rows >= Co read zero rows).
struct DirectW3 {
  const float* x;
  const float* dy;      // (Nb, H, W, Co) conv-output gradient, or (PL) the pooled-resolution gradient
  const uint8_t* amax;  // PL: the 2x2 max-pool argmax per pooled element
  float* ws;
  int Nb, H, W, Ci, Co, kh, kw, pad, R, lw;
  int J, PW, PH, CP, PS, blocks;
};

// SD_WD3_PRE (default 1): the input patch is staged PRE-SPLIT, each element as one 32-bit word (bf16 hi in the low
// half, bf16 lo in the high half: the same split2 values), so the inner loop forms a lane's 8 B-values of each plane
// with 4 v_perm_b32 instead of re-splitting 8 floats per use (every patch element feeds kh * kw taps x the column
// blocks): bit-identical products, the split VALU moved from the k loop to the stage.
#ifndef SD_WD3_PRE
#define SD_WD3_PRE 1
#endif
SD_DEV uint32_t pack_split(float v) {  // (bf16 hi | bf16 lo << 16), hi + lo = v up to 2^-17 |v| (split2's values)
  const f32x4 x = {v, 0.f, 0.f, 0.f};
  sdb::bf16x4 hi, lo;
  sdb::split2(x, hi, lo);
  return (uint32_t)__builtin_bit_cast(uint16_t, hi[0]) | ((uint32_t)__builtin_bit_cast(uint16_t, lo[0]) << 16);
}
// WS (wave split, as conv_wgrad_direct): for few column blocks (the 4-channel first stage: J + 1 = 101 -> 7 blocks)
// every wave covers all of them over every 8th 32-pixel step, and the 8 waves' tiles are summed through LDS at the end.
// PL: dy is the max-pool backward's pooled-resolution gradient + argmax (sd_pool_rms_bwd_compact), routed to its
// window position while fetched (conv_wgrad_direct's PL): the first stage's bwd-weight without the full-resolution
// conv gradient, on split-bf16.
template <int TM, int NBW, bool WS = false, bool PL = false>
__global__ __launch_bounds__(512) void conv_wgrad3_direct(DirectW3 d) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, q = lane >> 4;
  const int P = d.R * d.W;
  float* xp = lds;  // [PH][PW][CP]; channel Ci holds 1.0 (bias column), Ci+1 holds 0.0
  __bf16* dyh = reinterpret_cast<__bf16*>(lds + d.PH * d.PW * d.CP);  // [TM*16][PS]
  __bf16* dyl = dyh + TM * 16 * d.PS;
  for (int e = tid; e < TM * 16 * d.PS; e += 512) {  // rows >= Co stay zero; rows < Co are overwritten per block
    dyh[e] = (__bf16)0.f;
    dyl[e] = (__bf16)0.f;
  }
  int off[NBW];
#pragma unroll
  for (int b = 0; b < NBW; ++b) {
    const int j = 16 * (WS ? b : (blockIdx.x * NW_D + wave) * NBW + b) + l16;
    if (j < d.J) {
      const int t = j / d.Ci, ci = j - t * d.Ci, ky = t / d.kw, kx = t - ky * d.kw;
      off[b] = (ky * d.PW + kx) * d.CP + ci;
    } else {
      off[b] = d.Ci + (j == d.J ? 0 : 1);
    }
  }
  f32x4 acc[TM][NBW];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int b = 0; b < NBW; ++b) acc[i][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int rows_per_img = d.H / d.R, cq = d.Ci / 4, nP = d.PH * d.PW * cq;
  const int c4 = d.Co / 4, nD = c4 * (P / 4);  // 4x4 blocks: 8 pixel groups per 32-pixel step
  // this thread's dy block: 4 channels x 4 pixels (pixels c + 4 (4 ih + t) of 32-pixel step sb, t = 0..3)
  const int dq4 = tid % c4, drest = tid / c4;
  const int dc = drest % 4, dih = (drest / 4) % 2, dsb = drest / 8;
  f32x4 rd[4], rp[WD_VP];
  uint32_t aw[PL ? 4 : 1];  // PL: the 4 channels' argmax bytes of each pixel's pooled element
  int qd[PL ? 4 : 1];       // PL: the pixel's position in its 2x2 window
  auto fetch = [&](int rb) {
    const int n = rb / rows_per_img, y0 = (rb - n * rows_per_img) * d.R;
    [[maybe_unused]] const float* dsrc = d.dy + ((long)n * d.H + y0) * d.W * d.Co;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int px = 32 * dsb + dc + 4 * (4 * dih + t);
      if constexpr (PL) {  // the pooled element of pixel px (row y0 + px / W), loaded whole; masked in stage()
        const int yy = y0 + (px >> d.lw), xx = px & (d.W - 1);
        const long pp = (((long)n * (d.H >> 1) + (yy >> 1)) * (d.W >> 1) + (xx >> 1)) * d.Co + 4 * dq4;
        const bool ok = tid < nD;
        rd[t] = ok ? *reinterpret_cast<const f32x4*>(d.dy + pp) : f32x4{0.f, 0.f, 0.f, 0.f};
        aw[t] = ok ? *reinterpret_cast<const uint32_t*>(d.amax + pp) : 0xffffffffu;
        qd[t] = (yy & 1) * 2 + (xx & 1);
      } else {
        rd[t] = tid < nD ? *reinterpret_cast<const f32x4*>(dsrc + (long)px * d.Co + 4 * dq4)
                         : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
#pragma unroll
    for (int v = 0; v < WD_VP; ++v) {
      const int i = tid + 512 * v;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      if (i < nP) {
        const int pix = i / cq, c = 4 * (i - pix * cq);
        const int py = pix / d.PW, px = pix - py * d.PW;
        const int iy = y0 - d.pad + py, ix = px - d.pad;
        if (iy >= 0 && iy < d.H && ix >= 0 && ix < d.W)
          x = *reinterpret_cast<const f32x4*>(d.x + (((long)n * d.H + iy) * d.W + ix) * d.Ci + c);
      }
      rp[v] = x;
    }
  };
  auto stage = [&]() {
    if (tid < nD) {
      const int pos = 32 * dsb + 8 * dc + 4 * dih;
      if constexpr (PL) {  // route the pooled gradient to its argmax position of the 2x2 window, zeros elsewhere
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (((aw[t] >> (8 * k)) & 0xffu) != (uint32_t)qd[t]) rd[t][k] = 0.f;
      }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const f32x4 t = {rd[0][jj], rd[1][jj], rd[2][jj], rd[3][jj]};
        sdb::bf16x4 hi, lo;
        sdb::split2(t, hi, lo);
        const int o = (4 * dq4 + jj) * d.PS + pos;
        *reinterpret_cast<sdb::bf16x4*>(dyh + o) = hi;
        *reinterpret_cast<sdb::bf16x4*>(dyl + o) = lo;
      }
    }
#pragma unroll
    for (int v = 0; v < WD_VP; ++v) {
      const int i = tid + 512 * v;
      if (i < nP) {
        const int pix = i / cq, c = 4 * (i - pix * cq);
        if (SD_WD3_PRE) {
          sdb::bf16x4 hi, lo;
          sdb::split2(rp[v], hi, lo);
          const uint64_t h = __builtin_bit_cast(uint64_t, hi), l = __builtin_bit_cast(uint64_t, lo);
          typedef uint32_t u32x4_ __attribute__((ext_vector_type(4)));
          u32x4_ w;
#pragma unroll
          for (int k = 0; k < 4; ++k) w[k] = (uint32_t)((h >> (16 * k)) & 0xffffu) | ((uint32_t)((l >> (16 * k)) & 0xffffu) << 16);
          *reinterpret_cast<u32x4_*>(xp + pix * d.CP + c) = w;
        } else {
          *reinterpret_cast<f32x4*>(xp + pix * d.CP + c) = rp[v];
        }
      }
    }
  };
  for (int pix = tid; pix < d.PH * d.PW; pix += 512) {
    if (SD_WD3_PRE) {
      reinterpret_cast<uint32_t*>(xp)[pix * d.CP + d.Ci] = pack_split(1.f);
      reinterpret_cast<uint32_t*>(xp)[pix * d.CP + d.Ci + 1] = 0u;
    } else {
      xp[pix * d.CP + d.Ci] = 1.f;
      xp[pix * d.CP + d.Ci + 1] = 0.f;
    }
  }
  int rb = blockIdx.y;
  if (rb < d.blocks) fetch(rb);
  for (; rb < d.blocks; rb += gridDim.y) {
    __syncthreads();  // previous block's LDS reads are done
    stage();
    __syncthreads();
    if (rb + (int)gridDim.y < d.blocks) fetch(rb + gridDim.y);  // next block's loads overlap this block's MFMAs
    for (int s = WS ? wave : 0; s < P / 32; s += WS ? NW_D : 1) {
      sdb::bf16x8 ah[TM], al[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int o = (16 * i + l16) * d.PS + 32 * s + 8 * q;
        ah[i] = *reinterpret_cast<const sdb::bf16x8*>(dyh + o);
        al[i] = *reinterpret_cast<const sdb::bf16x8*>(dyl + o);
      }
      int pb[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int p = 32 * s + 4 * i + q, py = p >> d.lw, px = p & (d.W - 1);
        pb[i] = (py * d.PW + px) * d.CP;
      }
#pragma unroll
      for (int b = 0; b < NBW; ++b) {
        sdb::bf16x8 bh, bl;
        if (SD_WD3_PRE) {  // 8 packed words -> the two planes, 2 elements per v_perm_b32
          const uint32_t* xu = reinterpret_cast<const uint32_t*>(xp);
          uint32_t wv[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) wv[i] = xu[pb[i] + off[b]];
          typedef uint32_t u32x4_ __attribute__((ext_vector_type(4)));
          u32x4_ ph, pl;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            ph[i] = __builtin_amdgcn_perm(wv[2 * i + 1], wv[2 * i], 0x05040100u);  // lo halves: the hi plane
            pl[i] = __builtin_amdgcn_perm(wv[2 * i + 1], wv[2 * i], 0x07060302u);  // hi halves: the lo plane
          }
          bh = __builtin_bit_cast(sdb::bf16x8, ph);
          bl = __builtin_bit_cast(sdb::bf16x8, pl);
        } else {
          const f32x4 v0 = {xp[pb[0] + off[b]], xp[pb[1] + off[b]], xp[pb[2] + off[b]], xp[pb[3] + off[b]]};
          const f32x4 v1 = {xp[pb[4] + off[b]], xp[pb[5] + off[b]], xp[pb[6] + off[b]], xp[pb[7] + off[b]]};
          sdb::bf16x4 h0, h1, e0, e1;
          sdb::split2(v0, h0, e0);
          sdb::split2(v1, h1, e1);
          bh = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
          bl = __builtin_shufflevector(e0, e1, 0, 1, 2, 3, 4, 5, 6, 7);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          acc[i][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh, acc[i][b], 0, 0, 0);
          acc[i][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl, acc[i][b], 0, 0, 0);
          acc[i][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh, acc[i][b], 0, 0, 0);
        }
      }
    }
  }
  float* out = d.ws + (long)blockIdx.y * d.Co * (d.J + 1);
  if constexpr (WS) {  // sum the 8 waves' tiles through LDS (the staging area is free now), one 16x16 tile at a time
#pragma unroll
    for (int b = 0; b < NBW; ++b)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 4; ++r) lds[(wave * 4 + r) * 64 + lane] = acc[i][b][r];
        __syncthreads();
        if (tid < 256) {
          const int r = tid >> 6, ln = tid & 63;
          float v = 0.f;
#pragma unroll
          for (int w = 0; w < NW_D; ++w) v += lds[(w * 4 + r) * 64 + ln];
          const int j = 16 * b + (ln & 15), co = 16 * i + 4 * (ln >> 4) + r;
          if (j <= d.J && co < d.Co) out[(long)co * (d.J + 1) + j] = v;
        }
      }
    return;
  }
#pragma unroll
  for (int b = 0; b < NBW; ++b) {
    const int j = 16 * ((blockIdx.x * NW_D + wave) * NBW + b) + l16;
    if (j <= d.J) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = 16 * i + 4 * q + r;
          if (co < d.Co) out[(long)co * (d.J + 1) + j] = acc[i][b][r];
        }
    }
  }
}

// SDHIP_CONV_ALGO (benchmarking knob): 0 = auto, 1 = 32x32-tile kernels only, 2 = 16x16 kernels where eligible
int conv_algo() {
  static int a = -1;
  if (a < 0) {
    const char* e = getenv("SDHIP_CONV_ALGO");
    a = e ? atoi(e) : 0;
  }
  return a;
}

// SDHIP_CONV_ES (benchmarking knob): 1 (default) = 16x16 conv kernels on the early-store main loop with buffer-load
// operands, 0 = the double-buffered main loop with branchy loaders
bool conv_es() {
  static int a = -1;
  if (a < 0) {
    const char* e = getenv("SDHIP_CONV_ES");
    a = e ? atoi(e) : 1;
  }
  return a != 0;
}

int ilog2_exact(int v) {  // log2(v) if v is a power of two, else -1
  if (v <= 0 || (v & (v - 1))) return -1;
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

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

// COMPACT: dx is the pooled-resolution gradient (Nb, H/2, W/2, C) for sd_conv2d_wgrad_pool (no window scatter)
template <int T, int VPT, bool COMPACT = false>
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
        if constexpr (COMPACT) {
          dx[pix * C + c] = dp;
        } else {
          const int bi = amax[pix * C + c];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int yy = 2 * yo + (q >> 1), xx = 2 * xo + (q & 1);
            dx[(((long)n * H + yy) * W + xx) * C + c] = q == bi ? dp : 0.f;
          }
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
// host side of the direct bwd-weight: row-block size, j blocking, split count (shared with the workspace query)
struct DirectPlan {
  int R, nbw, gx, gy, slabs;
  bool ws;
  size_t lds;
};
int patch_stride(int Ci) {  // >= Ci + 2 (ones / zero channels), % 4 == 0, 16 or 48 (mod 64) for wide Ci
  if (Ci < 16) return (Ci + 2 + 3) / 4 * 4;
  int c = (Ci + 2 + 15) / 16 * 16;
  while (c % 64 != 16 && c % 64 != 48) c += 16;
  return c;
}

// pixels per staged row block of the max-pool-fused f32 direct bwd-weight (encoder first stage): more pixels per
// block = more MFMA steps per barrier (128 / 256 / 512 px: 397 / 337 / 305 us at 1024 images; default 512, falling
// back to smaller blocks where the staging does not fit, pool_plan); SDHIP_WGRAD_PIX overrides
int wgrad_pool_pix() {
  static int a = -1;
  if (a < 0) {
    const char* e = getenv("SDHIP_WGRAD_PIX");
    a = e ? atoi(e) : 512;
    if (a < 1) a = 512;
  }
  return a;
}

// pool_pix > 0: dy arrives at pooled resolution (a quarter of the block's pixels are fetched), blocks of pool_pix px
bool direct_plan(int Nb, int H, int W, int Ci, int Co, int kh, int kw, int ups, DirectPlan& pl, int pool_pix = 0) {
  const bool pool = pool_pix > 0;
  if (conv_algo() != 0 || ups != 0 || Co % 16 || Co > 64 || Ci % 4 || ilog2_exact(W) < 0) return false;
  const int pix = pool ? pool_pix : 128;
  pl.R = W >= pix ? 1 : (pix / W < H ? pix / W : H);
  if (H % pl.R || (pl.R * W) % 4) return false;
  const int SA = Co % 32 == 0 ? Co + 16 : Co, CP = patch_stride(Ci);
  const int PH = pl.R + kh - 1, PW = W + kw - 1;
  pl.lds = ((size_t)pl.R * W * SA + (size_t)PH * PW * CP) * 4;
  if (pl.lds > 160 * 1024) return false;
  if (pl.R * W * Co / (pool ? 16 : 4) > WD_VA * 512 || PH * PW * (Ci / 4) > WD_VP * 512) return false;
  const int J = kh * kw * Ci, JB = (J + 1 + 15) / 16;
  pl.ws = JB <= 7;  // few column blocks: split the pixels over the waves instead
  pl.nbw = pl.ws ? 7 : JB <= 16 ? 2 : JB <= 32 ? 4 : JB <= 56 ? 7 : (Co <= 48 ? 10 : 7);
  pl.gx = pl.ws ? 1 : (JB + NW_D * pl.nbw - 1) / (NW_D * pl.nbw);
  const int blocks = Nb * (H / pl.R);
  pl.gy = 256 / pl.gx;
  if (pl.gy > blocks) pl.gy = blocks;
  if (pl.gy < 1) pl.gy = 1;
  pl.slabs = pl.gy;
  return true;
}

int wgrad_direct(const float* in, const float* dout, float* dw_db, float* ws, long ws_floats, int Nb, int H, int W,
                 int Ci, int Co, int kh, int kw, int pad, int J, int lw, const DirectPlan& pl, hipStream_t s,
                 const uint8_t* amax, sd_wgrad_acc acc) {
  DirectW d;
  d.x = in; d.dy = dout; d.amax = amax; d.Nb = Nb; d.H = H; d.W = W; d.Ci = Ci; d.Co = Co; d.kh = kh; d.kw = kw; d.pad = pad;
  d.lw = lw; d.J = J; d.R = pl.R;
  d.PW = W + kw - 1; d.PH = d.R + kh - 1;
  d.SA = Co % 32 == 0 ? Co + 16 : Co;
  d.CP = patch_stride(Ci);
  d.blocks = Nb * (H / d.R);
  const size_t lds = pl.lds;
  const int nbw = pl.nbw, gx = pl.gx, gy = pl.gy;
  if (!ws || ws_floats < (long)pl.slabs * Co * (J + 1)) return SD_EARG;
  d.ws = ws;
  const dim3 grid(gx, gy);
  const int TM = Co / 16;
#define SD_WD_PL(TM_, NB_, WS_, PL_)                                                                       \
  if (TM == TM_ && nbw == NB_ && pl.ws == WS_ && (amax != nullptr) == PL_) {                               \
    static bool raised = false;                                                                            \
    if (!raised && lds > 65536) {                                                                          \
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(conv_wgrad_direct<TM_, NB_, WS_, PL_>),        \
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)       \
        return SD_EARG;                                                                                    \
      raised = true;                                                                                       \
    }                                                                                                      \
    conv_wgrad_direct<TM_, NB_, WS_, PL_><<<grid, 512, lds, s>>>(d);                                       \
    launched = true;                                                                                       \
  }
#define SD_WD(TM_, NB_, WS_) SD_WD_PL(TM_, NB_, WS_, false)
  bool launched = false;
  SD_WD(1, 7, true) SD_WD(2, 7, true) SD_WD(3, 7, true) SD_WD(4, 7, true)
  SD_WD_PL(1, 7, true, true) SD_WD_PL(2, 7, true, true) SD_WD_PL(3, 7, true, true) SD_WD_PL(4, 7, true, true)
  SD_WD(1, 2, false) SD_WD(1, 4, false) SD_WD(1, 7, false) SD_WD(1, 10, false)
  SD_WD(2, 2, false) SD_WD(2, 4, false) SD_WD(2, 7, false) SD_WD(2, 10, false)
  SD_WD(3, 2, false) SD_WD(3, 4, false) SD_WD(3, 7, false) SD_WD(3, 10, false)
  SD_WD(4, 2, false) SD_WD(4, 4, false) SD_WD(4, 7, false)
#undef SD_WD
#undef SD_WD_PL
  if (!launched) return SD_ESHAPE;
  SD_LAUNCH_CHECK();
  const long total = (long)Co * (J + 1);  // fixed-order sum of the row-block slabs (4 waves x unrolled loads)
  slab_reduce<<<(int)((total + 63) / 64), 256, 0, s>>>(ws, pl.slabs, total, dw_db, acc, J, Ci);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

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
  const bool va = (Ci % 4 == 0) && al16(in) && vb;
  const int lw = ilog2_exact(G.Wg), lhw = ilog2_exact(G.Hg * G.Wg);
  if (conv_algo() != 1 && va && lw >= 0 && lhw >= 0 && g.K / 4 <= MAX_TAPQ &&
      (Co == 32 || Co == 48 || Co == 64 || Co == 16)) {
    const dim3 grid(sd_cdiv(g.M, 128));
    const bool es = conv_es() && (long)Nb * Hs * Ws * Ci < (1L << 29);  // buffer offsets < 2 GiB
#define SD_FWD16(BN) (es ? conv_fwd16<BN, true><<<grid, 256, 0, s>>>(g, G, lw, lhw) \
                         : conv_fwd16<BN, false><<<grid, 256, 0, s>>>(g, G, lw, lhw))
    switch (Co) {
      case 16: SD_FWD16(16); break;
      case 32: SD_FWD16(32); break;
      case 48: SD_FWD16(48); break;
      default: SD_FWD16(64); break;
    }
#undef SD_FWD16
  } else if (Co <= 32) fwd_tile<128, 32, 32, 32>(g, G, va, vb, s);
  else fwd_tile<128, 64, 64, 32>(g, G, va, vb, s);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

// dw_db (Co, kh*kw*Ci + 1) = [dW | d bias] = sum over pixels of dout (Nb,Hg,Wg,Co) x im2col(in)
// fused ConvEncoder stage forward; SD_ESHAPE when the shape is outside the fused kernel (caller: conv + pool)
extern "C" int sd_conv2d_fwd_pool(const float* in, const float* w, const float* bias, const float* nw, float* pooled,
                                  uint8_t* amax, float* y, float* rstd, int Nb, int Hs, int Ws, int Ci, int Co, int kh,
                                  int kw, int pad, float eps, int nchw_flat, sd_stream stream_) {
  hipStream_t s = (hipStream_t)stream_;
  if (Nb <= 0) return SD_OK;
  Geom G{in, Nb, Hs, Ws, Ci, Hs, Ws, kh, kw, pad, 0};
  GemmArgs g{};
  g.B = w; g.bias = bias; g.ldb = (long)kh * kw * Ci; g.ldc = Co;
  g.M = Nb * Hs * Ws; g.N = Co; g.K = kh * kw * Ci; g.batch = 1; g.ksplit = 1; g.kchunk = g.K;
  g.alpha = 1.f; g.beta = 0.f;
  const bool vb = (((long)kh * kw * Ci) % 4 == 0) && al16(w);
  const bool va = (Ci % 4 == 0) && al16(in) && vb;
  const int lw = ilog2_exact(Ws), lhw = ilog2_exact(Hs * Ws);
  if (conv_algo() == 1 || !va || lw < 1 || lhw < 0 || g.K / 4 > MAX_TAPQ || Hs % 2 || 128 % (2 * Ws) ||
      g.M % 128)
    return SD_ESHAPE;
  const dim3 grid(g.M / 128);
  const bool es = conv_es() && (long)Nb * Hs * Ws * Ci < (1L << 29);  // buffer offsets < 2 GiB
  if (conv_direct_fwd() && es && Co == 48 && Ci == 32 && Ws == 32 && kh == 5 && kw == 5 && pad == 2 &&
      Hs % 4 == 0 && al16(in)) {
    const char* e = getenv("SDHIP_C32_TPW");
    const int tpw = e ? atoi(e) : 1;
#define SD_C32(TPW)                                                                                                \
  conv_fwd_direct_pool<48, 32, 5, 5, TPW><<<sd_cdiv(g.M / 128, TPW), 256, 0, s>>>(g, G, lhw, nw, pooled, amax, y, \
                                                                                 rstd, eps, nchw_flat)
    if (tpw == 4) SD_C32(4);
    else if (tpw == 1) SD_C32(1);
    else SD_C32(2);
#undef SD_C32
    SD_LAUNCH_CHECK();
    return SD_OK;
  }
  if (conv_direct_fwd() && es && Co == 32 && Ci == 4 && Ws == 64 && kh == 5 && kw == 5 && pad == 2 &&
      Hs % 2 == 0 && al16(in)) {
    // SDHIP_C4_TPW = n > 0: n tiles per workgroup (the round-5 default was 16: 2048 workgroups, 2.67 rounds of
    // the 768 then resident); default 0 = one round of resident workgroups (SDHIP_C4_OCC per CU, default 4).
    const char* e = getenv("SDHIP_C4_TPW");
    const char* eo = getenv("SDHIP_C4_OCC");
    const int occ = eo ? atoi(eo) : 4, tiles = g.M / 128;
    int tpw = e ? atoi(e) : 0;
    if (tpw <= 0) tpw = sd_cdiv(tiles, 256 * (occ > 0 ? occ : 4));
    const int nwg = sd_cdiv(tiles, tpw);
    conv_fwd_direct_pool_c4<32, 6, 5, 4><<<nwg, 256, 0, s>>>(g, G, lhw, tpw, nw, pooled, amax, y, rstd, eps,
                                                             nchw_flat);
    SD_LAUNCH_CHECK();
    return SD_OK;
  }
#define SD_FWDP(BN)                                                                                          \
  (es ? conv_fwd16_pool<BN, true><<<grid, 256, 0, s>>>(g, G, lw, lhw, nw, pooled, amax, y, rstd, eps, nchw_flat) \
      : conv_fwd16_pool<BN, false><<<grid, 256, 0, s>>>(g, G, lw, lhw, nw, pooled, amax, y, rstd, eps, nchw_flat))
  switch (Co) {
    case 16: SD_FWDP(16); break;
    case 32: SD_FWDP(32); break;
    case 48: SD_FWDP(48); break;
    case 64: SD_FWDP(64); break;
    default: return SD_ESHAPE;
  }
#undef SD_FWDP
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_conv2d_wgrad(const float* in, const float* dout, float* dw_db, float* workspace, long ws_floats,
                               int ksplit, int Nb, int Hs, int Ws, int Ci, int Co, int kh, int kw, int pad, int ups,
                               const sd_wgrad_acc* acc_p, sd_stream stream_) {
  hipStream_t s = (hipStream_t)stream_;
  if (Nb <= 0) return SD_OK;
  const sd_wgrad_acc acc = acc_p ? *acc_p : sd_wgrad_acc{nullptr, nullptr, 0};
  if (acc.dw && (!acc.db || acc.ci_w < 1 || acc.ci_w > Ci || !dw_db)) return SD_EARG;
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
  const int lw = ilog2_exact(G.Wg), lhw = ilog2_exact(G.Hg * G.Wg);
  DirectPlan pl;
  if (va && vb && direct_plan(Nb, Hs, Ws, Ci, Co, kh, kw, ups, pl))
    return wgrad_direct(in, dout, dw_db, workspace, ws_floats, Nb, Hs, Ws, Ci, Co, kh, kw, pad, J, lw, pl, s, nullptr,
                        acc);
  if (conv_algo() == 2 && va && vb && lw >= 0 && lhw >= 0 && (Co == 16 || Co == 32 || Co == 48 || Co == 64)) {
    const dim3 grid(sd_cdiv(g.N, 128), 1, ks);
    switch (Co) {
      case 16: conv_wgrad16<16><<<grid, 256, 0, s>>>(g, G, J, lw, lhw); break;
      case 32: conv_wgrad16<32><<<grid, 256, 0, s>>>(g, G, J, lw, lhw); break;
      case 48: conv_wgrad16<48><<<grid, 256, 0, s>>>(g, G, J, lw, lhw); break;
      default: conv_wgrad16<64><<<grid, 256, 0, s>>>(g, G, J, lw, lhw); break;
    }
  } else if (Co <= 32) wgrad_tile<32, 128, 32, 32>(g, G, J, va, vb, s);
  else wgrad_tile<64, 64, 32, 32>(g, G, J, va, vb, s);
  SD_LAUNCH_CHECK();
  if (ks > 1) {
    long total = (long)g.M * g.N;
    int blocks = (int)((total + 255) / 256);
    gemm_reduce_kernel<<<blocks, 256, 0, s>>>(g);
    SD_LAUNCH_CHECK();
  }
  if (acc.dw) {  // the implicit-GEMM path wrote dw_db: one pass adds it into the gradients
    const long total = (long)Co * (J + 1);
    slab_reduce<<<(int)((total + 63) / 64), 256, 0, s>>>(dw_db, 1, total, nullptr, acc, J, Ci);
    SD_LAUNCH_CHECK();
  }
  return SD_OK;
}

// number of partial slabs (each Co x (kh*kw*Ci+1) floats) sd_conv2d_wgrad will use with this `ksplit` request
extern "C" int sd_conv2d_wgrad_slabs(int Nb, int Hs, int Ws, int Ci, int Co, int kh, int kw, int ups, int ksplit) {
  DirectPlan pl;
  if (direct_plan(Nb, Hs, Ws, Ci, Co, kh, kw, ups, pl)) return pl.slabs;
  return ksplit < 1 ? 1 : ksplit;
}

// the pooled plan at the largest block (<= wgrad_pool_pix()) whose staging fits
static bool pool_plan(int Nb, int H, int W, int Ci, int Co, int kh, int kw, DirectPlan& pl) {
  if (H % 2 || W % 2) return false;
  for (int pix = wgrad_pool_pix(); pix >= 128; pix /= 2)
    if (direct_plan(Nb, H, W, Ci, Co, kh, kw, 0, pl, pix) && pl.ws && pl.nbw == 7 && pl.R % 2 == 0) return true;
  return false;
}
// bwd-weight of a pooled stage straight from the max-pool backward's pooled-resolution gradient + argmax
// (sd_pool_rms_bwd_compact): the direct f32 kernel expands it while staging. SD_ESHAPE outside the direct plan.
extern "C" int sd_conv2d_wgrad_pool_slabs(int Nb, int H, int W, int Ci, int Co, int kh, int kw) {
  DirectPlan pl;
  if (!pool_plan(Nb, H, W, Ci, Co, kh, kw, pl)) return 0;
  return pl.slabs;
}
extern "C" int sd_conv2d_wgrad_pool(const float* in, const float* dpool, const uint8_t* amax, float* dw_db,
                                    float* workspace, long ws_floats, int Nb, int H, int W, int Ci, int Co, int kh,
                                    int kw, int pad, const sd_wgrad_acc* acc_p, sd_stream stream_) {
  if (Nb <= 0) return SD_OK;
  const sd_wgrad_acc acc = acc_p ? *acc_p : sd_wgrad_acc{nullptr, nullptr, 0};
  if (acc.dw && (!acc.db || acc.ci_w < 1 || acc.ci_w > Ci)) return SD_EARG;
  DirectPlan pl;
  if (!pool_plan(Nb, H, W, Ci, Co, kh, kw, pl))
    return SD_ESHAPE;
  // amax is read as uint32 words (4 pooled pixels' argmax bytes per load)
  if (!al16(dpool) || !al16(in) || Co % 4 || Ci % 4 || !amax || reinterpret_cast<uintptr_t>(amax) % 4) return SD_EARG;
  return wgrad_direct(in, dpool, dw_db, workspace, ws_floats, Nb, H, W, Ci, Co, kh, kw, pad, kh * kw * Ci,
                      ilog2_exact(W), pl, (hipStream_t)stream_, amax, acc);
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
  // two-pass column sum of the per-block dw partials; its chunk workspace follows them in dw_partial
  return sd_colsum_ws(dw_partial, dw, grid, C, C, accumulate_dw, dw_partial + (long)grid * C, stream_);
}

extern "C" int sd_pool_rms_bwd_compact(const float* pooled, const uint8_t* amax, const float* w, const float* rstd,
                                       const float* dy, float* dpool, float* dw, float* dw_partial, int Nb, int H,
                                       int W, int C, int nchw_flat, int accumulate_dw, sd_stream stream_) {
  hipStream_t s = (hipStream_t)stream_;
  if (C > 128) return SD_ESHAPE;
  const int grid = sd_pool_rms_bwd_blocks(Nb, H, W);
  switch (vpt_for(C, 16)) {
    case 1: pool_rms_bwd<16, 1, true><<<grid, 256, 0, s>>>(pooled, amax, w, rstd, dy, dpool, dw_partial, Nb, H, W, C, nchw_flat); break;
    case 2: pool_rms_bwd<16, 2, true><<<grid, 256, 0, s>>>(pooled, amax, w, rstd, dy, dpool, dw_partial, Nb, H, W, C, nchw_flat); break;
    case 4: pool_rms_bwd<16, 4, true><<<grid, 256, 0, s>>>(pooled, amax, w, rstd, dy, dpool, dw_partial, Nb, H, W, C, nchw_flat); break;
    default: pool_rms_bwd<16, 8, true><<<grid, 256, 0, s>>>(pooled, amax, w, rstd, dy, dpool, dw_partial, Nb, H, W, C, nchw_flat); break;
  }
  SD_LAUNCH_CHECK();
  return sd_colsum_ws(dw_partial, dw, grid, C, C, accumulate_dw, dw_partial + (long)grid * C, stream_);
}

// ---------------------------------------------------------------- split-bf16 backward entry points
namespace {
}  // namespace


namespace {
// SDHIP_WGRAD3_CI4 (study knob): the split-bf16 direct bwd-weight also for 4-channel inputs (the encoder's first
// stage, which otherwise stays on the f32 direct kernel) — to measure that stage's gradient parity on split-bf16
bool wgrad3_ci4() {
  static int a = -1;
  if (a < 0) a = getenv("SDHIP_WGRAD3_CI4") ? 1 : 0;
  return a == 1;
}
bool direct3_plan(int Nb, int H, int W, int Ci, int Co, int kh, int kw, int ups, DirectPlan& pl) {
  if (ups != 0 || Co % 4 || Co > 64 || Ci % 4 || Ci < (wgrad3_ci4() ? 4 : 16) || W < 8 || ilog2_exact(W) < 0 ||
      W > 128)
    return false;
  pl.R = 128 / W < H ? 128 / W : H;
  const int P = pl.R * W;
  if (H % pl.R || P % 32) return false;
  const int TM = (Co + 15) / 16, CP = patch_stride(Ci);
  const int PH = pl.R + kh - 1, PW = W + kw - 1;
  pl.lds = (size_t)PH * PW * CP * 4 + (size_t)TM * 16 * (P + 8) * 2 * 2;
  if (pl.lds > 160 * 1024 || PH * PW * (Ci / 4) > WD_VP * 512 || (Co / 4) * (P / 4) > 512) return false;
  const int J = kh * kw * Ci, JB = (J + 1 + 15) / 16;
  pl.ws = false;
  // column blocks per wave: the accumulators (TM * NBW * 4 VGPRs) bound it; SDHIP_WGRAD3_NBW overrides (tuning knob)
  static int nbw_env = -1;
  if (nbw_env < 0) {
    const char* e = getenv("SDHIP_WGRAD3_NBW");
    nbw_env = e ? atoi(e) : 0;
  }
  const int nmax = nbw_env > 0 ? nbw_env : (TM <= 3 ? 7 : 4);
  pl.gx = (JB + NW_D * nmax - 1) / (NW_D * nmax);
  const int need = (JB + NW_D * pl.gx - 1) / (NW_D * pl.gx);
  pl.nbw = need <= 2 ? 2 : need <= 4 ? 4 : need <= 5 ? 5 : 7;
  const int blocks = Nb * (H / pl.R);
  pl.gy = 256 / pl.gx;
  if (pl.gy > blocks) pl.gy = blocks;
  if (pl.gy < 1) pl.gy = 1;
  pl.slabs = pl.gy;
  return true;
}

// the first stage's plan for conv_wgrad3_direct<TM, 7, WS, PL>: dy at pooled resolution (R even), every wave over
// all <= 7 column blocks (J + 1 <= 112), 32-pixel steps dealt to the 8 waves: R rows of W pixels with 8 steps per
// block (P = 256), one 4-channel x 4-pixel dy item per thread ((Co / 4) (P / 4) <= 512)
bool pool3_plan(int Nb, int H, int W, int Ci, int Co, int kh, int kw, DirectPlan& pl) {
  if (Co % 4 || Co > 64 || Ci % 4 || W < 8 || ilog2_exact(W) < 0 || W > 256 || H % 2) return false;
  const int J = kh * kw * Ci, JB = (J + 1 + 15) / 16;
  if (JB > 7) return false;
  pl.R = 256 / W;
  if (pl.R < 2 || pl.R % 2 || H % pl.R) return false;
  const int P = pl.R * W, TM = (Co + 15) / 16, CP = patch_stride(Ci);
  const int PH = pl.R + kh - 1, PW = W + kw - 1;
  if ((Co / 4) * (P / 4) > 512 || PH * PW * (Ci / 4) > WD_VP * 512) return false;
  pl.lds = (size_t)PH * PW * CP * 4 + (size_t)TM * 16 * (P + 8) * 2 * 2;
  if (pl.lds > 160 * 1024) return false;
  pl.ws = true;
  pl.nbw = 7;
  pl.gx = 1;
  const int blocks = Nb * (H / pl.R);
  pl.gy = blocks < 256 ? blocks : 256;
  pl.slabs = pl.gy;
  return true;
}

int wgrad3_direct(const float* in, const float* dout, float* dw_db, float* ws, long ws_floats, int Nb, int H, int W,
                  int Ci, int Co, int kh, int kw, int pad, const DirectPlan& pl, hipStream_t s, sd_wgrad_acc acc,
                  const uint8_t* amax = nullptr) {
  DirectW3 d;
  d.x = in; d.dy = dout; d.amax = amax; d.Nb = Nb; d.H = H; d.W = W; d.Ci = Ci; d.Co = Co; d.kh = kh; d.kw = kw;
  d.pad = pad;
  d.lw = ilog2_exact(W); d.J = kh * kw * Ci; d.R = pl.R;
  d.PW = W + kw - 1; d.PH = d.R + kh - 1;
  d.CP = patch_stride(Ci);
  d.PS = d.R * W + 8;
  d.blocks = Nb * (H / d.R);
  if (!ws || ws_floats < (long)pl.slabs * Co * (d.J + 1)) return SD_EARG;
  d.ws = ws;
  const dim3 grid(pl.gx, pl.gy);
  const int TM = (Co + 15) / 16;
  bool launched = false;
#define SD_WD3X(TM_, NB_, WS_, PL_)                                                                        \
  if (TM == TM_ && pl.nbw == NB_ && pl.ws == WS_ && (amax != nullptr) == PL_) {                            \
    static bool raised = false;                                                                            \
    if (!raised && pl.lds > 65536) {                                                                       \
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(conv_wgrad3_direct<TM_, NB_, WS_, PL_>),       \
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)       \
        return SD_EARG;                                                                                    \
      raised = true;                                                                                       \
    }                                                                                                      \
    conv_wgrad3_direct<TM_, NB_, WS_, PL_><<<grid, 512, pl.lds, s>>>(d);                                  \
    launched = true;                                                                                       \
  }
#define SD_WD3(TM_, NB_) SD_WD3X(TM_, NB_, false, false)
  SD_WD3(1, 2) SD_WD3(1, 4) SD_WD3(1, 5) SD_WD3(1, 7)
  SD_WD3(2, 2) SD_WD3(2, 4) SD_WD3(2, 5) SD_WD3(2, 7)
  SD_WD3(3, 2) SD_WD3(3, 4) SD_WD3(3, 5) SD_WD3(3, 7)
  SD_WD3(4, 2) SD_WD3(4, 4) SD_WD3(4, 5) SD_WD3(4, 7)
  SD_WD3X(1, 7, true, true) SD_WD3X(2, 7, true, true) SD_WD3X(3, 7, true, true) SD_WD3X(4, 7, true, true)
#undef SD_WD3
#undef SD_WD3X
  if (!launched) return SD_ESHAPE;
  SD_LAUNCH_CHECK();
  const long n = (long)Co * (d.J + 1);
  slab_reduce<<<(int)((n + 63) / 64), 256, 0, s>>>(ws, pl.slabs, n, dw_db, acc, d.J, Ci);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
}  // namespace

extern "C" int sd_conv2d_dgrad_bf16x3(const float* dout, const float* wflip, float* din, int Nb, int Hs, int Ws,
                                      int Ci, int Co, int kh, int kw, int pad, sd_stream stream_) {
  hipStream_t s = (hipStream_t)stream_;
  if (Nb <= 0) return SD_OK;
  Geom G{dout, Nb, Hs, Ws, Ci, Hs, Ws, kh, kw, pad, 0};
  GemmArgs g{};
  g.B = wflip; g.C = din; g.ldb = (long)kh * kw * Ci; g.ldc = Co;
  g.M = Nb * Hs * Ws; g.N = Co; g.K = kh * kw * Ci; g.batch = 1; g.ksplit = 1; g.kchunk = g.K;
  g.alpha = 1.f; g.beta = 0.f;
  const int lw = ilog2_exact(Ws), lhw = ilog2_exact(Hs * Ws);
  if (Ci % 4 || !al16(dout) || !al16(wflip) || lw < 0 || lhw < 0 || g.K / 4 > MAX_TAPQ ||
      (long)Nb * Hs * Ws * Ci >= (1L << 29))
    return SD_ESHAPE;
  const dim3 grid(sd_cdiv(g.M, 128));
  switch (Co) {
    case 16: conv_dgrad3<16><<<grid, 256, 0, s>>>(g, G, lw, lhw); break;
    case 32: conv_dgrad3<32><<<grid, 256, 0, s>>>(g, G, lw, lhw); break;
    case 48: conv_dgrad3<48><<<grid, 256, 0, s>>>(g, G, lw, lhw); break;
    case 64: conv_dgrad3<64><<<grid, 256, 0, s>>>(g, G, lw, lhw); break;
    default: return SD_ESHAPE;
  }
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_conv_split3_weight(const float* w, void* wsplit, int rows, int K, sd_stream stream_) {
  if (rows <= 0 || K <= 0 || !w || !wsplit) return SD_EARG;
  const int KP = (K + 31) / 32 * 32;
  const long total = (long)rows * KP;
  split3_weight<<<(int)((total + 255) / 256), 256, 0, (hipStream_t)stream_>>>(w, static_cast<__bf16*>(wsplit), rows,
                                                                               K, KP);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

namespace {
// SDHIP_CONV6_RING=0: the per-lane-weight kernel (conv_fwd6_direct_pool) instead of the LDS-ring one (A/B knob)
bool conv6_ring() {  // read per call (host only): tests toggle it in-process
  const char* e = getenv("SDHIP_CONV6_RING");
  return e ? atoi(e) != 0 : true;
}
// SDHIP_CONV6_PIPE=1: the ring kernel with the fragment register pipeline, one tile per workgroup (A/B knob; 1 %
// faster alone than without it, profiles/r06s3b, and slower than the prefetching multi-tile workgroups)
bool conv6_pipe() {
  const char* e = getenv("SDHIP_CONV6_PIPE");
  return e ? atoi(e) != 0 : false;
}
template <int BN, int CI, int LW, int KS, bool CG, bool PIPE, int TPW, int MT = 2, int BROW = 40, int NTH = 512>
int fwd6r_launch_t(const GemmArgs& g, const Geom& G, int lhw, const __bf16* wsp, const float* nw, float* pooled,
                   uint8_t* amax, float* y, float* rstd, float eps, int nchw_flat, size_t lds, hipStream_t s) {
  static bool raised = false;
  if (!raised) {
    if (hipFuncSetAttribute(
            reinterpret_cast<const void*>(conv_fwd6r_direct_pool<BN, CI, LW, KS, CG, PIPE, TPW, MT, BROW, NTH>),
            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return SD_EARG;
    raised = true;
  }
  const int nwg = (sd_cdiv(g.M / (16 * MT * (NTH / 64)), TPW) + 7) / 8 * 8;  // a multiple of 8: XCD-contiguous
  conv_fwd6r_direct_pool<BN, CI, LW, KS, CG, PIPE, TPW, MT, BROW, NTH><<<nwg, NTH, lds, s>>>(
      g, G, lhw, wsp, nw, pooled, amax, y, rstd, eps, nchw_flat);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
// SDHIP_CONV6_TPW: tiles per workgroup (1, 2, 4, 8, 16); default: enough for one workgroup per CU, at most 16.
// (The fragment pipeline, SDHIP_CONV6_PIPE=1, runs one tile per workgroup: with the prefetched patch it spills.)
template <int BN, int CI, int LW, int KS, bool CG>
int fwd6r_launch(const GemmArgs& g, const Geom& G, int lhw, const __bf16* wsp, const float* nw, float* pooled,
                 uint8_t* amax, float* y, float* rstd, float eps, int nchw_flat, size_t lds, hipStream_t s) {
  if (conv6_pipe())
    return fwd6r_launch_t<BN, CI, LW, KS, CG, true, 1>(g, G, lhw, wsp, nw, pooled, amax, y, rstd, eps, nchw_flat, lds,
                                                       s);
  // the 32 -> 48 stage: 512-pixel tiles, 64 pixels per wave, channel-group-major patch, packed ring (356 vs 392 us
  // alone, profiles/r06mt4), one tile per workgroup by default (its prefetch registers spill: 386 us); SDHIP_CONV6_MT=2:
  // the 256-pixel tiles
  if constexpr (CI == 32 && BN == 48) {
    const char* m = getenv("SDHIP_CONV6_MT");
    constexpr int R4 = 512 / (1 << LW);
    constexpr size_t lds4 = (size_t)3 * (R4 + KS - 1) * ((1 << LW) + KS - 1) * CI * 2 + (size_t)2 * 3 * BN * 32 * 2;
    if ((!m || atoi(m) == 4) && lds4 <= 160 * 1024 && g.M % 512 == 0 && G.Hs % R4 == 0) {
      const char* e = getenv("SDHIP_CONV6_TPW");
      const int want = e ? atoi(e) : 1;
#define SD_F6R4(T) \
  fwd6r_launch_t<BN, CI, LW, KS, true, false, T, 4, 32>(g, G, lhw, wsp, nw, pooled, amax, y, rstd, eps, nchw_flat, \
                                                        lds4, s)
      return want <= 1 ? SD_F6R4(1) : want <= 4 ? SD_F6R4(4) : SD_F6R4(8);
#undef SD_F6R4
    }
  }
  const char* e = getenv("SDHIP_CONV6_TPW");
  const int want = e ? atoi(e) : sd_cdiv(g.M / 256, 256);
#define SD_F6R(T) \
  fwd6r_launch_t<BN, CI, LW, KS, CG, false, T>(g, G, lhw, wsp, nw, pooled, amax, y, rstd, eps, nchw_flat, lds, s)
  return want <= 1 ? SD_F6R(1) : want <= 2 ? SD_F6R(2) : want <= 4 ? SD_F6R(4) : want <= 8 ? SD_F6R(8) : SD_F6R(16);
#undef SD_F6R
}
template <int BN, int CI, int LW>
int fwd6_launch(const GemmArgs& g, const Geom& G, int lhw, const __bf16* wsp, const float* nw, float* pooled,
                uint8_t* amax, float* y, float* rstd, float eps, int nchw_flat, hipStream_t s) {
  constexpr int W = 1 << LW, R = 128 / W, KS = 5;
  constexpr int R2 = 256 / W;
  // pixel-major patch with its pad where it fits (stage 2), channel-group-major otherwise (stage 3: 165 vs 146 KB)
  constexpr bool CG = (size_t)3 * (R2 + KS - 1) * (W + KS - 1) * (CI + 8) * 2 + (size_t)2 * 3 * BN * 40 * 2 > 160 * 1024;
  constexpr size_t lds2 =
      (size_t)3 * (R2 + KS - 1) * (W + KS - 1) * (CG ? CI : CI + 8) * 2 + (size_t)2 * 3 * BN * 40 * 2;
  if (conv6_ring() && lds2 <= 160 * 1024 && g.M % 256 == 0 && G.Hs % R2 == 0)
    return fwd6r_launch<BN, CI, LW, KS, CG>(g, G, lhw, wsp, nw, pooled, amax, y, rstd, eps, nchw_flat, lds2, s);
  const size_t lds = (size_t)3 * (R + KS - 1) * (W + KS - 1) * (CI + 8) * 2;
  static bool raised = false;
  if (!raised && lds > 65536) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(conv_fwd6_direct_pool<BN, CI, LW, KS>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return SD_EARG;
    raised = true;
  }
  conv_fwd6_direct_pool<BN, CI, LW, KS><<<g.M / 128, 256, lds, s>>>(g, G, lhw, wsp, nw, pooled, amax, y, rstd, eps,
                                                                   nchw_flat);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
}  // namespace

extern "C" int sd_conv2d_fwd_pool6(const float* in, const void* wsplit3, const float* bias, const float* nw,
                                   float* pooled, uint8_t* amax, float* y, float* rstd, int Nb, int Hs, int Ws, int Ci,
                                   int Co, int kh, int kw, int pad, float eps, int nchw_flat, sd_stream stream_) {
  hipStream_t s = (hipStream_t)stream_;
  if (Nb <= 0) return SD_OK;
  if (kh != 5 || kw != 5 || pad != 2 || Hs != Ws || Hs % 2 || !al16(in) || !al16(wsplit3)) return SD_ESHAPE;
  Geom G{in, Nb, Hs, Ws, Ci, Hs, Ws, kh, kw, pad, 0};
  GemmArgs g{};
  g.bias = bias; g.M = Nb * Hs * Ws; g.N = Co; g.K = kh * kw * Ci;
  const int lhw = ilog2_exact(Hs * Ws);
  if (lhw < 0 || g.M % 128) return SD_ESHAPE;
  const __bf16* wsp = static_cast<const __bf16*>(wsplit3);
  // a 128-pixel tile is 128 / Ws whole rows of one image
  if (Co == 48 && Ci == 32 && Ws == 32)
    return fwd6_launch<48, 32, 5>(g, G, lhw, wsp, nw, pooled, amax, y, rstd, eps, nchw_flat, s);
  if (Co == 64 && Ci == 48 && Ws == 16)
    return fwd6_launch<64, 48, 4>(g, G, lhw, wsp, nw, pooled, amax, y, rstd, eps, nchw_flat, s);
  return SD_ESHAPE;
}

extern "C" int sd_conv_split_weight(const float* w, void* wsplit, int rows, int K, sd_stream stream_) {
  if (rows <= 0 || K <= 0 || !w || !wsplit) return SD_EARG;
  const int KP = (K + 31) / 32 * 32;
  const long total = (long)rows * KP;
  split_weight<<<(int)((total + 255) / 256), 256, 0, (hipStream_t)stream_>>>(w, static_cast<__bf16*>(wsplit), rows, K,
                                                                              KP);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

namespace {
template <int CIN, int NT, int LW>
int dgrad_direct_launch(const float* dout, const __bf16* wsp, float* din, int Nb, int H, int pad, hipStream_t s) {
  constexpr int W = 1 << LW, R = 128 / W, KS = 5;
  const size_t lds = (size_t)2 * (R + KS - 1) * (W + KS - 1) * (CIN + 8) * 2 + (size_t)2 * 2 * (16 * NT) * 40 * 2;
  static bool raised = false;
  if (!raised && lds > 65536) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(conv_dgrad3_direct<CIN, NT, LW, KS>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return SD_EARG;
    raised = true;
  }
  conv_dgrad3_direct<CIN, NT, LW, KS><<<Nb * (H / R), 256, lds, s>>>(dout, wsp, din, Nb, H, pad);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
// 512-pixel tiles over 8 waves of 64 pixels, channel-group-major patch (one workgroup per CU); SDHIP_DGRAD_MT=2: the
// 128-pixel tiles of 32-pixel waves (two per CU)
template <int CIN, int NT, int LW>
int dgrad_direct_launch4(const float* dout, const __bf16* wsp, float* din, int Nb, int H, int pad, hipStream_t s) {
  constexpr int W = 1 << LW, R = 512 / W, KS = 5;
  constexpr size_t lds = (size_t)2 * (R + KS - 1) * (W + KS - 1) * CIN * 2 + (size_t)2 * 2 * (16 * NT) * 40 * 2;
  static_assert(lds <= 160 * 1024, "LDS");
  const char* e = getenv("SDHIP_DGRAD_MT");
  if ((e && atoi(e) == 2) || H % R) return dgrad_direct_launch<CIN, NT, LW>(dout, wsp, din, Nb, H, pad, s);
  static bool raised = false;
  if (!raised) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(conv_dgrad3_direct<CIN, NT, LW, KS, 4, true, 512>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
      return SD_EARG;
    raised = true;
  }
  conv_dgrad3_direct<CIN, NT, LW, KS, 4, true, 512><<<Nb * (H / R), 512, lds, s>>>(dout, wsp, din, Nb, H, pad);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
}  // namespace

extern "C" int sd_conv2d_dgrad_direct(const float* dout, const void* wsplit, float* din, int Nb, int Hs, int Ws,
                                      int Ci, int Co, int kh, int kw, int pad, sd_stream stream_) {
  hipStream_t s = (hipStream_t)stream_;
  if (Nb <= 0) return SD_OK;
  if (kh != 5 || kw != 5 || pad != 2 || Hs != Ws || !al16(dout) || !al16(wsplit) || !al16(din)) return SD_ESHAPE;
  const __bf16* wsp = static_cast<const __bf16*>(wsplit);
  // a workgroup takes 128 / Ws whole rows of one image
  if (Ci == 48 && Co == 32 && Ws == 32) return dgrad_direct_launch4<48, 2, 5>(dout, wsp, din, Nb, Hs, pad, s);
  if (Ci == 64 && Co == 48 && Ws == 16) {
    // whole-image 256-pixel tiles of four 64-pixel waves, channel-group-major patch (183 -> 131 us alone,
    // profiles/r06dg3); SDHIP_DGRAD3_MT=2: the 128-pixel tiles of 32-pixel waves
    const char* e = getenv("SDHIP_DGRAD3_MT");
    if (!(e && atoi(e) == 2) && Hs == 16) {
      constexpr size_t lds = (size_t)2 * 20 * 20 * 64 * 2 + (size_t)2 * 2 * 48 * 40 * 2;
      static bool raised = false;
      if (!raised) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(conv_dgrad3_direct<64, 3, 4, 5, 4, true, 256>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
          return SD_EARG;
        raised = true;
      }
      conv_dgrad3_direct<64, 3, 4, 5, 4, true, 256><<<Nb, 256, lds, s>>>(dout, wsp, din, Nb, Hs, pad);
      SD_LAUNCH_CHECK();
      return SD_OK;
    }
    return dgrad_direct_launch<64, 3, 4>(dout, wsp, din, Nb, Hs, pad, s);
  }
  return SD_ESHAPE;
}

extern "C" int sd_conv2d_wgrad_bf16x3_slabs(int Nb, int Hs, int Ws, int Ci, int Co, int kh, int kw, int ups) {
  DirectPlan pl;
  if (!direct3_plan(Nb, Hs, Ws, Ci, Co, kh, kw, ups, pl)) return SD_ESHAPE;
  return pl.slabs;
}

extern "C" int sd_conv2d_wgrad_pool_bf16x3_slabs(int Nb, int H, int W, int Ci, int Co, int kh, int kw) {
  DirectPlan pl;
  if (!pool3_plan(Nb, H, W, Ci, Co, kh, kw, pl)) return 0;
  return pl.slabs;
}
extern "C" int sd_conv2d_wgrad_pool_bf16x3(const float* in, const float* dpool, const uint8_t* amax, float* dw_db,
                                           float* workspace, long ws_floats, int Nb, int H, int W, int Ci, int Co,
                                           int kh, int kw, int pad, const sd_wgrad_acc* acc_p, sd_stream stream_) {
  if (Nb <= 0) return SD_OK;
  const sd_wgrad_acc acc = acc_p ? *acc_p : sd_wgrad_acc{nullptr, nullptr, 0};
  if (acc.dw && (!acc.db || acc.ci_w < 1 || acc.ci_w > Ci)) return SD_EARG;
  DirectPlan pl;
  if (!pool3_plan(Nb, H, W, Ci, Co, kh, kw, pl)) return SD_ESHAPE;
  if (!al16(dpool) || !al16(in) || !amax || reinterpret_cast<uintptr_t>(amax) % 4) return SD_EARG;
  return wgrad3_direct(in, dpool, dw_db, workspace, ws_floats, Nb, H, W, Ci, Co, kh, kw, pad, pl,
                       (hipStream_t)stream_, acc, amax);
}

extern "C" int sd_conv2d_wgrad_bf16x3(const float* in, const float* dout, float* dw_db, float* workspace,
                                      long ws_floats, int Nb, int Hs, int Ws, int Ci, int Co, int kh, int kw, int pad,
                                      const sd_wgrad_acc* acc_p, sd_stream stream_) {
  hipStream_t s = (hipStream_t)stream_;
  if (Nb <= 0) return SD_OK;
  const sd_wgrad_acc acc = acc_p ? *acc_p : sd_wgrad_acc{nullptr, nullptr, 0};
  if (acc.dw && (!acc.db || acc.ci_w < 1 || acc.ci_w > Ci)) return SD_EARG;
  DirectPlan pl;
  if (!direct3_plan(Nb, Hs, Ws, Ci, Co, kh, kw, 0, pl) || !al16(in) || !al16(dout)) return SD_ESHAPE;
  return wgrad3_direct(in, dout, dw_db, workspace, ws_floats, Nb, Hs, Ws, Ci, Co, kh, kw, pad, pl, s, acc);
}
