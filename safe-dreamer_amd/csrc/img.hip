// Fused imagination: Dreamer._imagine (dreamer.py:673-692) = for each of H1 steps: actor MLP on feat = [stoch, deter]
// (networks.py:313-377) -> action sample (bounded normal / one-hot) -> RSSM.img_step (rssm.py:180-187:
// Deter.forward rssm.py:36-75 + prior img_net + one-hot sample). N (= B*T) independent rows per step.
//
// 9 launches per step (the per-op path took ~28): each launch is a row-tiled fp32 MFMA contraction
// (v_mfma_f32_16x16x4_f32 via gemm16_mainloop) with
//   * A loaders that apply the previous layer's RMSNorm + SiLU while staging K-tiles into LDS — the per-row rstd
//     comes from row partial sums of squares that the PRODUCER's epilogue wrote (one float per row per 16*TN
//     output columns), so no normalised activation is ever materialised and no norm launch exists;
//   * epilogues that fuse the bias, those row partials, the GRU gate, the unimix one-hot prior sampler, and the
//     whole action branch (bounded-normal / one-hot action, action_norm, _dyn_in2 Linear + RMSNorm + SiLU);
//   * independent contractions that share an A operand grouped into one launch (actor layer 0 with _dyn_in1,
//     img_net_0 with the next step's _dyn_in0).
// Results land directly in the reference's (H1, N, F) feat and (H1, N, A) action layouts.
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "dist_core.h"
#include "gemm6_core.h"
#include "gemm_core.h"
#include "philox.h"
#include "sdhip.h"


namespace {
using namespace sdg;

SD_DEV f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }
SD_DEV f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

// ------------------------------------------------------------------------------------------- A loaders
// Row-major LDS image of a BM x BK tile; thread i holds row i / 8, k-quad i % 8 (float4 along k).
template <int BM>
struct AStage {
  static constexpr int NV = (BM * BK / 4 + 255) / 256;
  f32x4 r[NV];
  SD_DEV static int row(int v) { return (threadIdx.x + 256 * v) / (BK / 4); }
  SD_DEV static int kq(int v) { return (threadIdx.x + 256 * v) % (BK / 4); }
  // static when slot v is full for every thread (hipcc cannot see threadIdx.x < 256): no branch in the k loop
  SD_DEV static bool live(int v) { return 256 * (v + 1) <= BM * BK / 4 || threadIdx.x + 256 * v < BM * BK / 4; }
  SD_DEV void store(float* lds) const {
#pragma unroll
    for (int v = 0; v < NV; ++v)
      if (live(v)) *reinterpret_cast<f32x4*>(lds + row(v) * LDS_ROW + 4 * kq(v)) = r[v];
  }
  SD_DEV void store6(__bf16* lds) const {
#pragma unroll
    for (int v = 0; v < NV; ++v)
      if (live(v)) split3_store(lds + row(v) * LROW6 + 4 * kq(v), r[v]);
  }
};

// Per-row rstd of the workgroup's BM rows from `np` partial sums of squares part[p*M + m] over `width` columns,
// into LDS rs[BM]. 256 threads: row = tid % BM, partial group tid / BM; all loads issued at once (MAXP per thread),
// coalesced along rows. Fixed summation order.
template <int BM, int MAXP>
SD_DEV void wg_rstd(const float* part, int np, int M, int m0, int width, float eps, float* rs, float* red) {
  constexpr int G = 256 / BM;
  const int tid = threadIdx.x, row = tid % BM, grp = tid / BM;
  const sd_rsrc rp = sd_make_rsrc(part, (long)np * M * 4);
  float v[MAXP];
#pragma unroll
  for (int k = 0; k < MAXP; ++k) {
    const int p = grp + G * k;
    v[k] = sd_bload1(rp, (p < np && m0 + row < M) ? (uint32_t)(((long)p * M + m0 + row) * 4) : SD_OOB);
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < MAXP; ++k) s += v[k];
  red[tid] = s;
  __syncthreads();
  if (tid < BM) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < G; ++g) t += red[g * BM + tid];
    rs[tid] = rsqrtf(t / (float)width + eps);
  }
  __syncthreads();
}

template <int BM>
struct APlain : AStage<BM> {
  using AStage<BM>::r;
  sd_rsrc rx;
  long ld;
  int m0, M;
  SD_DEV APlain() = default;
  SD_DEV APlain(const float* X, long ld_, int m0_, int M_, int K) : ld(ld_), m0(m0_), M(M_) {
    rx = sd_make_rsrc(X, ((long)(M - 1) * ld + K) * 4);
  }
  SD_DEV void load(int k0, int) {
#pragma unroll
    for (int v = 0; v < AStage<BM>::NV; ++v) {
      const int m = m0 + this->row(v);
      r[v] = sd_bload4(rx, m < M ? (uint32_t)(((long)m * ld + k0 + 4 * this->kq(v)) * 4) : SD_OOB);
    }
  }
};

// A(m, k) = silu(X[m][k] * rstd[m] * w[k]), rstd of the tile's rows in LDS (wg_rstd). The loads only fill
// registers; the RMSNorm + SiLU is applied when the tile is staged into LDS (store), PF k tiles later, so the
// loads stay in flight behind the MFMAs instead of being waited for at issue.
template <int BM>
struct ARms : AStage<BM> {
  using AStage<BM>::r;
  using AStage<BM>::NV;
  sd_rsrc rx;
  const float* w;
  long ld;
  int m0, M;
  float rr[NV];
  f32x4 wr[NV];
  SD_DEV ARms() = default;
  SD_DEV ARms(const float* X, long ld_, const float* w_, const float* rs, int m0_, int M_, int K)
      : w(w_), ld(ld_), m0(m0_), M(M_) {
    rx = sd_make_rsrc(X, ((long)(M - 1) * ld + K) * 4);
#pragma unroll
    for (int v = 0; v < NV; ++v) rr[v] = rs[this->row(v)];
  }
  SD_DEV void load(int k0, int) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int gk = k0 + 4 * this->kq(v), m = m0 + this->row(v);
      r[v] = sd_bload4(rx, m < M ? (uint32_t)(((long)m * ld + gk) * 4) : SD_OOB);
      wr[v] = ld4(w + gk);
    }
  }
  SD_DEV f32x4 val(int v) const {
    f32x4 y;
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = siluf_(r[v][j] * rr[v] * wr[v][j]);
    return y;
  }
  SD_DEV void store(float* lds) const {
#pragma unroll
    for (int v = 0; v < NV; ++v)
      if (this->live(v)) *reinterpret_cast<f32x4*>(lds + this->row(v) * LDS_ROW + 4 * this->kq(v)) = val(v);
  }
  SD_DEV void store6(__bf16* lds) const {
#pragma unroll
    for (int v = 0; v < NV; ++v)
      if (this->live(v)) split3_store(lds + this->row(v) * LROW6 + 4 * this->kq(v), val(v));
  }
};

// B operand: rows of a k-contiguous weight matrix; local row lr -> global row base + (lr / seg) * stride + lr % seg
template <int BN>
struct BRows {
  static constexpr int NV = (BN * BK / 4 + 255) / 256;
  f32x4 r[NV];
  const float* W;
  long ld;
  int base, seg, stride, nrows;  // rows >= nrows read as 0 (the actor's output weight has only 2A or A rows)
  SD_DEV BRows() = default;
  SD_DEV BRows(const float* W_, long ld_, int base_, int seg_, int stride_, int nrows_ = 1 << 30)
      : W(W_), ld(ld_), base(base_), seg(seg_), stride(stride_), nrows(nrows_) {}
  SD_DEV void load(int k0, int) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + 256 * v;
      if (256 * (v + 1) <= BN * BK / 4 || i < BN * BK / 4) {
        const int lr = i / (BK / 4), kq = i % (BK / 4);
        const long gr = base + (lr / seg) * stride + lr % seg;
        r[v] = gr < nrows ? ld4(W + gr * ld + k0 + 4 * kq) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  SD_DEV void store(float* lds) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + 256 * v;
      if (256 * (v + 1) <= BN * BK / 4 || i < BN * BK / 4)
        *reinterpret_cast<f32x4*>(lds + (i / (BK / 4)) * LDS_ROW + 4 * (i % (BK / 4))) = r[v];
    }
  }
  SD_DEV void store6(__bf16* lds) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + 256 * v;
      if (256 * (v + 1) <= BN * BK / 4 || i < BN * BK / 4)
        split3_store(lds + (i / (BK / 4)) * LROW6 + 4 * (i % (BK / 4)), r[v]);
    }
  }
};

// B operand from a pre-split weight image (k_presplit6): the BN x 32 tile (ct, kt) is stored as its three bf16
// planes, [row][a0 32 | a1 32 | a2 32] (192 B a row), contiguous per tile, so a k tile is one coalesced read of
// 12 KB and store6 copies it into the LDS image in 16-B pieces with no VALU. The planes are split3_store's, so the
// contraction is bit-identical to BRows + store6 on the fp32 weight.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int PRE_ROW = 3 * BK6;  // bf16 per row of a pre-split tile
// TH: the image's tile height when it is taller than the BN rows read (rows sub .. sub + BN - 1 of each TH-row tile)
template <int BN, int TH = BN>
struct BPre6 {
  static constexpr int PCS = BN * PRE_ROW / 8, NV = (PCS + 255) / 256;  // 16-B pieces per tile
  u32x4 r[NV];
  const __bf16* tile0;
  SD_DEV BPre6() = default;
  SD_DEV BPre6(const __bf16* pre, int ct, int nkt, int kt0, int sub = 0)
      : tile0(pre + (((long)ct * nkt + kt0) * TH + sub) * PRE_ROW) {}
  SD_DEV static bool live(int v) { return 256 * (v + 1) <= PCS || threadIdx.x + 256 * v < PCS; }
  SD_DEV void load(int k0, int) {
    const __bf16* t = tile0 + (long)(k0 / BK6) * TH * PRE_ROW;
#pragma unroll
    for (int v = 0; v < NV; ++v)
      if (live(v)) r[v] = *reinterpret_cast<const u32x4*>(t + (threadIdx.x + 256 * v) * 8);
  }
  SD_DEV void store6(__bf16* lds) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + 256 * v;
      if (live(v)) *reinterpret_cast<u32x4*>(lds + (i / (PRE_ROW / 8)) * LROW6 + (i % (PRE_ROW / 8)) * 8) = r[v];
    }
  }
};
// W (rows, K) fp32, k contiguous -> the BPre6 image of BN-row column tiles: tile (n / BN, k / 32), row n % BN.
// One thread per (row, k quad). rows % BN == 0, K % 32 == 0 (the caller checks).
// _dyn_gru's weight for k_gate: tile ct = 32 deter columns c0 = 32 ct of block g = c0 / Dg, its 96 rows the r / c / u
// gate rows g*3Dg + {0, Dg, 2Dg} + c0 % Dg + (0..31) of Wg viewed as (3D, Dg); K = Dg.
__global__ __launch_bounds__(256) void k_presplit6_gate(const float* Wg, int D, int Dg, __bf16* out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const int nq = Dg / 4;
  if (i >= (long)3 * D * nq) return;
  const int rr = (int)(i / nq), k = 4 * (int)(i % nq), nkt = Dg / BK6;  // rr: row of the (3D) tile-ordered image
  const int ct = rr / 96, lr = rr % 96, c0 = ct * 32, g = c0 / Dg;
  const long wrow = (long)g * 3 * Dg + (lr / 32) * Dg + c0 % Dg + lr % 32;
  split3_store(out + (((long)ct * nkt + k / BK6) * 96 + lr) * PRE_ROW + k % BK6, ld4(Wg + wrow * Dg + k));
}
template <int BN>
__global__ __launch_bounds__(256) void k_presplit6(const float* W, int rows, int K, __bf16* out, long ldw = 0) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const int nq = K / 4;
  if (i >= (long)rows * nq) return;
  const int n = (int)(i / nq), k = 4 * (int)(i % nq), nkt = K / BK6;
  split3_store(out + (((long)(n / BN) * nkt + k / BK6) * BN + n % BN) * PRE_ROW + k % BK6,
               ld4(W + (long)n * (ldw ? ldw : K) + k));
}

// Pre-split ACTIVATION images (KH_APRE): the same BPre6 tile layout for a (rows, K) activation — tile (row / 64,
// col / 32), row % 64 — written once by the producer, so the k_hid tiles that read a row (D / 64 column tiles of it)
// copy its planes instead of each splitting it again (split3 of the same fp32 value: bit-identical operands).
#ifndef KH_APRE
#define KH_APRE 1
#endif
SD_DEV long pre_off(long row, int col, int K) {
  return (((row >> 6) * (K / BK6) + col / BK6) * 64 + (row & 63)) * PRE_ROW + (col % BK6);
}
// 4 consecutive columns (col % 4 == 0) of one row
SD_DEV void pre_store4(__bf16* img, long row, int col, int K, f32x4 v) { split3_store(img + pre_off(row, col, K), v); }
SD_DEV void pre_store4_nt(__bf16* img, long row, int col, int K, f32x4 v) {
  split3_store_nt(img + pre_off(row, col, K), v);
}
// IMG_NT (bitmask): step-kernel outputs written with non-temporal stores — 1 = k_gate's fp32 deter (feats; next read
// a step later), 2 = k_gate's deter image, 4 = k_hid's hp. All three (profiles/r05nt): the next launch's gap shrinks
// (k_lin 2.8 -> 1.5 us: less dirty L2 to write back at k_gate's end) but its reads of the image slow by more (mma
// 20.6 -> 23.8 us), step 130.6 -> 135.0 us; the fp32 deter alone (1): update 10.84 vs 10.85 ms, neutral
// (profiles/r05nt1). Off.
#ifndef IMG_NT
#define IMG_NT 0
#endif
// the image of a strided (rows, K) fp32 matrix (feats(0)'s deter at the first step)
__global__ __launch_bounds__(256) void k_presplit_rows(const float* X, long ldx, int rows, int K, __bf16* out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const int nq = K / 4;
  if (i >= (long)rows * nq) return;
  const long r = i / nq;
  const int k = 4 * (int)(i % nq);
  pre_store4(out, r, k, K, ld4(X + r * ldx + k));
}

// ------------------------------------------------------------------------------------------- contraction
// F6: the bf16x6 main loop (gemm6_core.h: fp32-accurate, 2.67x the fp32 MFMA rate) instead of v_mfma_f32_16x16x4_f32.
// ES (early store) applies to the fp32 loop only.
// FP: the fragment-prefetch loop order (LDS reads of tile k+1 issued ahead of tile k's MFMAs, gemm_core.h
// gemm16_mainloop_fp). The loaders are built from one prototype into PF register sets.
template <bool F6, bool FP, int BM, int BN, int WM, int WN, int PF, bool ES = false, class OpA, class OpB>
SD_DEV void mainloop(const OpA& a0, const OpB& b0, int kbeg, int kend, f32x4 (&acc)[WM / 16][WN / 16],
                     bool accumulate = false) {
  static_assert(BK == BK6, "tile depth");
  OpA la[PF];
  OpB lb[PF];
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    la[u] = a0;
    lb[u] = b0;
  }
  if constexpr (F6 && FP)
    gemm6_mainloop_fp<BM, BN, WM, WN, PF>(la, lb, kbeg, kend, acc, accumulate);
  else if constexpr (F6)
    gemm6_mainloop_pf<BM, BN, WM, WN, PF>(la, lb, kbeg, kend, acc, accumulate);
  else if constexpr (FP)
    gemm16_mainloop_fp<BM, BN, WM, WN, PF>(la, lb, kbeg, kend, acc, accumulate);
  else
    gemm16_mainloop_pf<BM, BN, WM, WN, PF, ES>(la, lb, kbeg, kend, acc, accumulate);
}
// per-kernel choice (measured, imagination alone, N = 1024): k_hid 54.0 -> 50.7 us and k_gate 41.9 -> 38.7 us on
// bf16x6; k_lin (28.6 vs 30.0) and the short-K latency-bound launches stay on fp32. These launches are bound by
// operand traffic and per-launch latency, not by the MFMA pipe (tools/pmc_table.py: k_hid MFMA busy ~0.45).
// (SD_IMG_F6 = bitmask over LIN, RMSLIN, HID, GATE, PRIOR, ACTION: a build-time A/B knob, tools/ab_variants.sh)
#ifndef SD_IMG_F6
#define SD_IMG_F6 0b001100
#endif
constexpr bool F6_LIN = SD_IMG_F6 & 1, F6_RMSLIN = SD_IMG_F6 & 2, F6_HID = SD_IMG_F6 & 4, F6_GATE = SD_IMG_F6 & 8,
               F6_PRIOR = SD_IMG_F6 & 16, F6_ACTION = SD_IMG_F6 & 32;
// fragment-prefetch loop order per kernel (same bit order) and a global prefetch-depth override (0: per-kernel)
#ifndef SD_IMG_FP
#define SD_IMG_FP 0b110011
#endif
#ifndef SD_IMG_PF
#define SD_IMG_PF 0
#endif
constexpr bool FP_LIN = SD_IMG_FP & 1, FP_RMSLIN = SD_IMG_FP & 2, FP_HID = SD_IMG_FP & 4, FP_GATE = SD_IMG_FP & 8,
               FP_PRIOR = SD_IMG_FP & 16, FP_ACTION = SD_IMG_FP & 32;
constexpr int pf_of(int d) { return SD_IMG_PF ? SD_IMG_PF : d; }
#ifndef KH_PF
#define KH_PF 1
#endif
#ifndef KG_PF
#define KG_PF 1
#endif
#ifndef KG_1S  // k_gate on the single-stage bf16x6 loop (gemm6_core.h gemm6_mainloop_1s)
#define KG_1S 1
#endif

// ------------------------------------------------------------------------------------------- epilogue helpers
// Wave (wr, wc) of a BM x BN tile owns rows wr*16 + 4q + r and columns wc*WN + 16j + l16 (gemm16_mainloop layout).
struct Lane {
  int l16, q, wr, wc;
};
template <int BN, int WN>
SD_DEV Lane lane_ids() {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  return Lane{lane & 15, lane >> 4, wave / (BN / WN), wave % (BN / WN)};
}

// out[m][n] = acc + bias[n] (+ add[m][n]); part[(n / PW) * M + m] = sum over each PW-column group of out^2 (the
// consumers' wg_rstd reads width / PW partials per row whatever the producer's tile shape: PW = 32 for the U-wide
// MLP layers, 64 for dyn_hid). WN % PW == 0.
template <int BM, int BN, int WN, int PW = 32>
SD_DEV void ep_bias_part(const f32x4 (&acc)[1][WN / 16], const float* bias, float* out, long ldo, float* part, int M,
                         int m0, int n0, const float* add = nullptr, const float* bvals = nullptr, bool nt = false) {
  constexpr int TN = WN / 16, TP = PW / 16;
  static_assert(WN % PW == 0, "whole row-partial groups per wave");
  const Lane L = lane_ids<BN, WN>();
  float ss[WN / PW][4] = {};
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + L.wc * WN + 16 * j + L.l16;
    const float bv = bvals ? bvals[j] : bias ? bias[n] : 0.f;  // (bvals: the bias values, loaded by the caller)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + L.wr * 16 + 4 * L.q + r;
      float v = acc[0][j][r] + bv;
      if (add && m < M) v += add[(long)m * ldo + n];
      if (m < M) {
        if (nt)
          __builtin_nontemporal_store(v, out + (long)m * ldo + n);
        else
          out[(long)m * ldo + n] = v;
      }
      ss[j / TP][r] += v * v;
    }
  }
#pragma unroll
  for (int p = 0; p < WN / PW; ++p)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float s = group_sum<16>(ss[p][r]);
      const int m = m0 + L.wr * 16 + 4 * L.q + r;
      if (L.l16 == 0 && part && m < M) part[(long)((n0 + L.wc * WN) / PW + p) * M + m] = s;
    }
}

// ------------------------------------------------------------------------------------------- kernels
// XCD-aware column-tile order for the block-diagonal (G blocks) layers: workgroups are dealt to the 8 XCDs round
// robin by linear id, and gridDim.x is a multiple of 8, so an XCD runs the x = xcd (mod 8) column tiles of every row
// tile. Mapping x -> tile (x % G) * tpb + x / G puts all tiles of block g = x % G on one XCD (G = 8): that XCD's L2
// then serves the block's input columns and weights to all of them, instead of every XCD streaming every block.
SD_DEV int xcd_col(int x, int nx, int tpb) {
  const int G = nx / tpb;
  return (x % G) * tpb + x / G;
}
// XCD-aware tile order for the grouped plain GEMMs (k_lin, grid (col tiles, row tiles, problems)): the 8 XCDs form a
// 4 (row groups) x 2 (column groups over all problems) grid, so an XCD's L2 serves a quarter of A and half of the
// weights instead of all of A (dispatch order deals linear ids round robin to the XCDs). Identity when the grid does
// not split that way.
#ifndef KL_XCD
#define KL_XCD 1
#endif
SD_DEV void xcd_tile(int& tx, int& ty, int& tz) {
  const int nx = gridDim.x, ny = gridDim.y, cols = nx * gridDim.z;
  if (ny % 4 || cols % 2) return;
  const int id = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z), xcd = id % 8, slot = id / 8;
  const int R4 = ny / 4, C2 = cols / 2;
  const int row = (xcd >> 1) * R4 + slot % R4, col = (xcd & 1) * C2 + slot / R4;
  tx = col % nx;
  ty = row;
  tz = col / nx;
}

struct LinProb {
  const float* A;
  long lda;
  int K;
  const float* W;  // (N, K) k-contiguous (ld = ldw)
  long ldw;
  const float* bias;
  float* out;
  long ldo;
  float* part;
  const float* add;  // optional (M, ldo) term added before the row partials (a K-split layer's first part)
};

// tile of the step's three (N, D) x (D, U) contractions (img_net_0 + _dyn_in0 + actor layer 0's deter part); build-time
// A/B knobs (tools/ab_variants.sh)
#ifndef KL3_BM
#define KL3_BM 32
#endif
#ifndef KL3_BN
#define KL3_BN 32
#endif
#ifndef KL_PF
#define KL_PF 2
#endif
// tile of the step's K = S*Kd launch (actor layer 0's stoch part + _dyn_in1)
#ifndef KL2_BN
#define KL2_BN 32
#endif
constexpr int KL2_WN = KL2_BN / 2, KL2_PW = KL2_WN < 32 ? KL2_WN : 32;
constexpr int KL3_WN = KL3_BN / (4 / (KL3_BM / 16)), KL3_PW = KL3_WN < 32 ? KL3_WN : 32;  // its row-partial width
// grouped plain-A linear layers (N = 256 each): out = A . W^T + b (+ add), with row partials. grid (N/BN, M/BM, nprob)
template <int BM, int BN>
__global__ __launch_bounds__(256) void k_lin(LinProb p0, LinProb p1, LinProb p2, int M, Tr tr) {
  SD_TR_BEGIN
  constexpr int WN = BN / (4 / (BM / 16));
  int tx = blockIdx.x, ty = blockIdx.y, tz = blockIdx.z;
  if (KL_XCD) xcd_tile(tx, ty, tz);
  const LinProb p = tz == 0 ? p0 : (tz == 1 ? p1 : p2);
  const int n0 = tx * BN, m0 = ty * BM;
  const APlain<BM> a0(p.A, p.lda, m0, M, p.K);
  const BRows<BN> b0(p.W, p.ldw, n0, BN, 0);
  f32x4 acc[1][WN / 16];
  SD_TR(1)
  mainloop<F6_LIN, FP_LIN, BM, BN, 16, WN, pf_of(KL_PF)>(a0, b0, 0, p.K, acc);
  SD_TR(2)
  ep_bias_part<BM, BN, WN, (WN < 32 ? WN : 32)>(acc, p.bias, p.out, p.ldo, p.part, M, m0, n0, p.add);
  SD_TR_END(tr.p, tr.slot)
}

// k_lin on the bf16x6 path with both operands pre-split (KL_PRE): A = deter' from the image k_gate already wrote for
// the next k_hid (64-row tiles), B = the three weights' images (built once per imagination), so the main loop only
// copies bf16 planes into LDS (no split VALU) and runs at the bf16 MFMA rate (six products per fp32 product:
// fp32-accurate, gemm6_core.h). Same outputs and row partials (KL3_PW wide) as k_lin<KL3_BM, KL3_BN>.
#ifndef KL_PRE
#define KL_PRE 1
#endif
#ifndef KL6_BM  // k_lin6 row tile: 32 (2 x 2 waves, half of each 64-row image tile: 768 workgroups, 3 per CU) or 64
#define KL6_BM 32  // (4 waves x 16 rows: 384 workgroups, two on half the CUs) — step trace 37.8 -> 33.1 us, r04y
#endif
template <int BM, int BN>
__global__ __launch_bounds__(256) void k_lin6(const __bf16* aimg, int K, const __bf16* w0, const __bf16* w1,
                                              const __bf16* w2, LinProb p0, LinProb p1, LinProb p2, int M, Tr tr) {
  SD_TR_BEGIN
  constexpr int WN = BN / (4 / (BM / 16));
  static_assert(WN % KL3_PW == 0 && BM <= 64, "row partials; rows of one 64-row image tile");
  int tx = blockIdx.x, ty = blockIdx.y, tz = blockIdx.z;
  if (KL_XCD) xcd_tile(tx, ty, tz);
  const LinProb p = tz == 0 ? p0 : (tz == 1 ? p1 : p2);
  const __bf16* wimg = tz == 0 ? w0 : (tz == 1 ? w1 : w2);
  const int n0 = tx * BN, m0 = ty * BM;
  f32x4 acc[1][WN / 16];
  SD_TR(1)
#ifndef KL_BWTEST  // timing probe only (wrong results): 1 = every workgroup reads column tile 0's weights, 2 = row
#define KL_BWTEST 0  // tile 0's deter rows, 3 = both (profiles/r05kl: 33.3 / 34.4 / 33.3 us — not operand traffic)
#endif
  const int ma = (KL_BWTEST & 2) ? 0 : m0, ta = (KL_BWTEST & 1) ? 0 : tx;
  mainloop<true, FP_LIN, BM, BN, 16, WN, pf_of(KL_PF)>(BPre6<BM, 64>(aimg, ma / 64, K / BK6, 0, ma % 64),
                                                      BPre6<BN>(wimg, ta, K / BK6, 0), 0, K, acc);
  SD_TR(2)
  ep_bias_part<BM, BN, WN, KL3_PW>(acc, p.bias, p.out, p.ldo, p.part, M, m0, n0, p.add);
  SD_TR_END(tr.p, tr.slot)
}

// The step's K = S*Kd contractions (actor layer 0's stoch part + _dyn_in1) read a straight-through one-hot sample:
// every categorical holds one nonzero (the sampler writes ((k == idx) - ys) + ys: exactly 0 off the index). So
// out[m] = b + add[m] + sum_s v_s WT[s*Kd + idx_s] — a gather of S rows of the pre-transposed weight WT (SK, U) per
// row, not a dense (N, SK) x (SK, U) GEMM. One wave per row, 4 columns per lane (U = 256); lane s finds categorical
// s's nonzero; the S row loads are issued in batches of OH_BATCH before their FMAs. A row with a categorical holding more
// than one nonzero takes the exact dense loop over all SK entries instead. Row partials per 16 columns, as k_lin's.
#ifndef KL_ONEHOT
#define KL_ONEHOT 1
#endif
#ifndef OH_SPLIT  // the two one-hot problems of a step as two grid rows (1) or one after the other per wave (0):
#define OH_SPLIT 1  // span 8.0 -> 5.7 us per step, update 11.47 -> 11.39 ms (3-round A/B, profiles/r04o)
#endif
#ifndef OH_BATCH  // weight-row loads issued before their FMAs
#define OH_BATCH 32
#endif
// k_onehot_lin writes one row partial per 16 columns (4 lanes x 4 columns); its consumers read U / KL2_PW partials
static_assert(!KL_ONEHOT || KL2_PW == 16, "k_onehot_lin's 16-column row partials need KL2_PW == 16 (KL2_BN = 32)");
struct OneHotProb {
  const float* WT;  // (SK, U) transposed weight
  const float* bias;
  const float* add;  // optional (M, U)
  float* out;        // (M, U)
  float* part;       // (U / 16, M)
  const float* nw;   // optional: RMSNorm weight -> img = pre-split image of silu(rms(out) * nw) (KH_APRE)
  __bf16* img;
  float eps;
};
__global__ __launch_bounds__(256) void k_onehot_lin(const float* X, long ldx, int SK, int Kd, OneHotProb p0,
                                                    OneHotProb p1, int nprob, int M, Tr tr) {
  SD_TR_BEGIN
  constexpr int U = 256;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long m = (long)blockIdx.x * 4 + wave;
  if (m >= M) return;
  const int S = SK / Kd;
  const float* x = X + m * ldx;
  // lane s < S: categorical s's first nonzero (index, value) and whether it holds another
  int idx = 0, many = 0;
  float val = 0.f;
  if (lane < S) {
    int cnt = 0;
    for (int j = 0; j < Kd; j += 4) {
      const f32x4 q = ld4(x + lane * Kd + j);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (q[e] != 0.f) {
          if (cnt == 0) { idx = j + e; val = q[e]; }
          ++cnt;
        }
    }
    many = cnt > 1;
  }
  const bool dense = __any(many);
  SD_TR(1)
  const int c = 4 * lane;
  // OH_SPLIT: one problem per workgroup row of the grid (blockIdx.y), both gathers in flight at once; else in turn
  const int pr0 = OH_SPLIT ? (int)blockIdx.y : 0, pr1 = OH_SPLIT ? pr0 + 1 : nprob;
#pragma unroll 1
  for (int pr = pr0; pr < pr1; ++pr) {
    const OneHotProb& p = pr == 0 ? p0 : p1;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    if (!dense) {
      for (int s0 = 0; s0 < S; s0 += OH_BATCH) {
        f32x4 w[OH_BATCH];
        float v[OH_BATCH];
#pragma unroll
        for (int u = 0; u < OH_BATCH; ++u) {
          const int s = s0 + u < S ? s0 + u : S - 1;
          const int k = s * Kd + __shfl(idx, s, 64);
          v[u] = s0 + u < S ? __shfl(val, s, 64) : 0.f;
          w[u] = ld4(p.WT + (long)k * U + c);
        }
#pragma unroll
        for (int u = 0; u < OH_BATCH; ++u)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[e] += v[u] * w[u][e];
      }
    } else {
      for (int k = 0; k < SK; ++k) {
        const float xv = x[k];
        if (xv != 0.f) {
          const f32x4 w = ld4(p.WT + (long)k * U + c);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[e] += xv * w[e];
        }
      }
    }
    const f32x4 b = p.bias ? ld4(p.bias + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    const f32x4 a = p.add ? ld4(p.add + m * U + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = acc[e] + b[e] + a[e];
    *reinterpret_cast<f32x4*>(p.out + m * U + c) = o;
    float ss = o[0] * o[0] + o[1] * o[1] + o[2] * o[2] + o[3] * o[3];
    ss += __shfl_xor(ss, 1, 64);
    ss += __shfl_xor(ss, 2, 64);
    if ((lane & 3) == 0 && p.part) p.part[(long)(lane >> 2) * M + m] = ss;
    if (p.img) {  // the row's normalised output, split once for k_hid (a wave holds the whole row)
      // rstd exactly as k_hid's wg_rstd<64, 8> forms it from these 16 partials (lane 4 p holds partial p): 4 groups
      // g of partials g, g + 4, g + 8, g + 12, summed in that order, then the groups in order -> bit-identical x1
      float pp[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) pp[q] = __shfl(ss, 4 * q, 64);
      float tsum = 0.f;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        float sg = 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) sg += pp[g + 4 * k];
        tsum += sg;
      }
      const float rs = rsqrtf(tsum / (float)U + p.eps);
      const f32x4 w = ld4(p.nw + c);
      f32x4 y;
#pragma unroll
      for (int e = 0; e < 4; ++e) y[e] = siluf_(o[e] * rs * w[e]);
      pre_store4(p.img, m, c, U, y);
    }
  }
  SD_TR(2)
  SD_TR_END(tr.p, tr.slot)
}
// WT (K, U) = W[:, 0:K]^T for a (U, ldw) weight
__global__ __launch_bounds__(256) void k_transpose_w(const float* W, long ldw, int U, int K, float* WT) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)U * K) return;
  const int k = (int)(i / U), c = (int)(i % U);
  WT[i] = W[(long)c * ldw + k];
}

// out = silu(rms(X)) . W^T + b (MLP hidden layer after the first), with row partials
// early-store main loop order (gemm16_mainloop_pf ES): measured faster here, slower in the other imagination kernels.
// Row partials per min(WN, 32) columns (16-row tiles: one wave per 16 columns -> 16-column partials).
#ifndef KR_BM
#define KR_BM 16
#endif
constexpr int KR_WN = 64 / (4 / (KR_BM / 16)), KR_PW = KR_WN < 32 ? KR_WN : 32;
template <int BM, int BN>
__global__ __launch_bounds__(256) void k_rmslin(const float* X, const float* nw, const float* part_in, int np, int K,
                                                const float* W, const float* bias, float* out, float* part, int M,
                                                float eps, Tr tr) {
  SD_TR_BEGIN
  constexpr int WN = BN / (4 / (BM / 16));
  __shared__ float rs[BM], red[256];
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  wg_rstd<BM, 8>(part_in, np, M, m0, K, eps, rs, red);
  SD_TR(1)
  const ARms<BM> a0(X, K, nw, rs, m0, M, K);
  const BRows<BN> b0(W, K, n0, BN, 0);
  f32x4 acc[1][WN / 16];
  mainloop<F6_RMSLIN, FP_RMSLIN, BM, BN, 16, WN, pf_of(FP_RMSLIN ? 2 : 3), true>(a0, b0, 0, K, acc);
  SD_TR(2)
  ep_bias_part<BM, BN, WN, (WN < 32 ? WN : 32)>(acc, bias, out, gridDim.x * BN, part, M, m0, n0);
  SD_TR_END(tr.p, tr.slot)
}

// ------------------------------------------------------------------------------------------- 16 x 64 register tiles
// The short-K (K = U = 256) layers on 16-row tiles — the actor / img_net hidden layers (k_rmslin) and the prior logits
// (k_prior) — measured as latency chains: an LDS-staged k loop of 8 tiles with a barrier each. Here each workgroup
// stages the RMSNorm + SiLU'd A panel (16 rows x K, from the producer's row partials) into LDS ONCE, every wave loads
// its weight fragments straight into registers at entry (column tile w % 4, K part w / 4: K / KS per wave), the MFMAs
// run from registers + LDS with no further barrier, and the KS k-parts are summed in a fixed order through LDS.
// v_mfma_f32_16x16x4_f32 (exact fp32 products): lane (l16, q) supplies k = 16c + 4q + j at MFMA j of chunk c.
template <int NWV>
struct RTile {
  static constexpr int U = 256, KS = NWV / 4, KP = U / KS, NCH = KP / 16, LDP = U + 4;
  f32x4 b[NCH];
  f32x4 acc;
  // weight rows of this wave's column tile (n0 + 16 (w % 4) + l16), its K part
  SD_DEV void load_w(const float* W, long ldw, int n0) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, q = lane >> 4;
    const float* p = W + (long)(n0 + 16 * (w % 4) + l16) * ldw + (w / 4) * KP + 4 * q;
#pragma unroll
    for (int c = 0; c < NCH; ++c) b[c] = ld4(p + 16 * c);
  }
  // panel P[16][LDP] = silu(X[m0 + r] * rstd_r * nw), rstd from np <= 16 partials part[p * M + m]; threads 0..255:
  // row tid / 16, 16 columns each (the row's 16 threads reduce its partials: no barrier before the norm)
  // the panel's operands in registers (threads 0..255): stage_load issues the loads, stage_store normalises and
  // writes P — split so a caller can issue its weight loads in between (RT_LOADFIRST) and the panel does not wait on
  // them (loads complete in issue order)
  struct Panel {
    f32x4 x[4], w[4];
    float pv;
    bool pok;  // pv is one of the np partials (else a clamped duplicate, masked in stage_store)
  };
  SD_DEV static void stage_load(Panel& q, const float* X, long ldx, const float* nw, const float* part, int np, int M,
                                int m0) {
    // unconditional loads (rows past M read row M - 1, partials past np read partial np - 1; stage_store masks
    // them): a "cond ? load : 0" made hipcc branch around the load and drain the vector-memory queue at the join
    const int tid = threadIdx.x;
    if (tid < 256) {
      const int r = tid >> 4, j = tid & 15;
      const long m = m0 + r < M ? m0 + r : M - 1;
      q.pv = part[(long)(j < np ? j : np - 1) * M + m];
      q.pok = j < np;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        q.x[i] = ld4(X + m * ldx + 16 * j + 4 * i);
        q.w[i] = ld4(nw + 16 * j + 4 * i);
      }
    }
  }
  SD_DEV static void stage_store(const Panel& q, float* P, int M, int m0, float eps) {
    const int tid = threadIdx.x;
    if (tid < 256) {
      const int r = tid >> 4, j = tid & 15;
      const bool rv = m0 + r < M;
      const float rs = rsqrtf(group_sum<16>(q.pok ? q.pv : 0.f) / (float)U + eps);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        f32x4 y;
#pragma unroll
        for (int e = 0; e < 4; ++e) y[e] = rv ? siluf_(q.x[i][e] * rs * q.w[i][e]) : 0.f;
        *reinterpret_cast<f32x4*>(P + r * LDP + 16 * j + 4 * i) = y;
      }
    }
  }
  SD_DEV static void stage(float* P, const float* X, long ldx, const float* nw, const float* part, int np, int M,
                           int m0, float eps) {
    Panel q;
    stage_load(q, X, ldx, nw, part, np, M, m0);
    stage_store(q, P, M, m0, eps);
  }
  SD_DEV void mma(const float* P) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, q = lane >> 4;
    acc = f32x4{0.f, 0.f, 0.f, 0.f};
    const float* a = P + l16 * LDP + (w / 4) * KP + 4 * q;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const f32x4 av = ld4(a + 16 * c);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], b[c][j], acc, 0, 0, 0);
    }
  }
  // sum of the KS k-parts into tile T[16][64 + 1] (row 4q + r, column 16 (w % 4) + l16), in k-part order
  SD_DEV void reduce(float* red, float* T) const {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, q = lane >> 4;
    if (KS > 1) {
#pragma unroll
      for (int r = 0; r < 4; ++r) red[(w * 4 + r) * 64 + lane] = acc[r];
      __syncthreads();
      if (w < 4) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = red[(w * 4 + r) * 64 + lane];
#pragma unroll
          for (int k = 1; k < KS; ++k) v += red[((w + 4 * k) * 4 + r) * 64 + lane];
          T[(4 * q + r) * 65 + 16 * w + l16] = v;
        }
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) T[(4 * q + r) * 65 + 16 * w + l16] = acc[r];
    }
    __syncthreads();
  }
};

// RTile<16>'s partition (16 virtual waves: column tile v % 4, k part v / 4) on 8 waves: wave w runs virtual waves w
// and w + 8 (same column tile, k parts w / 4 and w / 4 + 2) with one accumulator each, and the k parts are summed in
// RTile<16>'s order — bit-identical results with half the threads per workgroup (k_prior_rw<.., 512>).
struct RTile16h {
  static constexpr int U = 256, KS = 4, KP = U / KS, NCH = KP / 16, LDP = U + 4;
  f32x4 b[2][NCH];
  f32x4 acc[2];
  SD_DEV void load_w(const float* W, long ldw, int n0) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, q = lane >> 4;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int v = w + 8 * h;
      const float* p = W + (long)(n0 + 16 * (v % 4) + l16) * ldw + (v / 4) * KP + 4 * q;
#pragma unroll
      for (int c = 0; c < NCH; ++c) b[h][c] = ld4(p + 16 * c);
    }
  }
  using Panel = RTile<16>::Panel;
  SD_DEV static void stage_load(Panel& q, const float* X, long ldx, const float* nw, const float* part, int np, int M,
                                int m0) {
    RTile<16>::stage_load(q, X, ldx, nw, part, np, M, m0);
  }
  SD_DEV static void stage_store(const Panel& q, float* P, int M, int m0, float eps) {
    RTile<16>::stage_store(q, P, M, m0, eps);
  }
  SD_DEV static void stage(float* P, const float* X, long ldx, const float* nw, const float* part, int np, int M,
                           int m0, float eps) {
    RTile<16>::stage(P, X, ldx, nw, part, np, M, m0, eps);
  }
  SD_DEV void mma(const float* P) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, q = lane >> 4;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int v = w + 8 * h;
      acc[h] = f32x4{0.f, 0.f, 0.f, 0.f};
      const float* a = P + l16 * LDP + (v / 4) * KP + 4 * q;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        const f32x4 av = ld4(a + 16 * c);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j], b[h][c][j], acc[h], 0, 0, 0);
      }
    }
  }
  SD_DEV void reduce(float* red, float* T) const {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, l16 = lane & 15, q = lane >> 4;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[((w + 8 * h) * 4 + r) * 64 + lane] = acc[h][r];
    __syncthreads();
    if (w < 4) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = red[(w * 4 + r) * 64 + lane];
#pragma unroll
        for (int k = 1; k < KS; ++k) v += red[((w + 4 * k) * 4 + r) * 64 + lane];
        T[(4 * q + r) * 65 + 16 * w + l16] = v;
      }
    }
    __syncthreads();
  }
};

#ifndef RT_LOADFIRST  // k_rmslin_rw issues the A panel's loads before its weight loads (k_prior_rw would spill: 64 VGPRs):
#define RT_LOADFIRST 1  // step 156.5 -> 154.1 us, update 11.40 -> 11.36 ms (3-round A/B, profiles/r04l)
#endif
#ifndef KR_RW  // k_rmslin as register tiles (RTile<8>); 0: the LDS-staged k loop
#define KR_RW 1
#endif
#ifndef KP_RW  // k_prior as register tiles (RTile<16>, one sampler element per thread); 0: the LDS-staged k loop
#define KP_RW 1
#endif
#ifndef KP_NT  // k_prior_rw threads per workgroup: 1024 (RTile<16>) or 512 (RTile16h, two sampler elements per thread)
#define KP_NT 1024
#endif
// k_rmslin on RTile<8>: 512 threads, grid (U / 64, M / 16); the same outputs and 16-column row partials (part[p * M +
// m], p = column / 16) as k_rmslin<16, 64>
__global__ __launch_bounds__(512) void k_rmslin_rw(const float* X, const float* nw, const float* part_in, int np,
                                                   const float* W, const float* bias, float* out, float* part, int M,
                                                   float eps, Tr tr) {
  SD_TR_BEGIN
  using RT = RTile<8>;
  __shared__ __attribute__((aligned(16))) float P[16 * RT::LDP];
  __shared__ float red[8 * 4 * 64];
  __shared__ float T[16 * 65];
  const int n0 = blockIdx.x * 64, m0 = blockIdx.y * 16;
  RT rt;
  if (RT_LOADFIRST) {  // the panel's loads first: its normalisation waits only on them
    typename RT::Panel q;
    RT::stage_load(q, X, RT::U, nw, part_in, np, M, m0);
    rt.load_w(W, RT::U, n0);
    RT::stage_store(q, P, M, m0, eps);
  } else {
    rt.load_w(W, RT::U, n0);
    RT::stage(P, X, RT::U, nw, part_in, np, M, m0, eps);
  }
  __syncthreads();
  SD_TR(1)
  rt.mma(P);
  rt.reduce(red, T);
  SD_TR(2)
  const int tid = threadIdx.x;
  if (tid < 256) {  // row tid / 16, columns 4 (tid % 16) .. +3
    const int r = tid >> 4, j = tid & 15;
    const long m = m0 + r;
    const f32x4 bv = ld4(bias + n0 + 4 * j);
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = T[r * 65 + 4 * j + e] + bv[e];
    if (m < M) *reinterpret_cast<f32x4*>(out + m * RT::U + n0 + 4 * j) = v;
    float ss = v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
    ss += __shfl_xor(ss, 1, 64);
    ss += __shfl_xor(ss, 2, 64);  // 4 threads = 16 columns
    if ((j & 3) == 0 && m < M) part[(long)(n0 / 16 + (j >> 2)) * M + m] = ss;
  }
  SD_TR_END(tr.p, tr.slot)
}

// k_hid tiling knobs: 64 or 32 rows per workgroup, single-stage LDS loop, register budget (waves per SIMD)
#ifndef KH_BM
#define KH_BM 64
#endif
#ifndef KH_1S
#define KH_1S 1
#endif
#ifndef KH_PRE  // k_hid reads _dyn_hid's weight from the once-per-imagination pre-split image (BPre6)
#define KH_PRE 1
#endif
#ifndef KH_WAVES
#define KH_WAVES 2
#endif
constexpr int KH_WN = 64 / (4 / (KH_BM / 16)), KH_PW = KH_WN < 64 ? KH_WN : 64;  // hp row-partial width
template <int BM, int BN, int WN, class OpA, class OpB>
SD_DEV void hid_seg(const OpA& a0, const OpB& b0, int K, f32x4 (&acc)[1][WN / 16], bool accumulate) {
  if constexpr (KH_1S && F6_HID) {
    OpA la[KH_PF];
    OpB lb[KH_PF];
#pragma unroll
    for (int u = 0; u < KH_PF; ++u) {
      la[u] = a0;
      lb[u] = b0;
    }
    gemm6_mainloop_1s<BM, BN, 16, WN, KH_PF>(la, lb, 0, K, acc, accumulate);
  } else {
    mainloop<F6_HID, FP_HID, BM, BN, 16, WN, pf_of(KH_PF)>(a0, b0, 0, K, acc, accumulate);
  }
}

// hp = BlockLinear(dyn_hid_0)([h_g | x0 | x1 | x2]) + bh with x0 = silu(rms(x0p)), x1 = silu(rms(x1p)) applied by the
// A loaders (rssm.py:52-63): four main loops over the input segments accumulate into one tile. BM = BN = 64,
// grid (D/64, M/64); row partials per 64 columns (D/64 of them) for the gate norm.
template <bool APRE>
__global__ __launch_bounds__(256, KH_WAVES) void k_hid(sd_imagine d, const float* h, long ldh, const float* x0p, const float* x1p,
                                             const float* px0, const float* px1, int npx0, int npx1, const float* x2, float* hp,
                                             float* ph, const __bf16* wh6, const __bf16* himg, const __bf16* x1img,
                                             const __bf16* x2img, Tr tr) {
  SD_TR_BEGIN
  constexpr int BM = KH_BM, BN = 64, WN = BN / (4 / (BM / 16));
  static_assert(!APRE || BM == 64, "pre-split activation images are in 64-row tiles");
  __shared__ float rs0[BM], rs1[BM], red[256];
  const int Dg = d.D / d.G, U = d.U, Ig = Dg + 3 * U, M = d.N;
  const int n0 = xcd_col(blockIdx.x, gridDim.x, Dg / BN) * BN, m0 = blockIdx.y * BM, g = n0 / Dg;
  wg_rstd<BM, 8>(px0, npx0, M, m0, U, d.eps, rs0, red);
  if (!APRE) wg_rstd<BM, 8>(px1, npx1, M, m0, U, d.eps, rs1, red);
  SD_TR(1)
  const float* Wseg = d.Wh + (long)n0 * Ig;  // rows n0.. of Wh viewed as (D, Ig)
#ifndef KH_BWTEST  // timing probe only (wrong results): 1 = every workgroup reads column tile 0's weights, 2 = row tile
#define KH_BWTEST 0  // 0's activations, 3 = both — what k_hid costs without its L2 -> CU operand traffic
#endif
  const int ct = (KH_BWTEST & 1) ? 0 : n0 / BN, nkt = Ig / BK6;
  const int mt = (KH_BWTEST & 2) ? 0 : m0;
  // the four K segments of [h_g | x0 | x1 | x2]: B from the pre-split image (KH_PRE) or split while staged
  auto bseg = [&](int k0) {
    if constexpr (KH_PRE && F6_HID)
      return BPre6<BN>(wh6, ct, nkt, k0 / BK6);
    else
      return BRows<BN>(Wseg + k0, Ig, 0, BN, 0);
  };
  f32x4 acc[1][WN / 16];
  if constexpr (APRE) {  // h, x1 and x2 from their producers' pre-split images (64-row tiles of m0 / 64)
    hid_seg<BM, BN, WN>(BPre6<BM>(himg, mt / BM, d.D / BK6, g * Dg / BK6), bseg(0), Dg, acc, false);
  } else {
    const APlain<BM> a0(h + (long)g * Dg, ldh, m0, M, Dg);
    hid_seg<BM, BN, WN>(a0, bseg(0), Dg, acc, false);
  }
  {
    const ARms<BM> a0(x0p, U, d.n0, rs0, mt, M, U);
    hid_seg<BM, BN, WN>(a0, bseg(Dg), U, acc, true);
  }
  if constexpr (APRE) {
    hid_seg<BM, BN, WN>(BPre6<BM>(x1img, mt / BM, U / BK6, 0), bseg(Dg + U), U, acc, true);
    hid_seg<BM, BN, WN>(BPre6<BM>(x2img, mt / BM, U / BK6, 0), bseg(Dg + 2 * U), U, acc, true);
  } else {
    {
      const ARms<BM> a0(x1p, U, d.n1, rs1, m0, M, U);
      hid_seg<BM, BN, WN>(a0, bseg(Dg + U), U, acc, true);
    }
    {
      const APlain<BM> a0(x2, U, m0, M, U);
      hid_seg<BM, BN, WN>(a0, bseg(Dg + 2 * U), U, acc, true);
    }
  }
  SD_TR(2)
  ep_bias_part<BM, BN, WN, KH_PW>(acc, d.bh, hp, d.D, ph, M, m0, n0);
  SD_TR_END(tr.p, tr.slot)
}

// k_hid on register A operands (KH_AREG): the same 64 x 64 tile, bf16x6 products and k order as k_hid<true>
// (bit-identical), restructured around what bounds it. k_hid<true> runs its four K segments as four single-stage loops
// that stage A and B through LDS (two barriers per k tile, LDS writes and reads serialised with the MFMAs: mma phase
// ~28 us of a 36 us launch, MFMA busy ~0.3, and unchanged when every workgroup reads one tile's operands —
// profiles/r05n: not the L2 -> CU traffic). Here wave w's A operand is its own 16 rows, so each lane loads its
// fragment (row l16, k 8q..8q+7 of each plane) straight from the producers' pre-split images into registers — deter
// (k_gate), x0 (k_action_rows), x1 (k_onehot_lin), x2 (k_action_rows) — and only B (the weight tile the four waves
// share) goes through a double-buffered LDS stage; the whole K (NKT = Dg/32 + 24 tiles) is one fully unrolled loop
// with A two tiles ahead in three register sets, B's next tile stored between this tile's MFMAs, one barrier per tile.
// Step trace (profiles/r05s): k_hid 35.4 -> 27.0 us per step, the imagination step 149.7 -> 142.8 us; update A/B
// 11.09 -> 11.01 ms. (Measured against it, r05p / r05r: 32-row waves — 2 x 2 waves on 64 x 64, or 4 x 2 on 128 x 64
// tiles, B fragments reused by two row tiles — run slower, 36.4 / 33.6 vs 28.8 us: their fragment-shaped A loads
// double per lane.)
#ifndef KH_STAGES  // B's LDS stages: 3 = each tile's fragments read a step ahead, between the previous tile's MFMAs
#define KH_STAGES 2  // (3: 27.2 vs 27.0 us per launch, r05s — the reads were not what the MFMAs waited on)
#endif
template <int NKT>
__global__ __launch_bounds__(256, 2) void k_hid_areg(sd_imagine d, float* hp, float* ph, const __bf16* wh6,
                                                     const __bf16* himg, const __bf16* x0img, const __bf16* x1img,
                                                     const __bf16* x2img, Tr tr) {
  SD_TR_BEGIN
  constexpr int BM = 64, BN = 64, TN = 4, NH = NKT - 24;  // NH: deter tiles (Dg / 32); 8 tiles each of x0 / x1 / x2
  constexpr int STG = BN * LROW6, BP = BN * PRE_ROW / 8 / 256;  // LDS stage (bf16); 16-B B pieces per thread
  static_assert(BN * PRE_ROW / 8 == 256 * BP, "whole B pieces per thread");
  __bf16* smem = sd_smem6<KH_STAGES * STG>();
  const int Dg = d.D / d.G, M = d.N;
  const int n0 = xcd_col(blockIdx.x, gridDim.x, Dg / BN) * BN, m0 = blockIdx.y * BM, g = n0 / Dg;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l16 = lane & 15, q = lane >> 4;
  SD_TR(1)
  // this lane's A row in the 64-row image tiles (tile m0 / 64), plane offsets 0 / 32 / 64 at k 8q
  const long rt = m0 / 64, lrow = (long)(16 * wave + l16) * PRE_ROW + 8 * q;
  const __bf16* ah = himg + (rt * (d.D / BK6) + (long)g * Dg / BK6) * 64 * PRE_ROW + lrow;
  const __bf16* a0 = x0img + rt * 8 * 64 * PRE_ROW + lrow;
  const __bf16* a1 = x1img + rt * 8 * 64 * PRE_ROW + lrow;
  const __bf16* a2 = x2img + rt * 8 * 64 * PRE_ROW + lrow;
  const __bf16* bt = wh6 + (long)(n0 / BN) * NKT * BN * PRE_ROW + tid * 8;  // this thread's first B piece of tile 0
  auto aptr = [&](int kt) {  // (kt is a compile-time constant in the unrolled loop)
    return kt < NH ? ah + (long)kt * 64 * PRE_ROW
                   : (kt < NH + 8 ? a0 : kt < NH + 16 ? a1 : a2) + (long)((kt - NH) % 8) * 64 * PRE_ROW;
  };
  u32x4 A[3][3], B[2][BP];  // A: tiles kt, kt+1, kt+2 (3 planes each); B: pieces of the tiles two / three ahead
  auto load_a = [&](u32x4 (&a)[3], int kt) {
    const __bf16* p = aptr(kt);
#pragma unroll
    for (int s = 0; s < 3; ++s) a[s] = *reinterpret_cast<const u32x4*>(p + s * BK6);
  };
  auto load_b = [&](u32x4 (&b)[BP], int kt) {
#pragma unroll
    for (int u = 0; u < BP; ++u) b[u] = *reinterpret_cast<const u32x4*>(bt + ((long)kt * BN * PRE_ROW + u * 256 * 8));
  };
  auto store_b = [&](const u32x4 (&b)[BP], __bf16* st, int u) {
    const int i = tid + 256 * u;
    *reinterpret_cast<u32x4*>(st + (i / (PRE_ROW / 8)) * LROW6 + (i % (PRE_ROW / 8)) * 8) = b[u];
  };
  // B fragments of a stage: tile j's are read during step j - 1 (KH_STAGES 3: the stage was written a step earlier)
  // or at the start of step j (2 stages)
  bf16x8 fb[2][TN][3];
  auto read_b = [&](bf16x8 (&f)[TN][3], const __bf16* st, int j) {
    const __bf16* pb = st + (16 * j + l16) * LROW6 + 8 * q;
#pragma unroll
    for (int s = 0; s < 3; ++s) f[j][s] = *reinterpret_cast<const bf16x8*>(pb + s * BK6);
  };
  f32x4 acc[1][TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) acc[0][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bpre[TN];  // the epilogue's bias values, loaded ahead of the main loop
#pragma unroll
  for (int j = 0; j < TN; ++j) bpre[j] = d.bh[n0 + 16 * j + l16];
  constexpr int NS = KH_STAGES;
  load_a(A[0], 0);
  load_b(B[0], 0);
  load_a(A[1], 1);
  load_b(B[1], 1);
#pragma unroll
  for (int u = 0; u < BP; ++u) store_b(B[0], smem, u);
  if constexpr (NS == 3) {
#pragma unroll
    for (int u = 0; u < BP; ++u) store_b(B[1], smem + STG, u);
    load_b(B[0], 2);
  }
  __syncthreads();
  if constexpr (NS == 3) {
#pragma unroll
    for (int j = 0; j < TN; ++j) read_b(fb[0], smem, j);
  }
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    // B pieces in flight: 2 stages: tile kt+2 into set kt % 2 (tile kt+1, set (kt+1) % 2, is stored this step);
    // 3 stages: tile kt+3 into set (kt+1) % 2 (tile kt+2, set kt % 2, is stored this step)
    if (kt + NS < NKT) load_b(B[(kt + NS) % 2], kt + NS);
    if (kt + 2 < NKT) load_a(A[(kt + 2) % 3], kt + 2);
    __builtin_amdgcn_sched_barrier(0);  // the loads first
    const int ts = kt + NS - 1;  // the tile this step stages
    __bf16* stg = smem + (ts % NS) * STG;
    bf16x8(&f)[TN][3] = fb[kt % 2];
    if constexpr (NS == 2) {
#pragma unroll
      for (int j = 0; j < TN; ++j) read_b(f, smem + (kt % 2) * STG, j);
    }
    // gemm6_core.h's six products per accumulator in its order (a2b0, a1b1, a0b2, a1b0, a0b1, a0b0), as six passes over
    // the four accumulators; between the passes the staged tile's pieces and (3 stages) tile kt+1's fragments
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int as = u == 0 ? 2 : (u == 1 || u == 3) ? 1 : 0, bs = u == 0 || u == 3 || u == 5 ? 0 : u == 2 ? 2 : 1;
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, A[kt % 3][as]), f[j][bs],
                                                            acc[0][j], 0, 0, 0);
      if (ts < NKT && u < BP) store_b(B[ts % 2], stg, u);
      if (NS == 3 && kt + 1 < NKT && u >= 1 && u <= TN) read_b(fb[(kt + 1) % 2], smem + ((kt + 1) % NS) * STG, u - 1);
    }
    __syncthreads();
  }
  SD_TR(2)
  ep_bias_part<BM, BN, 64, KH_PW>(acc, d.bh, hp, d.D, ph, M, m0, n0, nullptr, bpre, (IMG_NT & 4) != 0);
  SD_TR_END(tr.p, tr.slot)
}

// k_lin6 on register A operands (KL_AREG): the step's three (N, D) x (D, U) deter contractions as one (N, D) x
// (D, nprob * U) product over the problems' concatenated columns, in 64-row x (16 NSUB)-column tiles of 512 threads
// whose K range is split between the two halves of the workgroup (waves 0-3: k tiles 0 .. NKH - 1, waves 4-7:
// NKH .. 2 NKH - 1). Each half has k_hid_areg's structure: wave w's 16 rows loaded per lane from the deter image into
// register fragments two tiles ahead, the half's weight tile through its own double-buffered LDS stage, 6 NSUB MFMAs
// per A fragment set (k_lin6's 32 x 32 tiles have 6, too few to pay for fragment-shaped loads, profiles/r05za); then
// the halves exchange half of their accumulators through LDS and each runs k_lin6's epilogue on two of every lane's
// four rows. NSUB = 3 (48 columns: 16 x 16 =
// 256 workgroups for three problems, one per CU) or 4 (the two-problem launch). The weight images are in 16-column
// tiles (k_presplit6<16>), so a tile's three or four 16-column pieces may come from different problems; the 16-column
// row-partial groups never straddle two. The halves' sums are added at the end, so the outputs agree with k_lin6's
// one pass to fp32 rounding, not bit for bit (test_lin6_areg_matches_lin6); NSUB 3 and 4 give the same values.
#ifndef KL_AREG
#define KL_AREG 1
#endif
#ifndef KL_KQ  // K parts per workgroup (256 threads each): 2, or 4 (1,024 threads, 4 waves per SIMD: k_lin span 25.6 ->
#define KL_KQ 2  // 24.7 us but the main loop unchanged at 20.8 us, update 10.82 -> 10.87 ms, profiles/r05kq)
#endif
#ifndef KL_NSUB  // 16-column pieces per tile of the three-problem launch
#define KL_NSUB 3
#endif
template <int NKH, int NSUB, int KQ>
__global__ __launch_bounds__(256 * KQ, KQ == 4 ? 4 : 2) void k_lin6_areg(const __bf16* aimg, int K, const __bf16* w0, const __bf16* w1,
                                                      const __bf16* w2, LinProb p0, LinProb p1, LinProb p2, int U,
                                                      int M, Tr tr) {
  SD_TR_BEGIN
  constexpr int BM = 64, BN = 16 * NSUB, NS = 2, PPS = 16 * PRE_ROW / 8;  // PPS: 16-B pieces per 16-column piece
  constexpr int STG = BN * LROW6, BP = (NSUB * PPS + 255) / 256;
  static_assert(KQ * BM * (BN + 4) * 4 <= KQ * NS * STG * 2, "reduce buffer within the stages");
  __bf16* smem = sd_smem6<KQ * NS * STG>();
  int tx = blockIdx.x, ty = blockIdx.y, tz = 0;
  if (KL_XCD) xcd_tile(tx, ty, tz);
  const int c0 = tx * BN, m0 = ty * BM, nkt = K / BK6;
  const int tid = threadIdx.x, half = tid >> 8, htid = tid & 255, lane = tid & 63, wave = (tid >> 6) & 3;  // half: K part
  const int l16 = lane & 15, q = lane >> 4;
  SD_TR(1)
  const int kt0 = half * NKH;
  const __bf16* ah = aimg + ((long)(m0 / 64) * nkt + kt0) * 64 * PRE_ROW + (long)(16 * wave + l16) * PRE_ROW + 8 * q;
  // this thread's B pieces: piece i = htid + 256 u of the tile, 16-column piece i / PPS (column c0 + 16 (i / PPS))
  const __bf16* bt[BP];
  int boff[BP];
#pragma unroll
  for (int u = 0; u < BP; ++u) {
    const int i = htid + 256 * u, sp = i < NSUB * PPS ? i / PPS : 0, c = c0 + 16 * sp, pz = c / U;
    const __bf16* img = pz == 0 ? w0 : (pz == 1 ? w1 : w2);
    bt[u] = img + (((long)((c % U) / 16) * nkt + kt0) * 16) * PRE_ROW + (i % PPS) * 8;
    boff[u] = (16 * sp + (i % PPS) / (PRE_ROW / 8)) * LROW6 + (i % (PRE_ROW / 8)) * 8;
  }
  auto live = [&](int u) { return 256 * (u + 1) <= NSUB * PPS || htid + 256 * u < NSUB * PPS; };
  __bf16* hs = smem + half * NS * STG;
  u32x4 A[3][3], B[2][BP];
  auto load_a = [&](u32x4 (&a)[3], int kt) {
    const __bf16* pa = ah + (long)kt * 64 * PRE_ROW;
#pragma unroll
    for (int s = 0; s < 3; ++s) a[s] = *reinterpret_cast<const u32x4*>(pa + s * BK6);
  };
  auto load_b = [&](u32x4 (&b)[BP], int kt) {
#pragma unroll
    for (int u = 0; u < BP; ++u)
      if (live(u)) b[u] = *reinterpret_cast<const u32x4*>(bt[u] + (long)kt * 16 * PRE_ROW);
  };
  auto store_b = [&](const u32x4 (&b)[BP], __bf16* st, int u) {
    if (live(u)) *reinterpret_cast<u32x4*>(st + boff[u]) = b[u];
  };
  bf16x8 f[NSUB][3];
  f32x4 acc[NSUB];
#pragma unroll
  for (int j = 0; j < NSUB; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the epilogue's bias values, loaded ahead of the main loop (a problem without a bias reads a valid dummy address,
  // unconditionally, and takes 0)
  float bpre[NSUB];
#pragma unroll
  for (int j = 0; j < NSUB; ++j) {
    const int c = c0 + 16 * j, pz = c / U;
    const float* bp = pz == 0 ? p0.bias : (pz == 1 ? p1.bias : p2.bias);
    const float bl = (bp ? bp : reinterpret_cast<const float*>(aimg))[c % U + l16];
    bpre[j] = bp ? bl : 0.f;
  }
  load_a(A[0], 0);
  load_b(B[0], 0);
  load_a(A[1], 1);
  load_b(B[1], 1);
#pragma unroll
  for (int u = 0; u < BP; ++u) store_b(B[0], hs, u);
  __syncthreads();
#pragma unroll
  for (int kt = 0; kt < NKH; ++kt) {
    if (kt + NS < NKH) load_b(B[(kt + NS) % 2], kt + NS);
    if (kt + 2 < NKH) load_a(A[(kt + 2) % 3], kt + 2);
    __builtin_amdgcn_sched_barrier(0);  // the loads first
    const int ts = kt + 1;  // the tile this step stages
    __bf16* stg = hs + (ts % NS) * STG;
#pragma unroll
    for (int j = 0; j < NSUB; ++j) {
      const __bf16* pb = hs + (kt % NS) * STG + (16 * j + l16) * LROW6 + 8 * q;
#pragma unroll
      for (int s = 0; s < 3; ++s) f[j][s] = *reinterpret_cast<const bf16x8*>(pb + s * BK6);
    }
    // gemm6_core.h's six products per accumulator in its order, as six passes over the accumulators
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int as = u == 0 ? 2 : (u == 1 || u == 3) ? 1 : 0, bs = u == 0 || u == 3 || u == 5 ? 0 : u == 2 ? 2 : 1;
#pragma unroll
      for (int j = 0; j < NSUB; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, A[kt % 3][as]), f[j][bs], acc[j],
                                                         0, 0, 0);
      if (ts < NKH && u < BP) store_b(B[ts % 2], stg, u);
    }
    __syncthreads();
  }
  SD_TR(2)
  // the K parts' sums meet through LDS (the stages are free after the loop's last barrier): part p finishes rows
  // r = p RPP .. of each lane's four, adding the KQ parts in index order (KQ = 2: a + b = b + a either way), so every
  // part runs the epilogue
  constexpr int LDR = BN + 4, RPP = 4 / KQ;
  float* red = reinterpret_cast<float*>(smem);
  const int rk = RPP * half;  // the rows this part keeps; it hands over the others
#pragma unroll
  for (int j = 0; j < NSUB; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (r / RPP != half) red[((half * BM) + 16 * wave + 4 * q + r) * LDR + 16 * j + l16] = acc[j][r];
  __syncthreads();
  // ep_bias_part's arithmetic per 16-column piece of its problem: out = acc + bias (+ add), part = the piece's sum
  // of squares (one 16-column group)
#pragma unroll
  for (int j = 0; j < NSUB; ++j) {
    const int c = c0 + 16 * j, pz = c / U, n = c % U + l16;
    const LinProb& p = pz == 0 ? p0 : (pz == 1 ? p1 : p2);
    const float bv = bpre[j];
    float ss[RPP];
#pragma unroll
    for (int i = 0; i < RPP; ++i) {
      const int r = rk + i, m = m0 + 16 * wave + 4 * q + r, o = (16 * wave + 4 * q + r) * LDR + 16 * j + l16;
      float sum = half == 0 ? acc[j][r] : red[o];
#pragma unroll
      for (int pp = 1; pp < KQ; ++pp) sum += pp == half ? acc[j][r] : red[pp * BM * LDR + o];
      float v = sum + bv;
      if (p.add && m < M) v += p.add[(long)m * p.ldo + n];
      if (m < M) p.out[(long)m * p.ldo + n] = v;
      ss[i] = 0.f;
      ss[i] += v * v;
    }
#pragma unroll
    for (int i = 0; i < RPP; ++i) {
      const float sv = group_sum<16>(ss[i]);
      const int m = m0 + 16 * wave + 4 * q + rk + i;
      if (l16 == 0 && p.part && m < M) p.part[(long)((c % U) / 16) * M + m] = sv;
    }
  }
  SD_TR_END(tr.p, tr.slot)
}

// gates = BlockLinear(dyn_gru)(silu(rms(hp))) + bg; deter' = GRU (rssm.py:65-75) -> feats[t+1][:, SK:].
// Tile: 64 rows x (r | c | u) for 32 deter columns of block g (BN = 96). grid (D/32, M/64)
// k_gate's B operand: the pre-split image of tile c0 / 32, or the r / c / u gate rows of Wg split while staged
template <bool PRE, int BN>
SD_DEV auto gate_b(const __bf16* wg6, int ct, int nkt, const float* Wblk, int Dg, int j0) {
  if constexpr (PRE)
    return BPre6<BN>(wg6, ct, nkt, 0);
  else
    return BRows<BN>(Wblk, Dg, j0, 32, Dg);
}
#ifndef KG_PRE  // k_gate reads _dyn_gru's weight from the once-per-imagination pre-split image (BPre6)
#define KG_PRE 1
#endif
#ifndef KG_HOLDPF  // k_gate loads its GRU epilogue operands before the main loop
#define KG_HOLDPF 1
#endif
#ifndef KG_WAVES  // minimum waves per SIMD for k_gate's register allocation (occupancy; its LDS admits 4 per CU)
#define KG_WAVES 4
#endif
__global__ __launch_bounds__(256, KG_WAVES) void k_gate(sd_imagine d, const float* hp, const float* ph, int nph,
                                              const float* hold, float* hnew, long ldf, const __bf16* wg6,
                                              __bf16* himg, Tr tr) {
  SD_TR_BEGIN
  constexpr int BM = 64, BN = 96;
  const int Dg = d.D / d.G;
  const int c0 = xcd_col(blockIdx.x, gridDim.x, Dg / 32) * 32, m0 = blockIdx.y * BM, g = c0 / Dg, j0 = c0 % Dg;
  __shared__ float rs[BM], red[256];
  wg_rstd<BM, 16>(ph, nph, d.N, m0, d.D, d.eps, rs, red);
  SD_TR(1)
  const ARms<BM> a0(hp + (long)g * Dg, d.D, d.nh + (long)g * Dg, rs, m0, d.N, Dg);
  constexpr bool PRE = KG_PRE && KG_1S && F6_GATE;
  using OpB = std::conditional_t<PRE, BPre6<BN>, BRows<BN>>;
  const OpB b0 = gate_b<PRE, BN>(wg6, c0 / 32, Dg / BK6, d.Wg + (long)g * 3 * Dg * Dg, Dg, j0);
  // the GRU epilogue's operands (old deter, gate biases) loaded before the main loop (KG_HOLDPF), rows clamped: they
  // arrive with the first k tile instead of as a dependent round trip after the last
  const Lane L = lane_ids<BN, BN>();
  const float* bg = d.bg + (long)g * 3 * Dg;
  float hold_[2][4], bias_[2][3];
  if (KG_HOLDPF) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int c = 16 * j + L.l16, jj = j0 + c, col = c0 + c;
      bias_[j][0] = bg[jj];
      bias_[j][1] = bg[Dg + jj];
      bias_[j][2] = bg[2 * Dg + jj];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long m = m0 + L.wr * 16 + 4 * L.q + r;
        hold_[j][r] = hold[(m < d.N ? m : d.N - 1) * ldf + col];
      }
    }
  }
  f32x4 acc[1][6];
  if constexpr (KG_1S && F6_GATE) {
    ARms<BM> la[KG_PF];
    OpB lb[KG_PF];
#pragma unroll
    for (int u = 0; u < KG_PF; ++u) {
      la[u] = a0;
      lb[u] = b0;
    }
    gemm6_mainloop_1s<BM, BN, 16, BN, KG_PF>(la, lb, 0, Dg, acc);
  } else {
    mainloop<F6_GATE, FP_GATE, BM, BN, 16, BN, pf_of(KG_PF)>(a0, b0, 0, Dg, acc);
  }
  SD_TR(2)
  float hv_[2][4] = {};
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = 16 * j + L.l16, jj = j0 + c, col = c0 + c;
    const float br = KG_HOLDPF ? bias_[j][0] : bg[jj], bc = KG_HOLDPF ? bias_[j][1] : bg[Dg + jj],
                bu = KG_HOLDPF ? bias_[j][2] : bg[2 * Dg + jj];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long m = m0 + L.wr * 16 + 4 * L.q + r;
      if (m >= d.N) continue;
      const float ra = acc[0][j][r] + br, ca = acc[0][2 + j][r] + bc, ua = acc[0][4 + j][r] + bu;
      const float rs = sigmoidf_(ra);
      const float cc = tanhf(rs * ca);
      const float u = sigmoidf_(ua - 1.f);
      const float hv = u * cc + (1.f - u) * (KG_HOLDPF ? hold_[j][r] : hold[m * ldf + col]);
      if (IMG_NT & 1)
        __builtin_nontemporal_store(hv, hnew + m * ldf + col);
      else
        hnew[m * ldf + col] = hv;
      hv_[j][r] = hv;
    }
  }
  if (himg) {  // the 64 x 32 tile of the new deter is exactly one pre-split image tile: staged in LDS, split, written
    constexpr int STG = (BM + BN) * LROW6;
    float* T = reinterpret_cast<float*>(sd_smem6<STG>());  // the main loop's image, free now
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) T[(L.wr * 16 + 4 * L.q + r) * 36 + 16 * j + L.l16] = hv_[j][r];
    __syncthreads();
    const int row = threadIdx.x >> 2, c8 = (threadIdx.x & 3) * 8;
    if (m0 + row < d.N) {
      if (IMG_NT & 2) {
        pre_store4_nt(himg, m0 + row, c0 + c8, d.D, *reinterpret_cast<const f32x4*>(T + row * 36 + c8));
        pre_store4_nt(himg, m0 + row, c0 + c8 + 4, d.D, *reinterpret_cast<const f32x4*>(T + row * 36 + c8 + 4));
      } else {
        pre_store4(himg, m0 + row, c0 + c8, d.D, *reinterpret_cast<const f32x4*>(T + row * 36 + c8));
        pre_store4(himg, m0 + row, c0 + c8 + 4, d.D, *reinterpret_cast<const f32x4*>(T + row * 36 + c8 + 4));
      }
    }
  }
  SD_TR_END(tr.p, tr.slot)
}

// prior logits = img_net_logit(silu(rms(x))) and the unimix one-hot ST sample -> feats[t+1][:, :SK].
// BM = 16, BN = 64 (4 waves along N), grid (SK/64, M/16): 512 workgroups at the bench shape so the sampler epilogue
// (Philox noise + unimix softmax per element) runs 4 elements per thread; the tile is staged through LDS and sampled
// by teams of KD threads.
template <int KD>
__global__ __launch_bounds__(256) void k_prior(sd_imagine d, const float* X, const float* nw, const float* part_in,
                                               int np, float* snew, long ldf, int t, Tr tr) {
  SD_TR_BEGIN
  constexpr int BM = 16, BN = 64, WN = 16;
  __shared__ float tile[BM][BN + 1];
  __shared__ float rs[BM], red[256];
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM, U = d.U, S = d.SK / KD;
  // the sampler's Gumbel noise depends on no operand: drawn first, so its Philox + f64 logs overlap the loads and
  // the MFMAs instead of following them
  constexpr int NK = BM * BN / 256;
  const uint64_t seed = d.seed + (d.seed_ptr ? *d.seed_ptr : 0ull);
  float gns[NK];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int i = threadIdx.x + 256 * k, rl = i / BN, c = i % BN;
    if (d.noise_img)  // drawn ahead (sd_imagine_noise): the same values
      gns[k] = m0 + rl < d.N ? d.noise_img[((long)t * d.N + m0 + rl) * d.SK + n0 + c] : 0.f;
    else
      gns[k] = sd_gumbel(seed, (uint32_t)d.stream_img, (uint32_t)t,
                         (uint64_t)((m0 + rl + d.row_offset) * S + (n0 + c) / KD) * KD + c % KD);
  }
  wg_rstd<BM, 8>(part_in, np, d.N, m0, U, d.eps, rs, red);
  SD_TR(1)
  const ARms<BM> a0(X, U, nw, rs, m0, d.N, U);
  const BRows<BN> b0(d.Wl, U, n0, BN, 0);
  f32x4 acc[1][1];
  mainloop<F6_PRIOR, FP_PRIOR, BM, BN, 16, WN, pf_of(FP_PRIOR ? 2 : 3)>(a0, b0, 0, U, acc);
  SD_TR(2)
  const Lane L = lane_ids<BN, WN>();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int c = L.wc * WN + L.l16;
    tile[4 * L.q + r][c] = acc[0][0][r] + d.bl[n0 + c];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int i = threadIdx.x + 256 * k;
    const int rl = i / BN, c = i % BN, lt = c % KD;
    const long m = m0 + rl;
    const float l = tile[rl][c];
    float p, pp, nl;
    unimix_forward<KD>(l, true, KD, d.unimix, p, pp, nl);
    float ys;
    int idx;
    st_soft<KD>(nl, gns[k], true, ys, idx, lt);
    if (m < d.N) snew[m * ldf + n0 + c] = ((lt == idx ? 1.f : 0.f) - ys) + ys;
  }
  SD_TR_END(tr.p, tr.slot)
}

// k_prior on RTile<16>: grid (SK / 64, M / 16); NT = 1024 threads (one sampler element per thread: row i / 64, column
// i % 64, teams of KD lanes) or NT = 512 (RTile16h, the same sums; elements tid and tid + 512); the noise drawn / read
// before the contraction
template <int KD, int NT>
__global__ __launch_bounds__(NT, NT == 1024 ? 8 : 4) void k_prior_rw(sd_imagine d, const float* X, const float* nw,
                                                                   const float* part_in, int np, float* snew, long ldf,
                                                                   int t, Tr tr) {
  SD_TR_BEGIN
  using RT = typename std::conditional<NT == 1024, RTile<16>, RTile16h>::type;
  constexpr int PE = 1024 / NT;  // sampler elements per thread
  __shared__ __attribute__((aligned(16))) float P[16 * RT::LDP];
  __shared__ float red[16 * 4 * 64];
  __shared__ float T[16 * 65];
  const int tid = threadIdx.x, n0 = blockIdx.x * 64, m0 = blockIdx.y * 16, S = d.SK / KD;
  RT rt;
  rt.load_w(d.Wl, RT::U, n0);
  float gn[PE], blv[PE];
#pragma unroll
  for (int e = 0; e < PE; ++e) {
    const int i = tid + NT * e, rl = i >> 6, c = i & 63;
    const long m = m0 + rl, mc = m < d.N ? m : d.N - 1;
    // drawn ahead (sd_imagine_noise, the same values): one unconditional load (address select), else drawn below
    gn[e] = *(d.noise_img ? d.noise_img + ((long)t * d.N + mc) * d.SK + n0 + c : d.bl + n0 + c);
    blv[e] = d.bl[n0 + c];
  }
  RT::stage(P, X, RT::U, nw, part_in, np, d.N, m0, d.eps);  // (its wait covers the noise loads issued before)
  if (!d.noise_img) {
    const uint64_t seed = d.seed + (d.seed_ptr ? *d.seed_ptr : 0ull);
#pragma unroll
    for (int e = 0; e < PE; ++e) {
      const int i = tid + NT * e, rl = i >> 6, c = i & 63, lt = c % KD;
      gn[e] = sd_gumbel(seed, (uint32_t)d.stream_img, (uint32_t)t,
                        (uint64_t)((m0 + rl + d.row_offset) * S + (n0 + c) / KD) * KD + lt);
    }
  }
  __syncthreads();
  SD_TR(1)
  rt.mma(P);
  rt.reduce(red, T);
  SD_TR(2)
#pragma unroll
  for (int e = 0; e < PE; ++e) {
    const int i = tid + NT * e, rl = i >> 6, c = i & 63, lt = c % KD;
    const long m = m0 + rl;
    const float l = T[rl * 65 + c] + blv[e];
    float p, pp, nl;
    unimix_forward<KD>(l, true, KD, d.unimix, p, pp, nl);
    float ys;
    int idx;
    st_soft<KD>(nl, gn[e], true, ys, idx, lt);
    if (m < d.N) snew[m * ldf + n0 + c] = ((lt == idx ? 1.f : 0.f) - ys) + ys;
  }
  SD_TR_END(tr.p, tr.slot)
}

// actor output layer + action sample (bounded normal: loc = tanh, scale in [min_std, max_std]; or unimix one-hot),
// action_norm, and the action branch of the next Deter step: x2 = silu(rms(_dyn_in2(a_n))) (rssm.py:40-46).
// BM = KA_BM rows (16: 64 workgroups at N = 1,024 — the sampler and the x2 epilogue loop over the tile's rows, so
// the per-workgroup chain halves against 32-row tiles), BN = 64 / 32 columns (2A or A <= 32 used), grid (1, M/BM).
#ifndef KA_BM
#define KA_BM 16
#endif
constexpr int KA_BN = KA_BM == 16 ? 64 : 32;  // 4 waves of 16 columns x 16 rows or 2 x 2 waves
__global__ __launch_bounds__(256) void k_action(sd_imagine d, const float* X, const float* nw, const float* part_in,
                                                int np, float* act, float* x2, int t, int want_x2, Tr tr) {
  SD_TR_BEGIN
  constexpr int BM = KA_BM, BN = KA_BN, WN = 16, RT = 256 / BM;  // RT threads per row in the row-sum pass
  __shared__ float tile[BM][BN + 1];
  __shared__ float an[BM][17];
  __shared__ float xs[BM][257];
  __shared__ float rsum[BM][RT + 1];
  const int m0 = blockIdx.y * BM, U = d.U, A = d.A;
  const int NO = d.act_discrete ? A : 2 * A;
  __shared__ float rs[BM], red[256];
  const int tid = threadIdx.x;
  // the action noise (one value per thread) depends on no operand: drawn before the contraction
  const uint64_t seed = d.seed + (d.seed_ptr ? *d.seed_ptr : 0ull);
  float nz = 0.f;
  if (d.act_discrete) {
    static_assert(BM * 16 <= 256, "one sampler element per thread");
    const int lt = tid % 16;
    if (lt < A) nz = sd_gumbel(seed, (uint32_t)d.stream_act, (uint32_t)t, (uint64_t)(m0 + tid / 16 + d.row_offset) * A + lt);
  } else if (tid < BM * A) {
    nz = sd_normal(seed, (uint32_t)d.stream_act, (uint32_t)t, (uint64_t)(m0 + tid / A + d.row_offset) * A + tid % A);
  }
  wg_rstd<BM, 8>(part_in, np, d.N, m0, U, d.eps, rs, red);
  SD_TR(1)
  const ARms<BM> a0(X, U, nw, rs, m0, d.N, U);
  const BRows<BN> b0(d.Wao, U, 0, BN, 0, NO);  // the output weight's NO rows, zeros past them
  f32x4 acc[1][1];
  mainloop<F6_ACTION, FP_ACTION, BM, BN, 16, WN, pf_of(FP_ACTION ? 2 : 3)>(a0, b0, 0, U, acc);
  SD_TR(2)
  const Lane L = lane_ids<BN, WN>();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int c = L.wc * WN + L.l16;
    tile[L.wr * 16 + 4 * L.q + r][c] = acc[0][0][r] + (c < NO ? d.bao[c] : 0.f);
  }
  __syncthreads();
  if (d.act_discrete) {  // team of 16 lanes per row (A <= 16), one-hot ST sample with the actor's unimix
    {
      const int i = tid, rl = i / 16, lt = i % 16;
      const bool on = lt < A;
      const long m = m0 + rl;
      const float l = on ? tile[rl][lt] : 0.f;
      float p, pp, nl;
      unimix_forward<16>(l, on, A, d.act_unimix, p, pp, nl);
      float ys;
      int idx;
      st_soft<16>(nl, nz, on, ys, idx, lt);
      if (on) {
        const float a = ((lt == idx ? 1.f : 0.f) - ys) + ys;
        if (m < d.N) act[m * A + lt] = a;
        an[rl][lt] = a / fmaxf(fabsf(a), 1.f);
      }
    }
  } else if (tid < BM * A) {
    const int rl = tid / A, j = tid % A;
    const long m = m0 + rl;
    const float loc = tanhf(tile[rl][j]);
    const float sc = (d.max_std - d.min_std) * sigmoidf_(tile[rl][A + j] + 2.f) + d.min_std;
    const float a = loc + nz * sc;
    if (m < d.N) act[m * A + j] = a;
    an[rl][j] = a / fmaxf(fabsf(a), 1.f);
  }
  if (!want_x2) {
    SD_TR_END(tr.p, tr.slot)
    return;
  }
  __syncthreads();
  // x2p[row][c] = a_n[row] . W2[c] + b2[c]; thread c = tid (U == 256 columns), all 32 rows
  {
    const int c = tid;
    float w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = j < A ? d.W2[(long)c * A + j] : 0.f;
    const float b = d.b2[c];
    for (int rl = 0; rl < BM; ++rl) {
      float v = b;
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (j < A) v += an[rl][j] * w[j];
      xs[rl][c] = v;
    }
  }
  __syncthreads();
  {  // row sums of squares: RT threads per row
    const int rl = tid / RT, part = tid % RT;
    float s = 0.f;
    for (int c = part; c < U; c += RT) s += xs[rl][c] * xs[rl][c];
    rsum[rl][part] = s;
  }
  __syncthreads();
  {
    const int c = tid;
    const float wn = d.n2[c];
    for (int rl = 0; rl < BM; ++rl) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < RT; ++k) s += rsum[rl][k];
      const float rs = rsqrtf(s / (float)U + d.eps);
      if (m0 + rl < d.N) x2[(long)(m0 + rl) * U + c] = siluf_(xs[rl][c] * rs * wn);
    }
  }
  SD_TR_END(tr.p, tr.slot)
}

// k_action by rows (KA_ROWS): one wave per row, 4 rows per workgroup (N / 4 workgroups: 256 at the bench shape instead
// of 64 16-row tiles). The chain has no workgroup barrier: the row's RMSNorm from the producer's partials, the actor
// output layer as fp32 dot products (4 columns per lane, one wave reduction per output), the action sample (bounded
// normal / unimix one-hot on lanes 0..15), action_norm, and the next Deter step's action branch x2 = silu(rms(a_n .
// W2^T + b2)) for the lane's 4 columns. Same noise indices as k_action; fp32 dot products in a different summation
// order than the MFMA tile (parity: continuous actions to tolerance, one-hot samples exact off near-ties).
#ifndef KA_ROWS
#define KA_ROWS 1
#endif
// X0: also the next k_hid's x0 operand as a pre-split image, x0img = split(silu(rms(x0p) * n0)) (k_hid_areg; the
// row's rstd summed from k_lin6's partials in wg_rstd<64, 8>'s association, so the planes are those k_hid's own ARms
// loader would stage)
struct X0Img {
  const float* x0p;
  const float* px0;
  int npx0;
  __bf16* img;
};
template <int MO>  // >= the output logits (2A or A): 16 or 32
__global__ __launch_bounds__(256) void k_action_rows(sd_imagine d, const float* X, const float* nw,
                                                     const float* part_in, int np, float* act, float* x2, int t,
                                                     int want_x2, __bf16* x2img, X0Img x0i, Tr tr) {
  SD_TR_BEGIN
  constexpr int U = 256, MA = 16;  // <= 16 actions
  __shared__ float w2s[U * MA];    // _dyn_in2's weight (U, A), staged coalesced while the logits chain runs
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long m = (long)blockIdx.x * 4 + wave;
  const int A = d.A, NO = d.act_discrete ? A : 2 * A, M = d.N;
  const bool live = m < M;
  const uint64_t seed = d.seed + (d.seed_ptr ? *d.seed_ptr : 0ull);
  // operand loads first, every one unconditional (clamped row / partial / output-row indices; values past them are
  // masked where used — a "cond ? load : 0" made hipcc branch around each load and drain the queue at the join): the
  // row's partials, its 4 columns, the norm weight, the output layer's rows, then _dyn_in2's weight (into registers,
  // stored to LDS after the logits, so the logits chain waits on none of it) and the drawn-ahead action noise
  const long mc = live ? m : M - 1;
  const float pv_ = part_in[(long)(lane < np ? lane : np - 1) * M + mc];
  const f32x4 xv = ld4(X + mc * U + 4 * lane);
  const f32x4 wn = ld4(nw + 4 * lane);
  f32x4 wo[MO];
#pragma unroll
  for (int o = 0; o < MO; ++o) wo[o] = ld4(d.Wao + (long)(o < NO ? o : NO - 1) * U + 4 * lane);
  const float bo_ = d.bao[lane < NO ? lane : NO - 1];
  const bool x2w = want_x2 != 0;
  constexpr int W2R = U * MA / 256;
  float w2r[W2R];
#pragma unroll
  for (int k = 0; k < W2R; ++k) {
    const int i = threadIdx.x + 256 * k;
    w2r[k] = d.W2[i < U * A ? i : U * A - 1];
  }
  const f32x4 b2 = ld4(d.b2 + 4 * lane), n2 = ld4(d.n2 + 4 * lane);
  const bool x0w = x0i.img != nullptr && want_x2 != 0;  // (uniform over the launch)
  const float* x0src = x0w ? x0i.x0p : X;  // (a valid row either way: the loads stay unconditional)
  const f32x4 x0v = ld4(x0src + mc * U + 4 * lane), n0v = ld4((x0w ? d.n0 : nw) + 4 * lane);
  const int np0 = x0w ? x0i.npx0 : np;
  const float p0_ = (x0w ? x0i.px0 : part_in)[(long)(lane < np0 ? lane : np0 - 1) * M + mc];
  const int la = lane < A ? lane : A - 1;
  float nz = *(d.noise_act ? d.noise_act + ((long)t * M + mc) * A + la : d.b2);
  if (!d.noise_act) {  // drawn here (the same counter-based values as the drawn-ahead noise)
    nz = 0.f;
    if (d.act_discrete) {
      if (lane < A) nz = sd_gumbel(seed, (uint32_t)d.stream_act, (uint32_t)t, (uint64_t)(m + d.row_offset) * A + lane);
    } else if (lane < A) {
      nz = sd_normal(seed, (uint32_t)d.stream_act, (uint32_t)t, (uint64_t)(m + d.row_offset) * A + lane);
    }
  } else if (!(live && lane < A)) {
    nz = 0.f;
  }
  const float pv = (live && lane < np) ? pv_ : 0.f, bo = lane < NO ? bo_ : 0.f;
  const float rs = rsqrtf(wave_sum(pv) / (float)U + d.eps);
  SD_TR(1)
  f32x4 y;
#pragma unroll
  for (int j = 0; j < 4; ++j) y[j] = siluf_(xv[j] * rs * wn[j]);
  // the NO dot products, reduced over the wave stage by stage (independent shuffles in flight together)
  float pd[MO];
#pragma unroll
  for (int o = 0; o < MO; ++o) {
    float v = y[0] * wo[o][0];
    v = fmaf(y[1], wo[o][1], v);
    v = fmaf(y[2], wo[o][2], v);
    pd[o] = fmaf(y[3], wo[o][3], v);
  }
#pragma unroll
  for (int sh = 32; sh > 0; sh >>= 1)
#pragma unroll
    for (int o = 0; o < MO; ++o)
      if (o < NO) pd[o] += __shfl_xor(pd[o], sh, 64);
  float lo = 0.f;  // lane o < NO: logit o (lanes past NO: 0, as with the former zero rows)
#pragma unroll
  for (int o = 0; o < MO; ++o)
    if (lane == o && o < NO) lo = pd[o];
  lo += bo;
  SD_TR(2)
  float a = 0.f;  // lane j < A: action element j
  if (d.act_discrete) {
    const bool on = lane < A;
    float p, pp, nl;
    unimix_forward<16>(lo, on, A, d.act_unimix, p, pp, nl);  // lanes 0..15 form the team
    float ys;
    int idx;
    st_soft<16>(nl, nz, on, ys, idx, lane & 15);
    if (on) a = ((lane == idx ? 1.f : 0.f) - ys) + ys;
  } else {
    const float ls = __shfl(lo, lane + A, 64);  // the scale logit of element lane
    if (lane < A) {
      const float loc = tanhf(lo);
      const float sc = (d.max_std - d.min_std) * sigmoidf_(ls + 2.f) + d.min_std;
      a = loc + nz * sc;
    }
  }
  if (live && lane < A) act[m * A + lane] = a;
  if (x0w) {  // wg_rstd<64, 8>: partial group g = p % 4 sums p = g, g + 4, ... in order, then the groups in order
    const float pp = lane < np0 ? p0_ : 0.f;
    float tt = 0.f;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      float sg = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) sg += __shfl(pp, g + 4 * k, 64);
      tt += sg;
    }
    const float r0 = rsqrtf(tt / (float)U + d.eps);
    f32x4 y0;
#pragma unroll
    for (int j = 0; j < 4; ++j) y0[j] = siluf_(x0v[j] * r0 * n0v[j]);
    if (live) pre_store4(x0i.img, m, 4 * lane, U, y0);
  }
  if (!x2w) {  // (uniform over the launch)
    SD_TR_END(tr.p, tr.slot)
    return;
  }
#pragma unroll
  for (int k = 0; k < W2R; ++k) {
    const int i = threadIdx.x + 256 * k;
    if (i < U * A) w2s[i] = w2r[k];
  }
  __syncthreads();  // w2s staged
  const float an = a / fmaxf(fabsf(a), 1.f);
  float anj[MA];
#pragma unroll
  for (int j = 0; j < MA; ++j) anj[j] = __shfl(an, j, 64);
  // x2p[4 lane + e] = b2 + sum_j a_n[j] W2[4 lane + e][j] (k_action's order: b2 first, then j = 0, 1, ...)
  f32x4 xp = b2;
#pragma unroll
  for (int j = 0; j < MA; ++j)
    if (j < A) {
#pragma unroll
      for (int e = 0; e < 4; ++e) xp[e] += anj[j] * w2s[(4 * lane + e) * A + j];
    }
  const float r2 = rsqrtf(wave_sum(xp[0] * xp[0] + xp[1] * xp[1] + xp[2] * xp[2] + xp[3] * xp[3]) / (float)U + d.eps);
  f32x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = siluf_(xp[e] * r2 * n2[e]);
  if (live) {
    *reinterpret_cast<f32x4*>(x2 + m * U + 4 * lane) = o;
    if (x2img) pre_store4(x2img, m, 4 * lane, U, o);
  }
  SD_TR_END(tr.p, tr.slot)
}

// The actor MLP after layer 0 in ONE launch per 16-row tile (networks.py:313-377): hidden layers 1..L-1
// (RMSNorm + SiLU of the previous layer, Linear), the output layer, the action sample and the x2 branch — what
// k_rmslin x (L-1) + k_action do in L launches. An MLP row needs only its own previous-layer row, so a workgroup that
// owns whole rows (all U = 256 columns: wave wc computes columns 64 wc .. 64 wc + 63) chains the layers through LDS
// with no grid-wide dependency. N / 16 workgroups (64 at the bench shape): the chain is latency-bound either way, and
// the CUs it leaves free run the update's filler phase beside the imagination.
// Arithmetic is bit-identical to the unfused launches: the same k order per output element (lane quad q supplies
// k = 32 kt + 8 q + s at MFMA step s, even steps into acc and odd steps into acc2, acc + acc2 at the end: the
// gemm16_mainloop_fp order at one 16-column tile per wave), the same bias / 16-column row-partial epilogue
// (ep_bias_part) and the same rstd summation order (wg_rstd). B fragments come straight from global memory (each
// wave owns its columns: nothing to share through LDS), three k tiles in flight.
#ifndef SD_FUSED_ACTOR  // measured slower (imagination alone 2.57 -> 2.68 ms): 64 workgroups are MFMA-bound
#define SD_FUSED_ACTOR 0
#endif
constexpr int FA_LD = 256 + 4;  // LDS row stride of the 16 x 256 activation panels (floats)
template <int NJ>
SD_DEV void fa_bload(f32x4 (&b)[NJ][2], const float* W, int ncol0, int nrows, int k0, int l16, int q) {
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int n = ncol0 + 16 * j + l16;
    const float* p = W + (long)n * 256 + k0 + 8 * q;
    b[j][0] = n < nrows ? ld4(p) : zero4();
    b[j][1] = n < nrows ? ld4(p + 4) : zero4();
  }
}
// acc[j] (+ acc2[j]) = P[0:16, :] . W[ncol0 + 16 j + (0..15), :]^T over K = 256, A from the LDS panel P
template <int NJ>
SD_DEV void fa_layer(const float* P, const float* W, int ncol0, int nrows, f32x4 (&acc)[NJ], int l16, int q) {
  constexpr int NKT = 256 / BK, RING = 3;
  f32x4 acc2[NJ], b[RING][NJ][2];
#pragma unroll
  for (int j = 0; j < NJ; ++j) acc[j] = acc2[j] = zero4();
#pragma unroll
  for (int u = 0; u < RING - 1; ++u) fa_bload<NJ>(b[u], W, ncol0, nrows, u * BK, l16, q);
#pragma unroll
  for (int kt = 0; kt < NKT; ++kt) {
    // the loads of tile kt + RING - 1 go out before this tile's MFMAs (the scheduler would otherwise sink them to
    // their use and wait on each L2 round trip)
    if (kt + RING - 1 < NKT) fa_bload<NJ>(b[(kt + RING - 1) % RING], W, ncol0, nrows, (kt + RING - 1) * BK, l16, q);
    __builtin_amdgcn_sched_barrier(0);
    const float* pa = P + l16 * FA_LD + kt * BK + 8 * q;
    const f32x4 a0 = *reinterpret_cast<const f32x4*>(pa), a1 = *reinterpret_cast<const f32x4*>(pa + 4);
    const int c = kt % RING;
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const float av = s < 4 ? a0[s & 3] : a1[s & 3], bv = b[c][j][s >> 2][s & 3];
        if (s & 1)
          acc2[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc2[j], 0, 0, 0);
        else
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[j], 0, 0, 0);
      }
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) acc[j] += acc2[j];
}
// rs[row] from the 16 LDS row partials part[p][row] (wg_rstd's order), then P = silu(O * rs * nw)
SD_DEV void fa_norm_panel(const float* O, const float (*part)[16], const float* nw, float eps, float* rs, float* P) {
  const int tid = threadIdx.x;
  if (tid < 16) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) t += part[g][tid];
    rs[tid] = rsqrtf(t / 256.f + eps);
  }
  __syncthreads();
  for (int i = tid; i < 16 * 64; i += 256) {
    const int row = i / 64, k = 4 * (i % 64);
    const f32x4 x = *reinterpret_cast<const f32x4*>(O + row * FA_LD + k), w = ld4(nw + k);
    f32x4 y;
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = siluf_(x[j] * rs[row] * w[j]);
    *reinterpret_cast<f32x4*>(P + row * FA_LD + k) = y;
  }
  __syncthreads();
}
__global__ __launch_bounds__(256) void k_actor(sd_imagine d, const float* X, const float* part_in, int np, float* act,
                                               float* x2, int t, int want_x2) {
  constexpr int BM = 16, RT = 256 / BM;
  __shared__ __attribute__((aligned(16))) float P[BM * FA_LD], O[BM * FA_LD];
  __shared__ float part[16][16], rs[BM], red[256];
  __shared__ float tile[BM][33];
  __shared__ float an[BM][17];
  __shared__ float rsum[BM][RT + 1];
  const int m0 = blockIdx.x * BM, U = d.U, A = d.A, L = d.actor_layers;
  const int NO = d.act_discrete ? A : 2 * A;
  const int tid = threadIdx.x, lane = tid & 63, wc = tid >> 6, l16 = lane & 15, q = lane >> 4;
  // layer 1's input panel: silu(rms(X)) of the tile's rows (X = actor layer 0's pre-norm output)
  wg_rstd<BM, 8>(part_in, np, d.N, m0, U, d.eps, rs, red);
  for (int i = tid; i < BM * 64; i += 256) {
    const int row = i / 64, k = 4 * (i % 64), m = m0 + row;
    const f32x4 x = m < d.N ? ld4(X + (long)m * U + k) : zero4(), w = ld4(d.na[0] + k);
    f32x4 y;
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = siluf_(x[j] * rs[row] * w[j]);
    *reinterpret_cast<f32x4*>(P + row * FA_LD + k) = y;
  }
  __syncthreads();
  for (int l = 1; l < L; ++l) {
    f32x4 acc[4];
    fa_layer<4>(P, d.Wa[l], 64 * wc, 1 << 30, acc, l16, q);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = 64 * wc + 16 * j + l16;
      const float bv = d.ba[l][n];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = acc[j][r] + bv;
        O[(4 * q + r) * FA_LD + n] = v;
        const float s = group_sum<16>(v * v);
        if (l16 == 0) part[4 * wc + j][4 * q + r] = s;
      }
    }
    __syncthreads();
    fa_norm_panel(O, part, d.na[l], d.eps, rs, P);
  }
  // output layer: waves 0-1 take columns 0..31 (NO <= 32 used; rows past NO read as 0)
  if (wc < 2) {
    f32x4 acc[1];
    fa_layer<1>(P, d.Wao, 16 * wc, NO, acc, l16, q);
    const int c = 16 * wc + l16;
#pragma unroll
    for (int r = 0; r < 4; ++r) tile[4 * q + r][c] = acc[0][r] + (c < NO ? d.bao[c] : 0.f);
  }
  __syncthreads();
  // action sample + action_norm + x2 = silu(rms(_dyn_in2(a_n))): k_action's epilogue
  const uint64_t seed = d.seed + (d.seed_ptr ? *d.seed_ptr : 0ull);
  if (d.act_discrete) {
    for (int i = tid; i < BM * 16; i += 256) {
      const int rl = i / 16, lt = i % 16;
      const bool on = lt < A;
      const long m = m0 + rl;
      const float lg = on ? tile[rl][lt] : 0.f;
      float p, pp, nl;
      unimix_forward<16>(lg, on, A, d.act_unimix, p, pp, nl);
      const float gn = on ? sd_gumbel(seed, (uint32_t)d.stream_act, (uint32_t)t, (uint64_t)(m + d.row_offset) * A + lt)
                          : 0.f;
      float ys;
      int idx;
      st_soft<16>(nl, gn, on, ys, idx, lt);
      if (on) {
        const float a = ((lt == idx ? 1.f : 0.f) - ys) + ys;
        if (m < d.N) act[m * A + lt] = a;
        an[rl][lt] = a / fmaxf(fabsf(a), 1.f);
      }
    }
  } else {
    for (int i = tid; i < BM * A; i += 256) {
      const int rl = i / A, j = i % A;
      const long m = m0 + rl;
      const float loc = tanhf(tile[rl][j]);
      const float sc = (d.max_std - d.min_std) * sigmoidf_(tile[rl][A + j] + 2.f) + d.min_std;
      const float a = loc + sd_normal(seed, (uint32_t)d.stream_act, (uint32_t)t, (uint64_t)(m + d.row_offset) * A + j) * sc;
      if (m < d.N) act[m * A + j] = a;
      an[rl][j] = a / fmaxf(fabsf(a), 1.f);
    }
  }
  if (!want_x2) return;
  __syncthreads();
  float* xs = O;  // x2 pre-norm rows (row stride FA_LD)
  {
    const int c = tid;
    float w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = j < A ? d.W2[(long)c * A + j] : 0.f;
    const float b = d.b2[c];
    for (int rl = 0; rl < BM; ++rl) {
      float v = b;
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (j < A) v += an[rl][j] * w[j];
      xs[rl * FA_LD + c] = v;
    }
  }
  __syncthreads();
  {
    const int rl = tid / RT, pt = tid % RT;
    float s = 0.f;
    for (int c = pt; c < U; c += RT) s += xs[rl * FA_LD + c] * xs[rl * FA_LD + c];
    rsum[rl][pt] = s;
  }
  __syncthreads();
  {
    const int c = tid;
    const float wn = d.n2[c];
    for (int rl = 0; rl < BM; ++rl) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < RT; ++k) s += rsum[rl][k];
      const float r = rsqrtf(s / (float)U + d.eps);
      if (m0 + rl < d.N) x2[(long)(m0 + rl) * U + c] = siluf_(xs[rl * FA_LD + c] * r * wn);
    }
  }
}

// img_net's hidden layers 1..L-1 + the prior logits + the unimix one-hot sample in ONE launch per (16-row tile,
// SK / NCT logit columns): what k_rmslin x (L-1) + k_prior do in L launches (rssm.py:180-195). Every workgroup of a
// row tile recomputes the tile's hidden rows (whole rows: the next norm needs them), then its logit columns (wave wc:
// SK / NCT / 4 columns), then samples them by teams of KD lanes as k_prior does. Bit-identical to the unfused launches
// (fa_layer's k order, ep_bias_part's partials, wg_rstd's sums). grid (NCT, N / 16).
#ifndef SD_FUSED_PRIOR  // measured slower (2.68 -> 2.85 ms with the fused actor): 4x recomputed hidden layer
#define SD_FUSED_PRIOR 0
#endif
#ifndef SD_PRIOR_NCT
#define SD_PRIOR_NCT 4
#endif
template <int KD, int NJ>
__global__ __launch_bounds__(256) void k_imgprior(sd_imagine d, const float* X, const float* part_in, int np,
                                                  float* snew, long ldf, int t) {
  constexpr int BM = 16, BNW = 64 * NJ;  // logit columns per workgroup (4 waves x 16 NJ)
  __shared__ __attribute__((aligned(16))) float P[BM * FA_LD], O[BM * FA_LD];
  __shared__ float part[16][16], rs[BM], red[256];
  __shared__ float tile[BM][BNW + 1];
  const int n0 = blockIdx.x * BNW, m0 = blockIdx.y * BM, U = d.U, S = d.SK / KD, L = d.img_layers;
  const int tid = threadIdx.x, lane = tid & 63, wc = tid >> 6, l16 = lane & 15, q = lane >> 4;
  wg_rstd<BM, 8>(part_in, np, d.N, m0, U, d.eps, rs, red);
  for (int i = tid; i < BM * 64; i += 256) {
    const int row = i / 64, k = 4 * (i % 64), m = m0 + row;
    const f32x4 x = m < d.N ? ld4(X + (long)m * U + k) : zero4(), w = ld4(d.ni[0] + k);
    f32x4 y;
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = siluf_(x[j] * rs[row] * w[j]);
    *reinterpret_cast<f32x4*>(P + row * FA_LD + k) = y;
  }
  __syncthreads();
  for (int l = 1; l < L; ++l) {
    f32x4 acc[4];
    fa_layer<4>(P, d.Wi[l], 64 * wc, 1 << 30, acc, l16, q);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = 64 * wc + 16 * j + l16;
      const float bv = d.bi[l][n];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = acc[j][r] + bv;
        O[(4 * q + r) * FA_LD + n] = v;
        const float s = group_sum<16>(v * v);
        if (l16 == 0) part[4 * wc + j][4 * q + r] = s;
      }
    }
    __syncthreads();
    fa_norm_panel(O, part, d.ni[l], d.eps, rs, P);
  }
  {
    f32x4 acc[NJ];
    fa_layer<NJ>(P, d.Wl, n0 + 16 * NJ * wc, 1 << 30, acc, l16, q);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int c = 16 * NJ * wc + 16 * j + l16;
#pragma unroll
      for (int r = 0; r < 4; ++r) tile[4 * q + r][c] = acc[j][r] + d.bl[n0 + c];
    }
  }
  __syncthreads();
  const uint64_t seed = d.seed + (d.seed_ptr ? *d.seed_ptr : 0ull);
#pragma unroll
  for (int k = 0; k < BM * BNW / 256; ++k) {
    const int i = tid + 256 * k;
    const int rl = i / BNW, c = i % BNW, lt = c % KD;
    const long m = m0 + rl;
    const int s = (n0 + c) / KD;
    const float lg = tile[rl][c];
    float p, pp, nl;
    unimix_forward<KD>(lg, true, KD, d.unimix, p, pp, nl);
    const float gn = sd_gumbel(seed, (uint32_t)d.stream_img, (uint32_t)t,
                               (uint64_t)((m + d.row_offset) * S + s) * KD + lt);
    float ys;
    int idx;
    st_soft<KD>(nl, gn, true, ys, idx, lt);
    if (m < d.N) snew[m * ldf + n0 + c] = ((lt == idx ? 1.f : 0.f) - ys) + ys;
  }
}

// noise[t][m][k] = sd_gumbel(seed, stream_img, t, (m + row_offset) * SK + k) for t < H1 - 1: one thread per 4
// consecutive k, which share one Philox block (sd_gumbel's word idx & 3), one float4 store
__global__ __launch_bounds__(256) void k_imag_noise(sd_imagine d, float* noise, float* noise_act) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x, per_t = (long)d.N * d.SK / 4;
  const long nact = noise_act ? (long)d.H1 * d.N * d.A : 0;
  if (i < nact) {  // the action noise: the value k_action_rows would draw for (step, row, element)
    const int t = (int)(i / ((long)d.N * d.A));
    const long r = i - (long)t * d.N * d.A, m = r / d.A;
    const int j = (int)(r % d.A);
    const uint64_t seed = d.seed + (d.seed_ptr ? *d.seed_ptr : 0ull);
    const uint64_t e = (uint64_t)(m + d.row_offset) * d.A + j;
    noise_act[i] = d.act_discrete ? sd_gumbel(seed, (uint32_t)d.stream_act, (uint32_t)t, e)
                                  : sd_normal(seed, (uint32_t)d.stream_act, (uint32_t)t, e);
  }
  if (i >= (long)(d.H1 - 1) * per_t) return;
  const int t = (int)(i / per_t);
  const long r = i - (long)t * per_t, m = r / (d.SK / 4), k = 4 * (r % (d.SK / 4));
  const uint64_t seed = d.seed + (d.seed_ptr ? *d.seed_ptr : 0ull);
  const uint64_t q = ((uint64_t)(m + d.row_offset) * d.SK + k) >> 2;
  const sd_u32x4 w = sd_philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), (uint32_t)t, (uint32_t)d.stream_img,
                                      (uint32_t)seed, (uint32_t)(seed >> 32));
  const f32x4 g{(float)(-log(-log(sd_u01(w.x)))), (float)(-log(-log(sd_u01(w.y)))),
                (float)(-log(-log(sd_u01(w.z)))), (float)(-log(-log(sd_u01(w.w))))};
  *reinterpret_cast<f32x4*>(noise + 4 * i) = g;
}

// ------------------------------------------------------------------------------------------- host side
struct IWork {
  float *a[2], *pa[2], *ad, *x0p, *px0, *x1p, *px1, *x2, *hp, *ph, *i[2], *pi[2];
  __bf16 *wh6, *wg6;  // pre-split _dyn_hid / _dyn_gru weights (BPre6 images, 3 bf16 per element)
  float *waT, *w1T;   // actor layer 0's stoch columns and _dyn_in1, transposed (SK, U) for k_onehot_lin
  __bf16 *h6, *x16, *x26;  // pre-split activation images (KH_APRE): deter, silu(rms(x1p)), x2; rows padded to 64
  __bf16* x06;             // and silu(rms(x0p)) for k_hid_areg (KH_AREG)
  __bf16 *wi6, *w06, *wad6;  // pre-split img_net_0 / _dyn_in0 / actor layer 0 (deter columns) weights (KL_PRE)
  long total;
};
long al64(long n) { return (n + 63) / 64 * 64; }
IWork iwork(const sd_imagine& d, float* base) {
  IWork w;
  long o = 0;
  auto take = [&](long n) { float* p = base ? base + o : nullptr; o += al64(n); return p; };
  const long NU = (long)d.N * d.U, NP = (long)d.N * (d.U / 16);  // up to 16-column row partials
  for (int k = 0; k < 2; ++k) { w.a[k] = take(NU); w.pa[k] = take(NP); }
  w.ad = take(NU);
  w.x0p = take(NU); w.px0 = take(NP);
  w.x1p = take(NU); w.px1 = take(NP);
  w.x2 = take(NU);
  w.hp = take((long)d.N * d.D);
  w.ph = take((long)d.N * (d.D / 32));
  for (int k = 0; k < 2; ++k) { w.i[k] = take(NU); w.pi[k] = take(NP); }
  const long Ig = d.D / d.G + 3L * d.U;
  w.wh6 = reinterpret_cast<__bf16*>(take((long)d.D * Ig * 3 / 2));
  w.wg6 = reinterpret_cast<__bf16*>(take((long)3 * d.D * (d.D / d.G) * 3 / 2));
  w.waT = take((long)d.SK * d.U);
  w.w1T = take((long)d.SK * d.U);
  const long rows = (d.N + 63L) / 64 * 64;
  w.h6 = reinterpret_cast<__bf16*>(take(rows * d.D * 3 / 2));
  w.x16 = reinterpret_cast<__bf16*>(take(rows * d.U * 3 / 2));
  w.x26 = reinterpret_cast<__bf16*>(take(rows * d.U * 3 / 2));
  w.x06 = reinterpret_cast<__bf16*>(take(rows * d.U * 3 / 2));
  w.wi6 = reinterpret_cast<__bf16*>(take((long)d.U * d.D * 3 / 2));
  w.w06 = reinterpret_cast<__bf16*>(take((long)d.U * d.D * 3 / 2));
  w.wad6 = reinterpret_cast<__bf16*>(take((long)d.U * d.D * 3 / 2));
  w.total = o;
  return w;
}

int icheck(const sd_imagine* d) {
  if (!d || !d->feats || !d->actions || !d->work) return SD_EARG;
  if (d->N < 1 || d->H1 < 1 || d->U != 256 || d->G < 1 || d->D % d->G || d->D > 4096) return SD_ESHAPE;
  const int Dg = d->D / d->G;
  if (Dg % 32 || Dg < 32 || d->SK % 64 || (d->Kd != 16 && d->Kd != 32) || d->SK % d->Kd) return SD_ESHAPE;
  if (d->A < 1 || (d->act_discrete ? d->A > 16 : 2 * d->A > 32)) return SD_ESHAPE;
  if (d->actor_layers < 1 || d->actor_layers > 4 || d->img_layers < 1 || d->img_layers > 4) return SD_ESHAPE;
  if ((d->SK + d->D) % 32) return SD_ESHAPE;
  if (d->t_begin < 0 || d->t_begin >= (d->t_end > 0 ? d->t_end : d->H1) || d->t_end > d->H1) return SD_EARG;
  return SD_OK;
}

}  // namespace

extern "C" int sd_imagine_noise(const sd_imagine* dp, float* noise, float* noise_act, sd_stream stream_) {
  if (!dp) return SD_EARG;
  sd_imagine dc = *dp;  // (feats / actions need not exist yet: the noise reads neither)
  if (!dc.feats) dc.feats = noise;
  if (!dc.actions) dc.actions = noise;
  const int rc = icheck(&dc);
  if (rc) return rc;
  if (!noise || ((uintptr_t)noise & 15)) return SD_EARG;
  long n = (long)(dp->H1 - 1) * dp->N * dp->SK / 4;
  if (noise_act) n = n > (long)dp->H1 * dp->N * dp->A ? n : (long)dp->H1 * dp->N * dp->A;
  if (n <= 0) return SD_OK;
  k_imag_noise<<<(int)((n + 255) / 256), 256, 0, (hipStream_t)stream_>>>(*dp, noise, noise_act);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_imagine_work_floats(const sd_imagine* d) {
  if (!d) return SD_EARG;
  return (int)iwork(*d, nullptr).total;
}

// k_hid reads deter / x1 / x2 from pre-split images when every producer writes one (k_gate, k_onehot_lin,
// k_action_rows); SDHIP_KH_NOAPRE set: the in-loader split, for tests comparing the two — bit-identical
static bool img_apre(const sd_imagine& d) {
  return KH_APRE && KH_1S && F6_HID && KH_PRE && KH_BM == 64 && KL_ONEHOT && d.SK / d.Kd <= 64 && KA_ROWS &&
         !SD_FUSED_ACTOR && d.U / KL2_PW == 16 && !getenv("SDHIP_KH_NOAPRE");
}
// k_hid on register A operands (k_hid_areg) at the block widths it is built for (Dg = 256 / 512); SDHIP_KH_NOAREG set:
// k_hid<true>, for A/B and the bit-identity test
#ifndef KH_AREG
#define KH_AREG 1
#endif
static int img_areg_nkt(const sd_imagine& d) {
  const int nkt = (d.D / d.G + 3 * d.U) / BK6;
  return (KH_AREG && img_apre(d) && (nkt == 32 || nkt == 40) && !getenv("SDHIP_KH_NOAREG")) ? nkt : 0;
}
static void launch_hid_areg(const sd_imagine& d, const IWork& w, int nkt, const float* feat_t, int F, Tr tr,
                            hipStream_t st) {
  (void)feat_t; (void)F;
  const dim3 grid(d.D / 64, sd_cdiv(d.N, 64));
  if (nkt == 32)
    k_hid_areg<32><<<grid, 256, 0, st>>>(d, w.hp, w.ph, w.wh6, w.h6, w.x06, w.x16, w.x26, tr);
  else
    k_hid_areg<40><<<grid, 256, 0, st>>>(d, w.hp, w.ph, w.wh6, w.h6, w.x06, w.x16, w.x26, tr);
}
// the deter contractions on pre-split operands (k_lin6): A the deter image (img_apre), B the weights split once per
// imagination; SDHIP_KL_NOPRE set: the fp32 k_lin, for A/B and tests
static bool img_lpre(const sd_imagine& d) {
  return KL_PRE && img_apre(d) && d.U % KL3_BN == 0 && d.D % BK6 == 0 && !getenv("SDHIP_KL_NOPRE");
}
// k_lin6_areg where it is built (D = 2048 / 4096: two halves of 32 / 64 k tiles, U = 256); SDHIP_KL_NOAREG set:
// k_lin6 (A/B, and the agreement test). Decides the weight images' column-tile width too (16 here, KL3_BN for k_lin6).
static bool img_lareg(const sd_imagine& d) {
  return KL_AREG && img_lpre(d) && (d.D == 64 * BK6 || d.D == 128 * BK6) && d.U == 256 && !getenv("SDHIP_KL_NOAREG");
}
// one k_lin6 / k_lin6_areg launch over nprob (2 or 3) problems sharing A = the deter image
static void launch_lin6(const sd_imagine& d, const IWork& w, const __bf16* wa, const __bf16* wb, const __bf16* wc,
                        const LinProb& pa, const LinProb& pb, const LinProb& pc, int nprob, Tr tr, hipStream_t st) {
  if (img_lareg(d)) {
    const bool n3 = nprob == 3 && KL_NSUB == 3 && !getenv("SDHIP_KL_NSUB4");  // (SDHIP_KL_NSUB4: 64-column tiles)
    const dim3 grid(n3 ? 3 * d.U / 48 : nprob * d.U / 64, sd_cdiv(d.N, 64));
#define SD_LIN6A(NKH_)                                                                                          \
  do {                                                                                                          \
    if (n3)                                                                                                     \
      k_lin6_areg<NKH_, 3, KL_KQ><<<grid, 256 * KL_KQ, 0, st>>>(w.h6, d.D, wa, wb, wc, pa, pb, pc, d.U, d.N, tr); \
    else                                                                                                        \
      k_lin6_areg<NKH_, 4, KL_KQ><<<grid, 256 * KL_KQ, 0, st>>>(w.h6, d.D, wa, wb, wc, pa, pb, pc, d.U, d.N, tr); \
  } while (0)
    if (d.D == 64 * BK6)
      SD_LIN6A(64 / KL_KQ);
    else
      SD_LIN6A(128 / KL_KQ);
#undef SD_LIN6A
  } else {
    k_lin6<KL6_BM, KL3_BN><<<dim3(d.U / KL3_BN, sd_cdiv(d.N, KL6_BM), nprob), 256, 0, st>>>(w.h6, d.D, wa, wb, wc, pa, pb,
                                                                                          pc, d.N, tr);
  }
}

// One launch of step t's k_lin / k_lin6 (img_net_0 + _dyn_in0 + actor layer 0's deter part: which = 0), k_hid (1) or
// k_gate (2), exactly as sd_imagine_run issues it (same descriptor and workspace; the launch recomputes the values that
// run already wrote, so it can be repeated): bench.py times the dominant kernel of the update this way.
extern "C" int sd_imagine_step_kernel(const sd_imagine* dp, int which, int t, sd_stream stream_) {
  int rc = icheck(dp);
  if (rc) return rc;
  const sd_imagine& d = *dp;
  if (t < 0 || t >= d.H1 - 1 || which < 0 || which > 2) return SD_EARG;
  hipStream_t st = (hipStream_t)stream_;
  const IWork w = iwork(d, d.work);
  const int N = d.N, U = d.U, SK = d.SK, D = d.D, F = SK + D;
  const long NF = (long)N * F;
  const int npU = U / KL2_PW;
  auto feats = [&](int s) { return d.feats + s * NF; };
  if (which == 0) {
    LinProb pi{feats(t + 1) + SK, F, D, d.Wi[0], D, d.bi[0], w.i[0], U, w.pi[0], nullptr};
    LinProb px{feats(t + 1) + SK, F, D, d.W0, D, d.b0, w.x0p, U, w.px0, nullptr};
    LinProb pd{feats(t + 1) + SK, F, D, d.Wa[0] + SK, F, nullptr, w.ad, U, nullptr, nullptr};
    if (img_lpre(d))  // the images the run built (the deter image holds its last step: the timing is the same)
      launch_lin6(d, w, w.wi6, w.w06, w.wad6, pi, px, pd, 3, Tr{}, st);
    else
      k_lin<KL3_BM, KL3_BN><<<dim3(U / KL3_BN, sd_cdiv(N, KL3_BM), 3), 256, 0, st>>>(pi, px, pd, N, Tr{});
  } else if (which == 1 && img_areg_nkt(d)) {  // (the images the run built)
    launch_hid_areg(d, w, img_areg_nkt(d), feats(t) + SK, F, Tr{}, st);
  } else if (which == 1) {
    k_hid<false><<<dim3(D / 64, sd_cdiv(N, KH_BM)), 256, 0, st>>>(d, feats(t) + SK, F, w.x0p, w.x1p, w.px0, w.px1,
                                                                 U / KL3_PW, npU, w.x2, w.hp, w.ph, w.wh6, nullptr,
                                                                 nullptr, nullptr, Tr{});
  } else {
    // k_gate reads hold = feats(t) deter and writes feats(t + 1) deter: the same values again
    k_gate<<<dim3(D / 32, sd_cdiv(N, 64)), 256, 0, st>>>(d, w.hp, w.ph, D / KH_PW, feats(t) + SK, feats(t + 1) + SK, F, w.wg6,
                                                         nullptr, Tr{});
  }
  SD_LAUNCH_CHECK();
  return SD_OK;
}

// the weight-only setup of an imagination: pre-split images and transposed one-hot weights (sd_imagine_prep)
static int imagine_prep(const sd_imagine& d, const IWork& w, hipStream_t st) {
  const int U = d.U, SK = d.SK, D = d.D, F = SK + D;
  const float* Wa0d = d.Wa[0] + SK;
  if (KH_PRE && F6_HID) {  // _dyn_hid's weight split into its bf16 planes once per imagination
    const long Ig = D / d.G + 3L * U;
    k_presplit6<64><<<(int)sd_cdiv((long)D * Ig / 4, 256), 256, 0, st>>>(d.Wh, D, (int)Ig, w.wh6);
    SD_LAUNCH_CHECK();
  }
  if (KL_ONEHOT) {  // the one-hot contractions' weights, transposed
    k_transpose_w<<<sd_cdiv((long)SK * U, 256), 256, 0, st>>>(d.Wa[0], F, U, SK, w.waT);
    k_transpose_w<<<sd_cdiv((long)SK * U, 256), 256, 0, st>>>(d.W1, SK, U, SK, w.w1T);
    SD_LAUNCH_CHECK();
  }
  if (KG_PRE && KG_1S && F6_GATE) {  // and _dyn_gru's
    k_presplit6_gate<<<(int)sd_cdiv((long)3 * D * (D / d.G) / 4, 256), 256, 0, st>>>(d.Wg, D, D / d.G, w.wg6);
    SD_LAUNCH_CHECK();
  }
  const bool lpre = img_lpre(d);  // the deter contractions' weights (img_net_0, _dyn_in0, actor layer 0's deter part)
  if (lpre) {
    const int gsz = (int)sd_cdiv((long)U * D / 4, 256);
    if (img_lareg(d)) {  // 16-column tiles for k_lin6_areg
      k_presplit6<16><<<gsz, 256, 0, st>>>(d.Wi[0], U, D, w.wi6, D);
      k_presplit6<16><<<gsz, 256, 0, st>>>(d.W0, U, D, w.w06, D);
      k_presplit6<16><<<gsz, 256, 0, st>>>(Wa0d, U, D, w.wad6, F);
    } else {
      k_presplit6<KL3_BN><<<gsz, 256, 0, st>>>(d.Wi[0], U, D, w.wi6, D);
      k_presplit6<KL3_BN><<<gsz, 256, 0, st>>>(d.W0, U, D, w.w06, D);
      k_presplit6<KL3_BN><<<gsz, 256, 0, st>>>(Wa0d, U, D, w.wad6, F);
    }
    SD_LAUNCH_CHECK();
  }
  return SD_OK;
}

extern "C" int sd_imagine_prep(const sd_imagine* dp, sd_stream stream_) {
  if (!dp) return SD_EARG;
  sd_imagine d = *dp;  // (feats / actions need not exist yet: the weight images read neither)
  if (!d.feats) d.feats = d.work;
  if (!d.actions) d.actions = d.work;
  const int rc = icheck(&d);
  if (rc) return rc;
  return imagine_prep(d, iwork(d, d.work), (hipStream_t)stream_);
}

extern "C" int sd_imagine_run(const sd_imagine* dp, sd_stream stream_) {
  int rc = icheck(dp);
  if (rc) return rc;
  const sd_imagine& d = *dp;
  hipStream_t st = (hipStream_t)stream_;
  const IWork w = iwork(d, d.work);
  const int N = d.N, U = d.U, SK = d.SK, D = d.D, F = SK + D;
  const long NF = (long)N * F;
  const int npU = U / KL2_PW;  // row partials per hidden row written by the K = S*Kd k_lin
  const dim3 gr(U / 64, sd_cdiv(N, KR_BM));
  const int npR = U / KR_PW;  // row partials written by k_rmslin
  auto feats = [&](int t) { return d.feats + t * NF; };
  // actor layer 0 on feat = [stoch, deter] is K-split: the deter part (no bias) runs in the launch that already
  // reads deter' (img_net_0 / _dyn_in0), the stoch part (+ bias + deter part, row partials) after the prior sample
  const float* Wa0d = d.Wa[0] + SK;  // (U, F) columns SK.. of the actor's first weight
  const int t_end = d.t_end > 0 ? d.t_end : d.H1;
  const bool apre = img_apre(d);  // pre-split k_hid operands
  const int areg = img_areg_nkt(d);  // k_hid_areg (and the x0 image k_action_rows writes for it)
  const X0Img x0i{w.x0p, w.px0, U / KL3_PW, areg ? w.x06 : nullptr};
  if (d.t_begin == 0 && apre) {  // the start state's deter image
    k_presplit_rows<<<(int)sd_cdiv((long)N * D / 4, 256), 256, 0, st>>>(feats(0) + SK, F, N, D, w.h6);
    SD_LAUNCH_CHECK();
  }
  if (d.t_begin == 0 && !d.prepped) {
    const int e = imagine_prep(d, w, st);
    if (e) return e;
  }
  const bool lpre = img_lpre(d);
  if (d.t_begin == 0) {  // x0p(0) = h0 . W0^T + b0 and the deter part of actor layer 0 at t = 0
    LinProb p{feats(0) + SK, F, D, d.W0, D, d.b0, w.x0p, U, w.px0, nullptr};
    LinProb pd{feats(0) + SK, F, D, Wa0d, F, nullptr, w.ad, U, nullptr, nullptr};
    // the 3-problem launch's tile, so x0p's row partials have one width for every step
    if (lpre)
      launch_lin6(d, w, w.w06, w.wad6, w.wad6, p, pd, pd, 2, Tr{}, st);
    else
      k_lin<KL3_BM, KL3_BN><<<dim3(U / KL3_BN, sd_cdiv(N, KL3_BM), 2), 256, 0, st>>>(p, pd, pd, N, Tr{});
    SD_LAUNCH_CHECK();
  }
  for (int t = d.t_begin; t < t_end; ++t) {
    const bool last = t == d.H1 - 1;
    auto tr = [&](int k) { return Tr{d.trace, t * 16 + k}; };  // launch k of step t (measurement builds)
    // actor layer 0's output: the caller's per-step buffer when given (read again by the policy loss), else scratch
    float* a0 = d.actor_h0 ? d.actor_h0 + (long)t * N * U : w.a[0];
    {  // actor layer 0, stoch part (+ deter part); _dyn_in1 on stoch
      LinProb pa{feats(t), F, SK, d.Wa[0], F, d.ba[0], a0, U, w.pa[0], w.ad};
      LinProb px{feats(t), F, SK, d.W1, SK, d.b1, w.x1p, U, w.px1, nullptr};
      if (KL_ONEHOT && d.SK / d.Kd <= 64) {
        const OneHotProb oa{w.waT, d.ba[0], w.ad, a0, w.pa[0], nullptr, nullptr, 0.f},
            ox{w.w1T, d.b1, nullptr, w.x1p, w.px1, apre ? d.n1 : nullptr, apre ? w.x16 : nullptr, d.eps};
        k_onehot_lin<<<dim3(sd_cdiv(N, 4), OH_SPLIT ? (last ? 1 : 2) : 1), 256, 0, st>>>(feats(t), F, SK, d.Kd, oa, ox,
                                                                                      last ? 1 : 2, N, tr(0));
      } else {
        k_lin<32, KL2_BN><<<dim3(U / KL2_BN, sd_cdiv(N, 32), last ? 1 : 2), 256, 0, st>>>(pa, px, px, N, tr(0));
      }
      SD_LAUNCH_CHECK();
    }
    if (SD_FUSED_ACTOR) {  // hidden layers 1.. + output layer + action sample + x2 in one launch
      k_actor<<<sd_cdiv(N, 16), 256, 0, st>>>(d, a0, w.pa[0], npU, d.actions + (long)t * N * d.A, w.x2, t,
                                              last ? 0 : 1);
    } else {
      int cur = 0, npa = npU;
      for (int l = 1; l < d.actor_layers; ++l) {
        if (KR_RW && U == 256 && npa <= 16)
          k_rmslin_rw<<<dim3(U / 64, sd_cdiv(N, 16)), 512, 0, st>>>(l == 1 ? a0 : w.a[cur], d.na[l - 1], w.pa[cur],
                                                                     npa, d.Wa[l], d.ba[l], w.a[cur ^ 1],
                                                                     w.pa[cur ^ 1], N, d.eps, tr(l));
        else
          k_rmslin<KR_BM, 64><<<gr, 256, 0, st>>>(l == 1 ? a0 : w.a[cur], d.na[l - 1], w.pa[cur], npa, U, d.Wa[l],
                                                  d.ba[l], w.a[cur ^ 1], w.pa[cur ^ 1], N, d.eps, tr(l));
        SD_LAUNCH_CHECK();
        cur ^= 1;
        npa = npR;
      }
      if (KA_ROWS) {
        const float* xa = d.actor_layers == 1 ? a0 : w.a[cur];
        float* acts = d.actions + (long)t * N * d.A;
        if ((d.act_discrete ? d.A : 2 * d.A) <= 16)
          k_action_rows<16><<<sd_cdiv(N, 4), 256, 0, st>>>(d, xa, d.na[d.actor_layers - 1], w.pa[cur], npa, acts,
                                                           w.x2, t, last ? 0 : 1, apre ? w.x26 : nullptr, x0i, tr(4));
        else
          k_action_rows<32><<<sd_cdiv(N, 4), 256, 0, st>>>(d, xa, d.na[d.actor_layers - 1], w.pa[cur], npa, acts,
                                                           w.x2, t, last ? 0 : 1, apre ? w.x26 : nullptr, x0i, tr(4));
      }
      else
        k_action<<<dim3(1, sd_cdiv(N, KA_BM)), 256, 0, st>>>(d, d.actor_layers == 1 ? a0 : w.a[cur],
                                                  d.na[d.actor_layers - 1], w.pa[cur], npa,
                                                  d.actions + (long)t * N * d.A, w.x2, t, last ? 0 : 1, tr(4));
    }
    SD_LAUNCH_CHECK();
    if (last) break;
    if (areg)
      launch_hid_areg(d, w, areg, feats(t) + SK, F, tr(5), st);
    else if (apre)
      k_hid<true><<<dim3(D / 64, sd_cdiv(N, KH_BM)), 256, 0, st>>>(d, feats(t) + SK, F, w.x0p, w.x1p, w.px0, w.px1,
                                                                  U / KL3_PW, npU, w.x2, w.hp, w.ph, w.wh6, w.h6,
                                                                  w.x16, w.x26, tr(5));
    else
      k_hid<false><<<dim3(D / 64, sd_cdiv(N, KH_BM)), 256, 0, st>>>(d, feats(t) + SK, F, w.x0p, w.x1p, w.px0, w.px1,
                                                                   U / KL3_PW, npU, w.x2, w.hp, w.ph, w.wh6, nullptr,
                                                                   nullptr, nullptr, tr(5));
    SD_LAUNCH_CHECK();
    k_gate<<<dim3(D / 32, sd_cdiv(N, 64)), 256, 0, st>>>(d, w.hp, w.ph, D / KH_PW, feats(t) + SK, feats(t + 1) + SK, F, w.wg6,
                                                         apre ? w.h6 : nullptr, tr(6));
    SD_LAUNCH_CHECK();
    {  // img_net_0, the next step's _dyn_in0 and the deter part of its actor layer 0 share A = deter'
      LinProb pi{feats(t + 1) + SK, F, D, d.Wi[0], D, d.bi[0], w.i[0], U, w.pi[0], nullptr};
      LinProb px{feats(t + 1) + SK, F, D, d.W0, D, d.b0, w.x0p, U, w.px0, nullptr};
      LinProb pd{feats(t + 1) + SK, F, D, Wa0d, F, nullptr, w.ad, U, nullptr, nullptr};
      if (lpre)
        launch_lin6(d, w, w.wi6, w.w06, w.wad6, pi, px, pd, 3, tr(7), st);
      else
        k_lin<KL3_BM, KL3_BN><<<dim3(U / KL3_BN, sd_cdiv(N, KL3_BM), 3), 256, 0, st>>>(pi, px, pd, N, tr(7));
      SD_LAUNCH_CHECK();
    }
    const int pj = SD_PRIOR_NCT > 0 && SK % (64 * SD_PRIOR_NCT) == 0 ? SK / (64 * SD_PRIOR_NCT) : 0;
    if (SD_FUSED_PRIOR && (pj == 1 || pj == 2 || pj == 4)) {  // img_net hidden layers + prior + sample, one launch
      const dim3 gp(SD_PRIOR_NCT, sd_cdiv(N, 16));
      const int npi = U / KL3_PW;
#define SD_PRIOR_LAUNCH(KD_, NJ_) \
  k_imgprior<KD_, NJ_><<<gp, 256, 0, st>>>(d, w.i[0], w.pi[0], npi, feats(t + 1), F, t)
      if (d.Kd == 16) {
        if (pj == 1) SD_PRIOR_LAUNCH(16, 1); else if (pj == 2) SD_PRIOR_LAUNCH(16, 2); else SD_PRIOR_LAUNCH(16, 4);
      } else {
        if (pj == 1) SD_PRIOR_LAUNCH(32, 1); else if (pj == 2) SD_PRIOR_LAUNCH(32, 2); else SD_PRIOR_LAUNCH(32, 4);
      }
#undef SD_PRIOR_LAUNCH
    } else {
      int ci = 0, npi = U / KL3_PW;
      for (int l = 1; l < d.img_layers; ++l) {
        if (KR_RW && U == 256 && npi <= 16)
          k_rmslin_rw<<<dim3(U / 64, sd_cdiv(N, 16)), 512, 0, st>>>(w.i[ci], d.ni[l - 1], w.pi[ci], npi, d.Wi[l],
                                                                     d.bi[l], w.i[ci ^ 1], w.pi[ci ^ 1], N, d.eps,
                                                                     tr(7 + l));
        else
          k_rmslin<KR_BM, 64><<<gr, 256, 0, st>>>(w.i[ci], d.ni[l - 1], w.pi[ci], npi, U, d.Wi[l], d.bi[l],
                                                  w.i[ci ^ 1], w.pi[ci ^ 1], N, d.eps, tr(7 + l));
        SD_LAUNCH_CHECK();
        ci ^= 1;
        npi = npR;
      }
      const dim3 gpr(SK / 64, sd_cdiv(N, 16));
      if (KP_RW && U == 256 && npi <= 16) {
        if (d.Kd == 16)
          k_prior_rw<16, KP_NT><<<gpr, KP_NT, 0, st>>>(d, w.i[ci], d.ni[d.img_layers - 1], w.pi[ci], npi, feats(t + 1), F, t,
                                               tr(12));
        else
          k_prior_rw<32, KP_NT><<<gpr, KP_NT, 0, st>>>(d, w.i[ci], d.ni[d.img_layers - 1], w.pi[ci], npi, feats(t + 1), F, t,
                                               tr(12));
      } else if (d.Kd == 16) {
        k_prior<16><<<gpr, 256, 0, st>>>(d, w.i[ci], d.ni[d.img_layers - 1], w.pi[ci], npi, feats(t + 1), F, t,
                                          tr(12));
      } else {
        k_prior<32><<<gpr, 256, 0, st>>>(d, w.i[ci], d.ni[d.img_layers - 1], w.pi[ci], npi, feats(t + 1), F, t,
                                          tr(12));
      }
    }
    SD_LAUNCH_CHECK();
  }
  return SD_OK;
}
