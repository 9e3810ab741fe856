// Shared fp32-MFMA GEMM block core (see gemm.hip for the design notes). Operand "loaders" supply BK-deep
// register tiles, so dense matrices (gemm.hip) and implicit-im2col convolution operands (conv.hip) share one
// MFMA/LDS pipeline and one epilogue.
#pragma once
#include "common.h"

namespace sdg {
namespace {  // internal linkage: the core is instantiated per translation unit

constexpr int BK = 32;
constexpr int LDS_ROW = BK + 4;  // floats (144-B rows: 9 is odd -> conflict-free b128 reads)

struct GemmArgs {
  const float* A;
  const float* B;
  float* C;
  const float* bias;
  float* ws;
  long lda, ldb, ldc;
  long sA, sB, sC, sBias;
  int M, N, K, batch, ksplit, kchunk;
  float alpha, beta;
  // split-bf16 weight-gradient GEMMs (sd_gemm_bf16x3_wgrad): rowsum[m] (+)= alpha * sum_k A[m, k] (the bias gradient
  // of C = dy^T x); with split-K each split writes its partial to rs_ws[split * M + m], summed by gemm_reduce_kernel
  float* rowsum;
  float* rs_ws;
  int rs_acc;
  // rows m >= rs_split sum into rowsum2[m - rs_split] (two heads' bias gradients from one weight-gradient GEMM over
  // their concatenated dy, sd_gemm_bf16x3_wgrad2); rs_split >= M: rowsum only
  int rs_split;
  float* rowsum2;
};

SD_DEV float* rowsum_at(const GemmArgs& g, int m) {
  return (!g.rowsum2 || m < g.rs_split) ? g.rowsum + m : g.rowsum2 + (m - g.rs_split);
}

// Load a ROWS x BK tile of an operand into registers (rows = m for A / n for B).
// KC: k contiguous (row-major in k, `ld` between rows) ; else rows contiguous (`ld` between k's).
template <int ROWS, bool KC, bool VEC>
struct TileLoader {
  static constexpr int NV = (ROWS * BK / 4 + 255) / 256;  // float4 per thread
  f32x4 r[NV];

  SD_DEV void load(const float* __restrict__ p, long ld, int row0, int nrows, int k0, int kend) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = tid + v * 256;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      if (i < ROWS * BK / 4) {
        if (KC) {
          const int row = i / (BK / 4), kq = i % (BK / 4);
          const int gr = row0 + row, gk = k0 + 4 * kq;
          if (gr < nrows) {
            const float* q = p + (long)gr * ld + gk;
            if (VEC && gk + 3 < kend) {
              x = *reinterpret_cast<const f32x4*>(q);
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j)
                if (gk + j < kend) x[j] = q[j];
            }
          }
        } else {
          const int k = i % BK, rq = i / BK;
          const int gk = k0 + k, gr = row0 + 4 * rq;
          if (gk < kend) {
            const float* q = p + (long)gk * ld + gr;
            if (VEC && gr + 3 < nrows) {
              x = *reinterpret_cast<const f32x4*>(q);
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j)
                if (gr + j < nrows) x[j] = q[j];
            }
          }
        }
      }
      r[v] = x;
    }
  }

  SD_DEV void store(float* lds) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = tid + v * 256;
      // (v + 1) * 256 <= ROWS * BK / 4: every thread's slot is inside the tile (static; hipcc cannot see tid < 256)
      if ((v + 1) * 256 <= ROWS * BK / 4 || i < ROWS * BK / 4) {
        if (KC) {
          const int row = i / (BK / 4), kq = i % (BK / 4);
          *reinterpret_cast<f32x4*>(lds + row * LDS_ROW + 4 * kq) = r[v];
        } else {
          const int k = i % BK, rq = i / BK;
#pragma unroll
          for (int j = 0; j < 4; ++j) lds[(4 * rq + j) * LDS_ROW + k] = r[v][j];
        }
      }
    }
  }
};

// Dense operand: ROWS x BK tiles of a strided matrix (rows = m for A / n for B).
template <int ROWS, bool KC, bool VEC>
struct DenseOperand {
  TileLoader<ROWS, KC, VEC> t;
  const float* p;
  long ld;
  int nrows, row0;
  SD_DEV DenseOperand(const float* base, long ld_, int nrows_, int row0_) : p(base), ld(ld_), nrows(nrows_), row0(row0_) {}
  SD_DEV void load(int k0, int kend) { t.load(p, ld, row0, nrows, k0, kend); }
  SD_DEV void store(float* lds) const { t.store(lds); }
};

template <int BM, int BN, int WM, int WN, class OpA, class OpB>
SD_DEV void gemm_block(const GemmArgs& g, OpA& la, OpB& lb, int bm0, int bn0, int b, int split, int kbeg, int kend) {
  constexpr int WAVES_N = BN / WN;
  constexpr int TM = WM / 32, TN = WN / 32;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves");
  __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * LDS_ROW];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / WAVES_N, wc = wave % WAVES_N;
  constexpr int STAGE = (BM + BN) * LDS_ROW;  // floats per pipeline stage: [A rows | B rows]

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int nk = (kend - kbeg + BK - 1) / BK;
  if (nk > 0) {
    la.load(kbeg, kend);
    lb.load(kbeg, kend);
    la.store(smem);
    lb.store(smem + BM * LDS_ROW);
    __syncthreads();
  }
  const int h = lane >> 5, l32 = lane & 31;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      la.load(kbeg + (kt + 1) * BK, kend);
      lb.load(kbeg + (kt + 1) * BK, kend);
    }
    constexpr int KH = BK / 2;  // k values per lane half per tile
    float af[TM][KH], bf[TN][KH];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const float* q = smem + cur * STAGE + (wr * WM + 32 * i + l32) * LDS_ROW + KH * h;
#pragma unroll
      for (int v = 0; v < KH / 4; ++v) {
        f32x4 x = *reinterpret_cast<const f32x4*>(q + 4 * v);
#pragma unroll
        for (int s = 0; s < 4; ++s) af[i][4 * v + s] = x[s];
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const float* q = smem + cur * STAGE + BM * LDS_ROW + (wc * WN + 32 * j + l32) * LDS_ROW + KH * h;
#pragma unroll
      for (int v = 0; v < KH / 4; ++v) {
        f32x4 x = *reinterpret_cast<const f32x4*>(q + 4 * v);
#pragma unroll
        for (int s = 0; s < 4; ++s) bf[j][4 * v + s] = x[s];
      }
    }
#pragma unroll
    for (int s = 0; s < KH; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
    if (kt + 1 < nk) {
      la.store(smem + (cur ^ 1) * STAGE);
      lb.store(smem + (cur ^ 1) * STAGE + BM * LDS_ROW);
    }
    __syncthreads();
  }

  // epilogue: reg r of a 32x32 tile -> row (r&3) + 8*(r>>2) + 4*h, col l32
  if (g.ksplit > 1) {
    float* W = g.ws + ((long)split * g.batch + b) * (long)g.M * g.N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = bn0 + wc * WN + 32 * j + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = bm0 + wr * WM + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
          if (m < g.M && n < g.N) W[(long)m * g.N + n] = g.alpha * acc[i][j][r];
        }
      }
    return;
  }
  float* C = g.C + (long)b * g.sC;
  const float* bias = g.bias ? g.bias + (long)b * g.sBias : nullptr;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = bn0 + wc * WN + 32 * j + l32;
      const float bv = (bias && n < g.N) ? bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = bm0 + wr * WM + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < g.M && n < g.N) {
          float v = g.alpha * acc[i][j][r] + bv;
          float* c = C + (long)m * g.ldc + n;
          if (g.beta != 0.f) v += g.beta * *c;
          *c = v;
        }
      }
    }
}

// k-major LDS image of a ROWS x BK operand tile whose global rows are contiguous along ROWS (A(m,k) at
// p[k*ld + m]): thread i loads the float4 (k = i / (ROWS/4), rows 4*(i % (ROWS/4)) ..+3) — consecutive lanes read
// consecutive 16 B of one k-row (coalesced) — and stores it as two 8-B writes into LDS[k][ROWS + 2]; the +2 pad
// makes the per-lane scalar fragment reads of gemm_block16 (lanes l16 along rows, 4 lane groups 8 k apart) hit
// 64 distinct banks.
template <int ROWS>
struct KMajor {
  static constexpr bool KMAJOR = true;
  static constexpr int LD = ROWS + 2;
  static constexpr int NQ = ROWS / 4;                       // float4 per k-row
  static constexpr int NV = (ROWS * BK / 4 + 255) / 256;    // float4 per thread
  f32x4 r[NV];
  SD_DEV static int kk(int i) { return i / NQ; }
  SD_DEV static int rq(int i) { return i % NQ; }
  SD_DEV void store(float* lds) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + v * 256;
      if (i < ROWS * BK / 4) {
        float* d = lds + kk(i) * LD + 4 * rq(i);
        *reinterpret_cast<float2*>(d) = float2{r[v][0], r[v][1]};
        *reinterpret_cast<float2*>(d + 2) = float2{r[v][2], r[v][3]};
      }
    }
  }
};

// dense k-major operand (rows m or n contiguous, `ld` between k's)
template <int ROWS, bool VEC>
struct DenseKM : KMajor<ROWS> {
  using KMajor<ROWS>::r;
  using KMajor<ROWS>::NV;
  const float* p;
  long ld;
  int nrows, row0;
  SD_DEV DenseKM(const float* base, long ld_, int nrows_, int row0_) : p(base), ld(ld_), nrows(nrows_), row0(row0_) {}
  SD_DEV void load(int k0, int kend) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + v * 256;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      const int gk = k0 + this->kk(i), gr = row0 + 4 * this->rq(i);
      if (i < ROWS * BK / 4 && gk < kend) {
        const float* q = p + (long)gk * ld + gr;
        if (VEC && gr + 3 < nrows) {
          x = *reinterpret_cast<const f32x4*>(q);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (gr + j < nrows) x[j] = q[j];
        }
      }
      r[v] = x;
    }
  }
};

// Same pipeline on v_mfma_f32_16x16x4_f32 (wave tiles in multiples of 16: e.g. N = 48 output channels exactly).
// Row-major LDS operands: lane (l16, q = lane>>4) reads k = 8q .. 8q+7 of its fragment row (two ds_read_b128);
// k-major operands (OpX::KMAJOR): the same k's as 8 scalar reads. MFMA step s consumes k = 8q + s in lane group q
// — a fixed k permutation shared by A and B.
template <class Op, class = void>
struct is_kmajor { static constexpr bool value = false; };
template <class Op>
struct is_kmajor<Op, decltype(void(Op::KMAJOR))> { static constexpr bool value = Op::KMAJOR; };

// PF = K-tiles in flight in registers (loader copies la[PF] / lb[PF]); the LDS image is double-buffered. With PF > 1
// a tile's global loads are issued PF iterations before its LDS store, hiding L2 latency behind PF tiles of MFMA work
// when a launch has too few waves per SIMD to hide it by occupancy. The k loop is unrolled by PF so every register
// set is statically indexed.
// Static LDS block of N floats, one per (kernel, N): lets an epilogue reuse a main loop's staging area.
template <int N>
SD_DEV float* sd_smem() {
  __shared__ __attribute__((aligned(16))) float s[N];
  return s;
}
// floats of gemm16_mainloop_pf's double-buffered staging area
template <int BM, int BN, bool AKM = false, bool BKM = false>
constexpr int gemm16_smem_floats() {
  return 2 * ((AKM ? BK * (BM + 2) : BM * LDS_ROW) + (BKM ? BK * (BN + 2) : BN * LDS_ROW));
}

// ES (early store): stage tile kt+1 and issue the loads of tile kt+1+PF BEFORE this tile's MFMAs (after its fragment
// reads), so the loads' address arithmetic fills the MFMA issue gaps; otherwise after them.
template <int BM, int BN, int WM, int WN, int PF = 1, bool ES = false, class OpA, class OpB>
SD_DEV void gemm16_mainloop_pf(OpA (&la)[PF], OpB (&lb)[PF], int kbeg, int kend, f32x4 (&acc)[WM / 16][WN / 16],
                               bool accumulate = false) {
  constexpr int WAVES_N = BN / WN;
  constexpr int TM = WM / 16, TN = WN / 16;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves");
  constexpr bool AKM = is_kmajor<OpA>::value, BKM = is_kmajor<OpB>::value;
  constexpr int LDA = AKM ? BM + 2 : LDS_ROW, LDB = BKM ? BN + 2 : LDS_ROW;
  constexpr int SA = AKM ? BK * LDA : BM * LDS_ROW, SB = BKM ? BK * LDB : BN * LDS_ROW;
  constexpr int STAGE = SA + SB;
  static_assert(2 * STAGE == gemm16_smem_floats<BM, BN, AKM, BKM>(), "staging size");
  float* smem = sd_smem<2 * STAGE>();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / WAVES_N, wc = wave % WAVES_N;
  const int l16 = lane & 15, q = lane >> 4;

  // fewer than 4 independent accumulator chains per wave: alternate two banks over the MFMA k steps so
  // dependent MFMAs do not serialise on the MFMA latency (one wave per SIMD in small-grid launches)
  constexpr int XC = TM * TN < 4 ? 2 : 1;
  f32x4 acc2[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (!accumulate) acc[i][j] = acc2[i][j];
    }

  const int nk = (kend - kbeg + BK - 1) / BK;
  if (nk <= 0) return;
  // tile t's k0; indices past the end are clamped to the last tile (a redundant reload that is never consumed), so
  // the steady-state body issues every load unconditionally: a load under a branch makes hipcc drain vmcnt(0) at
  // the merge, which would serialise the whole prefetch pipeline
  auto ktile = [&](int t) { return kbeg + (t < nk ? t : nk - 1) * BK; };
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    la[u].load(ktile(u), kend);
    lb[u].load(ktile(u), kend);
  }
  la[0].store(smem);
  lb[0].store(smem + SA);
  __syncthreads();
  la[0].load(ktile(PF), kend);
  lb[0].load(ktile(PF), kend);
  auto step = [&](int kt, int u) {
    const int cur = kt & 1;
    float af[TM][8], bf[TN][8];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wr * WM + 16 * i + l16;
      if (AKM) {
        const float* p = smem + cur * STAGE + 8 * q * LDA + row;
#pragma unroll
        for (int s = 0; s < 8; ++s) af[i][s] = p[s * LDA];
      } else {
        const float* p = smem + cur * STAGE + row * LDS_ROW + 8 * q;
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(p), x1 = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
        for (int s = 0; s < 4; ++s) { af[i][s] = x0[s]; af[i][4 + s] = x1[s]; }
      }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = wc * WN + 16 * j + l16;
      if (BKM) {
        const float* p = smem + cur * STAGE + SA + 8 * q * LDB + row;
#pragma unroll
        for (int s = 0; s < 8; ++s) bf[j][s] = p[s * LDB];
      } else {
        const float* p = smem + cur * STAGE + SA + row * LDS_ROW + 8 * q;
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(p), x1 = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
        for (int s = 0; s < 4; ++s) { bf[j][s] = x0[s]; bf[j][4 + s] = x1[s]; }
      }
    }
    // tile kt+1 lives in register set (u+1) % PF: stage it, then refill that set with tile kt+1+PF
    const int nx = (u + 1) % PF;  // static after unrolling
    if constexpr (ES) {
      la[nx].store(smem + (cur ^ 1) * STAGE);
      lb[nx].store(smem + (cur ^ 1) * STAGE + SA);
      la[nx].load(ktile(kt + 1 + PF), kend);
      lb[nx].load(ktile(kt + 1 + PF), kend);
    }
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if (XC == 2 && (s & 1))
            acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][s], bf[j][s], acc2[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
        }
    if constexpr (!ES) {
      // keep the LDS store of the next tile behind this tile's MFMAs: hoisted into them, its vmcnt(0) wait would
      // cut the window in which the global loads land from the whole k tile to a few MFMAs
#ifndef SD_NO_SCHED_BARRIER
      __builtin_amdgcn_sched_barrier(0);
#endif
      la[nx].store(smem + (cur ^ 1) * STAGE);
      lb[nx].store(smem + (cur ^ 1) * STAGE + SA);
      la[nx].load(ktile(kt + 1 + PF), kend);
      lb[nx].load(ktile(kt + 1 + PF), kend);
    }
    __syncthreads();
  };
  int kt = 0;
  for (; kt + PF <= nk; kt += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) step(kt + u, u);
  }
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (kt + u < nk) step(kt + u, u);
  if (XC == 2) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] += acc2[i][j];
  }
}

// Fragment-prefetch variant of gemm16_mainloop_pf (row-major LDS operands): iteration kt issues the LDS fragment
// reads of tile kt+1 BEFORE its own MFMAs, which run on fragments read one iteration earlier, so the LDS latency sits
// under the MFMAs instead of in front of them; the MFMA pipe only idles over the next tile's store and the barrier.
// Two LDS stages suffice: iteration kt stores tile kt+2 into stage kt&1, whose tile-kt fragments every wave read
// before iteration kt-1's barrier. Register tile t lives in set t % PF as in gemm16_mainloop_pf.
template <int BM, int BN, int WM, int WN, int PF = 1, class OpA, class OpB>
SD_DEV void gemm16_mainloop_fp(OpA (&la)[PF], OpB (&lb)[PF], int kbeg, int kend, f32x4 (&acc)[WM / 16][WN / 16],
                               bool accumulate = false) {
  constexpr int WAVES_N = BN / WN;
  constexpr int TM = WM / 16, TN = WN / 16;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves");
  static_assert(!is_kmajor<OpA>::value && !is_kmajor<OpB>::value, "row-major LDS operands");
  constexpr int SA = BM * LDS_ROW, STAGE = SA + BN * LDS_ROW;
  float* smem = sd_smem<2 * STAGE>();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / WAVES_N, wc = wave % WAVES_N;
  const int l16 = lane & 15, q = lane >> 4;
  constexpr int XC = TM * TN < 4 ? 2 : 1;
  f32x4 acc2[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (!accumulate) acc[i][j] = acc2[i][j];
    }
  const int nk = (kend - kbeg + BK - 1) / BK;
  if (nk <= 0) return;
  auto ktile = [&](int t) { return kbeg + (t < nk ? t : nk - 1) * BK; };
  f32x4 fa[TM][2], fb[TN][2], na[TM][2], nb[TN][2];
  auto frags = [&](int stage, f32x4 (&a)[TM][2], f32x4 (&b)[TN][2]) {
    const float* s = smem + stage * STAGE;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const float* p = s + (wr * WM + 16 * i + l16) * LDS_ROW + 8 * q;
      a[i][0] = *reinterpret_cast<const f32x4*>(p);
      a[i][1] = *reinterpret_cast<const f32x4*>(p + 4);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const float* p = s + SA + (wc * WN + 16 * j + l16) * LDS_ROW + 8 * q;
      b[j][0] = *reinterpret_cast<const f32x4*>(p);
      b[j][1] = *reinterpret_cast<const f32x4*>(p + 4);
    }
  };
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    la[u].load(ktile(u), kend);
    lb[u].load(ktile(u), kend);
  }
  la[0].store(smem);
  lb[0].store(smem + SA);
  la[0].load(ktile(PF), kend);
  lb[0].load(ktile(PF), kend);
  __syncthreads();
  frags(0, fa, fb);
  la[1 % PF].store(smem + STAGE);
  lb[1 % PF].store(smem + STAGE + SA);
  la[1 % PF].load(ktile(1 + PF), kend);
  lb[1 % PF].load(ktile(1 + PF), kend);
  __syncthreads();
  auto step = [&](int kt, int u) {
    frags((kt + 1) & 1, na, nb);  // tile kt+1 (a clamped, unused copy past the end)
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const float av = fa[i][s >> 2][s & 3], bv = fb[j][s >> 2][s & 3];
          if (XC == 2 && (s & 1))
            acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc2[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[i][j], 0, 0, 0);
        }
    const int nx = (u + 2) % PF;  // static after unrolling: register set of tile kt+2
    __builtin_amdgcn_sched_barrier(0);
    la[nx].store(smem + (kt & 1) * STAGE);
    lb[nx].store(smem + (kt & 1) * STAGE + SA);
    la[nx].load(ktile(kt + 2 + PF), kend);
    lb[nx].load(ktile(kt + 2 + PF), kend);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TM; ++i) { fa[i][0] = na[i][0]; fa[i][1] = na[i][1]; }
#pragma unroll
    for (int j = 0; j < TN; ++j) { fb[j][0] = nb[j][0]; fb[j][1] = nb[j][1]; }
  };
  int kt = 0;
  for (; kt + PF <= nk; kt += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) step(kt + u, u);
  }
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (kt + u < nk) step(kt + u, u);
  if (XC == 2) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] += acc2[i][j];
  }
}

// Early-store variant for row-major LDS operands (one register set): iteration kt reads its fragments from
// LDS[kt&1], stages tile kt+1 (loaded during iteration kt-1, so its loads had a whole MFMA phase to land) into the
// other buffer, issues the loads of tile kt+2, and only then runs its MFMAs — the loads are in flight under the
// MFMAs and their address arithmetic can fill the MFMA issue gaps. One barrier per k tile. Loaders should be
// branch-free (buffer loads) so the body stays one basic block the scheduler can interleave.
template <int BM, int BN, int WM, int WN, class OpA, class OpB>
SD_DEV void gemm16_mainloop_es(OpA& la, OpB& lb, int kbeg, int kend, f32x4 (&acc)[WM / 16][WN / 16]) {
  constexpr int WAVES_N = BN / WN;
  constexpr int TM = WM / 16, TN = WN / 16;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves");
  static_assert(!is_kmajor<OpA>::value && !is_kmajor<OpB>::value, "row-major LDS operands");
  constexpr int SA = BM * LDS_ROW, STAGE = (BM + BN) * LDS_ROW;
  static_assert(2 * STAGE == gemm16_smem_floats<BM, BN>(), "staging size");
  float* smem = sd_smem<2 * STAGE>();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / WAVES_N, wc = wave % WAVES_N;
  const int l16 = lane & 15, q = lane >> 4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (kend - kbeg + BK - 1) / BK;
  if (nk <= 0) return;
  auto ktile = [&](int t) { return kbeg + (t < nk ? t : nk - 1) * BK; };
  la.load(ktile(0), kend);
  lb.load(ktile(0), kend);
  la.store(smem);
  lb.store(smem + SA);
  la.load(ktile(1), kend);
  lb.load(ktile(1), kend);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const float* cur = smem + (kt & 1) * STAGE;
    float* nxt = smem + ((kt & 1) ^ 1) * STAGE;
    float af[TM][8], bf[TN][8];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const float* p = cur + (wr * WM + 16 * i + l16) * LDS_ROW + 8 * q;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(p), x1 = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
      for (int s = 0; s < 4; ++s) { af[i][s] = x0[s]; af[i][4 + s] = x1[s]; }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const float* p = cur + SA + (wc * WN + 16 * j + l16) * LDS_ROW + 8 * q;
      const f32x4 x0 = *reinterpret_cast<const f32x4*>(p), x1 = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
      for (int s = 0; s < 4; ++s) { bf[j][s] = x0[s]; bf[j][4 + s] = x1[s]; }
    }
    la.store(nxt);
    lb.store(nxt + SA);
    la.load(ktile(kt + 2), kend);
    lb.load(ktile(kt + 2), kend);
#pragma unroll
    for (int s = 0; s < 8; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][s], bf[j][s], acc[i][j], 0, 0, 0);
    __syncthreads();
  }
}

template <int BM, int BN, int WM, int WN, class OpA, class OpB>
SD_DEV void gemm16_mainloop(OpA& la, OpB& lb, int kbeg, int kend, f32x4 (&acc)[WM / 16][WN / 16]) {
  OpA (&a1)[1] = *reinterpret_cast<OpA(*)[1]>(&la);
  OpB (&b1)[1] = *reinterpret_cast<OpB(*)[1]>(&lb);
  gemm16_mainloop_pf<BM, BN, WM, WN, 1>(a1, b1, kbeg, kend, acc);
}

template <int BM, int BN, int WM, int WN, bool ES = false, class OpA, class OpB>
SD_DEV void gemm_block16(const GemmArgs& g, OpA& la, OpB& lb, int bm0, int bn0, int b, int split, int kbeg,
                         int kend) {
  constexpr int WAVES_N = BN / WN;
  constexpr int TM = WM / 16, TN = WN / 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / WAVES_N, wc = wave % WAVES_N;
  const int l16 = lane & 15, q = lane >> 4;
  f32x4 acc[TM][TN];
  if constexpr (ES)
    gemm16_mainloop_es<BM, BN, WM, WN>(la, lb, kbeg, kend, acc);
  else
    gemm16_mainloop<BM, BN, WM, WN>(la, lb, kbeg, kend, acc);

  // epilogue: reg r of a 16x16 tile -> row 4q + r, col l16
  if (g.ksplit > 1) {
    float* W = g.ws + ((long)split * g.batch + b) * (long)g.M * g.N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = bn0 + wc * WN + 16 * j + l16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = bm0 + wr * WM + 16 * i + 4 * q + r;
          if (m < g.M && n < g.N) W[(long)m * g.N + n] = g.alpha * acc[i][j][r];
        }
      }
    return;
  }
  float* C = g.C + (long)b * g.sC;
  const float* bias = g.bias ? g.bias + (long)b * g.sBias : nullptr;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = bn0 + wc * WN + 16 * j + l16;
      const float bv = (bias && n < g.N) ? bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = bm0 + wr * WM + 16 * i + 4 * q + r;
        if (m < g.M && n < g.N) {
          float v = g.alpha * acc[i][j][r] + bv;
          float* c = C + (long)m * g.ldc + n;
          if (g.beta != 0.f) v += g.beta * *c;
          *c = v;
        }
      }
    }
}

template <int BM, int BN, int WM, int WN, bool AK, bool BKC, bool VA, bool VB>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs g) {
  const int bn0 = blockIdx.x * BN, bm0 = blockIdx.y * BM;
  const int b = blockIdx.z / g.ksplit, split = blockIdx.z % g.ksplit;
  const int kbeg = split * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  DenseOperand<BM, AK, VA> la(g.A + (long)b * g.sA, g.lda, g.M, bm0);
  DenseOperand<BN, BKC, VB> lb(g.B + (long)b * g.sB, g.ldb, g.N, bn0);
  gemm_block<BM, BN, WM, WN>(g, la, lb, bm0, bn0, b, split, kbeg, kend);
}

__global__ void gemm_reduce_kernel(GemmArgs g) {
  const long MN = (long)g.M * g.N;
  const long total = MN * g.batch;
  for (long t = blockIdx.x * (long)blockDim.x + threadIdx.x; t < total; t += (long)gridDim.x * blockDim.x) {
    const int b = (int)(t / MN);
    const long mn = t % MN;
    const int m = (int)(mn / g.N), n = (int)(mn % g.N);
    float v = 0.f;
    for (int s = 0; s < g.ksplit; ++s) v += g.ws[((long)s * g.batch + b) * MN + mn];
    if (g.bias) v += g.bias[(long)b * g.sBias + n];
    float* c = g.C + (long)b * g.sC + (long)m * g.ldc + n;
    if (g.beta != 0.f) v += g.beta * *c;
    *c = v;
  }
  if (g.rowsum) {  // the bias gradient's split partials, fixed order (batch 1)
    for (long m = blockIdx.x * (long)blockDim.x + threadIdx.x; m < g.M; m += (long)gridDim.x * blockDim.x) {
      float v = 0.f;
      for (int s = 0; s < g.ksplit; ++s) v += g.rs_ws[(long)s * g.M + m];
      float* o = rowsum_at(g, (int)m);
      *o = (g.rs_acc ? *o : 0.f) + g.alpha * v;
    }
  }
}


}  // namespace
}  // namespace sdg
