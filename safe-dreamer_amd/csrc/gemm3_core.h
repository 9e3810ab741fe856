// Split-bf16 ("bf16x3") GEMM core on v_mfma_f32_16x16x32_bf16 (gfx950: 1024 FLOP/clk/SIMD, 16x the f32 MFMA).
//
// Every fp32 operand is split when it is staged into LDS: a = hi + lo with hi = bf16(a), lo = bf16(a - hi)
// (|a - hi - lo| <= 2^-17 |a|). The product a*b is taken as hi_a*hi_b + hi_a*lo_b + lo_a*hi_b — three bf16 MFMAs
// with exact products, accumulated in fp32 — dropping lo_a*lo_b (<= 2^-18 |ab|). A K-term dot product carries
// ~1e-5 relative error of the typical |term| * sqrt(K) (f32 MFMA: ~1e-7) at 16/3 = 5.3x the f32 MFMA rate.
// Used for the contractions whose results feed no sampled index: gradients (input and weight) of every linear
// and convolution, and the frozen imagined heads. Sampled latents and actions stay on the exact f32 path.
//
// LDS image per operand tile: [row][hi k0..31 | lo k0..31 | pad 8] bf16 (144-B rows, 36 banks: the 16 rows of a
// fragment read hit 16 distinct 4-bank groups). MFMA operand per lane: row l16 (A: m, B: n), k = 8q .. 8q+7
// (q = lane >> 4) as one ds_read_b128 per plane; accumulator reg r of a 16x16 tile -> row 4q + r, column l16.
#pragma once
#include "common.h"
#include "gemm_core.h"

namespace sdb {
namespace {
using sdg::GemmArgs;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 32;
#ifndef SD_G3_PAD  // bf16 of padding per LDS row (A/B knob)
#define SD_G3_PAD 8
#endif
constexpr int LROW = 2 * BK + SD_G3_PAD;  // bf16 per LDS row

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// v = hi + lo (+ <= 2^-17 |v|): hi as packed RNE pairs read back by shift / mask (hipcc otherwise converts each element
// back separately: 16 -> 10 VALU per float4), lo = bf16(v - hi)
SD_DEV void split2(f32x4 v, bf16x4& hi, bf16x4& lo) {
  const uint32_t p0 = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{v[0], v[1]}, bf16x2));
  const uint32_t p1 = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{v[2], v[3]}, bf16x2));
  const f32x4 h{__builtin_bit_cast(float, p0 << 16), __builtin_bit_cast(float, p0 & 0xffff0000u),
                __builtin_bit_cast(float, p1 << 16), __builtin_bit_cast(float, p1 & 0xffff0000u)};
  hi = __builtin_bit_cast(bf16x4, (uint64_t)p0 | ((uint64_t)p1 << 32));
  lo = __builtin_convertvector(v - h, bf16x4);
}

SD_DEV void split_store(__bf16* dst, f32x4 v) {
  bf16x4 hi, lo;
  split2(v, hi, lo);
  *reinterpret_cast<bf16x4*>(dst) = hi;
  *reinterpret_cast<bf16x4*>(dst + BK) = lo;
}

// Operand with k contiguous (row r, k at p[r * ld + k]): thread loads float4 runs along k.
template <int ROWS, bool VEC>
struct KC3 {
  static constexpr int NV = (ROWS * BK / 4 + 255) / 256;
  f32x4 r[NV];
  const float* p;
  long ld;
  int nrows, row0;
  SD_DEV KC3(const float* base, long ld_, int nrows_, int row0_) : p(base), ld(ld_), nrows(nrows_), row0(row0_) {}
  SD_DEV void load(int k0, int kend) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + v * 256;
      const int row = i / (BK / 4), gk = k0 + 4 * (i % (BK / 4)), gr = row0 + row;
      f32x4 x = {0.f, 0.f, 0.f, 0.f};
      if (i < ROWS * BK / 4 && gr < nrows) {
        const float* q = p + (long)gr * ld + gk;
        if (VEC && gk + 3 < kend) {
          x = *reinterpret_cast<const f32x4*>(q);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (gk + j < kend) x[j] = q[j];
        }
      }
      r[v] = x;
    }
  }
  SD_DEV void store(__bf16* lds) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + v * 256;
      if ((v + 1) * 256 <= ROWS * BK / 4 || i < ROWS * BK / 4)
        split_store(lds + (i / (BK / 4)) * LROW + 4 * (i % (BK / 4)), r[v]);
    }
  }
};

// Operand with rows contiguous (row r, k at p[k * ld + r]): thread loads a 4 (k) x 4 (rows) block as four float4
// runs along the rows (coalesced), transposes it in registers and stores four k-runs.
template <int ROWS, bool VEC>
struct KM3 {
  static constexpr int NBLK = ROWS * BK / 16;
  static constexpr int NV = (NBLK + 255) / 256;
  f32x4 r[NV][4];
  // sums over k of the thread's 4 rows per block (rowsum(): the bias gradient of a weight-gradient GEMM)
  SD_DEV void rowsum_add(f32x4 (&acc)[NV]) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) acc[v] += (r[v][0] + r[v][1]) + (r[v][2] + r[v][3]);
  }
  const float* p;
  long ld;
  int nrows, row0;
  SD_DEV KM3(const float* base, long ld_, int nrows_, int row0_) : p(base), ld(ld_), nrows(nrows_), row0(row0_) {}
  SD_DEV void load(int k0, int kend) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + v * 256;
      const int rq = i % (ROWS / 4), kq = i / (ROWS / 4);
      const int gr = row0 + 4 * rq;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const int gk = k0 + 4 * kq + kk;
        f32x4 x = {0.f, 0.f, 0.f, 0.f};
        if (i < NBLK && gk < kend) {
          const float* q = p + (long)gk * ld + gr;
          if (VEC && gr + 3 < nrows) {
            x = *reinterpret_cast<const f32x4*>(q);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (gr + j < nrows) x[j] = q[j];
          }
        }
        r[v][kk] = x;
      }
    }
  }
  SD_DEV void store(__bf16* lds) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + v * 256;
      if ((v + 1) * 256 <= NBLK || i < NBLK) {
        const int rq = i % (ROWS / 4), kq = i / (ROWS / 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x4 t = {r[v][0][j], r[v][1][j], r[v][2][j], r[v][3][j]};
          split_store(lds + (4 * rq + j) * LROW + 4 * kq, t);
        }
      }
    }
  }
};

// Row sums of an A loader's tiles over the K loop, in a fixed order: per thread in rowsum_add, then over the BK / 4
// k-quads of a row in row_sums_km3. Wraps the loader; the tile is added when it is staged into LDS (k-tile order, the
// loads' registers are consumed there anyway), not when its loads are issued — adding at issue made every k tile wait
// for its own loads before the MFMAs. Two wrappers may share one accumulator (gemm3_mainloop_d2's register sets).
template <class Op>
struct RowSumOp {
  Op& op;
  f32x4 (&acc)[Op::NV];
  static constexpr int NVv = Op::NV;
  SD_DEV RowSumOp(Op& o, f32x4 (&a)[Op::NV]) : op(o), acc(a) {}
  SD_DEV void load(int k0, int kend) { op.load(k0, kend); }
  SD_DEV void store(__bf16* lds) {
    op.rowsum_add(acc);
    op.store(lds);
  }
};
// KM3<ROWS> block i = (rq = i % (ROWS / 4), kq = i / (ROWS / 4)) holds rows 4rq..4rq+3; part: LDS (BK / 4) x ROWS
template <int ROWS, int NV>
SD_DEV void row_sums_km3(const f32x4 (&acc)[NV], float* part, float* out_rows) {
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int i = threadIdx.x + v * 256;
    if (i < ROWS * BK / 16) {
      const int rq = i % (ROWS / 4), kq = i / (ROWS / 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) part[kq * ROWS + 4 * rq + j] = acc[v][j];
    }
  }
  __syncthreads();
  for (int r = threadIdx.x; r < ROWS; r += 256) {
    float s = 0.f;
#pragma unroll
    for (int kq = 0; kq < BK / 4; ++kq) s += part[kq * ROWS + r];
    out_rows[r] = s;
  }
  __syncthreads();
}

template <int BM, int BN>
constexpr int gemm3_smem_bf16() {
  return 2 * (BM + BN) * LROW;
}

// Double-buffered main loop: the next k tile's global loads are issued before this tile's MFMAs and staged (split)
// into the other LDS buffer after them; one barrier per k tile.
template <int BM, int BN, int WM, int WN, class OpA, class OpB>
SD_DEV void gemm3_mainloop(OpA& la, OpB& lb, int kbeg, int kend, f32x4 (&acc)[WM / 16][WN / 16]) {
  constexpr int WAVES_N = BN / WN;
  constexpr int TM = WM / 16, TN = WN / 16;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves");
  constexpr int SA = BM * LROW, STAGE = (BM + BN) * LROW;
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * STAGE];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / WAVES_N, wc = wave % WAVES_N;
  const int l16 = lane & 15, q = lane >> 4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (kend - kbeg + BK - 1) / BK;
  if (nk <= 0) return;
  la.load(kbeg, kend);
  lb.load(kbeg, kend);
  la.store(smem);
  lb.store(smem + SA);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const __bf16* cur = smem + (kt & 1) * STAGE;
    if (kt + 1 < nk) {
      la.load(kbeg + (kt + 1) * BK, kend);
      lb.load(kbeg + (kt + 1) * BK, kend);
    }
    bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const __bf16* p = cur + (wr * WM + 16 * i + l16) * LROW + 8 * q;
      ah[i] = *reinterpret_cast<const bf16x8*>(p);
      al[i] = *reinterpret_cast<const bf16x8*>(p + BK);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const __bf16* p = cur + SA + (wc * WN + 16 * j + l16) * LROW + 8 * q;
      bh[j] = *reinterpret_cast<const bf16x8*>(p);
      bl[j] = *reinterpret_cast<const bf16x8*>(p + BK);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
      }
    if (kt + 1 < nk) {
      __bf16* nxt = smem + ((kt & 1) ^ 1) * STAGE;
      la.store(nxt);
      lb.store(nxt + SA);
    }
    __syncthreads();
  }
}

// Two-deep register prefetch: two register sets per operand (the loader copied), so tile kt+2's global loads are in
// flight across tile kt+1's MFMAs as well as tile kt's — two k tiles of L2 latency cover instead of one. Same LDS
// double buffer, products and k order as gemm3_mainloop (bit-identical results). Iteration kt: MFMAs on LDS stage
// kt & 1, stage tile kt+1 from register set X, reissue X's loads for tile kt+3; unrolled by two so X and Y swap.
// (la, lb) and (la2, lb2) are the two register sets: copies of one loader (RowSumOp: each wraps its own copy).
template <int BM, int BN, int WM, int WN, class OpA, class OpB>
SD_DEV void gemm3_mainloop_d2(OpA& la, OpB& lb, OpA& la2, OpB& lb2, int kbeg, int kend,
                              f32x4 (&acc)[WM / 16][WN / 16]) {
  constexpr int WAVES_N = BN / WN;
  constexpr int TM = WM / 16, TN = WN / 16;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves");
  constexpr int SA = BM * LROW, STAGE = (BM + BN) * LROW;
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * STAGE];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / WAVES_N, wc = wave % WAVES_N;
  const int l16 = lane & 15, q = lane >> 4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = (kend - kbeg + BK - 1) / BK;
  if (nk <= 0) return;
  la.load(kbeg, kend);
  lb.load(kbeg, kend);
  if (nk > 1) {
    la2.load(kbeg + BK, kend);
    lb2.load(kbeg + BK, kend);
  }
  la.store(smem);
  lb.store(smem + SA);
  if (nk > 2) {
    la.load(kbeg + 2 * BK, kend);
    lb.load(kbeg + 2 * BK, kend);
  }
  __syncthreads();
  auto step = [&](int kt, OpA& xa, OpB& xb) {  // x: the register set holding tile kt+1
    const __bf16* cur = smem + (kt & 1) * STAGE;
    bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const __bf16* p = cur + (wr * WM + 16 * i + l16) * LROW + 8 * q;
      ah[i] = *reinterpret_cast<const bf16x8*>(p);
      al[i] = *reinterpret_cast<const bf16x8*>(p + BK);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const __bf16* p = cur + SA + (wc * WN + 16 * j + l16) * LROW + 8 * q;
      bh[j] = *reinterpret_cast<const bf16x8*>(p);
      bl[j] = *reinterpret_cast<const bf16x8*>(p + BK);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
      }
    if (kt + 1 < nk) {
      __bf16* nxt = smem + ((kt & 1) ^ 1) * STAGE;
      xa.store(nxt);
      xb.store(nxt + SA);
    }
    if (kt + 3 < nk) {
      xa.load(kbeg + (kt + 3) * BK, kend);
      xb.load(kbeg + (kt + 3) * BK, kend);
    }
    __syncthreads();
  };
  int kt = 0;
  for (; kt + 2 <= nk; kt += 2) {
    step(kt, la2, lb2);
    step(kt + 1, la, lb);
  }
  if (kt < nk) step(kt, la2, lb2);
}

// Fragment-prefetch form (gemm_core.h gemm16_mainloop_fp): iteration kt reads tile kt+1's fragments from LDS before
// its MFMAs on tile kt (read one iteration earlier), then stages tile kt+2 into the stage tile kt came from and
// issues tile kt+3's loads. Branch-free (clamped tile indices); unrolled by two so the fragment sets swap roles
// instead of being copied.
template <int BM, int BN, int WM, int WN, class OpA, class OpB>
SD_DEV void gemm3_mainloop_fp(OpA& la, OpB& lb, int kbeg, int kend, f32x4 (&acc)[WM / 16][WN / 16]) {
  constexpr int WAVES_N = BN / WN;
  constexpr int TM = WM / 16, TN = WN / 16;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves");
  constexpr int SA = BM * LROW, STAGE = (BM + BN) * LROW;
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * STAGE];
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
  struct Frags {
    bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
  };
  auto frags = [&](int stage, Frags& f) {
    const __bf16* cur = smem + stage * STAGE;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const __bf16* p = cur + (wr * WM + 16 * i + l16) * LROW + 8 * q;
      f.ah[i] = *reinterpret_cast<const bf16x8*>(p);
      f.al[i] = *reinterpret_cast<const bf16x8*>(p + BK);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const __bf16* p = cur + SA + (wc * WN + 16 * j + l16) * LROW + 8 * q;
      f.bh[j] = *reinterpret_cast<const bf16x8*>(p);
      f.bl[j] = *reinterpret_cast<const bf16x8*>(p + BK);
    }
  };
  Frags f0, f1;
  la.load(ktile(0), kend);
  lb.load(ktile(0), kend);
  la.store(smem);
  lb.store(smem + SA);
  la.load(ktile(1), kend);
  lb.load(ktile(1), kend);
  __syncthreads();
  frags(0, f0);
  la.store(smem + STAGE);
  lb.store(smem + STAGE + SA);
  la.load(ktile(2), kend);
  lb.load(ktile(2), kend);
  __syncthreads();
  auto step = [&](int kt, const Frags& f, Frags& nf) {
    frags((kt + 1) & 1, nf);  // tile kt+1 (a clamped, unused copy past the end)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.al[i], f.bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.ah[i], f.bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.ah[i], f.bh[j], acc[i][j], 0, 0, 0);
      }
    __builtin_amdgcn_sched_barrier(0);
    la.store(smem + (kt & 1) * STAGE);  // tile kt+2
    lb.store(smem + (kt & 1) * STAGE + SA);
    la.load(ktile(kt + 3), kend);
    lb.load(ktile(kt + 3), kend);
    __syncthreads();
  };
  int kt = 0;
  for (; kt + 2 <= nk; kt += 2) {
    step(kt, f0, f1);
    step(kt + 1, f1, f0);
  }
  if (kt < nk) step(kt, f0, f1);
}

// C tile epilogue (alpha, bias, beta; or a split-K partial slab)
template <int BM, int BN, int WM, int WN>
SD_DEV void gemm3_epilogue(const GemmArgs& g, const f32x4 (&acc)[WM / 16][WN / 16], int bm0, int bn0, int b,
                           int split) {
  constexpr int WAVES_N = BN / WN;
  constexpr int TM = WM / 16, TN = WN / 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / WAVES_N, wc = wave % WAVES_N;
  const int l16 = lane & 15, q = lane >> 4;
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

}  // namespace
}  // namespace sdb
