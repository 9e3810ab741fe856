// Dense split-bf16 GEMM (gemm3_core.h): same contract as sd_gemm_f32 (gemm.hip) — C[b] = alpha * A[b] . B[b]
// (+ bias) (+ beta * C[b]), strided batch, either unit stride per operand, split-K slabs summed in a fixed order —
// at ~1e-5 relative accuracy instead of f32's ~1e-7. Shapes below one 64x64 tile per operand side go to the f32
// kernels (they are latency-bound there anyway).
#include "common.h"
#include "sdhip.h"

#include "gemm3_core.h"

namespace {
using namespace sdb;

#ifndef SD_G3_FP  // fragment-prefetch main loop (gemm3_core.h gemm3_mainloop_fp): measured no faster (4096^3 536 vs 540 us, update 13.85 vs 13.76 ms), off
#define SD_G3_FP 0
#endif

// (re-measured on the round-5 tree: 1 / 2 = 10.84 / 10.81 vs 10.80 ms, profiles/r05d2: off)
#ifndef SD_G3_D2  // two-deep register prefetch main loop (gemm3_core.h gemm3_mainloop_d2): 1 = 128-row tiles, 2 = all
#define SD_G3_D2 0
#endif
template <int BM>
constexpr bool g3_d2() {
  return SD_G3_D2 >= 2 || (SD_G3_D2 == 1 && BM >= 128);
}
#ifndef SD_G3_M256  // 256 x 128 tiles for the weight-gradient shape (gemm3_run)
#define SD_G3_M256 0  // measured slower: actor L0 dW 250.7 vs 194.2 us (1 workgroup per CU hides less latency)
#endif
#ifndef SD_G3_XCD  // XCD-contiguous tile order (below)
#define SD_G3_XCD 1
#endif
// Tile order. The dispatcher deals workgroups to the 8 XCDs round robin by linear id, and each XCD has its own L2:
// in the plain (x fastest) order the column tiles that share an A row panel run on different XCDs at the same time,
// so every XCD streams that panel from HBM. Remapped, XCD x runs a contiguous run of the logical order (x fastest,
// then the row tile, then batch x split), so the tiles sharing an A row panel (and, across the short row loop of a
// weight-gradient GEMM, a B column panel) are resident together on one XCD and read it once into its L2. When A is
// broadcast over the batch (strideA == 0, e.g. the imagined heads' first layers: one input, four weights), the batch
// loop moves inside the row loop, so one A panel feeds every batch entry's tiles from the same L2.
SD_DEV void g3_tile(const GemmArgs& g, int& tx, int& ty, int& tz) {
  const int nx = gridDim.x, ny = gridDim.y, nz = gridDim.z;
  int L = blockIdx.x + nx * (blockIdx.y + ny * blockIdx.z);
  if (SD_G3_XCD) {
    const int T = nx * ny * nz, per = T / 8, rem = T % 8, xcd = L % 8, slot = L / 8;
    L = xcd * per + (xcd < rem ? xcd : rem) + slot;  // XCD xcd holds per (+1 for the first rem XCDs) tiles
  }
  if (g.sA == 0 && g.batch > 1 && g.ksplit == 1) {  // A broadcast over the batch: x, then batch, then row tile
    tx = L % nx;
    tz = (L / nx) % nz;
    ty = L / (nx * nz);
  } else {
    tx = L % nx;
    ty = (L / nx) % ny;
    tz = L / (nx * ny);
  }
}

template <int BM, int BN, int WM, int WN, bool AK, bool BKC, bool VA, bool VB, bool RS = false>
__global__ __launch_bounds__(256, (BM >= 256 ? 1 : 2)) void gemm3_kernel(GemmArgs g) {
  int tx, ty, tz;
  g3_tile(g, tx, ty, tz);
  const int bn0 = tx * BN, bm0 = ty * BM;
  const int b = tz / g.ksplit, split = tz % g.ksplit;
  const int kbeg = split * g.kchunk;
  const int kend = min(g.K, kbeg + g.kchunk);
  const float* A = g.A + (long)b * g.sA;
  const float* Bp = g.B + (long)b * g.sB;
  using OA = typename std::conditional<AK, KC3<BM, VA>, KM3<BM, VA>>::type;
  using OB = typename std::conditional<BKC, KC3<BN, VB>, KM3<BN, VB>>::type;
  OA la(A, g.lda, g.M, bm0);
  OB lb(Bp, g.ldb, g.N, bn0);
  f32x4 acc[WM / 16][WN / 16];
  if constexpr (RS) {  // weight gradient: also the row sums of A (the bias gradient), written by column tile 0
    static_assert(!AK, "row sums need the rows-contiguous A loader");
    f32x4 rsum[OA::NV];
#pragma unroll
    for (int v = 0; v < OA::NV; ++v) rsum[v] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (g3_d2<BM>()) {
      OA la2 = la;
      OB lb2 = lb;
      RowSumOp<OA> ra(la, rsum), ra2(la2, rsum);
      gemm3_mainloop_d2<BM, BN, WM, WN>(ra, lb, ra2, lb2, kbeg, kend, acc);
    } else {
      RowSumOp<OA> ra(la, rsum);
      gemm3_mainloop<BM, BN, WM, WN>(ra, lb, kbeg, kend, acc);
    }
    if (tx == 0) {
      __shared__ float part[(BK / 4) * BM], rows[BM];
      row_sums_km3<BM>(rsum, part, rows);
      for (int r = threadIdx.x; r < BM; r += 256) {
        const int m = bm0 + r;
        if (m >= g.M) continue;
        if (g.ksplit > 1)
          g.rs_ws[(long)split * g.M + m] = rows[r];
        else {
          float* o = rowsum_at(g, m);
          *o = (g.rs_acc ? *o : 0.f) + g.alpha * rows[r];
        }
      }
    }
  } else if (SD_G3_FP) {
    gemm3_mainloop_fp<BM, BN, WM, WN>(la, lb, kbeg, kend, acc);
  } else if (g3_d2<BM>()) {
    OA la2 = la;
    OB lb2 = lb;
    gemm3_mainloop_d2<BM, BN, WM, WN>(la, lb, la2, lb2, kbeg, kend, acc);
  } else {
    gemm3_mainloop<BM, BN, WM, WN>(la, lb, kbeg, kend, acc);
  }
  gemm3_epilogue<BM, BN, WM, WN>(g, acc, bm0, bn0, b, split);
}

template <int BM, int BN, int WM, int WN, bool AK, bool BKC>
void launch3_tile(const GemmArgs& g, bool va, bool vb, hipStream_t st) {
  dim3 grid(sd_cdiv(g.N, BN), sd_cdiv(g.M, BM), g.batch * g.ksplit);
  if constexpr (!AK) {
    if (g.rowsum) {
      if (va && vb) SD_PAD_LAUNCH((gemm3_kernel<BM, BN, WM, WN, AK, BKC, true, true, true>), grid, 256, st, g);
      else if (va) SD_PAD_LAUNCH((gemm3_kernel<BM, BN, WM, WN, AK, BKC, true, false, true>), grid, 256, st, g);
      else if (vb) SD_PAD_LAUNCH((gemm3_kernel<BM, BN, WM, WN, AK, BKC, false, true, true>), grid, 256, st, g);
      else SD_PAD_LAUNCH((gemm3_kernel<BM, BN, WM, WN, AK, BKC, false, false, true>), grid, 256, st, g);
      return;
    }
  }
  if (va && vb) SD_PAD_LAUNCH((gemm3_kernel<BM, BN, WM, WN, AK, BKC, true, true>), grid, 256, st, g);
  else if (va) SD_PAD_LAUNCH((gemm3_kernel<BM, BN, WM, WN, AK, BKC, true, false>), grid, 256, st, g);
  else if (vb) SD_PAD_LAUNCH((gemm3_kernel<BM, BN, WM, WN, AK, BKC, false, true>), grid, 256, st, g);
  else SD_PAD_LAUNCH((gemm3_kernel<BM, BN, WM, WN, AK, BKC, false, false>), grid, 256, st, g);
}

template <bool AK, bool BKC>
void launch3_layout(const GemmArgs& g, int tile, bool va, bool vb, hipStream_t st) {
  if (tile == 0) launch3_tile<128, 128, 64, 64, AK, BKC>(g, va, vb, st);
  else if (tile == 2 && !AK && !BKC) launch3_tile<256, 128, 128, 64, AK, BKC>(g, va, vb, st);
  else launch3_tile<64, 64, 32, 32, AK, BKC>(g, va, vb, st);
}

bool al16_3(const void* p) { return ((uintptr_t)p & 15) == 0; }

// ---- MLP layer on the split-bf16 core (sd_gemm_bf16x3_mlp): C[b] = act(rms(A[b]) * nw[b]) . B[b] + bias[b], the
// RMSNorm (nn.RMSNorm, eps) + SiLU of the previous layer applied to A rows while they are staged into LDS (rstd from
// the producer's per-row partial sums of squares), and optionally this layer's own per-row partials written by the
// epilogue (one per 64 output columns) for the next layer. No normalised tensor is ever materialised.
struct MlpExt {
  const float* nw;
  long sNw;
  const float* pin;
  long sPin;
  int npin, act;
  float eps;
  float* pout;
  long sPout;
  const float* wp[SD_MLP_MAXB];  // per-entry operands (sd_mlp_ext): null = the strided batch
  const float* bp[SD_MLP_MAXB];
  const float* nwp[SD_MLP_MAXB];
  int wrows[SD_MLP_MAXB];
};

// entry b of a per-entry array as a chain of selects (a dynamic index into a kernel-argument array would copy it to
// scratch)
template <class T>
SD_DEV T pick_b(const T (&a)[SD_MLP_MAXB], int b) {
  static_assert(SD_MLP_MAXB == 4, "pick_b");
  return b == 0 ? a[0] : b == 1 ? a[1] : b == 2 ? a[2] : b == 3 ? a[3] : T{};
}

// A operand, k contiguous, rows normalised (x * rs[row] * nw[k], then SiLU if act) when stored into LDS
template <int ROWS>
struct KC3Rms {
  static constexpr int NV = (ROWS * BK / 4 + 255) / 256;
  f32x4 r[NV], w[NV];
  const float* p;
  const float* nw;
  const float* rs;  // LDS, ROWS entries (this tile's rows)
  long ld;
  int nrows, row0, act;
  SD_DEV KC3Rms(const float* base, long ld_, int nrows_, int row0_, const float* nw_, const float* rs_, int act_)
      : p(base), nw(nw_), rs(rs_), ld(ld_), nrows(nrows_), row0(row0_), act(act_) {}
  SD_DEV void load(int k0, int kend) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + v * 256;
      const int row = i / (BK / 4), gk = k0 + 4 * (i % (BK / 4)), gr = row0 + row;
      const bool ok = i < ROWS * BK / 4 && gr < nrows;
      r[v] = ok ? *reinterpret_cast<const f32x4*>(p + (long)gr * ld + gk) : f32x4{0.f, 0.f, 0.f, 0.f};
      w[v] = *reinterpret_cast<const f32x4*>(nw + gk);
    }
  }
  SD_DEV void store(__bf16* lds) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const int i = threadIdx.x + v * 256;
      if ((v + 1) * 256 <= ROWS * BK / 4 || i < ROWS * BK / 4) {
        const int row = i / (BK / 4);
        const float s = rs[row];
        f32x4 x;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float y = r[v][j] * s * w[v][j];
          x[j] = act ? y * sigmoidf_(y) : y;
        }
        split_store(lds + row * LROW + 4 * (i % (BK / 4)), x);
      }
    }
  }
};

// BN = 128: 2 x 2 waves of 64 x 64 (2 workgroups per CU). BN = 256 (the heads' 256-column layers): 2 x 2 waves of
// 64 x 128, one workgroup per CU — each B fragment read from LDS feeds 4 row tiles and each A fragment 8 column tiles,
// 1.33x the MFMAs per LDS byte of the 64 x 64 wave tile (whose main loop the LDS traffic bounds: MFMA busy ~0.35)
#ifndef SD_MLP_WIDE  // measured slower on the imagined heads' first layer (335 vs 274 us alone, r04e), neutral on the
                     // normed hidden layers once that layer moved to gemm3_w256 (update 10.84 vs 10.84 ms, r05mw): off
#define SD_MLP_WIDE 0
#endif
template <bool RMS, bool POUT, int BN>
__global__ __launch_bounds__(256, BN == 128 ? 2 : 1) void gemm3_mlp_kernel(GemmArgs g, MlpExt e) {
  constexpr int BM = 128, WM = 64, WN = BN / 2, TM = WM / 16, TN = WN / 16, NP = WN / 64;
  int tx, ty, tz;
  g3_tile(g, tx, ty, tz);
  const int bn0 = tx * BN, bm0 = ty * BM, b = tz;
  __shared__ float rs[BM];
  const float* A = g.A + (long)b * g.sA;
  const float* wpb = pick_b(e.wp, b);
  const float* Bp = wpb ? wpb : g.B + (long)b * g.sB;
  const int wr_b = pick_b(e.wrows, b), nb = wr_b > 0 ? wr_b : g.N;  // entry b's weight rows (columns >= nb: 0)
  if (RMS) {  // this tile's rows: rstd from the producer's partial sums of squares
    const float* pin = e.pin + (long)b * e.sPin;
    for (int r = threadIdx.x; r < BM; r += 256) {
      const int m = bm0 + r;
      float s = 0.f;
      if (m < g.M)
        for (int q = 0; q < e.npin; ++q) s += pin[(long)q * g.M + m];
      rs[r] = rsqrtf(s / (float)g.K + e.eps);
    }
    __syncthreads();
  }
  f32x4 acc[TM][TN];
  KC3<BN, true> lb(Bp, g.ldb, nb, bn0);
  if constexpr (RMS) {
    const float* nwb = pick_b(e.nwp, b);
    KC3Rms<BM> la(A, g.lda, g.M, bm0, nwb ? nwb : e.nw + (long)b * e.sNw, rs, e.act);
    if constexpr (g3_d2<BM>()) {
      KC3Rms<BM> la2 = la;
      KC3<BN, true> lb2 = lb;
      gemm3_mainloop_d2<BM, BN, WM, WN>(la, lb, la2, lb2, 0, g.K, acc);
    } else {
      gemm3_mainloop<BM, BN, WM, WN>(la, lb, 0, g.K, acc);
    }
  } else {
    KC3<BM, true> la(A, g.lda, g.M, bm0);
    if constexpr (g3_d2<BM>()) {
      KC3<BM, true> la2 = la;
      KC3<BN, true> lb2 = lb;
      gemm3_mainloop_d2<BM, BN, WM, WN>(la, lb, la2, lb2, 0, g.K, acc);
    } else {
      gemm3_mainloop<BM, BN, WM, WN>(la, lb, 0, g.K, acc);
    }
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / (BN / WN), wc = wave % (BN / WN), l16 = lane & 15, q = lane >> 4;
  float* C = g.C + (long)b * g.sC;
  const float* bpb = pick_b(e.bp, b);
  const float* bias = bpb ? bpb : g.bias ? g.bias + (long)b * g.sBias : nullptr;
  float ss[NP][TM][4];
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) ss[p][i][r] = 0.f;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = bn0 + wc * WN + 16 * j + l16;
    const float bv = (bias && n < nb) ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = bm0 + wr * WM + 16 * i + 4 * q + r;
        const float v = g.alpha * acc[i][j][r] + bv;
        if (m < g.M && n < g.N) C[(long)m * g.ldc + n] = v;
        ss[j / 4][i][r] += n < g.N ? v * v : 0.f;
      }
  }
  if (POUT) {  // partials (per 64 columns) of every row's sum of squares
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      float* pout = e.pout + (long)b * e.sPout + (long)((bn0 + wc * WN) / 64 + p) * g.M;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = ss[p][i][r];
          v += __shfl_xor(v, 1, 64);
          v += __shfl_xor(v, 2, 64);
          v += __shfl_xor(v, 4, 64);
          v += __shfl_xor(v, 8, 64);
          const int m = bm0 + wr * WM + 16 * i + 4 * q + r;
          if (l16 == 0 && m < g.M) pout[m] = v;
        }
    }
  }
}

// ---- The wide form for long layers without an input norm (SD_MLP_W256; the imagined heads' first layers: M = H1 * N
// = 16,384 rows, K = feat 2,560, four 256-wide heads on one input). One 256 x 256 tile per workgroup = one entry's
// whole width over 256 rows: 512 threads as 2 (rows) x 4 (columns) waves of 128 x 64, on v_mfma_f32_32x32x16_bf16
// (twice the FLOP per fragment byte of the 16x16x32 tile, so the LDS reads stay under half the MFMA time). Against
// gemm3_mlp_kernel's 128 x 128 tiles every A row panel is read by 4 workgroups instead of 8 and every B panel by 64
// instead of 128; the four entries of a row panel run back to back on one XCD (its L2 serves the panel). One
// workgroup per CU (147 KB of LDS): the next k tile's global loads are issued before this tile's MFMAs and split into
// the other LDS stage after them, one barrier per k tile. Same split products as gemm3_core.h (lo*hi, hi*lo, hi*hi per
// 16-deep step); the 32x32 MFMA sums its 16 k in its own order, so the results differ from the 128 x 128 kernel's at
// the split's ~1e-5 level, not bit for bit.
#ifndef SD_MLP_W256
#define SD_MLP_W256 1
#endif
#ifndef SD_W256_PASSES
#define SD_W256_PASSES 1
#endif
typedef float f32x16 __attribute__((ext_vector_type(16)));
namespace w256 {
constexpr int BM = 256, BN = 256, NT = 512, WM = 128, WN = 64, TM = WM / 32, TN = WN / 32;
constexpr int NV = BM * BK / 4 / NT;  // float4 per thread per operand per k tile (= TM: one per MFMA group)
constexpr int SA = BM * LROW, STAGE = (BM + BN) * LROW;
}  // namespace w256

template <bool POUT>
__global__ __launch_bounds__(512, 1) void gemm3_w256_kernel(GemmArgs g, MlpExt e) {
  using namespace w256;
  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, wr = wave >> 2, wc = wave & 3;
  const int l32 = lane & 31, h = lane >> 5;
  // tile order: the batch entries of one row panel consecutive, runs of T / 8 consecutive tiles per XCD
  const int T = (int)gridDim.x, per = T / 8, rem = T % 8, xcd = (int)blockIdx.x % 8, slot = (int)blockIdx.x / 8;
  const int L = xcd * per + (xcd < rem ? xcd : rem) + slot;
  const int b = L % g.batch, bm0 = (L / g.batch) * BM;
  const float* A = g.A + (long)b * g.sA;
  const float* wpb = pick_b(e.wp, b);
  const float* Bp = wpb ? wpb : g.B + (long)b * g.sB;
  const int wr_b = pick_b(e.wrows, b), nb = wr_b > 0 ? wr_b : g.N;
  // loader slots: float4 v of thread tid = row (tid + NT v) / 8, k quad tid % 8 of the 256 x 32 tile, as byte offsets
  // into range-checked buffer descriptors: rows past M and weight rows past nb get an offset past the range and read
  // 0 (no branch around any load; past-M rows are never stored)
  const sd_rsrc rsa = sd_make_rsrc(A, ((long)(g.M - 1) * g.lda + g.K) * 4);
  const sd_rsrc rsb = sd_make_rsrc(Bp, ((long)(nb - 1) * g.ldb + g.K) * 4);
  uint32_t oa[NV], ob[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int r = (tid + NT * v) >> 3, kq = tid & 7;
    oa[v] = bm0 + r < g.M ? (uint32_t)(((long)(bm0 + r) * g.lda + 4 * kq) * 4) : SD_OOB;
    ob[v] = r < nb ? (uint32_t)(((long)r * g.ldb + 4 * kq) * 4) : SD_OOB;
  }
  const int nk = g.K / BK;
  struct Set {
    f32x4 a[NV], b[NV];
  };
  auto load = [&](Set& x, int kt) {  // tile kt (clamped to the last: the loop's loads are unconditional)
    const uint32_t kb = (uint32_t)((kt < nk ? kt : nk - 1) * BK * 4);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      x.a[v] = sd_bload4(rsa, oa[v] == SD_OOB ? SD_OOB : oa[v] + kb);
      x.b[v] = sd_bload4(rsb, ob[v] == SD_OOB ? SD_OOB : ob[v] + kb);
    }
  };
  const int sr = (tid >> 3) * LROW + 4 * (tid & 7);  // this thread's LDS element in row-slot v = 0
  auto store1 = [&](const Set& x, __bf16* st, int v, int opb) {  // float4 v of operand A (opb 0) / B, split
    split_store(st + (opb ? SA : 0) + sr + v * (NT / 8) * LROW, opb ? x.b[v] : x.a[v]);
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // tile kt's MFMAs in 8 groups of 6 (one row tile i of one 16-deep step s each), each followed by the split + store
  // of one float4 slot of tile kt + 1 (A's slots in step 0, B's in step 1; held in register set y since the previous
  // iteration) into the other stage, so
  // the split's VALU work and LDS writes run between this tile's MFMAs instead of after them
  auto step = [&](int kt, Set& x, Set& y) {  // x: free now (tile kt is staged) -> tile kt + 2; y: tile kt + 1
    load(x, kt + 2);
    __builtin_amdgcn_sched_barrier(0);  // issued first: hipcc otherwise sinks them behind the MFMAs
    const __bf16* cur = smem + (kt & 1) * STAGE;
    __bf16* nxt = smem + ((kt & 1) ^ 1) * STAGE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const __bf16* p = cur + SA + (wc * WN + 32 * j + l32) * LROW + 16 * s + 8 * h;
        bh[j] = *reinterpret_cast<const bf16x8*>(p);
        bl[j] = *reinterpret_cast<const bf16x8*>(p + BK);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const __bf16* p = cur + (wr * WM + 32 * i + l32) * LROW + 16 * s + 8 * h;
        ah[i] = *reinterpret_cast<const bf16x8*>(p);
        al[i] = *reinterpret_cast<const bf16x8*>(p + BK);
      }
#if SD_W256_PASSES  // the three products as three passes over the 8 accumulators (no dependent MFMA back to back)
#pragma unroll
      for (int u = 0; u < 3 * TM * TN; ++u) {
        const int pass = u / (TM * TN), i = (u / TN) % TM, j = u % TN;
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pass == 1 ? ah[i] : pass ? ah[i] : al[i],
                                                           pass == 0 ? bh[j] : pass == 1 ? bl[j] : bh[j],
                                                           acc[i][j], 0, 0, 0);
        if (u % 6 == 5) store1(y, nxt, u / 6, s);
      }
#else
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
        }
        store1(y, nxt, i, s);
      }
#endif
    }
    __syncthreads();
  };
  Set x0, x1;
  load(x0, 0);
  load(x1, 1);
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    store1(x0, smem, v, 0);
    store1(x0, smem, v, 1);
  }
  __syncthreads();
  int kt = 0;
  for (; kt + 2 <= nk; kt += 2) {
    step(kt, x0, x1);
    step(kt + 1, x1, x0);
  }
  if (kt < nk) step(kt, x0, x1);
  // epilogue: register r of tile (i, j) = row 32 i + (r & 3) + 8 (r >> 2) + 4 h, column 32 j + l32 of the wave tile
  float* C = g.C + (long)b * g.sC;
  const float* bpb = pick_b(e.bp, b);
  const float* bias = bpb ? bpb : g.bias ? g.bias + (long)b * g.sBias : nullptr;
  float bv[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = wc * WN + 32 * j + l32;
    bv[j] = (bias && n < nb) ? bias[n] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = bm0 + wr * WM + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
      float ss = 0.f;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = wc * WN + 32 * j + l32;
        const float v = g.alpha * acc[i][j][r] + bv[j];
        if (m < g.M && n < g.N) C[(long)m * g.ldc + n] = v;
        ss += n < g.N ? v * v : 0.f;
      }
      if (POUT) {  // the wave's 64 columns = one partial of the row's sum of squares
        ss += __shfl_xor(ss, 1, 64);
        ss += __shfl_xor(ss, 2, 64);
        ss += __shfl_xor(ss, 4, 64);
        ss += __shfl_xor(ss, 8, 64);
        ss += __shfl_xor(ss, 16, 64);
        if (l32 == 0 && m < g.M) e.pout[(long)b * e.sPout + (long)wc * g.M + m] = ss;
      }
    }
}

}  // namespace

extern "C" int sd_gemm_bf16x3_mlp(const sd_gemm_desc* d, const sd_mlp_ext* x, sd_stream stream_) {
  if (!d || !x || !d->A || !d->B || !d->C) return SD_EARG;
  if (d->M <= 0 || d->N <= 0 || d->batch <= 0) return SD_OK;
  // the fused path's shapes: k-contiguous A and B (C = A . W^T), 16-B aligned, whole 32-deep k tiles, no split-K
  if (!d->a_kcontig || !d->b_kcontig || d->K % BK || d->K < BK || d->N < 64 || d->beta != 0.f) return SD_ESHAPE;
  if (!al16_3(d->A) || !al16_3(d->B) || d->lda % 4 || d->ldb % 4 || (d->batch > 1 && (d->strideA % 4 || d->strideB % 4)))
    return SD_ESHAPE;
  bool any_nw = false;
  for (int b = 0; b < SD_MLP_MAXB && b < d->batch; ++b) any_nw = any_nw || x->norm_w_ptr[b];
  const bool rms = x->norm_w != nullptr || any_nw, pout = x->part_out != nullptr;
  if (rms && (!x->part_in || x->npart_in <= 0 || (x->norm_w && (!al16_3(x->norm_w) || x->stride_norm_w % 4))))
    return SD_EARG;
  if (rms && !x->norm_w)  // every entry needs its own norm weight then
    for (int b = 0; b < d->batch; ++b)
      if (b >= SD_MLP_MAXB || !x->norm_w_ptr[b]) return SD_EARG;
  if (pout && d->N % 64) return SD_ESHAPE;
  bool per_entry = false;
  for (int b = 0; b < SD_MLP_MAXB; ++b) {
    if (x->w_rows[b] < 0 || x->w_rows[b] > d->N) return SD_EARG;
    if ((x->w_ptr[b] && !al16_3(x->w_ptr[b])) || (x->norm_w_ptr[b] && !al16_3(x->norm_w_ptr[b]))) return SD_ESHAPE;
    per_entry = per_entry || x->w_ptr[b] || x->bias_ptr[b] || x->norm_w_ptr[b] || x->w_rows[b];
  }
  if (per_entry && d->batch > SD_MLP_MAXB) return SD_EARG;
  GemmArgs g{};
  g.A = d->A; g.B = d->B; g.C = d->C; g.bias = d->bias; g.ws = nullptr;
  g.lda = d->lda; g.ldb = d->ldb; g.ldc = d->ldc;
  g.sA = d->strideA; g.sB = d->strideB; g.sC = d->strideC; g.sBias = d->strideBias;
  g.M = d->M; g.N = d->N; g.K = d->K; g.batch = d->batch;
  g.alpha = d->alpha; g.beta = 0.f; g.ksplit = 1; g.kchunk = d->K;
  MlpExt e{x->norm_w, x->stride_norm_w, x->part_in, x->stride_part_in, x->npart_in, x->act, x->eps, x->part_out,
           x->stride_part_out, {}, {}, {}, {}};
  for (int b = 0; b < SD_MLP_MAXB; ++b) {
    e.wp[b] = x->w_ptr[b];
    e.bp[b] = x->bias_ptr[b];
    e.nwp[b] = x->norm_w_ptr[b];
    e.wrows[b] = x->w_rows[b];
  }
  hipStream_t st = (hipStream_t)stream_;
  // long layers without an input norm, one 256-wide entry per tile: the 256 x 256 kernel once it fills the chip
  // (SDHIP_MLP_NOW256 set: the 128-tile kernel instead, for the agreement test of the two paths)
  if (SD_MLP_W256 && !rms && g.N == 256 && (long)sd_cdiv(g.M, 256) * g.batch >= 192 && !getenv("SDHIP_MLP_NOW256")) {
    const dim3 grid(sd_cdiv(g.M, 256) * g.batch);
    // (no LDS pad: its 147 KB already hold the CU)
    if (pout) hipLaunchKernelGGL((gemm3_w256_kernel<true>), grid, dim3(512), 0, st, g, e);
    else hipLaunchKernelGGL((gemm3_w256_kernel<false>), grid, dim3(512), 0, st, g, e);
    SD_LAUNCH_CHECK();
    return SD_OK;
  }
  // 256-column tiles where the layer is exactly that wide (every imagined head's hidden layers), else 128
  const bool wide = SD_MLP_WIDE && g.N % 256 == 0;
#define SD_MLP_LAUNCH(BN_)                                                                             \
  do {                                                                                                 \
    const dim3 grid(sd_cdiv(g.N, BN_), sd_cdiv(g.M, 128), g.batch);                                    \
    if (rms && pout) SD_PAD_LAUNCH((gemm3_mlp_kernel<true, true, BN_>), grid, 256, st, g, e);                    \
    else if (rms) SD_PAD_LAUNCH((gemm3_mlp_kernel<true, false, BN_>), grid, 256, st, g, e);                      \
    else if (pout) SD_PAD_LAUNCH((gemm3_mlp_kernel<false, true, BN_>), grid, 256, st, g, e);                     \
    else SD_PAD_LAUNCH((gemm3_mlp_kernel<false, false, BN_>), grid, 256, st, g, e);                              \
  } while (0)
  if (wide) SD_MLP_LAUNCH(256);
  else SD_MLP_LAUNCH(128);
#undef SD_MLP_LAUNCH
  SD_LAUNCH_CHECK();
  return SD_OK;
}

namespace {
int gemm3_run(const sd_gemm_desc* d, float* workspace, long workspace_floats, float* rowsum, int rs_acc,
              sd_stream stream_, int rs_split = 1 << 30, float* rowsum2 = nullptr);
}

extern "C" int sd_gemm_bf16x3(const sd_gemm_desc* d, float* workspace, long workspace_floats, sd_stream stream_) {
  if (!d || !d->A || !d->B || !d->C) return SD_EARG;
  if (d->M <= 0 || d->N <= 0 || d->batch <= 0) return SD_OK;
  if (d->M < 64 || d->N < 64 || d->K < 64) return sd_gemm_f32(d, workspace, workspace_floats, stream_);
  return gemm3_run(d, workspace, workspace_floats, nullptr, 0, stream_);
}

extern "C" int sd_gemm_bf16x3_wgrad(const sd_gemm_desc* d, float* workspace, long workspace_floats, float* rowsum,
                                    int accumulate, sd_stream stream_) {
  if (!d || !d->A || !d->B || !d->C || !rowsum) return SD_EARG;
  if (d->M <= 0 || d->N <= 0) return SD_OK;
  if (d->M < 64 || d->N < 64 || d->K < 64 || d->batch != 1 || d->a_kcontig) return SD_ESHAPE;
  return gemm3_run(d, workspace, workspace_floats, rowsum, accumulate, stream_);
}

extern "C" int sd_gemm_bf16x3_wgrad2(const sd_gemm_desc* d, float* workspace, long workspace_floats, float* rowsum,
                                     float* rowsum2, int rs_split, int accumulate, sd_stream stream_) {
  if (!d || !d->A || !d->B || !d->C || !rowsum || !rowsum2) return SD_EARG;
  if (d->M <= 0 || d->N <= 0) return SD_OK;
  if (d->M < 64 || d->N < 64 || d->K < 64 || d->batch != 1 || d->a_kcontig) return SD_ESHAPE;
  if (rs_split <= 0 || rs_split >= d->M) return SD_ESHAPE;
  return gemm3_run(d, workspace, workspace_floats, rowsum, accumulate, stream_, rs_split, rowsum2);
}

namespace {
#ifndef SD_G3_T128  // 128 x 128 tiles once the launch has this many of them (else 64 x 64). 192 (was 256): the S2
#define SD_G3_T128 192  // input-gradient GEMMs of the imagined actor / value (240 tiles of 128) on 128 x 128 tiles, one
#endif              // round of workgroups: update 10.86 -> 10.79 ms over 6 same-box rounds, bit-identical (r05t128*)
int gemm3_run(const sd_gemm_desc* d, float* workspace, long workspace_floats, float* rowsum, int rs_acc,
              sd_stream stream_, int rs_split, float* rowsum2) {
  hipStream_t stream = (hipStream_t)stream_;
  GemmArgs g{};
  g.rowsum = rowsum;
  g.rs_acc = rs_acc;
  g.rs_split = rs_split;
  g.rowsum2 = rowsum2;
  g.rs_ws = nullptr;
  g.A = d->A; g.B = d->B; g.C = d->C; g.bias = d->bias; g.ws = workspace;
  g.lda = d->lda; g.ldb = d->ldb; g.ldc = d->ldc;
  g.sA = d->strideA; g.sB = d->strideB; g.sC = d->strideC; g.sBias = d->strideBias;
  g.M = d->M; g.N = d->N; g.K = d->K; g.batch = d->batch;
  g.alpha = d->alpha; g.beta = d->beta;
  int ks = d->ksplit < 1 ? 1 : d->ksplit;
  const long slabs = (long)ks * d->batch * d->M * d->N;
  if (ks > 1 && (!workspace || workspace_floats < slabs + (rowsum ? (long)ks * d->M : 0))) return SD_EARG;
  if (ks > 1 && rowsum) g.rs_ws = workspace + slabs;
  g.ksplit = ks;
  long kc = ((long)d->K + ks - 1) / ks;
  g.kchunk = (int)((kc + BK - 1) / BK * BK);
  const bool va = al16_3(d->A) && d->lda % 4 == 0 && (d->batch == 1 || d->strideA % 4 == 0);
  const bool vb = al16_3(d->B) && d->ldb % 4 == 0 && (d->batch == 1 || d->strideB % 4 == 0);
  int tile = d->tile;
  const bool ak = d->a_kcontig != 0, bk = d->b_kcontig != 0;
  if (tile != 0 && tile != 1 && tile != 2) {
    const long tiles128 = (long)sd_cdiv(d->M, 128) * sd_cdiv(d->N, 128) * d->batch * ks;
    tile = tiles128 >= SD_G3_T128 ? 0 : 1;
    // weight-gradient shape (M <= 256 output rows, long split K, both operands rows-contiguous: dW = dy^T x): one
    // 256-row tile covers every M, so each k chunk of x is read once instead of once per 128-row tile
    if (SD_G3_M256 && !ak && !bk && d->M > 128 && d->M <= 256 && ks > 1 && g.kchunk >= 512 && tile == 0) tile = 2;
  }
  if (tile == 2 && (ak || bk)) tile = 0;
  if (ak && bk) launch3_layout<true, true>(g, tile, va, vb, stream);
  else if (ak) launch3_layout<true, false>(g, tile, va, vb, stream);
  else if (bk) launch3_layout<false, true>(g, tile, va, vb, stream);
  else launch3_layout<false, false>(g, tile, va, vb, stream);
  SD_LAUNCH_CHECK();
  if (ks > 1) {
    long total = (long)d->batch * d->M * d->N;
    int blocks = (int)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    sdg::gemm_reduce_kernel<<<blocks, 256, 0, stream>>>(g);
    SD_LAUNCH_CHECK();
  }
  return SD_OK;
}
}  // namespace
