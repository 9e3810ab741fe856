// fp32 GEMM on the gfx950 matrix cores (v_mfma_f32_32x32x2_f32: exact f32 fma chains, 64 FLOP/clk/SIMD).
//
//   C[b] = alpha * A[b] . B[b] (+ bias[n]) (+ beta * C[b])      A: M x K, B: K x N, C: M x N row-major (ldc)
//
// Every dense contraction of the Dreamer update is routed here: nn.Linear forward (A=x rows, B=W rows: both
// K-contiguous), its input gradient (B=W, N-contiguous), its weight gradient (A=dy^T, B=x: both M/N-contiguous,
// long K -> split-K), BlockLinear (networks.py:24-56) as a strided batch over the G blocks, and the Barlow
// cross-correlation (dreamer.py:528). Operand layout is a compile-time choice (A_K / B_K: "k is the contiguous
// index"), so every global->LDS copy is a coalesced float4 stream.
//
// Tiling: 256 threads = 4 waves, a BM x BN block tile, BK = 16, register-staged double-buffered LDS.
// LDS image per operand is [row][BK+4] (80-byte rows): each lane reads its 8 k-values for one MFMA row as two
// ds_read_b128, conflict-free (5 is odd -> the 16 lanes of a b128 group hit 16 distinct 16-B slots).
// The MFMA's k order is permuted (lane half h supplies k = s + 8h at step s) — the product is a sum, so any
// k order is valid as long as A and B agree.
// Split-K writes fp32 partial slabs that sd_gemm_reduce sums in a fixed order (deterministic, no atomics).
#include "common.h"
#include "sdhip.h"

#include "gemm_core.h"

namespace {
using namespace sdg;

template <int BM, int BN, int WM, int WN, bool AK, bool BKC>
void launch_tile(const GemmArgs& g, bool va, bool vb, hipStream_t st) {
  dim3 grid(sd_cdiv(g.N, BN), sd_cdiv(g.M, BM), g.batch * g.ksplit);
  if (va && vb) gemm_kernel<BM, BN, WM, WN, AK, BKC, true, true><<<grid, 256, 0, st>>>(g);
  else if (va) gemm_kernel<BM, BN, WM, WN, AK, BKC, true, false><<<grid, 256, 0, st>>>(g);
  else if (vb) gemm_kernel<BM, BN, WM, WN, AK, BKC, false, true><<<grid, 256, 0, st>>>(g);
  else gemm_kernel<BM, BN, WM, WN, AK, BKC, false, false><<<grid, 256, 0, st>>>(g);
}

template <bool AK, bool BKC>
void launch_layout(const GemmArgs& g, int tile, bool va, bool vb, hipStream_t st) {
  switch (tile) {
    case 0: launch_tile<128, 128, 64, 64, AK, BKC>(g, va, vb, st); break;
    case 1: launch_tile<64, 64, 32, 32, AK, BKC>(g, va, vb, st); break;
    case 2: launch_tile<32, 128, 32, 32, AK, BKC>(g, va, vb, st); break;
    default: launch_tile<128, 64, 64, 32, AK, BKC>(g, va, vb, st); break;
  }
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" int sd_gemm_f32(const sd_gemm_desc* d, float* workspace, long workspace_floats, sd_stream stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  if (!d || !d->A || !d->B || !d->C) return SD_EARG;
  if (d->M <= 0 || d->N <= 0 || d->batch <= 0) return SD_OK;
  GemmArgs g;
  g.A = d->A; g.B = d->B; g.C = d->C; g.bias = d->bias; g.ws = workspace;
  g.lda = d->lda; g.ldb = d->ldb; g.ldc = d->ldc;
  g.sA = d->strideA; g.sB = d->strideB; g.sC = d->strideC; g.sBias = d->strideBias;
  g.M = d->M; g.N = d->N; g.K = d->K; g.batch = d->batch;
  g.alpha = d->alpha; g.beta = d->beta;
  int ks = d->ksplit < 1 ? 1 : d->ksplit;
  if (d->K <= 0) ks = 1;
  if (ks > 1 && (!workspace || workspace_floats < (long)ks * d->batch * d->M * d->N)) return SD_EARG;
  g.ksplit = ks;
  long kc = ((long)(d->K > 0 ? d->K : 1) + ks - 1) / ks;
  kc = (kc + BK - 1) / BK * BK;
  g.kchunk = (int)kc;
  const bool ak = d->a_kcontig != 0, bk = d->b_kcontig != 0;
  // float4 staging needs 16-B aligned bases, ld % 4 == 0 and batch strides % 4 == 0
  const bool va = aligned16(d->A) && d->lda % 4 == 0 && (d->batch == 1 || d->strideA % 4 == 0);
  const bool vb = aligned16(d->B) && d->ldb % 4 == 0 && (d->batch == 1 || d->strideB % 4 == 0);
  int tile = d->tile;
  if (tile < 0) {
    long tiles128 = (long)sd_cdiv(d->M, 128) * sd_cdiv(d->N, 128) * d->batch * ks;
    if (d->M <= 32) tile = 2;
    else if (tiles128 >= 256) tile = 0;
    else tile = 1;
  }
  if (ak && bk) launch_layout<true, true>(g, tile, va, vb, stream);
  else if (ak) launch_layout<true, false>(g, tile, va, vb, stream);
  else if (bk) launch_layout<false, true>(g, tile, va, vb, stream);
  else launch_layout<false, false>(g, tile, va, vb, stream);
  SD_LAUNCH_CHECK();
  if (ks > 1) {
    long total = (long)d->batch * d->M * d->N;
    int blocks = (int)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    gemm_reduce_kernel<<<blocks, 256, 0, stream>>>(g);
    SD_LAUNCH_CHECK();
  }
  return SD_OK;
}
