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
  if (va && vb) SD_PAD_LAUNCH((gemm_kernel<BM, BN, WM, WN, AK, BKC, true, true>), grid, 256, st, g);
  else if (va) SD_PAD_LAUNCH((gemm_kernel<BM, BN, WM, WN, AK, BKC, true, false>), grid, 256, st, g);
  else if (vb) SD_PAD_LAUNCH((gemm_kernel<BM, BN, WM, WN, AK, BKC, false, true>), grid, 256, st, g);
  else SD_PAD_LAUNCH((gemm_kernel<BM, BN, WM, WN, AK, BKC, false, false>), grid, 256, st, g);
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

// ---------------------------------------------------------------- skinny GEMM (M <= 32), e.g. the per-step
// contractions of the RSSM observe scan (B = 16 rows). Weight-streaming bound: no LDS staging, each lane loads
// its A row and B column as float4 straight to registers, 4 independent 8-deep k chunks in flight per lane,
// the 4 waves of a workgroup take interleaved k chunks and are summed through LDS at the end; K is further split
// across workgroups (slabs + the deterministic reduce) so a 16 x 256 x 2048 GEMV still spans ~128 CUs.
template <bool BKC, bool VA, bool VB>
__global__ __launch_bounds__(256) void gemm_skinny(GemmArgs g) {
  constexpr int U = 4;
  __shared__ float red[4][16][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l32 = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.x * 32;
  const int split = blockIdx.y, b = blockIdx.z;
  const int kbeg = split * g.kchunk, kend = min(g.K, kbeg + g.kchunk);
  const float* A = g.A + (long)b * g.sA;
  const float* Bp = g.B + (long)b * g.sB;
  const int m = l32, n = n0 + l32;
  const bool mv = m < g.M, nv = n < g.N;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  for (int k = kbeg + 8 * wave; k < kend; k += 32 * U) {
    f32x4 a[U], bb[U];
#pragma unroll
    for (int i = 0; i < U; ++i) {
      const int kk = k + 32 * i + 4 * h;
      f32x4 x = {0.f, 0.f, 0.f, 0.f}, y = {0.f, 0.f, 0.f, 0.f};
      if (kk < kend) {
        if (mv) {
          const float* q = A + (long)m * g.lda + kk;
          if (VA && kk + 3 < kend) x = *reinterpret_cast<const f32x4*>(q);
          else {
#pragma unroll
            for (int j = 0; j < 4; ++j) if (kk + j < kend) x[j] = q[j];
          }
        }
        if (nv) {
          if (BKC) {
            const float* q = Bp + (long)n * g.ldb + kk;
            if (VB && kk + 3 < kend) y = *reinterpret_cast<const f32x4*>(q);
            else {
#pragma unroll
              for (int j = 0; j < 4; ++j) if (kk + j < kend) y[j] = q[j];
            }
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) if (kk + j < kend) y[j] = Bp[(long)(kk + j) * g.ldb + n];
          }
        }
      }
      a[i] = x;
      bb[i] = y;
    }
#pragma unroll
    for (int i = 0; i < U; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][j], bb[i][j], acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) red[wave][r][lane] = acc[r];
  __syncthreads();
  // wave w finalises registers r = 4w .. 4w+3
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int r = 4 * wave + q;
    const float v = (red[0][r][lane] + red[1][r][lane]) + (red[2][r][lane] + red[3][r][lane]);
    const int row = (r & 3) + 8 * (r >> 2) + 4 * h;
    if (row < g.M && nv) {
      if (g.ksplit > 1) {
        g.ws[((long)split * g.batch + b) * (long)g.M * g.N + (long)row * g.N + n] = g.alpha * v;
      } else {
        float o = g.alpha * v + (g.bias ? g.bias[(long)b * g.sBias + n] : 0.f);
        float* c = g.C + (long)b * g.sC + (long)row * g.ldc + n;
        if (g.beta != 0.f) o += g.beta * *c;
        *c = o;
      }
    }
  }
}


// ---------------------------------------------------------------- 16-row GEMM (M <= 16) on v_mfma_f32_16x16x4_f32
// One workgroup = 8 waves = one 16-column tile over the whole K (no split-K launch): wave w streams k chunks
// w, w+8, ... (16 k per chunk: lane group q = lane>>4 holds k = 4q..4q+3 of its A row / B column as one float4),
// 4 chunks in flight per lane; the 8 partial 16x16 tiles are summed through LDS. Used by the observe scan
// (M = B rows per GPU) where every step streams the RSSM weights once from L2 / Infinity Cache.
template <bool BKC, bool VA, bool VB>
__global__ __launch_bounds__(512) void gemm_m16(GemmArgs g) {
  constexpr int U = 4, NW = 8;
  __shared__ float red[NW][4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l16 = lane & 15, q = lane >> 4;
  const int n0 = blockIdx.x * 16;
  const int split = blockIdx.y, b = blockIdx.z;
  const int kbeg = split * g.kchunk, kend = min(g.K, kbeg + g.kchunk);
  const float* A = g.A + (long)b * g.sA;
  const float* Bp = g.B + (long)b * g.sB;
  const int m = l16, n = n0 + l16;
  const bool mv = m < g.M, nv = n < g.N;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k = kbeg + 16 * wave; k < kend; k += 16 * NW * U) {
    f32x4 a[U], bb[U];
#pragma unroll
    for (int i = 0; i < U; ++i) {
      const int kk = k + 16 * NW * i + 4 * q;
      f32x4 x = {0.f, 0.f, 0.f, 0.f}, y = {0.f, 0.f, 0.f, 0.f};
      if (kk < kend) {
        if (mv) {
          const float* p = A + (long)m * g.lda + kk;
          if (VA && kk + 3 < kend) x = *reinterpret_cast<const f32x4*>(p);
          else {
#pragma unroll
            for (int j = 0; j < 4; ++j) if (kk + j < kend) x[j] = p[j];
          }
        }
        if (nv) {
          if (BKC) {
            const float* p = Bp + (long)n * g.ldb + kk;
            if (VB && kk + 3 < kend) y = *reinterpret_cast<const f32x4*>(p);
            else {
#pragma unroll
              for (int j = 0; j < 4; ++j) if (kk + j < kend) y[j] = p[j];
            }
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) if (kk + j < kend) y[j] = Bp[(long)(kk + j) * g.ldb + n];
          }
        }
      }
      a[i] = x;
      bb[i] = y;
    }
#pragma unroll
    for (int i = 0; i < U; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][j], bb[i][j], acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[wave][r][lane] = acc[r];
  __syncthreads();
  if (wave < 4) {  // wave w finalises accumulator register r = w: row = 4*(lane>>4) + r, col = lane & 15
    const int r = wave;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[w][r][lane];
    const int row = 4 * q + r;
    if (row < g.M && nv) {
      if (g.ksplit > 1) {
        g.ws[((long)split * g.batch + b) * (long)g.M * g.N + (long)row * g.N + n] = g.alpha * v;
      } else {
        float o = g.alpha * v + (g.bias ? g.bias[(long)b * g.sBias + n] : 0.f);
        float* c = g.C + (long)b * g.sC + (long)row * g.ldc + n;
        if (g.beta != 0.f) o += g.beta * *c;
        *c = o;
      }
    }
  }
}

void launch_m16(const GemmArgs& g, bool bk, bool va, bool vb, hipStream_t st) {
  dim3 grid(sd_cdiv(g.N, 16), g.ksplit, g.batch);
#define M16_L(B_, A_, V_) gemm_m16<B_, A_, V_><<<grid, 512, 0, st>>>(g)
  if (bk) {
    if (va && vb) M16_L(true, true, true); else if (va) M16_L(true, true, false);
    else if (vb) M16_L(true, false, true); else M16_L(true, false, false);
  } else {
    if (va) M16_L(false, true, false); else M16_L(false, false, false);
  }
#undef M16_L
}

void launch_skinny(const GemmArgs& g, bool bk, bool va, bool vb, hipStream_t st) {
  dim3 grid(sd_cdiv(g.N, 32), g.ksplit, g.batch);
#define SK_L(B_, A_, V_) gemm_skinny<B_, A_, V_><<<grid, 256, 0, st>>>(g)
  if (bk) {
    if (va && vb) SK_L(true, true, true); else if (va) SK_L(true, true, false);
    else if (vb) SK_L(true, false, true); else SK_L(true, false, false);
  } else {
    if (va) SK_L(false, true, false); else SK_L(false, false, false);
  }
#undef SK_L
}

}  // namespace

extern "C" int sd_gemm_f32(const sd_gemm_desc* d, float* workspace, long workspace_floats, sd_stream stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  if (!d || !d->A || !d->B || !d->C) return SD_EARG;
  if (d->M <= 0 || d->N <= 0 || d->batch <= 0) return SD_OK;
  GemmArgs g{};
  g.A = d->A; g.B = d->B; g.C = d->C; g.bias = d->bias; g.ws = workspace;
  g.lda = d->lda; g.ldb = d->ldb; g.ldc = d->ldc;
  g.sA = d->strideA; g.sB = d->strideB; g.sC = d->strideC; g.sBias = d->strideBias;
  g.M = d->M; g.N = d->N; g.K = d->K; g.batch = d->batch;
  g.alpha = d->alpha; g.beta = d->beta;
  int ks = d->ksplit < 1 ? 1 : d->ksplit;
  if (d->K <= 0) ks = 1;
  if (ks > 1 && (!workspace || workspace_floats < (long)ks * d->batch * d->M * d->N)) return SD_EARG;
  g.ksplit = ks;
  const bool skinny = d->M <= 32 && d->a_kcontig && d->tile < 0;
  const bool m16 = skinny && d->M <= 16;
  const int kgran = m16 ? 16 : skinny ? 32 : BK;
  long kc = ((long)(d->K > 0 ? d->K : 1) + ks - 1) / ks;
  kc = (kc + kgran - 1) / kgran * kgran;
  g.kchunk = (int)kc;
  const bool ak = d->a_kcontig != 0, bk = d->b_kcontig != 0;
  // float4 staging needs 16-B aligned bases, ld % 4 == 0 and batch strides % 4 == 0
  const bool va = aligned16(d->A) && d->lda % 4 == 0 && (d->batch == 1 || d->strideA % 4 == 0);
  const bool vb = aligned16(d->B) && d->ldb % 4 == 0 && (d->batch == 1 || d->strideB % 4 == 0);
  if (skinny) {
    if (m16) launch_m16(g, bk, va, vb, stream);
    else launch_skinny(g, bk, va, vb, stream);
    SD_LAUNCH_CHECK();
    if (ks > 1) {
      long total = (long)d->batch * d->M * d->N;
      int blocks = (int)((total + 255) / 256);
      gemm_reduce_kernel<<<blocks, 256, 0, stream>>>(g);
      SD_LAUNCH_CHECK();
    }
    return SD_OK;
  }
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
