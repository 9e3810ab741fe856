// Three-way split-bf16 ("bf16x6") GEMM main loop: an fp32-accurate contraction on v_mfma_f32_16x16x32_bf16.
//
// Each fp32 operand is split where it is staged into LDS: a = a0 + a1 + a2, a0 = bf16(a), a1 = bf16(a - a0),
// a2 = bf16(a - a0 - a1) (both differences are exact by Sterbenz; |a - a0 - a1 - a2| <= 2^-27 |a|). The product
// keeps every term down to 2^-18 relative, a2*b0 + a1*b1 + a0*b2 + a1*b0 + a0*b1 + a0*b0 — six bf16 MFMAs with
// exact products and fp32 accumulation, smallest terms first — and drops a1*b2, a2*b1, a2*b2 (<= 2^-26 |ab|).
// The result carries fp32-level error (measured on K = 2048 dot products: max |err| / sum|a||b| 8e-8 vs 1.5e-7
// for an fp32 fma chain), at 6 x 16 = 96 MFMA cycles per 16x16x32 tile step against 8 x 32 = 256 for
// v_mfma_f32_16x16x4_f32 over the same K: 2.67x the fp32 MFMA rate. Unlike the two-way split of gemm3_core.h
// (~1e-5 relative, used only where no sampled index depends on the result) this is a drop-in for the exact fp32
// path on the sampling chain (imagination, encoder forward).
//
// LDS image per operand tile: [row][a0 k0..31 | a1 k0..31 | a2 k0..31 | pad 16] bf16 = 224-B rows (56 dwords:
// the 16 rows x 4 lane groups of a ds_read_b128 fragment read hit 64 distinct banks). MFMA operand per lane: row
// l16, k = 8q .. 8q+7 (q = lane >> 4), one ds_read_b128 per plane; accumulator register r of a 16x16 tile holds
// row 4q + r, column l16 (the layout of gemm16_mainloop_pf, so epilogues are shared).
//
// Loaders are gemm16_mainloop_pf's (load(k0, kend) into registers) plus store6(__bf16*), which writes the three
// planes of their BM/BN x 32 register tile (split3_store per float4).
#pragma once
#include "common.h"

namespace sdg {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int BK6 = 32;            // fp32-equivalent k per tile (one 16x16x32 step per plane pair)
constexpr int LROW6 = 3 * BK6 + 16;  // bf16 per LDS row

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// RNE bf16 pair of (a, b) in one v_cvt_pk_bf16_f32, and the two floats it represents read back from the packed bits
// (a shift and a mask: hipcc otherwise re-converts each element separately to get them back)
SD_DEV uint32_t bf16_pair(float a, float b, float& ra, float& rb) {
  const uint32_t p = __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{a, b}, bf16x2));
  ra = __builtin_bit_cast(float, p << 16);
  rb = __builtin_bit_cast(float, p & 0xffff0000u);
  return p;
}

SD_DEV void split3_store(__bf16* dst, f32x4 v) {
  float h0, h1, h2, h3, m0, m1, m2, m3;
  const u32x2 h{bf16_pair(v[0], v[1], h0, h1), bf16_pair(v[2], v[3], h2, h3)};
  const float r0 = v[0] - h0, r1 = v[1] - h1, r2 = v[2] - h2, r3 = v[3] - h3;
  const u32x2 m{bf16_pair(r0, r1, m0, m1), bf16_pair(r2, r3, m2, m3)};
  const f32x4 l{r0 - m0, r1 - m1, r2 - m2, r3 - m3};
  *reinterpret_cast<u32x2*>(dst) = h;
  *reinterpret_cast<u32x2*>(dst + BK6) = m;
  *reinterpret_cast<bf16x4*>(dst + 2 * BK6) = __builtin_convertvector(l, bf16x4);
}

// split3_store with non-temporal stores (written for another XCD's next launch: streamed out of this XCD's L2)
SD_DEV void split3_store_nt(__bf16* dst, f32x4 v) {
  float h0, h1, h2, h3, m0, m1, m2, m3;
  const u32x2 h{bf16_pair(v[0], v[1], h0, h1), bf16_pair(v[2], v[3], h2, h3)};
  const float r0 = v[0] - h0, r1 = v[1] - h1, r2 = v[2] - h2, r3 = v[3] - h3;
  const u32x2 m{bf16_pair(r0, r1, m0, m1), bf16_pair(r2, r3, m2, m3)};
  const f32x4 l{r0 - m0, r1 - m1, r2 - m2, r3 - m3};
  __builtin_nontemporal_store(h, reinterpret_cast<u32x2*>(dst));
  __builtin_nontemporal_store(m, reinterpret_cast<u32x2*>(dst + BK6));
  __builtin_nontemporal_store(__builtin_bit_cast(u32x2, __builtin_convertvector(l, bf16x4)),
                              reinterpret_cast<u32x2*>(dst + 2 * BK6));
}

template <int N>
SD_DEV __bf16* sd_smem6() {
  __shared__ __attribute__((aligned(16))) __bf16 s[N];
  return s;
}
template <int BM, int BN>
constexpr int gemm6_smem_bf16() {
  return 2 * (BM + BN) * LROW6;
}

// acc += A . B^T over [kbeg, kend) with PF k tiles in flight in registers and a double-buffered LDS image (one
// barrier per tile), the structure of gemm16_mainloop_pf (late store behind a sched_barrier).
template <int BM, int BN, int WM, int WN, int PF, class OpA, class OpB>
SD_DEV void gemm6_mainloop_pf(OpA (&la)[PF], OpB (&lb)[PF], int kbeg, int kend, f32x4 (&acc)[WM / 16][WN / 16],
                              bool accumulate = false) {
  constexpr int WAVES_N = BN / WN;
  constexpr int TM = WM / 16, TN = WN / 16;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves");
  constexpr int SA = BM * LROW6, STAGE = (BM + BN) * LROW6;
  __bf16* smem = sd_smem6<2 * STAGE>();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / WAVES_N, wc = wave % WAVES_N;
  const int l16 = lane & 15, q = lane >> 4;
  if (!accumulate) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int nk = (kend - kbeg + BK6 - 1) / BK6;
  if (nk <= 0) return;
  auto ktile = [&](int t) { return kbeg + (t < nk ? t : nk - 1) * BK6; };  // clamped: branch-free steady state
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    la[u].load(ktile(u), kend);
    lb[u].load(ktile(u), kend);
  }
  la[0].store6(smem);
  lb[0].store6(smem + SA);
  __syncthreads();
  la[0].load(ktile(PF), kend);
  lb[0].load(ktile(PF), kend);
  auto step = [&](int kt, int u) {
    const __bf16* cur = smem + (kt & 1) * STAGE;
    bf16x8 a[TM][3], b[TN][3];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const __bf16* p = cur + (wr * WM + 16 * i + l16) * LROW6 + 8 * q;
#pragma unroll
      for (int s = 0; s < 3; ++s) a[i][s] = *reinterpret_cast<const bf16x8*>(p + s * BK6);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const __bf16* p = cur + SA + (wc * WN + 16 * j + l16) * LROW6 + 8 * q;
#pragma unroll
      for (int s = 0; s < 3; ++s) b[j][s] = *reinterpret_cast<const bf16x8*>(p + s * BK6);
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x4 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][2], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b[j][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[j][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[j][1], c, 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[j][0], c, 0, 0, 0);
      }
    const int nx = (u + 1) % PF;
    __builtin_amdgcn_sched_barrier(0);
    la[nx].store6(smem + ((kt & 1) ^ 1) * STAGE);
    lb[nx].store6(smem + ((kt & 1) ^ 1) * STAGE + SA);
    la[nx].load(ktile(kt + 1 + PF), kend);
    lb[nx].load(ktile(kt + 1 + PF), kend);
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
}

// Single-stage form: half the LDS of gemm6_mainloop_pf (one staging buffer), two barriers per k tile (stage ->
// barrier -> fragment reads -> barrier -> MFMAs, which run from registers while the next tile is staged). For
// launches whose double-buffered LDS footprint would cap residency below the grid (k_gate: 2 -> 4 workgroups per CU,
// its 1,024 workgroups in one round instead of two).
template <int BM, int BN, int WM, int WN, int PF, class OpA, class OpB>
SD_DEV void gemm6_mainloop_1s(OpA (&la)[PF], OpB (&lb)[PF], int kbeg, int kend, f32x4 (&acc)[WM / 16][WN / 16],
                              bool accumulate = false) {
  constexpr int WAVES_N = BN / WN;
  constexpr int TM = WM / 16, TN = WN / 16;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves");
  constexpr int SA = BM * LROW6, STAGE = (BM + BN) * LROW6;
  __bf16* smem = sd_smem6<STAGE>();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / WAVES_N, wc = wave % WAVES_N;
  const int l16 = lane & 15, q = lane >> 4;
  if (!accumulate) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int nk = (kend - kbeg + BK6 - 1) / BK6;
  if (nk <= 0) return;
  auto ktile = [&](int t) { return kbeg + (t < nk ? t : nk - 1) * BK6; };
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    la[u].load(ktile(u), kend);
    lb[u].load(ktile(u), kend);
  }
  auto step = [&](int kt, int u) {
    la[u].store6(smem);
    lb[u].store6(smem + SA);
    la[u].load(ktile(kt + PF), kend);
    lb[u].load(ktile(kt + PF), kend);
    __syncthreads();
    bf16x8 a[TM][3], b[TN][3];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const __bf16* p = smem + (wr * WM + 16 * i + l16) * LROW6 + 8 * q;
#pragma unroll
      for (int s = 0; s < 3; ++s) a[i][s] = *reinterpret_cast<const bf16x8*>(p + s * BK6);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const __bf16* p = smem + SA + (wc * WN + 16 * j + l16) * LROW6 + 8 * q;
#pragma unroll
      for (int s = 0; s < 3; ++s) b[j][s] = *reinterpret_cast<const bf16x8*>(p + s * BK6);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x4 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][2], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b[j][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[j][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][1], b[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[j][1], c, 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][0], b[j][0], c, 0, 0, 0);
      }
  };
  int kt = 0;
  for (; kt + PF <= nk; kt += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) step(kt + u, u);
  }
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (kt + u < nk) step(kt + u, u);
}

// Fragment-prefetch form (gemm_core.h gemm16_mainloop_fp): iteration kt reads tile kt+1's three planes from LDS
// before running tile kt's MFMAs on fragments read one iteration earlier, then stores tile kt+2 into stage kt&1.
template <int BM, int BN, int WM, int WN, int PF, class OpA, class OpB>
SD_DEV void gemm6_mainloop_fp(OpA (&la)[PF], OpB (&lb)[PF], int kbeg, int kend, f32x4 (&acc)[WM / 16][WN / 16],
                              bool accumulate = false) {
  constexpr int WAVES_N = BN / WN;
  constexpr int TM = WM / 16, TN = WN / 16;
  static_assert((BM / WM) * (BN / WN) == 4, "4 waves");
  constexpr int SA = BM * LROW6, STAGE = (BM + BN) * LROW6;
  __bf16* smem = sd_smem6<2 * STAGE>();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave / WAVES_N, wc = wave % WAVES_N;
  const int l16 = lane & 15, q = lane >> 4;
  if (!accumulate) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int nk = (kend - kbeg + BK6 - 1) / BK6;
  if (nk <= 0) return;
  auto ktile = [&](int t) { return kbeg + (t < nk ? t : nk - 1) * BK6; };
  bf16x8 fa[TM][3], fb[TN][3], na[TM][3], nb[TN][3];
  auto frags = [&](int stage, bf16x8 (&a)[TM][3], bf16x8 (&b)[TN][3]) {
    const __bf16* cur = smem + stage * STAGE;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const __bf16* p = cur + (wr * WM + 16 * i + l16) * LROW6 + 8 * q;
#pragma unroll
      for (int s = 0; s < 3; ++s) a[i][s] = *reinterpret_cast<const bf16x8*>(p + s * BK6);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const __bf16* p = cur + SA + (wc * WN + 16 * j + l16) * LROW6 + 8 * q;
#pragma unroll
      for (int s = 0; s < 3; ++s) b[j][s] = *reinterpret_cast<const bf16x8*>(p + s * BK6);
    }
  };
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    la[u].load(ktile(u), kend);
    lb[u].load(ktile(u), kend);
  }
  la[0].store6(smem);
  lb[0].store6(smem + SA);
  la[0].load(ktile(PF), kend);
  lb[0].load(ktile(PF), kend);
  __syncthreads();
  frags(0, fa, fb);
  la[1 % PF].store6(smem + STAGE);
  lb[1 % PF].store6(smem + STAGE + SA);
  la[1 % PF].load(ktile(1 + PF), kend);
  lb[1 % PF].load(ktile(1 + PF), kend);
  __syncthreads();
  auto step = [&](int kt, int u) {
    frags((kt + 1) & 1, na, nb);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        f32x4 c = acc[i][j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][2], fb[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[j][1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], fb[j][0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][1], c, 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], fb[j][0], c, 0, 0, 0);
      }
    const int nx = (u + 2) % PF;
    __builtin_amdgcn_sched_barrier(0);
    la[nx].store6(smem + (kt & 1) * STAGE);
    lb[nx].store6(smem + (kt & 1) * STAGE + SA);
    la[nx].load(ktile(kt + 2 + PF), kend);
    lb[nx].load(ktile(kt + 2 + PF), kend);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int s = 0; s < 3; ++s) fa[i][s] = na[i][s];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int s = 0; s < 3; ++s) fb[j][s] = nb[j][s];
  };
  int kt = 0;
  for (; kt + PF <= nk; kt += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) step(kt + u, u);
  }
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (kt + u < nk) step(kt + u, u);
}

}  // namespace
}  // namespace sdg
