// Fused RSSM posterior scan: RSSM.observe (rssm.py:140-156) -> obs_step (rssm.py:158-178) -> Deter.forward
// (rssm.py:36-75), forward and BPTT backward, for B <= 16 rows per step.
//
// Why launches and not one persistent kernel: on MI355X a dependent kernel boundary costs ~1.5 us, an XCD-
// hierarchical grid barrier ~4-5 us (MI355X_MICROARCH.md price list), so the win is in FEWER, FATTER launches:
// the ~15 kernels of a forward step (mask, GEMM, norm, GEMM, norm, GEMM, block GEMM, norm, block GEMM, GRU, GEMM,
// norm, GEMM, sampler) become 5, the ~20 of a backward step become 6. Every launch is an M=16 MFMA contraction
// (v_mfma_f32_16x16x4_f32, exact fp32) over weights streamed once from L2/MALL:
//   * 512-thread workgroups, one 16-column output tile (or 3 / Kd/16 tiles) each; the 8 waves take interleaved
//     16-deep k chunks, all of a wave's weight float4s are issued BEFORE the prologue runs, so the weight stream
//     overlaps the prologue's own loads;
//   * the A panel (16 rows x K) is built in LDS by a fused prologue: split-K slab reduction + bias + RMSNorm + SiLU,
//     the straight-through sampler's backward (noise recomputed from the counter-based Philox stream), or an
//     RMSNorm backward; row stride K+4 floats keeps the ds_read_b128 fragment loads conflict-free;
//   * the epilogue fuses bias, the GRU gate (fwd and bwd), the unimix one-hot sampler, the reset masks of the next
//     step, and per-tile row partials that the next launch needs for its RMSNorm (deterministic, no atomics).
// Split-K partial slabs are summed by the CONSUMER's prologue (it needs whole rows anyway for its norm), so no
// reduce launch sits between a producer and its consumer.
#include "common.h"
#include "dist_core.h"
#include "philox.h"
#include "sdhip.h"

namespace {

constexpr int NW = 8;
constexpr int NTHR = 64 * NW;
constexpr int MR = 16;

SD_DEV f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }
SD_DEV f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
SD_DEV void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
SD_DEV float dsilu(float z) {
  const float s = sigmoidf_(z);
  return s * (1.f + z * (1.f - s));
}

// ------------------------------------------------------------------------------------------- contraction core
// acc[t] += A[0:16, span] . W_t[n_t + 0:16, span]^T.  Wave w owns k chunks c = w, w+8, ...; lane group q = lane>>4
// supplies k = 16c + 4q .. +3 as one float4 and the MFMA consumes them in 4 steps (a permuted but consistent k order).
template <int NT, int CPW>
struct Core {
  f32x4 b[CPW][NT];
  f32x4 acc[NT];

  // Wt[t]: row (n_t + l16) of a k-contiguous weight matrix, at the span's first k
  SD_DEV void load_b(const float* const* Wt, int nch, int wave, int q) {
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
      const int ch = wave + NW * c;
#pragma unroll
      for (int t = 0; t < NT; ++t) b[c][t] = ch < nch ? ld4(Wt[t] + ch * 16 + 4 * q) : zero4();
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = zero4();
  }
  SD_DEV void mma(const f32x4& a, int c) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], b[c][t][j], acc[t], 0, 0, 0);
  }
  // A from an LDS panel with row stride lda (lda % 64 == 4)
  SD_DEV void run_lds(const float* P, int lda, int nch, int wave, int l16, int q) {
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
      const int ch = wave + NW * c;
      if (ch < nch) mma(ld4(P + l16 * lda + ch * 16 + 4 * q), c);
    }
  }
  // A straight from global memory (rows >= M are zero); all loads issued before the first MFMA
  SD_DEV void run_glb(const float* A, long lda, int M, int nch, int wave, int l16, int q) {
    f32x4 a[CPW];
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
      const int ch = wave + NW * c;
      a[c] = (ch < nch && l16 < M) ? ld4(A + (long)l16 * lda + ch * 16 + 4 * q) : zero4();
    }
#pragma unroll
    for (int c = 0; c < CPW; ++c)
      if (wave + NW * c < nch) mma(a[c], c);
  }
  // sum the 8 waves' partial tiles into C (16 x 16NT, row-major) in LDS
  SD_DEV void reduce(float* red, float* C, int tid, int wave, int lane) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[((wave * NT + t) * 4 + r) * 64 + lane] = acc[t][r];
    __syncthreads();
    for (int i = tid; i < NT * 256; i += NTHR) {
      const int t = i >> 8, r = (i >> 6) & 3, ln = i & 63;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) v += red[((w * NT + t) * 4 + r) * 64 + ln];
      C[(4 * (ln >> 4) + r) * (16 * NT) + t * 16 + (ln & 15)] = v;
    }
    __syncthreads();
  }
};

template <int NT>
constexpr int core_lds_floats() { return NW * NT * 256 + MR * 16 * NT; }

#define SD_THREAD_IDS                                      \
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6; \
  const int l16 = lane & 15, q = lane >> 4;                \
  (void)l16; (void)q;

// ------------------------------------------------------------------------------------------- prologue pieces
// 32 threads per row (16 rows). x = sum_s slab[s] (+ bias) (+ add); y = silu(x * rsqrt(mean(x^2)+eps) * w) into the
// LDS panel P (stride ldp). Rows >= M are zero. Saves x / y (row stride ldys) / r when the pointers are non-null.
SD_DEV void pro_rms(const float* slab, int ks, long sstride, const float* bias, const float* add, int N, int M,
                    const float* w, float eps, float* P, int ldp, float* sx, float* sy, long ldys, float* sr, int tid) {
  const int row = tid >> 5, t32 = tid & 31;
  const bool rv = row < M;
  float ss = 0.f;
  for (int c = 4 * t32; c < N; c += 128) {
    f32x4 x = zero4();
    if (rv) {
      for (int s = 0; s < ks; ++s) x += ld4(slab + s * sstride + (long)row * N + c);
      if (bias) x += ld4(bias + c);
      if (add) x += ld4(add + (long)row * N + c);
      if (sx) st4(sx + (long)row * N + c, x);
    }
    st4(P + row * ldp + c, x);
    ss += x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3];
  }
  ss = group_sum<32>(ss);
  const float r = rsqrtf(ss / (float)N + eps);
  if (sr && rv && t32 == 0) sr[row] = r;
  for (int c = 4 * t32; c < N; c += 128) {
    const f32x4 x = ld4(P + row * ldp + c), wv = ld4(w + c);
    f32x4 y;
#pragma unroll
    for (int j = 0; j < 4; ++j) y[j] = rv ? siluf_(x[j] * r * wv[j]) : 0.f;
    st4(P + row * ldp + c, y);
    if (sy && rv) st4(sy + (long)row * ldys + c, y);
  }
}

// RMSNorm+SiLU backward of full rows: dx = r (g - xh mean(g xh)), g = dy silu'(xh w) w, xh = x r.  dy, x: (M,N).
// Result into P (stride ldp); saved to sdx when non-null.
SD_DEV void pro_rms_bwd(const float* x, const float* rstd, const float* w, const float* dy, int N, int M, float* P,
                        int ldp, float* sdx, int tid) {
  const int row = tid >> 5, t32 = tid & 31;
  const bool rv = row < M;
  const float r = rv ? rstd[row] : 0.f;
  float dot = 0.f;
  for (int c = 4 * t32; c < N; c += 128) {
    f32x4 g = zero4();
    if (rv) {
      const f32x4 xv = ld4(x + (long)row * N + c), wv = ld4(w + c), d = ld4(dy + (long)row * N + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float xh = xv[j] * r;
        g[j] = d[j] * dsilu(xh * wv[j]) * wv[j];
        dot += g[j] * xh;
      }
    }
    st4(P + row * ldp + c, g);
  }
  dot = group_sum<32>(dot) / (float)N;
  for (int c = 4 * t32; c < N; c += 128) {
    f32x4 o = zero4();
    if (rv) {
      const f32x4 g = ld4(P + row * ldp + c), xv = ld4(x + (long)row * N + c);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = r * (g[j] - xv[j] * r * dot);
      if (sdx) st4(sdx + (long)row * N + c, o);
    }
    st4(P + row * ldp + c, o);
  }
}

// per-row sum of `tiles` partials part[i*16 + row] (fixed order per thread + fixed tree): 32 threads per row
SD_DEV float row_partials(const float* part, int tiles, int tid) {
  const int row = tid >> 5, t32 = tid & 31;
  float s = 0.f;
  for (int i = t32; i < tiles; i += 32) s += part[i * MR + row];
  return group_sum<32>(s);
}

// rows [0, M) of a (M, ld) global matrix, columns [0, N) -> LDS panel; rows >= M zero
SD_DEV void pro_copy(const float* src, long ld, int N, int M, float* P, int ldp, int tid) {
  const int row = tid >> 5, t32 = tid & 31;
  for (int c = 4 * t32; c < N; c += 128) st4(P + row * ldp + c, row < M ? ld4(src + (long)row * ld + c) : zero4());
}

// ------------------------------------------------------------------------------------------- scratch layout
struct Work {
  float *x0s, *x1s, *ops, *ssh, *dotp, *dxs, *dhin, *gq, *cs, *ch;
  long total;
};
long al64(long n) { return (n + 63) / 64 * 64; }
Work work_layout(const sd_rssm_scan& d, float* base) {
  Work w;
  long o = 0;
  const long BU = (long)d.B * d.U;
  auto take = [&](long n) { float* p = base ? base + o : nullptr; o += al64(n); return p; };
  w.x0s = take(d.ks_d * BU);
  w.x1s = take(d.ks_s * BU);
  w.ops = take(d.ks_d * BU);
  w.ssh = take((long)d.D);
  w.dotp = take((long)d.D);
  w.dxs = take((long)d.G * d.B * 3 * d.U);
  w.dhin = take((long)d.B * d.D);
  w.gq = take((long)d.B * d.D);
  w.cs = take((long)d.B * d.SK);
  w.ch = take((long)d.B * d.D);
  w.total = o;
  return w;
}

// ------------------------------------------------------------------------------------------- forward kernels
struct SlabProb {
  const float* A;
  long lda;
  const float* W;
  long ldw;
  float* out;                 // slab s at out + s*M*N
  const unsigned char* mask;  // rows whose input is reset (output row forced to 0), or null
};

// plain M=16 GEMM into split-K slabs: out[s][m][n] = A[m, span_s] . W[n, span_s]; grid (N/16, ks, nprob)
template <int CPW>
__global__ __launch_bounds__(NTHR) void k_slab(SlabProb p0, SlabProb p1, int M, int N, int span) {
  extern __shared__ float smem[];
  SD_THREAD_IDS
  const SlabProb p = blockIdx.z ? p1 : p0;
  const int n0 = blockIdx.x * 16, s = blockIdx.y, kb = s * span, nch = span / 16;
  Core<1, CPW> core;
  const float* wt[1] = {p.W + (long)(n0 + l16) * p.ldw + kb};
  core.load_b(wt, nch, wave, q);
  core.run_glb(p.A + kb, p.lda, M, nch, wave, l16, q);
  float* C = smem + NW * 256;
  core.reduce(smem, C, tid, wave, lane);
  if (tid < 256) {
    const int row = tid >> 4, c = tid & 15;
    if (row < M) {
      float v = C[row * 16 + c];
      if (p.mask && p.mask[row]) v = 0.f;
      p.out[(long)s * M * N + (long)row * N + n0 + c] = v;
    }
  }
}

// s_in[0] = mask(stoch0), h_in[0] = mask(deter0)   (rssm.py:161-165 on the initial state)
__global__ void k_init(sd_rssm_scan d) {
  const long nS = (long)d.B * d.SK, nD = (long)d.B * d.D;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nS + nD; i += (long)gridDim.x * blockDim.x) {
    if (i < nS) {
      const int row = (int)(i / d.SK);
      d.s_in[i] = d.reset[row] ? 0.f : d.stoch0[i];
    } else {
      const long j = i - nS;
      const int row = (int)(j / d.D);
      d.h_in[j] = d.reset[row] ? 0.f : d.deter0[j];
    }
  }
}

// hp[t] = BlockLinear(dyn_hid_0)([h_g | x0 | x1 | x2]) + bh, with x0 = silu(rms(x0p)), x1 = silu(rms(x1p)) built
// in the prologue (rssm.py:52-63). grid (D/16); also the per-tile row sums of hp^2 for the next norm.
template <int CPW>
__global__ __launch_bounds__(NTHR) void k_hid(sd_rssm_scan d, Work w, int t) {
  extern __shared__ float smem[];
  SD_THREAD_IDS
  const int B = d.B, U = d.U, D = d.D, Dg = D / d.G, Ig = Dg + 3 * U, ldp = Ig + 4;
  const int tile = blockIdx.x, n0 = tile * 16, g = n0 / Dg;
  Core<1, CPW> core;
  const float* wt[1] = {d.Wh + (long)(n0 + l16) * Ig};
  core.load_b(wt, Ig / 16, wave, q);
  float* P = smem + core_lds_floats<1>();
  const long tBU = (long)t * B * U;
  pro_copy(d.h_in + (long)t * B * D + (long)g * Dg, D, Dg, B, P, ldp, tid);
  pro_rms(w.x0s, d.ks_d, (long)B * U, d.b0, nullptr, U, B, d.n0, d.eps, P + Dg, ldp,
          tile == 0 ? d.x0p + tBU : nullptr, tile == 0 ? d.xcat + 3 * tBU : nullptr, 3 * U,
          tile == 0 ? d.r0 + (long)t * B : nullptr, tid);
  pro_rms(w.x1s, d.ks_s, (long)B * U, d.b1, nullptr, U, B, d.n1, d.eps, P + Dg + U, ldp,
          tile == 1 ? d.x1p + tBU : nullptr, tile == 1 ? d.xcat + 3 * tBU + U : nullptr, 3 * U,
          tile == 1 ? d.r1 + (long)t * B : nullptr, tid);
  pro_copy(d.x2 + tBU, U, U, B, P + Dg + 2 * U, ldp, tid);
  if (tile == 2) {
    const int row = tid >> 5, t32 = tid & 31;
    if (row < B)
      for (int c = 4 * t32; c < U; c += 128) st4(d.xcat + 3 * tBU + (long)row * 3 * U + 2 * U + c, ld4(P + row * ldp + Dg + 2 * U + c));
  }
  __syncthreads();
  core.run_lds(P, ldp, Ig / 16, wave, l16, q);
  float* C = smem + NW * 256;
  core.reduce(smem, C, tid, wave, lane);
  if (tid < 256) {
    const int row = tid >> 4, c = tid & 15;
    const float v = C[row * 16 + c] + d.bh[n0 + c];
    if (row < B) d.hp[(long)t * B * D + (long)row * D + n0 + c] = v;
    const float ss = group_sum<16>(row < B ? v * v : 0.f);
    if (c == 0) w.ssh[tile * MR + row] = ss;
  }
}

// gates = BlockLinear(dyn_gru)(silu(rms(hp))) + bg; deter = GRU(gates, h_in) (rssm.py:65-75); h_in[t+1] masked.
// grid (D/16): workgroup = 16 deter columns of one block, with their r / c / u gate rows (3 tiles).
template <int CPW>
__global__ __launch_bounds__(NTHR) void k_gate(sd_rssm_scan d, Work w, int t) {
  extern __shared__ float smem[];
  SD_THREAD_IDS
  const int B = d.B, D = d.D, Dg = D / d.G, ldp = Dg + 4;
  const int tile = blockIdx.x, n0 = tile * 16, g = n0 / Dg, j0 = n0 % Dg;
  Core<3, CPW> core;
  const float* wg = d.Wg + (long)g * 3 * Dg * Dg;
  const float* wt[3] = {wg + (long)(j0 + l16) * Dg, wg + (long)(Dg + j0 + l16) * Dg, wg + (long)(2 * Dg + j0 + l16) * Dg};
  core.load_b(wt, Dg / 16, wave, q);
  float* P = smem + core_lds_floats<3>();
  {
    const int row = tid >> 5, t32 = tid & 31;
    const float ss = row_partials(w.ssh, D / 16, tid);
    const float r = rsqrtf(ss / (float)D + d.eps);
    const bool rv = row < B;
    if (rv && t32 == 0 && tile == 0) d.rh[(long)t * B + row] = r;
    const float* hrow = d.hp + (long)t * B * D + (long)row * D + (long)g * Dg;
    float* hhrow = d.hh + (long)t * B * D + (long)row * D + (long)g * Dg;
    for (int c = 4 * t32; c < Dg; c += 128) {
      f32x4 y = zero4();
      if (rv) {
        const f32x4 x = ld4(hrow + c), wv = ld4(d.nh + (long)g * Dg + c);
#pragma unroll
        for (int j = 0; j < 4; ++j) y[j] = siluf_(x[j] * r * wv[j]);
        if (j0 == 0) st4(hhrow + c, y);
      }
      st4(P + row * ldp + c, y);
    }
  }
  __syncthreads();
  core.run_lds(P, ldp, Dg / 16, wave, l16, q);
  float* C = smem + NW * 3 * 256;
  core.reduce(smem, C, tid, wave, lane);
  if (tid < 256) {
    const int row = tid >> 4, c = tid & 15;
    if (row < B) {
      const int j = j0 + c, col = n0 + c;
      const float* bg = d.bg + (long)g * 3 * Dg;
      const float ra = C[row * 48 + c] + bg[j];
      const float ca = C[row * 48 + 16 + c] + bg[Dg + j];
      const float ua = C[row * 48 + 32 + c] + bg[2 * Dg + j];
      float* gr = d.gates + (long)t * B * 3 * D + (long)row * 3 * D + (long)g * 3 * Dg;
      gr[j] = ra;
      gr[Dg + j] = ca;
      gr[2 * Dg + j] = ua;
      const float rs = sigmoidf_(ra);
      const float cc = tanhf(rs * ca);
      const float u = sigmoidf_(ua - 1.f);
      const float h = d.h_in[(long)t * B * D + (long)row * D + col];
      const float out = u * cc + (1.f - u) * h;
      d.deter[(long)t * B * D + (long)row * D + col] = out;
      if (t + 1 < d.T) d.h_in[(long)(t + 1) * B * D + (long)row * D + col] = d.reset[(t + 1) * B + row] ? 0.f : out;
    }
  }
}

// logits = obs_net_logit(silu(rms(op))) and the straight-through unimix one-hot sample (rssm.py:172-177,
// distributions.py:16-33); op = sum of the obs_net_0 slabs + (embed half + bias). grid (S): one categorical / WG.
template <int CPW, int KD>
__global__ __launch_bounds__(NTHR) void k_logit(sd_rssm_scan d, Work w, int t) {
  extern __shared__ float smem[];
  SD_THREAD_IDS
  constexpr int NT = KD / 16;
  const int B = d.B, U = d.U, SK = d.SK, S = SK / KD, ldp = U + 4;
  const int s = blockIdx.x, n0 = s * KD;
  Core<NT, CPW> core;
  const float* wt[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) wt[i] = d.Wl + (long)(n0 + 16 * i + l16) * U;
  core.load_b(wt, U / 16, wave, q);
  float* P = smem + core_lds_floats<NT>();
  const long tBU = (long)t * B * U;
  const bool sv = s == 0;
  pro_rms(w.ops, d.ks_d, (long)B * U, nullptr, d.eproj + tBU, U, B, d.no, d.eps, P, ldp, sv ? d.op + tBU : nullptr,
          sv ? d.oo + tBU : nullptr, U, sv ? d.ro + (long)t * B : nullptr, tid);
  __syncthreads();
  core.run_lds(P, ldp, U / 16, wave, l16, q);
  float* C = smem + NW * NT * 256;
  core.reduce(smem, C, tid, wave, lane);
  const uint64_t seed = d.seed + (d.seed_ptr ? *d.seed_ptr : 0ull);
  for (int i = tid; i < MR * KD; i += NTHR) {  // team of KD lanes per (row, categorical)
    const int row = i / KD, lt = i % KD;
    const float l = C[row * KD + lt] + d.bl[n0 + lt];
    float p, pp, nl;
    unimix_forward<KD>(l, true, KD, d.unimix, p, pp, nl);
    const float gn = sd_gumbel(seed, (uint32_t)d.stream_id, (uint32_t)t,
                               (uint64_t)((long)row * S + s + d.group_offset) * KD + lt);
    float ys;
    int idx;
    st_soft<KD>(nl, gn, true, ys, idx, lt);
    if (row < B) {
      const float y = ((lt == idx ? 1.f : 0.f) - ys) + ys;
      const long o = (long)t * B * SK + (long)row * SK + n0 + lt;
      d.logit[o] = l;
      d.stoch[o] = y;
      if (t + 1 < d.T) d.s_in[o + (long)B * SK] = d.reset[(t + 1) * B + row] ? 0.f : y;
    }
  }
}

// ------------------------------------------------------------------------------------------- backward kernels
// dl = d_logit + ST-sampler backward(logit, d_stoch + carry_s) (prologue, noise recomputed);  d_o = dl . Wl.
// grid (U/16)
template <int CPW, int KD>
__global__ __launch_bounds__(NTHR) void k_dlogit(sd_rssm_scan d, Work w, int t) {
  extern __shared__ float smem[];
  SD_THREAD_IDS
  const int B = d.B, U = d.U, SK = d.SK, S = SK / KD, ldp = SK + 4;
  const int n0 = blockIdx.x * 16;
  Core<1, CPW> core;
  const float* wt[1] = {d.WlT + (long)(n0 + l16) * SK};
  core.load_b(wt, SK / 16, wave, q);
  float* P = smem + core_lds_floats<1>();
  const uint64_t seed = d.seed + (d.seed_ptr ? *d.seed_ptr : 0ull);
  const long tBS = (long)t * B * SK;
  for (int i = tid; i < MR * SK; i += NTHR) {
    const int row = i / SK, k = i % SK, lt = k % KD, s = k / KD;
    const bool rv = row < B;
    const long o = tBS + (long)row * SK + k;
    const float l = rv ? d.logit[o] : 0.f;
    float p, pp, nl;
    unimix_forward<KD>(l, true, KD, d.unimix, p, pp, nl);
    const float gn = sd_gumbel(seed, (uint32_t)d.stream_id, (uint32_t)t,
                               (uint64_t)((long)row * S + s + d.group_offset) * KD + lt);
    float ys;
    int idx;
    st_soft<KD>(nl, gn, true, ys, idx, lt);
    const float ds = rv ? (d.d_stoch ? d.d_stoch[o] : 0.f) + w.cs[(long)row * SK + k] : 0.f;
    const float sd = group_sum<KD>(ds * ys);
    const float dlv = unimix_backward<KD>(ys * (ds - sd), p, pp, nl, true, d.unimix);
    const float v = rv ? (d.d_logit ? d.d_logit[o] : 0.f) + dlv : 0.f;
    P[row * ldp + k] = v;
    if (rv && blockIdx.x == 0) d.dl[o] = v;
  }
  __syncthreads();
  core.run_lds(P, ldp, SK / 16, wave, l16, q);
  float* C = smem + NW * 256;
  core.reduce(smem, C, tid, wave, lane);
  if (tid < 256) {
    const int row = tid >> 4, c = tid & 15;
    if (row < B) d.d_o[(long)t * B * U + (long)row * U + n0 + c] = C[row * 16 + c];
  }
}

// d_op = RMSNorm-SiLU backward (prologue); dh = d_deter + carry_h + d_op . Wo[:, :D]; GRU backward (epilogue).
// grid (D/16)
template <int CPW>
__global__ __launch_bounds__(NTHR) void k_dgru(sd_rssm_scan d, Work w, int t) {
  extern __shared__ float smem[];
  SD_THREAD_IDS
  const int B = d.B, U = d.U, D = d.D, Dg = D / d.G, ldp = U + 4;
  const int tile = blockIdx.x, n0 = tile * 16;
  Core<1, CPW> core;
  const float* wt[1] = {d.WoDT + (long)(n0 + l16) * U};
  core.load_b(wt, U / 16, wave, q);
  float* P = smem + core_lds_floats<1>();
  const long tBU = (long)t * B * U;
  pro_rms_bwd(d.op + tBU, d.ro + (long)t * B, d.no, d.d_o + tBU, U, B, P, ldp, tile == 0 ? d.d_op + tBU : nullptr,
              tid);
  __syncthreads();
  core.run_lds(P, ldp, U / 16, wave, l16, q);
  float* C = smem + NW * 256;
  core.reduce(smem, C, tid, wave, lane);
  if (tid < 256) {
    const int row = tid >> 4, c = tid & 15;
    if (row < B) {
      const int col = n0 + c, g = col / Dg, j = col % Dg;
      const long od = (long)t * B * D + (long)row * D + col;
      const float dh = (d.d_deter ? d.d_deter[od] : 0.f) + w.ch[(long)row * D + col] + C[row * 16 + c];
      const long gb = (long)t * B * 3 * D + (long)row * 3 * D + (long)g * 3 * Dg;
      const float ra = d.gates[gb + j], ca = d.gates[gb + Dg + j], ua = d.gates[gb + 2 * Dg + j];
      const float rs = sigmoidf_(ra);
      const float cc = tanhf(rs * ca);
      const float u = sigmoidf_(ua - 1.f);
      const float hv = d.h_in[od];
      const float dtc = dh * u * (1.f - cc * cc);
      d.d_gates[gb + j] = dtc * ca * rs * (1.f - rs);
      d.d_gates[gb + Dg + j] = dtc * rs;
      d.d_gates[gb + 2 * Dg + j] = dh * (cc - hv) * u * (1.f - u);
      w.dhin[(long)row * D + col] = dh * (1.f - u);
    }
  }
}

// d_hh = d_gates_g . Wg[g] (block GEMM); epilogue: RMSNorm-SiLU backward pieces of dyn_hid's norm (g*w and the
// per-tile row partials of sum g*xhat). grid (D/16)
template <int CPW>
__global__ __launch_bounds__(NTHR) void k_dhh(sd_rssm_scan d, Work w, int t) {
  extern __shared__ float smem[];
  SD_THREAD_IDS
  const int B = d.B, D = d.D, Dg = D / d.G;
  const int tile = blockIdx.x, n0 = tile * 16, g = n0 / Dg, j0 = n0 % Dg;
  Core<1, CPW> core;
  const float* wt[1] = {d.WgT + ((long)g * Dg + j0 + l16) * 3 * Dg};
  core.load_b(wt, 3 * Dg / 16, wave, q);
  core.run_glb(d.d_gates + (long)t * B * 3 * D + (long)g * 3 * Dg, 3 * (long)D, B, 3 * Dg / 16, wave, l16, q);
  float* C = smem + NW * 256;
  core.reduce(smem, C, tid, wave, lane);
  if (tid < 256) {
    const int row = tid >> 4, c = tid & 15, col = n0 + c;
    float part = 0.f;
    if (row < B) {
      const float dy = C[row * 16 + c];
      const long o = (long)t * B * D + (long)row * D + col;
      d.d_hh[o] = dy;
      const float xh = d.hp[o] * d.rh[(long)t * B + row], wv = d.nh[col];
      const float gq = dy * dsilu(xh * wv) * wv;
      w.gq[(long)row * D + col] = gq;
      part = gq * xh;
    }
    part = group_sum<16>(part);
    if (c == 0) w.dotp[tile * MR + row] = part;
  }
}

// d_hp_g = RMSNorm backward (prologue, from g*w and the row partials); then two problems in one grid:
//   P0: d_xcat slab g = d_hp_g . Wsh[g-rows]   ((3U/16) * G workgroups)
//   P1: d_hin[:, g] += d_hp_g . Wbd[g]          (D/16 workgroups)
template <int CPW>
__global__ __launch_bounds__(NTHR) void k_dhp(sd_rssm_scan d, Work w, int t) {
  extern __shared__ float smem[];
  SD_THREAD_IDS
  const int B = d.B, U = d.U, D = d.D, Dg = D / d.G, ldp = Dg + 4, X = 3 * U;
  const int NX = (X / 16) * d.G;
  const int blk = blockIdx.x;
  const bool p0 = blk < NX;
  int g, n0;
  const float* wrow;
  if (p0) {
    g = blk / (X / 16);
    n0 = (blk % (X / 16)) * 16;
    wrow = d.WshT + (long)(n0 + l16) * D + (long)g * Dg;
  } else {
    n0 = (blk - NX) * 16;
    g = n0 / Dg;
    wrow = d.WbdT + ((long)g * Dg + n0 % Dg + l16) * Dg;
  }
  Core<1, CPW> core;
  const float* wt[1] = {wrow};
  core.load_b(wt, Dg / 16, wave, q);
  float* P = smem + core_lds_floats<1>();
  {
    const int row = tid >> 5, t32 = tid & 31;
    const float dot = row_partials(w.dotp, D / 16, tid) / (float)D;
    const bool rv = row < B;
    const float r = rv ? d.rh[(long)t * B + row] : 0.f;
    const bool save = !p0 && (n0 % Dg) == 0;
    for (int c = 4 * t32; c < Dg; c += 128) {
      f32x4 o = zero4();
      if (rv) {
        const long ob = (long)row * D + (long)g * Dg + c;
        const f32x4 gq = ld4(w.gq + ob), x = ld4(d.hp + (long)t * B * D + ob);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = r * (gq[j] - x[j] * r * dot);
        if (save) st4(d.d_hp + (long)t * B * D + ob, o);
      }
      st4(P + row * ldp + c, o);
    }
  }
  __syncthreads();
  core.run_lds(P, ldp, Dg / 16, wave, l16, q);
  float* C = smem + NW * 256;
  core.reduce(smem, C, tid, wave, lane);
  if (tid < 256) {
    const int row = tid >> 4, c = tid & 15;
    if (row < B) {
      if (p0) w.dxs[(long)g * B * X + (long)row * X + n0 + c] = C[row * 16 + c];
      else w.dhin[(long)row * D + n0 + c] += C[row * 16 + c];
    }
  }
}

// d_xcat = sum over blocks of the slabs; d_x0p / d_x1p = RMSNorm-SiLU backward of the _dyn_in0 / _dyn_in1 norms.
// grid (B): one workgroup per row; waves 0-3 take x0, waves 4-7 x1.
__global__ __launch_bounds__(NTHR) void k_dx01(sd_rssm_scan d, Work w, int t) {
  __shared__ float red[NW];
  extern __shared__ float smem[];
  const int tid = threadIdx.x, wave = tid >> 6;
  const int B = d.B, U = d.U, X = 3 * U, b = blockIdx.x;
  const long tB = (long)t * B;
  float* dx = smem;
  for (int c = tid; c < X; c += NTHR) {
    float v = 0.f;
    for (int g = 0; g < d.G; ++g) v += w.dxs[(long)g * B * X + (long)b * X + c];
    dx[c] = v;
    d.d_xcat[(tB + b) * X + c] = v;
  }
  __syncthreads();
  const int half = wave >> 2, ht = tid & 255;
  const float* x = (half ? d.x1p : d.x0p) + (tB + b) * U;
  const float* wn = half ? d.n1 : d.n0;
  const float r = (half ? d.r1 : d.r0)[tB + b];
  float* out = (half ? d.d_x1p : d.d_x0p) + (tB + b) * U;
  float dot = 0.f;
  for (int c = ht; c < U; c += 256) {
    const float xh = x[c] * r, wv = wn[c];
    const float gg = dx[half * U + c] * dsilu(xh * wv) * wv;
    dx[X + half * U + c] = gg;
    dot += gg * xh;
  }
  dot = wave_sum(dot);
  if ((tid & 63) == 0) red[wave] = dot;
  __syncthreads();
  dot = (red[4 * half] + red[4 * half + 1] + red[4 * half + 2] + red[4 * half + 3]) / (float)U;
  for (int c = ht; c < U; c += 256) out[c] = r * (dx[X + half * U + c] - x[c] * r * dot);
}

// carry_h = mask(d_hin + d_x0p . W0), carry_s = mask(d_x1p . W1) for step t-1 (rssm.py:161-165 backward).
// grid (D/16 + SK/16)
template <int CPW>
__global__ __launch_bounds__(NTHR) void k_carry(sd_rssm_scan d, Work w, int t) {
  extern __shared__ float smem[];
  SD_THREAD_IDS
  const int B = d.B, U = d.U, D = d.D, SK = d.SK;
  const bool p0 = (int)blockIdx.x < D / 16;
  const int n0 = p0 ? blockIdx.x * 16 : (blockIdx.x - D / 16) * 16;
  Core<1, CPW> core;
  const float* wt[1] = {(p0 ? d.W0T : d.W1T) + (long)(n0 + l16) * U};
  core.load_b(wt, U / 16, wave, q);
  core.run_glb((p0 ? d.d_x0p : d.d_x1p) + (long)t * B * U, U, B, U / 16, wave, l16, q);
  float* C = smem + NW * 256;
  core.reduce(smem, C, tid, wave, lane);
  if (tid < 256) {
    const int row = tid >> 4, c = tid & 15;
    if (row < B) {
      const bool rs = d.reset[t * B + row] != 0;
      if (p0) {
        const long o = (long)row * D + n0 + c;
        w.ch[o] = rs ? 0.f : w.dhin[o] + C[row * 16 + c];
      } else {
        w.cs[(long)row * SK + n0 + c] = rs ? 0.f : C[row * 16 + c];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------- host side
int cpw_for(int k) {  // chunks per wave for a k span (16-deep chunks over 8 waves), rounded to an instantiation
  const int c = (k / 16 + NW - 1) / NW;
  return c <= 2 ? 2 : c <= 4 ? 4 : c <= 8 ? 8 : c <= 12 ? 12 : c <= 16 ? 16 : -1;
}

#define SD_CPW_SWITCH(cpw, ...)                            \
  switch (cpw) {                                           \
    case 2: { constexpr int CP = 2; __VA_ARGS__; } break;  \
    case 4: { constexpr int CP = 4; __VA_ARGS__; } break;  \
    case 8: { constexpr int CP = 8; __VA_ARGS__; } break;  \
    case 12: { constexpr int CP = 12; __VA_ARGS__; } break; \
    case 16: { constexpr int CP = 16; __VA_ARGS__; } break; \
    default: return SD_ESHAPE;                             \
  }

#define SD_KD_SWITCH(kd, ...)                              \
  switch (kd) {                                            \
    case 16: { constexpr int KD = 16; __VA_ARGS__; } break; \
    case 32: { constexpr int KD = 32; __VA_ARGS__; } break; \
    case 64: { constexpr int KD = 64; __VA_ARGS__; } break; \
    default: return SD_ESHAPE;                             \
  }

// dynamic LDS above 64 KB needs the per-function limit raised; done once per instantiation (the first call runs
// eagerly, before any graph capture)
template <auto KERN>
bool raise_lds(size_t bytes) {
  static size_t done = 65536;
  if (bytes <= done) return true;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(KERN), hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)bytes) != hipSuccess)
    return false;
  done = bytes;
  return true;
}

int check(const sd_rssm_scan* d) {
  if (!d) return SD_EARG;
  if (d->B < 1 || d->B > MR || d->T < 1 || d->G < 1 || d->D % d->G) return SD_ESHAPE;
  const int Dg = d->D / d->G;
  if (d->U % 64 || Dg % 64 || d->SK % 64 || d->D % 64) return SD_ESHAPE;
  if (d->Kd != 16 && d->Kd != 32 && d->Kd != 64) return SD_ESHAPE;
  if (d->SK % d->Kd) return SD_ESHAPE;
  if (d->ks_d < 1 || d->ks_s < 1 || d->D % (d->ks_d * 16) || d->SK % (d->ks_s * 16)) return SD_ESHAPE;
  if (!d->work) return SD_EARG;
  return SD_OK;
}

}  // namespace

extern "C" int sd_rssm_scan_work_floats(const sd_rssm_scan* d) {
  if (!d) return SD_EARG;
  return (int)work_layout(*d, nullptr).total;
}

extern "C" int sd_rssm_scan_fwd(const sd_rssm_scan* dp, sd_stream stream_) {
  int rc = check(dp);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream_;
  const sd_rssm_scan& d = *dp;
  const Work w = work_layout(d, d.work);
  const int B = d.B, U = d.U, D = d.D, SK = d.SK, Dg = D / d.G, Ig = Dg + 3 * U;
  const int span_d = D / d.ks_d, span_s = SK / d.ks_s;
  const int cp_d = cpw_for(span_d), cp_s = cpw_for(span_s), cp_h = cpw_for(Ig), cp_g = cpw_for(Dg),
            cp_u = cpw_for(U);
  if (cp_d < 0 || cp_s < 0 || cp_h < 0 || cp_g < 0 || cp_u < 0) return SD_ESHAPE;
  const size_t core1 = core_lds_floats<1>() * 4;
  const size_t lds_hid = core1 + (size_t)MR * (Ig + 4) * 4;
  const size_t lds_gate = core_lds_floats<3>() * 4 + (size_t)MR * (Dg + 4) * 4;
  const long BD = (long)B * D, BS = (long)B * SK, BU = (long)B * U;

  k_init<<<64, 256, 0, st>>>(d);
  SD_LAUNCH_CHECK();
  {  // x0p(0) = h_in[0] . W0^T
    SlabProb p{d.h_in, D, d.W0, D, w.x0s, nullptr};
    SD_CPW_SWITCH(cp_d, k_slab<CP><<<dim3(U / 16, d.ks_d, 1), NTHR, core1, st>>>(p, p, B, U, span_d));
    SD_LAUNCH_CHECK();
  }
  for (int t = 0; t < d.T; ++t) {
    {
      SlabProb p{d.s_in + t * BS, SK, d.W1, SK, w.x1s, nullptr};
      SD_CPW_SWITCH(cp_s, k_slab<CP><<<dim3(U / 16, d.ks_s, 1), NTHR, core1, st>>>(p, p, B, U, span_s));
      SD_LAUNCH_CHECK();
    }
    SD_CPW_SWITCH(cp_h, if (!raise_lds<k_hid<CP>>(lds_hid)) return SD_EARG;
                  k_hid<CP><<<D / 16, NTHR, lds_hid, st>>>(d, w, t));
    SD_LAUNCH_CHECK();
    SD_CPW_SWITCH(cp_g, if (!raise_lds<k_gate<CP>>(lds_gate)) return SD_EARG;
                  k_gate<CP><<<D / 16, NTHR, lds_gate, st>>>(d, w, t));
    SD_LAUNCH_CHECK();
    {
      SlabProb po{d.deter + t * BD, D, d.WoD, D, w.ops, nullptr};
      SlabProb px{d.deter + t * BD, D, d.W0, D, w.x0s, d.reset + (t + 1) * B};
      const int np = t + 1 < d.T ? 2 : 1;
      SD_CPW_SWITCH(cp_d, k_slab<CP><<<dim3(U / 16, d.ks_d, np), NTHR, core1, st>>>(po, px, B, U, span_d));
      SD_LAUNCH_CHECK();
    }
    SD_KD_SWITCH(d.Kd, {
      constexpr int NT = KD / 16;
      const size_t lds = core_lds_floats<NT>() * 4 + (size_t)MR * (U + 4) * 4;
      SD_CPW_SWITCH(cp_u, if (!(raise_lds<k_logit<CP, KD>>(lds))) return SD_EARG;
                    k_logit<CP, KD><<<SK / KD, NTHR, lds, st>>>(d, w, t));
    });
    SD_LAUNCH_CHECK();
  }
  (void)BU;
  return SD_OK;
}

extern "C" int sd_rssm_scan_bwd(const sd_rssm_scan* dp, sd_stream stream_) {
  int rc = check(dp);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream_;
  const sd_rssm_scan& d = *dp;
  const Work w = work_layout(d, d.work);
  const int B = d.B, U = d.U, D = d.D, SK = d.SK, Dg = D / d.G;
  const int cp_sk = cpw_for(SK), cp_u = cpw_for(U), cp_g3 = cpw_for(3 * Dg), cp_g = cpw_for(Dg);
  if (cp_sk < 0 || cp_u < 0 || cp_g3 < 0 || cp_g < 0) return SD_ESHAPE;
  const size_t core1 = core_lds_floats<1>() * 4;
  const size_t lds_dl = core1 + (size_t)MR * (SK + 4) * 4;
  const size_t lds_dgru = core1 + (size_t)MR * (U + 4) * 4;
  const size_t lds_dhp = core1 + (size_t)MR * (Dg + 4) * 4;
  const size_t lds_dx = (size_t)(3 * U + 2 * U) * 4;
  hipError_t e = hipMemsetAsync(w.cs, 0, sizeof(float) * (size_t)B * SK, st);
  if (e != hipSuccess) return (int)e;
  e = hipMemsetAsync(w.ch, 0, sizeof(float) * (size_t)B * D, st);
  if (e != hipSuccess) return (int)e;
  const int NX = (3 * U / 16) * d.G;
  for (int t = d.T - 1; t >= 0; --t) {
    SD_KD_SWITCH(d.Kd, SD_CPW_SWITCH(cp_sk, if (!(raise_lds<k_dlogit<CP, KD>>(lds_dl))) return SD_EARG;
                                     k_dlogit<CP, KD><<<U / 16, NTHR, lds_dl, st>>>(d, w, t)));
    SD_LAUNCH_CHECK();
    SD_CPW_SWITCH(cp_u, k_dgru<CP><<<D / 16, NTHR, lds_dgru, st>>>(d, w, t));
    SD_LAUNCH_CHECK();
    SD_CPW_SWITCH(cp_g3, k_dhh<CP><<<D / 16, NTHR, core1, st>>>(d, w, t));
    SD_LAUNCH_CHECK();
    SD_CPW_SWITCH(cp_g, if (!raise_lds<k_dhp<CP>>(lds_dhp)) return SD_EARG;
                  k_dhp<CP><<<NX + D / 16, NTHR, lds_dhp, st>>>(d, w, t));
    SD_LAUNCH_CHECK();
    k_dx01<<<B, NTHR, lds_dx, st>>>(d, w, t);
    SD_LAUNCH_CHECK();
    if (t > 0) {
      SD_CPW_SWITCH(cp_u, k_carry<CP><<<D / 16 + SK / 16, NTHR, core1, st>>>(d, w, t));
      SD_LAUNCH_CHECK();
    }
  }
  return SD_OK;
}
