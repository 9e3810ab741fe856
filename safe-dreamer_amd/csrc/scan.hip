// Fused RSSM posterior scan: RSSM.observe (rssm.py:140-156) -> obs_step (rssm.py:158-178) -> Deter.forward
// (rssm.py:36-75), forward and BPTT backward; B <= 4096 rows per step as ceil(B / row_tile) row tiles of <= 16 rows
// side by side in each launch's grid (grid z).
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
// acc[t] += A[0:16, span] . W_t[n_t + 0:16, span]^T.  Wave w owns 16-deep k chunks; lane group q = lane>>4 supplies
// k = 16c + 4q .. +3 as one float4 and the MFMA consumes them in 4 steps (a permuted but consistent k order).
// SD_CORE_PAIR: a wave's chunks come in adjacent pairs (2w, 2w + 1, 2w + 16, 2w + 17, ...), so the two loads it issues
// back to back for a row cover one whole 128-B line (with single chunks c = w, w + 8, ... each 128-B line of a weight
// row was split between two waves' loads, issued at different times).
#ifndef SD_CORE_PAIR
#define SD_CORE_PAIR 1
#endif
SD_DEV int core_chunk(int wave, int c) {
  return SD_CORE_PAIR ? 2 * (wave + NW * (c >> 1)) + (c & 1) : wave + NW * c;
}
template <int NT, int CPW>
struct Core {
  static_assert(!SD_CORE_PAIR || CPW % 2 == 0, "chunk pairs");
  f32x4 b[CPW][NT];
  f32x4 acc[NT];

  // Wt[t]: row (n_t + l16) of a k-contiguous weight matrix, at the span's first k (a valid row for EVERY lane: the
  // extra lanes of an 8-column tile point at a real row, their output columns are discarded). Chunks past nch load
  // chunk nch - 1 and are never multiplied: every load is unconditional (no branch around it, so hipcc has no join at
  // which to drain the queue — see "load helpers" below).
  SD_DEV void load_b(const float* const* Wt, int nch, int wave, int q) {
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
      const int ch = core_chunk(wave, c), chc = ch < nch ? ch : nch - 1;
#pragma unroll
      for (int t = 0; t < NT; ++t) b[c][t] = ld4(Wt[t] + chc * 16 + 4 * q);
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
      const int ch = core_chunk(wave, c);
      if (ch < nch) mma(ld4(P + l16 * lda + ch * 16 + 4 * q), c);
    }
  }
  // A straight from global memory; rows >= M read row M - 1 (their output rows are discarded by the callers), all
  // loads issued before the first MFMA
  SD_DEV void run_glb(const float* A, long lda, int M, int nch, int wave, int l16, int q) {
    f32x4 a[CPW];
    const int lr = l16 < M ? l16 : M - 1;
#pragma unroll
    for (int c = 0; c < CPW; ++c) {
      const int ch = core_chunk(wave, c), chc = ch < nch ? ch : nch - 1;
      a[c] = ld4(A + (long)lr * lda + chc * 16 + 4 * q);
    }
#pragma unroll
    for (int c = 0; c < CPW; ++c)
      if (core_chunk(wave, c) < nch) mma(a[c], c);
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

// row tile of a workgroup (grid z): batch rows rb .. rb + nr (d.row_tile rows, normalised on the host)
#define SD_ROW_TILE                                               \
  const int rb = (int)blockIdx.z * d.row_tile, nr = min(d.row_tile, d.B - rb); \
  (void)rb; (void)nr;

#define SD_THREAD_IDS                                      \
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6; \
  const int l16 = lane & 15, q = lane >> 4;                \
  (void)l16; (void)q;

// XCD-contiguous tiles: the dispatcher deals workgroup i to XCD i % 8, so tile (i % 8) * (n / 8) + i / 8 gives XCD x
// the n / 8 consecutive column tiles [x n / 8, (x + 1) n / 8) (with 16-column tiles over D = 2048: exactly block x).
// Each XCD then writes whole 128-B lines of every output row (two or four neighbouring tiles share a line), and the
// lines left dirty at the launch's end are not split between XCDs. Speed only: any tile order gives the same result.
#ifndef SD_SCAN_XCD
#define SD_SCAN_XCD 1
#endif
SD_DEV int xcd_tile(int i, int n) { return (SD_SCAN_XCD && n % 8 == 0) ? (i % 8) * (n / 8) + i / 8 : i; }

// ------------------------------------------------------------------------------------------- load helpers
// Prologues use 32 threads per row (16 rows): thread t32 owns the float4 columns c = 4*t32 + 128*i. Every load a
// launch needs is issued before the first use, and every load is UNCONDITIONAL: rows past the tile read a valid row
// (the callers clamp the row index; those rows' results are discarded), slabs past ks read slab ks - 1 (masked when
// summed). A predicated "cond ? load : 0" made hipcc branch around each load and drain the whole vector-memory queue
// (s_waitcnt vmcnt(0)) at the join, so the weight stream issued first and the prologue loads behind it became two
// dependent round trips (round 5: tools/isa_waits.py listed such drains in every scan kernel).
// Rows are exactly 128 * NI floats wide (every caller's width: U = 256, D/G, S*Kd are multiples of 128).
template <int NI>
SD_DEV void ld_row(f32x4 (&v)[NI], const float* rowp, int t32) {
#pragma unroll
  for (int i = 0; i < NI; ++i) v[i] = ld4(rowp + 4 * t32 + 128 * i);
}
// KS <= slab loads of ks split-K slabs (sum_slabs adds the first ks in fixed order, after the launch's other loads)
template <int NI, int KS>
SD_DEV void ld_slabs(f32x4 (&part)[KS][NI], const float* rowp, long sstride, int ks, int t32) {
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int sc = s < ks ? s : ks - 1;
#pragma unroll
    for (int i = 0; i < NI; ++i) part[s][i] = ld4(rowp + sc * sstride + 4 * t32 + 128 * i);
  }
}
template <int NI, int KS>
SD_DEV void sum_slabs(f32x4 (&v)[NI], const f32x4 (&part)[KS][NI], int ks) {
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    v[i] = part[0][i];
#pragma unroll
    for (int s = 1; s < KS; ++s)
      if (s < ks) v[i] += part[s][i];
  }
}
// per-tile row partials, row-major: part[row * tiles + i], i < tiles <= 128*NP (tiles % 4 == 0): a row's partials
// are one contiguous run, read as float4s by the row's 32 threads (the column-major layout cost 64 cache lines per
// wave instruction); entries past `tiles` re-read the last float4 and are masked in sum_parts
template <int NP>
SD_DEV void ld_parts(f32x4 (&v)[NP], const float* rowp, int tiles, int t32) {
#pragma unroll
  for (int j = 0; j < NP; ++j) {
    const int i = 4 * (t32 + 32 * j);
    v[j] = *reinterpret_cast<const f32x4*>(rowp + (i < tiles ? i : tiles - 4));
  }
}
template <int NP>
SD_DEV float sum_parts(const f32x4 (&v)[NP], int tiles, int t32) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NP; ++j)
    if (4 * (t32 + 32 * j) < tiles) s += (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
  return group_sum<32>(s);
}
SD_DEV float sumsq4(f32x4 x) { return x[0] * x[0] + x[1] * x[1] + x[2] * x[2] + x[3] * x[3]; }

// y = silu(x * r * w) (rows >= M -> 0), x already holds the row (incl. bias)
template <int NI>
SD_DEV float rms_silu_rows(f32x4 (&x)[NI], const f32x4 (&w)[NI], int N, float eps, bool rv, f32x4 (&y)[NI]) {
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NI; ++i) ss += sumsq4(x[i]);
  ss = group_sum<32>(ss);
  const float r = rsqrtf(ss / (float)N + eps);
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) y[i][j] = rv ? siluf_(x[i][j] * r * w[i][j]) : 0.f;
  return r;
}

template <int NI>
SD_DEV void st_row(float* rowp, const f32x4 (&v)[NI], int N, int t32) {
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int c = 4 * t32 + 128 * i;
    if (c < N) st4(rowp + c, v[i]);
  }
}

constexpr int KSM = 8;         // max split-K slabs (ks_d, ks_s)
#ifndef SD_LR_NG
#define SD_LR_NG 8  // 4: 12.03 / 12.01 ms, 8: 11.98 / 11.95 ms per update (same box, profiles/r03ng_env.txt); again
                    // on round-5 code, 4: 11.01 vs 8: 10.88 ms (k_logit_rows 6.2 -> 8.2 us, k_hid 6.9 -> 6.7, r05ng)
#endif
constexpr int LR_NG = SD_LR_NG;                 // x1p slabs written by k_logit_rows (categorical groups per row)
constexpr int KS1 = LR_NG > KSM ? LR_NG : KSM;  // max x1p slabs k_hid sums
constexpr int lr_cpg(int SK, int KD) { return SK / (LR_NG * KD) > 0 ? SK / (LR_NG * KD) : 1; }
// output columns per workgroup of k_hid / k_gate: 16, or 8 (twice the workgroups, half the weight rows each; the
// 16-wide MFMA tile then carries 8 zero weight rows in k_hid, and r|c + u|0 gate rows in k_gate)
#ifndef SD_SCAN_HCW
#define SD_SCAN_HCW 16
#endif
#ifndef SD_SCAN_GCW
#define SD_SCAN_GCW 8
#endif
// output columns per workgroup of k_dlogit / k_dgru / k_dhh (16 or 8)
#ifndef SD_SCAN_DLCW
#define SD_SCAN_DLCW 16
#endif
#ifndef SD_SCAN_DGCW
#define SD_SCAN_DGCW 16
#endif
#ifndef SD_SCAN_DHCW
#define SD_SCAN_DHCW 16
#endif
// ------------------------------------------------------------------------------------------- scratch layout
struct Work {
  float *x0s, *x1s, *ops, *ssh, *dotp, *dxs, *dhin, *gq, *ch, *w1t;
  long total;
};
long al64(long n) { return (n + 63) / 64 * 64; }
int row_tile_of(const sd_rssm_scan& d) { return d.row_tile > 0 ? d.row_tile : MR; }
int row_tiles(const sd_rssm_scan& d) { return (d.B + row_tile_of(d) - 1) / row_tile_of(d); }
Work work_layout(const sd_rssm_scan& d, float* base) {
  Work w;
  long o = 0;
  const long NT = row_tiles(d);
  const long BU = (long)d.B * d.U;
  auto take = [&](long n) { float* p = base ? base + o : nullptr; o += al64(n); return p; };
  w.x0s = take(d.ks_d * BU);
  w.x1s = take((long)KS1 * BU);  // ks_s slabs, or k_logit_rows' LR_NG
  w.ops = take(d.ks_d * BU);
  w.ssh = take(NT * MR * (d.D / 8));  // per row tile: 16 rows x (D/16 or D/8 column tiles) partials
  w.dotp = take(NT * MR * (d.D / 8));  // per row tile: 16 rows x (D/16 or D/8 column tiles) partials
  w.dxs = take((long)d.G * d.B * 3 * d.U);
  w.dhin = take((long)d.B * d.D);
  w.gq = take((long)d.B * d.D);
  w.ch = take((long)d.B * d.D);
  w.w1t = take((long)d.SK * d.U);  // _dyn_in1's weight transposed (SK, U): k_logit_rows' gather rows
  w.total = o;
  return w;
}

constexpr int UH = 256;        // hidden width of the fused path (base.yaml: hidden 256)
constexpr int NU = UH / 128;   // float4 columns per prologue thread over a hidden row

// ------------------------------------------------------------------------------------------- forward kernels
// reset flag of (step t, batch row b): (T, B) time-major, or (B, T) batch-major when d.reset_bm (read in place)
SD_DEV bool reset_at(const sd_rssm_scan& d, int t, int b) {
  return d.reset[d.reset_bm ? (long)b * d.T + t : (long)t * d.B + b] != 0;
}
// the raw flag byte of (min(t, T - 1), b), for an unconditional load whose value is only tested later
SD_DEV unsigned char reset_byte(const sd_rssm_scan& d, int t, int b) {
  const int tc = t < d.T ? t : d.T - 1;
  return d.reset[d.reset_bm ? (long)b * d.T + tc : (long)tc * d.B + b];
}

struct SlabProb {
  const float* A;
  long lda;
  const float* W;
  long ldw;
  float* out;                 // slab s at out + s*M*N
  const unsigned char* mask;  // reset flags (a valid pointer even when unused); row r at mask[r * mstride]
  uint64_t* trace;            // SD_SCAN_TRACE builds: phase timestamps (sd_rssm_scan.trace), slot below
  int slot;
  int mstride;
  int use_mask;               // 1: rows whose flag is set are forced to 0 (their input was reset)
};

// row-tiled GEMM into split-K slabs: out[s][m][n] = A[m, span_s] . W[n, span_s]; grid (N/16, ks * row tiles, nprob)
// (blockIdx.y = s + ks * row tile: the row tiles of one column tile stay 16 * ks blocks apart, i.e. on one XCD)
template <int CPW>
__global__ __launch_bounds__(NTHR) void k_slab(SlabProb p0, SlabProb p1, int M, int N, int span, int ks, int rt) {
  extern __shared__ float smem[];
  SD_THREAD_IDS
  SD_TR_BEGIN
  const SlabProb p = blockIdx.z ? p1 : p0;
  const int s = (int)blockIdx.y % ks, rb = ((int)blockIdx.y / ks) * rt, nr = min(rt, M - rb);
  const int n0 = xcd_tile(blockIdx.x, gridDim.x) * 16, kb = s * span, nch = span / 16;
  Core<1, CPW> core;
  const float* wt[1] = {p.W + (long)(n0 + l16) * p.ldw + kb};
  core.load_b(wt, nch, wave, q);
  const int erow = tid >> 4;
  const unsigned char mflag = p.mask[(long)(rb + (erow < nr ? erow : nr - 1)) * p.mstride];  // read unconditionally
  core.run_glb(p.A + (long)rb * p.lda + kb, p.lda, nr, nch, wave, l16, q);
  const bool masked = p.use_mask && mflag;
  SD_TR(1)
  float* C = smem + NW * 256;
  core.reduce(smem, C, tid, wave, lane);
  SD_TR(2)
  if (tid < 256 && erow < nr) {
    const int c = tid & 15;
    p.out[(long)s * M * N + (long)(rb + erow) * N + n0 + c] = masked ? 0.f : C[erow * 16 + c];
  }
  SD_TR_END(p.trace, p.slot)
}

// s_in[0] = mask(stoch0), h_in[0] = mask(deter0)   (rssm.py:161-165 on the initial state)
__global__ void k_zero(float* p, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0.f;
}

// (and w1t = W1^T for k_logit_rows)
__global__ void k_init(sd_rssm_scan d, float* w1t) {
  const long nS = (long)d.B * d.SK, nD = (long)d.B * d.D, nW = w1t ? (long)d.SK * d.U : 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nW; i += (long)gridDim.x * blockDim.x) {
    const long k = i / d.U, c = i % d.U;  // w1t[k][c] = W1[c][k]
    w1t[i] = d.W1[c * d.SK + k];
  }
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nS + nD; i += (long)gridDim.x * blockDim.x) {
    if (i < nS) {
      const int row = (int)(i / d.SK);
      d.s_in[i] = reset_at(d, 0, row) ? 0.f : d.stoch0[i];
    } else {
      const long j = i - nS;
      const int row = (int)(j / d.D);
      d.h_in[j] = reset_at(d, 0, row) ? 0.f : d.deter0[j];
    }
  }
}

// hp[t] = BlockLinear(dyn_hid_0)([h_g | x0 | x1 | x2]) + bh, with x0 = silu(rms(x0p)), x1 = silu(rms(x1p)) built
// in the prologue (rssm.py:52-63). grid (D/16); also the per-tile row sums of hp^2 for the next norm.
// row (t, b) of the hoisted per-step inputs x2 / eproj: time-major (T, B, U), or batch-major (B, T, U) when
// d.bm_inputs (computed on the batch-major rows, no transpose)
SD_DEV long in_row(const sd_rssm_scan& d, int t, int b) {
  return d.bm_inputs ? (long)b * d.T + t : (long)t * d.B + b;
}

// X0F: x0 = silu(rms(x0p)) was formed by the previous step's k_logit_rows (written into xcat), read as it stands;
// otherwise (t = 0, or the k_logit path) summed from the split-K slabs and normalised here. CW: output columns per
// workgroup (16 or 8; grid D / CW), the row partials of hp^2 then come per CW-column tile.
template <int CPW, int NG, bool X0F, int CW>
__global__ __launch_bounds__(NTHR) void k_hid(sd_rssm_scan d, Work w, int t) {
  extern __shared__ float smem[];
  SD_TR_BEGIN
  SD_THREAD_IDS
  SD_ROW_TILE
  const int B = d.B, D = d.D, Dg = D / d.G, Ig = Dg + 3 * UH, ldp = Ig + 4;
  const int tile = xcd_tile(blockIdx.x, gridDim.x), n0 = tile * CW, g = n0 / Dg;
  Core<1, CPW> core;
  const float* wt[1] = {d.Wh + (long)(n0 + (l16 & (CW - 1))) * Ig};  // CW 8: lanes 8..15 repeat rows (discarded)
  core.load_b(wt, Ig / 16, wave, q);
  const int row = tid >> 5, t32 = tid & 31, gr = rb + row;
  const bool rv = row < nr;
  const int grc = rv ? gr : rb + nr - 1;  // rows past the tile read the tile's last row (results discarded)
  const long tBU = (long)t * B * UH;
  f32x4 h[NG], x0[NU], x1[NU], x2v[NU], b0v[NU], b1v[NU], n0v[NU], n1v[NU];
#ifndef SD_SCAN_PROBE_SLABS  // timing probe only (wrong results): k_hid reads / sums one x1p slab instead of ks_s
#define SD_SCAN_PROBE_SLABS 0
#endif
  constexpr int KX1 = SD_SCAN_PROBE_SLABS ? 1 : KS1;
  const int ks1 = SD_SCAN_PROBE_SLABS ? 1 : d.ks_s;
  f32x4 x0p[X0F ? 1 : KSM][NU], x1p[KX1][NU];
  ld_row(h, d.h_in + (long)t * B * D + (long)grc * D + (long)g * Dg, t32);
  if constexpr (X0F) {
    ld_row(x0, d.xcat + 3 * tBU + (long)grc * 3 * UH, t32);
  } else {
    ld_slabs<NU, KSM>(x0p, w.x0s + (long)grc * UH, (long)B * UH, d.ks_d, t32);
    ld_row(b0v, d.b0, t32);
    ld_row(n0v, d.n0, t32);
  }
  ld_slabs<NU, KX1>(x1p, w.x1s + (long)grc * UH, (long)B * UH, ks1, t32);
  ld_row(b1v, d.b1, t32);
  ld_row(n1v, d.n1, t32);
  ld_row(x2v, d.x2 + in_row(d, t, grc) * UH, t32);
  const int ec = tid & 15;
  const float bhv = d.bh[n0 + (ec & (CW - 1))];
  // every load is in flight: now the prologue arithmetic
  f32x4 y0[NU], y1[NU];
  float r0 = 0.f;
  if constexpr (X0F) {
#pragma unroll
    for (int i = 0; i < NU; ++i) y0[i] = x0[i];
  } else {
    sum_slabs(x0, x0p, d.ks_d);
#pragma unroll
    for (int i = 0; i < NU; ++i) x0[i] += b0v[i];
    r0 = rms_silu_rows(x0, n0v, UH, d.eps, rv, y0);
  }
  sum_slabs(x1, x1p, ks1);
#pragma unroll
  for (int i = 0; i < NU; ++i) x1[i] += b1v[i];
  const float r1 = rms_silu_rows(x1, n1v, UH, d.eps, rv, y1);
  float* P = smem + core_lds_floats<1>() + row * ldp;
  st_row(P, h, Dg, t32);
  st_row(P + Dg, y0, UH, t32);
  st_row(P + Dg + UH, y1, UH, t32);
  st_row(P + Dg + 2 * UH, x2v, UH, t32);
  if (rv && tile < 3) {
    float* xc = d.xcat + 3 * tBU + (long)gr * 3 * UH;
    if (tile == 0) {
      if (!X0F) {  // (X0F: written by the previous step's k_logit_rows)
        st_row(d.x0p + tBU + (long)gr * UH, x0, UH, t32);
        st_row(xc, y0, UH, t32);
        if (t32 == 0) d.r0[(long)t * B + gr] = r0;
      }
    } else if (tile == 1) {
      st_row(d.x1p + tBU + (long)gr * UH, x1, UH, t32);
      st_row(xc + UH, y1, UH, t32);
      if (t32 == 0) d.r1[(long)t * B + gr] = r1;
    } else {
      st_row(xc + 2 * UH, x2v, UH, t32);
    }
  }
  __syncthreads();
  SD_TR(1)
  core.run_lds(smem + core_lds_floats<1>(), ldp, Ig / 16, wave, l16, q);
  float* C = smem + NW * 256;
  core.reduce(smem, C, tid, wave, lane);
  SD_TR(2)
  if (tid < 256) {
    const int er = tid >> 4, c = tid & 15;
    const bool ok = er < nr && (CW == 16 || c < CW);
    const float v = C[er * 16 + c] + bhv;
    if (ok) d.hp[(long)t * B * D + (long)(rb + er) * D + n0 + c] = v;
    const float ss = group_sum<16>(ok ? v * v : 0.f);
    if (c == 0) w.ssh[((long)blockIdx.z * MR + er) * (D / CW) + tile] = ss;
  }
  SD_TR_END(d.trace, d.trace_slot)
}

// gates = BlockLinear(dyn_gru)(silu(rms(hp))) + bg; deter = GRU(gates, h_in) (rssm.py:65-75); h_in[t+1] masked.
// grid (D/CW): workgroup = CW deter columns of one block with their r / c / u gate rows: CW 16 = 3 MFMA tiles (r, c,
// u); CW 8 = 2 tiles (r | c, u | zero rows). HCW: k_hid's column tile (D / HCW row partials of hp^2 per row).
template <int CPW, int NG, int CW, int HCW>
__global__ __launch_bounds__(NTHR) void k_gate(sd_rssm_scan d, Work w, int t) {
  extern __shared__ float smem[];
  SD_TR_BEGIN
  SD_THREAD_IDS
  SD_ROW_TILE
  constexpr int NTL = CW == 16 ? 3 : 2, CL = 16 * NTL;
  const int B = d.B, D = d.D, Dg = D / d.G, ldp = Dg + 4;
  const int tile = xcd_tile(blockIdx.x, gridDim.x), n0 = tile * CW, g = n0 / Dg, j0 = n0 % Dg;
  Core<NTL, CPW> core;
  const float* wg = d.Wg + (long)g * 3 * Dg * Dg;
  const float* wt[NTL];
  if constexpr (CW == 16) {
    wt[0] = wg + (long)(j0 + l16) * Dg;
    wt[1] = wg + (long)(Dg + j0 + l16) * Dg;
    wt[NTL - 1] = wg + (long)(2 * Dg + j0 + l16) * Dg;
  } else {  // tile 1's lanes 8..15 repeat the u rows (their output columns are discarded)
    wt[0] = wg + (long)(l16 < 8 ? j0 + l16 : Dg + j0 + l16 - 8) * Dg;
    wt[NTL - 1] = wg + (long)(2 * Dg + j0 + (l16 & 7)) * Dg;
  }
  core.load_b(wt, Dg / 16, wave, q);
  const int row = tid >> 5, t32 = tid & 31, gr = rb + row;
  const bool rv = row < nr;
  const int grc = rv ? gr : rb + nr - 1;
  constexpr int NPP = (4096 / HCW + 127) / 128;  // float4 partial loads per thread (D <= 4096)
  f32x4 pv[NPP];
  ld_parts(pv, w.ssh + ((long)blockIdx.z * MR + row) * (D / HCW), D / HCW, t32);
  f32x4 hv[NG], nv[NG];
  ld_row(hv, d.hp + (long)t * B * D + (long)grc * D + (long)g * Dg, t32);
  ld_row(nv, d.nh + (long)g * Dg, t32);
  // epilogue operands (thread = (row er, column c < CW)), read unconditionally at clamped indices
  const int er = (tid >> 4) & 15, c = tid & 15, j = j0 + c, col = n0 + c, ger = rb + er;
  const bool ev = tid < 256 && er < nr && (CW == 16 || c < CW);
  const int cc_ = c & (CW - 1), gerc = er < nr ? ger : rb + nr - 1;
  const float* bg = d.bg + (long)g * 3 * Dg;
  const float bra = bg[j0 + cc_], bca = bg[Dg + j0 + cc_], bua = bg[2 * Dg + j0 + cc_];
  const float hprev = d.h_in[(long)t * B * D + (long)gerc * D + n0 + cc_];
  const unsigned char rflag = reset_byte(d, t + 1, gerc);
  const float r = rsqrtf(sum_parts(pv, D / HCW, t32) / (float)D + d.eps);
  if (rv && t32 == 0 && tile == 0) d.rh[(long)t * B + gr] = r;
  f32x4 y[NG];
#pragma unroll
  for (int i = 0; i < NG; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) y[i][k] = rv ? siluf_(hv[i][k] * r * nv[i][k]) : 0.f;
  st_row(smem + core_lds_floats<NTL>() + row * ldp, y, Dg, t32);
  if (rv && j0 == 0) st_row(d.hh + (long)t * B * D + (long)gr * D + (long)g * Dg, y, Dg, t32);
  __syncthreads();
  SD_TR(1)
  core.run_lds(smem + core_lds_floats<NTL>(), ldp, Dg / 16, wave, l16, q);
  float* C = smem + NW * NTL * 256;
  core.reduce(smem, C, tid, wave, lane);
  SD_TR(2)
  if (ev) {
    const float ra = C[er * CL + c] + bra;
    const float ca = C[er * CL + (CW == 16 ? 16 : 8) + c] + bca;
    const float ua = C[er * CL + (CW == 16 ? 32 : 16) + c] + bua;
    float* gw = d.gates + (long)t * B * 3 * D + (long)ger * 3 * D + (long)g * 3 * Dg;
    gw[j] = ra;
    gw[Dg + j] = ca;
    gw[2 * Dg + j] = ua;
    const float rs = sigmoidf_(ra);
    const float cc = tanhf(rs * ca);
    const float u = sigmoidf_(ua - 1.f);
    const float out = u * cc + (1.f - u) * hprev;
    d.deter[(long)t * B * D + (long)ger * D + col] = out;
    if (d.post_deter) d.post_deter[((long)ger * d.T + t) * D + col] = out;  // batch-major copy (RSSM.observe's output)
    if (t + 1 < d.T) d.h_in[(long)(t + 1) * B * D + (long)ger * D + col] = rflag ? 0.f : out;
  }
  SD_TR_END(d.trace, d.trace_slot)
}

// logits = obs_net_logit(silu(rms(op))) and the straight-through unimix one-hot sample (rssm.py:172-177,
// distributions.py:16-33); op = sum of the obs_net_0 slabs + (embed half + bias). grid (S): one categorical / WG.
template <int KD>
__global__ __launch_bounds__(NTHR) void k_logit(sd_rssm_scan d, Work w, int t) {
  extern __shared__ float smem[];
  SD_THREAD_IDS
  SD_ROW_TILE
  constexpr int NT = KD / 16, NE = (MR * KD + NTHR - 1) / NTHR;
  const int B = d.B, SK = d.SK, S = SK / KD, ldp = UH + 4;
  const int s = blockIdx.x, n0 = s * KD;
  Core<NT, 2> core;
  const float* wt[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) wt[i] = d.Wl + (long)(n0 + 16 * i + l16) * UH;
  core.load_b(wt, UH / 16, wave, q);
  const int row = tid >> 5, t32 = tid & 31, gr = rb + row;
  const bool rv = row < nr;
  const int grc = rv ? gr : rb + nr - 1;
  const long tBU = (long)t * B * UH;
  f32x4 x[NU], e[NU], nv[NU], xs[KSM][NU];
  ld_slabs<NU, KSM>(xs, w.ops + (long)grc * UH, (long)B * UH, d.ks_d, t32);
  ld_row(e, d.eproj + in_row(d, t, grc) * UH, t32);
  ld_row(nv, d.no, t32);
  sum_slabs(x, xs, d.ks_d);
  // sampler operands + noise, independent of the contraction
  const uint64_t seed = d.seed + (d.seed_ptr ? *d.seed_ptr : 0ull);
  float blv[NE], gn[NE];
  bool rnext[NE];
#pragma unroll
  for (int k = 0; k < NE; ++k) {
    const int i = tid + NTHR * k, er = (i / KD) & 15, lt = i % KD;
    blv[k] = d.bl[n0 + lt];
    gn[k] = sd_gumbel(seed, (uint32_t)d.stream_id, (uint32_t)t,
                      (uint64_t)((long)(rb + er) * S + s + d.group_offset) * KD + lt);
    rnext[k] = er < nr && t + 1 < d.T && reset_at(d, t + 1, rb + er);
  }
#pragma unroll
  for (int i = 0; i < NU; ++i) x[i] += e[i];
  f32x4 y[NU];
  const float r = rms_silu_rows(x, nv, UH, d.eps, rv, y);
  st_row(smem + core_lds_floats<NT>() + row * ldp, y, UH, t32);
  if (rv && s == 0) {
    st_row(d.op + tBU + (long)gr * UH, x, UH, t32);
    st_row(d.oo + tBU + (long)gr * UH, y, UH, t32);
    if (t32 == 0) d.ro[(long)t * B + gr] = r;
  }
  __syncthreads();
  core.run_lds(smem + core_lds_floats<NT>(), ldp, UH / 16, wave, l16, q);
  float* C = smem + NW * NT * 256;
  core.reduce(smem, C, tid, wave, lane);
#pragma unroll
  for (int k = 0; k < NE; ++k) {  // team of KD lanes per (row, categorical)
    const int i = tid + NTHR * k;
    if (i < MR * KD) {
      const int er = i / KD, lt = i % KD;
      const float l = C[er * KD + lt] + blv[k];
      float p, pp, nl;
      unimix_forward<KD>(l, true, KD, d.unimix, p, pp, nl);
      float ys;
      int idx;
      st_soft<KD>(nl, gn[k], true, ys, idx, lt);
      if (er < nr) {
        const float yv = ((lt == idx ? 1.f : 0.f) - ys) + ys;
        const long o = (long)t * B * SK + (long)(rb + er) * SK + n0 + lt;
        d.logit[o] = l;
        if (d.stoch) d.stoch[o] = yv;
        if (d.post_logit) {  // batch-major copies (RSSM.observe's outputs)
          const long ob = ((long)(rb + er) * d.T + t) * SK + n0 + lt;
          d.post_logit[ob] = l;
          d.post_stoch[ob] = yv;
        }
        if (t + 1 < d.T) d.s_in[o + (long)B * SK] = rnext[k] ? 0.f : yv;
      }
    }
  }
}

// k_logit by rows, with the next step's _dyn_in1 folded in: workgroup (g, b) takes batch row b and the CPG
// categoricals g*CPG.. of the obs_net logits (rssm.py:172-177): obs_net RMSNorm + SiLU of its row, the CPG*KD logits
// (fp32 dot products, K = U split over TPC lanes), the unimix one-hot ST sample (distributions.py:16-33), and then
// slab g of x1p[t+1] = the sample's _dyn_in1 pre-activation (rssm.py:52-56). A straight-through one-hot row holds one
// nonzero per categorical (((k == idx) - ys) + ys is exactly 0 off the index), so its contraction with W1 is a gather
// of CPG rows of W1^T: the NG = S / CPG slabs of a row sum (in k_hid's prologue, fixed order) to the dense product.
// That removes the x1p k_slab launch from every step (4 dependent launches per step instead of 5).
#ifndef LR_STAGE
#define LR_STAGE 0  // measured slower in the update: 9.8 vs 8.9 us (128 KB of LDS: one workgroup per CU)
#endif
template <int KD, int CPG>
__global__ __launch_bounds__(NTHR) void k_logit_rows(sd_rssm_scan d, Work w, int t) {
  constexpr int NC = CPG * KD, TPC = NTHR / NC, KPT = UH / TPC, NQ = KPT / 4;
  static_assert(NTHR % NC == 0 && UH % (4 * TPC) == 0, "column split");
  __shared__ __attribute__((aligned(16))) float y[UH];
  __shared__ float red[NW], red0[NW], lg[NC], hv[CPG];
  __shared__ int hot[CPG];
  SD_TR_BEGIN
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int B = d.B, SK = d.SK, S = SK / KD, g = blockIdx.x, b = blockIdx.y, n0 = g * NC;
  const long tBU = (long)t * B * UH;
  // the gather's candidate rows — W1^T rows n0 .. n0 + NC (the group's categoricals x every index) — are loaded
  // before the sample exists and staged in LDS (LR_STAGE: NC x U floats), so the gather after the sampler is an LDS
  // read instead of a dependent global round trip
  constexpr bool STAGE = LR_STAGE && NC * UH * 4 <= 131072;
  constexpr int NW1 = STAGE ? NC * UH / 4 / NTHR : 1;
  extern __shared__ __attribute__((aligned(16))) float w1s[];
  f32x4 w1r[NW1];
  const bool more = t + 1 < d.T;
  if (STAGE && more) {
#pragma unroll
    for (int i = 0; i < NW1; ++i) w1r[i] = ld4(w.w1t + (long)n0 * UH + 4 * (tid + NTHR * i));
  }
  // independent of the contraction: the column's weight slice, bias, noise, reset mask
  const int col = tid / TPC, kp = tid % TPC;
  f32x4 wv[NQ];
#pragma unroll
  for (int i = 0; i < NQ; ++i) wv[i] = ld4(d.Wl + (long)(n0 + col) * UH + kp * KPT + 4 * i);
  const uint64_t seed = d.seed + (d.seed_ptr ? *d.seed_ptr : 0ull);
  const bool ts = tid < NC;
  const int lt = tid % KD;
  // every load of the launch is issued unconditionally (threads past U / NC read valid duplicates), values used later
  const float blv = d.bl[n0 + (tid % NC)];
  const unsigned char rflag = reset_byte(d, t + 1, b);
  const int uc = tid % UH;
  float part[KSM], ev_ = 0.f, nw_ = 0.f;
  if (tid < UH) {  // (waves 0-3: a wave-uniform branch; the slab index is clamped, not predicated)
#pragma unroll
    for (int s = 0; s < KSM; ++s) part[s] = w.ops[(long)(s < d.ks_d ? s : d.ks_d - 1) * B * UH + (long)b * UH + uc];
    ev_ = d.eproj[in_row(d, t, b) * UH + uc];
    nw_ = d.no[uc];
  }
  // one workgroup per row also forms the NEXT step's x0 = silu(rms(x0p)), x0p = sum of the _dyn_in0 slabs k_slab
  // wrote before this launch + b0 (rssm.py:52-56), so k_hid stages the finished row instead of every column tile
  // summing the slabs and normalising again (same slab order and bias add as k_hid's own path). Its loads come last:
  // the branch around them may drain the queue, which by then holds nothing that is not needed anyway.
  const bool x0w = more && g == (gridDim.x > 1 ? 1 : 0);
  float part0[KSM], b0_ = 0.f, n0w = 0.f;
  if (x0w && tid < UH) {
#pragma unroll
    for (int s = 0; s < KSM; ++s) part0[s] = w.x0s[(long)(s < d.ks_d ? s : d.ks_d - 1) * B * UH + (long)b * UH + uc];
    b0_ = d.b0[uc];
    n0w = d.n0[uc];
  }
  const bool rnext = t + 1 < d.T && rflag;
  float gn = 0.f;
  if (ts)
    gn = sd_gumbel(seed, (uint32_t)d.stream_id, (uint32_t)t,
                   (uint64_t)((long)b * S + g * CPG + tid / KD + d.group_offset) * KD + lt);
  // obs_net_0 output row (sum of the deter-half slabs + the hoisted embed half with bias), RMSNorm + SiLU
  float x = 0.f, nw = 0.f;
  if (tid < UH) {
    x = part[0];
#pragma unroll
    for (int s = 1; s < KSM; ++s)
      if (s < d.ks_d) x += part[s];
    x += ev_;
    nw = nw_;
  }
  float x0v = 0.f;
  if (x0w && tid < UH) {
    x0v = part0[0];
#pragma unroll
    for (int s = 1; s < KSM; ++s)
      if (s < d.ks_d) x0v += part0[s];
    x0v += b0_;
  }
  float ss = wave_sum(x * x);
  const float ss0 = wave_sum(x0v * x0v);
  if (lane == 0) {
    red[wave] = ss;
    red0[wave] = ss0;
  }
  __syncthreads();
  SD_TR(1)
  ss = 0.f;
#pragma unroll
  for (int i = 0; i < UH / 64; ++i) ss += red[i];
  const float r = rsqrtf(ss / (float)UH + d.eps);
  if (x0w && tid < UH) {
    float s0 = 0.f;
#pragma unroll
    for (int i = 0; i < UH / 64; ++i) s0 += red0[i];
    const float r0 = rsqrtf(s0 / (float)UH + d.eps);
    const long o = (long)(t + 1) * B * UH + (long)b * UH + tid;
    d.x0p[o] = x0v;
    d.xcat[2 * (long)(t + 1) * B * UH + o + (long)b * 2 * UH] = siluf_(x0v * r0 * n0w);  // xcat (T, B, 3U), cols 0..U
    if (tid == 0) d.r0[(long)(t + 1) * B + b] = r0;
  }
  if (tid < UH) {
    const float yv = siluf_(x * r * nw);
    y[tid] = yv;
    if (g == 0) {
      d.op[tBU + (long)b * UH + tid] = x;
      d.oo[tBU + (long)b * UH + tid] = yv;
      if (tid == 0) d.ro[(long)t * B + b] = r;
    }
  }
  __syncthreads();
  // logits: TPC adjacent lanes per column, KPT k each, fixed-order pairwise combine
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const f32x4 yy = *reinterpret_cast<const f32x4*>(y + kp * KPT + 4 * i);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = fmaf(yy[j], wv[i][j], acc);
  }
#pragma unroll
  for (int o = 1; o < TPC; o <<= 1) acc += __shfl_xor(acc, o, 64);
  if (kp == 0) lg[col] = acc;
  __syncthreads();
  SD_TR(2)
  if (ts) {
    const float l = lg[tid] + blv;
    float p, pp, nl;
    unimix_forward<KD>(l, true, KD, d.unimix, p, pp, nl);
    float ysoft;
    int idx;
    st_soft<KD>(nl, gn, true, ysoft, idx, lt);
    const float yv = ((lt == idx ? 1.f : 0.f) - ysoft) + ysoft;
    const long o = (long)t * B * SK + (long)b * SK + n0 + tid;
    d.logit[o] = l;
    if (d.stoch) d.stoch[o] = yv;
    if (d.post_logit) {
      const long ob = ((long)b * d.T + t) * SK + n0 + tid;
      d.post_logit[ob] = l;
      d.post_stoch[ob] = yv;
    }
    if (t + 1 < d.T) d.s_in[o + (long)B * SK] = rnext ? 0.f : yv;
    if (lt == idx) {
      hot[tid / KD] = tid;  // local column of the categorical's nonzero
      hv[tid / KD] = yv;
    }
  }
  if (!more) {
    SD_TR_END(d.trace, d.trace_slot)
    return;
  }
  if (STAGE) {
#pragma unroll
    for (int i = 0; i < NW1; ++i) *reinterpret_cast<f32x4*>(w1s + 4 * (tid + NTHR * i)) = w1r[i];
  }
  __syncthreads();
  if (tid < UH) {  // slab g of x1p[t+1]: sum over the group's categoricals of v_s * W1^T[hot_s]
    float v = 0.f;
    if (!rnext) {
      float wr[CPG];
#pragma unroll
      for (int s = 0; s < CPG; ++s) wr[s] = STAGE ? w1s[hot[s] * UH + tid] : w.w1t[(long)(n0 + hot[s]) * UH + tid];
#pragma unroll
      for (int s = 0; s < CPG; ++s) v = fmaf(hv[s], wr[s], v);
    }
    w.x1s[(long)g * B * UH + (long)b * UH + tid] = v;
  }
  SD_TR_END(d.trace, d.trace_slot)
}

// ------------------------------------------------------------------------------------------- backward kernels
// straight-through sampler backward of one categorical (team of KD lanes): d logits += d/dl <ds, y_soft>. The part
// that needs only the logit and the noise (sampler_fwd) can run before the incoming gradient exists (k_carry: before
// its contraction); sampler_bwd_tail finishes it.
struct STFwd {
  float p, pp, nl, ys;
};
template <int KD>
SD_DEV STFwd sampler_fwd(float l, float gn, float unimix, int lt) {
  STFwd f;
  unimix_forward<KD>(l, true, KD, unimix, f.p, f.pp, f.nl);
  int idx;
  st_soft<KD>(f.nl, gn, true, f.ys, idx, lt);
  return f;
}
template <int KD>
SD_DEV float sampler_bwd_tail(const STFwd& f, float ds, float unimix) {
  const float sd = group_sum<KD>(ds * f.ys);
  return unimix_backward<KD>(f.ys * (ds - sd), f.p, f.pp, f.nl, true, unimix);
}
template <int KD>
SD_DEV float sampler_bwd(float l, float gn, float ds, float unimix, int lt) {
  return sampler_bwd_tail<KD>(sampler_fwd<KD>(l, gn, unimix, lt), ds, unimix);
}

// incoming gradient of posterior element (t, row, col) of a width-W output: time-major, or batch-major (bm_grads) plus
// an optional second summand g2 (rows of ld_g2 floats), summed as g + g2 (the caller's former torch.add order)
SD_DEV float in_grad(const sd_rssm_scan& d, const float* g, const float* g2, int t, int row, int col, int W) {
  if (!d.bm_grads) return g ? g[((long)t * d.B + row) * W + col] : 0.f;
  const long r = (long)row * d.T + t;
  const float a = g ? g[r * W + col] : 0.f;
  return g2 ? a + g2[r * d.ld_g2 + col] : a;
}
// the same as two unconditional loads (a missing summand reads `dummy`, any valid float) and a later combine, so the
// loads can be issued with the rest of a launch's prologue (see "load helpers")
struct InGrad {
  float a, b;
  SD_DEV void load(const sd_rssm_scan& d, const float* g, const float* g2, int t, int row, int col, int W,
                   const float* dummy) {
    const long r = d.bm_grads ? (long)row * d.T + t : (long)t * d.B + row;
    const float* pa = g ? g + r * W + col : dummy;  // address selects, one load each
    const float* pb = (d.bm_grads && g2) ? g2 + r * d.ld_g2 + col : dummy;
    a = *pa;
    b = *pb;
  }
  SD_DEV float value(const sd_rssm_scan& d, const float* g, const float* g2) const {
    const float av = g ? a : 0.f;
    return (d.bm_grads && g2) ? av + b : av;
  }
};

// dl[T-1] = d_logit + sampler backward (no carry yet). Elementwise, teams of KD lanes.
template <int KD>
__global__ __launch_bounds__(256) void k_sbwd_last(sd_rssm_scan d) {
  const int t = d.T - 1, SK = d.SK, S = SK / KD;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const int row = (int)(i / SK), k = (int)(i % SK), lt = k % KD, s = k / KD;
  const bool v = row < d.B;
  const long o = (long)t * d.B * SK + (long)row * SK + k;
  const uint64_t seed = d.seed + (d.seed_ptr ? *d.seed_ptr : 0ull);
  const float l = v ? d.logit[o] : 0.f;
  const float gn = sd_gumbel(seed, (uint32_t)d.stream_id, (uint32_t)t, (uint64_t)((long)row * S + s + d.group_offset) * KD + lt);
  const float ds = v ? in_grad(d, d.d_stoch, d.d_stoch2, t, row, k, SK) : 0.f;
  const float dl = sampler_bwd<KD>(l, gn, ds, d.unimix, lt);
  if (v) d.dl[o] = in_grad(d, d.d_logit, nullptr, t, row, k, SK) + dl;
}

// d_o = dl[t] . Wl   (dl built by the previous launch). grid (U/CW)
template <int CPW, int NS, int CW>
__global__ __launch_bounds__(NTHR) void k_dlogit(sd_rssm_scan d, Work w, int t) {
  extern __shared__ float smem[];
  SD_TR_BEGIN
  SD_THREAD_IDS
  SD_ROW_TILE
  const int B = d.B, SK = d.SK, ldp = SK + 4;
  const int n0 = xcd_tile(blockIdx.x, gridDim.x) * CW;
  Core<1, CPW> core;
  const float* wt[1] = {d.WlT + (long)(n0 + (l16 & (CW - 1))) * SK};
  core.load_b(wt, SK / 16, wave, q);
  const int row = tid >> 5, t32 = tid & 31;
  f32x4 v[NS];
  ld_row(v, d.dl + (long)t * B * SK + (long)(rb + (row < nr ? row : nr - 1)) * SK, t32);
  st_row(smem + core_lds_floats<1>() + row * ldp, v, SK, t32);
  __syncthreads();
  SD_TR(1)
  core.run_lds(smem + core_lds_floats<1>(), ldp, SK / 16, wave, l16, q);
  float* C = smem + NW * 256;
  core.reduce(smem, C, tid, wave, lane);
  SD_TR(2)
  if (tid < 256) {
    const int er = tid >> 4, c = tid & 15;
    if (er < nr && (CW == 16 || c < CW)) d.d_o[(long)t * B * UH + (long)(rb + er) * UH + n0 + c] = C[er * 16 + c];
  }
  SD_TR_END(d.trace, d.trace_slot)
}

// d_op = RMSNorm-SiLU backward (prologue); dh = d_deter + carry_h + d_op . Wo[:, :D]; GRU backward (epilogue).
// grid (D/CW)
template <int CW>
__global__ __launch_bounds__(NTHR) void k_dgru(sd_rssm_scan d, Work w, int t) {
  extern __shared__ float smem[];
  SD_TR_BEGIN
  SD_THREAD_IDS
  SD_ROW_TILE
  const int B = d.B, D = d.D, Dg = D / d.G, ldp = UH + 4;
  const int tile = xcd_tile(blockIdx.x, gridDim.x), n0 = tile * CW;
  Core<1, 2> core;
  const float* wt[1] = {d.WoDT + (long)(n0 + (l16 & (CW - 1))) * UH};
  core.load_b(wt, UH / 16, wave, q);
  const int row = tid >> 5, t32 = tid & 31, gr = rb + row;
  const bool rv = row < nr;
  const int grc = rv ? gr : rb + nr - 1;
  const long tBU = (long)t * B * UH;
  f32x4 xv[NU], dy[NU], nv[NU];
  ld_row(xv, d.op + tBU + (long)grc * UH, t32);
  ld_row(dy, d.d_o + tBU + (long)grc * UH, t32);
  ld_row(nv, d.no, t32);
  const float r_ = d.ro[(long)t * B + grc];
  // epilogue operands, read unconditionally at clamped indices
  const int er = (tid >> 4) & 15, c = tid & 15, col = n0 + (c & (CW - 1)), g = col / Dg, j = col % Dg;
  const int ger = er < nr ? rb + er : rb + nr - 1;
  const bool ev = tid < 256 && er < nr && (CW == 16 || c < CW);
  const long od = (long)t * B * D + (long)ger * D + col;
  const long gb = (long)t * B * 3 * D + (long)ger * 3 * D + (long)g * 3 * Dg;
  InGrad ig;
  ig.load(d, d.d_deter, d.d_deter2, t, ger, col, D, w.ch);
  const float chv = w.ch[(long)ger * D + col];
  const float ra = d.gates[gb + j], ca = d.gates[gb + Dg + j], ua = d.gates[gb + 2 * Dg + j];
  const float hv = d.h_in[od];
  const float r = rv ? r_ : 0.f;
  float dot = 0.f;
  f32x4 gq[NU];
#pragma unroll
  for (int i = 0; i < NU; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float xh = xv[i][k] * r;
      gq[i][k] = dy[i][k] * dsilu(xh * nv[i][k]) * nv[i][k];
      dot += gq[i][k] * xh;
    }
  dot = group_sum<32>(dot) / (float)UH;
  f32x4 o[NU];
#pragma unroll
  for (int i = 0; i < NU; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) o[i][k] = rv ? r * (gq[i][k] - xv[i][k] * r * dot) : 0.f;
  st_row(smem + core_lds_floats<1>() + row * ldp, o, UH, t32);
  if (rv && tile == 0) {
    st_row(d.d_op + tBU + (long)gr * UH, o, UH, t32);
    if (d.d_op_bm) st_row(d.d_op_bm + ((long)gr * d.T + t) * UH, o, UH, t32);
  }
  __syncthreads();
  SD_TR(1)
  core.run_lds(smem + core_lds_floats<1>(), ldp, UH / 16, wave, l16, q);
  float* C = smem + NW * 256;
  core.reduce(smem, C, tid, wave, lane);
  SD_TR(2)
  if (ev) {
    const float dh = (ig.value(d, d.d_deter, d.d_deter2) + chv) + C[er * 16 + c];
    const float rs = sigmoidf_(ra);
    const float cc = tanhf(rs * ca);
    const float u = sigmoidf_(ua - 1.f);
    const float dtc = dh * u * (1.f - cc * cc);
    d.d_gates[gb + j] = dtc * ca * rs * (1.f - rs);
    d.d_gates[gb + Dg + j] = dtc * rs;
    d.d_gates[gb + 2 * Dg + j] = dh * (cc - hv) * u * (1.f - u);
    w.dhin[(long)ger * D + col] = dh * (1.f - u);
  }
  SD_TR_END(d.trace, d.trace_slot)
}

// d_hh = d_gates_g . Wg[g] (block GEMM); epilogue: RMSNorm-SiLU backward pieces of dyn_hid's norm (g*w and the
// per-tile row partials of sum g*xhat). grid (D/CW)
template <int CPW, int CW>
__global__ __launch_bounds__(NTHR) void k_dhh(sd_rssm_scan d, Work w, int t) {
  extern __shared__ float smem[];
  SD_TR_BEGIN
  SD_THREAD_IDS
  SD_ROW_TILE
  const int B = d.B, D = d.D, Dg = D / d.G;
  const int tile = xcd_tile(blockIdx.x, gridDim.x), n0 = tile * CW, g = n0 / Dg, j0 = n0 % Dg;
  Core<1, CPW> core;
  const float* wt[1] = {d.WgT + ((long)g * Dg + j0 + (l16 & (CW - 1))) * 3 * Dg};
  core.load_b(wt, 3 * Dg / 16, wave, q);
  const int er = (tid >> 4) & 15, c = tid & 15, col = n0 + (c & (CW - 1));
  const int ger = er < nr ? rb + er : rb + nr - 1;
  const bool ev = tid < 256 && er < nr && (CW == 16 || c < CW);
  const long o = (long)t * B * D + (long)ger * D + col;
  const float hpv = d.hp[o], rhv = d.rh[(long)t * B + ger], wv = d.nh[col];  // unconditional, clamped
  core.run_glb(d.d_gates + ((long)t * B + rb) * 3 * D + (long)g * 3 * Dg, 3 * (long)D, nr, 3 * Dg / 16, wave, l16, q);
  const float xh = hpv * rhv;
  SD_TR(1)
  float* C = smem + NW * 256;
  core.reduce(smem, C, tid, wave, lane);
  SD_TR(2)
  if (tid < 256) {
    float part = 0.f;
    if (ev) {
      const float dy = C[er * 16 + c];
      d.d_hh[o] = dy;
      const float gq = dy * dsilu(xh * wv) * wv;
      w.gq[(long)ger * D + col] = gq;
      part = gq * xh;
    }
    part = group_sum<16>(part);
    if (c == 0) w.dotp[((long)blockIdx.z * MR + er) * (D / CW) + tile] = part;
  }
  SD_TR_END(d.trace, d.trace_slot)
}

// d_xcat slabs k_dhp writes: slab s covers G / KX consecutive blocks (KX = 8 = G: one per block). Fewer slabs mean
// fewer, larger P0 workgroups and less for k_carry to stage (each of its workgroups sums KX slabs of 16 rows)
#ifndef SD_SCAN_KX
#define SD_SCAN_KX 8
#endif
__host__ __device__ inline int kx_of(int G) { return G % SD_SCAN_KX == 0 ? SD_SCAN_KX : G; }

// d_hp = RMSNorm backward (prologue, from g*w and the row partials) over the workgroup's K span; then two problems in
// one grid:
//   P0: d_xcat slab s = d_hp[:, blocks of s] . Wsh[those rows]   ((3U/16) * KX workgroups, K = G/KX blocks)
//   P1: d_hin[:, g] += d_hp_g . Wbd[g]                            (D/16 workgroups, K = one block)
// CPW / NGX cover the longest span (P0); P1 masks the chunks past its block. DHC: k_dhh's column tile (D / DHC row
// partials).
template <int CPW, int NGX, int DHC>
__global__ __launch_bounds__(NTHR) void k_dhp(sd_rssm_scan d, Work w, int t) {
  extern __shared__ float smem[];
  SD_TR_BEGIN
  SD_THREAD_IDS
  SD_ROW_TILE
  const int B = d.B, D = d.D, Dg = D / d.G, X = 3 * UH;
  const int KX = kx_of(d.G), NX = (X / 16) * KX;
  const int blk = blockIdx.x;
  const bool p0 = blk < NX;
  int n0, k0, K, sl = 0;
  const float* wrow;
  if (p0) {  // (X / 16 = 48 column tiles per slab: blk % 8 = tile % 8, so the remap stays within a slab)
    sl = blk / (X / 16);
    n0 = xcd_tile(blk % (X / 16), X / 16) * 16;
    K = (d.G / KX) * Dg;
    k0 = sl * K;
    wrow = d.WshT + (long)(n0 + l16) * D + k0;
  } else {  // (NX = 48 KX is a multiple of 8)
    n0 = xcd_tile(blk - NX, D / 16) * 16;
    const int g = n0 / Dg;
    K = Dg;
    k0 = g * Dg;
    wrow = d.WbdT + ((long)g * Dg + n0 % Dg + l16) * Dg;
  }
  const int ldp = K + 4;
  Core<1, CPW> core;
  const float* wt[1] = {wrow};
  core.load_b(wt, K / 16, wave, q);
  const int row = tid >> 5, t32 = tid & 31, gr = rb + row;
  const bool rv = row < nr;
  constexpr int NPP = (4096 / DHC + 127) / 128;
  f32x4 pv[NPP];
  ld_parts(pv, w.dotp + ((long)blockIdx.z * MR + row) * (D / DHC), D / DHC, t32);
  const int grc = rv ? gr : rb + nr - 1;
  const long ob = (long)gr * D + k0, obc = (long)grc * D + k0;
  f32x4 gq[NGX], xv[NGX];  // (K = D/G = 128 * NGX on both problems: G / KX = 1)
  ld_row(gq, w.gq + obc, t32);
  ld_row(xv, d.hp + (long)t * B * D + obc, t32);
  const float r_ = d.rh[(long)t * B + grc];
  const int er = (tid >> 4) & 15, c = tid & 15, ger = rb + er;
  const bool ev = tid < 256 && er < nr;
  const float dh_ = w.dhin[(long)(er < nr ? ger : rb + nr - 1) * D + n0 + c];  // unconditional, used by P1 only
  const float r = rv ? r_ : 0.f, dh_old = (!p0 && ev) ? dh_ : 0.f;
  const float dot = sum_parts(pv, D / DHC, t32) / (float)D;
  f32x4 o[NGX];
#pragma unroll
  for (int i = 0; i < NGX; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) o[i][k] = rv ? r * (gq[i][k] - xv[i][k] * r * dot) : 0.f;
  st_row(smem + core_lds_floats<1>() + row * ldp, o, K, t32);
  if (rv && !p0 && (n0 % Dg) == 0) st_row(d.d_hp + (long)t * B * D + ob, o, K, t32);
  __syncthreads();
  SD_TR(1)
  core.run_lds(smem + core_lds_floats<1>(), ldp, K / 16, wave, l16, q);
  float* C = smem + NW * 256;
  core.reduce(smem, C, tid, wave, lane);
  SD_TR(2)
  if (ev) {
    if (p0) w.dxs[(long)sl * B * X + (long)ger * X + n0 + c] = C[er * 16 + c];
    else w.dhin[(long)ger * D + n0 + c] = dh_old + C[er * 16 + c];
  }
  SD_TR_END(d.trace, d.trace_slot)
}

// d_xcat = sum over blocks of the slabs; d_x0p / d_x1p = RMSNorm-SiLU backward of the _dyn_in0 / _dyn_in1 norms.
// grid (B): one workgroup per row; waves 0-3 take x0, waves 4-7 x1 (one column per thread).
__global__ __launch_bounds__(NTHR) void k_dx01(sd_rssm_scan d, Work w, int t) {
  __shared__ float red[NW];
  __shared__ float dx[3 * UH];
  constexpr int X = 3 * UH, NC = (X + NTHR - 1) / NTHR, GM = 8;
  const int tid = threadIdx.x, wave = tid >> 6;
  const int B = d.B, b = blockIdx.x;
  const long tB = (long)t * B;
  float part[GM][NC];
#pragma unroll
  for (int g = 0; g < GM; ++g)
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const int c = tid + NTHR * k;
      part[g][k] = (g < kx_of(d.G) && c < X) ? w.dxs[(long)g * B * X + (long)b * X + c] : 0.f;
    }
  const int half = wave >> 2, ht = tid & 255;
  const float* x = (half ? d.x1p : d.x0p) + (tB + b) * UH;
  const float xv = x[ht], wv = (half ? d.n1 : d.n0)[ht];
  const float r = (half ? d.r1 : d.r0)[tB + b];
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    const int c = tid + NTHR * k;
    float v = part[0][k];
#pragma unroll
    for (int g = 1; g < GM; ++g) v += part[g][k];
    if (c < X) {
      dx[c] = v;
      d.d_xcat[(tB + b) * X + c] = v;
      if (d.d_x2_bm && c >= 2 * d.U) d.d_x2_bm[((long)b * d.T + t) * d.U + (c - 2 * d.U)] = v;
    }
  }
  __syncthreads();
  const float xh = xv * r;
  const float gg = dx[half * UH + ht] * dsilu(xh * wv) * wv;
  float dot = wave_sum(gg * xh);
  if ((tid & 63) == 0) red[wave] = dot;
  __syncthreads();
  dot = (red[4 * half] + red[4 * half + 1] + red[4 * half + 2] + red[4 * half + 3]) / (float)UH;
  ((half ? d.d_x1p : d.d_x0p) + (tB + b) * UH)[ht] = r * (gg - xh * dot);
}

// carry_h = mask(d_hin + d_x0p . W0) and carry_s = mask(d_x1p . W1) into step t-1 (rssm.py:161-165 backward); the
// carry_s workgroups (one categorical each) then run the sampler backward of step t-1:
// dl[t-1] = d_logit[t-1] + ST-backward(logit[t-1], d_stoch[t-1] + carry_s). grid (D/KD + S)
// The A operand d_x0p (carry_h workgroups) / d_x1p (carry_s workgroups) is built by the prologue, as k_dx01 builds it:
// sum of the G d_xcat slabs of k_dhp + the _dyn_in0 / _dyn_in1 RMSNorm-SiLU backward, 16 rows into an LDS panel. The
// first workgroup of each half also writes its d_xcat part and d_x0p / d_x1p (read by the deferred weight gradients);
// one extra workgroup (the last) writes the x2 part of d_xcat and does nothing else, so the others hold no registers
// for it (188 -> 128 VGPRs: two workgroups per CU, so deter 4096's 288 workgroups run as one round instead of two).
// So k_dx01 runs only at t = 0 (no k_carry there).
template <int KD>
__global__ __launch_bounds__(NTHR) void k_carry(sd_rssm_scan d, Work w, int t) {
  extern __shared__ float smem[];
  SD_TR_BEGIN
  SD_THREAD_IDS
  SD_ROW_TILE
  constexpr int NT = KD / 16, NE = (MR * KD + NTHR - 1) / NTHR, GM = 8, X = 3 * UH, ldp = UH + 4;
  const int B = d.B, D = d.D, SK = d.SK, S = SK / KD;
  if ((int)blockIdx.x == D / KD + SK / KD) {  // the x2 part of d_xcat: sum of k_dhp's slabs (k_dx01's order)
    const int row = tid >> 5, t32 = tid & 31, gr = rb + row, KX = kx_of(d.G);
    const int grc = row < nr ? gr : rb + nr - 1;
    const long tB = (long)t * B;
    f32x4 part2[GM][NU], dx[NU];
#pragma unroll
    for (int g = 0; g < GM; ++g) ld_row(part2[g], w.dxs + (long)(g < KX ? g : KX - 1) * B * X + (long)grc * X + 2 * UH, t32);
    sum_slabs(dx, part2, KX);
    if (row < nr) {
      st_row(d.d_xcat + (tB + gr) * X + 2 * UH, dx, UH, t32);
      if (d.d_x2_bm) st_row(d.d_x2_bm + ((long)gr * d.T + t) * UH, dx, UH, t32);
    }
    SD_TR(1)
    SD_TR(2)
    SD_TR_END(d.trace, d.trace_slot)
    return;
  }
  const bool p0 = (int)blockIdx.x < D / KD;
  const int wid = p0 ? xcd_tile(blockIdx.x, D / KD) : xcd_tile(blockIdx.x - D / KD, SK / KD), n0 = wid * KD;
  Core<NT, 2> core;
  const float* wt[NT];
#pragma unroll
  for (int i = 0; i < NT; ++i) wt[i] = (p0 ? d.W0T : d.W1T) + (long)(n0 + 16 * i + l16) * UH;
  core.load_b(wt, UH / 16, wave, q);
  // prologue loads: the G slabs of this half's d_xcat part, its pre-norm input and norm weight (unconditional, rows
  // clamped; slabs past KX re-read slab KX - 1 and are not summed)
  const int row = tid >> 5, t32 = tid & 31, gr = rb + row;
  const bool rv = row < nr;
  const int grc = rv ? gr : rb + nr - 1, KX = kx_of(d.G);
  const long tB = (long)t * B;
  const int hoff = p0 ? 0 : UH;
  f32x4 part[GM][NU], xv[NU], nv[NU];
#pragma unroll
  for (int g = 0; g < GM; ++g) ld_row(part[g], w.dxs + (long)(g < KX ? g : KX - 1) * B * X + (long)grc * X + hoff, t32);
  const float rr_ = (p0 ? d.r0 : d.r1)[tB + grc];
  ld_row(xv, (p0 ? d.x0p : d.x1p) + (tB + grc) * UH, t32);
  ld_row(nv, p0 ? d.n0 : d.n1, t32);
  // epilogue operands: element i = (row er, column lt) of the 16 x KD tile, read unconditionally (clamped rows; the
  // carry_h workgroups read column 0 of the sampler operands and never use them)
  const uint64_t seed = d.seed + (d.seed_ptr ? *d.seed_ptr : 0ull);
  const int tp = t - 1;
  float e0[NE], gn[NE];
  InGrad e1[NE], e2[NE];
  unsigned char rf[NE];
#pragma unroll
  for (int k = 0; k < NE; ++k) {
    const int i = tid + NTHR * k, er = (i / KD) & 15, lt = i % KD;
    const int gerc = er < nr ? rb + er : rb + nr - 1, cs = p0 ? 0 : n0 + lt;
    rf[k] = reset_byte(d, t, gerc);
    e0[k] = *(p0 ? w.dhin + (long)gerc * D + n0 + lt : d.logit + (long)tp * B * SK + (long)gerc * SK + cs);
    e1[k].load(d, d.d_stoch, d.d_stoch2, tp, gerc, cs, SK, w.ch);
    e2[k].load(d, d.d_logit, nullptr, tp, gerc, cs, SK, w.ch);
  }
  const float rr = rv ? rr_ : 0.f;
  bool rs[NE];
#pragma unroll
  for (int k = 0; k < NE; ++k) {
    const int i = tid + NTHR * k, er = (i / KD) & 15, lt = i % KD, ger = rb + er;
    const bool ev = i < MR * KD && er < nr;
    rs[k] = ev && rf[k] != 0;
    gn[k] = 0.f;
    if (!p0)
      gn[k] = sd_gumbel(seed, (uint32_t)d.stream_id, (uint32_t)tp,
                        (uint64_t)((long)ger * S + n0 / KD + d.group_offset) * KD + lt);
  }
  // the sampler's forward half of step t - 1 (carry_s workgroups): needs only the logit and the noise, so it runs
  // here, beside the prologue loads, instead of after the contraction
  STFwd sf[NE];
  if (!p0) {
#pragma unroll
    for (int k = 0; k < NE; ++k)
      if (tid + NTHR * k < MR * KD) sf[k] = sampler_fwd<KD>(e0[k], gn[k], d.unimix, (tid + NTHR * k) % KD);
  }
  // d_xcat part = sum of the slabs (k_dx01's order)
  f32x4 dx[NU];
  sum_slabs(dx, part, KX);
  float dot = 0.f;
  f32x4 gg[NU], xh[NU];
#pragma unroll
  for (int i = 0; i < NU; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      xh[i][k] = xv[i][k] * rr;
      gg[i][k] = dx[i][k] * dsilu(xh[i][k] * nv[i][k]) * nv[i][k];
      dot += gg[i][k] * xh[i][k];
    }
  dot = group_sum<32>(dot) / (float)UH;
  f32x4 o[NU];
#pragma unroll
  for (int i = 0; i < NU; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) o[i][k] = rv ? rr * (gg[i][k] - xh[i][k] * dot) : 0.f;
  float* P = smem + core_lds_floats<NT>();
  st_row(P + row * ldp, o, UH, t32);
  if (rv && wid == 0) {
    st_row(d.d_xcat + (tB + gr) * X + hoff, dx, UH, t32);
    st_row((p0 ? d.d_x0p : d.d_x1p) + (tB + gr) * UH, o, UH, t32);
  }
  __syncthreads();
  SD_TR(1)
  core.run_lds(P, ldp, UH / 16, wave, l16, q);
  float* C = smem + NW * NT * 256;
  core.reduce(smem, C, tid, wave, lane);
  SD_TR(2)
#pragma unroll
  for (int k = 0; k < NE; ++k) {
    const int i = tid + NTHR * k;
    if (i < MR * KD) {
      const int er = i / KD, lt = i % KD, ger = rb + er;
      const bool ev = er < nr;
      if (p0) {
        if (ev) w.ch[(long)ger * D + n0 + lt] = rs[k] ? 0.f : e0[k] + C[er * KD + lt];
      } else {
        const float cs = rs[k] ? 0.f : C[er * KD + lt];
        const float dlv = sampler_bwd_tail<KD>(sf[k], ev ? e1[k].value(d, d.d_stoch, d.d_stoch2) + cs : 0.f, d.unimix);
        if (ev) d.dl[(long)tp * B * SK + (long)ger * SK + n0 + lt] = e2[k].value(d, d.d_logit, nullptr) + dlv;
      }
    }
  }
  SD_TR_END(d.trace, d.trace_slot)
}

// ------------------------------------------------------------------------------------------- host side
int cpw_for(int k) {  // chunks per wave for a k span (16-deep chunks over 8 waves), rounded to an instantiation
  const int c = (k / 16 + NW - 1) / NW;
  return c <= 2 ? 2 : c <= 4 ? 4 : c <= 6 ? 6 : c <= 8 ? 8 : c <= 12 ? 12 : c <= 16 ? 16 : -1;
}

#define SD_CPW_SWITCH(cpw, ...)                            \
  switch (cpw) {                                           \
    case 2: { constexpr int CP = 2; __VA_ARGS__; } break;  \
    case 4: { constexpr int CP = 4; __VA_ARGS__; } break;  \
    case 6: { constexpr int CP = 6; __VA_ARGS__; } break;  \
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
  if (d->B < 1 || d->B > 4096 || d->T < 1 || d->G < 1 || d->G > 8 || d->D % d->G) return SD_ESHAPE;
  if (d->row_tile < 0 || d->row_tile > MR) return SD_EARG;
  const int Dg = d->D / d->G;
  if (d->U != UH || (Dg != 256 && Dg != 512) || (d->SK != 512 && d->SK != 1024) || d->D > 4096) return SD_ESHAPE;
  if (d->Kd != 16 && d->Kd != 32 && d->Kd != 64) return SD_ESHAPE;
  if (d->SK % d->Kd || d->D % d->Kd) return SD_ESHAPE;
  if (d->ks_d < 1 || d->ks_s < 1 || d->ks_d > KSM || d->ks_s > KSM || d->D % (d->ks_d * 16) ||
      d->SK % (d->ks_s * 16))
    return SD_ESHAPE;
  if (!d->work) return SD_EARG;
  if (d->ld_wod < 0 || (d->ld_wod > 0 && (d->ld_wod < d->D || d->ld_wod % 4))) return SD_EARG;
  if ((d->post_logit != nullptr) != (d->post_stoch != nullptr)) return SD_EARG;
  if ((d->d_stoch2 || d->d_deter2) && (!d->bm_grads || d->ld_g2 < 1)) return SD_EARG;
  return SD_OK;
}

#define SD_NG_SWITCH(dg, ...)                                 \
  switch (dg) {                                               \
    case 256: { constexpr int NG = 2; __VA_ARGS__; } break;   \
    case 512: { constexpr int NG = 4; __VA_ARGS__; } break;   \
    default: return SD_ESHAPE;                                \
  }

#ifndef SD_SCAN_LROWS
#define SD_SCAN_LROWS 1
#endif
// the forward's per-step phases (0: x1p k_slab, 1: k_hid, 2: k_gate, 3: obs_net_0 + next x0p k_slab, 4: logits +
// sampler [+ next x1p slabs when lrows]); one definition for sd_rssm_scan_fwd and the measurement aid
int fwd_phase(const sd_rssm_scan& d, const Work& w, bool lrows, int which, int t, hipStream_t st) {
  const int B = d.B, D = d.D, SK = d.SK, Dg = D / d.G, Ig = Dg + 3 * UH;
  const int ks_s = lrows ? LR_NG : d.ks_s;
  const int span_d = D / d.ks_d, span_s = SK / ks_s;
  const int cp_d = cpw_for(span_d), cp_s = cpw_for(span_s), cp_h = cpw_for(Ig);
  if (cp_d < 0 || cp_s < 0 || cp_h < 0) return SD_ESHAPE;
  const size_t core1 = core_lds_floats<1>() * 4;
  const size_t lds_hid = core1 + (size_t)MR * (Ig + 4) * 4;
  const size_t lds_gate = core_lds_floats<SD_SCAN_GCW == 16 ? 3 : 2>() * 4 + (size_t)MR * (Dg + 4) * 4;
  const long BD = (long)B * D, BS = (long)B * SK;
  const long wod_ld = d.ld_wod > 0 ? d.ld_wod : D;
  sd_rssm_scan dd = d;
  dd.ks_s = ks_s;  // x1p slabs k_hid sums
  const int rt = dd.row_tile = row_tile_of(d), nt = row_tiles(d);
  dd.trace_slot = t * 8 + which;
  if (which == 0) {
    SlabProb p{d.s_in + t * BS, SK, d.W1, SK, w.x1s, d.reset, d.trace, dd.trace_slot, 1, 0};
    SD_CPW_SWITCH(cp_s, k_slab<CP><<<dim3(UH / 16, ks_s * nt, 1), NTHR, core1, st>>>(p, p, B, UH, span_s, ks_s, rt));
  } else if (which == 1) {
    // x0 finished by the previous step's k_logit_rows (lrows, t > 0)
    constexpr int HC = SD_SCAN_HCW;
    if (lrows && t > 0) {
      SD_NG_SWITCH(Dg, SD_CPW_SWITCH(cp_h, if (!(raise_lds<k_hid<CP, NG, true, HC>>(lds_hid))) return SD_EARG;
                                     k_hid<CP, NG, true, HC><<<dim3(D / HC, 1, nt), NTHR, lds_hid, st>>>(dd, w, t)));
    } else {
      SD_NG_SWITCH(Dg, SD_CPW_SWITCH(cp_h, if (!(raise_lds<k_hid<CP, NG, false, HC>>(lds_hid))) return SD_EARG;
                                     k_hid<CP, NG, false, HC><<<dim3(D / HC, 1, nt), NTHR, lds_hid, st>>>(dd, w, t)));
    }
  } else if (which == 2) {
    constexpr int GC = SD_SCAN_GCW, HC = SD_SCAN_HCW;
    SD_NG_SWITCH(Dg, if (!(raise_lds<k_gate<NG, NG, GC, HC>>(lds_gate))) return SD_EARG;
                 k_gate<NG, NG, GC, HC><<<dim3(D / GC, 1, nt), NTHR, lds_gate, st>>>(dd, w, t));
  } else if (which == 3) {
    SlabProb po{d.deter + t * BD, D, d.WoD, wod_ld, w.ops, d.reset, d.trace, dd.trace_slot, 1, 0};
    SlabProb px{d.deter + t * BD, D, d.W0, D, w.x0s, d.reset_bm ? d.reset + (t + 1) : d.reset + (t + 1) * B, d.trace,
                dd.trace_slot, d.reset_bm ? d.T : 1, 1};
    const int np = t + 1 < d.T ? 2 : 1;
    SD_CPW_SWITCH(cp_d, k_slab<CP><<<dim3(UH / 16, d.ks_d * nt, np), NTHR, core1, st>>>(po, px, B, UH, span_d,
                                                                                        d.ks_d, rt));
  } else if (lrows) {
    const dim3 gr(LR_NG, B);
#define SD_LR(KD_, CPG_)                                                                                 \
  do {                                                                                                    \
    constexpr size_t lds = LR_STAGE && (size_t)CPG_ * KD_ * UH * 4 <= 131072 ? (size_t)CPG_ * KD_ * UH * 4 : 0; \
    if (!(raise_lds<k_logit_rows<KD_, CPG_>>(lds))) return SD_EARG;                                       \
    k_logit_rows<KD_, CPG_><<<gr, NTHR, lds, st>>>(dd, w, t);                                             \
  } while (0)
    // CPG = S / LR_NG categoricals per workgroup (use_lrows: S % LR_NG == 0, so CPG >= 1 where it launches)
    if (d.Kd == 16) { if (SK == 512) SD_LR(16, lr_cpg(512, 16)); else SD_LR(16, lr_cpg(1024, 16)); }
    else if (d.Kd == 32) { if (SK == 512) SD_LR(32, lr_cpg(512, 32)); else SD_LR(32, lr_cpg(1024, 32)); }
    else { if (SK == 512) SD_LR(64, lr_cpg(512, 64)); else SD_LR(64, lr_cpg(1024, 64)); }
#undef SD_LR
  } else {
    SD_KD_SWITCH(d.Kd, {
      const size_t lds = core_lds_floats<KD / 16>() * 4 + (size_t)MR * (UH + 4) * 4;
      if (!(raise_lds<k_logit<KD>>(lds))) return SD_EARG;
      k_logit<KD><<<dim3(SK / KD, 1, nt), NTHR, lds, st>>>(dd, w, t);
    });
  }
  SD_LAUNCH_CHECK();
  return SD_OK;
}
bool use_lrows(const sd_rssm_scan& d) { return SD_SCAN_LROWS && (d.SK / d.Kd) % LR_NG == 0; }

}  // namespace

extern "C" int sd_rssm_scan_work_floats(const sd_rssm_scan* d) {
  if (!d) return SD_EARG;
  return (int)work_layout(*d, nullptr).total;
}

extern "C" int sd_rssm_scan_fwd(const sd_rssm_scan* dp, sd_stream stream_) {
  int rc = check(dp);
  if (rc) return rc;
  if (!dp->stoch && !dp->post_stoch) return SD_EARG;  // the sample goes somewhere
  hipStream_t st = (hipStream_t)stream_;
  const sd_rssm_scan& d = *dp;
  const Work w = work_layout(d, d.work);
  const int B = d.B, D = d.D;
  const int cp_d = cpw_for(D / d.ks_d);
  if (cp_d < 0) return SD_ESHAPE;
  const bool lrows = use_lrows(d);
  k_init<<<lrows ? 256 : 64, 256, 0, st>>>(d, lrows ? w.w1t : nullptr);
  SD_LAUNCH_CHECK();
  {  // x0p(0) = h_in[0] . W0^T
    SlabProb p{d.h_in, D, d.W0, D, w.x0s, d.reset, nullptr, 0, 1, 0};
    SD_CPW_SWITCH(cp_d, k_slab<CP><<<dim3(UH / 16, d.ks_d * row_tiles(d), 1), NTHR, core_lds_floats<1>() * 4, st>>>(
                            p, p, B, UH, D / d.ks_d, d.ks_d, row_tile_of(d)));
    SD_LAUNCH_CHECK();
  }
  for (int t = 0; t < d.T; ++t) {
    for (int which = 0; which < 5; ++which) {
      if (which == 0 && lrows && t > 0) continue;  // x1p[t] slabs written by step t-1's k_logit_rows
      rc = fwd_phase(d, w, lrows, which, t, st);
      if (rc) return rc;
    }
  }
  return SD_OK;
}

// One launch of forward step t's phase `which` exactly as sd_rssm_scan_fwd issues it (same descriptor, workspace and
// grid): 0 = k_slab (x1p; issued only at t = 0 when k_logit_rows writes the next step's x1p slabs), 1 = k_hid,
// 2 = k_gate, 3 = k_slab (obs_net_0 deter half + next x0p), 4 = k_logit / k_logit_rows. A measurement aid (bench.py
// times the scan's phases with it, after a full sd_rssm_scan_fwd on the same descriptor); only t = T - 1 rewrites
// exactly the values the run wrote (the workspace slabs hold the last step's partials).
extern "C" int sd_rssm_scan_step_kernel(const sd_rssm_scan* dp, int which, int t, sd_stream stream_) {
  int rc = check(dp);
  if (rc) return rc;
  const sd_rssm_scan& d = *dp;
  if (t < 0 || t >= d.T || which < 0 || which > 4) return SD_EARG;
  return fwd_phase(d, work_layout(d, d.work), use_lrows(d), which, t, (hipStream_t)stream_);
}

extern "C" int sd_rssm_scan_bwd(const sd_rssm_scan* dp, sd_stream stream_) {
  int rc = check(dp);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream_;
  sd_rssm_scan d = *dp;
  d.row_tile = row_tile_of(*dp);
  const int nt = row_tiles(d);
  const Work w = work_layout(d, d.work);
  const int B = d.B, D = d.D, SK = d.SK, Dg = D / d.G;
  const int cp_g3 = cpw_for(3 * Dg);
  if (cp_g3 < 0) return SD_ESHAPE;
  const size_t core1 = core_lds_floats<1>() * 4;
  const size_t lds_dl = core1 + (size_t)MR * (SK + 4) * 4;
  const size_t lds_dgru = core1 + (size_t)MR * (UH + 4) * 4;
  const int kspan = (d.G / kx_of(d.G)) * Dg;  // k_dhp's longest K span (P0)
  const size_t lds_dhp = core1 + (size_t)MR * (kspan + 4) * 4;
  // carry of the step after T-1 is zero. A kernel, not hipMemsetAsync: in a captured HIP graph the memset node was
  // observed not to be ordered before the first k_dgru (garbage carry in replays)
  k_zero<<<sd_cdiv(B * D, 256), 256, 0, st>>>(w.ch, (long)B * D);
  SD_LAUNCH_CHECK();
  constexpr int DLC = SD_SCAN_DLCW, DGC = SD_SCAN_DGCW, DHC = SD_SCAN_DHCW;
  const int NX = (3 * UH / 16) * kx_of(d.G);
  SD_KD_SWITCH(d.Kd, k_sbwd_last<KD><<<(int)(((long)B * SK + 255) / 256), 256, 0, st>>>(d));
  SD_LAUNCH_CHECK();
  for (int t = d.T - 1; t >= 0; --t) {
    d.trace_slot = (d.T + t) * 8;
    if (SK == 512) {
      if (!(raise_lds<k_dlogit<4, 4, DLC>>(lds_dl))) return SD_EARG;
      k_dlogit<4, 4, DLC><<<dim3(UH / DLC, 1, nt), NTHR, lds_dl, st>>>(d, w, t);
    } else {
      if (!(raise_lds<k_dlogit<8, 8, DLC>>(lds_dl))) return SD_EARG;
      k_dlogit<8, 8, DLC><<<dim3(UH / DLC, 1, nt), NTHR, lds_dl, st>>>(d, w, t);
    }
    SD_LAUNCH_CHECK();
    d.trace_slot = (d.T + t) * 8 + 1;
    k_dgru<DGC><<<dim3(D / DGC, 1, nt), NTHR, lds_dgru, st>>>(d, w, t);
    SD_LAUNCH_CHECK();
    d.trace_slot = (d.T + t) * 8 + 2;
    SD_CPW_SWITCH(cp_g3, k_dhh<CP, DHC><<<dim3(D / DHC, 1, nt), NTHR, core1, st>>>(d, w, t));
    SD_LAUNCH_CHECK();
    d.trace_slot = (d.T + t) * 8 + 3;
    SD_CPW_SWITCH(kspan / 128, if (!(raise_lds<k_dhp<CP, CP, DHC>>(lds_dhp))) return SD_EARG;
                  k_dhp<CP, CP, DHC><<<dim3(NX + D / 16, 1, nt), NTHR, lds_dhp, st>>>(d, w, t));
    SD_LAUNCH_CHECK();
    d.trace_slot = (d.T + t) * 8 + 4;
    if (t > 0) {  // k_carry builds d_x0p / d_x1p itself (the k_dx01 work in its prologue)
      SD_KD_SWITCH(d.Kd, k_carry<KD><<<dim3(D / KD + SK / KD + 1, 1, nt), NTHR,
                                       core_lds_floats<KD / 16>() * 4 + (size_t)MR * (UH + 4) * 4, st>>>(d, w, t));
    } else {
      k_dx01<<<B, NTHR, 0, st>>>(d, w, t);
    }
    SD_LAUNCH_CHECK();
  }
  return SD_OK;
}
