// Small elementwise / reduction kernels of the update path and the Barlow (r2dreamer) loss.
//
//  * image uint8 -> f32 (Dreamer.preprocess, dreamer.py:710-713) with the encoder's "-0.5" (networks.py:224);
//  * symlog inputs (MLP encoder, networks.py:333-334); action normalisation a / max(|a|, 1) (rssm.py:44);
//    reset masking of the recurrent state (rssm.py:161-165);
//  * Barlow twins loss (dreamer.py:525-532): column mean / unbiased std, standardisation fwd/bwd, the
//    invariance + redundancy reduction over the E x E cross-correlation and its gradient;
//  * noise buffers (philox.h) for tests and diagnostics.
#include "common.h"
#include "philox.h"
#include "sdhip.h"

namespace {

__global__ void u8_to_f32(const uint8_t* __restrict__ in, float* __restrict__ out, long n, float shift) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (float)in[i] / 255.0f - shift;
}

// the replay image to both float forms in one pass: img[p][c] = u8 / 255 (Dreamer.preprocess; nullable) and the
// ConvEncoder input enc[p][c] = u8 / 255 - shift, zero-padded to Cp channels (the same two roundings as
// sd_u8_to_f32 followed by sd_pad_channels). One thread per pixel.
__global__ void u8_image_inputs_kernel(const uint8_t* __restrict__ in, float* __restrict__ img, float* __restrict__ enc,
                                       long pixels, int C, int Cp, float shift) {
  const long pix = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= pixels) return;
  for (int c = 0; c < Cp; ++c) {
    float v = 0.f;
    if (c < C) {
      const float f = (float)in[pix * C + c] / 255.0f;
      if (img) img[pix * C + c] = f;
      v = f - shift;
    }
    enc[pix * Cp + c] = v;
  }
}

// out[p][c] = in[p][c] - shift for c < C, 0 for C <= c < Cp (channel-pad an NHWC image to a float4 multiple)
__global__ void pad_channels_kernel(const float* __restrict__ in, float* __restrict__ out, long pixels, int C, int Cp,
                                    float shift) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= pixels * Cp) return;
  const long pix = i / Cp;
  const int c = (int)(i - pix * Cp);
  out[i] = c < C ? in[pix * C + c] - shift : 0.f;
}

__global__ void symlog_kernel(const float* __restrict__ x, float* __restrict__ y, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const float v = x[i];
    const float s = v > 0.f ? 1.f : (v < 0.f ? -1.f : 0.f);
    y[i] = s * log1pf(fabsf(v));
  }
}

__global__ void action_norm_kernel(const float* __restrict__ a, float* __restrict__ y, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = a[i] / fmaxf(fabsf(a[i]), 1.f);
}

// y[r, :] = mask[r] ? 0 : x[r, :]   (mask is bool/uint8)
__global__ void mask_rows_kernel(const float* __restrict__ x, const uint8_t* __restrict__ mask, long mask_stride,
                                 float* __restrict__ y, long rows, int width) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * width) return;
  const long r = i / width;
  y[i] = mask[r * mask_stride] ? 0.f : x[i];
}

__global__ void fill_gumbel(float* out, long n, uint64_t seed, uint32_t stream, uint32_t step, long offset) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = sd_gumbel(seed, stream, step, (uint64_t)(i + offset));
}
__global__ void fill_normal(float* out, long n, uint64_t seed, uint32_t stream, uint32_t step, long offset) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = sd_normal(seed, stream, step, (uint64_t)(i + offset));
}

// column mean and unbiased std of x (R x C): two passes over rows, NP row-partials per column (64 x NP threads per
// workgroup, so a 1024-row batch is 64 dependent loads per thread, not 256), fixed summation order
constexpr int CS_NP = 16;
__global__ __launch_bounds__(64 * CS_NP) void colstats_kernel(const float* __restrict__ x, int R, int C,
                                                             float* __restrict__ mean, float* __restrict__ stdv) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int part = threadIdx.x >> 6;
  __shared__ float red[CS_NP][64];
  __shared__ float mu_s[64];
  float s = 0.f;
  if (c < C)
    for (int r = part; r < R; r += CS_NP) s += x[(long)r * C + c];
  red[part][threadIdx.x & 63] = s;
  __syncthreads();
  if (part == 0) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < CS_NP; ++k) t += red[k][threadIdx.x];
    const float mu = t / (float)R;
    mu_s[threadIdx.x] = mu;
    if (c < C) mean[c] = mu;
  }
  __syncthreads();
  const float mu = mu_s[threadIdx.x & 63];
  float q = 0.f;
  if (c < C)
    for (int r = part; r < R; r += CS_NP) {
      const float d = x[(long)r * C + c] - mu;
      q += d * d;
    }
  __syncthreads();  // every thread has read mu_s / red from the first pass
  red[part][threadIdx.x & 63] = q;
  __syncthreads();
  if (part == 0 && c < C) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < CS_NP; ++k) t += red[k][threadIdx.x];
    stdv[c] = sqrtf(t / (float)(R - 1));
  }
}

__global__ void standardize_kernel(const float* __restrict__ x, const float* __restrict__ mean,
                                   const float* __restrict__ stdv, float* __restrict__ y, long R, int C, float eps) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R * C) return;
  const int c = (int)(i % C);
  y[i] = (x[i] - mean[c]) / (stdv[c] + eps);
}

// dx = (dn - mean_r dn)/s - (x - mu) * A / (s^2 (R-1) sigma),  A = sum_r dn (x - mu),  s = sigma + eps
__global__ __launch_bounds__(64 * CS_NP) void standardize_bwd_kernel(const float* __restrict__ x,
                                                                    const float* __restrict__ mean,
                                                                    const float* __restrict__ stdv,
                                                                    const float* __restrict__ dn,
                                                                    float* __restrict__ dx, int R, int C, float eps) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int part = threadIdx.x >> 6;
  __shared__ float red0[CS_NP][64], red1[CS_NP][64];
  __shared__ float mdn[64], aa[64];
  const float mu = c < C ? mean[c] : 0.f;
  float s0 = 0.f, s1 = 0.f;
  if (c < C)
    for (int r = part; r < R; r += CS_NP) {
      const float d = dn[(long)r * C + c];
      s0 += d;
      s1 += d * (x[(long)r * C + c] - mu);
    }
  red0[part][threadIdx.x & 63] = s0;
  red1[part][threadIdx.x & 63] = s1;
  __syncthreads();
  if (part == 0) {
    const int l = threadIdx.x;
    float t0 = 0.f, t1 = 0.f;
#pragma unroll
    for (int k = 0; k < CS_NP; ++k) { t0 += red0[k][l]; t1 += red1[k][l]; }
    mdn[l] = t0 / (float)R;
    aa[l] = t1;
  }
  __syncthreads();
  if (c >= C) return;
  const float sg = stdv[c];
  const float sc = sg + eps;
  const float m = mdn[threadIdx.x & 63], A = aa[threadIdx.x & 63];
  const float k2 = A / (sc * sc * (float)(R - 1) * sg);
  for (int r = part; r < R; r += CS_NP) {
    const long o = (long)r * C + c;
    dx[o] = (dn[o] - m) / sc - (x[o] - mu) * k2;
  }
}

// loss = sum_i (c_ii - 1)^2 + lambd * sum_{i!=j} c_ij^2 ; partial per block, then 1 block finishes
__global__ void barlow_partial(const float* __restrict__ c, int E, float lambd, float* __restrict__ part) {
  __shared__ float red[4];
  float inv = 0.f, rd = 0.f;
  const long n = (long)E * E;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int r = (int)(i / E), col = (int)(i % E);
    const float v = c[i];
    if (r == col) inv += (v - 1.f) * (v - 1.f);
    else rd += v * v;
  }
  inv = block_sum<256>(inv, red);
  rd = block_sum<256>(rd, red);
  if (threadIdx.x == 0) { part[2 * blockIdx.x] = inv; part[2 * blockIdx.x + 1] = rd; }
}

__global__ void barlow_final(const float* __restrict__ part, int nb, float lambd, float* __restrict__ loss) {
  __shared__ float red[4];
  float inv = 0.f, rd = 0.f;
  for (int i = threadIdx.x; i < nb; i += 256) { inv += part[2 * i]; rd += part[2 * i + 1]; }
  inv = block_sum<256>(inv, red);
  rd = block_sum<256>(rd, red);
  if (threadIdx.x == 0) loss[0] = inv + lambd * rd;
}

// dc_ij = g * (i == j ? 2 (c_ii - 1) : 2 lambd c_ij)
__global__ void barlow_dc(const float* __restrict__ c, const float* __restrict__ g, float* __restrict__ dc, int E,
                          float lambd) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)E * E) return;
  const int r = (int)(i / E), col = (int)(i % E);
  const float v = c[i];
  dc[i] = g[0] * (r == col ? 2.f * (v - 1.f) : 2.f * lambd * v);
}

int nb(long n) { return (int)((n + 255) / 256); }

// ---- data-parallel Barlow (parallel.barlow_dist; dreamer.py:525-532 over the GLOBAL batch of Nt rows, this rank
// holding R of them). Forward: local column sums -> all-reduce -> barlow_center (centred rows, local column sums of
// squares) -> d1^T d2 (GEMM) -> all-reduce -> barlow_finish. Backward: barlow_dc, dn1 = n2 dc^T / Nt (GEMM),
// barlow_rowstats, barlow_dist_dx.
// d_k = x_k - sums_k / Nt, q_k = sum over this rank's rows of d_k^2 (k = 0: x1, 1: x2); grid (E / 64, 2)
__global__ __launch_bounds__(64 * CS_NP) void barlow_center_kernel(const float* __restrict__ x1,
                                                                   const float* __restrict__ x2,
                                                                   const float* __restrict__ sums, float Nt, int R, int E,
                                                                   float* __restrict__ d1, float* __restrict__ d2,
                                                                   float* __restrict__ q) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), part = threadIdx.x >> 6, k = blockIdx.y;
  const float* x = k ? x2 : x1;
  float* d = k ? d2 : d1;
  __shared__ float red[CS_NP][64];
  const float m = c < E ? sums[(long)k * E + c] / Nt : 0.f;
  float s = 0.f;
  if (c < E)
    for (int r = part; r < R; r += CS_NP) {
      const float v = x[(long)r * E + c] - m;
      d[(long)r * E + c] = v;
      s += v * v;
    }
  red[part][threadIdx.x & 63] = s;
  __syncthreads();
  if (part == 0 && c < E) {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < CS_NP; ++j) t += red[j][threadIdx.x];
    q[(long)k * E + c] = t;
  }
}
// stats = [q (2, E) | craw (E, E)] summed over ranks -> s = sqrt(q / (Nt - 1)) (2, E), c = craw / (sc1_i sc2_j) / Nt,
// n2 = d2 / sc2 (this rank's rows), z2 = (sums2 - Nt * (sums2 / Nt)) / sc2; sc = s + 1e-8. One flat index space.
__global__ void barlow_finish_kernel(const float* __restrict__ stats, const float* __restrict__ sums, float Nt, int E,
                                     const float* __restrict__ d2, int R, float* __restrict__ c,
                                     float* __restrict__ s, float* __restrict__ n2, float* __restrict__ z2) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long EE = (long)E * E, RE = (long)R * E;
  const float* q = stats;
  auto sc_of = [&](int k, int j) { return sqrtf(q[(long)k * E + j] / (Nt - 1.f)) + 1e-8f; };
  if (i < EE) {
    const int r = (int)(i / E), col = (int)(i % E);
    c[i] = stats[2L * E + i] / (sc_of(0, r) * sc_of(1, col)) / Nt;
  } else if (i < EE + RE) {
    const long o = i - EE;
    n2[o] = d2[o] / sc_of(1, (int)(o % E));
  } else if (i < EE + RE + 2L * E) {
    const long o = i - EE - RE;
    s[o] = sqrtf(q[o] / (Nt - 1.f));
  } else if (i < EE + RE + 3L * E) {
    const int j = (int)(i - EE - RE - 2L * E);
    const float t = sums[(long)E + j];
    z2[j] = (t - Nt * (t / Nt)) / sc_of(1, j);
  }
}
// s0_j = (sum_k dc[j, k] z2[k]) / Nt, A_j = (s1_j + 1e-8) sum_k dc[j, k] c[j, k]; one wave per row j
__global__ __launch_bounds__(256) void barlow_rowstats_kernel(const float* __restrict__ dc, const float* __restrict__ c,
                                                              const float* __restrict__ z2,
                                                              const float* __restrict__ s1, float Nt, int E,
                                                              float* __restrict__ s0, float* __restrict__ A) {
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (j >= E) return;
  float a = 0.f, b = 0.f;
  for (int k = lane; k < E; k += 64) {
    const float g = dc[(long)j * E + k];
    a += g * z2[k];
    b += g * c[(long)j * E + k];
  }
  a = wave_sum(a);
  b = wave_sum(b);
  if (lane == 0) {
    s0[j] = a / Nt;
    A[j] = (s1[j] + 1e-8f) * b;
  }
}
// dx1 = world * ((dn1 - s0 / Nt) / sc - (x1 - m1) * A / (sc^2 (Nt - 1) s1)), m1 = sums1 / Nt, sc = s1 + 1e-8
__global__ void barlow_dist_dx_kernel(const float* __restrict__ x1, const float* __restrict__ dn1,
                                      const float* __restrict__ sums, const float* __restrict__ s1,
                                      const float* __restrict__ s0, const float* __restrict__ A, float Nt, float world,
                                      long R, int E, float* __restrict__ dx1) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R * E) return;
  const int j = (int)(i % E);
  const float sg = s1[j], sc = sg + 1e-8f, m = sums[j] / Nt;
  dx1[i] = ((dn1[i] - s0[j] / Nt) / sc - (x1[i] - m) * (A[j] / (sc * sc * (Nt - 1.f) * sg))) * world;
}

// Metric vector: out[b] = sum over the requests r with r.out == b, in request order, of r.scale * stat_r(x_r[0:n_r])
// (stat: mean, unbiased std, min, max). Pass 1: every request is cut into chunks of SD_STAT_CHUNK elements, one
// workgroup per chunk holds its elements in registers (all loads in flight at once) and writes the chunk's
// (count, mean, M2, min, max); pass 2: one workgroup per output slot merges its requests' chunks in order (Chan's
// pairwise update) and sums the scaled statistics. Fixed order everywhere: deterministic.
constexpr int ST_PER = SD_STAT_CHUNK / 256;  // elements per thread of a chunk
__global__ __launch_bounds__(256) void stats_chunk_kernel(sd_stats s, float* __restrict__ ws) {
  __shared__ float red[8];
  const int c = blockIdx.x, tid = threadIdx.x;
  int q = 0;
  while (q + 1 < s.nreq && s.r[q + 1].chunk0 <= c) ++q;
  const sd_stat_req r = s.r[q];
  const long lo = (long)(c - r.chunk0) * SD_STAT_CHUNK;
  const long cnt = r.n - lo < SD_STAT_CHUNK ? r.n - lo : SD_STAT_CHUNK;
  float v[ST_PER];
#pragma unroll
  for (int k = 0; k < ST_PER; ++k) {
    const long i = (long)k * 256 + tid;
    v[k] = i < cnt ? r.x[lo + i] : 0.f;
  }
  float t = 0.f, mn = INFINITY, mx = -INFINITY;
#pragma unroll
  for (int k = 0; k < ST_PER; ++k) {
    const bool ok = (long)k * 256 + tid < cnt;
    t += v[k];
    mn = ok ? fminf(mn, v[k]) : mn;
    mx = ok ? fmaxf(mx, v[k]) : mx;
  }
  const float mean = block_sum<256>(t, red) / (float)cnt;
  float q2 = 0.f;
#pragma unroll
  for (int k = 0; k < ST_PER; ++k) {
    const float d = (long)k * 256 + tid < cnt ? v[k] - mean : 0.f;
    q2 += d * d;
  }
  q2 = block_sum<256>(q2, red);
  mn = -block_max<256>(-mn, red);
  mx = block_max<256>(mx, red);
  if (tid == 0) {
    float* o = ws + 5L * c;
    o[0] = (float)cnt;
    o[1] = mean;
    o[2] = q2;
    o[3] = mn;
    o[4] = mx;
  }
}
__global__ __launch_bounds__(64) void stats_merge_kernel(sd_stats s, const float* __restrict__ ws,
                                                         float* __restrict__ out) {
  const int b = blockIdx.x;
  if (threadIdx.x) return;
  float acc = 0.f;
  for (int q = 0; q < s.nreq; ++q) {
    if (s.r[q].out != b) continue;
    const sd_stat_req r = s.r[q];
    const int nc = (int)((r.n + SD_STAT_CHUNK - 1) / SD_STAT_CHUNK);
    double n = 0.0, mean = 0.0, m2 = 0.0;
    float mn = INFINITY, mx = -INFINITY;
    for (int k = 0; k < nc; ++k) {
      const float* o = ws + 5L * (r.chunk0 + k);
      const double nb = o[0], d = (double)o[1] - mean, tot = n + nb;
      mean += d * nb / tot;
      m2 += (double)o[2] + d * d * n * nb / tot;
      n = tot;
      mn = fminf(mn, o[3]);
      mx = fmaxf(mx, o[4]);
    }
    float v = (float)mean;
    if (r.kind == SD_STAT_STD) v = (float)sqrt(m2 / (n - 1.0));
    else if (r.kind == SD_STAT_MIN) v = mn;
    else if (r.kind == SD_STAT_MAX) v = mx;
    if (r.sub) v -= r.sub[0];
    if (r.div) v /= r.div[0];
    acc += r.scale * v;
  }
  out[b] = acc;
}

// weighted loss total (dreamer.py:571-576: the loss dict's `sum(v * scale)`): term i = coef_i * mean(x_i) (fixed
// reduction order), total = ((0 + s_0 m_0) + s_1 m_1) + ... in the dict's order. One workgroup.
__global__ __launch_bounds__(256) void loss_terms_fwd_kernel(sd_loss_terms L, float* __restrict__ means,
                                                             float* __restrict__ total) {
  __shared__ float red[4];
  float tot = 0.f;
  for (int i = 0; i < L.n; ++i) {
    const sd_loss_term t = L.t[i];
    float acc = 0.f;
    for (long j = threadIdx.x; j < t.n; j += 256) acc += t.x[j];
    const float m = t.coef * (block_sum<256>(acc, red) / (float)t.n);
    tot = __fadd_rn(tot, __fmul_rn(t.scale, m));
    if (threadIdx.x == 0 && means) means[i] = m;
  }
  if (threadIdx.x == 0) total[0] = tot;
}
// g_i[j] = (g_total * scale_i + g_means[i]) * coef_i / n_i: every term's input gradient in one launch (grid.y = term)
__global__ __launch_bounds__(256) void loss_terms_bwd_kernel(sd_loss_terms L, const float* __restrict__ g_total,
                                                             const float* __restrict__ g_means) {
  const sd_loss_term t = L.t[blockIdx.y];
  if (!t.g) return;
  const float g = ((g_total ? g_total[0] * t.scale : 0.f) + (g_means ? g_means[blockIdx.y] : 0.f)) * t.coef / (float)t.n;
  for (long j = (long)blockIdx.x * 256 + threadIdx.x; j < t.n; j += (long)gridDim.x * 256) t.g[j] = g;
}

// Weight layout copies, one launch for a list: mode 0 = transpose dst[b][c][r] = src[b * sb + r * sr + c]; mode 1 =
// column pad dst[b * rows + r][c] = c < cols ? src[b * sb + r * sr + c] : 0 for c < dcols. One workgroup per 64 x 64
// tile, the tiles of all entries numbered in one flat range (no workgroup idles on a small entry while another walks
// a large one); a transpose moves the tile through LDS with 16-byte loads and stores on both HBM sides where the
// entry's strides allow it (4-byte accesses otherwise and at ragged edges).
namespace lcopy {
constexpr int TS = 64, LD = TS + 4;
__device__ inline int tiles_of(const sd_layout_copy& e) {
  return e.batch * ((e.rows + TS - 1) / TS) * (((e.mode ? e.dcols : e.cols) + TS - 1) / TS);
}
}  // namespace lcopy

__global__ __launch_bounds__(256) void layout_copy_kernel(sd_layout_copies L) {
  using namespace lcopy;
  __shared__ float tile[TS * LD];
  int id = blockIdx.x, ei = 0;
  for (; ei < L.n; ++ei) {
    const int n = tiles_of(L.e[ei]);
    if (id < n) break;
    id -= n;
  }
  if (ei >= L.n) return;
  const sd_layout_copy& e = L.e[ei];
  const int tc = ((e.mode ? e.dcols : e.cols) + TS - 1) / TS, tr = (e.rows + TS - 1) / TS;
  const int b = id / (tr * tc), rem = id % (tr * tc), r0 = (rem / tc) * TS, c0 = (rem % tc) * TS;
  const float* src = e.src + (long)b * e.sb;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;  // 16 rows of 16 four-column groups
  if (e.mode == 1) {
    const long ld = e.dld ? e.dld : e.dcols;
    const int c = c0 + (int)(threadIdx.x & 63);  // a wave per row, lanes on consecutive columns
    for (int i = threadIdx.x >> 6; i < TS; i += 4) {
      const int r = r0 + i;
      if (r >= e.rows) break;
      if (c < e.dcols) e.dst[((long)b * e.rows + r) * ld + c] = c < e.cols ? src[(long)r * e.sr + c] : 0.f;
    }
    return;
  }
  const bool vin = ((e.sr | e.sb) & 3) == 0 && ((uintptr_t)e.src & 15) == 0;
  const bool vout = (e.rows & 3) == 0 && ((uintptr_t)e.dst & 15) == 0;
  const int c = c0 + 4 * tx;
#pragma unroll
  for (int i = 0; i < TS / 16; ++i) {
    const int rl = ty + 16 * i, r = r0 + rl;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < e.rows) {
      const float* p = src + (long)r * e.sr + c;
      if (vin && c + 3 < e.cols) {
        v = *reinterpret_cast<const float4*>(p);
      } else {
        if (c < e.cols) v.x = p[0];
        if (c + 1 < e.cols) v.y = p[1];
        if (c + 2 < e.cols) v.z = p[2];
        if (c + 3 < e.cols) v.w = p[3];
      }
    }
    *reinterpret_cast<float4*>(&tile[rl * LD + 4 * tx]) = v;
  }
  __syncthreads();
  float* dst = e.dst + (long)b * e.rows * e.cols;
  const int r = r0 + 4 * tx;  // dst columns r .. r + 3
#pragma unroll
  for (int i = 0; i < TS / 16; ++i) {
    const int cl = ty + 16 * i, cc = c0 + cl;  // dst row
    if (cc >= e.cols) break;
    float4 v;
    v.x = tile[(4 * tx + 0) * LD + cl];
    v.y = tile[(4 * tx + 1) * LD + cl];
    v.z = tile[(4 * tx + 2) * LD + cl];
    v.w = tile[(4 * tx + 3) * LD + cl];
    float* p = dst + (long)cc * e.rows + r;
    if (vout && r + 3 < e.rows) {
      *reinterpret_cast<float4*>(p) = v;
    } else {
      if (r < e.rows) p[0] = v.x;
      if (r + 1 < e.rows) p[1] = v.y;
      if (r + 2 < e.rows) p[2] = v.z;
      if (r + 3 < e.rows) p[3] = v.w;
    }
  }
}

// episode flags of a batch (dreamer.py:571-660 operands): is_last / is_terminal (bool bytes) -> f32 last, term and
// cont = 1 - term, for the continue-head target, the replay lambda-return and the replay-value weights
__global__ void episode_flags_kernel(const unsigned char* __restrict__ is_last, const unsigned char* __restrict__ is_term,
                                     long n, float* __restrict__ last, float* __restrict__ term,
                                     float* __restrict__ cont) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float l = is_last[i] ? 1.f : 0.f, t = is_term[i] ? 1.f : 0.f;
  last[i] = l;
  term[i] = t;
  cont[i] = 1.f - t;
}

// an empty dispatch whose name and grid (tag workgroups) a kernel trace can find: bench.py brackets its timed steps
// with tags 1 and 2 so tools/kernel_table.py counts only the dispatches of those steps
__global__ void k_trace_mark(int tag) {}

// Shader clock under an f32 MFMA load (MI355X_MICROARCH.md 'DVFS give-back' item 6): every wave runs `iters` dependent
// v_mfma_f32_16x16x4_f32 chains on non-trivial operands; lane 0 of wave 0 stamps s_memtime (shader cycles) and
// s_memrealtime (100 MHz) around the loop and writes (cycles, ticks) for its workgroup to stamps[2 * wg]. The stamps go
// to their own buffer; the accumulators feed one guarded store that never fires (keeps the loop).
__global__ __launch_bounds__(256) void k_clock_probe(long long* stamps, float* sink, int iters) {
  const int lane = threadIdx.x & 63;
  float a = 1.f + 1e-3f * lane, b = 0.5f - 1e-4f * threadIdx.x;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
  const long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, a, acc1, 0, 0, 0);
    acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, acc2, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, b, acc3, 0, 0, 0);
  }
  const long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    stamps[2 * blockIdx.x] = t1 - t0;
    stamps[2 * blockIdx.x + 1] = r1 - r0;
  }
  const float s = acc0[0] + acc1[1] + acc2[2] + acc3[3];
  if (s == -1.2345e30f) sink[blockIdx.x] = s;
}

}  // namespace

extern "C" int sd_clock_probe(long long* stamps, float* sink, int nwg, int iters, sd_stream s) {
  if (nwg < 1 || nwg > 4096 || iters < 1) return SD_EARG;
  k_clock_probe<<<nwg, 256, 0, (hipStream_t)s>>>(stamps, sink, iters);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_multi_stats(const sd_stats* s, float* workspace, float* out, int nout, sd_stream st) {
  if (!s || s->nreq <= 0 || s->nreq > SD_MAX_STATS || nout <= 0 || !workspace) return SD_EARG;
  int chunks = 0;
  for (int q = 0; q < s->nreq; ++q) {
    const sd_stat_req& r = s->r[q];
    if (r.out < 0 || r.out >= nout || r.n <= 0 || !r.x || r.chunk0 != chunks) return SD_EARG;
    chunks += (int)((r.n + SD_STAT_CHUNK - 1) / SD_STAT_CHUNK);
  }
  stats_chunk_kernel<<<chunks, 256, 0, (hipStream_t)st>>>(*s, workspace);
  SD_LAUNCH_CHECK();
  stats_merge_kernel<<<nout, 64, 0, (hipStream_t)st>>>(*s, workspace, out);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_loss_terms_fwd(const sd_loss_terms* L, float* means, float* total, sd_stream s) {
  if (!L || L->n < 1 || L->n > SD_MAX_LOSS_TERMS || !total) return SD_EARG;
  for (int i = 0; i < L->n; ++i)
    if (!L->t[i].x || L->t[i].n <= 0) return SD_EARG;
  loss_terms_fwd_kernel<<<1, 256, 0, (hipStream_t)s>>>(*L, means, total);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_loss_terms_bwd(const sd_loss_terms* L, const float* g_total, const float* g_means, sd_stream s) {
  if (!L || L->n < 1 || L->n > SD_MAX_LOSS_TERMS) return SD_EARG;
  long nmax = 0;
  for (int i = 0; i < L->n; ++i) nmax = L->t[i].n > nmax ? L->t[i].n : nmax;
  if (nmax <= 0) return SD_EARG;
  const int gx = (int)(nmax < 256L * 64 ? (nmax + 255) / 256 : 64);
  loss_terms_bwd_kernel<<<dim3(gx, L->n), 256, 0, (hipStream_t)s>>>(*L, g_total, g_means);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_layout_copies_run(const sd_layout_copies* L, sd_stream s) {
  if (!L || L->n < 1 || L->n > SD_MAX_LAYOUT_COPIES) return SD_EARG;
  long total = 0;
  for (int i = 0; i < L->n; ++i) {
    const sd_layout_copy& e = L->e[i];
    if (!e.src || !e.dst || e.batch < 1 || e.rows < 1 || e.cols < 1 || e.mode < 0 || e.mode > 1) return SD_EARG;
    if (e.mode == 1 && e.dcols < e.cols) return SD_EARG;
    total += (long)e.batch * ((e.rows + lcopy::TS - 1) / lcopy::TS) *
             (((e.mode ? e.dcols : e.cols) + lcopy::TS - 1) / lcopy::TS);
  }
  if (total > 0x7fffffffL) return SD_ESHAPE;
  layout_copy_kernel<<<dim3((unsigned)total), 256, 0, (hipStream_t)s>>>(*L);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_episode_flags(const uint8_t* is_last, const uint8_t* is_term, long n, float* last, float* term,
                                float* cont, sd_stream s) {
  if (n <= 0) return SD_OK;
  if (!is_last || !is_term || !last || !term || !cont) return SD_EARG;
  episode_flags_kernel<<<nb(n), 256, 0, (hipStream_t)s>>>(is_last, is_term, n, last, term, cont);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_trace_mark(int tag, sd_stream s) {
  if (tag < 1 || tag > 64) return SD_EARG;
  k_trace_mark<<<tag, 64, 0, (hipStream_t)s>>>(tag);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_u8_to_f32(const uint8_t* in, float* out, long n, float shift, sd_stream s) {
  if (n <= 0) return SD_OK;
  u8_to_f32<<<nb(n), 256, 0, (hipStream_t)s>>>(in, out, n, shift);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
extern "C" int sd_u8_image_inputs(const uint8_t* in, float* img, float* enc, long pixels, int C, int Cp, float shift,
                                  sd_stream s) {
  if (pixels <= 0) return SD_OK;
  if (C < 1 || Cp < C || !in || !enc) return SD_EARG;
  u8_image_inputs_kernel<<<nb(pixels), 256, 0, (hipStream_t)s>>>(in, img, enc, pixels, C, Cp, shift);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
extern "C" int sd_pad_channels(const float* in, float* out, long pixels, int C, int Cp, float shift, sd_stream s) {
  if (pixels <= 0) return SD_OK;
  if (C < 1 || Cp < C) return SD_ESHAPE;
  pad_channels_kernel<<<nb(pixels * Cp), 256, 0, (hipStream_t)s>>>(in, out, pixels, C, Cp, shift);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
extern "C" int sd_symlog(const float* x, float* y, long n, sd_stream s) {
  if (n <= 0) return SD_OK;
  symlog_kernel<<<nb(n), 256, 0, (hipStream_t)s>>>(x, y, n);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
extern "C" int sd_action_norm(const float* a, float* y, long n, sd_stream s) {
  if (n <= 0) return SD_OK;
  action_norm_kernel<<<nb(n), 256, 0, (hipStream_t)s>>>(a, y, n);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
extern "C" int sd_mask_rows(const float* x, const uint8_t* mask, long mask_stride, float* y, long rows, int width,
                            sd_stream s) {
  if (rows <= 0) return SD_OK;
  mask_rows_kernel<<<nb(rows * width), 256, 0, (hipStream_t)s>>>(x, mask, mask_stride, y, rows, width);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
extern "C" int sd_fill_gumbel(float* out, long n, uint64_t seed, int stream_id, int step, long offset, sd_stream s) {
  if (n <= 0) return SD_OK;
  fill_gumbel<<<nb(n), 256, 0, (hipStream_t)s>>>(out, n, seed, stream_id, step, offset);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
extern "C" int sd_fill_normal(float* out, long n, uint64_t seed, int stream_id, int step, long offset, sd_stream s) {
  if (n <= 0) return SD_OK;
  fill_normal<<<nb(n), 256, 0, (hipStream_t)s>>>(out, n, seed, stream_id, step, offset);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
extern "C" int sd_colstats(const float* x, int R, int C, float* mean, float* stdv, sd_stream s) {
  if (R <= 1 || C <= 0) return SD_EARG;
  colstats_kernel<<<(C + 63) / 64, 64 * CS_NP, 0, (hipStream_t)s>>>(x, R, C, mean, stdv);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
extern "C" int sd_standardize(const float* x, const float* mean, const float* stdv, float* y, long R, int C, float eps,
                              sd_stream s) {
  if (R <= 0) return SD_OK;
  standardize_kernel<<<nb(R * C), 256, 0, (hipStream_t)s>>>(x, mean, stdv, y, R, C, eps);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
extern "C" int sd_standardize_bwd(const float* x, const float* mean, const float* stdv, const float* dn, float* dx,
                                  int R, int C, float eps, sd_stream s) {
  if (R <= 1) return SD_EARG;
  standardize_bwd_kernel<<<(C + 63) / 64, 64 * CS_NP, 0, (hipStream_t)s>>>(x, mean, stdv, dn, dx, R, C, eps);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
extern "C" int sd_barlow_loss(const float* c, int E, float lambd, float* partial, int nblocks, float* loss,
                              sd_stream s) {
  barlow_partial<<<nblocks, 256, 0, (hipStream_t)s>>>(c, E, lambd, partial);
  SD_LAUNCH_CHECK();
  barlow_final<<<1, 256, 0, (hipStream_t)s>>>(partial, nblocks, lambd, loss);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
extern "C" int sd_barlow_center(const float* x1, const float* x2, const float* sums, float Nt, int R, int E, float* d1,
                                float* d2, float* q, sd_stream s) {
  if (R < 0 || E <= 0) return SD_ESHAPE;
  barlow_center_kernel<<<dim3((E + 63) / 64, 2), 64 * CS_NP, 0, (hipStream_t)s>>>(x1, x2, sums, Nt, R, E, d1, d2, q);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
extern "C" int sd_barlow_finish(const float* stats, const float* sums, float Nt, int E, const float* d2, int R, float* c,
                                float* stdv, float* n2, float* z2, sd_stream s) {
  if (R < 0 || E <= 0) return SD_ESHAPE;
  const long n = (long)E * E + (long)R * E + 3L * E;
  barlow_finish_kernel<<<nb(n), 256, 0, (hipStream_t)s>>>(stats, sums, Nt, E, d2, R, c, stdv, n2, z2);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
extern "C" int sd_barlow_rowstats(const float* dc, const float* c, const float* z2, const float* s1, float Nt, int E,
                                  float* s0, float* A, sd_stream s) {
  if (E <= 0) return SD_ESHAPE;
  barlow_rowstats_kernel<<<(E + 3) / 4, 256, 0, (hipStream_t)s>>>(dc, c, z2, s1, Nt, E, s0, A);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
extern "C" int sd_barlow_dist_dx(const float* x1, const float* dn1, const float* sums, const float* s1, const float* s0,
                                 const float* A, float Nt, float world, long R, int E, float* dx1, sd_stream s) {
  if (R < 0 || E <= 0) return SD_ESHAPE;
  if (R == 0) return SD_OK;
  barlow_dist_dx_kernel<<<nb(R * E), 256, 0, (hipStream_t)s>>>(x1, dn1, sums, s1, s0, A, Nt, world, R, E, dx1);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
extern "C" int sd_barlow_dc(const float* c, const float* g, float* dc, int E, float lambd, sd_stream s) {
  barlow_dc<<<nb((long)E * E), 256, 0, (hipStream_t)s>>>(c, g, dc, E, lambd);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

// ---- InfoNCE (dreamer.py:533-542): cross_entropy(logits - rowmax, arange) over the rows of x1 x2^T.
// Row r's label column is r + label_off (data parallel: this rank's rows against every rank's x2). One workgroup
// per row: max, log-sum-exp (fixed-order block reductions), loss_r = lse_r - l[r][r + off]; the mean over rows is a
// second single-block kernel (deterministic). Backward: dl[r][c] = g * scale * (softmax(l_r)[c] - [c == r + off]).
namespace {
__global__ __launch_bounds__(256) void infonce_rows(const float* __restrict__ l, long ld, int ncol, long off,
                                                    float* __restrict__ row_loss, float* __restrict__ lse) {
  __shared__ float red[4];
  const int r = blockIdx.x;
  const float* x = l + (long)r * ld;
  float m = -INFINITY;
  for (int c = threadIdx.x; c < ncol; c += 256) m = fmaxf(m, x[c]);
  m = wave_max(m);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float s = 0.f;
  for (int c = threadIdx.x; c < ncol; c += 256) s += expf(x[c] - m);
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) {
    const float v = m + logf(s);
    lse[r] = v;
    row_loss[r] = v - x[r + off];
  }
}
__global__ __launch_bounds__(256) void mean_kernel(const float* __restrict__ v, int n, float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += v[i];
  s = block_sum<256>(s, red);
  if (threadIdx.x == 0) out[0] = s / (float)n;
}
__global__ void infonce_bwd_kernel(const float* __restrict__ l, long ld, int n, int ncol, long off,
                                   const float* __restrict__ lse, const float* __restrict__ g, float scale,
                                   float* __restrict__ dl) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)n * ncol) return;
  const int r = (int)(i / ncol), c = (int)(i - (long)r * ncol);
  const float p = expf(l[(long)r * ld + c] - lse[r]);
  dl[(long)r * ncol + c] = g[0] * scale * (p - (c == r + off ? 1.f : 0.f));
}
}  // namespace

extern "C" int sd_infonce_fwd(const float* logits, long ld, int n, int ncol, long label_off, float* row_loss,
                              float* lse, float* loss, sd_stream s) {
  if (n <= 0) return SD_OK;
  if (label_off < 0 || label_off + n > ncol) return SD_EARG;
  infonce_rows<<<n, 256, 0, (hipStream_t)s>>>(logits, ld, ncol, label_off, row_loss, lse);
  SD_LAUNCH_CHECK();
  mean_kernel<<<1, 256, 0, (hipStream_t)s>>>(row_loss, n, loss);
  SD_LAUNCH_CHECK();
  return SD_OK;
}
extern "C" int sd_infonce_bwd(const float* logits, long ld, int n, int ncol, long label_off, const float* lse,
                              const float* g, float scale, float* dlogits, sd_stream s) {
  if (n <= 0) return SD_OK;
  infonce_bwd_kernel<<<nb((long)n * ncol), 256, 0, (hipStream_t)s>>>(logits, ld, n, ncol, label_off, lse, g, scale,
                                                                     dlogits);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

// ---- replay slices (utils/buffer.py:27-53 semantics, HBM storage laid out (capacity, env, row)): every key of a
// batch of B slices gathered in ONE launch straight into the consumer's buffers, and the latent write-back as one
// scatter. Slice b starts at (t0, e) = starts[pick[b]]; key k copies steps j = 0..steps-1 of time (t0 + shift + j) %
// cap (data keys: shift 1, the action one step back: shift 0, the initial latent: steps 1, shift 0). A storage row
// that several slices write back takes the value of the slice with the largest b.
namespace {
__global__ __launch_bounds__(256) void slices_kernel(sd_slice_keys ks, const int64_t* __restrict__ starts,
                                                     const int64_t* __restrict__ pick, int B, int L, long cap, int E,
                                                     int64_t* __restrict__ t_out, int64_t* __restrict__ e_out,
                                                     int scatter) {
  const int row = blockIdx.x, k = blockIdx.y;
  const sd_slice_key key = ks.k[k];
  const int b = row / L, j = row - b * L;
  if (b >= B || j >= key.steps) return;
  const int64_t t0 = starts[2 * pick[b]], e = starts[2 * pick[b] + 1];
  const long t = (t0 + key.shift + j) % cap;
  if (scatter) {
    // overlapping slices write one storage row several times: the slice with the largest b wins (a sequential
    // scatter in row order), so the write-back is deterministic (torch's index_put with duplicates is not)
    for (int b2 = b + 1; b2 < B; ++b2) {
      const int64_t s2 = starts[2 * pick[b2]];
      if (starts[2 * pick[b2] + 1] == e && ((t - s2 - key.shift) % cap + cap) % cap < key.steps) return;
    }
  }
  if (k == 0 && threadIdx.x == 0 && t_out && !scatter) {  // index of the data rows for the write-back
    const long tt = (t0 + 1 + j) % cap;
    t_out[(long)b * L + j] = tt;
    e_out[(long)b * L + j] = e;
  }
  char* st = (char*)key.storage + ((long)t * E + e) * key.row_bytes;
  char* bf = (char*)key.batch + ((long)b * key.steps + j) * key.row_bytes;
  const char* src = scatter ? bf : st;
  char* dst = scatter ? st : bf;
  if ((key.row_bytes & 15) == 0 && (((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
    for (long i = threadIdx.x; i < key.row_bytes / 16; i += 256)
      reinterpret_cast<int4*>(dst)[i] = reinterpret_cast<const int4*>(src)[i];
  } else {
    for (long i = threadIdx.x; i < key.row_bytes; i += 256) dst[i] = src[i];
  }
}
}  // namespace

namespace {
__global__ void replay_pick_kernel(uint64_t seed, uint32_t draw, long nstarts, int B, int64_t* __restrict__ pick) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) pick[b] = sd_uniform_int(seed, SD_STREAM_REPLAY, draw, (uint64_t)b, (int)nstarts);
}
}  // namespace

extern "C" int sd_replay_pick(uint64_t seed, uint32_t draw, long nstarts, int B, int64_t* pick, sd_stream s) {
  if (B < 0 || nstarts < 1 || nstarts > 0x7fffffffL || (B > 0 && !pick)) return SD_EARG;
  if (B == 0) return SD_OK;
  replay_pick_kernel<<<(B + 255) / 256, 256, 0, (hipStream_t)s>>>(seed, draw, nstarts, B, pick);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_replay_slices(const sd_slice_keys* keys, const int64_t* starts, const int64_t* pick, int B, int L,
                                long cap, int E, int64_t* t_idx, int64_t* e_idx, int scatter, sd_stream s) {
  if (!keys || keys->n < 0 || keys->n > SD_MAX_SLICE_KEYS) return SD_EARG;
  if (B <= 0 || keys->n == 0) return SD_OK;
  for (int k = 0; k < keys->n; ++k)
    if (keys->k[k].steps > L || keys->k[k].steps < 0 || !keys->k[k].storage || !keys->k[k].batch) return SD_EARG;
  slices_kernel<<<dim3(B * L, keys->n), 256, 0, (hipStream_t)s>>>(*keys, starts, pick, B, L, cap, E, t_idx, e_idx,
                                                                    scatter);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

// ---- r2dreamer image augmentation (Dreamer._augment_images / random_translate, dreamer.py:716-729,845-880):
// replicate-pad by `pad`, shift by an integer (sx, sy) in [0, 2 pad] per slice (same_across_time) or per image.
// Shifts from Philox (SD_STREAM_AUG, step 0): index (row * 2 + axis) or ((row * T + t) * 2 + axis), axis 0 = x,
// 1 = y; row = global slice row (row_offset + b).
//   nearest (aug.bilinear False): out[y][x] = in[clamp(y + sy - pad)][clamp(x + sx - pad)], the pixel centres the
//     reference's grid lands on;
//   bilinear (aug.bilinear True, the default): the reference's F.grid_sample(bilinear, zeros, align_corners False)
//     arithmetic restated in f32 — the linspace grid (fma(step, k, start) below half, fma(-step, n-1-k, end) above),
//     + shift * 2 / padded size, unnormalised as fma(g + 1, size / 2, -0.5), corner weights from floor, and the
//     four corners accumulated as one fma chain (nw first). The grid misses the pixel centres by float rounding,
//     so weights of ~6e-8 mix in the neighbours; the restatement reproduces them bit for bit (torch CPU, pinned by
//     tests/test_gpu_ops.py::test_random_translate_bilinear_matches_grid_sample). The Barlow targets are
//     sensitive enough to those last bits that the first conv layer's gradient moves visibly without them.
namespace {
// torch.linspace(-1 + 1/n, 1 - 1/n, n)[k] in f32 (CPU kernel: f32 step, fma from the nearer end)
SD_DEV float grid_coord(int n, int k) {
  const float start = (float)(-1.0 + 1.0 / n), end = (float)(1.0 - 1.0 / n);
  const float step = __fdiv_rn(__fsub_rn(end, start), (float)(n - 1));
  return k < n / 2 ? __builtin_fmaf(step, (float)k, start) : __builtin_fmaf(-step, (float)(n - 1 - k), end);
}

// padded-image pixel (zeros outside the padded frame, replicate edges inside)
SD_DEV float padded_px(const float* img, int H, int W, int C, int pad, int yp, int xp, int c) {
  if (yp < 0 || yp >= H + 2 * pad || xp < 0 || xp >= W + 2 * pad) return 0.f;
  const int yy = min(max(yp - pad, 0), H - 1), xx = min(max(xp - pad, 0), W - 1);
  return img[((long)yy * W + xx) * C + c];
}

__global__ void random_translate_kernel(const float* __restrict__ in, float* __restrict__ out, int N, int T, int H,
                                        int W, int C, int pad, uint64_t seed, const uint64_t* seed_ptr,
                                        long row_offset, int same_across_time, int bilinear) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)N * H * W * C;
  if (i >= total) return;
  const int c = (int)(i % C);
  long r = i / C;
  const int x = (int)(r % W);
  r /= W;
  const int y = (int)(r % H);
  const int n = (int)(r / H);
  const int b = n / T, t = n - b * T;
  const uint64_t sd = seed + (seed_ptr ? *seed_ptr : 0ull);
  const uint64_t base = same_across_time ? (uint64_t)(row_offset + b) * 2 : ((uint64_t)(row_offset + b) * T + t) * 2;
  const int sx = sd_uniform_int(sd, SD_STREAM_AUG, 0, base, 2 * pad + 1);
  const int sy = sd_uniform_int(sd, SD_STREAM_AUG, 0, base + 1, 2 * pad + 1);
  const float* img = in + (long)n * H * W * C;
  if (!bilinear) {
    const int yy = min(max(y + sy - pad, 0), H - 1), xx = min(max(x + sx - pad, 0), W - 1);
    out[i] = img[((long)yy * W + xx) * C + c];
    return;
  }
  const int Hp = H + 2 * pad, Wp = W + 2 * pad;
  const float gx = __fadd_rn(grid_coord(Wp, x), __fdiv_rn((float)sx * 2.f, (float)Wp));
  const float gy = __fadd_rn(grid_coord(Hp, y), __fdiv_rn((float)sy * 2.f, (float)Hp));
  const float ix = __builtin_fmaf(__fadd_rn(gx, 1.f), (float)Wp * 0.5f, -0.5f);
  const float iy = __builtin_fmaf(__fadd_rn(gy, 1.f), (float)Hp * 0.5f, -0.5f);
  const float x0 = floorf(ix), y0 = floorf(iy);
  const float we = __fsub_rn(ix, x0), ww = __fsub_rn(1.f, we), ws = __fsub_rn(iy, y0), wn = __fsub_rn(1.f, ws);
  const int xi = (int)x0, yi = (int)y0;
  const float nw = padded_px(img, H, W, C, pad, yi, xi, c), ne = padded_px(img, H, W, C, pad, yi, xi + 1, c);
  const float sw = padded_px(img, H, W, C, pad, yi + 1, xi, c), se = padded_px(img, H, W, C, pad, yi + 1, xi + 1, c);
  float v = __fmul_rn(nw, __fmul_rn(wn, ww));
  v = __builtin_fmaf(ne, __fmul_rn(wn, we), v);
  v = __builtin_fmaf(sw, __fmul_rn(ws, ww), v);
  out[i] = __builtin_fmaf(se, __fmul_rn(ws, we), v);
}
}  // namespace

extern "C" int sd_random_translate(const float* in, float* out, int B, int T, int H, int W, int C, int pad,
                                   uint64_t seed, const uint64_t* seed_ptr, long row_offset, int same_across_time,
                                   int bilinear, sd_stream s) {
  const long total = (long)B * T * H * W * C;
  if (total <= 0) return SD_OK;
  if (pad < 0) return SD_EARG;
  random_translate_kernel<<<nb(total), 256, 0, (hipStream_t)s>>>(in, out, B * T, T, H, W, C, pad, seed, seed_ptr,
                                                                 row_offset, same_across_time, bilinear);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

// ---- timeline marks (profiling aid): one thread stores the constant-rate wall clock into buf[idx]; enqueued on a
// stream (and capturable into a HIP graph) it timestamps the point the stream has reached
namespace {
__global__ void mark_kernel(unsigned long long* buf, int idx) { buf[idx] = wall_clock64(); }
}  // namespace

extern "C" int sd_mark(uint64_t* buf, int idx, sd_stream stream) {
  if (!buf || idx < 0) return SD_EARG;
  mark_kernel<<<1, 1, 0, (hipStream_t)stream>>>(reinterpret_cast<unsigned long long*>(buf), idx);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_wall_clock_khz(int device) {
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, device) != hipSuccess) return SD_EARG;
  return v;
}
