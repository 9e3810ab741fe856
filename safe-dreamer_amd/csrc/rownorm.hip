// Row-wise RMSNorm (+ SiLU) forward/backward: the `Linear -> RMSNorm(eps) -> SiLU` body of every MLP in the
// model (rssm.py:16-31,106-130; networks.py:88-96,252-255,313-336) and RMSNorm2D on channels-last conv
// activations (a channels-last row is exactly the reference's permuted RMSNorm row).
//
// One "team" of TEAM lanes owns a row (TEAM = 16/32/64 inside one wave, or 256 = the whole block for wide
// rows); each lane keeps VPT columns in registers, so x is read once and y written once (HBM-bound: 8 B/elt).
// Backward recomputes xhat and the SiLU derivative from (x, rstd) and emits the RMSNorm-weight gradient as
// per-block partial sums (reduced by sd_colsum in a fixed order: deterministic).
#include "common.h"
#include "sdhip.h"

extern "C" int sd_colsum_ws(const float* in, float* out, int R, int N, long ld, int accumulate, float* workspace,
                            sd_stream stream);

namespace {

template <int TEAM>
SD_DEV float team_sum(float v, float* red) {
  if (TEAM <= 64) return group_sum<TEAM>(v);
  return block_sum<256>(v, red);
}

template <int TEAM, int VPT>
__global__ __launch_bounds__(256) void rms_fwd(const float* __restrict__ x, const float* __restrict__ w,
                                               float* __restrict__ y, float* __restrict__ rstd, int M, int N,
                                               float eps, int act, long ldy) {
  constexpr int TPB = 256 / TEAM;  // teams per block
  __shared__ float red[4];
  const int team = threadIdx.x / TEAM, t = threadIdx.x % TEAM;
  for (long row = (long)blockIdx.x * TPB + team; row < M; row += (long)gridDim.x * TPB) {
    const float* xr = x + row * N;
    float v[VPT];
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int c = t + j * TEAM;
      v[j] = c < N ? xr[c] : 0.f;
      ss += v[j] * v[j];
    }
    ss = team_sum<TEAM>(ss, red);
    const float r = rsqrtf(ss / (float)N + eps);
    if (t == 0 && rstd) rstd[row] = r;
    float* yr = y + row * ldy;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int c = t + j * TEAM;
      if (c < N) {
        float z = v[j] * r * w[c];
        yr[c] = act ? siluf_(z) : z;
      }
    }
    if (TEAM == 256) __syncthreads();
  }
}

// dx = r * (g - xhat * mean(g * xhat)),  g = dz * w,  dz = dy * silu'(z);  dw_part[block] = sum_rows dz * xhat
template <int TEAM, int VPT>
__global__ __launch_bounds__(256) void rms_bwd(const float* __restrict__ x, const float* __restrict__ w,
                                               const float* __restrict__ rstd, const float* __restrict__ dy,
                                               float* __restrict__ dx, float* __restrict__ dw_part, int M, int N,
                                               int act, int accumulate_dx, long ldy, long ldx) {
  constexpr int TPB = 256 / TEAM;
  __shared__ float red[4];
  __shared__ float wpart[TEAM == 256 ? 1 : TPB * TEAM * VPT];
  const int team = threadIdx.x / TEAM, t = threadIdx.x % TEAM;
  float dwacc[VPT];
#pragma unroll
  for (int j = 0; j < VPT; ++j) dwacc[j] = 0.f;
  for (long row = (long)blockIdx.x * TPB + team; row < M; row += (long)gridDim.x * TPB) {
    const float* xr = x + row * N;
    const float* dyr = dy + row * ldy;
    const float r = rstd[row];
    float xh[VPT], g[VPT];
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int c = t + j * TEAM;
      xh[j] = 0.f;
      g[j] = 0.f;
      if (c < N) {
        const float xv = xr[c] * r;
        const float wv = w[c];
        float dz = dyr[c];
        if (act) {
          const float z = xv * wv;
          const float s = sigmoidf_(z);
          dz *= s * (1.f + z * (1.f - s));
        }
        xh[j] = xv;
        g[j] = dz * wv;
        dwacc[j] += dz * xv;
        dot += g[j] * xv;
      }
    }
    dot = team_sum<TEAM>(dot, red) / (float)N;
    float* dxr = dx + row * ldx;
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int c = t + j * TEAM;
      if (c < N) {
        const float v = r * (g[j] - xh[j] * dot);
        dxr[c] = accumulate_dx ? dxr[c] + v : v;
      }
    }
    if (TEAM == 256) __syncthreads();
  }
  if (!dw_part) return;
  if (TEAM == 256) {
#pragma unroll
    for (int j = 0; j < VPT; ++j) {
      const int c = t + j * TEAM;
      if (c < N) dw_part[(long)blockIdx.x * N + c] = dwacc[j];
    }
  } else {
#pragma unroll
    for (int j = 0; j < VPT; ++j) wpart[(team * VPT + j) * TEAM + t] = dwacc[j];
    __syncthreads();
    for (int c = threadIdx.x; c < N; c += 256) {
      const int j = c / TEAM, tt = c % TEAM;
      float s = 0.f;
      for (int tm = 0; tm < TPB; ++tm) s += wpart[(tm * VPT + j) * TEAM + tt];
      dw_part[(long)blockIdx.x * N + c] = s;
    }
  }
}

// Vector forms for rows of N = 256 * NV (the MLPs' 256..1024-wide layers): a wave per row, each lane NV float4 of
// contiguous columns (lane t: columns 256 j + 4 t .. + 3), so every load / store is one dwordx4 instead of four
// strided dwords (rms_fwd / rms_bwd above: 1.5 TB/s on the imagined actor / value layers, round-5 kernel table)
template <int NV>
__global__ __launch_bounds__(256) void rms_fwd_v(const float* __restrict__ x, const float* __restrict__ w,
                                                 float* __restrict__ y, float* __restrict__ rstd, int M, float eps,
                                                 int act, long ldy) {
  constexpr int N = 256 * NV;
  const int team = threadIdx.x >> 6, t = threadIdx.x & 63;
  f32x4 wv[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) wv[j] = *reinterpret_cast<const f32x4*>(w + j * 256 + 4 * t);
  for (long row = (long)blockIdx.x * 4 + team; row < M; row += (long)gridDim.x * 4) {
    f32x4 v[NV];
    float ss = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      v[j] = *reinterpret_cast<const f32x4*>(x + row * N + j * 256 + 4 * t);
      ss += (v[j][0] * v[j][0] + v[j][1] * v[j][1]) + (v[j][2] * v[j][2] + v[j][3] * v[j][3]);
    }
    ss = group_sum<64>(ss);
    const float r = rsqrtf(ss / (float)N + eps);
    if (t == 0 && rstd) rstd[row] = r;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float z = v[j][e] * r * wv[j][e];
        o[e] = act ? siluf_(z) : z;
      }
      *reinterpret_cast<f32x4*>(y + row * ldy + j * 256 + 4 * t) = o;
    }
  }
}

template <int NV>
__global__ __launch_bounds__(256) void rms_bwd_v(const float* __restrict__ x, const float* __restrict__ w,
                                                 const float* __restrict__ rstd, const float* __restrict__ dy,
                                                 float* __restrict__ dx, float* __restrict__ dw_part, int M, int act,
                                                 int accumulate_dx, long ldy, long ldx) {
  constexpr int N = 256 * NV;
  __shared__ f32x4 wpart[4][64 * NV];
  const int team = threadIdx.x >> 6, t = threadIdx.x & 63;
  f32x4 wv[NV], dwacc[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    wv[j] = *reinterpret_cast<const f32x4*>(w + j * 256 + 4 * t);
    dwacc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (long row = (long)blockIdx.x * 4 + team; row < M; row += (long)gridDim.x * 4) {
    const float r = rstd[row];
    f32x4 xh[NV], g[NV];
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const f32x4 xv = *reinterpret_cast<const f32x4*>(x + row * N + j * 256 + 4 * t);
      const f32x4 dv = *reinterpret_cast<const f32x4*>(dy + row * ldy + j * 256 + 4 * t);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xn = xv[e] * r, wn = wv[j][e];
        float dz = dv[e];
        if (act) {
          const float z = xn * wn;
          const float sg = sigmoidf_(z);
          dz *= sg * (1.f + z * (1.f - sg));
        }
        xh[j][e] = xn;
        g[j][e] = dz * wn;
        dwacc[j][e] += dz * xn;
        dot += g[j][e] * xn;
      }
    }
    dot = group_sum<64>(dot) / (float)N;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      float* q = dx + row * ldx + j * 256 + 4 * t;
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = r * (g[j][e] - xh[j][e] * dot);
      if (accumulate_dx) o += *reinterpret_cast<const f32x4*>(q);
      *reinterpret_cast<f32x4*>(q) = o;
    }
  }
  if (!dw_part) return;
#pragma unroll
  for (int j = 0; j < NV; ++j) wpart[team][j * 64 + t] = dwacc[j];
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * NV; i += 256) {  // float4 i = columns 256 (i / 64) + 4 (i % 64) ..
    const f32x4 a = (wpart[0][i] + wpart[1][i]) + (wpart[2][i] + wpart[3][i]);
    *reinterpret_cast<f32x4*>(dw_part + (long)blockIdx.x * N + (i / 64) * 256 + 4 * (i % 64)) = a;
  }
}

// Column sums in a fixed order (deterministic). Pass 1: block (64 columns x RCH rows), 4 row-phases x 8 independent
// accumulators per thread (memory-level parallelism); writes part[chunk][n]. Pass 2 sums the chunks.
constexpr int COLSUM_RCH = 512;

__global__ void colsum_pass1(const float* __restrict__ in, float* __restrict__ part, int R, int N, long ld) {
  const int n = blockIdx.x * 64 + (threadIdx.x & 63);
  const int ph = threadIdx.x >> 6;
  const int r0 = blockIdx.y * COLSUM_RCH;
  const int r1 = min(R, r0 + COLSUM_RCH);
  __shared__ float red[4][64];
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (n < N) {
    int r = r0 + ph;
    for (; r + 28 < r1; r += 32) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += in[(long)(r + 4 * j) * ld + n];
    }
    for (; r < r1; r += 4) a[0] += in[(long)r * ld + n];
  }
  red[ph][threadIdx.x & 63] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (ph == 0 && n < N) {
    const int l = threadIdx.x;
    part[(long)blockIdx.y * N + n] = (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
  }
}

__global__ void colsum_pass2(const float* __restrict__ part, float* __restrict__ out, int chunks, int N,
                             int accumulate) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int c = 0; c < chunks; ++c) s += part[(long)c * N + n];
  out[n] = accumulate ? out[n] + s : s;
}

// single-chunk fast path: sum all rows straight into out
__global__ void colsum_kernel(const float* __restrict__ in, float* __restrict__ out, int R, int N, long ld,
                              int accumulate) {
  const int n = blockIdx.x * 64 + (threadIdx.x & 63);
  const int ph = threadIdx.x >> 6;
  __shared__ float red[4][64];
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (n < N) {
    int r = ph;
    for (; r + 28 < R; r += 32) {
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += in[(long)(r + 4 * j) * ld + n];
    }
    for (; r < R; r += 4) a[0] += in[(long)r * ld + n];
  }
  red[ph][threadIdx.x & 63] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (ph == 0 && n < N) {
    const int l = threadIdx.x;
    const float v = (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
    out[n] = accumulate ? out[n] + v : v;
  }
}

// short columns (R <= COLSUM_RCH, e.g. the RMSNorm weight-gradient partials of sd_rmsnorm_bwd): 32 columns x 32 row
// phases per 1024-thread block, so a 512 x 256 partial block is summed by 8 x 1024 threads at 16 loads each instead
// of 4 x 256 threads at 128 (colsum_kernel: 7 us per launch, round-5 kernel table); fixed order, deterministic
__global__ __launch_bounds__(1024) void colsum_short(const float* __restrict__ in, float* __restrict__ out, int R,
                                                     int N, long ld, int accumulate) {
  const int cl = threadIdx.x & 31, ph = threadIdx.x >> 5;
  const int n = blockIdx.x * 32 + cl;
  __shared__ float red[32][33];
  __shared__ float red4[4][32];
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (n < N) {
    int r = ph;
    for (; r + 96 < R; r += 128) {
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] += in[(long)(r + 32 * j) * ld + n];
    }
    for (; r < R; r += 32) a[0] += in[(long)r * ld + n];
  }
  red[ph][cl] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (ph < 4) {  // 4 x 8 partial rows, then one lane per column adds the 4
    float s = 0.f;
#pragma unroll
    for (int p = 0; p < 8; ++p) s += red[ph * 8 + p][cl];
    red4[ph][cl] = s;
  }
  __syncthreads();
  if (ph == 0 && n < N) {
    const float v = (red4[0][cl] + red4[1][cl]) + (red4[2][cl] + red4[3][cl]);
    out[n] = accumulate ? out[n] + v : v;
  }
}

int pick_vpt(int n) {
  if (n <= 1) return 1;
  if (n <= 2) return 2;
  if (n <= 3) return 3;
  if (n <= 4) return 4;
  if (n <= 8) return 8;
  return 16;
}

template <int TEAM>
int grid_for(int M) {
  long teams = (M + 0L);
  long blocks = (teams + 256 / TEAM - 1) / (256 / TEAM);
  return (int)(blocks < 8192 ? blocks : 8192);
}
// backward: fewer, longer-lived blocks so the weight-gradient partials stay few
template <int TEAM>
int grid_bwd(int M) {
  const int g = grid_for<TEAM>(M);
  return g < 512 ? g : 512;
}

#define SD_RMS_DISPATCH(KERNEL, TEAMV, ...)                                             \
  switch (pick_vpt((N + TEAMV - 1) / TEAMV)) {                                          \
    case 1: KERNEL<TEAMV, 1><<<grid, 256, 0, stream>>>(__VA_ARGS__); break;              \
    case 2: KERNEL<TEAMV, 2><<<grid, 256, 0, stream>>>(__VA_ARGS__); break;              \
    case 3: KERNEL<TEAMV, 3><<<grid, 256, 0, stream>>>(__VA_ARGS__); break;              \
    case 4: KERNEL<TEAMV, 4><<<grid, 256, 0, stream>>>(__VA_ARGS__); break;              \
    case 8: KERNEL<TEAMV, 8><<<grid, 256, 0, stream>>>(__VA_ARGS__); break;              \
    default: KERNEL<TEAMV, 16><<<grid, 256, 0, stream>>>(__VA_ARGS__); break;            \
  }

// the vector forms: N = 256, 512 or 1024, every row start 16-B aligned
bool vec_ok(int N, const void* a, const void* b, const void* c, long ld) {
  const bool al = (((uintptr_t)a | (uintptr_t)b | (uintptr_t)c) & 15) == 0;
  return al && (N == 256 || N == 512 || N == 1024) && ld % 4 == 0;
}

int team_for(int N) {
  if (N <= 64) return 16;
  if (N <= 1024) return 64;
  return 256;
}

}  // namespace

extern "C" int sd_rmsnorm_fwd(const float* x, const float* w, float* y, float* rstd, int M, int N, float eps,
                              int act, sd_stream stream_) {
  return sd_rmsnorm_fwd_ld(x, w, y, N, rstd, M, N, eps, act, stream_);
}

extern "C" int sd_rmsnorm_fwd_ld(const float* x, const float* w, float* y, long ldy, float* rstd, int M, int N,
                                 float eps, int act, sd_stream stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  if (M <= 0) return SD_OK;
  if (N <= 0 || N > 4096) return SD_ESHAPE;
  const int team = team_for(N);
  if (vec_ok(N, x, w, y, ldy)) {
    const int grid = grid_for<64>(M);
    switch (N / 256) {
      case 1: rms_fwd_v<1><<<grid, 256, 0, stream>>>(x, w, y, rstd, M, eps, act, ldy); break;
      case 2: rms_fwd_v<2><<<grid, 256, 0, stream>>>(x, w, y, rstd, M, eps, act, ldy); break;
      default: rms_fwd_v<4><<<grid, 256, 0, stream>>>(x, w, y, rstd, M, eps, act, ldy); break;
    }
    SD_LAUNCH_CHECK();
    return SD_OK;
  }
  if (team == 16) { int grid = grid_for<16>(M); SD_RMS_DISPATCH(rms_fwd, 16, x, w, y, rstd, M, N, eps, act, ldy) }
  else if (team == 64) { int grid = grid_for<64>(M); SD_RMS_DISPATCH(rms_fwd, 64, x, w, y, rstd, M, N, eps, act, ldy) }
  else { int grid = grid_for<256>(M); SD_RMS_DISPATCH(rms_fwd, 256, x, w, y, rstd, M, N, eps, act, ldy) }
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_rmsnorm_bwd_blocks(int M, int N) {
  const int team = team_for(N);
  return team == 16 ? grid_bwd<16>(M) : team == 64 ? grid_bwd<64>(M) : grid_bwd<256>(M);
}

extern "C" int sd_rmsnorm_bwd(const float* x, const float* w, const float* rstd, const float* dy, float* dx,
                              float* dw, float* dw_partial, int M, int N, int act, int accumulate_dx,
                              int accumulate_dw, sd_stream stream_) {
  return sd_rmsnorm_bwd_ld(x, w, rstd, dy, N, dx, dw, dw_partial, M, N, act, accumulate_dx, accumulate_dw, stream_);
}

extern "C" int sd_rmsnorm_bwd_ld(const float* x, const float* w, const float* rstd, const float* dy, long ldy,
                                 float* dx, float* dw, float* dw_partial, int M, int N, int act, int accumulate_dx,
                                 int accumulate_dw, sd_stream stream_) {
  return sd_rmsnorm_bwd_ldx(x, w, rstd, dy, ldy, dx, N, dw, dw_partial, M, N, act, accumulate_dx, accumulate_dw,
                            stream_);
}

extern "C" int sd_rmsnorm_bwd_ldx(const float* x, const float* w, const float* rstd, const float* dy, long ldy,
                                  float* dx, long ldx, float* dw, float* dw_partial, int M, int N, int act,
                                  int accumulate_dx, int accumulate_dw, sd_stream stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  if (M <= 0) return SD_OK;
  if (N <= 0 || N > 4096 || ldx < N || ldy < N) return SD_ESHAPE;
  const int team = team_for(N);
  float* part = dw ? dw_partial : nullptr;
  int grid;
  if (vec_ok(N, x, w, dx, ldx) && vec_ok(N, dy, w, dx, ldy)) {
    grid = grid_bwd<64>(M);
    switch (N / 256) {
      case 1: rms_bwd_v<1><<<grid, 256, 0, stream>>>(x, w, rstd, dy, dx, part, M, act, accumulate_dx, ldy, ldx); break;
      case 2: rms_bwd_v<2><<<grid, 256, 0, stream>>>(x, w, rstd, dy, dx, part, M, act, accumulate_dx, ldy, ldx); break;
      default: rms_bwd_v<4><<<grid, 256, 0, stream>>>(x, w, rstd, dy, dx, part, M, act, accumulate_dx, ldy, ldx); break;
    }
  } else if (team == 16) { grid = grid_bwd<16>(M); SD_RMS_DISPATCH(rms_bwd, 16, x, w, rstd, dy, dx, part, M, N, act, accumulate_dx, ldy, ldx) }
  else if (team == 64) { grid = grid_bwd<64>(M); SD_RMS_DISPATCH(rms_bwd, 64, x, w, rstd, dy, dx, part, M, N, act, accumulate_dx, ldy, ldx) }
  else { grid = grid_bwd<256>(M); SD_RMS_DISPATCH(rms_bwd, 256, x, w, rstd, dy, dx, part, M, N, act, accumulate_dx, ldy, ldx) }
  SD_LAUNCH_CHECK();
  if (dw) return sd_colsum_ws(dw_partial, dw, grid, N, N, accumulate_dw, nullptr, stream_);
  return SD_OK;
}

extern "C" int sd_colsum_chunks(int R) { return (R + COLSUM_RCH - 1) / COLSUM_RCH; }

// workspace (>= sd_colsum_chunks(R) * N floats) is only needed when R > COLSUM_RCH
extern "C" int sd_colsum_ws(const float* in, float* out, int R, int N, long ld, int accumulate, float* workspace,
                            sd_stream stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  if (N <= 0) return SD_OK;
  const int chunks = (R + COLSUM_RCH - 1) / COLSUM_RCH;
  if (chunks <= 1 && N <= 4096) {
    colsum_short<<<(N + 31) / 32, 1024, 0, stream>>>(in, out, R, N, ld, accumulate);
    SD_LAUNCH_CHECK();
    return SD_OK;
  }
  if (chunks <= 1 || !workspace) {
    colsum_kernel<<<(N + 63) / 64, 256, 0, stream>>>(in, out, R, N, ld, accumulate);
    SD_LAUNCH_CHECK();
    return SD_OK;
  }
  colsum_pass1<<<dim3((N + 63) / 64, chunks), 256, 0, stream>>>(in, workspace, R, N, ld);
  SD_LAUNCH_CHECK();
  colsum_pass2<<<(N + 255) / 256, 256, 0, stream>>>(workspace, out, chunks, N, accumulate);
  SD_LAUNCH_CHECK();
  return SD_OK;
}

extern "C" int sd_colsum(const float* in, float* out, int R, int N, long ld, int accumulate, sd_stream stream_) {
  return sd_colsum_ws(in, out, R, N, ld, accumulate, nullptr, stream_);
}
