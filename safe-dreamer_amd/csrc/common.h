// Shared helpers for the safe-dreamer MI355X (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SD_DEV __device__ __forceinline__

// status codes returned across the C ABI (0 = ok, >0 = hipError_t, <0 = argument errors)
enum { SD_OK = 0, SD_EARG = -1, SD_ESHAPE = -2, SD_EALIGN = -3 };

#define SD_LAUNCH_CHECK()                                  \
  do {                                                     \
    hipError_t _e = hipGetLastError();                     \
    if (_e != hipSuccess) return (int)_e;                  \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

SD_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
SD_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// sum over groups of `W` consecutive lanes (W power of two <= 64)
template <int W>
SD_DEV float group_sum(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
template <int W>
SD_DEV float group_max(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide sum for blockDim.x = NT (multiple of 64); `red` = __shared__ float[NT/64]
template <int NT>
SD_DEV float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) s += red[i];
  return s;
}

SD_DEV float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }
SD_DEV float siluf_(float x) { return x / (1.f + expf(-x)); }

static inline int sd_cdiv(long a, long b) { return (int)((a + b - 1) / b); }
