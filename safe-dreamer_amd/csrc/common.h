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

template <int NT>
SD_DEV float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float s = red[0];
#pragma unroll
  for (int i = 1; i < NT / 64; ++i) s = fmaxf(s, red[i]);
  return s;
}

// Branch-free bounded loads: a buffer descriptor (range-checked by the hardware) plus a per-lane byte offset; an
// invalid element gets an offset >= the range (SD_OOB) and reads 0. A "cond ? load : 0" on a runtime condition
// instead makes hipcc branch around the load and drain vmcnt(0) there, serialising every prefetch behind it.
// Descriptor inputs go through readfirstlane so hipcc knows they are wave-uniform (no waterfall loops).
typedef __amdgpu_buffer_rsrc_t sd_rsrc;
constexpr uint32_t SD_OOB = 0x80000000u;
SD_DEV sd_rsrc sd_make_rsrc(const void* base, long bytes) {
  const uint64_t p = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p), hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
  const uint32_t nb = __builtin_amdgcn_readfirstlane((uint32_t)(bytes < 0x7ffffff0L ? bytes : 0x7ffffff0L));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, (int)nb, 0x00020000);
}
SD_DEV f32x4 sd_bload4(sd_rsrc r, uint32_t byte_off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}
SD_DEV float sd_bload1(sd_rsrc r, uint32_t byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, byte_off, 0, 0));
}

// hardware exp2 + reciprocal forms (v_exp_f32, v_rcp_f32): ~1e-7 relative error, 4 VALU instead of the
// ~25-instruction IEEE expf/division expansions — these sit on the A-operand path of the fused GEMM loaders.
// (__fdividef is NOT the fast form on ROCm 7.2 / gfx950: it lowers to the 13-instruction v_div_scale/fmas/fixup
// IEEE sequence; __builtin_amdgcn_rcpf is one v_rcp_f32.) exp(-x) = inf for x << 0 gives rcp = 0: silu -> -0.
SD_DEV float sigmoidf_(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
SD_DEV float siluf_(float x) { return x * __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

static inline int sd_cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// sd_set_lds_pad (abi.cpp): the dynamic LDS a GEMM launch reserves beyond its own (0 = none)
size_t sd_lds_pad_for(const void* kern);
#define SD_PAD_LAUNCH(KERN, GRID, BLOCK, ST, ...)                                             \
  do {                                                                                       \
    auto* k_ = KERN;                                                                         \
    hipLaunchKernelGGL(k_, GRID, BLOCK, sd_lds_pad_for(reinterpret_cast<const void*>(k_)), ST, __VA_ARGS__); \
  } while (0)

// Phase timestamps (measurement build, -DSD_SCAN_TRACE; scan.hip and img.hip kernels): thread 0 of every workgroup keeps entry / operands staged /
// contraction reduced / exit (s_memrealtime, 100 MHz) and stores them at exit into trace[slot][workgroup][4].
// SD_CHAIN_PRIO (1..3): the latency-bound chains' kernels (the observe scan's and the imagination's step launches, the
// ones that open with SD_TR_BEGIN) raise their waves' issue priority (s_setprio) at entry, so on a SIMD shared with a
// filler phase's waves (the other stream's GEMMs, priority 0) their instructions issue first (MI355X_MICROARCH.md:
// VALU issue is arbitrated by priority, then age). 0 = off.
#ifndef SD_CHAIN_PRIO
#define SD_CHAIN_PRIO 0
#endif
#define SD_CHAIN_PRIO_SET                                     \
  if constexpr (SD_CHAIN_PRIO > 0) __builtin_amdgcn_s_setprio(SD_CHAIN_PRIO);
#ifdef SD_SCAN_TRACE
constexpr int TR_WG = 2048;  // workgroup slots per launch
#define SD_TR_BEGIN SD_CHAIN_PRIO_SET uint64_t tr_[4] = {__builtin_amdgcn_s_memrealtime(), 0ull, 0ull, 0ull};
#define SD_TR(k) tr_[k] = __builtin_amdgcn_s_memrealtime();
#define SD_TR_END(buf, slot)                                                                               \
  if (threadIdx.x == 0 && (buf)) {                                                                         \
    tr_[3] = __builtin_amdgcn_s_memrealtime();                                                             \
    const long wg_ = blockIdx.x + (long)gridDim.x * (blockIdx.y + (long)gridDim.y * blockIdx.z);           \
    if (wg_ < TR_WG) {                                                                                     \
      uint64_t* o_ = (buf) + ((long)(slot) * TR_WG + wg_) * 4;                                             \
      for (int i_ = 0; i_ < 4; ++i_) o_[i_] = tr_[i_];                                                      \
    }                                                                                                      \
  }
#else
#define SD_TR_BEGIN SD_CHAIN_PRIO_SET
#define SD_TR(k)
#define SD_TR_END(buf, slot)
#endif
// a launch's trace destination (img.hip kernels: the buffer of sd_imagine.trace, slot t * 16 + launch of the step)
struct Tr {
  uint64_t* p;
  int slot;
};
