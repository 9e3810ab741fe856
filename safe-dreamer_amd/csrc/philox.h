// Counter-based sampling noise, bit-identical to oracle/noise.py (see its docstring for the definition).
// The reference draws Gumbel noise inside F.gumbel_softmax (OneHotDist.rsample, distributions.py:32-33) and
// N(0,1) inside Normal.rsample (bounded_normal, distributions.py:217-222) from torch's global RNG; here each
// sampling site derives its noise from (seed, stream, step, global element index) inside the consuming kernel,
// so no noise tensor is ever written to HBM and data-parallel shards draw exactly the 1-GPU noise.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SD_STREAM_OBS 1
#define SD_STREAM_IMG 2
#define SD_STREAM_ACT 3
#define SD_STREAM_POLICY 4
#define SD_STREAM_POLICY_ACT 5
#define SD_STREAM_AUG 6
#define SD_STREAM_REPLAY 8  // replay slice picks (sd_replay_pick); 7 is DreamerPro's augmented posterior scan

struct sd_u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ sd_u32x4 sd_philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                     uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}

__device__ __forceinline__ double sd_u01(uint32_t w) { return ((double)(w >> 8) + 0.5) * (1.0 / 16777216.0); }

__device__ __forceinline__ float sd_gumbel(uint64_t seed, uint32_t stream, uint32_t step, uint64_t idx) {
#ifdef SD_TIMING_CHEAP_NOISE  // measurement-only build (tools/ab_variants.sh): what the noise costs the chains
  return (float)((idx * 2654435761u + step) & 1023u) * 1e-3f;
#endif
  const uint64_t q = idx >> 2;
  sd_u32x4 r = sd_philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), step, stream, (uint32_t)seed,
                                (uint32_t)(seed >> 32));
  const uint32_t sel = (uint32_t)(idx & 3);
  const uint32_t w = sel == 0 ? r.x : sel == 1 ? r.y : sel == 2 ? r.z : r.w;
  const double u = sd_u01(w);
  return (float)(-log(-log(u)));
}

__device__ __forceinline__ float sd_normal(uint64_t seed, uint32_t stream, uint32_t step, uint64_t idx) {
#ifdef SD_TIMING_CHEAP_NOISE
  return (float)((idx * 2654435761u + step) & 1023u) * 1e-3f - 0.5f;
#endif
  sd_u32x4 r = sd_philox4x32_10((uint32_t)idx, (uint32_t)(idx >> 32), step, stream, (uint32_t)seed,
                                (uint32_t)(seed >> 32));
  const double u1 = sd_u01(r.x), u2 = sd_u01(r.y);
  return (float)(sqrt(-2.0 * log(u1)) * cos(2.0 * 3.141592653589793 * u2));
}

// uniform integer in [0, n) from the same word as sd_gumbel(seed, stream, step, idx) (augmentation shifts)
__device__ __forceinline__ int sd_uniform_int(uint64_t seed, uint32_t stream, uint32_t step, uint64_t idx, int n) {
  const uint64_t q = idx >> 2;
  sd_u32x4 r = sd_philox4x32_10((uint32_t)q, (uint32_t)(q >> 32), step, stream, (uint32_t)seed,
                                (uint32_t)(seed >> 32));
  const uint32_t sel = (uint32_t)(idx & 3);
  const uint32_t w = sel == 0 ? r.x : sel == 1 ? r.y : sel == 2 ? r.z : r.w;
  const int v = (int)(sd_u01(w) * (double)n);
  return v < n ? v : n - 1;
}
