// fp32 MFMA throughput probe: register-only MFMA chains (no memory), by instruction, independent accumulator
// chains per wave and waves per SIMD. Prints TFLOP/s over the whole GPU.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int CH>
__global__ void k16(float* out, int iters) {
  f32x4 acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[c], 0, 0, 0);
  float s = 0.f;
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int CH>
__global__ void k32(float* out, int iters) {
  f32x16 acc[CH];
  for (int c = 0; c < CH; ++c)
    for (int r = 0; r < 16; ++r) acc[c][r] = 0.f;
  float a = threadIdx.x * 1e-3f, b = 1.0001f;
  for (int i = 0; i < iters; ++i)
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[c], 0, 0, 0);
  float s = 0.f;
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][5];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class K>
void run(const char* name, K kern, int ch, int flop_per_mfma, int wps, float* out) {
  const int iters = 4096, blocks = 256 * 4 * wps / 4;  // 256 CUs x 4 SIMDs x wps waves, 256-thread blocks
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  kern<<<blocks, 256>>>(out, iters);
  hipEventRecord(a);
  kern<<<blocks, 256>>>(out, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double flops = (double)blocks * 4 * iters * ch * flop_per_mfma;
  printf("%-10s chains %2d waves/SIMD %d : %7.1f TFLOP/s\n", name, ch, wps, flops / ms / 1e9);
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 4 * 8 * 256 * sizeof(float));
  for (int wps = 1; wps <= 2; ++wps) {
    run("16x16x4", k16<1>, 1, 2048, wps, out);
    run("16x16x4", k16<2>, 2, 2048, wps, out);
    run("16x16x4", k16<4>, 4, 2048, wps, out);
    run("16x16x4", k16<8>, 8, 2048, wps, out);
    run("32x32x2", k32<1>, 1, 4096, wps, out);
    run("32x32x2", k32<2>, 2, 4096, wps, out);
    run("32x32x2", k32<4>, 4, 4096, wps, out);
  }
  return 0;
}
