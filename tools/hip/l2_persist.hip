// Does a weight slice stay in an XCD's L2 from one launch to the next? (decides the observe scan's design, DESIGN.md
// §4). Buffer W (bytes MB) is split into 32 slices; launch grid 256 x 256 threads: workgroup w (XCD w % 8 under
// round-robin dispatch) reads slice w / 8, so every XCD reads all of W once per launch (<= 4 MiB per XCD L2).
// Sequence, each launch timed with events: cold read, warm read, warm read after an 8 MB write burst to another
// buffer (the scan's saved activations), and the same with non-temporal stores for the burst.
// Run under `rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum TCC_MISS_sum --kernel-trace` to read the past-L2 bytes per launch.
// Build: hipcc --offload-arch=gfx950 -O3 tools/hip/l2_persist.hip -o tools/hip/l2_persist
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ __launch_bounds__(256) void rd(const float4* __restrict__ W, long slice_f4, float* out) {
  const long base = (long)(blockIdx.x / 8) * slice_f4;
  float4 acc = {0.f, 0.f, 0.f, 0.f};
  for (long i = threadIdx.x; i < slice_f4; i += 256) {
    const float4 v = W[base + i];
    acc.x += v.x;
    acc.y += v.y;
    acc.z += v.z;
    acc.w += v.w;
  }
  const float s = acc.x + acc.y + acc.z + acc.w;
  if (s == 12345.678f) out[blockIdx.x] = s;  // keeps the loads; never true for the zero-filled buffer
}

__global__ __launch_bounds__(256) void wr(float4* __restrict__ X, long n_f4, int nt) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n_f4; i += (long)gridDim.x * 256) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const f4 v = {1.f, 2.f, 3.f, (float)i};
    f4* p = reinterpret_cast<f4*>(X) + i;
    if (nt)
      __builtin_nontemporal_store(v, p);
    else
      *p = v;
  }
}

int main(int argc, char** argv) {
  const double mb = argc > 1 ? atof(argv[1]) : 2.0;
  const long bytes = (long)(mb * 1048576.0), slice_f4 = bytes / 16 / 32;
  float4 *W, *X;
  float* out;
  (void)hipMalloc(&W, bytes);
  (void)hipMalloc(&X, 8l << 20);
  (void)hipMalloc(&out, 4096);
  (void)hipMemset(W, 0, bytes);
  (void)hipMemset(X, 0, 8l << 20);
  hipDeviceSynchronize();
  hipEvent_t e[2];
  hipEventCreate(&e[0]);
  hipEventCreate(&e[1]);
  auto timed_rd = [&](const char* what) {
    hipEventRecord(e[0]);
    rd<<<256, 256>>>(W, slice_f4, out);
    hipEventRecord(e[1]);
    hipEventSynchronize(e[1]);
    float ms;
    hipEventElapsedTime(&ms, e[0], e[1]);
    printf("%-40s %8.2f us\n", what, ms * 1e3);
  };
  for (int rep = 0; rep < 3; ++rep) {
    wr<<<1024, 256>>>(X, (8l << 20) / 16, 0);  // 8 MB plain-store burst
    timed_rd("read after 8 MB plain-store burst");
    timed_rd("read again (warm)");
    timed_rd("read again (warm)");
    wr<<<1024, 256>>>(X, (8l << 20) / 16, 1);
    timed_rd("read after 8 MB nt-store burst");
  }
  hipDeviceSynchronize();
  printf("W = %.1f MB per XCD\n", mb);
  return 0;
}
