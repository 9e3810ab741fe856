// The observe scan's 4-launch floor at deter 2048 and 4096 (measurement aid, not product code).
// persist_scan_proto.hip's launch variant — 4 dependent phases per step as graph-captured launches of 256 workgroups x
// 512 threads, each re-staging its weights (HBM / MALL -> LDS) and a 16-row A panel written by 16 other workgroups —
// with the per-workgroup weight and K sizes of the forward step scaled by S: S = 1 is the dmc / atari geometry
// (_dyn_hid K 512 per half-block tile, _dyn_gru K 256, obs_net_0 + _dyn_in0 K 256, logits K 256), S = 2 the
// memory-maze one (deter 4096: the three D-dependent phases' K and weights per workgroup doubled; the logits phase,
// K = U, unchanged). Each phase allocates only its own weights' LDS (dynamic), so S = 2 fits.
// Build: hipcc --offload-arch=gfx950 -O3 tools/hip/scan_floor_proto.hip -o tools/hip/scan_floor_proto
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int NWG = 256, NT = 512, NWAVE = 8, M = 16, STEPS = 64, NPH = 4, OUT_PER_WG = 512;
constexpr int PN[NPH] = {1, 2, 1, 2};  // 16-column tiles per phase

template <int S>
struct Geo {
  static constexpr int K(int p) { return p == 3 ? 256 : (p == 0 ? 512 * S : 256 * S); }
  static constexpr int WF(int p) { return 16 * PN[p] * (K(p) + 4); }  // weight floats of phase p per workgroup
  static constexpr int WTOT = WF(0) + WF(1) + WF(2) + WF(3);
  static constexpr int WOFF(int p) { return p == 0 ? 0 : WOFF(p - 1) + WF(p - 1); }
  static constexpr int ASTR = 512 * S + 4;
};

template <int S, int P>
__global__ __launch_bounds__(NT, 1) void phase(const float* wg, float* const* bufs) {
  using G = Geo<S>;
  constexpr int K = G::K(P), NTL = PN[P], WFP = G::WF(P);
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* wl = sm;          // this phase's weights [col][K + 4]
  float* al = sm + WFP;    // A panel [16][ASTR], reused for the cross-wave reduction
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  {  // weights: this workgroup's slice, float4 copies
    const f32x4* src = reinterpret_cast<const f32x4*>(wg + (long)blockIdx.x * G::WTOT + G::WOFF(P));
    f32x4* dst = reinterpret_cast<f32x4*>(wl);
    for (int i = threadIdx.x; i < WFP / 4; i += NT) dst[i] = src[i];
  }
  {  // A panel: 16 rows x K from the previous phase's outputs (16 producer workgroups' slots, read contiguously)
    const float* in = bufs[(P + 3) % 4];
    const f32x4* src = reinterpret_cast<const f32x4*>(in + (long)((blockIdx.x % 16) * 16) * OUT_PER_WG);
    constexpr int N4 = M * K / 4, PER = (N4 + NT - 1) / NT;
    f32x4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) v[i] = threadIdx.x + i * NT < N4 ? src[threadIdx.x + i * NT] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = (threadIdx.x + i * NT) * 4, r = e / K, c = e % K;
      if (threadIdx.x + i * NT < N4) *reinterpret_cast<f32x4*>(al + r * G::ASTR + c) = v[i];
    }
  }
  __syncthreads();
  f32x4 acc[NTL];
#pragma unroll
  for (int t = 0; t < NTL; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int KW = K / NWAVE;
#pragma unroll 8
  for (int k0 = 0; k0 < KW; k0 += 4) {
    const int k = wave * KW + k0 + (lane >> 4);
    const float a = al[(lane & 15) * G::ASTR + k];
#pragma unroll
    for (int t = 0; t < NTL; ++t) {
      const float b = wl[(t * 16 + (lane & 15)) * (K + 4) + k];
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[t], 0, 0, 0);
    }
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < NTL; ++t) *reinterpret_cast<f32x4*>(al + ((wave * NTL + t) * 64 + lane) * 4) = acc[t];
  __syncthreads();
  if (threadIdx.x < NTL * 256) {
    const int t = threadIdx.x >> 8, e = threadIdx.x & 255;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) s += al[((w * NTL + t) * 64 + (e >> 2)) * 4 + (e & 3)];
    s = s / (1.f + __expf(-s)) * 0.5f;
    bufs[P][(long)blockIdx.x * OUT_PER_WG + t * 256 + e] = s;
  }
}

template <int S>
int run(float* const* bufs, hipStream_t st) {
  using G = Geo<S>;
  float* wg;
  if (hipMalloc(&wg, (long)NWG * G::WTOT * 4) != hipSuccess) return 1;
  if (hipMemset(wg, 0, (long)NWG * G::WTOT * 4) != hipSuccess) return 1;
  size_t lds[NPH];
  const void* kern[NPH] = {reinterpret_cast<const void*>(phase<S, 0>), reinterpret_cast<const void*>(phase<S, 1>),
                           reinterpret_cast<const void*>(phase<S, 2>), reinterpret_cast<const void*>(phase<S, 3>)};
  for (int p = 0; p < NPH; ++p) {
    lds[p] = (size_t)(G::WF(p) + M * G::ASTR) * 4;
    if (lds[p] > 160 * 1024) {
      printf("S=%d phase %d needs %zu B of LDS: not run\n", S, p, lds[p]);
      return 1;
    }
    if (hipFuncSetAttribute(kern[p], hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds[p]) != hipSuccess) return 1;
  }
  hipGraph_t graph;
  hipGraphExec_t exec;
  if (hipStreamBeginCapture(st, hipStreamCaptureModeGlobal) != hipSuccess) return 1;
  for (int s = 0; s < STEPS; ++s) {
    phase<S, 0><<<NWG, NT, lds[0], st>>>(wg, bufs);
    phase<S, 1><<<NWG, NT, lds[1], st>>>(wg, bufs);
    phase<S, 2><<<NWG, NT, lds[2], st>>>(wg, bufs);
    phase<S, 3><<<NWG, NT, lds[3], st>>>(wg, bufs);
  }
  if (hipStreamEndCapture(st, &graph) != hipSuccess || hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) != hipSuccess)
    return 1;
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 1;
  for (int rep = 0; rep < 4; ++rep) {
    if (hipEventRecord(e0, st) != hipSuccess || hipGraphLaunch(exec, st) != hipSuccess ||
        hipEventRecord(e1, st) != hipSuccess || hipEventSynchronize(e1) != hipSuccess)
      return 1;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e0, e1) != hipSuccess) return 1;
    printf("S=%d (weights per workgroup %d / %d / %d / %d KB) rep %d: %d steps x 4 launches %.1f us = %.2f us per step\n",
           S, G::WF(0) / 256, G::WF(1) / 256, G::WF(2) / 256, G::WF(3) / 256, rep, STEPS, ms * 1e3, ms * 1e3 / STEPS);
  }
  return hipFree(wg) != hipSuccess;
}

int main() {
  float *buf[4], **bufs;
  const long n = (long)NWG * OUT_PER_WG * 4;  // 4x a phase's outputs: the S = 2 A panels read past the 16 producers
  for (auto& b : buf)
    if (hipMalloc(&b, n * 4) != hipSuccess || hipMemset(b, 0, n * 4) != hipSuccess) return 1;
  if (hipMalloc(&bufs, sizeof(buf)) != hipSuccess || hipMemcpy(bufs, buf, sizeof(buf), hipMemcpyHostToDevice) != hipSuccess)
    return 1;
  hipStream_t st;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
  if (run<1>(bufs, st) || run<2>(bufs, st)) {
    printf("failed\n");
    return 1;
  }
  return 0;
}
