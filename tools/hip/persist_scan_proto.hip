// Weights-stationary persistent observe-scan SKELETON vs the same phase bodies as one launch per phase (VERDICT r03
// item 2(b); measurement aid, not product code). Geometry of the real forward step at dmc/cnn (D 2048, U 256, 8 blocks,
// B 16, scan.hip): 4 dependent phases per step, each an M = 16 fp32 MFMA contraction whose A panel (16 rows x K) is
// the previous phase's output written by OTHER workgroups:
//   phase 0  _dyn_hid  (block input 1024, split over 2 WGs): K 512, one 16-col tile, 32 KB weights per WG
//   phase 1  _dyn_gru  (block 256 -> 3 gates):              K 256, two tiles,        32 KB
//   phase 2  obs_net_0 deter half + _dyn_in0 (2048 -> 512): K 256, one tile,         16 KB
//   phase 3  obs_net logits (256 -> 512):                   K 256, two tiles,        32 KB
// 256 workgroups x 512 threads, one per CU. `persist`: one launch for all 64 steps, each WG's 112 KB of weights loaded
// into LDS once, an XCD-hierarchical grid barrier between phases (per-group counter -> top counter -> per-group
// generation flag; groups = blockIdx % 8, which share an XCD under round-robin dispatch; speed only, not correctness);
// producers: plain stores -> every wave's vmcnt(0) -> workgroup barrier -> lane-0 release fence -> vmcnt(0) -> add;
// consumers: relaxed poll -> acquire fence. Every spin is bounded: on timeout an error flag is set and every later
// barrier is skipped, so the grid drains (the run then reports the failure instead of timing).
// `launch`: the same body as 4 x 64 launches, each re-staging its weights from HBM/MALL (what the product does).
// Thread 0 of every workgroup stamps s_memrealtime (100 MHz) at arrive / released / staged / reduced per phase.
// Build: hipcc --offload-arch=gfx950 -O3 tools/hip/persist_scan_proto.hip -o tools/hip/persist_scan_proto
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int NWG = 256, NT = 512, NWAVE = 8, M = 16, STEPS = 64, NPH = 4;
constexpr int PK[NPH] = {512, 256, 256, 256};  // K per phase
constexpr int PN[NPH] = {1, 2, 1, 2};          // 16-col tiles per phase
// weights [col][K + 4] (the pad puts a 16-lane column read on distinct banks)
constexpr int W_OFF[NPH + 1] = {0, 16 * 516, 16 * 516 + 32 * 260, 16 * 516 + 48 * 260, 16 * 516 + 80 * 260};
constexpr int W_FLOATS = W_OFF[NPH];          // 29056 floats = 113.5 KB
constexpr int A_STRIDE = 512 + 4;             // A panel row stride (floats)
constexpr int A_FLOATS = M * A_STRIDE;        // 33 KB, reused as the cross-wave reduction scratch
constexpr int OUT_PER_WG = 512;               // floats each WG writes per phase (2 tiles of 16 x 16)
constexpr long SPIN_LIMIT = 1l << 21;

struct Sync {
  unsigned grp[8 * 32];  // per-group arrive counters, one 128-B line each
  unsigned top[32];
  unsigned gen[8 * 32];  // per-group generation flags
  unsigned err[32];
};

__device__ __forceinline__ uint64_t now() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ unsigned ld_relaxed(unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// grid barrier number `g` (0-based, monotonic); returns false once any workgroup has timed out
__device__ bool grid_barrier(Sync* s, unsigned g, volatile int* lds_ok) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    int ok = ld_relaxed(&s->err[0]) == 0;
    if (ok) {
      const int grp = blockIdx.x & 7;
      const unsigned per = NWG / 8;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned old = __hip_atomic_fetch_add(&s->grp[grp * 32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      long spins = 0;
      if (old + 1 == (g + 1) * per) {  // last arriver of the group: group leader
        __hip_atomic_fetch_add(&s->top[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (ld_relaxed(&s->top[0]) < (g + 1) * 8u) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > SPIN_LIMIT) break;
        }
        __hip_atomic_store(&s->gen[grp * 32], g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        while (ld_relaxed(&s->gen[grp * 32]) < g + 1) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > SPIN_LIMIT) break;
        }
      }
      if (spins > SPIN_LIMIT) {
        __hip_atomic_store(&s->err[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *lds_ok = ok;
  }
  __syncthreads();
  return *lds_ok;
}

__device__ void stage_weights(float* wl, const float* wg, int p) {
  const int n = (W_OFF[p + 1] - W_OFF[p]);
  const float4* src = reinterpret_cast<const float4*>(wg + (long)blockIdx.x * W_FLOATS + W_OFF[p]);
  float4* dst = reinterpret_cast<float4*>(wl + W_OFF[p]);
  for (int i = threadIdx.x; i < n / 4; i += NT) dst[i] = src[i];
}

// one phase: A panel <- 16 x K of the previous phase's outputs (other WGs'), contraction with the LDS weights,
// cross-wave reduction, SiLU, plain stores of this WG's outputs
typedef __attribute__((address_space(1))) unsigned gu32;  // global (never flat) for every handed-off word

__device__ __forceinline__ float4 ld_sc1(const float4* p) {  // four 4-B global_load_dword sc1 (bypass this CU's L1)
  gu32* q = (gu32*)(p);
  float4 v;
  v.x = __uint_as_float(__hip_atomic_load(q + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  v.y = __uint_as_float(__hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  v.z = __uint_as_float(__hip_atomic_load(q + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  v.w = __uint_as_float(__hip_atomic_load(q + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  return v;
}

// SC1: the A panel was handed over inside this launch (pair variant): every load of it sc1; the outputs are stored
// sc1 (write-through) for a consumer in the same launch
template <int P, bool SC1 = false, bool SC1_OUT = false>
__device__ void phase_body(float* wl, float* al, const float* in, float* out, uint64_t* st) {
  constexpr int K = PK[P], NTL = PN[P];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  {  // A panel: 16 rows of K floats from WGs (b % 16) * 16 .. +15's outputs (8 KB each side of the XCDs)
    const float4* src = reinterpret_cast<const float4*>(in + (long)((blockIdx.x % 16) * 16) * OUT_PER_WG);
    constexpr int N4 = M * K / 4, PER = N4 / NT;
    float4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) v[i] = SC1 ? ld_sc1(src + threadIdx.x + i * NT) : src[threadIdx.x + i * NT];
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int e = (threadIdx.x + i * NT) * 4, r = e / K, c = e % K;
      *reinterpret_cast<float4*>(al + r * A_STRIDE + c) = v[i];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) st[1] = now();
  f32x4 acc[NTL];
#pragma unroll
  for (int t = 0; t < NTL; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int KW = K / NWAVE;  // k span of a wave
  const float* wp = wl + W_OFF[P];
#pragma unroll
  for (int k0 = 0; k0 < KW; k0 += 4) {
    const int k = wave * KW + k0 + (lane >> 4);
    const float a = al[(lane & 15) * A_STRIDE + k];
#pragma unroll
    for (int t = 0; t < NTL; ++t) {
      const float b = wp[(t * 16 + (lane & 15)) * (K + 4) + k];
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[t], 0, 0, 0);
    }
  }
  __syncthreads();  // A panel reads done: reuse as reduction scratch
#pragma unroll
  for (int t = 0; t < NTL; ++t)
    *reinterpret_cast<f32x4*>(al + ((wave * NTL + t) * 64 + lane) * 4) = acc[t];
  __syncthreads();
  if (threadIdx.x == 0) st[2] = now();
  if (threadIdx.x < NTL * 256) {
    const int t = threadIdx.x >> 8, e = threadIdx.x & 255;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NWAVE; ++w) s += al[((w * NTL + t) * 64 + (e >> 2)) * 4 + (e & 3)];
    s = s / (1.f + __expf(-s)) * 0.5f;
    if (SC1_OUT)
      __hip_atomic_store((gu32*)(out + (long)blockIdx.x * OUT_PER_WG + t * 256 + e), __float_as_uint(s),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      out[(long)blockIdx.x * OUT_PER_WG + t * 256 + e] = s;
  }
}

__global__ __launch_bounds__(NT, 1) void persist(const float* wg, float* const* bufs, Sync* s, uint64_t* tr,
                                                  uint64_t* t0) {
  __shared__ __attribute__((aligned(16))) float wl[W_FLOATS];
  __shared__ __attribute__((aligned(16))) float al[A_FLOATS];
  __shared__ int ok;
  for (int p = 0; p < NPH; ++p) stage_weights(wl, wg, p);
  unsigned g = 0;
  if (!grid_barrier(s, g++, &ok)) return;
  if (threadIdx.x == 0 && blockIdx.x == 0) t0[0] = now();
  for (int step = 0; step < STEPS; ++step) {
#define SD_PHASE(P)                                                                    \
  {                                                                                    \
    uint64_t* st = tr + (((long)step * NPH + P) * NWG + blockIdx.x) * 4;               \
    if (threadIdx.x == 0) st[0] = now();                                               \
    if (!grid_barrier(s, g++, &ok)) return;                                            \
    if (threadIdx.x == 0) st[3] = now(); /* released */                                \
    phase_body<P>(wl, al, bufs[(P + 3) % 4], bufs[P], st);                             \
  }
    SD_PHASE(0) SD_PHASE(1) SD_PHASE(2) SD_PHASE(3)
#undef SD_PHASE
  }
  grid_barrier(s, g++, &ok);
  if (threadIdx.x == 0 && blockIdx.x == 0) t0[1] = now();
}

template <int P>
__global__ __launch_bounds__(NT, 1) void launch_phase(const float* wg, float* const* bufs, uint64_t* tr, int step) {
  __shared__ __attribute__((aligned(16))) float wl[W_FLOATS];
  __shared__ __attribute__((aligned(16))) float al[A_FLOATS];
  uint64_t* st = tr + (((long)step * NPH + P) * NWG + blockIdx.x) * 4;
  if (threadIdx.x == 0) st[0] = now();
  stage_weights(wl, wg, P);
  if (threadIdx.x == 0) st[3] = now();  // weights issued (the A panel load below waits for them too)
  phase_body<P>(wl, al, bufs[(P + 3) % 4], bufs[P], st);
}

// ---- round 6: the block-local pair _dyn_hid -> _dyn_gru (phases 0 and 1) as ONE launch per step,
// phases 2 and 3 as launches: 3 launches per step. Every WG stages both phases' weights up front (phase 1's weight
// staging overlaps phase 0), runs phase 0, publishes its outputs write-through (sc1 stores, every storing wave drained,
// barrier, one lane's sc1 flag = step + 1), then polls its producers' flags with sc1 loads: the 16 WGs whose outputs
// form its phase-1 A panel, or with NORM all 256 (the RMSNorm between _dyn_hid and _dyn_gru needs every column
// tile's partial sums of squares of the rows: an all-to-all edge), and loads the panel with sc1 loads (the handoff
// table's first row: hipMalloc'd, one WG per CU, 4-B sc1 stores and loads). Spins are bounded (error word).
template <bool NORM>
__global__ __launch_bounds__(NT, 1) void pair_launch(const float* wg, float* const* bufs, uint64_t* tr, int step,
                                                      unsigned* flags, unsigned* err) {
  __shared__ __attribute__((aligned(16))) float wl[W_FLOATS];
  __shared__ __attribute__((aligned(16))) float al[A_FLOATS];
  __shared__ int ok;
  const unsigned epoch = step + 1;
  uint64_t* st0 = tr + (((long)step * NPH + 0) * NWG + blockIdx.x) * 4;
  uint64_t* st1 = tr + (((long)step * NPH + 1) * NWG + blockIdx.x) * 4;
  if (threadIdx.x == 0) st0[0] = now();
  stage_weights(wl, wg, 0);
  stage_weights(wl, wg, 1);
  if (threadIdx.x == 0) st0[3] = now();
  phase_body<0, false, true>(wl, al, bufs[3], bufs[0], st0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x == 0) {
    st1[0] = now();
    __hip_atomic_store((gu32*)&flags[blockIdx.x * 32], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x == 0) ok = 1;
  __syncthreads();
  constexpr int NPOLL = NORM ? NWG : 16;
  if (threadIdx.x < NPOLL) {
    const int src = NORM ? threadIdx.x : (blockIdx.x % 16) * 16 + threadIdx.x;
    long spins = 0;
    while (__hip_atomic_load((gu32*)&flags[src * 32], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != epoch) {
      if (++spins > SPIN_LIMIT || __hip_atomic_load((gu32*)err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        __hip_atomic_store((gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  if (!ok) return;
  if (threadIdx.x == 0) st1[3] = now();  // released: every producer's flag seen
  phase_body<1, true, false>(wl, al, bufs[0], bufs[1], st1);
}

static double med(std::vector<double> v) {
  if (v.empty()) return 0.0;
  std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
  return v[v.size() / 2];
}

static void report(const char* what, const std::vector<uint64_t>& tr, bool persistent) {
  // per step/phase: arrive = median st[0]; released = st[3]; staged st[1]; reduced st[2]; exit of phase = next arrive
  printf("%s: per phase, median over steps (us)\n", what);
  printf("  phase  %s  stage  mma+red  body_span\n", persistent ? "barrier(last arrive->median release)" : "weights(entry->issued)");
  for (int p = 0; p < NPH; ++p) {
    std::vector<double> bar, stg, mma, span;
    for (int s = 1; s < STEPS; ++s) {
      const uint64_t* x = &tr[((long)s * NPH + p) * NWG * 4];
      std::vector<double> a, r, b, c;
      uint64_t last_arrive = 0, first_rel = ~0ull, last_red = 0;
      for (int w = 0; w < NWG; ++w) {
        const uint64_t* q = x + w * 4;
        last_arrive = std::max(last_arrive, q[0]);
        first_rel = std::min(first_rel, q[3]);
        last_red = std::max(last_red, q[2]);
        r.push_back((double)q[3]);
        b.push_back(((double)q[1] - (double)q[3]) * 0.01);
        c.push_back(((double)q[2] - (double)q[1]) * 0.01);
      }
      if (persistent)
        bar.push_back((med(r) - (double)last_arrive) * 0.01);
      else {
        std::vector<double> wgt;
        for (int w = 0; w < NWG; ++w) wgt.push_back(((double)x[w * 4 + 3] - (double)x[w * 4 + 0]) * 0.01);
        bar.push_back(med(wgt));
      }
      stg.push_back(med(b));
      mma.push_back(med(c));
      span.push_back(((double)last_red - (double)first_rel) * 0.01);
    }
    printf("  %d      %8.2f  %6.2f  %6.2f  %8.2f\n", p, med(bar), med(stg), med(mma), med(span));
  }
}

int main() {
  int dev = 0, ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (ncu < NWG) {
    printf("needs %d CUs resident, device has %d: not run\n", NWG, ncu);
    return 0;
  }
  int occ = 0;
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, persist, NT, 0);
  printf("CUs %d, persist blocks per CU %d\n", ncu, occ);
  if (occ < 1) return 1;
  float *wg, *buf[4], **bufs;
  Sync* s;
  uint64_t *tr, *t0;
  const long trn = (long)STEPS * NPH * NWG * 4;
  hipMalloc(&wg, (long)NWG * W_FLOATS * 4);
  for (auto& b : buf) hipMalloc(&b, (long)NWG * OUT_PER_WG * 4), hipMemset(b, 0, (long)NWG * OUT_PER_WG * 4);
  hipMalloc(&bufs, sizeof(buf));
  hipMemcpy(bufs, buf, sizeof(buf), hipMemcpyHostToDevice);
  hipMalloc(&s, sizeof(Sync));
  hipMalloc(&tr, trn * 8);
  hipMalloc(&t0, 16);
  std::vector<float> hw((long)NWG * W_FLOATS);
  for (size_t i = 0; i < hw.size(); ++i) hw[i] = ((i * 2654435761u) % 1000) * 1e-6f - 5e-4f;
  hipMemcpy(wg, hw.data(), hw.size() * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  std::vector<uint64_t> h(trn);
  for (int rep = 0; rep < 3; ++rep) {  // persistent: rep 0 warms up
    hipMemset(s, 0, sizeof(Sync));
    hipMemset(tr, 0, trn * 8);
    hipEventRecord(e0);
    persist<<<NWG, NT>>>(wg, bufs, s, tr, t0);
    hipEventRecord(e1);
    if (hipEventSynchronize(e1) != hipSuccess) {
      printf("persist: launch failed\n");
      return 1;
    }
    unsigned err = 0;
    uint64_t tt[2];
    hipMemcpy(&err, &s->err[0], 4, hipMemcpyDeviceToHost);
    hipMemcpy(tt, t0, 16, hipMemcpyDeviceToHost);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    if (err) {
      printf("persist: a barrier timed out (not all %d workgroups resident?): no timing\n", NWG);
      return 1;
    }
    printf("persist rep %d: launch %.1f us, %d steps after weight load %.2f us = %.2f us per step\n", rep, ms * 1e3,
           STEPS, (tt[1] - tt[0]) * 0.01, (tt[1] - tt[0]) * 0.01 / STEPS);
  }
  hipMemcpy(h.data(), tr, trn * 8, hipMemcpyDeviceToHost);
  report("persistent (weights in LDS, grid barrier between phases)", h, true);
  // the product replays its launches from HIP graphs: capture the 4 x 64 launches once
  hipStream_t stream;
  hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
  hipGraph_t graph;
  hipGraphExec_t exec;
  hipStreamBeginCapture(stream, hipStreamCaptureModeGlobal);
  for (int st = 0; st < STEPS; ++st) {
    launch_phase<0><<<NWG, NT, 0, stream>>>(wg, bufs, tr, st);
    launch_phase<1><<<NWG, NT, 0, stream>>>(wg, bufs, tr, st);
    launch_phase<2><<<NWG, NT, 0, stream>>>(wg, bufs, tr, st);
    launch_phase<3><<<NWG, NT, 0, stream>>>(wg, bufs, tr, st);
  }
  hipStreamEndCapture(stream, &graph);
  if (hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) != hipSuccess) {
    printf("graph instantiate failed\n");
    return 1;
  }
  for (int rep = 0; rep < 3; ++rep) {
    hipMemset(tr, 0, trn * 8);
    hipDeviceSynchronize();
    hipEventRecord(e0, stream);
    hipGraphLaunch(exec, stream);
    hipEventRecord(e1, stream);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    printf("launch (graph) rep %d: %d steps x 4 launches %.2f us = %.2f us per step\n", rep, STEPS, ms * 1e3,
           ms * 1e3 / STEPS);
  }
  hipMemcpy(h.data(), tr, trn * 8, hipMemcpyDeviceToHost);
  report("launches (weights re-staged every launch)", h, false);
  // the pair variants: phases 0 + 1 in one launch, phases 2, 3 as launches (3 launches per step)
  unsigned *flags, *err;
  hipMalloc(&flags, NWG * 32 * 4);
  hipMalloc(&err, 128);
  for (int norm = 0; norm < 2; ++norm) {
    hipGraph_t pg;
    hipGraphExec_t pe;
    hipStreamBeginCapture(stream, hipStreamCaptureModeGlobal);
    for (int st = 0; st < STEPS; ++st) {
      if (norm)
        pair_launch<true><<<NWG, NT, 0, stream>>>(wg, bufs, tr, st, flags, err);
      else
        pair_launch<false><<<NWG, NT, 0, stream>>>(wg, bufs, tr, st, flags, err);
      launch_phase<2><<<NWG, NT, 0, stream>>>(wg, bufs, tr, st);
      launch_phase<3><<<NWG, NT, 0, stream>>>(wg, bufs, tr, st);
    }
    hipStreamEndCapture(stream, &pg);
    if (hipGraphInstantiate(&pe, pg, nullptr, nullptr, 0) != hipSuccess) {
      printf("pair graph instantiate failed\n");
      return 1;
    }
    for (int rep = 0; rep < 3; ++rep) {
      hipMemset(tr, 0, trn * 8);
      hipMemset(flags, 0, NWG * 32 * 4);
      hipMemset(err, 0, 128);
      hipDeviceSynchronize();
      hipEventRecord(e0, stream);
      hipGraphLaunch(pe, stream);
      hipEventRecord(e1, stream);
      hipEventSynchronize(e1);
      unsigned herr = 0;
      hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      if (herr) {
        printf("pair%s: a hand-off wait timed out: no timing\n", norm ? "+norm" : "");
        return 1;
      }
      printf("pair%s (graph) rep %d: %d steps x 3 launches %.2f us = %.2f us per step\n", norm ? "+norm" : "", rep,
             STEPS, ms * 1e3, ms * 1e3 / STEPS);
    }
    hipMemcpy(h.data(), tr, trn * 8, hipMemcpyDeviceToHost);
    report(norm ? "pair + all-256 norm wait (phase 1: entry = published, 'weights' = the hand-off wait)"
                : "pair, 16-producer panel wait (phase 1: entry = published, 'weights' = the hand-off wait)", h, false);
  }
  return 0;
}
