// ABI version probe + misc host helpers of libsdhip.so (see include/sdhip.h).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <mutex>
#include "common.h"
#include "sdhip.h"

extern "C" int sd_abi_version(void) { return SDHIP_ABI_VERSION; }

extern "C" int sd_stream_create_cumask(int first_cu, int ncu, sd_stream* out) {
  int dev = 0, ncus = 0;
  if (!out || ncu <= 0 || first_cu < 0 || hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || first_cu + ncu > ncus)
    return SD_EARG;
  uint32_t mask[32] = {};
  const int words = (ncus + 31) / 32;
  if (words > 32) return SD_EARG;
  for (int c = first_cu; c < first_cu + ncu; ++c) mask[c / 32] |= 1u << (c % 32);
  hipStream_t s = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask);
  if (e != hipSuccess) return (int)e;
  *out = (sd_stream)s;
  return SD_OK;
}

extern "C" int sd_stream_destroy(sd_stream stream) { return (int)hipStreamDestroy((hipStream_t)stream); }

static int g_lds_pad = 0;
extern "C" int sd_set_lds_pad(int bytes) {
  if (bytes < 0 || bytes > 65536) return SD_EARG;
  const int old = g_lds_pad;
  g_lds_pad = bytes;
  return old;
}
int sd_lds_pad_bytes() { return g_lds_pad; }
// the pad for one kernel: raises the kernel's dynamic-LDS limit once per (kernel, size); 0 when unset. The table is
// shared by every launching thread (mutex). A failed hipFuncSetAttribute (e.g. static + pad LDS over the CU's limit)
// launches that kernel without the pad, but is reported — on stderr once per kernel and by sd_lds_pad_failures() —
// so an SDREAMER_FILL_LDS A/B cannot measure "no pad" as "pad neutral".
static std::mutex g_pad_mu;
static int g_pad_failures = 0;
extern "C" int sd_lds_pad_failures(void) {
  std::lock_guard<std::mutex> lk(g_pad_mu);
  return g_pad_failures;
}
size_t sd_lds_pad_for(const void* kern) {
  static const void* done_k[256];
  static int done_b[256], n = 0;
  static const void* bad_k[256];
  static int nbad = 0;
  const int p = g_lds_pad;
  if (p <= 0) return 0;
  std::lock_guard<std::mutex> lk(g_pad_mu);
  for (int i = 0; i < n; ++i)
    if (done_k[i] == kern && done_b[i] >= p) return (size_t)p;
  const hipError_t e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, p);
  if (e != hipSuccess) {
    ++g_pad_failures;
    bool seen = false;
    for (int i = 0; i < nbad; ++i) seen |= bad_k[i] == kern;
    if (!seen) {
      if (nbad < 256) bad_k[nbad++] = kern;
      fprintf(stderr, "libsdhip: LDS pad of %d B refused for kernel %p (%s): launched without the pad\n", p, kern,
              hipGetErrorString(e));
    }
    return 0;
  }
  if (n < 256) {
    done_k[n] = kern;
    done_b[n++] = p;
  }
  return (size_t)p;
}
