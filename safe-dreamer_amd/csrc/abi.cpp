// ABI version probe + misc host helpers of libsdhip.so (see include/sdhip.h).
#include <hip/hip_runtime.h>
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
