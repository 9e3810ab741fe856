// ABI version probe + misc host helpers of libsdhip.so (see include/sdhip.h).
#include <hip/hip_runtime.h>
#include "sdhip.h"

extern "C" int sd_abi_version(void) { return SDHIP_ABI_VERSION; }
