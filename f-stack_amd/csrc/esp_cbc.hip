// esp_cbc.hip — ESP AES-CBC + HMAC-SHA1-96 (CSP_MODE_ETA) kernels.  (stub)
#include <hip/hip_runtime.h>

#include "espgpu_internal.h"

namespace espgpu {
int launch_eta(const EtaParams &, int, int, void *) { return -1; }
}  // namespace espgpu
