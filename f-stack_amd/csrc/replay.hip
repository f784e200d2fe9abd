// replay.hip — the ESP replay-window pre-filter for a device-resident batch.
//
// esp_input checks every inbound record against its SA's replay window before
// handing it to crypto (freebsd/netipsec/xform_esp.c:329-340:
// ipsec_chkreplay, ipsec.c:1248-1331) and takes the ESN high word for the AAD
// from that check (:339, :372-402).  Here every record of a batch is checked
// in parallel against the windows as they stand when the batch starts, which
// is what esp_input sees for records that are in flight together (the window
// only moves in esp_input_cb, after authentication: ipsec_updatereplay,
// ipsec.c:1338-1436, espgpu_replay_update on the host).
//
// One lane per record: a 16-byte descriptor, the 4-byte sequence number from
// the record header and one bitmap word; integer compares only.  A replayed
// record gets status ESPGPU_EACCES and descriptor len 0 (the decrypt kernels
// then drop it as EINVAL without crypto work; espgpu_replay_merge restores
// EACCES in the batch status).
#include <hip/hip_runtime.h>

#include "espgpu_internal.h"

namespace espgpu {

namespace {

__device__ __forceinline__ uint32_t be32(uint32_t x) { return __builtin_amdgcn_perm(x, x, 0x00010203u); }

// check_window (ipsec.c:1191-1201): bit (seq & 31) of word (seq >> 5) masked
// by the power-of-two bitmap size (IPSEC_REDUNDANT_BIT_SHIFTS, :1177-1180).
__device__ __forceinline__ bool seen(const espgpu_replay &r, const uint32_t *bitmap, uint32_t seq) {
  return (bitmap[r.bitmap_off + ((seq >> 5) & (r.bitmap_size - 1))] >> (seq & 31)) & 1u;
}

// ipsec_chkreplay (ipsec.c:1248-1331): true = permitted, *seqhigh set.
__device__ bool chkreplay(const espgpu_replay &r, const uint32_t *bitmap, uint32_t seq, uint32_t *seqhigh) {
  if (seq == 0 && r.last == 0) return false;
  const uint32_t window = r.wsize << 3;
  const uint32_t tl = (uint32_t)r.last, th = (uint32_t)(r.last >> 32);
  const uint32_t bl = tl - window + 1;
  // the high part stays when seq is in [bl, 2^32) with the window in one
  // subspace, or in [0, bl) with the window spanning two
  if ((tl >= window - 1 && seq >= bl) || (tl < window - 1 && seq < bl)) {
    *seqhigh = th;
    return !(seq <= tl && seen(r, bitmap, seq));
  }
  // top of a non-ESN space reached: only SADB_X_EXT_CYCSEQ SAs go on
  if (tl == 0xffffffffu && !(r.flags & ESPGPU_REPLAY_ESN) && !(r.flags & ESPGPU_REPLAY_CYCSEQ))
    return false;
  if (tl < window - 1 && seq >= bl) {         // in the window, previous subspace
    if (th == 0) return false;
    *seqhigh = th - 1;
    return !seen(r, bitmap, seq);
  }
  *seqhigh = th + 1;                           // wrapped into the next subspace
  return !(th + 1 == 0 && !(r.flags & ESPGPU_REPLAY_CYCSEQ));
}

__global__ __launch_bounds__(256) void replay_check_kernel(const uint8_t *arena, espgpu_desc *desc, uint32_t n,
                                                           const espgpu_replay *rp, uint32_t nrp,
                                                           const uint32_t *bitmap, uint8_t *rstatus) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const espgpu_desc d = desc[i];
  uint8_t st = 0;
  if (d.sa < nrp && d.len >= 8) {
    const espgpu_replay r = rp[d.sa];
    if (r.wsize != 0) {                        // esp_input: replay != NULL && wsize != 0
      const uint32_t seq = be32(*reinterpret_cast<const uint32_t *>(arena + (size_t)d.off4 * 4 + 4));
      uint32_t seqh = 0;
      if (!chkreplay(r, bitmap, seq, &seqh)) {
        st = ESPGPU_EACCES;
        desc[i].len = 0;
      } else if (r.flags & ESPGPU_REPLAY_ESN) {
        desc[i].esn_hi = seqh;
      }
    }
  }
  rstatus[i] = st;
}

__global__ __launch_bounds__(256) void replay_merge_kernel(uint8_t *status, const uint8_t *rstatus, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && rstatus[i]) status[i] = rstatus[i];
}

}  // namespace

int launch_replay_check(const uint8_t *arena, espgpu_desc *desc, uint32_t n, const espgpu_replay *rp,
                        uint32_t nrp, const uint32_t *bitmap, uint8_t *rstatus, void *stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(replay_check_kernel, dim3((n + 255) / 256), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), arena, desc, n, rp, nrp, bitmap, rstatus);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_replay_merge(uint8_t *status, const uint8_t *rstatus, uint32_t n, void *stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(replay_merge_kernel, dim3((n + 255) / 256), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), status, rstatus, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace espgpu
