// xfer.hip — the opencrypto path's staging copies as a kernel.
//
// A batch staged by espgpu_process moves host -> device before its crypto
// kernels and device -> host after them.  Two kinds of span:
//   * the staging region of a slot (records gathered by process(), the
//     descriptors, the status bytes): pinned hipHostMalloc memory;
//   * records that stay where the caller put them, in memory registered with
//     espgpu_register_host (hipHostRegister: DPDK mbuf pages, lib/ff_veth.c:
//     367-389): read into the device arena before the kernels, the results
//     written back in place after them, with no CPU gather / scatter.
// Both are read or written by the GPU through the host mapping (PCIe), one
// workgroup per <= kXferPiece-byte piece; a piece with rec != ~0u is skipped
// unless that record's status byte is 0 (a rejected record's buffer stays as
// it is, as complete_slot leaves it).
//
// Records in mbufs start at any byte (ESP follows a 14-byte Ethernet and a
// 20- or 40-byte IP header: 2 mod 4): the copy itself is xfer_copy.h.
#include <hip/hip_runtime.h>

#include "espgpu_internal.h"
#include "xfer_copy.h"

namespace espgpu {

namespace {

constexpr int kXferThreads = 256;

__global__ __launch_bounds__(kXferThreads) void xfer_kernel(const XferSpan *spans, const uint8_t *status) {
  const XferSpan sp = spans[blockIdx.x];
  if (sp.rec != ~0u && status[sp.rec] != 0) return;
  xfer_copy(sp.src, sp.dst, sp.len, threadIdx.x, kXferThreads);
}

}  // namespace

int launch_xfer(const XferSpan *spans, uint32_t nspans, const uint8_t *status, void *stream) {
  if (nspans == 0) return 0;
  hipLaunchKernelGGL(xfer_kernel, dim3(nspans), dim3(kXferThreads), 0, (hipStream_t)stream, spans, status);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace espgpu
