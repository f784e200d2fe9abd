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
// Records in mbufs start at any byte: ESP follows a 14-byte Ethernet and a
// 20- or 40-byte IP header, 2 mod 4.  The copy works on destination-aligned
// dwords, each assembled from the two source dwords it straddles
// (alignbyte), so every load and store is an aligned dword and never touches
// a dword that holds no byte of the span; the <= 3-byte head and tail go
// bytewise.  Both sides 16-byte aligned: dwordx4.
#include <hip/hip_runtime.h>

#include "espgpu_internal.h"

namespace espgpu {

namespace {

constexpr int kXferThreads = 256;

__global__ __launch_bounds__(kXferThreads) void xfer_kernel(const XferSpan *spans, const uint8_t *status) {
  const XferSpan sp = spans[blockIdx.x];
  if (sp.rec != ~0u && status[sp.rec] != 0) return;
  const uint8_t *src = reinterpret_cast<const uint8_t *>(sp.src);
  uint8_t *dst = reinterpret_cast<uint8_t *>(sp.dst);
  const uint32_t len = sp.len, t = threadIdx.x;
  if (((sp.src | sp.dst) & 15) == 0) {
    const uint32_t n16 = len >> 4;
    for (uint32_t i = t; i < n16; i += kXferThreads)
      reinterpret_cast<uint4 *>(dst)[i] = reinterpret_cast<const uint4 *>(src)[i];
    for (uint32_t i = (n16 << 4) + t; i < len; i += kXferThreads) dst[i] = src[i];
    return;
  }
  // head: bytes up to the first 4-byte-aligned destination address
  const uint32_t head = min(len, (uint32_t)((4u - (uint32_t)(sp.dst & 3)) & 3u));
  if (t < head) dst[t] = src[t];
  const uint32_t m = (len - head) >> 2;                 // whole destination dwords
  const uint32_t tail0 = head + (m << 2);
  if (t < len - tail0) dst[tail0 + t] = src[tail0 + t];
  if (m == 0) return;
  uint32_t *d32 = reinterpret_cast<uint32_t *>(dst + head);
  const uint64_t p = sp.src + head;                     // source of d32[0]
  const uint32_t sh = (uint32_t)(p & 3);
  const uint32_t *s32 = reinterpret_cast<const uint32_t *>(p & ~(uint64_t)3);
  if (sh == 0) {
    for (uint32_t j = t; j < m; j += kXferThreads) d32[j] = s32[j];
  } else {
    // d32[j] = source bytes p+4j .. p+4j+3 = the high (4-sh) bytes of s32[j]
    // and the low sh bytes of s32[j+1]; both dwords hold bytes of the span
    for (uint32_t j = t; j < m; j += kXferThreads)
      d32[j] = __builtin_amdgcn_alignbyte(s32[j + 1], s32[j], sh);
  }
}

}  // namespace

int launch_xfer(const XferSpan *spans, uint32_t nspans, const uint8_t *status, void *stream) {
  if (nspans == 0) return 0;
  hipLaunchKernelGGL(xfer_kernel, dim3(nspans), dim3(kXferThreads), 0, (hipStream_t)stream, spans, status);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace espgpu
