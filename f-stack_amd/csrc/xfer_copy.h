// xfer_copy.h — the byte-span copy of the opencrypto path's staging, as a
// device function shared by the xfer kernel (xfer.hip) and the crypto kernels
// that stage their own records (esp_gcm.hip, small single-session batches).
//
// Copies len bytes from src to dst (device or host-mapped addresses) with the
// nt threads t = 0..nt-1 of the caller.  Both 16-byte aligned: dwordx4.
// Otherwise destination-aligned dwords, each assembled from the two source
// dwords it straddles (alignbyte), so every load and store is an aligned
// dword and never touches a dword that holds no byte of the span; the
// <= 3-byte head and tail go bytewise.  Records in mbufs start 2 mod 4.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace espgpu {

// Every load of a batch is issued before its stores (source and destination
// never overlap), so a thread pays the read latency -- a PCIe round trip for
// host memory -- once per kU elements, not once per element; the head and
// tail bytes load with the first batch and store after the last.
template <int kU = 8>
__device__ __forceinline__ void xfer_copy(uint64_t src_a, uint64_t dst_a, uint32_t len, uint32_t t,
                                          uint32_t nt) {
  const uint8_t *__restrict__ src = reinterpret_cast<const uint8_t *>(src_a);
  uint8_t *__restrict__ dst = reinterpret_cast<uint8_t *>(dst_a);
  if (((src_a | dst_a) & 15) == 0) {
    const uint32_t n16 = len >> 4, tb = (n16 << 4) + t;
    const uint8_t tv = tb < len ? src[tb] : 0;
    const uint4 *__restrict__ s16 = reinterpret_cast<const uint4 *>(src);
    uint4 *__restrict__ d16 = reinterpret_cast<uint4 *>(dst);
    for (uint32_t i0 = t; i0 < n16; i0 += nt * kU) {
      uint4 v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (i0 + u * nt < n16) v[u] = s16[i0 + u * nt];
#pragma unroll
      for (int u = 0; u < kU; ++u)
        if (i0 + u * nt < n16) d16[i0 + u * nt] = v[u];
    }
    if (tb < len) dst[tb] = tv;
    return;
  }
  // head: bytes up to the first 4-byte-aligned destination address
  const uint32_t head = min(len, (uint32_t)((4u - (uint32_t)(dst_a & 3)) & 3u));
  const uint32_t m = (len - head) >> 2;                 // whole destination dwords
  const uint32_t tail0 = head + (m << 2);
  const bool hb = t < head, tb = t < len - tail0;
  const uint8_t hv = hb ? src[t] : 0, tv = tb ? src[tail0 + t] : 0;
  uint32_t *__restrict__ d32 = reinterpret_cast<uint32_t *>(dst + head);
  const uint64_t p = src_a + head;                      // source of d32[0]
  const uint32_t sh = (uint32_t)(p & 3);
  const uint32_t *__restrict__ s32 = reinterpret_cast<const uint32_t *>(p & ~(uint64_t)3);
  // d32[j] = source bytes p+4j .. p+4j+3 = the high (4-sh) bytes of s32[j]
  // and the low sh bytes of s32[j+1]; both dwords hold bytes of the span
  // (sh == 0: s32[j] alone)
  for (uint32_t j0 = t; j0 < m; j0 += nt * kU) {
    uint32_t a[kU], b[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const uint32_t j = j0 + u * nt;
      if (j < m) {
        a[u] = s32[j];
        b[u] = sh ? s32[j + 1] : 0u;
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const uint32_t j = j0 + u * nt;
      if (j < m) d32[j] = sh ? __builtin_amdgcn_alignbyte(b[u], a[u], sh) : a[u];
    }
  }
  if (hb) dst[t] = hv;
  if (tb) dst[tail0 + t] = tv;
}

}  // namespace espgpu
