// hybridprobe.hip -- measurement only: can the VALU-bound bitsliced AES
// (aes_bs.h) and the LDS-bound T-table rounds run at once on the same CUs?
// Two persistent kernels, one per stream: bs (256-thread workgroups, two per
// CU: two waves per SIMD at <= 192 VGPRs) and tt (256-thread workgroups, one
// per CU by its 64 KiB LDS: one wave per SIMD at <= 128 VGPRs, T-table-shaped
// rounds of 32 conflict-free ds_read_b32 each, as tools/ldsprobe.hip).  Times
// each alone and both launched together; block-rounds per second of each.
//   hipcc --offload-arch=gfx950 -O3 -I tools -I f-stack_amd/csrc -o tools/hybridprobe tools/hybridprobe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "aes_bs.h"

using namespace espgpu;
typedef const __attribute__((address_space(4))) uint32_t *rkptr;

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2), amdgpu_num_vgpr(192)))
void bs_kernel(const uint32_t *__restrict__ rk_g, uint32_t *out, int iters) {
  const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
  uint32_t st[128];
#pragma unroll
  for (int i = 0; i < 128; ++i) st[i] = gid * (i + 1) * 2654435761u;
  const rkptr rk = (rkptr)(const void *)rk_g;
  for (int it = 0; it < iters; ++it) {
#pragma unroll 1
    for (int r = 1; r <= 9; ++r) {
      uint32_t k[4] = {rk[4 * (r - 1)], rk[4 * (r - 1) + 1], rk[4 * (r - 1) + 2], rk[4 * (r - 1) + 3]};
      bs::round<true>(st, k);
    }
    uint32_t k[4] = {rk[36], rk[37], rk[38], rk[39]};
    bs::round<false>(st, k);
  }
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 128; ++i) acc ^= st[i] * (i + 1);
  out[gid] = acc;
}

// T-table-shaped rounds: 2 blocks per lane, 16 data-dependent conflict-free
// ds_read_b32 per block-round (entry x at x*256 + (lane&31)*4), XOR-folded
template <int N>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1), amdgpu_num_vgpr(128)))
void tt_kernel(uint32_t *out, int rounds) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[65536];
  for (int i = threadIdx.x; i < 65536 / 4; i += 256) reinterpret_cast<uint32_t *>(lds)[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t slot = (threadIdx.x & 31) * 4;
  uint32_t s[N];
#pragma unroll
  for (int k = 0; k < N; ++k) s[k] = threadIdx.x * 77 + k * 13 + blockIdx.x;
  for (int r = 0; r < rounds; ++r) {
    uint32_t t[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
      const uint32_t a = __builtin_amdgcn_perm(s[(k + 1) % N], slot, 0x0c0c0000u | ((4u + (k & 3)) << 8));
      t[k] = *reinterpret_cast<const uint32_t *>(lds + a);
    }
#pragma unroll
    for (int k = 0; k < N; ++k) s[k] = __builtin_amdgcn_bitop3_b32(s[k], t[k], t[(k + 1) % N], 0x96);
  }
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) acc ^= s[k];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  uint32_t hk[44];
  for (int i = 0; i < 44; ++i) hk[i] = 0x9e3779b9u * (i + 1);
  uint32_t *drk, *dout, *dout2;
  hipMalloc(&drk, sizeof hk);
  hipMemcpy(drk, hk, sizeof hk, hipMemcpyHostToDevice);
  hipMalloc(&dout, 512 * 256 * 4);
  hipMalloc(&dout2, 256 * 256 * 4);
  hipStream_t sa, sb;
  hipStreamCreateWithFlags(&sa, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&sb, hipStreamNonBlocking);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int BSI = 30, TTR = 3000;   // iterations sized for ~ms-scale kernels
  auto run = [&](bool bs, bool tt) {
    hipDeviceSynchronize();
    hipEventRecord(e0, 0);
    hipStreamWaitEvent(sa, e0, 0);
    hipStreamWaitEvent(sb, e0, 0);
    if (bs) hipLaunchKernelGGL(bs_kernel, dim3(512), dim3(256), 0, sa, drk, dout, BSI);
    if (tt) hipLaunchKernelGGL(tt_kernel<32>, dim3(256), dim3(256), 0, sb, dout2, TTR);
    hipEvent_t ea, eb;
    hipEventCreateWithFlags(&ea, hipEventDisableTiming);
    hipEventCreateWithFlags(&eb, hipEventDisableTiming);
    hipEventRecord(ea, sa);
    hipEventRecord(eb, sb);
    hipStreamWaitEvent(0, ea, 0);
    hipStreamWaitEvent(0, eb, 0);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(ea);
    hipEventDestroy(eb);
    return ms;
  };
  run(true, true);   // warm-up
  for (int rep = 0; rep < 3; ++rep) {
    const float a = run(true, false), b = run(false, true), c = run(true, true);
    const double bs_br = 512.0 * 256 * 32 * BSI * 10, tt_br = 256.0 * 256 * 32 * TTR / 16;   // block-rounds
    printf("{\"bs_alone_ms\": %.3f, \"tt_alone_ms\": %.3f, \"both_ms\": %.3f, \"sum_ms\": %.3f, "
           "\"bs_Gblockrounds_s\": %.1f, \"tt_Gblockrounds_s\": %.1f, \"both_Gblockrounds_s\": %.1f}\n",
           a, b, c, a + b, bs_br / a / 1e6, tt_br / b / 1e6, (bs_br + tt_br) / c / 1e6);
  }
  return 0;
}
