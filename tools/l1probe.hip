// l1probe.hip -- measurement only: can the vector L1 serve T-table lookups
// beside the LDS?  Each lane runs R dependent "rounds" of N independent
// lookups at data-dependent addresses (as ldsprobe.hip / an AES round):
//   KIND 0: N ds_read_b32 from a 64 KiB LDS table (conflict-free lane slots)
//   KIND 1: N global_load_dword from a 1 KiB table in global memory (L1-resident)
//   KIND 2: N - M LDS lookups and M L1 lookups per round (both pipes at once)
// Prints lookups per CU-cycle (at 2.1 GHz) per variant and waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o tools/l1probe tools/l1probe.hip && ./tools/l1probe
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int KIND, int N, int M>
__global__ __launch_bounds__(1024) void probe(const uint32_t *__restrict__ gt, uint32_t *out, int rounds) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[65536];
  for (int i = threadIdx.x; i < 65536 / 4; i += blockDim.x)
    reinterpret_cast<uint32_t *>(lds)[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t slot = (lane & 31) * 4;
  constexpr int NL1 = KIND == 0 ? 0 : (KIND == 1 ? N : M);   // lookups through L1 per round
  uint32_t s[N];
#pragma unroll
  for (int k = 0; k < N; ++k) s[k] = threadIdx.x * 77 + k * 13;
  for (int r = 0; r < rounds; ++r) {
    uint32_t t[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
      if (k < N - NL1) {
        const uint32_t a = __builtin_amdgcn_perm(s[(k + 1) % N], slot, 0x0c0c0000u | ((4u + (k & 3)) << 8));
        t[k] = *reinterpret_cast<const uint32_t *>(lds + a);
      } else {
        const uint32_t x = (s[(k + 1) % N] >> (8 * (k & 3))) & 0xffu;
        t[k] = gt[x];
      }
    }
#pragma unroll
    for (int k = 0; k < N; ++k) s[k] = __builtin_amdgcn_bitop3_b32(s[k], t[k], t[(k + 1) % N], 0x96);
  }
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) acc ^= s[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int KIND, int N, int M>
static void run(const uint32_t *gt, int wg, int rounds) {
  const int grid = 256;
  uint32_t *d;
  hipMalloc(&d, (size_t)grid * 1024 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((probe<KIND, N, M>), dim3(grid), dim3(wg), 0, 0, gt, d, rounds);
  hipEventRecord(e0, 0);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((probe<KIND, N, M>), dim3(grid), dim3(wg), 0, 0, gt, d, rounds);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  const double looks = (double)grid * (wg / 64) * rounds * N;     // wave-level lookups
  const double cyc = ms * 1e-3 * 2.1e9;
  printf("{\"kind\": %d, \"n\": %d, \"m_l1\": %d, \"wg\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, "
         "\"lookups_per_cu_cycle\": %.3f}\n",
         KIND, N, KIND == 1 ? N : (KIND == 2 ? M : 0), wg, wg / 256, ms, looks / 256.0 / cyc);
  hipFree(d);
}

int main() {
  uint32_t *gt;
  hipMalloc(&gt, 1024 * 4);
  uint32_t h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = (uint32_t)i * 2246822519u + 7u;
  hipMemcpy(gt, h, sizeof h, hipMemcpyHostToDevice);
  const int R = 4000;
  for (int wg : {256, 512, 1024}) {
    run<0, 16, 0>(gt, wg, R);
    run<1, 16, 0>(gt, wg, R);
    run<2, 16, 2>(gt, wg, R);
    run<2, 16, 4>(gt, wg, R);
    run<2, 16, 6>(gt, wg, R);
  }
  hipFree(gt);
  return 0;
}
