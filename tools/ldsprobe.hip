// ldsprobe.hip -- measurement only: T-table-style LDS lookup throughput on
// gfx950.  Each lane runs R dependent "rounds"; a round issues N independent
// lookups at data-dependent, conflict-free addresses (one v_perm each, slot =
// lane & 31) and folds them into the state that addresses the next round,
// as an AES round does.  Variants (KIND): 0 ds_read_b32 (4-byte entries),
// 1 ds_read_b64 (8-byte entries, both halves folded in), 2 ds_read_b128
// (16-byte entries in 16 lane slots, all four words folded in, as the GHASH
// table reads), 3 the GCM kernel's mix: N ds_read_b32 and N/8 ds_read_b128
// per round (133 : 16 per block there); waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ldsprobe tools/ldsprobe.hip && ./tools/ldsprobe
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int KIND, int N>
__global__ __launch_bounds__(1024) void probe(uint32_t *out, int rounds) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[65536];
  for (int i = threadIdx.x; i < 65536 / 4; i += blockDim.x)
    reinterpret_cast<uint32_t *>(lds)[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t slot = KIND == 1 ? (lane & 31) * 8 : KIND == 2 ? (lane & 15) * 16 : (lane & 31) * 4;
  const uint32_t slot16 = (lane & 15) * 16;
  constexpr int NW = KIND == 3 ? N / 8 : 0;          // the mix's b128 lookups per round
  uint32_t s[N];
#pragma unroll
  for (int k = 0; k < N; ++k) s[k] = threadIdx.x * 77 + k * 13;
  for (int r = 0; r < rounds; ++r) {
    uint32_t t[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
      // entry x = byte (k&3) of s[k], at x*256 + slot
      const uint32_t a = __builtin_amdgcn_perm(s[(k + 1) % N], slot, 0x0c0c0000u | ((4u + (k & 3)) << 8));
      if (KIND == 1) {
        const uint2 v = *reinterpret_cast<const uint2 *>(lds + a);
        t[k] = v.x ^ v.y;
      } else if (KIND == 2) {
        const uint4 v = *reinterpret_cast<const uint4 *>(lds + a);
        t[k] = __builtin_amdgcn_bitop3_b32(v.x, v.y, v.z, 0x96) ^ v.w;
      } else {
        t[k] = *reinterpret_cast<const uint32_t *>(lds + a);
      }
    }
    uint32_t w[NW > 0 ? NW : 1];
#pragma unroll
    for (int k = 0; k < NW; ++k) {
      const uint32_t a = __builtin_amdgcn_perm(s[(k + 3) % N], slot16, 0x0c0c0000u | ((4u + (k & 3)) << 8));
      const uint4 v = *reinterpret_cast<const uint4 *>(lds + a);
      w[k] = __builtin_amdgcn_bitop3_b32(v.x, v.y, v.z, 0x96) ^ v.w;
    }
#pragma unroll
    for (int k = 0; k < N; ++k) s[k] = __builtin_amdgcn_bitop3_b32(s[k], t[k], t[(k + 1) % N], 0x96);
#pragma unroll
    for (int k = 0; k < NW; ++k) s[k] ^= w[k];
  }
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) acc ^= s[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int KIND, int N>
static void run(int wg, int rounds) {
  const int grid = 256 * (1024 / wg > 1 ? 1 : 1);
  uint32_t *d;
  hipMalloc(&d, (size_t)grid * 1024 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((probe<KIND, N>), dim3(grid), dim3(wg), 0, 0, d, rounds);
  hipEventRecord(e0, 0);
  for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((probe<KIND, N>), dim3(grid), dim3(wg), 0, 0, d, rounds);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  constexpr int NI = N + (KIND == 3 ? N / 8 : 0);
  const double instrs = (double)grid * (wg / 64) * rounds * NI;  // wave-level LDS instructions
  const double per_cu_cycles = ms * 1e-3 * 2.1e9;                 // at ~2.1 GHz
  printf("{\"kind\": \"%s\", \"n\": %d, \"wg\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, "
         "\"lds_instr_per_cu_cycle\": %.3f}\n",
         KIND == 0 ? "b32" : KIND == 1 ? "b64" : KIND == 2 ? "b128" : "mix_b32_8:1_b128", N, wg, wg / 256, ms,
         instrs / 256 / per_cu_cycles);
  hipFree(d);
}

int main() {
  const int R = 20000;
  for (int wg : {768, 1024}) {
    run<0, 16>(wg, R);
    run<0, 32>(wg, R);
    run<2, 16>(wg, R);
    run<3, 16>(wg, R);
    run<3, 32>(wg, R);
  }
  return 0;
}
