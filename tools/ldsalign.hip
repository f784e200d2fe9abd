// ldsalign.hip -- measurement only: are 16-byte LDS writes at 4-byte (not
// 16-byte) alignment correct on gfx950 (SH_MEM_CONFIG unaligned mode), and
// what do they cost against aligned ones and against dword writes?
// The compiler splits a 4-byte-aligned 16-byte LDS store into two
// ds_write2_b32; the GCM output ring (esp_gcm.hip, GCM_RING) issues
// ds_write_b128 itself (inline asm), so this checks that form.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ldsalign tools/ldsalign.hip && ./tools/ldsalign
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

__device__ __forceinline__ void ds_w128(uint32_t addr, uint4 v) {
  typedef uint32_t V4 __attribute__((ext_vector_type(4)));
  V4 u = {v.x, v.y, v.z, v.w};
  asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(u) : "memory");
}

// correctness: lane t writes 16 bytes at byte offset 4*off[t] of a 4 KiB
// window (offsets chosen so no two lanes overlap), then every dword is read
// back as a dword
__global__ void check(const uint32_t *off, uint32_t *out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[1024 + 64];
  for (int i = threadIdx.x; i < 1024 + 64; i += blockDim.x) lds[i] = 0xdeadbeefu;
  __syncthreads();
  const uint32_t base = (uint32_t)(uintptr_t)(void *)lds;
  const uint32_t t = threadIdx.x;
  ds_w128(base + 4 * off[t], make_uint4(4 * t, 4 * t + 1, 4 * t + 2, 4 * t + 3));
  __syncthreads();
  for (int i = threadIdx.x; i < 1024 + 64; i += blockDim.x) out[i] = lds[i];
}

// throughput: each lane writes 4 times per iteration to its own 16-byte
// slots, lanes contiguous (a wave's write covers 1 KiB: conflict-free when
// aligned), KIND 0 aligned b128, 1 b128 at +4 bytes, 2 four ds_write_b32, 3
// two ds_write2_b32 (the compiler's split form), with one dependent read per
// iteration so the writes stay live
template <int KIND>
__global__ __launch_bounds__(1024) void tput(uint32_t *out, int iters) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[65536 + 64];
  const uint32_t base = (uint32_t)(uintptr_t)(void *)lds;
  const uint32_t t = threadIdx.x;
  const uint32_t a = base + (t >> 6) * 4096 + (t & 63) * 16 + (KIND == 1 || KIND == 3 ? 4 : 0);
  uint32_t x = t;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t ar = a + r * 1024;
      if (KIND <= 1) {
        ds_w128(ar, make_uint4(x, x + 1, x + 2, x + 3));
      } else if (KIND == 2) {
        asm volatile("ds_write_b32 %0, %1\n\tds_write_b32 %0, %2 offset:4\n\tds_write_b32 %0, %3 offset:8\n\tds_write_b32 %0, %4 offset:12"
                     ::"v"(ar), "v"(x), "v"(x + 1), "v"(x + 2), "v"(x + 3) : "memory");
      } else {
        asm volatile("ds_write2_b32 %0, %1, %2 offset1:1\n\tds_write2_b32 %0, %3, %4 offset0:2 offset1:3"
                     ::"v"(ar), "v"(x), "v"(x + 1), "v"(x + 2), "v"(x + 3) : "memory");
      }
    }
    x += *reinterpret_cast<volatile uint32_t *>(lds + (t >> 6) * 4096 + (t & 63) * 16 + (it & 3) * 4);
  }
  out[blockIdx.x * 1024 + t] = x;
}

int main() {
  uint32_t h_off[64], *d_off, *d_out, h_out[1088];
  // lane t at dword 17*t (+0..3): distinct 4-byte alignments mod 16
  for (int t = 0; t < 64; ++t) h_off[t] = 17 * t;
  hipMalloc(&d_off, sizeof h_off);
  hipMalloc(&d_out, 1 << 24);
  hipMemcpy(d_off, h_off, sizeof h_off, hipMemcpyHostToDevice);
  check<<<1, 64>>>(d_off, d_out);
  hipMemcpy(h_out, d_out, sizeof h_out, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 1088; ++i) {
    uint32_t want = 0xdeadbeefu;
    const int t = i / 17, k = i % 17;
    if (t < 64 && k < 4) want = 4 * t + k;
    if (h_out[i] != want) ++bad;
  }
  printf("{\"probe\": \"ds_write_b128 at 4-byte alignment\", \"correct\": %s, \"bad_dwords\": %d}\n",
         bad ? "false" : "true", bad);
  const int iters = 20000, grid = 256 * 4;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char *names[4] = {"b128 aligned", "b128 at +4", "4x b32", "2x write2_b32 at +4"};
  for (int kind = 0; kind < 4; ++kind) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      if (kind == 0) tput<0><<<grid, 1024>>>(d_out, iters);
      if (kind == 1) tput<1><<<grid, 1024>>>(d_out, iters);
      if (kind == 2) tput<2><<<grid, 1024>>>(d_out, iters);
      if (kind == 3) tput<3><<<grid, 1024>>>(d_out, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep == 1) {
        const double waves = grid * 16.0, writes = waves * iters * 4;   // 16-byte writes (wave-level)
        printf("{\"kind\": \"%s\", \"ms\": %.3f, \"wave_writes16_per_cu_cycle_at_2.1GHz\": %.3f}\n", names[kind], ms,
               writes / (ms * 1e-3 * 2.1e9 * 256));
      }
    }
  }
  return 0;
}
