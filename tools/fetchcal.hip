// FETCH_SIZE calibration for the ETA kernels' read patterns (measurement only).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/fetchcal tools/fetchcal.hip
//   rocprofv3 --kernel-trace --pmc FETCH_SIZE -- ./tools/fetchcal
//
// MI355X_MICROARCH.md §HBM calibrates FETCH_SIZE only for 16 B/lane streaming
// reads (it reports half their bytes).  The verify pass and the CBC cipher
// pass read each record through its quad (hmac_quad / cbc_enc_quad: lane
// 4Q+k loads piece k of one 64-byte group of each of the quad's 4 records),
// so one instruction covers 16 separate 64-byte spans.  Each kernel below
// reads the same 1M x 1500-byte arena (the bench layout) once:
//   flat    16 B/lane, 1 KiB contiguous per instruction (the reference case)
//   quad1   64-byte groups through the quad, one group per iteration
//   quad2   two groups per iteration (a record's 128 contiguous bytes)
//   lane16  lane = record, 16 bytes per lane per instruction (no quad)
// and prints the bytes it read; FETCH_SIZE (KiB) per kernel comes from the
// profiler's counter file.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

typedef uint32_t V4 __attribute__((ext_vector_type(4), aligned(4)));

constexpr uint32_t kRec = 1500, kN = 1u << 20;

__device__ __forceinline__ uint32_t fold(V4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

__global__ void flat(const uint8_t *a, size_t bytes, uint32_t *out) {
  uint32_t acc = 0;
  const size_t n16 = bytes / 16;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    acc ^= fold(*reinterpret_cast<const V4 *>(a + 16 * i));
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int NB>
__global__ void quad(const uint8_t *a, uint32_t *out) {
  const int lane = threadIdx.x & 63, q = lane & 3;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t nwaves = (gridDim.x * blockDim.x) >> 6;
  uint32_t acc = 0;
  for (uint32_t u = wave; u < kN / 64; u += nwaves) {
    const uint32_t base = u * 64 + (lane & ~3);           // the quad's first record
    for (uint32_t g = 0; g < (kRec + 63) / 64; g += NB) {
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t o = 64 * (g + nb) + 16 * q;
          if (o + 16 <= kRec) acc ^= fold(*reinterpret_cast<const V4 *>(a + (size_t)(base + i) * kRec + o));
        }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ void lane16(const uint8_t *a, uint32_t *out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, nt = gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint32_t r = t; r < kN; r += nt)
    for (uint32_t o = 0; o + 16 <= kRec; o += 16) acc ^= fold(*reinterpret_cast<const V4 *>(a + (size_t)r * kRec + o));
  out[t] = acc;
}

int main() {
  const size_t bytes = (size_t)kN * kRec;
  uint8_t *a;
  uint32_t *out;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&out, 1024 * 1024 * 4));
  CK(hipMemset(a, 0x5a, bytes));
  // a 512 MiB write between kernels evicts the arena from the 256 MiB Infinity Cache
  uint8_t *flush;
  CK(hipMalloc(&flush, 512u << 20));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char *names[] = {"flat", "quad1", "quad2", "lane16"};
  for (int rep = 0; rep < 3; ++rep)
    for (int k = 0; k < 4; ++k) {
      CK(hipMemset(flush, rep + k, 512u << 20));
      CK(hipEventRecord(e0));
      if (k == 0) hipLaunchKernelGGL(flat, dim3(1024), dim3(1024), 0, 0, a, bytes, out);
      if (k == 1) hipLaunchKernelGGL(quad<1>, dim3(256), dim3(1024), 0, 0, a, out);
      if (k == 2) hipLaunchKernelGGL(quad<2>, dim3(256), dim3(1024), 0, 0, a, out);
      if (k == 3) hipLaunchKernelGGL(lane16, dim3(256), dim3(1024), 0, 0, a, out);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("{\"kernel\": \"%s\", \"rep\": %d, \"bytes\": %zu, \"ms\": %.4f, \"GBps\": %.1f}\n", names[k], rep,
             (size_t)kN * (kRec / 16 * 16), ms, (double)kN * (kRec / 16 * 16) / ms / 1e6);
    }
  CK(hipFree(a));
  CK(hipFree(out));
  CK(hipFree(flush));
  return 0;
}
