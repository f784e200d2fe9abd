// Memory-pattern probe for the GCM kernel's record layout (measurement only).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/memprobe tools/memprobe.hip
//   ./tools/memprobe
//
// Streams N records of `len` bytes laid out `stride` bytes apart starting at
// byte offset `off` (the bench arena's layout: 1480-byte records in 1500-byte
// slots, 20 bytes in), S lanes per record, 16 bytes per lane per access, two
// accesses per step (blocks i and i+S, as the GCM pair step does), and
//   kind 0: copy (load + store to a second buffer at the same offsets)
//   kind 1: load only (xor-reduce, one word per record written)
//   kind 2: store only
// against a flat fully coalesced copy of the same bytes.  The result is the
// HBM rate this access pattern can reach with no arithmetic in the way.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

struct U4 {
  uint32_t x, y, z, w;
} __attribute__((aligned(4)));

// U accesses per lane per step (blocks i, i+S, ..., i+(U-1)S); NT bit 1 =
// nontemporal loads, bit 2 = nontemporal stores
template <typename T>
__device__ __forceinline__ T ldv(const T *p, bool nt) {
  return nt ? __builtin_nontemporal_load(p) : *p;
}
template <typename T>
__device__ __forceinline__ void stv(T *p, T v, bool nt) {
  if (nt)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}

template <int S, int KIND, int U, int NT>
__global__ __launch_bounds__(1024) void rec_kernel(const uint8_t *in, uint8_t *out, uint32_t *sink, int n,
                                                   int len, int stride, int off) {
  constexpr int RPW = 64 / S;
  const int lane = threadIdx.x & 63, l = lane & (S - 1);
  const int wave = (blockIdx.x * (blockDim.x / 64)) + threadIdx.x / 64;
  const int nw = gridDim.x * (blockDim.x / 64);
  const int nb = (len + 15) / 16;
  for (int r0 = wave * RPW; r0 < n; r0 += nw * RPW) {
    const int r = r0 + lane / S;
    if (r >= n) break;
    const size_t base = (size_t)r * stride + off;
    uint32_t acc = 0;
    for (int i = l; i < nb; i += U * S) {
      uint32_t v[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int ib = i + u * S;
        v[u][0] = v[u][1] = v[u][2] = v[u][3] = ib;
        if (KIND != 2 && ib < nb) {
          const uint32_t *q = reinterpret_cast<const uint32_t *>(in + base + 16 * ib);
          v[u][0] = ldv(q, NT & 1);
          v[u][1] = ldv(q + 1, NT & 1);
          v[u][2] = ldv(q + 2, NT & 1);
          v[u][3] = ldv(q + 3, NT & 1);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int ib = i + u * S;
        if (KIND != 1) {
          if (ib < nb) {
            uint32_t *q = reinterpret_cast<uint32_t *>(out + base + 16 * ib);
            stv(q, v[u][0], NT & 2);
            stv(q + 1, v[u][1], NT & 2);
            stv(q + 2, v[u][2], NT & 2);
            stv(q + 3, v[u][3], NT & 2);
          }
        } else {
          acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
        }
      }
    }
    if (KIND == 1 && acc == 0x12345678u) sink[r] = acc;
  }
}

__global__ __launch_bounds__(1024) void flat_copy(const uint4 *in, uint4 *out, size_t n16) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}

static int g_block = 1024;
template <int S, int KIND, int U, int NT>
static float run(const uint8_t *in, uint8_t *out, uint32_t *sink, int n, int len, int stride, int off, int grid) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 2; ++w) rec_kernel<S, KIND, U, NT><<<grid, g_block>>>(in, out, sink, n, len, stride, off);
  CK(hipEventRecord(e0));
  const int reps = 10;
  for (int w = 0; w < reps; ++w) rec_kernel<S, KIND, U, NT><<<grid, g_block>>>(in, out, sink, n, len, stride, off);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char **argv) {
  const int n = 1 << 20, len = 1480 + 16, stride = 1500;
  const size_t bytes = (size_t)n * stride + 4096;
  uint8_t *in, *out;
  uint32_t *sink;
  CK(hipMalloc(&in, bytes));
  CK(hipMalloc(&out, bytes));
  CK(hipMalloc(&sink, n * 4));
  CK(hipMemset(in, 1, bytes));
  {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t n16 = (size_t)n * len / 16;
    flat_copy<<<4096, 1024>>>((const uint4 *)in, (uint4 *)out, n16);
    CK(hipEventRecord(e0));
    for (int w = 0; w < 10; ++w) flat_copy<<<4096, 1024>>>((const uint4 *)in, (uint4 *)out, n16);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 10;
    printf("{\"pattern\": \"flat_copy\", \"ms\": %.4f, \"GBps\": %.1f}\n", ms, 2.0 * n16 * 16 / ms / 1e6);
  }
  const char *kn[3] = {"copy", "load", "store"};
  const int off = 36, grid = 256;
  for (int inplace = 0; inplace < 2; ++inplace) {
    uint8_t *o = inplace ? in : out;
#define ONE(SS, KK, UU, NN)                                                                               \
  {                                                                                                       \
    float ms = run<SS, KK, UU, NN>(in, o, sink, n, len, stride, off, grid);                               \
    double b = (double)n * len * (KK == 0 ? 2 : 1);                                                       \
    printf("{\"block\": %d, \"S\": %d, \"kind\": \"%s\", \"U\": %d, \"nt\": %d, \"inplace\": %d, \"ms\": %.4f, " \
           "\"GBps\": %.1f}\n",                                                                           \
           g_block, SS, kn[KK], UU, NN, inplace, ms, b / ms / 1e6);                                       \
  }
    for (int blk : {768}) {
      g_block = blk;
      ONE(4, 0, 2, 0) ONE(4, 0, 4, 0) ONE(4, 0, 8, 0) ONE(8, 0, 2, 0) ONE(8, 0, 4, 0) ONE(16, 0, 1, 0) ONE(16, 0, 2, 0)
      ONE(4, 2, 2, 0) ONE(4, 1, 2, 0)
      ONE(1, 1, 4, 0) ONE(1, 0, 4, 0) ONE(1, 2, 4, 0)   // lane = record, 64 B per step (the ETA kernel's pattern)
      ONE(1, 0, 4, 1) ONE(1, 0, 4, 2) ONE(1, 0, 4, 3) ONE(1, 0, 8, 0) ONE(2, 0, 4, 0) ONE(4, 0, 4, 2)
    }
  }
  CK(hipDeviceSynchronize());
  return 0;
}
