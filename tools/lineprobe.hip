// Line-alignment probe for the GCM kernel's memory pattern (measurement only).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/lineprobe tools/lineprobe.hip && ./tools/lineprobe
//
// 1M records of 1448 payload bytes at the bench layout (1500-byte slots, the
// payload 36 bytes in, so 4-byte but not 16-byte aligned), S = 4 lanes per
// record, one pair step = 8 x 16 bytes per record, copy in -> out:
//   mode 0 "blocks": the kernel today -- lane l takes the payload's 16-byte
//          blocks l and l+4 of the step (addresses P + 16*(8m + l [+4])),
//          single 16-byte accesses at 4-byte alignment;
//   mode 1 "lines":  lane l takes the 16-byte-aligned chunks l and l+4 of the
//          128-byte line L + 128m (L = P & ~127): every pair step reads and
//          writes one whole aligned line per record (partial chunks at the
//          record's ends are skipped here; the kernel stores them by dwords);
//   mode 2 "lines+1": mode 1 with the next line's loads issued one step ahead.
// `spin` adds that many dependent VALU ops per step (the AES/GHASH work
// between a step's loads and its stores, so the memory can hide under it).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

typedef uint32_t V4a __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t V4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ V4 spinv(V4 v, int spin) {
  for (int k = 0; k < spin; ++k) v.x = __builtin_amdgcn_alignbit(v.x, v.y, 7) ^ v.z;
  return v;
}

template <int MODE>
__global__ __launch_bounds__(1024) void probe(const uint8_t *in, uint8_t *out, int n, int plen, int stride,
                                              int off, int spin, uint32_t *q) {
  const int lane = threadIdx.x & 63, l = lane & 3;
  for (;;) {
    __shared__ uint32_t tk;
    if (threadIdx.x == 0) tk = atomicAdd(q, 1u);
    __syncthreads();
    const uint32_t c = tk;
    __syncthreads();
    if ((int)(c * 256) >= n) break;
    const int r = c * 256 + (threadIdx.x >> 2);
    if (r >= n) continue;
    const size_t P = (size_t)r * stride + off;
    if (MODE == 0) {
      const int nb = (plen + 15) / 16;
      for (int i = l; i < nb; i += 8) {
        const int ib = i + 4;
        V4 a = {0, 0, 0, 0}, b = {0, 0, 0, 0};
        a = *reinterpret_cast<const V4a *>(in + P + 16 * i);
        if (ib < nb) b = *reinterpret_cast<const V4a *>(in + P + 16 * ib);
        a = spinv(a, spin);
        *reinterpret_cast<V4a *>(out + P + 16 * i) = a;
        if (ib < nb) *reinterpret_cast<V4a *>(out + P + 16 * ib) = b;
      }
    } else {
      const size_t L = P & ~(size_t)127, E = P + plen;
      const int nl = (int)((E - L + 127) / 128);
      V4 na = {0, 0, 0, 0}, nb2 = {0, 0, 0, 0};
      auto ld = [&](int m, int h) -> V4 {
        const size_t a = L + 128 * (size_t)m + 64 * h + 16 * l;
        V4 v = {0, 0, 0, 0};
        if (a >= P && a + 16 <= E) v = *reinterpret_cast<const V4 *>(in + a);
        return v;
      };
      if (MODE == 2) {
        na = ld(0, 0);
        nb2 = ld(0, 1);
      }
      for (int m = 0; m < nl; ++m) {
        V4 a, b;
        if (MODE == 2) {
          a = na;
          b = nb2;
          if (m + 1 < nl) {
            na = ld(m + 1, 0);
            nb2 = ld(m + 1, 1);
          }
        } else {
          a = ld(m, 0);
          b = ld(m, 1);
        }
        a = spinv(a, spin);
        const size_t s0 = L + 128 * (size_t)m + 16 * l, s1 = s0 + 64;
        if (s0 >= P && s0 + 16 <= E) *reinterpret_cast<V4 *>(out + s0) = a;
        if (s1 >= P && s1 + 16 <= E) *reinterpret_cast<V4 *>(out + s1) = b;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && atomicAdd(q + 1, 1u) == gridDim.x - 1) {
    atomicExch(q, 0u);
    atomicExch(q + 1, 0u);
  }
}

template <int MODE>
static float run(const uint8_t *in, uint8_t *out, int n, int spin, uint32_t *q) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) probe<MODE><<<256, 1024>>>(in, out, n, 1448, 1500, 36, spin, q);
  CK(hipEventRecord(e0));
  const int reps = 20;
  for (int w = 0; w < reps; ++w) probe<MODE><<<256, 1024>>>(in, out, n, 1448, 1500, 36, spin, q);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main() {
  const int n = 1 << 20;
  const size_t bytes = (size_t)n * 1500 + 4096;
  uint8_t *in, *out;
  uint32_t *q;
  CK(hipMalloc(&in, bytes));
  CK(hipMalloc(&out, bytes));
  CK(hipMalloc(&q, 8));
  CK(hipMemset(q, 0, 8));
  CK(hipMemset(in, 1, bytes));
  const char *names[3] = {"blocks", "lines", "lines+1"};
  for (int spin : {0, 64, 256}) {
    float t[3] = {run<0>(in, out, n, spin, q), run<1>(in, out, n, spin, q), run<2>(in, out, n, spin, q)};
    for (int k = 0; k < 3; ++k)
      printf("{\"mode\": \"%s\", \"spin\": %d, \"ms\": %.4f, \"GBps_copy\": %.1f}\n", names[k], spin, t[k],
             2.0 * n * 1448 / t[k] / 1e6);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
