// bsprobe.hip -- measurement only: bitsliced AES-128 (tools/aes_bs.h)
// throughput on gfx950, checked against a host AES first.  Each lane encrypts
// 32 counter blocks nonce||ctr (ctr low 5 bits = the slice), all 10 rounds on
// the VALU; the timing loop chains the state through `iters` encryptions.
//   hipcc --offload-arch=gfx950 -O3 -I tools -I f-stack_amd/csrc -o tools/bsprobe tools/bsprobe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include "aes_bs.h"

using namespace espgpu;

typedef const __attribute__((address_space(4))) uint32_t *rkptr;

template <int WG>
__global__ __launch_bounds__(WG) void bsprobe(const uint32_t *__restrict__ rk_g, uint32_t *out, int iters,
                                              int verify) {
  const uint32_t gid = blockIdx.x * WG + threadIdx.x;
  uint32_t st[128];
  // nonce byte j = f(gid, j), counter = gid * 32 + slice (big-endian bytes 12..15)
  uint8_t blk[16];
#pragma unroll
  for (int j = 0; j < 12; ++j) blk[j] = (uint8_t)(gid * 131u + j * 29u + 7u);
  const uint32_t cb = gid * 32u;
  blk[12] = cb >> 24, blk[13] = cb >> 16, blk[14] = cb >> 8, blk[15] = cb;
  const uint32_t pat[5] = {0xAAAAAAAAu, 0xCCCCCCCCu, 0xF0F0F0F0u, 0xFF00FF00u, 0xFFFF0000u};
#pragma unroll
  for (int j = 0; j < 16; ++j)
#pragma unroll
    for (int v = 0; v < 8; ++v)
      st[8 * j + v] = (j == 15 && v < 5) ? pat[v] : (((blk[j] >> v) & 1) ? 0xffffffffu : 0u);
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
  if (verify) {
#pragma unroll
    for (int i = 0; i < 128; ++i) out[gid * 128 + i] = st[i];
  } else {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 128; ++i) acc ^= st[i] * (i + 1);
    out[gid] = acc;
  }
}

// ---- host reference AES-128 ----
static uint8_t S[256];
static uint8_t gmul(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
    b >>= 1;
  }
  return r;
}
static void init_sbox() {
  for (int x = 0; x < 256; ++x) {
    uint8_t inv = 0;
    for (int y = 1; y < 256 && x; ++y)
      if (gmul((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
    uint8_t s = inv;
    for (int k = 1; k < 5; ++k) s ^= (uint8_t)((inv << k) | (inv >> (8 - k)));
    S[x] = s ^ 0x63;
  }
}
static void expand(const uint8_t key[16], uint8_t rk[11][16]) {
  memcpy(rk[0], key, 16);
  uint8_t rc = 1;
  for (int r = 1; r <= 10; ++r) {
    const uint8_t *p = rk[r - 1];
    uint8_t t[4] = {S[p[13]], S[p[14]], S[p[15]], S[p[12]]};
    t[0] ^= rc;
    rc = gmul(rc, 2);
    for (int i = 0; i < 4; ++i) rk[r][i] = p[i] ^ t[i];
    for (int i = 4; i < 16; ++i) rk[r][i] = p[i] ^ rk[r][i - 4];
  }
}
static void encrypt(const uint8_t rk[11][16], const uint8_t in[16], uint8_t out[16]) {
  uint8_t s[16];
  for (int i = 0; i < 16; ++i) s[i] = in[i] ^ rk[0][i];
  for (int r = 1; r <= 10; ++r) {
    uint8_t t[16];
    for (int c = 0; c < 4; ++c)
      for (int rw = 0; rw < 4; ++rw) t[4 * c + rw] = S[s[4 * ((c + rw) & 3) + rw]];
    if (r < 10) {
      for (int c = 0; c < 4; ++c) {
        uint8_t *a = &t[4 * c], b[4];
        for (int rw = 0; rw < 4; ++rw)
          b[rw] = gmul(a[rw], 2) ^ gmul(a[(rw + 1) & 3], 3) ^ a[(rw + 2) & 3] ^ a[(rw + 3) & 3];
        memcpy(a, b, 4);
      }
    }
    for (int i = 0; i < 16; ++i) s[i] = t[i] ^ rk[r][i];
  }
  memcpy(out, s, 16);
}

template <int WG>
static void timeit(uint32_t *drk, uint32_t *dout, int blocks_per_cu, int iters) {
  const int grid = 256 * blocks_per_cu;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(bsprobe<WG>, dim3(grid), dim3(WG), 0, 0, drk, dout, iters, 0);
  hipEventRecord(e0, 0);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(bsprobe<WG>, dim3(grid), dim3(WG), 0, 0, drk, dout, iters, 0);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= 3;
  const double blocks = (double)grid * WG * 32 * iters;  // AES blocks
  const double cu_cycles = ms * 1e-3 * 2.0e9;            // per CU at ~2.0 GHz
  printf("{\"wg\": %d, \"wgs_per_cu\": %d, \"ms\": %.3f, \"Mblocks_per_s\": %.0f, "
         "\"cu_cycles_per_block_round_at_2GHz\": %.4f}\n",
         WG, blocks_per_cu, ms, blocks / ms / 1e3, cu_cycles * 256 / (blocks * 10));
}

int main() {
  init_sbox();
  uint8_t key[16], rk[11][16];
  for (int i = 0; i < 16; ++i) key[i] = (uint8_t)(0x2b + 17 * i);
  expand(key, rk);
  uint32_t hk[44];
  for (int r = 0; r <= 10; ++r)
    for (int w = 0; w < 4; ++w) {
      uint32_t v = 0;
      for (int b = 0; b < 4; ++b) v |= (uint32_t)(rk[r][4 * w + b] ^ (r ? 0x63 : 0)) << (8 * b);
      hk[4 * r + w] = v;
    }
  uint32_t *drk, *dout;
  hipMalloc(&drk, sizeof hk);
  hipMemcpy(drk, hk, sizeof hk, hipMemcpyHostToDevice);
  const int vl = 256;
  hipMalloc(&dout, (size_t)256 * 8 * 1024 * 128 * 4);
  hipLaunchKernelGGL(bsprobe<256>, dim3(1), dim3(vl), 0, 0, drk, dout, 1, 1);
  static uint32_t h[256 * 128];
  hipMemcpy(h, dout, sizeof h, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int g = 0; g < vl; ++g)
    for (int s = 0; s < 32; ++s) {
      uint8_t blk[16], ref[16];
      for (int j = 0; j < 12; ++j) blk[j] = (uint8_t)(g * 131u + j * 29u + 7u);
      const uint32_t c = g * 32u + s;
      blk[12] = c >> 24, blk[13] = c >> 16, blk[14] = c >> 8, blk[15] = c;
      encrypt(rk, blk, ref);
      for (int j = 0; j < 16; ++j) {
        uint8_t d = 0;
        for (int v = 0; v < 8; ++v) d |= ((h[g * 128 + 8 * j + v] >> s) & 1) << v;
        d ^= rk[10][j] ^ 0x63;
        if (d != ref[j]) ++bad;
      }
    }
  printf("{\"verify_bad_bytes\": %d, \"of\": %d}\n", bad, vl * 32 * 16);
  if (bad) return 1;
  for (int bpc : {1, 2, 3, 4}) timeit<256>(drk, dout, bpc, 40);
  for (int bpc : {1, 2}) timeit<512>(drk, dout, bpc, 40);
  return 0;
}
