// Host self-test of the bitsliced AES (tools/aes_bs.h) that the measurement
// probes run (tools/bsprobe.hip; round 3's bitsliced ctr pass, measured
// slower and no longer built):
// the header is built for the CPU with its two gfx950 builtins emulated
// (v_bitop3_b32's truth table over a=0xf0, b=0xcc, c=0xaa; v_perm_b32's byte
// select), and 32 counter blocks nonce || ctr are encrypted the kernel's way
// -- bitsliced input, K0 then K_r ^ 0x63.. folded into the S-box inputs, the
// last key added after the 32x32 transposes -- for AES-128/192/256 and
// compared with host_crypto.cpp's table AES.  Built and run by
// tests/test_host_selftests.py.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <initializer_list>

static uint32_t host_bitop3(uint32_t a, uint32_t b, uint32_t c, uint32_t tt) {
  uint32_t r = 0;
  for (int idx = 0; idx < 8; ++idx)
    if ((tt >> idx) & 1)
      r |= ((idx & 4) ? a : ~a) & ((idx & 2) ? b : ~b) & ((idx & 1) ? c : ~c);
  return r;
}
// v_perm_b32 (selectors 0..7 only): byte k of the result = byte sel_k of {hi, lo}
static uint32_t host_perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  const uint64_t v = ((uint64_t)hi << 32) | lo;
  uint32_t r = 0;
  for (int k = 0; k < 4; ++k) r |= (uint32_t)((v >> (8 * ((sel >> (8 * k)) & 7))) & 0xff) << (8 * k);
  return r;
}
#define ESPGPU_HOST_SHIM 1
#define __device__
#define __forceinline__ inline
#define __builtin_amdgcn_bitop3_b32(a, b, c, t) host_bitop3((a), (b), (c), (t))
#define __builtin_amdgcn_perm(hi, lo, sel) host_perm((hi), (lo), (sel))
#include "aes_bs.h"
#include "host_crypto.h"

using namespace espgpu;

static uint32_t bswap(uint32_t v) { return __builtin_bswap32(v); }

int main() {
  int bad = 0, checked = 0;
  uint32_t seed = 12345;
  auto rnd = [&]() { seed = seed * 1664525u + 1013904223u; return seed >> 8; };
  for (int klen : {16, 24, 32}) {
    for (int trial = 0; trial < 8; ++trial) {
      uint8_t key[32];
      for (int i = 0; i < klen; ++i) key[i] = (uint8_t)rnd();
      uint32_t rk[60];
      const int nr = hc::aes_expand_enc(key, klen, rk);
      // the DevSA::dk form (espgpu.cpp newsession): little-endian words, K_r ^ 0x63.. for r >= 1
      uint32_t dk[60];
      for (int i = 0; i < 4 * (nr + 1); ++i) dk[i] = bswap(rk[i]) ^ (i >= 4 ? 0x63636363u : 0u);
      // a window: counters 32w .. 32w+31 of one record's nonce (salt || IV)
      uint8_t nonce[12];
      for (int i = 0; i < 12; ++i) nonce[i] = (uint8_t)rnd();
      const uint32_t w = trial * 37 % 300;
      uint32_t W[4];
      memcpy(W, nonce, 12);
      W[3] = bswap(32u * w);
      uint32_t st[128];
      for (int j = 0; j < 16; ++j)
        for (int b = 0; b < 8; ++b)
          st[8 * j + b] = (uint32_t)((int32_t)(W[j >> 2] << (31 - (8 * (j & 3) + b))) >> 31);
      const uint32_t pat[5] = {0xAAAAAAAAu, 0xCCCCCCCCu, 0xF0F0F0F0u, 0xFF00FF00u, 0xFFFF0000u};
      for (int b = 0; b < 5; ++b) st[120 + b] = pat[b];
      for (int r = 0; r < nr - 1; ++r) bs::round<true>(st, &dk[4 * r]);
      bs::round<false>(st, &dk[4 * (nr - 1)]);
      for (int g = 0; g < 4; ++g) {
        bs::transpose32(&st[32 * g]);
        for (int s = 0; s < 32; ++s) st[32 * g + s] ^= dk[4 * nr + g];
      }
      for (int s = 0; s < 32; ++s) {
        uint8_t blk[16], ref[16], got[16];
        memcpy(blk, nonce, 12);
        const uint32_t ctr = 32u * w + (uint32_t)s;
        blk[12] = ctr >> 24, blk[13] = ctr >> 16, blk[14] = ctr >> 8, blk[15] = ctr;
        hc::aes_encrypt_block(rk, nr, blk, ref);
        for (int g = 0; g < 4; ++g) memcpy(got + 4 * g, &st[32 * g + s], 4);
        ++checked;
        if (memcmp(got, ref, 16)) ++bad;
      }
    }
  }
  printf("%s: %d of %d blocks differ\n", bad ? "FAIL" : "OK", bad, checked);
  return bad != 0;
}
