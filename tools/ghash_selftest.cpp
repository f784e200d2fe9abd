// Host self-test of the GHASH table layout the GCM kernel uses
// (host_crypto.cpp ghash_tables): the 4-bit H^1..H^8 and H^16 tables, each
// evaluated exactly the way esp_gcm.hip indexes them, against gf128_mul
// (SP 800-38D Alg. 1).  Also the paired stride-8 Horner (Y*H^16 ^ Ba*H^8 ^ Bb,
// Y*H^8 ^ Ba on an odd last step) + final H^(8-l) combination against a
// serial GHASH.  Built and run by tests/test_host_selftests.py.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

// layout constants, mirrored from espgpu_internal.h (which needs HIP vector types)
static constexpr unsigned kGhPowerBytes = 8192, kGh16Off = 8 * 8192, kGhTableBytes = 73728;
#include "host_crypto.h"

using namespace espgpu;
static_assert(kGhTableBytes == kGh16Off + kGhPowerBytes, "layout");

static void xor16(uint8_t *a, const uint8_t *b) { for (int i = 0; i < 16; ++i) a[i] ^= b[i]; }

// as gf_mul4_global: nibble position j = 2p (low) / 2p+1 (high), row j*256
static void mul4(const uint8_t *t, const uint8_t x[16], uint8_t out[16]) {
  memset(out, 0, 16);
  for (int p = 0; p < 16; ++p) {
    xor16(out, t + (2 * p) * 256 + (x[p] & 15) * 16);
    xor16(out, t + (2 * p + 1) * 256 + (x[p] >> 4) * 16);
  }
}

int main() {
  std::vector<uint8_t> tabs(kGhTableBytes);
  srand(7);
  for (int trial = 0; trial < 20; ++trial) {
    uint8_t h[16], pw[9][16];
    for (auto &b : h) b = rand() & 0xff;
    hc::ghash_tables(h, tabs.data());
    memcpy(pw[1], h, 16);
    for (int e = 2; e <= 8; ++e) hc::gf128_mul(pw[e - 1], h, pw[e]);
    for (int it = 0; it < 50; ++it) {
      uint8_t x[16], a[16], b[16];
      for (auto &v : x) v = rand() & 0xff;
      for (int e = 1; e <= 8; ++e) {
        hc::gf128_mul(x, pw[e], a);
        mul4(tabs.data() + (e - 1) * kGhPowerBytes, x, b);
        if (memcmp(a, b, 16)) { printf("4-bit H^%d table mismatch\n", e); return 1; }
      }
      uint8_t h16[16];
      hc::gf128_mul(pw[8], pw[8], h16);
      hc::gf128_mul(x, h16, a);
      mul4(tabs.data() + kGh16Off, x, b);
      if (memcmp(a, b, 16)) { printf("4-bit H^16 table mismatch\n"); return 1; }
    }
    // stride-8 Horner over N blocks (front-padded to 8M) vs serial GHASH
    for (int N : {1, 3, 8, 9, 93, 562}) {
      std::vector<uint8_t> X(16 * N);
      for (auto &v : X) v = rand() & 0xff;
      uint8_t ser[16] = {0}, t[16];
      for (int i = 0; i < N; ++i) { xor16(ser, &X[16 * i]); hc::gf128_mul(ser, h, t); memcpy(ser, t, 16); }
      const int M = (N + 7) / 8, pad = 8 * M - N;
      uint8_t Z[16] = {0};
      for (int l = 0; l < 8; ++l) {
        uint8_t Y[16] = {0};
        // paired steps as esp_gcm.hip: Y*H^16 ^ Ba*H^8 ^ Bb, or Y*H^8 ^ Ba
        for (int m = 0; m < M; m += 2) {
          const int ia = 8 * m + l - pad, ib = ia + 8;
          uint8_t Ba[16] = {0}, Bb[16] = {0}, p1[16], p2[16];
          if (ia >= 0) memcpy(Ba, &X[16 * ia], 16);
          if (m + 1 < M) {
            memcpy(Bb, &X[16 * ib], 16);
            mul4(tabs.data() + kGh16Off, Y, p1);
            mul4(tabs.data() + 7 * kGhPowerBytes, Ba, p2);
            xor16(p1, p2);
            xor16(p1, Bb);
          } else {
            mul4(tabs.data() + 7 * kGhPowerBytes, Y, p1);
            xor16(p1, Ba);
          }
          memcpy(Y, p1, 16);
        }
        mul4(tabs.data() + (7 - l) * kGhPowerBytes, Y, t);
        xor16(Z, t);
      }
      if (memcmp(Z, ser, 16)) { printf("Horner mismatch N=%d\n", N); return 1; }
    }
  }
  printf("ghash selftest OK\n");
  return 0;
}
