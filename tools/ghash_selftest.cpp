// Host self-test of the GHASH table layouts the GCM kernel uses
// (host_crypto.cpp ghash_tables): the 4-bit H^1..H^8 tables (global,
// gf_mul4_global) and the 8-bit H^4 / H^8 Horner tables the kernels expand
// from them in LDS (stage_h8_lds; ghash_expand8 is its host mirror, gf_mul8),
// each evaluated exactly the way esp_gcm.hip indexes it, against gf128_mul
// (SP 800-38D Alg. 1).  Also the
// stride-S Horner + final H^(S-l) combination, S = 4 and 8, against a serial
// GHASH.  Built and run by tests/test_host_selftests.py.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

// layout constants, mirrored from espgpu_internal.h (which needs HIP vector types)
static constexpr int S = 4;   // kGcmLanesPerRec: lanes per record = Horner stride
static constexpr int S2 = 8;  // kGcmLanesSmall: the small-batch kernel's stride
static constexpr unsigned kGhPowerBytes = 8192, kGh8Bytes = 65536, kGhTableBytes = 8 * kGhPowerBytes;
#include "host_crypto.h"

using namespace espgpu;
static_assert(kGhTableBytes == 65536, "layout");

static void xor16(uint8_t *a, const uint8_t *b) { for (int i = 0; i < 16; ++i) a[i] ^= b[i]; }

// as gf_mul8: byte position p (memory order), value v at v*256 + p*16
static void mul8(const uint8_t *tab, const uint8_t x[16], uint8_t out[16]) {
  memset(out, 0, 16);
  for (int p = 0; p < 16; ++p) xor16(out, tab + x[p] * 256 + p * 16);
}
// as gf_mul4_global: nibble position j = 2p (low) / 2p+1 (high), row j*256
static void mul4(const uint8_t *t, const uint8_t x[16], uint8_t out[16]) {
  memset(out, 0, 16);
  for (int p = 0; p < 16; ++p) {
    xor16(out, t + (2 * p) * 256 + (x[p] & 15) * 16);
    xor16(out, t + (2 * p + 1) * 256 + (x[p] >> 4) * 16);
  }
}

int main() {
  std::vector<uint8_t> tabs(kGhTableBytes), t8s(kGh8Bytes), t88(kGh8Bytes);
  srand(7);
  for (int trial = 0; trial < 20; ++trial) {
    uint8_t h[16], pw[9][16];
    for (auto &b : h) b = rand() & 0xff;
    hc::ghash_tables(h, tabs.data());
    hc::ghash_expand8(tabs.data() + (S - 1) * kGhPowerBytes, t8s.data());
    hc::ghash_expand8(tabs.data() + (S2 - 1) * kGhPowerBytes, t88.data());
    memcpy(pw[1], h, 16);
    for (int e = 2; e <= 8; ++e) hc::gf128_mul(pw[e - 1], h, pw[e]);
    for (int it = 0; it < 50; ++it) {
      uint8_t x[16], a[16], b[16];
      for (auto &v : x) v = rand() & 0xff;
      hc::gf128_mul(x, pw[S], a);
      mul8(t8s.data(), x, b);
      if (memcmp(a, b, 16)) { printf("8-bit H^S table mismatch\n"); return 1; }
      hc::gf128_mul(x, pw[S2], a);
      mul8(t88.data(), x, b);
      if (memcmp(a, b, 16)) { printf("8-bit H^8 table mismatch\n"); return 1; }
      for (int e = 1; e <= 8; ++e) {
        hc::gf128_mul(x, pw[e], a);
        mul4(tabs.data() + (e - 1) * kGhPowerBytes, x, b);
        if (memcmp(a, b, 16)) { printf("4-bit H^%d table mismatch\n", e); return 1; }
      }
    }
    // stride-S Horner over N blocks (front-padded to S*M) vs serial GHASH
    for (int st : {S, S2})
    for (int N : {1, 3, 8, 9, 93, 562}) {
      const int S = st;
      const uint8_t *g8 = S == 4 ? t8s.data() : t88.data();
      std::vector<uint8_t> X(16 * N);
      for (auto &v : X) v = rand() & 0xff;
      uint8_t ser[16] = {0}, t[16];
      for (int i = 0; i < N; ++i) { xor16(ser, &X[16 * i]); hc::gf128_mul(ser, h, t); memcpy(ser, t, 16); }
      const int M = (N + S - 1) / S, pad = S * M - N;
      uint8_t Z[16] = {0};
      for (int l = 0; l < S; ++l) {
        uint8_t Y[16] = {0};
        for (int m = 0; m < M; ++m) {
          if (m > 0) { mul8(g8, Y, t); memcpy(Y, t, 16); }
          const int i = S * m + l - pad;
          if (i >= 0) xor16(Y, &X[16 * i]);
        }
        mul4(tabs.data() + (S - 1 - l) * kGhPowerBytes, Y, t);
        xor16(Z, t);
      }
      if (memcmp(Z, ser, 16)) { printf("Horner mismatch S=%d N=%d\n", S, N); return 1; }
    }
  }
  printf("ghash selftest OK\n");
  return 0;
}
