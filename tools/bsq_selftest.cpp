// Host model of the quad-bitsliced AES-CTR step (esp_gcm.hip aes_ctr8_bsq,
// GCM_HYBRID): the 4 lanes of one record compute the 8 counter blocks of a
// pair step together, lane q holding row q of the state as 8 bit planes
// (bit 8c + b of plane i = bit i of state byte (q, c) of block b).  S-box:
// aes_bs.h's circuit (S' = S ^ 0x63, so the round keys are DevSA::dk's
// K_r ^ 0x63..); ShiftRows: rotate right by 8q; MixColumns: rows q+1 and q+2
// come from the quad's other lanes (DPP quad_perm on the device).  The 4
// lanes are emulated explicitly here, each device step mirrored one to one,
// and every keystream block is compared with host_crypto.cpp's table AES.
// Built and run by tests/test_host_selftests.py.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <initializer_list>

static uint32_t host_bitop3(uint32_t a, uint32_t b, uint32_t c, uint32_t tt) {
  uint32_t r = 0;
  for (int idx = 0; idx < 8; ++idx)
    if ((tt >> idx) & 1) r |= ((idx & 4) ? a : ~a) & ((idx & 2) ? b : ~b) & ((idx & 1) ? c : ~c);
  return r;
}
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
static uint32_t rotr(uint32_t x, int s) { return s ? (x >> s) | (x << (32 - s)) : x; }

// swapmove ladder: afterwards bit i (within each byte) of a[s] = bit s of the old a[i]
static void transpose8(uint32_t a[8]) {
  const uint32_t M[3] = {0x0F0F0F0Fu, 0x33333333u, 0x55555555u};
  for (int q = 0; q < 3; ++q) {
    const int j = 4 >> q;
    for (int k = 0; k < 8; ++k) {
      if (k & j) continue;
      const uint32_t t = ((a[k] >> j) ^ a[k + j]) & M[q];
      a[k + j] ^= t;
      a[k] ^= t << j;
    }
  }
}

int main() {
  uint32_t seed = 777;
  auto rnd = [&]() { seed = seed * 1664525u + 1013904223u; return seed >> 8; };
  int bad = 0, checked = 0;
  for (int trial = 0; trial < 200; ++trial) {
    uint8_t key[16];
    for (auto &k : key) k = (uint8_t)rnd();
    uint32_t rk[60];
    const int nr = hc::aes_expand_enc(key, 16, rk);
    uint32_t dk[60];                                  // DevSA::dk: LE words, K_r ^ 0x63 for r >= 1
    for (int i = 0; i < 4 * (nr + 1); ++i) dk[i] = bswap(rk[i]) ^ (i >= 4 ? 0x63636363u : 0u);
    // kernel form of round 0 (BE words) and the state words entering round 1
    uint8_t nonce[12];
    for (auto &v : nonce) v = (uint8_t)rnd();
    uint32_t nw[3];
    memcpy(nw, nonce, 12);
    const uint32_t s0c = bswap(nw[0]) ^ rk[0], s1c = bswap(nw[1]) ^ rk[1], s2c = bswap(nw[2]) ^ rk[2];
    const uint32_t rk3 = rk[3];
    // counters of the step's 8 blocks: ctr0 + b (slot 4a + b -> counter 4a + 2 + b);
    // include runs that carry across bytes
    uint32_t ctr0 = trial < 100 ? 4u * (rnd() % 600) + 2u : (rnd() | 0xf8u) - (rnd() & 3u);
    // key planes as the workgroup builds them in LDS: KP[r-1][q][i], byte c =
    // bit i of key byte (q, c) of K'_r = byte q of dk[4r + c]
    uint32_t KP[10][4][8];
    for (int r = 1; r <= nr; ++r)
      for (int q = 0; q < 4; ++q)
        for (int i = 0; i < 8; ++i) {
          uint32_t w = 0;
          for (int c = 0; c < 4; ++c) w |= (((dk[4 * r + c] >> (8 * q + i)) & 1u) * 0xffu) << (8 * c);
          KP[r - 1][q][i] = w;
        }
    // ---- per lane (row q): input words W[b] (byte c = state byte (q, c) of block b) ----
    uint32_t P[4][8];
    for (int q = 0; q < 4; ++q) {
      const int sh = 24 - 8 * q;                      // byte q of a BE word
      const uint32_t R = ((s0c >> sh) & 0xff) | (((s1c >> sh) & 0xff) << 8) | (((s2c >> sh) & 0xff) << 16);
      uint32_t W[8];
      for (int b = 0; b < 8; ++b) W[b] = R | ((((ctr0 + (uint32_t)b) ^ rk3) << (8 * q)) & 0xff000000u);
      transpose8(W);                                  // W[i] now plane i
      memcpy(P[q], W, sizeof W);
    }
    for (int r = 1; r <= nr; ++r) {
      for (int q = 0; q < 4; ++q) {
        bs::sbox(P[q], 0);                            // S'(x) = S(x) ^ 0x63
        for (int i = 0; i < 8; ++i) P[q][i] = rotr(P[q][i], 8 * q);   // ShiftRows
      }
      if (r < nr) {
        uint32_t t[4][8], u[4][8], o[4][8];
        for (int q = 0; q < 4; ++q)
          for (int i = 0; i < 8; ++i) t[q][i] = P[q][i] ^ P[(q + 1) & 3][i];      // dpp quad_perm [1,2,3,0]
        for (int q = 0; q < 4; ++q)
          for (int i = 0; i < 8; ++i) u[q][i] = t[q][i] ^ t[(q + 2) & 3][i];      // dpp quad_perm [2,3,0,1]
        for (int q = 0; q < 4; ++q) {
          const uint32_t *T = t[q], h = T[7];
          const uint32_t xt[8] = {h, T[0] ^ h, T[1], T[2] ^ h, T[3] ^ h, T[4], T[5], T[6]};
          for (int i = 0; i < 8; ++i) o[q][i] = xt[i] ^ u[q][i] ^ P[q][i];
        }
        memcpy(P, o, sizeof o);
      }
      for (int q = 0; q < 4; ++q)
        for (int i = 0; i < 8; ++i) P[q][i] ^= KP[r - 1][q][i];
    }
    // ---- output: planes -> words, quad 4x4 transposes, byte transposes ----
    uint32_t A[4][8];
    for (int q = 0; q < 4; ++q) {
      memcpy(A[q], P[q], sizeof P[q]);
      transpose8(A[q]);                               // A[q][b]: byte c = keystream byte (q, c) of block b
    }
    for (int d : {2, 1})
      for (int half = 0; half < 2; ++half)
        for (int b = 0; b < 4; ++b) {
          if (b & d) continue;
          const int x0 = 4 * half + b, x1 = x0 + d;
          uint32_t send[4];
          for (int q = 0; q < 4; ++q) send[q] = (q & d) ? A[q][x0] : A[q][x1];
          for (int q = 0; q < 4; ++q) {
            const uint32_t y = send[q ^ d];           // dpp quad_perm xor d
            if (q & d) A[q][x0] = y; else A[q][x1] = y;
          }
        }
    for (int q = 0; q < 4; ++q)
      for (int half = 0; half < 2; ++half) {
        const uint32_t *X = &A[q][4 * half];          // X[r]: byte c = keystream byte (r, c) of block q + 4*half
        const uint32_t T0 = host_perm(X[1], X[0], 0x05010400u), T1 = host_perm(X[1], X[0], 0x07030602u);
        const uint32_t T2 = host_perm(X[3], X[2], 0x05010400u), T3 = host_perm(X[3], X[2], 0x07030602u);
        const uint32_t C[4] = {host_perm(T2, T0, 0x05040100u), host_perm(T2, T0, 0x07060302u),
                               host_perm(T3, T1, 0x05040100u), host_perm(T3, T1, 0x07060302u)};
        // reference: E_K(nonce || BE32(ctr0 + block))
        const uint32_t blk = (uint32_t)q + 4u * (uint32_t)half;
        uint8_t in[16], ref[16];
        memcpy(in, nonce, 12);
        const uint32_t cv = ctr0 + blk;
        in[12] = (uint8_t)(cv >> 24), in[13] = (uint8_t)(cv >> 16), in[14] = (uint8_t)(cv >> 8), in[15] = (uint8_t)cv;
        hc::aes_encrypt_block(rk, nr, in, ref);
        ++checked;
        if (memcmp(C, ref, 16)) {
          if (bad < 5) printf("mismatch trial %d block %u\n", trial, blk);
          ++bad;
        }
      }
  }
  if (bad) {
    printf("FAIL %d of %d\n", bad, checked);
    return 1;
  }
  printf("OK quad-bitsliced AES-128: %d keystream blocks\n", checked);
  return 0;
}
