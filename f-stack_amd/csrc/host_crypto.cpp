// host_crypto.cpp — see host_crypto.h.
#include "host_crypto.h"
#include "sha512_consts.h"

#include <string.h>

namespace espgpu {
namespace hc {

namespace {

uint8_t xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

uint8_t mul8(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  for (; b; b >>= 1, a = xt(a))
    if (b & 1) r ^= a;
  return r;
}

Tables build() {
  Tables t;
  // log/antilog over generator 3 gives inverses without a search
  uint8_t lg[256] = {0}, alg[256] = {0};
  uint8_t v = 1;
  for (int i = 0; i < 255; ++i) {
    alg[i] = v;
    lg[v] = (uint8_t)i;
    v = mul8(v, 3);
  }
  for (int x = 0; x < 256; ++x) {
    uint8_t inv = x ? alg[(255 - lg[x]) % 255] : 0;
    uint8_t s = inv;
    for (int r = 1; r <= 4; ++r) s ^= (uint8_t)((inv << r) | (inv >> (8 - r)));
    s ^= 0x63;
    t.sbox[x] = s;
    t.isbox[s] = (uint8_t)x;
  }
  for (int x = 0; x < 256; ++x) {
    uint8_t s = t.sbox[x], i = t.isbox[x];
    t.te0[x] = ((uint32_t)mul8(s, 2) << 24) | ((uint32_t)s << 16) | ((uint32_t)s << 8) | mul8(s, 3);
    t.td0[x] = ((uint32_t)mul8(i, 14) << 24) | ((uint32_t)mul8(i, 9) << 16) |
               ((uint32_t)mul8(i, 13) << 8) | mul8(i, 11);
  }
  return t;
}

uint32_t be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
void put_be32(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
}
uint32_t rotr(uint32_t v, int n) { return n ? (v >> n) | (v << (32 - n)) : v; }

uint32_t sub_word(uint32_t w) {
  const Tables &t = tables();
  return ((uint32_t)t.sbox[w >> 24] << 24) | ((uint32_t)t.sbox[(w >> 16) & 255] << 16) |
         ((uint32_t)t.sbox[(w >> 8) & 255] << 8) | t.sbox[w & 255];
}

uint32_t inv_mix(uint32_t w) {
  uint8_t a[4] = {(uint8_t)(w >> 24), (uint8_t)(w >> 16), (uint8_t)(w >> 8), (uint8_t)w};
  static const uint8_t m[4][4] = {{14, 11, 13, 9}, {9, 14, 11, 13}, {13, 9, 14, 11}, {11, 13, 9, 14}};
  uint32_t r = 0;
  for (int i = 0; i < 4; ++i) {
    uint8_t b = 0;
    for (int j = 0; j < 4; ++j) b ^= mul8(a[j], m[i][j]);
    r = (r << 8) | b;
  }
  return r;
}

}  // namespace

const Tables &tables() {
  static const Tables t = build();
  return t;
}

int aes_expand_enc(const uint8_t *key, int klen, uint32_t rk[60]) {
  if (klen != 16 && klen != 24 && klen != 32) return 0;
  const int nk = klen / 4, nr = nk + 6, total = 4 * (nr + 1);
  uint32_t rcon = 0x01000000u;
  for (int i = 0; i < nk; ++i) rk[i] = be32(key + 4 * i);
  for (int i = nk; i < total; ++i) {
    uint32_t t = rk[i - 1];
    if (i % nk == 0) {
      t = sub_word((t << 8) | (t >> 24)) ^ rcon;
      rcon = (uint32_t)xt((uint8_t)(rcon >> 24)) << 24;
    } else if (nk == 8 && i % nk == 4) {
      t = sub_word(t);
    }
    rk[i] = rk[i - nk] ^ t;
  }
  return nr;
}

int aes_expand_dec(const uint8_t *key, int klen, uint32_t dk[60]) {
  uint32_t ek[60];
  const int nr = aes_expand_enc(key, klen, ek);
  if (!nr) return 0;
  for (int r = 0; r <= nr; ++r)
    for (int c = 0; c < 4; ++c) {
      uint32_t w = ek[4 * (nr - r) + c];
      dk[4 * r + c] = (r == 0 || r == nr) ? w : inv_mix(w);
    }
  return nr;
}

void aes_encrypt_block(const uint32_t *rk, int nr, const uint8_t in[16], uint8_t out[16]) {
  const Tables &t = tables();
  uint32_t s[4], n[4];
  for (int c = 0; c < 4; ++c) s[c] = be32(in + 4 * c) ^ rk[c];
  for (int r = 1; r < nr; ++r) {
    for (int c = 0; c < 4; ++c)
      n[c] = t.te0[s[c] >> 24] ^ rotr(t.te0[(s[(c + 1) & 3] >> 16) & 255], 8) ^
             rotr(t.te0[(s[(c + 2) & 3] >> 8) & 255], 16) ^ rotr(t.te0[s[(c + 3) & 3] & 255], 24) ^
             rk[4 * r + c];
    memcpy(s, n, sizeof s);
  }
  for (int c = 0; c < 4; ++c) {
    uint32_t w = ((uint32_t)t.sbox[s[c] >> 24] << 24) | ((uint32_t)t.sbox[(s[(c + 1) & 3] >> 16) & 255] << 16) |
                 ((uint32_t)t.sbox[(s[(c + 2) & 3] >> 8) & 255] << 8) | t.sbox[s[(c + 3) & 3] & 255];
    put_be32(out + 4 * c, w ^ rk[4 * nr + c]);
  }
}

void gf128_mul(const uint8_t x[16], const uint8_t y[16], uint8_t out[16]) {
  uint64_t zh = 0, zl = 0;
  uint64_t vh = 0, vl = 0;
  for (int i = 0; i < 8; ++i) {
    vh = (vh << 8) | y[i];
    vl = (vl << 8) | y[8 + i];
  }
  for (int i = 0; i < 128; ++i) {
    if ((x[i >> 3] >> (7 - (i & 7))) & 1) {
      zh ^= vh;
      zl ^= vl;
    }
    const bool lsb = vl & 1;
    vl = (vl >> 1) | (vh << 63);
    vh >>= 1;
    if (lsb) vh ^= 0xE100000000000000ull;
  }
  for (int i = 0; i < 8; ++i) {
    out[i] = (uint8_t)(zh >> (56 - 8 * i));
    out[8 + i] = (uint8_t)(zl >> (56 - 8 * i));
  }
}

void ghash_tables(const uint8_t h[16], uint8_t *out) {
  // H^1..H^8 (index 0..7) with 4-bit indices: power p, nibble position j
  // (byte j>>1, low nibble if j even), value n at p*8192 + j*256 + n*16 =
  // (the block whose nibble j is n) * H^(p+1).  The kernels' 8-bit Horner
  // tables are expanded from these on the device (ghash_expand8).
  uint8_t pw[8][16];
  memcpy(pw[0], h, 16);
  for (int p = 1; p < 8; ++p) gf128_mul(pw[p - 1], h, pw[p]);
  for (int p = 0; p < 8; ++p) {
    // products of every single-bit block with H^(p+1)
    uint8_t bit[128][16];
    for (int b = 0; b < 128; ++b) {
      uint8_t e[16] = {0};
      e[b >> 3] = (uint8_t)(1u << (b & 7));   // bit (b&7) of byte b>>3 (LSB = 0)
      gf128_mul(e, pw[p], bit[b]);
    }
    for (int j = 0; j < 32; ++j) {
      const int byte = j >> 1, sh = (j & 1) * 4;
      for (int n = 0; n < 16; ++n) {
        uint8_t acc[16] = {0};
        for (int t = 0; t < 4; ++t)
          if (n & (1 << t))
            for (int k = 0; k < 16; ++k) acc[k] ^= bit[byte * 8 + sh + t][k];
        memcpy(out + ((size_t)p * 32 * 16 + (size_t)j * 16 + n) * 16, acc, 16);
      }
    }
  }
}

void ghash_expand8(const uint8_t *t4, uint8_t *t8) {
  // the multiply is GF(2)-linear in the block: byte q = v contributes the
  // low nibble's product plus the high nibble's (esp_gcm.hip stage_h8)
  for (int q = 0; q < 16; ++q)
    for (int v = 0; v < 256; ++v) {
      const uint8_t *lo = t4 + (2 * q) * 256 + (v & 15) * 16;
      const uint8_t *hi = t4 + (2 * q + 1) * 256 + (v >> 4) * 16;
      for (int k = 0; k < 16; ++k) t8[(size_t)v * 256 + (size_t)q * 16 + k] = lo[k] ^ hi[k];
    }
}

void sha1_compress(uint32_t h[5], const uint8_t blk[64]) {
  uint32_t w[80];
  for (int i = 0; i < 16; ++i) w[i] = be32(blk + 4 * i);
  for (int i = 16; i < 80; ++i) {
    uint32_t x = w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16];
    w[i] = (x << 1) | (x >> 31);
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
  for (int i = 0; i < 80; ++i) {
    uint32_t f, k;
    if (i < 20) { f = (b & c) | (~b & d); k = 0x5a827999u; }
    else if (i < 40) { f = b ^ c ^ d; k = 0x6ed9eba1u; }
    else if (i < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8f1bbcdcu; }
    else { f = b ^ c ^ d; k = 0xca62c1d6u; }
    uint32_t t = ((a << 5) | (a >> 27)) + f + e + k + w[i];
    e = d; d = c; c = (b << 30) | (b >> 2); b = a; a = t;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

static void sha1_full(const uint8_t *m, int len, uint8_t out[20]) {
  uint32_t h[5] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u, 0xc3d2e1f0u};
  int off = 0;
  for (; len - off >= 64; off += 64) sha1_compress(h, m + off);
  uint8_t tail[128] = {0};
  const int rem = len - off;
  memcpy(tail, m + off, (size_t)rem);
  tail[rem] = 0x80;
  const int tl = (rem + 9 <= 64) ? 64 : 128;
  const uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; ++i) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
  sha1_compress(h, tail);
  if (tl == 128) sha1_compress(h, tail + 64);
  for (int i = 0; i < 5; ++i) put_be32(out + 4 * i, h[i]);
}

void hmac_sha1_pad_state(const uint8_t *key, int klen, uint8_t padval, uint32_t h[5]) {
  uint8_t k[64] = {0};
  if (klen > 64) sha1_full(key, klen, k);
  else if (klen > 0) memcpy(k, key, (size_t)klen);
  for (int i = 0; i < 64; ++i) k[i] ^= padval;
  h[0] = 0x67452301u; h[1] = 0xefcdab89u; h[2] = 0x98badcfeu; h[3] = 0x10325476u; h[4] = 0xc3d2e1f0u;
  sha1_compress(h, k);
}

// SHA-256 (FIPS 180-4; freebsd/crypto/sha2/sha256c.c SHA256_Transform :135)
static const uint32_t K256[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u,
};
static inline uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

void sha256_compress(uint32_t h[8], const uint8_t blk[64]) {
  uint32_t w[64], v[8];
  for (int i = 0; i < 16; ++i) w[i] = be32(blk + 4 * i);
  for (int i = 16; i < 64; ++i) {
    const uint32_t s0 = rotr32(w[i - 15], 7) ^ rotr32(w[i - 15], 18) ^ (w[i - 15] >> 3);
    const uint32_t s1 = rotr32(w[i - 2], 17) ^ rotr32(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  for (int i = 0; i < 8; ++i) v[i] = h[i];
  for (int i = 0; i < 64; ++i) {
    const uint32_t t1 = v[7] + (rotr32(v[4], 6) ^ rotr32(v[4], 11) ^ rotr32(v[4], 25)) +
                        ((v[4] & v[5]) ^ (~v[4] & v[6])) + K256[i] + w[i];
    const uint32_t t2 = (rotr32(v[0], 2) ^ rotr32(v[0], 13) ^ rotr32(v[0], 22)) +
                        ((v[0] & v[1]) ^ (v[0] & v[2]) ^ (v[1] & v[2]));
    v[7] = v[6]; v[6] = v[5]; v[5] = v[4]; v[4] = v[3] + t1;
    v[3] = v[2]; v[2] = v[1]; v[1] = v[0]; v[0] = t1 + t2;
  }
  for (int i = 0; i < 8; ++i) h[i] += v[i];
}

static const uint32_t kSha256Iv[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                      0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

static void sha256_full(const uint8_t *m, int len, uint8_t out[32]) {
  uint32_t h[8];
  memcpy(h, kSha256Iv, sizeof h);
  int off = 0;
  for (; len - off >= 64; off += 64) sha256_compress(h, m + off);
  uint8_t tail[128] = {0};
  const int rem = len - off;
  memcpy(tail, m + off, (size_t)rem);
  tail[rem] = 0x80;
  const int tl = (rem + 9 <= 64) ? 64 : 128;
  const uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; ++i) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
  sha256_compress(h, tail);
  if (tl == 128) sha256_compress(h, tail + 64);
  for (int i = 0; i < 8; ++i) put_be32(out + 4 * i, h[i]);
}

// hmac_init_pad (crypto.c:413-441) for HMAC-SHA2-256: the chaining state
// after the padded key block (the key is hashed first when longer than 64)
void hmac_sha256_pad_state(const uint8_t *key, int klen, uint8_t padval, uint32_t h[8]) {
  uint8_t k[64] = {0};
  if (klen > 64) sha256_full(key, klen, k);
  else if (klen > 0) memcpy(k, key, (size_t)klen);
  for (int i = 0; i < 64; ++i) k[i] ^= padval;
  memcpy(h, kSha256Iv, 32);
  sha256_compress(h, k);
}

// SHA-512 / SHA-384 (FIPS 180-4; freebsd/crypto/sha2/sha512c.c SHA512_Transform
// :196): 128-byte blocks of 64-bit words; constants from sha512_consts.h
static const uint64_t K512[80] = ESPGPU_SHA512_K;
static const uint64_t kSha512Iv[8] = ESPGPU_SHA512_IV, kSha384Iv[8] = ESPGPU_SHA384_IV;
static inline uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
static inline uint64_t be64(const uint8_t *p) { return ((uint64_t)be32(p) << 32) | be32(p + 4); }

void sha512_compress(uint64_t h[8], const uint8_t blk[128]) {
  uint64_t w[80], v[8];
  for (int i = 0; i < 16; ++i) w[i] = be64(blk + 8 * i);
  for (int i = 16; i < 80; ++i) {
    const uint64_t s0 = rotr64(w[i - 15], 1) ^ rotr64(w[i - 15], 8) ^ (w[i - 15] >> 7);
    const uint64_t s1 = rotr64(w[i - 2], 19) ^ rotr64(w[i - 2], 61) ^ (w[i - 2] >> 6);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  for (int i = 0; i < 8; ++i) v[i] = h[i];
  for (int i = 0; i < 80; ++i) {
    const uint64_t t1 = v[7] + (rotr64(v[4], 14) ^ rotr64(v[4], 18) ^ rotr64(v[4], 41)) +
                        ((v[4] & v[5]) ^ (~v[4] & v[6])) + K512[i] + w[i];
    const uint64_t t2 = (rotr64(v[0], 28) ^ rotr64(v[0], 34) ^ rotr64(v[0], 39)) +
                        ((v[0] & v[1]) ^ (v[0] & v[2]) ^ (v[1] & v[2]));
    v[7] = v[6]; v[6] = v[5]; v[5] = v[4]; v[4] = v[3] + t1;
    v[3] = v[2]; v[2] = v[1]; v[1] = v[0]; v[0] = t1 + t2;
  }
  for (int i = 0; i < 8; ++i) h[i] += v[i];
}

static void sha512_full(const uint8_t *m, int len, bool is384, uint8_t out[64]) {
  uint64_t h[8];
  memcpy(h, is384 ? kSha384Iv : kSha512Iv, sizeof h);
  int off = 0;
  for (; len - off >= 128; off += 128) sha512_compress(h, m + off);
  uint8_t tail[256] = {0};
  const int rem = len - off;
  memcpy(tail, m + off, (size_t)rem);
  tail[rem] = 0x80;
  const int tl = (rem + 17 <= 128) ? 128 : 256;
  const uint64_t bits = (uint64_t)len * 8;          // the high 64 bits of the 128-bit length are 0
  for (int i = 0; i < 8; ++i) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
  sha512_compress(h, tail);
  if (tl == 256) sha512_compress(h, tail + 128);
  for (int i = 0; i < (is384 ? 6 : 8); ++i) {
    put_be32(out + 8 * i, (uint32_t)(h[i] >> 32));
    put_be32(out + 8 * i + 4, (uint32_t)h[i]);
  }
}

// hmac_init_pad (crypto.c:413-441) for HMAC-SHA2-384/512: the state after the
// key padded to 128 bytes (hashed first when longer), as 16 words: word 2k is
// the high half of state word k, 2k+1 the low half
void hmac_sha512_pad_state(const uint8_t *key, int klen, uint8_t padval, bool is384, uint32_t out[16]) {
  uint8_t k[128] = {0};
  if (klen > 128) sha512_full(key, klen, is384, k);
  else if (klen > 0) memcpy(k, key, (size_t)klen);
  for (int i = 0; i < 128; ++i) k[i] ^= padval;
  uint64_t h[8];
  memcpy(h, is384 ? kSha384Iv : kSha512Iv, sizeof h);
  sha512_compress(h, k);
  for (int i = 0; i < 8; ++i) {
    out[2 * i] = (uint32_t)(h[i] >> 32);
    out[2 * i + 1] = (uint32_t)h[i];
  }
}

}  // namespace hc
}  // namespace espgpu
