// host_crypto.h — session-setup arithmetic run on the host at newsession time
// (the work swcr_setup_gcm / swcr_setup_cipher / swcr_setup_auth do in
// freebsd/opencrypto/cryptosoft.c:976-1128): AES key schedules, H = E_K(0),
// GHASH power tables, HMAC-SHA1 ipad/opad chaining states.  Nothing here runs
// per packet; the per-packet work is all in the HIP kernels.
#pragma once
#include <stdint.h>

namespace espgpu {
namespace hc {

struct Tables {
  uint8_t sbox[256], isbox[256];
  uint32_t te0[256], td0[256];   // big-endian T-table words
};
const Tables &tables();

// FIPS-197 key expansion; returns Nr (10/12/14) or 0 on a bad length.
int aes_expand_enc(const uint8_t *key, int klen_bytes, uint32_t rk[60]);
// Equivalent-inverse-cipher schedule (rijndaelKeySetupDec layout).
int aes_expand_dec(const uint8_t *key, int klen_bytes, uint32_t dk[60]);
void aes_encrypt_block(const uint32_t *rk, int nr, const uint8_t in[16], uint8_t out[16]);

// GF(2^128) product in GCM bit order (SP 800-38D Algorithm 1).
void gf128_mul(const uint8_t x[16], const uint8_t y[16], uint8_t out[16]);

// GHASH table set for the GCM kernels (kGhTableBytes, espgpu_internal.h):
// H^1..H^8 with 4-bit indices (8 KiB each).
void ghash_tables(const uint8_t h[16], uint8_t *out);
// The 8-bit table (64 KiB, value-major) of the power whose 4-bit table is t4:
// what esp_gcm.hip stage_h8 builds in LDS (host mirror for the self-test).
void ghash_expand8(const uint8_t *t4, uint8_t *t8);

// SHA-1 compression of one 64-byte block into state h[5].
void sha1_compress(uint32_t h[5], const uint8_t block[64]);
// HMAC pad state: h = SHA1-compress(IV, (key or SHA1(key)) ^ padval).
void hmac_sha1_pad_state(const uint8_t *key, int klen, uint8_t padval, uint32_t h[5]);
void sha256_compress(uint32_t h[8], const uint8_t block[64]);
void hmac_sha256_pad_state(const uint8_t *key, int klen, uint8_t padval, uint32_t h[8]);
void sha512_compress(uint64_t h[8], const uint8_t block[128]);
void hmac_sha512_pad_state(const uint8_t *key, int klen, uint8_t padval, bool is384, uint32_t h[16]);

}  // namespace hc
}  // namespace espgpu
