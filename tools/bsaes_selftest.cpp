// Host self-test of csrc/bsaes.h: T-table rounds up to round nr-KR, the
// bitsliced tail for the rest, against hc::aes_encrypt_block (FIPS-197),
// for AES-128/192/256 and KR = 1..4.  Built and run by tests/test_bsaes.py.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>

#include "bsaes.h"
#include "host_crypto.h"

using namespace espgpu;

static uint32_t ror8(uint32_t x) { return (x >> 8) | (x << 24); }

// State entering round `upto` (big-endian column words), T-table rounds.
static void rounds_to(const uint32_t *rk, const uint8_t in[16], int upto, uint32_t s[4]) {
  const hc::Tables &t = hc::tables();
  for (int c = 0; c < 4; ++c)
    s[c] = ((uint32_t)in[4 * c] << 24 | (uint32_t)in[4 * c + 1] << 16 | (uint32_t)in[4 * c + 2] << 8 |
            in[4 * c + 3]) ^ rk[c];
  for (int r = 1; r < upto; ++r) {
    uint32_t n[4];
    for (int c = 0; c < 4; ++c)
      n[c] = t.te0[s[c] >> 24] ^ ror8(t.te0[(s[(c + 1) & 3] >> 16) & 0xff]) ^
             ror8(ror8(t.te0[(s[(c + 2) & 3] >> 8) & 0xff])) ^
             ror8(ror8(ror8(t.te0[s[(c + 3) & 3] & 0xff]))) ^ rk[4 * r + c];
    memcpy(s, n, sizeof n);
  }
}

template <int KR>
static int check(int klen, unsigned seed) {
  srand(seed);
  uint8_t key[32], a[16], b[16], ea[16], eb[16];
  for (auto &x : key) x = rand() & 0xff;
  for (int i = 0; i < 16; ++i) { a[i] = rand() & 0xff; b[i] = rand() & 0xff; }
  uint32_t rk[60];
  const int nr = hc::aes_expand_enc(key, klen, rk);
  hc::aes_encrypt_block(rk, nr, a, ea);
  hc::aes_encrypt_block(rk, nr, b, eb);
  uint32_t sa[4], sb[4], oa[4], ob[4], keys[8 * 4];
  rounds_to(rk, a, nr - KR + 1, sa);
  rounds_to(rk, b, nr - KR + 1, sb);
  bs::round_keys(rk, nr, 4, keys);                   // one 4-round set serves every KR
  bs::tail_rounds<KR>(sa, sb, (const uint32_t *)keys + 8 * (4 - KR), oa, ob);
  for (int c = 0; c < 4; ++c)
    for (int r = 0; r < 4; ++r) {
      if (((oa[c] >> (24 - 8 * r)) & 0xff) != ea[4 * c + r] ||
          ((ob[c] >> (24 - 8 * r)) & 0xff) != eb[4 * c + r]) {
        printf("MISMATCH klen=%d KR=%d seed=%u col=%d row=%d\n", klen, KR, seed, c, r);
        return 1;
      }
    }
  return 0;
}

int main() {
  // the S-box circuit alone, all 256 inputs (each input byte in every lane slot)
  const hc::Tables &t = hc::tables();
  for (int v = 0; v < 256; ++v) {
    uint32_t q[8];
    for (int j = 0; j < 8; ++j) q[j] = ((v >> j) & 1) ? 0xffffffffu : 0u;
    bs::sbox(q);
    int o = 0;
    for (int j = 0; j < 8; ++j) o |= (q[j] & 1) << j;
    if (o != t.sbox[v]) { printf("SBOX MISMATCH %02x -> %02x (want %02x)\n", v, o, t.sbox[v]); return 1; }
  }
  int bad = 0;
  for (unsigned s = 0; s < 200; ++s)
    for (int klen : {16, 24, 32}) {
      bad |= check<1>(klen, s);
      bad |= check<2>(klen, s);
      bad |= check<3>(klen, s);
      bad |= check<4>(klen, s);
    }
  if (bad) return 1;
  printf("bsaes selftest OK\n");
  return 0;
}
