// esp_cbc.hip — ESP AES-CBC + HMAC-SHA1-96 (CSP_MODE_ETA) kernels for gfx950.
//
// Replaces swcr_eta (freebsd/opencrypto/cryptosoft.c:874-888) =
//   decrypt: swcr_authcompute (verify, :317-382) then swcr_encdec (CBC, :101-284)
//   encrypt: swcr_encdec then swcr_authcompute (compute, ICV written)
// for the request esp_input / esp_output build (xform_esp.c:296-461):
//   AAD = ESP header + IV (hlen = 8 + 16 bytes), payload = CBC ciphertext,
//   HMAC-SHA1 over AAD || payload (|| ESN high 32 bits, CSP_F_ESN), ICV = the
//   first mlen (12) bytes, IV = the 16 bytes before the payload.
//
// Mapping: a wave owns 64 records (lane = record for everything serial).
//  * HMAC-SHA1 is a serial chain per record, so lane = record: each lane runs
//    its record's SHA-1 compressions from the precomputed ipad/opad chaining
//    states (hmac_init_pad, crypto.c:413-441), 80 rounds fully unrolled in
//    registers, no tables.
//  * Out-of-place decrypt (MODE 0, the benchmarked path) is ONE pass per
//    record (eta_decrypt_fused): every 64-byte HMAC chunk the lane loads also
//    completes up to four CBC blocks, which it decrypts with four AES states
//    in flight (aes_dec4) and stores, so the record is read once.
//  * In-place verify-first decrypt (MODE 2) must authenticate before it may
//    overwrite: HMAC pass first, then the CBC pass is block-parallel -- the
//    wave walks its records as one flat block list, 64 consecutive blocks per
//    pass (1 KiB contiguous per instruction), last pass first, so in-place
//    decryption never reads a block another lane already overwrote.
//  * AES decryption uses Td0/Td1 tables replicated 32x in LDS (conflict-free
//    ds_read_b32, one v_perm_b32 per address, as in esp_gcm.hip) and a
//    replicated inverse S-box for the last round.
//  * CBC encryption is serial per record (lane = record), Te0/Te1 in LDS.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "espgpu_internal.h"

namespace espgpu {

namespace {

constexpr uint32_t LDS_T = 0;          // Td0/Td1 (decrypt) or Te0/Te1 (encrypt), 64 KiB
constexpr uint32_t LDS_SI = 65536;     // inverse S-box as dwords, [256][32], 32 KiB
constexpr uint32_t LDS_BYTES = 65536 + 32768;

typedef const __attribute__((address_space(4))) uint32_t *kptr;

struct __attribute__((aligned(4))) U4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}
__device__ __forceinline__ uint32_t ror16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return perm(x, x, 0x00010203u); }
__device__ __forceinline__ uint4 ld16(const uint8_t *p) {
  U4 v = *reinterpret_cast<const U4 *>(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st16(uint8_t *p, uint4 v) {
  *reinterpret_cast<U4 *>(p) = U4{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) {
  return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}
__device__ __forceinline__ uint4 bswap4(uint4 v) {
  return make_uint4(bswap32(v.x), bswap32(v.y), bswap32(v.z), bswap32(v.w));
}

// T-table addressing, see esp_gcm.hip: entry x at x*256, T0 in lane slots
// (lane&31)*4, T1 128 bytes later.
__device__ __forceinline__ uint32_t tpa(uint32_t w, uint32_t slot, int k) {
  return perm(w, slot, 0x0c0c0000u | ((4u + (uint32_t)k) << 8));
}
__device__ __forceinline__ uint32_t t0(const uint8_t *lds, uint32_t a) {
  return *reinterpret_cast<const uint32_t *>(lds + a);
}
__device__ __forceinline__ uint32_t t1(const uint8_t *lds, uint32_t a) {
  return *reinterpret_cast<const uint32_t *>(lds + a + 128);
}

// ---- AES decryption (rijndaelDecrypt, rijndael-alg-fst.c:1044-1222) --------
// dk = rijndaelKeySetupDec schedule (big-endian words).  Input/output are
// little-endian memory words.
template <typename KP>
__device__ __forceinline__ uint4 aes_dec(uint4 in, KP dk, int nr, const uint8_t *lds, uint32_t slot) {
  uint32_t s0 = bswap32(in.x) ^ dk[0], s1 = bswap32(in.y) ^ dk[1];
  uint32_t s2 = bswap32(in.z) ^ dk[2], s3 = bswap32(in.w) ^ dk[3];
#pragma unroll 1
  for (int r = 1; r < nr; ++r) {
    const uint32_t k0 = ror16(dk[4 * r]), k1 = ror16(dk[4 * r + 1]);
    const uint32_t k2 = ror16(dk[4 * r + 2]), k3 = ror16(dk[4 * r + 3]);
    // t_c = Td0[s_c.b3] ^ Td1[s_c-1.b2] ^ ror16(Td0[s_c+2.b1] ^ Td1[s_c+1.b0] ^ ror16(rk))
    const uint32_t a0 = t0(lds, tpa(s0, slot, 3)), b0 = t1(lds, tpa(s3, slot, 2));
    const uint32_t c0 = t0(lds, tpa(s2, slot, 1)), d0 = t1(lds, tpa(s1, slot, 0));
    const uint32_t a1 = t0(lds, tpa(s1, slot, 3)), b1 = t1(lds, tpa(s0, slot, 2));
    const uint32_t c1 = t0(lds, tpa(s3, slot, 1)), d1 = t1(lds, tpa(s2, slot, 0));
    const uint32_t a2 = t0(lds, tpa(s2, slot, 3)), b2 = t1(lds, tpa(s1, slot, 2));
    const uint32_t c2 = t0(lds, tpa(s0, slot, 1)), d2 = t1(lds, tpa(s3, slot, 0));
    const uint32_t a3 = t0(lds, tpa(s3, slot, 3)), b3 = t1(lds, tpa(s2, slot, 2));
    const uint32_t c3 = t0(lds, tpa(s1, slot, 1)), d3 = t1(lds, tpa(s0, slot, 0));
    s0 = xor3(a0, b0, ror16(xor3(c0, d0, k0)));
    s1 = xor3(a1, b1, ror16(xor3(c1, d1, k1)));
    s2 = xor3(a2, b2, ror16(xor3(c2, d2, k2)));
    s3 = xor3(a3, b3, ror16(xor3(c3, d3, k3)));
    __builtin_amdgcn_sched_barrier(0);
  }
  // last round: Si bytes from the replicated inverse S-box (dword per entry)
  const uint32_t *si = reinterpret_cast<const uint32_t *>(lds + LDS_SI);
  const uint32_t ls = slot >> 2;
  uint32_t ss[4] = {s0, s1, s2, s3}, o[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const uint32_t a = si[((ss[c] >> 24) << 5) | ls];
    const uint32_t b = si[(((ss[(c + 3) & 3] >> 16) & 0xff) << 5) | ls];
    const uint32_t cc = si[(((ss[(c + 2) & 3] >> 8) & 0xff) << 5) | ls];
    const uint32_t d = si[((ss[(c + 1) & 3] & 0xff) << 5) | ls];
    o[c] = (a | (b << 8) | (cc << 16) | (d << 24)) ^ bswap32(dk[4 * nr + c]);
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// Four independent blocks through the same rounds: 64 table reads in flight
// per lane per round instead of 16 (the decrypt of one 64-byte HMAC chunk).
template <typename KP>
__device__ __forceinline__ void aes_dec4(uint4 (&v)[4], KP dk, int nr, const uint8_t *lds, uint32_t slot) {
  uint32_t s[4][4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    s[q][0] = bswap32(v[q].x) ^ dk[0];
    s[q][1] = bswap32(v[q].y) ^ dk[1];
    s[q][2] = bswap32(v[q].z) ^ dk[2];
    s[q][3] = bswap32(v[q].w) ^ dk[3];
  }
#pragma unroll 1
  for (int r = 1; r < nr; ++r) {
    const uint32_t k0 = ror16(dk[4 * r]), k1 = ror16(dk[4 * r + 1]);
    const uint32_t k2 = ror16(dk[4 * r + 2]), k3 = ror16(dk[4 * r + 3]);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t s0 = s[q][0], s1 = s[q][1], s2 = s[q][2], s3 = s[q][3];
      const uint32_t a0 = t0(lds, tpa(s0, slot, 3)), b0 = t1(lds, tpa(s3, slot, 2));
      const uint32_t c0 = t0(lds, tpa(s2, slot, 1)), d0 = t1(lds, tpa(s1, slot, 0));
      const uint32_t a1 = t0(lds, tpa(s1, slot, 3)), b1 = t1(lds, tpa(s0, slot, 2));
      const uint32_t c1 = t0(lds, tpa(s3, slot, 1)), d1 = t1(lds, tpa(s2, slot, 0));
      const uint32_t a2 = t0(lds, tpa(s2, slot, 3)), b2 = t1(lds, tpa(s1, slot, 2));
      const uint32_t c2 = t0(lds, tpa(s0, slot, 1)), d2 = t1(lds, tpa(s3, slot, 0));
      const uint32_t a3 = t0(lds, tpa(s3, slot, 3)), b3 = t1(lds, tpa(s2, slot, 2));
      const uint32_t c3 = t0(lds, tpa(s1, slot, 1)), d3 = t1(lds, tpa(s0, slot, 0));
      s[q][0] = xor3(a0, b0, ror16(xor3(c0, d0, k0)));
      s[q][1] = xor3(a1, b1, ror16(xor3(c1, d1, k1)));
      s[q][2] = xor3(a2, b2, ror16(xor3(c2, d2, k2)));
      s[q][3] = xor3(a3, b3, ror16(xor3(c3, d3, k3)));
    }
  }
  const uint32_t *si = reinterpret_cast<const uint32_t *>(lds + LDS_SI);
  const uint32_t ls = slot >> 2;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t o[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t a = si[((s[q][c] >> 24) << 5) | ls];
      const uint32_t b = si[(((s[q][(c + 3) & 3] >> 16) & 0xff) << 5) | ls];
      const uint32_t cc = si[(((s[q][(c + 2) & 3] >> 8) & 0xff) << 5) | ls];
      const uint32_t d = si[((s[q][(c + 1) & 3] & 0xff) << 5) | ls];
      o[c] = (a | (b << 8) | (cc << 16) | (d << 24)) ^ bswap32(dk[4 * nr + c]);
    }
    v[q] = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// ---- AES encryption (rijndaelEncrypt) with Te0/Te1 in LDS ------------------
template <typename KP>
__device__ __forceinline__ uint4 aes_enc(uint4 in, KP ek, int nr, const uint8_t *lds, uint32_t slot) {
  uint32_t s0 = bswap32(in.x) ^ ek[0], s1 = bswap32(in.y) ^ ek[1];
  uint32_t s2 = bswap32(in.z) ^ ek[2], s3 = bswap32(in.w) ^ ek[3];
#pragma unroll 1
  for (int r = 1; r < nr; ++r) {
    const uint32_t k0 = ror16(ek[4 * r]), k1 = ror16(ek[4 * r + 1]);
    const uint32_t k2 = ror16(ek[4 * r + 2]), k3 = ror16(ek[4 * r + 3]);
    const uint32_t a0 = t0(lds, tpa(s0, slot, 3)), b0 = t1(lds, tpa(s1, slot, 2));
    const uint32_t c0 = t0(lds, tpa(s2, slot, 1)), d0 = t1(lds, tpa(s3, slot, 0));
    const uint32_t a1 = t0(lds, tpa(s1, slot, 3)), b1 = t1(lds, tpa(s2, slot, 2));
    const uint32_t c1 = t0(lds, tpa(s3, slot, 1)), d1 = t1(lds, tpa(s0, slot, 0));
    const uint32_t a2 = t0(lds, tpa(s2, slot, 3)), b2 = t1(lds, tpa(s3, slot, 2));
    const uint32_t c2 = t0(lds, tpa(s0, slot, 1)), d2 = t1(lds, tpa(s1, slot, 0));
    const uint32_t a3 = t0(lds, tpa(s3, slot, 3)), b3 = t1(lds, tpa(s0, slot, 2));
    const uint32_t c3 = t0(lds, tpa(s1, slot, 1)), d3 = t1(lds, tpa(s2, slot, 0));
    s0 = xor3(a0, b0, ror16(xor3(c0, d0, k0)));
    s1 = xor3(a1, b1, ror16(xor3(c1, d1, k1)));
    s2 = xor3(a2, b2, ror16(xor3(c2, d2, k2)));
    s3 = xor3(a3, b3, ror16(xor3(c3, d3, k3)));
    __builtin_amdgcn_sched_barrier(0);
  }
  uint32_t ss[4] = {s0, s1, s2, s3}, o[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const uint32_t a = t0(lds, tpa(ss[c], slot, 3));
    const uint32_t b = t0(lds, tpa(ss[(c + 1) & 3], slot, 2));
    const uint32_t cc = t0(lds, tpa(ss[(c + 2) & 3], slot, 1));
    const uint32_t d = t0(lds, tpa(ss[(c + 3) & 3], slot, 0));
    o[c] = xor3(perm(b, a, 0x0c0c0501u), perm(d, cc, 0x05010c0cu), bswap32(ek[4 * nr + c]));
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// ---- SHA-1 compression (sha1_step, freebsd/crypto/sha1.c:94-176) ----------
__device__ __forceinline__ void sha1_compress(uint32_t h[5], uint32_t w[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#pragma unroll
  for (int t = 0; t < 80; ++t) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      wt = rotl(xor3(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^ w[t & 15], 1);
      w[t & 15] = wt;
    }
    uint32_t f, k;
    if (t < 20) {
      f = __builtin_amdgcn_bitop3_b32(b, c, d, 0xCA);   // (b & c) | (~b & d)
      k = 0x5a827999u;
    } else if (t < 40) {
      f = xor3(b, c, d);
      k = 0x6ed9eba1u;
    } else if (t < 60) {
      f = __builtin_amdgcn_bitop3_b32(b, c, d, 0xE8);   // majority
      k = 0x8f1bbcdcu;
    } else {
      f = xor3(b, c, d);
      k = 0xca62c1d6u;
    }
    const uint32_t tmp = rotl(a, 5) + f + e + k + wt;
    e = d;
    d = c;
    c = rotl(b, 30);
    b = a;
    a = tmp;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

// HMAC-SHA1 of msg = rec[0, L0) || (esn ? be32(esn_hi) : "") from the SA's
// ipad/opad chaining states (already past the 64-byte key block).
__device__ void hmac_sha1(const uint8_t *rec, uint32_t L0, bool esn, uint32_t esn_hi,
                          kptr ipad, kptr opad, uint32_t out[5]) {
  const uint32_t L = L0 + (esn ? 4u : 0u);              // multiple of 4 for ESP records
  const uint32_t nfull = L0 / 64;                       // blocks entirely from memory
  const uint32_t total = (L + 9 + 63) / 64;             // inner blocks incl. padding
  const uint64_t bits = (uint64_t)(64 + L) * 8;         // the ipad block counts
  uint32_t h[5] = {ipad[0], ipad[1], ipad[2], ipad[3], ipad[4]};
  uint32_t w[16];
  // One compression site for every block (inner data, inner padding, outer)
  // keeps a single inlined copy of the 80 rounds.
  for (uint32_t b = 0; b <= total; ++b) {
    if (b < nfull) {
      const uint8_t *p = rec + 64 * b;
      const uint4 q0 = bswap4(ld16(p)), q1 = bswap4(ld16(p + 16)), q2 = bswap4(ld16(p + 32)),
                  q3 = bswap4(ld16(p + 48));
      w[0] = q0.x; w[1] = q0.y; w[2] = q0.z; w[3] = q0.w;
      w[4] = q1.x; w[5] = q1.y; w[6] = q1.z; w[7] = q1.w;
      w[8] = q2.x; w[9] = q2.y; w[10] = q2.z; w[11] = q2.w;
      w[12] = q3.x; w[13] = q3.y; w[14] = q3.z; w[15] = q3.w;
    } else if (b < total) {
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const uint32_t o = 64 * b + 4 * k;
        uint32_t v;
        if (o + 4 <= L0) v = bswap32(*reinterpret_cast<const uint32_t *>(rec + o));
        else if (esn && o == L0) v = esn_hi;
        else if (o == L) v = 0x80000000u;
        else v = 0;
        if (b == total - 1 && k == 14) v = (uint32_t)(bits >> 32);
        if (b == total - 1 && k == 15) v = (uint32_t)bits;
        w[k] = v;
      }
    } else {
      // outer: opad state, block = inner digest || 0x80 || 0... || (64+20)*8
#pragma unroll
      for (int k = 0; k < 5; ++k) w[k] = h[k];
      w[5] = 0x80000000u;
#pragma unroll
      for (int k = 6; k < 15; ++k) w[k] = 0;
      w[15] = (64 + 20) * 8;
#pragma unroll
      for (int k = 0; k < 5; ++k) h[k] = opad[k];
    }
    sha1_compress(h, w);
  }
  for (int k = 0; k < 5; ++k) out[k] = h[k];
}

__device__ __forceinline__ kptr kp(const void *p) { return (kptr)p; }

// One pass over an ETA record for the out-of-place decrypt: the record is
// read once, in 64-byte HMAC chunks (lane = record); each chunk feeds the
// SHA-1 compression AND the CBC decryption of the CT blocks it completes, so
// the ciphertext is not fetched a second time for the cipher.  ESP places CT
// block i at 24 + 16i: chunk 0 holds the IV (C_-1) and blocks 0, 1; chunk
// b >= 1 holds the 8-byte tail of block 4b-2 and blocks 4b-1 .. 4b+1, whose
// other 8 bytes came at the end of chunk b-1 (carried in two registers).
// The <= 4 blocks after the last full chunk are decrypted on the way through
// the first partial chunk.  Writes plaintext to out (MODE 0 decrypts records
// whose ICV fails too; the status byte says so, as in the GCM kernel).
// Returns whether the first mlen bytes of the HMAC match the ICV; *trl gets
// the esp_input_cb trailer word from the last block.
__device__ bool eta_decrypt_fused(const uint8_t *rec, uint8_t *orec, uint32_t plen, uint32_t mlen, bool esn,
                                  uint32_t esn_hi, kptr ipad, kptr opad, kptr dk, int nr, const uint8_t *lds,
                                  uint32_t slot, bool act, uint32_t *trl) {
  const uint32_t L0 = 24 + plen, L = L0 + (esn ? 4u : 0u);
  const uint32_t nfull = L0 / 64, total = (L + 9 + 63) / 64, nblk = plen / 16;
  const uint64_t bits = (uint64_t)(64 + L) * 8;
  uint32_t T = act ? total : 0;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) T = max(T, (uint32_t)__shfl_xor((int)T, o));
  uint32_t h[5] = {ipad[0], ipad[1], ipad[2], ipad[3], ipad[4]};
  uint4 prev = make_uint4(0, 0, 0, 0);
  uint32_t cy0 = 0, cy1 = 0;
  for (uint32_t b = 0; b <= T; ++b) {
    const bool on = act && b <= total;
    uint32_t w[16];
    uint32_t m[16];
    if (on && b < nfull) {
      const uint8_t *q = rec + 64 * b;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint4 v = ld16(q + 16 * k);
        m[4 * k] = v.x; m[4 * k + 1] = v.y; m[4 * k + 2] = v.z; m[4 * k + 3] = v.w;
      }
      uint4 blk[4];
      int i0, nb;
      if (b == 0) {                       // wave-uniform: every lane is at chunk 0 together
        prev = make_uint4(m[2], m[3], m[4], m[5]);
        blk[0] = make_uint4(m[6], m[7], m[8], m[9]);
        blk[1] = make_uint4(m[10], m[11], m[12], m[13]);
        blk[2] = blk[3] = make_uint4(0, 0, 0, 0);
        i0 = 0;
        nb = 2;
      } else {
        blk[0] = make_uint4(cy0, cy1, m[0], m[1]);
        blk[1] = make_uint4(m[2], m[3], m[4], m[5]);
        blk[2] = make_uint4(m[6], m[7], m[8], m[9]);
        blk[3] = make_uint4(m[10], m[11], m[12], m[13]);
        i0 = 4 * (int)b - 2;
        nb = 4;
      }
      cy0 = m[14];
      cy1 = m[15];
      uint4 d[4] = {blk[0], blk[1], blk[2], blk[3]};
      aes_dec4(d, dk, nr, lds, slot);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (k < nb) {
          st16(orec + 24 + 16 * (i0 + k), xor4(d[k], prev));
          prev = blk[k];
        }
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = bswap32(m[k]);
    } else if (on && b < total) {
      if (b == nfull) {
        // the CT blocks after the last full chunk (1..4 of them)
        const int i0 = nfull == 0 ? 0 : 4 * (int)nfull - 2;
        if (nfull == 0) prev = ld16(rec + 8);
        uint4 blk[4], d[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          blk[k] = make_uint4(0, 0, 0, 0);
          if (i0 + k < (int)nblk) blk[k] = ld16(rec + 24 + 16 * (i0 + k));
          d[k] = blk[k];
        }
        aes_dec4(d, dk, nr, lds, slot);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (i0 + k < (int)nblk) {
            const uint4 pt = xor4(d[k], prev);
            st16(orec + 24 + 16 * (i0 + k), pt);
            if (i0 + k == (int)nblk - 1) *trl = esp_trailer_word(pt.w, plen);
            prev = blk[k];
          }
        }
      }
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const uint32_t o = 64 * b + 4 * k;
        uint32_t v;
        if (o + 4 <= L0) v = bswap32(*reinterpret_cast<const uint32_t *>(rec + o));
        else if (esn && o == L0) v = esn_hi;
        else if (o == L) v = 0x80000000u;
        else v = 0;
        if (b == total - 1 && k == 14) v = (uint32_t)(bits >> 32);
        if (b == total - 1 && k == 15) v = (uint32_t)bits;
        w[k] = v;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 5; ++k) w[k] = h[k];
      w[5] = 0x80000000u;
#pragma unroll
      for (int k = 6; k < 15; ++k) w[k] = 0;
      w[15] = (64 + 20) * 8;
      if (on) {
#pragma unroll
        for (int k = 0; k < 5; ++k) h[k] = opad[k];
      }
    }
    uint32_t hn[5] = {h[0], h[1], h[2], h[3], h[4]};
    sha1_compress(hn, w);
    if (on) {
#pragma unroll
      for (int k = 0; k < 5; ++k) h[k] = hn[k];
    }
  }
  uint32_t diff = 0;
  if (act)
    for (uint32_t k = 0; k < mlen / 4; ++k)
      diff |= bswap32(h[k]) ^ *reinterpret_cast<const uint32_t *>(rec + L0 + 4 * k);
  return act && diff == 0;
}

// MODE 0: decrypt out-of-place; 1: encrypt in place; 2: decrypt in place (verify first)
template <int MODE, int WG>
__global__ __launch_bounds__(WG) void eta_kernel(EtaParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t slot = (uint32_t)(lane & 31) * 4;
  const uint2 *tab = MODE == 1 ? p.tpair : p.dpair;
  for (int idx = tid; idx < 256 * 32; idx += WG) {
    const int x = idx >> 5, r = idx & 31;
    const uint2 t = tab[x];
    *reinterpret_cast<uint32_t *>(lds + LDS_T + x * 256 + r * 4) = t.x;
    *reinterpret_cast<uint32_t *>(lds + LDS_T + x * 256 + 128 + r * 4) = t.y;
    if (MODE != 1) *reinterpret_cast<uint32_t *>(lds + LDS_SI + idx * 4) = p.isbox[x];
  }
  __syncthreads();

  // Work units are one wave's worth of records: a 64-record ETA chunk of one
  // session from the planner, or (implicit) 64 consecutive descriptors.
  // Waves draw units from a queue; the last wave to retire resets it.
  const bool implicit = p.chunks == nullptr;
  const uint32_t u0 = implicit ? 0u : p.nchunks[0];
  const uint32_t u1 = implicit ? (p.n + 63) / 64 : p.nchunks[1];
  for (;;) {
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(&p.queue[0], 1u);
    const uint32_t u = u0 + __builtin_amdgcn_readfirstlane(t);
    if (u >= u1) break;
    uint32_t di = 0;
    bool have;
    if (implicit) {
      di = u * 64 + lane;
      have = di < p.n;
    } else {
      const Chunk ch = p.chunks[u];
      have = (uint32_t)lane < ch.count;
      if (have) di = p.order[ch.start + lane];
    }
    // ---- lane = record: descriptor, HMAC (verify or compute) ----
    bool valid = false, ok = false;
    uint32_t off = 0, len = 0, sa = 0, plen = 0;
    if (have) {
      const uint4 dv = *reinterpret_cast<const uint4 *>(p.desc + di);
      off = dv.x * 4;
      len = dv.y & 0xffffu;
      sa = dv.y >> 16;
      const DevSA *s = sa < p.nsas ? p.sas + sa : nullptr;
      if (!s || s->mode != ESPGPU_CSP_MODE_ETA) {
        have = false;                                       // not ours (GCM kernel / EINVAL)
        if (!s || s->mode == 0) {
          p.status[di] = ESPGPU_EINVAL;
          if (MODE != 1 && p.trailer) p.trailer[di] = 0;
        }
      } else {
        const uint32_t mlen = s->mlen;
        const int pl = (int)len - 24 - (int)mlen;           // hlen 24, alen = mlen (12)
        valid = pl > 0 && (pl & 15) == 0 && (len & 3) == 0;  // xform_esp.c:316-324
        plen = valid ? (uint32_t)pl : 0;
        if (valid && MODE == 2) {
          uint32_t dg[5];
          const uint8_t *rec = p.arena + off;
          hmac_sha1(rec, 24 + plen, (s->flags & ESPGPU_CSP_F_ESN) != 0, dv.z, kp(s->ipad),
                    kp(s->opad), dg);
          uint32_t diff = 0;
          for (uint32_t k = 0; k < mlen / 4; ++k)
            diff |= bswap32(dg[k]) ^ *reinterpret_cast<const uint32_t *>(rec + 24 + plen + 4 * k);
          ok = diff == 0;
        }
      }
    }
    if (MODE == 1) {
      // ---- encrypt: CBC chain is serial, lane = record ----
      if (have && valid) {
        const DevSA *s = p.sas + sa;
        uint8_t *rec = p.arena + off;
        uint4 prev = ld16(rec + 8);                         // IV
        const int nr = (int)s->nr;
        for (uint32_t b = 0; b < plen / 16; ++b) {
          const uint4 c = aes_enc(xor4(ld16(rec + 24 + 16 * b), prev), s->rk, nr, lds, slot);
          st16(rec + 24 + 16 * b, c);
          prev = c;
        }
        uint32_t dg[5];
        hmac_sha1(rec, 24 + plen, (s->flags & ESPGPU_CSP_F_ESN) != 0, p.desc[di].esn_hi,
                  kp(s->ipad), kp(s->opad), dg);
        for (uint32_t k = 0; k < s->mlen / 4; ++k)
          *reinterpret_cast<uint32_t *>(rec + 24 + plen + 4 * k) = bswap32(dg[k]);
      }
      if (have) p.status[di] = valid ? ESPGPU_OK : ESPGPU_EINVAL;
      continue;
    }
    if (MODE == 0) {
      // ---- out-of-place decrypt: one fused pass per record (lane = record),
      // one session at a time so round keys and pads stay in SGPRs ----
      bool run = have && valid;
      uint64_t todo = __ballot(run);
      while (todo) {
        const uint32_t sau = __builtin_amdgcn_readfirstlane(__shfl(sa, __builtin_ctzll(todo)));
        const bool mine = run && sa == sau;
        todo &= ~__ballot(mine);
        run = run && !mine;
        const DevSA *s = p.sas + sau;
        uint32_t trl = 0;
        const bool good = eta_decrypt_fused(p.arena + off, p.out + off, plen, s->mlen,
                                            (s->flags & ESPGPU_CSP_F_ESN) != 0, mine ? p.desc[di].esn_hi : 0,
                                            kp(s->ipad), kp(s->opad), kp(s->dk), (int)s->nr, lds, slot, mine,
                                            &trl);
        if (mine) {
          ok = good;
          if (p.trailer) p.trailer[di] = good ? trl : 0u;
        }
      }
      if (have) p.status[di] = !valid ? ESPGPU_EINVAL : (ok ? ESPGPU_OK : ESPGPU_EBADMSG);
      if (have && p.trailer && !valid) p.trailer[di] = 0;
      continue;
    }
    if (have) p.status[di] = !valid ? ESPGPU_EINVAL : (ok ? ESPGPU_OK : ESPGPU_EBADMSG);
    // trailer word: 0 now for records that will not be decrypted; the lane
    // decrypting a record's last block writes the others'
    if (have && p.trailer && !(valid && ok)) p.trailer[di] = 0;

    // ---- decrypt: all of the wave's blocks of one session as one flat list ----
    // Records to decrypt (one session at a time, so the round keys stay
    // wave-uniform in SGPRs: one pass for planner chunks) are concatenated;
    // every lane takes one block per pass, last pass first.  Within a pass all
    // lanes load C_i and C_{i-1} before any lane stores, and a pass only
    // overwrites blocks no later (lower) pass reads: in-place decryption is
    // safe without holding records in registers.
    bool run = have && valid && (MODE == 0 || ok);
    uint64_t todo = __ballot(run);
    while (todo) {
      const uint32_t sau = __builtin_amdgcn_readfirstlane(__shfl(sa, __builtin_ctzll(todo)));
      const bool mine = run && sa == sau;
      todo &= ~__ballot(mine);
      run = run && !mine;
      const uint32_t nb = mine ? plen / 16 : 0;
      uint32_t incl = nb;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
      }
      const uint32_t start = incl - nb;
      const int total = (int)__builtin_amdgcn_readfirstlane(__shfl(incl, 63));
      const DevSA *s = p.sas + sau;
      const int nr = (int)s->nr;
      const kptr dk = kp(s->dk);
      uint8_t *const obase = MODE == 0 ? p.out : p.arena;
      for (int base = total - 64; base > -64; base -= 64) {
        const int f = base + lane;
        // the record holding flat block f: the last lane whose start <= f
        int j = 0;
        uint32_t sj = 0;
#pragma unroll
        for (int step = 32; step >= 1; step >>= 1) {
          const uint32_t sc = __shfl(start, j + step);
          if ((int)sc <= f) {
            j += step;
            sj = sc;
          }
        }
        const uint32_t ro = __shfl(off, j);
        const uint32_t rpl = __shfl(plen, j), rdi = __shfl(di, j);
        const int rok = __shfl((int)ok, j);        // MODE 0 also decrypts failed records
        if (f >= 0) {
          const uint32_t i = (uint32_t)f - sj;
          const uint8_t *rec = p.arena + ro;
          const uint4 c = ld16(rec + 24 + 16 * i);
          const uint4 prev = ld16(rec + 8 + 16 * i);         // C_{i-1}, or the IV for i = 0
          const uint4 pt = xor4(aes_dec(c, dk, nr, lds, slot), prev);
          st16(obase + ro + 24 + 16 * i, pt);
          if (p.trailer && i == rpl / 16 - 1 && rok) p.trailer[rdi] = esp_trailer_word(pt.w, rpl);
        }
      }
    }
  }
  // Every wave leaves the loop after drawing one ticket past the end, so once
  // all have retired no ticket is drawn again: reset for the next launch.
  if (lane == 0 && atomicAdd(&p.queue[1], 1u) == gridDim.x * (WG / 64) - 1) {
    atomicExch(&p.queue[0], 0u);
    atomicExch(&p.queue[1], 0u);
  }
}

}  // namespace

// Decrypt runs 768-thread workgroups: 3 waves/SIMD at up to 170 VGPRs (the
// unrolled SHA-1 schedule needs ~150 and spills at 128), one workgroup per CU
// (96 KiB LDS); encrypt runs 1024.
int launch_eta(const EtaParams &p, int encrypt, int grid, void *stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (grid <= 0) grid = 256;
  // implicit units (64 records, one wave each): no more workgroups than units
  if (p.chunks == nullptr) {
    const int units = (int)((p.n + 63) / 64), wpg = (encrypt ? 1024 : 768) / 64;
    grid = std::max(1, std::min(grid, (units + wpg - 1) / wpg));
  }
  const int two_pass = !encrypt && p.out == p.arena;
  if (encrypt)
    hipLaunchKernelGGL((eta_kernel<1, 1024>), dim3(grid), dim3(1024), 0, st, p);
  else if (two_pass)
    hipLaunchKernelGGL((eta_kernel<2, 768>), dim3(grid), dim3(768), 0, st, p);
  else
    hipLaunchKernelGGL((eta_kernel<0, 768>), dim3(grid), dim3(768), 0, st, p);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace espgpu
