// esp_cbc.hip — ESP encrypt-then-MAC (CSP_MODE_ETA) kernels for gfx950:
// AES-CBC or AES-CTR (RFC 3686) with HMAC-SHA1 or HMAC-SHA2-256.
//
// Replaces swcr_eta (freebsd/opencrypto/cryptosoft.c:874-888) =
//   decrypt: swcr_authcompute (verify, :317-382) then swcr_encdec (:101-284)
//   encrypt: swcr_encdec then swcr_authcompute (compute, ICV written)
// for the request esp_input / esp_output build (xform_esp.c:296-461):
//   CBC: record = SPI|SN|IV16|CT|ICV, hlen 24, IV = the 16 bytes before the CT,
//        CT a multiple of 16 (rijndael blocksize);
//   CTR: record = SPI|SN|IV8|CT|ICV, hlen 16, counter block of CT block i =
//        nonce(4) || IV8 || be32(i+1) (xform_esp.c:453-458, RFC 3686; the nonce
//        is the SA key's last 4 bytes, carried in the descriptor's salt), any
//        4-byte-multiple CT (blocksize 1, esp_output pads to 4);
//   HMAC over SPI|SN|IV|CT (|| ESN high word, CSP_F_ESN); ICV = its first mlen
//   bytes (12 for SHA1-96, 16 for SHA2-256-128: xform_ah_authsize).
//
// Mapping: a wave owns 64 records (lane = record for everything serial).
//  * HMAC is a serial chain per record, so lane = record: each lane runs its
//    record's SHA-1 / SHA-256 compressions from the precomputed ipad/opad
//    chaining states (hmac_init_pad, crypto.c:413-441), rounds fully
//    unrolled in registers, no tables.  The in-place verify and the MAC pass
//    move the bytes through the quad (hmac_quad: lane 4Q+k loads piece k of
//    the quad's four records, a DPP transpose hands each lane its own), two
//    64-byte blocks per load.
//  * Decrypt is verify-first: an HMAC pass (lane = record), then a
//    block-parallel decrypt of the verified records (MODE 3 out of place;
//    MODE 2 in place, the opencrypto contract).
//  * In-place verify-first decrypt (MODE 2) must authenticate before it may
//    overwrite: HMAC pass first, then a block-parallel pass -- the wave walks
//    its records as one flat block list, 64 consecutive blocks per pass
//    (1 KiB contiguous per instruction), last pass first, so in-place CBC
//    decryption never reads a block another lane already overwrote.
//  * AES uses T-table pairs replicated 32x in LDS (conflict-free ds_read_b32,
//    one v_perm_b32 per address, as in esp_gcm.hip): Td0/Td1 + a replicated
//    inverse S-box for CBC decryption, Te0/Te1 for CBC encryption and CTR.
//  * CBC encryption is serial per record (lane = record; its 64-byte groups
//    moved through the quad as the hash blocks, cbc_enc_quad); CTR encryption
//    runs the same lane = record loop with independent blocks.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "espgpu_internal.h"
#include "sha512_consts.h"

namespace espgpu {

namespace {

// LDS: decrypt modes hold Td pair, inverse S-box and Te pair (CBC and CTR
// sessions can share a launch); encrypt holds the Te pair only.
constexpr uint32_t LDS_T = 0;          // Td0/Td1 (decrypt) or Te0/Te1 (encrypt), 64 KiB
constexpr uint32_t LDS_SI = 65536;     // inverse S-box as dwords, [256][32], 32 KiB
constexpr uint32_t LDS_TE = 98304;     // Te0/Te1 in the decrypt modes (CTR keystream), 64 KiB
constexpr uint32_t lds_bytes(int mode) { return mode == 1 || mode == 4 ? 65536u : 163840u; }

// cipher kinds (MODE 4): the CTR keystream, or the CBC chain with the
// encrypt-then-MAC HMAC-SHA1 / SHA2-256 ICV in the same pass
constexpr int CK_CTR = 1, CK_CBCMAC = 2;
// MODE 1 / 2 / 3 session sets (the CKS template argument), split by hash so
// that the common kernel carries no SHA-512 code (its registers then fit
// without spilling): HMAC-SHA1 / SHA2-256 / none, or HMAC-SHA2-384 / 512 only
constexpr int CK_NARROW = -2, CK_WIDEH = -3;
constexpr int kEtaU = 4;               // blocks per lane per pass of the block-parallel decrypt
constexpr int HS_SHA1 = 0, HS_SHA256 = 1;

typedef const __attribute__((address_space(4))) uint32_t *kptr;

// Measurement knobs for the decrypt kernels, compiled in only by `make knobs`
// (bench.py --tuning eta_opts=N with ESPGPU_LIB pointing at
// libespgpu_knobs.so): 0x10000 skips the verify pass (every record decrypts),
// 0x20000 the HMAC compressions (the loads stay), 0x40000 the decrypt pass's
// AES, 0x80000 its loads and stores; in the fused CBC + HMAC encrypt pass
// 0x100000 skips the stores, 0x200000 the loads, 0x400000 the compressions,
// 0x800000 the AES.  They break results on purpose, to split the kernel's time.
#ifdef ESPGPU_KNOBS
__device__ uint32_t e_opts;
__device__ __forceinline__ uint32_t eopts() {
  return *(const __attribute__((address_space(4))) uint32_t *)(const void *)&e_opts;
}
#else
__device__ __forceinline__ constexpr uint32_t eopts() { return 0; }
#endif

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}
__device__ __forceinline__ uint32_t ror16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return perm(x, x, 0x00010203u); }
// single 16- / 8-byte vector accesses at 4-byte alignment (see esp_gcm.hip)
typedef uint32_t V4a __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t V2a __attribute__((ext_vector_type(2), aligned(4)));
__device__ __forceinline__ uint4 ld16(const uint8_t *p) {
  const V4a v = *reinterpret_cast<const V4a *>(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st16(uint8_t *p, uint4 v) {
  V4a u = {v.x, v.y, v.z, v.w};
  *reinterpret_cast<V4a *>(p) = u;
}
// first `rem` bytes (4, 8, 12 or >= 16) of v; no store shared with the full
// path, so full blocks stay single 16-byte stores
__device__ __forceinline__ void st_partial(uint8_t *p, uint4 v, int rem) {
  if (rem >= 16) {
    st16(p, v);
    return;
  }
  if (rem > 4) {
    V2a u = {v.x, v.y};
    *reinterpret_cast<V2a *>(p) = u;
  } else {
    *reinterpret_cast<uint32_t *>(p) = v.x;
  }
  if (rem > 8) *reinterpret_cast<uint32_t *>(p + 8) = v.z;
}
__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) {
  return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}
__device__ __forceinline__ uint4 bswap4(uint4 v) {
  return make_uint4(bswap32(v.x), bswap32(v.y), bswap32(v.z), bswap32(v.w));
}
// the dword of a block holding the last 3 plaintext bytes, rem = bytes of the
// block that are payload (4, 8, 12 or 16)
__device__ __forceinline__ uint32_t last_word(uint4 v, int rem) {
  return rem >= 16 ? v.w : (rem > 8 ? v.z : (rem > 4 ? v.y : v.x));
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
template <int N, typename KP>
__device__ __forceinline__ void aes_dec4(uint4 (&v)[N], KP dk, int nr, const uint8_t *lds, uint32_t slot) {
  uint32_t s[N][4];
#pragma unroll
  for (int q = 0; q < N; ++q) {
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
    for (int q = 0; q < N; ++q) {
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
  for (int q = 0; q < N; ++q) {
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

// Four independent blocks through the encryption rounds (CTR keystream of
// one 64-byte chunk): Te0/Te1 at `lds`, round keys `ek` (enc schedule).
template <int N, typename KP>
__device__ __forceinline__ void aes_enc4(uint4 (&v)[N], KP ek, int nr, const uint8_t *lds, uint32_t slot) {
  uint32_t s[N][4];
#pragma unroll
  for (int q = 0; q < N; ++q) {
    s[q][0] = bswap32(v[q].x) ^ ek[0];
    s[q][1] = bswap32(v[q].y) ^ ek[1];
    s[q][2] = bswap32(v[q].z) ^ ek[2];
    s[q][3] = bswap32(v[q].w) ^ ek[3];
  }
#pragma unroll 1
  for (int r = 1; r < nr; ++r) {
    const uint32_t k0 = ror16(ek[4 * r]), k1 = ror16(ek[4 * r + 1]);
    const uint32_t k2 = ror16(ek[4 * r + 2]), k3 = ror16(ek[4 * r + 3]);
#pragma unroll
    for (int q = 0; q < N; ++q) {
      const uint32_t s0 = s[q][0], s1 = s[q][1], s2 = s[q][2], s3 = s[q][3];
      const uint32_t a0 = t0(lds, tpa(s0, slot, 3)), b0 = t1(lds, tpa(s1, slot, 2));
      const uint32_t c0 = t0(lds, tpa(s2, slot, 1)), d0 = t1(lds, tpa(s3, slot, 0));
      const uint32_t a1 = t0(lds, tpa(s1, slot, 3)), b1 = t1(lds, tpa(s2, slot, 2));
      const uint32_t c1 = t0(lds, tpa(s3, slot, 1)), d1 = t1(lds, tpa(s0, slot, 0));
      const uint32_t a2 = t0(lds, tpa(s2, slot, 3)), b2 = t1(lds, tpa(s3, slot, 2));
      const uint32_t c2 = t0(lds, tpa(s0, slot, 1)), d2 = t1(lds, tpa(s1, slot, 0));
      const uint32_t a3 = t0(lds, tpa(s3, slot, 3)), b3 = t1(lds, tpa(s0, slot, 2));
      const uint32_t c3 = t0(lds, tpa(s1, slot, 1)), d3 = t1(lds, tpa(s2, slot, 0));
      s[q][0] = xor3(a0, b0, ror16(xor3(c0, d0, k0)));
      s[q][1] = xor3(a1, b1, ror16(xor3(c1, d1, k1)));
      s[q][2] = xor3(a2, b2, ror16(xor3(c2, d2, k2)));
      s[q][3] = xor3(a3, b3, ror16(xor3(c3, d3, k3)));
    }
  }
#pragma unroll
  for (int q = 0; q < N; ++q) {
    uint32_t o[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t a = t0(lds, tpa(s[q][c], slot, 3));
      const uint32_t b = t0(lds, tpa(s[q][(c + 1) & 3], slot, 2));
      const uint32_t cc = t0(lds, tpa(s[q][(c + 2) & 3], slot, 1));
      const uint32_t d = t0(lds, tpa(s[q][(c + 3) & 3], slot, 0));
      o[c] = xor3(perm(b, a, 0x0c0c0501u), perm(d, cc, 0x05010c0cu), bswap32(ek[4 * nr + c]));
    }
    v[q] = make_uint4(o[0], o[1], o[2], o[3]);
  }
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
    // e + K + W_t does not depend on a: summed first (and materialized, so
    // the adds are not reassociated), the round's critical path is a ->
    // {rotl 5, f} -> one add3 instead of a -> f -> add3 -> add3
    uint32_t ekw = e + k + wt;
    asm volatile("" : "+v"(ekw));
    const uint32_t tmp = rotl(a, 5) + f + ekw;
    e = d;
    d = c;
    c = rotl(b, 30);
    b = a;
    a = tmp;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

// ---- SHA-256 compression (SHA256_Transform, freebsd/crypto/sha2/sha256c.c:135) ----
__constant__ uint32_t kK256[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u,
};

__device__ __forceinline__ void sha256_compress(uint32_t h[8], uint32_t w[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int t = 0; t < 64; ++t) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      const uint32_t x = w[(t - 15) & 15], y = w[(t - 2) & 15];
      const uint32_t s0 = xor3(rotr(x, 7), rotr(x, 18), x >> 3);
      const uint32_t s1 = xor3(rotr(y, 17), rotr(y, 19), y >> 10);
      wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
      w[t & 15] = wt;
    }
    // h + K_t + W_t (and d + that) do not depend on this round's e or a:
    // summed first, so e' = S1 + ch + (d+h+K+W) and t1 are one add3 each
    uint32_t hkw = hh + kK256[t] + wt;
    asm volatile("" : "+v"(hkw));
    uint32_t dhkw = d + hkw;
    asm volatile("" : "+v"(dhkw));
    const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
    const uint32_t ch = __builtin_amdgcn_bitop3_b32(e, f, g, 0xCA);     // (e & f) | (~e & g)
    const uint32_t t1 = S1 + ch + hkw;
    const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
    const uint32_t mj = __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);     // majority
    hh = g; g = f; f = e; e = S1 + ch + dhkw;
    d = c; c = b; b = a; a = t1 + S0 + mj;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// The two HMAC hashes behind one interface: W chaining words.
template <int HS> struct Hash;
template <> struct Hash<HS_SHA1> {
  static constexpr int W = 5;
  static __device__ __forceinline__ void compress(uint32_t h[8], uint32_t w[16]) { sha1_compress(h, w); }
};
template <> struct Hash<HS_SHA256> {
  static constexpr int W = 8;
  static __device__ __forceinline__ void compress(uint32_t h[8], uint32_t w[16]) { sha256_compress(h, w); }
};

// message word k of the padded block b of the inner HMAC message
// rec[0, L0) || (esn ? be32(esn_hi) : "") once past the full blocks
__device__ __forceinline__ uint32_t tail_word(const uint8_t *rec, uint32_t b, int k, uint32_t L0, uint32_t L,
                                              bool esn, uint32_t esn_hi, uint32_t total, uint64_t bits) {
  const uint32_t o = 64 * b + 4 * k;
  uint32_t v;
  if (o + 4 <= L0) v = bswap32(*reinterpret_cast<const uint32_t *>(rec + o));
  else if (esn && o == L0) v = esn_hi;
  else if (o == L) v = 0x80000000u;
  else v = 0;
  if (b == total - 1 && k == 14) v = (uint32_t)(bits >> 32);
  if (b == total - 1 && k == 15) v = (uint32_t)bits;
  return v;
}

// the outer block: inner digest || 0x80 || 0... || bit length of (64 + digest)
template <int HS>
__device__ __forceinline__ void outer_block(const uint32_t h[8], uint32_t w[16]) {
  constexpr int W = Hash<HS>::W;
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = k < W ? h[k] : (k == W ? 0x80000000u : 0u);
  w[15] = (64 + 4 * W) * 8;
}

// HMAC of msg = rec[0, L0) || (esn ? be32(esn_hi) : "") from the SA's
// ipad/opad chaining states (already past the 64-byte key block).
template <int HS>
__device__ void hmac_t(const uint8_t *rec, uint32_t L0, bool esn, uint32_t esn_hi, kptr ipad, kptr opad,
                       uint32_t out[8]) {
  constexpr int W = Hash<HS>::W;
  const uint32_t L = L0 + (esn ? 4u : 0u);              // multiple of 4 for ESP records
  const uint32_t nfull = L0 / 64;                       // blocks entirely from memory
  const uint32_t total = (L + 9 + 63) / 64;             // inner blocks incl. padding
  const uint64_t bits = (uint64_t)(64 + L) * 8;         // the ipad block counts
  uint32_t h[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) h[k] = k < W ? ipad[k] : 0u;
  uint32_t w[16];
  // One compression site for every block (inner data, inner padding, outer)
  // keeps a single inlined copy of the rounds.  (Prefetching the next block,
  // or two blocks per step, measured equal or slower: DESIGN.md §6.)
  for (uint32_t b = 0; b <= total; ++b) {
    if (b < nfull) {
      const uint8_t *p = rec + 64 * b;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint4 v = bswap4(ld16(p + 16 * q));
        w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
      }
    } else if (b < total) {
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = tail_word(rec, b, k, L0, L, esn, esn_hi, total, bits);
    } else {
      outer_block<HS>(h, w);
#pragma unroll
      for (int k = 0; k < W; ++k) h[k] = opad[k];
    }
    if (eopts() & 0x20000) {                   // knob: the loads without the compression
#pragma unroll
      for (int k = 0; k < 16; ++k) h[k & 7] ^= w[k];
    } else {
      Hash<HS>::compress(h, w);
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) out[k] = h[k];
}

// hmac_t for a whole wave whose lanes each verify one record (MODE 2's
// verify, MODE 1's ICVs): the same hash, but a block's 64 bytes reach their lane by
// a coalesced load.  Lane 4Q+k loads piece k (16 bytes) of block b of each of
// the quad's 4 records, so one load instruction covers 16 records x 64
// contiguous bytes (16 lines) instead of 64 records x 16 bytes (64 lines), and
// a 4x4 transpose across the quad (DPP) hands each lane its record's pieces.
// Every lane of the wave must call it (act = this lane's record is hashed);
// the block loop runs to the wave's longest message.
template <int CTRL>
__device__ __forceinline__ uint32_t qdpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xf, 0xf, true);
}
template <int I>
__device__ __forceinline__ uint32_t qbcast(uint32_t x) { return qdpp<I * 0x55>(x); }   // quad_perm [I,I,I,I]

// A record address rebuilt from its broadcast halves, as a global-memory
// pointer: a plain integer-to-pointer cast is a generic (flat) address, and
// flat loads and stores count in lgkmcnt too, beside the LDS table reads
// (measured equal in time: profiles/r6_cfg3_encrypt_pipe_ab.txt).
__device__ __forceinline__ uint8_t *gptr(uint64_t a) {
  return (uint8_t *)(__attribute__((address_space(1))) uint8_t *)(uintptr_t)a;
}

// lane q of a quad: A[i] (i = 0..3) -> lane q holds, in A[k], lane k's A[q]
__device__ __forceinline__ void quad_transpose4(uint32_t (&A)[4], bool qb0, bool qb1) {
#pragma unroll
  for (int b = 0; b < 2; ++b) {                  // distance 2: pairs (0,2), (1,3)
    const uint32_t y = qdpp<0x4E>(qb1 ? A[b] : A[b + 2]);
    A[b] = qb1 ? y : A[b];
    A[b + 2] = qb1 ? A[b + 2] : y;
  }
#pragma unroll
  for (int b = 0; b < 4; b += 2) {               // distance 1: pairs (0,1), (2,3)
    const uint32_t y = qdpp<0xB1>(qb0 ? A[b] : A[b + 1]);
    A[b] = qb0 ? y : A[b];
    A[b + 1] = qb0 ? A[b + 1] : y;
  }
}

// NB = 2: each iteration loads blocks b and b + 1 together (a record's 128
// contiguous bytes at once, so the line they share is fetched once), then
// compresses them one after the other.
template <int HS, int NB = 1>
__device__ void hmac_quad(bool act, const uint8_t *rec, uint32_t L0, bool esn, uint32_t esn_hi, kptr ipad,
                          kptr opad, uint32_t out[8]) {
  constexpr int W = Hash<HS>::W;
  const int lane = threadIdx.x & 63, q = lane & 3;
  const bool qb0 = (q & 1) != 0, qb1 = (q & 2) != 0;
  const uint32_t L = act ? L0 + (esn ? 4u : 0u) : 0u;
  const uint32_t nfull = act ? L0 / 64 : 0u;
  const uint32_t total = act ? (L + 9 + 63) / 64 : 0u;
  const uint64_t bits = (uint64_t)(64 + L) * 8;
  uint32_t h[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) h[k] = (act && k < W) ? ipad[k] : 0u;
  // the quad's record pointers and full-block counts
  const uint64_t rp = (uint64_t)(uintptr_t)rec;
  const uint32_t rlo = (uint32_t)rp, rhi = (uint32_t)(rp >> 32);
  const uint8_t *pr[4] = {
      gptr(((uint64_t)qbcast<0>(rhi) << 32) | qbcast<0>(rlo)),
      gptr(((uint64_t)qbcast<1>(rhi) << 32) | qbcast<1>(rlo)),
      gptr(((uint64_t)qbcast<2>(rhi) << 32) | qbcast<2>(rlo)),
      gptr(((uint64_t)qbcast<3>(rhi) << 32) | qbcast<3>(rlo))};
  const uint32_t pn[4] = {qbcast<0>(nfull), qbcast<1>(nfull), qbcast<2>(nfull), qbcast<3>(nfull)};
  uint32_t tw = total;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) tw = max(tw, (uint32_t)__shfl_xor((int)tw, o));
  for (uint32_t b0 = 0; b0 <= tw; b0 += NB) {     // wave-uniform trip count
  uint4 PP[NB][4];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      PP[nb][i] = b0 + nb < pn[i] ? ld16(pr[i] + 64 * (b0 + nb) + 16 * q) : make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const uint32_t b = b0 + nb;
    if (nb > 0 && b > tw) continue;               // (wave-uniform)
    const uint4 *P = PP[nb];
    uint32_t X[4] = {P[0].x, P[1].x, P[2].x, P[3].x}, Y[4] = {P[0].y, P[1].y, P[2].y, P[3].y};
    uint32_t Z[4] = {P[0].z, P[1].z, P[2].z, P[3].z}, V[4] = {P[0].w, P[1].w, P[2].w, P[3].w};
    quad_transpose4(X, qb0, qb1);
    quad_transpose4(Y, qb0, qb1);
    quad_transpose4(Z, qb0, qb1);
    quad_transpose4(V, qb0, qb1);
    uint32_t w[16];
    if (b < nfull) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {             // piece k of this lane's record
        w[4 * k] = bswap32(X[k]);
        w[4 * k + 1] = bswap32(Y[k]);
        w[4 * k + 2] = bswap32(Z[k]);
        w[4 * k + 3] = bswap32(V[k]);
      }
    } else if (b < total) {
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = tail_word(rec, b, k, L0, L, esn, esn_hi, total, bits);
    } else if (b == total) {                     // (lanes past their total keep their digest)
      outer_block<HS>(h, w);
      if (act) {
#pragma unroll
        for (int k = 0; k < W; ++k) h[k] = opad[k];
      }
    }
    if (b <= total) {
      if (eopts() & 0x20000) {
#pragma unroll
        for (int k = 0; k < 16; ++k) h[k & 7] ^= w[k];
      } else {
        Hash<HS>::compress(h, w);
      }
    }
  }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) out[k] = h[k];
}

// MODE 4's CBC chain with hmac_quad's coalesced access: the record is still
// one lane's serial chain, but its 64-byte groups move between memory and the
// lane through the quad -- lane 4Q+k loads / stores piece k (16 bytes) of
// each of the quad's 4 records, and a 4x4 DPP transpose hands each lane its
// record's 4 blocks (and back).  One instruction covers 16 records x 64
// contiguous bytes instead of 64 records x 16 bytes.  Every lane of the wave
// calls it (act = this lane's record is encrypted); the loop runs to the
// wave's longest record.  ek: the wave-uniform encryption schedule.
template <int NB>
__device__ void cbc_enc_quad(bool act, uint8_t *rec, uint32_t nb0, kptr ek, int nr, const uint8_t *lds,
                             uint32_t slot) {
  const int lane = threadIdx.x & 63, q = lane & 3;
  const bool qb0 = (q & 1) != 0, qb1 = (q & 2) != 0;
  const uint32_t nb = act ? nb0 : 0u;
  // (the quad's record addresses and lengths are broadcast where used, not
  // kept: 12 fewer live VGPRs across the rounds; every broadcast runs on all
  // lanes, never inside a lane-dependent branch -- a DPP read of a lane the
  // branch switched off returns 0)
  const uint64_t rp = (uint64_t)(uintptr_t)rec;
  const uint32_t rlo = (uint32_t)rp, rhi = (uint32_t)(rp >> 32);
  auto pr = [&](auto I) {
    constexpr int i = decltype(I)::value;
    return gptr(((uint64_t)qbcast<i>(rhi) << 32) | qbcast<i>(rlo));
  };
  auto pn = [&](auto I) { return qbcast<decltype(I)::value>(nb); };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  uint32_t nw = nb;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) nw = max(nw, (uint32_t)__shfl_xor((int)nw, o));
  nw = __builtin_amdgcn_readfirstlane(nw);        // (equal on every lane: a scalar loop)
  uint4 prev = act ? ld16(rec + 8) : make_uint4(0, 0, 0, 0);   // IV
  // NB 64-byte groups (4 blocks each) per iteration: loaded together, chained,
  // stored together (NB = 2: a record's 128 contiguous bytes move at once)
  for (uint32_t b0 = 0; b0 < nw; b0 += 4 * NB) {  // wave-uniform trip count
    uint32_t X[NB][4], Y[NB][4], Z[NB][4], V[NB][4];
#pragma unroll
    for (int g = 0; g < NB; ++g) {
      const uint32_t b = b0 + 4 * g;
      uint4 P[4];
      auto ld = [&](auto I) {
        constexpr int i = decltype(I)::value;
        const uint8_t *a = pr(I);                  // (DPP: every lane, outside the branch)
        P[i] = b + q < pn(I) ? ld16(a + 24 + 16 * (b + q)) : make_uint4(0, 0, 0, 0);
      };
      ld(I0{});
      ld(I1{});
      ld(I2{});
      ld(I3{});
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        X[g][i] = P[i].x;
        Y[g][i] = P[i].y;
        Z[g][i] = P[i].z;
        V[g][i] = P[i].w;
      }
    }
#pragma unroll
    for (int g = 0; g < NB; ++g) {
      const uint32_t b = b0 + 4 * g;
      quad_transpose4(X[g], qb0, qb1);
      quad_transpose4(Y[g], qb0, qb1);
      quad_transpose4(Z[g], qb0, qb1);
      quad_transpose4(V[g], qb0, qb1);
#pragma unroll
      for (int k = 0; k < 4; ++k) {               // block b + k of this lane's record
        if (b + k < nb) {
          prev = aes_enc(xor4(make_uint4(X[g][k], Y[g][k], Z[g][k], V[g][k]), prev), ek, nr, lds, slot);
          X[g][k] = prev.x;
          Y[g][k] = prev.y;
          Z[g][k] = prev.z;
          V[g][k] = prev.w;
        }
      }
      quad_transpose4(X[g], qb0, qb1);            // (its own inverse)
      quad_transpose4(Y[g], qb0, qb1);
      quad_transpose4(Z[g], qb0, qb1);
      quad_transpose4(V[g], qb0, qb1);
    }
#pragma unroll
    for (int g = 0; g < NB; ++g) {
      const uint32_t b = b0 + 4 * g;
      auto st = [&](auto I) {
        constexpr int i = decltype(I)::value;
        uint8_t *a = pr(I);                        // (DPP: every lane, outside the branch)
        const bool in = b + q < pn(I);
        if (in) st16(a + 24 + 16 * (b + q), make_uint4(X[g][i], Y[g][i], Z[g][i], V[g][i]));
      };
      st(I0{});
      st(I1{});
      st(I2{});
      st(I3{});
    }
  }
}

// MODE 4 CK_CBCMAC: cbc_enc_quad's CBC chain with the HMAC of
// encrypt-then-MAC in the same pass (xform_esp.c:673-961's output order:
// encrypt, then the ICV over SPI|SN|IV|CT (|ESN hi), cryptosoft.c:874-888).
// Each 64-byte ciphertext group the chain produces is hashed from the
// lane's registers right away instead of being read back by a MAC pass:
// SHA block g is message words 16g..16g+15, i.e. the 6 words before the
// group (the 24-byte header for g = 0, else the previous group's last 6
// ciphertext words) and the group's first 10 words.  The inner hash runs to
// the wave's longest message (tail words as tail_word()), then the outer
// hash and the ICV (mlen bytes after the ciphertext).  Every lane of the
// wave calls it (act = this lane's record); ek / ipad / opad wave-uniform.
template <int HS>
__device__ void cbc_mac_quad(bool act, uint8_t *rec, uint32_t plen, kptr ek, int nr, const uint8_t *lds,
                             uint32_t slot, bool esn, uint32_t esn_hi, kptr ipad, kptr opad, uint32_t mlen) {
  constexpr int W = Hash<HS>::W;
  const int lane = threadIdx.x & 63, q = lane & 3;
  const bool qb0 = (q & 1) != 0, qb1 = (q & 2) != 0;
  const uint32_t nb = act ? plen / 16 : 0u;
  const uint32_t l0w = 6u + plen / 4;                    // message words from the record
  const uint32_t L = 4 * l0w + (esn ? 4u : 0u);          // message bytes
  const uint32_t total = act ? (L + 9 + 63) / 64 : 0u;   // inner blocks incl. padding
  const uint64_t bits = (uint64_t)(64 + L) * 8;          // the ipad block counts
  const uint64_t rp = (uint64_t)(uintptr_t)rec;
  const uint32_t rlo = (uint32_t)rp, rhi = (uint32_t)(rp >> 32);
  auto pr = [&](auto I) {
    constexpr int i = decltype(I)::value;
    return gptr(((uint64_t)qbcast<i>(rhi) << 32) | qbcast<i>(rlo));
  };
  auto pn = [&](auto I) { return qbcast<decltype(I)::value>(nb); };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  uint32_t nw = nb, gw = total;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    nw = max(nw, (uint32_t)__shfl_xor((int)nw, o));
    gw = max(gw, (uint32_t)__shfl_xor((int)gw, o));
  }
  nw = __builtin_amdgcn_readfirstlane(nw);
  gw = __builtin_amdgcn_readfirstlane(gw);
  uint4 prev = act ? ld16(rec + 8) : make_uint4(0, 0, 0, 0);   // IV
  // the 6 message words before the current group: SPI, SN, IV
  uint32_t pw[6] = {act ? *reinterpret_cast<const uint32_t *>(rec) : 0u,
                    act ? *reinterpret_cast<const uint32_t *>(rec + 4) : 0u, prev.x, prev.y, prev.z, prev.w};
  uint32_t h[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) h[k] = (act && k < W) ? ipad[k] : 0u;
  for (uint32_t g = 0; g < gw; ++g) {                 // wave-uniform trip count
    const uint32_t b = 4 * g;
    uint32_t X[4] = {0, 0, 0, 0}, Y[4] = {0, 0, 0, 0}, Z[4] = {0, 0, 0, 0}, V[4] = {0, 0, 0, 0};
    if (b < nw) {                                     // (wave-uniform)
      uint4 P[4];
      auto ld = [&](auto I) {
        constexpr int i = decltype(I)::value;
        const uint8_t *a = pr(I);                      // (DPP: every lane, outside the branch)
        P[i] = b + q < pn(I) && !(eopts() & 0x200000) ? ld16(a + 24 + 16 * (b + q)) : make_uint4(0, 0, 0, 0);
      };
      ld(I0{});
      ld(I1{});
      ld(I2{});
      ld(I3{});
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        X[i] = P[i].x;
        Y[i] = P[i].y;
        Z[i] = P[i].z;
        V[i] = P[i].w;
      }
      quad_transpose4(X, qb0, qb1);
      quad_transpose4(Y, qb0, qb1);
      quad_transpose4(Z, qb0, qb1);
      quad_transpose4(V, qb0, qb1);
#pragma unroll
      for (int k = 0; k < 4; ++k) {                   // block b + k of this lane's record
        if (b + k < nb) {
          prev = (eopts() & 0x800000) ? xor4(make_uint4(X[k], Y[k], Z[k], V[k]), prev)
                                      : aes_enc(xor4(make_uint4(X[k], Y[k], Z[k], V[k]), prev), ek, nr, lds, slot);
          X[k] = prev.x;
          Y[k] = prev.y;
          Z[k] = prev.z;
          V[k] = prev.w;
        }
      }
    }
    // SHA block g from the 6 words before the group and its first 10
    const uint32_t c[16] = {X[0], Y[0], Z[0], V[0], X[1], Y[1], Z[1], V[1],
                            X[2], Y[2], Z[2], V[2], X[3], Y[3], Z[3], V[3]};
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t m = 16 * g + (uint32_t)k;
      uint32_t v = bswap32(k < 6 ? pw[k] : c[k - 6]);
      if (m >= l0w) v = (esn && m == l0w) ? esn_hi : (4 * m == L ? 0x80000000u : 0u);
      if (g + 1 == total && k == 14) v = (uint32_t)(bits >> 32);
      if (g + 1 == total && k == 15) v = (uint32_t)bits;
      w[k] = v;
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) pw[k] = c[10 + k];
    if (b < nw) {                                     // the ciphertext back, quad-coalesced
      quad_transpose4(X, qb0, qb1);
      quad_transpose4(Y, qb0, qb1);
      quad_transpose4(Z, qb0, qb1);
      quad_transpose4(V, qb0, qb1);
      auto st = [&](auto I) {
        constexpr int i = decltype(I)::value;
        uint8_t *a = pr(I);                            // (DPP: every lane, outside the branch)
        if (b + q < pn(I) && !(eopts() & 0x100000)) st16(a + 24 + 16 * (b + q), make_uint4(X[i], Y[i], Z[i], V[i]));
      };
      st(I0{});
      st(I1{});
      st(I2{});
      st(I3{});
    }
    if (g < total && !(eopts() & 0x400000)) Hash<HS>::compress(h, w);
  }
  if (act) {
    uint32_t w[16], o[8];
    outer_block<HS>(h, w);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = k < W ? opad[k] : 0u;
    Hash<HS>::compress(o, w);
    for (uint32_t k = 0; k < mlen / 4; ++k) *reinterpret_cast<uint32_t *>(rec + 24 + plen + 4 * k) = bswap32(o[k]);
  }
}

// ---- SHA-512 / SHA-384 compression (SHA512_Transform, freebsd/crypto/sha2/sha512c.c:196) ----
// 64-bit words held as uint64_t; rotations as two v_alignbit on the halves.
__constant__ uint64_t kK512[80] = ESPGPU_SHA512_K;

__device__ __forceinline__ uint64_t rotr64(uint64_t x, int n) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  uint32_t rl, rh;
  if (n < 32) {
    rl = __builtin_amdgcn_alignbit(hi, lo, n);
    rh = __builtin_amdgcn_alignbit(lo, hi, n);
  } else {
    rl = __builtin_amdgcn_alignbit(lo, hi, n - 32);
    rh = __builtin_amdgcn_alignbit(hi, lo, n - 32);
  }
  return ((uint64_t)rh << 32) | rl;
}

__device__ __forceinline__ void sha512_compress(uint64_t h[8], uint64_t w[16]) {
  uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int t = 0; t < 80; ++t) {
    uint64_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      const uint64_t x = w[(t - 15) & 15], y = w[(t - 2) & 15];
      const uint64_t s0 = rotr64(x, 1) ^ rotr64(x, 8) ^ (x >> 7);
      const uint64_t s1 = rotr64(y, 19) ^ rotr64(y, 61) ^ (y >> 6);
      wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
      w[t & 15] = wt;
    }
    const uint64_t S1 = rotr64(e, 14) ^ rotr64(e, 18) ^ rotr64(e, 41);
    const uint64_t ch = (e & f) ^ (~e & g);
    const uint64_t t1 = hh + S1 + ch + kK512[t] + wt;
    const uint64_t S0 = rotr64(a, 28) ^ rotr64(a, 34) ^ rotr64(a, 39);
    const uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
    hh = g; g = f; f = e; e = d + t1;
    d = c; c = b; b = a; a = t1 + S0 + mj;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// 32-bit message word k (0..31) of the padded 128-byte block b of the inner
// message rec[0, L0) || (esn ? be32(esn_hi) : ""); the 128-bit length field
// is words 28..31 of the last block (its high 64 bits are zero)
__device__ __forceinline__ uint32_t tail_word128(const uint8_t *rec, uint32_t b, int k, uint32_t L0, uint32_t L,
                                                 bool esn, uint32_t esn_hi, uint32_t total, uint64_t bits) {
  const uint32_t o = 128 * b + 4 * k;
  uint32_t v;
  if (o + 4 <= L0) v = bswap32(*reinterpret_cast<const uint32_t *>(rec + o));
  else if (esn && o == L0) v = esn_hi;
  else if (o == L) v = 0x80000000u;
  else v = 0;
  if (b == total - 1 && k == 30) v = (uint32_t)(bits >> 32);
  if (b == total - 1 && k == 31) v = (uint32_t)bits;
  return v;
}

// HMAC-SHA2-384 / -512 (hmac_init_pad states from the host: 16 words each,
// word 2k = high half of state word k) of msg = rec[0, L0) || (esn ? be32(esn_hi) : "");
// out = the 48- or 64-byte digest as big-endian 32-bit words
__device__ void hmac_wide(const uint8_t *rec, uint32_t L0, bool esn, uint32_t esn_hi, bool is384, kptr ipad,
                          kptr opad, uint32_t out[16]) {
  const uint32_t L = L0 + (esn ? 4u : 0u);
  const uint32_t nfull = L0 / 128;                      // blocks entirely from memory
  const uint32_t total = (L + 17 + 127) / 128;          // inner blocks incl. padding
  const uint64_t bits = (uint64_t)(128 + L) * 8;        // the ipad block counts
  const int dw = is384 ? 6 : 8;                         // digest words (64-bit)
  uint64_t h[8], w[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) h[k] = ((uint64_t)ipad[2 * k] << 32) | ipad[2 * k + 1];
  for (uint32_t b = 0; b <= total; ++b) {
    if (b < nfull) {
      const uint8_t *p = rec + 128 * b;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const uint4 v = ld16(p + 16 * q);
        w[2 * q] = ((uint64_t)bswap32(v.x) << 32) | bswap32(v.y);
        w[2 * q + 1] = ((uint64_t)bswap32(v.z) << 32) | bswap32(v.w);
      }
    } else if (b < total) {
#pragma unroll
      for (int k = 0; k < 16; ++k)
        w[k] = ((uint64_t)tail_word128(rec, b, 2 * k, L0, L, esn, esn_hi, total, bits) << 32) |
               tail_word128(rec, b, 2 * k + 1, L0, L, esn, esn_hi, total, bits);
    } else {
      // outer block: inner digest || 0x80 || 0... || bit length of (128 + digest)
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = k < dw ? h[k] : (k == dw ? 0x8000000000000000ull : 0ull);
      w[15] = (uint64_t)(128 + 8 * dw) * 8;
#pragma unroll
      for (int k = 0; k < 8; ++k) h[k] = ((uint64_t)opad[2 * k] << 32) | opad[2 * k + 1];
    }
    sha512_compress(h, w);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    out[2 * k] = (uint32_t)(h[k] >> 32);
    out[2 * k + 1] = (uint32_t)h[k];
  }
}

__device__ __forceinline__ bool wide_hash(uint32_t aalg) {
  return aalg == ESPGPU_CRYPTO_SHA2_384_HMAC || aalg == ESPGPU_CRYPTO_SHA2_512_HMAC;
}

__device__ __forceinline__ kptr kp(const void *p) { return (kptr)p; }

// out: the digest as big-endian words (5 / 8 / 12 / 16 of them)
__device__ __forceinline__ void hmac_any(int aalg, const uint8_t *rec, uint32_t L0, bool esn, uint32_t esn_hi,
                                         kptr ipad, kptr opad, uint32_t out[16]) {
  if (wide_hash((uint32_t)aalg))
    hmac_wide(rec, L0, esn, esn_hi, aalg == ESPGPU_CRYPTO_SHA2_384_HMAC, ipad, opad, out);
  else if (aalg == ESPGPU_CRYPTO_SHA2_256_HMAC)
    hmac_t<HS_SHA256>(rec, L0, esn, esn_hi, ipad, opad, out);
  else
    hmac_t<HS_SHA1>(rec, L0, esn, esn_hi, ipad, opad, out);
}

__device__ __forceinline__ void fill_pair(uint8_t *lds, uint32_t base, const uint2 *tab, int tid, int wg) {
  for (int idx = tid; idx < 256 * 32; idx += wg) {
    const int x = idx >> 5, r = idx & 31;
    const uint2 t = tab[x];
    *reinterpret_cast<uint32_t *>(lds + base + x * 256 + r * 4) = t.x;
    *reinterpret_cast<uint32_t *>(lds + base + x * 256 + 128 + r * 4) = t.y;
  }
}

// The verified decrypt of a wave unit (MODE 2 in place, MODE 3 to p.out):
// run = this lane's record passed verification; (sa, off, plen, di, salt) its
// session, offset, payload length, descriptor index and salt.  All of the
// wave's blocks of one session as one flat list: records to decrypt (one
// session at a time, so the round keys stay wave-uniform in SGPRs) are
// concatenated; every lane takes one block per pass, last pass first.
// Within a pass all lanes load their blocks (and C_{i-1}) before any lane
// stores, and a pass only overwrites blocks no later (lower) pass reads:
// in-place decryption is safe without holding records in registers.
template <int MODE>
__device__ __forceinline__ void verified_decrypt(const EtaParams &p, const uint8_t *lds, uint32_t slot, int lane,
                                                 bool run, uint32_t sa, uint32_t off, uint32_t plen, uint32_t di,
                                                 uint32_t salt) {
  uint64_t todo = __ballot(run);
  while (todo) {
    const uint32_t sau = __builtin_amdgcn_readfirstlane(__shfl(sa, __builtin_ctzll(todo)));
    const bool mine = run && sa == sau;
    todo &= ~__ballot(mine);
    run = run && !mine;
    const DevSA *s = p.sas + sau;
    const bool ctr = s->calg == ESPGPU_CRYPTO_AES_ICM;      // wave-uniform
    const bool null = s->calg == ESPGPU_CRYPTO_NULL_CBC;    // ESP-NULL: the identity
    const uint32_t nb = mine ? (plen + 15) / 16 : 0;
    uint32_t incl = nb;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(incl, o);
      if (lane >= o) incl += v;
    }
    const uint32_t start = incl - nb;
    const int total = (int)__builtin_amdgcn_readfirstlane(__shfl(incl, 63));
    const int nr = (int)s->nr;
    // Equal-length records in lanes 0..m-1 and none after (a planner unit
    // of one MTU, as cfg3's): flat block f is block f - j*nbu of lane j =
    // f / nbu, a multiply-shift (exact: f * nbu < 2^32) instead of the
    // shuffle search's six ds_bpermutes on the LDS pipe
    const uint64_t mm = __ballot(mine);
    const uint32_t nbu = __builtin_amdgcn_readfirstlane(nb);   // lane 0's (mm has bit 0 if uniform)
    const bool uni = (mm & (mm + 1)) == 0 && (mm & 1) && __all(!mine || nb == nbu) && nbu > 0;
    const uint64_t inv = uni ? ((1ull << 32) + nbu - 1) / nbu : 0u;   // ceil(2^32 / nbu)
    // kEtaU blocks per lane per pass, 64 apart (each load instruction
    // covers 64 consecutive blocks), decrypted together for ILP
    constexpr int U = kEtaU;
    for (int base = total - 64 * U; base > -64 * U; base -= 64 * U) {
      int fk[U];
      uint32_t ik[U], rok[U], rplk[U], rdik[U], rsk[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const int f = base + lane + 64 * k;
        // the record holding flat block f: the last lane whose start <= f
        // (6-step shuffle search; by ballot and v_readlane it measured equal)
        int j = 0;
        uint32_t sj = 0;
        if (uni) {                                    // (wave-uniform)
          j = f < 0 ? 0 : (int)(((uint64_t)(uint32_t)f * inv) >> 32);   // = f / nbu
          sj = (uint32_t)j * nbu;
        } else {
#pragma unroll
          for (int step = 32; step >= 1; step >>= 1) {
            const uint32_t sc = __shfl(start, j + step);
            if ((int)sc <= f) {
              j += step;
              sj = sc;
            }
          }
        }
        fk[k] = f;
        ik[k] = (uint32_t)f - sj;
        rok[k] = __shfl(off, j);
        // (each __shfl is a ds_bpermute on the LDS pipe the AES lookups
        // bound: only what the session kind uses, wave-uniform conditions)
        rplk[k] = (ctr || null || p.trailer) ? __shfl(plen, j) : 0u;
        rdik[k] = p.trailer ? __shfl(di, j) : 0u;
        rsk[k] = ctr ? __shfl(salt, j) : 0u;
      }
      // all loads of the pass before any store (in place: see above)
      uint4 v[U], pv[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        v[k] = pv[k] = make_uint4(0, 0, 0, 0);
        if (fk[k] >= 0 && !(eopts() & 0x80000)) {             // knob: no decrypt-pass loads
          const uint8_t *rec = p.arena + rok[k];
          if (null) {
            v[k] = ld16(rec + 8 + 16 * ik[k]);                                     // P_i = C_i
          } else if (ctr) {
            pv[k] = ld16(rec + 16 + 16 * ik[k]);                                   // C_i
            v[k] = make_uint4(rsk[k], *reinterpret_cast<const uint32_t *>(rec + 8),
                              *reinterpret_cast<const uint32_t *>(rec + 12), bswap32(ik[k] + 1));
          } else {
            v[k] = ld16(rec + 24 + 16 * ik[k]);                                    // C_i
            pv[k] = ld16(rec + 8 + 16 * ik[k]);                // C_{i-1}, or the IV for i = 0
          }
        }
      }
      if (null) {
      } else if (ctr) {
        aes_enc4(v, kp(s->rk), nr, lds + LDS_TE, slot);
      } else if (!(eopts() & 0x40000)) {                       // knob: no decrypt-pass AES
        aes_dec4(v, kp(s->dk), nr, lds, slot);
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        if (fk[k] >= 0 && !(eopts() & 0x80000)) {             // knob: no decrypt-pass stores
          uint8_t *dst = (MODE == 2 ? p.arena : p.out) + rok[k];   // MODE 3: p.out (may be p.arena)
          const uint32_t i = ik[k], rpl = rplk[k];
          const int rem = (int)rpl - 16 * (int)i;
          const uint4 pt = xor4(v[k], pv[k]);
          if (null) {
            if (MODE != 2 && p.out != p.arena) st_partial(dst + 8 + 16 * i, pt, rem);   // in place: as is
          } else if (ctr) {
            st_partial(dst + 16 + 16 * i, pt, rem);
          } else {
            st16(dst + 24 + 16 * i, pt);
          }
          if (p.trailer && i == (rpl + 15) / 16 - 1) p.trailer[rdik[k]] = esp_trailer_word(last_word(pt, rem), rpl);
        }
      }
    }
  }
}

// MODE 1: encrypt, MAC pass over the ciphertext MODE 4 wrote (lane = record
//         HMAC, ICV written) for AES-CTR / ESP-NULL records and, at SHA2-384 /
//         512, CBC ones;
// MODE 2: decrypt in place, verify first: the verify pass (lane = record
//         HMAC), then the block-parallel decrypt of the verified records;
// MODE 3: decrypt out of place: the same two passes, plaintext to p.out;
// MODE 4: encrypt, cipher pass (lane = record CBC chain, with the HMAC-SHA1 /
//         SHA2-256 ICV in the same pass; CTR keystream).
// CKS: MODE 4 is built once per cipher (CK_CBCMAC / CK_CTR); MODE 1 / 2 / 3 once
// per hash width (CK_NARROW: HMAC-SHA1 / SHA2-256 / no auth, no SHA-512 code,
// so the registers fit without spilling; CK_WIDEH: HMAC-SHA2-384/512).
// (Measured slower and not built: the one-pass out-of-place decrypt, the
// verify and decrypt passes as separate kernels, side by side on two streams,
// or interleaved per wave; the in-place one pass with CBC rollback; wave-
// specialised verify / decrypt roles and lagging waves; a CBC cipher pass at
// 8 waves / SIMD followed by a MAC pass: DESIGN.md §3.2, §5.1, §5.2, §6.)
template <int MODE, int WG, int CKS>
__global__ __launch_bounds__(WG, 1) void eta_kernel(EtaParams p) {
  static_assert(MODE >= 1 && MODE <= 4, "MAC pass, in-place / out-of-place decrypt, cipher pass");
  __shared__ __attribute__((aligned(16))) uint8_t lds[lds_bytes(MODE)];
  const int tid = threadIdx.x, lane = tid & 63;
  const uint32_t slot = (uint32_t)(lane & 31) * 4;
  if (MODE == 4) {
    fill_pair(lds, LDS_T, p.tpair, tid, WG);
  } else if (MODE != 1) {                         // MODE 1 (the MAC pass) reads no table
    fill_pair(lds, LDS_T, p.dpair, tid, WG);
    for (int idx = tid; idx < 256 * 32; idx += WG)
      *reinterpret_cast<uint32_t *>(lds + LDS_SI + idx * 4) = p.isbox[idx >> 5];
    fill_pair(lds, LDS_TE, p.tpair, tid, WG);
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
    uint32_t off = 0, len = 0, sa = 0, plen = 0, hl = 24, salt = 0, esnh = 0;
    int hq = 0;                                  // MODE 2 narrow: 1 SHA-1 / 2 SHA2-256 record to hash
    bool hq_esn = false;
    uint32_t hq_mlen = 0;
    if (have) {
      const uint4 dv = *reinterpret_cast<const uint4 *>(p.desc + di);
      off = dv.x * 4;
      len = dv.y & 0xffffu;
      sa = dv.y >> 16;
      esnh = dv.z;
      salt = dv.w;
      const DevSA *s = sa < p.nsas ? p.sas + sa : nullptr;
      if (!s || s->mode != ESPGPU_CSP_MODE_ETA) {
        have = false;                                       // not ours (GCM kernel / EINVAL)
        if (!s || s->mode == 0) {
          p.status[di] = ESPGPU_EINVAL;
          if (MODE != 1 && p.trailer) p.trailer[di] = 0;
        }
      } else if (MODE == 4 && (s->calg == ESPGPU_CRYPTO_NULL_CBC ||
                               (s->calg == ESPGPU_CRYPTO_AES_ICM) != (CKS == CK_CTR))) {
        have = false;                                       // the other cipher's pass / no cipher
      } else if (MODE != 4 && ((CKS == CK_NARROW && wide_hash(s->aalg)) || (CKS == CK_WIDEH && !wide_hash(s->aalg)))) {
        have = false;                                       // the other hash set's launch
      } else {
        const bool ctr = s->calg == ESPGPU_CRYPTO_AES_ICM, null = s->calg == ESPGPU_CRYPTO_NULL_CBC;
        const uint32_t mlen = s->mlen;
        hl = ctr ? 16u : null ? 8u : 24u;                   // SPI|SN|IV8, SPI|SN, SPI|SN|IV16
        const int pl = (int)len - (int)hl - (int)mlen;      // alen = mlen (0: no auth)
        // xform_esp.c:316-324: payload > 0 and a multiple of the cipher's
        // blocksize (16 for CBC, 1 for CTR, 4 for NULL; records are 4-byte
        // multiples)
        valid = pl > 0 && (ctr || null || (pl & 15) == 0) && (len & 3) == 0;
        plen = valid ? (uint32_t)pl : 0;
        if (valid && (MODE == 2 || MODE == 3) && s->aalg == 0) {
          ok = true;                                        // CSP_MODE_CIPHER: nothing to verify
        } else if (valid && (MODE == 2 || MODE == 3) && (eopts() & 0x10000)) {
          ok = true;                                        // knob: no verify pass at all
        } else if (valid && MODE == 2 && CKS == CK_NARROW) {
          hq = s->aalg == ESPGPU_CRYPTO_SHA2_256_HMAC ? 2 : 1;   // hashed below, by the whole wave
          hq_esn = (s->flags & ESPGPU_CSP_F_ESN) != 0;
          hq_mlen = mlen;
        } else if (valid && (MODE == 2 || MODE == 3)) {
          uint32_t dg[16];
          const uint8_t *rec = p.arena + off;
          if (CKS == CK_NARROW) {              // SHA-1 / SHA2-256 only: no SHA-512 code, fewer VGPRs
            if (s->aalg == ESPGPU_CRYPTO_SHA2_256_HMAC)
              hmac_t<HS_SHA256>(rec, hl + plen, (s->flags & ESPGPU_CSP_F_ESN) != 0, esnh, kp(s->ipad),
                                kp(s->opad), dg);
            else
              hmac_t<HS_SHA1>(rec, hl + plen, (s->flags & ESPGPU_CSP_F_ESN) != 0, esnh, kp(s->ipad),
                              kp(s->opad), dg);
          } else {
            hmac_any((int)s->aalg, rec, hl + plen, (s->flags & ESPGPU_CSP_F_ESN) != 0, esnh, kp(s->ipad),
                     kp(s->opad), dg);
          }
          uint32_t diff = 0;
          for (uint32_t k = 0; k < mlen / 4; ++k)
            diff |= bswap32(dg[k]) ^ *reinterpret_cast<const uint32_t *>(rec + hl + plen + 4 * k);
          ok = diff == 0 || (eopts() & 0x20000);            // (knob: no compression, decrypt anyway)
        }
      }
    }
    if (MODE == 2 && CKS == CK_NARROW) {
      // the verify of this unit's records, the whole wave at once
      // (hmac_quad: quad-coalesced loads, two hash blocks per load)
      for (int hs = 1; hs <= 2; ++hs) {           // (not unrolled: two hmac_quad bodies)
        if (!__any(hq == hs)) continue;           // wave-uniform
        const bool act = hq == hs;
        const DevSA *s = p.sas + (act ? sa : 0u);
        const uint8_t *rec = p.arena + off;
        uint32_t dg[16];
        if (hs == 2)
          hmac_quad<HS_SHA256, 2>(act, rec, hl + plen, hq_esn, esnh, kp(s->ipad), kp(s->opad), dg);
        else
          hmac_quad<HS_SHA1, 2>(act, rec, hl + plen, hq_esn, esnh, kp(s->ipad), kp(s->opad), dg);
        if (act) {
          uint32_t diff = 0;
          for (uint32_t k = 0; k < hq_mlen / 4; ++k)
            diff |= bswap32(dg[k]) ^ *reinterpret_cast<const uint32_t *>(rec + hl + plen + 4 * k);
          ok = diff == 0 || (eopts() & 0x20000);
        }
      }
    }
    if (MODE == 4) {
      // ---- encrypt, cipher pass (one kernel per cipher): lane = record.
      // CK_CBCMAC: the serial CBC chain (one AES state per lane) with the
      // record's HMAC-SHA1 / SHA2-256 hashed from its registers (cbc_mac_quad,
      // 113 VGPRs, 16 waves per CU; at 5 waves/SIMD it spills and runs 18 %
      // slower); CK_CTR: the keystream 4 blocks at a time (the MAC pass
      // follows) ----
      // One session at a time (a planner chunk has one): the session pointer
      // is wave-uniform, so the round keys come through the scalar cache into
      // SGPRs instead of a vector load per round on the CBC chain's critical
      // path (per-lane keys: 2.87 ms for cfg3's 1M x 1496-B records)
      bool run = have && valid;
      uint64_t todo = __ballot(run);
      while (todo) {
        const uint32_t sau = __builtin_amdgcn_readfirstlane(__shfl(sa, __builtin_ctzll(todo)));
        const bool mine = run && sa == sau;
        todo &= ~__ballot(mine);
        run = run && !mine;
        const DevSA *s = p.sas + sau;
        const int nr = (int)s->nr;
        if (CKS == CK_CBCMAC) {                   // the chain and, for SHA-1 / SHA2-256, the ICV
          const bool esn = (s->flags & ESPGPU_CSP_F_ESN) != 0;
          if (s->aalg == ESPGPU_CRYPTO_SHA1_HMAC)
            cbc_mac_quad<HS_SHA1>(mine, p.arena + off, plen, kp(s->rk), nr, lds, slot, esn, esnh, kp(s->ipad),
                                  kp(s->opad), s->mlen);
          else if (s->aalg == ESPGPU_CRYPTO_SHA2_256_HMAC)
            cbc_mac_quad<HS_SHA256>(mine, p.arena + off, plen, kp(s->rk), nr, lds, slot, esn, esnh,
                                    kp(s->ipad), kp(s->opad), s->mlen);
          else                                    // no auth, or SHA2-384/512 (the wide MAC pass)
            cbc_enc_quad<1>(mine, p.arena + off, plen / 16, kp(s->rk), nr, lds, slot);
          continue;
        }
        if (CKS != CK_CTR || !mine) continue;
        uint8_t *rec = p.arena + off;
        const uint32_t iv0 = *reinterpret_cast<const uint32_t *>(rec + 8);
        const uint32_t iv1 = *reinterpret_cast<const uint32_t *>(rec + 12);
        const uint32_t nb = (plen + 15) / 16;
        for (uint32_t b = 0; b < nb; b += 4) {
          uint4 ks[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) ks[k] = make_uint4(salt, iv0, iv1, bswap32(b + (uint32_t)k + 1));
          aes_enc4(ks, kp(s->rk), nr, lds, slot);
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (b + k < nb)
              st_partial(rec + 16 + 16 * (b + k), xor4(ld16(rec + 16 + 16 * (b + k)), ks[k]),
                         (int)(plen - 16 * (b + k)));
        }
      }
      // the fused pass may be the only one for its records (no MAC pass when
      // the ctx has no AES-CTR / ESP-NULL session)
      if (CKS == CK_CBCMAC && have) p.status[di] = valid ? ESPGPU_OK : ESPGPU_EINVAL;
      continue;
    }
    if (MODE == 1) {
      // ---- encrypt, MAC pass (after MODE 4 wrote the ciphertext): HMAC over
      // SPI|SN|IV|CT (|ESN), ICV = its first mlen bytes ----
      // SHA-1 / SHA2-256 ICVs with hmac_quad's coalesced block loads (the whole
      // wave calls it), SHA2-384/512 with hmac_any
      int hq1 = 0;
      if (have && valid && p.sas[sa].calg != ESPGPU_CRYPTO_AES_CBC) {   // (CBC: the fused cipher pass's)
        const uint32_t aa = p.sas[sa].aalg;
        hq1 = aa == ESPGPU_CRYPTO_SHA1_HMAC ? 1 : aa == ESPGPU_CRYPTO_SHA2_256_HMAC ? 2 : 0;
      }
      for (int hs = 1; hs <= 2; ++hs) {           // (not unrolled: two hmac_quad bodies)
        if (!__any(hq1 == hs)) continue;          // wave-uniform
        const bool act = hq1 == hs;
        const DevSA *s = p.sas + (act ? sa : 0u);
        uint8_t *rec = p.arena + off;
        uint32_t dg[16];
        if (hs == 2)
          hmac_quad<HS_SHA256, 2>(act, rec, hl + plen, act && (s->flags & ESPGPU_CSP_F_ESN) != 0, esnh,
                                  kp(s->ipad), kp(s->opad), dg);
        else
          hmac_quad<HS_SHA1, 2>(act, rec, hl + plen, act && (s->flags & ESPGPU_CSP_F_ESN) != 0, esnh,
                                kp(s->ipad), kp(s->opad), dg);
        if (act)
          for (uint32_t k = 0; k < s->mlen / 4; ++k)
            *reinterpret_cast<uint32_t *>(rec + hl + plen + 4 * k) = bswap32(dg[k]);
      }
      if (CKS != CK_NARROW && have && valid && hq1 == 0 && p.sas[sa].aalg != 0) {   // CSP_MODE_CIPHER: no ICV
        const DevSA *s = p.sas + sa;
        uint8_t *rec = p.arena + off;
        uint32_t dg[16];
        hmac_any((int)s->aalg, rec, hl + plen, (s->flags & ESPGPU_CSP_F_ESN) != 0, esnh, kp(s->ipad),
                 kp(s->opad), dg);
        for (uint32_t k = 0; k < s->mlen / 4; ++k)
          *reinterpret_cast<uint32_t *>(rec + hl + plen + 4 * k) = bswap32(dg[k]);
      }
      if (have) p.status[di] = valid ? ESPGPU_OK : ESPGPU_EINVAL;
      continue;
    }
    if (have) p.status[di] = !valid ? ESPGPU_EINVAL : (ok ? ESPGPU_OK : ESPGPU_EBADMSG);
    // trailer word: 0 now for records that will not be decrypted; the lane
    // decrypting a record's last block writes the others'
    if (have && p.trailer && !(valid && ok)) p.trailer[di] = 0;

    verified_decrypt<MODE>(p, lds, slot, lane, have && valid && ok, sa, off, plen, di, salt);
  }
  // Every wave leaves the loop after drawing one ticket past the end, so once
  // all have retired no ticket is drawn again: reset for the next launch.
  if (lane == 0 && atomicAdd(&p.queue[1], 1u) == gridDim.x * (WG / 64) - 1) {
    atomicExch(&p.queue[0], 0u);
    atomicExch(&p.queue[1], 0u);
  }
}

}  // namespace

int set_eta_opts(uint32_t opts) {
#ifdef ESPGPU_KNOBS
  return hipMemcpyToSymbol(HIP_SYMBOL(e_opts), &opts, 4) == hipSuccess ? 0 : -1;
#else
  return opts ? -1 : 0;
#endif
}

// Decrypt: 160 KiB of LDS, one workgroup per CU; the in-place SHA-1 /
// SHA2-256 launch at 1024 threads (hmac_quad: 128 VGPRs, 4 waves/SIMD), the
// others at 768 (3 waves/SIMD at up to 170 VGPRs: the unrolled hash schedules
// need ~150).  Encrypt: the fused CBC + HMAC pass and the CTR cipher pass at
// 1024 threads (the CTR pass up to two workgroups per CU), then the MAC pass
// for the CTR / ESP-NULL records only.
int launch_eta(const EtaParams &p, int encrypt, int kinds, int grid, void *stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (grid <= 0) grid = 256;
  // implicit units (64 records, one wave each): no more workgroups than units
  auto clamp = [&](int g, int wg) {
    if (p.chunks != nullptr) return g;
    const int units = (int)((p.n + 63) / 64), wpg = wg / 64;
    return std::max(1, std::min(g, (units + wpg - 1) / wpg));
  };
  const int in_place = !encrypt && p.out == p.arena;
  if (encrypt) {
    // Every CBC record's chain, and the ICV of the HMAC-SHA1 / SHA2-256
    // ones, in one pass (CK_CBCMAC: the ciphertext is hashed from registers,
    // not read back; cfg3 encrypt 2.56 -> 2.37 ms against a cipher pass then
    // a MAC pass, profiles/r6_cfg3_fused_encrypt_ab.txt); the MAC pass then
    // serves only AES-CTR / ESP-NULL records (none: not launched)
    if (kinds & 5)
      hipLaunchKernelGGL((eta_kernel<4, 1024, CK_CBCMAC>), dim3(clamp(grid, 1024)), dim3(1024), 0, st, p);
    if (kinds & 10) hipLaunchKernelGGL((eta_kernel<4, 1024, CK_CTR>), dim3(clamp(2 * grid, 1024)), dim3(1024), 0, st, p);
    // MAC pass by hash width, as the decrypt: SHA-1 / SHA2-256 / no auth
    // without the SHA-512 code (1024 threads), SHA2-384/512 apart
    if (kinds & 10)
      hipLaunchKernelGGL((eta_kernel<1, 1024, CK_NARROW>), dim3(clamp(grid, 1024)), dim3(1024), 0, st, p);
    if (kinds & 16) hipLaunchKernelGGL((eta_kernel<1, 768, CK_WIDEH>), dim3(clamp(grid, 768)), dim3(768), 0, st, p);
  } else if (in_place) {
    hipLaunchKernelGGL((eta_kernel<2, 1024, CK_NARROW>), dim3(clamp(grid, 1024)), dim3(1024), 0, st, p);
    if (kinds & 16) hipLaunchKernelGGL((eta_kernel<2, 768, CK_WIDEH>), dim3(clamp(grid, 768)), dim3(768), 0, st, p);
  } else {
    hipLaunchKernelGGL((eta_kernel<3, 768, CK_NARROW>), dim3(clamp(grid, 768)), dim3(768), 0, st, p);
    if (kinds & 16) hipLaunchKernelGGL((eta_kernel<3, 768, CK_WIDEH>), dim3(clamp(grid, 768)), dim3(768), 0, st, p);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace espgpu
