// esp_gcm.hip — ESP AES-GCM-16 verify+decrypt / encrypt kernel for gfx950.
//
// Replaces swcr_gcm (freebsd/opencrypto/cryptosoft.c:465-645) as reached from
// esp_input / esp_output (freebsd/netipsec/xform_esp.c:260-463, 673-961):
//   AAD   = SPI||SN (8 B) or SPI||ESN_hi||SN (12 B, CSP_F_SEPARATE_AAD)
//   nonce = salt(4) || explicit IV(8);  J0 = nonce||1;  CT block c uses nonce||c+2
//   tag   = GHASH_H(AAD, CT, len) ^ E_K(J0), compared on mlen bytes; a mismatch
//           sets EBADMSG and the record's plaintext is not released.
//   ICV   = the last mlen (16, 12 or 8) bytes of the record, so the payload is
//           len - 16 - mlen bytes (cryptosoft.c:1112-1117 honours mlen < 16).
//
// Mapping (MI355X-first, not a translation of the 16-byte-at-a-time loop):
//  * 8 lanes per ESP record, 8 records per wave, 16 waves per workgroup
//    (a 256-record "chunk" of ONE session per workgroup iteration, two passes).
//  * GHASH is reassociated so every lane runs a Horner chain over blocks
//    l, l+8, l+16, ... of its record (front-padded with zero blocks to a
//    multiple of 8, which leaves the hash unchanged), two steps at a time:
//    Y <- Y*H^16 ^ B_m*H^8 ^ B_m+1.  Each lane then multiplies by H^(8-l) and
//    the 8 partials are XOR-reduced across the lane group.  Multiplication by
//    a fixed power is X*H^e = XOR_j T_e[j][nibble_j(X)] with 4-bit tables:
//    a 256-byte position row spans the 64 LDS banks once, so ds_read_b128
//    lookups never bank-conflict (equal nibbles broadcast).  H^8 and H^16
//    live in LDS; the per-lane final H^(8-l) is gathered from L2.
//  * AES-CTR uses the four T-tables Te0..Te3 replicated 32x in LDS (entry x
//    at x*256 of its 64 KiB pair: Te0/Te2 in lane slots (lane&31)*4, Te1/Te3
//    128 bytes later): every lane of a 32-lane ds_read_b32 group hits its own
//    bank whatever the indices, and the address is one v_perm_b32 of
//    (state byte, lane slot).  A column is then two v_bitop3 XORs.
//  * The lane that owns GHASH block i also computes AES(nonce||i+1): block 0
//    (the AAD block) gets J0, CT block c = i-1 gets counter c+2, so the CTR
//    work is aligned with the hash work and plaintext is stored from the same
//    registers that fed GHASH.
//  * LDS throughput is the binding resource (T-table and GHASH lookups; HBM
//    traffic is ~1/3 of its time), so each paired step interleaves the two
//    GHASH products' 64 table reads with the 8+ AES rounds of the two counter
//    blocks, phase by phase: every phase has independent LDS reads from both
//    chains in flight.  Rounds 1-2 of a counter block are cached per 256
//    counters (only the low counter byte changes): 5 lookups instead of 32.
//  * Records and descriptors are read with 16-byte loads, 128 contiguous bytes
//    per lane group per step, one paired step ahead of use.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "espgpu_internal.h"

namespace espgpu {

namespace {

constexpr uint32_t LDS_TA = 0;                       // Te0 | Te1 pairs, 64 KiB
constexpr uint32_t LDS_TB = 65536;                   // Te2 | Te3 pairs, 64 KiB
constexpr uint32_t LDS_H8 = 131072;                  // H^8, 4-bit indices, 8 KiB
constexpr uint32_t LDS_H16 = LDS_H8 + kGhPowerBytes; // H^16, 4-bit indices, 8 KiB
constexpr uint32_t LDS_BYTES = LDS_H16 + kGhPowerBytes;
constexpr int S = 8;                                 // lanes per record
static_assert(LDS_TA == 0 && LDS_TB == 1u << 16 && (LDS_H8 >> 16) == 2, "perm-built LDS addresses");

// Round keys are read through the constant address space: uniform loads from
// it become s_load (SGPRs, scalar cache) instead of vector loads or LDS reads.
typedef const __attribute__((address_space(4))) uint32_t *rkptr;
__device__ __forceinline__ uint4 ldk4(rkptr p) { return make_uint4(p[0], p[1], p[2], p[3]); }

struct __attribute__((aligned(4))) U4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return perm(x, x, 0x00010203u); }

__device__ __forceinline__ uint4 ld16(const uint8_t *p) {
  U4 v = *reinterpret_cast<const U4 *>(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st16(uint8_t *p, uint4 v) {
  U4 u{v.x, v.y, v.z, v.w};
  *reinterpret_cast<U4 *>(p) = u;
}
__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) {
  return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}
__device__ __forceinline__ uint4 zero4() { return make_uint4(0, 0, 0, 0); }
__device__ __forceinline__ uint4 sel4(bool c, uint4 a, uint4 b) {
  return make_uint4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}

// Keep the first `rem` bytes of a 16-byte block, zero the rest.  Valid ESP
// payloads are 4-byte multiples (the kernel rejects len % 4 != 0, as
// esp_output pads to 4, xform_esp.c:710-716), so rem is 4, 8, 12 or >= 16.
__device__ __forceinline__ uint4 mask_block(uint4 v, int rem) {
  return make_uint4(v.x, rem > 4 ? v.y : 0u, rem > 8 ? v.z : 0u, rem > 12 ? v.w : 0u);
}

// Store the first `rem` bytes (a multiple of 4) of v.
__device__ __forceinline__ void st_partial(uint8_t *p, uint4 v, int rem) {
  if (rem >= 16) {
    st16(p, v);
    return;
  }
  uint32_t *q = reinterpret_cast<uint32_t *>(p);
  q[0] = v.x;
  if (rem > 4) q[1] = v.y;
  if (rem > 8) q[2] = v.z;
}

// ---- AES (rijndaelEncrypt, rijndael-alg-fst.c:863-1042) on LDS T-tables -----
// Byte k (0 = LSB) of state word w indexes Te(3-k).  The address is ONE
// v_perm_b32: byte0 = the lane slot (lane&31)*4, byte1 = w.byte k, byte2 =
// the table pair (0: Te0/Te1, 1: Te2/Te3) from `slot`; Te1/Te3 sit 128 bytes
// further (DS immediate offset).
struct Slots {
  uint32_t a, b;   // (lane&31)*4 | pair << 16
};
__device__ __forceinline__ uint32_t tpa(uint32_t w, uint32_t slot, int k) {
  return perm(w, slot, 0x0c020000u | ((4u + (uint32_t)k) << 8));
}
__device__ __forceinline__ uint32_t lds32(const uint8_t *lds, uint32_t a, uint32_t off) {
  return *reinterpret_cast<const uint32_t *>(lds + a + off);
}
__device__ __forceinline__ uint32_t T0(const uint8_t *lds, Slots s, uint32_t w) { return lds32(lds, tpa(w, s.a, 3), 0); }
__device__ __forceinline__ uint32_t T1(const uint8_t *lds, Slots s, uint32_t w) { return lds32(lds, tpa(w, s.a, 2), 128); }
__device__ __forceinline__ uint32_t T2(const uint8_t *lds, Slots s, uint32_t w) { return lds32(lds, tpa(w, s.b, 1), 0); }
__device__ __forceinline__ uint32_t T3(const uint8_t *lds, Slots s, uint32_t w) { return lds32(lds, tpa(w, s.b, 0), 128); }

struct St {
  uint32_t s0, s1, s2, s3;
};

// One middle round on big-endian state words, raw round key k.
__device__ __forceinline__ St aes_round(St s, uint4 k, const uint8_t *lds, Slots sl) {
  const uint32_t a0 = T0(lds, sl, s.s0), b0 = T1(lds, sl, s.s1), c0 = T2(lds, sl, s.s2), d0 = T3(lds, sl, s.s3);
  const uint32_t a1 = T0(lds, sl, s.s1), b1 = T1(lds, sl, s.s2), c1 = T2(lds, sl, s.s3), d1 = T3(lds, sl, s.s0);
  const uint32_t a2 = T0(lds, sl, s.s2), b2 = T1(lds, sl, s.s3), c2 = T2(lds, sl, s.s0), d2 = T3(lds, sl, s.s1);
  const uint32_t a3 = T0(lds, sl, s.s3), b3 = T1(lds, sl, s.s0), c3 = T2(lds, sl, s.s1), d3 = T3(lds, sl, s.s2);
  return St{xor3(xor3(a0, b0, c0), d0, k.x), xor3(xor3(a1, b1, c1), d1, k.y),
            xor3(xor3(a2, b2, c2), d2, k.z), xor3(xor3(a3, b3, c3), d3, k.w)};
}

// Last round: S[x] is byte 1 of Te0[x]; emit little-endian (memory order)
// words directly; the last round key is stored byte-swapped.
__device__ __forceinline__ uint4 aes_last(St s, uint4 k, const uint8_t *lds, Slots sl) {
  const uint32_t ss[4] = {s.s0, s.s1, s.s2, s.s3};
  const uint32_t kk[4] = {k.x, k.y, k.z, k.w};
  uint32_t o[4];
#pragma unroll
  for (int col = 0; col < 4; ++col) {
    const uint32_t a = T0(lds, sl, ss[col]) ;
    const uint32_t b = lds32(lds, tpa(ss[(col + 1) & 3], sl.a, 2), 0);
    const uint32_t c = lds32(lds, tpa(ss[(col + 2) & 3], sl.a, 1), 0);
    const uint32_t d = lds32(lds, tpa(ss[(col + 3) & 3], sl.a, 0), 0);
    o[col] = xor3(perm(b, a, 0x0c0c0501u), perm(d, c, 0x05010c0cu), kk[col]);
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// The same rounds split into "issue" (16 T-table reads) and "combine" (the
// XORs), so the paired step can software-pipeline its two blocks: block b's
// reads are in flight while block a's results are combined, and vice versa.
struct R16 {
  uint32_t v[16];
};
__device__ __forceinline__ R16 issue_round(St s, const uint8_t *lds, Slots sl) {
  R16 r;
  r.v[0] = T0(lds, sl, s.s0); r.v[1] = T1(lds, sl, s.s1); r.v[2] = T2(lds, sl, s.s2); r.v[3] = T3(lds, sl, s.s3);
  r.v[4] = T0(lds, sl, s.s1); r.v[5] = T1(lds, sl, s.s2); r.v[6] = T2(lds, sl, s.s3); r.v[7] = T3(lds, sl, s.s0);
  r.v[8] = T0(lds, sl, s.s2); r.v[9] = T1(lds, sl, s.s3); r.v[10] = T2(lds, sl, s.s0); r.v[11] = T3(lds, sl, s.s1);
  r.v[12] = T0(lds, sl, s.s3); r.v[13] = T1(lds, sl, s.s0); r.v[14] = T2(lds, sl, s.s1); r.v[15] = T3(lds, sl, s.s2);
  return r;
}
__device__ __forceinline__ St combine_round(const R16 &r, uint4 k) {
  return St{xor3(xor3(r.v[0], r.v[1], r.v[2]), r.v[3], k.x), xor3(xor3(r.v[4], r.v[5], r.v[6]), r.v[7], k.y),
            xor3(xor3(r.v[8], r.v[9], r.v[10]), r.v[11], k.z), xor3(xor3(r.v[12], r.v[13], r.v[14]), r.v[15], k.w)};
}
__device__ __forceinline__ R16 issue_last(St s, const uint8_t *lds, Slots sl) {
  const uint32_t ss[4] = {s.s0, s.s1, s.s2, s.s3};
  R16 r;
#pragma unroll
  for (int col = 0; col < 4; ++col) {
    r.v[4 * col] = lds32(lds, tpa(ss[col], sl.a, 3), 0);
    r.v[4 * col + 1] = lds32(lds, tpa(ss[(col + 1) & 3], sl.a, 2), 0);
    r.v[4 * col + 2] = lds32(lds, tpa(ss[(col + 2) & 3], sl.a, 1), 0);
    r.v[4 * col + 3] = lds32(lds, tpa(ss[(col + 3) & 3], sl.a, 0), 0);
  }
  return r;
}
__device__ __forceinline__ uint4 combine_last(const R16 &r, uint4 k) {
  const uint32_t kk[4] = {k.x, k.y, k.z, k.w};
  uint32_t o[4];
#pragma unroll
  for (int col = 0; col < 4; ++col)
    o[col] = xor3(perm(r.v[4 * col + 1], r.v[4 * col], 0x0c0c0501u),
                  perm(r.v[4 * col + 3], r.v[4 * col + 2], 0x05010c0cu), kk[col]);
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// Round keys of the group's session as wave-uniform values (SGPRs): loaded
// once per record group and laundered, so that under SGPR pressure they are
// spilled to VGPR lanes (v_readlane) instead of being re-loaded with s_load
// in the step loop -- an s_load's s_waitcnt lgkmcnt(0) would also drain every
// LDS read in flight.
template <int NR>
struct Keys {
  uint32_t k[4 * (NR + 1)];
  __device__ __forceinline__ uint4 operator[](int r) const {
    return make_uint4(k[4 * r], k[4 * r + 1], k[4 * r + 2], k[4 * r + 3]);
  }
};
template <int NR, bool LAUNDER = true>
__device__ __forceinline__ Keys<NR> load_keys(rkptr rk) {
  Keys<NR> K;
#pragma unroll
  for (int i = 0; i < 4 * (NR + 1); ++i) {
    uint32_t v = rk[i];
    if (LAUNDER) asm volatile("" : "+s"(v));
    K.k[i] = v;
  }
  return K;
}

// ---- counter-mode caching of rounds 1-2 ------------------------------------
// Every counter block of a record is nonce(12 B) || ctr, and within a run of
// 256 counters only ctr's low byte changes.  Entering round 1 that byte is
// s3.b0, which feeds exactly one T-table lookup (column 0, Te3); after round
// 1 only column 0 (t0) varies, and in round 2 each output column has exactly
// one lookup on t0.  So for a fixed nonce and ctr>>8 the other 15 + 12
// lookups are constants: K0 (round 1, column 0 without its Te3 term) and
// L0..L3 (round 2 without their t0 terms): 5 lookups per block for rounds
// 1-2 instead of 32.
struct CtrCache {
  uint32_t K0, L0, L1, L2, L3;
  int hi;
};

// n0..n2: the nonce words XOR round key 0.
template <int NR>
__device__ __forceinline__ void ctr_cache_build(CtrCache &cc, uint32_t n0, uint32_t n1, uint32_t n2, int hi,
                                                const Keys<NR> &K, const uint8_t *lds, Slots sl) {
  // (the nonce words are laundered so the 12 address computations on them are
  // not hoisted out of the step loop into 12 loop-long VGPRs)
  asm volatile("" : "+v"(n0), "+v"(n1), "+v"(n2));
  const uint32_t n3 = ((uint32_t)hi << 8) ^ K.k[3];    // bytes 1..3 valid; byte 0 varies
  const uint4 k1 = K[1], k2 = K[2];
  cc.K0 = xor3(T0(lds, sl, n0), T1(lds, sl, n1), T2(lds, sl, n2)) ^ k1.x;
  const uint32_t t1 = xor3(xor3(T0(lds, sl, n1), T1(lds, sl, n2), T2(lds, sl, n3)), T3(lds, sl, n0), k1.y);
  const uint32_t t2 = xor3(xor3(T0(lds, sl, n2), T1(lds, sl, n3), T2(lds, sl, n0)), T3(lds, sl, n1), k1.z);
  const uint32_t t3 = xor3(xor3(T0(lds, sl, n3), T1(lds, sl, n0), T2(lds, sl, n1)), T3(lds, sl, n2), k1.w);
  cc.L0 = xor3(T1(lds, sl, t1), T2(lds, sl, t2), T3(lds, sl, t3)) ^ k2.x;    // minus Te0[t0.b3]
  cc.L1 = xor3(T0(lds, sl, t1), T1(lds, sl, t2), T2(lds, sl, t3)) ^ k2.y;    // minus Te3[t0.b0]
  cc.L2 = xor3(T0(lds, sl, t2), T1(lds, sl, t3), T3(lds, sl, t1)) ^ k2.z;    // minus Te2[t0.b1]
  cc.L3 = xor3(T0(lds, sl, t3), T2(lds, sl, t1), T3(lds, sl, t2)) ^ k2.w;    // minus Te1[t0.b2]
  cc.hi = hi;
}

// State entering round 3 of E_K(nonce || ctr) from the cache (built for ctr >> 8).
__device__ __forceinline__ St ctr_r12(const CtrCache &cc, uint32_t ctr, uint32_t rk3, const uint8_t *lds, Slots sl) {
  const uint32_t t0 = cc.K0 ^ T3(lds, sl, ctr ^ rk3);
  return St{cc.L0 ^ T0(lds, sl, t0), cc.L1 ^ T3(lds, sl, t0), cc.L2 ^ T2(lds, sl, t0), cc.L3 ^ T1(lds, sl, t0)};
}

// The same without the cache (a counter block in a different 256-run than
// the cache: rare, only where a record's counters cross a multiple of 256).
template <int NR>
__device__ __forceinline__ St ctr_r12_full(uint32_t n0, uint32_t n1, uint32_t n2, uint32_t ctr, const Keys<NR> &K,
                                           const uint8_t *lds, Slots sl) {
  St s{n0, n1, n2, ctr ^ K.k[3]};
  s = aes_round(s, K[1], lds, sl);
  return aes_round(s, K[2], lds, sl);
}

// ---- GHASH: products by fixed powers with 4-bit LDS tables -------------------
// (gf_mul, gfmult.c:219-229).  Table of a power: nibble position j (byte j>>1
// of the block in memory order, low nibble if j even), value n at j*256 + n*16.
// gh_byte<B> folds byte B (word B>>2, byte B&3) of v into acc:
// acc ^= T[2B][lo nibble] ^ T[2B+1][hi nibble].  The nibble lands in address
// bits 4..7 ((w << 4) & F0F0F0F0 for low, w & F0F0F0F0 for high nibbles);
// pb = the table's LDS base (bits 8..23; per lane for the Y product, which
// uses H^16 or H^8 by lane).
__device__ __forceinline__ uint4 lds128(const uint8_t *lds, uint32_t a, uint32_t off) {
  return *reinterpret_cast<const uint4 *>(lds + a + off);
}
__device__ __forceinline__ uint32_t word(uint4 v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }
// Y * H^e with the 4-bit table of that power in global memory (t = its 8 KiB).
// Used once per record per lane (the final x H^(8-l)), where the power differs
// per lane: from LDS that would be bank conflicts, from L2 it is a gather.
__device__ __forceinline__ uint4 gf_mul4_global(uint4 x, const uint8_t *t) {
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0;
  uint32_t w = x.x, w1 = x.y, w2 = x.z, w3 = x.w;
  // two words (16 positions, 4 KiB of table) per iteration: 16 gathers in
  // flight, two L2 round trips per record group, one table pointer
#pragma unroll 2
  for (int k = 0; k < 4; ++k) {
    const uint32_t hi = w & 0xF0F0F0F0u, lo = (w << 4) & 0xF0F0F0F0u;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint4 e = *reinterpret_cast<const uint4 *>(t + (2 * q) * 256 + ((lo >> (8 * q)) & 0xffu));
      const uint4 f = *reinterpret_cast<const uint4 *>(t + (2 * q + 1) * 256 + ((hi >> (8 * q)) & 0xffu));
      r0 = xor3(r0, e.x, f.x);
      r1 = xor3(r1, e.y, f.y);
      r2 = xor3(r2, e.z, f.z);
      r3 = xor3(r3, e.w, f.w);
    }
    w = w1;
    w1 = w2;
    w2 = w3;
    t += 8 * 256;
  }
  return make_uint4(r0, r1, r2, r3);
}

__device__ __forceinline__ uint4 shfl_xor4(uint4 v, int m) {
  return make_uint4(__shfl_xor(v.x, m), __shfl_xor(v.y, m), __shfl_xor(v.z, m), __shfl_xor(v.w, m));
}
__device__ __forceinline__ uint4 shfl4(uint4 v, int src) {
  return make_uint4(__shfl(v.x, src), __shfl(v.y, src), __shfl(v.z, src), __shfl(v.w, src));
}

// ---- the paired step --------------------------------------------------------
// AES rounds 3..NR of the two counter blocks (states a, b entering round 3)
// with the paired step's GHASH products interleaved, as a software pipeline
// of "halves": half h issues the 16 T-table reads of round 3 + h/2 of block
// (h odd ? b : a), then combines the reads the previous half issued for the
// other block, so one block's reads are in flight while the other's are
// XORed.  Half h < 16 also carries GHASH bytes 2h, 2h+1 of one product
// (halves 0..7: Y*T_Y, Y known at step start; halves 8..15: X*H^8, X = this
// step's data block, loaded at step start and first needed half a step
// later), issued first in the half and folded at its end.  Per wave at most
// 32 T-table reads and 4 GHASH rows are in flight (lgkmcnt saturates at 15,
// so a combine waits for all but the 15 youngest reads).
// AES = false: 16 halves of GHASH only; GH = false: AES only.
// GHASH rows of half H: bytes 2h, 2h+1 of the Y product (H < 8) or of the X
// product (8 <= H < 16), two rows per byte.
template <int B>
__device__ __forceinline__ void gh_rows(uint4 &e, uint4 &f, uint4 v, uint32_t pb, const uint8_t *lds) {
  constexpr int K = B >> 2, Q = B & 3;
  const uint32_t w = word(v, K);
  const uint32_t sel = 0x0c060500u | (uint32_t)Q;
  constexpr uint32_t off = (uint32_t)(8 * K + 2 * Q) * 256;
  e = lds128(lds, perm(pb, (w << 4) & 0xF0F0F0F0u, sel), off);
  f = lds128(lds, perm(pb, w & 0xF0F0F0F0u, sel), off + 256);
}
template <int H>
__device__ __forceinline__ void gh_issue(uint4 &g0, uint4 &g1, uint4 &g2, uint4 &g3, uint4 Y, uint32_t pY,
                                         uint4 X, const uint8_t *lds) {
  if constexpr (H < 8) {
    gh_rows<2 * H>(g0, g1, Y, pY, lds);
    gh_rows<2 * H + 1>(g2, g3, Y, pY, lds);
  } else {
    gh_rows<2 * (H - 8)>(g0, g1, X, LDS_H8, lds);
    gh_rows<2 * (H - 8) + 1>(g2, g3, X, LDS_H8, lds);
  }
}
__device__ __forceinline__ void gh_fold(uint4 &acc, uint4 g0, uint4 g1, uint4 g2, uint4 g3) {
  acc.x = xor3(acc.x, g0.x, g1.x);
  acc.y = xor3(acc.y, g0.y, g1.y);
  acc.z = xor3(acc.z, g0.z, g1.z);
  acc.w = xor3(acc.w, g0.w, g1.w);
  acc.x = xor3(acc.x, g2.x, g3.x);
  acc.y = xor3(acc.y, g2.y, g3.y);
  acc.z = xor3(acc.z, g2.z, g3.z);
  acc.w = xor3(acc.w, g2.w, g3.w);
  // Materialize the sum here: XOR is associative, and otherwise the chain is
  // re-associated into one tree at the end of the step, keeping all 64 rows
  // (256 VGPRs) live.
  asm volatile("" : "+v"(acc.x), "+v"(acc.y), "+v"(acc.z), "+v"(acc.w));
}
template <int NR, bool AES, bool GH, int H>
__device__ __forceinline__ void halves(St &a, St &b, R16 &ra, R16 &rb, uint4 &ka, uint4 &kb, uint4 &acc,
                                       uint4 Y, uint32_t pY, uint4 X, const Keys<NR> &K, const uint8_t *lds,
                                       Slots sl) {
  constexpr int NH = AES ? 2 * (NR - 2) : 16;   // halves of the step
  if constexpr (H < NH) {
    // GHASH rows first, then the half's T-table reads, then the combines: the
    // GHASH fold waits for its rows but not for the 16 younger T-table reads
    uint4 g0, g1, g2, g3;
    if constexpr (GH && H < 16) gh_issue<H>(g0, g1, g2, g3, Y, pY, X, lds);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (AES) {
      constexpr int r = 3 + H / 2;               // round this half issues
      constexpr bool blk_b = (H & 1) != 0;
      if constexpr (!blk_b) ra = (r < NR) ? issue_round(a, lds, sl) : issue_last(a, lds, sl);
      else rb = (r < NR) ? issue_round(b, lds, sl) : issue_last(b, lds, sl);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (GH && H < 16) gh_fold(acc, g0, g1, g2, g3);
    if constexpr (AES && H > 0) {
      // combine what the previous half issued (the other block)
      constexpr int pr = 3 + (H - 1) / 2;
      constexpr bool blk_b = (H & 1) != 0;
      if constexpr (!blk_b) {
        if constexpr (pr < NR) b = combine_round(rb, K[pr]);
      } else {
        if constexpr (pr < NR) a = combine_round(ra, K[pr]);
        else ka = combine_last(ra, K[NR]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    halves<NR, AES, GH, H + 1>(a, b, ra, rb, ka, kb, acc, Y, pY, X, K, lds, sl);
  } else if constexpr (AES) {
    kb = combine_last(rb, K[NR]);                 // the last half issued b's last round
  }
}
// Alternative schedules of the same work (kernel template SCHED & 3, for A/B):
// 0: halves (above); 1: per AES round both blocks' 32 reads + 8 GHASH rows in
// one region (production); 2: all AES rounds (32 reads per region), then the
// 64 GHASH rows.  All three measured within 3 % of each other on cfg1.
template <int NR, bool AES, bool GH, int P>
__device__ __forceinline__ void rounds_both(St &a, St &b, uint4 &ka, uint4 &kb, uint4 &acc, uint4 Y, uint32_t pY,
                                           uint4 X, const Keys<NR> &K, const uint8_t *lds, Slots sl) {
  constexpr int r = 3 + P;
  if constexpr (AES && r < NR) {
    a = aes_round(a, K[r], lds, sl);
    b = aes_round(b, K[r], lds, sl);
  } else if constexpr (AES && r == NR) {
    ka = aes_last(a, K[NR], lds, sl);
    kb = aes_last(b, K[NR], lds, sl);
  }
  if constexpr (GH && P < 8) {
    uint4 g0, g1, g2, g3;
    gh_issue<2 * P>(g0, g1, g2, g3, Y, pY, X, lds);
    gh_fold(acc, g0, g1, g2, g3);
    gh_issue<2 * P + 1>(g0, g1, g2, g3, Y, pY, X, lds);
    gh_fold(acc, g0, g1, g2, g3);
  }
  __builtin_amdgcn_sched_barrier(0);
  constexpr int last = (AES ? NR - 3 : 7);
  if constexpr (P < last) rounds_both<NR, AES, GH, P + 1>(a, b, ka, kb, acc, Y, pY, X, K, lds, sl);
}
template <int H>
__device__ __forceinline__ void gh_all(uint4 &acc, uint4 Y, uint32_t pY, uint4 X, const uint8_t *lds) {
  uint4 g0, g1, g2, g3;
  gh_issue<H>(g0, g1, g2, g3, Y, pY, X, lds);
  gh_fold(acc, g0, g1, g2, g3);
  if constexpr (H & 1) __builtin_amdgcn_sched_barrier(0);
  if constexpr (H < 15) gh_all<H + 1>(acc, Y, pY, X, lds);
}

template <int NR, bool AES, bool GH, int SCHED>
__device__ __forceinline__ void phases(St &a, St &b, uint4 &ka, uint4 &kb, uint4 &acc, uint4 Y, uint32_t pY,
                                       uint4 X, const Keys<NR> &K, const uint8_t *lds, Slots sl) {
  if constexpr ((SCHED & 3) == 0) {
    R16 ra, rb;
    halves<NR, AES, GH, 0>(a, b, ra, rb, ka, kb, acc, Y, pY, X, K, lds, sl);
  } else if constexpr ((SCHED & 3) == 1) {
    rounds_both<NR, AES, GH, 0>(a, b, ka, kb, acc, Y, pY, X, K, lds, sl);
  } else {
    if constexpr (AES) rounds_both<NR, true, false, 0>(a, b, ka, kb, acc, Y, pY, X, K, lds, sl);
    if constexpr (GH) gh_all<0>(acc, Y, pY, X, lds);
  }
}

// Per-lane record state for one 8-record group of a wave.
struct Rec {
  uint8_t *rec, *orec;
  int valid, ct_len, nct, N, M, pad;
  uint32_t esnh;
  uint32_t n0, n1, n2;      // nonce words ^ rk[0..2]
};

// GHASH block i's data: the ciphertext block (1 <= i <= nct) or the record
// header for the AAD block (i = 0: SPI||SN, masked to 8 bytes); zeros for the
// front padding, the length block (added after the loop) and invalid records.
// The load is exec-masked, not redirected to a shared zero line: every
// wave's padding lanes reading one address made an L2-channel hot spot that
// cost 20 % of the kernel time.
__device__ __forceinline__ uint4 ld_blk(const Rec &r, int i) {
  uint4 v = zero4();
  if (r.valid && i >= 0 && i <= r.nct) v = ld16(r.rec + 16 * i);
  return v;
}
// GHASH input from the loaded block: the partial last CT block is zero-padded,
// the AAD block keeps 8 bytes (SPI||SN) or becomes SPI||ESN_hi||SN (ESN SAs,
// CSP_F_SEPARATE_AAD, xform_esp.c:372-397).
__device__ __forceinline__ uint4 ghash_in(const Rec &r, int i, uint4 C, bool sep) {
  const int rem = i == 0 ? 8 : r.ct_len - 16 * (i - 1);
  if (rem < 16) {
    C = mask_block(C, rem);
    if (sep && i == 0) C = make_uint4(C.x, r.esnh, C.y, 0);
  }
  return C;
}
__device__ __forceinline__ uint4 len_block(const Rec &r, bool sep) {
  return make_uint4(0, bswap32(sep ? 96u : 64u), 0, bswap32((uint32_t)r.ct_len * 8));
}
__device__ __forceinline__ uint32_t trailer_of(uint4 pt, int rem, int ct_len) {
  return esp_trailer_word(rem >= 16 ? pt.w : (rem > 8 ? pt.z : (rem > 4 ? pt.y : pt.x)), (uint32_t)ct_len);
}

// ---- one 8-record group per wave ---------------------------------------------
// MODE 0: decrypt, single pass, plaintext to p.out (out-of-place device staging)
// MODE 1: encrypt in place + ICV
// MODE 2: decrypt in place, verify first (pass 1 GHASH + tag, pass 2 CTR)
template <int MODE, int NR, int SCHED>
__device__ __forceinline__ void do_group(const GcmParams &p, const uint8_t *lds, uint32_t di, bool have,
                                         uint4 dv, uint32_t sa, uint32_t sa_flags, uint32_t mlen, rkptr rk) {
  const int lane = threadIdx.x & 63;
  const int l = lane & (S - 1);
  // (SCHED bit 2, measurement only: Te2/Te3 reads go to the Te0/Te1 pair --
  // wrong results, same instruction stream, to time the LDS placement)
  const Slots sl{(uint32_t)(lane & 31) * 4, ((uint32_t)(lane & 31) * 4) | ((SCHED & 4) ? 0u : 0x10000u)};
  const bool sep = (sa_flags & ESPGPU_CSP_F_SEPARATE_AAD) != 0;

  // -- descriptor and record header ------------------------------------------
  Rec r{};
  r.rec = p.arena;
  uint32_t len = 0;
  if (have) {                                                 // dv: prefetched by the caller
    len = dv.y & 0xffffu;
    r.ct_len = (int)len - 16 - (int)mlen;                     // 8 hdr + 8 IV + ICV
    r.valid = ((dv.y >> 16) == sa) && r.ct_len > 0 && (len & 3) == 0;   // xform_esp.c:279-324
    if (r.valid) {
      r.rec = p.arena + (size_t)dv.x * 4;
      const uint4 h = ld16(r.rec);                            // SPI, SN, explicit IV
      r.esnh = bswap32(dv.z);
      r.nct = (r.ct_len + 15) >> 4;
      r.N = r.nct + 2;
      r.M = (r.N + S - 1) / S;
      r.pad = S * r.M - r.N;
      r.n0 = bswap32(dv.w) ^ rk[0];                          // salt
      r.n1 = bswap32(h.z) ^ rk[1];
      r.n2 = bswap32(h.w) ^ rk[2];
    }
  }
  int Mw = r.M;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) Mw = max(Mw, __shfl_xor(Mw, o));
  if (Mw == 0) {
    if (have && l == 0 && !r.valid) p.status[di] = ESPGPU_EINVAL;
    if (have && l == 0 && MODE != 1 && p.trailer) p.trailer[di] = 0;
    return;
  }
  const int Sw = (Mw + 1) >> 1;                              // paired steps
  const Keys<NR> K = load_keys<NR, !(SCHED & 16)>(rk);
  const uint32_t rk3 = K.k[3];
  r.orec = (MODE == 0 ? p.out - p.arena + r.rec : r.rec);
  CtrCache cc;
  cc.hi = -1;
  uint32_t trl = 0;                                          // fused esp_input_cb trailer word
  const bool want_trl = MODE != 1 && p.trailer != nullptr;

  uint4 Y = zero4(), EJ0 = zero4();

  // rounds 1-2 of the counter blocks of GHASH indices ia, ia+8 (counters
  // ia+1 and ia+9; block ia < 0 is front padding and gets J0's counter)
  auto rounds12 = [&](int ia, St &a, St &b) {
    const uint32_t ca = ia >= 0 ? (uint32_t)ia + 1 : 1u, cb = (uint32_t)ia + 9;
    if ((int)(ca >> 8) != cc.hi) ctr_cache_build(cc, r.n0, r.n1, r.n2, (int)(ca >> 8), K, lds, sl);
    a = ctr_r12(cc, ca, rk3, lds, sl);
    b = ctr_r12(cc, cb, rk3, lds, sl);
    if ((int)(cb >> 8) != cc.hi) b = ctr_r12_full(r.n0, r.n1, r.n2, cb, K, lds, sl);
    __builtin_amdgcn_sched_barrier(0);
  };
  // store the output block of CT index i (1..nct) and note the trailer
  auto put = [&](bool run, uint8_t *base, int i, uint4 v, bool trailer) {
    if (run && i >= 1 && i <= r.nct) {
      const int rem = r.ct_len - 16 * (i - 1);
      st_partial(base + 16 * i, v, rem);
      if (trailer && want_trl && i == r.nct) trl = trailer_of(v, rem, r.ct_len);
    }
  };

  if constexpr (MODE == 0) {
    // ---- single pass: AES and GHASH of the same blocks interleaved ----------
    int ia = l - r.pad;
    constexpr bool PF = (SCHED & 128) != 0;   // next step's blocks in flight during this one
    uint4 Ca = zero4(), Cb = zero4();
    if constexpr (PF) {
      Ca = ld_blk(r, ia);
      Cb = ld_blk(r, ia + 8);
    }
    for (int s = 0; s < Sw; ++s, ia += 16) {
      const int ib = ia + 8;
      uint4 Na = zero4(), Nb = zero4();
      if constexpr (PF) {
        Na = ld_blk(r, ia + 16);
        Nb = ld_blk(r, ib + 16);
      } else {
        Ca = ld_blk(r, ia);
        Cb = ld_blk(r, ib);
      }
      const bool two = 2 * s + 1 < r.M, one = 2 * s < r.M;
      // two: Y*H^16 ^ Ba*H^8 ^ Bb;  one: Y*H^8 ^ Ba (the X product is 0*H^8)
      const uint32_t pY = two ? LDS_H16 : LDS_H8;
      St a, b;
      rounds12(ia, a, b);
      uint4 ka, kb, acc = zero4();
      const uint4 Ba = ghash_in(r, ia, Ca, sep), Bb = ghash_in(r, ib, Cb, sep);
      // (SCHED bits 5/6, measurement only: skip the GHASH / the AES rounds)
      phases<NR, !(SCHED & 64), !(SCHED & 32), SCHED>(a, b, ka, kb, acc, Y, pY, two ? Ba : zero4(), K, lds, sl);
      if (one) Y = xor4(acc, two ? Bb : Ba);
      if (s == 0) EJ0 = sel4(ia == 0, ka, EJ0);
      put(r.valid, r.orec, ia, xor4(Ca, ka), true);
      put(r.valid, r.orec, ib, xor4(Cb, kb), true);
      if constexpr (PF) {
        Ca = Na;
        Cb = Nb;
      }
    }
  } else if constexpr (MODE == 1) {
    // ---- encrypt: the GHASH input is this step's output, so the hash runs
    // one paired step behind the cipher (Ba/Bb/two/one of the previous step)
    uint4 Ba = zero4(), Bb = zero4();
    bool ptwo = false, pone = false;
    int ia = l - r.pad;
    for (int s = 0; s <= Sw; ++s, ia += 16) {
      const int ib = ia + 8;
      const uint32_t pY = ptwo ? LDS_H16 : LDS_H8;
      uint4 acc = zero4();
      const uint4 X = ptwo ? Ba : zero4();
      if (s < Sw) {
        const uint4 Pa = ld_blk(r, ia), Pb = ld_blk(r, ib);
        St a, b;
        rounds12(ia, a, b);
        uint4 ka, kb;
        phases<NR, true, true, SCHED>(a, b, ka, kb, acc, Y, pY, X, K, lds, sl);
        if (pone) Y = xor4(acc, ptwo ? Bb : Ba);
        if (s == 0) EJ0 = sel4(ia == 0, ka, EJ0);
        // output blocks; outside the CT the loaded block passes through (the
        // AAD header for ia == 0, zeros elsewhere)
        const uint4 Oa = sel4(ia >= 1 && ia <= r.nct, xor4(Pa, ka), Pa);
        const uint4 Ob = sel4(ib <= r.nct, xor4(Pb, kb), Pb);
        put(r.valid, r.rec, ia, Oa, false);
        put(r.valid, r.rec, ib, Ob, false);
        Ba = ghash_in(r, ia, Oa, sep);
        Bb = ghash_in(r, ib, Ob, sep);
        ptwo = 2 * s + 1 < r.M;
        pone = 2 * s < r.M;
      } else {
        uint4 ka, kb;
        St a{}, b{};
        phases<NR, false, true, SCHED>(a, b, ka, kb, acc, Y, pY, X, K, lds, sl);
        if (pone) Y = xor4(acc, ptwo ? Bb : Ba);
      }
    }
  } else {
    // ---- MODE 2 pass 1: GHASH over the ciphertext, E_K(J0) ------------------
    {
      ctr_cache_build(cc, r.n0, r.n1, r.n2, 0, K, lds, sl);
      St a = ctr_r12(cc, 1u, rk3, lds, sl), b = a;
      uint4 kb, acc = zero4();
      phases<NR, true, false, SCHED>(a, b, EJ0, kb, acc, Y, LDS_H8, zero4(), K, lds, sl);
    }
    int ia = l - r.pad;
    constexpr bool PF = (SCHED & 128) != 0;   // next step's blocks in flight during this one
    uint4 Ca = zero4(), Cb = zero4();
    if constexpr (PF) {
      Ca = ld_blk(r, ia);
      Cb = ld_blk(r, ia + 8);
    }
    for (int s = 0; s < Sw; ++s, ia += 16) {
      const int ib = ia + 8;
      uint4 Na = zero4(), Nb = zero4();
      if constexpr (PF) {
        Na = ld_blk(r, ia + 16);
        Nb = ld_blk(r, ib + 16);
      } else {
        Ca = ld_blk(r, ia);
        Cb = ld_blk(r, ib);
      }
      const bool two = 2 * s + 1 < r.M, one = 2 * s < r.M;
      const uint32_t pY = two ? LDS_H16 : LDS_H8;
      const uint4 Ba = ghash_in(r, ia, Ca, sep), Bb = ghash_in(r, ib, Cb, sep);
      St a{}, b{};
      uint4 ka, kb, acc = zero4();
      phases<NR, false, true, SCHED>(a, b, ka, kb, acc, Y, pY, two ? Ba : zero4(), K, lds, sl);
      if (one) Y = xor4(acc, two ? Bb : Ba);
      if constexpr (PF) {
        Ca = Na;
        Cb = Nb;
      }
    }
  }
  // the length block is GHASH block N-1, the last block of lane 7: it is
  // added after every multiply, so it can be folded in here
  if (l == S - 1 && r.valid) Y = xor4(Y, len_block(r, sep));

  // the received ICV, loaded before the final multiply's L2 gathers so the
  // two latencies overlap
  uint4 tag = zero4();
  if (MODE != 1 && r.valid) {
    const uint32_t *q = reinterpret_cast<const uint32_t *>(r.rec + len - mlen);
    if (mlen == 16) {
      tag = ld16(r.rec + len - mlen);
    } else {
      tag.x = q[0];
      tag.y = q[1];
      if (mlen > 8) tag.z = q[2];
    }
  }
  // X = sum_l Y_l * H^(8-l)  (power index 7-l)
  uint4 Z = gf_mul4_global(Y, p.gtab + (size_t)sa * kGhTableBytes + (uint32_t)(7 - l) * kGhPowerBytes);
  Z = xor4(Z, shfl_xor4(Z, 1));
  Z = xor4(Z, shfl_xor4(Z, 2));
  Z = xor4(Z, shfl_xor4(Z, 4));
  // E_K(J0) sits in the lane owning GHASH block 0 (lane pad); MODE 2 has it everywhere
  const uint4 ej0 = MODE == 2 ? EJ0 : shfl4(EJ0, (lane & ~(S - 1)) | r.pad);
  const uint4 T = xor4(Z, ej0);

  int ok = 1;
  if (r.valid) {
    const uint32_t icv = len - mlen;
    if (MODE == 1) {
      if (l == 0) st_partial(r.rec + icv, T, (int)mlen);
    } else {
      const uint4 d = mask_block(xor4(T, tag), (int)mlen);
      ok = ((d.x | d.y | d.z | d.w) == 0);
    }
  }
  if constexpr (MODE == 2) {
    // pass 2: CTR decrypt in place, only for authenticated records
    const int run = r.valid && ok;
    int Mr = run ? r.M : 0;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) Mr = max(Mr, __shfl_xor(Mr, o));
    const int Sr = (Mr + 1) >> 1;
    Rec rr = r;
    rr.valid = run;
    int ia = l - r.pad;
    for (int s = 0; s < Sr; ++s, ia += 16) {
      const int ib = ia + 8;
      const uint4 Ca = ld_blk(rr, ia), Cb = ld_blk(rr, ib);
      St a, b;
      rounds12(ia, a, b);
      uint4 ka, kb, acc = zero4();
      phases<NR, true, false, SCHED>(a, b, ka, kb, acc, Y, LDS_H8, zero4(), K, lds, sl);
      put(run, r.rec, ia, xor4(Ca, ka), true);
      put(run, r.rec, ib, xor4(Cb, kb), true);
    }
  }
  if (want_trl) {
    // exactly one lane of the record holds it: OR over the 8 lanes
    trl |= __shfl_xor(trl, 1);
    trl |= __shfl_xor(trl, 2);
    trl |= __shfl_xor(trl, 4);
    if (have && l == 0) p.trailer[di] = (r.valid && ok) ? trl : 0u;
  }
  if (have && l == 0)
    p.status[di] = !r.valid ? ESPGPU_EINVAL : (ok ? ESPGPU_OK : ESPGPU_EBADMSG);
}

// One instantiation per key size (NR = 10/12/14 rounds): the launcher starts
// the NR = 10 kernel always (it also fails invalid-session records) and the
// others only when sessions of that key size exist; each skips the chunks of
// the other key sizes.
template <int MODE, int NR, int WG, int SCHED>
__global__ __launch_bounds__(WG) void gcm_kernel(GcmParams p) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
  __shared__ uint32_t s_ticket[2];
  const int tid = threadIdx.x;

  // T-tables: per entry 32 lane slots of Te0 then 32 of Te1 (pair A), and of
  // Te2 = ror16(Te0), Te3 = ror16(Te1) (pair B), see tpa().
  for (int idx = tid; idx < 256 * 32; idx += WG) {
    const int x = idx >> 5, s = idx & 31;
    const uint2 t = p.tpair[x];
    uint32_t *e = reinterpret_cast<uint32_t *>(lds + x * 256 + s * 4);
    e[0] = t.x;
    e[32] = t.y;
    e[16384] = __builtin_amdgcn_alignbit(t.x, t.x, 16);
    e[16384 + 32] = __builtin_amdgcn_alignbit(t.y, t.y, 16);
  }

  const bool implicit = (p.chunks == nullptr);
  const uint32_t nch = implicit ? (p.n + kChunkRecs - 1) / kChunkRecs : *p.nchunks;
  uint32_t cur_sa = 0xffffffffu, nr = 0, flags = 0, mlen = 16, mode = 0;
  const int wave = tid >> 6;
  // Dynamic chunk queue: chunk costs differ by up to ~300x (64-B vs 9000-B
  // records) and the planner emits the largest first, so grabbing tickets
  // balances the chip where a static split would leave most CUs idle.
  // s_ticket is double-buffered by iteration parity: slot it&1 is rewritten
  // only at it+2, after every thread passed iteration it+1's barrier.
  for (uint32_t it = 0;; ++it) {
    if (tid == 0) s_ticket[it & 1] = atomicAdd(&p.queue[0], 1u);
    __syncthreads();
    const uint32_t c = s_ticket[it & 1];
    if (c >= nch) break;
    uint32_t sa, start, count;
    if (implicit) {
      start = c * kChunkRecs;
      count = min((uint32_t)kChunkRecs, p.n - start);
      sa = p.desc[start].sa;
    } else {
      const Chunk ch = p.chunks[c];
      sa = ch.sa;
      start = ch.start;
      count = ch.count;
    }
    sa = __builtin_amdgcn_readfirstlane(sa);
    if (sa != cur_sa) {
      __syncthreads();
      if (sa < p.nsas) {
        const DevSA *s = p.sas + sa;
        nr = s->nr;
        flags = s->flags;
        mlen = s->mlen;
        mode = s->mode;
        if (mode == ESPGPU_CSP_MODE_AEAD) {
          // H^8 and H^16 4-bit tables: 16 KiB, one 16-byte row per thread
          const uint8_t *tab = p.gtab + (size_t)sa * kGhTableBytes;
          const uint4 *s8 = reinterpret_cast<const uint4 *>(tab + 7 * kGhPowerBytes);
          const uint4 *s16 = reinterpret_cast<const uint4 *>(tab + kGh16Off);
          uint4 *dst = reinterpret_cast<uint4 *>(lds + LDS_H8);
          constexpr int Q = (int)(kGhPowerBytes / 16);
          for (int q = tid; q < 2 * Q; q += WG) dst[q] = q < Q ? s8[q] : s16[q - Q];
        }
      } else {
        mode = 0;
      }
      cur_sa = sa;
      __syncthreads();
    }
    // a chunk takes kChunkRecs / (WG/8) passes of the workgroup; each pass
    // loads the next pass's descriptor ahead (its latency then overlaps the
    // current record group instead of stalling the whole workgroup)
    constexpr uint32_t kPass = (uint32_t)(WG / 64) * S;
    const uint32_t lrec = (uint32_t)wave * S + ((tid & 63) >> 3);
    auto desc_of = [&](uint32_t sub, uint32_t &di, bool &have, uint4 &dv) {
      const uint32_t rl = sub + lrec;
      have = rl < count;
      const uint32_t pos = start + (have ? rl : 0);
      di = p.order ? p.order[pos] : pos;
      dv = have ? *reinterpret_cast<const uint4 *>(p.desc + di) : zero4();
    };
    uint32_t ndi;
    bool nhave;
    uint4 ndv;
    desc_of(0, ndi, nhave, ndv);
    for (uint32_t sub = 0; sub < count; sub += kPass) {
      const uint32_t di = ndi;
      const bool have = nhave;
      const uint4 dv = ndv;
      if (sub + kPass < count) desc_of(sub + kPass, ndi, nhave, ndv);
      // Session check per record: a chunk is one session (planner), but a
      // caller-grouped batch (implicit chunks) is trusted only this far: a
      // record whose own session is not this chunk's AEAD session is EINVAL
      // here unless it is an ETA record, which the ETA kernel owns.
      if (mode == ESPGPU_CSP_MODE_AEAD && nr != NR) break;       // another kernel's chunk
      if (mode != ESPGPU_CSP_MODE_AEAD) {
        if (NR == 10 && have && (tid & 7) == 0) {
          const uint32_t rsa = p.desc[di].sa;
          const bool eta = rsa < p.nsas && p.sas[rsa].mode == ESPGPU_CSP_MODE_ETA;
          if (!eta) {
            p.status[di] = ESPGPU_EINVAL;
            if (MODE != 1 && p.trailer) p.trailer[di] = 0;
          }
        }
        continue;
      }
      do_group<MODE, NR, SCHED>(p, lds, di, have, dv, sa, flags, mlen, (rkptr)(const void *)(p.sas[sa].rk));
    }
  }
  // Every workgroup leaves the loop after drawing exactly one ticket >= nch,
  // so once all have retired no ticket is drawn again: reset for the next launch.
  if (tid == 0 && atomicAdd(&p.queue[1], 1u) == gridDim.x - 1) {
    atomicExch(&p.queue[0], 0u);
    atomicExch(&p.queue[1], 0u);
  }
}

}  // namespace

// Production schedule: per AES round both blocks' reads + 8 GHASH rows in
// one region (SCHED 1), the next step's data in flight (bit 7).  Measured
// against the alternatives on cfg1 (tools/gcm_timing.py).
constexpr int kSched = 1 | 128;

template <int NR, int SCHED>
static void launch_nr(const GcmParams &p, int encrypt, int two_pass, int grid, hipStream_t st) {
  if (encrypt)
    hipLaunchKernelGGL((gcm_kernel<1, NR, 1024, SCHED>), dim3(grid), dim3(1024), 0, st, p);
  else if (two_pass)
    hipLaunchKernelGGL((gcm_kernel<2, NR, 1024, SCHED>), dim3(grid), dim3(1024), 0, st, p);
  else
    hipLaunchKernelGGL((gcm_kernel<0, NR, 1024, SCHED>), dim3(grid), dim3(1024), 0, st, p);
}

int launch_gcm(const GcmParams &p, int encrypt, int two_pass, int grid, uint32_t nr_mask, int sched,
               void *stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (grid <= 0) grid = 256;
#ifdef ESPGPU_KNOBS
  // measurement-only variants (make KNOBS=1; tools/gcm_timing.py): AES-128
  // decrypt out of place.  SCHED bits: 0-1 schedule (0 pipelined halves, 1
  // per-round regions, 2 AES then GHASH), 2 Te2/Te3 reads on the Te0/Te1
  // pair (wrong results), 4 keys re-loadable, 5 skip GHASH, 6 skip AES
  // rounds 3+, 7 prefetch.
  if (sched > 0 && !encrypt && !two_pass) {
#define KNOB(V) \
  case V: hipLaunchKernelGGL((gcm_kernel<0, 10, 1024, V>), dim3(grid), dim3(1024), 0, st, p); break;
    switch (sched) {
      KNOB(1) KNOB(2) KNOB(128) KNOB(130) KNOB(133) KNOB(145) KNOB(161) KNOB(193) KNOB(224)
      default: return -1;
    }
#undef KNOB
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
#else
  (void)sched;
#endif
  launch_nr<10, kSched>(p, encrypt, two_pass, grid, st);
  if (nr_mask & 2) launch_nr<12, kSched>(p, encrypt, two_pass, grid, st);
  if (nr_mask & 4) launch_nr<14, kSched>(p, encrypt, two_pass, grid, st);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace espgpu
