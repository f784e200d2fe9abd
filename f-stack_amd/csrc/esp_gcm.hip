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
//  * S = kGcmLanesPerRec = 4 lanes per ESP record, 16 records per wave, 16
//    waves per workgroup, one workgroup per CU (128 KiB LDS); workgroups take
//    256-record chunks of ONE session from a ticket counter.  Batches below
//    kGcmSmallBatch records run with S = kGcmLanesSmall = 8 (half the serial
//    steps per record) in smaller chunks spread over the CUs (launch_gcm).
//  * GHASH is reassociated so every lane runs a Horner chain with the SAME
//    multiplier H^S over blocks l, l+S, l+2S, ... of its record (the block
//    list is front-padded with zero blocks to a multiple of S, which leaves
//    the hash unchanged), then multiplies by H^(S-l) and the S partials are
//    XOR-reduced across the lane group.  Multiplication by a fixed H^e uses
//    tables indexed per byte or nibble POSITION, so there is no shift/reduce
//    step: X*H^e = XOR_j T_e[j][digit_j(X)].  The Horner multiplier H^S is in
//    LDS with 8-bit indices (16 ds_read_b128 per block, value-major and read
//    in a lane-dependent position order, so conflict-free: gf_mul8); the
//    per-lane final H^(S-l) is gathered from L2 (4-bit tables).
//  * AES-CTR uses T-tables Te0 and Te1 replicated 32x in LDS (entry x at x*256:
//    Te0 in lane slots (lane&31)*4, Te1 128 bytes later): ds_read_b32 with every
//    lane of a 32-lane group on its own bank -> conflict-free; the LDS address
//    is a single v_perm_b32 of (state byte, lane slot).  Te2/Te3 are folded
//    through one ror16 per column: t = Te0[a]^Te1[b]^ror16(Te0[c]^Te1[d]^ror16(rk)).
//    Rounds 1-2 come from a per-lane cache keyed on ctr>>8 (counter mode only
//    changes the low byte inside 256 blocks).
//  * The lane that owns GHASH block i also computes AES(nonce||i+1): block 0
//    (the AAD block) gets J0, CT block c = i-1 gets counter c+2, so the CTR
//    work is aligned with the hash work and plaintext is stored from the same
//    registers that fed GHASH.  Steps run in pairs (blocks i and i+S: two
//    independent AES states per lane, GHASH (Y*H^S ^ Ba)*H^S ^ Bb).
//  * Records are read and written with single 16-byte vector accesses, 128
//    contiguous bytes per record per paired step.  HBM traffic per record =
//    record + descriptor + plaintext + status byte.
//  * In place (d_out == d_arena, the opencrypto contract) the same single
//    pass decrypts over the ciphertext it hashes (MODE 3); a record whose tag
//    fails gets the same keystream XORed over it once more, which restores its
//    ciphertext exactly (cryptosoft.c:595-633 never decrypts such a record).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "espgpu_internal.h"
#include "xfer_copy.h"

namespace espgpu {

namespace {
constexpr int kGcmInPlaceMode = 3;     // do_group MODE of an in-place decrypt (one pass, verify-first)

// LDS: the 8-bit H^S GHASH table at 0 (value-major, gf_mul8), the AES
// T-table at 64 KiB.
constexpr uint32_t LDS_GT = 0;          // H^S, 256 values x 16 positions x 16 B
constexpr uint32_t LDS_TP = 65536;      // 256 entries x 32 lane slots x 8 B
constexpr uint32_t LDS_BYTES = LDS_TP + 65536;
// then the staging scratch of a session change (stage_h8_lds): one 4-bit power table
constexpr uint32_t LDS_ALL = LDS_BYTES + kGhPowerBytes;

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
__device__ __forceinline__ uint32_t ror16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return perm(x, x, 0x00010203u); }

// 16- and 8-byte accesses at 4-byte alignment as single vector memory
// operations (one IR access each, so the backend never splits or re-merges them)
typedef uint32_t V4a __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t V2a __attribute__((ext_vector_type(2), aligned(4)));
// (nontemporal hints on these measured 4-14 % slower: DESIGN.md §6)
__device__ __forceinline__ uint4 ld16(const uint8_t *p) {
  const V4a v = *reinterpret_cast<const V4a *>(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st16(uint8_t *p, uint4 v) {
  V4a u = {v.x, v.y, v.z, v.w};
  *reinterpret_cast<V4a *>(p) = u;
}
__device__ __forceinline__ void st8(uint8_t *p, uint32_t a, uint32_t b) {
  V2a u = {a, b};
  *reinterpret_cast<V2a *>(p) = u;
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
  // the last block of a record: 4, 8 or 12 bytes, no store shared with the
  // full-block path (a common first-word store would be hoisted out of both
  // branches and split every full block into three stores)
  if (rem > 4)
    st8(p, v.x, v.y);
  else
    *reinterpret_cast<uint32_t *>(p) = v.x;
  if (rem > 8) *reinterpret_cast<uint32_t *>(p + 8) = v.z;
}

// ---- AES (rijndaelEncrypt, rijndael-alg-fst.c:863-1042) on the pair table ----

// T-table layout (64 KiB at LDS_TP): entry x occupies 256 bytes = Te0[x]
// replicated in 32 lane slots (bytes 0..127) followed by Te1[x] =
// ror8(Te0[x]) in 32 slots (bytes 128..255).  Lane L reads slot L&31, so for
// ds_read_b32 (32 banks, bank = dword index mod 32, 32-lane groups) every lane
// of a group hits its own bank whatever the indices: conflict-free.  The
// address of Te0[byte k of w] for this lane is ONE v_perm_b32: byte0 =
// (L&31)*4 and byte2 = LDS_TP>>16 from `slot`, byte1 = w.byte k; Te1 is the
// same address + 128 (DS immediate offset).
__device__ __forceinline__ uint32_t tpa(uint32_t w, uint32_t slot, int k) {
  return perm(w, slot, 0x0c020000u | ((4u + (uint32_t)k) << 8));
}
__device__ __forceinline__ uint32_t te0(const uint8_t *lds, uint32_t a) {
  return *reinterpret_cast<const uint32_t *>(lds + a);
}
__device__ __forceinline__ uint32_t te1(const uint8_t *lds, uint32_t a) {
  return *reinterpret_cast<const uint32_t *>(lds + a + 128);
}

// One middle round on big-endian state words; k = ror16(round key) (kernel form).
// W (lone-wave kernels): a scheduling barrier between the 16 lookups and the
// XORs, so every lookup is issued before the wave waits on the first; the
// throughput kernels leave the interleaving (fewer live registers) to the
// compiler and hide the latency with other waves.
template <bool W = false>
__device__ __forceinline__ void aes_round(uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &s3, uint4 k,
                                          const uint8_t *lds, uint32_t slot) {
  // column c: Te0[s_c.b3] ^ Te1[s_c+1.b2] ^ ror16(Te0[s_c+2.b1] ^ Te1[s_c+3.b0] ^ ror16(rk))
  const uint32_t a0 = te0(lds, tpa(s0, slot, 3)), b0 = te1(lds, tpa(s1, slot, 2));
  const uint32_t c0 = te0(lds, tpa(s2, slot, 1)), d0 = te1(lds, tpa(s3, slot, 0));
  const uint32_t a1 = te0(lds, tpa(s1, slot, 3)), b1 = te1(lds, tpa(s2, slot, 2));
  const uint32_t c1 = te0(lds, tpa(s3, slot, 1)), d1 = te1(lds, tpa(s0, slot, 0));
  const uint32_t a2 = te0(lds, tpa(s2, slot, 3)), b2 = te1(lds, tpa(s3, slot, 2));
  const uint32_t c2 = te0(lds, tpa(s0, slot, 1)), d2 = te1(lds, tpa(s1, slot, 0));
  const uint32_t a3 = te0(lds, tpa(s3, slot, 3)), b3 = te1(lds, tpa(s0, slot, 2));
  const uint32_t c3 = te0(lds, tpa(s1, slot, 1)), d3 = te1(lds, tpa(s2, slot, 0));
  if (W) __builtin_amdgcn_sched_barrier(0);
  s0 = xor3(a0, b0, ror16(xor3(c0, d0, k.x)));
  s1 = xor3(a1, b1, ror16(xor3(c1, d1, k.y)));
  s2 = xor3(a2, b2, ror16(xor3(c2, d2, k.z)));
  s3 = xor3(a3, b3, ror16(xor3(c3, d3, k.w)));
}

// Measurement knobs, compiled in only by `make knobs` (libespgpu_knobs.so;
// tools/gcm_timing.py --opts, bench.py --tuning gcm_opts=N): bit0 skips the
// record loads and plaintext stores, bit1 the GHASH multiplies, bit2 the AES
// rounds after round 2, bit3 the stores only, bit4 the loads only, bit5 the
// per-session GHASH table staging, bit6 the per-record final multiply, bit7
// takes every tag as matching (so that MODE 3 runs no rollback while the other
// bits break the tags).  They break results on purpose, to split the kernel's
// time between memory, GHASH, AES and per-session setup.
#ifdef ESPGPU_KNOBS
__device__ uint32_t g_opts;
__device__ __forceinline__ uint32_t gopts() {
  return *(const __attribute__((address_space(4))) uint32_t *)(const void *)&g_opts;
}
// Phase clock of the small-batch kernel (knobs build only): workgroup 0's
// thread 0 records (shader clock, 100 MHz real-time clock) at each phase
// boundary of its first chunk; read with espgpu_debug_phases().
__device__ uint64_t g_phase[32];
#define GCM_PHASE_T(i, first, thr)                                          \
  do {                                                                     \
    if (S == kGcmLanesSmall && blockIdx.x == 0 && threadIdx.x == (thr) && (first)) { \
      g_phase[2 * (i)] = __builtin_readcyclecounter();                     \
      g_phase[2 * (i) + 1] = __builtin_amdgcn_s_memrealtime();             \
    }                                                                      \
  } while (0)
#define GCM_PHASE(i, first) GCM_PHASE_T(i, first, 0)
#else
__device__ __forceinline__ constexpr uint32_t gopts() { return 0; }
#define GCM_PHASE(i, first) do {} while (0)
#define GCM_PHASE_T(i, first, thr) do {} while (0)
#endif

// Last round: S[x] is byte 1 of Te0[x]; emit little-endian (memory order)
// words directly; the last round key is stored byte-swapped.
template <bool W = false>
__device__ __forceinline__ uint4 aes_last(uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3, uint4 k,
                                          const uint8_t *lds, uint32_t slot) {
  uint32_t o[4], a[4], b[4], c[4], d[4];
  const uint32_t ss[4] = {s0, s1, s2, s3};
  const uint32_t kk[4] = {k.x, k.y, k.z, k.w};
#pragma unroll
  for (int col = 0; col < 4; ++col) {
    a[col] = te0(lds, tpa(ss[col], slot, 3));
    b[col] = te0(lds, tpa(ss[(col + 1) & 3], slot, 2));
    c[col] = te0(lds, tpa(ss[(col + 2) & 3], slot, 1));
    d[col] = te0(lds, tpa(ss[(col + 3) & 3], slot, 0));
  }
  if (W) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int col = 0; col < 4; ++col)
    o[col] = xor3(perm(b[col], a[col], 0x0c0c0501u), perm(d[col], c[col], 0x05010c0cu), kk[col]);
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// Rounds r0..nr-1 (middle) and the last round.  s* = state entering round r0.
template <bool W = false>
__device__ __forceinline__ uint4 aes_rounds(uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3, int r0,
                                            int nr, rkptr rk, const uint8_t *lds,
                                            uint32_t slot) {
  // nr and rk are wave-uniform (one session per chunk): one loop body serves
  // AES-128/192/256, and the round keys come in through scalar loads (SGPRs),
  // not LDS, which is the bottleneck resource.
#pragma unroll 1
  for (int r = r0; r < nr; ++r) {
    aes_round<W>(s0, s1, s2, s3, ldk4(rk + 4 * r), lds, slot);
    __builtin_amdgcn_sched_barrier(0);
  }
  return aes_last<W>(s0, s1, s2, s3, ldk4(rk + 4 * nr), lds, slot);
}

// ---- counter-mode caching of rounds 1-2 ------------------------------------
// Every counter block of a record is nonce(12 B) || ctr, and within a run of
// 256 counters only ctr's low byte changes.  Entering round 1 that byte is
// s3.b0, which feeds exactly one T-table lookup (column 0); after round 1 only
// column 0 (t0) varies, and in round 2 each output column has exactly one
// lookup on t0.  So for a fixed nonce and ctr>>8 the other 15 + 12 lookups are
// constants: K0 (round 1, column 0 without its s3.b0 term) and L0..L3 (round 2
// without their t0 terms).  Per block this leaves 1 + 4 lookups for rounds 1-2
// instead of 32 (the whole AES-128 block: 133 LDS lookups instead of 160).
struct CtrCache {
  uint32_t K0, L0, L1, L2, L3;
  int hi;
};

__device__ __forceinline__ void ctr_cache_build(CtrCache &cc, uint32_t s0, uint32_t s1, uint32_t s2,
                                                int hi, rkptr rk, const uint8_t *lds,
                                                uint32_t slot) {
  const uint32_t s3 = ((uint32_t)hi << 8) ^ rk[3];   // bytes 1..3 valid; byte 0 varies
  const uint4 k1 = ldk4(rk + 4);
  const uint4 k2 = ldk4(rk + 8);
  // round 1 (k1 = ror16(rk[4..7]))
  cc.K0 = xor3(te0(lds, tpa(s0, slot, 3)), te1(lds, tpa(s1, slot, 2)),
               ror16(te0(lds, tpa(s2, slot, 1)) ^ k1.x));
  const uint32_t t1 = xor3(te0(lds, tpa(s1, slot, 3)), te1(lds, tpa(s2, slot, 2)),
                           ror16(xor3(te0(lds, tpa(s3, slot, 1)), te1(lds, tpa(s0, slot, 0)), k1.y)));
  const uint32_t t2 = xor3(te0(lds, tpa(s2, slot, 3)), te1(lds, tpa(s3, slot, 2)),
                           ror16(xor3(te0(lds, tpa(s0, slot, 1)), te1(lds, tpa(s1, slot, 0)), k1.z)));
  const uint32_t t3 = xor3(te0(lds, tpa(s3, slot, 3)), te1(lds, tpa(s0, slot, 2)),
                           ror16(xor3(te0(lds, tpa(s1, slot, 1)), te1(lds, tpa(s2, slot, 0)), k1.w)));
  __builtin_amdgcn_sched_barrier(0);
  // round 2, each column without its t0 lookup
  cc.L0 = te1(lds, tpa(t1, slot, 2)) ^ ror16(xor3(te0(lds, tpa(t2, slot, 1)), te1(lds, tpa(t3, slot, 0)), k2.x));
  cc.L1 = xor3(te0(lds, tpa(t1, slot, 3)), te1(lds, tpa(t2, slot, 2)),
               ror16(te0(lds, tpa(t3, slot, 1)) ^ k2.y));
  cc.L2 = xor3(te0(lds, tpa(t2, slot, 3)), te1(lds, tpa(t3, slot, 2)),
               ror16(te1(lds, tpa(t1, slot, 0)) ^ k2.z));
  cc.L3 = te0(lds, tpa(t3, slot, 3)) ^ ror16(xor3(te0(lds, tpa(t1, slot, 1)), te1(lds, tpa(t2, slot, 0)), k2.w));
  cc.hi = hi;
}

// E_K(nonce || ctr) using the cache (which must be built for ctr >> 8).
template <bool W = false>
__device__ __forceinline__ uint4 aes_ctr(const CtrCache &cc, uint32_t ctr, uint32_t rk3, int nr,
                                         rkptr rk, const uint8_t *lds, uint32_t slot) {
  const uint32_t t0 = cc.K0 ^ ror16(te1(lds, tpa(ctr ^ rk3, slot, 0)));
  const uint32_t v0 = cc.L0 ^ te0(lds, tpa(t0, slot, 3));
  const uint32_t v1 = cc.L1 ^ ror16(te1(lds, tpa(t0, slot, 0)));
  const uint32_t v2 = cc.L2 ^ ror16(te0(lds, tpa(t0, slot, 1)));
  const uint32_t v3 = cc.L3 ^ te1(lds, tpa(t0, slot, 2));
  return aes_rounds<W>(v0, v1, v2, v3, 3, nr, rk, lds, slot);
}

// Two blocks' round with all 32 lookups issued before the XORs (lone wave).
__device__ __forceinline__ void aes_round2w(uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &s3, uint32_t &u0,
                                            uint32_t &u1, uint32_t &u2, uint32_t &u3, uint4 k,
                                            const uint8_t *lds, uint32_t slot) {
  const uint32_t ss[4] = {s0, s1, s2, s3}, uu[4] = {u0, u1, u2, u3};
  uint32_t a[4], b[4], c[4], d[4], e[4], f[4], g[4], h[4];
#pragma unroll
  for (int col = 0; col < 4; ++col) {
    a[col] = te0(lds, tpa(ss[col], slot, 3));
    b[col] = te1(lds, tpa(ss[(col + 1) & 3], slot, 2));
    c[col] = te0(lds, tpa(ss[(col + 2) & 3], slot, 1));
    d[col] = te1(lds, tpa(ss[(col + 3) & 3], slot, 0));
    e[col] = te0(lds, tpa(uu[col], slot, 3));
    f[col] = te1(lds, tpa(uu[(col + 1) & 3], slot, 2));
    g[col] = te0(lds, tpa(uu[(col + 2) & 3], slot, 1));
    h[col] = te1(lds, tpa(uu[(col + 3) & 3], slot, 0));
  }
  __builtin_amdgcn_sched_barrier(0);
  const uint32_t kk[4] = {k.x, k.y, k.z, k.w};
  uint32_t o[4], q[4];
#pragma unroll
  for (int col = 0; col < 4; ++col) {
    o[col] = xor3(a[col], b[col], ror16(xor3(c[col], d[col], kk[col])));
    q[col] = xor3(e[col], f[col], ror16(xor3(g[col], h[col], kk[col])));
  }
  s0 = o[0], s1 = o[1], s2 = o[2], s3 = o[3];
  u0 = q[0], u1 = q[1], u2 = q[2], u3 = q[3];
}

__device__ __forceinline__ void aes_last2w(uint32_t s0, uint32_t s1, uint32_t s2, uint32_t s3, uint32_t u0,
                                           uint32_t u1, uint32_t u2, uint32_t u3, uint4 k, const uint8_t *lds,
                                           uint32_t slot, uint4 &ka, uint4 &kb) {
  const uint32_t ss[4] = {s0, s1, s2, s3}, uu[4] = {u0, u1, u2, u3};
  const uint32_t kk[4] = {k.x, k.y, k.z, k.w};
  uint32_t a[4], b[4], c[4], d[4], e[4], f[4], g[4], h[4];
#pragma unroll
  for (int col = 0; col < 4; ++col) {
    a[col] = te0(lds, tpa(ss[col], slot, 3));
    b[col] = te0(lds, tpa(ss[(col + 1) & 3], slot, 2));
    c[col] = te0(lds, tpa(ss[(col + 2) & 3], slot, 1));
    d[col] = te0(lds, tpa(ss[(col + 3) & 3], slot, 0));
    e[col] = te0(lds, tpa(uu[col], slot, 3));
    f[col] = te0(lds, tpa(uu[(col + 1) & 3], slot, 2));
    g[col] = te0(lds, tpa(uu[(col + 2) & 3], slot, 1));
    h[col] = te0(lds, tpa(uu[(col + 3) & 3], slot, 0));
  }
  __builtin_amdgcn_sched_barrier(0);
  uint32_t o[4], q[4];
#pragma unroll
  for (int col = 0; col < 4; ++col) {
    o[col] = xor3(perm(b[col], a[col], 0x0c0c0501u), perm(d[col], c[col], 0x05010c0cu), kk[col]);
    q[col] = xor3(perm(f[col], e[col], 0x0c0c0501u), perm(h[col], g[col], 0x05010c0cu), kk[col]);
  }
  ka = make_uint4(o[0], o[1], o[2], o[3]);
  kb = make_uint4(q[0], q[1], q[2], q[3]);
}

// Two counter blocks (both covered by the cache) interleaved round by round:
// each round issues 32 independent LDS lookups before the wave waits, halving
// the dependent LDS round trips per block.
template <bool W = false>
__device__ __forceinline__ void aes_ctr2(const CtrCache &cc, uint32_t ca, uint32_t cb, uint32_t rk3,
                                         int nr, rkptr rk, const uint8_t *lds, uint32_t slot, uint4 &ka,
                                         uint4 &kb) {
  const uint32_t ta = cc.K0 ^ ror16(te1(lds, tpa(ca ^ rk3, slot, 0)));
  const uint32_t tb = cc.K0 ^ ror16(te1(lds, tpa(cb ^ rk3, slot, 0)));
  uint32_t a0 = cc.L0 ^ te0(lds, tpa(ta, slot, 3)), b0 = cc.L0 ^ te0(lds, tpa(tb, slot, 3));
  uint32_t a1 = cc.L1 ^ ror16(te1(lds, tpa(ta, slot, 0))), b1 = cc.L1 ^ ror16(te1(lds, tpa(tb, slot, 0)));
  uint32_t a2 = cc.L2 ^ ror16(te0(lds, tpa(ta, slot, 1))), b2 = cc.L2 ^ ror16(te0(lds, tpa(tb, slot, 1)));
  uint32_t a3 = cc.L3 ^ te1(lds, tpa(ta, slot, 2)), b3 = cc.L3 ^ te1(lds, tpa(tb, slot, 2));
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll 1
  for (int r = 3; r < ((gopts() & 4) ? 3 : nr); ++r) {
    const uint4 k = ldk4(rk + 4 * r);
    if (W) {
      aes_round2w(a0, a1, a2, a3, b0, b1, b2, b3, k, lds, slot);
    } else {
      aes_round(a0, a1, a2, a3, k, lds, slot);
      aes_round(b0, b1, b2, b3, k, lds, slot);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  const uint4 kl = ldk4(rk + 4 * nr);
  if (W) {
    aes_last2w(a0, a1, a2, a3, b0, b1, b2, b3, kl, lds, slot, ka, kb);
  } else {
    ka = aes_last(a0, a1, a2, a3, kl, lds, slot);
    kb = aes_last(b0, b1, b2, b3, kl, lds, slot);
  }
}

// ---- GHASH multiply by a fixed power (gf_mul, gfmult.c:219-229) ----------
// Y * H^S with 8-bit tables in LDS: 16 lookups, one per byte position p, of the
// 16-byte product (the block whose byte p is v) * H^S, XOR-accumulated.
//
// Bank-conflict-free by construction.  A ds_read_b128 is serviced in four
// 16-lane groups ({0-3,12-15,20-27}, {4-11,16-19,28-31} and the same +32) and
// its bank quad is address bits 4..7.  The table is value-major, entry (v, p)
// at v*256 + p*16 (host_crypto.cpp ghash_tables), and in lookup t lane L reads
// position p = t ^ (L & 15): the 16 lanes of every group have distinct L & 15,
// so they hit 16 distinct quads whatever their data (a position-major table
// puts entry v on quad v mod 16: random bytes made 2-4-way conflicts, a quarter
// of all LDS cycles).  Each lane walks its positions in its own order: its Y
// words are permuted by (L >> 2) & 3 and the bytes inside each word by L & 3,
// then each address is one v_perm of (value byte, position << 4).
struct GhLane {
  uint32_t selb;      // v_perm selector: byte b <- byte b ^ (L & 3)
  uint32_t cpos0;     // byte b: (b ^ (L & 15)) << 4 (positions 0..3 of word 0)
  bool sw1, sw2;      // lane bits 2 and 3: the word permutation
};

__device__ __forceinline__ GhLane gh_lane(int lane) {
  GhLane g;
  const uint32_t jl = (uint32_t)lane & 3u, jj = (uint32_t)lane & 15u;
  g.selb = (0u ^ jl) | ((1u ^ jl) << 8) | ((2u ^ jl) << 16) | ((3u ^ jl) << 24);
  g.cpos0 = ((0u ^ jj) << 4) | (((1u ^ jj) << 4) << 8) | (((2u ^ jj) << 4) << 16) | (((3u ^ jj) << 4) << 24);
  g.sw1 = (lane & 4) != 0;
  g.sw2 = (lane & 8) != 0;
  return g;
}

__device__ __forceinline__ uint4 gf_mul8(uint4 x, const uint8_t *lds, const GhLane &g) {
  // slot k <- word k ^ ((L >> 2) & 3)
  const uint32_t a0 = g.sw1 ? x.y : x.x, a1 = g.sw1 ? x.x : x.y;
  const uint32_t a2 = g.sw1 ? x.w : x.z, a3 = g.sw1 ? x.z : x.w;
  const uint32_t w[4] = {g.sw2 ? a2 : a0, g.sw2 ? a3 : a1, g.sw2 ? a0 : a2, g.sw2 ? a1 : a3};
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    // byte b of c = byte b ^ (L & 3) of slot k: position p = (4k + b) ^ (L & 15)
    const uint32_t c = perm(w[k], w[k], g.selb);
    const uint32_t cp = g.cpos0 ^ ((uint32_t)k * 0x40404040u);    // p << 4, bytes 0..3
#pragma unroll
    for (int b = 0; b < 4; b += 2) {
      const uint32_t ea = perm(c, cp, 0x0c0c0000u | ((4u + b) << 8) | (uint32_t)b);
      const uint32_t eb = perm(c, cp, 0x0c0c0000u | ((5u + b) << 8) | (uint32_t)(b + 1));
      const uint4 e = *reinterpret_cast<const uint4 *>(lds + LDS_GT + ea);
      const uint4 f = *reinterpret_cast<const uint4 *>(lds + LDS_GT + eb);
      r0 = xor3(r0, e.x, f.x);
      r1 = xor3(r1, e.y, f.y);
      r2 = xor3(r2, e.z, f.z);
      r3 = xor3(r3, e.w, f.w);
    }
    // Materialize the partial sums here: otherwise the XORs sink into the
    // caller's `if (m < M)` and all 16 rows (64 VGPRs) stay live -> spills.
    asm volatile("" : "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3));
  }
  return make_uint4(r0, r1, r2, r3);
}

// gf_mul8 for a lone wave (burst kernel, 256 VGPRs): all 16 lookups are
// issued before any XOR (a scheduling barrier keeps them together), so the
// multiply waits one LDS latency instead of the eight the register-lean form
// above serializes (each pair's XOR frees its registers for the next pair).
__device__ __forceinline__ uint4 gf_mul8_wide(uint4 x, const uint8_t *lds, const GhLane &g) {
  const uint32_t a0 = g.sw1 ? x.y : x.x, a1 = g.sw1 ? x.x : x.y;
  const uint32_t a2 = g.sw1 ? x.w : x.z, a3 = g.sw1 ? x.z : x.w;
  const uint32_t w[4] = {g.sw2 ? a2 : a0, g.sw2 ? a3 : a1, g.sw2 ? a0 : a2, g.sw2 ? a1 : a3};
  uint4 e[16];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t c = perm(w[k], w[k], g.selb);
    const uint32_t cp = g.cpos0 ^ ((uint32_t)k * 0x40404040u);
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t ea = perm(c, cp, 0x0c0c0000u | ((4u + b) << 8) | (uint32_t)b);
      e[4 * k + b] = *reinterpret_cast<const uint4 *>(lds + LDS_GT + ea);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0;
#pragma unroll
  for (int q = 0; q < 16; q += 2) {
    r0 = xor3(r0, e[q].x, e[q + 1].x);
    r1 = xor3(r1, e[q].y, e[q + 1].y);
    r2 = xor3(r2, e[q].z, e[q + 1].z);
    r3 = xor3(r3, e[q].w, e[q + 1].w);
  }
  return make_uint4(r0, r1, r2, r3);
}

// Y * H^e with the 4-bit table of that power in global memory (t = its 8 KiB:
// nibble position j (byte j>>1, low nibble if j even), value n at j*256+n*16).
// Used once per record per lane (the final x H^(8-l)), where the power differs
// per lane: from LDS that would be bank conflicts, from L2 it is a gather.
// ROLLED: rolled over the 4 words (8 positions, 2 KiB of table each), so the
// table addresses stay one pointer instead of 16 hoisted 64-bit ones (the
// throughput kernels); unrolled, all 32 gathers are in flight at once instead
// of four dependent L2 round trips (the small-batch kernels' latency).
template <int UNR = 1>
__device__ __forceinline__ uint4 gf_mul4_global(uint4 x, const uint8_t *t) {
  uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0;
  uint32_t w = x.x, w1 = x.y, w2 = x.z, w3 = x.w;
  constexpr int kUnroll = UNR;
#pragma unroll kUnroll
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
__device__ __forceinline__ uint4 xor4(uint4 a, uint4 b) {
  return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}

// The cold work of the chunk loop (session-change table staging, the first
// T-table fill, MODE 3's rollback of a failed record) runs as real calls:
// kept out of the record loop's register allocation (gcm_kernel<3,1024,4>:
// 16 -> 0 VGPRs spilled).
#define GCM_COLD __noinline__

// The Te0/Te1 pair table, 32 replicas, into LDS (a workgroup's first AEAD
// chunk; out of line like the table staging)
template <int WG>
__device__ GCM_COLD void fill_tp(uint8_t *lds, const uint2 *tpair, int tid) {
  for (int idx = tid; idx < 256 * 32; idx += WG) {
    const int x = idx >> 5, r = idx & 31;
    const uint2 t = tpair[x];
    *reinterpret_cast<uint32_t *>(lds + LDS_TP + x * 256 + r * 4) = t.x;
    *reinterpret_cast<uint32_t *>(lds + LDS_TP + x * 256 + 128 + r * 4) = t.y;
  }
}

// The Horner multiplier's 8-bit table (value-major, entry (v, q) at v*256 +
// q*16) built in LDS from the same power's 4-bit table in gtab (nibble
// position j, value n at j*256 + n*16; host_crypto.cpp ghash_tables).  The
// multiply is GF(2)-linear in the block, so T8[v][q] = T4[2q][v & 15] ^
// T4[2q+1][v >> 4]: a workgroup that changes session reads 8 KiB (which the
// final multiply's gathers share) instead of copying the 64-KiB table.  The
// reference precomputes its tables once per key (gmac.c:48-63 -> gfmult.c:87
// gf128_genmultable4); here the 8-bit expansion is redone per workgroup.
// The 8 KiB come into `scratch` with one coalesced 16-byte load per thread
// (one L2/HBM round trip: at a session change of every chunk, as in cfg4,
// four dependent ones per thread were the staging's cost), then the 8-bit
// entries from LDS.  Entry slot e takes q = e & 15 and v = (e >> 4) + 17q
// (mod 256), so a 16-lane group reads 16 different bank quads for the low
// nibble's row, at most 2 lanes per quad for the high one, and writes 16
// different quads.  Contains a barrier: call it workgroup-uniformly, after
// the workgroup's last read of dst and scratch.
template <int WG>
__device__ GCM_COLD void stage_h8_lds(uint8_t *dst, const uint8_t *t4, int tid, uint8_t *scratch) {
  for (int i = tid; i < (int)(kGhPowerBytes / 16); i += WG)
    reinterpret_cast<uint4 *>(scratch)[i] = reinterpret_cast<const uint4 *>(t4)[i];
  __syncthreads();
#pragma unroll 1
  for (int k = 0; k < (4096 + WG - 1) / WG; ++k) {
    const int e = tid + k * WG;
    if (4096 % WG == 0 || e < 4096) {
      const int q = e & 15, v = ((e >> 4) + 17 * q) & 255;
      const uint4 lo = *reinterpret_cast<const uint4 *>(scratch + (2 * q) * 256 + (v & 15) * 16);
      const uint4 hi = *reinterpret_cast<const uint4 *>(scratch + (2 * q + 1) * 256 + (v >> 4) * 16);
      *reinterpret_cast<uint4 *>(dst + (v * 16 + q) * 16) = xor4(lo, hi);
    }
  }
}

// In place, one pass (MODE 3): a record whose tag
// failed already holds plaintext; XORing the same keystream over it again
// restores the ciphertext exactly, so the buffer ends as cryptosoft's
// verify-first leaves it (cryptosoft.c:595-633: a failed record is not
// decrypted).  Rare path, one block per lane per step, with its own counter
// cache: it runs only in a wave with a failed record, after the wave's stores
// are complete (the block-to-lane map here differs from the GHASH
// schedule's), and out of line, so the record loop does not hold registers
// for it.  Every lane of the wave calls it (back: this lane's record).
template <int S>
__device__ GCM_COLD void gcm_rollback(uint8_t *rec, int nct, int ct_len, bool back, int l, uint32_t s0c,
                                          uint32_t s1c, uint32_t s2c, rkptr rk, uint32_t rk3, int nr,
                                          const uint8_t *lds, uint32_t slot) {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  CtrCache cc;
  cc.hi = -1;
  int Mr = back ? (nct + S - 1) / S : 0;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) Mr = max(Mr, __shfl_xor(Mr, o));
  for (int a = 0; a < Mr; ++a) {
    const int c = S * a + l;
    const uint32_t t = (uint32_t)c + 2;
    uint4 P = make_uint4(0, 0, 0, 0);
    if (back && c < nct) P = ld16(rec + 16 + 16 * c);
    if ((int)(t >> 8) != cc.hi) ctr_cache_build(cc, s0c, s1c, s2c, (int)(t >> 8), rk, lds, slot);
    const uint4 ks = aes_ctr(cc, t, rk3, nr, rk, lds, slot);
    if (back && c < nct) st_partial(rec + 16 + 16 * c, xor4(P, ks), ct_len - 16 * c);
  }
}

// ---- one record group per wave (64 / S records) --------------------------------
// MODE 0: decrypt, single pass, plaintext to p.out (out of place)
// MODE 1: encrypt in place + ICV
// MODE 3: decrypt in place, verify first, in one pass: MODE 0 over the record
//         itself, then a failed record's keystream XORed over it again
// (the two-pass in-place form, GHASH + tag then CTR over the verified
// records, measured 1.60-1.64 vs 1.39-1.46 ms on cfg1: DESIGN.md §3.1)
// Steps m, m+1 of a lane run together: 2 independent AES blocks, then
// GHASH as (Y*H^S ^ B_m)*H^S ^ B_m+1 with the 8-bit table.
template <int MODE, int S>
__device__ __forceinline__ void do_group(const GcmParams &p, const uint8_t *lds, uint32_t di, bool have,
                                         uint32_t sa, uint32_t sa_flags, uint32_t mlen, int nr, rkptr rk) {
  static_assert(MODE == 0 || MODE == 1 || MODE == 3, "decrypt out of place, encrypt, decrypt in place");
  const int lane = threadIdx.x & 63;
  const int l = lane & (S - 1);
  const uint32_t slot = ((uint32_t)(lane & 31) * 4) | (LDS_TP & 0xff0000u);
  const int sep = (sa_flags & ESPGPU_CSP_F_SEPARATE_AAD) != 0;
  const GhLane gl = gh_lane(lane);

  // -- descriptor and record header ------------------------------------------
  int valid = 0, ct_len = 0, nct = 0, N = 0, M = 0, pad = 0;
  uint8_t *rec = p.arena;
  uint32_t len = 0, spi = 0, sn = 0, esnh = 0;
  uint32_t s0c = 0, s1c = 0, s2c = 0;
  if (have) {
    const uint4 dv = *reinterpret_cast<const uint4 *>(p.desc + di);
    len = dv.y & 0xffffu;
    ct_len = (int)len - 16 - (int)mlen;                      // 8 hdr + 8 IV + ICV
    valid = ((dv.y >> 16) == sa) && ct_len > 0 && (len & 3) == 0 &&   // xform_esp.c:279-324
            (MODE != 0 || p.out_stride == 0 || ct_len <= (int)p.out_stride);   // packed output: fits its slot
    if (valid) {
      rec = p.arena + (size_t)dv.x * 4;
      const uint4 h = ld16(rec);                             // SPI, SN, explicit IV
      spi = h.x;
      sn = h.y;
      esnh = bswap32(dv.z);
      nct = (ct_len + 15) >> 4;
      N = nct + 2;
      M = (N + S - 1) / S;
      pad = S * M - N;
      s0c = bswap32(dv.w) ^ rk[0];                           // salt
      s1c = bswap32(h.z) ^ rk[1];
      s2c = bswap32(h.w) ^ rk[2];
    }
  }
  int Mw = M;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) Mw = max(Mw, __shfl_xor(Mw, o));
  GCM_PHASE(8, true);
  const bool want_trl = MODE != 1 && p.trailer != nullptr;
  if (Mw == 0) {
    if (have && l == 0 && !valid) p.status[di] = ESPGPU_EINVAL;
    if (have && l == 0 && want_trl) p.trailer[di] = 0;
    return;
  }
  const uint32_t rk3 = rk[3];
  // out of place: the record's own offset in out, or (packed output) slot di
  // of out_stride bytes; orec is where the record's header would be, the
  // plaintext starts 16 bytes after it
  uint8_t *orec = (MODE == 0 ? (p.out_stride ? p.out + (size_t)di * p.out_stride - 16 : p.out - p.arena + rec)
                             : rec);
  CtrCache cc;
  cc.hi = -1;                                               // built on first use

  // fused esp_input_cb trailer word, from the lane holding the last CT block
  uint32_t trl = 0;
  auto note_trailer = [&](int i, uint4 pt, int rem) {
    if (want_trl && i == nct)
      trl = esp_trailer_word(rem >= 16 ? pt.w : (rem > 8 ? pt.z : (rem > 4 ? pt.y : pt.x)),
                             (uint32_t)ct_len);
  };

  // GHASH input block of GHASH index i (>= 1) given its ciphertext C and
  // keystream ks; stores the output block (MODE 0: plaintext, MODE 1: CT).
  auto block_in = [&](int i, bool has_ct, uint4 C, uint4 ks) -> uint4 {
    if (has_ct) {
      const int c = i - 1;
      const int rem = ct_len - 16 * c;
      if (MODE == 1) {
        const uint4 o = xor4(C, ks);
        st_partial(orec + 16 + 16 * c, o, rem);
        return mask_block(o, rem);
      }
      if (MODE == 0 || MODE == 3) {
        const uint4 pt = xor4(C, ks);
        if (!(gopts() & 9)) st_partial(orec + 16 + 16 * c, pt, rem);
        note_trailer(i, pt, rem);
      }
      return mask_block(C, rem);
    }
    if (valid && i == N - 1)                                     // length block
      return make_uint4(0, bswap32(sep ? 96u : 64u), 0, bswap32((uint32_t)ct_len * 8));
    return make_uint4(0, 0, 0, 0);
  };

  uint4 Y = make_uint4(0, 0, 0, 0), EJ0 = make_uint4(0, 0, 0, 0);
  // Aligned schedule (MODE 0 / 1, S = 4, every record of the wave with pad =
  // S - 1, i.e. nct + 1 a multiple of S, as 1500-byte packets are): the AES
  // work is decoupled from the GHASH positions.  GHASH is unchanged (block i
  // = S*g + l - pad at step g), but the counter blocks are dealt out densely,
  // lane l of AES step a taking slot j = S*a + l (CT block j, or J0 in slot
  // nct), so a record runs nct + 1 = S*Ma block encryptions instead of S*M =
  // S*(Ma + 1): the front padding and the length block get none.  With pad =
  // S - 1 GHASH step a + 1 of lane l hashes exactly slot j of AES step a, so
  // the ciphertext a lane loaded (or, encrypting, produced) is hashed one step
  // later from its own registers.
  const bool aligned = S == kGcmLanesPerRec && __all(!valid || pad == S - 1);
  int m = aligned ? Mw : 0;
  if (aligned) {
    const int Ma = valid ? M - 1 : 0;
    int Maw = Ma;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) Maw = max(Maw, __shfl_xor(Maw, o));
    // GHASH block of AES slot j: the (masked) ciphertext, the length block in
    // slot nct; C = this slot's ciphertext, ks its keystream; also stores
    // the slot's output and notes E_K(J0) / the trailer word
    auto slot_out = [&](int j, uint4 C, uint4 ks) -> uint4 {
      if (!valid || j > nct) return make_uint4(0, 0, 0, 0);
      if (j == nct) {
        EJ0 = ks;
        return make_uint4(0, bswap32(sep ? 96u : 64u), 0, bswap32((uint32_t)ct_len * 8));
      }
      const int rem = ct_len - 16 * j;
      const uint4 o = xor4(C, ks);
      if (!(gopts() & 9)) st_partial(orec + 16 + 16 * j, o, rem);
      if (MODE == 0 || MODE == 3) note_trailer(j + 1, o, rem);
      return mask_block(MODE == 1 ? o : C, rem);
    };
    uint4 prev = (valid && l == S - 1) ? (sep ? make_uint4(spi, esnh, sn, 0) : make_uint4(spi, sn, 0, 0))
                                       : make_uint4(0, 0, 0, 0);      // GHASH step 0: AAD / padding
    for (int a = 0; a < Maw; a += 2) {
      const int ja = S * a + l, jb = ja + S;
      const uint32_t ca = ja < nct ? (uint32_t)ja + 2 : 1u, cb = jb < nct ? (uint32_t)jb + 2 : 1u;
      const bool two = a + 1 < Maw;                                  // wave-uniform
      if (two && a > 0 && __all(!valid || 16 * (jb + 1) <= ct_len)) {
        // interior: both slots full ciphertext blocks for every record
        if ((int)(ca >> 8) != cc.hi) ctr_cache_build(cc, s0c, s1c, s2c, (int)(ca >> 8), rk, lds, slot);
        if (__all((int)(cb >> 8) == cc.hi)) {
          uint4 Ca = make_uint4(0, 0, 0, 0), Cb = make_uint4(0, 0, 0, 0);
          if (valid && !(gopts() & 17)) {
            Ca = ld16(rec + 16 + 16 * ja);
            Cb = ld16(rec + 16 + 16 * jb);
          }
          uint4 ka, kb;
          aes_ctr2(cc, ca, cb, rk3, nr, rk, lds, slot, ka, kb);
          const uint4 Oa = xor4(Ca, ka), Ob = xor4(Cb, kb);
          if (valid && !(gopts() & 9)) {
            st16(orec + 16 + 16 * ja, Oa);
            st16(orec + 16 + 16 * jb, Ob);
          }
          const uint4 Ba = MODE == 1 ? Oa : Ca;
          if (gopts() & 2)
            Y = xor4(xor4(Y, prev), Ba);
          else
            Y = xor4(gf_mul8(xor4(gf_mul8(Y, lds, gl), prev), lds, gl), Ba);
          prev = MODE == 1 ? Ob : Cb;
          continue;
        }
      }
      // general pair (or single last AES step): per-lane slot kinds
      uint4 Ca = make_uint4(0, 0, 0, 0), Cb = make_uint4(0, 0, 0, 0);
      if (valid && ja < nct && !(gopts() & 17)) Ca = ld16(rec + 16 + 16 * ja);
      if (two && valid && jb < nct && !(gopts() & 17)) Cb = ld16(rec + 16 + 16 * jb);
      // (the edge steps of a record: one block at a time, so the general path
      // holds one keystream block and inlines no second pair round)
      if ((int)(ca >> 8) != cc.hi) ctr_cache_build(cc, s0c, s1c, s2c, (int)(ca >> 8), rk, lds, slot);
      const uint4 ka = aes_ctr(cc, ca, rk3, nr, rk, lds, slot);
      const uint4 Ba = a < Ma ? slot_out(ja, Ca, ka) : make_uint4(0, 0, 0, 0);
      uint4 Bb = make_uint4(0, 0, 0, 0), kb = make_uint4(0, 0, 0, 0);
      if (two) {
        if ((int)(cb >> 8) != cc.hi) ctr_cache_build(cc, s0c, s1c, s2c, (int)(cb >> 8), rk, lds, slot);
        kb = aes_ctr(cc, cb, rk3, nr, rk, lds, slot);
        if (a + 1 < Ma) Bb = slot_out(jb, Cb, kb);
      }
      // GHASH steps a (block prev) and a + 1 (block Ba), each only if <= Ma
      const uint4 Ym = a == 0 ? prev : xor4((gopts() & 2) ? Y : gf_mul8(Y, lds, gl), prev);
      if (valid && a <= Ma) Y = Ym;
      const uint4 Yn = xor4((gopts() & 2) ? Y : gf_mul8(Y, lds, gl), Ba);
      if (valid && a + 1 <= Ma) Y = Yn;
      prev = Bb;
    }
    if ((Maw & 1) == 0 && Maw > 0) {
      // GHASH step Maw (the last block of the records with Ma == Maw)
      const uint4 Yn = xor4((gopts() & 2) ? Y : gf_mul8(Y, lds, gl), prev);
      if (valid && Ma == Maw) Y = Yn;
    }
  }
  while (m < Mw) {
    const int i = S * m + l - pad;
    if (m + 1 < Mw) {
      // The pair needs the counter cache valid for both blocks (i < 0 is
      // front padding: J0's counter).
      const uint32_t ca = i >= 0 ? (uint32_t)i + 1 : 1u, cb = (uint32_t)(i + S) + 1;
      if ((int)(ca >> 8) != cc.hi) ctr_cache_build(cc, s0c, s1c, s2c, (int)(ca >> 8), rk, lds, slot);
      if (__all((int)(cb >> 8) == cc.hi)) {
        const int ib = i + S;
        // Interior pair, wave-uniform: for every record of the wave both
        // blocks are full ciphertext blocks and neither is the last one (no
        // AAD, length block, partial block or trailer word), so loads and
        // stores are unconditional 16-byte accesses and GHASH takes them
        // unmasked.  Most pairs of a record take this path.
        if (__all(!valid || (i >= 1 && 16 * ib < ct_len))) {
          uint4 Ca = make_uint4(0, 0, 0, 0), Cb = make_uint4(0, 0, 0, 0);
          if (valid && !(gopts() & 17)) {
            Ca = ld16(rec + 16 * i);
            Cb = ld16(rec + 16 * ib);
          }
          uint4 ka, kb;
          aes_ctr2(cc, ca, cb, rk3, nr, rk, lds, slot, ka, kb);
          uint4 Ba = Ca, Bb = Cb;
          if (MODE == 1) {
            Ba = xor4(Ca, ka);
            Bb = xor4(Cb, kb);
          }
          if (valid && !(gopts() & 9)) {
            st16(orec + 16 * i, MODE == 1 ? Ba : xor4(Ca, ka));
            st16(orec + 16 * ib, MODE == 1 ? Bb : xor4(Cb, kb));
          }
          if (gopts() & 2)
            Y = xor4(xor4(Y, Ba), Bb);
          else
            Y = xor4(gf_mul8(xor4(gf_mul8(Y, lds, gl), Ba), lds, gl), Bb);
          m += 2;
          continue;
        }
        const bool hca = valid && i >= 1 && i <= nct, hcb = valid && ib <= nct;
        uint4 Ca = make_uint4(0, 0, 0, 0), Cb = make_uint4(0, 0, 0, 0);
        if (hca && !(gopts() & 17)) Ca = ld16(rec + 16 * i);
        if (hcb && !(gopts() & 17)) Cb = ld16(rec + 16 * ib);
        uint4 ka, kb;
        aes_ctr2(cc, ca, cb, rk3, nr, rk, lds, slot, ka, kb);
        uint4 Ba;
        if (valid && i == 0) {                                     // AAD block
          Ba = sep ? make_uint4(spi, esnh, sn, 0) : make_uint4(spi, sn, 0, 0);
          EJ0 = ka;
        } else {
          Ba = block_in(i, hca, Ca, ka);
        }
        const uint4 Bb = block_in(ib, hcb, Cb, kb);
        // M >= m+2: Y = (Y*H^8 ^ Ba)*H^8 ^ Bb;  M == m+1: Y = Y*H^8 ^ Ba
        const uint4 P = (gopts() & 2) ? Y : gf_mul8(Y, lds, gl);
        if (M >= m + 1) {
          const uint4 Ym = xor4(P, Ba);
          Y = Ym;
          if (M >= m + 2) Y = xor4((gopts() & 2) ? Ym : gf_mul8(Ym, lds, gl), Bb);
        }
        m += 2;
        continue;
      }
    }
    const uint32_t ctr = i >= 0 ? (uint32_t)(i + 1) : 1u;     // J0 for block 0, c+2 for CT c
    // Issue this step's ciphertext load before the AES/GHASH work so its HBM
    // latency hides under the round computation.
    const bool has_ct = valid && i >= 1 && i <= nct;
    uint4 C = make_uint4(0, 0, 0, 0);
    if (has_ct) C = ld16(rec + 16 * i);
    if ((int)(ctr >> 8) != cc.hi) ctr_cache_build(cc, s0c, s1c, s2c, (int)(ctr >> 8), rk, lds, slot);
    if (m > 0) {
      const uint4 Yn = gf_mul8(Y, lds, gl);
      if (m < M) Y = Yn;
    }
    const uint4 ks = aes_ctr(cc, ctr, rk3, nr, rk, lds, slot);
    uint4 B;
    if (valid && i == 0) {
      B = sep ? make_uint4(spi, esnh, sn, 0) : make_uint4(spi, sn, 0, 0);     // AAD block
      EJ0 = ks;
    } else {
      B = block_in(i, has_ct, C, ks);
    }
    Y = xor4(Y, B);
    ++m;
  }
  GCM_PHASE(9, true);
  // the received ICV, loaded before the final multiply's L2 gathers so the
  // two latencies overlap
  uint4 tag = make_uint4(0, 0, 0, 0);
  if (MODE != 1 && valid) {
    const uint32_t *q = reinterpret_cast<const uint32_t *>(rec + len - mlen);
    if (mlen == 16) {
      tag = ld16(rec + len - mlen);
    } else {
      tag.x = q[0];
      tag.y = q[1];
      if (mlen > 8) tag.z = q[2];
    }
  }
  // X = sum_l Y_l * H^(8-l)  (power index 7-l)
  uint4 Z;
  // (from LDS tables -- 24 KiB more per session -- measured +0.6 % on cfg4,
  // -1.7 % on cfg2; in 2 or 4 round trips instead of 4, equal or slower:
  // DESIGN.md §5.1, §6)
  if (gopts() & 64)
    Z = Y;
  else
    Z = gf_mul4_global(Y, p.gtab + (size_t)sa * kGhTableBytes + (uint32_t)(S - 1 - l) * kGhPowerBytes);
#pragma unroll
  for (int o = 1; o < S; o <<= 1) Z = xor4(Z, shfl_xor4(Z, o));
  const uint4 ej0 = shfl4(EJ0, (lane & ~(S - 1)) | pad);
  const uint4 T = xor4(Z, ej0);
  GCM_PHASE(10, true);

  int ok = 1;
  if (valid) {
    if (MODE == 1) {
      if (l == 0) st_partial(rec + len - mlen, T, (int)mlen);
    } else {
      const uint4 d = mask_block(xor4(T, tag), (int)mlen);
      ok = ((d.x | d.y | d.z | d.w) == 0) || (gopts() & 128);
    }
  }
  if (MODE == 3 && __any(valid && !ok))
    gcm_rollback<S>(rec, nct, ct_len, valid && !ok, l, s0c, s1c, s2c, rk, rk3, nr, lds, slot);
  if (want_trl) {
    // exactly one lane of the record holds it: OR over the 8 lanes
#pragma unroll
    for (int o = 1; o < S; o <<= 1) trl |= __shfl_xor(trl, o);
    if (have && l == 0) p.trailer[di] = (valid && ok) ? trl : 0u;
  }
  if (have && l == 0)
    p.status[di] = !valid ? ESPGPU_EINVAL : (ok ? ESPGPU_OK : ESPGPU_EBADMSG);
}

// ---- the burst design's two halves: a CTR pass and a GHASH / tag pass ----------
// For latency (gcm_burst_kernel, gcm_door_kernel below) the halves of GCM run
// side by side with the mapping each one wants:
//  * ctr pass (ctr_group): AES-CTR only, kBurstCtrLanes = 32 lanes per
//    record, three counter blocks per lane, all lookups of a round issued
//    before the wave waits (W); it also writes E_K(J0) (p.ej0[record]) and the
//    fused trailer word;
//  * tag pass (tag_group): GHASH only, S = 8 lanes per record with the 8-bit
//    H^8 table; T = GHASH ^ E_K(J0).
// decrypt out of place: ctr (DIR 0) beside the hash, then tag_finish
// (verify: status; a failed record's trailer word is zeroed); encrypt: ctr
// (DIR 1, in place) then tag (writes the ICV).  (As a throughput design --
// two kernels, 16 ctr lanes per record -- it measured 1.72-1.74 vs 1.50 ms on
// cfg1, and with a bitsliced ctr pass 2.26 ms: DESIGN.md §6.)
// Burst kernel (gcm_burst_kernel below): 512-thread workgroups, because two
// waves per SIMD leave 256 VGPRs per lane (at 1024 threads the 128-VGPR cap
// spilled 20-28) and a burst never needs the occupancy; its ctr pass runs 32
// lanes per record on waves [0, kBurstCtrWaves), its hash pass the rest.
constexpr int kBurstWG = 512, kBurstCtrLanes = 32, kBurstCtrWaves = 5;
constexpr uint32_t kBurstChunk = 4;     // records per burst chunk (at least; spread over the CUs)

template <int DIR, int S, bool W>
__device__ __forceinline__ void ctr_group(const GcmParams &p, const uint8_t *lds, uint32_t di, bool have,
                                          uint32_t sa, uint32_t mlen, int nr, rkptr rk, uint32_t tbase = 0) {
  const int lane = threadIdx.x & 63;
  const int l = lane & (S - 1);
  const uint32_t slot = (uint32_t)(lane & 31) * 4 | tbase;  // T-table at LDS offset tbase (64 KiB aligned)
  int valid = 0, ct_len = 0, nct = 0, K = 0;
  uint8_t *rec = p.arena;
  uint32_t s0c = 0, s1c = 0, s2c = 0;
  if (have) {
    const uint4 dv = *reinterpret_cast<const uint4 *>(p.desc + di);
    const uint32_t len = dv.y & 0xffffu;
    ct_len = (int)len - 16 - (int)mlen;
    valid = ((dv.y >> 16) == sa) && ct_len > 0 && (len & 3) == 0;
    if (valid) {
      rec = p.arena + (size_t)dv.x * 4;
      const uint4 h = ld16(rec);
      nct = (ct_len + 15) >> 4;
      K = (nct + S) / S;                                   // J0 + nct blocks over S lanes
      s0c = bswap32(dv.w) ^ rk[0];
      s1c = bswap32(h.z) ^ rk[1];
      s2c = bswap32(h.w) ^ rk[2];
    }
  }
  int Kw = K;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) Kw = max(Kw, __shfl_xor(Kw, o));
  if (Kw == 0) return;
  const bool want_trl = DIR == 0 && p.trailer != nullptr;
  uint8_t *orec = DIR == 0 ? p.out - p.arena + rec : rec;
  const uint32_t rk3 = rk[3];
  CtrCache cc;
  cc.hi = -1;
  // block i of the lane: -1 = J0 (counter 1), CT block i has counter i + 2
  auto emit = [&](int i, bool loaded, uint4 C, uint4 ks) {
    if (!valid) return;
    if (i == -1) {
      p.ej0[di] = ks;
      return;
    }
    if (!loaded) return;
    const int rem = ct_len - 16 * i;
    const uint4 o = xor4(C, ks);
    st_partial(orec + 16 + 16 * i, o, rem);
    if (want_trl && i == nct - 1)
      p.trailer[di] = esp_trailer_word(rem >= 16 ? o.w : (rem > 8 ? o.z : (rem > 4 ? o.y : o.x)),
                                       (uint32_t)ct_len);
  };
  for (int k = 0; k < Kw; k += 2) {
    const int ia = l - 1 + S * k, ib = ia + S;
    const bool two = k + 1 < Kw;                           // wave-uniform
    const bool la = valid && ia >= 0 && ia < nct;
    const bool lb = valid && two && ib < nct;
    uint4 Ca = make_uint4(0, 0, 0, 0), Cb = make_uint4(0, 0, 0, 0);
    if (la) Ca = ld16(rec + 16 + 16 * ia);
    if (lb) Cb = ld16(rec + 16 + 16 * ib);
    const uint32_t ca = (uint32_t)(ia + 2), cb = (uint32_t)(ib + 2);
    if ((int)(ca >> 8) != cc.hi) ctr_cache_build(cc, s0c, s1c, s2c, (int)(ca >> 8), rk, lds, slot);
    uint4 ka, kb = make_uint4(0, 0, 0, 0);
    if (two && __all((int)(cb >> 8) == cc.hi)) {
      aes_ctr2<W>(cc, ca, cb, rk3, nr, rk, lds, slot, ka, kb);
    } else {
      ka = aes_ctr<W>(cc, ca, rk3, nr, rk, lds, slot);
      if (two) {
        if ((int)(cb >> 8) != cc.hi) ctr_cache_build(cc, s0c, s1c, s2c, (int)(cb >> 8), rk, lds, slot);
        kb = aes_ctr<W>(cc, cb, rk3, nr, rk, lds, slot);
      }
    }
    emit(ia, la, Ca, ka);
    if (two) emit(ib, lb, Cb, kb);
  }
}

// zs != nullptr (burst kernel, decrypt): only the GHASH value, Z = sum of the
// lanes' Y x H^(S-1-l), goes to zs[zi] (LDS); tag_finish completes the record
// once E_K(J0) exists.
template <int DIR, int S>
__device__ __forceinline__ void tag_group(const GcmParams &p, const uint8_t *lds, uint32_t di, bool have,
                                          uint32_t sa, uint32_t sa_flags, uint32_t mlen,
                                          uint4 *zs = nullptr, uint32_t zi = 0) {
  const int lane = threadIdx.x & 63;
  const int l = lane & (S - 1);
  const int sep = (sa_flags & ESPGPU_CSP_F_SEPARATE_AAD) != 0;
  const GhLane gl = gh_lane(lane);
  int valid = 0, ct_len = 0, nct = 0, N = 0, M = 0, pad = 0;
  uint8_t *rec = p.arena;
  uint32_t len = 0, spi = 0, sn = 0, esnh = 0;
  if (have) {
    const uint4 dv = *reinterpret_cast<const uint4 *>(p.desc + di);
    len = dv.y & 0xffffu;
    ct_len = (int)len - 16 - (int)mlen;
    valid = ((dv.y >> 16) == sa) && ct_len > 0 && (len & 3) == 0;
    if (valid) {
      rec = p.arena + (size_t)dv.x * 4;
      const uint4 h = ld16(rec);
      spi = h.x;
      sn = h.y;
      esnh = bswap32(dv.z);
      nct = (ct_len + 15) >> 4;
      N = nct + 2;
      M = (N + S - 1) / S;
      pad = S * M - N;
    }
  }
  int Mw = M;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) Mw = max(Mw, __shfl_xor(Mw, o));
  GCM_PHASE_T(8, true, kBurstCtrWaves * 64);
  const bool want_trl = DIR == 0 && p.trailer != nullptr;
  if (Mw == 0) {
    if (zs == nullptr && have && l == 0 && !valid) {
      p.status[di] = ESPGPU_EINVAL;
      if (want_trl) p.trailer[di] = 0;
    }
    return;
  }
  // GHASH input block i: 0 = AAD, 1..nct = ciphertext, N-1 = lengths, < 0 = front padding
  auto blk = [&](int i, bool loaded, uint4 C) -> uint4 {
    if (loaded) return mask_block(C, ct_len - 16 * (i - 1));
    if (valid && i == 0) return sep ? make_uint4(spi, esnh, sn, 0) : make_uint4(spi, sn, 0, 0);
    if (valid && i == N - 1) return make_uint4(0, bswap32(sep ? 96u : 64u), 0, bswap32((uint32_t)ct_len * 8));
    return make_uint4(0, 0, 0, 0);
  };
  // lone-wave form for the burst kernel's S = 8 lanes
  auto gmul = [&](uint4 v) { return S == kGcmLanesSmall ? gf_mul8_wide(v, lds, gl) : gf_mul8(v, lds, gl); };
  uint4 Y = make_uint4(0, 0, 0, 0);
  // Small-batch lanes (S = 8) load their first kPre blocks (a 1500-byte
  // packet's all) before the first multiply: a lone wave would otherwise wait
  // a full load latency per step pair.
  constexpr int kPre = S == kGcmLanesSmall ? 12 : 0;
  uint4 Cp[kPre > 0 ? kPre : 1];
#pragma unroll
  for (int m = 0; m < kPre; ++m) {
    const int i = S * m + l - pad;
    Cp[m] = make_uint4(0, 0, 0, 0);
    if (valid && m < M && i >= 1 && i <= nct) Cp[m] = ld16(rec + 16 * i);
  }
  GCM_PHASE_T(9, true, kBurstCtrWaves * 64);
  for (int m = 0; m < Mw; m += 2) {
    const int i = S * m + l - pad, ib = i + S;
    const bool two = m + 1 < Mw;                           // wave-uniform
    const bool la = valid && i >= 1 && i <= nct, lb = valid && two && ib >= 1 && ib <= nct;
    uint4 Ca = make_uint4(0, 0, 0, 0), Cb = make_uint4(0, 0, 0, 0);
    if (kPre && m + 1 < kPre) {
      // m is even: select the preloaded pair without dynamic register indexing
#pragma unroll
      for (int q = 0; q < kPre; q += 2)
        if (q == m) {
          Ca = Cp[q];
          Cb = Cp[q + 1];
        }
    } else {
      if (la) Ca = ld16(rec + 16 * i);
      if (lb) Cb = ld16(rec + 16 * ib);
    }
    const uint4 Ba = blk(i, la, Ca), Bb = blk(ib, lb, Cb);
    const uint4 Ya = xor4(m == 0 ? Y : gmul(Y), Ba);
    if (m < M) Y = Ya;
    if (two) {
      const uint4 Yb = xor4(gmul(Y), Bb);
      if (m + 1 < M) Y = Yb;
    }
  }
  GCM_PHASE_T(10, true, kBurstCtrWaves * 64);
  if (zs != nullptr) {
    uint4 Z = gf_mul4_global<S != kGcmLanesSmall ? 1 : 4>(Y, p.gtab + (size_t)sa * kGhTableBytes + (uint32_t)(S - 1 - l) * kGhPowerBytes);
#pragma unroll
    for (int o = 1; o < S; o <<= 1) Z = xor4(Z, shfl_xor4(Z, o));
    if (have && l == 0) zs[zi] = Z;
    GCM_PHASE_T(11, true, kBurstCtrWaves * 64);
    return;
  }
  uint4 tag = make_uint4(0, 0, 0, 0), ej0 = make_uint4(0, 0, 0, 0);
  if (valid) {
    ej0 = p.ej0[di];
    if (DIR == 0) {
      const uint32_t *q = reinterpret_cast<const uint32_t *>(rec + len - mlen);
      if (mlen == 16) {
        tag = ld16(rec + len - mlen);
      } else {
        tag.x = q[0];
        tag.y = q[1];
        if (mlen > 8) tag.z = q[2];
      }
    }
  }
  uint4 Z = gf_mul4_global<S != kGcmLanesSmall ? 1 : 4>(Y, p.gtab + (size_t)sa * kGhTableBytes + (uint32_t)(S - 1 - l) * kGhPowerBytes);
#pragma unroll
  for (int o = 1; o < S; o <<= 1) Z = xor4(Z, shfl_xor4(Z, o));
  const uint4 T = xor4(Z, ej0);
  int ok = 1;
  if (valid) {
    if (DIR == 1) {
      if (l == 0) st_partial(rec + len - mlen, T, (int)mlen);
    } else {
      const uint4 d = mask_block(xor4(T, tag), (int)mlen);
      ok = ((d.x | d.y | d.z | d.w) == 0);
    }
  }
  if (have && l == 0) {
    p.status[di] = !valid ? ESPGPU_EINVAL : (ok ? ESPGPU_OK : ESPGPU_EBADMSG);
    if (want_trl && !(valid && ok)) p.trailer[di] = 0;
  }
}

// The rest of tag_group for a record whose GHASH value Z is known (one thread
// per record, burst kernel decrypt, after the ctr pass wrote E_K(J0) and the
// trailer word): verify, status, trailer word zeroed on failure.
__device__ __forceinline__ void tag_finish(const GcmParams &p, uint32_t di, uint32_t sa, uint32_t mlen, uint4 Z) {
  const uint4 dv = *reinterpret_cast<const uint4 *>(p.desc + di);
  const uint32_t len = dv.y & 0xffffu;
  const int ct_len = (int)len - 16 - (int)mlen;
  const bool valid = ((dv.y >> 16) == sa) && ct_len > 0 && (len & 3) == 0;
  int ok = 0;
  if (valid) {
    const uint8_t *rec = p.arena + (size_t)dv.x * 4;
    const uint32_t *q = reinterpret_cast<const uint32_t *>(rec + len - mlen);
    uint4 tag = make_uint4(0, 0, 0, 0);
    if (mlen == 16) {
      tag = ld16(rec + len - mlen);
    } else {
      tag.x = q[0];
      tag.y = q[1];
      if (mlen > 8) tag.z = q[2];
    }
    const uint4 d = mask_block(xor4(xor4(Z, p.ej0[di]), tag), (int)mlen);
    ok = ((d.x | d.y | d.z | d.w) == 0);
  }
  p.status[di] = !valid ? ESPGPU_EINVAL : (ok ? ESPGPU_OK : ESPGPU_EBADMSG);
  if (p.trailer && !(valid && ok)) p.trailer[di] = 0;
}

// Self-staging prologue of one chunk (gcm_kernel<..., STAGE>): copies the
// chunk's descriptors (p.hdesc -> p.desc) and records (p.xin) from host memory
// through the mapping and keeps its result spans (p.xout) in LDS for the
// epilogue.  Two dependent host reads per chunk: the spans and descriptor
// words together, then every record's bytes at once (tpr threads per record,
// one batch of loads each for records up to 2 KiB).
template <int WG>
__device__ __forceinline__ void stage_in(const GcmParams &p, uint32_t start, uint32_t count, XferSpan *s_xout) {
  const uint32_t tid = threadIdx.x;
  uint32_t tpr = 64;                                    // threads per record: count x tpr <= WG
  while (tpr > 1 && tpr * count > (uint32_t)WG) tpr >>= 1;
  const uint32_t r = tid / tpr, sub = tid % tpr;
  constexpr uint32_t kDW = sizeof(espgpu_desc) / 4;
  static_assert(kChunkRecs * kDW <= 4 * WG, "descriptor words per thread");
  const uint32_t nd = count * kDW;
  const uint32_t *hd = reinterpret_cast<const uint32_t *>(p.hdesc + start);
  uint32_t *dd = reinterpret_cast<uint32_t *>(const_cast<espgpu_desc *>(p.desc) + start);
  uint32_t dv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (tid + k * WG < nd) dv[k] = hd[tid + k * WG];
  XferSpan sp{0, 0, 0, 0}, so{0, 0, 0, 0};
  if (r < count) {
    sp = p.xin[start + r];
    if (sub < 2) so = p.xout[2 * (start + r) + sub];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (tid + k * WG < nd) dd[tid + k * WG] = dv[k];
  if (r < count) {
    if (sub < 2) s_xout[2 * r + sub] = so;
    xfer_copy<16>(sp.src, sp.dst, sp.len, sub, tpr);
  }
  __syncthreads();
}

// S lanes per record: kGcmLanesPerRec for throughput, kGcmLanesSmall for
// batches too small to fill the chip (half the serial steps per record).
// STAGE: the batch stages its own records (p.xin / p.xout, implicit chunks):
// each chunk's records are copied in by the workgroup that runs the chunk and
// its results copied out after it, so a burst is one launch.
template <int MODE, int WG, int S, bool STAGE = false>
__global__ __launch_bounds__(WG) void gcm_kernel(GcmParams p) {
  static_assert(S == kGcmLanesPerRec || S == kGcmLanesSmall, "GHASH tables exist for these strides");
  constexpr int RPW = 64 / S;             // records per wave
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALL];
  const int tid = threadIdx.x;
  GCM_PHASE(0, true);
  // The T-table (per entry 32 slots of Te0 then 32 slots of Te1, see tpa())
  // is filled with the first session's GHASH table: a workgroup that draws no
  // chunk (a launch with few GCM chunks, e.g. a batch of ETA records whose
  // invalid records the GCM kernel marks) leaves without the 64 KiB fill.
  bool tfilled = false;

  const bool implicit = (p.chunks == nullptr);
  const uint32_t nch = implicit ? (p.n + p.chunk - 1) / p.chunk : *p.nchunks;
  uint32_t cur_sa = 0xffffffffu, nr = 0, flags = 0, mlen = 16, mode = 0;
  const int wave = tid >> 6;
  // Dynamic chunk queue: chunk costs differ by up to ~300x (64-B vs 9000-B
  // records) and the planner emits the largest first, so grabbing tickets
  // balances the chip where a static split would leave most CUs idle.
  // s_ticket is double-buffered by iteration parity: slot it&1 is rewritten
  // only at it+2, after every thread passed iteration it+1's barrier.
  // (Per-XCD ticket counters measured equal on cfg4 and 13 % slower on
  // cfg2, whose largest-first order they break: DESIGN.md §6.)
  __shared__ uint32_t s_ticket[2];
  __shared__ XferSpan s_xout[STAGE ? 2 * kChunkRecs : 1];
  for (uint32_t it = 0;; ++it) {
    if (tid == 0) s_ticket[it & 1] = atomicAdd(&p.queue[0], 1u);
    __syncthreads();
    const uint32_t c = s_ticket[it & 1];
    GCM_PHASE(2, it == 0);
    if (c >= nch) break;
    uint32_t sa, start, count;
    if (implicit) {
      start = c * p.chunk;
      count = min(p.chunk, p.n - start);
      if (STAGE) stage_in<WG>(p, start, count, s_xout);
      GCM_PHASE(3, it == 0);
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
        if (mode == ESPGPU_CSP_MODE_AEAD && !tfilled) {
          fill_tp<WG>(lds, p.tpair, tid);
          tfilled = true;
          GCM_PHASE(1, true);
        }
        if (mode == ESPGPU_CSP_MODE_AEAD && !(gopts() & 32))
          stage_h8_lds<WG>(lds + LDS_GT, p.gtab + (size_t)sa * kGhTableBytes + (size_t)(S - 1) * kGhPowerBytes,
                           tid, lds + LDS_BYTES);
      } else {
        mode = 0;
      }
      cur_sa = sa;
      __syncthreads();
    }
    GCM_PHASE(4, it == 0);
    // a chunk takes kChunkRecs / (WG/8) passes of the workgroup
    for (uint32_t sub = 0; sub < count; sub += (uint32_t)(WG / 64) * RPW) {
      const uint32_t rl = sub + (uint32_t)wave * RPW + (uint32_t)((tid & 63) / S);
      const bool have = rl < count;
      const uint32_t pos = start + (have ? rl : 0);
      const uint32_t di = p.order ? p.order[pos] : pos;
      // Session check per record: a chunk is one session (planner), but a
      // caller-grouped batch (implicit chunks) is trusted only this far: a
      // record whose own session is not this chunk's AEAD session is EINVAL
      // here (do_group: valid requires desc.sa == sa) unless it is an ETA
      // record, which the ETA kernel owns.
      if (mode != ESPGPU_CSP_MODE_AEAD) {
        if (have && (tid & (S - 1)) == 0) {
          const uint32_t rsa = p.desc[di].sa;
          const bool eta = rsa < p.nsas && p.sas[rsa].mode == ESPGPU_CSP_MODE_ETA;
          if (!eta) {
            p.status[di] = ESPGPU_EINVAL;
            if (MODE != 1 && p.trailer) p.trailer[di] = 0;
          }
        }
        continue;
      }
      do_group<MODE, S>(p, lds, di, have, sa, flags, mlen, (int)nr, (rkptr)(const void *)(p.sas[sa].rk));
    }
    GCM_PHASE(5, it == 0);
    if (STAGE) {
      // statuses and the results of the records that passed back to the host
      __syncthreads();
      // (spans from LDS: no host read on the way out, the writes are posted)
      for (uint32_t r = (uint32_t)wave; r < count; r += (uint32_t)(WG / 64)) {
        const uint32_t di = start + r;
        const uint8_t st = p.status[di];
        if ((tid & 63) == 0) p.hstat[di] = st;
        if (st == ESPGPU_OK) {
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const XferSpan sp = s_xout[2 * r + k];
            if (sp.len) xfer_copy(sp.src, sp.dst, sp.len, (uint32_t)(tid & 63), 64u);
          }
        }
      }
      GCM_PHASE(6, it == 0);
    }
  }
  GCM_PHASE(7, true);
  // Every workgroup leaves the loop after drawing exactly one ticket >= nch,
  // so once all have retired no ticket is drawn again: reset for the next launch.
  if (tid == 0 && atomicAdd(&p.queue[1], 1u) == gridDim.x - 1) {
    atomicExch(&p.queue[0], 0u);
    atomicExch(&p.queue[1], 0u);
  }
}

// ---- burst kernel: the split design in one launch, for latency ----------------
// A burst leaves the chip idle and the fused kernel's time is the serial chain
// of each lane: S = 8 lanes walk a 1480-byte record in 12 AES + GHASH steps,
// VALU-issue-bound in a lone wave (~7.7 K cycles per step pair, phase clock of
// a 32-record burst, tools/burst_bench with the knobs library).  Here a chunk
// runs the ctr pass with kBurstCtrLanes = 32 lanes per record (3 counter
// blocks per lane) and the GHASH with kGcmLanesSmall = 8 lanes (12 multiplies,
// the H^8 table), E_K(J0) handed over through p.ej0 as in the two-kernel split
// design; both tables stay in LDS (T-table at LDS_TP, H^8 table at LDS_GT).
// DIR 0, decrypt out of place: the GHASH of the ciphertext does not wait for
// the ctr pass, so waves [0, kBurstCtrWaves) run the ctr pass while the others
// hash (Z to LDS); after a barrier one thread per record verifies.
// DIR 1, encrypt in place: the ctr pass, a barrier, then the tag pass over the
// ciphertext it wrote (ICV, status).
// STAGE: the batch stages its own records (stage_in / the epilogue, as
// gcm_kernel<..., true>): one launch per burst.
// The per-session state a burst workgroup keeps across chunks (the H^8
// table in LDS belongs to cur_sa).
struct BurstSA {
  uint32_t cur = 0xffffffffu, nr = 0, flags = 0, mlen = 16, mode = 0;
};

// One chunk of the burst design (gcm_burst_kernel; gcm_door_kernel runs the
// same body per claimed chunk): records [start, start + count) of p, session
// `sa` (~0u: the chunk's first descriptor's, read after staging).  `first`
// only gates the phase clock.
template <int DIR, int WG, bool STAGE>
__device__ __forceinline__ void burst_chunk(const GcmParams &p, uint8_t *lds, uint32_t start, uint32_t count,
                                            uint32_t sa, BurstSA &ss, uint4 *s_z, XferSpan *s_xout, bool first) {
  constexpr int ST = kGcmLanesSmall;
  [[maybe_unused]] constexpr int S = ST;    // for the phase clock
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  if (STAGE) stage_in<WG>(p, start, count, s_xout);
  if (sa == 0xffffffffu) sa = p.desc[start].sa;
  sa = __builtin_amdgcn_readfirstlane(sa);
  if (sa != ss.cur) {
    __syncthreads();
    if (sa < p.nsas) {
      const DevSA *s = p.sas + sa;
      ss.nr = s->nr;
      ss.flags = s->flags;
      ss.mlen = s->mlen;
      ss.mode = s->mode;
      if (ss.mode == ESPGPU_CSP_MODE_AEAD)    // H^8 (power index 7)
        stage_h8_lds<WG>(lds + LDS_GT, p.gtab + (size_t)sa * kGhTableBytes + 7 * kGhPowerBytes, tid,
                         lds + LDS_BYTES);
    } else {
      ss.mode = 0;
    }
    ss.cur = sa;
    __syncthreads();
  }
  const uint32_t nr = ss.nr, flags = ss.flags, mlen = ss.mlen;
  if (ss.mode != ESPGPU_CSP_MODE_AEAD) {
    // as gcm_kernel: EINVAL unless the ETA kernel's record
    for (uint32_t r = (uint32_t)tid; r < count; r += WG) {
      const uint32_t pos = start + r;
      const uint32_t di = p.order ? p.order[pos] : pos;
      const uint32_t rsa = p.desc[di].sa;
      const bool eta = rsa < p.nsas && p.sas[rsa].mode == ESPGPU_CSP_MODE_ETA;
      if (!eta) {
        p.status[di] = ESPGPU_EINVAL;
        if (DIR == 0 && p.trailer) p.trailer[di] = 0;
      }
    }
    if (STAGE) {
      // the statuses go back to the host (no results: nothing verified)
      __syncthreads();
      for (uint32_t r = (uint32_t)tid; r < count; r += WG) p.hstat[start + r] = p.status[start + r];
    }
    return;
  }
  GCM_PHASE(3, first);
  const rkptr rk = (rkptr)(const void *)(p.sas[sa].rk);
  constexpr uint32_t kCtrRpw = 64 / kBurstCtrLanes, kTagRpw = 64 / ST;
  if (DIR == 0) {
    constexpr uint32_t kCw = kBurstCtrWaves, kTw = WG / 64 - kBurstCtrWaves;
    if ((uint32_t)wave < kCw) {
      for (uint32_t sub = 0; sub < count; sub += kCw * kCtrRpw) {
        const uint32_t rl = sub + (uint32_t)wave * kCtrRpw + (uint32_t)((tid & 63) / kBurstCtrLanes);
        const bool have = rl < count;
        const uint32_t pos = start + (have ? rl : 0);
        const uint32_t di = p.order ? p.order[pos] : pos;
        if (__any(have)) ctr_group<0, kBurstCtrLanes, true>(p, lds, di, have, sa, mlen, (int)nr, rk, LDS_TP);
      }
    } else {
      for (uint32_t sub = 0; sub < count; sub += kTw * kTagRpw) {
        const uint32_t rl = sub + ((uint32_t)wave - kCw) * kTagRpw + (uint32_t)((tid & 63) / ST);
        const bool have = rl < count;
        const uint32_t pos = start + (have ? rl : 0);
        const uint32_t di = p.order ? p.order[pos] : pos;
        if (__any(have)) tag_group<0, ST>(p, lds, di, have, sa, flags, mlen, s_z, rl);
      }
    }
    GCM_PHASE(4, first);
    __syncthreads();
    GCM_PHASE(5, first);
    for (uint32_t r = (uint32_t)tid; r < count; r += WG) {
      const uint32_t pos = start + r;
      tag_finish(p, p.order ? p.order[pos] : pos, sa, mlen, s_z[r]);
    }
    // s_z is rewritten by the next chunk's hash waves
    __syncthreads();
  } else {
    for (uint32_t sub = 0; sub < count; sub += (uint32_t)(WG / 64) * kCtrRpw) {
      const uint32_t rl = sub + (uint32_t)wave * kCtrRpw + (uint32_t)((tid & 63) / kBurstCtrLanes);
      const bool have = rl < count;
      const uint32_t pos = start + (have ? rl : 0);
      const uint32_t di = p.order ? p.order[pos] : pos;
      if (__any(have)) ctr_group<1, kBurstCtrLanes, true>(p, lds, di, have, sa, mlen, (int)nr, rk, LDS_TP);
    }
    // the ciphertext and E_K(J0) written above are read below by other waves
    __syncthreads();
    for (uint32_t sub = 0; sub < count; sub += (uint32_t)(WG / 64) * kTagRpw) {
      const uint32_t rl = sub + (uint32_t)wave * kTagRpw + (uint32_t)((tid & 63) / ST);
      const bool have = rl < count;
      const uint32_t pos = start + (have ? rl : 0);
      const uint32_t di = p.order ? p.order[pos] : pos;
      if (__any(have)) tag_group<1, ST>(p, lds, di, have, sa, flags, mlen);
    }
  }
  if (STAGE) {
    // statuses and the results of the records that passed back to the host
    __syncthreads();
    for (uint32_t r = (uint32_t)wave; r < count; r += (uint32_t)(WG / 64)) {
      const uint32_t di = start + r;
      const uint8_t st = p.status[di];
      if ((tid & 63) == 0) p.hstat[di] = st;
      if (st == ESPGPU_OK) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const XferSpan sp = s_xout[2 * r + k];
          if (sp.len) xfer_copy(sp.src, sp.dst, sp.len, (uint32_t)(tid & 63), 64u);
        }
      }
    }
  }
  GCM_PHASE(6, first);
}

// The T-table pair into LDS (entry x: 32 slots of Te0, then 32 of Te1; tpa()).
template <int WG>
__device__ __forceinline__ void load_tpair(uint8_t *lds, const uint2 *tpair) {
  for (int idx = threadIdx.x; idx < 256 * 32; idx += WG) {
    const int x = idx >> 5, r = idx & 31;
    const uint2 t = tpair[x];
    *reinterpret_cast<uint32_t *>(lds + LDS_TP + x * 256 + r * 4) = t.x;
    *reinterpret_cast<uint32_t *>(lds + LDS_TP + x * 256 + 128 + r * 4) = t.y;
  }
}

template <int DIR, int WG, bool STAGE = false>
__global__ __launch_bounds__(WG) void gcm_burst_kernel(GcmParams p) {
  [[maybe_unused]] constexpr int S = kGcmLanesSmall;    // for the phase clock
  GCM_PHASE(0, true);
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALL];
  const int tid = threadIdx.x;
  load_tpair<WG>(lds, p.tpair);
  GCM_PHASE(1, true);
  const bool implicit = (p.chunks == nullptr);
  const uint32_t nch = implicit ? (p.n + p.chunk - 1) / p.chunk : *p.nchunks;
  BurstSA ss;
  __shared__ uint4 s_z[DIR == 0 ? kChunkRecs : 1];
  __shared__ XferSpan s_xout[STAGE ? 2 * kChunkRecs : 1];
  __shared__ uint32_t s_ticket[2];
  for (uint32_t it = 0;; ++it) {
    if (tid == 0) s_ticket[it & 1] = atomicAdd(&p.queue[0], 1u);
    __syncthreads();
    const uint32_t c = s_ticket[it & 1];
    GCM_PHASE(2, it == 0);
    if (c >= nch) break;
    if (implicit) {
      const uint32_t start = c * p.chunk;
      burst_chunk<DIR, WG, STAGE>(p, lds, start, min(p.chunk, p.n - start), 0xffffffffu, ss, s_z, s_xout, it == 0);
    } else {
      const Chunk ch = p.chunks[c];
      burst_chunk<DIR, WG, STAGE>(p, lds, ch.start, ch.count, ch.sa, ss, s_z, s_xout, it == 0);
    }
  }
  GCM_PHASE(7, true);
  if (tid == 0 && atomicAdd(&p.queue[1], 1u) == gridDim.x - 1) {
    atomicExch(&p.queue[0], 0u);
    atomicExch(&p.queue[1], 0u);
  }
}

// ---- doorbell kernel: the burst kernel as a persistent service -------------
// (espgpu_internal.h DoorCtl / DoorDev; set_tuning "door").  What a launched
// burst pays besides its crypto (phase clock, 32 registered records: 40 us
// per burst, 21 us of it in the kernel) is the launch and completion
// signalling and, inside the kernel, the T-table and H^8-table fills (3 us)
// and a cold ticket atomic.  Here the workgroups stay resident with both
// tables in LDS: thread 0 polls the job ring in host memory (one 16-byte
// read per poll over PCIe), claims chunk (job, c) with a CAS on the device
// claim counter, and the workgroup runs burst_chunk on it, staging records in
// from and results out to host memory as the launched burst kernel does.
// Every wave reaches the exit: stop set by the host, or idle_ticks without a
// claim (poll() relaunches the kernel for a job published after that).
template <int WG>
__global__ __launch_bounds__(WG) void gcm_door_kernel(DoorArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_ALL];
  __shared__ uint4 s_z[kChunkRecs];
  __shared__ XferSpan s_xout[2 * kChunkRecs];
  __shared__ uint32_t s_cmd[2][4];                 // job, chunk, n, slot_op (double-buffered by parity)
  const int tid = threadIdx.x;
  load_tpair<WG>(lds, a.tpair);
  BurstSA ss;
  constexpr uint32_t kExit = 0xffffffffu;
  // thread 0's view of the ring: the job it claims in, and that job's entry
  uint32_t cur = 0, en = 0, eso = 0, enc = 0;
  bool have = false;
  for (uint32_t it = 0;; ++it) {
    uint32_t *cmd = s_cmd[it & 1];
    if (tid == 0) {
      uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint32_t job = kExit, c = 0, n = 0, so = 0, stop = 0;
      typedef uint32_t V4 __attribute__((ext_vector_type(4)));
      for (uint32_t poll = 0;; ++poll) {
        // stop (read on every 4th poll: each read is a PCIe round trip):
        // kDoorStopNow exits between chunks; kDoorStopIdle (the host is about
        // to launch other kernels, which may share this kernel's hardware
        // queue) exits as soon as no published job is waiting
        if ((poll & 3) == 0) {
          stop = *reinterpret_cast<volatile uint32_t *>(&a.ctl->stop);
          if (stop == kDoorStopNow) break;
        }
        if (!have) {
          const uint32_t hint = __hip_atomic_load(&a.dev->next, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if ((int32_t)(hint - cur) > 0) cur = hint;
          const V4 e = *reinterpret_cast<const volatile V4 *>(&a.ctl->ring[cur % kDoorRing]);   // one 16-byte read
          if (e.w == cur + 1 && e.z == (e.x ^ e.y ^ e.w ^ kDoorChk)) {
            have = true;
            en = e.x, eso = e.y, enc = (e.x + a.chunk - 1) / a.chunk;
            // jobs are still arriving: the idle clock restarts even if other
            // workgroups win every chunk of this one
            t0 = __builtin_amdgcn_s_memrealtime();
          } else if ((int32_t)(e.w - (cur + 1)) > 0) {
            ++cur;                         // the entry holds a later job: job cur is long done
            continue;
          } else {
            if (stop == kDoorStopIdle) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > a.idle_ticks) break;
            __builtin_amdgcn_s_sleep(4);
            continue;
          }
        }
        unsigned long long *tw = &a.dev->tick[cur % kDoorRing];
        const unsigned long long w = __hip_atomic_load(tw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((int32_t)((uint32_t)(w >> 32) - (cur + 1)) < 0) {
          // install job cur's generation (it is published: this thread saw it)
          unsigned long long exp = w;
          __hip_atomic_compare_exchange_strong(tw, &exp, (unsigned long long)(cur + 1) << 32, __ATOMIC_RELAXED,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          continue;
        }
        const unsigned long long t = __hip_atomic_fetch_add(tw, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t g = (uint32_t)(t >> 32), cc = (uint32_t)t;
        if (g == cur + 1) {
          if (cc < enc) {
            job = cur, c = cc, n = en, so = eso;
            break;
          }
          // every chunk of job cur is claimed: on to the next job
          __hip_atomic_fetch_max(&a.dev->next, cur + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ++cur;
          have = false;
          continue;
        }
        // the add landed on a later job's generation (g - 1, published when
        // it was installed): chunk cc of that job is this workgroup's unless
        // the job already had all its chunks claimed
        const uint32_t jj = g - 1;
        const V4 e = *reinterpret_cast<const volatile V4 *>(&a.ctl->ring[jj % kDoorRing]);
        cur = jj;
        have = false;
        if (e.w == jj + 1 && e.z == (e.x ^ e.y ^ e.w ^ kDoorChk)) {
          have = true;
          en = e.x, eso = e.y, enc = (e.x + a.chunk - 1) / a.chunk;
          if (cc < enc) {
            job = jj, c = cc, n = en, so = eso;
            break;
          }
        }
      }
      // the job's host data (descriptors, spans, records) as published: no
      // line cached from an earlier job at the same addresses survives
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      cmd[0] = job;
      cmd[1] = c;
      cmd[2] = n;
      cmd[3] = so;
    }
    __syncthreads();
    const uint32_t job = cmd[0];
    if (job == kExit) break;
    const uint32_t c = cmd[1], n = cmd[2], slot = cmd[3] & 0xffffu, op = cmd[3] >> 16;
    if (slot < a.nslots) {
      const DoorSlot sl = a.slots[slot];
      GcmParams p{};
      uint8_t *res = op ? sl.arena : sl.out;
      p.arena = sl.arena;
      p.out = res;
      p.desc = reinterpret_cast<const espgpu_desc *>(sl.arena + sl.desc_off);
      p.n = n;
      p.sas = a.sas;
      p.gtab = a.gtab;
      p.tpair = a.tpair;
      p.status = res + sl.stat_off;
      p.nsas = a.nsas;
      p.chunk = a.chunk;
      p.ej0 = sl.ej0;
      p.xin = sl.xin;
      p.xout = sl.xout;
      p.hstat = sl.hstat;
      p.hdesc = reinterpret_cast<const espgpu_desc *>(sl.hdesc);
      const uint32_t start = c * a.chunk, count = min(a.chunk, n - start);
      if (op)
        burst_chunk<1, WG, true>(p, lds, start, count, 0xffffffffu, ss, s_z, s_xout, false);
      else
        burst_chunk<0, WG, true>(p, lds, start, count, 0xffffffffu, ss, s_z, s_xout, false);
    }
    // every wave's host writes (results, statuses) complete and visible
    // before the job can be signalled done
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __syncthreads();
    if (tid == 0) {
      const uint32_t nch = (n + a.chunk - 1) / a.chunk;
      const uint32_t f = __hip_atomic_fetch_add(&a.dev->fin[job % kDoorRing], 1u, __ATOMIC_ACQ_REL,
                                                __HIP_MEMORY_SCOPE_AGENT);
      if (f == nch - 1) {
        __hip_atomic_store(&a.dev->fin[job % kDoorRing], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&a.ctl->done[job % kDoorRing], job + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

}  // namespace

#ifdef ESPGPU_KNOBS
extern "C" __attribute__((visibility("default"))) int espgpu_debug_phases(uint64_t *out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), sizeof(g_phase)) == hipSuccess ? 0 : -1;
}
#endif

int set_gcm_opts(uint32_t opts) {
#ifdef ESPGPU_KNOBS
  return hipMemcpyToSymbol(HIP_SYMBOL(g_opts), &opts, 4) == hipSuccess ? 0 : -1;
#else
  return opts ? -1 : 0;
#endif
}

int launch_gcm_door(const DoorArgs &a, int grid, void *stream) {
  hipLaunchKernelGGL((gcm_door_kernel<kBurstWG>), dim3(grid), dim3(kBurstWG), 0,
                     reinterpret_cast<hipStream_t>(stream), a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_gcm(const GcmParams &pp, int encrypt, int two_pass, int grid, int lanes, void *stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (grid <= 0) grid = 256;
  constexpr int W = kGcmLanesSmall;
  const bool small = pp.xin != nullptr || (lanes ? lanes == W : pp.n < kGcmSmallBatch);
  GcmParams p = pp;
  // implicit chunks (caller-grouped batch): kChunkRecs records each, or for a
  // batch of fewer than grid x kChunkRecs records as few as four waves'
  // records, so that it spreads over up to `grid` CUs instead of queueing on a
  // few (one wave per workgroup would stage 128 KiB of LDS tables for 8
  // records and hold every CU, starving a concurrent burst's kernel); no more
  // workgroups than chunks (a 32-record burst is one workgroup, not 256 that
  // only fill LDS and leave)
  // Chunk sizes are powers of two, so every chunk lies inside one aligned run
  // of kChunkRecs records (the grouping contract, include/espgpu.h).
  // burst kernel (small, E_K(J0) scratch given, out of place or encrypt):
  // chunks of one ctr wave's records, so a burst spreads over CUs
  const bool burst = small && pp.ej0 != nullptr && !two_pass;
  const uint32_t per = (pp.n + (uint32_t)grid - 1) / (uint32_t)grid;
  p.chunk = burst ? kBurstChunk : small ? 64 / W : 4 * (64 / kGcmLanesPerRec);
  while (p.chunk < per && p.chunk < (uint32_t)kChunkRecs) p.chunk <<= 1;
  if (p.chunks == nullptr) grid = std::max(1, std::min(grid, (int)((p.n + p.chunk - 1) / p.chunk)));
  if (!small && p.ej0 != nullptr) return -1;          // (the burst design serves small batches only)
  if (burst) {
    if (p.xin != nullptr && p.chunks != nullptr) return -1;   // self-staging: implicit chunks only
    if (p.xin != nullptr && encrypt)
      hipLaunchKernelGGL((gcm_burst_kernel<1, kBurstWG, true>), dim3(grid), dim3(kBurstWG), 0, st, p);
    else if (p.xin != nullptr)
      hipLaunchKernelGGL((gcm_burst_kernel<0, kBurstWG, true>), dim3(grid), dim3(kBurstWG), 0, st, p);
    else if (encrypt)
      hipLaunchKernelGGL((gcm_burst_kernel<1, kBurstWG>), dim3(grid), dim3(kBurstWG), 0, st, p);
    else
      hipLaunchKernelGGL((gcm_burst_kernel<0, kBurstWG>), dim3(grid), dim3(kBurstWG), 0, st, p);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  if (p.xin != nullptr) {   // self-staging small batch (implicit chunks, S = 8, never in place)
    if (p.chunks != nullptr || two_pass) return -1;
    if (encrypt)
      hipLaunchKernelGGL((gcm_kernel<1, 1024, W, true>), dim3(grid), dim3(1024), 0, st, p);
    else
      hipLaunchKernelGGL((gcm_kernel<0, 1024, W, true>), dim3(grid), dim3(1024), 0, st, p);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  if (small) {
    if (encrypt)
      hipLaunchKernelGGL((gcm_kernel<1, 1024, W>), dim3(grid), dim3(1024), 0, st, p);
    else if (two_pass)
      hipLaunchKernelGGL((gcm_kernel<kGcmInPlaceMode, 1024, W>), dim3(grid), dim3(1024), 0, st, p);
    else
      hipLaunchKernelGGL((gcm_kernel<0, 1024, W>), dim3(grid), dim3(1024), 0, st, p);
  } else if (encrypt) {
    hipLaunchKernelGGL((gcm_kernel<1, 1024, kGcmLanesPerRec>), dim3(grid), dim3(1024), 0, st, p);
  } else if (two_pass) {
    hipLaunchKernelGGL((gcm_kernel<kGcmInPlaceMode, 1024, kGcmLanesPerRec>), dim3(grid), dim3(1024), 0, st, p);
  } else {
    hipLaunchKernelGGL((gcm_kernel<0, 1024, kGcmLanesPerRec>), dim3(grid), dim3(1024), 0, st, p);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace espgpu
