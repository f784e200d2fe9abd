// bsaes.h — bitsliced AES tail rounds for TWO blocks held by one lane.
//
// Why: the T-table rounds of esp_gcm.hip are bound by LDS issue (each round
// is 16 ds_read_b32 per block) while the VALU is ~40 % busy.  Running the
// last K rounds of a lane's two counter blocks in bitsliced form moves that
// work from LDS to VALU.  Same function as the T-table rounds
// (rijndaelEncrypt, rijndael-alg-fst.c:863-1042), different data layout.
//
// Layout: 2 blocks x 16 bytes = 256 bits in 8 plane words q[0..7]; q[j]
// holds bit j of every byte.  Bit position of state byte (row r, column c)
// of block b in a plane word: 8*(3-r) + 4*b + c', where c' = (c + k*r) mod 4
// is the PHYSICAL column: ShiftRows is never executed, it only advances the
// offset k (logical column c of row r lives k*r columns further right), and
// MixColumns / the round keys are written for the offset they meet.
//
// Input : state entering round R (before SubBytes) as big-endian column
//         words (the T-table rounds' s0..s3) for blocks a and b.
// Output: the ciphertext blocks as little-endian memory words.
// Keys  : per bitsliced round, 8 plane words (key bytes replicated for both
//         blocks, laid out for that round's offset), from bs_round_keys().
//
// Plain C++ operators: hipcc folds the XOR/AND chains into v_bitop3_b32 and
// the rotations into v_alignbit_b32 / v_perm_b32.
#ifndef ESPGPU_BSAES_H
#define ESPGPU_BSAES_H

#include <stdint.h>

#if defined(__HIPCC__)
#define BS_FN __host__ __device__ __forceinline__
#else
#define BS_FN static inline
#endif

namespace espgpu {
namespace bs {

BS_FN uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

// swap the bits of a selected by mask m<<n with the bits of b selected by m
BS_FN void swapmove(uint32_t &a, uint32_t &b, uint32_t m, int n) {
  const uint32_t t = ((a >> n) ^ b) & m;
  b ^= t;
  a ^= t << n;
}

// 8 words W[m] (byte k of each) -> planes: q[j] byte k bit m = bit j of W[m] byte k.
BS_FN void transpose8(uint32_t w[8]) {
  swapmove(w[0], w[1], 0x55555555u, 1);
  swapmove(w[2], w[3], 0x55555555u, 1);
  swapmove(w[4], w[5], 0x55555555u, 1);
  swapmove(w[6], w[7], 0x55555555u, 1);
  swapmove(w[0], w[2], 0x33333333u, 2);
  swapmove(w[1], w[3], 0x33333333u, 2);
  swapmove(w[4], w[6], 0x33333333u, 2);
  swapmove(w[5], w[7], 0x33333333u, 2);
  swapmove(w[0], w[4], 0x0f0f0f0fu, 4);
  swapmove(w[1], w[5], 0x0f0f0f0fu, 4);
  swapmove(w[2], w[6], 0x0f0f0f0fu, 4);
  swapmove(w[3], w[7], 0x0f0f0f0fu, 4);
}

// Rotate every nibble right by s (bit c <- bit c+s mod 4).
template <int S>
BS_FN uint32_t nrotr(uint32_t x) {
  if (S == 0) return x;
  const uint32_t lo = (0xfu >> S) * 0x11111111u;
  return ((x >> S) & lo) | ((x << (4 - S)) & ~lo);
}

// R1 of MixColumns at offset K: value of row r+1, logical same column.
template <int K>
BS_FN uint32_t term1(uint32_t x) { return nrotr<(K & 3)>(rol(x, 8)); }
template <int K>
BS_FN uint32_t term2(uint32_t x) { return nrotr<((2 * K) & 3)>(rol(x, 16)); }

// Boyar-Peralta S-box circuit (32 AND, 83 XOR/XNOR); x0 = bit 7 ... x7 = bit 0.
BS_FN void sbox(uint32_t q[8]) {
  const uint32_t x0 = q[7], x1 = q[6], x2 = q[5], x3 = q[4];
  const uint32_t x4 = q[3], x5 = q[2], x6 = q[1], x7 = q[0];
  // top linear layer
  const uint32_t y14 = x3 ^ x5, y13 = x0 ^ x6, y9 = x0 ^ x3, y8 = x0 ^ x5;
  const uint32_t t0 = x1 ^ x2;
  const uint32_t y1 = t0 ^ x7, y4 = y1 ^ x3, y12 = y13 ^ y14, y2 = y1 ^ x0;
  const uint32_t y5 = y1 ^ x6, y3 = y5 ^ y8;
  const uint32_t t1 = x4 ^ y12;
  const uint32_t y15 = t1 ^ x5, y20 = t1 ^ x1, y6 = y15 ^ x7, y10 = y15 ^ t0;
  const uint32_t y11 = y20 ^ y9, y7 = x7 ^ y11, y17 = y10 ^ y11, y19 = y10 ^ y8;
  const uint32_t y16 = t0 ^ y11, y21 = y13 ^ y16, y18 = x0 ^ y16;
  // nonlinear middle
  const uint32_t t2 = y12 & y15, t3 = y3 & y6, t4 = t3 ^ t2, t5 = y4 & x7, t6 = t5 ^ t2;
  const uint32_t t7 = y13 & y16, t8 = y5 & y1, t9 = t8 ^ t7, t10 = y2 & y7, t11 = t10 ^ t7;
  const uint32_t t12 = y9 & y11, t13 = y14 & y17, t14 = t13 ^ t12, t15 = y8 & y10;
  const uint32_t t16 = t15 ^ t12, t17 = t4 ^ t14, t18 = t6 ^ t16, t19 = t9 ^ t14;
  const uint32_t t20 = t11 ^ t16, t21 = t17 ^ y20, t22 = t18 ^ y19, t23 = t19 ^ y21;
  const uint32_t t24 = t20 ^ y18;
  const uint32_t t25 = t21 ^ t22, t26 = t21 & t23, t27 = t24 ^ t26, t28 = t25 & t27;
  const uint32_t t29 = t28 ^ t22, t30 = t23 ^ t24, t31 = t22 ^ t26, t32 = t31 & t30;
  const uint32_t t33 = t32 ^ t24, t34 = t23 ^ t33, t35 = t27 ^ t33, t36 = t24 & t35;
  const uint32_t t37 = t36 ^ t34, t38 = t27 ^ t36, t39 = t29 & t38, t40 = t25 ^ t39;
  const uint32_t t41 = t40 ^ t37, t42 = t29 ^ t33, t43 = t29 ^ t40, t44 = t33 ^ t37;
  const uint32_t t45 = t42 ^ t41;
  const uint32_t z0 = t44 & y15, z1 = t37 & y6, z2 = t33 & x7, z3 = t43 & y16;
  const uint32_t z4 = t40 & y1, z5 = t29 & y7, z6 = t42 & y11, z7 = t45 & y17;
  const uint32_t z8 = t41 & y10, z9 = t44 & y12, z10 = t37 & y3, z11 = t33 & y4;
  const uint32_t z12 = t43 & y13, z13 = t40 & y5, z14 = t29 & y2, z15 = t42 & y9;
  const uint32_t z16 = t45 & y14, z17 = t41 & y8;
  // bottom linear layer
  const uint32_t t46 = z15 ^ z16, t47 = z10 ^ z11, t48 = z5 ^ z13, t49 = z9 ^ z10;
  const uint32_t t50 = z2 ^ z12, t51 = z2 ^ z5, t52 = z7 ^ z8, t53 = z0 ^ z3;
  const uint32_t t54 = z6 ^ z7, t55 = z16 ^ z17, t56 = z12 ^ t48, t57 = t50 ^ t53;
  const uint32_t t58 = z4 ^ t46, t59 = z3 ^ t54, t60 = t46 ^ t57, t61 = z14 ^ t57;
  const uint32_t t62 = t52 ^ t58, t63 = t49 ^ t58, t64 = z4 ^ t59, t65 = t61 ^ t62;
  const uint32_t t66 = z1 ^ t63;
  const uint32_t s0 = t59 ^ t63, s6 = t56 ^ ~t62, s7 = t48 ^ ~t60;
  const uint32_t t67 = t64 ^ t65;
  const uint32_t s3 = t53 ^ t66, s4 = t51 ^ t66, s5 = t47 ^ t65;
  const uint32_t s1 = t64 ^ ~s3, s2 = t55 ^ ~t67;
  q[7] = s0; q[6] = s1; q[5] = s2; q[4] = s3;
  q[3] = s4; q[2] = s5; q[1] = s6; q[0] = s7;
}

// MixColumns at offset K fused with AddRoundKey (key planes k[8]).
template <int K>
BS_FN void mixcolumns_ark(uint32_t q[8], const uint32_t k[8]) {
  uint32_t r1[8], t[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    r1[j] = term1<K>(q[j]);
    t[j] = q[j] ^ r1[j];
  }
  // xtime on planes: 2*t (mod x^8+x^4+x^3+x+1)
  const uint32_t xt[8] = {t[7], t[0] ^ t[7], t[1], t[2] ^ t[7], t[3] ^ t[7], t[4], t[5], t[6]};
#pragma unroll
  for (int j = 0; j < 8; ++j) q[j] = xt[j] ^ r1[j] ^ term2<K>(t[j]) ^ k[j];
}

BS_FN void ark(uint32_t q[8], const uint32_t k[8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) q[j] ^= k[j];
}

// Byte r of big-endian column word w (row 0 = top byte).
BS_FN uint32_t bget(uint32_t w, int r) { return (w >> (24 - 8 * r)) & 0xffu; }

// Column word of PHYSICAL column cp at offset K: byte of row r comes from
// logical column (cp - K*r) mod 4.
template <int K>
BS_FN uint32_t gather_col(const uint32_t s[4], int cp) {
  if ((K & 3) == 0) return s[cp];
  uint32_t w = 0;
#pragma unroll
  for (int r = 0; r < 4; ++r) w |= bget(s[(cp - K * r) & 3], r) << (24 - 8 * r);
  return w;
}

template <int K0>
BS_FN void pack(const uint32_t sa[4], const uint32_t sb[4], uint32_t q[8]) {
  uint32_t w[8];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    w[c] = gather_col<K0>(sa, c);
    w[4 + c] = gather_col<K0>(sb, c);
  }
  transpose8(w);
#pragma unroll
  for (int j = 0; j < 8; ++j) q[j] = w[j];
}

// Planes at offset KF -> logical big-endian column words of both blocks.
template <int KF>
BS_FN void unpack(const uint32_t q[8], uint32_t oa[4], uint32_t ob[4]) {
  uint32_t w[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) w[j] = q[j];
  transpose8(w);   // the bit transpose is an involution
  // physical column cp holds logical (r, cp - KF*r): logical (r, c) is in
  // physical column c + KF*r
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if ((KF & 3) == 0) {
      oa[c] = w[c];
      ob[c] = w[4 + c];
    } else {
      uint32_t a = 0, b = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        a |= bget(w[(c + KF * r) & 3], r) << (24 - 8 * r);
        b |= bget(w[4 + ((c + KF * r) & 3)], r) << (24 - 8 * r);
      }
      oa[c] = a;
      ob[c] = b;
    }
  }
}

// Offset a bitsliced segment starts at, so that its final offset is 0 (no
// output gather): K rounds advance the offset by K.
template <int KR>
struct Plan {
  static constexpr int k0 = (4 - (KR & 3)) & 3;
};

// Rounds nr-KR+1..nr on two blocks.  sa/sb: state entering round nr-KR+1
// (big-endian column words).  keys: KR x 8 plane words (any pointer type:
// the kernel passes a constant-address-space pointer so they load into
// SGPRs).  Output: big-endian column words of the two ciphertext blocks.
template <int KR, typename KP>
BS_FN void tail_rounds(const uint32_t sa[4], const uint32_t sb[4], KP keys, uint32_t oa[4],
                       uint32_t ob[4]) {
  constexpr int k0 = Plan<KR>::k0;
  uint32_t q[8], kk[8];
  pack<k0>(sa, sb, q);
#pragma unroll
  for (int i = 0; i < KR - 1; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) kk[j] = keys[8 * i + j];
    sbox(q);
    // offset after this round's ShiftRows: k0 + i + 1
    switch ((k0 + i + 1) & 3) {
      case 0: mixcolumns_ark<0>(q, kk); break;
      case 1: mixcolumns_ark<1>(q, kk); break;
      case 2: mixcolumns_ark<2>(q, kk); break;
      default: mixcolumns_ark<3>(q, kk); break;
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) kk[j] = keys[8 * (KR - 1) + j];
  sbox(q);
  ark(q, kk);
  unpack<0>(q, oa, ob);
}

// Host: plane round keys for the last kr rounds of a schedule of big-endian
// round-key words rk[4*(nr+1)] (rijndaelKeySetupEnc form).  The offset a
// round's AddRoundKey meets is (r - nr) mod 4 whatever kr is (a segment always
// ends at offset 0), so the keys of the last 4 rounds serve every kr <= 4:
// kr rounds use out + 8*(4 - kr) of a 4-round set.
BS_FN void round_keys(const uint32_t *rk, int nr, int kr, uint32_t *out) {
  for (int i = 0; i < kr; ++i) {
    const int r = nr - kr + 1 + i;
    const int off = (r - nr) & 3;
    uint32_t w[8];
    for (int cp = 0; cp < 4; ++cp) {
      uint32_t v = 0;
      for (int row = 0; row < 4; ++row)
        v |= bget(rk[4 * r + ((cp - off * row) & 3)], row) << (24 - 8 * row);
      w[cp] = v;
      w[4 + cp] = v;
    }
    transpose8(w);
    for (int j = 0; j < 8; ++j) out[8 * i + j] = w[j];
  }
}

}  // namespace bs
}  // namespace espgpu

#endif  // ESPGPU_BSAES_H
