// aes_bs.h — bitsliced AES rounds on the VALU for gfx950 (device code).
//
// The T-table AES of esp_gcm.hip is bound by the LDS lookup rate (16
// ds_read_b32 per block-round).  Here a lane holds 32 AES blocks
// bitsliced: register st[8*j + v] carries bit v (value 2^v) of state byte j
// (FIPS-197 input order, j = 4*column + row) for the 32 blocks, one per bit.
// A round is then pure VALU: the S-box is the Boyar-Peralta circuit
// (tools/sbox_circuit.py checks it against the S-box), ShiftRows is register
// renaming at compile time, MixColumns is 84 XORs per column, and the round
// key is folded into the next S-box's linear input layer as wave-uniform
// masks (SGPRs), so no XOR of the key is spent on the state.
//
// Affine constant.  The S-box circuit is evaluated without its four NOTs,
// i.e. it computes S'(x) = S(x) ^ 0x63.  A state of all-0x63 bytes is fixed by
// ShiftRows and MixColumns (2 ^ 3 ^ 1 ^ 1 = 1), so the NOT-free rounds equal
// the real ones when every round key after the first is XORed with 0x63 in
// every byte: the caller passes K'_r = K_r ^ 0x63..63 for r >= 1
// (rijndaelEncrypt's round structure, rijndael-alg-fst.c:863-1042).
#pragma once
#ifndef ESPGPU_HOST_SHIM   // tools/aes_bs_selftest.cpp builds this header for the CPU
#include <hip/hip_runtime.h>
#endif
#include <stdint.h>

namespace espgpu {
namespace bs {

__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// mask of bit (7 - i) of a uniform key byte: all ones or zero (x_i order)
__device__ __forceinline__ uint32_t kmask(uint32_t kb, int i) {
  return (uint32_t)(((int32_t)(kb << (24 + i))) >> 31);
}

// S'(x ^ k) on one bitsliced byte, in place.  b[v] = bit v; kb = the
// (uniform) key byte XORed into the input first.
__device__ __forceinline__ void sbox(uint32_t *b, uint32_t kb) {
  const uint32_t xi0 = b[7], x1 = b[6], x2 = b[5], xi3 = b[4];   // x0, x3 (x3 names the XOR)
  const uint32_t x4 = b[3], x5 = b[2], x6 = b[1], x7 = b[0];
  const uint32_t k0 = kmask(kb, 0), k1 = kmask(kb, 1), k2 = kmask(kb, 2), k3 = kmask(kb, 3);
  const uint32_t k4 = kmask(kb, 4), k5 = kmask(kb, 5), k6 = kmask(kb, 6), k7 = kmask(kb, 7);
  // linear input layer with the key folded in (every term below is x ^ k)
  const uint32_t y14 = x3(xi3, x5, k3 ^ k5);
  const uint32_t y13 = x3(xi0, x6, k0 ^ k6);
  const uint32_t y9 = x3(xi0, xi3, k0 ^ k3);
  const uint32_t y8 = x3(xi0, x5, k0 ^ k5);
  const uint32_t t0 = x3(x1, x2, k1 ^ k2);
  const uint32_t y1 = x3(t0, x7, k7);
  const uint32_t y4 = x3(y1, xi3, k3);
  const uint32_t y12 = y13 ^ y14;
  const uint32_t y2 = x3(y1, xi0, k0);
  const uint32_t y5 = x3(y1, x6, k6);
  const uint32_t y3 = y5 ^ y8;
  const uint32_t t1 = x3(x4, y12, k4);
  const uint32_t y15 = x3(t1, x5, k5);
  const uint32_t y20 = x3(t1, x1, k1);
  const uint32_t X7 = x7 ^ k7;
  const uint32_t y6 = y15 ^ X7;
  const uint32_t y10 = y15 ^ t0;
  const uint32_t y11 = y20 ^ y9;
  const uint32_t y7 = X7 ^ y11;
  const uint32_t y17 = y10 ^ y11;
  const uint32_t y19 = y10 ^ y8;
  const uint32_t y16 = t0 ^ y11;
  const uint32_t y21 = y13 ^ y16;
  const uint32_t y18 = x3(xi0, y16, k0);
  // nonlinear middle and output layer: the circuit's gates packed greedily
  // into 3-input v_bitop3_b32 (truth table over a=0xf0, b=0xcc, c=0xaa;
  // generated from tools/sbox_circuit.py by tools/sbox_lut3.py)
  // 62 ops (92 gates, 30 absorbed)
  const uint32_t t2 = y12 & y15;
  const uint32_t t4 = __builtin_amdgcn_bitop3_b32(y3, y6, t2, 0x6a);
  const uint32_t t6 = __builtin_amdgcn_bitop3_b32(y4, X7, t2, 0x6a);
  const uint32_t t7 = y13 & y16;
  const uint32_t t9 = __builtin_amdgcn_bitop3_b32(y5, y1, t7, 0x6a);
  const uint32_t t11 = __builtin_amdgcn_bitop3_b32(y2, y7, t7, 0x6a);
  const uint32_t t12 = y9 & y11;
  const uint32_t t14 = __builtin_amdgcn_bitop3_b32(y14, y17, t12, 0x6a);
  const uint32_t t16 = __builtin_amdgcn_bitop3_b32(y8, y10, t12, 0x6a);
  const uint32_t t21 = __builtin_amdgcn_bitop3_b32(t4, t14, y20, 0x96);
  const uint32_t t22 = __builtin_amdgcn_bitop3_b32(t6, t16, y19, 0x96);
  const uint32_t t23 = __builtin_amdgcn_bitop3_b32(t9, t14, y21, 0x96);
  const uint32_t t24 = __builtin_amdgcn_bitop3_b32(t11, t16, y18, 0x96);
  const uint32_t t25 = t21 ^ t22;
  const uint32_t t26 = t21 & t23;
  const uint32_t t27 = t24 ^ t26;
  const uint32_t t29 = __builtin_amdgcn_bitop3_b32(t25, t27, t22, 0x6a);
  const uint32_t t30 = t23 ^ t24;
  const uint32_t t32 = __builtin_amdgcn_bitop3_b32(t22, t26, t30, 0x28);
  const uint32_t t33 = t32 ^ t24;
  const uint32_t t36 = __builtin_amdgcn_bitop3_b32(t24, t27, t33, 0x60);
  const uint32_t t37 = __builtin_amdgcn_bitop3_b32(t36, t23, t33, 0x96);
  const uint32_t t39 = __builtin_amdgcn_bitop3_b32(t29, t27, t36, 0x60);
  const uint32_t t40 = t25 ^ t39;
  const uint32_t t41 = t40 ^ t37;
  const uint32_t t42 = t29 ^ t33;
  const uint32_t t43 = t29 ^ t40;
  const uint32_t t44 = t33 ^ t37;
  const uint32_t t45 = t42 ^ t41;
  const uint32_t z2 = t33 & X7;
  const uint32_t z3 = t43 & y16;
  const uint32_t z4 = t40 & y1;
  const uint32_t z5 = t29 & y7;
  const uint32_t z7 = t45 & y17;
  const uint32_t z10 = t37 & y3;
  const uint32_t z12 = t43 & y13;
  const uint32_t z16 = t45 & y14;
  const uint32_t t46 = __builtin_amdgcn_bitop3_b32(t42, y9, z16, 0x6a);
  const uint32_t t47 = __builtin_amdgcn_bitop3_b32(z10, t33, y4, 0x78);
  const uint32_t t48 = __builtin_amdgcn_bitop3_b32(z5, t40, y5, 0x78);
  const uint32_t t49 = __builtin_amdgcn_bitop3_b32(t44, y12, z10, 0x6a);
  const uint32_t t52 = __builtin_amdgcn_bitop3_b32(z7, t41, y10, 0x78);
  const uint32_t t53 = __builtin_amdgcn_bitop3_b32(t44, y15, z3, 0x6a);
  const uint32_t t54 = __builtin_amdgcn_bitop3_b32(t42, y11, z7, 0x6a);
  const uint32_t t55 = __builtin_amdgcn_bitop3_b32(z16, t41, y8, 0x78);
  const uint32_t t57 = __builtin_amdgcn_bitop3_b32(z2, z12, t53, 0x96);
  const uint32_t t58 = z4 ^ t46;
  const uint32_t t59 = z3 ^ t54;
  const uint32_t t61 = __builtin_amdgcn_bitop3_b32(t29, y2, t57, 0x6a);
  const uint32_t t62 = t52 ^ t58;
  const uint32_t t63 = t49 ^ t58;
  const uint32_t t64 = z4 ^ t59;
  const uint32_t t65 = t61 ^ t62;
  const uint32_t t66 = __builtin_amdgcn_bitop3_b32(t37, y6, t63, 0x6a);
  const uint32_t s0 = t59 ^ t63;
  const uint32_t s6 = __builtin_amdgcn_bitop3_b32(z12, t48, t62, 0x96);
  const uint32_t s7 = __builtin_amdgcn_bitop3_b32(t48, t46, t57, 0x96);
  const uint32_t s3 = t53 ^ t66;
  const uint32_t s4 = __builtin_amdgcn_bitop3_b32(z2, z5, t66, 0x96);
  const uint32_t s5 = t47 ^ t65;
  const uint32_t s1 = t64 ^ s3;
  const uint32_t s2 = __builtin_amdgcn_bitop3_b32(t55, t64, t65, 0x96);
  b[7] = s0, b[6] = s1, b[5] = s2, b[4] = s3;
  b[3] = s4, b[2] = s5, b[1] = s6, b[0] = s7;
}

// key byte j of a round key given as 4 little-endian-loaded words (byte j of
// the key at bits 8*(j&3) of word j>>2)
__device__ __forceinline__ uint32_t kbyte(const uint32_t *kw, int j) { return (kw[j >> 2] >> (8 * (j & 3))) & 0xffu; }

// One round: S'(state ^ kprev) (all 16 bytes), ShiftRows, MixColumns if mix.
// kprev = the previous round's key (K0, or K'_r for r >= 1), little-endian
// words, wave-uniform.
template <bool MIX>
__device__ __forceinline__ void round(uint32_t (&st)[128], const uint32_t *kprev) {
#pragma unroll
  for (int j = 0; j < 16; ++j) sbox(&st[8 * j], kbyte(kprev, j));
  uint32_t o[128];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    // after ShiftRows, row r of column c is the byte at (row r, column c + r)
    const uint32_t *a[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) a[r] = &st[8 * (4 * ((c + r) & 3) + r)];
    if (!MIX) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int v = 0; v < 8; ++v) o[8 * (4 * c + r) + v] = a[r][v];
      continue;
    }
    // out_r = xtime(a_r ^ a_r+1) ^ (a0 ^ a1 ^ a2 ^ a3) ^ a_r
    uint32_t t[4][8], tot[8];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int v = 0; v < 8; ++v) t[r][v] = a[r][v] ^ a[(r + 1) & 3][v];
#pragma unroll
    for (int v = 0; v < 8; ++v) tot[v] = t[0][v] ^ t[2][v];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      uint32_t *q = &o[8 * (4 * c + r)];
      const uint32_t h = t[r][7];
      q[0] = x3(h, tot[0], a[r][0]);
      q[1] = x3(x3(t[r][0], h, tot[1]), a[r][1], 0u);
      q[2] = x3(t[r][1], tot[2], a[r][2]);
      q[3] = x3(x3(t[r][2], h, tot[3]), a[r][3], 0u);
      q[4] = x3(x3(t[r][3], h, tot[4]), a[r][4], 0u);
      q[5] = x3(t[r][4], tot[5], a[r][5]);
      q[6] = x3(t[r][5], tot[6], a[r][6]);
      q[7] = x3(t[r][6], tot[7], a[r][7]);
    }
  }
#pragma unroll
  for (int i = 0; i < 128; ++i) st[i] = o[i];
}

// 32x32 bit transpose: afterwards bit i of a[s] = bit s of the old a[i]
// (swapmove ladder; the 16- and 8-bit stages are byte moves).  Applied to the
// 32 registers of state bytes 4g..4g+3 it turns them into word g (memory
// order) of each of the 32 blocks.
__device__ __forceinline__ void transpose32(uint32_t *a) {
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const uint32_t x = a[k], y = a[k + 16];
    a[k] = __builtin_amdgcn_perm(y, x, 0x05040100u);
    a[k + 16] = __builtin_amdgcn_perm(y, x, 0x07060302u);
  }
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    if (k & 8) continue;
    const uint32_t x = a[k], y = a[k + 8];
    a[k] = __builtin_amdgcn_perm(y, x, 0x06020400u);
    a[k + 8] = __builtin_amdgcn_perm(y, x, 0x07030501u);
  }
  constexpr uint32_t M[3] = {0x0F0F0F0Fu, 0x33333333u, 0x55555555u};
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int j = 4 >> q;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
      if (k & j) continue;
      const uint32_t t = ((a[k] >> j) ^ a[k + j]) & M[q];
      a[k + j] ^= t;
      a[k] ^= t << j;
    }
  }
}

}  // namespace bs
}  // namespace espgpu
