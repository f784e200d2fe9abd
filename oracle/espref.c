/*
 * espref.c — CPU restatement of FreeBSD's ESP bulk-crypto path (see espref.h).
 *
 * TEST INFRASTRUCTURE ONLY (parity oracle + "port" CPU baseline).  Not part of
 * the product; the product never links it.
 *
 * Written from the reference's algorithms, not copied: the AES tables are
 * generated from the field arithmetic instead of the constant arrays of
 * rijndael-alg-fst.c:57-733, and the GHASH reduction table is derived from
 * the polynomial rather than taken from gfmult.c:129.  The per-request
 * structure (context copy per op, 16-byte GHASH updates, verify-then-decrypt)
 * deliberately mirrors cryptosoft.c so that its timing is "cryptosoft-shaped".
 */
#include "espref.h"
#include "sha512_consts.h"

#include <errno.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------------ */
/* Byte helpers (GETU32/PUTU32 of rijndael_local.h, be64dec/enc of gfmult.h) */

static inline uint32_t ld_be32(const uint8_t *p)
{
	return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) |
	    ((uint32_t)p[2] << 8) | p[3];
}

static inline void st_be32(uint8_t *p, uint32_t v)
{
	p[0] = v >> 24; p[1] = v >> 16; p[2] = v >> 8; p[3] = v;
}

static inline uint64_t ld_be64(const uint8_t *p)
{
	return ((uint64_t)ld_be32(p) << 32) | ld_be32(p + 4);
}

static inline void st_be64(uint8_t *p, uint64_t v)
{
	st_be32(p, (uint32_t)(v >> 32));
	st_be32(p + 4, (uint32_t)v);
}

static inline uint32_t ror32(uint32_t v, int n)
{
	return n ? (v >> n) | (v << (32 - n)) : v;
}

/* ------------------------------------------------------------------------ */
/* Generated tables                                                          */

static uint8_t SBOX[256], ISBOX[256];
static uint32_t TE[4][256], TD[4][256];   /* Te0..Te3 / Td0..Td3 */
static uint16_t GHRED[16];                /* gfmult.c:129 reduction[] */
static pthread_once_t tables_once = PTHREAD_ONCE_INIT;

static uint8_t xtime8(uint8_t a)
{
	return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
}

static uint8_t gmul8(uint8_t a, uint8_t b)
{
	uint8_t r = 0;

	while (b) {
		if (b & 1)
			r ^= a;
		a = xtime8(a);
		b >>= 1;
	}
	return r;
}

static uint8_t rotl8(uint8_t v, int n)
{
	return (uint8_t)((v << n) | (v >> (8 - n)));
}

static void gen_tables(void)
{
	/* S-box: inverse in GF(2^8) mod x^8+x^4+x^3+x+1, then the affine map. */
	for (int x = 0; x < 256; x++) {
		uint8_t inv = 0;
		if (x != 0)
			for (int y = 1; y < 256; y++)
				if (gmul8((uint8_t)x, (uint8_t)y) == 1) {
					inv = (uint8_t)y;
					break;
				}
		uint8_t s = inv ^ rotl8(inv, 1) ^ rotl8(inv, 2) ^ rotl8(inv, 3) ^
		    rotl8(inv, 4) ^ 0x63;
		SBOX[x] = s;
		ISBOX[s] = (uint8_t)x;
	}
	/* Te0[x] = S[x].[02,01,01,03], Td0[x] = Si[x].[0e,09,0d,0b]
	 * (rijndael-alg-fst.c:43-55); TeN/TdN are byte rotations. */
	for (int x = 0; x < 256; x++) {
		uint8_t s = SBOX[x], si = ISBOX[x];
		uint32_t te = ((uint32_t)gmul8(s, 2) << 24) | ((uint32_t)s << 16) |
		    ((uint32_t)s << 8) | gmul8(s, 3);
		uint32_t td = ((uint32_t)gmul8(si, 14) << 24) |
		    ((uint32_t)gmul8(si, 9) << 16) | ((uint32_t)gmul8(si, 13) << 8) |
		    gmul8(si, 11);
		for (int k = 0; k < 4; k++) {
			TE[k][x] = ror32(te, 8 * k);
			TD[k][x] = ror32(td, 8 * k);
		}
	}
	/*
	 * GHASH x^4 reduction (gfmult.c:125-132): bit j of the four bits shifted
	 * out of v[1] has degree 127-j; times x^4 it becomes R*x^(3-j) with
	 * R = x^7+x^2+x+1, i.e. 0xE1 in the reflected top byte.
	 */
	for (int r = 0; r < 16; r++) {
		uint16_t v = 0;
		for (int j = 0; j < 4; j++)
			if (r & (1 << j))
				v ^= (uint16_t)(0xE100 >> (3 - j));
		GHRED[r] = v;
	}
}

static void init_tables(void)
{
	pthread_once(&tables_once, gen_tables);
}

/* ------------------------------------------------------------------------ */
/* AES (rijndael-alg-fst.c)                                                  */

static uint32_t subword(uint32_t w)
{
	return ((uint32_t)SBOX[w >> 24] << 24) | ((uint32_t)SBOX[(w >> 16) & 0xff] << 16) |
	    ((uint32_t)SBOX[(w >> 8) & 0xff] << 8) | SBOX[w & 0xff];
}

/* rijndaelKeySetupEnc, rijndael-alg-fst.c:735-821 (FIPS-197 5.2, any Nk). */
int oref_aes_setkey_enc(uint32_t rk[60], const uint8_t *key, int keybits)
{
	int nk = keybits / 32, nr, i;
	uint32_t rcon = 0x01000000;

	init_tables();
	if (keybits != 128 && keybits != 192 && keybits != 256)
		return 0;
	nr = nk + 6;
	for (i = 0; i < nk; i++)
		rk[i] = ld_be32(key + 4 * i);
	for (; i < 4 * (nr + 1); i++) {
		uint32_t t = rk[i - 1];
		if (i % nk == 0) {
			t = subword((t << 8) | (t >> 24)) ^ rcon;
			rcon = (uint32_t)xtime8((uint8_t)(rcon >> 24)) << 24;
		} else if (nk > 6 && i % nk == 4) {
			t = subword(t);
		}
		rk[i] = rk[i - nk] ^ t;
	}
	return nr;
}

static uint32_t inv_mixcol(uint32_t w)
{
	uint8_t a0 = w >> 24, a1 = w >> 16, a2 = w >> 8, a3 = w;
	uint8_t b0 = gmul8(a0, 14) ^ gmul8(a1, 11) ^ gmul8(a2, 13) ^ gmul8(a3, 9);
	uint8_t b1 = gmul8(a0, 9) ^ gmul8(a1, 14) ^ gmul8(a2, 11) ^ gmul8(a3, 13);
	uint8_t b2 = gmul8(a0, 13) ^ gmul8(a1, 9) ^ gmul8(a2, 14) ^ gmul8(a3, 11);
	uint8_t b3 = gmul8(a0, 11) ^ gmul8(a1, 13) ^ gmul8(a2, 9) ^ gmul8(a3, 14);
	return ((uint32_t)b0 << 24) | ((uint32_t)b1 << 16) | ((uint32_t)b2 << 8) | b3;
}

/* rijndaelKeySetupDec, rijndael-alg-fst.c:823-861: reverse the round order,
 * InvMixColumns on every round key but the first and last. */
int oref_aes_setkey_dec(uint32_t rk[60], const uint8_t *key, int keybits)
{
	int nr = oref_aes_setkey_enc(rk, key, keybits);

	for (int i = 0, j = 4 * nr; i < j; i += 4, j -= 4)
		for (int k = 0; k < 4; k++) {
			uint32_t t = rk[i + k];
			rk[i + k] = rk[j + k];
			rk[j + k] = t;
		}
	for (int i = 4; i < 4 * nr; i++)
		rk[i] = inv_mixcol(rk[i]);
	return nr;
}

/* rijndaelEncrypt, rijndael-alg-fst.c:863-1042 */
void oref_aes_encrypt(const uint32_t *rk, int nr, const uint8_t in[16], uint8_t out[16])
{
	/* scalar state words as rijndaelEncrypt keeps them (s0..s3 / t0..t3) */
	uint32_t s0 = ld_be32(in) ^ rk[0], s1 = ld_be32(in + 4) ^ rk[1];
	uint32_t s2 = ld_be32(in + 8) ^ rk[2], s3 = ld_be32(in + 12) ^ rk[3];
	uint32_t t0, t1, t2, t3;

	for (int r = 1; r < nr; r++) {
		rk += 4;
		t0 = TE[0][s0 >> 24] ^ TE[1][(s1 >> 16) & 0xff] ^ TE[2][(s2 >> 8) & 0xff] ^ TE[3][s3 & 0xff] ^ rk[0];
		t1 = TE[0][s1 >> 24] ^ TE[1][(s2 >> 16) & 0xff] ^ TE[2][(s3 >> 8) & 0xff] ^ TE[3][s0 & 0xff] ^ rk[1];
		t2 = TE[0][s2 >> 24] ^ TE[1][(s3 >> 16) & 0xff] ^ TE[2][(s0 >> 8) & 0xff] ^ TE[3][s1 & 0xff] ^ rk[2];
		t3 = TE[0][s3 >> 24] ^ TE[1][(s0 >> 16) & 0xff] ^ TE[2][(s1 >> 8) & 0xff] ^ TE[3][s2 & 0xff] ^ rk[3];
		s0 = t0; s1 = t1; s2 = t2; s3 = t3;
	}
	rk += 4;
#define SB4(a, b, c, d) (((uint32_t)SBOX[(a) >> 24] << 24) | ((uint32_t)SBOX[((b) >> 16) & 0xff] << 16) | \
	((uint32_t)SBOX[((c) >> 8) & 0xff] << 8) | SBOX[(d) & 0xff])
	st_be32(out, SB4(s0, s1, s2, s3) ^ rk[0]);
	st_be32(out + 4, SB4(s1, s2, s3, s0) ^ rk[1]);
	st_be32(out + 8, SB4(s2, s3, s0, s1) ^ rk[2]);
	st_be32(out + 12, SB4(s3, s0, s1, s2) ^ rk[3]);
#undef SB4
}

/* rijndaelDecrypt, rijndael-alg-fst.c:1044-1222 (equivalent inverse cipher) */
void oref_aes_decrypt(const uint32_t *rk, int nr, const uint8_t in[16], uint8_t out[16])
{
	uint32_t s0 = ld_be32(in) ^ rk[0], s1 = ld_be32(in + 4) ^ rk[1];
	uint32_t s2 = ld_be32(in + 8) ^ rk[2], s3 = ld_be32(in + 12) ^ rk[3];
	uint32_t t0, t1, t2, t3;

	for (int r = 1; r < nr; r++) {
		rk += 4;
		t0 = TD[0][s0 >> 24] ^ TD[1][(s3 >> 16) & 0xff] ^ TD[2][(s2 >> 8) & 0xff] ^ TD[3][s1 & 0xff] ^ rk[0];
		t1 = TD[0][s1 >> 24] ^ TD[1][(s0 >> 16) & 0xff] ^ TD[2][(s3 >> 8) & 0xff] ^ TD[3][s2 & 0xff] ^ rk[1];
		t2 = TD[0][s2 >> 24] ^ TD[1][(s1 >> 16) & 0xff] ^ TD[2][(s0 >> 8) & 0xff] ^ TD[3][s3 & 0xff] ^ rk[2];
		t3 = TD[0][s3 >> 24] ^ TD[1][(s2 >> 16) & 0xff] ^ TD[2][(s1 >> 8) & 0xff] ^ TD[3][s0 & 0xff] ^ rk[3];
		s0 = t0; s1 = t1; s2 = t2; s3 = t3;
	}
	rk += 4;
#define ISB4(a, b, c, d) (((uint32_t)ISBOX[(a) >> 24] << 24) | ((uint32_t)ISBOX[((b) >> 16) & 0xff] << 16) | \
	((uint32_t)ISBOX[((c) >> 8) & 0xff] << 8) | ISBOX[(d) & 0xff])
	st_be32(out, ISB4(s0, s3, s2, s1) ^ rk[0]);
	st_be32(out + 4, ISB4(s1, s0, s3, s2) ^ rk[1]);
	st_be32(out + 8, ISB4(s2, s1, s0, s3) ^ rk[2]);
	st_be32(out + 12, ISB4(s3, s2, s1, s0) ^ rk[3]);
#undef ISB4
}

/* ------------------------------------------------------------------------ */
/* GHASH (gfmult.c / gfmult.h): bit-reflected GF(2^128), v[0] = bytes 0-7   */
/* big-endian, 4-bit tables with bit-reversed indexes striped in 4 columns. */

typedef struct { uint64_t v[2]; } gf128;
struct gftab { uint32_t a[16], b[16], c[16], d[16]; };   /* gfmult.h:56-61 */
struct gftab4 { struct gftab t[4]; };                       /* h, h^2, h^3, h^4 */

static const uint8_t NIBREV[16] = {   /* bit reversal of a nibble */
	0, 8, 4, 12, 2, 10, 6, 14, 1, 9, 5, 13, 3, 11, 7, 15 };

static inline gf128 gf_read(const uint8_t *b)
{
	gf128 r = { { ld_be64(b), ld_be64(b + 8) } };
	return r;
}

static inline void gf_write(gf128 x, uint8_t *b)
{
	st_be64(b, x.v[0]);
	st_be64(b + 8, x.v[1]);
}

static inline gf128 gf_add(gf128 a, gf128 b)
{
	a.v[0] ^= b.v[0];
	a.v[1] ^= b.v[1];
	return a;
}

/* multiply by alpha (x): right shift with 0xE1 reduction, gfmult.c:44-55 */
static gf128 gf_mulalpha(gf128 v)
{
	uint64_t carry = v.v[1] & 1;

	v.v[1] = (v.v[1] >> 1) | (v.v[0] << 63);
	v.v[0] = (v.v[0] >> 1) ^ (carry ? (uint64_t)0xE1 << 56 : 0);
	return v;
}

/* gf128_genmultable, gfmult.c:62-84 */
static void gf_genmultable(gf128 h, struct gftab *t)
{
	gf128 m[16];

	m[0].v[0] = m[0].v[1] = 0;
	m[1] = h;
	for (int i = 2; i < 16; i += 2) {
		m[i] = gf_mulalpha(m[i / 2]);
		m[i + 1] = gf_add(m[i], h);
	}
	for (int i = 0; i < 16; i++) {
		t->a[NIBREV[i]] = (uint32_t)(m[i].v[0] >> 32);
		t->b[NIBREV[i]] = (uint32_t)m[i].v[0];
		t->c[NIBREV[i]] = (uint32_t)(m[i].v[1] >> 32);
		t->d[NIBREV[i]] = (uint32_t)m[i].v[1];
	}
}

static inline gf128 gf_row(const struct gftab *t, unsigned n)   /* readrow, :111-122 */
{
	gf128 r;

	n &= 15;
	r.v[0] = ((uint64_t)t->a[n] << 32) | t->b[n];
	r.v[1] = ((uint64_t)t->c[n] << 32) | t->d[n];
	return r;
}

static inline gf128 gf_shift4(gf128 x)   /* x * alpha^4 */
{
	unsigned red = x.v[1] & 15;

	x.v[1] = (x.v[1] >> 4) | (x.v[0] << 60);
	x.v[0] = (x.v[0] >> 4) ^ ((uint64_t)GHRED[red] << 48);
	return x;
}

/* gfmultword, gfmult.c:138-162: Horner over the 16 nibbles of one word,
 * highest-degree nibble (the low bits) first. */
static gf128 gf_multword(uint64_t w, gf128 x, const struct gftab *t)
{
	for (int i = 0; i < 16; i++, w >>= 4) {
		gf128 row = gf_row(t, (unsigned)w);
		x = gf_add(gf_shift4(x), row);
	}
	return x;
}

static gf128 gf_mul(gf128 v, const struct gftab *t)   /* gf128_mul, :219-229 */
{
	gf128 r = { { 0, 0 } };

	r = gf_multword(v.v[1], r, t);
	return gf_multword(v.v[0], r, t);
}

/* gfmultword4, gfmult.c:174-216: four words against h^4,h^3,h^2,h */
static gf128 gf_multword4(uint64_t wa, uint64_t wb, uint64_t wc, uint64_t wd,
    gf128 x, const struct gftab4 *t)
{
	for (int i = 0; i < 16; i++) {
		gf128 row = gf_add(gf_row(&t->t[3], (unsigned)wa),
		    gf_add(gf_row(&t->t[2], (unsigned)wb),
		    gf_add(gf_row(&t->t[1], (unsigned)wc), gf_row(&t->t[0], (unsigned)wd))));
		x = gf_add(gf_shift4(x), row);
		wa >>= 4; wb >>= 4; wc >>= 4; wd >>= 4;
	}
	return x;
}

/* gf128_mul4b, gfmult.c:262-275 */
static gf128 gf_mul4b(gf128 r, const uint8_t *v, const struct gftab4 *t)
{
	gf128 a = gf_add(r, gf_read(v)), b = gf_read(v + 16), c = gf_read(v + 32),
	    d = gf_read(v + 48), x = { { 0, 0 } };

	x = gf_multword4(a.v[1], b.v[1], c.v[1], d.v[1], x, t);
	return gf_multword4(a.v[0], b.v[0], c.v[0], d.v[0], x, t);
}

/* gf128_genmultable4, gfmult.c:89-106 */
static void gf_genmultable4(gf128 h, struct gftab4 *t)
{
	gf128 h2, h3, h4;

	gf_genmultable(h, &t->t[0]);
	h2 = gf_mul(h, &t->t[0]);
	gf_genmultable(h2, &t->t[1]);
	h3 = gf_mul(h, &t->t[1]);
	gf_genmultable(h3, &t->t[2]);
	h4 = gf_mul(h2, &t->t[1]);
	gf_genmultable(h4, &t->t[3]);
}

void oref_gf128_mul(const uint8_t h[16], const uint8_t x[16], uint8_t out[16])
{
	struct gftab t;

	init_tables();
	gf_genmultable(gf_read(h), &t);
	gf_write(gf_mul(gf_read(x), &t), out);
}

/* ------------------------------------------------------------------------ */
/* AES-GMAC context (gmac.h:42-48, gmac.c:39-131)                            */

struct gmac_ctx {
	struct gftab4 tbl;
	gf128 hash;
	uint32_t ks[60];
	uint8_t counter[16];
	int rounds;
};

static void gmac_setkey(struct gmac_ctx *g, const uint8_t *key, int klen)
{
	static const uint8_t zero[16];
	uint8_t hb[16];

	memset(g, 0, sizeof(*g));                       /* AES_GMAC_Init */
	g->rounds = oref_aes_setkey_enc(g->ks, key, klen * 8);
	oref_aes_encrypt(g->ks, g->rounds, zero, hb);   /* H = E_K(0^128) */
	gf_genmultable4(gf_read(hb), &g->tbl);
}

static void gmac_update(struct gmac_ctx *g, const uint8_t *p, unsigned len)
{
	gf128 v = g->hash;

	while (len > 0) {
		unsigned n;
		if (len >= 64) {
			n = 64;
			v = gf_mul4b(v, p, &g->tbl);
		} else if (len >= 16) {
			n = 16;
			v = gf_mul(gf_add(v, gf_read(p)), &g->tbl.t[0]);
		} else {
			uint8_t buf[16] = { 0 };
			n = len;
			memcpy(buf, p, n);
			v = gf_mul(gf_add(v, gf_read(buf)), &g->tbl.t[0]);
		}
		len -= n;
		p += n;
	}
	g->hash = v;
}

static void gmac_final(uint8_t tag[16], struct gmac_ctx *g)
{
	uint8_t e[16];

	g->counter[15] = 1;                             /* J0 = IV || 0^31 || 1 */
	oref_aes_encrypt(g->ks, g->rounds, g->counter, e);
	gf_write(gf_add(g->hash, gf_read(e)), tag);
}

/* ------------------------------------------------------------------------ */
/* AES-ICM in GCM mode (xform_aes_icm.c:126-194)                             */

struct icm_ctx {
	uint32_t ek[60];
	int nr;
	uint8_t block[16];
};

static void icm_gcm_reinit(struct icm_ctx *c, const uint8_t iv[12])
{
	memcpy(c->block, iv, 12);
	c->block[12] = c->block[13] = c->block[14] = 0;
	c->block[15] = 2;                               /* counter 1 is the tag's */
}

static void icm_crypt_last(struct icm_ctx *c, const uint8_t *in, uint8_t *out, int n)
{
	uint8_t ks[16];

	oref_aes_encrypt(c->ek, c->nr, c->block, ks);
	for (int i = 0; i < n; i++)
		out[i] = in[i] ^ ks[i];
}

static void icm_crypt(struct icm_ctx *c, const uint8_t *in, uint8_t *out)
{
	icm_crypt_last(c, in, out, 16);
	for (int i = 15; i >= 0; i--)                   /* full 128-bit increment */
		if (++c->block[i])
			break;
}

/* ------------------------------------------------------------------------ */
/* SHA-1 (sha1.c) and HMAC (crypto.c:413-457)                                */

struct sha1_ctx {
	uint32_t h[5];
	uint64_t nbytes;
	uint8_t buf[64];
	unsigned fill;
};

static void sha1_block(uint32_t h[5], const uint8_t *m)   /* sha1_step, sha1.c:94-176 */
{
	uint32_t w[80], a, b, c, d, e;

	for (int t = 0; t < 16; t++)
		w[t] = ld_be32(m + 4 * t);
	for (int t = 16; t < 80; t++) {
		uint32_t x = w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16];
		w[t] = (x << 1) | (x >> 31);
	}
	a = h[0]; b = h[1]; c = h[2]; d = h[3]; e = h[4];
	for (int t = 0; t < 80; t++) {
		uint32_t f, k;
		if (t < 20) {
			f = (b & c) | (~b & d); k = 0x5a827999;
		} else if (t < 40) {
			f = b ^ c ^ d; k = 0x6ed9eba1;
		} else if (t < 60) {
			f = (b & c) | (b & d) | (c & d); k = 0x8f1bbcdc;
		} else {
			f = b ^ c ^ d; k = 0xca62c1d6;
		}
		uint32_t tmp = ((a << 5) | (a >> 27)) + f + e + w[t] + k;
		e = d; d = c; c = (b << 30) | (b >> 2); b = a; a = tmp;
	}
	h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

static void sha1_init(struct sha1_ctx *s)   /* sha1_init, sha1.c:178-188 */
{
	static const uint32_t iv[5] = { 0x67452301, 0xefcdab89, 0x98badcfe,
	    0x10325476, 0xc3d2e1f0 };
	memcpy(s->h, iv, sizeof(iv));
	s->nbytes = 0;
	s->fill = 0;
}

static void sha1_update(struct sha1_ctx *s, const uint8_t *p, size_t n)   /* sha1_loop */
{
	s->nbytes += n;
	while (n > 0) {
		size_t k = 64 - s->fill;
		if (k > n)
			k = n;
		memcpy(s->buf + s->fill, p, k);
		s->fill += (unsigned)k;
		p += k;
		n -= k;
		if (s->fill == 64) {
			sha1_block(s->h, s->buf);
			s->fill = 0;
		}
	}
}

static void sha1_final(uint8_t out[20], struct sha1_ctx *s)   /* sha1_pad + sha1_result */
{
	uint64_t bits = s->nbytes * 8;
	uint8_t pad = 0x80, z = 0, lb[8];

	sha1_update(s, &pad, 1);
	while (s->fill != 56)
		sha1_update(s, &z, 1);
	st_be64(lb, bits);
	sha1_update(s, lb, 8);
	for (int i = 0; i < 5; i++)
		st_be32(out + 4 * i, s->h[i]);
}

void oref_sha1(const uint8_t *msg, size_t len, uint8_t out[20])
{
	struct sha1_ctx s;

	sha1_init(&s);
	sha1_update(&s, msg, len);
	sha1_final(out, &s);
}

/* hmac_init_pad, crypto.c:413-441 */
static void hmac_pad(const uint8_t *key, int klen, struct sha1_ctx *s, uint8_t padval)
{
	uint8_t k[64];

	memset(k, 0, sizeof(k));
	if (klen > 64) {
		oref_sha1(key, (size_t)klen, k);
		klen = 20;
	} else {
		memcpy(k, key, (size_t)klen);
	}
	for (int i = 0; i < 64; i++)
		k[i] ^= padval;
	sha1_init(s);
	sha1_update(s, k, 64);
}

void oref_hmac_sha1(const uint8_t *key, int klen, const uint8_t *msg, size_t len, uint8_t out[20])
{
	struct sha1_ctx i, o;
	uint8_t inner[20];

	hmac_pad(key, klen, &i, 0x36);
	hmac_pad(key, klen, &o, 0x5c);
	sha1_update(&i, msg, len);
	sha1_final(inner, &i);
	sha1_update(&o, inner, 20);
	sha1_final(out, &o);
}

/* ------------------------------------------------------------------------ */
/* SHA-256 (freebsd/crypto/sha2/sha256c.c: K[] :83, SHA256_Transform :135,   */
/* SHA256_Init :229) in the same context shape as SHA-1 above                 */

static const uint32_t SHA256_K[64] = {
	0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
	0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
	0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
	0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
	0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
	0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
	0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
	0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2,
};

static void sha256_block(uint32_t h[8], const uint8_t *m)
{
	uint32_t w[64], v[8];

	for (int t = 0; t < 16; t++)
		w[t] = ld_be32(m + 4 * t);
	for (int t = 16; t < 64; t++) {
		uint32_t s0 = ror32(w[t - 15], 7) ^ ror32(w[t - 15], 18) ^ (w[t - 15] >> 3);
		uint32_t s1 = ror32(w[t - 2], 17) ^ ror32(w[t - 2], 19) ^ (w[t - 2] >> 10);
		w[t] = w[t - 16] + s0 + w[t - 7] + s1;
	}
	memcpy(v, h, sizeof(v));
	for (int t = 0; t < 64; t++) {
		uint32_t S1 = ror32(v[4], 6) ^ ror32(v[4], 11) ^ ror32(v[4], 25);
		uint32_t ch = (v[4] & v[5]) ^ (~v[4] & v[6]);
		uint32_t t1 = v[7] + S1 + ch + SHA256_K[t] + w[t];
		uint32_t S0 = ror32(v[0], 2) ^ ror32(v[0], 13) ^ ror32(v[0], 22);
		uint32_t maj = (v[0] & v[1]) ^ (v[0] & v[2]) ^ (v[1] & v[2]);
		uint32_t t2 = S0 + maj;
		v[7] = v[6]; v[6] = v[5]; v[5] = v[4]; v[4] = v[3] + t1;
		v[3] = v[2]; v[2] = v[1]; v[1] = v[0]; v[0] = t1 + t2;
	}
	for (int i = 0; i < 8; i++)
		h[i] += v[i];
}

/* ------------------------------------------------------------------------ */
/* SHA-512 / SHA-384 (freebsd/crypto/sha2/sha512c.c: K[] :152, SHA512_Transform */
/* :196, SHA512_Init :440, SHA384_Init :493); 128-byte blocks, 64-bit words,  */
/* a 128-bit length field.  Constants: sha512_consts.h (FIPS 180-4).          */

static const uint64_t SHA512_K[80] = OREF_SHA512_K;

static uint64_t ror64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

static void sha512_block(uint64_t h[8], const uint8_t *m)
{
	uint64_t w[80], v[8];

	for (int t = 0; t < 16; t++)
		w[t] = ld_be64(m + 8 * t);
	for (int t = 16; t < 80; t++) {
		uint64_t s0 = ror64(w[t - 15], 1) ^ ror64(w[t - 15], 8) ^ (w[t - 15] >> 7);
		uint64_t s1 = ror64(w[t - 2], 19) ^ ror64(w[t - 2], 61) ^ (w[t - 2] >> 6);
		w[t] = w[t - 16] + s0 + w[t - 7] + s1;
	}
	memcpy(v, h, sizeof(v));
	for (int t = 0; t < 80; t++) {
		uint64_t S1 = ror64(v[4], 14) ^ ror64(v[4], 18) ^ ror64(v[4], 41);
		uint64_t ch = (v[4] & v[5]) ^ (~v[4] & v[6]);
		uint64_t t1 = v[7] + S1 + ch + SHA512_K[t] + w[t];
		uint64_t S0 = ror64(v[0], 28) ^ ror64(v[0], 34) ^ ror64(v[0], 39);
		uint64_t maj = (v[0] & v[1]) ^ (v[0] & v[2]) ^ (v[1] & v[2]);
		v[7] = v[6]; v[6] = v[5]; v[5] = v[4]; v[4] = v[3] + t1;
		v[3] = v[2]; v[2] = v[1]; v[1] = v[0]; v[0] = t1 + S0 + maj;
	}
	for (int i = 0; i < 8; i++)
		h[i] += v[i];
}

/* A hash context for any auth algorithm of an ETA session. */
struct hctx {
	int alg;                /* OREF_CRYPTO_SHA1_HMAC, _SHA2_256/384/512_HMAC */
	uint32_t h[8];          /* SHA-1 / SHA-256 state */
	uint64_t h64[8];        /* SHA-384 / SHA-512 state */
	uint64_t nbytes;
	uint8_t buf[128];
	unsigned fill;
};

static int wide(int alg) { return alg == OREF_CRYPTO_SHA2_384_HMAC || alg == OREF_CRYPTO_SHA2_512_HMAC; }
static int block_len(int alg) { return wide(alg) ? 128 : 64; }
static int hash_len(int alg)
{
	switch (alg) {
	case OREF_CRYPTO_SHA2_256_HMAC: return 32;
	case OREF_CRYPTO_SHA2_384_HMAC: return 48;
	case OREF_CRYPTO_SHA2_512_HMAC: return 64;
	default: return 20;
	}
}

static void h_init(struct hctx *c, int alg)
{
	static const uint32_t iv256[8] = { 0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
	    0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19 };
	static const uint64_t iv512[8] = OREF_SHA512_IV, iv384[8] = OREF_SHA384_IV;
	struct sha1_ctx s1;

	memset(c, 0, sizeof(*c));
	c->alg = alg;
	if (alg == OREF_CRYPTO_SHA2_256_HMAC) {
		memcpy(c->h, iv256, sizeof(iv256));
	} else if (alg == OREF_CRYPTO_SHA2_384_HMAC) {
		memcpy(c->h64, iv384, sizeof(iv384));
	} else if (alg == OREF_CRYPTO_SHA2_512_HMAC) {
		memcpy(c->h64, iv512, sizeof(iv512));
	} else {
		sha1_init(&s1);
		memcpy(c->h, s1.h, sizeof(s1.h));
	}
}

static void h_block(struct hctx *c, const uint8_t *m)
{
	if (wide(c->alg))
		sha512_block(c->h64, m);
	else if (c->alg == OREF_CRYPTO_SHA2_256_HMAC)
		sha256_block(c->h, m);
	else
		sha1_block(c->h, m);
}

static void h_update(struct hctx *c, const uint8_t *p, size_t n)
{
	const unsigned bl = (unsigned)block_len(c->alg);

	c->nbytes += n;
	while (n > 0) {
		size_t k = bl - c->fill;
		if (k > n)
			k = n;
		memcpy(c->buf + c->fill, p, k);
		c->fill += (unsigned)k;
		p += k;
		n -= k;
		if (c->fill == bl) {
			h_block(c, c->buf);
			c->fill = 0;
		}
	}
}

/* padding: 0x80, zeros, then the bit length in 8 (SHA-1/256) or 16 bytes */
static void h_final(uint8_t *out, struct hctx *c)
{
	const unsigned bl = (unsigned)block_len(c->alg), lf = wide(c->alg) ? 16 : 8;
	uint64_t bits = c->nbytes * 8;
	uint8_t pad = 0x80, z = 0, lb[16];

	h_update(c, &pad, 1);
	while (c->fill != bl - lf)
		h_update(c, &z, 1);
	memset(lb, 0, sizeof(lb));
	st_be64(lb + lf - 8, bits);
	h_update(c, lb, lf);
	if (wide(c->alg)) {
		for (int i = 0; i < hash_len(c->alg) / 8; i++) {
			st_be32(out + 8 * i, (uint32_t)(c->h64[i] >> 32));
			st_be32(out + 8 * i + 4, (uint32_t)c->h64[i]);
		}
	} else {
		for (int i = 0; i < hash_len(c->alg) / 4; i++)
			st_be32(out + 4 * i, c->h[i]);
	}
}

void oref_sha256(const uint8_t *msg, size_t len, uint8_t out[32])
{
	struct hctx c;

	h_init(&c, OREF_CRYPTO_SHA2_256_HMAC);
	h_update(&c, msg, len);
	h_final(out, &c);
}

/* hmac_init_pad (crypto.c:413-441) for any hash: the key padded to the
 * hash's block (64 or 128 bytes), hashed first when longer */
static void h_hmac_pad(const uint8_t *key, int klen, struct hctx *c, int alg, uint8_t padval)
{
	const int bl = block_len(alg);
	uint8_t k[128];

	memset(k, 0, sizeof(k));
	if (klen > bl) {
		struct hctx t;
		h_init(&t, alg);
		h_update(&t, key, (size_t)klen);
		h_final(k, &t);
	} else {
		memcpy(k, key, (size_t)klen);
	}
	for (int i = 0; i < bl; i++)
		k[i] ^= padval;
	h_init(c, alg);
	h_update(c, k, (size_t)bl);
}

void oref_hash(int alg, const uint8_t *msg, size_t len, uint8_t *out)
{
	struct hctx c;

	h_init(&c, alg);
	h_update(&c, msg, len);
	h_final(out, &c);
}

void oref_hmac(int alg, const uint8_t *key, int klen, const uint8_t *msg, size_t len, uint8_t *out)
{
	struct hctx i, o;
	uint8_t inner[64];

	h_hmac_pad(key, klen, &i, alg, 0x36);
	h_hmac_pad(key, klen, &o, alg, 0x5c);
	h_update(&i, msg, len);
	h_final(inner, &i);
	h_update(&o, inner, (size_t)hash_len(alg));
	h_final(out, &o);
}

/* AES-ICM over data from an explicit 16-byte initial counter block
 * (aes_icm_reinit + aes_icm_crypt/_last, xform_aes_icm.c:113-181) */
void oref_aes_ctr(const uint8_t *key, int klen, const uint8_t ctr[16], uint8_t *data, int len)
{
	struct icm_ctx c;
	int resid;

	init_tables();
	c.nr = oref_aes_setkey_enc(c.ek, key, klen * 8);
	memcpy(c.block, ctr, 16);
	for (resid = len; resid >= 16; resid -= 16, data += 16)
		icm_crypt(&c, data, data);
	if (resid > 0)
		icm_crypt_last(&c, data, data, resid);
}

/* ------------------------------------------------------------------------ */
/* Sessions (cryptosoft.c:976-1128, 1309-1409)                               */

struct oref_sa {
	int mode, flags, mlen, klen;
	int calg, aalg;         /* ETA: AES_CBC or AES_ICM; SHA1_HMAC or SHA2_256_HMAC */
	uint8_t salt[4];
	/* GCM: sw_ictx (AES-GMAC ctx) + sw_kschedule (ICM ctx) */
	struct gmac_ctx gictx;
	struct icm_ctx icm;
	/* ETA: rijndael ctx + HMAC ipad/opad contexts */
	uint32_t ek[60], dk[60];
	int nr;
	struct hctx ictx, octx;
};

oref_sa *oref_sa_new(int mode, int flags, const uint8_t *ckey, int cklen,
    const uint8_t salt[4], const uint8_t *akey, int aklen, int mlen)
{
	return oref_sa_new2(mode, flags, mode == OREF_CSP_MODE_AEAD ? OREF_CRYPTO_AES_NIST_GCM_16 :
	    OREF_CRYPTO_AES_CBC, ckey, cklen, salt, OREF_CRYPTO_SHA1_HMAC, akey, aklen, mlen);
}

oref_sa *oref_sa_new2(int mode, int flags, int calg, const uint8_t *ckey, int cklen,
    const uint8_t salt[4], int aalg, const uint8_t *akey, int aklen, int mlen)
{
	oref_sa *sa;

	init_tables();
	if (calg == OREF_CRYPTO_NULL_CBC ? cklen != 0 : (cklen != 16 && cklen != 24 && cklen != 32))
		return NULL;
	sa = calloc(1, sizeof(*sa));
	if (sa == NULL)
		return NULL;
	sa->mode = mode;
	sa->flags = flags;
	sa->klen = cklen;
	if (mode == OREF_CSP_MODE_AEAD) {               /* swcr_setup_gcm :1087 */
		sa->mlen = (mlen == 0) ? 16 : mlen;
		gmac_setkey(&sa->gictx, ckey, cklen);
		sa->icm.nr = oref_aes_setkey_enc(sa->icm.ek, ckey, cklen * 8);
		if (salt)
			memcpy(sa->salt, salt, 4);
	} else if (mode == OREF_CSP_MODE_ETA || mode == OREF_CSP_MODE_CIPHER) {   /* swcr_setup_cipher/auth */
		const int auth = mode == OREF_CSP_MODE_ETA;
		if ((calg != OREF_CRYPTO_AES_CBC && calg != OREF_CRYPTO_AES_ICM && calg != OREF_CRYPTO_NULL_CBC) ||
		    (auth && aalg != OREF_CRYPTO_SHA1_HMAC && aalg != OREF_CRYPTO_SHA2_256_HMAC &&
		     aalg != OREF_CRYPTO_SHA2_384_HMAC && aalg != OREF_CRYPTO_SHA2_512_HMAC)) {
			free(sa);
			return NULL;
		}
		sa->calg = calg;
		sa->aalg = auth ? aalg : 0;
		sa->mlen = !auth ? 0 : (mlen == 0) ? hash_len(aalg) : mlen;   /* :1013-1018 */
		if (calg != OREF_CRYPTO_NULL_CBC) {
			sa->nr = oref_aes_setkey_enc(sa->ek, ckey, cklen * 8);
			oref_aes_setkey_dec(sa->dk, ckey, cklen * 8);
		}
		if (salt)
			memcpy(sa->salt, salt, 4);      /* AES-ICM nonce (RFC 3686) */
		if (auth) {
			h_hmac_pad(akey, aklen, &sa->ictx, aalg, 0x36);
			h_hmac_pad(akey, aklen, &sa->octx, aalg, 0x5c);
		}
	} else {
		free(sa);
		return NULL;
	}
	return sa;
}

void oref_sa_free(oref_sa *sa)
{
	free(sa);
}

/* ------------------------------------------------------------------------ */
/* swcr_gcm on a contiguous buffer (cryptosoft.c:465-645)                    */

struct req {
	uint8_t *buf;
	const uint8_t *aad;     /* separate AAD or NULL (then aad_start) */
	int aad_start, aad_len;
	int payload_start, payload_len, digest_start, iv_start;
	uint8_t iv[16];
	uint8_t esn[4];
	int encrypt;
};

static int swcr_gcm_c(const oref_sa *sa, struct req *r)
{
	struct gmac_ctx ctx;
	struct icm_ctx icm;
	uint8_t blk[16], tag[16], lenblk[16];
	int resid, len;

	memcpy(&ctx, &sa->gictx, sizeof(ctx));          /* bcopy(sw_ictx) :485 */
	memcpy(&icm, &sa->icm, sizeof(icm));
	memcpy(ctx.counter, r->iv, 12);                 /* AES_GMAC_Reinit */

	if (r->aad != NULL) {                           /* :505-515 */
		len = r->aad_len & ~15;
		if (len)
			gmac_update(&ctx, r->aad, (unsigned)len);
		if (r->aad_len != len) {
			memset(blk, 0, 16);
			memcpy(blk, r->aad + len, (size_t)(r->aad_len - len));
			gmac_update(&ctx, blk, 16);
		}
	} else {                                        /* :517-537 */
		const uint8_t *p = r->buf + r->aad_start;
		len = r->aad_len & ~15;
		if (len)
			gmac_update(&ctx, p, (unsigned)len);
		if (r->aad_len != len) {
			memset(blk, 0, 16);
			memcpy(blk, p + len, (size_t)(r->aad_len - len));
			gmac_update(&ctx, blk, 16);
		}
	}

	icm_gcm_reinit(&icm, r->iv);                    /* :540 */
	uint8_t *p = r->buf + r->payload_start;
	for (resid = r->payload_len; resid >= 16; resid -= 16, p += 16) {   /* :550-572 */
		if (r->encrypt) {
			icm_crypt(&icm, p, p);
			gmac_update(&ctx, p, 16);
		} else {
			gmac_update(&ctx, p, 16);
		}
	}
	if (resid > 0) {                                /* :573-580 */
		memcpy(blk, p, (size_t)resid);
		if (r->encrypt) {
			icm_crypt_last(&icm, blk, blk, resid);
			memcpy(p, blk, (size_t)resid);
		}
		gmac_update(&ctx, blk, (unsigned)resid);
	}
	memset(lenblk, 0, 16);                          /* :583-588 */
	st_be32(lenblk + 4, (uint32_t)r->aad_len * 8);
	st_be32(lenblk + 12, (uint32_t)r->payload_len * 8);
	gmac_update(&ctx, lenblk, 16);
	gmac_final(tag, &ctx);

	if (!r->encrypt) {                              /* :593-633 */
		uint8_t diff = 0;
		for (int i = 0; i < sa->mlen; i++)
			diff |= tag[i] ^ r->buf[r->digest_start + i];
		if (diff != 0)
			return EBADMSG;
		p = r->buf + r->payload_start;
		for (resid = r->payload_len; resid > 16; resid -= 16, p += 16)
			icm_crypt(&icm, p, p);
		if (resid > 0)
			icm_crypt_last(&icm, p, p, resid);
	} else {
		memcpy(r->buf + r->digest_start, tag, (size_t)sa->mlen);   /* :636 */
	}
	return 0;
}

/* swcr_encdec for AES-CBC / AES-ICM on a contiguous buffer (cryptosoft.c:101-284) */
static int swcr_encdec_cbc(const oref_sa *sa, struct req *r)
{
	uint8_t iv[16], niv[16];
	uint8_t *p = r->buf + r->payload_start;

	if (sa->calg == OREF_CRYPTO_AES_ICM) {          /* stream cipher: any length */
		struct icm_ctx c;
		int resid;

		memcpy(c.ek, sa->ek, sizeof(c.ek));
		c.nr = sa->nr;
		memcpy(c.block, r->iv, 16);             /* aes_icm_reinit, IV_SEPARATE */
		for (resid = r->payload_len; resid >= 16; resid -= 16, p += 16)
			icm_crypt(&c, p, p);
		if (resid > 0)
			icm_crypt_last(&c, p, p, resid);
		return 0;
	}
	if (r->payload_len % 16)
		return EINVAL;
	memcpy(iv, r->buf + r->iv_start, 16);           /* crypto_read_iv */
	for (int resid = r->payload_len; resid >= 16; resid -= 16, p += 16) {
		if (r->encrypt) {
			for (int i = 0; i < 16; i++)
				p[i] ^= iv[i];
			oref_aes_encrypt(sa->ek, sa->nr, p, p);
			memcpy(iv, p, 16);
		} else {
			memcpy(niv, p, 16);             /* keep C_i for the next block */
			oref_aes_decrypt(sa->dk, sa->nr, p, p);
			for (int i = 0; i < 16; i++)
				p[i] ^= iv[i];
			memcpy(iv, niv, 16);
		}
	}
	return 0;
}

/* swcr_authcompute for HMAC-SHA1 / HMAC-SHA2 (cryptosoft.c:317-382) */
static int swcr_authcompute_c(const oref_sa *sa, struct req *r)
{
	struct hctx ctx;
	uint8_t a[64];

	memcpy(&ctx, &sa->ictx, sizeof(ctx));
	h_update(&ctx, r->buf + r->aad_start, (size_t)r->aad_len);
	h_update(&ctx, r->buf + r->payload_start, (size_t)r->payload_len);
	if (sa->flags & OREF_CSP_F_ESN)
		h_update(&ctx, r->esn, 4);
	h_final(a, &ctx);
	memcpy(&ctx, &sa->octx, sizeof(ctx));
	h_update(&ctx, a, (size_t)hash_len(sa->aalg));
	h_final(a, &ctx);
	if (!r->encrypt) {
		uint8_t diff = 0;
		for (int i = 0; i < sa->mlen; i++)
			diff |= a[i] ^ r->buf[r->digest_start + i];
		return diff ? EBADMSG : 0;
	}
	memcpy(r->buf + r->digest_start, a, (size_t)sa->mlen);
	return 0;
}

static int swcr_eta_c(const oref_sa *sa, struct req *r)   /* cryptosoft.c:874-888 */
{
	int e;

	if (sa->mode == OREF_CSP_MODE_CIPHER)            /* swcr_encdec / swcr_null, :1339-1350 */
		return sa->calg == OREF_CRYPTO_NULL_CBC ? 0 : swcr_encdec_cbc(sa, r);
	if (sa->calg == OREF_CRYPTO_NULL_CBC)            /* digest only, :1394-1398 */
		return swcr_authcompute_c(sa, r);
	if (r->encrypt) {
		e = swcr_encdec_cbc(sa, r);
		return e ? e : swcr_authcompute_c(sa, r);
	}
	e = swcr_authcompute_c(sa, r);
	return e ? e : swcr_encdec_cbc(sa, r);
}

/* Build the request as esp_input does (xform_esp.c:296-461, skip = 0) and
 * as esp_output does for the encrypt direction (xform_esp.c:673-961). */
static int esp_process(const oref_sa *sa, uint8_t *esp, int len, uint32_t esn_hi, int encrypt)
{
	struct req r;
	uint8_t aadbuf[12];
	int gcm = (sa->mode == OREF_CSP_MODE_AEAD);
	int ctr = !gcm && sa->calg == OREF_CRYPTO_AES_ICM;
	int null = !gcm && sa->calg == OREF_CRYPTO_NULL_CBC;
	/* RFC 4106 / 3686: 8-byte IV; CBC 16 (txform->ivsize); NULL none */
	int ivlen = (gcm || ctr) ? 8 : null ? 0 : 16, hlen = 8 + ivlen;
	/* ICV bytes = the session's sw_mlen (cryptosoft.c:1112-1117): 16 for GCM
	 * and 12 for HMAC-SHA1-96 as ESP sets them up (xform_ah_authsize), 8/12
	 * for a truncated GCM session, 20 for an untruncated HMAC-SHA1 one */
	int alen = sa->mlen;
	int plen = len - hlen - alen;

	/* :279-324: payload a multiple of the cipher's blocksize (CBC 16, CTR 1,
	 * NULL 4) and records 4-byte multiples */
	if ((len & 3) || plen <= 0 || (!gcm && !ctr && !null && (plen & 15)))
		return EINVAL;
	memset(&r, 0, sizeof(r));
	r.buf = esp;
	r.encrypt = encrypt;
	r.payload_start = hlen;
	r.payload_len = plen;
	r.digest_start = len - alen;
	st_be32(r.esn, esn_hi);                         /* seqh = htonl(seqh) */
	if (gcm) {
		r.aad_len = 8;                          /* RFC 4106: SPI + SN */
		if (sa->flags & OREF_CSP_F_SEPARATE_AAD) {   /* :375-397 */
			memcpy(aadbuf, esp, 4);
			memcpy(aadbuf + 4, r.esn, 4);
			memcpy(aadbuf + 8, esp + 4, 4);
			r.aad = aadbuf;
			r.aad_len = 12;
		}
		memcpy(r.iv, sa->salt, 4);              /* :453-455 */
		memcpy(r.iv + 4, esp + 8, 8);
		return swcr_gcm_c(sa, &r);
	}
	r.aad_start = 0;
	r.aad_len = hlen;                               /* :369 */
	r.iv_start = hlen - ivlen;                      /* :460-461 */
	if (ctr) {                                      /* :453-458: salt | IV | be32(1) */
		memcpy(r.iv, sa->salt, 4);
		memcpy(r.iv + 4, esp + 8, 8);
		st_be32(r.iv + 12, 1);
	}
	return swcr_eta_c(sa, &r);
}

int oref_esp_decrypt(const oref_sa *sa, uint8_t *esp, int len, uint32_t esn_hi)
{
	return esp_process(sa, esp, len, esn_hi, 0);
}

int oref_esp_encrypt(const oref_sa *sa, uint8_t *esp, int len, uint32_t esn_hi)
{
	return esp_process(sa, esp, len, esn_hi, 1);
}

int oref_gcm(const uint8_t *key, int klen, const uint8_t iv[12],
    const uint8_t *aad, int aadlen, uint8_t *data, int len,
    uint8_t *tag, int mlen, int encrypt)
{
	oref_sa *sa = oref_sa_new(OREF_CSP_MODE_AEAD, 0, key, klen, NULL, NULL, 0, mlen);
	struct req r;
	uint8_t *buf;
	int e;

	if (sa == NULL)
		return EINVAL;
	/* contiguous [data | tag] so digest_start addresses the tag */
	buf = malloc((size_t)len + 16);
	memcpy(buf, data, (size_t)len);
	memcpy(buf + len, tag, 16);
	memset(&r, 0, sizeof(r));
	r.buf = buf;
	r.aad = aadlen ? aad : (const uint8_t *)"";
	r.aad_len = aadlen;
	r.payload_start = 0;
	r.payload_len = len;
	r.digest_start = len;
	r.encrypt = encrypt;
	memcpy(r.iv, iv, 12);
	e = swcr_gcm_c(sa, &r);
	if (e == 0) {
		memcpy(data, buf, (size_t)len);
		if (encrypt)
			memcpy(tag, buf + len, (size_t)sa->mlen);
	}
	free(buf);
	oref_sa_free(sa);
	return e;
}

/* Generic AES-CBC + HMAC-SHA1 EtA (swcr_eta) on [aad | payload | digest]. */
int oref_eta(const uint8_t *ckey, int cklen, const uint8_t *akey, int aklen,
    const uint8_t iv[16], const uint8_t *aad, int aadlen, uint8_t *data, int len,
    uint8_t *digest, int mlen, int encrypt)
{
	oref_sa *sa = oref_sa_new(OREF_CSP_MODE_ETA, 0, ckey, cklen, NULL, akey, aklen, mlen);
	struct req r;
	uint8_t *buf;
	int e;

	if (sa == NULL)
		return EINVAL;
	buf = malloc((size_t)(16 + aadlen + len + 20));
	memcpy(buf, iv, 16);
	memcpy(buf + 16, aad, (size_t)aadlen);
	memcpy(buf + 16 + aadlen, data, (size_t)len);
	memcpy(buf + 16 + aadlen + len, digest, 20);
	memset(&r, 0, sizeof(r));
	r.buf = buf;
	r.iv_start = 0;
	r.aad_start = 16;
	r.aad_len = aadlen;
	r.payload_start = 16 + aadlen;
	r.payload_len = len;
	r.digest_start = 16 + aadlen + len;
	r.encrypt = encrypt;
	e = swcr_eta_c(sa, &r);
	if (e == 0) {
		memcpy(data, buf + r.payload_start, (size_t)len);
		if (encrypt)
			memcpy(digest, buf + r.digest_start, (size_t)sa->mlen);
	}
	free(buf);
	oref_sa_free(sa);
	return e;
}

/* ------------------------------------------------------------------------ */
/* Multi-threaded batch driver (CPU baseline)                                */

struct job {
	oref_sa *const *sas;
	uint8_t *arena;
	const uint32_t *off4;
	const uint16_t *len, *sa_idx;
	const uint32_t *esn_hi;
	uint8_t *status;
	long lo, hi;
	int encrypt;
};

static void *worker(void *arg)
{
	struct job *j = arg;

	for (long i = j->lo; i < j->hi; i++) {
		uint32_t e = j->esn_hi ? j->esn_hi[i] : 0;
		int rc = esp_process(j->sas[j->sa_idx[i]], j->arena + (size_t)j->off4[i] * 4,
		    j->len[i], e, j->encrypt);
		if (j->status)
			j->status[i] = (uint8_t)rc;
	}
	return NULL;
}

static double now_s(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static double run_batch(oref_sa *const *sas, uint8_t *arena, const uint32_t *off4,
    const uint16_t *len, const uint16_t *sa_idx, const uint32_t *esn_hi,
    uint8_t *status, long n, int nthreads, int encrypt)
{
	pthread_t th[256];
	struct job jobs[256];
	double t0, t1;

	init_tables();
	if (nthreads < 1)
		nthreads = 1;
	if (nthreads > 256)
		nthreads = 256;
	for (int t = 0; t < nthreads; t++) {
		jobs[t] = (struct job){ sas, arena, off4, len, sa_idx, esn_hi, status,
		    n * t / nthreads, n * (t + 1) / nthreads, encrypt };
	}
	t0 = now_s();
	if (nthreads == 1) {
		worker(&jobs[0]);
	} else {
		for (int t = 0; t < nthreads; t++)
			pthread_create(&th[t], NULL, worker, &jobs[t]);
		for (int t = 0; t < nthreads; t++)
			pthread_join(th[t], NULL);
	}
	t1 = now_s();
	return t1 - t0;
}

double oref_batch_decrypt(oref_sa *const *sas, uint8_t *arena, const uint32_t *off4,
    const uint16_t *len, const uint16_t *sa_idx, const uint32_t *esn_hi,
    uint8_t *status, long n, int nthreads)
{
	return run_batch(sas, arena, off4, len, sa_idx, esn_hi, status, n, nthreads, 0);
}

double oref_batch_encrypt(oref_sa *const *sas, uint8_t *arena, const uint32_t *off4,
    const uint16_t *len, const uint16_t *sa_idx, const uint32_t *esn_hi,
    long n, int nthreads)
{
	return run_batch(sas, arena, off4, len, sa_idx, esn_hi, NULL, n, nthreads, 1);
}

/* ---- replay window: freebsd/netipsec/ipsec.c:1177-1436 -------------------
 * Bit b of the window is bit (b & 31) of word (b >> 5) & (bitmap_size - 1)
 * (IPSEC_REDUNDANT_BIT_SHIFTS 5, IPSEC_BITMAP_INDEX_MASK, :1177-1180); the
 * window spans wsize * 8 sequence numbers below and including `last`. */
static int rp_check_window(const oref_replay *r, uint64_t seq)      /* :1191-1201 */
{
	return (r->bitmap[(seq >> 5) & (r->bitmap_size - 1)] >> (seq & 31)) & 1u;
}

static void rp_advance_window(const oref_replay *r, uint64_t seq)   /* :1203-1221 */
{
	uint64_t cur = r->last >> 5, idx = seq >> 5, diff = idx - cur, i;
	if (diff > r->bitmap_size)
		diff = r->bitmap_size;
	for (i = 0; i < diff; i++)
		r->bitmap[(i + cur + 1) & (r->bitmap_size - 1)] = 0;
}

static void rp_set_window(const oref_replay *r, uint64_t seq)       /* :1223-1232 */
{
	r->bitmap[(seq >> 5) & (r->bitmap_size - 1)] |= 1u << (seq & 31);
}

int oref_chkreplay(uint32_t seq, uint32_t *seqhigh, oref_replay *r)  /* :1248-1331 */
{
	uint32_t window, tl, th, bl;
	if (r->wsize == 0)
		return 1;
	if (seq == 0 && r->last == 0)
		return 0;
	window = r->wsize << 3;
	tl = (uint32_t)r->last;
	th = (uint32_t)(r->last >> 32);
	bl = tl - window + 1;
	if ((tl >= window - 1 && seq >= bl) || (tl < window - 1 && seq < bl)) {
		*seqhigh = th;
		if (seq <= tl && rp_check_window(r, seq))
			return 0;
		return 1;
	}
	if (tl == 0xffffffffu && !(r->flags & OREF_REPLAY_ESN)) {
		r->overflow++;
		if (!(r->flags & OREF_REPLAY_CYCSEQ))
			return 0;
	}
	if (tl < window - 1 && seq >= bl) {
		if (th == 0)
			return 0;
		*seqhigh = th - 1;
		if (rp_check_window(r, seq))
			return 0;
		return 1;
	}
	*seqhigh = th + 1;
	if (th + 1 == 0) {
		r->overflow++;
		if (!(r->flags & OREF_REPLAY_CYCSEQ))
			return 0;
	}
	return 1;
}

int oref_updatereplay(uint32_t seq, oref_replay *r)                   /* :1338-1436 */
{
	uint32_t window, tl, th, bl, seqh;
	if (r->wsize == 0)
		return 0;
	if (seq == 0 && r->last == 0)
		return 1;
	window = r->wsize << 3;
	tl = (uint32_t)r->last;
	th = (uint32_t)(r->last >> 32);
	bl = tl - window + 1;
	if ((tl >= window - 1 && seq >= bl) || (tl < window - 1 && seq < bl)) {
		seqh = th;
		if (seq <= tl) {
			if (rp_check_window(r, seq))
				return 1;
			rp_set_window(r, seq);
		} else {
			rp_advance_window(r, ((uint64_t)seqh << 32) | seq);
			rp_set_window(r, seq);
			r->last = ((uint64_t)seqh << 32) | seq;
		}
		r->count++;
		return 0;
	}
	if (!(r->flags & OREF_REPLAY_ESN))
		return 1;
	if (tl < window - 1 && seq >= bl) {
		if (th == 0)
			return 1;
		if (rp_check_window(r, seq))
			return 1;
		rp_set_window(r, seq);
		r->count++;
		return 0;
	}
	seqh = th + 1;
	if (seqh == 0)
		return 1;
	rp_advance_window(r, ((uint64_t)seqh << 32) | seq);
	rp_set_window(r, seq);
	r->last = ((uint64_t)seqh << 32) | seq;
	r->count++;
	return 0;
}
