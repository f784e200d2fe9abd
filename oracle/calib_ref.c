/*
 * calib_ref.c — TEST INFRASTRUCTURE ONLY (never shipped, never on the GPU box).
 *
 * Composes the reference's OWN compiled primitives (rijndael-alg-fst.c
 * rijndaelKeySetupEnc/rijndaelEncrypt, gfmult.c gf128_genmultable4/gf128_mul,
 * built from /root/reference into oracle/_ref by `make calib`) in swcr_gcm's
 * per-block order for an ESP record (cryptosoft.c:465-645: GHASH over AAD and
 * ciphertext one 16-byte gmac Update at a time, length block, tag = GHASH ^
 * E(J0), compare, then AES-ICM decrypt), and:
 *   1. checks that espref.c's oref_esp_decrypt produces the same plaintext
 *      and status on the same records (a pin of the restatement against the
 *      reference's primitives composed the reference's way);
 *   2. times both on one core: the ratio calibrates bench.py's cpu_baseline
 *      (the restatement, which can travel to the GPU box) against the
 *      reference's own arithmetic (which cannot).
 * Prints one JSON line.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/types.h>
#include <time.h>

#include <crypto/rijndael/rijndael.h>
#include "gfmult.h"

#include "espref.h"

struct refgcm {
	uint32_t ks[60];
	int nr;
	struct gf128table4 tbl;
};

static void ref_setkey(struct refgcm *k, const uint8_t *key, int klen)
{
	static const uint8_t zero[16];
	uint8_t h[16];

	k->nr = rijndaelKeySetupEnc(k->ks, key, klen * 8);
	rijndaelEncrypt(k->ks, k->nr, zero, h);
	gf128_genmultable4(gf128_read(h), &k->tbl);
}

static struct gf128 upd(struct gf128 v, const uint8_t *p, int n, struct gf128table *t)
{
	uint8_t b[16] = { 0 };

	memcpy(b, p, (size_t)n);
	return gf128_mul(gf128_add(v, gf128_read(b)), t);
}

/* ESP record: SPI|SN (8) | IV (8) | CT | ICV (16); nonce = salt || IV */
static int ref_record(const struct refgcm *k, const uint8_t salt[4], uint8_t *rec, int len)
{
	struct gf128table *t = (struct gf128table *)&k->tbl.tbls[0];
	const int ct = len - 32;
	uint8_t ctr[16], e[16], tag[16], lb[16] = { 0 };
	struct gf128 v = MAKE_GF128(0, 0);

	v = upd(v, rec, 8, t);                            /* AAD: SPI|SN */
	for (int o = 0; o < ct; o += 16)
		v = upd(v, rec + 16 + o, ct - o < 16 ? ct - o : 16, t);
	lb[7] = 64;                                       /* be64(aadlen*8) */
	lb[12] = (uint8_t)((ct * 8) >> 24);
	lb[13] = (uint8_t)((ct * 8) >> 16);
	lb[14] = (uint8_t)((ct * 8) >> 8);
	lb[15] = (uint8_t)(ct * 8);
	v = gf128_mul(gf128_add(v, gf128_read(lb)), t);
	memcpy(ctr, salt, 4);
	memcpy(ctr + 4, rec + 8, 8);
	ctr[12] = ctr[13] = ctr[14] = 0;
	ctr[15] = 1;
	rijndaelEncrypt(k->ks, k->nr, ctr, e);
	gf128_write(gf128_add(v, gf128_read(e)), tag);
	uint8_t d = 0;
	for (int i = 0; i < 16; i++)
		d |= tag[i] ^ rec[len - 16 + i];
	if (d)
		return 74;                                /* EBADMSG */
	for (int o = 0; o < ct; o += 16) {
		for (int i = 15; i >= 12 && ++ctr[i] == 0; i--)
			;
		rijndaelEncrypt(k->ks, k->nr, ctr, e);
		for (int i = 0; i < 16 && o + i < ct; i++)
			rec[16 + o + i] ^= e[i];
	}
	return 0;
}

static double now(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int main(int argc, char **argv)
{
	const int n = argc > 1 ? atoi(argv[1]) : 16384, len = 1480, reps = 3;
	uint8_t key[20];
	srand(11);
	for (int i = 0; i < 20; i++)
		key[i] = (uint8_t)rand();
	oref_sa *sa = oref_sa_new(OREF_CSP_MODE_AEAD, 0, key, 16, key + 16, NULL, 0, 16);
	struct refgcm rk;
	ref_setkey(&rk, key, 16);
	uint8_t *ct = malloc((size_t)n * len), *a = malloc((size_t)n * len), *b = malloc((size_t)n * len);
	for (long i = 0; i < (long)n * len; i++)
		ct[i] = (uint8_t)rand();
	for (int r = 0; r < n; r++) {
		uint8_t *p = ct + (size_t)r * len;
		p[4] = (uint8_t)(r >> 24); p[5] = (uint8_t)(r >> 16); p[6] = (uint8_t)(r >> 8); p[7] = (uint8_t)r;
		if (oref_esp_encrypt(sa, p, len, 0)) { printf("{\"error\": \"encrypt\"}\n"); return 1; }
		if (r % 97 == 5)
			p[len - 1] ^= 1;                  /* some tag failures */
	}
	double t_or = 1e30, t_ref = 1e30;
	int mism = 0, fails = 0;
	for (int rep = 0; rep < reps; rep++) {
		memcpy(a, ct, (size_t)n * len);
		memcpy(b, ct, (size_t)n * len);
		double t0 = now();
		int so[1];
		(void)so;
		for (int r = 0; r < n; r++)
			oref_esp_decrypt(sa, a + (size_t)r * len, len, 0);
		double t1 = now();
		for (int r = 0; r < n; r++)
			fails += ref_record(&rk, key + 16, b + (size_t)r * len, len) != 0;
		double t2 = now();
		if (t1 - t0 < t_or) t_or = t1 - t0;
		if (t2 - t1 < t_ref) t_ref = t2 - t1;
	}
	/* the oracle leaves EBADMSG records untouched, so do both */
	mism = memcmp(a, b, (size_t)n * len) != 0;
	/* AES block primitives alone (CBC decrypt of the ETA path uses the
	 * inverse cipher): reference vs restatement, same key, same blocks */
	uint32_t ek[60], dk[60], oek[60], odk[60];
	int nr = rijndaelKeySetupEnc(ek, key, 128);
	rijndaelKeySetupDec(dk, key, 128);
	oref_aes_setkey_enc(oek, key, 128);
	oref_aes_setkey_dec(odk, key, 128);
	uint8_t x[16] = { 0 }, y[16] = { 0 };
	const int nb = 1 << 20;
	double u0 = now();
	for (int i = 0; i < nb; i++) rijndaelEncrypt(ek, nr, x, x);
	double u1 = now();
	for (int i = 0; i < nb; i++) oref_aes_encrypt(oek, nr, y, y);
	double u2 = now();
	for (int i = 0; i < nb; i++) rijndaelDecrypt(dk, nr, x, x);
	double u3 = now();
	for (int i = 0; i < nb; i++) oref_aes_decrypt(odk, nr, y, y);
	double u4 = now();
	mism |= memcmp(x, y, 16) != 0;
	printf("{\"records\": %d, \"record_bytes\": %d, \"oracle_ns_per_record\": %.1f, "
	       "\"ref_primitives_ns_per_record\": %.1f, \"ratio_oracle_over_ref\": %.3f, "
	       "\"tag_failures\": %d, \"outputs_identical\": %s, "
	       "\"aes128_enc_ns_ref\": %.1f, \"aes128_enc_ns_oracle\": %.1f, "
	       "\"aes128_dec_ns_ref\": %.1f, \"aes128_dec_ns_oracle\": %.1f}\n",
	       n, len, t_or / n * 1e9, t_ref / n * 1e9, t_or / t_ref, fails / reps,
	       mism ? "false" : "true", (u1 - u0) / nb * 1e9, (u2 - u1) / nb * 1e9,
	       (u3 - u2) / nb * 1e9, (u4 - u3) / nb * 1e9);
	return mism;
}
