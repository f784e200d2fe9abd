/* The whole F-Stack binding on the GPU: kernel-domain driver (ff_gpucrypto.c
 * over the kmock KPI) -> host-domain shim (ff_gpucrypto_host.c) ->
 * libespgpu.so.  The staging area is configured small (4 records, one slot)
 * so a burst of 6 requests makes process() answer ERESTART: the framework
 * must see ERESTART (-1), queue and later retry.  ESP AES-GCM records are
 * encrypted and then decrypted through the driver; one tampered ICV must come
 * back as crp_etype 89 (FreeBSD EBADMSG) with its buffer untouched, the rest
 * as 0 with the original plaintext.
 *
 * F-Stack mode (no-queue: no crypto_proc thread to requeue): requests that
 * find the slot in flight go to the engine's host overflow and launch from
 * the next poll; no ERESTART reaches the framework, and no process() call
 * waits for the GPU (the longest of a 48-request burst, timed, stays under
 * PROCESS_BOUND_US).  With the overflow off the same requests complete as
 * ENOBUFS (55) drops.  Then the buffers are registered memory
 * (espgpu_register_host): the records are read and written by the GPU in
 * place, bit-exact with the gathered path. */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "kmock.h"
#include "espgpu.h"

extern const struct kmock_cryptodev ff_gpucrypto_kmock;
int  ff_gpucrypto_host_configure(const struct espgpu_config *c);
void ff_gpucrypto_host_set_noqueue(int on);
void ff_gpucrypto_host_fini(void);
int  ff_gpucrypto_host_register(void *base, uint64_t len);
int  ff_gpucrypto_host_stats(struct espgpu_stats *st);
int  ff_gpucrypto_host_tune(const char *key, int value);
int  ff_gpucrypto_poll(void);

#define CHECK(c) do { if (!(c)) { printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); exit(1); } } while (0)
#define NREC 6
#define NBIG 48
#define PROCESS_BOUND_US 500.0

static int plen_of(int i) { return 64 + 48 * i; }          /* 4-byte multiples */
static uint8_t buf[NREC][512], orig[NREC][512];
static uint8_t big[NBIG][512], big_orig[NBIG][512], big_ct[NBIG][512];
static const uint8_t salt[4] = { 0xca, 0xfe, 0xba, 0xbe };
static int ndone;
static int cb(struct cryptop *crp) { (void)crp; ndone++; return 0; }

static void esp_crp_buf(struct cryptop *crp, crypto_session_t ses, uint8_t *b, int plen, int encrypt)
{

	memset(crp, 0, sizeof(*crp));
	crp->crp_session = ses;
	crp->crp_op = encrypt ? CRYPTO_OP_ENCRYPT | CRYPTO_OP_COMPUTE_DIGEST
	                      : CRYPTO_OP_DECRYPT | CRYPTO_OP_VERIFY_DIGEST;
	crp->crp_flags = CRYPTO_F_CBIFSYNC | CRYPTO_F_IV_SEPARATE;     /* xform_esp.c:453 */
	crp->crp_buf.cb_type = CRYPTO_BUF_CONTIG;
	crp->crp_buf.cb_buf = (char *)b;
	crp->crp_buf.cb_buf_len = 16 + plen + 16;
	crp->crp_aad_start = 0;                      /* SPI || SN */
	crp->crp_aad_length = 8;
	crp->crp_payload_start = 16;
	crp->crp_payload_length = plen;
	crp->crp_digest_start = 16 + plen;
	memcpy(crp->crp_iv, salt, 4);
	memcpy(crp->crp_iv + 4, b + 8, 8);
	crp->crp_callback = cb;
}

static void esp_crp(struct cryptop *crp, crypto_session_t ses, int i, int encrypt)
{
	esp_crp_buf(crp, ses, buf[i], plen_of(i), encrypt);
}

static double now_us(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec * 1e6 + t.tv_nsec / 1e3;
}

/* a burst of NBIG requests over big[]: the longest kmock_dispatch (us) */
static double run_big(struct cryptop *crp, crypto_session_t ses, int encrypt)
{
	const struct kmock_stats *st = kmock_stats();
	double worst = 0;
	int guard = 0;

	ndone = 0;
	for (int i = 0; i < NBIG; i++) {
		esp_crp_buf(&crp[i], ses, big[i], 16 * (i % 20) + 64, encrypt);
		double t0 = now_us();
		CHECK(kmock_dispatch(&crp[i]) == 0);
		double dt = now_us() - t0;
		worst = dt > worst ? dt : worst;
	}
	while (ndone < NBIG) {
		CHECK(ff_gpucrypto_poll() >= 0);
		CHECK(++guard < 1000000);
	}
	CHECK(st->queued == 0 && st->blocked == 0);
	return worst;
}
static void run_burst(struct cryptop *crp, int n)
{
	const struct kmock_stats *st = kmock_stats();
	int guard = 0;

	ndone = 0;
	for (int i = 0; i < n; i++)
		CHECK(kmock_dispatch(&crp[i]) == 0);
	while (ndone < n) {
		CHECK(ff_gpucrypto_poll() >= 0);
		kmock_run_queue();
		CHECK(++guard < 1000000);
	}
	CHECK(st->queued == 0 && st->blocked == 0);
}

int main(void)
{
	struct espgpu_config cfg;
	struct crypto_session_params csp;
	crypto_session_t ses;
	struct cryptop crp[NREC];
	const struct kmock_stats *st = kmock_stats();
	uint8_t key[16];

	memset(&cfg, 0, sizeof(cfg));
	cfg.batch_records = 4;
	cfg.nbatches = 1;
	cfg.batch_bytes = 1 << 16;
	CHECK(ff_gpucrypto_host_configure(&cfg) == 0);
	CHECK(kmock_attach(&ff_gpucrypto_kmock) == 0);
	for (int i = 0; i < 16; i++)
		key[i] = (uint8_t)(0x30 + 7 * i);
	memset(&csp, 0, sizeof(csp));
	csp.csp_mode = 4;
	csp.csp_ivlen = 12;
	csp.csp_cipher_alg = 25;
	csp.csp_cipher_klen = 16;
	csp.csp_cipher_key = key;
	CHECK(kmock_newsession(&ses, &csp) == 0);

	srand(7);
	for (int i = 0; i < NREC; i++) {
		int L = 16 + plen_of(i) + 16;
		for (int k = 0; k < L; k++)
			buf[i][k] = (uint8_t)rand();
		buf[i][0] = 0; buf[i][1] = 0; buf[i][2] = 0x12; buf[i][3] = 0x34;   /* SPI */
		memset(buf[i] + L - 16, 0, 16);
		memcpy(orig[i], buf[i], sizeof(buf[i]));
	}
	/* encrypt: 4 stage, the 5th gets ERESTART from the engine */
	for (int i = 0; i < NREC; i++)
		esp_crp(&crp[i], ses, i, 1);
	run_burst(crp, NREC);
	CHECK(st->erestarts >= 1);
	for (int i = 0; i < NREC; i++) {
		int plen = plen_of(i);
		CHECK(crp[i].crp_etype == 0);
		CHECK(memcmp(buf[i], orig[i], 16) == 0);                     /* header, IV */
		CHECK(memcmp(buf[i] + 16, orig[i] + 16, plen) != 0);        /* encrypted */
	}
	/* decrypt, one ICV tampered */
	uint8_t tampered[512];
	buf[2][16 + plen_of(2) + 5] ^= 0x20;
	memcpy(tampered, buf[2], sizeof(tampered));
	int e0 = st->erestarts;
	for (int i = 0; i < NREC; i++)
		esp_crp(&crp[i], ses, i, 0);
	run_burst(crp, NREC);
	CHECK(st->erestarts > e0);
	for (int i = 0; i < NREC; i++) {
		if (i == 2) {
			CHECK(crp[i].crp_etype == 89);
			CHECK(memcmp(buf[i], tampered, sizeof(tampered)) == 0);
		} else {
			CHECK(crp[i].crp_etype == 0);
			CHECK(memcmp(buf[i] + 16, orig[i] + 16, plen_of(i)) == 0);
		}
	}
	/* F-Stack mode (no crypto_proc thread): the same burst with no-queue
	 * set never reaches the framework as ERESTART */
	ff_gpucrypto_host_set_noqueue(1);
	e0 = st->erestarts;
	memcpy(buf[2], orig[2], sizeof(buf[2]));
	for (int i = 0; i < NREC; i++)
		esp_crp(&crp[i], ses, i, 1);
	run_burst(crp, NREC);
	CHECK(st->erestarts == e0);
	for (int i = 0; i < NREC; i++)
		esp_crp(&crp[i], ses, i, 0);
	run_burst(crp, NREC);
	CHECK(st->erestarts == e0);
	for (int i = 0; i < NREC; i++) {
		CHECK(crp[i].crp_etype == 0);
		CHECK(memcmp(buf[i], orig[i], 16 + plen_of(i)) == 0);
	}

	/* a 48-request burst through 4-record staging: 44 wait in the overflow;
	 * no process() call waits for the GPU */
	struct cryptop bcrp[NBIG];
	struct espgpu_stats es0, es1;
	for (int i = 0; i < NBIG; i++) {
		const int L = 16 + 16 * (i % 20) + 64 + 16;
		for (int k = 0; k < L; k++)
			big[i][k] = (uint8_t)rand();
		memset(big[i] + L - 16, 0, 16);
		memcpy(big_orig[i], big[i], sizeof(big[i]));
	}
	CHECK(ff_gpucrypto_host_stats(&es0) == 0);
	double w_enc = run_big(bcrp, ses, 1);
	CHECK(ff_gpucrypto_host_stats(&es1) == 0);
	CHECK(es1.overflow - es0.overflow >= NBIG - 8);
	CHECK(st->erestarts == e0);
	for (int i = 0; i < NBIG; i++)
		CHECK(bcrp[i].crp_etype == 0);
	memcpy(big_ct, big, sizeof(big));
	double w_dec = run_big(bcrp, ses, 0);
	for (int i = 0; i < NBIG; i++) {
		CHECK(bcrp[i].crp_etype == 0);
		CHECK(memcmp(big[i], big_orig[i], 16 + 16 * (i % 20) + 64) == 0);
	}
	printf("max process() us: encrypt %.1f decrypt %.1f (bound %.0f)\n", w_enc, w_dec, PROCESS_BOUND_US);
	CHECK(w_enc < PROCESS_BOUND_US && w_dec < PROCESS_BOUND_US);

	/* overflow off: what finds the slot in flight is dropped (ENOBUFS) */
	CHECK(ff_gpucrypto_host_tune("overflow_mb", 0) == 0);
	for (int i = 0; i < NREC; i++)
		esp_crp(&crp[i], ses, i, 1);
	run_burst(crp, NREC);
	CHECK(st->erestarts == e0);
	int drops = 0;
	for (int i = 0; i < NREC; i++) {
		CHECK(crp[i].crp_etype == 0 || crp[i].crp_etype == ENOBUFS);
		drops += crp[i].crp_etype == ENOBUFS;
	}
	CHECK(drops >= 1);
	ff_gpucrypto_host_set_noqueue(1);

	/* zero-copy: the same ciphertexts from registered memory decrypt to the
	 * same plaintexts, the buffers written by the GPU */
	memcpy(big, big_ct, sizeof(big));
	CHECK(ff_gpucrypto_host_register(big, sizeof(big)) == 0);
	CHECK(ff_gpucrypto_host_stats(&es0) == 0);
	run_big(bcrp, ses, 0);
	CHECK(ff_gpucrypto_host_stats(&es1) == 0);
	CHECK(es1.zerocopy - es0.zerocopy == NBIG);
	for (int i = 0; i < NBIG; i++) {
		CHECK(bcrp[i].crp_etype == 0);
		CHECK(memcmp(big[i], big_orig[i], 16 + 16 * (i % 20) + 64) == 0);
		/* the ICV stays the ciphertext's */
		CHECK(memcmp(big[i] + 16 + 16 * (i % 20) + 64, big_ct[i] + 16 + 16 * (i % 20) + 64, 16) == 0);
	}
	kmock_freesession(ses);
	kmock_detach();
	ff_gpucrypto_host_fini();
	printf("kmock gpu OK erestarts=%d\n", st->erestarts);
	return 0;
}
