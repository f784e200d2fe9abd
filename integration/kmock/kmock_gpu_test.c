/* The whole F-Stack binding on the GPU: kernel-domain driver (ff_gpucrypto.c
 * over the kmock KPI) -> host-domain shim (ff_gpucrypto_host.c) ->
 * libespgpu.so.  The staging area is configured small (4 records, one slot)
 * so a burst of 6 requests makes process() answer ERESTART: the framework
 * must see ERESTART (-1), queue and later retry.  ESP AES-GCM records are
 * encrypted and then decrypted through the driver; one tampered ICV must come
 * back as crp_etype 89 (FreeBSD EBADMSG) with its buffer untouched, the rest
 * as 0 with the original plaintext. */
#include <stdio.h>
#include <stdlib.h>

#include "kmock.h"
#include "espgpu.h"

extern const struct kmock_cryptodev ff_gpucrypto_kmock;
int  ff_gpucrypto_host_configure(const struct espgpu_config *c);
void ff_gpucrypto_host_set_noqueue(int on);
void ff_gpucrypto_host_fini(void);
int  ff_gpucrypto_poll(void);

#define CHECK(c) do { if (!(c)) { printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); exit(1); } } while (0)
#define NREC 6

static int plen_of(int i) { return 64 + 48 * i; }          /* 4-byte multiples */
static uint8_t buf[NREC][512], orig[NREC][512];
static const uint8_t salt[4] = { 0xca, 0xfe, 0xba, 0xbe };
static int ndone;
static int cb(struct cryptop *crp) { (void)crp; ndone++; return 0; }

static void esp_crp(struct cryptop *crp, crypto_session_t ses, int i, int encrypt)
{
	int plen = plen_of(i);

	memset(crp, 0, sizeof(*crp));
	crp->crp_session = ses;
	crp->crp_op = encrypt ? CRYPTO_OP_ENCRYPT | CRYPTO_OP_COMPUTE_DIGEST
	                      : CRYPTO_OP_DECRYPT | CRYPTO_OP_VERIFY_DIGEST;
	crp->crp_flags = CRYPTO_F_CBIFSYNC | CRYPTO_F_IV_SEPARATE;     /* xform_esp.c:453 */
	crp->crp_buf.cb_type = CRYPTO_BUF_CONTIG;
	crp->crp_buf.cb_buf = (char *)buf[i];
	crp->crp_buf.cb_buf_len = 16 + plen + 16;
	crp->crp_aad_start = 0;                      /* SPI || SN */
	crp->crp_aad_length = 8;
	crp->crp_payload_start = 16;
	crp->crp_payload_length = plen;
	crp->crp_digest_start = 16 + plen;
	memcpy(crp->crp_iv, salt, 4);
	memcpy(crp->crp_iv + 4, buf[i] + 8, 8);
	crp->crp_callback = cb;
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
	kmock_freesession(ses);
	kmock_detach();
	ff_gpucrypto_host_fini();
	printf("kmock gpu OK erestarts=%d\n", st->erestarts);
	return 0;
}
