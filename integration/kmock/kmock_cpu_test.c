/* The kernel-domain driver (ff_gpucrypto.c) over the kmock crypto KPI and a
 * scripted host layer (fake_host.c): attach flags, probe/new/free session,
 * ERESTART reaching the framework as ERESTART (-1) with the request queued
 * and the driver blocked, unblock + retry, and the ABI -> FreeBSD errno map
 * on completions (ICV failure -> crp_etype 89).  No GPU. */
#include <stdio.h>
#include <stdlib.h>

#include "kmock.h"
#include "espgpu.h"

extern const struct kmock_cryptodev ff_gpucrypto_kmock;
int gpucrypto_errno(int abi);
int fake_poll(void);
void fake_gpu_fail(void);
extern int fake_freed_sid, fake_last_nsegs;

#define CHECK(c) do { if (!(c)) { printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); exit(1); } } while (0)

static int ncb;
static int ndone[8];           /* crypto_done callbacks per request slot (crp_opaque) */
static int cb(struct cryptop *crp)
{
	ncb++;
	if (crp->crp_opaque)
		(*(int *)crp->crp_opaque)++;
	return 0;
}

static uint8_t bufs[8][96];

static void esp_gcm_crp(struct cryptop *crp, crypto_session_t ses, int i, uint8_t icv0)
{
	memset(crp, 0, sizeof(*crp));
	memset(bufs[i], 0x11 * i, sizeof(bufs[i]));
	bufs[i][96 - 16] = icv0;
	crp->crp_session = ses;
	crp->crp_op = CRYPTO_OP_DECRYPT | CRYPTO_OP_VERIFY_DIGEST;
	crp->crp_flags = CRYPTO_F_CBIFSYNC | CRYPTO_F_IV_SEPARATE;
	crp->crp_buf.cb_type = CRYPTO_BUF_CONTIG;
	crp->crp_buf.cb_buf = (char *)bufs[i];
	crp->crp_buf.cb_buf_len = 96;
	crp->crp_aad_start = 0;
	crp->crp_aad_length = 8;
	crp->crp_payload_start = 16;
	crp->crp_payload_length = 96 - 32;
	crp->crp_digest_start = 96 - 16;
	crp->crp_callback = cb;
}

int main(void)
{
	static const uint8_t key[16];
	struct crypto_session_params csp;
	crypto_session_t ses, s2, s3, s4;
	struct cryptop crp[8];
	const struct kmock_stats *st = kmock_stats();

	/* ABI -> FreeBSD errno */
	CHECK(gpucrypto_errno(ESPGPU_OK) == 0);
	CHECK(gpucrypto_errno(ESPGPU_EIO) == 5);
	CHECK(gpucrypto_errno(ESPGPU_EBADMSG) == 89);
	CHECK(gpucrypto_errno(ESPGPU_ERESTART) == -1);
	CHECK(gpucrypto_errno(ESPGPU_EAGAIN) == 35);
	CHECK(gpucrypto_errno(ESPGPU_EINVAL) == 22);
	CHECK(gpucrypto_errno(ESPGPU_ENOTSUP) == 45);
	CHECK(gpucrypto_errno(ESPGPU_ENOBUFS) == 55);
	CHECK(gpucrypto_errno(12345) == EIO);

	CHECK(kmock_attach(&ff_gpucrypto_kmock) == 0);
	CHECK(st->caps == (CRYPTOCAP_F_HARDWARE | CRYPTOCAP_F_SYNC));
	CHECK(st->session_size == sizeof(int32_t));

	memset(&csp, 0, sizeof(csp));
	csp.csp_mode = 4;                       /* CSP_MODE_AEAD */
	csp.csp_ivlen = 12;
	csp.csp_cipher_alg = 25;                /* CRYPTO_AES_NIST_GCM_16 */
	csp.csp_cipher_klen = 16;
	csp.csp_cipher_key = key;
	CHECK(kmock_newsession(&ses, &csp) == 0);
	csp.csp_ivlen = 16;                     /* not ours: probesession says EINVAL */
	CHECK(kmock_newsession(&s2, &csp) == EINVAL && s2 == NULL);
	csp.csp_ivlen = 12;
	CHECK(kmock_newsession(&s3, &csp) == 0);
	CHECK(kmock_newsession(&s4, &csp) == 0);
	/* the SA table is full: the probe declines (ENOMEM), and with the
	 * software driver present crypto_newsession selects it instead */
	CHECK(kmock_newsession(&s2, &csp) == ENOMEM && s2 == NULL);
	kmock_soft_enable(1);
	CHECK(kmock_newsession(&s2, &csp) == 0 && crypto_ses2hid(s2) == KMOCK_SOFT_ID);
	CHECK(st->soft_sessions == 1);
	kmock_freesession(s2);
	CHECK(st->soft_sessions == 0);
	kmock_soft_enable(0);

	/* four stage; the fifth hits a full staging area: ERESTART reaches the
	 * framework, which queues it and blocks the driver; the sixth queues
	 * behind it without reaching the driver */
	for (int i = 0; i < 4; i++) {
		esp_gcm_crp(&crp[i], ses, i, i == 2 ? 0xBA : 0x00);
		CHECK(kmock_dispatch(&crp[i]) == 0);
	}
	CHECK(st->erestarts == 0 && st->done == 0);
	esp_gcm_crp(&crp[4], ses, 4, 0x00);
	CHECK(kmock_dispatch(&crp[4]) == 0);
	CHECK(st->erestarts == 1 && st->blocked == 1 && st->queued == 1 && st->done == 0);
	esp_gcm_crp(&crp[5], ses, 5, 0xE1);
	CHECK(kmock_dispatch(&crp[5]) == 0);
	CHECK(st->erestarts == 1 && st->queued == 2);

	/* the poll completes the staged four and unblocks the driver */
	CHECK(fake_poll() == 4);
	CHECK(st->done == 4 && ncb == 4 && st->blocked == 0 && st->unblocks == 1);
	CHECK(crp[0].crp_etype == 0 && crp[1].crp_etype == 0 && crp[3].crp_etype == 0);
	CHECK(crp[2].crp_etype == 89);          /* ICV mismatch: FreeBSD EBADMSG */
	CHECK(kmock_run_queue() == 2 && st->queued == 0);
	CHECK(fake_poll() == 2);
	CHECK(crp[4].crp_etype == 0 && crp[5].crp_etype == 22);

	/* driver-side rejects complete at once through crypto_done, process() = 0 */
	{
		struct mbuf m[17];
		for (int i = 0; i < 17; i++) {
			m[i].m_next = i < 16 ? &m[i + 1] : NULL;
			m[i].m_len = 4;
			m[i].m_data = (char *)bufs[7] + 4 * i;
		}
		esp_gcm_crp(&crp[6], ses, 6, 0);
		crp[6].crp_buf.cb_type = CRYPTO_BUF_MBUF;
		crp[6].crp_buf.cb_mbuf = &m[0];
		CHECK(kmock_dispatch(&crp[6]) == 0);
		CHECK(crp[6].crp_etype == EINVAL && (crp[6].crp_flags & CRYPTO_F_DONE));
		m[15].m_next = NULL;                    /* 16 segments: accepted */
		esp_gcm_crp(&crp[6], ses, 6, 0);
		crp[6].crp_buf.cb_type = CRYPTO_BUF_MBUF;
		crp[6].crp_buf.cb_mbuf = &m[0];
		crp[6].crp_payload_length = 64 - 32;
		crp[6].crp_digest_start = 64 - 16;
		CHECK(kmock_dispatch(&crp[6]) == 0 && fake_last_nsegs == 16);
		CHECK(fake_poll() == 1 && crp[6].crp_etype == 0);
		esp_gcm_crp(&crp[7], ses, 7, 0);
		crp[7].crp_obuf.cb_type = CRYPTO_BUF_CONTIG;      /* separate output */
		CHECK(kmock_dispatch(&crp[7]) == 0 && crp[7].crp_etype == EINVAL);
		esp_gcm_crp(&crp[7], ses, 7, 0);
		crp[7].crp_cipher_key = key;                      /* per-request key */
		CHECK(kmock_dispatch(&crp[7]) == 0 && crp[7].crp_etype == EINVAL);
	}

	/* GPU failure: three requests staged, then the GPU
	 * fails.  The staged ones complete exactly once with EIO (a clean drop);
	 * the next request on the session moves it to the software driver
	 * (EAGAIN with a new session in crp_session, as crypto_invoke's
	 * CRYPTOCAP_F_CLEANUP branch does) and, re-dispatched as esp_input_cb
	 * does, completes there; new sessions go to the software driver. */
	{
		crypto_session_t s5;
		const int done0 = st->done;

		kmock_soft_enable(1);
		memset(ndone, 0, sizeof(ndone));
		for (int i = 0; i < 3; i++) {
			esp_gcm_crp(&crp[i], ses, i, 0x00);
			crp[i].crp_opaque = &ndone[i];
			CHECK(kmock_dispatch(&crp[i]) == 0);
		}
		CHECK(st->done == done0);
		fake_gpu_fail();
		esp_gcm_crp(&crp[3], ses, 3, 0x00);
		crp[3].crp_opaque = &ndone[3];
		CHECK(kmock_dispatch(&crp[3]) == 0);
		CHECK(ndone[3] == 1 && crp[3].crp_etype == EAGAIN);
		CHECK(crp[3].crp_session != ses && crypto_ses2hid(crp[3].crp_session) == KMOCK_SOFT_ID);
		CHECK(st->soft_sessions == 1);
		CHECK(kmock_dispatch(&crp[3]) == 0);              /* esp_input_cb's re-dispatch */
		CHECK(ndone[3] == 2 && crp[3].crp_etype == 0 && st->soft_done == 1);
		CHECK(fake_poll() == 3);
		for (int i = 0; i < 3; i++)
			CHECK(ndone[i] == 1 && crp[i].crp_etype == EIO);
		CHECK(fake_poll() == 0);
		for (int i = 0; i < 3; i++)
			CHECK(ndone[i] == 1);                          /* exactly once */
		/* the probe declines now: a new session lands on the software driver */
		CHECK(kmock_newsession(&s5, &csp) == 0 && crypto_ses2hid(s5) == KMOCK_SOFT_ID);
		CHECK(st->soft_sessions == 2);
		kmock_freesession(s5);
		kmock_freesession(crp[3].crp_session);
		CHECK(st->soft_sessions == 0);
	}

	kmock_freesession(s3);
	CHECK(fake_freed_sid == 1);
	kmock_freesession(ses);
	CHECK(fake_freed_sid == 0);
	kmock_freesession(s4);
	kmock_detach();
	CHECK(st->driverid == -1);
	CHECK(st->sessions == 0);                 /* every session freed */
	printf("kmock cpu OK\n");
	return 0;
}
