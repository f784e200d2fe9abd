/*
 * kmock_py.c -- flat C entry points over the kernel-domain driver
 * (ff_gpucrypto.c over the kmock KPI) and the host shim
 * (ff_gpucrypto_host.c -> libespgpu.so), so that the Python parity tests
 * (tests/test_kmock_driver_gpu.py) can drive the very C driver F-Stack links
 * with the reference's golden packets and check it against the oracle.
 *
 * Built into integration/libkmockdrv.so by integration/Makefile.  Each call
 * is what the framework side of a request does in the kernel:
 *   kd_newsession  crypto_newsession: probesession must bid -100, then
 *                  CRYPTODEV_NEWSESSION                 (crypto.c:622-659, :910)
 *   kd_request     crypto_getreq + the fields esp_input / esp_output fill
 *                  (xform_esp.c:364-458, :862-931), over an mbuf chain
 *                  (CRYPTO_BUF_MBUF, one mbuf per caller segment) or a
 *                  contiguous buffer (CRYPTO_BUF_CONTIG)
 *   kd_dispatch    crypto_dispatch                      (crypto.c:1413-1460)
 *   kd_poll        F-Stack's main_loop hook: ff_gpucrypto_poll() (flush,
 *                  completions through crypto_done), then the framework's
 *                  re-dispatch of ERESTARTed requests after crypto_unblock
 * The caller owns the segment buffers: the engine writes results into them.
 */
#include <stdlib.h>

#include "kmock.h"
#include "espgpu.h"

extern const struct kmock_cryptodev ff_gpucrypto_kmock;
int  ff_gpucrypto_host_configure(const struct espgpu_config *c);
int  ff_gpucrypto_host_init_proc(int proc_id);
void ff_gpucrypto_host_set_noqueue(int on);
void ff_gpucrypto_host_fini(void);
int  ff_gpucrypto_host_register(void *base, uint64_t len);
int  ff_gpucrypto_host_stats(struct espgpu_stats *st);
int  ff_gpucrypto_host_tune(const char *key, int value);
int  ff_gpucrypto_host_failed(void);
int  ff_gpucrypto_poll(void);

#define KD_MAX_SEGS 16

struct kd_req {
	struct cryptop crp;
	struct mbuf    m[KD_MAX_SEGS];
	uint8_t        aad[16];
	int            done;               /* crp_callback runs (crypto_done calls) */
};

static int
kd_cb(struct cryptop *crp)
{
	((struct kd_req *)crp)->done++;    /* crp is the first member */
	return (0);
}

/* open the GPU context (staging: batch_records x nbatches slots), attach the
 * driver; noqueue = F-Stack mode (host overflow, never ERESTART) */
int
kd_open(int batch_records, int nbatches, int batch_bytes, int noqueue)
{
	struct espgpu_config c = { 0 };
	int e;

	c.batch_records = (uint32_t)batch_records;
	c.nbatches = (uint32_t)nbatches;
	c.batch_bytes = (uint32_t)batch_bytes;
	c.max_sessions = 64;
	if ((e = ff_gpucrypto_host_configure(&c)) != 0)
		return (e);
	if ((e = kmock_attach(&ff_gpucrypto_kmock)) != 0)
		return (e);
	ff_gpucrypto_host_set_noqueue(noqueue);
	return (0);
}

/* as ff_init() opens it: ff_gpucrypto_host_init_proc (device proc_id mod
 * n, F-Stack mode, FF_GPUCRYPTO_DOOR from the environment), then attach */
int
kd_open_proc(int proc_id)
{
	int e;

	if ((e = ff_gpucrypto_host_init_proc(proc_id)) != 0)
		return (e);
	return (kmock_attach(&ff_gpucrypto_kmock));
}

void
kd_close(void)
{
	kmock_detach();
	ff_gpucrypto_host_fini();
}

/* -> 0 and *out, or a FreeBSD errno (the driver declined or failed) */
int
kd_newsession(int mode, int flags, int ivlen, int calg, int cklen, const void *ckey, int aalg,
    int aklen, const void *akey, int mlen, void **out)
{
	struct crypto_session_params csp;

	memset(&csp, 0, sizeof(csp));
	csp.csp_mode = mode;
	csp.csp_flags = flags;
	csp.csp_ivlen = ivlen;
	csp.csp_cipher_alg = calg;
	csp.csp_cipher_klen = cklen;
	csp.csp_cipher_key = ckey;
	csp.csp_auth_alg = aalg;
	csp.csp_auth_klen = aklen;
	csp.csp_auth_key = akey;
	csp.csp_auth_mlen = mlen;
	return (kmock_newsession((crypto_session_t *)out, &csp));
}

void
kd_freesession(void *ses)
{
	kmock_freesession((crypto_session_t)ses);
}

/* A request over nsegs caller buffers: mbuf chain (mbuf != 0) or one
 * contiguous buffer (nsegs 1).  aad: the separate AAD (GCM with ESN, 12
 * bytes) or NULL; esn: the ESN high word bytes for ETA (crp_esn); iv: 16
 * bytes for CRYPTO_F_IV_SEPARATE requests. */
void *
kd_request(void *ses, int op, int flags, int mbuf, void **bases, const int *lens, int nsegs,
    const void *aad, int aad_start, int aad_len, const uint8_t *esn, const uint8_t *iv, int iv_start,
    int payload_start, int payload_len, int digest_start)
{
	struct kd_req *r;
	int i;

	if (nsegs < 1 || nsegs > KD_MAX_SEGS || (!mbuf && nsegs != 1) || (aad != NULL && aad_len > 16))
		return (NULL);
	r = calloc(1, sizeof(*r));
	if (r == NULL)
		return (NULL);
	r->crp.crp_session = (crypto_session_t)ses;
	r->crp.crp_op = op;
	r->crp.crp_flags = flags;
	if (mbuf) {
		for (i = 0; i < nsegs; i++) {
			r->m[i].m_data = bases[i];
			r->m[i].m_len = lens[i];
			r->m[i].m_next = i + 1 < nsegs ? &r->m[i + 1] : NULL;
		}
		r->crp.crp_buf.cb_type = CRYPTO_BUF_MBUF;
		r->crp.crp_buf.cb_mbuf = &r->m[0];
	} else {
		r->crp.crp_buf.cb_type = CRYPTO_BUF_CONTIG;
		r->crp.crp_buf.cb_buf = bases[0];
		r->crp.crp_buf.cb_buf_len = lens[0];
	}
	if (aad != NULL) {
		memcpy(r->aad, aad, (size_t)aad_len);
		r->crp.crp_aad = r->aad;
	}
	r->crp.crp_aad_start = aad_start;
	r->crp.crp_aad_length = aad_len;
	if (esn != NULL)
		memcpy(r->crp.crp_esn, esn, 4);
	if (iv != NULL)
		memcpy(r->crp.crp_iv, iv, 16);
	r->crp.crp_iv_start = iv_start;
	r->crp.crp_payload_start = payload_start;
	r->crp.crp_payload_length = payload_len;
	r->crp.crp_digest_start = digest_start;
	r->crp.crp_callback = kd_cb;
	return (r);
}

int
kd_dispatch(void *r)
{
	return (kmock_dispatch(&((struct kd_req *)r)->crp));
}

/* one main_loop iteration: completions delivered, queued requests retried */
int
kd_poll(void)
{
	int n = ff_gpucrypto_poll();

	kmock_run_queue();
	return (n);
}

/* -1 while pending, else crp_etype (FreeBSD errno) */
int
kd_result(void *r)
{
	struct kd_req *q = r;

	return (q->done ? q->crp.crp_etype : -1);
}

void
kd_free(void *r)
{
	free(r);
}

int
kd_register(void *base, uint64_t len)
{
	return (ff_gpucrypto_host_register(base, len));
}

/* framework counters: erestarts, queued, blocked, done */
void
kd_counters(int *out4)
{
	const struct kmock_stats *st = kmock_stats();

	out4[0] = st->erestarts;
	out4[1] = st->queued;
	out4[2] = st->blocked;
	out4[3] = st->done;
}

/* engine counters: zero-copy records, overflow entries, doorbell batches,
 * GPU failures, requests completed or refused with EIO because of one */
void
kd_engine(uint64_t *out5)
{
	struct espgpu_stats s;

	memset(&s, 0, sizeof(s));
	ff_gpucrypto_host_stats(&s);
	out5[0] = s.zerocopy;
	out5[1] = s.overflow;
	out5[2] = s.door;
	out5[3] = s.gpu_fail;
	out5[4] = s.fail_eio;
}

/* the GPU-failure path */
int
kd_tune(const char *key, int value)
{
	return (ff_gpucrypto_host_tune(key, value));
}

int
kd_failed(void)
{
	return (ff_gpucrypto_host_failed());
}

/* crypto_done calls so far for the request (exactly one is the contract) */
int
kd_done_count(void *r)
{
	return (((struct kd_req *)r)->done);
}

/* the driver id of the request's session now (gpucrypto_migrate moves it) */
int
kd_session_hid(void *r)
{
	return ((int)crypto_ses2hid(((struct kd_req *)r)->crp.crp_session));
}

/* esp_input_cb's EAGAIN path: re-dispatch on the session the request now names */
int
kd_redispatch(void *r)
{
	struct kd_req *q = r;

	q->crp.crp_flags &= ~CRYPTO_F_DONE;
	return (kmock_dispatch(&q->crp));
}

void
kd_soft_enable(int on)
{
	kmock_soft_enable(on);
}

/* software stand-in and session counters: soft sessions, soft completions,
 * sessions alive, the driver's own id */
void
kd_soft(int *out4)
{
	const struct kmock_stats *st = kmock_stats();

	out4[0] = st->soft_sessions;
	out4[1] = st->soft_done;
	out4[2] = st->sessions;
	out4[3] = st->driverid;
}

void
kd_freesession_of(void *r)
{
	kmock_freesession(((struct kd_req *)r)->crp.crp_session);
}
