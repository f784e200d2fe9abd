/*
 * ff_crypto_selftest.c -- kernel-domain half of integration/fstack_run: the
 * framework calls esp_init / esp_input / esp_output make, against the real
 * freebsd/opencrypto compiled by F-Stack's own lib/Makefile rules
 * (integration/fstack_run.py compiles this file with the same NORMAL_C
 * command line and links it into libfstack.ro before the symbol
 * localisation, exporting only the ffst_* entry points below).
 *
 *   ffst_newsession   crypto_newsession(&cses, &csp, crid)       crypto.c:910
 *                     (esp_init passes V_crypto_support =
 *                     CRYPTOCAP_F_HARDWARE | CRYPTOCAP_F_SOFTWARE,
 *                     xform_esp.c:242, ipsec.c:151); crypto_select_driver
 *                     picks the highest probesession bid       crypto.c:622-659
 *   ffst_request      crypto_getreq + crypto_use_mbuf / crypto_use_buf and the
 *                     fields esp_input / esp_output fill     xform_esp.c:364-458
 *                     over a real mbuf chain (m_getcl clusters, one per
 *                     caller segment)
 *   ffst_dispatch     crypto_dispatch                        crypto.c:1413
 *   ffst_result       the callback's record: crypto_done ran it inline
 *                     (CRYPTO_F_CBIFSYNC and a CRYPTOCAP_F_SYNC driver,
 *                     crypto.c:1802-1826), and m_copydata of the result
 *   ffst_redispatch   esp_input_cb's EAGAIN path (xform_esp.c:505-512): the
 *                     request names the session the driver moved it to;
 *                     crypto_dispatch it again (the GPU-failure phase)
 * The host half (host_main.c) drives these after ff_freebsd_init().
 */
#include <sys/param.h>
#include <sys/systm.h>
#include <sys/errno.h>
#include <sys/malloc.h>
#include <sys/mbuf.h>
#include <opencrypto/cryptodev.h>

int   ffst_find_driver(const char *name);
void *ffst_newsession(const int *p, const void *ckey, const void *akey, int crid, int *err, int *hid);
void  ffst_freesession(void *ses);
void *ffst_request(void *ses, const int *f, const void *aad, const void *esn, const void *iv,
    const void *buf, int len, const int *cuts, int ncuts);
int   ffst_dispatch(void *r);
int   ffst_result(void *r, void *out, int len, int *flags);
int   ffst_ndone(void *r);
int   ffst_redispatch(void *r, int *etype0, int *hid);
void  ffst_free(void *r);

struct ffst_req {
	struct cryptop	*crp;
	struct mbuf	*m;		/* NULL: contiguous buffer */
	char		*buf;
	int		 len;
	int		 done;		/* the callback ran */
	int		 ndone;		/* how many times */
	int		 done_flag;	/* CRYPTO_F_DONE was set when it ran */
	crypto_session_t moved;	/* the session a GPU failure moved it to (freed with it) */
	uint8_t		 aad[16];
};

static int
ffst_cb(struct cryptop *crp)
{
	struct ffst_req *r = crp->crp_opaque;

	r->done_flag = (crp->crp_flags & CRYPTO_F_DONE) != 0;
	r->done = 1;
	r->ndone++;
	return (0);
}

int
ffst_find_driver(const char *name)
{
	return (crypto_find_driver(name));
}

/* p: mode, flags, ivlen, cipher alg, cipher klen, auth alg, auth klen, mlen */
void *
ffst_newsession(const int *p, const void *ckey, const void *akey, int crid, int *err, int *hid)
{
	struct crypto_session_params csp;
	crypto_session_t cses = NULL;

	memset(&csp, 0, sizeof(csp));
	csp.csp_mode = p[0];
	csp.csp_flags = p[1];
	csp.csp_ivlen = p[2];
	csp.csp_cipher_alg = p[3];
	csp.csp_cipher_klen = p[4];
	csp.csp_cipher_key = p[4] ? ckey : NULL;
	csp.csp_auth_alg = p[5];
	csp.csp_auth_klen = p[6];
	csp.csp_auth_key = p[6] ? akey : NULL;
	csp.csp_auth_mlen = p[7];
	*err = crypto_newsession(&cses, &csp, crid);
	*hid = *err == 0 ? crypto_ses2hid(cses) : -1;
	return (*err == 0 ? cses : NULL);
}

void
ffst_freesession(void *ses)
{
	crypto_freesession(ses);
}

/* f: op, flags, aad_start, aad_len, iv_start, payload_start, payload_len,
 * digest_start, has_aad, has_iv, mbuf.  cuts: segment boundaries of the mbuf
 * chain (each segment <= MCLBYTES). */
void *
ffst_request(void *ses, const int *f, const void *aad, const void *esn, const void *iv,
    const void *buf, int len, const int *cuts, int ncuts)
{
	struct ffst_req *r;
	struct cryptop *crp;
	struct mbuf *m, *tail = NULL;
	int i, a, b;

	r = malloc(sizeof(*r), M_TEMP, M_NOWAIT | M_ZERO);
	if (r == NULL)
		return (NULL);
	crp = crypto_getreq(ses, M_NOWAIT);
	if (crp == NULL) {
		free(r, M_TEMP);
		return (NULL);
	}
	r->crp = crp;
	r->len = len;
	if (f[10]) {
		for (i = 0; i <= ncuts; i++) {
			a = i == 0 ? 0 : cuts[i - 1];
			b = i == ncuts ? len : cuts[i];
			if (b - a > MCLBYTES || b < a)
				goto fail;
			m = m_getcl(M_NOWAIT, MT_DATA, i == 0 ? M_PKTHDR : 0);
			if (m == NULL)
				goto fail;
			memcpy(mtod(m, char *), (const char *)buf + a, b - a);
			m->m_len = b - a;
			if (tail == NULL)
				r->m = m;
			else
				tail->m_next = m;
			tail = m;
		}
		r->m->m_pkthdr.len = len;
		crypto_use_mbuf(crp, r->m);
	} else {
		r->buf = malloc(len, M_TEMP, M_NOWAIT);
		if (r->buf == NULL)
			goto fail;
		memcpy(r->buf, buf, len);
		crypto_use_buf(crp, r->buf, len);
	}
	crp->crp_op = f[0];
	crp->crp_flags = f[1];
	crp->crp_aad_start = f[2];
	crp->crp_aad_length = f[3];
	if (f[8]) {
		memcpy(r->aad, aad, f[3]);
		crp->crp_aad = r->aad;
	}
	memcpy(crp->crp_esn, esn, 4);
	crp->crp_iv_start = f[4];
	if (f[9])
		memcpy(crp->crp_iv, iv, EALG_MAX_BLOCK_LEN);
	crp->crp_payload_start = f[5];
	crp->crp_payload_length = f[6];
	crp->crp_digest_start = f[7];
	crp->crp_opaque = r;
	crp->crp_callback = ffst_cb;
	return (r);
fail:
	ffst_free(r);
	return (NULL);
}

int
ffst_dispatch(void *rp)
{
	struct ffst_req *r = rp;

	return (crypto_dispatch(r->crp));
}

/* -1 while pending; else crp_etype, the buffer copied to out, flags bit 0 =
 * the callback saw CRYPTO_F_DONE */
int
ffst_result(void *rp, void *out, int len, int *flags)
{
	struct ffst_req *r = rp;

	if (!r->done)
		return (-1);
	if (len > r->len)
		len = r->len;
	if (r->m != NULL)
		m_copydata(r->m, 0, len, out);
	else
		memcpy(out, r->buf, len);
	*flags = r->done_flag;
	return (r->crp->crp_etype);
}

int
ffst_ndone(void *rp)
{
	return (((struct ffst_req *)rp)->ndone);
}

/* The request completed with EAGAIN and a new session (gpucrypto_migrate):
 * what esp_input_cb does next -- dispatch it again on that session.  The
 * request's own session becomes the moved one (freed with the request: here
 * no SA keeps it, as ipsec_updateid would). */
int
ffst_redispatch(void *rp, int *etype0, int *hid)
{
	struct ffst_req *r = rp;

	*etype0 = r->crp->crp_etype;
	*hid = (int)crypto_ses2hid(r->crp->crp_session);
	if (r->crp->crp_etype != EAGAIN)
		return (-1);
	r->moved = r->crp->crp_session;
	r->done = 0;
	r->crp->crp_etype = 0;
	r->crp->crp_flags &= ~CRYPTO_F_DONE;
	return (crypto_dispatch(r->crp));
}

void
ffst_free(void *rp)
{
	struct ffst_req *r = rp;

	if (r->crp != NULL)
		crypto_freereq(r->crp);
	if (r->moved != NULL)
		crypto_freesession(r->moved);
	if (r->m != NULL)
		m_freem(r->m);
	if (r->buf != NULL)
		free(r->buf, M_TEMP);
	free(r, M_TEMP);
}
