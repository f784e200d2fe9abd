/*
 * oracle_engine.c -- a CPU stand-in for the host shim (ff_gpucrypto_host.c)
 * so that integration/fstack_run runs F-Stack's opencrypto with the MI355X
 * driver attached on a machine without a GPU.  TEST INFRASTRUCTURE: the
 * crypto is the oracle's (oracle/espref.c, a restatement of cryptosoft),
 * never the product.  It keeps the engine's contract: probesession is the
 * real espgpu_probesession (device-free), process() stages the request and
 * returns at once, ff_gpucrypto_poll() completes staged requests through
 * ff_gpucrypto_done() (so crypto_done runs from the poll, as on the GPU),
 * results are written back into the request's segments, at that poll, only
 * for etype 0.  oracle_engine_fail() plays a GPU failure as the engine
 * reports it: staged requests complete with ESPGPU_EIO and untouched
 * buffers, process() answers ESPGPU_EIO, the probe ENXIO.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "espgpu.h"
#include "espref.h"

void ff_gpucrypto_done(void *opaque, int abi_etype);
void ff_gpucrypto_unblock(void);

#define OE_MAX_SES 64
#define OE_MAX_PENDING 4096

static struct oe_ses {
	int used, mode, flags, calg, aalg, cklen, aklen, mlen;
	uint8_t ckey[32], akey[128];
	oref_sa *sa;                  /* made at the first request (salt = crp_iv[0..3]) */
} g_ses[OE_MAX_SES];

/* a staged request: its result is written back at the poll that completes it */
static struct oe_pend {
	void *opaque;
	int etype;
	struct espgpu_seg segs[16];
	int nsegs;
	uint8_t *rec;                 /* the processed record (malloc'ed) */
	uint32_t rec0, wb_off, wb_len;  /* write-back: [wb_off, wb_off + wb_len) of the record */
} g_pend[OE_MAX_PENDING];
static int g_npend, g_ready, g_failed;

int  ff_gpucrypto_host_ready(void) { return (g_ready); }
void oracle_engine_init(void) { g_ready = 1; }
int  ff_gpucrypto_host_failed(void) { return (g_failed); }
void oracle_engine_fail(void) { g_failed = 1; }

int
ff_gpucrypto_host_probe(const struct espgpu_session_params *csp)
{
	int r;

	if (g_failed)
		return (ESPGPU_ENXIO);
	r = espgpu_probesession(csp);
	if (r != ESPGPU_PROBE_HARDWARE)
		return (r);
	/* a full SA table declines (ff_gpucrypto_host.c: espgpu_session_room) */
	for (int i = 0; i < OE_MAX_SES; i++)
		if (!g_ses[i].used)
			return (r);
	return (ESPGPU_ENOMEM);
}

int
ff_gpucrypto_host_newsession(const struct espgpu_session_params *csp, int32_t *sid)
{
	if (g_failed)
		return (ESPGPU_ENXIO);
	for (int i = 0; i < OE_MAX_SES; i++) {
		struct oe_ses *s = &g_ses[i];
		if (s->used)
			continue;
		memset(s, 0, sizeof(*s));
		s->used = 1;
		s->mode = csp->csp_mode;
		s->flags = csp->csp_flags;
		s->calg = csp->csp_cipher_alg;
		s->aalg = csp->csp_auth_alg;
		s->cklen = csp->csp_cipher_klen;
		s->aklen = csp->csp_auth_klen;
		s->mlen = csp->csp_auth_mlen;
		if (s->cklen)
			memcpy(s->ckey, csp->csp_cipher_key, (size_t)s->cklen);
		if (s->aklen)
			memcpy(s->akey, csp->csp_auth_key, (size_t)s->aklen);
		*sid = i;
		return (ESPGPU_OK);
	}
	return (ESPGPU_ENOMEM);
}

void
ff_gpucrypto_host_freesession(int32_t sid)
{
	if (sid >= 0 && sid < OE_MAX_SES && g_ses[sid].used) {
		if (g_ses[sid].sa)
			oref_sa_free(g_ses[sid].sa);
		g_ses[sid].used = 0;
		g_ses[sid].sa = NULL;
	}
}

static void
seg_io(const struct espgpu_seg *segs, int nsegs, uint32_t off, uint8_t *p, uint32_t n, int out)
{
	for (int i = 0; i < nsegs && n; i++) {
		uint32_t l = segs[i].len;
		if (off >= l) {
			off -= l;
			continue;
		}
		uint32_t k = l - off < n ? l - off : n;
		if (out)
			memcpy(p, (uint8_t *)segs[i].base + off, k);
		else
			memcpy((uint8_t *)segs[i].base + off, p, k);
		p += k;
		n -= k;
		off = 0;
	}
}

static uint32_t be32(const uint8_t *p) { return ((uint32_t)p[0] << 24 | p[1] << 16 | p[2] << 8 | p[3]); }

int
ff_gpucrypto_host_process(const struct espgpu_req *r, int hint)
{
	struct oe_ses *s;
	int gcm, ctr, null, hlen, mlen, e, enc;
	uint32_t rec0, rlen, esn_hi = 0;
	uint8_t *rec;

	(void)hint;
	if (g_failed)
		return (ESPGPU_EIO);
	if (r->session < 0 || r->session >= OE_MAX_SES || !g_ses[r->session].used)
		return (ESPGPU_EINVAL);
	if (g_npend == OE_MAX_PENDING || r->nsegs > 16)
		return (ESPGPU_ERESTART);
	s = &g_ses[r->session];
	gcm = s->mode == ESPGPU_CSP_MODE_AEAD;
	ctr = s->calg == ESPGPU_CRYPTO_AES_ICM;
	null = s->calg == ESPGPU_CRYPTO_NULL_CBC;
	hlen = 8 + (gcm || ctr ? 8 : null ? 0 : 16);
	mlen = gcm ? (s->mlen ? s->mlen : 16) : s->mode == ESPGPU_CSP_MODE_CIPHER ? 0 :
	    s->mlen ? s->mlen : (s->aalg == ESPGPU_CRYPTO_SHA1_HMAC ? 20 : s->aalg == ESPGPU_CRYPTO_SHA2_256_HMAC ? 32 :
	    s->aalg == ESPGPU_CRYPTO_SHA2_384_HMAC ? 48 : 64);
	if (s->sa == NULL) {
		if (gcm)
			s->sa = oref_sa_new(OREF_CSP_MODE_AEAD, s->flags, s->ckey, s->cklen, r->crp_iv, NULL, 0, mlen);
		else
			s->sa = oref_sa_new2(s->mode, s->flags, s->calg, s->ckey, s->cklen, r->crp_iv, s->aalg,
			    s->akey, s->aklen, mlen);
	}
	rec0 = (uint32_t)(r->crp_payload_start - hlen);
	rlen = (uint32_t)(hlen + r->crp_payload_length + mlen);
	rec = malloc(rlen);
	seg_io(r->segs, r->nsegs, rec0, rec, rlen, 1);
	if (gcm && (s->flags & ESPGPU_CSP_F_SEPARATE_AAD) && r->crp_aad != NULL)
		esn_hi = be32((const uint8_t *)r->crp_aad + 4);      /* SPI | ESN high | SN */
	else if (!gcm && (s->flags & ESPGPU_CSP_F_ESN))
		esn_hi = be32(r->crp_esn);
	enc = (r->crp_op & ESPGPU_CRYPTO_OP_ENCRYPT) != 0;
	e = enc ? oref_esp_encrypt(s->sa, rec, (int)rlen, esn_hi) : oref_esp_decrypt(s->sa, rec, (int)rlen, esn_hi);
	struct oe_pend *p = &g_pend[g_npend++];
	p->opaque = r->opaque;
	p->etype = e == 0 ? ESPGPU_OK : e == 74 ? ESPGPU_EBADMSG : ESPGPU_EINVAL;
	memcpy(p->segs, r->segs, (size_t)r->nsegs * sizeof(r->segs[0]));
	p->nsegs = r->nsegs;
	p->rec = rec;
	p->rec0 = rec0;
	p->wb_off = (uint32_t)hlen;                                       /* payload (+ ICV) */
	p->wb_len = rlen - (uint32_t)hlen - (enc ? 0 : (uint32_t)mlen);
	return (ESPGPU_OK);
}

/* main_loop hook: every staged request completes through crypto_done, its
 * result written back first (etype 0 only; a failed engine writes nothing
 * and completes it with EIO) */
int
ff_gpucrypto_poll(void)
{
	int n = g_npend;

	g_npend = 0;
	for (int i = 0; i < n; i++) {
		struct oe_pend *p = &g_pend[i];
		if (g_failed)
			p->etype = ESPGPU_EIO;
		if (p->etype == ESPGPU_OK)
			seg_io(p->segs, p->nsegs, p->rec0 + p->wb_off, p->rec + p->wb_off, p->wb_len, 0);
		free(p->rec);
		ff_gpucrypto_done(p->opaque, p->etype);
	}
	if (n)
		ff_gpucrypto_unblock();
	return (n);
}
