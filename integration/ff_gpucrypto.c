/*
 * ff_gpucrypto.c -- kernel-domain opencrypto driver for libespgpu
 * (INTEGRATION.md section 1).  In F-Stack it is lib/ff_gpucrypto.c, an
 * OPENCRYPTO_SRCS file built with the FreeBSD headers; here it is built with
 * -DFF_GPUCRYPTO_KMOCK against integration/kmock (a test double of the crypto
 * KPI) so that the same source is compiled, linked and exercised by the
 * tests (tests/test_integration.py).
 *
 * It plays cryptosoft's part (freebsd/opencrypto/cryptosoft.c:1440-1510) for
 * the ESP transforms the engine serves:
 *   attach        crypto_get_driverid(dev, sizeof(session),
 *                     CRYPTOCAP_F_HARDWARE | CRYPTOCAP_F_SYNC)    crypto.c:990
 *                 -- HARDWARE so probesession's -100 beats cryptosoft's -500
 *                 (crypto.c:621-659); SYNC so CRYPTO_F_CBIFSYNC callbacks run
 *                 inline from the poll (cryptodev.h:592)
 *   probesession  cryptodev_if.m:72-75   -> espgpu_probesession
 *   newsession    cryptodev_if.m:93-97   -> espgpu_newsession
 *   freesession   cryptodev_if.m:113-116 -> espgpu_freesession
 *   process       cryptodev_if.m:143-147 -> espgpu_process: 0, or ERESTART
 *                 when the staging slots are full (crypto.c:1451-1459 then
 *                 queues the request and blocks the driver until
 *                 crypto_unblock); every other failure completes the request
 *                 through crypto_done with crp_etype set, as swcr_process does.
 *   GPU failure   requests the engine held complete with EIO (a clean drop);
 *                 later ones move their session to cryptosoft
 *                 (gpucrypto_migrate: EAGAIN with a new session, the
 *                 framework's own CRYPTOCAP_F_CLEANUP protocol); the probe
 *                 declines, so new sessions go to cryptosoft.
 * Completions come back on the lcore thread from ff_gpucrypto_poll() (host
 * domain, main_loop) through ff_gpucrypto_done() below.
 *
 * Built two ways: with the FreeBSD headers in F-Stack's kernel domain, where
 * it is a DRIVER_MODULE on lib/ff_newbus.c's nexus0
 * (tests/test_fstack_build.py compiles and link-checks that build), and with
 * -DFF_GPUCRYPTO_KMOCK against integration/kmock, a test double of the
 * crypto KPI that the CPU and GPU tests drive.
 *
 * Errors cross the boundary as libespgpu's ABI codes (include/espgpu.h) and
 * are translated to FreeBSD kernel errno here, in gpucrypto_errno().
 */
#ifdef FF_GPUCRYPTO_KMOCK
#include "kmock/kmock.h"
#else
#include <sys/param.h>
#include <sys/systm.h>
#include <sys/bus.h>
#include <sys/errno.h>
#include <sys/kernel.h>
#include <sys/mbuf.h>
#include <sys/module.h>
#include <opencrypto/cryptodev.h>
#include "cryptodev_if.h"
#endif

#include "espgpu.h"

#define GPUCRYPTO_MAX_SEGS 16      /* ESP chains are <= 5 mbufs for 9000-B jumbos */

struct gpucrypto_session {
	int32_t sid;               /* libespgpu session slot */
};

/* host-domain entry points (lib/ff_gpucrypto_host.c) */
int  ff_gpucrypto_host_probe(const struct espgpu_session_params *csp);
int  ff_gpucrypto_host_newsession(const struct espgpu_session_params *csp, int32_t *sid);
void ff_gpucrypto_host_freesession(int32_t sid);
int  ff_gpucrypto_host_process(const struct espgpu_req *r, int hint);
int  ff_gpucrypto_host_failed(void);

/* kernel-domain entry points the host domain calls (lib/ff_api.symlist) */
void ff_gpucrypto_done(void *opaque, int abi_etype);
void ff_gpucrypto_unblock(void);

static int32_t gpucrypto_id = -1;

int gpucrypto_errno(int abi);

/* libespgpu ABI code -> FreeBSD errno (sys/errno.h) */
int
gpucrypto_errno(int abi)
{
	switch (abi) {
	case ESPGPU_OK:       return (0);
	case ESPGPU_EIO:      return (EIO);          /* GPU failure: a clean drop */
	case ESPGPU_EINVAL:   return (EINVAL);
	case ESPGPU_EBADMSG:  return (EBADMSG);      /* 89 */
	case ESPGPU_ERESTART: return (ERESTART);     /* -1 */
	case ESPGPU_EAGAIN:   return (EAGAIN);       /* 35 */
	case ESPGPU_ENOMEM:   return (ENOMEM);
	case ESPGPU_ENOBUFS:  return (ENOBUFS);
	case ESPGPU_ENXIO:    return (ENXIO);
	case ESPGPU_ENODEV:   return (ENODEV);
	case ESPGPU_ENOENT:   return (ENOENT);
	case ESPGPU_ENOTSUP:  return (EOPNOTSUPP);   /* 45 */
	default:              return (EIO);
	}
}

static void
gpucrypto_csp(const struct crypto_session_params *csp, struct espgpu_session_params *m)
{
	m->csp_mode = csp->csp_mode;
	m->csp_flags = csp->csp_flags;
	m->csp_ivlen = csp->csp_ivlen;
	m->csp_cipher_alg = csp->csp_cipher_alg;
	m->csp_cipher_klen = csp->csp_cipher_klen;
	m->csp_cipher_key = csp->csp_cipher_key;
	m->csp_auth_alg = csp->csp_auth_alg;
	m->csp_auth_klen = csp->csp_auth_klen;
	m->csp_auth_key = csp->csp_auth_key;
	m->csp_auth_mlen = csp->csp_auth_mlen;
}

static int
gpucrypto_probesession(device_t dev, const struct crypto_session_params *csp)
{
	struct espgpu_session_params m;
	int r;

	(void)dev;
	gpucrypto_csp(csp, &m);
	r = ff_gpucrypto_host_probe(&m);
	return (r == ESPGPU_PROBE_HARDWARE ? CRYPTODEV_PROBE_HARDWARE : gpucrypto_errno(r));
}

static int
gpucrypto_newsession(device_t dev, crypto_session_t cses, const struct crypto_session_params *csp)
{
	struct gpucrypto_session *s = crypto_get_driver_session(cses);
	struct espgpu_session_params m;

	(void)dev;
	gpucrypto_csp(csp, &m);
	return (gpucrypto_errno(ff_gpucrypto_host_newsession(&m, &s->sid)));
}

static void
gpucrypto_freesession(device_t dev, crypto_session_t cses)
{
	struct gpucrypto_session *s = crypto_get_driver_session(cses);

	(void)dev;
	ff_gpucrypto_host_freesession(s->sid);
	s->sid = -1;
}

static int
gpucrypto_fail(struct cryptop *crp, int error)
{
	crp->crp_etype = error;
	crypto_done(crp);
	return (0);
}

/*
 * The GPU failed (the engine's espgpu_health; its held requests complete
 * with EIO through ff_gpucrypto_done).  This driver cannot unregister:
 * crypto_unregister_all waits in mtx_sleep until the driver's sessions are
 * gone (crypto.c:1178-1179) and F-Stack's _sleep returns at once
 * (lib/ff_kern_synch.c:87-92), so it would spin forever.  Instead it does for
 * each of its sessions, on that session's next request, what crypto_invoke
 * does for a driver that did unregister (the CRYPTOCAP_F_CLEANUP branch,
 * crypto.c:1684-1725): a new session on the same parameters -- the probe
 * now declines, so crypto_newsession selects cryptosoft -- goes into the
 * request, which completes with EAGAIN; esp_input_cb / esp_output_cb then
 * move the SA to that session and re-dispatch (xform_esp.c:505-512,
 * ipsec_updateid ipsec.c:1451-1495).  Unlike that branch the old session is
 * not freed here (its requests still held by the engine complete with EIO,
 * and a second request naming it would free it twice): once the SA has moved
 * nothing uses it, and it is left, one per SA.  Without another driver, or
 * should the new session land on this one, the request is a clean drop (EIO).
 */
static int
gpucrypto_migrate(struct cryptop *crp)
{
	crypto_session_t nses;

	if (crypto_newsession(&nses, crypto_get_params(crp->crp_session),
	    CRYPTOCAP_F_HARDWARE | CRYPTOCAP_F_SOFTWARE) != 0)
		return (gpucrypto_fail(crp, EIO));
	if (gpucrypto_id >= 0 && crypto_ses2hid(nses) == (uint32_t)gpucrypto_id) {
		crypto_freesession(nses);
		return (gpucrypto_fail(crp, EIO));
	}
	crp->crp_session = nses;
	return (gpucrypto_fail(crp, EAGAIN));
}

static int
gpucrypto_process(device_t dev, struct cryptop *crp, int hint)
{
	struct gpucrypto_session *s = crypto_get_driver_session(crp->crp_session);
	struct espgpu_seg segs[GPUCRYPTO_MAX_SEGS];
	struct espgpu_req r;
	struct mbuf *m;
	int n = 0, e;

	(void)dev;
	if (ff_gpucrypto_host_failed())
		return (gpucrypto_migrate(crp));
	/* in place only; session keys only (ESP never rekeys per request) */
	if (CRYPTO_HAS_OUTPUT_BUFFER(crp) || crp->crp_cipher_key != NULL ||
	    crp->crp_auth_key != NULL)
		return (gpucrypto_fail(crp, EINVAL));
	switch (crp->crp_buf.cb_type) {
	case CRYPTO_BUF_MBUF:
		for (m = crp->crp_buf.cb_mbuf; m != NULL; m = m->m_next) {
			if (n == GPUCRYPTO_MAX_SEGS)
				return (gpucrypto_fail(crp, EINVAL));
			segs[n].base = mtod(m, void *);
			segs[n].len = (uint32_t)m->m_len;
			n++;
		}
		break;
	case CRYPTO_BUF_CONTIG:
		segs[0].base = crp->crp_buf.cb_buf;
		segs[0].len = (uint32_t)crp->crp_buf.cb_buf_len;
		n = 1;
		break;
	default:
		return (gpucrypto_fail(crp, EINVAL));
	}
	memset(&r, 0, sizeof(r));
	r.session = s->sid;
	r.crp_op = crp->crp_op;
	r.crp_flags = crp->crp_flags;
	r.segs = segs;
	r.nsegs = n;
	r.crp_aad = crp->crp_aad;
	r.crp_aad_start = crp->crp_aad_start;
	r.crp_aad_length = crp->crp_aad_length;
	memcpy(r.crp_esn, crp->crp_esn, 4);
	r.crp_iv_start = crp->crp_iv_start;
	r.crp_payload_start = crp->crp_payload_start;
	r.crp_payload_length = crp->crp_payload_length;
	r.crp_digest_start = crp->crp_digest_start;
	memcpy(r.crp_iv, crp->crp_iv, sizeof(r.crp_iv));
	r.opaque = crp;
	/* segs[] is copied by the engine before it returns */
	e = ff_gpucrypto_host_process(&r, hint);
	if (e == ESPGPU_OK)
		return (0);
	if (e == ESPGPU_ERESTART)
		return (ERESTART);                  /* framework queues + blocks */
	if (e == ESPGPU_EIO && ff_gpucrypto_host_failed())
		return (gpucrypto_migrate(crp));    /* the GPU failed under this request */
	return (gpucrypto_fail(crp, gpucrypto_errno(e)));
}

void
ff_gpucrypto_done(void *opaque, int abi_etype)
{
	struct cryptop *crp = opaque;

	crp->crp_etype = gpucrypto_errno(abi_etype);
	crypto_done(crp);                         /* crypto.c:1802, inline for CBIFSYNC */
}

void
ff_gpucrypto_unblock(void)
{
	if (gpucrypto_id >= 0)
		crypto_unblock((uint32_t)gpucrypto_id, CRYPTO_SYMQ);   /* crypto.c:1191 */
}

static int
gpucrypto_attach(device_t dev)
{
	gpucrypto_id = crypto_get_driverid(dev, sizeof(struct gpucrypto_session),
	    CRYPTOCAP_F_HARDWARE | CRYPTOCAP_F_SYNC);
	if (gpucrypto_id < 0)
		return (ENXIO);
	return (0);
}

static int
gpucrypto_detach(device_t dev)
{
	(void)dev;
	if (gpucrypto_id >= 0)
		crypto_unregister_all((uint32_t)gpucrypto_id);
	gpucrypto_id = -1;
	return (0);
}

#ifdef FF_GPUCRYPTO_KMOCK
const struct kmock_cryptodev ff_gpucrypto_kmock = {
	"gpucrypto", gpucrypto_attach, gpucrypto_detach, gpucrypto_probesession,
	gpucrypto_newsession, gpucrypto_freesession, gpucrypto_process,
};
#else
/*
 * In F-Stack: a newbus driver on nexus0 (lib/ff_newbus.c), attached like
 * cryptosoft (cryptosoft.c:1443-1510) when mi_startup loads the
 * DRIVER_MODULEs, after cryptosoft's own module has run crypto_init
 * (SI_ORDER_ANY sorts after DRIVER_MODULE's SI_ORDER_MIDDLE).  ff_init()
 * opens the GPU context before ff_freebsd_init() (ff_gpucrypto_host_init_proc);
 * without one the probe declines and cryptosoft keeps every session.
 */
#include "bus_if.h"
#include "device_if.h"

int ff_gpucrypto_host_ready(void);

static void
gpucrypto_identify(driver_t *drv, device_t parent)
{
	(void)drv;
	if (device_find_child(parent, "gpucrypto", -1) == NULL)
		BUS_ADD_CHILD(parent, 0, "gpucrypto", 0);
}

static int
gpucrypto_probe(device_t dev)
{
	if (!ff_gpucrypto_host_ready())
		return (ENXIO);
	device_set_desc(dev, "MI355X ESP bulk crypto (libespgpu)");
	return (BUS_PROBE_NOWILDCARD);
}

static device_method_t gpucrypto_methods[] = {
	DEVMETHOD(device_identify,	gpucrypto_identify),
	DEVMETHOD(device_probe,		gpucrypto_probe),
	DEVMETHOD(device_attach,	gpucrypto_attach),
	DEVMETHOD(device_detach,	gpucrypto_detach),

	DEVMETHOD(cryptodev_probesession, gpucrypto_probesession),
	DEVMETHOD(cryptodev_newsession,	gpucrypto_newsession),
	DEVMETHOD(cryptodev_freesession, gpucrypto_freesession),
	DEVMETHOD(cryptodev_process,	gpucrypto_process),

	DEVMETHOD_END
};

static driver_t gpucrypto_driver = {
	"gpucrypto",
	gpucrypto_methods,
	0,		/* no softc */
};
static devclass_t gpucrypto_devclass;

EARLY_DRIVER_MODULE_ORDERED(gpucrypto, nexus, gpucrypto_driver, gpucrypto_devclass,
    NULL, NULL, SI_ORDER_ANY, BUS_PASS_DEFAULT);
MODULE_VERSION(gpucrypto, 1);
MODULE_DEPEND(gpucrypto, crypto, 1, 1, 1);
#endif
