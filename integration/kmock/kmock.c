/* kmock.c -- the framework side of kmock.h (see there). */
#include <stdlib.h>

#include "kmock.h"

struct crypto_session {
	const struct kmock_cryptodev *drv;
	struct crypto_session_params csp;
	void *softc;                    /* cc_session_size bytes for the driver */
};

static const struct kmock_cryptodev *g_drv;
static struct kmock_stats g_st;
static struct cryptop *q_head, *q_tail;
static struct kmock_device { int unit; } g_dev;
static int g_soft;

/* cryptosoft's part (kmock_soft_enable): bids for everything, completes a
 * request with etype 0, transforms nothing */
static int soft_probe(device_t dev, const struct crypto_session_params *csp)
{
	(void)dev; (void)csp;
	return CRYPTODEV_PROBE_SOFTWARE;
}
static int soft_newsession(device_t dev, crypto_session_t cses, const struct crypto_session_params *csp)
{
	(void)dev; (void)cses; (void)csp;
	g_st.soft_sessions++;
	return 0;
}
static void soft_freesession(device_t dev, crypto_session_t cses)
{
	(void)dev; (void)cses;
	g_st.soft_sessions--;
}
static int soft_process(device_t dev, struct cryptop *crp, int hint)
{
	(void)dev; (void)hint;
	g_st.soft_done++;
	crp->crp_etype = 0;
	crypto_done(crp);
	return 0;
}
static const struct kmock_cryptodev g_soft_drv = {
	"cryptosoft", NULL, NULL, soft_probe, soft_newsession, soft_freesession, soft_process,
};

void kmock_soft_enable(int on) { g_soft = on; }

void *crypto_get_driver_session(crypto_session_t cses) { return cses->softc; }

const struct crypto_session_params *crypto_get_params(crypto_session_t cses) { return &cses->csp; }

uint32_t crypto_ses2hid(crypto_session_t cses)
{
	return cses->drv == &g_soft_drv ? KMOCK_SOFT_ID : (uint32_t)g_st.driverid;
}

int32_t crypto_get_driverid(device_t dev, size_t session_size, int flags)
{
	(void)dev;
	if ((flags & (CRYPTOCAP_F_HARDWARE | CRYPTOCAP_F_SOFTWARE)) == 0)
		return -1;                                   /* crypto.c:995 */
	g_st.driverid = 7;
	g_st.caps = flags;
	g_st.session_size = session_size;
	return g_st.driverid;
}

int crypto_unregister_all(uint32_t driverid)
{
	if ((int32_t)driverid != g_st.driverid)
		return ENOENT;
	g_st.driverid = -1;
	return 0;
}

int crypto_unblock(uint32_t driverid, int what)
{
	if ((int32_t)driverid != g_st.driverid)
		return EINVAL;
	if (what & CRYPTO_SYMQ)
		g_st.blocked = 0;
	g_st.unblocks++;
	return 0;
}

void crypto_done(struct cryptop *crp)
{
	crp->crp_flags |= CRYPTO_F_DONE;
	g_st.done++;
	if (crp->crp_callback)
		crp->crp_callback(crp);
}

int kmock_attach(const struct kmock_cryptodev *drv)
{
	memset(&g_st, 0, sizeof(g_st));
	g_st.driverid = -1;
	q_head = q_tail = NULL;
	g_drv = drv;
	g_soft = 0;
	return drv->attach(&g_dev);
}

void kmock_detach(void)
{
	if (g_drv && g_drv->detach)
		g_drv->detach(&g_dev);
	g_drv = NULL;
}

int crypto_newsession(crypto_session_t *out, const struct crypto_session_params *csp, int crid)
{
	const struct kmock_cryptodev *drv = g_drv;
	struct crypto_session *s;
	int e, pr;

	(void)crid;
	*out = NULL;
	/* the driver under test if attached and bidding hardware, else the
	 * software stand-in if enabled (crypto_select_driver's order) */
	pr = g_st.driverid >= 0 ? g_drv->probesession(&g_dev, csp) : EOPNOTSUPP;
	if (pr != CRYPTODEV_PROBE_HARDWARE) {
		if (!g_soft)
			return pr > 0 ? pr : EOPNOTSUPP;   /* an errno: this driver declines */
		drv = &g_soft_drv;
	}
	s = calloc(1, sizeof(*s));
	s->softc = calloc(1, g_st.session_size ? g_st.session_size : 1);
	s->drv = drv;
	s->csp = *csp;
	e = drv->newsession(&g_dev, s, csp);
	if (e) {
		free(s->softc);
		free(s);
		return e;
	}
	g_st.sessions++;
	*out = s;
	return 0;
}

int kmock_newsession(crypto_session_t *out, const struct crypto_session_params *csp)
{
	return crypto_newsession(out, csp, CRYPTOCAP_F_HARDWARE | CRYPTOCAP_F_SOFTWARE);
}

void crypto_freesession(crypto_session_t s)
{
	if (!s)
		return;
	s->drv->freesession(&g_dev, s);
	free(s->softc);
	free(s);
	g_st.sessions--;
}

void kmock_freesession(crypto_session_t s) { crypto_freesession(s); }

static void enqueue(struct cryptop *crp)
{
	crp->kmock_next = NULL;
	if (q_tail)
		q_tail->kmock_next = crp;
	else
		q_head = crp;
	q_tail = crp;
	g_st.queued++;
}

int kmock_dispatch(struct cryptop *crp)
{
	if (crp->crp_session->drv == &g_soft_drv)
		return g_soft_drv.process(&g_dev, crp, 0);
	if (!g_st.blocked) {
		int r = g_drv->process(&g_dev, crp, 0);
		if (r != ERESTART)
			return r;
		g_st.erestarts++;
		g_st.blocked = 1;          /* crypto_invoke's ERESTART: cc_qblocked */
	}
	enqueue(crp);
	return 0;
}

int kmock_run_queue(void)
{
	int n = 0;

	while (q_head && !g_st.blocked) {
		struct cryptop *crp = q_head;
		int r = g_drv->process(&g_dev, crp, 0);
		if (r == ERESTART) {
			g_st.erestarts++;
			g_st.blocked = 1;
			break;
		}
		q_head = crp->kmock_next;
		if (!q_head)
			q_tail = NULL;
		g_st.queued--;
		n++;
	}
	return n;
}

const struct kmock_stats *kmock_stats(void) { return &g_st; }
