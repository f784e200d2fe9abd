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

void *crypto_get_driver_session(crypto_session_t cses) { return cses->softc; }

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
	return drv->attach(&g_dev);
}

void kmock_detach(void)
{
	if (g_drv && g_drv->detach)
		g_drv->detach(&g_dev);
	g_drv = NULL;
}

int kmock_newsession(crypto_session_t *out, const struct crypto_session_params *csp)
{
	struct crypto_session *s;
	int e, pr = g_drv->probesession(&g_dev, csp);

	*out = NULL;
	if (pr > 0)
		return pr;                 /* an errno: this driver declines */
	if (pr != CRYPTODEV_PROBE_HARDWARE)
		return EOPNOTSUPP;
	s = calloc(1, sizeof(*s));
	s->softc = calloc(1, g_st.session_size ? g_st.session_size : 1);
	s->drv = g_drv;
	s->csp = *csp;
	e = g_drv->newsession(&g_dev, s, csp);
	if (e) {
		free(s->softc);
		free(s);
		return e;
	}
	*out = s;
	return 0;
}

void kmock_freesession(crypto_session_t s)
{
	if (!s)
		return;
	s->drv->freesession(&g_dev, s);
	free(s->softc);
	free(s);
}

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
