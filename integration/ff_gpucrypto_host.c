/*
 * ff_gpucrypto_host.c — host-domain half of the F-Stack binding (INTEGRATION.md
 * section 2).  It would live in lib/ as an FF_HOST_SRCS file: libc/HIP
 * headers only, no FreeBSD kernel headers.  The kernel-domain driver
 * (lib/ff_gpucrypto.c) converts struct cryptop /
 * crypto_session_params into the espgpu_* mirrors and calls these entry
 * points; ff_gpucrypto_poll() runs once per main_loop iteration
 * (lib/ff_dpdk_if.c:2363) and hands completions back through
 * ff_gpucrypto_done() (kernel domain, listed in lib/ff_api.symlist).
 *
 * Built here against include/espgpu.h and f-stack_amd/libespgpu.so by
 * `make -C integration` (tests/test_integration.py), so the binding a
 * maintainer adds is compile- and link-checked, and with the kernel-domain
 * driver (ff_gpucrypto.c over integration/kmock) into kmock_gpu_test, which
 * runs the whole driver path on the GPU.  Return codes are libespgpu's ABI
 * codes; ff_gpucrypto.c translates them to FreeBSD errno.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include "espgpu.h"

/* kernel-domain callbacks (weak so this file links standalone for tests) */
void ff_gpucrypto_done(void *opaque, int etype) __attribute__((weak));
void ff_gpucrypto_unblock(void) __attribute__((weak));

static espgpu_ctx *g_ctx;          /* one F-Stack process = one lcore = one ctx */
/* F-Stack runs no crypto_proc thread (its kproc/kthread stubs never start
 * one, lib/ff_compat.c:156-171), so a request that crypto_dispatch queues on
 * ERESTART (crypto.c:1450-1459) would never be re-dispatched there.  With
 * no-queue set, the engine keeps requests that arrive while every staging
 * slot is in flight in a host overflow (set_tuning "overflow_mb"), launched
 * by the next ff_gpucrypto_poll(): process() never waits for the GPU
 * (cryptodev_if.m:143-147).  Past the overflow's size a request completes
 * with ENOBUFS: esp_input_cb drops it, as esp_input drops a packet it cannot
 * get a cryptop for (xform_esp.c:348-354). */
static int g_noqueue;
#define FF_GPUCRYPTO_OVERFLOW_MB 256

void ff_gpucrypto_host_set_noqueue(int on)
{
	g_noqueue = on;
	if (g_ctx)
		espgpu_set_tuning(g_ctx, "overflow_mb", on ? FF_GPUCRYPTO_OVERFLOW_MB : 0);
}

int ff_gpucrypto_host_init(int gpu)
{
	struct espgpu_config c = { 0 };

	c.device = gpu;
	return espgpu_init(&c, &g_ctx);
}

/* ff_init(): F-Stack process proc_id (one lcore) opens device
 * proc_id mod (visible devices): the GPUs are split by lcore, i.e. by the RSS
 * queues NIC steers to each lcore.
 * FF_GPUCRYPTO_DOOR=N (1..256) starts the doorbell path on N CUs: bursts are
 * handed to a resident kernel through pinned host memory instead of a launch
 * each (a 32-record burst 42 -> 25 us).  Off by default:
 * the resident kernel keeps N CUs while bursts arrive (it exits after 20 ms
 * without one). */
int ff_gpucrypto_host_init_proc(int proc_id)
{
	int n = espgpu_device_count(), e;
	const char *door;

	if (n <= 0)
		return ESPGPU_ENODEV;
	e = ff_gpucrypto_host_init(proc_id % n);
	if (e == ESPGPU_OK) {
		ff_gpucrypto_host_set_noqueue(1);
		door = getenv("FF_GPUCRYPTO_DOOR");
		if (door && atoi(door) > 0)
			espgpu_set_tuning(g_ctx, "door", atoi(door));
	}
	return e;
}

/* as ff_gpucrypto_host_init, with explicit staging sizes (batch_records,
 * batch_bytes, nbatches: how much a burst may stage before process() answers
 * ERESTART) */
int ff_gpucrypto_host_configure(const struct espgpu_config *c)
{
	return espgpu_init(c, &g_ctx);
}

/* Register mbuf memory (one DPDK mempool memory chunk; the patched
 * ff_dpdk_if.c walks the pktmbuf pools with rte_mempool_mem_iter after
 * ff_gpucrypto_host_init_proc): records in it are read and written back by
 * the GPU, with no gather into the staging buffer. */
int ff_gpucrypto_host_register(void *base, uint64_t len)
{
	return g_ctx ? espgpu_register_host(g_ctx, base, len) : ESPGPU_ENXIO;
}

/* the kernel-domain driver's device_probe: attach only with a GPU context */
int ff_gpucrypto_host_ready(void)
{
	return g_ctx != NULL;
}

void ff_gpucrypto_host_fini(void)
{
	if (g_ctx) {
		espgpu_drain(g_ctx);
		espgpu_fini(g_ctx);
		g_ctx = NULL;
	}
}

/* engine counters (overflow / zero-copy records, ERESTARTs) and knobs, for
 * the tests and an operator's sysctl-style view */
int ff_gpucrypto_host_stats(struct espgpu_stats *st)
{
	return g_ctx ? espgpu_get_stats(g_ctx, st) : ESPGPU_ENXIO;
}

int ff_gpucrypto_host_tune(const char *key, int value)
{
	return g_ctx ? espgpu_set_tuning(g_ctx, key, value) : ESPGPU_ENXIO;
}

/* the GPU context has failed (espgpu_health): the driver stops taking work */
int ff_gpucrypto_host_failed(void)
{
	return g_ctx != NULL && espgpu_health(g_ctx) != ESPGPU_OK;
}

/* CRYPTODEV_PROBESESSION: -100 (CRYPTODEV_PROBE_HARDWARE) or EINVAL; ENXIO
 * once the GPU has failed, so crypto_newsession picks cryptosoft.
 * Host-only, valid before ff_gpucrypto_host_init. */
int ff_gpucrypto_host_probe(const struct espgpu_session_params *csp)
{
	int r;

	if (ff_gpucrypto_host_failed())
		return ESPGPU_ENXIO;
	r = espgpu_probesession(csp);
	/* a full SA table declines here, so that crypto_newsession selects
	 * cryptosoft rather than failing the SA in CRYPTODEV_NEWSESSION
	 * (crypto.c:954-958) */
	if (r == ESPGPU_PROBE_HARDWARE && g_ctx && espgpu_session_room(g_ctx) == 0)
		return ESPGPU_ENOMEM;
	return r;
}

int ff_gpucrypto_host_newsession(const struct espgpu_session_params *csp, int32_t *sid)
{
	if (ff_gpucrypto_host_failed())
		return ESPGPU_ENXIO;
	return g_ctx ? espgpu_newsession(g_ctx, csp, sid) : ESPGPU_ENXIO;
}

void ff_gpucrypto_host_freesession(int32_t sid)
{
	if (g_ctx)
		espgpu_freesession(g_ctx, sid);
}

/* CRYPTODEV_PROCESS: ESPGPU_OK or ESPGPU_ERESTART (the driver returns
 * ERESTART and the framework requeues); the driver maps any other code
 * (ESPGPU_EIO on a failed GPU: the driver then moves the session) */
int ff_gpucrypto_host_process(const struct espgpu_req *r, int hint)
{
	int e;

	if (!g_ctx)
		return ESPGPU_ENXIO;
	e = espgpu_process(g_ctx, r, hint);
	if (e == ESPGPU_ERESTART && g_noqueue)
		e = ESPGPU_ENOBUFS;         /* overflow full: the driver completes it as a drop */
	return e;
}

/* main_loop hook: launch the burst's staged records, deliver completions */
int ff_gpucrypto_poll(void)
{
	struct espgpu_completion c[256];
	int n, i, total = 0, blocked;

	if (!g_ctx)
		return 0;
	blocked = espgpu_flush(g_ctx);
	while ((n = espgpu_poll(g_ctx, c, 256)) > 0) {
		for (i = 0; i < n; i++)
			if (ff_gpucrypto_done)
				ff_gpucrypto_done(c[i].opaque, c[i].etype);
		total += n;
	}
	/* slots the poll retired take the overflow now, not one loop later */
	if (total && !blocked)
		blocked = espgpu_flush(g_ctx);
	if (total && ff_gpucrypto_unblock)
		ff_gpucrypto_unblock();     /* crypto_unblock(id, CRYPTO_SYMQ), crypto.c:1191 */
	return blocked ? -blocked : total;
}
