/* fake_host.c -- a scripted stand-in for the host-domain shim
 * (ff_gpucrypto_host.c) so the kernel-domain driver's error paths run without
 * a GPU: up to FAKE_CAP requests stage, the next process() answers
 * ESPGPU_ERESTART; fake_poll() completes the staged ones with an etype the
 * request carries in the first ICV byte (0xBA -> ESPGPU_EBADMSG,
 * 0xE1 -> ESPGPU_EINVAL), then unblocks, exactly as ff_gpucrypto_poll does.
 * Probe is the real espgpu_probesession (device-free).
 * fake_gpu_fail() plays a GPU failure as the engine reports it (espgpu_health):
 * the staged requests complete with ESPGPU_EIO at the next fake_poll, process()
 * answers ESPGPU_EIO, probe and newsession ENXIO. */
#include <stdint.h>
#include <string.h>

#include "espgpu.h"

#define FAKE_CAP 4

void ff_gpucrypto_done(void *opaque, int abi_etype);
void ff_gpucrypto_unblock(void);

static struct { void *opaque; int etype; } staged[FAKE_CAP];
static int nstaged, next_sid, nfreed, failed;
int fake_freed_sid = -1, fake_last_nsegs;

void fake_gpu_fail(void)
{
	failed = 1;
	for (int i = 0; i < nstaged; i++)
		staged[i].etype = ESPGPU_EIO;
}

int ff_gpucrypto_host_failed(void) { return failed; }

int ff_gpucrypto_host_probe(const struct espgpu_session_params *csp)
{
	int r;

	if (failed)
		return ESPGPU_ENXIO;
	r = espgpu_probesession(csp);
	/* the 3-slot SA table below is full: decline, as the real shim does on
	 * espgpu_session_room() == 0 */
	return r == ESPGPU_PROBE_HARDWARE && next_sid - nfreed >= 3 ? ESPGPU_ENOMEM : r;
}

int ff_gpucrypto_host_newsession(const struct espgpu_session_params *csp, int32_t *sid)
{
	(void)csp;
	if (failed)
		return ESPGPU_ENXIO;
	*sid = next_sid++;
	return next_sid > 3 ? ESPGPU_ENOMEM : ESPGPU_OK;     /* a 3-slot SA table */
}

void ff_gpucrypto_host_freesession(int32_t sid)
{
	fake_freed_sid = sid;
	nfreed++;
}

static uint8_t byte_at(const struct espgpu_req *r, uint32_t off)
{
	for (int i = 0; i < r->nsegs; i++) {
		if (off < r->segs[i].len)
			return ((const uint8_t *)r->segs[i].base)[off];
		off -= r->segs[i].len;
	}
	return 0;
}

int ff_gpucrypto_host_process(const struct espgpu_req *r, int hint)
{
	uint8_t tag;

	(void)hint;
	if (failed)
		return ESPGPU_EIO;
	if (nstaged == FAKE_CAP)
		return ESPGPU_ERESTART;
	fake_last_nsegs = r->nsegs;
	tag = byte_at(r, (uint32_t)r->crp_digest_start);
	staged[nstaged].opaque = r->opaque;
	staged[nstaged].etype = tag == 0xBA ? ESPGPU_EBADMSG : tag == 0xE1 ? ESPGPU_EINVAL : ESPGPU_OK;
	nstaged++;
	return ESPGPU_OK;
}

int fake_poll(void)
{
	int n = nstaged;

	for (int i = 0; i < n; i++)
		ff_gpucrypto_done(staged[i].opaque, staged[i].etype);
	nstaged = 0;
	if (n)
		ff_gpucrypto_unblock();
	return n;
}
