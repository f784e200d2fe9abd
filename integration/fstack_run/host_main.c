/*
 * host_main.c -- runs F-Stack's kernel domain (libfstack.ro, compiled by
 * lib/Makefile's own rules) with cryptosoft and the MI355X opencrypto driver
 * attached, and pushes ESP requests through the reference's crypto.c:
 *
 *   1. the engine comes up before the FreeBSD stack, as in the patched
 *      ff_init() (ff_gpucrypto_host_init_proc before ff_freebsd_init):
 *      the GPU build opens device 0 (F-Stack mode, host overflow), the CPU
 *      build the oracle stand-in (oracle_engine.c);
 *   2. ff_freebsd_init() -> mi_startup(): SYSINITs, DRIVER_MODULE(cryptosoft)
 *      -> lib/ff_newbus.c driver_module_handler -> crypto_modevent ->
 *      crypto_init (crypto.c:320), cryptosoft and gpucrypto attach
 *      (crypto_get_driverid);
 *   3. per session two crypto_newsession calls: crid = HARDWARE|SOFTWARE
 *      (esp_init's V_crypto_support: crypto_select_driver must pick the
 *      driver bidding -100 over cryptosoft's -500) and crid = SOFTWARE
 *      (cryptosoft, the reference path itself);
 *   4. every request crypto_dispatch'ed on both (mbuf chains or contiguous
 *      buffers), main_loop's ff_gpucrypto_poll() until each callback has run
 *      (crypto_done inline: no crypto_ret thread runs in F-Stack);
 *   4b. without --fail, a full SA table: the next session goes to cryptosoft
 *   5. with --fail, the GPU-failure path: the engine
 *      fails (GPU build: set_tuning "fault" 1, the next launch fails; CPU
 *      build: the stand-in fails with the requests staged), every request is
 *      dispatched again on the gpucrypto sessions and must complete exactly
 *      once, with EIO and its buffer untouched; then once more: each now
 *      completes with EAGAIN and a cryptosoft session (gpucrypto_migrate,
 *      the framework's CRYPTOCAP_F_CLEANUP protocol), and its re-dispatch
 *      (esp_input_cb's EAGAIN path) runs on cryptosoft.
 *
 *   fstack_crypto_run <requests.bin> <results.bin> [--fail]
 * File formats: integration/fstack_run.py (pack_requests / read_results).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ff_config.h"

#define CAP_HW 0x01000000         /* CRYPTOCAP_F_HARDWARE, cryptodev.h:641 */
#define CAP_SW 0x02000000         /* CRYPTOCAP_F_SOFTWARE */

int   ff_freebsd_init(void);
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
int   ff_gpucrypto_poll(void);
int   ff_gpucrypto_host_failed(void);

#ifdef FSR_GPU
int ff_gpucrypto_host_init_proc(int proc_id);
void ff_gpucrypto_host_fini(void);
int ff_gpucrypto_host_tune(const char *key, int value);
#else
void oracle_engine_init(void);
void oracle_engine_fail(void);
#endif

struct ses_rec {                  /* 8 ints, 32 + 128 key bytes */
	int32_t p[8];
	uint8_t ckey[32], akey[128];
};
struct req_hdr {                  /* 11 ints, aad 16, esn 4, iv 16, ncuts, cuts[16], len */
	int32_t ses, f[11];
	uint8_t aad[16], esn[4], iv[16];
	int32_t ncuts, cuts[16], len;
};

static void
die(const char *m)
{
	fprintf(stderr, "fstack_crypto_run: %s\n", m);
	exit(2);
}

static void
rd(FILE *f, void *p, size_t n)
{
	if (fread(p, 1, n, f) != n)
		die("short read");
}

static double
now(void)
{
	struct timespec t;

	clock_gettime(CLOCK_MONOTONIC, &t);
	return (t.tv_sec + t.tv_nsec * 1e-9);
}

int
main(int argc, char **argv)
{
	FILE *in, *out;
	uint32_t magic, nses, nreq;

	const int fail = argc == 4 && strcmp(argv[3], "--fail") == 0;
	if (argc != 3 && !fail)
		die("usage: fstack_crypto_run <requests.bin> <results.bin> [--fail]");
	in = fopen(argv[1], "rb");
	if (in == NULL)
		die("cannot open requests");
	rd(in, &magic, 4);
	rd(in, &nses, 4);
	rd(in, &nreq, 4);
	if (magic != 0x52435346u)                 /* "FSCR" */
		die("bad magic");

	/* lib/ff_config.c defaults for the [freebsd] section */
	ff_global_cfg.freebsd.hz = 100;
	ff_global_cfg.freebsd.physmem = 1048576 * 256;
	ff_global_cfg.freebsd.fd_reserve = 0;
#ifdef FSR_GPU
	if (ff_gpucrypto_host_init_proc(0) != 0)
		die("no GPU context");
#else
	oracle_engine_init();
#endif
	if (ff_freebsd_init() != 0)
		die("ff_freebsd_init failed");
	const int gpu_hid = ffst_find_driver("gpucrypto"), sw_hid = ffst_find_driver("cryptosoft");

	struct ses_rec *ss = calloc(nses, sizeof(*ss));
	void **sdef = calloc(nses, sizeof(void *)), **ssw = calloc(nses, sizeof(void *));
	int32_t *sinfo = calloc(4 * (size_t)nses, sizeof(int32_t));
	for (uint32_t i = 0; i < nses; i++) {
		rd(in, &ss[i], sizeof(ss[i]));
		sdef[i] = ffst_newsession(ss[i].p, ss[i].ckey, ss[i].akey, CAP_HW | CAP_SW, &sinfo[4 * i], &sinfo[4 * i + 1]);
		ssw[i] = ffst_newsession(ss[i].p, ss[i].ckey, ss[i].akey, CAP_SW, &sinfo[4 * i + 2], &sinfo[4 * i + 3]);
	}
	struct req_hdr *rh = calloc(nreq, sizeof(*rh));
	uint8_t **bufs = calloc(nreq, sizeof(void *));
	void **rdef = calloc(nreq, sizeof(void *)), **rsw = calloc(nreq, sizeof(void *));
	int32_t *disp = calloc(2 * (size_t)nreq, sizeof(int32_t));
	for (uint32_t i = 0; i < nreq; i++) {
		rd(in, &rh[i], sizeof(rh[i]));
		bufs[i] = malloc((size_t)rh[i].len);
		rd(in, bufs[i], (size_t)rh[i].len);
	}
	fclose(in);

	/* the burst through the default (selected) driver: all dispatched,
	 * then main_loop iterations until every callback ran */
	double t0 = now();
	for (uint32_t i = 0; i < nreq; i++) {
		if (sdef[rh[i].ses] == NULL)
			continue;
		rdef[i] = ffst_request(sdef[rh[i].ses], rh[i].f, rh[i].aad, rh[i].esn, rh[i].iv, bufs[i], rh[i].len,
		    rh[i].cuts, rh[i].ncuts);
		if (rdef[i] == NULL)
			die("request");
		disp[2 * i] = ffst_dispatch(rdef[i]);
	}
	uint8_t *tmp = malloc(65536 + 64);
	for (;;) {
		int pending = 0, fl;
		for (uint32_t i = 0; i < nreq; i++)
			if (rdef[i] && ffst_result(rdef[i], tmp, 0, &fl) < 0)
				pending++;
		if (!pending)
			break;
		ff_gpucrypto_poll();
		if (now() - t0 > 60)
			die("requests did not complete");
	}
	/* the same requests through cryptosoft (synchronous: done at dispatch) */
	for (uint32_t i = 0; i < nreq; i++) {
		if (ssw[rh[i].ses] == NULL)
			continue;
		rsw[i] = ffst_request(ssw[rh[i].ses], rh[i].f, rh[i].aad, rh[i].esn, rh[i].iv, bufs[i], rh[i].len,
		    rh[i].cuts, rh[i].ncuts);
		if (rsw[i] == NULL)
			die("request");
		disp[2 * i + 1] = ffst_dispatch(rsw[i]);
	}

	/* 4b. a full SA table: new sessions on the parameters of a session the
	 * driver holds, until one lands on cryptosoft -- the probe declines on a
	 * full table, where CRYPTODEV_NEWSESSION failing would fail the SA
	 * (crypto.c:954-958) -- then, with one GPU session freed, the next lands
	 * on the GPU again */
	if (!fail) {
		enum { MAXS = 8192 };
		void **xs = calloc(MAXS, sizeof(void *));
		int nx = 0, ngpu = 0, err = 0, hid = -1, g = -1;
		for (uint32_t i = 0; i < nses && g < 0; i++)
			if (sinfo[4 * i + 1] == gpu_hid)
				g = (int)i;
		if (g < 0)
			die("SA-table fill: no session on gpucrypto");
		while (nx < MAXS) {
			xs[nx] = ffst_newsession(ss[g].p, ss[g].ckey, ss[g].akey, CAP_HW | CAP_SW, &err, &hid);
			if (xs[nx] == NULL)
				die("SA-table fill: crypto_newsession failed");
			nx++;
			if (hid != gpu_hid)
				break;
			ngpu++;
		}
		if (hid != sw_hid || ngpu == 0)
			die("SA-table fill: the full table did not hand the session to cryptosoft");
		ffst_freesession(xs[0]);
		xs[0] = ffst_newsession(ss[g].p, ss[g].ckey, ss[g].akey, CAP_HW | CAP_SW, &err, &hid);
		if (xs[0] == NULL || hid != gpu_hid)
			die("SA-table fill: a freed slot was not reused");
		for (int i = 0; i < nx; i++)
			ffst_freesession(xs[i]);
		free(xs);
		printf("SA table full after %d more sessions on gpucrypto: the next went to cryptosoft\n", ngpu);
	}

	/* 5. the GPU-failure phase: f1 = the requests the engine holds when it
	 * fails, f2 = requests after it */
	void **rf1 = calloc(nreq, sizeof(void *)), **rf2 = calloc(nreq, sizeof(void *));
	int32_t *fv = calloc(8 * (size_t)nreq, sizeof(int32_t));
	if (fail) {
#ifdef FSR_GPU
		if (ff_gpucrypto_host_tune("fault", 1) != 0)
			die("fault injection refused");
#endif
		for (uint32_t i = 0; i < nreq; i++) {
			if (sdef[rh[i].ses] == NULL || sinfo[4 * rh[i].ses + 1] != gpu_hid)
				continue;
			rf1[i] = ffst_request(sdef[rh[i].ses], rh[i].f, rh[i].aad, rh[i].esn, rh[i].iv, bufs[i],
			    rh[i].len, rh[i].cuts, rh[i].ncuts);
			if (rf1[i] == NULL)
				die("request");
			fv[8 * i] = ffst_dispatch(rf1[i]);
		}
#ifndef FSR_GPU
		oracle_engine_fail();
#endif
		double t1 = now();
		for (;;) {
			int pending = 0, fl;
			for (uint32_t i = 0; i < nreq; i++)
				if (rf1[i] && ffst_result(rf1[i], tmp, 0, &fl) < 0)
					pending++;
			if (!pending)
				break;
			ff_gpucrypto_poll();
			if (now() - t1 > 30)
				die("requests held at the failure did not complete");
		}
		for (int k = 0; k < 16; k++)           /* more main-loop iterations deliver nothing twice */
			ff_gpucrypto_poll();
		if (!ff_gpucrypto_host_failed())
			die("the engine does not report the failure");
		for (uint32_t i = 0; i < nreq; i++) {
			int hid;
			if (rf1[i] == NULL)
				continue;
			/* a request dispatched as the engine failed (the one whose staging
			 * found the slot full and the launch failing) was refused, not
			 * held: it completed with EAGAIN on a cryptosoft session, and
			 * esp_input_cb re-dispatches it */
			fv[8 * i + 1] = ffst_ndone(rf1[i]);
			if (ffst_redispatch(rf1[i], &fv[8 * i + 2], &hid) != -1 && hid != sw_hid)
				die("moved to a session not on cryptosoft");
			fv[8 * i + 3] = ffst_ndone(rf1[i]);
			rf2[i] = ffst_request(sdef[rh[i].ses], rh[i].f, rh[i].aad, rh[i].esn, rh[i].iv, bufs[i],
			    rh[i].len, rh[i].cuts, rh[i].ncuts);
			if (rf2[i] == NULL)
				die("request");
			if (ffst_dispatch(rf2[i]) != 0)                /* completes at once (EAGAIN) */
				die("dispatch after the failure");
			fv[8 * i + 4] = ffst_redispatch(rf2[i], &fv[8 * i + 5], &fv[8 * i + 6]);
			fv[8 * i + 7] = ffst_ndone(rf2[i]);
		}
	}

	out = fopen(argv[2], "wb");
	if (out == NULL)
		die("cannot open results");
	magic = 0x53525346u;                      /* "FSRS" */
	fwrite(&magic, 4, 1, out);
	fwrite(&nses, 4, 1, out);
	fwrite(&nreq, 4, 1, out);
	fwrite(&gpu_hid, 4, 1, out);
	fwrite(&sw_hid, 4, 1, out);
	fwrite(sinfo, 4, 4 * (size_t)nses, out);
	for (uint32_t i = 0; i < nreq; i++) {
		int32_t v[6] = { -2, 0, -2, 0, disp[2 * i], disp[2 * i + 1] };
		uint8_t *b0 = calloc(1, (size_t)rh[i].len + 1), *b1 = calloc(1, (size_t)rh[i].len + 1);
		if (rdef[i])
			v[0] = ffst_result(rdef[i], b0, rh[i].len, &v[1]);
		if (rsw[i])
			v[2] = ffst_result(rsw[i], b1, rh[i].len, &v[3]);
		fwrite(v, 4, 6, out);
		fwrite(b0, 1, (size_t)rh[i].len, out);
		fwrite(b1, 1, (size_t)rh[i].len, out);
		if (fail) {
			/* f1: dispatch, crypto_done calls when the poll had run, the first
			 * etype, crypto_done calls in all, final etype, buffer; f2: redispatch
			 * rc, etype before it (EAGAIN), session hid after the move, crypto_done
			 * calls, final etype, buffer */
			int32_t w[10] = { fv[8 * i], fv[8 * i + 1], fv[8 * i + 2], fv[8 * i + 3], -2, fv[8 * i + 4],
			    fv[8 * i + 5], fv[8 * i + 6], fv[8 * i + 7], -2 };
			int fl;
			memset(b0, 0, (size_t)rh[i].len);
			memset(b1, 0, (size_t)rh[i].len);
			if (rf1[i])
				w[4] = ffst_result(rf1[i], b0, rh[i].len, &fl);
			if (rf2[i])
				w[9] = ffst_result(rf2[i], b1, rh[i].len, &fl);
			fwrite(w, 4, 10, out);
			fwrite(b0, 1, (size_t)rh[i].len, out);
			fwrite(b1, 1, (size_t)rh[i].len, out);
			if (rf1[i])
				ffst_free(rf1[i]);
			if (rf2[i])
				ffst_free(rf2[i]);
		}
		free(b0);
		free(b1);
		if (rdef[i])
			ffst_free(rdef[i]);
		if (rsw[i])
			ffst_free(rsw[i]);
	}
	fclose(out);
	for (uint32_t i = 0; i < nses; i++) {
		if (sdef[i])
			ffst_freesession(sdef[i]);
		if (ssw[i])
			ffst_freesession(ssw[i]);
	}
#ifdef FSR_GPU
	ff_gpucrypto_host_fini();
#endif
	printf("fstack_crypto_run OK: %u sessions, %u requests, gpucrypto hid %d, cryptosoft hid %d\n", nses, nreq,
	    gpu_hid, sw_hid);
	return (0);
}
