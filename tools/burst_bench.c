/*
 * burst_bench.c -- the opencrypto driver path (espgpu_process / flush / poll)
 * at F-Stack burst sizes: what one main_loop iteration sees (INTEGRATION.md
 * section 3: requests staged during the RX burst, one flush, completions
 * polled).  Measurement only.
 *
 *   make -C tools burst_bench && ./tools/burst_bench [burst ...]
 *
 * For each burst size B (default 32 = MAX_PKT_BURST, lib/ff_dpdk_if.c):
 *   latency   B decrypt requests staged, flushed, polled until all B have
 *             completed (one burst in flight); median / p99 over 2000 bursts
 *   pipelined bursts issued back to back, up to `nbatches` (2) in flight,
 *             completions polled between them: sustained records/s
 * Records: ESP AES-128-GCM, 1500-byte packets (1480-byte ESP records, one
 * contiguous buffer each), encrypted by the engine first, restored from a
 * copy before every decrypt so every tag verifies.  One JSON line per B.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "espgpu.h"

#define REC 1480
#define CK(x) do { int e_ = (x); if (e_) { fprintf(stderr, "%s -> %d (%s)\n", #x, e_, espgpu_last_error(ctx)); exit(1); } } while (0)

static espgpu_ctx *ctx;

static double now_us(void)
{
	struct timespec t;
	clock_gettime(CLOCK_MONOTONIC, &t);
	return t.tv_sec * 1e6 + t.tv_nsec / 1e3;
}

static int cmp_d(const void *a, const void *b)
{
	double x = *(const double *)a, y = *(const double *)b;
	return x < y ? -1 : x > y;
}

static void make_req(struct espgpu_req *r, struct espgpu_seg *seg, uint8_t *buf, int32_t sid, int enc,
                     const uint8_t salt[4], void *opaque)
{
	memset(r, 0, sizeof(*r));
	seg->base = buf;
	seg->len = REC;
	r->session = sid;
	r->crp_op = enc ? ESPGPU_CRYPTO_OP_ENCRYPT : ESPGPU_CRYPTO_OP_VERIFY_DIGEST;
	r->crp_flags = ESPGPU_CRYPTO_F_IV_SEPARATE;
	r->segs = seg;
	r->nsegs = 1;
	r->crp_aad_start = 0;
	r->crp_aad_length = 8;
	r->crp_payload_start = 16;
	r->crp_payload_length = REC - 32;
	r->crp_digest_start = REC - 16;
	memcpy(r->crp_iv, salt, 4);
	memcpy(r->crp_iv + 4, buf + 8, 8);
	r->opaque = opaque;
}

/* stage n requests (retrying ERESTART after a poll), return completions seen */
static int submit(struct espgpu_req *r, int n, int *done, int *bad)
{
	struct espgpu_completion c[1024];
	for (int i = 0; i < n; i++) {
		int e;
		while ((e = espgpu_process(ctx, &r[i], 0)) == ESPGPU_ERESTART) {
			espgpu_flush(ctx);
			int k = espgpu_poll(ctx, c, 1024);
			for (int j = 0; j < k; j++) *bad += c[j].etype != 0;
			*done += k;
		}
		if (e) {
			fprintf(stderr, "process: %d\n", e);
			exit(1);
		}
	}
	return 0;
}

int main(int argc, char **argv)
{
	int bursts[16], nb = 0;
	for (int i = 1; i < argc && nb < 16; i++) bursts[nb++] = atoi(argv[i]);
	if (!nb) { bursts[0] = 32; bursts[1] = 256; bursts[2] = 2048; nb = 3; }
	int maxb = 0;
	for (int i = 0; i < nb; i++) maxb = bursts[i] > maxb ? bursts[i] : maxb;

	struct espgpu_config cfg;
	memset(&cfg, 0, sizeof(cfg));
	CK(espgpu_init(&cfg, &ctx));
	uint8_t key[16], salt[4] = {1, 2, 3, 4};
	for (int i = 0; i < 16; i++) key[i] = (uint8_t)(i * 13 + 5);
	struct espgpu_session_params p;
	memset(&p, 0, sizeof(p));
	p.csp_mode = ESPGPU_CSP_MODE_AEAD;
	p.csp_ivlen = 12;
	p.csp_cipher_alg = ESPGPU_CRYPTO_AES_NIST_GCM_16;
	p.csp_cipher_klen = 16;
	p.csp_cipher_key = key;
	int32_t sid;
	CK(espgpu_newsession(ctx, &p, &sid));

	const int pool = maxb * 4;          /* distinct buffers so bursts in flight do not alias */
	uint8_t *bufs = malloc((size_t)pool * REC), *ct = malloc((size_t)pool * REC);
	struct espgpu_req *req = malloc(sizeof(*req) * pool);
	struct espgpu_seg *seg = malloc(sizeof(*seg) * pool);
	srand(3);
	for (size_t i = 0; i < (size_t)pool * REC; i++) bufs[i] = (uint8_t)rand();
	int done = 0, bad = 0;
	for (int i = 0; i < pool; i++) {
		memset(bufs + (size_t)i * REC + REC - 16, 0, 16);
		make_req(&req[i], &seg[i], bufs + (size_t)i * REC, sid, 1, salt, NULL);
	}
	submit(req, pool, &done, &bad);
	CK(espgpu_drain(ctx));
	struct espgpu_completion c[4096];
	while (espgpu_poll(ctx, c, 4096) > 0) {}
	memcpy(ct, bufs, (size_t)pool * REC);
	for (int i = 0; i < pool; i++)
		make_req(&req[i], &seg[i], bufs + (size_t)i * REC, sid, 0, salt, NULL);

	for (int bi = 0; bi < nb; bi++) {
		const int B = bursts[bi];
		const int iters = B <= 64 ? 2000 : (B <= 512 ? 400 : 60);
		double *lat = malloc(sizeof(double) * iters);
		bad = 0;
		/* latency: one burst in flight */
		for (int it = -20; it < iters; it++) {
			const int base = (it & 3) * B;
			memcpy(bufs + (size_t)base * REC, ct + (size_t)base * REC, (size_t)B * REC);
			done = 0;
			double t0 = now_us();
			submit(req + base, B, &done, &bad);
			espgpu_flush(ctx);
			while (done < B) {
				int k = espgpu_poll(ctx, c, 4096);
				for (int j = 0; j < k; j++) bad += c[j].etype != 0;
				done += k;
			}
			if (it >= 0) lat[it] = now_us() - t0;
		}
		const int bad_latency = bad;
		qsort(lat, iters, sizeof(double), cmp_d);
		const double med = lat[iters / 2], p99 = lat[(int)(iters * 0.99)];
		/* pipelined: bursts back to back, completions polled in between */
		const int total_bursts = iters;
		done = 0;
		double t0 = now_us();
		for (int it = 0; it < total_bursts; it++) {
			const int base = (it & 3) * B;
			/* a fresh burst of ciphertext arrives (inside the timed loop: the
			 * 4-burst buffer ring is only reused after its results are back) */
			while (done < (it - 3) * B) {
				int k = espgpu_poll(ctx, c, 4096);
				for (int j = 0; j < k; j++) bad += c[j].etype != 0;
				done += k;
			}
			memcpy(bufs + (size_t)base * REC, ct + (size_t)base * REC, (size_t)B * REC);
			submit(req + base, B, &done, &bad);
			espgpu_flush(ctx);
			int k = espgpu_poll(ctx, c, 4096);
			for (int j = 0; j < k; j++) bad += c[j].etype != 0;
			done += k;
		}
		while (done < total_bursts * B) {
			espgpu_flush(ctx);
			int k = espgpu_poll(ctx, c, 4096);
			for (int j = 0; j < k; j++) bad += c[j].etype != 0;
			done += k;
		}
		const double dt = now_us() - t0;
		printf("{\"burst\": %d, \"record_bytes\": %d, \"latency_us_median\": %.1f, \"latency_us_p99\": %.1f, "
		       "\"latency_records_per_s\": %.0f, \"pipelined_records_per_s\": %.0f, \"pipelined_GBps\": %.3f, "
		       "\"iters\": %d, \"auth_fail\": [%d, %d]}\n",
		       B, REC, med, p99, B / med * 1e6, total_bursts * (double)B / dt * 1e6,
		       total_bursts * (double)B * REC / dt / 1e3, iters, bad_latency, bad - bad_latency);
		fflush(stdout);
		free(lat);
	}
	espgpu_freesession(ctx, sid);
	espgpu_fini(ctx);
	return 0;
}
