/*
 * burst_bench.c -- the opencrypto driver path (espgpu_process / flush / poll)
 * at F-Stack burst sizes: what one main_loop iteration sees (INTEGRATION.md
 * section 3: requests staged during the RX burst, one flush, completions
 * polled).  Measurement only.
 *
 *   make -C tools burst_bench && ./tools/burst_bench [burst ...]
 *
 * For each burst size B (default 32 = MAX_PKT_BURST, lib/ff_dpdk_if.c) and
 * each way the records reach the GPU:
 *   mode   "gather"      records in ordinary (pageable) memory: process()
 *                        copies them into the pinned staging buffer;
 *          "registered"  the record buffers registered once
 *                        (espgpu_register_host, as F-Stack registers its mbuf
 *                        pools): the GPU reads them and writes the results
 *                        back, no CPU copy;
 *   xfer   1 = a small batch's staging region moved by the xfer kernel,
 *          0 = by hipMemcpyAsync (set_tuning "xfer");
 * it reports
 *   latency     B decrypt requests staged, flushed, polled until all B have
 *               completed (one burst in flight); median / p99 over the bursts
 *   pipelined   bursts issued back to back, completions polled in between,
 *               ERESTART answered by flush + poll + retry (overflow off)
 *   fstack      the F-Stack main_loop shape: per iteration stage B, flush,
 *               poll once, never wait; process() never sees ERESTART (host
 *               overflow on, set_tuning "overflow_mb")
 * Records: ESP AES-128-GCM, 1500-byte packets (1480-byte ESP records), each
 * in its own 2176-byte buffer at offset 162 = DPDK headroom 128 + Ethernet 14
 * + IPv4 20 (2 mod 4, where an mbuf puts them); encrypted by the engine first,
 * restored from a copy before every decrypt so every tag verifies.  One JSON
 * line per (B, mode, xfer).
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <dlfcn.h>

#include "espgpu.h"

#define REC 1480
#define STRIDE 2176                   /* RTE_MBUF_DEFAULT_BUF_SIZE: 2048 data room + 128 headroom */
#define OFF 162
#define RING 16                       /* bursts of buffers in the ring */
#define CK(x) do { int e_ = (x); if (e_) { fprintf(stderr, "%s -> %d (%s)\n", #x, e_, espgpu_last_error(ctx)); exit(1); } } while (0)

static espgpu_ctx *ctx;
static uint8_t *bufs, *ct;
static struct espgpu_req *req;
static struct espgpu_seg *seg;
static int pool;

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

/* the TSC, for timing single process() calls cheaply (clock_gettime around
 * every call costs as much as the call); ticks -> us calibrated at start */
static double tsc_us;
static inline unsigned long long tsc(void) { return __builtin_ia32_rdtsc(); }
static void calibrate_tsc(void)
{
	double t0 = now_us();
	unsigned long long c0 = tsc();
	while (now_us() - t0 < 20000) {}
	tsc_us = (now_us() - t0) / (double)(tsc() - c0);
}

static uint8_t *rec_of(int i) { return bufs + (size_t)i * STRIDE + OFF; }

static void make_req(struct espgpu_req *r, struct espgpu_seg *sg, uint8_t *buf, int32_t sid, int enc,
                     const uint8_t salt[4])
{
	memset(r, 0, sizeof(*r));
	sg->base = buf;
	sg->len = REC;
	r->session = sid;
	r->crp_op = enc ? ESPGPU_CRYPTO_OP_ENCRYPT : ESPGPU_CRYPTO_OP_VERIFY_DIGEST;
	r->crp_flags = ESPGPU_CRYPTO_F_IV_SEPARATE;
	r->segs = sg;
	r->nsegs = 1;
	r->crp_aad_start = 0;
	r->crp_aad_length = 8;
	r->crp_payload_start = 16;
	r->crp_payload_length = REC - 32;
	r->crp_digest_start = REC - 16;
	memcpy(r->crp_iv, salt, 4);
	memcpy(r->crp_iv + 4, buf + 8, 8);
}

static int poll_some(int *bad)
{
	struct espgpu_completion c[4096];
	int k = espgpu_poll(ctx, c, 4096);
	for (int j = 0; j < k; j++) *bad += c[j].etype != 0;
	return k;
}

/* stage n requests (retrying ERESTART after a flush + poll), return completions seen */
static void submit(struct espgpu_req *r, int n, int *done, int *bad)
{
	for (int i = 0; i < n; i++) {
		int e;
		while ((e = espgpu_process(ctx, &r[i], 0)) == ESPGPU_ERESTART) {
			espgpu_flush(ctx);
			*done += poll_some(bad);
		}
		if (e) {
			fprintf(stderr, "process: %d\n", e);
			exit(1);
		}
	}
}

static void restore(int base, int B)
{
	for (int i = base; i < base + B; i++)
		memcpy(rec_of(i), ct + (size_t)i * REC, REC);
}

/* bursts back to back; the ring of RING bursts is only reused once its
 * results are back.  fstack: process() must never answer ERESTART. */
static double pipelined(int B, int iters, int fstack, int *bad, double *worst_process_us)
{
	int done = 0;
	*worst_process_us = 0;
	double t0 = now_us();
	for (int it = 0; it < iters; it++) {
		const int base = (it % RING) * B;
		while (done < (it - (RING - 1)) * B) {
			espgpu_flush(ctx);
			done += poll_some(bad);
		}
		restore(base, B);
		if (fstack) {
			for (int i = 0; i < B; i++) {
				unsigned long long p0 = tsc();
				int e = espgpu_process(ctx, &req[base + i], 0);
				double dp = (double)(tsc() - p0) * tsc_us;
				*worst_process_us = dp > *worst_process_us ? dp : *worst_process_us;
				if (e) {
					fprintf(stderr, "fstack mode: process -> %d\n", e);
					exit(1);
				}
			}
		} else {
			submit(req + base, B, &done, bad);
		}
		espgpu_flush(ctx);
		done += poll_some(bad);
	}
	while (done < iters * B) {
		espgpu_flush(ctx);
		done += poll_some(bad);
	}
	return now_us() - t0;
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
	calibrate_tsc();
	/* BURST_TUNING="key=v,key=v": set_tuning before the runs (measurement knobs) */
	const char *tun = getenv("BURST_TUNING");
	if (tun) {
		char buf[256];
		snprintf(buf, sizeof buf, "%s", tun);
		for (char *kv = strtok(buf, ","); kv; kv = strtok(NULL, ",")) {
			char *eq = strchr(kv, '=');
			if (!eq) continue;
			*eq = 0;
			CK(espgpu_set_tuning(ctx, kv, atoi(eq + 1)));
		}
	}
	const int only_mode = getenv("BURST_MODE") ? atoi(getenv("BURST_MODE")) : -1;
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

	pool = maxb * RING;
	const size_t bytes = (size_t)pool * STRIDE;
	if (posix_memalign((void **)&bufs, 4096, bytes)) return 1;
	ct = malloc((size_t)pool * REC);
	req = malloc(sizeof(*req) * pool);
	seg = malloc(sizeof(*seg) * pool);
	srand(3);
	for (size_t i = 0; i < bytes; i++) bufs[i] = (uint8_t)rand();
	int done = 0, bad = 0;
	for (int i = 0; i < pool; i++) {
		memset(rec_of(i) + REC - 16, 0, 16);
		make_req(&req[i], &seg[i], rec_of(i), sid, 1, salt);
	}
	submit(req, pool, &done, &bad);
	CK(espgpu_drain(ctx));
	struct espgpu_completion c[4096];
	while (espgpu_poll(ctx, c, 4096) > 0) {}
	for (int i = 0; i < pool; i++) {
		memcpy(ct + (size_t)i * REC, rec_of(i), REC);
		make_req(&req[i], &seg[i], rec_of(i), sid, 0, salt);
	}

	int registered = 0;
	for (int mode = 0; mode < 2; mode++) {
		if (only_mode >= 0 && mode != only_mode) continue;
		if (mode == 1) {
			CK(espgpu_register_host(ctx, bufs, bytes));
			registered = 1;
		}
		for (int xfer = 1; xfer >= 0; xfer--) {
			CK(espgpu_set_tuning(ctx, "xfer", xfer));
			for (int bi = 0; bi < nb; bi++) {
				const int B = bursts[bi];
				const int iters = B <= 64 ? 2000 : (B <= 512 ? 400 : 60);
				double *lat = malloc(sizeof(double) * iters);
				struct espgpu_stats s0, s1;
				CK(espgpu_get_stats(ctx, &s0));
				bad = 0;
				/* latency: one burst in flight */
				for (int it = -20; it < iters; it++) {
					const int base = ((it + 20) % RING) * B;
					restore(base, B);
					done = 0;
					double t0 = now_us();
					submit(req + base, B, &done, &bad);
					espgpu_flush(ctx);
					while (done < B) done += poll_some(&bad);
					if (it >= 0) lat[it] = now_us() - t0;
				}
				const int bad_latency = bad;
				/* knobs library only: the small GCM kernel's phase clock of the
				 * last latency burst (workgroup 0, first chunk) */
				int (*phases)(unsigned long long *) =
					(int (*)(unsigned long long *))dlsym(RTLD_DEFAULT, "espgpu_debug_phases");
				unsigned long long ph[32];
				if (phases && phases(ph) == 0) {
					printf("{\"phases\": %d, \"mode\": %d, \"xfer\": %d, \"clk\": [", B, mode, xfer);
					for (int k = 1; k < 12; k++)
						printf("%s%lld", k > 1 ? ", " : "", (long long)(ph[2 * k] - ph[0]));
					printf("], \"real_10ns\": [");
					for (int k = 1; k < 12; k++)
						printf("%s%lld", k > 1 ? ", " : "", (long long)(ph[2 * k + 1] - ph[1]));
					printf("]}\n");
				}
				qsort(lat, iters, sizeof(double), cmp_d);
				const double med = lat[iters / 2], p99 = lat[(int)(iters * 0.99)];
				double wp;
				CK(espgpu_set_tuning(ctx, "overflow_mb", 0));
				const double dt = pipelined(B, iters, 0, &bad, &wp);
				CK(espgpu_set_tuning(ctx, "overflow_mb", 256));
				double wf;
				const double df = pipelined(B, iters, 1, &bad, &wf);
				CK(espgpu_set_tuning(ctx, "overflow_mb", 0));
				CK(espgpu_get_stats(ctx, &s1));
				printf("{\"burst\": %d, \"tuning\": \"%s\", \"mode\": \"%s\", \"xfer\": %d, \"record_bytes\": %d, "
				       "\"latency_us_median\": %.1f, \"latency_us_p99\": %.1f, \"latency_records_per_s\": %.0f, "
				       "\"pipelined_records_per_s\": %.0f, \"pipelined_GBps\": %.3f, "
				       "\"fstack_records_per_s\": %.0f, \"fstack_GBps\": %.3f, \"fstack_max_process_us\": %.1f, "
				       "\"batches\": %llu, \"overflow\": %llu, \"zerocopy\": %llu, "
				       "\"iters\": %d, \"auth_fail\": [%d, %d]}\n",
				       B, tun ? tun : "", mode ? "registered" : "gather", xfer, REC, med, p99, B / med * 1e6,
				       iters * (double)B / dt * 1e6, iters * (double)B * REC / dt / 1e3,
				       iters * (double)B / df * 1e6, iters * (double)B * REC / df / 1e3, wf,
				       (unsigned long long)(s1.batches - s0.batches),
				       (unsigned long long)(s1.overflow - s0.overflow),
				       (unsigned long long)(s1.zerocopy - s0.zerocopy), iters, bad_latency, bad - bad_latency);
				fflush(stdout);
				free(lat);
			}
		}
	}
	if (registered) CK(espgpu_unregister_host(ctx, bufs));
	espgpu_freesession(ctx, sid);
	espgpu_fini(ctx);
	return 0;
}
