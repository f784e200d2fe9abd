/*
 * espgpu.h — C ABI of the MI355X-native ESP bulk-crypto engine (libespgpu.so).
 *
 * Drop-in boundary: this library plays the part of an opencrypto *driver*
 * (freebsd/opencrypto/cryptodev_if.m) beneath the unchanged opencrypto
 * framework, i.e. it replaces the software driver "cryptosoft"
 * (freebsd/opencrypto/cryptosoft.c) for the ESP ciphers F-Stack's IPsec uses:
 *   AES-GCM-16 (CSP_MODE_AEAD)                  -> swcr_gcm      cryptosoft.c:465-645
 *   AES-CBC, AES-CTR (RFC 3686) or NULL + HMAC-SHA1-96
 *     or HMAC-SHA2-256-128 / -384-192 / -512-256
 *     (CSP_MODE_ETA)                            -> swcr_eta      cryptosoft.c:874-888
 *                                                  (NULL: swcr_authcompute, :1394-1398)
 *   AES-CBC or AES-CTR with no auth, or NULL
 *     (CSP_MODE_CIPHER)                         -> swcr_encdec   cryptosoft.c:101-284
 *                                                  (NULL: swcr_null, :91-95)
 * Every entry point is plain C: integers, pointers, sizes.  No exceptions,
 * no C++ or torch types cross it.  Errors are errno values, as in opencrypto.
 * One espgpu_ctx per lcore thread (thread-compatible, not thread-safe), the
 * way F-Stack runs one FreeBSD stack per lcore (lib/ff_dpdk_if.c:2235).
 *
 * Two ways in:
 *  (1) the opencrypto driver path (host buffers): probesession / newsession /
 *      freesession / process / flush / poll  — what a kernel-domain driver shim
 *      in F-Stack binds;
 *  (2) the device-resident batch path: records already in HBM, a 16-byte
 *      descriptor per record — what bench.py times and what a GPU-direct RX
 *      path would call.
 */
#ifndef ESPGPU_H
#define ESPGPU_H

#if defined(_KERNEL) && defined(__FreeBSD__)
/* F-Stack's kernel domain (lib/Makefile: -nostdinc, FreeBSD headers only):
 * the driver ff_gpucrypto.c includes this header for the request mirrors */
#include <sys/types.h>
#else
#include <stddef.h>
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define ESPGPU_ABI_VERSION 6

/* ---- constants, numerically identical to freebsd/opencrypto/cryptodev.h ---- */
#define ESPGPU_CSP_MODE_CIPHER      2        /* cryptodev.h:362: ESP without auth */
#define ESPGPU_CSP_MODE_AEAD        4        /* cryptodev.h:364 */
#define ESPGPU_CSP_MODE_ETA         5        /* cryptodev.h:365 */
#define ESPGPU_CSP_F_SEPARATE_AAD   0x0002   /* cryptodev.h:370 */
#define ESPGPU_CSP_F_ESN            0x0004   /* cryptodev.h:371 */
#define ESPGPU_CRYPTO_SHA1_HMAC     7        /* cryptodev.h:150 */
#define ESPGPU_CRYPTO_AES_CBC       11       /* cryptodev.h:155 */
#define ESPGPU_CRYPTO_NULL_CBC      16       /* cryptodev.h:160: ESP-NULL (enc_xform_null) */
#define ESPGPU_CRYPTO_SHA2_256_HMAC 18     /* cryptodev.h:162 */
#define ESPGPU_CRYPTO_SHA2_384_HMAC 19     /* cryptodev.h:163 */
#define ESPGPU_CRYPTO_SHA2_512_HMAC 20     /* cryptodev.h:164 */
#define ESPGPU_CRYPTO_AES_ICM       23       /* AES-CTR, cryptodev.h:167 */
#define ESPGPU_CRYPTO_AES_NIST_GCM_16 25     /* cryptodev.h:169 */
#define ESPGPU_CRYPTO_OP_DECRYPT    0x0      /* cryptodev.h:598 */
#define ESPGPU_CRYPTO_OP_ENCRYPT    0x1
#define ESPGPU_CRYPTO_OP_VERIFY_DIGEST 0x2
#define ESPGPU_CRYPTO_F_IV_SEPARATE 0x0200   /* cryptodev.h:470 */
#define ESPGPU_CRYPTO_HINT_MORE     0x1      /* cryptodev.h:612 */
#define ESPGPU_PROBE_HARDWARE       (-100)   /* CRYPTODEV_PROBE_HARDWARE, cryptodev.h:345 */

/*
 * Error codes returned by every entry point and written as the per-record
 * status byte.  They are this ABI's own numbers (they coincide with Linux
 * errno, the host the library runs on), NOT FreeBSD kernel errno: a
 * kernel-domain shim translates them before they reach opencrypto, e.g.
 * ESPGPU_EBADMSG -> EBADMSG (89), ESPGPU_ERESTART -> ERESTART (-1),
 * ESPGPU_EAGAIN -> EAGAIN (35); see integration/ff_gpucrypto.c
 * gpucrypto_errno().
 */
#define ESPGPU_OK       0
#define ESPGPU_ENOENT   2     /* unknown tuning key                            */
#define ESPGPU_EIO      5     /* HIP runtime failure (espgpu_last_error says)  */
#define ESPGPU_ENXIO    6
#define ESPGPU_EAGAIN   11
#define ESPGPU_ENOMEM   12    /* SA table full / allocation failure            */
#define ESPGPU_ENODEV   19    /* no HIP device                                 */
#define ESPGPU_EINVAL   22    /* malformed request or unsupported parameters   */
#define ESPGPU_EBADMSG  74    /* ICV mismatch (status byte / crp_etype)        */
#define ESPGPU_ERESTART 85    /* process(): staging full, requeue (cc_qblocked) */
#define ESPGPU_ENOTSUP  95
#define ESPGPU_ENOBUFS  105   /* F-Stack mode: host overflow full, request dropped */

/* Mirror of struct crypto_session_params (cryptodev.h:357-384). */
struct espgpu_session_params {
	int         csp_mode;
	int         csp_flags;
	int         csp_ivlen;
	int         csp_cipher_alg;
	int         csp_cipher_klen;
	const void *csp_cipher_key;
	int         csp_auth_alg;
	int         csp_auth_klen;
	const void *csp_auth_key;
	int         csp_auth_mlen;
};

/* One buffer segment (an mbuf in the chain, or the whole contiguous buffer). */
struct espgpu_seg {
	void    *base;
	uint32_t len;
};

/*
 * Mirror of the struct cryptop fields a driver consumes (cryptodev.h:427-504).
 * The buffer is crp_buf (CRYPTO_BUF_CONTIG = 1 segment, CRYPTO_BUF_MBUF = the
 * chain as segments), processed in place.  `opaque` comes back in the
 * completion (a kernel-domain shim passes the cryptop pointer itself).
 */
struct espgpu_req {
	int32_t                  session;
	int                      crp_op;
	int                      crp_flags;
	const struct espgpu_seg *segs;
	int                      nsegs;
	const void              *crp_aad;          /* separate AAD or NULL */
	int                      crp_aad_start;
	int                      crp_aad_length;
	uint8_t                  crp_esn[4];
	int                      crp_iv_start;
	int                      crp_payload_start;
	int                      crp_payload_length;
	int                      crp_digest_start;
	uint8_t                  crp_iv[16];
	void                    *opaque;
};

struct espgpu_completion {
	void *opaque;
	int   etype;            /* crp_etype: 0, EBADMSG, EINVAL, EIO (GPU failure) */
};

/* Device-resident descriptor: one per ESP record (16 bytes). */
struct espgpu_desc {
	uint32_t off4;          /* record start in the arena, in 4-byte units       */
	uint16_t len;           /* ESP record length: SPI|SN|IV|payload|ICV          */
	uint16_t sa;            /* session slot (espgpu_newsession's id)             */
	uint32_t esn_hi;        /* high 32 bits of the ESN (SAs with CSP_F_ESN/SEP)  */
	uint32_t salt;          /* GCM salt / AES-CTR nonce = crp_iv[0..3], in memory order */
};

struct espgpu_config {
	int      device;          /* HIP device ordinal                               */
	uint32_t max_sessions;    /* SA table capacity (default 1024)                 */
	uint32_t batch_records;   /* records per host batch (default 65536)           */
	uint32_t batch_bytes;     /* staging bytes per host batch (default 64 MiB)    */
	uint32_t nbatches;        /* staging slots in flight (default 2)              */
	uint32_t grid;            /* workgroups for the crypto kernels (0 = auto)     */
};

struct espgpu_stats {
	uint64_t records, bytes, auth_fail, einval;
	uint64_t batches, kernel_ns;   /* kernel_ns: device time measured with events */
	uint64_t erestart;
	uint64_t overflow;             /* requests staged through the host overflow      */
	uint64_t zerocopy;             /* records moved from / to registered memory      */
	uint64_t door;                 /* batches served by the doorbell kernel (ABI 3)  */
	uint64_t ovf_reserved;         /* host bytes the overflow's fixed rings hold (ABI 4):
	                                  set once by set_tuning "overflow_mb", never grown */
	uint64_t ovf_peak;             /* most record bytes the overflow held at once    */
	uint64_t ovf_process_ns_max;   /* longest overflow placement inside process()    */
	uint64_t gpu_fail;             /* GPU failures detected (ABI 5): 0, or 1 once failed */
	uint64_t fail_eio;             /* requests completed or refused with EIO because of it */
};

typedef struct espgpu_ctx espgpu_ctx;

/* ---- lifecycle (a kernel-domain shim calls crypto_get_driverid(...,
 *      CRYPTOCAP_F_HARDWARE|CRYPTOCAP_F_SYNC), crypto.c:989, around these) ---- */
int  espgpu_abi_version(void);
/* Visible HIP devices (>= 0), or ESPGPU_ENODEV.  One F-Stack process (lcore)
 * opens one context; process k of a node takes device k mod count
 * (ff_gpucrypto_host_init_proc). */
int  espgpu_device_count(void);
int  espgpu_init(const struct espgpu_config *cfg, espgpu_ctx **out);
void espgpu_fini(espgpu_ctx *ctx);
const char *espgpu_last_error(espgpu_ctx *ctx);
/* GPU health: ESPGPU_OK, or ESPGPU_EIO once the context has seen a GPU
 * failure -- a launch or copy that could not be queued, a completion query
 * that returned an error, or a batch outstanding longer than set_tuning
 * "deadline_ms" (default 2000).  From then on the context launches nothing:
 * every request it held completes exactly once through espgpu_poll with
 * etype ESPGPU_EIO (unless its batch is seen to complete after all),
 * espgpu_process / flush / drain / newsession and the batch entry points
 * answer ESPGPU_EIO, and espgpu_last_error names the cause.  The F-Stack
 * shim's probe declines on a failed context, so new sessions go to
 * cryptosoft. */
int  espgpu_health(espgpu_ctx *ctx);

/* ---- opencrypto driver methods (cryptodev_if.m) ---- */
/* CRYPTODEV_PROBESESSION (cryptodev_if.m:72-75): ESPGPU_PROBE_HARDWARE or EINVAL.
 * Host-only; no device needed. */
int  espgpu_probesession(const struct espgpu_session_params *csp);
/* CRYPTODEV_NEWSESSION (cryptodev_if.m:93-97): expands keys (AES schedule,
 * GHASH power tables, HMAC ipad/opad states) into the device SA table. */
int  espgpu_newsession(espgpu_ctx *ctx, const struct espgpu_session_params *csp,
                       int32_t *session_out);
/* CRYPTODEV_FREESESSION (cryptodev_if.m:113-116) */
void espgpu_freesession(espgpu_ctx *ctx, int32_t session);
/* Free SA-table slots (ABI 6; >= 0, or ESPGPU_EINVAL without a context):
 * at 0 espgpu_newsession answers ESPGPU_ENOMEM.  The F-Stack shim's probe
 * declines then, so crypto_newsession selects cryptosoft instead of failing
 * the SA in CRYPTODEV_NEWSESSION (crypto.c:954-958). */
int  espgpu_session_room(espgpu_ctx *ctx);
/* CRYPTODEV_PROCESS (cryptodev_if.m:143-147): never blocks.  On a failed
 * context (espgpu_health) it answers ESPGPU_EIO at once: never ERESTART or
 * EAGAIN, which would hand the request back to this dead engine.  Stages the
 * request; returns 0, or ERESTART when every staging slot is in flight (the
 * framework then sets cc_qblocked and requeues, crypto.c:1451-1459).  With
 * set_tuning "overflow_mb" > 0 such a request is kept in a host overflow
 * instead (ERESTART only once that many MiB are held), which the next
 * espgpu_flush moves into the slots as they free: F-Stack runs no
 * crypto_proc thread to requeue.  A record lying
 * in one segment of memory registered with espgpu_register_host is not
 * copied by the CPU: the GPU reads it and writes the results back in place.
 * Malformed requests complete with crp_etype = EINVAL via poll(), as
 * crypto_done would.  `hint` (CRYPTO_HINT_MORE) is accepted and ignored:
 * staged requests launch at espgpu_flush (once per RX burst) or when a
 * staging slot fills. */
int  espgpu_process(espgpu_ctx *ctx, const struct espgpu_req *req, int hint);
/* Launch everything staged so far, then move the overflow into the slots
 * that are free: a small batch runs copy, kernels, copy in order on its
 * slot's stream; a large one H2D, kernels and D2H on three ctx streams
 * chained by events, so consecutive batches overlap copies with kernels.
 * Never waits.  F-Stack's main_loop calls this once per RX burst
 * (lib/ff_dpdk_if.c:2363). */
int  espgpu_flush(espgpu_ctx *ctx);
/* Complete finished requests: copies results back into the caller's segments
 * (only for etype 0: EBADMSG leaves the buffer unchanged) and returns up to
 * `max` completions; the shim calls crypto_done() for each. */
int  espgpu_poll(espgpu_ctx *ctx, struct espgpu_completion *out, int max);
/* Block until everything staged, flushed or in the overflow has completed
 * (teardown / tests); the completions wait for espgpu_poll. */
int  espgpu_drain(espgpu_ctx *ctx);
/* Register host memory the requests' buffers live in (DPDK mbuf pools:
 * F-Stack's mbuf data is the mbuf's own hugepage buffer, lib/ff_veth.c:
 * 367-389; ff_dpdk_register_gpu_mem walks the pools with
 * rte_mempool_mem_iter).  hipHostRegister maps it
 * for the device once; process() then stages a record that lies in it by
 * reference, and the xfer kernel reads it into the device batch and writes
 * the results back (payload; ICV when encrypting; nothing for a record that
 * fails) with no CPU copy.  Memory already pinned (hipHostMalloc) is mapped
 * as is.  Regions must not overlap: EINVAL.  Unregister drains first. */
int  espgpu_register_host(espgpu_ctx *ctx, void *base, uint64_t len);
int  espgpu_unregister_host(espgpu_ctx *ctx, void *base);
int  espgpu_get_stats(espgpu_ctx *ctx, struct espgpu_stats *st);

/* ---- device-resident batch path ----
 * d_arena: device buffer holding the records (padded by >= 16 bytes at its
 * end); d_desc[n]; d_status[n] receives one errno byte per record.
 * decrypt: plaintext goes to d_out at the same offsets (d_out may equal
 * d_arena: verify-first in place; an EBADMSG record ends byte-identical to
 * its ciphertext: AES-GCM in one pass that XORs the keystream back over a
 * failed record, CBC/CTR + HMAC verifying before it decrypts).
 * encrypt: payload encrypted in place, ICV written.
 * `flags`: ESPGPU_BATCH_GROUPED if d_desc is already grouped by session with
 * at most one session per aligned run of 256 records (skips the device
 * planner; records of another session than their run's come back EINVAL).
 * `stream` is a hipStream_t (NULL = default stream).  Asynchronous.
 * Launches on one ctx are stream-ordered by the library: the work-queue
 * counters and planner workspace belong to the ctx, so a launch on a stream
 * other than the ctx's previous one first waits on an event recorded after
 * that launch (never two kernels of one ctx at once).  Use one ctx per
 * stream for concurrent batches. */
#define ESPGPU_BATCH_GROUPED 0x1
int  espgpu_decrypt_batch(espgpu_ctx *ctx, uint8_t *d_arena, const struct espgpu_desc *d_desc,
                          uint32_t n, uint8_t *d_status, uint8_t *d_out, uint32_t flags,
                          void *stream);
int  espgpu_encrypt_batch(espgpu_ctx *ctx, uint8_t *d_arena, const struct espgpu_desc *d_desc,
                          uint32_t n, uint8_t *d_status, uint32_t flags, void *stream);

/* espgpu_decrypt_batch with a packed output: the plaintext (ESP payload) of
 * record i lands at d_out + i * out_stride instead of the record's own offset,
 * every 128-byte line of it written whole (out_stride a nonzero multiple of
 * 128; d_out 128-byte aligned, n * out_stride bytes, not overlapping d_arena:
 * EINVAL for an unaligned d_out or d_out == d_arena; a partial overlap cannot
 * be detected and races with the ciphertext reads).  A record whose payload
 * is longer than out_stride is EINVAL.  Single pass, like the out-of-place
 * espgpu_decrypt_batch: a record whose status is nonzero (EBADMSG) still has
 * its unverified plaintext in its slot, which the consumer must ignore
 * (swcr_gcm releases no plaintext for it, cryptosoft.c:600-603).  For a
 * device-side consumer of the plaintext; the line-aligned stores make the
 * kernel ≈ 4-6 % faster than the record layout's.  GCM
 * contexts only: ENOTSUP when the context has ETA sessions.  No esp_input_cb
 * trailer words. */
int  espgpu_decrypt_batch_packed(espgpu_ctx *ctx, uint8_t *d_arena, const struct espgpu_desc *d_desc,
                                 uint32_t n, uint8_t *d_status, uint8_t *d_out, uint32_t out_stride,
                                 uint32_t flags, void *stream);

/* Decrypt + the ESP trailer checks of esp_input_cb (xform_esp.c:597-630)
 * fused into the kernels: d_trailer[i] (one 32-bit word per record) gets
 *   bits 0-7  next header, bits 8-15 pad length (the last 3 plaintext bytes),
 *   ESPGPU_TR_BADLEN  pad length + 2 > payload length       (esps_badilen),
 *   ESPGPU_TR_BADPAD  last pad byte != pad length != 0       (esps_badenc; the
 *                     caller ignores it for SADB_X_EXT_PRAND SAs),
 *   ESPGPU_TR_NONE    next header == IPPROTO_NONE (59)       (silent drop),
 *   ESPGPU_TR_VALID   set for every record whose status is 0;
 * and 0 for records that failed (status != 0).  Otherwise as
 * espgpu_decrypt_batch. */
#define ESPGPU_TR_BADLEN 0x00010000u
#define ESPGPU_TR_BADPAD 0x00020000u
#define ESPGPU_TR_NONE   0x00040000u
#define ESPGPU_TR_VALID  0x80000000u
int  espgpu_decrypt_batch_trailer(espgpu_ctx *ctx, uint8_t *d_arena,
                                  const struct espgpu_desc *d_desc, uint32_t n,
                                  uint8_t *d_status, uint8_t *d_out, uint32_t *d_trailer,
                                  uint32_t flags, void *stream);

/* Host-to-host pipelined decrypt of a large host-resident batch (the shape of
 * an offload from DPDK hugepage mbufs): records in h_arena (pinned: hipHostMalloc
 * or hipHostRegister), descriptors in ascending arena order; `chunk` records per
 * step (0 = 65536).  Step k's H2D, step k-1's kernels and step k-2's D2H run
 * concurrently on three HIP streams.  Plaintext lands in h_out at the same
 * offsets; returns when everything is back. */
int  espgpu_decrypt_host(espgpu_ctx *ctx, const uint8_t *h_arena, uint64_t arena_bytes,
                         const struct espgpu_desc *h_desc, uint32_t n, uint8_t *h_status,
                         uint8_t *h_out, uint32_t chunk, uint32_t flags);

/* ---- replay window (esp_input's pre-crypto check and esp_input_cb's
 *      update, freebsd/netipsec/xform_esp.c:329-340, :565-580) ----
 * One SA's window as ipsec_chkreplay reads it (struct secreplay,
 * netipsec/keydb.h:206-213): `last` = ESN high << 32 | low of the window
 * top, `wsize` in bytes (window = wsize * 8 packets, 0 = no replay check),
 * `bitmap_size` u32 words (a power of two, key.c:3346-3351) starting at word
 * `bitmap_off` of a shared bitmap array. */
#define ESPGPU_REPLAY_ESN    0x1     /* SADB_X_SAFLAGS_ESN  */
#define ESPGPU_REPLAY_CYCSEQ 0x2     /* SADB_X_EXT_CYCSEQ   */
#define ESPGPU_EACCES        13      /* replayed (esp_input's EACCES, esps_replay) */
struct espgpu_replay {
	uint64_t last;
	uint32_t wsize;
	uint32_t bitmap_size;
	uint32_t bitmap_off;
	uint32_t flags;
};

/* 1 if r's window parameters are usable: wsize 0 (no check), or bitmap_size
 * a power of two with bitmap_size * 32 >= wsize * 8 bits; else 0.  Both the
 * batch check and espgpu_replay_update index the bitmap with
 * bitmap_size - 1 as a mask: the caller of espgpu_replay_check_batch must
 * pass only windows this accepts (espgpu_replay_update returns EINVAL). */
int  espgpu_replay_params_ok(const struct espgpu_replay *r);
/* Pre-filter a device-resident batch against the windows as they stand
 * (ipsec_chkreplay, ipsec.c:1248-1331, for every record in parallel; the
 * record's SA indexes d_replay[nreplay]): d_rstatus[i] = 0 or ESPGPU_EACCES.
 * A replayed record's descriptor gets len = 0, so the decrypt kernels drop
 * it (status EINVAL) without crypto work; an accepted record of an ESN SA
 * gets esn_hi = the window's high word, as esp_input fills crp_esn.  Run it
 * before espgpu_decrypt_batch, then espgpu_replay_merge.  Asynchronous. */
int  espgpu_replay_check_batch(espgpu_ctx *ctx, const uint8_t *d_arena, struct espgpu_desc *d_desc,
                               uint32_t n, const struct espgpu_replay *d_replay, uint32_t nreplay,
                               const uint32_t *d_bitmap, uint8_t *d_rstatus, void *stream);
/* d_status[i] = d_rstatus[i] where that is nonzero. */
int  espgpu_replay_merge(espgpu_ctx *ctx, uint8_t *d_status, const uint8_t *d_rstatus, uint32_t n,
                         void *stream);
/* Host: ipsec_updatereplay (ipsec.c:1338-1436) for one authenticated record,
 * in arrival order per SA: 0 (window advanced / bit set) or ESPGPU_EACCES. */
int  espgpu_replay_update(struct espgpu_replay *r, uint32_t *bitmap, uint32_t seq);

/* Device time of the last timed batch's crypto kernels (ms, from HIP events
 * on the batch stream).  Process-path batches of <= 128 KiB (a burst on its
 * slot's own stream) are not timed: the two event markers cost a 32-record
 * burst 8 us of its 65. */
float espgpu_last_kernel_ms(espgpu_ctx *ctx);

/* Tuning knobs (engine-internal, for A/B measurement):
 *   "grid"      workgroups per launch (0 = 256, one per CU);
 *   "gcm_lanes" GCM lanes per record: 0 (default) 8 below 32768 records,
 *               else 4; 4 or 8 forces one kernel; others EINVAL;
 *   "overflow_mb" host overflow for process() while every staging slot is
 *               in flight, in MiB (0, the default: ERESTART; 0..4095; only
 *               requests not yet moved into a slot count against it);
 *   "xfer"      small batches' staging region moved by the xfer kernel (1,
 *               default) or by hipMemcpyAsync (0);
 *   "gcm_burst" GCM batches of up to this many records (default 4096) that
 *               run the small-batch design, out of place or encrypt, use the
 *               burst kernel (a 32-lane CTR pass and an 8-lane GHASH in one
 *               launch, for latency); 0 = the fused small-batch kernel;
 *   "door"      doorbell path (0, the default: off): N > 0 keeps a
 *               persistent kernel of N workgroups (one per CU) resident that
 *               serves the process path's single-session GCM batches of up
 *               to gcm_burst records -- flush() publishes a 16-byte job in
 *               pinned host memory instead of launching, the kernel stages
 *               the records in and the results out through the mapping, and
 *               poll() reads its done word -- so a burst pays no launch or
 *               completion signal; other kernels of the ctx then use the
 *               remaining CUs; 1..256, others EINVAL; changing it drains;
 *   "door_idle_us" the doorbell kernel exits after this long without a
 *               job (default 20000; 100..10^7): flush / poll relaunch it;
 *   "stage_fused" a process-path burst of one GCM session stages its own
 *               records inside the crypto kernel (1, default: one launch per
 *               burst) instead of xfer kernels around it (0);
 *   "deadline_ms" a batch outstanding this long (launch to completion) is a
 *               GPU failure (espgpu_health); 1..600000, default 2000;
 *   "fault"     fault injection for the GPU-failure path's tests: a mask of
 *               ESPGPU_FAULT_LAUNCH (the next launch fails), _QUERY (the next
 *               completion query of an in-flight batch returns an error) and
 *               _STUCK (the next batch launched is never seen to complete, so
 *               it meets the deadline); each bit is consumed once;
 *   "gcm_opts" / "eta_opts" measurement knobs that skip work on purpose
 *               (results wrong): only in libespgpu_knobs.so, ENOTSUP in the
 *               product library unless 0.
 * (The keys of designs measured slower and removed -- "gcm_split", "gcm_bs",
 * "eta_fused", "eta_ws", "eta_lag" -- are unknown: ENOENT.)
 * Returns 0, EINVAL, ENOTSUP or ENOENT (unknown key). */
#define ESPGPU_FAULT_LAUNCH 0x1
#define ESPGPU_FAULT_QUERY  0x2
#define ESPGPU_FAULT_STUCK  0x4
int  espgpu_set_tuning(espgpu_ctx *ctx, const char *key, int value);

#ifdef __cplusplus
}
#endif
#endif /* ESPGPU_H */
