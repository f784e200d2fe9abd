/*
 * kmock.h -- a user-space stand-in for the slice of the FreeBSD kernel crypto
 * KPI that integration/ff_gpucrypto.c uses, so that the kernel-domain driver
 * compiles, links and runs in this repository's tests (built with
 * -DFF_GPUCRYPTO_KMOCK).  It is OUR test double, not the reference's headers:
 * the declarations follow the shapes in freebsd/opencrypto/cryptodev.h
 * (struct cryptop :438-504, struct crypto_buffer :400-415,
 * struct crypto_session_params :357-384, CRYPTOCAP_* :641-656) and the
 * FreeBSD errno values in freebsd/sys/errno.h, and kmock.c restates the
 * framework behaviour the driver relies on:
 *   crypto_dispatch -> crypto_invoke -> CRYPTODEV_PROCESS, ERESTART puts the
 *     request on the queue and marks the driver blocked   crypto.c:1413-1460
 *   crypto_unblock clears the block, the queue is retried crypto.c:1191-1210
 *   crypto_done runs the callback (CBIFSYNC: inline)      crypto.c:1802-1830
 *   crypto_newsession picks the driver whose probe bids best (hardware -100
 *     over software -500; a positive errno declines)      crypto.c:622-659, 910
 * With kmock_soft_enable(1) a software driver stand-in (cryptosoft's part:
 * probe -500 for everything, process completes the request with etype 0 and
 * leaves the data as is) sits beside the driver under test, so the GPU-failure
 * path's session migration can be followed (ff_gpucrypto.c gpucrypto_migrate).
 * Inside F-Stack the driver is built against the real headers instead.
 */
#ifndef KMOCK_H
#define KMOCK_H

#include <stddef.h>
#include <stdint.h>
#include <string.h>

/* freebsd/sys/errno.h values (not the host's) */
#define ENOENT      2
#define EIO         5
#define ENXIO       6
#define ENOMEM      12
#define ENODEV      19
#define EINVAL      22
#define EAGAIN      35
#define EOPNOTSUPP  45
#define ENOBUFS     55
#define EBADMSG     89
#define ERESTART    (-1)

typedef struct kmock_device *device_t;

struct mbuf {
	struct mbuf *m_next;
	int          m_len;
	char        *m_data;
};
#define mtod(m, t) ((t)((m)->m_data))

enum crypto_buffer_type {
	CRYPTO_BUF_NONE = 0,
	CRYPTO_BUF_CONTIG,
	CRYPTO_BUF_UIO,
	CRYPTO_BUF_MBUF,
	CRYPTO_BUF_VMPAGE,
};

struct crypto_buffer {
	union {
		struct {
			char *cb_buf;
			int   cb_buf_len;
		};
		struct mbuf *cb_mbuf;
	};
	enum crypto_buffer_type cb_type;
};

struct crypto_session_params {
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

typedef struct crypto_session *crypto_session_t;

#define EALG_MAX_BLOCK_LEN 16
struct cryptop {
	crypto_session_t crp_session;
	int              crp_etype;
	int              crp_flags;
	int              crp_op;
	struct crypto_buffer crp_buf;
	struct crypto_buffer crp_obuf;
	void            *crp_aad;
	int              crp_aad_start;
	int              crp_aad_length;
	uint8_t          crp_esn[4];
	int              crp_iv_start;
	int              crp_payload_start;
	int              crp_payload_output_start;
	int              crp_payload_length;
	int              crp_digest_start;
	uint8_t          crp_iv[EALG_MAX_BLOCK_LEN];
	const void      *crp_cipher_key;
	const void      *crp_auth_key;
	void            *crp_opaque;
	int            (*crp_callback)(struct cryptop *);
	struct cryptop  *kmock_next;          /* framework queue link (crp_next) */
};

#define CRYPTO_F_DONE           0x0020
#define CRYPTO_F_CBIFSYNC       0x0040
#define CRYPTO_F_IV_SEPARATE    0x0200
#define CRYPTO_OP_DECRYPT       0x0
#define CRYPTO_OP_ENCRYPT       0x1
#define CRYPTO_OP_COMPUTE_DIGEST 0x0
#define CRYPTO_OP_VERIFY_DIGEST 0x2
#define CRYPTO_HAS_OUTPUT_BUFFER(crp) ((crp)->crp_obuf.cb_type != CRYPTO_BUF_NONE)

#define CRYPTOCAP_F_HARDWARE    0x01000000
#define CRYPTOCAP_F_SOFTWARE    0x02000000
#define CRYPTOCAP_F_SYNC        0x04000000
#define CRYPTO_SYMQ             0x1
#define CRYPTODEV_PROBE_HARDWARE (-100)
#define CRYPTODEV_PROBE_SOFTWARE (-500)

void   *crypto_get_driver_session(crypto_session_t cses);
const struct crypto_session_params *crypto_get_params(crypto_session_t cses);
uint32_t crypto_ses2hid(crypto_session_t cses);
int32_t crypto_get_driverid(device_t dev, size_t session_size, int flags);
int     crypto_unregister_all(uint32_t driverid);
int     crypto_unblock(uint32_t driverid, int what);
void    crypto_done(struct cryptop *crp);
int     crypto_newsession(crypto_session_t *cses, const struct crypto_session_params *csp, int crid);
void    crypto_freesession(crypto_session_t cses);

/* The driver's method table (what DEVMETHOD/kobj provide in the kernel). */
struct kmock_cryptodev {
	const char *name;
	int  (*attach)(device_t dev);
	int  (*detach)(device_t dev);
	int  (*probesession)(device_t dev, const struct crypto_session_params *csp);
	int  (*newsession)(device_t dev, crypto_session_t cses, const struct crypto_session_params *csp);
	void (*freesession)(device_t dev, crypto_session_t cses);
	int  (*process)(device_t dev, struct cryptop *crp, int hint);
};

/* ---- test-side framework (crypto.c's role) ---- */
struct kmock_stats {
	int32_t driverid;
	int     caps;                 /* flags passed to crypto_get_driverid      */
	size_t  session_size;
	int     blocked;              /* cc_qblocked                             */
	int     erestarts;            /* CRYPTODEV_PROCESS returned ERESTART      */
	int     queued;               /* requests waiting on the crypto queue     */
	int     done;                 /* crypto_done calls                        */
	int     unblocks;
	int     soft_sessions;        /* sessions on the software stand-in        */
	int     soft_done;            /* requests it completed                    */
	int     sessions;             /* sessions alive (either driver)           */
};
int  kmock_attach(const struct kmock_cryptodev *drv);
void kmock_detach(void);
/* crypto_newsession: probesession must report hardware (-100), then newsession */
int  kmock_newsession(crypto_session_t *out, const struct crypto_session_params *csp);
void kmock_freesession(crypto_session_t cses);
/* crypto_dispatch for a request without CRYPTO_F_BATCH */
int  kmock_dispatch(struct cryptop *crp);
/* crypto_proc's pass over the queue after an unblock: re-dispatch in order */
int  kmock_run_queue(void);
const struct kmock_stats *kmock_stats(void);
/* the software driver stand-in beside the driver under test (off: only it) */
void kmock_soft_enable(int on);
/* crypto_ses2hid of a session on the software stand-in */
#define KMOCK_SOFT_ID 8

#endif /* KMOCK_H */
