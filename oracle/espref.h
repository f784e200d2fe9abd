/*
 * espref.h — CPU restatement of the F-Stack/FreeBSD ESP bulk-crypto path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle (and the "port"
 * CPU baseline) for the MI355X engine in f-stack_amd/.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product path never links or calls anything in oracle/.
 *
 * What it restates (reference = /root/reference, F-Stack 1.25):
 *   freebsd/crypto/rijndael/rijndael-alg-fst.c   AES T-table cipher + key schedules
 *   freebsd/opencrypto/gfmult.c, gmac.c          GHASH (4-bit Shoup tables) / AES-GMAC
 *   freebsd/opencrypto/xform_aes_icm.c           GCM counter mode (counter starts at 2)
 *   freebsd/crypto/sha1.c, opencrypto/crypto.c   SHA-1 and HMAC ipad/opad precompute
 *   freebsd/opencrypto/cryptosoft.c              swcr_gcm / swcr_eta / swcr_encdec /
 *                                                swcr_authcompute request processing
 *   freebsd/netipsec/xform_esp.c                 esp_input / esp_output request layout
 *   freebsd/netipsec/ipsec.c                     replay window: ipsec_chkreplay /
 *                                                ipsec_updatereplay
 *
 * Pinning: primitives are checked against the reference's own
 * rijndael-alg-fst.c / gfmult.c compiled from /root/reference (oracle/_ref),
 * and whole-path results against DPDK's ESP / AEAD / CBC+HMAC-SHA1 known-answer
 * vectors held in the reference tree (tests/golden/).
 */
#ifndef ESPREF_H
#define ESPREF_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Session modes (values of crypto_session_params.csp_mode, cryptodev.h:360-365). */
#define OREF_CSP_MODE_CIPHER 2          /* cipher only: ESP without auth (esp_init :230-231) */
#define OREF_CSP_MODE_AEAD 4
#define OREF_CSP_MODE_ETA  5
/* csp_flags (cryptodev.h:369-371) */
#define OREF_CSP_F_SEPARATE_AAD 0x0002
#define OREF_CSP_F_ESN          0x0004
/* algorithms (cryptodev.h:150-169) */
#define OREF_CRYPTO_SHA1_HMAC      7
#define OREF_CRYPTO_AES_CBC        11
#define OREF_CRYPTO_NULL_CBC       16     /* enc_xform_null: blocksize 4, no IV (xform_null.c:65-76) */
#define OREF_CRYPTO_SHA2_256_HMAC  18
#define OREF_CRYPTO_SHA2_384_HMAC  19     /* cryptodev.h:163 */
#define OREF_CRYPTO_SHA2_512_HMAC  20     /* cryptodev.h:164 */
#define OREF_CRYPTO_AES_ICM        23          /* AES-CTR */
#define OREF_CRYPTO_AES_NIST_GCM_16 25

typedef struct oref_sa oref_sa;

/* --- primitives (for pinning against oracle/_ref and KATs) --- */
int  oref_aes_setkey_enc(uint32_t rk[60], const uint8_t *key, int keybits);   /* returns Nr */
int  oref_aes_setkey_dec(uint32_t rk[60], const uint8_t *key, int keybits);
void oref_aes_encrypt(const uint32_t *rk, int nr, const uint8_t in[16], uint8_t out[16]);
void oref_aes_decrypt(const uint32_t *rk, int nr, const uint8_t in[16], uint8_t out[16]);
/* out = x * h in GF(2^128), GCM bit order (gfmult.c representation) */
void oref_gf128_mul(const uint8_t h[16], const uint8_t x[16], uint8_t out[16]);
void oref_sha1(const uint8_t *msg, size_t len, uint8_t out[20]);
void oref_hmac_sha1(const uint8_t *key, int klen, const uint8_t *msg, size_t len, uint8_t out[20]);
void oref_sha256(const uint8_t *msg, size_t len, uint8_t out[32]);
/* hash / HMAC with alg = OREF_CRYPTO_SHA1_HMAC (20-byte out), _SHA2_256_HMAC
 * (32), _SHA2_384_HMAC (48) or _SHA2_512_HMAC (64) */
void oref_hash(int alg, const uint8_t *msg, size_t len, uint8_t *out);
void oref_hmac(int alg, const uint8_t *key, int klen, const uint8_t *msg, size_t len, uint8_t *out);
/* AES-ICM (counter mode, full 128-bit big-endian increment) from ctr[16] */
void oref_aes_ctr(const uint8_t *key, int klen, const uint8_t ctr[16], uint8_t *data, int len);

/* Generic AES-GCM AEAD (12-byte IV) as swcr_gcm computes it; in place.
 * encrypt: writes tag[16].  decrypt: verifies tag[0..mlen) and returns
 * 0 or EBADMSG (buffer untouched on EBADMSG). */
int oref_gcm(const uint8_t *key, int klen, const uint8_t iv[12],
             const uint8_t *aad, int aadlen, uint8_t *data, int len,
             uint8_t *tag, int mlen, int encrypt);

/* Generic AES-CBC + HMAC-SHA1 encrypt-then-MAC (swcr_eta) over
 * [aad | data]; digest[20] written (encrypt) or its first mlen bytes checked. */
int oref_eta(const uint8_t *ckey, int cklen, const uint8_t *akey, int aklen,
             const uint8_t iv[16], const uint8_t *aad, int aadlen, uint8_t *data, int len,
             uint8_t *digest, int mlen, int encrypt);

/* --- sessions (swcr_newsession/swcr_setup_gcm/swcr_setup_cipher/auth) ---
 * GCM: ckey is the SA key WITHOUT the 4-byte salt (esp_init strips it,
 * xform_esp.c:169); salt is passed separately.
 * ETA: AES-CBC cipher key + HMAC-SHA1 key, mlen 12 (AH_HMAC_HASHLEN). */
oref_sa *oref_sa_new(int mode, int flags, const uint8_t *ckey, int cklen,
                     const uint8_t salt[4], const uint8_t *akey, int aklen, int mlen);
/* ETA with a chosen cipher (OREF_CRYPTO_AES_CBC, _AES_ICM: RFC 3686 ESP
 * AES-CTR, salt = the 4-byte nonce esp_init strips from the key, or
 * _NULL_CBC: no key, swcr_newsession degrades the session to the digest,
 * cryptosoft.c:1394-1398) and HMAC (OREF_CRYPTO_SHA1_HMAC or
 * _SHA2_256/384/512_HMAC; mlen 0 = the full hash).  CIPHER: the same ciphers
 * with no auth (aalg 0; NULL_CBC is swcr_null, cryptosoft.c:1339-1342). */
oref_sa *oref_sa_new2(int mode, int flags, int calg, const uint8_t *ckey, int cklen,
                      const uint8_t salt[4], int aalg, const uint8_t *akey, int aklen, int mlen);
void oref_sa_free(oref_sa *sa);

/* ESP record = [SPI 4][SN 4][IV ivlen][payload][ICV alen], i.e. the buffer
 * esp_input sees at `skip` (xform_esp.c:260-463).  In place.
 * Returns 0, EBADMSG (ICV mismatch, buffer untouched) or EINVAL (length). */
int oref_esp_decrypt(const oref_sa *sa, uint8_t *esp, int len, uint32_t esn_hi);
/* esp_output direction over an already padded record: encrypts payload and
 * writes the ICV (xform_esp.c:673-961, cryptosoft.c:558-568,636). */
int oref_esp_encrypt(const oref_sa *sa, uint8_t *esp, int len, uint32_t esn_hi);

/* Batch decrypt with `nthreads` workers, each taking a contiguous slice
 * (one private session per worker, like one F-Stack stack per lcore).
 * rec i is at arena + off4[i]*4, length len[i], SA sas[sa_idx[i]].
 * Returns wall seconds of the decrypt loop only. */
double oref_batch_decrypt(oref_sa *const *sas, uint8_t *arena, const uint32_t *off4,
                          const uint16_t *len, const uint16_t *sa_idx,
                          const uint32_t *esn_hi, uint8_t *status, long n, int nthreads);
double oref_batch_encrypt(oref_sa *const *sas, uint8_t *arena, const uint32_t *off4,
                          const uint16_t *len, const uint16_t *sa_idx,
                          const uint32_t *esn_hi, long n, int nthreads);

/* Replay window (struct secreplay, netipsec/keydb.h:206-213), with the SA
 * flags the checks read: bit 0 SADB_X_SAFLAGS_ESN, bit 1 SADB_X_EXT_CYCSEQ. */
typedef struct {
	uint64_t count;
	uint64_t last;
	uint32_t wsize;            /* bytes: window = wsize * 8 packets */
	uint32_t bitmap_size;      /* u32 words, a power of two */
	uint32_t *bitmap;
	int overflow;
	int flags;
} oref_replay;
#define OREF_REPLAY_ESN    1
#define OREF_REPLAY_CYCSEQ 2
/* ipsec_chkreplay (ipsec.c:1248-1331): 1 permitted (seqhigh set), 0 not. */
int oref_chkreplay(uint32_t seq, uint32_t *seqhigh, oref_replay *r);
/* ipsec_updatereplay (ipsec.c:1338-1436): 0 OK (window updated), 1 NG. */
int oref_updatereplay(uint32_t seq, oref_replay *r);

#ifdef __cplusplus
}
#endif
#endif
