/* OpenSSL EVP comparison point for bench.py ("optionally an
 * OpenSSL EVP line, labelled not the reference path").
 *
 * Decrypts ESP records laid out as in the GPU batch ABI (arena + off4/len/sa
 * per record) on the host, in place or out of place, with the same verify-first semantics as
 * cryptosoft (swcr_gcm cryptosoft.c:465-645, swcr_eta :874-888): a record
 * whose ICV does not match is EBADMSG (74) and its payload is not used.
 * This is NOT the reference's algorithm: OpenSSL runs AES-NI/VAES and
 * PCLMULQDQ code paths the F-Stack kernel crypto does not have.  It is timed
 * only to show what a modern CPU library does on the same records.
 *
 *   alg 0: ESP AES-GCM-16 (RFC 4106): SPI|SN|IV8|CT|ICV(mlen), AAD = SPI|SN,
 *          nonce = salt|IV8 (xform_esp.c:430-458)
 *   alg 1: ESP AES-CBC + HMAC-SHA1 (truncated to mlen): SPI|SN|IV16|CT|ICV,
 *          HMAC over SPI|SN|IV|CT (swcr_authcompute, cryptosoft.c:317-382)
 *
 * Build: gcc -O2 -fPIC -shared ossl_esp.c -o libossl_esp.so -lcrypto -pthread
 */
#define OPENSSL_SUPPRESS_DEPRECATED 1
#include <openssl/evp.h>
#include <openssl/hmac.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

enum { ST_OK = 0, ST_EINVAL = 22, ST_EBADMSG = 74 };

struct job {
  int alg, nsa, cklen, aklen, mlen;
  const uint8_t *ckeys, *akeys, *salts;
  const uint8_t *arena;
  uint8_t *out;
  int reps;
  const uint32_t *off4;
  const uint16_t *len, *sa_idx;
  uint8_t *status;
  uint32_t lo, hi;
  double t0, t1;   // the record loop's start and end (CLOCK_MONOTONIC)
  int err;
};

static const EVP_CIPHER *gcm_cipher(int klen) {
  return klen == 16 ? EVP_aes_128_gcm() : klen == 24 ? EVP_aes_192_gcm() : EVP_aes_256_gcm();
}
static const EVP_CIPHER *cbc_cipher(int klen) {
  return klen == 16 ? EVP_aes_128_cbc() : klen == 24 ? EVP_aes_192_cbc() : EVP_aes_256_cbc();
}

static uint8_t gcm_one(EVP_CIPHER_CTX *c, const uint8_t *salt, const uint8_t *rec, uint8_t *orec, int len,
                       int mlen) {
  const int ct_len = len - 16 - mlen;
  if (ct_len <= 0 || (len & 3)) return ST_EINVAL;
  uint8_t nonce[12], tag[16];
  int ol = 0, fl = 0;
  memcpy(nonce, salt, 4);
  memcpy(nonce + 4, rec + 8, 8);
  memcpy(tag, rec + len - mlen, (size_t)mlen);
  if (EVP_DecryptInit_ex(c, NULL, NULL, NULL, nonce) != 1) return ST_EINVAL;
  if (EVP_DecryptUpdate(c, NULL, &ol, rec, 8) != 1) return ST_EINVAL;
  if (EVP_DecryptUpdate(c, orec + 16, &ol, rec + 16, ct_len) != 1) return ST_EINVAL;
  if (EVP_CIPHER_CTX_ctrl(c, EVP_CTRL_GCM_SET_TAG, mlen, tag) != 1) return ST_EINVAL;
  return EVP_DecryptFinal_ex(c, orec + 16 + ol, &fl) > 0 ? ST_OK : ST_EBADMSG;
}

static uint8_t eta_one(EVP_CIPHER_CTX *c, HMAC_CTX *h, const uint8_t *rec, uint8_t *orec, int len, int mlen) {
  const int plen = len - 24 - mlen;
  if (plen <= 0 || (plen & 15) || (len & 3)) return ST_EINVAL;
  uint8_t dg[EVP_MAX_MD_SIZE];
  unsigned dl = 0;
  if (HMAC_Init_ex(h, NULL, 0, NULL, NULL) != 1 || HMAC_Update(h, rec, (size_t)(24 + plen)) != 1 ||
      HMAC_Final(h, dg, &dl) != 1)
    return ST_EINVAL;
  if (memcmp(dg, rec + 24 + plen, (size_t)mlen) != 0) return ST_EBADMSG;   // verify first
  int ol = 0;
  if (EVP_DecryptInit_ex(c, NULL, NULL, NULL, rec + 8) != 1) return ST_EINVAL;
  if (EVP_DecryptUpdate(c, orec + 24, &ol, rec + 24, plen) != 1) return ST_EINVAL;
  return ST_OK;
}

static double now_s(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void *worker(void *arg) {
  struct job *j = (struct job *)arg;
  EVP_CIPHER_CTX **cc = calloc((size_t)j->nsa, sizeof(*cc));
  HMAC_CTX **hh = calloc((size_t)j->nsa, sizeof(*hh));
  /* per-session contexts (key schedules, HMAC pads) outside the timed region,
   * as the oracle's sessions are made before it is timed */
  for (int s = 0; s < j->nsa && cc && hh; ++s) {
    cc[s] = EVP_CIPHER_CTX_new();
    const uint8_t *k = j->ckeys + (size_t)s * (size_t)j->cklen;
    if (j->alg == 0) {
      if (EVP_DecryptInit_ex(cc[s], gcm_cipher(j->cklen), NULL, NULL, NULL) != 1 ||
          EVP_CIPHER_CTX_ctrl(cc[s], EVP_CTRL_GCM_SET_IVLEN, 12, NULL) != 1 ||
          EVP_DecryptInit_ex(cc[s], NULL, NULL, k, NULL) != 1)
        j->err = 1;
    } else {
      hh[s] = HMAC_CTX_new();
      if (EVP_DecryptInit_ex(cc[s], cbc_cipher(j->cklen), NULL, k, NULL) != 1 ||
          EVP_CIPHER_CTX_set_padding(cc[s], 0) != 1 ||
          HMAC_Init_ex(hh[s], j->akeys + (size_t)s * (size_t)j->aklen, j->aklen, EVP_sha1(), NULL) != 1)
        j->err = 1;
    }
  }
  if (!cc || !hh) j->err = 1;
  j->t0 = now_s();
  for (int r = 0; r < j->reps && !j->err; ++r) {
    for (uint32_t i = j->lo; i < j->hi; ++i) {
      const int s = j->sa_idx[i];
      const size_t o = (size_t)j->off4[i] * 4;
      j->status[i] = j->alg == 0 ? gcm_one(cc[s], j->salts + 4 * (size_t)s, j->arena + o, j->out + o, j->len[i],
                                           j->mlen)
                                 : eta_one(cc[s], hh[s], j->arena + o, j->out + o, j->len[i], j->mlen);
    }
  }
  j->t1 = now_s();
  for (int s = 0; s < j->nsa && cc && hh; ++s) {
    EVP_CIPHER_CTX_free(cc[s]);
    if (hh[s]) HMAC_CTX_free(hh[s]);
  }
  free(cc);
  free(hh);
  return NULL;
}

/* Decrypts n records with nthreads threads (contiguous record ranges), reps
 * times over: plaintext to the same offsets of `out` (out == arena: in
 * place; then reps must be 1); fills status.  Returns the seconds from the
 * first thread's start of its record loop to the last one's end (session
 * setup excluded), or a negative value on error. */
double ossl_esp_batch_decrypt(int alg, int nsa, const uint8_t *ckeys, int cklen, const uint8_t *akeys,
                              int aklen, const uint8_t *salts, int mlen, const uint8_t *arena, uint8_t *out,
                              const uint32_t *off4, const uint16_t *len, const uint16_t *sa_idx,
                              uint8_t *status, uint32_t n, int nthreads, int reps) {
  if (nthreads < 1 || nsa < 1 || (alg != 0 && alg != 1) || mlen < 4 || mlen > 20 || reps < 1 ||
      (reps > 1 && out == arena))
    return -1.0;
  pthread_t *th = calloc((size_t)nthreads, sizeof(*th));
  struct job *jobs = calloc((size_t)nthreads, sizeof(*jobs));
  if (!th || !jobs) {
    free(th);
    free(jobs);
    return -1.0;
  }
  int made = 0, err = 0;
  for (int t = 0; t < nthreads; ++t) {
    struct job *j = &jobs[t];
    j->alg = alg, j->nsa = nsa, j->cklen = cklen, j->aklen = aklen, j->mlen = mlen;
    j->ckeys = ckeys, j->akeys = akeys, j->salts = salts;
    j->arena = arena, j->out = out, j->reps = reps, j->off4 = off4, j->len = len, j->sa_idx = sa_idx, j->status = status;
    j->lo = (uint32_t)((uint64_t)n * (uint64_t)t / (uint64_t)nthreads);
    j->hi = (uint32_t)((uint64_t)n * (uint64_t)(t + 1) / (uint64_t)nthreads);
    if (pthread_create(&th[t], NULL, worker, j) != 0) {
      err = 1;   // the threads already running finish and are joined
      break;
    }
    ++made;
  }
  double t0 = 0, t1 = 0;
  for (int t = 0; t < made; ++t) {
    pthread_join(th[t], NULL);
    err |= jobs[t].err;
    if (t == 0 || jobs[t].t0 < t0) t0 = jobs[t].t0;
    if (t == 0 || jobs[t].t1 > t1) t1 = jobs[t].t1;
  }
  free(th);
  free(jobs);
  return err ? -1.0 : t1 - t0;
}
