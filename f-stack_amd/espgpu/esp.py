"""ESP request builders, the caller side of the hot path (unchanged semantics).

  esp_csp()           esp_init           freebsd/netipsec/xform_esp.c:143-244
  esp_input_crp()     esp_input          xform_esp.c:260-463
  esp_output_crp()    esp_output         xform_esp.c:673-961 (padding :710-716, :810-843)
  esp_trailer_ok()    esp_input_cb tail  xform_esp.c:597-636
Records are IPv4 packets with the ESP header at `skip` (tunnel mode: skip = IP
header length), in a bytearray (or an mbuf-like list of bytearrays).
"""
import struct

from . import _lib as L
from .opencrypto import crypto_session_params

GCM, CBC_SHA1 = "aes-gcm-16", "aes-cbc-hmac-sha1-96"
CBC_SHA256, CBC_SHA384, CBC_SHA512 = ("aes-cbc-hmac-sha2-256-128", "aes-cbc-hmac-sha2-384-192",
                                      "aes-cbc-hmac-sha2-512-256")
CTR_SHA1, CTR_SHA256 = "aes-ctr-hmac-sha1-96", "aes-ctr-hmac-sha2-256-128"   # RFC 3686
CTR_SHA384, CTR_SHA512 = "aes-ctr-hmac-sha2-384-192", "aes-ctr-hmac-sha2-512-256"
# ESP-NULL (SADB_EALG_NULL, key.c:588; RFC 2410) with HMAC: encrypt-then-MAC
# sessions whose cipher is CRYPTO_NULL_CBC (no key, no IV, blocksize 4)
NULL_SHA1, NULL_SHA256 = "null-hmac-sha1-96", "null-hmac-sha2-256-128"
NULL_SHA384, NULL_SHA512 = "null-hmac-sha2-384-192", "null-hmac-sha2-512-256"
# encryption without authentication (esp_init's CSP_MODE_CIPHER, xform_esp.c:230-231)
CBC, CTR = "aes-cbc", "aes-ctr"
# auth algorithm and ICV bytes (xform_ah_authsize, xform_ah.c:117-131: 12 for
# SHA1-96, hashsize/2 for SHA2 per RFC 4868)
_AUTH = {CBC_SHA1: (L.CRYPTO_SHA1_HMAC, 12), CTR_SHA1: (L.CRYPTO_SHA1_HMAC, 12),
         CBC_SHA256: (L.CRYPTO_SHA2_256_HMAC, 16), CTR_SHA256: (L.CRYPTO_SHA2_256_HMAC, 16),
         CBC_SHA384: (L.CRYPTO_SHA2_384_HMAC, 24), CTR_SHA384: (L.CRYPTO_SHA2_384_HMAC, 24),
         CBC_SHA512: (L.CRYPTO_SHA2_512_HMAC, 32), CTR_SHA512: (L.CRYPTO_SHA2_512_HMAC, 32),
         NULL_SHA1: (L.CRYPTO_SHA1_HMAC, 12), NULL_SHA256: (L.CRYPTO_SHA2_256_HMAC, 16),
         NULL_SHA384: (L.CRYPTO_SHA2_384_HMAC, 24), NULL_SHA512: (L.CRYPTO_SHA2_512_HMAC, 32)}
_CTR_ALGS = (CTR_SHA1, CTR_SHA256, CTR_SHA384, CTR_SHA512, CTR)
_NULL_ALGS = (NULL_SHA1, NULL_SHA256, NULL_SHA384, NULL_SHA512)
ETA_ALGS = tuple(_AUTH)
CIPHER_ALGS = (CBC, CTR)
IPPROTO_NONE = 59


class SecAssoc:
    """What key_setsaval leaves in struct secasvar for the two ESP transforms."""

    def __init__(self, spi, alg, key, auth_key=b"", esn=False, mlen=None):
        self.spi = spi
        self.alg = alg
        self.key = bytes(key)          # GCM: cipher key || 4-byte salt (RFC 4106 8.1)
        self.auth_key = bytes(auth_key)
        self.esn = esn
        # ICV bytes: xform_ah_authsize (GMAC 16, SHA1-HMAC 12, SHA2-HMAC
        # hashsize/2); a GCM SA may carry a truncated 12- or 8-byte ICV
        # (RFC 4106 s3.3, csp_auth_mlen)
        self.mlen = mlen if mlen is not None else (
            16 if alg == GCM else _AUTH[alg][1] if alg in _AUTH else 0)

    @property
    def ctr(self):
        return self.alg in _CTR_ALGS

    @property
    def null(self):
        return self.alg in _NULL_ALGS

    @property
    def auth(self):
        """An ICV to verify / compute (every transform but the CIPHER ones)."""
        return self.alg == GCM or self.alg in _AUTH

    @property
    def cipher_alg(self):
        return L.CRYPTO_AES_ICM if self.ctr else L.CRYPTO_NULL_CBC if self.null else L.CRYPTO_AES_CBC

    @property
    def auth_alg(self):
        return _AUTH[self.alg][0] if self.alg in _AUTH else 0

    @property
    def ivlen(self):
        # RFC 4106 / 3686: 8-byte IV; enc_xform_null: none; CBC: 16
        return 8 if self.alg == GCM or self.ctr else 0 if self.null else 16

    @property
    def hlen(self):
        return 8 + self.ivlen           # struct newesp + IV

    @property
    def alen(self):
        return self.mlen

    @property
    def blocksize(self):
        # enc_xform blocksize (ESP pads to 4 anyway): GCM / CTR 1, NULL 4, CBC 16
        return 1 if self.alg == GCM or self.ctr else 4 if self.null else 16

    @property
    def salt(self):
        # the 4-byte salt / nonce esp_init strips off the key (RFC 4106 8.1, RFC 3686 5.1)
        return self.key[-4:] if self.alg == GCM or self.ctr else b"\0\0\0\0"

    def csp(self):
        if self.alg == GCM:
            return crypto_session_params(
                csp_mode=L.CSP_MODE_AEAD,
                csp_flags=L.CSP_F_SEPARATE_AAD if self.esn else 0,
                csp_ivlen=12, csp_cipher_alg=L.CRYPTO_AES_NIST_GCM_16,
                csp_cipher_klen=len(self.key) - 4, csp_cipher_key=self.key[:-4],
                csp_auth_mlen=0 if self.mlen == 16 else self.mlen)
        ckey = self.key[:-4] if self.ctr else b"" if self.null else self.key
        ivsize = 0 if self.null else 16                      # csp_ivlen = txform->ivsize (:240)
        if not self.auth:                                     # esp_init :230-231
            return crypto_session_params(
                csp_mode=L.CSP_MODE_CIPHER, csp_ivlen=ivsize, csp_cipher_alg=self.cipher_alg,
                csp_cipher_klen=len(ckey), csp_cipher_key=ckey)
        return crypto_session_params(
            csp_mode=L.CSP_MODE_ETA, csp_flags=L.CSP_F_ESN if self.esn else 0,
            csp_ivlen=ivsize, csp_cipher_alg=self.cipher_alg, csp_cipher_klen=len(ckey),
            csp_cipher_key=ckey if ckey else None, csp_auth_alg=self.auth_alg,
            csp_auth_klen=len(self.auth_key), csp_auth_key=self.auth_key, csp_auth_mlen=self.mlen)


def _flat(buf):
    return bytes(buf) if not isinstance(buf, list) else b"".join(bytes(b) for b in buf)


def esp_input_crp(fw, ses, sa, pkt, skip, esn_hi=0):
    """Build the decrypt+verify cryptop exactly as esp_input does."""
    total = len(_flat(pkt))
    crp = fw.crypto_getreq(ses)
    seqh = struct.pack(">I", esn_hi)
    data = _flat(pkt)
    if sa.auth:                                                               # :364-405
        crp.crp_op = L.CRYPTO_OP_VERIFY_DIGEST
        crp.crp_aad_length = 8 if sa.alg == GCM else sa.hlen                  # :366-369
        if sa.alg == GCM and sa.esn:                                          # :372-397
            crp.crp_aad = data[skip:skip + 4] + seqh + data[skip + 4:skip + 8]
            crp.crp_aad_length = 12
        else:
            crp.crp_aad_start = skip
        if sa.alg != GCM and sa.esn:
            crp.crp_esn = seqh                                                # :400-402
        crp.crp_digest_start = total - sa.alen                                # :404
    crp.crp_op |= L.CRYPTO_OP_DECRYPT                                         # :420
    crp.crp_flags = L.CRYPTO_F_CBIFSYNC
    crp.crp_buf = pkt
    crp.crp_payload_start = skip + sa.hlen                                    # :424-425
    crp.crp_payload_length = total - (skip + sa.hlen + sa.alen)
    if sa.alg == GCM or sa.ctr:                                               # :430-458
        ctr0 = struct.pack(">I", 1) if sa.ctr else b"\0" * 4
        crp.crp_iv = bytearray(sa.salt + data[skip + sa.hlen - sa.ivlen:skip + sa.hlen] + ctr0)
        crp.crp_flags |= L.CRYPTO_F_IV_SEPARATE
    elif sa.ivlen:
        crp.crp_iv_start = skip + sa.hlen - sa.ivlen
    return crp


def esp_output_crp(fw, ses, sa, pkt, skip, esn_hi=0):
    """The encrypt cryptop esp_output builds over an already padded packet."""
    total = len(_flat(pkt))
    data = _flat(pkt)
    crp = fw.crypto_getreq(ses)
    crp.crp_op = L.CRYPTO_OP_ENCRYPT | (L.CRYPTO_OP_COMPUTE_DIGEST if sa.auth else 0)
    crp.crp_flags = L.CRYPTO_F_CBIFSYNC
    crp.crp_buf = pkt
    crp.crp_payload_start = skip + sa.hlen
    crp.crp_payload_length = total - (skip + sa.hlen + sa.alen)
    seqh = struct.pack(">I", esn_hi)
    if not sa.auth:                                                   # :862-887, no esph
        if sa.ctr:
            crp.crp_iv = bytearray(sa.salt + data[skip + 8:skip + 16] + struct.pack(">I", 1))
            crp.crp_flags |= L.CRYPTO_F_IV_SEPARATE
        elif sa.ivlen:
            crp.crp_iv_start = skip + 8
        return crp
    crp.crp_digest_start = total - sa.alen
    if sa.alg == GCM:
        if sa.esn:
            crp.crp_aad = data[skip:skip + 4] + seqh + data[skip + 4:skip + 8]
            crp.crp_aad_length = 12
        else:
            crp.crp_aad_start = skip
            crp.crp_aad_length = 8
        crp.crp_iv = bytearray(sa.salt + data[skip + 8:skip + 16] + b"\0" * 4)
        crp.crp_flags |= L.CRYPTO_F_IV_SEPARATE
    else:
        crp.crp_aad_start = skip
        crp.crp_aad_length = sa.hlen
        if sa.ctr:
            crp.crp_iv = bytearray(sa.salt + data[skip + 8:skip + 16] + struct.pack(">I", 1))
            crp.crp_flags |= L.CRYPTO_F_IV_SEPARATE
        elif sa.ivlen:
            crp.crp_iv_start = skip + 8
        if sa.esn:
            crp.crp_esn = seqh
    return crp


def esp_pad(inner, blocksize=4, next_header=4):
    """Self-describing padding 1,2,3,... + pad length + next header (xform_esp.c:810-843)."""
    rlen = len(inner)
    padding = ((blocksize - ((rlen + 2) % blocksize)) % blocksize) + 2
    pad = bytes(range(1, padding - 1)) + bytes([padding - 2, next_header])
    return bytes(inner) + pad


def trailer_word(plain_payload):
    """The 32-bit word the kernels' fused trailer check produces for a
    decrypted payload (espgpu_decrypt_batch_trailer, include/espgpu.h):
    next header | pad length << 8 | TR_* flags | TR_VALID."""
    from . import _lib as L
    p = bytes(plain_payload)
    l0, padlen, nh = p[-3], p[-2], p[-1]
    t = nh | (padlen << 8) | L.TR_VALID
    if padlen + 2 > len(p):
        t |= L.TR_BADLEN
    if padlen != l0 and padlen != 0:
        t |= L.TR_BADPAD
    if nh == IPPROTO_NONE:
        t |= L.TR_NONE
    return t


def trailer_accepts(word, prand=False):
    """esp_input_cb's verdict (xform_esp.c:597-630) from a trailer word:
    True = keep the packet.  prand: the SA uses random padding
    (SADB_X_EXT_PRAND), which skips the pad-content check."""
    from . import _lib as L
    if not word & L.TR_VALID or word & (L.TR_BADLEN | L.TR_NONE):
        return False
    return prand or not word & L.TR_BADPAD


def esp_trailer_ok(plain_payload):
    """The checks esp_input_cb makes on the last three plaintext bytes
    (xform_esp.c:597-630, default SADB_X_EXT_PSEQ padding)."""
    p = bytes(plain_payload)
    last = p[-3:]
    if last[1] + 2 > len(p):
        return False
    if last[1] != last[0] and last[1] != 0:
        return False
    return last[2] != IPPROTO_NONE
