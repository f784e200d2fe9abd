"""CPU tests of the drop-in boundary: libespgpu.so loads, exports every
function include/espgpu.h declares, its structs have the ABI layout, and the
host-only driver logic (probesession = swcr_probesession + check_csp for the
ESP ciphers) answers like the reference.  No compute calls: no GPU here."""
import ctypes as C

import pytest

from espgpu import _lib as L
from espgpu.esp import CBC_SHA1, GCM, SecAssoc, esp_pad, esp_trailer_ok
from espgpu.opencrypto import GpuCryptoDriver, crypto_session_params


def test_library_exports_header_symbols():
    lib = L.lib()
    syms = L.header_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(lib, s), "missing export %s" % s
    assert lib.espgpu_abi_version() == 6    # ABI 6: espgpu_session_room


def test_struct_layouts():
    assert C.sizeof(L.Desc) == 16
    assert C.sizeof(L.Completion) == 16
    assert L.Req.crp_iv.offset % 1 == 0
    # espgpu_req must match the C layout: check a few offsets against natural alignment
    assert L.Req.segs.offset == 16 and L.Req.crp_aad.offset == 32
    # struct espgpu_stats: 15 uint64 counters (ABI 5 appended gpu_fail, fail_eio)
    assert C.sizeof(L.Stats) == 15 * 8 and L.Stats.fail_eio.offset == 14 * 8


def _probe(**kw):
    return GpuCryptoDriver.probesession(crypto_session_params(**kw))


@pytest.mark.parametrize("klen", [16, 24, 32])
def test_probesession_accepts_esp_gcm(klen):
    assert _probe(csp_mode=L.CSP_MODE_AEAD, csp_ivlen=12, csp_cipher_alg=L.CRYPTO_AES_NIST_GCM_16,
                  csp_cipher_klen=klen, csp_cipher_key=b"k" * klen) == L.CRYPTODEV_PROBE_HARDWARE
    assert _probe(csp_mode=L.CSP_MODE_AEAD, csp_flags=L.CSP_F_SEPARATE_AAD, csp_ivlen=12,
                  csp_cipher_alg=L.CRYPTO_AES_NIST_GCM_16, csp_cipher_klen=klen,
                  csp_cipher_key=b"k" * klen) == L.CRYPTODEV_PROBE_HARDWARE
    for mlen in (8, 12, 16):            # RFC 4106 ICV lengths
        assert _probe(csp_mode=L.CSP_MODE_AEAD, csp_ivlen=12, csp_cipher_alg=L.CRYPTO_AES_NIST_GCM_16,
                      csp_cipher_klen=klen, csp_cipher_key=b"k" * klen,
                      csp_auth_mlen=mlen) == L.CRYPTODEV_PROBE_HARDWARE


@pytest.mark.parametrize("calg", [L.CRYPTO_AES_CBC, L.CRYPTO_AES_ICM])
@pytest.mark.parametrize("aalg,mlen", [(L.CRYPTO_SHA1_HMAC, 12), (L.CRYPTO_SHA2_256_HMAC, 16),
                                       (L.CRYPTO_SHA2_256_HMAC, 0), (L.CRYPTO_SHA2_384_HMAC, 24),
                                       (L.CRYPTO_SHA2_384_HMAC, 48), (L.CRYPTO_SHA2_512_HMAC, 32),
                                       (L.CRYPTO_SHA2_512_HMAC, 0)])
def test_probesession_accepts_eta_variants(calg, aalg, mlen):
    """AES-CBC / AES-CTR (enc_xform ivsize 16, xform_aes_icm.c:69) with
    HMAC-SHA1 or HMAC-SHA2-256/384/512 (esp_init, xform_esp.c:225-241; ICV
    up to the hash size, swcr_setup_auth)."""
    for klen in (16, 24, 32):
        assert _probe(csp_mode=L.CSP_MODE_ETA, csp_ivlen=16, csp_cipher_alg=calg, csp_cipher_klen=klen,
                      csp_cipher_key=b"k" * klen, csp_auth_alg=aalg, csp_auth_klen=32,
                      csp_auth_key=b"a" * 32, csp_auth_mlen=mlen) == L.CRYPTODEV_PROBE_HARDWARE


@pytest.mark.parametrize("calg,klen,ivlen", [(L.CRYPTO_AES_CBC, 16, 16), (L.CRYPTO_AES_CBC, 32, 16),
                                             (L.CRYPTO_AES_ICM, 24, 16), (L.CRYPTO_NULL_CBC, 0, 0)])
def test_probesession_accepts_cipher_only(calg, klen, ivlen):
    """ESP with encryption and no auth: esp_init's CSP_MODE_CIPHER
    (xform_esp.c:230-231; swcr_probesession :1257-1266)."""
    assert _probe(csp_mode=L.CSP_MODE_CIPHER, csp_ivlen=ivlen, csp_cipher_alg=calg, csp_cipher_klen=klen,
                  csp_cipher_key=b"k" * klen if klen else None) == L.CRYPTODEV_PROBE_HARDWARE


@pytest.mark.parametrize("aalg,mlen", [(L.CRYPTO_SHA1_HMAC, 12), (L.CRYPTO_SHA2_256_HMAC, 16),
                                       (L.CRYPTO_SHA2_384_HMAC, 24), (L.CRYPTO_SHA2_512_HMAC, 32)])
def test_probesession_accepts_esp_null(aalg, mlen):
    """ESP-NULL with HMAC (SADB_EALG_NULL, key.c:588): CSP_MODE_ETA with
    CRYPTO_NULL_CBC, no cipher key, csp_ivlen 0 (enc_xform_null's ivsize)."""
    assert _probe(csp_mode=L.CSP_MODE_ETA, csp_ivlen=0, csp_cipher_alg=L.CRYPTO_NULL_CBC, csp_auth_alg=aalg,
                  csp_auth_klen=32, csp_auth_key=b"a" * 32, csp_auth_mlen=mlen) == L.CRYPTODEV_PROBE_HARDWARE


def test_probesession_accepts_esp_cbc_sha1():
    assert _probe(csp_mode=L.CSP_MODE_ETA, csp_ivlen=16, csp_cipher_alg=L.CRYPTO_AES_CBC,
                  csp_cipher_klen=32, csp_cipher_key=b"k" * 32, csp_auth_alg=L.CRYPTO_SHA1_HMAC,
                  csp_auth_klen=20, csp_auth_key=b"a" * 20, csp_auth_mlen=12) == -100


@pytest.mark.parametrize("kw", [
    dict(csp_mode=L.CSP_MODE_AEAD, csp_ivlen=16, csp_cipher_alg=25, csp_cipher_klen=16),   # ivlen != 12
    dict(csp_mode=L.CSP_MODE_AEAD, csp_ivlen=12, csp_cipher_alg=25, csp_cipher_klen=20),   # bad key length
    dict(csp_mode=L.CSP_MODE_AEAD, csp_ivlen=12, csp_cipher_alg=11, csp_cipher_klen=16),   # CBC as AEAD
    dict(csp_mode=L.CSP_MODE_ETA, csp_ivlen=16, csp_cipher_alg=25, csp_cipher_klen=16,
         csp_auth_alg=7, csp_auth_klen=20),                                                 # GCM as ETA
    dict(csp_mode=L.CSP_MODE_ETA, csp_ivlen=16, csp_cipher_alg=11, csp_cipher_klen=16,
         csp_auth_alg=9, csp_auth_klen=32),                                                 # auth alg not served
    dict(csp_mode=L.CSP_MODE_ETA, csp_ivlen=16, csp_cipher_alg=11, csp_cipher_klen=16,
         csp_auth_alg=19, csp_auth_klen=48, csp_auth_mlen=52),                              # mlen > SHA-384
    dict(csp_mode=L.CSP_MODE_ETA, csp_ivlen=16, csp_cipher_alg=11, csp_cipher_klen=16,
         csp_auth_alg=20, csp_auth_klen=64, csp_auth_mlen=30),                              # ICV not dwords
    dict(csp_mode=L.CSP_MODE_ETA, csp_ivlen=16, csp_cipher_alg=11, csp_cipher_klen=16,
         csp_auth_alg=8, csp_auth_klen=20),                                                 # RIPEMD-160 not served
    dict(csp_mode=L.CSP_MODE_ETA, csp_ivlen=12, csp_cipher_alg=23, csp_cipher_klen=16,
         csp_auth_alg=7, csp_auth_klen=20),                                                 # CTR ivlen != 16
    dict(csp_mode=L.CSP_MODE_ETA, csp_ivlen=16, csp_cipher_alg=23, csp_cipher_klen=16,
         csp_auth_alg=18, csp_auth_klen=32, csp_auth_mlen=36),                              # mlen > SHA-256
    dict(csp_mode=2, csp_ivlen=16, csp_cipher_alg=11, csp_cipher_klen=16, csp_auth_alg=7,
         csp_auth_klen=20),                                                                 # cipher-only with auth
    dict(csp_mode=2, csp_flags=0x4, csp_ivlen=16, csp_cipher_alg=11, csp_cipher_klen=16),   # cipher-only with ESN
    dict(csp_mode=2, csp_ivlen=16, csp_cipher_alg=11, csp_cipher_klen=20),                  # cipher-only, bad key
    dict(csp_mode=2, csp_ivlen=0, csp_cipher_alg=16, csp_cipher_klen=8),                    # NULL with a key
    dict(csp_mode=L.CSP_MODE_ETA, csp_ivlen=0, csp_cipher_alg=16, csp_cipher_klen=16,
         csp_auth_alg=7, csp_auth_klen=20),                                                 # ESP-NULL with a key
    dict(csp_mode=L.CSP_MODE_AEAD, csp_ivlen=12, csp_cipher_alg=25, csp_cipher_klen=16,
         csp_auth_mlen=4),                                                                  # GCM ICV 4 (not RFC 4106)
    # ESP AES-GMAC (SADB_X_EALG_AESGMAC, key.c:591, RFC 4543): esp_init makes
    # it CSP_MODE_CIPHER with CRYPTO_AES_NIST_GMAC (xform_esp.c:230-236), which
    # check_csp refuses (alg_is_cipher: GMAC is ALG_KEYED_DIGEST, crypto.c:682,
    # :747-783), so crypto_newsession fails on the reference too
    dict(csp_mode=2, csp_ivlen=12, csp_cipher_alg=24, csp_cipher_klen=16),
    dict(csp_mode=L.CSP_MODE_AEAD, csp_flags=0x1, csp_ivlen=12, csp_cipher_alg=25,
         csp_cipher_klen=16),                                                               # SEPARATE_OUTPUT
    dict(csp_mode=L.CSP_MODE_AEAD, csp_ivlen=12, csp_cipher_alg=25, csp_cipher_klen=16,
         csp_auth_mlen=10),                                                                 # ICV not dwords
])
def test_probesession_rejects(kw):
    assert _probe(**kw) == L.EINVAL


def test_sa_session_params_follow_esp_init():
    sa = SecAssoc(0x1234, GCM, bytes(20))
    csp = sa.csp()
    assert csp.csp_cipher_klen == 16 and csp.csp_ivlen == 12 and csp.csp_mode == L.CSP_MODE_AEAD
    sa2 = SecAssoc(0x1234, CBC_SHA1, bytes(32), bytes(20), esn=True)
    c2 = sa2.csp()
    assert c2.csp_flags == L.CSP_F_ESN and c2.csp_auth_mlen == 12 and sa2.hlen == 24 and sa2.alen == 12


def test_esp_padding_and_trailer_checks():
    for n in range(40, 60):
        p = esp_pad(bytes(n), blocksize=4)
        assert len(p) % 4 == 0 and esp_trailer_ok(p)
    p = bytearray(esp_pad(bytes(41), 16))
    assert len(p) % 16 == 0
    p[-2] = 200
    assert not esp_trailer_ok(p)


def test_init_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        GpuCryptoDriver()
