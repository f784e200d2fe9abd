"""ctypes bindings for the oracle (oracle/liboracle.so, oracle/_ref/libref.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libref.so")

CSP_MODE_CIPHER = 2          # cryptodev.h:362, ESP without auth
CSP_MODE_AEAD = 4
CSP_MODE_ETA = 5
CRYPTO_SHA1_HMAC = 7
CRYPTO_AES_CBC = 11
CRYPTO_SHA2_256_HMAC = 18
CRYPTO_SHA2_384_HMAC = 19
CRYPTO_SHA2_512_HMAC = 20
HASH_LEN = {CRYPTO_SHA1_HMAC: 20, CRYPTO_SHA2_256_HMAC: 32, CRYPTO_SHA2_384_HMAC: 48, CRYPTO_SHA2_512_HMAC: 64}
CRYPTO_AES_ICM = 23
CRYPTO_NULL_CBC = 16         # cryptodev.h:160, enc_xform_null
CSP_F_SEPARATE_AAD = 0x2
CSP_F_ESN = 0x4
EBADMSG = 74
EINVAL = 22

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("oracle not built: run `make -C oracle`")
        L = C.CDLL(LIB_PATH)
        u8p, u32p, u16p = C.POINTER(C.c_uint8), C.POINTER(C.c_uint32), C.POINTER(C.c_uint16)
        L.oref_sa_new.restype = C.c_void_p
        L.oref_sa_new.argtypes = [C.c_int, C.c_int, C.c_char_p, C.c_int, C.c_char_p,
                                  C.c_char_p, C.c_int, C.c_int]
        L.oref_sa_new2.restype = C.c_void_p
        L.oref_sa_new2.argtypes = [C.c_int, C.c_int, C.c_int, C.c_char_p, C.c_int, C.c_char_p,
                                   C.c_int, C.c_char_p, C.c_int, C.c_int]
        L.oref_sa_free.argtypes = [C.c_void_p]
        L.oref_sha256.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p]
        L.oref_hmac.argtypes = [C.c_int, C.c_char_p, C.c_int, C.c_char_p, C.c_size_t, C.c_void_p]
        L.oref_hash.argtypes = [C.c_int, C.c_char_p, C.c_size_t, C.c_void_p]
        L.oref_aes_ctr.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_void_p, C.c_int]
        L.oref_esp_decrypt.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_uint32]
        L.oref_esp_encrypt.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_uint32]
        L.oref_gcm.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_char_p, C.c_int,
                               C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int]
        L.oref_eta.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_int, C.c_char_p, C.c_char_p,
                               C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int]
        L.oref_aes_setkey_enc.argtypes = [u32p, C.c_char_p, C.c_int]
        L.oref_aes_setkey_dec.argtypes = [u32p, C.c_char_p, C.c_int]
        L.oref_aes_encrypt.argtypes = [u32p, C.c_int, C.c_char_p, C.c_void_p]
        L.oref_aes_decrypt.argtypes = [u32p, C.c_int, C.c_char_p, C.c_void_p]
        L.oref_gf128_mul.argtypes = [C.c_char_p, C.c_char_p, C.c_void_p]
        L.oref_sha1.argtypes = [C.c_char_p, C.c_size_t, C.c_void_p]
        L.oref_hmac_sha1.argtypes = [C.c_char_p, C.c_int, C.c_char_p, C.c_size_t, C.c_void_p]
        L.oref_batch_decrypt.restype = C.c_double
        L.oref_batch_decrypt.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, u32p, u16p, u16p,
                                         u32p, u8p, C.c_long, C.c_int]
        L.oref_batch_encrypt.restype = C.c_double
        L.oref_batch_encrypt.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, u32p, u16p, u16p,
                                         u32p, C.c_long, C.c_int]
        L.oref_chkreplay.argtypes = [C.c_uint32, u32p, C.c_void_p]
        L.oref_updatereplay.argtypes = [C.c_uint32, C.c_void_p]
        _lib = L
    return _lib


class _ReplayC(C.Structure):
    _fields_ = [("count", C.c_uint64), ("last", C.c_uint64), ("wsize", C.c_uint32),
                ("bitmap_size", C.c_uint32), ("bitmap", C.POINTER(C.c_uint32)),
                ("overflow", C.c_int), ("flags", C.c_int)]


REPLAY_ESN, REPLAY_CYCSEQ = 1, 2


class Replay:
    """An SA's replay window (struct secreplay, keydb.h:206-213) driven by the
    restated ipsec_chkreplay / ipsec_updatereplay (ipsec.c:1248-1436).  The
    bitmap size follows key_setsaval (key.c:3346-3351): the smallest power of
    two >= wsize + 4 bytes, in 32-bit words."""

    def __init__(self, wsize, last=0, flags=0):
        import numpy as np
        words = 1
        while wsize + 4 > words:
            words <<= 1
        words = max(words // 4, 1)
        self.bitmap = np.zeros(words, dtype=np.uint32)
        self.c = _ReplayC(0, last, wsize, words,
                          self.bitmap.ctypes.data_as(C.POINTER(C.c_uint32)), 0, flags)

    def check(self, seq):
        """(permitted, seqhigh)"""
        sh = C.c_uint32(0xFFFFFFFF)
        ok = lib().oref_chkreplay(seq & 0xFFFFFFFF, C.byref(sh), C.byref(self.c))
        return bool(ok), sh.value

    def update(self, seq):
        """True if the window accepted seq (ipsec_updatereplay returned 0)"""
        return lib().oref_updatereplay(seq & 0xFFFFFFFF, C.byref(self.c)) == 0

    @property
    def last(self):
        return self.c.last


class SA:
    """A cryptosoft-style session (swcr_newsession)."""

    def __init__(self, mode, ckey, salt=b"\0\0\0\0", akey=b"", mlen=0, flags=0,
                 calg=CRYPTO_AES_CBC, aalg=CRYPTO_SHA1_HMAC):
        """ETA: calg CRYPTO_AES_CBC or CRYPTO_AES_ICM (ESP AES-CTR, salt = the
        RFC 3686 nonce), aalg CRYPTO_SHA1_HMAC or CRYPTO_SHA2_256/384/512_HMAC."""
        self.mode = mode
        self.h = lib().oref_sa_new2(mode, flags, calg, bytes(ckey), len(ckey), bytes(salt),
                                    aalg, bytes(akey), len(akey), mlen)
        if not self.h:
            raise ValueError("oref_sa_new failed")

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.oref_sa_free(self.h)
            self.h = None

    def esp_decrypt(self, rec, esn_hi=0):
        """-> (etype, bytes) ; in-place semantics on a copy."""
        buf = C.create_string_buffer(bytes(rec), len(rec))
        e = lib().oref_esp_decrypt(self.h, buf, len(rec), esn_hi)
        return e, buf.raw

    def esp_encrypt(self, rec, esn_hi=0):
        buf = C.create_string_buffer(bytes(rec), len(rec))
        e = lib().oref_esp_encrypt(self.h, buf, len(rec), esn_hi)
        return e, buf.raw


def gcm(key, iv, aad, data, tag=b"\0" * 16, mlen=16, encrypt=True):
    buf = C.create_string_buffer(bytes(data), max(1, len(data)))
    t = C.create_string_buffer(bytes(tag).ljust(16, b"\0"), 16)
    e = lib().oref_gcm(bytes(key), len(key), bytes(iv), bytes(aad), len(aad), buf, len(data),
                       t, mlen, 1 if encrypt else 0)
    return e, buf.raw[:len(data)], t.raw


def eta(ckey, akey, iv, aad, data, digest=b"\0" * 20, mlen=20, encrypt=True):
    """AES-CBC + HMAC-SHA1 EtA -> (etype, data', digest20)."""
    buf = C.create_string_buffer(bytes(data), max(1, len(data)))
    d = C.create_string_buffer(bytes(digest).ljust(20, b"\0"), 20)
    e = lib().oref_eta(bytes(ckey), len(ckey), bytes(akey), len(akey), bytes(iv), bytes(aad),
                       len(aad), buf, len(data), d, mlen, 1 if encrypt else 0)
    return e, buf.raw[:len(data)], d.raw


def sha256(msg):
    out = C.create_string_buffer(32)
    lib().oref_sha256(bytes(msg), len(msg), out)
    return out.raw


def hash(alg, msg):
    """Plain SHA-1 / SHA-256 / SHA-384 / SHA-512 (alg = the HMAC algorithm id)."""
    out = C.create_string_buffer(64)
    lib().oref_hash(alg, bytes(msg), len(msg), out)
    return out.raw[:HASH_LEN[alg]]


def hmac(alg, key, msg):
    out = C.create_string_buffer(64)
    lib().oref_hmac(alg, bytes(key), len(key), bytes(msg), len(msg), out)
    return out.raw[:HASH_LEN[alg]]


def aes_ctr(key, ctr16, data):
    """AES-ICM (full 128-bit counter increment) starting at ctr16."""
    buf = C.create_string_buffer(bytes(data), max(1, len(data)))
    lib().oref_aes_ctr(bytes(key), len(key), bytes(ctr16), buf, len(data))
    return buf.raw[:len(data)]


def aes_encrypt_block(key, block):
    rk = (C.c_uint32 * 60)()
    nr = lib().oref_aes_setkey_enc(rk, bytes(key), len(key) * 8)
    out = C.create_string_buffer(16)
    lib().oref_aes_encrypt(rk, nr, bytes(block), out)
    return out.raw


def aes_decrypt_block(key, block):
    rk = (C.c_uint32 * 60)()
    nr = lib().oref_aes_setkey_dec(rk, bytes(key), len(key) * 8)
    out = C.create_string_buffer(16)
    lib().oref_aes_decrypt(rk, nr, bytes(block), out)
    return out.raw


def aes_round_keys(key, decrypt=False):
    rk = (C.c_uint32 * 60)()
    f = lib().oref_aes_setkey_dec if decrypt else lib().oref_aes_setkey_enc
    nr = f(rk, bytes(key), len(key) * 8)
    return nr, list(rk)[: 4 * (nr + 1)]


def gf128_mul(h, x):
    out = C.create_string_buffer(16)
    lib().oref_gf128_mul(bytes(h), bytes(x), out)
    return out.raw


def sha1(msg):
    out = C.create_string_buffer(20)
    lib().oref_sha1(bytes(msg), len(msg), out)
    return out.raw


def hmac_sha1(key, msg):
    out = C.create_string_buffer(20)
    lib().oref_hmac_sha1(bytes(key), len(key), bytes(msg), len(msg), out)
    return out.raw


def _ptr(a, ct):
    return a.ctypes.data_as(C.POINTER(ct))


def batch(sas, arena, off4, lens, sa_idx, esn_hi=None, nthreads=1, encrypt=False):
    """Process records in a numpy uint8 arena in place. -> (seconds, status)."""
    n = len(off4)
    arr = (C.c_void_p * len(sas))(*[s.h for s in sas])
    off4 = np.ascontiguousarray(off4, dtype=np.uint32)
    lens = np.ascontiguousarray(lens, dtype=np.uint16)
    sa_idx = np.ascontiguousarray(sa_idx, dtype=np.uint16)
    eh = None if esn_hi is None else _ptr(np.ascontiguousarray(esn_hi, dtype=np.uint32), C.c_uint32)
    assert arena.dtype == np.uint8 and arena.flags.c_contiguous
    if encrypt:
        t = lib().oref_batch_encrypt(arr, arena.ctypes.data, _ptr(off4, C.c_uint32),
                                     _ptr(lens, C.c_uint16), _ptr(sa_idx, C.c_uint16), eh, n,
                                     nthreads)
        return t, None
    status = np.zeros(n, dtype=np.uint8)
    t = lib().oref_batch_decrypt(arr, arena.ctypes.data, _ptr(off4, C.c_uint32),
                                 _ptr(lens, C.c_uint16), _ptr(sa_idx, C.c_uint16), eh,
                                 _ptr(status, C.c_uint8), n, nthreads)
    return t, status


# ---------------------------------------------------------------------------
# The reference's own primitives, compiled from /root/reference (oracle/_ref).

class _GF128(C.Structure):
    _fields_ = [("v", C.c_uint64 * 2)]


_ref = None


def ref_available():
    return os.path.exists(REF_PATH)


def ref():
    global _ref
    if _ref is None:
        R = C.CDLL(REF_PATH)
        R.rijndaelKeySetupEnc.argtypes = [C.POINTER(C.c_uint32), C.c_char_p, C.c_int]
        R.rijndaelKeySetupDec.argtypes = [C.POINTER(C.c_uint32), C.c_char_p, C.c_int]
        R.rijndaelEncrypt.argtypes = [C.POINTER(C.c_uint32), C.c_int, C.c_char_p, C.c_void_p]
        R.rijndaelDecrypt.argtypes = [C.POINTER(C.c_uint32), C.c_int, C.c_char_p, C.c_void_p]
        R.gf128_genmultable.argtypes = [_GF128, C.c_void_p]
        R.gf128_mul.argtypes = [_GF128, C.c_void_p]
        R.gf128_mul.restype = _GF128
        _ref = R
    return _ref


def ref_aes_encrypt_block(key, block, decrypt=False):
    R = ref()
    rk = (C.c_uint32 * 60)()
    nr = (R.rijndaelKeySetupDec if decrypt else R.rijndaelKeySetupEnc)(rk, bytes(key), len(key) * 8)
    out = C.create_string_buffer(16)
    (R.rijndaelDecrypt if decrypt else R.rijndaelEncrypt)(rk, nr, bytes(block), out)
    return out.raw, nr, list(rk)[: 4 * (nr + 1)]


def ref_gf128_mul(h, x):
    """gf128_genmultable + gf128_mul from the reference's gfmult.c."""
    R = ref()
    raw = np.zeros(256 + 64, dtype=np.uint8)          # struct gf128table, 64-B aligned
    off = (-raw.ctypes.data) % 64
    tbl = raw.ctypes.data + off
    hv = _GF128((C.c_uint64 * 2)(int.from_bytes(h[:8], "big"), int.from_bytes(h[8:], "big")))
    xv = _GF128((C.c_uint64 * 2)(int.from_bytes(x[:8], "big"), int.from_bytes(x[8:], "big")))
    R.gf128_genmultable(hv, C.c_void_p(tbl))
    r = R.gf128_mul(xv, C.c_void_p(tbl))
    return r.v[0].to_bytes(8, "big") + r.v[1].to_bytes(8, "big")
