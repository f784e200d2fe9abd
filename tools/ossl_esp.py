"""ctypes binding of tools/libossl_esp.so (OpenSSL EVP ESP decrypt, the
comparison point bench.py reports as `cpu_openssl`; not the reference path,
see ossl_esp.c)."""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "libossl_esp.so")
_lib = None


def available():
    return os.path.exists(LIB)


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(LIB)
        f = _lib.ossl_esp_batch_decrypt
        f.restype = C.c_double
        f.argtypes = [C.c_int, C.c_int, C.c_char_p, C.c_int, C.c_char_p, C.c_int, C.c_char_p, C.c_int,
                      C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                      C.c_int, C.c_int]
    return _lib


def batch_decrypt(alg, ckeys, arena, off4, lens, sa_idx, akeys=None, salts=None, mlen=16, nthreads=1,
                  out=None, reps=1):
    """Decrypt records of `arena` (numpy uint8): in place, or with `out` (same
    size) to the same offsets of out, `reps` times over (out of place only).
    alg 'gcm': ckeys = AES keys (one per SA), salts = 4-byte salts;
    alg 'cbc_sha1': ckeys = AES keys, akeys = HMAC keys (20 B each).
    -> (seconds, status array: 0 ok, 74 EBADMSG, 22 EINVAL)."""
    a = 0 if alg == "gcm" else 1
    nsa = len(ckeys)
    cklen = len(ckeys[0])
    assert all(len(k) == cklen for k in ckeys)
    ck = b"".join(bytes(k) for k in ckeys)
    if a == 0:
        ak, aklen = b"\0", 0
        sl = b"".join(bytes(s) for s in salts)
        assert len(sl) == 4 * nsa
    else:
        aklen = len(akeys[0])
        ak = b"".join(bytes(k) for k in akeys)
        sl = b"\0" * 4
    off4 = np.ascontiguousarray(off4, dtype=np.uint32)
    lens = np.ascontiguousarray(lens, dtype=np.uint16)
    sa_idx = np.ascontiguousarray(sa_idx, dtype=np.uint16)
    assert arena.dtype == np.uint8 and arena.flags.c_contiguous
    n = len(off4)
    status = np.zeros(n, dtype=np.uint8)
    if out is None:
        out = arena
    assert out.dtype == np.uint8 and out.flags.c_contiguous and out.size >= arena.size
    t = lib().ossl_esp_batch_decrypt(a, nsa, ck, cklen, ak, aklen, sl, mlen, arena.ctypes.data, out.ctypes.data,
                                     off4.ctypes.data, lens.ctypes.data, sa_idx.ctypes.data,
                                     status.ctypes.data, n, nthreads, reps)
    if t < 0:
        raise RuntimeError("ossl_esp_batch_decrypt failed")
    return t, status
