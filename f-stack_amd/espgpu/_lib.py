"""ctypes binding of libespgpu.so (include/espgpu.h).

The product path: every call here goes to the HIP engine.  There is no CPU
fallback; if the library is missing or no GPU is present the calls fail loudly.
"""
import ctypes as C
import os
import re

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))   # f-stack_amd/
LIB_PATH = os.environ.get("ESPGPU_LIB", os.path.join(PKG_ROOT, "libespgpu.so"))
HEADER = os.path.join(os.path.dirname(PKG_ROOT), "include", "espgpu.h")

# constants (cryptodev.h values, see include/espgpu.h)
CSP_MODE_CIPHER = 2
CSP_MODE_AEAD = 4
CSP_MODE_ETA = 5
CSP_F_SEPARATE_AAD = 0x2
CSP_F_ESN = 0x4
CRYPTO_SHA1_HMAC = 7
CRYPTO_AES_CBC = 11
CRYPTO_NULL_CBC = 16
CRYPTO_SHA2_256_HMAC = 18
CRYPTO_SHA2_384_HMAC = 19
CRYPTO_SHA2_512_HMAC = 20
CRYPTO_AES_ICM = 23
CRYPTO_AES_NIST_GCM_16 = 25
CRYPTO_OP_DECRYPT = 0x0
CRYPTO_OP_ENCRYPT = 0x1
CRYPTO_OP_VERIFY_DIGEST = 0x2
CRYPTO_OP_COMPUTE_DIGEST = 0x0
CRYPTO_F_CBIFSYNC = 0x0040
CRYPTO_F_IV_SEPARATE = 0x0200
CRYPTO_HINT_MORE = 0x1
CRYPTODEV_PROBE_HARDWARE = -100
BATCH_GROUPED = 0x1
TR_BADLEN = 0x00010000
TR_BADPAD = 0x00020000
TR_NONE = 0x00040000
TR_VALID = 0x80000000
EIO = 5
EINVAL = 22
EBADMSG = 74
ERESTART = 85
FAULT_LAUNCH, FAULT_QUERY, FAULT_STUCK = 0x1, 0x2, 0x4   # set_tuning "fault" (espgpu.h)


class SessionParams(C.Structure):
    _fields_ = [("csp_mode", C.c_int), ("csp_flags", C.c_int), ("csp_ivlen", C.c_int),
                ("csp_cipher_alg", C.c_int), ("csp_cipher_klen", C.c_int),
                ("csp_cipher_key", C.c_void_p), ("csp_auth_alg", C.c_int),
                ("csp_auth_klen", C.c_int), ("csp_auth_key", C.c_void_p),
                ("csp_auth_mlen", C.c_int)]


class Seg(C.Structure):
    _fields_ = [("base", C.c_void_p), ("len", C.c_uint32)]


class Req(C.Structure):
    _fields_ = [("session", C.c_int32), ("crp_op", C.c_int), ("crp_flags", C.c_int),
                ("segs", C.POINTER(Seg)), ("nsegs", C.c_int), ("crp_aad", C.c_void_p),
                ("crp_aad_start", C.c_int), ("crp_aad_length", C.c_int),
                ("crp_esn", C.c_uint8 * 4), ("crp_iv_start", C.c_int),
                ("crp_payload_start", C.c_int), ("crp_payload_length", C.c_int),
                ("crp_digest_start", C.c_int), ("crp_iv", C.c_uint8 * 16),
                ("opaque", C.c_void_p)]


class Completion(C.Structure):
    _fields_ = [("opaque", C.c_void_p), ("etype", C.c_int)]


class Desc(C.Structure):
    _fields_ = [("off4", C.c_uint32), ("len", C.c_uint16), ("sa", C.c_uint16),
                ("esn_hi", C.c_uint32), ("salt", C.c_uint32)]


class Replay(C.Structure):
    """struct espgpu_replay: one SA's replay window (secreplay, keydb.h:206-213)."""
    _fields_ = [("last", C.c_uint64), ("wsize", C.c_uint32), ("bitmap_size", C.c_uint32),
                ("bitmap_off", C.c_uint32), ("flags", C.c_uint32)]


REPLAY_ESN, REPLAY_CYCSEQ, EACCES = 0x1, 0x2, 13


class Config(C.Structure):
    _fields_ = [("device", C.c_int), ("max_sessions", C.c_uint32),
                ("batch_records", C.c_uint32), ("batch_bytes", C.c_uint32),
                ("nbatches", C.c_uint32), ("grid", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("records", C.c_uint64), ("bytes", C.c_uint64), ("auth_fail", C.c_uint64),
                ("einval", C.c_uint64), ("batches", C.c_uint64), ("kernel_ns", C.c_uint64),
                ("erestart", C.c_uint64), ("overflow", C.c_uint64), ("zerocopy", C.c_uint64),
                ("door", C.c_uint64), ("ovf_reserved", C.c_uint64), ("ovf_peak", C.c_uint64),
                ("ovf_process_ns_max", C.c_uint64), ("gpu_fail", C.c_uint64), ("fail_eio", C.c_uint64)]


_lib = None


def lib():
    """Load libespgpu.so; raises if it has not been built (no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("libespgpu.so not found at %s: build it with "
                               "`make -C f-stack_amd` (hipcc, gfx950)" % LIB_PATH)
        # One HIP runtime per process: torch bundles its own libamdhip64 (same
        # soname, libamdhip64.so.7).  Loaded first, it satisfies our DT_NEEDED;
        # loaded after us it would come in as a second runtime that sees no
        # devices.  So bring torch in first when it is installed.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        vp = C.c_void_p
        L.espgpu_abi_version.restype = C.c_int
        L.espgpu_device_count.restype = C.c_int
        L.espgpu_init.argtypes = [C.POINTER(Config), C.POINTER(vp)]
        L.espgpu_fini.argtypes = [vp]
        L.espgpu_fini.restype = None
        L.espgpu_last_error.argtypes = [vp]
        L.espgpu_last_error.restype = C.c_char_p
        L.espgpu_health.argtypes = [vp]
        L.espgpu_probesession.argtypes = [C.POINTER(SessionParams)]
        L.espgpu_newsession.argtypes = [vp, C.POINTER(SessionParams), C.POINTER(C.c_int32)]
        L.espgpu_freesession.argtypes = [vp, C.c_int32]
        L.espgpu_freesession.restype = None
        L.espgpu_session_room.argtypes = [vp]
        L.espgpu_session_room.restype = C.c_int
        L.espgpu_process.argtypes = [vp, C.POINTER(Req), C.c_int]
        L.espgpu_flush.argtypes = [vp]
        L.espgpu_poll.argtypes = [vp, C.POINTER(Completion), C.c_int]
        L.espgpu_drain.argtypes = [vp]
        L.espgpu_get_stats.argtypes = [vp, C.POINTER(Stats)]
        L.espgpu_register_host.argtypes = [vp, vp, C.c_uint64]
        L.espgpu_unregister_host.argtypes = [vp, vp]
        L.espgpu_decrypt_batch.argtypes = [vp, vp, vp, C.c_uint32, vp, vp, C.c_uint32, vp]
        L.espgpu_encrypt_batch.argtypes = [vp, vp, vp, C.c_uint32, vp, C.c_uint32, vp]
        L.espgpu_decrypt_batch_trailer.argtypes = [vp, vp, vp, C.c_uint32, vp, vp, vp, C.c_uint32, vp]
        if hasattr(L, "espgpu_decrypt_batch_packed"):   # (absent from older builds used in A/B runs)
            L.espgpu_decrypt_batch_packed.argtypes = [vp, vp, vp, C.c_uint32, vp, vp, C.c_uint32, C.c_uint32, vp]
        L.espgpu_replay_check_batch.argtypes = [vp, vp, vp, C.c_uint32, vp, C.c_uint32, vp, vp, vp]
        L.espgpu_replay_merge.argtypes = [vp, vp, vp, C.c_uint32, vp]
        L.espgpu_replay_update.argtypes = [C.POINTER(Replay), C.POINTER(C.c_uint32), C.c_uint32]
        L.espgpu_replay_params_ok.argtypes = [C.POINTER(Replay)]
        L.espgpu_last_kernel_ms.argtypes = [vp]
        L.espgpu_last_kernel_ms.restype = C.c_float
        L.espgpu_set_tuning.argtypes = [vp, C.c_char_p, C.c_int]
        L.espgpu_decrypt_host.argtypes = [vp, vp, C.c_uint64, vp, C.c_uint32, vp, vp, C.c_uint32,
                                          C.c_uint32]
        _lib = L
    return _lib


def header_symbols(path=HEADER):
    """Function names declared in include/espgpu.h."""
    src = open(path).read()
    return sorted(set(re.findall(r"\b(espgpu_[a-z_0-9]+)\s*\(", src)))
