"""Host-side mirror of the opencrypto framework API for the GPU driver.

Same names, argument meaning and error behaviour as freebsd/opencrypto:
  crypto_session_params   cryptodev.h:357-384
  cryptop                 cryptodev.h:427-504 (the fields a driver reads)
  crypto_newsession       crypto.c:909   (driver selection by probesession priority)
  crypto_freesession      crypto.c:972
  crypto_getreq           crypto.c:1787
  crypto_dispatch         crypto.c:1413  (ERESTART -> queued, retried: cc_qblocked)
  crypto_done             crypto.c:1802  (CRYPTO_F_DONE, callback run inline:
                                          the driver registers CRYPTOCAP_F_SYNC)
The only registered driver is GpuCryptoDriver (libespgpu.so, cryptodev_if.m
methods).  In F-Stack the burst loop (lib/ff_dpdk_if.c main_loop) calls
crypto_flush()/crypto_poll() once per RX burst; tests call crypto_drain().
"""
import ctypes as C
import itertools

from . import _lib as L
from ._lib import (CRYPTO_F_IV_SEPARATE, CSP_MODE_AEAD, CSP_MODE_ETA, EINVAL,  # noqa: F401
                   EIO, ERESTART)

CRYPTO_F_DONE = 0x0020
EOPNOTSUPP = 95


class crypto_session_params:
    def __init__(self, csp_mode=0, csp_flags=0, csp_ivlen=0, csp_cipher_alg=0,
                 csp_cipher_klen=0, csp_cipher_key=None, csp_auth_alg=0, csp_auth_klen=0,
                 csp_auth_key=None, csp_auth_mlen=0):
        self.csp_mode = csp_mode
        self.csp_flags = csp_flags
        self.csp_ivlen = csp_ivlen
        self.csp_cipher_alg = csp_cipher_alg
        self.csp_cipher_klen = csp_cipher_klen
        self.csp_cipher_key = csp_cipher_key
        self.csp_auth_alg = csp_auth_alg
        self.csp_auth_klen = csp_auth_klen
        self.csp_auth_key = csp_auth_key
        self.csp_auth_mlen = csp_auth_mlen

    def _c(self):
        """-> (SessionParams, keepalive)"""
        ck = C.create_string_buffer(bytes(self.csp_cipher_key or b""), max(1, self.csp_cipher_klen))
        ak = C.create_string_buffer(bytes(self.csp_auth_key or b""), max(1, self.csp_auth_klen))
        p = L.SessionParams(self.csp_mode, self.csp_flags, self.csp_ivlen, self.csp_cipher_alg,
                            self.csp_cipher_klen,
                            C.cast(ck, C.c_void_p) if self.csp_cipher_key is not None else None,
                            self.csp_auth_alg, self.csp_auth_klen,
                            C.cast(ak, C.c_void_p) if self.csp_auth_key is not None else None,
                            self.csp_auth_mlen)
        return p, (ck, ak)


class crypto_session:
    def __init__(self, driver, sid, csp):
        self.driver = driver
        self.sid = sid
        self.csp = csp


class cryptop:
    """struct cryptop: the buffer is crp_buf, a bytearray (CRYPTO_BUF_CONTIG) or a
    list of bytearrays (an mbuf chain, CRYPTO_BUF_MBUF); processed in place."""

    def __init__(self, session):
        self.crp_session = session
        self.crp_olen = 0
        self.crp_etype = 0
        self.crp_flags = 0
        self.crp_op = 0
        self.crp_buf = None
        self.crp_aad = None
        self.crp_aad_start = 0
        self.crp_aad_length = 0
        self.crp_esn = b"\0\0\0\0"
        self.crp_iv_start = 0
        self.crp_payload_start = 0
        self.crp_payload_output_start = 0
        self.crp_payload_length = 0
        self.crp_digest_start = 0
        self.crp_iv = bytearray(16)
        self.crp_opaque = None
        self.crp_callback = None


def crypto_use_buf(crp, buf):
    crp.crp_buf = buf


def crypto_use_mbuf(crp, chain):
    crp.crp_buf = list(chain)


class GpuCryptoDriver:
    """The cryptodev_if.m driver methods, backed by libespgpu.so."""

    def __init__(self, device=0, max_sessions=1024, batch_records=65536,
                 batch_bytes=64 << 20, nbatches=2):
        self.lib = L.lib()
        cfg = L.Config(device, max_sessions, batch_records, batch_bytes, nbatches, 0)
        h = C.c_void_p()
        rc = self.lib.espgpu_init(C.byref(cfg), C.byref(h))
        if rc != 0:
            raise RuntimeError("espgpu_init failed (errno %d): no usable MI355X / HIP device?" % rc)
        self.ctx = h
        self._inflight = {}
        self._ids = itertools.count(1)

    def close(self):
        if self.ctx:
            self.lib.espgpu_fini(self.ctx)
            self.ctx = None

    def last_error(self):
        return self.lib.espgpu_last_error(self.ctx).decode()

    @staticmethod
    def probesession(csp):
        p, _keep = csp._c()
        return L.lib().espgpu_probesession(C.byref(p))

    def newsession(self, csp):
        p, _keep = csp._c()
        sid = C.c_int32(-1)
        rc = self.lib.espgpu_newsession(self.ctx, C.byref(p), C.byref(sid))
        return rc, sid.value

    def freesession(self, sid):
        self.lib.espgpu_freesession(self.ctx, sid)

    def process(self, crp, hint=0):
        bufs = crp.crp_buf if isinstance(crp.crp_buf, list) else [crp.crp_buf]
        segs = (L.Seg * len(bufs))()
        keep = []
        for i, b in enumerate(bufs):
            arr = (C.c_char * max(1, len(b))).from_buffer(b)
            keep.append(arr)
            segs[i] = L.Seg(C.addressof(arr), len(b))
        aad = None
        if crp.crp_aad is not None:
            aad = C.create_string_buffer(bytes(crp.crp_aad), len(crp.crp_aad))
            keep.append(aad)
        tok = next(self._ids)
        r = L.Req()
        r.session = crp.crp_session.sid
        r.crp_op = crp.crp_op
        r.crp_flags = crp.crp_flags
        r.segs = segs
        r.nsegs = len(bufs)
        r.crp_aad = C.cast(aad, C.c_void_p) if aad is not None else None
        r.crp_aad_start = crp.crp_aad_start
        r.crp_aad_length = crp.crp_aad_length
        r.crp_esn[:] = list(bytes(crp.crp_esn)[:4])
        r.crp_iv_start = crp.crp_iv_start
        r.crp_payload_start = crp.crp_payload_start
        r.crp_payload_length = crp.crp_payload_length
        r.crp_digest_start = crp.crp_digest_start
        r.crp_iv[:] = list(bytes(crp.crp_iv).ljust(16, b"\0")[:16])
        r.opaque = tok
        rc = self.lib.espgpu_process(self.ctx, C.byref(r), hint)
        if rc == 0:
            self._inflight[tok] = (crp, segs, keep)
        return rc

    def health(self):
        """0, or EIO once the GPU failed (espgpu_health)"""
        return self.lib.espgpu_health(self.ctx)

    def session_room(self):
        """Free SA-table slots (espgpu_session_room): at 0 newsession is ENOMEM"""
        return self.lib.espgpu_session_room(self.ctx)

    def flush(self):
        rc = self.lib.espgpu_flush(self.ctx)
        # EIO: the GPU failed; the held requests come back through poll()
        if rc and rc != EIO:
            raise RuntimeError("espgpu_flush: %s" % self.last_error())
        return rc

    def poll(self, max_n=4096):
        out = (L.Completion * max_n)()
        n = self.lib.espgpu_poll(self.ctx, out, max_n)
        done = []
        for i in range(n):
            crp, _segs, _keep = self._inflight.pop(out[i].opaque)
            crp.crp_etype = out[i].etype
            done.append(crp)
        return done

    def drain(self):
        rc = self.lib.espgpu_drain(self.ctx)
        if rc and rc != EIO:
            raise RuntimeError("espgpu_drain: %s" % self.last_error())
        return rc

    def set_tuning(self, key, value):
        return self.lib.espgpu_set_tuning(self.ctx, key.encode(), value)

    def register_host(self, arr):
        """Register a host buffer (numpy array / bytearray) that request
        buffers live in: its records are moved by the GPU, not gathered
        (espgpu_register_host).  Keep `arr` alive until unregister_host."""
        addr, n = _addr_len(arr)
        rc = self.lib.espgpu_register_host(self.ctx, addr, n)
        if rc:
            raise RuntimeError("espgpu_register_host: %s" % self.last_error())

    def unregister_host(self, arr):
        rc = self.lib.espgpu_unregister_host(self.ctx, _addr_len(arr)[0])
        if rc:
            raise RuntimeError("espgpu_unregister_host: %d" % rc)

    def stats(self):
        s = L.Stats()
        self.lib.espgpu_get_stats(self.ctx, C.byref(s))
        return {k: getattr(s, k) for k, _ in L.Stats._fields_}


def _addr_len(arr):
    if hasattr(arr, "ctypes"):                     # numpy
        return arr.ctypes.data, arr.nbytes
    return C.addressof((C.c_char * len(arr)).from_buffer(arr)), len(arr)


# ---------------------------------------------------------------------------
# framework functions (crypto.c), single registered driver

class CryptoFramework:
    def __init__(self, driver):
        self.driver = driver
        self._blocked = []            # ERESTART'd requests (cc_qblocked queue)

    def crypto_newsession(self, csp):
        """-> (error, crypto_session) ; EINVAL/EOPNOTSUPP like crypto.c:909-970."""
        if self.driver.probesession(csp) >= 0:
            return EOPNOTSUPP, None
        rc, sid = self.driver.newsession(csp)
        if rc:
            return rc, None
        return 0, crypto_session(self.driver, sid, csp)

    def crypto_freesession(self, ses):
        self.driver.freesession(ses.sid)

    def crypto_getreq(self, ses):
        return cryptop(ses)

    def crypto_dispatch(self, crp, hint=0):
        if self._blocked:
            self._blocked.append(crp)
            return 0
        rc = self.driver.process(crp, hint)
        if rc == ERESTART:
            self._blocked.append(crp)
            return 0
        if rc:
            # a request the engine refuses (EIO once the GPU failed) completes
            # at once, as the kernel-domain driver's gpucrypto_fail does
            crp.crp_etype = rc
            self._done([crp])
        return 0

    def _done(self, crps):
        for crp in crps:
            crp.crp_flags |= CRYPTO_F_DONE
            if crp.crp_callback is not None:
                crp.crp_callback(crp)

    def crypto_flush(self):
        self.driver.flush()

    def crypto_poll(self):
        done = self.driver.poll()
        self._done(done)
        # crypto_unblock: retry queued requests now that a slot may be free
        while self._blocked:
            crp = self._blocked[0]
            rc = self.driver.process(crp)
            if rc == ERESTART:
                break
            self._blocked.pop(0)
            if rc:
                crp.crp_etype = rc
                self._done([crp])
        return len(done)

    def crypto_drain(self):
        total = 0
        while True:
            self.driver.drain()
            total += self.crypto_poll()
            if not self._blocked:
                self.driver.drain()
                total += self.crypto_poll()
                return total
