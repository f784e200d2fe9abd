"""The kernel-domain opencrypto driver F-Stack links, checked against the
reference's golden packets and the oracle (not against itself).

The chain under test is the C code of the F-Stack build:
  integration/ff_gpucrypto.c    gpucrypto_process: struct cryptop -> espgpu_req
                                (crp_iv, crp_aad, crp_esn, payload / digest
                                offsets, mbuf chain -> segments), the errno map,
                                crypto_done through ff_gpucrypto_done
  integration/ff_gpucrypto_host.c  the host shim (overflow in F-Stack mode)
  f-stack_amd/libespgpu.so      the engine
driven over integration/kmock (crypto_newsession / crypto_dispatch /
crypto_done / crypto_unblock, crypto.c:622-659, :1413-1460, :1802-1830) by
integration/libkmockdrv.so (kmock/kmock_py.c).  The requests are the ones
esp_input / esp_output build (espgpu.esp.esp_input_crp / esp_output_crp,
xform_esp.c:364-458, :862-931), as contiguous buffers and as mbuf chains cut
inside the header, IV, payload and ICV.

* DPDK's ESP known-answer packets (tests/golden: AES-GCM-128/192/256, IPv4
  and IPv6, AES-CBC + HMAC-SHA2-256/384/512, AES-CBC without
  authentication) decrypt to their inner packets; a flipped ICV bit gives
  crp_etype 89 (FreeBSD EBADMSG) with the buffer untouched.
* Oracle-built records of every session kind the driver serves, with ESN
  (GCM: the 12-byte separate AAD in crp_aad; ETA: crp_esn), truncated GCM
  ICVs, CTR, ESP-NULL and cipher-only sessions: encrypt gives the oracle's
  record byte for byte (ciphertext and ICV); decrypt with flipped bits gives
  the oracle's statuses and plaintext.
* Mixed bursts through small staging, in F-Stack mode (the host overflow,
  no ERESTART reaches the framework) and in queue mode (ERESTART -> queued
  -> re-dispatched after crypto_unblock), and from registered (zero-copy)
  memory."""
import ctypes as C
import os
import time

import numpy as np
import pytest

import oracle as O
from helpers import EtaSA, GcmSA, build_records, golden

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KD_LIB = os.path.join(ROOT, "integration", "libkmockdrv.so")
BSD_EBADMSG, BSD_EINVAL = 89, 22          # freebsd/sys/errno.h, what crypto_done delivers


class _Fw:
    """What esp_input_crp / esp_output_crp need from the framework."""

    def crypto_getreq(self, ses):
        from espgpu.opencrypto import cryptop
        return cryptop(ses)


class KmockDriver:
    """ff_gpucrypto.c over the kmock KPI, host shim, libespgpu.so."""

    def __init__(self, batch_records=64, nbatches=2, batch_bytes=4 << 20, noqueue=True, proc_id=None):
        if not torch.cuda.is_available():
            pytest.fail("GPU test run without a visible HIP device")
        L = C.CDLL(KD_LIB)
        vp, i = C.c_void_p, C.c_int
        L.kd_open.argtypes = [i, i, i, i]
        L.kd_newsession.argtypes = [i, i, i, i, i, vp, i, i, vp, i, C.POINTER(vp)]
        L.kd_freesession.argtypes = [vp]
        L.kd_request.restype = vp
        L.kd_request.argtypes = [vp, i, i, i, C.POINTER(vp), C.POINTER(i), i, vp, i, i, vp, vp, i, i, i, i]
        L.kd_dispatch.argtypes = [vp]
        L.kd_result.argtypes = [vp]
        L.kd_free.argtypes = [vp]
        L.kd_register.argtypes = [vp, C.c_uint64]
        self.L = L
        if proc_id is not None:               # as ff_init() opens it (ff_gpucrypto_host_init_proc)
            rc = L.kd_open_proc(proc_id)
        else:
            rc = L.kd_open(batch_records, nbatches, batch_bytes, int(noqueue))
        assert rc == 0, rc
        self._keep = []

    def close(self):
        self.L.kd_close()

    def newsession(self, sa):
        csp = sa.csp()
        ck = C.create_string_buffer(bytes(csp.csp_cipher_key or b""), max(1, csp.csp_cipher_klen))
        ak = C.create_string_buffer(bytes(csp.csp_auth_key or b""), max(1, csp.csp_auth_klen))
        h = C.c_void_p()
        e = self.L.kd_newsession(csp.csp_mode, csp.csp_flags, csp.csp_ivlen, csp.csp_cipher_alg,
                                 csp.csp_cipher_klen, C.cast(ck, C.c_void_p) if csp.csp_cipher_key else None,
                                 csp.csp_auth_alg, csp.csp_auth_klen,
                                 C.cast(ak, C.c_void_p) if csp.csp_auth_key else None, csp.csp_auth_mlen,
                                 C.byref(h))
        return e, h.value

    def freesession(self, h):
        self.L.kd_freesession(h)

    def request(self, ses, crp, bufs):
        """A kernel cryptop from an esp_input_crp / esp_output_crp request
        over `bufs` (one bytearray: contiguous; a list: an mbuf chain)."""
        chain = isinstance(bufs, list)
        segs = bufs if chain else [bufs]
        arrs = [(C.c_char * len(b)).from_buffer(b) for b in segs]
        bases = (C.c_void_p * len(segs))(*[C.addressof(a) for a in arrs])
        lens = (C.c_int * len(segs))(*[len(b) for b in segs])
        aad = bytes(crp.crp_aad) if crp.crp_aad is not None else None
        esn = C.create_string_buffer(bytes(crp.crp_esn)[:4], 4)
        iv = C.create_string_buffer(bytes(crp.crp_iv).ljust(16, b"\0")[:16], 16)
        r = self.L.kd_request(ses, crp.crp_op, crp.crp_flags, int(chain), bases, lens, len(segs),
                              aad, crp.crp_aad_start, crp.crp_aad_length, esn, iv, crp.crp_iv_start,
                              crp.crp_payload_start, crp.crp_payload_length, crp.crp_digest_start)
        assert r
        self._keep.append((arrs, bases, lens))
        return r

    def dispatch(self, r):
        return self.L.kd_dispatch(r)

    def wait(self, reqs, timeout_s=60.0):
        """main_loop iterations until every request has completed -> etypes"""
        t_end = time.monotonic() + timeout_s
        while time.monotonic() < t_end:
            res = [self.L.kd_result(r) for r in reqs]
            if min(res) >= 0:
                return res
            for _ in range(64):
                self.L.kd_poll()
        raise AssertionError("requests did not complete")

    def counters(self):
        a = (C.c_int * 4)()
        self.L.kd_counters(a)
        return dict(zip(("erestarts", "queued", "blocked", "done"), list(a)))

    def engine(self):
        a = (C.c_uint64 * 5)()
        self.L.kd_engine(a)
        return dict(zip(("zerocopy", "overflow", "door", "gpu_fail", "fail_eio"), list(a)))

    def free(self, reqs):
        for r in reqs:
            self.L.kd_free(r)
        self._keep.clear()


@pytest.fixture
def kd():
    d = KmockDriver()
    yield d
    d.close()


def _chain(pkt, cuts):
    """pkt cut at the given offsets into an mbuf chain (bytearrays)."""
    cuts = sorted({c for c in cuts if 0 < c < len(pkt)})
    edges = [0] + cuts + [len(pkt)]
    return [bytearray(pkt[a:b]) for a, b in zip(edges, edges[1:])]


def _flat(bufs):
    return bytes(bufs) if not isinstance(bufs, list) else b"".join(bytes(b) for b in bufs)


def _layouts(skip, hlen, total, alen):
    """contiguous; a 3-mbuf chain (header / payload / tail); a fine chain cut
    inside the ESP header, the IV, the payload (at odd offsets) and the ICV"""
    return {
        "contig": None,
        "chain3": [skip + 5, skip + 37],
        "fine": [skip + 3, skip + hlen - 3, skip + hlen + 1, skip + hlen + 7, (skip + total) // 2 + 3,
                 total - alen - 5, total - alen // 2],
    }


def _run_one(kd, ses, crp, bufs):
    r = kd.request(ses, crp, bufs)
    assert kd.dispatch(r) == 0
    (et,) = kd.wait([r])
    kd.free([r])
    return et


# ---------------------------------------------------------------------------
# DPDK known-answer packets through the kernel-domain driver

@pytest.mark.parametrize("layout", ["contig", "chain3", "fine"])
@pytest.mark.parametrize("v", golden("esp_packets.json"), ids=lambda v: v["name"])
def test_gcm_kat_through_kernel_driver(kd, v, layout):
    from espgpu.esp import GCM, SecAssoc, esp_input_crp, esp_trailer_ok
    sa = SecAssoc(v["spi"], GCM, bytes.fromhex(v["key"]) + bytes.fromhex(v["salt"]))
    e, ses = kd.newsession(sa)
    assert e == 0
    skip = v["outer_hdr_len"]
    rec = bytes.fromhex(v["esp_record"])
    pkt = bytes([0x45]) + bytes(skip - 1) + rec
    cuts = _layouts(skip, sa.hlen, len(pkt), sa.alen)[layout]
    bufs = bytearray(pkt) if cuts is None else _chain(pkt, cuts)
    crp = esp_input_crp(_Fw(), ses, sa, bufs, skip)
    assert _run_one(kd, ses, crp, bufs) == 0
    flat = _flat(bufs)
    pt = flat[skip + 16:len(flat) - 16]
    inner = bytes.fromhex(v["inner_packet"])
    assert pt[:len(inner)] == inner and esp_trailer_ok(pt)
    assert flat[:skip + 16] == pkt[:skip + 16] and flat[-16:] == pkt[-16:]   # header, IV, ICV as they were
    # a flipped ICV bit: EBADMSG, and not a byte of the buffer changes
    bad = bytearray(pkt)
    bad[-3] ^= 0x10
    bufs = bad if cuts is None else _chain(bad, cuts)
    crp = esp_input_crp(_Fw(), ses, sa, bufs, skip)
    assert _run_one(kd, ses, crp, bufs) == BSD_EBADMSG
    assert _flat(bufs) == bytes(bad)
    kd.freesession(ses)


@pytest.mark.parametrize("layout", ["contig", "fine"])
@pytest.mark.parametrize("v", golden("eta_esp_packets.json"), ids=lambda v: v["name"])
def test_cbc_sha2_kat_through_kernel_driver(kd, v, layout):
    from espgpu import esp as E
    alg = {"cbc-hmac-sha256": E.CBC_SHA256, "cbc-hmac-sha384": E.CBC_SHA384, "cbc-hmac-sha512": E.CBC_SHA512}
    sa = E.SecAssoc(v["spi"], alg[v["mode"]], bytes.fromhex(v["cipher_key"]), bytes.fromhex(v["auth_key"]))
    assert sa.mlen == v["digest_len"]
    e, ses = kd.newsession(sa)
    assert e == 0
    skip = v["outer_hdr_len"]
    pkt = bytes(skip) + bytes.fromhex(v["esp_record"])
    cuts = _layouts(skip, sa.hlen, len(pkt), sa.alen)[layout]
    bufs = bytearray(pkt) if cuts is None else _chain(pkt, cuts)
    crp = E.esp_input_crp(_Fw(), ses, sa, bufs, skip)
    assert _run_one(kd, ses, crp, bufs) == 0
    inner = bytes.fromhex(v["inner_packet"])
    assert _flat(bufs)[skip + 24:skip + 24 + len(inner)] == inner
    bad = bytearray(pkt)
    bad[-1] ^= 0x01
    bufs = bad if cuts is None else _chain(bad, cuts)
    crp = E.esp_input_crp(_Fw(), ses, sa, bufs, skip)
    assert _run_one(kd, ses, crp, bufs) == BSD_EBADMSG
    assert _flat(bufs) == bytes(bad)
    kd.freesession(ses)


@pytest.mark.parametrize("v", golden("cipher_esp_packets.json"), ids=lambda v: v["name"])
def test_cipher_only_kat_through_kernel_driver(kd, v):
    """CSP_MODE_CIPHER (esp_init, xform_esp.c:230-231): decrypt to the inner
    packet, then encrypt the plaintext back to the reference's packet."""
    from espgpu import esp as E
    sa = E.SecAssoc(v["spi"], E.CBC, bytes.fromhex(v["cipher_key"]))
    e, ses = kd.newsession(sa)
    assert e == 0
    skip = v["outer_hdr_len"]
    rec = bytes.fromhex(v["esp_record"])
    pkt = bytearray(bytes(skip) + rec)
    assert _run_one(kd, ses, E.esp_input_crp(_Fw(), ses, sa, pkt, skip), pkt) == 0
    inner = bytes.fromhex(v["inner_packet"])
    assert bytes(pkt[skip + 24:skip + 24 + len(inner)]) == inner
    chain = _chain(bytes(pkt), [skip + 9, skip + 30, len(pkt) - 7])
    assert _run_one(kd, ses, E.esp_output_crp(_Fw(), ses, sa, chain, skip), chain) == 0
    assert _flat(chain)[skip:] == rec
    kd.freesession(ses)


# ---------------------------------------------------------------------------
# oracle-built records of every session kind

def _kinds(rng):
    return {
        "gcm128": GcmSA(rng, 16),
        "gcm256-esn": GcmSA(rng, 32, esn=True),
        "gcm192-icv12": GcmSA(rng, 24, mlen=12),
        "gcm128-esn-icv8": GcmSA(rng, 16, esn=True, mlen=8),
        "cbc256-sha1-esn": EtaSA(rng, 32, esn=True),
        "ctr128-sha256": EtaSA(rng, 16, ctr=True, sha256=True),
        "cbc192-sha384-esn": EtaSA(rng, 24, sha=384, esn=True),
        "ctr256-sha512": EtaSA(rng, 32, ctr=True, sha=512),
        "null-sha256-esn": EtaSA(rng, 0, null=True, sha=256, esn=True),
        "cbc128-cipher": EtaSA(rng, 16, noauth=True),
        "ctr256-cipher": EtaSA(rng, 32, ctr=True, noauth=True),
    }


KINDS = list(_kinds(np.random.default_rng(0)))


def _records(kind, n=24, seed=0):
    rng = np.random.default_rng(4100 + seed + KINDS.index(kind))
    sa = _kinds(rng)[kind]
    blk = 16 if (isinstance(sa, EtaSA) and not sa.ctr and not sa.null) else 4
    cts = rng.integers(1, 400, n) * blk
    cts[:3] = [blk, 1440 - 1440 % blk, 8944 - 8944 % blk]
    esn_hi = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) if sa.esn else None
    plain, ct, descs, eh = build_records(rng, [sa], np.zeros(n, dtype=np.int64), cts, esn_hi=esn_hi)
    return rng, sa, plain, ct, descs, eh


def _pkt(arena, descs, i, skip=20):
    o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
    return bytes([0x45]) + bytes(skip - 1) + arena[o:o + L].tobytes()


@pytest.mark.parametrize("kind", KINDS)
def test_encrypt_through_kernel_driver_vs_oracle(kd, kind):
    """esp_output's cryptop over the plaintext record (contiguous and mbuf
    chains): the buffer ends up as the oracle's record, ciphertext and ICV."""
    from espgpu.esp import esp_output_crp
    rng, sa, plain, ct, descs, eh = _records(kind)
    esa = sa.esp_sa()
    e, ses = kd.newsession(esa)
    assert e == 0
    reqs, bufs_all = [], []
    for i in range(len(descs)):
        pkt = _pkt(plain, descs, i)
        L = len(pkt)
        bufs = bytearray(pkt) if i % 2 == 0 else _chain(pkt, sorted(rng.integers(21, L, 5)))
        crp = esp_output_crp(_Fw(), ses, esa, bufs, 20, esn_hi=int(eh[i]))
        r = kd.request(ses, crp, bufs)
        assert kd.dispatch(r) == 0
        reqs.append(r)
        bufs_all.append(bufs)
    ets = kd.wait(reqs)
    kd.free(reqs)
    for i, (et, bufs) in enumerate(zip(ets, bufs_all)):
        assert et == 0, (i, et)
        assert _flat(bufs) == _pkt(ct, descs, i), i
    kd.freesession(ses)


@pytest.mark.parametrize("kind", KINDS)
def test_decrypt_through_kernel_driver_vs_oracle(kd, kind):
    """esp_input's cryptop over the oracle's ciphertext, 1 in 3 records with a
    flipped bit anywhere past the outer header: statuses (EBADMSG 89) and
    plaintext as the oracle's, failed records untouched."""
    from espgpu.esp import esp_input_crp
    rng, sa, plain, ct, descs, eh = _records(kind, seed=1)
    n = len(descs)
    bad = ct.copy()
    for i in range(0, n, 3):
        o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
        bad[o + 8 + int(rng.integers(0, L - 8))] ^= 1 << int(rng.integers(0, 8))
    ref = bad.copy()
    _, ref_st = O.batch([sa.oracle], ref, descs["off4"], descs["len"], descs["sa"], esn_hi=eh)
    esa = sa.esp_sa()
    e, ses = kd.newsession(esa)
    assert e == 0
    reqs, bufs_all = [], []
    for i in range(n):
        pkt = _pkt(bad, descs, i)
        bufs = bytearray(pkt) if i % 2 else _chain(pkt, sorted(rng.integers(21, len(pkt), 6)))
        crp = esp_input_crp(_Fw(), ses, esa, bufs, 20, esn_hi=int(eh[i]))
        r = kd.request(ses, crp, bufs)
        assert kd.dispatch(r) == 0
        reqs.append(r)
        bufs_all.append(bufs)
    ets = kd.wait(reqs)
    kd.free(reqs)
    want = {0: 0, O.EBADMSG: BSD_EBADMSG, O.EINVAL: BSD_EINVAL}
    for i, (et, bufs) in enumerate(zip(ets, bufs_all)):
        assert et == want[int(ref_st[i])], (i, et, ref_st[i])
        got = _flat(bufs)[20:]
        o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
        if et == 0:
            h, a = sa.hlen, sa.mlen
            assert got[h:L - a] == ref[o + h:o + L - a].tobytes(), i
            assert got[:h] == bad[o:o + h].tobytes() and got[L - a:] == bad[o + L - a:o + L].tobytes()
        else:
            assert got == bad[o:o + L].tobytes(), i
    if sa.mlen:
        assert (ref_st != 0).sum() >= n // 3 - 1      # the flips were seen
    kd.freesession(ses)


# ---------------------------------------------------------------------------
# bursts: staging full, overflow or ERESTART, registered memory

@pytest.mark.parametrize("noqueue", [True, False], ids=["fstack-overflow", "erestart-queue"])
def test_mixed_burst_small_staging_vs_oracle(noqueue):
    """240 decrypts over four sessions (GCM, GCM ESN, CBC-SHA1, CTR-SHA256)
    through two 8-record staging slots.  F-Stack mode: the overflow takes
    what finds both slots in flight, no ERESTART reaches the framework.
    Queue mode: process() answers ERESTART, crypto_dispatch queues the
    request (cc_qblocked) and re-dispatches after crypto_unblock.  Either
    way every record's status and plaintext equal the oracle's."""
    from espgpu.esp import esp_input_crp
    kd = KmockDriver(batch_records=8, nbatches=2, noqueue=noqueue)
    try:
        rng = np.random.default_rng(4300 + noqueue)
        sas = [GcmSA(rng, 16), GcmSA(rng, 16, esn=True), EtaSA(rng, 32), EtaSA(rng, 16, ctr=True, sha256=True)]
        n = 240
        idx = rng.integers(0, len(sas), n)
        cts = np.array([int(rng.integers(1, 95)) * 16 for _ in range(n)])
        eh = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        plain, ct, descs, eh = build_records(rng, sas, idx, cts, esn_hi=eh)
        bad = ct.copy()
        for i in range(0, n, 7):
            o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
            bad[o + L - 1] ^= 0x80
        ref = bad.copy()
        _, ref_st = O.batch([s.oracle for s in sas], ref, descs["off4"], descs["len"], descs["sa"], esn_hi=eh)
        ses = []
        for s in sas:
            e, h = kd.newsession(s.esp_sa())
            assert e == 0
            ses.append(h)
        c0 = kd.counters()
        reqs, bufs_all = [], []
        for i in range(n):
            pkt = _pkt(bad, descs, i)
            bufs = _chain(pkt, [20 + 4, len(pkt) // 2])
            esa = sas[idx[i]].esp_sa()
            crp = esp_input_crp(_Fw(), ses[idx[i]], esa, bufs, 20,
                                esn_hi=int(eh[i]) if sas[idx[i]].esn else 0)
            r = kd.request(ses[idx[i]], crp, bufs)
            assert kd.dispatch(r) == 0
            reqs.append(r)
            bufs_all.append(bufs)
        ets = kd.wait(reqs)
        kd.free(reqs)
        c1 = kd.counters()
        if noqueue:
            assert c1["erestarts"] == c0["erestarts"] and kd.engine()["overflow"] > 0
        else:
            assert c1["erestarts"] > c0["erestarts"]
        assert c1["queued"] == 0 and c1["blocked"] == 0
        for i in range(n):
            assert ets[i] == (BSD_EBADMSG if ref_st[i] == O.EBADMSG else 0), (i, ets[i], ref_st[i])
            o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
            got = _flat(bufs_all[i])[20:]
            if ets[i] == 0:
                h, a = sas[idx[i]].hlen, sas[idx[i]].mlen
                assert got[h:L - a] == ref[o + h:o + L - a].tobytes(), i
            else:
                assert got == bad[o:o + L].tobytes(), i
        for h in ses:
            kd.freesession(h)
    finally:
        kd.close()


def test_registered_memory_through_kernel_driver_vs_oracle(kd):
    """The packets lie in one registered region (the mbuf pools,
    espgpu_register_host): every record is moved by the GPU (zero-copy count =
    all), GCM and CBC-SHA1 sessions, encrypt then tampered decrypt, bytes
    equal the oracle's."""
    from espgpu.esp import esp_input_crp, esp_output_crp
    rng = np.random.default_rng(4400)
    sas = [GcmSA(rng, 16), EtaSA(rng, 32)]
    n, slot = 64, 2048
    idx = rng.integers(0, 2, n)
    cts = rng.integers(1, 90, n) * 16
    plain, ct, descs, eh = build_records(rng, sas, idx, cts)
    region = np.zeros(n * slot, dtype=np.uint8)
    mv = memoryview(region)
    ses = []
    for s in sas:
        e, h = kd.newsession(s.esp_sa())
        assert e == 0
        ses.append(h)
    assert kd.L.kd_register(region.ctypes.data, region.nbytes) == 0

    def views():      # each packet at an mbuf's data offset (headroom 128 + 14 + 20: 2 mod 4)
        return [mv[i * slot + 162:i * slot + 182 + int(descs["len"][i])] for i in range(n)]

    for i in range(n):
        region[i * slot + 162:i * slot + 162 + 20 + int(descs["len"][i])] = np.frombuffer(_pkt(plain, descs, i), np.uint8)
    z0 = kd.engine()["zerocopy"]
    reqs = []
    for i, v in enumerate(views()):
        r = _req_view(kd, esp_output_crp, ses[idx[i]], sas[idx[i]].esp_sa(), v)
        reqs.append(r)
    assert kd.wait(reqs) == [0] * n
    kd.free(reqs)
    for i in range(n):
        L = int(descs["len"][i])
        assert region[i * slot + 182:i * slot + 182 + L].tobytes() == _pkt(ct, descs, i)[20:], i
    flip = rng.random(n) < 0.25
    for i in np.flatnonzero(flip):
        region[i * slot + 182 + int(descs["len"][i]) - 1] ^= 0x02
    before = region.copy()
    reqs = [_req_view(kd, esp_input_crp, ses[idx[i]], sas[idx[i]].esp_sa(), v) for i, v in enumerate(views())]
    ets = kd.wait(reqs)
    kd.free(reqs)
    assert kd.engine()["zerocopy"] - z0 == 2 * n
    for i in range(n):
        L, h, a = int(descs["len"][i]), sas[idx[i]].hlen, sas[idx[i]].mlen
        base = i * slot + 182
        o = int(descs["off4"][i]) * 4
        if flip[i]:
            assert ets[i] == BSD_EBADMSG
            assert (region[base:base + L] == before[base:base + L]).all()
        else:
            assert ets[i] == 0
            assert region[base + h:base + L - a].tobytes() == plain[o + h:o + L - a].tobytes(), i
    for h in ses:
        kd.freesession(h)


def test_doorbell_through_kernel_driver_vs_oracle(monkeypatch):
    """F-Stack's init path with FF_GPUCRYPTO_DOOR set
    (ff_gpucrypto_host_init_proc): 32-packet GCM bursts from registered mbuf
    memory go to the resident doorbell kernel (door count), encrypt equals the
    oracle's ciphertext, a tampered decrypt the oracle's statuses and
    plaintext, failed packets untouched."""
    from espgpu.esp import esp_input_crp, esp_output_crp
    monkeypatch.setenv("FF_GPUCRYPTO_DOOR", "16")
    kd = KmockDriver(proc_id=0)
    try:
        rng = np.random.default_rng(4500)
        sa = GcmSA(rng, 16)
        n, slot = 32, 2048
        idx = np.zeros(n, dtype=np.int64)
        cts = rng.integers(1, 90, n) * 16
        plain, ct, descs, eh = build_records(rng, [sa], idx, cts)
        region = np.zeros(n * slot, dtype=np.uint8)
        mv = memoryview(region)
        e, ses = kd.newsession(sa.esp_sa())
        assert e == 0
        assert kd.L.kd_register(region.ctypes.data, region.nbytes) == 0
        views = [mv[i * slot + 162:i * slot + 182 + int(descs["len"][i])] for i in range(n)]
        for i in range(n):
            region[i * slot + 162:i * slot + 182 + int(descs["len"][i])] = np.frombuffer(_pkt(plain, descs, i), np.uint8)
        d0 = kd.engine()["door"]
        reqs = [_req_view(kd, esp_output_crp, ses, sa.esp_sa(), v) for v in views]
        assert kd.wait(reqs) == [0] * n
        kd.free(reqs)
        for i in range(n):
            L = int(descs["len"][i])
            assert region[i * slot + 182:i * slot + 182 + L].tobytes() == _pkt(ct, descs, i)[20:], i
        flip = rng.random(n) < 0.25
        for i in np.flatnonzero(flip):
            region[i * slot + 182 + int(descs["len"][i]) - 1] ^= 0x02
        before = region.copy()
        reqs = [_req_view(kd, esp_input_crp, ses, sa.esp_sa(), v) for v in views]
        ets = kd.wait(reqs)
        kd.free(reqs)
        assert kd.engine()["door"] > d0
        for i in range(n):
            L, h, a = int(descs["len"][i]), sa.hlen, sa.mlen
            base = i * slot + 182
            o = int(descs["off4"][i]) * 4
            if flip[i]:
                assert ets[i] == BSD_EBADMSG
                assert (region[base:base + L] == before[base:base + L]).all()
            else:
                assert ets[i] == 0
                assert region[base + h:base + L - a].tobytes() == plain[o + h:o + L - a].tobytes(), i
        kd.freesession(ses)
    finally:
        kd.close()


def _req_view(kd, build, ses, esa, view):
    """A request over a memoryview into the registered region (one mbuf)."""
    arr = (C.c_char * len(view)).from_buffer(view)
    bases = (C.c_void_p * 1)(C.addressof(arr))
    lens = (C.c_int * 1)(len(view))
    crp = build(_Fw(), ses, esa, bytearray(bytes(view)), 20)
    aad = bytes(crp.crp_aad) if crp.crp_aad is not None else None
    esn = C.create_string_buffer(bytes(crp.crp_esn)[:4], 4)
    iv = C.create_string_buffer(bytes(crp.crp_iv).ljust(16, b"\0")[:16], 16)
    r = kd.L.kd_request(ses, crp.crp_op, crp.crp_flags, 1, bases, lens, 1, aad, crp.crp_aad_start,
                        crp.crp_aad_length, esn, iv, crp.crp_iv_start, crp.crp_payload_start,
                        crp.crp_payload_length, crp.crp_digest_start)
    assert r
    kd._keep.append((arr, bases, lens))
    assert kd.dispatch(r) == 0
    return r


# ---------------------------------------------------------------------------
# GPU failure: every cryptop completes exactly once

KMOCK_SOFT_ID, BSD_EIO, BSD_EAGAIN = 8, 5, 35
def test_full_sa_table_sends_the_next_session_to_software(kd):
    """kd_open's engine holds 64 SAs (espgpu_config.max_sessions).  The 65th
    session is declined at probe (espgpu_session_room == 0): ENOMEM with no
    software driver, and with one crypto_newsession selects it -- the SA is
    never failed in CRYPTODEV_NEWSESSION (crypto.c:954-958).  A freed GPU
    session's slot takes the next SA, whose requests decrypt as the oracle."""
    from espgpu.esp import esp_input_crp
    L = kd.L
    L.kd_soft.argtypes = [C.c_void_p]
    soft = (C.c_int * 4)()
    rng = np.random.default_rng(6464)
    hs = []
    for _ in range(64):
        e, h = kd.newsession(GcmSA(rng, 16).esp_sa())
        assert e == 0
        hs.append(h)
    L.kd_soft(soft)
    assert soft[0] == 0 and soft[2] == 64
    sa = GcmSA(rng, 16)
    esa = sa.esp_sa()
    e, h = kd.newsession(esa)
    assert e == 12 and not h                             # ENOMEM: the probe declined
    L.kd_soft_enable(1)
    e, hsw = kd.newsession(esa)
    assert e == 0
    L.kd_soft(soft)
    assert soft[0] == 1 and soft[2] == 65                # on the software driver
    kd.freesession(hs.pop(5))
    e, ses = kd.newsession(esa)
    assert e == 0
    L.kd_soft(soft)
    assert soft[0] == 1                                  # the freed GPU slot, not software
    n = 24
    plain, ct, descs, _ = build_records(rng, [sa], np.zeros(n, dtype=np.int64), rng.integers(1, 92, n) * 16)
    ref = ct.copy()
    _, ref_st = O.batch([sa.oracle], ref, descs["off4"], descs["len"], descs["sa"])
    reqs, bufs_all = [], []
    for i in range(n):
        bufs = bytearray(_pkt(ct, descs, i))
        r = kd.request(ses, esp_input_crp(_Fw(), ses, esa, bufs, 20), bufs)
        assert kd.dispatch(r) == 0
        reqs.append(r)
        bufs_all.append(bufs)
    assert kd.wait(reqs) == [0] * n
    kd.free(reqs)
    for i, bufs in enumerate(bufs_all):
        o, Ln = int(descs["off4"][i]) * 4, int(descs["len"][i])
        assert ref_st[i] == 0 and bytes(bufs[20 + 16:20 + Ln - 16]) == ref[o + 16:o + Ln - 16].tobytes(), i
    for h in hs + [hsw, ses]:
        kd.freesession(h)
    L.kd_soft(soft)
    assert soft[0] == 0 and soft[2] == 0


FAULT_LAUNCH, FAULT_QUERY, FAULT_STUCK = 1, 2, 4     # set_tuning "fault" (include/espgpu.h)


@pytest.mark.parametrize("fault,door", [(FAULT_LAUNCH, 0), (FAULT_QUERY, 0), (FAULT_STUCK, 0),
                                        (FAULT_LAUNCH, 16), (FAULT_STUCK, 16)],
                         ids=["launch", "query", "stuck", "launch-door", "stuck-door"])
def test_gpu_failure_completes_every_request_once(fault, door):
    """F-Stack mode (two 16-record slots and the host overflow), optionally on
    the doorbell path.  After 16 requests complete normally, a fault is
    injected (set_tuning "fault": the next launch fails / the next completion
    query returns an error / the next batch is never seen to complete, which
    meets deadline_ms) and 80 more requests are dispatched.  Main-loop
    iterations then complete every one of them exactly once -- crypto_done
    called once per cryptop, with no hang -- either with the oracle's
    plaintext (its batch completed) or with EIO and the buffer untouched (a
    clean drop, esp_input_cb's esps_noxform); the engine counts one failure
    and as many EIO completions.  Afterwards the next request of the session
    completes with EAGAIN and a session on the software driver, and its
    re-dispatch (esp_input_cb's EAGAIN path) completes there; a new session
    goes to the software driver (the probe declines)."""
    from espgpu.esp import esp_input_crp
    kd = KmockDriver(batch_records=16, nbatches=2, noqueue=True)
    L = kd.L
    L.kd_tune.argtypes = [C.c_char_p, C.c_int]
    for f in ("kd_done_count", "kd_session_hid", "kd_redispatch", "kd_freesession_of"):
        getattr(L, f).argtypes = [C.c_void_p]
    try:
        if door:
            assert L.kd_tune(b"door", door) == 0
        rng = np.random.default_rng(4700 + fault + door)
        sa = GcmSA(rng, 16)
        n = 96
        cts = rng.integers(1, 92, n) * 16
        plain, ct, descs, eh = build_records(rng, [sa], np.zeros(n, dtype=np.int64), cts)
        ref = ct.copy()
        _, ref_st = O.batch([sa.oracle], ref, descs["off4"], descs["len"], descs["sa"])
        assert (ref_st == 0).all()
        esa = sa.esp_sa()
        e, ses = kd.newsession(esa)
        assert e == 0

        def mk(i):
            bufs = bytearray(_pkt(ct, descs, i))
            return kd.request(ses, esp_input_crp(_Fw(), ses, esa, bufs, 20), bufs), bufs

        def check_pt(i, bufs):
            o, Ln = int(descs["off4"][i]) * 4, int(descs["len"][i])
            assert bytes(bufs[20 + 16:20 + Ln - 16]) == ref[o + 16:o + Ln - 16].tobytes(), i

        warm = [mk(i) for i in range(16)]
        for r, _ in warm:
            assert kd.dispatch(r) == 0
        assert kd.wait([r for r, _ in warm]) == [0] * 16
        for i, (_, b) in enumerate(warm):
            check_pt(i, b)
        assert L.kd_failed() == 0
        if fault == FAULT_STUCK:
            assert L.kd_tune(b"deadline_ms", 200) == 0
        assert L.kd_tune(b"fault", fault) == 0
        reqs = [mk(i) for i in range(16, n)]
        for r, _ in reqs:
            assert kd.dispatch(r) == 0
        t0 = time.monotonic()
        ets = kd.wait([r for r, _ in reqs], timeout_s=30.0)
        assert time.monotonic() - t0 < 10.0
        assert L.kd_failed() == 1
        for _ in range(64):                              # more main-loop iterations deliver nothing twice
            L.kd_poll()
        assert [L.kd_done_count(r) for r, _ in reqs] == [1] * len(reqs)
        n_eio = 0
        for k, (et, (r, bufs)) in enumerate(zip(ets, reqs)):
            i = 16 + k
            if et == 0:
                check_pt(i, bufs)
            else:
                assert et == BSD_EIO, (i, et)
                assert bytes(bufs) == _pkt(ct, descs, i), i          # untouched
                n_eio += 1
        assert n_eio >= 48 if fault != FAULT_LAUNCH else n_eio == len(reqs)
        eng = kd.engine()
        # the engine counts what it dropped or refused; after the failure the
        # driver stops calling it (launch: the 16 staged + the one whose
        # staging launched them; the other 63 failed in the driver)
        assert eng["gpu_fail"] == 1 and eng["fail_eio"] == (17 if fault == FAULT_LAUNCH else n_eio), eng
        kd.free([r for r, _ in warm + reqs])
        # after the failure: the session moves to the software driver
        L.kd_soft_enable(1)
        r, bufs = mk(0)
        assert kd.dispatch(r) == 0
        assert L.kd_done_count(r) == 1 and L.kd_result(r) == BSD_EAGAIN
        assert L.kd_session_hid(r) == KMOCK_SOFT_ID
        assert L.kd_redispatch(r) == 0
        assert L.kd_done_count(r) == 2 and L.kd_result(r) == 0
        soft = (C.c_int * 4)()
        L.kd_soft(soft)
        assert soft[0] == 1 and soft[1] == 1
        L.kd_freesession_of(r)
        kd.free([r])
        e2, ses2 = kd.newsession(esa)                    # the probe declines: software
        assert e2 == 0
        L.kd_soft(soft)
        assert soft[0] == 1
        kd.freesession(ses2)
        kd.freesession(ses)
        L.kd_soft(soft)
        assert soft[0] == 0 and soft[2] == 0             # every session freed
    finally:
        kd.close()                                       # bounded: the failed ctx waits on nothing
