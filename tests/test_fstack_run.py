"""F-Stack's own opencrypto framework running the MI355X driver.

integration/fstack_run.py builds F-Stack's kernel domain (lib/Makefile's own
rules, FF_IPSEC=1 FF_IPSEC_GPU=1) into an executable that boots it with
ff_freebsd_init() and pushes ESP requests through the reference's
crypto.c (integration/fstack_run/host_main.c):
  * ff_newbus.c's driver_module_handler -> crypto_modevent -> crypto_init
    (crypto.c:320, :2265); cryptosoft and gpucrypto attach;
  * crypto_newsession with esp_init's crid (HARDWARE|SOFTWARE,
    xform_esp.c:242) must select gpucrypto (probesession -100 beats
    cryptosoft's -500, crypto_select_driver crypto.c:622-659); a transform
    the engine does not serve (AH's HMAC digest, CSP_MODE_DIGEST) stays on
    cryptosoft;
  * crypto_dispatch (crypto.c:1413) of every request, as a real FreeBSD mbuf
    chain or a contiguous buffer; the callback runs inline from crypto_done
    (CBIFSYNC + CRYPTOCAP_F_SYNC, crypto.c:1802-1826) during F-Stack's
    main_loop poll (ff_gpucrypto_poll);
  * the same requests on a cryptosoft-only session (crid SOFTWARE): the
    reference's software path itself runs beside the driver, and every
    result (crp_etype and the whole buffer) must be identical, and equal to
    the DPDK known answers and the oracle.
The CPU executable (fstack_crypto_run_cpu) has the oracle stand-in
(integration/fstack_run/oracle_engine.c) behind the host shim's interface;
the GPU one (fstack_crypto_run_gpu) the real shim and libespgpu.so.  Both
are built here, where /root/reference exists, and travel to the GPU box.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle as O
from helpers import EtaSA, GcmSA, build_records, golden

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "integration"))
import fstack_run as FR  # noqa: E402

BSD_EBADMSG = 89
CSP_MODE_DIGEST = 3


class _Fw:
    def crypto_getreq(self, ses):
        from espgpu.opencrypto import cryptop
        c = cryptop(ses)
        return c


def _sess(csp):
    return dict(mode=csp.csp_mode, flags=csp.csp_flags, ivlen=csp.csp_ivlen, calg=csp.csp_cipher_alg,
                cklen=csp.csp_cipher_klen, aalg=csp.csp_auth_alg, aklen=csp.csp_auth_klen,
                mlen=csp.csp_auth_mlen, ckey=csp.csp_cipher_key, akey=csp.csp_auth_key)


def _req(si, crp, pkt, cuts):
    return dict(ses=si, op=crp.crp_op, flags=crp.crp_flags, aad_start=crp.crp_aad_start,
                aad_len=crp.crp_aad_length, iv_start=crp.crp_iv_start, payload_start=crp.crp_payload_start,
                payload_len=crp.crp_payload_length, digest_start=crp.crp_digest_start,
                aad=bytes(crp.crp_aad) if crp.crp_aad is not None else None, esn=bytes(crp.crp_esn),
                iv=bytes(crp.crp_iv), mbuf=cuts is not None, cuts=cuts or [], buf=bytes(pkt))


def _cuts(rng, n, k):
    """k cut points, every mbuf at most MCLBYTES (2048) long"""
    c = set(int(x) for x in rng.integers(1, n, k))
    c |= set(range(2000, n, 2000))
    return sorted(c)[:16]


def _workload():
    """sessions, requests and what each request must produce"""
    from espgpu import esp as E
    sessions, reqs, want = [], [], []
    rng = np.random.default_rng(5100)

    def add_session(csp):
        sessions.append(_sess(csp))
        return len(sessions) - 1

    # DPDK known-answer packets, contiguous and as mbuf chains, plus a tampered copy
    for v in golden("esp_packets.json"):
        sa = E.SecAssoc(v["spi"], E.GCM, bytes.fromhex(v["key"]) + bytes.fromhex(v["salt"]))
        si = add_session(sa.csp())
        skip = v["outer_hdr_len"]
        pkt = bytes([0x45]) + bytes(skip - 1) + bytes.fromhex(v["esp_record"])
        inner = bytes.fromhex(v["inner_packet"])
        for cuts in (None, [skip + 5, skip + 37], [skip + 3, skip + 13, skip + 17, len(pkt) - 9]):
            reqs.append(_req(si, E.esp_input_crp(_Fw(), si, sa, bytearray(pkt), skip), pkt, cuts))
            want.append(("kat", 0, skip + 16, inner))
        bad = bytearray(pkt)
        bad[-3] ^= 0x10
        reqs.append(_req(si, E.esp_input_crp(_Fw(), si, sa, bad, skip), bad, [skip + 11]))
        want.append(("bad", BSD_EBADMSG, 0, bytes(bad)))
    alg = {"cbc-hmac-sha256": E.CBC_SHA256, "cbc-hmac-sha384": E.CBC_SHA384, "cbc-hmac-sha512": E.CBC_SHA512}
    for v in golden("eta_esp_packets.json"):
        sa = E.SecAssoc(v["spi"], alg[v["mode"]], bytes.fromhex(v["cipher_key"]), bytes.fromhex(v["auth_key"]))
        si = add_session(sa.csp())
        skip = v["outer_hdr_len"]
        pkt = bytes(skip) + bytes.fromhex(v["esp_record"])
        for cuts in (None, [skip + 9, skip + 30, len(pkt) - 5]):
            reqs.append(_req(si, E.esp_input_crp(_Fw(), si, sa, bytearray(pkt), skip), pkt, cuts))
            want.append(("kat", 0, skip + 24, bytes.fromhex(v["inner_packet"])))
        bad = bytearray(pkt)
        bad[-1] ^= 0x01
        reqs.append(_req(si, E.esp_input_crp(_Fw(), si, sa, bad, skip), bad, None))
        want.append(("bad", BSD_EBADMSG, 0, bytes(bad)))
    for v in golden("cipher_esp_packets.json"):
        sa = E.SecAssoc(v["spi"], E.CBC, bytes.fromhex(v["cipher_key"]))
        si = add_session(sa.csp())
        skip = v["outer_hdr_len"]
        pkt = bytes(skip) + bytes.fromhex(v["esp_record"])
        reqs.append(_req(si, E.esp_input_crp(_Fw(), si, sa, bytearray(pkt), skip), pkt, [skip + 7]))
        want.append(("kat", 0, skip + 24, bytes.fromhex(v["inner_packet"])))

    # oracle-built records of every session kind, both directions
    kinds = [GcmSA(rng, 16), GcmSA(rng, 32, esn=True), GcmSA(rng, 24, mlen=12), GcmSA(rng, 16, esn=True, mlen=8),
             EtaSA(rng, 32, esn=True), EtaSA(rng, 16, ctr=True, sha256=True), EtaSA(rng, 24, sha=384, esn=True),
             EtaSA(rng, 32, ctr=True, sha=512), EtaSA(rng, 0, null=True, sha=256, esn=True),
             EtaSA(rng, 16, noauth=True), EtaSA(rng, 32, ctr=True, noauth=True)]
    for sa in kinds:
        esa = sa.esp_sa()
        si = add_session(esa.csp())
        blk = 16 if (isinstance(sa, EtaSA) and not sa.ctr and not sa.null) else 4
        n = 10
        cts = rng.integers(1, 300, n) * blk
        cts[0] = 8944 - 8944 % blk
        eh = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) if sa.esn else None
        plain, ct, descs, eh = build_records(rng, [sa], np.zeros(n, dtype=np.int64), cts, esn_hi=eh)
        bad = ct.copy()
        for i in range(0, n, 3):
            o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
            bad[o + 8 + int(rng.integers(0, L - 8))] ^= 0x04
        ref = bad.copy()
        _, ref_st = O.batch([sa.oracle], ref, descs["off4"], descs["len"], descs["sa"], esn_hi=eh)
        for i in range(n):
            o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
            hdr = bytes([0x45]) + bytes(19)
            p_in = hdr + plain[o:o + L].tobytes()
            cuts = _cuts(rng, len(p_in), 4) if i % 2 else None
            reqs.append(_req(si, E.esp_output_crp(_Fw(), si, esa, bytearray(p_in), 20, esn_hi=int(eh[i])), p_in, cuts))
            want.append(("exact", 0, 0, hdr + ct[o:o + L].tobytes()))
            p_bad = hdr + bad[o:o + L].tobytes()
            reqs.append(_req(si, E.esp_input_crp(_Fw(), si, esa, bytearray(p_bad), 20, esn_hi=int(eh[i])), p_bad,
                             _cuts(rng, len(p_bad), 5) if i % 2 == 0 else None))
            if ref_st[i] == 0:
                h, a = sa.hlen, sa.mlen
                exp = hdr + bad[o:o + h].tobytes() + ref[o + h:o + L - a].tobytes() + bad[o + L - a:o + L].tobytes()
                want.append(("exact", 0, 0, exp))
            else:
                want.append(("exact", BSD_EBADMSG, 0, p_bad))
    # AH-style HMAC digest session: not served by the engine, stays on cryptosoft
    from espgpu.opencrypto import crypto_session_params
    ah = crypto_session_params(csp_mode=CSP_MODE_DIGEST, csp_auth_alg=O.CRYPTO_SHA1_HMAC, csp_auth_klen=20,
                               csp_auth_key=bytes(range(20)), csp_auth_mlen=12)
    add_session(ah)
    return sessions, reqs, want


@pytest.fixture(scope="module")
def workload():
    return _workload()


def _run(exe, workload, tmp_path, fail=False):
    sessions, reqs, want = workload
    rq, rs = str(tmp_path / "req.bin"), str(tmp_path / "res.bin")
    FR.pack_requests(rq, sessions, reqs)
    p = subprocess.run([exe, rq, rs] + (["--fail"] if fail else []), capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, (p.returncode, p.stdout[-2000:], p.stderr[-4000:])
    assert "fstack_crypto_run OK" in p.stdout
    if not fail:                                     # host_main.c 4b: a full SA table -> cryptosoft
        assert "the next went to cryptosoft" in p.stdout
    return FR.read_results(rs, [len(r["buf"]) for r in reqs], fail=fail)


BSD_EIO, BSD_EAGAIN = 5, 35


def _check_failure(res, workload):
    """The GPU-failure phase (host_main.c --fail), after
    the normal run checked by _check: every request the engine held when it
    failed completed exactly once, with EIO and its buffer untouched (a
    request dispatched at the moment of the failure -- its staging launched
    the failing batch -- was refused instead, and moved as below); every
    request after it completed with EAGAIN and a cryptosoft session (the
    driver's session move, crypto.c:1684-1725's protocol) and, re-dispatched
    as esp_input_cb does, exactly as cryptosoft's own run of it."""
    sessions, reqs, want = workload
    gpu_hid, sw_hid, ses, out = res
    n = n_eio = 0
    for i, (q, r) in enumerate(zip(reqs, out)):
        if ses[q["ses"]][1] != gpu_hid:
            continue
        n += 1
        assert r["f1_dispatch"] == 0 and r["f1_ndone0"] == 1, (i, r["f1_dispatch"], r["f1_ndone0"])
        if r["f1_etype0"] == BSD_EIO:
            n_eio += 1
            assert r["f1_ndone"] == 1 and r["f1_etype"] == BSD_EIO, (i, r["f1_ndone"], r["f1_etype"])
            assert r["f1_buf"] == q["buf"], i                           # untouched
        else:
            assert r["f1_etype0"] == BSD_EAGAIN, (i, r["f1_etype0"])
            assert r["f1_ndone"] == 2 and r["f1_etype"] == r["etype_sw"] and r["f1_buf"] == r["buf_sw"], i
        assert r["f2_etype0"] == BSD_EAGAIN and r["f2_hid"] == sw_hid, (i, r["f2_etype0"], r["f2_hid"])
        assert r["f2_redispatch"] == 0 and r["f2_ndone"] == 2, (i, r["f2_redispatch"], r["f2_ndone"])
        assert r["f2_etype"] == r["etype_sw"], (i, r["f2_etype"], r["etype_sw"])
        assert r["f2_buf"] == r["buf_sw"], i                            # cryptosoft's result
    assert n == len(reqs) and n_eio >= 1, (n, n_eio)      # (the GPU build holds until the first op change)


def _check(res, workload):
    sessions, reqs, want = workload
    gpu_hid, sw_hid, ses, out = res
    assert gpu_hid >= 0 and sw_hid >= 0 and gpu_hid != sw_hid
    for i, (err_d, hid_d, err_s, hid_s) in enumerate(ses[:-1]):
        assert err_d == 0 and hid_d == gpu_hid, (i, err_d, hid_d)        # esp_init's crid picks gpucrypto
        assert err_s == 0 and hid_s == sw_hid, (i, err_s, hid_s)         # SOFTWARE: cryptosoft
    err_d, hid_d, err_s, hid_s = ses[-1]
    assert err_d == 0 and hid_d == sw_hid and hid_s == sw_hid            # not served: cryptosoft keeps it
    for i, (r, (kind, etype, off, exp)) in enumerate(zip(out, want)):
        assert r["dispatch"] == 0 and r["dispatch_sw"] == 0, i
        assert r["done_flag"] == 1 and r["done_flag_sw"] == 1, i          # callback ran from crypto_done
        assert r["etype"] == etype, (i, kind, r["etype"], etype)
        assert r["etype_sw"] == etype, (i, kind, r["etype_sw"], etype)   # the reference's own software path
        assert r["buf"] == r["buf_sw"], (i, kind)                        # byte for byte as cryptosoft
        if kind == "kat":
            assert r["buf"][off:off + len(exp)] == exp, i
        else:
            assert r["buf"] == exp, (i, kind)


HAVE_REF = os.path.isdir("/root/reference/lib")


@pytest.fixture(scope="module")
def built():
    if HAVE_REF:
        FR.build("/root/reference", "/tmp/fstack_run_build_%d" % os.getpid())
    return FR.EXE_CPU, FR.EXE_GPU


def test_fstack_opencrypto_with_gpucrypto_cpu(built, workload, tmp_path):
    """The CPU executable (oracle stand-in behind the host shim interface)."""
    exe = built[0]
    if not os.path.exists(exe):
        pytest.skip("needs the F-Stack tree to build integration/fstack_crypto_run_cpu")
    _check(_run(exe, workload, tmp_path), workload)


@pytest.mark.gpu
def test_fstack_opencrypto_with_gpucrypto_gpu(workload, tmp_path):
    """The GPU executable: F-Stack's crypto.c, the kernel-domain driver, the
    real host shim and libespgpu.so on the MI355X, against cryptosoft run in
    the same process, the DPDK known answers and the oracle."""
    exe = FR.EXE_GPU
    # built where the F-Stack tree exists (__graft_entry__.build) and shipped
    # with the tree: a GPU run without it has lost the only F-Stack-level GPU
    # check, which must show as a failure, not a skip
    assert os.path.exists(exe), "integration/fstack_crypto_run_gpu missing: run __graft_entry__.build() where /root/reference exists"
    _check(_run(exe, workload, tmp_path), workload)


def test_fstack_gpu_failure_cpu(built, workload, tmp_path):
    """The GPU-failure path under F-Stack's crypto.c (CPU executable: the
    oracle stand-in fails with the requests staged)."""
    exe = built[0]
    if not os.path.exists(exe):
        pytest.skip("needs the F-Stack tree to build integration/fstack_crypto_run_cpu")
    res = _run(exe, workload, tmp_path, fail=True)
    _check(res, workload)
    _check_failure(res, workload)


@pytest.mark.gpu
def test_fstack_gpu_failure_gpu(workload, tmp_path):
    """The GPU-failure path under F-Stack's crypto.c on the MI355X: the
    engine's next launch fails (set_tuning "fault" 1) with every request
    staged; each completes once with EIO, later requests move to cryptosoft."""
    exe = FR.EXE_GPU
    assert os.path.exists(exe), "integration/fstack_crypto_run_gpu missing: run __graft_entry__.build() where /root/reference exists"
    res = _run(exe, workload, tmp_path, fail=True)
    _check(res, workload)
    _check_failure(res, workload)
