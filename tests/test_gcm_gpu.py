"""GPU parity tests for the AES-GCM-16 ESP path (MI355X).  Bit-exact against
the oracle (CPU restatement of swcr_gcm) and the DPDK ESP known answers, through
both boundaries: the opencrypto driver path (process/flush/poll on host
buffers, incl. mbuf-style segment chains) and the device-resident batch path."""
import numpy as np
import pytest

import oracle as O
from helpers import GcmSA, build_records, golden, oracle_decrypt

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def drv():
    from espgpu.opencrypto import GpuCryptoDriver
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible HIP device")
    d = GpuCryptoDriver(max_sessions=256)
    yield d
    d.close()


@pytest.fixture(scope="module")
def fw(drv):
    from espgpu.opencrypto import CryptoFramework
    return CryptoFramework(drv)


def payload_mask(descs, size, hlen=16, alen=16):
    """alen: ICV bytes, one int or one per record."""
    m = np.zeros(size, dtype=bool)
    alens = np.broadcast_to(np.asarray(alen), (len(descs),))
    for o4, L, a in zip(descs["off4"], descs["len"], alens):
        o = int(o4) * 4
        m[o + hlen:o + int(L) - int(a)] = True
    return m


# ---------------------------------------------------------------------------
# opencrypto driver path

def _run_esp(fw, sa, pkt, skip):
    from espgpu.esp import esp_input_crp
    err, ses = fw.crypto_newsession(sa.csp())
    assert err == 0
    crp = esp_input_crp(fw, ses, sa, pkt, skip)
    seen = []
    crp.crp_callback = lambda c: seen.append(c.crp_etype)
    assert fw.crypto_dispatch(crp) == 0
    fw.crypto_drain()
    fw.crypto_freesession(ses)
    assert len(seen) == 1
    return seen[0]


@pytest.mark.parametrize("v", golden("esp_packets.json"), ids=lambda v: v["name"])
@pytest.mark.parametrize("chain", [False, True], ids=["contig", "mbuf-chain"])
def test_dpdk_esp_kat_opencrypto(fw, v, chain):
    from espgpu.esp import GCM, SecAssoc, esp_trailer_ok
    key = bytes.fromhex(v["key"]) + bytes.fromhex(v["salt"])
    sa = SecAssoc(v["spi"], GCM, key)
    skip = v["outer_hdr_len"]
    pkt = bytearray(b"\x45" + bytes(skip - 1)) + bytearray(bytes.fromhex(v["esp_record"]))
    bufs = [pkt[:skip + 5], pkt[skip + 5:skip + 37], pkt[skip + 37:]] if chain else pkt
    et = _run_esp(fw, sa, bufs, skip)
    assert et == 0
    flat = b"".join(bytes(b) for b in bufs) if chain else bytes(pkt)
    pt = flat[skip + 16:len(flat) - 16]
    inner = bytes.fromhex(v["inner_packet"])
    assert pt[:len(inner)] == inner and esp_trailer_ok(pt)
    # ICV bit flip -> EBADMSG and the buffer is left as it was
    bad = bytearray(bytes([0x45]) + bytes(skip - 1)) + bytearray(bytes.fromhex(v["esp_record"]))
    bad[-3] ^= 0x10
    before = bytes(bad)
    assert _run_esp(fw, sa, bad, skip) == O.EBADMSG
    assert bytes(bad) == before


def test_opencrypto_encrypt_then_decrypt(fw):
    """esp_output -> esp_input through the driver, ciphertext bit-exact vs oracle."""
    from espgpu.esp import GCM, SecAssoc, esp_input_crp, esp_output_crp, esp_pad
    rng = np.random.default_rng(5)
    for klen in (16, 24, 32):
        key = rng.integers(0, 256, klen + 4, dtype=np.uint8).tobytes()
        sa = SecAssoc(0x1000 + klen, GCM, key)
        err, ses = fw.crypto_newsession(sa.csp())
        assert err == 0
        orc = O.SA(O.CSP_MODE_AEAD, key[:-4], key[-4:])
        pkts, refs = [], []
        for n in (20, 61, 1400, 8900):
            inner = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            body = esp_pad(inner)
            rec = (sa.spi.to_bytes(4, "big") + (7).to_bytes(4, "big") +
                   rng.integers(0, 256, 8, dtype=np.uint8).tobytes() + body + bytes(16))
            pkt = bytearray(bytes(20) + rec)
            pkts.append(pkt)
            e, ref = orc.esp_encrypt(rec)
            assert e == 0
            refs.append(ref)
            crp = esp_output_crp(fw, ses, sa, pkt, 20)
            assert fw.crypto_dispatch(crp) == 0
        fw.crypto_drain()
        for pkt, ref in zip(pkts, refs):
            assert bytes(pkt[20:]) == ref
        crps = []
        for pkt in pkts:
            crp = esp_input_crp(fw, ses, sa, pkt, 20)
            crps.append(crp)
            assert fw.crypto_dispatch(crp) == 0
        fw.crypto_drain()
        for crp, pkt, ref in zip(crps, pkts, refs):
            assert crp.crp_etype == 0
            e, dec = orc.esp_decrypt(ref)
            assert bytes(pkt[20 + 16:-16]) == dec[16:-16]
        fw.crypto_freesession(ses)


# ---------------------------------------------------------------------------
# device-resident batch path

def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _descs_dev(descs):
    return torch.from_numpy(np.ascontiguousarray(descs).view(np.uint8).copy()).cuda()


def _sessions(drv, sas):
    from espgpu.esp import GCM, SecAssoc
    sids = []
    for s in sas:
        rc, sid = drv.newsession(SecAssoc(s.spi, GCM, s.key + s.salt, esn=s.esn, mlen=s.mlen).csp())
        assert rc == 0
        sids.append(sid)
    return sids


@pytest.mark.parametrize("klen", [16, 24, 32])
@pytest.mark.parametrize("esn", [False, True])
def test_batch_decrypt_vs_oracle(drv, klen, esn, gcm_lanes):
    from espgpu.batch import decrypt_batch
    rng = np.random.default_rng(100 + klen + esn)
    sas = [GcmSA(rng, klen, esn=esn)]
    sids = _sessions(drv, sas)
    n = 1000
    cts = rng.choice([4, 12, 16, 20, 44, 204, 1000, 1448, 1452, 8948], n)
    plain, ct, descs, eh = build_records(rng, sas, np.zeros(n, dtype=np.int64), cts,
                                         esn_hi=rng.integers(0, 2**32, n, dtype=np.uint32)
                                         if esn else None)
    descs["sa"] = sids[0]
    bad = ct.copy()
    flip = rng.random(n) < 0.05
    for i in np.nonzero(flip)[0]:
        bad[int(descs["off4"][i]) * 4 + int(descs["len"][i]) - 1 - int(rng.integers(0, 16))] ^= 0x40
    ref_out, ref_st = oracle_decrypt(sas, bad, _oracle_descs(descs), eh)
    arena, out = _dev(bad), torch.zeros(len(bad), dtype=torch.uint8, device="cuda")
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    decrypt_batch(drv, arena, _descs_dev(descs), n, st, out=out, grouped=True)
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    assert (st == ref_st).all(), np.nonzero(st != ref_st)[0][:10]
    assert (st[flip] == O.EBADMSG).all() and (st[~flip] == 0).all()
    ok_mask = payload_mask(descs[~flip], len(bad))
    assert (out.cpu().numpy()[ok_mask] == ref_out[ok_mask]).all()
    assert (ref_out[ok_mask] == plain[ok_mask]).all()
    for s in sids:
        drv.freesession(s)


def _oracle_descs(descs):
    d = descs.copy()
    d["sa"] = 0
    return d


def test_batch_encrypt_vs_oracle(drv, gcm_lanes):
    from espgpu.batch import encrypt_batch
    rng = np.random.default_rng(9)
    sas = [GcmSA(rng, 16), GcmSA(rng, 32, esn=True)]
    sids = _sessions(drv, sas)
    n = 512
    sa_idx = np.repeat([0, 1], n // 2)
    cts = rng.choice([12, 204, 1448, 8948, 36], n)
    eh = rng.integers(0, 2**32, n, dtype=np.uint32)
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts, esn_hi=eh)
    d = descs.copy()
    d["sa"] = [sids[s] for s in sa_idx]
    arena = _dev(plain)
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    encrypt_batch(drv, arena, _descs_dev(d), n, st, grouped=False)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    assert (arena.cpu().numpy() == ct).all()
    for s in sids:
        drv.freesession(s)


def test_batch_inplace_verify_first(drv, gcm_lanes):
    """d_out == d_arena: EBADMSG records keep their ciphertext (esp_input_cb contract)."""
    from espgpu.batch import decrypt_batch
    rng = np.random.default_rng(21)
    sas = [GcmSA(rng, 16)]
    sids = _sessions(drv, sas)
    n = 600
    cts = rng.choice([12, 204, 1448, 8948], n)
    plain, ct, descs, eh = build_records(rng, sas, np.zeros(n, dtype=np.int64), cts)
    descs["sa"] = sids[0]
    bad = ct.copy()
    flip = np.arange(n) % 7 == 3
    for i in np.nonzero(flip)[0]:
        bad[int(descs["off4"][i]) * 4 + 3] ^= 0x01      # corrupt the SN (AAD)
    arena = _dev(bad)
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    decrypt_batch(drv, arena, _descs_dev(descs), n, st, out=None, grouped=True)
    torch.cuda.synchronize()
    st, res = st.cpu().numpy(), arena.cpu().numpy()
    assert (st[flip] == O.EBADMSG).all() and (st[~flip] == 0).all()
    m_ok, m_bad = payload_mask(descs[~flip], len(bad)), payload_mask(descs[flip], len(bad))
    assert (res[m_ok] == plain[m_ok]).all()
    assert (res[m_bad] == bad[m_bad]).all()
    drv.freesession(sids[0])


@pytest.mark.parametrize("grouped", [True, False])
@pytest.mark.parametrize("shape", ["aligned", "mixed"])
def test_inplace_failed_records_restored_vs_oracle(drv, gcm_lanes, grouped, shape):
    """In place, verify first, with forged records in every schedule the 4-lane
    kernel has: it decrypts in one pass and XORs the keystream back over a
    record whose tag failed (esp_gcm.hip GCM_INPLACE_ONEPASS), so the whole
    arena must equal the oracle's in-place result byte for byte (a failed
    record untouched, cryptosoft.c:595-633).  "aligned": 1448-byte payloads
    only (the dense-AES schedule); "mixed": sizes that break it.  Forgeries in
    the AAD, the ciphertext (first, middle and last block) and the ICV, one
    whole wave of failed records, and single failures among good ones."""
    from espgpu.batch import decrypt_batch
    rng = np.random.default_rng(4106)
    nsa = 1 if grouped else 12
    sas = [GcmSA(rng, int(rng.choice([16, 32])), esn=bool(k % 2)) for k in range(nsa)]
    sids = _sessions(drv, sas)
    n = 2048
    sa_idx = np.zeros(n, dtype=np.int64) if grouped else rng.integers(0, nsa, n)
    cts = np.full(n, 1448) if shape == "aligned" else rng.choice([12, 204, 1448, 8948, 1452], n)
    esn = rng.integers(0, 2**32, n, dtype=np.uint32)
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts, esn_hi=esn)
    d = descs.copy()
    d["sa"] = [sids[s] for s in sa_idx]
    bad = ct.copy()
    flip = rng.random(n) < 0.05
    flip[64:80] = True                       # a whole wave (16 records of 4 lanes) fails
    for k, i in enumerate(np.nonzero(flip)[0]):
        o, L, alen = int(descs["off4"][i]) * 4, int(descs["len"][i]), sas[sa_idx[i]].mlen
        ctl = L - 16 - alen
        pos = [o + 5, o + 16, o + 16 + ctl // 2, o + 16 + ctl - 1, o + L - 1][k % 5]
        bad[pos] ^= 1 << (k % 8)
    ref, ref_st = oracle_decrypt(sas, bad, descs, eh)
    assert (ref_st[flip] == O.EBADMSG).all() and (ref_st[~flip] == 0).all()
    arena = _dev(bad)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    decrypt_batch(drv, arena, _descs_dev(d), n, st, out=None, grouped=grouped)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == ref_st).all()
    res = arena.cpu().numpy()
    assert (res == ref).all(), "first differing byte %d" % int(np.argmax(res != ref))
    for s in sids:
        drv.freesession(s)


def test_planner_many_sessions_mixed_sizes(drv, gcm_lanes):
    """Random SA per record (the cfg2 shape, scaled down): device planner path."""
    from espgpu.batch import decrypt_batch
    rng = np.random.default_rng(33)
    nsa = 40
    sas = [GcmSA(rng, int(rng.choice([16, 32]))) for _ in range(nsa)]
    sids = _sessions(drv, sas)
    n = 3000
    sa_idx = rng.integers(0, nsa, n)
    cts = rng.choice([12, 204, 1448, 8948], n)
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts)
    d = descs.copy()
    d["sa"] = [sids[s] for s in sa_idx]
    ref_out, ref_st = oracle_decrypt(sas, ct, descs, eh)
    arena, out = _dev(ct), torch.zeros(len(ct), dtype=torch.uint8, device="cuda")
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    decrypt_batch(drv, arena, _descs_dev(d), n, st, out=out, grouped=False)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    m = payload_mask(descs, len(ct))
    assert (out.cpu().numpy()[m] == plain[m]).all()
    for s in sids:
        drv.freesession(s)


def test_invalid_records_einval(drv):
    from espgpu.batch import decrypt_batch
    rng = np.random.default_rng(4)
    sas = [GcmSA(rng)]
    sids = _sessions(drv, sas)
    plain, ct, descs, eh = build_records(rng, sas, np.zeros(6, dtype=np.int64), [100] * 6)
    descs["sa"] = sids[0]
    descs["len"][0] = 32          # no payload: plen <= 0
    descs["len"][1] = 130         # not a multiple of 4
    descs["sa"][2] = 250          # no such session
    for grouped in (True, False):
        arena = _dev(ct)
        out = torch.zeros_like(arena)
        st = torch.full((6,), 0xEE, dtype=torch.uint8, device="cuda")
        decrypt_batch(drv, arena, _descs_dev(descs), 6, st, out=out, grouped=grouped)
        torch.cuda.synchronize()
        s = st.cpu().numpy()
        assert list(s[:3]) == [O.EINVAL] * 3 and (s[3:] == 0).all(), (grouped, s)
    drv.freesession(sids[0])


def test_full_size_1m_x_1500_vs_oracle(drv):
    """cfg1 at full size (1M x 1500-B packets, one AES-128-GCM SA), every
    record against the oracle: GPU encrypt gives the oracle's arena byte for
    byte; with 1% of the ICVs flipped, GPU decrypt gives the oracle's 1M
    statuses, out of place the oracle's plaintext for every verified record,
    in place the oracle's whole arena (failed records untouched)."""
    import os
    from espgpu.batch import decrypt_batch, encrypt_batch
    rng = np.random.default_rng(1500)
    sas = [GcmSA(rng, 16)]
    sids = _sessions(drv, sas)
    n, rec, size = 1 << 20, 1480, (1 << 20) * 1500 + 64
    plain = np.frombuffer(rng.bytes(size), dtype=np.uint8).copy()
    d = np.zeros(n, dtype=[("off4", "<u4"), ("len", "<u2"), ("sa", "<u2"), ("esn_hi", "<u4"), ("salt", "<u4")])
    d["off4"] = (np.arange(n, dtype=np.int64) * 1500 + 20) // 4
    d["len"] = rec
    d["salt"] = int.from_bytes(sas[0].salt, "little")
    nth = min(16, os.cpu_count() or 1)
    ct = plain.copy()
    O.batch([sas[0].oracle], ct, d["off4"], d["len"], d["sa"], nthreads=nth, encrypt=True)
    d["sa"] = sids[0]
    desc = _descs_dev(d)
    arena = torch.from_numpy(plain).cuda()
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    encrypt_batch(drv, arena, desc, n, st, grouped=True)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    assert np.array_equal(arena.cpu().numpy(), ct)
    del arena

    flip = rng.random(n) < 0.01
    fi = np.nonzero(flip)[0]
    bad = ct.copy()
    bad[fi * 1500 + 20 + rec - 1 - rng.integers(0, 16, len(fi))] ^= 0x40
    ref_out = bad.copy()
    d["sa"] = 0
    _, ref_st = O.batch([sas[0].oracle], ref_out, d["off4"], d["len"], d["sa"], nthreads=nth)
    assert (ref_st[flip] == O.EBADMSG).all() and (ref_st[~flip] == 0).all()
    pm = np.zeros(1500, dtype=bool)
    pm[20 + 16:20 + rec - 16] = True
    ok_mask = np.concatenate([(pm[None, :] & ~flip[:, None]).reshape(-1), np.zeros(64, dtype=bool)])
    assert np.array_equal(ref_out[ok_mask], plain[ok_mask])
    for inplace in (False, True):
        src = torch.from_numpy(bad).cuda()
        out = src if inplace else torch.zeros_like(src)
        st.fill_(0xEE)
        decrypt_batch(drv, src, desc, n, st, out=None if inplace else out, grouped=True)
        torch.cuda.synchronize()
        assert np.array_equal(st.cpu().numpy(), ref_st), inplace
        res = out.cpu().numpy()
        if inplace:
            assert np.array_equal(res, ref_out)
        else:
            assert np.array_equal(res[ok_mask], ref_out[ok_mask])
        del src, out, res
    drv.freesession(sids[0])


def test_freesession_waits_for_batch_on_user_stream(drv):
    """espgpu_freesession zeroes the session's device keys: a device-resident
    batch still running on the caller's own stream must finish under the old
    keys first (the ctx's last-launch event), so every record verifies."""
    from espgpu.batch import decrypt_batch, encrypt_batch
    rng = np.random.default_rng(4242)
    sas = [GcmSA(rng, 16)]
    sids = _sessions(drv, sas)
    n, rec = 1 << 20, 1480
    g = torch.Generator(device="cuda").manual_seed(11)
    arena = torch.randint(0, 256, (n * 1500 + 64,), dtype=torch.uint8, device="cuda", generator=g)
    d = np.zeros(n, dtype=[("off4", "<u4"), ("len", "<u2"), ("sa", "<u2"), ("esn_hi", "<u4"), ("salt", "<u4")])
    d["off4"] = (np.arange(n, dtype=np.int64) * 1500 + 20) // 4
    d["len"] = rec
    d["sa"] = sids[0]
    d["salt"] = int.from_bytes(sas[0].salt, "little")
    desc = _descs_dev(d)
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    encrypt_batch(drv, arena, desc, n, st, grouped=True)
    torch.cuda.synchronize()
    user = torch.cuda.Stream()
    out = torch.zeros_like(arena)
    st.fill_(0xEE)
    torch.cuda.synchronize()
    with torch.cuda.stream(user):
        for _ in range(4):          # several ms of work queued behind the free
            decrypt_batch(drv, arena, desc, n, st, out=out, grouped=True, stream=user)
    drv.freesession(sids[0])        # host returns only after the batches ran
    assert user.query()
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0


@pytest.mark.parametrize("inplace", [False, True])
def test_every_line_alignment_vs_oracle(drv, gcm_lanes, inplace):
    """Every payload alignment (all 32 four-byte offsets in a 128-byte line,
    out of place also with the output at another alignment than the input),
    payloads that end anywhere in a 16-byte block or a line, cross the
    counter-256 run, and the three ICV lengths: decrypt and encrypt bit-exact
    vs the oracle, trailer words included, through both GCM kernels."""
    from espgpu.batch import decrypt_batch, encrypt_batch
    rng = np.random.default_rng(9000 + gcm_lanes + 2 * inplace)
    sas = [GcmSA(rng, 16), GcmSA(rng, 32, esn=True), GcmSA(rng, 16, mlen=12), GcmSA(rng, 24, mlen=8)]
    sids = _sessions(drv, sas)
    cts = [4, 8, 12, 16, 20, 60, 64, 108, 112, 124, 128, 132, 236, 240, 252, 256, 260, 1448, 4092, 4100, 8948]
    n = 32 * len(cts)
    sa_idx = rng.integers(0, len(sas), n)
    ct_l = np.array([cts[i % len(cts)] for i in range(n)])
    # one record per (alignment, size): stride_pad rotates the start offsets
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, ct_l, stride_pad=4,
                                         esn_hi=rng.integers(0, 2**32, n, dtype=np.uint32))
    offs = descs["off4"].astype(np.int64) * 4 + 16
    assert len(set((offs % 128).tolist())) == 32
    bad = ct.copy()
    flip = rng.random(n) < 0.1
    for i in np.nonzero(flip)[0]:
        bad[int(descs["off4"][i]) * 4 + int(rng.integers(0, int(descs["len"][i])))] ^= 0x08
    ref_out, ref_st = oracle_decrypt(sas, bad, descs, eh)
    d = descs.copy()
    d["sa"] = [sids[s] for s in sa_idx]
    for shift in ((0,) if inplace else (0, 4, 68)):
        arena = _dev(bad)
        obuf = torch.zeros(len(bad) + 128, dtype=torch.uint8, device="cuda")
        out = arena if inplace else obuf[shift:shift + len(bad)]
        st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
        tr = torch.zeros(n, dtype=torch.int32, device="cuda")
        decrypt_batch(drv, arena, _descs_dev(d), n, st, out=None if inplace else out, trailer=tr)
        torch.cuda.synchronize()
        got = st.cpu().numpy()
        assert (got == ref_st).all(), (shift, np.nonzero(got != ref_st)[0][:10])
        alens = np.array([sas[s].mlen for s in sa_idx])
        m = payload_mask(descs[got == 0], len(bad), 16, alens[got == 0])
        assert (out.cpu().numpy()[m] == ref_out[m]).all(), shift
        from espgpu.esp import trailer_word
        trw = tr.cpu().numpy().view(np.uint32)
        for i in np.nonzero(got == 0)[0][:200]:
            o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
            assert trw[i] == trailer_word(bytes(ref_out[o + 16:o + L - int(alens[i])])), i
        assert (trw[got != 0] == 0).all()
    arena = _dev(plain)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    encrypt_batch(drv, arena, _descs_dev(d), n, st)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    assert (arena.cpu().numpy() == ct).all()
    for s in sids:
        drv.freesession(s)


@pytest.mark.parametrize("chunk", [0, 97, 1000])
def test_host_pipeline_vs_oracle(drv, chunk):
    """espgpu_decrypt_host: pinned host records -> chunked H2D/kernel/D2H on
    three streams -> pinned host plaintext; same results as the oracle."""
    from espgpu.batch import decrypt_host
    rng = np.random.default_rng(500 + chunk)
    sas = [GcmSA(rng, 16), GcmSA(rng, 32, esn=True)]
    sids = _sessions(drv, sas)
    n = 2500
    sa_idx = rng.integers(0, 2, n)
    cts = rng.choice([4, 16, 204, 1448, 8948], n)
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts,
                                         esn_hi=rng.integers(0, 2**32, n, dtype=np.uint32))
    bad = ct.copy()
    flip = rng.random(n) < 0.05
    for i in np.nonzero(flip)[0]:
        bad[int(descs["off4"][i]) * 4 + int(descs["len"][i]) - 3] ^= 0x01
    ref_out, ref_st = oracle_decrypt(sas, bad, descs, eh)
    d = descs.copy()
    d["sa"] = [sids[s] for s in sa_idx]
    h_arena = torch.from_numpy(bad.copy()).pin_memory()
    h_desc = torch.from_numpy(np.ascontiguousarray(d).view(np.uint8).copy()).pin_memory()
    h_out = torch.zeros(len(bad), dtype=torch.uint8).pin_memory()
    h_st = torch.full((n,), 0xEE, dtype=torch.uint8).pin_memory()
    decrypt_host(drv, h_arena, h_desc, n, h_st, h_out, chunk=chunk)
    st = h_st.numpy()
    assert (st == ref_st).all(), np.nonzero(st != ref_st)[0][:10]
    m = payload_mask(descs[st == 0], len(bad))
    assert (h_out.numpy()[m] == ref_out[m]).all()
    assert (h_out.numpy()[m] == plain[m]).all()
    for s in sids:
        drv.freesession(s)


@pytest.mark.parametrize("grid", [0, 7, 300])
def test_kernel_grids_vs_oracle(drv, grid, gcm_lanes):
    """The GCM kernel decrypts (out of place and verify-first in place),
    verifies and encrypts bit-exactly at the default and at odd grid sizes
    (work-queue drain with fewer and more workgroups than CUs), for
    AES-128/256, ESN, and records crossing counter 256 mid-pair."""
    from espgpu.batch import decrypt_batch, encrypt_batch
    rng = np.random.default_rng(700 + grid)
    sas = [GcmSA(rng, 16), GcmSA(rng, 32, esn=True)]
    sids = _sessions(drv, sas)
    n = 1200
    sa_idx = rng.integers(0, 2, n)
    cts = rng.choice([4, 12, 100, 204, 1448, 4000, 8948, 8940], n)
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts,
                                         esn_hi=rng.integers(0, 2**32, n, dtype=np.uint32))
    bad = ct.copy()
    flip = rng.random(n) < 0.05
    for i in np.nonzero(flip)[0]:
        bad[int(descs["off4"][i]) * 4 + 16 + int(rng.integers(0, int(descs["len"][i]) - 16))] ^= 0x10
    ref_out, ref_st = oracle_decrypt(sas, bad, descs, eh)
    d = descs.copy()
    d["sa"] = [sids[s] for s in sa_idx]
    assert drv.lib.espgpu_set_tuning(drv.ctx, b"grid", grid) == 0
    try:
        for inplace in (False, True):
            arena = _dev(bad)
            out = arena if inplace else torch.zeros_like(arena)
            st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
            decrypt_batch(drv, arena, _descs_dev(d), n, st, out=None if inplace else out)
            torch.cuda.synchronize()
            got = st.cpu().numpy()
            assert (got == ref_st).all(), (inplace, np.nonzero(got != ref_st)[0][:10])
            m = payload_mask(descs[got == 0], len(bad))
            assert (out.cpu().numpy()[m] == ref_out[m]).all()
            if inplace:
                mb = payload_mask(descs[got != 0], len(bad), 0, 0)
                assert (out.cpu().numpy()[mb] == bad[mb]).all()
        arena = _dev(plain)
        st = torch.zeros(n, dtype=torch.uint8, device="cuda")
        encrypt_batch(drv, arena, _descs_dev(d), n, st)
        torch.cuda.synchronize()
        assert (st.cpu().numpy() == 0).all()
        assert (arena.cpu().numpy() == ct).all()
    finally:
        drv.lib.espgpu_set_tuning(drv.ctx, b"grid", 0)
        for s in sids:
            drv.freesession(s)


# ---------------------------------------------------------------------------
# truncated ICVs (csp_auth_mlen 12 / 8: cryptosoft.c:1112-1117 keeps sw_mlen
# bytes of the tag and compares that many, swcr_gcm :598-600, :636)

@pytest.mark.parametrize("mlen", [12, 8])
def test_truncated_icv_batch_vs_oracle(drv, mlen, gcm_lanes):
    """Decrypt (out of place and verify-first in place) and encrypt with
    truncated-ICV sessions mixed with a full-ICV one through the planner."""
    from espgpu.batch import decrypt_batch, encrypt_batch
    rng = np.random.default_rng(800 + mlen)
    sas = [GcmSA(rng, 16, mlen=mlen), GcmSA(rng, 32, esn=True, mlen=mlen), GcmSA(rng, 16)]
    sids = _sessions(drv, sas)
    n = 1500
    sa_idx = rng.integers(0, 3, n)
    cts = rng.choice([4, 12, 204, 1448, 8948], n)
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts,
                                         esn_hi=rng.integers(0, 2**32, n, dtype=np.uint32))
    alens = np.array([sas[i].mlen for i in sa_idx])
    bad = ct.copy()
    flip = rng.random(n) < 0.05
    for i in np.nonzero(flip)[0]:       # a bit inside the (truncated) ICV
        bad[int(descs["off4"][i]) * 4 + int(descs["len"][i]) - 1 - int(rng.integers(0, alens[i]))] ^= 0x02
    ref_out, ref_st = oracle_decrypt(sas, bad, descs, eh)
    assert (ref_st[flip] == O.EBADMSG).all() and (ref_st[~flip] == 0).all()
    d = descs.copy()
    d["sa"] = [sids[s] for s in sa_idx]
    for inplace in (False, True):
        arena = _dev(bad)
        out = arena if inplace else torch.zeros_like(arena)
        st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
        decrypt_batch(drv, arena, _descs_dev(d), n, st, out=None if inplace else out)
        torch.cuda.synchronize()
        got = st.cpu().numpy()
        assert (got == ref_st).all(), (inplace, np.nonzero(got != ref_st)[0][:10])
        m = payload_mask(descs[~flip], len(bad), alen=alens[~flip])
        assert (out.cpu().numpy()[m] == plain[m]).all()
    arena = _dev(plain)
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    encrypt_batch(drv, arena, _descs_dev(d), n, st)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    assert (arena.cpu().numpy() == ct).all()        # CT and the mlen-byte ICVs
    for s in sids:
        drv.freesession(s)


@pytest.mark.parametrize("mlen", [12, 8])
def test_truncated_icv_opencrypto(fw, mlen):
    """esp_output -> esp_input through the driver path with a truncated-ICV
    session: ciphertext and ICV bit-exact vs the oracle, a flipped ICV bit is
    EBADMSG with the buffer untouched."""
    from espgpu.esp import GCM, SecAssoc, esp_input_crp, esp_output_crp, esp_pad
    rng = np.random.default_rng(900 + mlen)
    key = rng.integers(0, 256, 20, dtype=np.uint8).tobytes()
    sa = SecAssoc(0x3000 + mlen, GCM, key, mlen=mlen)
    err, ses = fw.crypto_newsession(sa.csp())
    assert err == 0
    orc = O.SA(O.CSP_MODE_AEAD, key[:-4], key[-4:], mlen=mlen)
    pkts, refs = [], []
    for nbytes in (20, 61, 1400, 8900):
        body = esp_pad(rng.integers(0, 256, nbytes, dtype=np.uint8).tobytes())
        rec = (sa.spi.to_bytes(4, "big") + (9).to_bytes(4, "big") +
               rng.integers(0, 256, 8, dtype=np.uint8).tobytes() + body + bytes(mlen))
        pkt = bytearray(bytes(20) + rec)
        e, ref = orc.esp_encrypt(rec)
        assert e == 0
        pkts.append(pkt)
        refs.append((rec, ref))
        assert fw.crypto_dispatch(esp_output_crp(fw, ses, sa, pkt, 20)) == 0
    fw.crypto_drain()
    for pkt, (rec, ref) in zip(pkts, refs):
        assert bytes(pkt[20:]) == ref
    crps = [esp_input_crp(fw, ses, sa, pkt, 20) for pkt in pkts]
    bad = bytearray(pkts[1])
    bad[-1] ^= 0x80
    before = bytes(bad)
    crps.append(esp_input_crp(fw, ses, sa, bad, 20))
    for c in crps:
        assert fw.crypto_dispatch(c) == 0
    fw.crypto_drain()
    for c, pkt, (rec, ref) in zip(crps, pkts, refs):
        assert c.crp_etype == 0
        assert bytes(pkt[20 + 16:-mlen]) == rec[16:-mlen]
    assert crps[-1].crp_etype == O.EBADMSG and bytes(bad) == before
    fw.crypto_freesession(ses)


def test_two_streams_one_ctx(drv):
    """One ctx used from two streams back to back (no host sync between):
    the ctx's work-queue counters and planner workspace are shared, so the
    second launch must be ordered after the first (run_batch waits on the
    ctx's last-launch event); both batches come out bit-exact."""
    from espgpu.batch import decrypt_batch
    rng = np.random.default_rng(77)
    sas = [GcmSA(rng, 16), GcmSA(rng, 32)]
    sids = _sessions(drv, sas)
    jobs = []
    for k in range(2):
        n = 3000 + 500 * k
        sa_idx = rng.integers(0, 2, n)
        plain, ct, descs, eh = build_records(rng, sas, sa_idx, rng.choice([12, 204, 1448, 8948], n))
        d = descs.copy()
        d["sa"] = [sids[s] for s in sa_idx]
        jobs.append((n, plain, ct, descs, _descs_dev(d)))
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for rep in range(4):
        outs = []
        for (n, plain, ct, descs, ddev), s in zip(jobs, streams):
            with torch.cuda.stream(s):
                arena = _dev(ct)
                out = torch.zeros_like(arena)
                st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
            s.synchronize()
            outs.append((arena, out, st))
        for (n, plain, ct, descs, ddev), s, (arena, out, st) in zip(jobs, streams, outs):
            decrypt_batch(drv, arena, ddev, n, st, out=out, grouped=False, stream=s)
        torch.cuda.synchronize()
        for (n, plain, ct, descs, ddev), (arena, out, st) in zip(jobs, outs):
            assert (st.cpu().numpy() == 0).all(), rep
            m = payload_mask(descs, len(ct))
            assert (out.cpu().numpy()[m] == plain[m]).all(), rep
    for s in sids:
        drv.freesession(s)


@pytest.mark.parametrize("n", [1, 7, 33, 257, 4097, 32767, 32768, 40000])
def test_grouped_batch_sizes_across_the_small_batch_path(drv, n):
    """Caller-grouped batches on both sides of the small-batch switch
    (kGcmSmallBatch = 32768: 8 lanes per record and power-of-two chunks of
    32..256 records below it, 4 lanes and 256-record chunks at and above it),
    decrypted out of place, in place and re-encrypted: statuses and bytes
    bit-exact vs the oracle, tag failures included."""
    from espgpu.batch import decrypt_batch, encrypt_batch
    rng = np.random.default_rng(4000 + n)
    sas = [GcmSA(rng, 16, esn=True, mlen=16)]
    sids = _sessions(drv, sas)
    cts = rng.choice([4, 44, 204, 1448, 2996], n)
    eh = rng.integers(0, 2**32, n, dtype=np.uint32)
    plain, ct, descs, eh = build_records(rng, sas, np.zeros(n, dtype=np.int64), cts, esn_hi=eh)
    descs["sa"] = sids[0]
    bad = ct.copy()
    flip = rng.random(n) < 0.05
    for i in np.nonzero(flip)[0]:
        o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
        bad[o + int(rng.integers(0, L))] ^= 0x02
    ref_out, ref_st = oracle_decrypt(sas, bad, _oracle_descs(descs), eh)
    ok_mask = payload_mask(descs[ref_st == 0], len(bad))
    for inplace in (False, True):
        arena = _dev(bad)
        out = arena if inplace else torch.zeros_like(arena)
        st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
        decrypt_batch(drv, arena, _descs_dev(descs), n, st, out=None if inplace else out, grouped=True)
        torch.cuda.synchronize()
        got = st.cpu().numpy()
        assert (got == ref_st).all(), (inplace, np.nonzero(got != ref_st)[0][:10])
        assert (out.cpu().numpy()[ok_mask] == plain[ok_mask]).all(), inplace
    arena = _dev(plain)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    encrypt_batch(drv, arena, _descs_dev(descs), n, st, grouped=True)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    assert (arena.cpu().numpy() == ct).all()
    for s in sids:
        drv.freesession(s)


@pytest.mark.parametrize("lanes,burst", [(0, 4096), (4, 4096), (8, 4096), (0, 1 << 30)],
                         ids=["auto", "lanes4", "lanes8", "burst"])
@pytest.mark.parametrize("n,grouped", [(700, False), (40000, False), (40000, True)])
def test_packed_output_vs_oracle(n, grouped, lanes, burst):
    """espgpu_decrypt_batch_packed: record i's plaintext at out + i*stride
    (128-byte aligned), mixed sizes and sessions (planner) or one session
    (caller-grouped), small (S = 8) and large batches, and with the burst
    kernel enabled for every size (packed output always takes the fused
    kernel); statuses and verified plaintext vs the oracle, a record longer
    than the stride is EINVAL, the bytes of each slot past its payload are
    never written.  A record that fails its tag (EBADMSG) holds its
    unverified plaintext, as the header says: the consumer ignores it."""
    from espgpu.batch import decrypt_batch_packed
    from espgpu.opencrypto import GpuCryptoDriver
    d = GpuCryptoDriver(max_sessions=16)
    try:
        assert d.lib.espgpu_set_tuning(d.ctx, b"gcm_lanes", lanes) == 0      # 0: by batch size
        assert d.lib.espgpu_set_tuning(d.ctx, b"gcm_burst", burst) == 0
        rng = np.random.default_rng(2100 + n + grouped)
        nsa = 1 if grouped else 3
        sas = [GcmSA(rng, klen=16 + 8 * (i % 3), mlen=(16, 12, 8)[i % 3]) for i in range(nsa)]
        sids = _sessions(d, sas)
        sa_idx = np.zeros(n, dtype=np.int64) if grouped else rng.integers(0, nsa, n)
        stride = 1536
        cts = rng.choice([12, 204, 1448, 1452, 1536, 1540], n)     # 1540 > stride: EINVAL
        plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts)
        bad = ct.copy()
        flip = rng.random(n) < 0.05
        for i in np.flatnonzero(flip):
            bad[int(descs["off4"][i]) * 4 + int(descs["len"][i]) - 1] ^= 0x10
        ref_out, ref_st = oracle_decrypt(sas, bad, descs, eh)
        want_st = np.where(cts > stride, O.EINVAL, ref_st)
        dd = descs.copy()
        dd["sa"] = [sids[s] for s in sa_idx]
        arena = _dev(bad)
        out = torch.full((n * stride,), 0xA5, dtype=torch.uint8, device="cuda")
        st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
        decrypt_batch_packed(d, arena, _descs_dev(dd), n, st, out, stride, grouped=grouped)
        torch.cuda.synchronize()
        got = st.cpu().numpy()
        assert (got == want_st).all(), np.flatnonzero(got != want_st)[:10]
        res = out.cpu().numpy().reshape(n, stride)
        for i in np.flatnonzero(got == 0):
            o, L, ml = int(descs["off4"][i]) * 4, int(descs["len"][i]), sas[sa_idx[i]].mlen
            c = L - 16 - ml
            assert res[i, :c].tobytes() == plain[o + 16:o + 16 + c].tobytes(), i
            assert (res[i, c:] == 0xA5).all(), i
        for i in np.flatnonzero(cts > stride):
            assert (res[i] == 0xA5).all(), i
        # only the ICV was flipped: the unverified plaintext is the true one
        for i in np.flatnonzero(got == O.EBADMSG):
            o, L, ml = int(descs["off4"][i]) * 4, int(descs["len"][i]), sas[sa_idx[i]].mlen
            c = L - 16 - ml
            assert res[i, :c].tobytes() == plain[o + 16:o + 16 + c].tobytes(), i
        assert (got == O.EBADMSG).sum() > 0
        for s in sids:
            d.freesession(s)
    finally:
        d.close()


def test_packed_output_rejects(drv):
    """Stride not a multiple of 128, in place, an unaligned output, or a
    context holding ETA sessions: EINVAL / ENOTSUP."""
    from espgpu.esp import CBC_SHA1, SecAssoc
    z = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    dsc = torch.zeros(16, dtype=torch.uint8, device="cuda")
    st = torch.zeros(1, dtype=torch.uint8, device="cuda")
    L = drv.lib
    assert L.espgpu_decrypt_batch_packed(drv.ctx, z.data_ptr(), dsc.data_ptr(), 1, st.data_ptr(), z.data_ptr(),
                                         1536, 0, None) == 22
    out = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    assert L.espgpu_decrypt_batch_packed(drv.ctx, z.data_ptr(), dsc.data_ptr(), 1, st.data_ptr(), out.data_ptr(),
                                         1500, 0, None) == 22
    assert L.espgpu_decrypt_batch_packed(drv.ctx, z.data_ptr(), dsc.data_ptr(), 1, st.data_ptr(), out.data_ptr(),
                                         0, 0, None) == 22
    # d_out not 128-byte aligned
    assert L.espgpu_decrypt_batch_packed(drv.ctx, z.data_ptr(), dsc.data_ptr(), 1, st.data_ptr(),
                                         out.data_ptr() + 64, 1536, 0, None) == 22
    rc, sid = drv.newsession(SecAssoc(0x4242, CBC_SHA1, bytes(16), bytes(20)).csp())
    assert rc == 0
    try:
        assert L.espgpu_decrypt_batch_packed(drv.ctx, z.data_ptr(), dsc.data_ptr(), 1, st.data_ptr(),
                                             out.data_ptr(), 1536, 0, None) == 95
    finally:
        drv.freesession(sid)


def test_gpu_failure_batch_and_driver_path():
    """The GPU-failure path on the engine directly (its own context, the
    module's stays healthy): a device-resident batch whose launch fails
    (set_tuning "fault" 1) returns EIO and fails the context; every later
    batch, newsession, process, flush and drain answers EIO (never
    ERESTART), a request the Python framework dispatches completes at once
    with EIO, espgpu_health and the stats say so, and close does not hang.
    A healthy batch before the fault decrypts as the oracle does."""
    from espgpu.batch import decrypt_batch, descs_to_tensor
    from espgpu.esp import esp_input_crp
    from espgpu.opencrypto import CryptoFramework, GpuCryptoDriver
    d = GpuCryptoDriver(max_sessions=8, batch_records=64, nbatches=2)
    try:
        fw = CryptoFramework(d)
        rng = np.random.default_rng(4800)
        sa = GcmSA(rng, 16)
        err, cs = fw.crypto_newsession(sa.esp_sa().csp())
        assert err == 0 and cs.sid == 0
        n = 512
        plain, ct, descs, _ = build_records(rng, [sa], np.zeros(n, dtype=np.int64),
                                            rng.integers(1, 92, n) * 16)
        ref = ct.copy()
        _, ref_st = O.batch([sa.oracle], ref, descs["off4"], descs["len"], descs["sa"])
        dev = torch.device("cuda:0")
        arena = torch.from_numpy(np.concatenate([ct, np.zeros(64, np.uint8)])).to(dev)
        desc = descs_to_tensor(descs, dev)
        status = torch.zeros(n, dtype=torch.uint8, device=dev)
        decrypt_batch(d, arena, desc, n, status)
        torch.cuda.synchronize()
        assert (status.cpu().numpy() == ref_st).all()
        m = payload_mask(descs, len(ct))
        assert (arena.cpu().numpy()[:len(ct)][m] == ref[m]).all()
        assert d.health() == 0
        assert d.set_tuning("fault", 8) == O.EINVAL            # unknown bit
        assert d.set_tuning("fault", 1) == 0
        arena.copy_(torch.from_numpy(np.concatenate([ct, np.zeros(64, np.uint8)])).to(dev))
        with pytest.raises(RuntimeError):
            decrypt_batch(d, arena, desc, n, status)
        EIO = 5
        assert d.health() == EIO and "GPU failure" in d.last_error()
        assert d.lib.espgpu_decrypt_batch(d.ctx, arena.data_ptr(), desc.data_ptr(), n, status.data_ptr(),
                                          None, 0, None) == EIO
        assert d.newsession(sa.esp_sa().csp())[0] == EIO
        pkt = bytearray(bytes(20)) + bytearray(ct[int(descs["off4"][0]) * 4:][:int(descs["len"][0])].tobytes())
        before = bytes(pkt)
        crp = esp_input_crp(fw, cs, sa.esp_sa(), pkt, 20)
        seen = []
        crp.crp_callback = lambda c: seen.append(c.crp_etype)
        assert fw.crypto_dispatch(crp) == 0
        assert seen == [EIO] and bytes(pkt) == before          # completed at once, untouched
        assert d.flush() == EIO and d.drain() == EIO
        fw.crypto_poll()
        assert seen == [EIO]                                   # once
        st = d.stats()
        assert st["gpu_fail"] == 1 and st["fail_eio"] == 1
        assert d.set_tuning("deadline_ms", 0) == O.EINVAL
        fw.crypto_freesession(cs)                              # host bookkeeping only
    finally:
        d.close()
