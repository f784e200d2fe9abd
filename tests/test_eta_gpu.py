"""GPU parity tests for the AES-CBC + HMAC-SHA1-96 ESP path (CSP_MODE_ETA):
bit-exact against the oracle (swcr_eta restatement), ICV failures, ESN,
in-place verify-first, mixed GCM + ETA batches through the planner."""
import numpy as np
import pytest

import oracle as O
from helpers import EtaSA, GcmSA, build_records, oracle_decrypt

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


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _descs_dev(descs):
    return torch.from_numpy(np.ascontiguousarray(descs).view(np.uint8).copy()).cuda()


def _sessions(drv, sas):
    from espgpu.esp import CBC_SHA1, GCM, SecAssoc
    sids = []
    for s in sas:
        if isinstance(s, EtaSA):
            sa = SecAssoc(s.spi, CBC_SHA1, s.key, s.akey, esn=s.esn)
        else:
            sa = SecAssoc(s.spi, GCM, s.key + s.salt, esn=s.esn)
        rc, sid = drv.newsession(sa.csp())
        assert rc == 0, drv.last_error()
        sids.append(sid)
    return sids


def _mask(descs, size, hlen, alen):
    m = np.zeros(size, dtype=bool)
    for o4, L in zip(descs["off4"], descs["len"]):
        m[int(o4) * 4 + hlen:int(o4) * 4 + int(L) - alen] = True
    return m


@pytest.mark.parametrize("klen", [16, 24, 32])
@pytest.mark.parametrize("esn", [False, True])
@pytest.mark.parametrize("inplace", [False, True])
def test_eta_decrypt_vs_oracle(drv, klen, esn, inplace):
    from espgpu.batch import decrypt_batch
    rng = np.random.default_rng(300 + klen + 2 * esn + 4 * inplace)
    sas = [EtaSA(rng, klen, esn=esn) for _ in range(3)]
    sids = _sessions(drv, sas)
    n = 700
    sa_idx = rng.integers(0, 3, n)
    cts = rng.choice([16, 32, 48, 208, 1440, 1456, 8944], n)
    eh = rng.integers(0, 2**32, n, dtype=np.uint32)
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts, gcm=False, esn_hi=eh)
    bad = ct.copy()
    flip = rng.random(n) < 0.07
    for i in np.nonzero(flip)[0]:
        o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
        bad[o + int(rng.integers(0, L))] ^= 0x08        # anywhere: hdr, IV, CT or ICV
    ref_out, ref_st = oracle_decrypt(sas, bad, descs, eh)
    d = descs.copy()
    d["sa"] = [sids[s] for s in sa_idx]
    arena = _dev(bad)
    out = arena if inplace else torch.zeros_like(arena)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    decrypt_batch(drv, arena, _descs_dev(d), n, st, out=None if inplace else out, grouped=False)
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    assert (st == ref_st).all(), np.nonzero(st != ref_st)[0][:10]
    ok = st == 0
    m_ok = _mask(descs[ok], len(bad), 24, 12)
    res = out.cpu().numpy()
    assert (res[m_ok] == ref_out[m_ok]).all()
    assert (res[m_ok] == plain[m_ok]).all()
    if inplace:
        m_bad = _mask(descs[~ok], len(bad), 0, 0)
        assert (res[m_bad] == bad[m_bad]).all()       # EBADMSG records untouched
    for s in sids:
        drv.freesession(s)


def test_eta_encrypt_vs_oracle(drv):
    from espgpu.batch import encrypt_batch
    rng = np.random.default_rng(77)
    sas = [EtaSA(rng, 32), EtaSA(rng, 16, esn=True)]
    sids = _sessions(drv, sas)
    n = 400
    sa_idx = rng.integers(0, 2, n)
    cts = rng.choice([16, 1440, 8944, 64], n)
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts, gcm=False,
                                         esn_hi=rng.integers(0, 2**32, n, dtype=np.uint32))
    d = descs.copy()
    d["sa"] = [sids[s] for s in sa_idx]
    arena = _dev(plain)
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    encrypt_batch(drv, arena, _descs_dev(d), n, st)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    assert (arena.cpu().numpy() == ct).all()
    for s in sids:
        drv.freesession(s)


def test_mixed_gcm_and_eta_batch(drv):
    """One batch holding GCM and ETA records of several sessions (planner path)."""
    from espgpu.batch import decrypt_batch
    rng = np.random.default_rng(88)
    gsas = [GcmSA(rng, 16), GcmSA(rng, 32)]
    esas = [EtaSA(rng, 32), EtaSA(rng, 16)]
    gs, es = _sessions(drv, gsas), _sessions(drv, esas)
    n = 500
    pg, cg, dg, eg = build_records(rng, gsas, rng.integers(0, 2, n), rng.choice([12, 1448, 204], n))
    pe, ce, de, ee = build_records(rng, esas, rng.integers(0, 2, n), rng.choice([16, 1440], n), gcm=False)
    shift = len(cg)
    arena_np = np.concatenate([cg, ce])
    d = np.concatenate([dg.copy(), de.copy()])
    d["sa"][:n] = [gs[s] for s in dg["sa"]]
    d["sa"][n:] = [es[s] for s in de["sa"]]
    d["off4"][n:] += shift // 4
    perm = rng.permutation(2 * n)
    d = d[perm]
    arena, out = _dev(arena_np), torch.zeros(len(arena_np), dtype=torch.uint8, device="cuda")
    st = torch.full((2 * n,), 0xEE, dtype=torch.uint8, device="cuda")
    decrypt_batch(drv, arena, _descs_dev(d), 2 * n, st, out=out, grouped=False)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    res = out.cpu().numpy()
    mg = _mask(dg, len(cg), 16, 16)
    me = _mask(de, len(ce), 24, 12)
    assert (res[:shift][mg] == pg[mg]).all()
    assert (res[shift:][me] == pe[me]).all()
    for s in gs + es:
        drv.freesession(s)


def test_eta_opencrypto_roundtrip(drv):
    """esp_output -> esp_input through process/flush/poll, CBC_SHA1 SAs."""
    from espgpu.esp import CBC_SHA1, SecAssoc, esp_input_crp, esp_output_crp, esp_pad
    from espgpu.opencrypto import CryptoFramework
    fw = CryptoFramework(drv)
    rng = np.random.default_rng(99)
    key, akey = rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), rng.integers(0, 256, 20, dtype=np.uint8).tobytes()
    for esn in (False, True):
        sa = SecAssoc(0x4242, CBC_SHA1, key, akey, esn=esn)
        err, ses = fw.crypto_newsession(sa.csp())
        assert err == 0
        orc = O.SA(O.CSP_MODE_ETA, key, akey=akey, mlen=12, flags=O.CSP_F_ESN if esn else 0)
        pkts, refs = [], []
        for n in (30, 1400, 8900):
            body = esp_pad(rng.integers(0, 256, n, dtype=np.uint8).tobytes(), blocksize=16)
            rec = (sa.spi.to_bytes(4, "big") + (9).to_bytes(4, "big") +
                   rng.integers(0, 256, 16, dtype=np.uint8).tobytes() + body + bytes(12))
            e, ref = orc.esp_encrypt(rec, esn_hi=5 if esn else 0)
            assert e == 0
            pkt = bytearray(bytes(20) + rec)
            pkts.append(pkt)
            refs.append(ref)
            assert fw.crypto_dispatch(esp_output_crp(fw, ses, sa, pkt, 20, esn_hi=5 if esn else 0)) == 0
        fw.crypto_drain()
        for pkt, ref in zip(pkts, refs):
            assert bytes(pkt[20:]) == ref
        crps = []
        for pkt in pkts:
            c = esp_input_crp(fw, ses, sa, pkt, 20, esn_hi=5 if esn else 0)
            crps.append(c)
            assert fw.crypto_dispatch(c) == 0
        fw.crypto_drain()
        for c, pkt, ref in zip(crps, pkts, refs):
            assert c.crp_etype == 0
            assert bytes(pkt[20 + 24:-12]) == orc.esp_decrypt(ref, esn_hi=5 if esn else 0)[1][24:-12]
        # wrong ESN high bits -> EBADMSG when the SA uses ESN
        if esn:
            c = esp_input_crp(fw, ses, sa, bytearray(bytes(20) + refs[0]), 20, esn_hi=6)
            fw.crypto_dispatch(c)
            fw.crypto_drain()
            assert c.crp_etype == O.EBADMSG
        fw.crypto_freesession(ses)
