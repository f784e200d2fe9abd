"""Fused esp_input_cb trailer checks (xform_esp.c:597-630):
espgpu_decrypt_batch_trailer's per-record word against the Python
restatement applied to the oracle's plaintext; and (CPU) that the word's
verdict agrees with esp_trailer_ok, the direct restatement of the reference."""
import numpy as np
import pytest

from helpers import EtaSA, GcmSA, build_records, oracle_decrypt


def _tails(rng, n):
    """A mix of trailers: valid monotonic padding, bad pad content, bad pad
    length, IPPROTO_NONE and random bytes."""
    t = {}
    for i in range(n):
        k = i % 5
        if k == 0:
            pl = int(rng.integers(0, 12))
            t[i] = bytes([pl if pl else int(rng.integers(0, 256)), pl, 4])       # ok (IPv4)
        elif k == 1:
            t[i] = bytes([3, 7, 41])                                           # bad pad content
        elif k == 2:
            t[i] = bytes([250, 250, 6])                                        # pad length too big
        elif k == 3:
            t[i] = bytes([2, 2, 59])                                           # IPPROTO_NONE
    return t


def test_trailer_word_matches_reference_checks():
    from espgpu.esp import esp_trailer_ok, trailer_accepts, trailer_word
    rng = np.random.default_rng(5)
    for _ in range(5000):
        n = int(rng.integers(3, 40))
        p = rng.integers(0, 256, n, dtype=np.uint8)
        if rng.random() < 0.5:
            pl = int(rng.integers(0, n - 1))
            p[-2] = pl
            p[-3] = pl if rng.random() < 0.7 else p[-3]
        if rng.random() < 0.1:
            p[-1] = 59
        assert trailer_accepts(trailer_word(p)) == esp_trailer_ok(p)


torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def drv():
    from espgpu.opencrypto import GpuCryptoDriver
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible HIP device")
    d = GpuCryptoDriver(max_sessions=64)
    yield d
    d.close()


def _sessions(drv, sas):
    from espgpu.esp import CBC_SHA1, GCM, SecAssoc
    out = []
    for s in sas:
        sa = (SecAssoc(s.spi, CBC_SHA1, s.key, s.akey, esn=s.esn) if isinstance(s, EtaSA)
              else SecAssoc(s.spi, GCM, s.key + s.salt, esn=s.esn))
        rc, sid = drv.newsession(sa.csp())
        assert rc == 0
        out.append(sid)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["gcm", "eta"])
@pytest.mark.parametrize("inplace", [False, True])
def test_fused_trailer_vs_oracle(drv, kind, inplace, gcm_lanes):
    from espgpu.batch import decrypt_batch
    from espgpu.esp import trailer_word
    rng = np.random.default_rng(17 + inplace + 2 * (kind == "eta"))
    gcm = kind == "gcm"
    sas = [GcmSA(rng, 16), GcmSA(rng, 32)] if gcm else [EtaSA(rng, 32), EtaSA(rng, 16)]
    sids = _sessions(drv, sas)
    n = 600
    sa_idx = rng.integers(0, 2, n)
    cts = rng.choice([4, 8, 12, 16, 20, 204, 1448] if gcm else [16, 32, 208, 1440], n)
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts, gcm=gcm, tails=_tails(rng, n))
    bad = ct.copy()
    flip = rng.random(n) < 0.05
    for i in np.nonzero(flip)[0]:
        bad[int(descs["off4"][i]) * 4 + int(descs["len"][i]) - 2] ^= 0x01          # ICV bit
    ref_out, ref_st = oracle_decrypt(sas, bad, descs, eh)
    hlen, alen = (16, 16) if gcm else (24, 12)
    want = np.zeros(n, dtype=np.uint32)
    for i in range(n):
        if ref_st[i] == 0:
            o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
            want[i] = trailer_word(ref_out[o + hlen:o + L - alen])
    d = descs.copy()
    d["sa"] = [sids[s] for s in sa_idx]
    arena = torch.from_numpy(bad.copy()).cuda()
    out = arena if inplace else torch.zeros_like(arena)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    tr = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    dd = torch.from_numpy(np.ascontiguousarray(d).view(np.uint8).copy()).cuda()
    decrypt_batch(drv, arena, dd, n, st, out=None if inplace else out, trailer=tr)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == ref_st).all()
    got = tr.cpu().numpy().view(np.uint32)
    assert (got == want).all(), np.nonzero(got != want)[0][:10]
    for s in sids:
        drv.freesession(s)
