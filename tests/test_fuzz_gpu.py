"""Seeded differential test across every session kind the engine serves, in
one planner batch: AES-GCM-16 (AES-128/192/256, ICV 16 / 12 / 8, with and
without ESN) beside AES-CBC / AES-CTR x HMAC-SHA1 / SHA2-256 / 384 / 512 ETA
sessions (xform_esp.c:143-244 session shapes; swcr_gcm cryptosoft.c:465-645,
swcr_eta :874-888).  Per seed: random record sizes, ESN high words, bit flips
anywhere in the record, and malformed records (length not a multiple of 4,
a CBC payload that is not whole blocks, a descriptor naming a freed session:
esp_input's plen checks, xform_esp.c:316-324, give EINVAL).  Decrypted in
place and out of place with the fused trailer word: every status, every
plaintext byte of an authenticated record and every trailer word must equal
the oracle's; in place, rejected records stay untouched."""
import numpy as np
import pytest

import oracle as O
from helpers import EtaSA, GcmSA, build_records

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def drv():
    from espgpu.opencrypto import GpuCryptoDriver
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible HIP device")
    d = GpuCryptoDriver(max_sessions=128)
    yield d
    d.close()


def _all_sas(rng):
    g = [GcmSA(rng, k, esn=e, mlen=m) for k, m in ((16, 16), (24, 12), (32, 8)) for e in (False, True)]
    t = [EtaSA(rng, k, esn=e, ctr=c, sha=h) for (k, c, h) in
         ((32, False, 1), (16, True, 1), (16, False, 256), (32, True, 256), (24, False, 384), (16, True, 512))
         for e in (False, True)]
    nul = [EtaSA(rng, esn=e, null=True, sha=h) for h in (1, 256, 512) for e in (False, True)]   # ESP-NULL
    return g + t + nul


def _cts(rng, sas, idx):
    # GCM and CTR payloads: any 4-byte multiple; CBC: whole 16-byte blocks
    free = rng.choice([4, 12, 44, 100, 204, 1444, 1448, 2996, 8948], len(idx))
    cbc = rng.choice([16, 48, 208, 1440, 1456, 8944], len(idx))
    is_cbc = np.array([isinstance(sas[i], EtaSA) and not sas[i].ctr and not sas[i].null for i in idx])
    return np.where(is_cbc, cbc, free)


@pytest.mark.parametrize("seed", [11, 12, 13, 14])
def test_every_session_kind_mixed_vs_oracle(drv, seed, gcm_lanes):
    from espgpu.batch import decrypt_batch
    from espgpu.esp import trailer_word
    rng = np.random.default_rng(9000 + seed)
    sas = _all_sas(rng)
    sids = []
    for s in sas:
        rc, sid = drv.newsession(s.esp_sa().csp())
        assert rc == 0, drv.last_error()
        sids.append(sid)
    # a session slot that is freed again: records naming it must be EINVAL
    rc, dead = drv.newsession(sas[0].esp_sa().csp())
    assert rc == 0
    drv.freesession(dead)

    n = 1500
    idx = rng.integers(0, len(sas), n)
    cts = _cts(rng, sas, idx)
    eh = rng.integers(0, 2**32, n, dtype=np.uint32)
    plain, ct, descs, eh = build_records(rng, sas, idx, cts, esn_hi=eh)
    bad = ct.copy()
    flip = rng.random(n) < 0.08
    for i in np.nonzero(flip)[0]:
        o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
        bad[o + int(rng.integers(0, L))] ^= 1 << int(rng.integers(0, 8))
    ref_out = bad.copy()
    _, ref_st = O.batch([s.oracle for s in sas], ref_out, descs["off4"], descs["len"], descs["sa"],
                        esn_hi=eh, nthreads=8)
    assert (ref_st[flip] == O.EBADMSG).all() and (ref_st[~flip] == 0).all()

    d = descs.copy()
    d["sa"] = [sids[s] for s in idx]
    want_st = ref_st.copy()
    # malformed descriptors (the record bytes stay as they are)
    cand = np.nonzero(~flip)[0]
    odd = rng.choice(cand, 12, replace=False)
    d["len"][odd] -= 2                                   # len % 4 != 0
    want_st[odd] = O.EINVAL
    cbc = [i for i in cand if isinstance(sas[idx[i]], EtaSA) and not sas[idx[i]].ctr and not sas[idx[i]].null
           and i not in odd]
    short = rng.choice(cbc, min(8, len(cbc)), replace=False)
    d["len"][short] -= 4                                 # CBC payload not whole blocks
    want_st[short] = O.EINVAL
    rest = [i for i in cand if i not in odd and i not in short]
    gone = rng.choice(rest, 6, replace=False)
    d["sa"][gone] = dead                                 # freed session
    want_st[gone] = O.EINVAL

    ok = want_st == 0
    hl = np.array([sas[i].hlen for i in idx])
    ml = np.array([sas[i].mlen for i in idx])
    want_trl = np.array([trailer_word(plain[int(o) * 4 + h:int(o) * 4 + int(L) - a]) if k else 0
                         for o, L, h, a, k in zip(descs["off4"], descs["len"], hl, ml, ok)], dtype=np.uint32)
    m_ok = np.zeros(len(bad), dtype=bool)
    m_rej = np.zeros(len(bad), dtype=bool)
    for o4, L, h, a, k in zip(descs["off4"], descs["len"], hl, ml, ok):
        if k:
            m_ok[int(o4) * 4 + int(h):int(o4) * 4 + int(L) - int(a)] = True
        else:
            m_rej[int(o4) * 4:int(o4) * 4 + int(L)] = True
    ddev = torch.from_numpy(np.ascontiguousarray(d).view(np.uint8).copy()).cuda()
    for inplace in (False, True):
        arena = torch.from_numpy(bad.copy()).cuda()
        out = arena if inplace else torch.zeros_like(arena)
        st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
        trl = torch.full((n,), -1, dtype=torch.int32, device="cuda")
        decrypt_batch(drv, arena, ddev, n, st, out=None if inplace else out, grouped=False, trailer=trl)
        torch.cuda.synchronize()
        got = st.cpu().numpy()
        assert (got == want_st).all(), (inplace, np.nonzero(got != want_st)[0][:10])
        res = out.cpu().numpy()
        assert (res[m_ok] == plain[m_ok]).all(), inplace
        assert (res[m_ok] == ref_out[m_ok]).all(), inplace
        assert (trl.cpu().numpy().view(np.uint32) == want_trl).all(), inplace
        if inplace:
            assert (res[m_rej] == bad[m_rej]).all()      # verify-first: rejected records untouched
    for s in sids:
        drv.freesession(s)
