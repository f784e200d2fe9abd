"""GPU parity tests for the AES-CBC + HMAC-SHA1-96 ESP path (CSP_MODE_ETA):
bit-exact against the oracle (swcr_eta restatement), ICV failures, ESN,
in-place verify-first, mixed GCM + ETA batches through the planner."""
import numpy as np
import pytest

import oracle as O
from helpers import EtaSA, GcmSA, build_records, golden, oracle_decrypt

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
    sids = []
    for s in sas:
        rc, sid = drv.newsession(s.esp_sa().csp())
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


@pytest.mark.parametrize("grouped", [False, True])
def test_eta_encrypt_mixed_wave_vs_oracle(drv, grouped):
    """Encrypt with every ETA transform mixed record by record (grouped: the
    64-record units hold several sessions, so the cipher pass walks them one
    session at a time and the quad-coalesced CBC chain and MAC pass run with
    lanes switched off inside each quad), ragged payloads from one block to
    jumbo, and records of no session or with a CBC payload that is not a
    block multiple among them (EINVAL, bytes untouched): ciphertext and ICV
    bit-exact vs the oracle."""
    from espgpu.batch import encrypt_batch
    rng = np.random.default_rng(91 + grouped)
    sas = [EtaSA(rng, 32), EtaSA(rng, 16, esn=True, sha=256), EtaSA(rng, 24, sha=384),
           EtaSA(rng, 32, ctr=True, sha=1), EtaSA(rng, 16, noauth=True), EtaSA(rng, null=True, sha=256)]
    sids = _sessions(drv, sas)
    n = 1000
    sa_idx = rng.integers(0, len(sas), n)
    cts = _variant_cts(rng, sas, sa_idx)
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts,
                                         esn_hi=rng.integers(0, 2**32, n, dtype=np.uint32))
    d = descs.copy()
    d["sa"] = [sids[s] for s in sa_idx]
    orphan = rng.random(n) < 0.05
    d["sa"][orphan] = 0xFFFF                                  # no such session
    # CBC records whose payload is not a block multiple (xform_esp.c:316-324)
    cbc = np.array([not (sas[i].ctr or sas[i].null) for i in sa_idx])
    ragged = cbc & ~orphan & (rng.random(n) < 0.05)
    d["len"][ragged] -= 4
    orphan |= ragged
    arena = _dev(plain)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    encrypt_batch(drv, arena, _descs_dev(d), n, st, grouped=grouped)
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    assert (st[orphan] == O.EINVAL).all() and (st[~orphan] == 0).all()
    res = arena.cpu().numpy()
    keep = np.zeros(len(plain), dtype=bool)
    for i in range(n):
        o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
        keep[o:o + L] = True
        want = plain[o:o + L] if orphan[i] else ct[o:o + L]   # refused records keep their bytes
        assert (res[o:o + L] == want).all(), (i, sa_idx[i], int(cts[i]), bool(orphan[i]))
    assert (res[~keep] == plain[~keep]).all()                 # nothing outside the records
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


# ---------------------------------------------------------------------------
# AES-CTR (RFC 3686) and HMAC-SHA2-256 ETA sessions

def _variant_sas(rng, esn=False):
    """Every cipher x hash pair; SHA2-384/512 SAs (the MODE 3 launch beside the
    fused ones) include auth keys longer than the 128-byte block (hashed
    first, hmac_init_pad) and a short one."""
    return [EtaSA(rng, 16, esn=esn, ctr=c, sha256=h) for c in (False, True) for h in (False, True)] + \
           [EtaSA(rng, 32, esn=esn, ctr=True, sha256=True), EtaSA(rng, 24, esn=esn, ctr=True),
            EtaSA(rng, 16, esn=esn, sha=384), EtaSA(rng, 24, esn=esn, sha=512),
            EtaSA(rng, 32, esn=esn, ctr=True, sha=512, aklen=150), EtaSA(rng, 16, esn=esn, ctr=True, sha=384, aklen=7)] + \
           _f4_sas(rng, esn)


def _f4_sas(rng, esn=False):
    """The rest of key.c's ESP transforms the engine serves: encryption
    without auth (CSP_MODE_CIPHER, AES-CBC and AES-CTR) and ESP-NULL with
    every HMAC (CRYPTO_NULL_CBC: the payload unencrypted, only the ICV)."""
    return [EtaSA(rng, 16, noauth=True), EtaSA(rng, 32, ctr=True, noauth=True)] + \
           [EtaSA(rng, esn=esn, null=True, sha=h) for h in (1, 256, 384, 512)]


def _variant_cts(rng, sas, sa_idx):
    """CBC payloads are 16-byte multiples; CTR and NULL ones any 4-byte multiple."""
    cbc = rng.choice([16, 32, 48, 208, 1440, 1456, 8944], len(sa_idx))
    ctr = rng.choice([4, 8, 12, 20, 44, 100, 1444, 1448, 8948], len(sa_idx))
    return np.where([sas[i].ctr or sas[i].null for i in sa_idx], ctr, cbc)


def _hl(sas, idx):
    return np.array([sas[i].hlen for i in idx]), np.array([sas[i].mlen for i in idx])


def _mask_var(descs, size, hl, ml):
    m = np.zeros(size, dtype=bool)
    for o4, L, h, a in zip(descs["off4"], descs["len"], hl, ml):
        m[int(o4) * 4 + int(h):int(o4) * 4 + int(L) - int(a)] = True
    return m


@pytest.mark.parametrize("esn", [False, True])
@pytest.mark.parametrize("inplace", [False, True])
def test_eta_variants_decrypt_vs_oracle(drv, esn, inplace):
    """AES-CBC / AES-CTR x HMAC-SHA1-96 / HMAC-SHA2 sessions mixed in one
    batch (planner path), AES-128/192/256, tag failures anywhere in the
    record: statuses and plaintext bit-exact vs the oracle, failed records
    untouched in place (MODE 2 in place, MODE 3 out of place)."""
    _eta_variants_decrypt(drv, esn, inplace)


def _full_icv_sas(rng):
    """Untruncated ICVs: HMAC-SHA1 with csp_auth_mlen 20 and HMAC-SHA2 with
    csp_auth_mlen 0, which swcr_setup_auth (cryptosoft.c:1013-1018) reads as
    the whole hash (32 / 48 / 64 bytes), plus SHA2-512 with mlen 64 given
    explicitly; CBC, CTR and NULL ciphers."""
    sas = [EtaSA(rng, 16, sha=1, mlen=20), EtaSA(rng, 32, ctr=True, sha=1, mlen=20, esn=True),
           EtaSA(rng, 24, sha=256, mlen=32), EtaSA(rng, 16, ctr=True, sha=384, mlen=48),
           EtaSA(rng, 32, sha=512, mlen=64, esn=True), EtaSA(rng, null=True, sha=512, mlen=64),
           EtaSA(rng, null=True, sha=256, mlen=32)]
    zero = [False, False, True, True, False, False, True]    # these go in with csp_auth_mlen 0
    return sas, zero


def _full_icv_sessions(drv, sas, zero):
    sids = []
    for s, z in zip(sas, zero):
        csp = s.esp_sa().csp()
        if z:
            csp.csp_auth_mlen = 0
        rc, sid = drv.newsession(csp)
        assert rc == 0, drv.last_error()
        sids.append(sid)
    return sids


@pytest.mark.parametrize("inplace", [False, True])
def test_eta_full_hash_icv_vs_oracle(drv, inplace):
    """Full-length HMAC ICVs (20 / 32 / 48 / 64 bytes) through the planner:
    decrypt with bit flips (statuses and plaintext vs the oracle, rejected
    records untouched in place) and encrypt (ciphertext and ICV vs the
    oracle)."""
    from espgpu.batch import decrypt_batch, encrypt_batch
    rng = np.random.default_rng(1350 + inplace)
    sas, zero = _full_icv_sas(rng)
    sids = _full_icv_sessions(drv, sas, zero)
    n = 700
    sa_idx = rng.integers(0, len(sas), n)
    cts = _variant_cts(rng, sas, sa_idx)
    eh = rng.integers(0, 2**32, n, dtype=np.uint32)
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts, esn_hi=eh)
    d = descs.copy()
    d["sa"] = [sids[s] for s in sa_idx]
    arena = _dev(plain)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    encrypt_batch(drv, arena, _descs_dev(d), n, st)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    assert (arena.cpu().numpy() == ct).all()

    bad = ct.copy()
    flip = rng.random(n) < 0.1
    for i in np.nonzero(flip)[0]:
        o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
        bad[o + L - 1 - int(rng.integers(0, sas[sa_idx[i]].mlen))] ^= 0x04   # inside the ICV
    ref_out, ref_st = oracle_decrypt(sas, bad, descs, eh)
    assert (ref_st[flip] == O.EBADMSG).all() and (ref_st[~flip] == 0).all()
    arena = _dev(bad)
    out = arena if inplace else torch.zeros_like(arena)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    decrypt_batch(drv, arena, _descs_dev(d), n, st, out=None if inplace else out, grouped=False)
    torch.cuda.synchronize()
    got = st.cpu().numpy()
    assert (got == ref_st).all(), np.nonzero(got != ref_st)[0][:10]
    hl, ml = _hl(sas, sa_idx)
    ok = got == 0
    m_ok = _mask_var(descs[ok], len(bad), hl[ok], ml[ok])
    res = out.cpu().numpy()
    assert (res[m_ok] == plain[m_ok]).all()
    if inplace:
        m_bad = _mask_var(descs[~ok], len(bad), np.zeros((~ok).sum()), np.zeros((~ok).sum()))
        assert (res[m_bad] == bad[m_bad]).all()
    for s in sids:
        drv.freesession(s)


def test_eta_inplace_cbc_context_vs_oracle():
    """In-place decrypt (MODE 2) of a CBC-only context at ~94 wave units:
    SHA-1 and SHA2-256 sessions of every key size with ESN, beside SHA2-384
    and cipher-only CBC sessions (the wide kernel's records), records of no
    session and ragged CBC payloads (EINVAL), bit flips anywhere.  Statuses
    and plaintext bit-exact vs the oracle, rejected records untouched, twice
    (the retire resets the unit queue)."""
    from espgpu.batch import decrypt_batch
    from espgpu.opencrypto import GpuCryptoDriver
    d0 = GpuCryptoDriver(max_sessions=64)
    try:
        rng = np.random.default_rng(1700)
        sas = [EtaSA(rng, k, esn=e, sha=h) for k in (16, 24, 32) for e in (False, True) for h in (1, 256)] + \
              [EtaSA(rng, 16, sha=384), EtaSA(rng, 32, noauth=True)]
        sids = _sessions(d0, sas)
        n = 6000                                  # ~94 units: several per wave
        sa_idx = rng.integers(0, len(sas), n)
        cts = rng.choice([16, 32, 48, 208, 1440, 1456, 8944], n)
        eh = rng.integers(0, 2**32, n, dtype=np.uint32)
        plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts, esn_hi=eh)
        bad = ct.copy()
        flip = rng.random(n) < 0.07
        for i in np.nonzero(flip)[0]:
            o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
            bad[o + int(rng.integers(0, L))] ^= 0x20
        ref_out, ref_st = oracle_decrypt(sas, bad, descs, eh)
        d = descs.copy()
        d["sa"] = [sids[s] for s in sa_idx]
        orphan = rng.random(n) < 0.02
        d["sa"][orphan] = 0xFFFF
        ragged = ~orphan & (rng.random(n) < 0.02)
        d["len"][ragged] -= 4
        ref_st = ref_st.copy()
        ref_st[orphan | ragged] = O.EINVAL
        arena = _dev(bad)
        st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
        for _ in range(2):
            arena.copy_(_dev(bad))
            st.fill_(0xEE)
            decrypt_batch(d0, arena, _descs_dev(d), n, st, grouped=False)
            torch.cuda.synchronize()
            got = st.cpu().numpy()
            assert (got == ref_st).all(), np.nonzero(got != ref_st)[0][:10]
            hl, ml = _hl(sas, sa_idx)
            ok = got == 0
            m_ok = _mask_var(descs[ok], len(bad), hl[ok], ml[ok])
            res = arena.cpu().numpy()
            assert (res[m_ok] == ref_out[m_ok]).all()
            m_bad = _mask_var(d[~ok], len(bad), np.zeros((~ok).sum()), np.zeros((~ok).sum()))
            assert (res[m_bad] == bad[m_bad]).all()
        for s in sids:
            d0.freesession(s)
    finally:
        d0.close()


def test_removed_design_knobs_are_unknown(drv):
    """The measured-slower designs are not built: their old
    set_tuning keys are unknown (ENOENT), not silently accepted."""
    for k in (b"eta_fused", b"gcm_split", b"gcm_bs", b"eta_ws", b"eta_lag"):
        assert drv.lib.espgpu_set_tuning(drv.ctx, k, 0) == 2


def _eta_variants_decrypt(drv, esn, inplace):
    from espgpu.batch import decrypt_batch
    rng = np.random.default_rng(1300 + 2 * esn + inplace)
    sas = _variant_sas(rng, esn)
    sids = _sessions(drv, sas)
    n = 900
    sa_idx = rng.integers(0, len(sas), n)
    cts = _variant_cts(rng, sas, sa_idx)
    eh = rng.integers(0, 2**32, n, dtype=np.uint32)
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts, esn_hi=eh)
    bad = ct.copy()
    flip = rng.random(n) < 0.07
    for i in np.nonzero(flip)[0]:
        o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
        bad[o + int(rng.integers(0, L))] ^= 0x10
    ref_out, ref_st = oracle_decrypt(sas, bad, descs, eh)
    # a flipped bit fails the ICV check; without auth it decrypts (to garbage)
    auth = np.array([not sas[i].noauth for i in sa_idx])
    assert (ref_st[flip & auth] == O.EBADMSG).all() and (ref_st[~(flip & auth)] == 0).all()
    d = descs.copy()
    d["sa"] = [sids[s] for s in sa_idx]
    arena = _dev(bad)
    out = arena if inplace else torch.zeros_like(arena)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    decrypt_batch(drv, arena, _descs_dev(d), n, st, out=None if inplace else out, grouped=False)
    torch.cuda.synchronize()
    got = st.cpu().numpy()
    assert (got == ref_st).all(), np.nonzero(got != ref_st)[0][:10]
    hl, ml = _hl(sas, sa_idx)
    ok = got == 0
    m_ok = _mask_var(descs[ok], len(bad), hl[ok], ml[ok])
    res = out.cpu().numpy()
    assert (res[m_ok] == ref_out[m_ok]).all()
    clean = ok & ~flip
    m_clean = _mask_var(descs[clean], len(bad), hl[clean], ml[clean])
    assert (res[m_clean] == plain[m_clean]).all()
    if inplace:
        m_bad = _mask_var(descs[~ok], len(bad), np.zeros((~ok).sum()), np.zeros((~ok).sum()))
        assert (res[m_bad] == bad[m_bad]).all()
    for s in sids:
        drv.freesession(s)


def test_eta_variants_encrypt_vs_oracle(drv):
    from espgpu.batch import encrypt_batch
    rng = np.random.default_rng(1400)
    sas = _variant_sas(rng, esn=True)
    sids = _sessions(drv, sas)
    n = 600
    sa_idx = rng.integers(0, len(sas), n)
    cts = _variant_cts(rng, sas, sa_idx)
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts,
                                         esn_hi=rng.integers(0, 2**32, n, dtype=np.uint32))
    d = descs.copy()
    d["sa"] = [sids[s] for s in sa_idx]
    arena = _dev(plain)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    encrypt_batch(drv, arena, _descs_dev(d), n, st)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    assert (arena.cpu().numpy() == ct).all()
    for s in sids:
        drv.freesession(s)


def test_eta_variants_trailer(drv):
    """The fused esp_input_cb trailer word for CTR records (partial last
    block) and SHA2-256 sessions, out of place and in place; a record whose
    ICV fails gets EBADMSG and trailer word 0."""
    from espgpu.batch import decrypt_batch
    from espgpu.esp import trailer_word
    _eta_variants_trailer(drv, decrypt_batch, trailer_word)


def _eta_variants_trailer(drv, decrypt_batch, trailer_word):
    rng = np.random.default_rng(1500)
    sas = _variant_sas(rng)
    sids = _sessions(drv, sas)
    n = 400
    sa_idx = rng.integers(0, len(sas), n)
    cts = _variant_cts(rng, sas, sa_idx)
    tails = {i: bytes([int(rng.integers(0, 4)), int(rng.integers(0, 40)), int(rng.choice([4, 41, 59]))])
             for i in range(n)}
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts, tails=tails)
    d = descs.copy()
    d["sa"] = [sids[s] for s in sa_idx]
    hl, ml = _hl(sas, sa_idx)
    want = np.array([trailer_word(plain[int(o) * 4 + h:int(o) * 4 + int(L) - a])
                     for o, L, h, a in zip(descs["off4"], descs["len"], hl, ml)], dtype=np.uint32)
    # every 7th authenticated record: a flipped ICV bit
    bad = ct.copy()
    flip = np.array([i % 7 == 3 and ml[i] > 0 for i in range(n)])
    for i in np.flatnonzero(flip):
        bad[int(descs["off4"][i]) * 4 + int(descs["len"][i]) - 1] ^= 0x01
    want[flip] = 0
    for inplace in (False, True):
        arena = _dev(bad)
        out = arena if inplace else torch.zeros_like(arena)
        st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
        trl = torch.zeros(n, dtype=torch.int32, device="cuda")
        decrypt_batch(drv, arena, _descs_dev(d), n, st, out=None if inplace else out, grouped=False, trailer=trl)
        torch.cuda.synchronize()
        got = st.cpu().numpy()
        assert (got[flip] == 74).all() and (got[~flip] == 0).all()
        assert (trl.cpu().numpy().view(np.uint32) == want).all(), inplace
    for s in sids:
        drv.freesession(s)


@pytest.mark.parametrize("alg", ["ctr-sha1", "ctr-sha256", "cbc-sha256", "cbc-sha384", "ctr-sha512"])
def test_eta_variants_opencrypto_roundtrip(drv, alg):
    """esp_output -> esp_input through process/flush/poll for the AES-CTR
    (crp_iv = nonce || IV || be32(1), xform_esp.c:453-458) and HMAC-SHA2
    SAs: ciphertext and ICV bit-exact vs the oracle, flipped ICV -> EBADMSG."""
    from espgpu import esp as E
    from espgpu.esp import SecAssoc, esp_input_crp, esp_output_crp, esp_pad
    from espgpu.opencrypto import CryptoFramework
    fw = CryptoFramework(drv)
    rng = np.random.default_rng(1600 + len(alg) + 7 * alg.endswith("384"))
    ctr, bits = alg.startswith("ctr"), int(alg.split("sha")[1])
    name = {"ctr-sha1": E.CTR_SHA1, "ctr-sha256": E.CTR_SHA256, "cbc-sha256": E.CBC_SHA256,
            "cbc-sha384": E.CBC_SHA384, "ctr-sha512": E.CTR_SHA512}[alg]
    aalg = {1: O.CRYPTO_SHA1_HMAC, 256: O.CRYPTO_SHA2_256_HMAC, 384: O.CRYPTO_SHA2_384_HMAC,
            512: O.CRYPTO_SHA2_512_HMAC}[bits]
    ckey = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
    nonce = rng.integers(0, 256, 4, dtype=np.uint8).tobytes() if ctr else b""
    akey = rng.integers(0, 256, {1: 20, 256: 32, 384: 48, 512: 64}[bits], dtype=np.uint8).tobytes()
    sa = SecAssoc(0x5150, name, ckey + nonce, akey)
    assert sa.mlen == {1: 12, 256: 16, 384: 24, 512: 32}[bits]
    err, ses = fw.crypto_newsession(sa.csp())
    assert err == 0
    orc = O.SA(O.CSP_MODE_ETA, ckey, nonce or b"\0\0\0\0", akey=akey, mlen=sa.mlen,
               calg=O.CRYPTO_AES_ICM if ctr else O.CRYPTO_AES_CBC, aalg=aalg)
    pkts, refs = [], []
    for nbytes in (30, 61, 1400, 8900):
        body = esp_pad(rng.integers(0, 256, nbytes, dtype=np.uint8).tobytes(), blocksize=4 if ctr else 16)
        rec = (sa.spi.to_bytes(4, "big") + (3).to_bytes(4, "big") +
               rng.integers(0, 256, sa.ivlen, dtype=np.uint8).tobytes() + body + bytes(sa.mlen))
        e, ref = orc.esp_encrypt(rec)
        assert e == 0
        pkt = bytearray(bytes(20) + rec)
        pkts.append(pkt)
        refs.append((rec, ref))
        assert fw.crypto_dispatch(esp_output_crp(fw, ses, sa, pkt, 20)) == 0
    fw.crypto_drain()
    for pkt, (rec, ref) in zip(pkts, refs):
        assert bytes(pkt[20:]) == ref
    crps = [esp_input_crp(fw, ses, sa, pkt, 20) for pkt in pkts]
    bad = bytearray(pkts[2])
    bad[-3] ^= 0x20
    before = bytes(bad)
    crps.append(esp_input_crp(fw, ses, sa, bad, 20))
    for c in crps:
        assert fw.crypto_dispatch(c) == 0
    fw.crypto_drain()
    for c, pkt, (rec, ref) in zip(crps, pkts, refs):
        assert c.crp_etype == 0
        assert bytes(pkt[20 + sa.hlen:-sa.mlen]) == rec[sa.hlen:-sa.mlen]
    assert crps[-1].crp_etype == O.EBADMSG and bytes(bad) == before
    fw.crypto_freesession(ses)


@pytest.mark.parametrize("v", golden("eta_esp_packets.json"), ids=lambda v: v["name"])
def test_dpdk_cbc_sha2_esp_kat_opencrypto(drv, v):
    """DPDK's AES-CBC + HMAC-SHA2-256-128 / -384-192 / -512-256 ESP tunnel
    packets decrypt through the driver path to the expected inner packets."""
    from espgpu import esp as E
    from espgpu.esp import SecAssoc, esp_input_crp
    from espgpu.opencrypto import CryptoFramework
    fw = CryptoFramework(drv)
    alg = {"cbc-hmac-sha256": E.CBC_SHA256, "cbc-hmac-sha384": E.CBC_SHA384, "cbc-hmac-sha512": E.CBC_SHA512}
    sa = SecAssoc(v["spi"], alg[v["mode"]], bytes.fromhex(v["cipher_key"]), bytes.fromhex(v["auth_key"]))
    assert sa.mlen == v["digest_len"]
    err, ses = fw.crypto_newsession(sa.csp())
    assert err == 0
    skip = v["outer_hdr_len"]
    pkt = bytearray(bytes(skip)) + bytearray(bytes.fromhex(v["esp_record"]))
    c = esp_input_crp(fw, ses, sa, pkt, skip)
    assert fw.crypto_dispatch(c) == 0
    fw.crypto_drain()
    assert c.crp_etype == 0
    inner = bytes.fromhex(v["inner_packet"])
    assert bytes(pkt[skip + 24:skip + 24 + len(inner)]) == inner
    fw.crypto_freesession(ses)


@pytest.mark.parametrize("v", golden("cipher_esp_packets.json"), ids=lambda v: v["name"])
def test_cipher_only_esp_kat_opencrypto(drv, v):
    """DPDK's AES-128-CBC ESP packet with no authentication through the
    driver path: a CSP_MODE_CIPHER session (xform_esp.c:230-231) decrypts it
    to the inner packet and encrypts the plaintext back to the packet."""
    from espgpu import esp as E
    from espgpu.esp import SecAssoc, esp_input_crp, esp_output_crp
    from espgpu.opencrypto import CryptoFramework
    fw = CryptoFramework(drv)
    sa = SecAssoc(v["spi"], E.CBC, bytes.fromhex(v["cipher_key"]))
    assert sa.mlen == 0 and sa.csp().csp_mode == O.CSP_MODE_CIPHER
    err, ses = fw.crypto_newsession(sa.csp())
    assert err == 0
    skip = v["outer_hdr_len"]
    rec = bytes.fromhex(v["esp_record"])
    pkt = bytearray(bytes(skip)) + bytearray(rec)
    c = esp_input_crp(fw, ses, sa, pkt, skip)
    assert fw.crypto_dispatch(c) == 0
    fw.crypto_drain()
    assert c.crp_etype == 0
    inner = bytes.fromhex(v["inner_packet"])
    assert bytes(pkt[skip + 24:skip + 24 + len(inner)]) == inner
    c = esp_output_crp(fw, ses, sa, pkt, skip)
    assert fw.crypto_dispatch(c) == 0
    fw.crypto_drain()
    assert c.crp_etype == 0 and bytes(pkt[skip:]) == rec
    fw.crypto_freesession(ses)


@pytest.mark.parametrize("alg", ["null-sha1", "null-sha256", "null-sha512"])
def test_esp_null_opencrypto_roundtrip(drv, alg):
    """ESP-NULL + HMAC through process/flush/poll: esp_output leaves the
    payload as it is and appends the oracle's ICV; esp_input verifies it,
    a flipped payload bit is EBADMSG with the packet untouched."""
    from espgpu import esp as E
    from espgpu.esp import SecAssoc, esp_input_crp, esp_output_crp, esp_pad
    from espgpu.opencrypto import CryptoFramework
    fw = CryptoFramework(drv)
    bits = int(alg.split("sha")[1])
    rng = np.random.default_rng(1650 + bits)
    name = {1: E.NULL_SHA1, 256: E.NULL_SHA256, 512: E.NULL_SHA512}[bits]
    aalg = {1: O.CRYPTO_SHA1_HMAC, 256: O.CRYPTO_SHA2_256_HMAC, 512: O.CRYPTO_SHA2_512_HMAC}[bits]
    akey = rng.integers(0, 256, {1: 20, 256: 32, 512: 64}[bits], dtype=np.uint8).tobytes()
    sa = SecAssoc(0x6160, name, b"", akey)
    assert sa.hlen == 8 and sa.mlen == {1: 12, 256: 16, 512: 32}[bits]
    err, ses = fw.crypto_newsession(sa.csp())
    assert err == 0
    orc = O.SA(O.CSP_MODE_ETA, b"", akey=akey, mlen=sa.mlen, calg=O.CRYPTO_NULL_CBC, aalg=aalg)
    pkts, refs = [], []
    for nbytes in (30, 61, 1400, 8900):
        body = esp_pad(rng.integers(0, 256, nbytes, dtype=np.uint8).tobytes(), blocksize=4)
        rec = sa.spi.to_bytes(4, "big") + (9).to_bytes(4, "big") + body + bytes(sa.mlen)
        e, ref = orc.esp_encrypt(rec)
        assert e == 0 and ref[:-sa.mlen] == rec[:-sa.mlen]
        pkt = bytearray(bytes(20) + rec)
        pkts.append(pkt)
        refs.append(ref)
        assert fw.crypto_dispatch(esp_output_crp(fw, ses, sa, pkt, 20)) == 0
    fw.crypto_drain()
    for pkt, ref in zip(pkts, refs):
        assert bytes(pkt[20:]) == ref
    crps = [esp_input_crp(fw, ses, sa, pkt, 20) for pkt in pkts]
    bad = bytearray(pkts[1])
    bad[40] ^= 0x02
    before = bytes(bad)
    crps.append(esp_input_crp(fw, ses, sa, bad, 20))
    for c in crps:
        assert fw.crypto_dispatch(c) == 0
    fw.crypto_drain()
    for c, pkt, ref in zip(crps, pkts, refs):
        assert c.crp_etype == 0 and bytes(pkt[20:]) == ref
    assert crps[-1].crp_etype == O.EBADMSG and bytes(bad) == before
    fw.crypto_freesession(ses)


def test_grouped_mode_mixed_run_fails_closed(drv):
    """ESPGPU_BATCH_GROUPED trusts the caller's grouping only per record: in a
    GCM chunk led by an ETA record the GCM records come back EINVAL (never an
    unauthenticated 0), GCM records of another session than their chunk's are
    EINVAL, and ETA records anywhere are still decrypted and verified by the
    ETA kernel.  The implicit chunk size depends on the batch size (256
    records, or down to 8 for small batches: launch_gcm), so a record whose
    chunk happens to be led by its own session may also come back 0; every 0
    must then carry the oracle's plaintext."""
    from espgpu.batch import decrypt_batch
    rng = np.random.default_rng(1700)
    g1, g2, e1 = GcmSA(rng, 16), GcmSA(rng, 16), EtaSA(rng, 16)
    sids = _sessions(drv, [g1, g2, e1])
    # chunk 0 (records 0..255): ETA first, then GCM(g1); chunk 1: GCM(g1) first,
    # then ETA and GCM(g2) records mixed in
    n = 512
    kinds = np.zeros(n, dtype=np.int64)          # 0 = g1, 1 = g2, 2 = e1
    kinds[0] = 2
    kinds[10:20] = 2
    kinds[300:310] = 2
    kinds[400:405] = 1
    sas = [g1, g2, e1]
    cts = np.where(kinds == 2, 1440, 1448)
    plain, ct, descs, eh = build_records(rng, sas, kinds, cts)
    d = descs.copy()
    d["sa"] = [sids[k] for k in kinds]
    ref_out, ref_st = oracle_decrypt(sas, ct, descs, eh)
    assert (ref_st == 0).all()
    arena, out = _dev(ct), torch.zeros(len(ct), dtype=torch.uint8, device="cuda")
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    decrypt_batch(drv, arena, _descs_dev(d), n, st, out=out, grouped=True)
    torch.cuda.synchronize()
    got = st.cpu().numpy()
    eta = kinds == 2
    assert (got[eta] == 0).all()                                 # ETA kernel owns them
    assert np.isin(got, [0, O.EINVAL]).all()                     # nothing else, no 0xEE left
    assert got[1] == O.EINVAL                                    # chunk 0 is ETA-led: GCM fails closed
    assert (got[256:300] == 0).all()                             # g1-led chunks: decrypted
    assert got[405] == O.EINVAL or got[400] == O.EINVAL          # g1 and g2 share a chunk either way
    res = out.cpu().numpy()
    hl, ml = _hl(sas, kinds)
    okm = got == 0
    m = _mask_var(descs[okm], len(ct), hl[okm], ml[okm])
    assert (res[m] == plain[m]).all()
    for s in sids:
        drv.freesession(s)


def test_eta_mixed_sessions_in_one_wave_unit(drv):
    """Caller-grouped batch whose 64-record units mix ETA sessions (CBC +
    HMAC-SHA1, CTR + HMAC-SHA2-256, CBC + HMAC-SHA2-384): one session at a
    time through the verified decrypt, the wide-hash records in their own
    launch; statuses and verified plaintext vs the oracle, out of place, with
    tampered ICVs."""
    from espgpu.batch import decrypt_batch
    rng = np.random.default_rng(1902)
    sas = [EtaSA(rng, 16), EtaSA(rng, 32, ctr=True, sha256=True), EtaSA(rng, 24, sha=384)]
    sids = _sessions(drv, sas)
    try:
        n = 640
        kinds = rng.integers(0, 3, n)
        cts = rng.choice([16, 208, 1440], n)
        plain, ct, descs, eh = build_records(rng, sas, kinds, cts)
        bad = ct.copy()
        flip = rng.random(n) < 0.1
        for i in np.flatnonzero(flip):
            bad[int(descs["off4"][i]) * 4 + int(descs["len"][i]) - 1] ^= 0x02
        ref_out, ref_st = oracle_decrypt(sas, bad, descs, eh)
        assert (ref_st[flip] == O.EBADMSG).all() and (ref_st[~flip] == 0).all()
        d = descs.copy()
        d["sa"] = [sids[k] for k in kinds]
        arena, out = _dev(bad), torch.zeros(len(bad), dtype=torch.uint8, device="cuda")
        st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
        decrypt_batch(drv, arena, _descs_dev(d), n, st, out=out, grouped=True)
        torch.cuda.synchronize()
        got = st.cpu().numpy()
        assert (got == ref_st).all(), np.flatnonzero(got != ref_st)[:10]
        hl, ml = _hl(sas, kinds)
        ok = got == 0
        m_ok = _mask_var(descs[ok], len(bad), hl[ok], ml[ok])
        assert (out.cpu().numpy()[m_ok] == plain[m_ok]).all()
    finally:
        for s in sids:
            drv.freesession(s)


def test_planner_as_the_session_table_grows():
    """Planner batches while the session table grows between them (the key
    count is 5 x sessions + 1, so each batch's key range is larger than the
    last): the per-key counts a batch starts from must be zero over the whole
    range, whatever the earlier batches left in the workspace.  GCM and ETA
    sessions added in rounds of 1, 4, 16 and 40, a batch over all sessions so
    far after each round: statuses and plaintext vs the oracle."""
    from espgpu.batch import decrypt_batch
    from espgpu.opencrypto import GpuCryptoDriver
    d = GpuCryptoDriver(max_sessions=128)
    try:
        rng = np.random.default_rng(1700)
        sas, sids = [], []
        for grow in (1, 4, 16, 40):
            new = [GcmSA(rng, 16) if rng.random() < 0.5 else EtaSA(rng, 16, sha256=bool(rng.random() < 0.5))
                   for _ in range(grow)]
            sids += _sessions(d, new)
            sas += new
            n = 200 + 10 * len(sas)
            sa_idx = rng.integers(0, len(sas), n)
            cts = np.where([isinstance(sas[i], GcmSA) for i in sa_idx], rng.integers(1, 90, n) * 16 - 4,
                           rng.integers(1, 90, n) * 16)
            eh = np.zeros(n, dtype=np.uint32)
            plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts, esn_hi=eh)
            bad = ct.copy()
            flip = rng.random(n) < 0.1
            for i in np.nonzero(flip)[0]:
                o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
                bad[o + L - 1] ^= 0x01                          # inside the ICV
            ref_out, ref_st = oracle_decrypt(sas, bad, descs, eh)
            dd = descs.copy()
            dd["sa"] = [sids[s] for s in sa_idx]
            arena = _dev(bad)
            out = torch.zeros_like(arena)
            st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
            decrypt_batch(d, arena, _descs_dev(dd), n, st, out=out, grouped=False)
            torch.cuda.synchronize()
            got = st.cpu().numpy()
            assert (got == ref_st).all(), (len(sas), np.nonzero(got != ref_st)[0][:10])
            hl, ml = _hl(sas, sa_idx)
            ok = got == 0
            m_ok = _mask_var(descs[ok], len(bad), hl[ok], ml[ok])
            assert (out.cpu().numpy()[m_ok] == ref_out[m_ok]).all()
    finally:
        d.close()


def test_planner_past_the_lds_key_arrays():
    """A session table with more planner keys (5 x sessions + 1) than the
    LDS arrays hold (16384: 3276 sessions) takes the global-memory plan
    (plan.hip plan_*_g).  A batch at 3276 sessions (the LDS plan's last size)
    and one at 3400, GCM and ETA sessions mixed, records in random session
    order with 10 % tampered ICVs, out of place and in place: statuses and
    plaintext vs the oracle, the tampered records in place restored."""
    from espgpu.batch import decrypt_batch
    from espgpu.opencrypto import GpuCryptoDriver
    d = GpuCryptoDriver(max_sessions=4096)
    try:
        rng = np.random.default_rng(3276)
        sas, sids = [], []
        for total in (3276, 3400):
            new = [GcmSA(rng, 16) if rng.random() < 0.8 else EtaSA(rng, 16, sha256=bool(rng.random() < 0.5))
                   for _ in range(total - len(sas))]
            sids += _sessions(d, new)
            sas += new
            n = 12000
            sa_idx = rng.integers(0, len(sas), n)
            cts = np.where([isinstance(sas[i], GcmSA) for i in sa_idx], rng.integers(1, 90, n) * 16 - 4,
                           rng.integers(1, 90, n) * 16)
            eh = np.zeros(n, dtype=np.uint32)
            plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts, esn_hi=eh)
            bad = ct.copy()
            for i in np.nonzero(rng.random(n) < 0.1)[0]:
                o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
                bad[o + L - 1] ^= 0x01                          # inside the ICV
            ref_out, ref_st = oracle_decrypt(sas, bad, descs, eh)
            assert (ref_st != 0).any() and (ref_st == 0).any()
            dd = descs.copy()
            dd["sa"] = [sids[s] for s in sa_idx]
            hl, ml = _hl(sas, sa_idx)
            for inplace in (False, True):
                arena = _dev(bad)
                out = arena if inplace else torch.zeros_like(arena)
                st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
                decrypt_batch(d, arena, _descs_dev(dd), n, st, out=None if inplace else out, grouped=False)
                torch.cuda.synchronize()
                got = st.cpu().numpy()
                assert (got == ref_st).all(), (len(sas), inplace, np.nonzero(got != ref_st)[0][:10])
                ok = got == 0
                m_ok = _mask_var(descs[ok], len(bad), hl[ok], ml[ok])
                res = out.cpu().numpy()
                assert (res[m_ok] == ref_out[m_ok]).all(), (len(sas), inplace)
                if inplace:
                    m_bad = _mask_var(descs[~ok], len(bad), hl[~ok], ml[~ok])
                    assert (res[m_bad] == bad[m_bad]).all(), len(sas)      # failed records untouched
    finally:
        d.close()
