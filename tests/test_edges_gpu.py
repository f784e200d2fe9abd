"""GPU parity at the edges of the descriptor format: empty batches and records
of the largest length a descriptor can carry (len is 16 bits and ESP records
are 4-byte multiples: 65532 bytes, i.e. a 65535-byte IP datagram's ESP
payload).  A 65532-byte GCM record runs 4093 counter blocks (the counter's
low byte wraps 16 times: the counter cache is rebuilt mid-record); an ETA
record runs 1023 HMAC-SHA1/256 or 512 SHA-512 blocks.  Bit-exact vs the
oracle, tampered records EBADMSG."""
import numpy as np
import pytest

import oracle as O
from helpers import EtaSA, GcmSA, build_records, oracle_decrypt

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

MAXLEN = 65532


@pytest.fixture(scope="module")
def drv():
    from espgpu.opencrypto import GpuCryptoDriver
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible HIP device")
    d = GpuCryptoDriver(max_sessions=64)
    yield d
    d.close()


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _descs_dev(descs):
    return torch.from_numpy(np.ascontiguousarray(descs).view(np.uint8).copy()).cuda()


def test_empty_batches(drv):
    """n = 0: decrypt, in-place decrypt and encrypt return 0 and write nothing."""
    from espgpu.batch import decrypt_batch, encrypt_batch
    arena = torch.full((256,), 0x5A, dtype=torch.uint8, device="cuda")
    out = torch.full((256,), 0xA5, dtype=torch.uint8, device="cuda")
    desc = torch.zeros(16, dtype=torch.uint8, device="cuda")
    st = torch.full((1,), 0xEE, dtype=torch.uint8, device="cuda")
    decrypt_batch(drv, arena, desc, 0, st, out=out)
    decrypt_batch(drv, arena, desc, 0, st, out=None)
    encrypt_batch(drv, arena, desc, 0, st)
    torch.cuda.synchronize()
    assert (arena.cpu().numpy() == 0x5A).all() and (out.cpu().numpy() == 0xA5).all()
    assert int(st.item()) == 0xEE


def _run(drv, sas, ct_lens, rng, inplace, tamper=(1,)):
    from espgpu.batch import decrypt_batch
    sids = []
    for s in sas:
        rc, sid = drv.newsession(s.esp_sa().csp())
        assert rc == 0, drv.last_error()
        sids.append(sid)
    n = len(ct_lens)
    sa_idx = np.arange(n) % len(sas)
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, ct_lens,
                                         esn_hi=rng.integers(0, 2**32, n, dtype=np.uint32))
    assert int(descs["len"].max()) == MAXLEN
    bad = ct.copy()
    for i in tamper:
        o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
        bad[o + L // 2] ^= 0x08                                  # mid-record ciphertext bit
    ref_out, ref_st = oracle_decrypt(sas, bad, descs, eh)
    d = descs.copy()
    d["sa"] = [sids[s] for s in sa_idx]
    arena = _dev(bad)
    out = arena if inplace else torch.zeros_like(arena)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    decrypt_batch(drv, arena, _descs_dev(d), n, st, out=None if inplace else out, grouped=False)
    torch.cuda.synchronize()
    got = st.cpu().numpy()
    assert (got == ref_st).all(), (got, ref_st)
    assert all(ref_st[i] == O.EBADMSG for i in tamper) and (np.delete(ref_st, list(tamper)) == 0).all()
    res = out.cpu().numpy()
    for i in range(n):
        o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
        s = sas[sa_idx[i]]
        lo, hi = o + s.hlen, o + L - s.mlen
        if got[i] == 0:
            assert (res[lo:hi] == plain[lo:hi]).all(), i
        elif inplace:
            assert (res[o:o + L] == bad[o:o + L]).all(), i        # failed: untouched in place
    for sid in sids:
        drv.freesession(sid)


@pytest.mark.parametrize("inplace", [False, True])
def test_gcm_max_length_records(drv, inplace, gcm_lanes):
    rng = np.random.default_rng(4100 + inplace)
    sas = [GcmSA(rng, 16), GcmSA(rng, 32, esn=True)]
    ct = MAXLEN - 32                                             # SPI|SN|IV8 + 16-byte ICV
    _run(drv, sas, [ct, ct, 4, 1448, ct, 8948], rng, inplace)


@pytest.mark.parametrize("inplace", [False, True])
def test_eta_max_length_records(drv, inplace):
    rng = np.random.default_rng(4200 + inplace)
    sas = [EtaSA(rng, 32), EtaSA(rng, 16, ctr=True, sha256=True, esn=True), EtaSA(rng, 24, sha=512)]
    # the longest payload each layout allows within 65532 bytes: CTR (header
    # 16, any 4-byte multiple) fills it exactly; CBC (header 24, payload a
    # multiple of 16) stops at 65524 / 65528 with a 12- / 32-byte ICV
    lens = [65488, MAXLEN - 16 - 16, 65472, 16, 44, 1440]
    _run(drv, sas, lens, rng, inplace, tamper=(0, 2))
