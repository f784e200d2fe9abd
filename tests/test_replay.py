"""Replay window (esp_input's ipsec_chkreplay before crypto, esp_input_cb's
ipsec_updatereplay after it; freebsd/netipsec/ipsec.c:1177-1436,
xform_esp.c:329-340, :565-580).

The oracle restates both functions (oracle/espref.c, oref_chkreplay /
oref_updatereplay).  No fixture in the reference tree exercises them (DPDK's
own replay tests drive rte_ipsec's window, a different implementation), so
the oracle is pinned by the RFC 4303 3.4.3 properties the code implements
(tests below) and is parity-unpinned beyond them.  Against it:
  * CPU: espgpu_replay_update (host, the engine's window update) step by step,
    window state included, over random arrival orders, ESN and not;
  * GPU: the batch pre-filter kernel (espgpu_replay_check_batch) record by
    record, and the whole inbound sequence check -> decrypt -> merge on GCM
    records whose ESN high word only the window knows."""
import ctypes as C

import numpy as np
import pytest

import oracle as O
from helpers import GcmSA, build_records, oracle_decrypt


def _windows():
    """(wsize bytes, flags, start `last`) combinations: small and large
    windows, the low edge, subspace edges and a non-zero ESN high word."""
    out = []
    for wsize in (4, 8, 32, 128):
        w = wsize * 8
        for flags in (0, O.REPLAY_ESN, O.REPLAY_CYCSEQ):
            for last in (0, 5, w - 3, w + 1000, 0xFFFFFFFF - 10, (7 << 32) | 3, (7 << 32) | 0xFFFFFFF0):
                if last >> 32 and not flags & O.REPLAY_ESN:
                    continue
                out.append((wsize, flags, last))
    return out


def _seqs(rng, last, w, k):
    """Sequence numbers around the window top: in the window, just above it,
    far above, below it, across the 2^32 boundary, zero."""
    tl = last & 0xFFFFFFFF
    c = [tl - rng.integers(0, w), tl + rng.integers(1, 3 * w), tl - w - rng.integers(0, 64),
         rng.integers(0, 2**32), tl + (1 << 31), 0, tl, tl + 1]
    pick = rng.integers(0, len(c), k)
    return [int(c[j]) & 0xFFFFFFFF for j in pick]


def test_oracle_replay_rfc4303_properties():
    r = O.Replay(8)                                   # 64-packet window
    assert r.check(0) == (False, 0xFFFFFFFF)          # SN 0 never valid on an empty window
    for sn in range(1, 101):                          # in order: all accepted, once
        assert r.check(sn)[0] and r.update(sn)
        assert not r.update(sn) and not r.check(sn)[0]
    assert r.last == 100
    assert r.check(100 - 63)[0] is False              # seen, inside the window
    r2 = O.Replay(8)
    for sn in (10, 5, 7, 70, 8):                      # out of order inside the window
        assert r2.update(sn)
    assert not r2.update(8) and not r2.update(70)
    assert not r2.update(6)                           # below the window [7, 70]
    assert r2.check(69) == (True, 0)                  # unseen, inside the window
    # ESN: a window across 2^32 -- a low SN belongs to the next subspace
    r3 = O.Replay(8, last=(2 << 32) | 0xFFFFFFF0, flags=O.REPLAY_ESN)
    assert r3.check(5) == (True, 3) and r3.update(5) and r3.last == (3 << 32) | 5
    assert r3.check(0xFFFFFFF8) == (True, 2)          # previous subspace, inside the window
    assert not O.Replay(8, last=0xFFFFFFFF).check(3)[0]   # non-ESN space exhausted


def _lib():
    import espgpu
    return espgpu.lib()


@pytest.mark.parametrize("wsize,flags,last", _windows())
def test_host_update_matches_oracle(wsize, flags, last):
    from espgpu._lib import Replay
    L = _lib()
    rng = np.random.default_rng(wsize * 7919 + flags * 31 + (last & 0xFFFF))
    ref = O.Replay(wsize, last=last, flags=flags)
    bitmap = np.zeros(ref.bitmap.size + 3, dtype=np.uint32)      # window at word 3
    bitmap[:3] = 0xDEADBEEF
    rp = Replay(last, wsize, ref.bitmap.size, 3, flags)
    for sn in _seqs(rng, last, wsize * 8, 300):
        want = ref.update(sn)
        got = L.espgpu_replay_update(C.byref(rp), bitmap.ctypes.data_as(C.POINTER(C.c_uint32)), sn)
        assert (got == 0) == want and got in (0, 13), (sn, got, want)
        assert rp.last == ref.last
        assert np.array_equal(bitmap[3:], ref.bitmap)
    assert (bitmap[:3] == 0xDEADBEEF).all()


@pytest.mark.parametrize("wsize,bsize,ok", [
    (0, 0, True),          # no replay check: the bitmap is never read
    (8, 0, False),         # no bitmap words
    (8, 3, False),         # not a power of two: bitmap_size - 1 is no mask
    (8, 1, False),         # 64 window bits in one 32-bit word
    (8, 2, True), (8, 4, True),
    (128, 16, False), (128, 32, True),
])
def test_replay_update_rejects_unusable_windows(wsize, bsize, ok):
    """espgpu_replay_update indexes the bitmap with bitmap_size - 1 as a
    mask: a window whose bitmap is empty, not a power of two or smaller than
    wsize * 8 bits is EINVAL, not an out-of-bounds read or write."""
    from espgpu._lib import Replay
    L = _lib()
    rp = Replay(100, wsize, bsize, 0, 0)
    assert L.espgpu_replay_params_ok(C.byref(rp)) == int(ok)
    bitmap = np.full(max(bsize, 1) + 4, 0xA5A5A5A5, dtype=np.uint32)
    got = L.espgpu_replay_update(C.byref(rp), bitmap.ctypes.data_as(C.POINTER(C.c_uint32)), 101)
    if ok:
        assert got == 0
    else:
        assert got == 22 and rp.last == 100 and (bitmap == 0xA5A5A5A5).all()


# ---------------------------------------------------------------- GPU ------

def _torch():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible HIP device")
    return torch


@pytest.fixture(scope="module")
def drv():
    _torch()
    from espgpu.opencrypto import GpuCryptoDriver
    d = GpuCryptoDriver(max_sessions=64)
    yield d
    d.close()


def _replay_tables(refs):
    from espgpu.batch import REPLAY_DTYPE
    tab = np.zeros(len(refs), dtype=REPLAY_DTYPE)
    words, off = [], 0
    for k, r in enumerate(refs):
        tab[k] = (r.c.last, r.c.wsize, r.c.bitmap_size, off, r.c.flags)
        words.append(r.bitmap.copy())
        off += r.bitmap.size
    return tab, np.concatenate(words)


@pytest.mark.gpu
def test_replay_check_kernel_matches_oracle(drv):
    torch = _torch()
    from espgpu.batch import replay_check
    rng = np.random.default_rng(11)
    refs = []
    for wsize, flags, last in _windows():
        r = O.Replay(wsize, last=last, flags=flags)
        for sn in _seqs(rng, last, wsize * 8, 200):       # a used window
            r.update(sn)
        refs.append(r)
    refs.append(O.Replay(0))                                  # replay check disabled
    n = 40000
    sa = rng.integers(0, len(refs), n).astype(np.uint16)
    seq = np.array([_seqs(rng, refs[s].last, max(refs[s].c.wsize, 1) * 8, 1)[0] for s in sa],
                   dtype=np.uint32)
    arena = rng.integers(0, 256, n * 16 + 64, dtype=np.uint8)
    for k in range(4):
        arena[np.arange(n) * 16 + 4 + k] = (seq >> (24 - 8 * k)) & 0xFF
    desc = np.zeros(n, dtype=[("off4", "<u4"), ("len", "<u2"), ("sa", "<u2"), ("esn_hi", "<u4"),
                              ("salt", "<u4")])
    desc["off4"] = np.arange(n) * 4
    desc["len"] = 16
    desc["sa"] = sa
    desc["esn_hi"] = 0xA5A5A5A5
    tab, words = _replay_tables(refs)
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).cuda()
    rst = torch.full((n,), 0x77, dtype=torch.uint8, device="cuda")
    replay_check(drv, torch.from_numpy(arena).cuda(), d_desc, n,
                 torch.from_numpy(tab.view(np.uint8).copy()).cuda(),
                 torch.from_numpy(words.view(np.int32)).cuda(), rst)
    torch.cuda.synchronize()
    got = d_desc.cpu().numpy().view(desc.dtype)
    rs = rst.cpu().numpy()
    for i in range(n):
        r = refs[sa[i]]
        ok, sh = r.check(int(seq[i]))
        assert rs[i] == (0 if ok else 13), (i, sa[i], seq[i])
        assert got["len"][i] == (16 if ok else 0)
        want_hi = sh if (ok and r.c.wsize and r.c.flags & O.REPLAY_ESN) else 0xA5A5A5A5
        assert got["esn_hi"][i] == want_hi, (i, seq[i], r.c.last, sh)
    assert (rs == 13).any() and (rs == 0).any()


@pytest.mark.gpu
def test_replay_prefilter_then_decrypt(drv):
    """esp_input's order on a batch: window check (which supplies the ESN
    high word), verify + decrypt, merge.  Replayed records end EACCES and keep
    their bytes; the rest decrypt exactly as the oracle with the window's
    ESN high word, which the descriptors did not carry."""
    torch = _torch()
    from espgpu.batch import decrypt_batch, descs_to_tensor, replay_check, replay_merge
    rng = np.random.default_rng(5)
    sas = [GcmSA(rng, esn=True), GcmSA(rng)]
    sids = []
    for s in sas:
        rc, sid = drv.newsession(s.esp_sa().csp())
        assert rc == 0
        sids.append(sid)
    refs = {sids[0]: O.Replay(16, last=(4 << 32) | 0xFFFFFF00, flags=O.REPLAY_ESN),
            sids[1]: O.Replay(16, last=5000)}
    for sn in (0xFFFFFF00 - 5, 0xFFFFFF00 - 9):
        refs[sids[0]].update(sn)
    for sn in range(4900, 5000, 3):
        refs[sids[1]].update(sn)
    n = 600
    sa_idx = rng.integers(0, 2, n)
    seqs, his = [], []
    for s in sa_idx:
        r = refs[sids[s]]
        cand = ([0xFFFFFF00 - 5, 0xFFFFFF00 - 9, 0xFFFFFF00 - 7, 0xFFFFFF10, 3, 0xFFFFFF00]
                if s == 0 else [4903, 4904, 4997, 5001, 6000, 100, 4999])
        sn = int(cand[rng.integers(0, len(cand))])
        ok, sh = r.check(sn)
        seqs.append(sn)
        his.append(sh if ok and s == 0 else 0)
    plain, ct, descs, esn_hi = build_records(rng, sas, sa_idx, [96] * n, seqs=seqs,
                                             esn_hi=np.array(his, dtype=np.uint32))
    want, wst = oracle_decrypt(sas, ct, descs, esn_hi)
    descs["sa"] = [sids[s] for s in sa_idx]
    descs["esn_hi"] = 0                                  # only the window knows it
    # the replay table is indexed by session id, like the SA table
    tab, words = _replay_tables([refs.get(k, O.Replay(0)) for k in range(max(sids) + 1)])
    d_arena = torch.from_numpy(ct.copy()).cuda()
    d_desc = descs_to_tensor(descs, "cuda")
    rst = torch.zeros(n, dtype=torch.uint8, device="cuda")
    replay_check(drv, d_arena, d_desc, n, torch.from_numpy(tab.view(np.uint8).copy()).cuda(),
                 torch.from_numpy(words.view(np.int32)).cuda(), rst)
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    out = torch.zeros_like(d_arena)
    decrypt_batch(drv, d_arena, d_desc, n, st, out=out)
    replay_merge(drv, st, rst, n)
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    out = out.cpu().numpy()
    n_rep = 0
    for i in range(n):
        r = refs[sids[sa_idx[i]]]
        ok, _ = r.check(seqs[i])
        if not ok:
            assert st[i] == 13
            n_rep += 1
            continue
        assert st[i] == wst[i] == 0, (i, seqs[i], st[i], wst[i])
        o, L = int(descs["off4"][i]) * 4, int(descs["len"][i])
        assert np.array_equal(out[o + 16:o + L - 16], want[o + 16:o + L - 16])
    assert 0 < n_rep < n
    for s in sids:
        drv.freesession(s)
