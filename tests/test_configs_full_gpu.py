"""GPU parity at the FULL size of BASELINE.json configs 2-4 (1M records
each, as bench.py runs them), every record against the oracle (the threaded
C restatement, oracle/espref.c):

  cfg2  1M mixed-MTU packets {64, 256, 1500, 9000} B over 1024 AES-128-GCM SAs;
  cfg3  1M x 1496-B packets over 1024 AES-256-CBC + HMAC-SHA1-96 SAs;
  cfg4  1M x 1500-B packets over rank 0's share of 8192 random SPIs' SAs
        (fnv1_32(spi) mod 8, key.c:295-299) -- one GPU's cfg4 workload.

Encrypt: the GPU's arena equals the oracle's byte for byte.  Decrypt with 1 %
of the ICVs flipped: the GPU's 1M statuses equal the oracle's, out of place
every verified record's plaintext, in place the oracle's whole arena (failed
records keep their ciphertext).  Records sit back to back at their packet
strides, 20 bytes in (an IPv4 header's room), as in bench.py."""
import os

import numpy as np
import pytest

import oracle as O
from helpers import EtaSA, GcmSA

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

DESC = [("off4", "<u4"), ("len", "<u2"), ("sa", "<u2"), ("esn_hi", "<u4"), ("salt", "<u4")]


@pytest.fixture(scope="module")
def drv():
    from espgpu.opencrypto import GpuCryptoDriver
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible HIP device")
    d = GpuCryptoDriver(max_sessions=2048)
    yield d
    d.close()


def _layout(pkt_sizes):
    """Records back to back at packet strides, 20 B in: (off4, len, size)."""
    pkt = np.asarray(pkt_sizes, dtype=np.int64)
    starts = np.concatenate([[0], np.cumsum(pkt)[:-1]])
    return ((starts + 20) // 4).astype(np.uint32), (pkt - 20).astype(np.uint16), int(pkt.sum()) + 64


def _full_check(drv, sas, sa_idx, pkt_sizes, hlen, alen, seed):
    from espgpu.batch import decrypt_batch, encrypt_batch
    rng = np.random.default_rng(seed)
    n = len(sa_idx)
    off4, lens, size = _layout(pkt_sizes)
    d = np.zeros(n, dtype=DESC)
    d["off4"], d["len"], d["sa"] = off4, lens, sa_idx
    if isinstance(sas[0], GcmSA):
        salts = np.array([int.from_bytes(s.salt, "little") for s in sas], dtype=np.uint32)
        d["salt"] = salts[sa_idx]
    nth = min(16, os.cpu_count() or 1)
    osas = [s.oracle for s in sas]
    plain = np.frombuffer(rng.bytes(size), dtype=np.uint8).copy()
    ct = plain.copy()
    O.batch(osas, ct, d["off4"], d["len"], d["sa"], nthreads=nth, encrypt=True)
    sids = []
    for s in sas:
        rc, sid = drv.newsession(s.esp_sa().csp())
        assert rc == 0, drv.last_error()
        sids.append(sid)
    gd = d.copy()
    gd["sa"] = np.array(sids)[sa_idx]
    desc = torch.from_numpy(np.ascontiguousarray(gd).view(np.uint8).copy()).cuda()
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    arena = torch.from_numpy(plain).cuda()
    encrypt_batch(drv, arena, desc, n, st, grouped=False)
    torch.cuda.synchronize()
    assert int((st != 0).sum()) == 0
    assert np.array_equal(arena.cpu().numpy(), ct)
    del arena

    flip = rng.random(n) < 0.01
    fi = np.nonzero(flip)[0]
    bad = ct.copy()
    bad[d["off4"][fi].astype(np.int64) * 4 + d["len"][fi].astype(np.int64) - 1 - rng.integers(0, alen, len(fi))] ^= 0x40
    ref_out = bad.copy()
    _, ref_st = O.batch(osas, ref_out, d["off4"], d["len"], d["sa"], nthreads=nth)
    assert (ref_st[flip] == O.EBADMSG).all() and (ref_st[~flip] == 0).all()
    # payload bytes of the verified records
    edge = np.zeros(size + 1, dtype=np.int32)
    ok = ~flip
    np.add.at(edge, d["off4"][ok].astype(np.int64) * 4 + hlen, 1)
    np.add.at(edge, d["off4"][ok].astype(np.int64) * 4 + d["len"][ok].astype(np.int64) - alen, -1)
    ok_mask = np.cumsum(edge[:-1]) > 0
    assert np.array_equal(ref_out[ok_mask], plain[ok_mask])
    for inplace in (False, True):
        src = torch.from_numpy(bad).cuda()
        out = src if inplace else torch.zeros_like(src)
        st.fill_(0xEE)
        decrypt_batch(drv, src, desc, n, st, out=None if inplace else out, grouped=False)
        torch.cuda.synchronize()
        assert np.array_equal(st.cpu().numpy(), ref_st), inplace
        res = out.cpu().numpy()
        if inplace:
            assert np.array_equal(res, ref_out)
        else:
            assert np.array_equal(res[ok_mask], ref_out[ok_mask])
        del src, out, res
    for s in sids:
        drv.freesession(s)


def test_cfg2_full_size(drv):
    rng = np.random.default_rng(0xF2)
    nsa, n = 1024, 1 << 20
    sas = [GcmSA(rng, 16) for _ in range(nsa)]
    sa_idx = rng.integers(0, nsa, n).astype(np.uint16)
    pkts = rng.choice([64, 256, 1500, 9000], n)
    _full_check(drv, sas, sa_idx, pkts, 16, 16, 0xF20)


def test_cfg3_full_size(drv):
    rng = np.random.default_rng(0xF3)
    nsa, n = 1024, 1 << 20
    sas = [EtaSA(rng, 32) for _ in range(nsa)]
    sa_idx = rng.integers(0, nsa, n).astype(np.uint16)
    _full_check(drv, sas, sa_idx, np.full(n, 1496), 24, 12, 0xF30)


def test_cfg4_full_size_rank0(drv):
    from espgpu.shard import random_spis, shard_plan
    world, nsa_glob, n = 8, 8192, 1 << 20
    spis = random_spis(nsa_glob, 0xF4)
    sa_glob = np.random.default_rng(0xF40).integers(0, nsa_glob, n * world * 21 // 20)
    local_sas, local_pkts = shard_plan(spis, sa_glob, 0, world)
    assert len(local_pkts) >= n and 900 < len(local_sas) < 1150
    remap = np.full(nsa_glob, -1, dtype=np.int64)
    remap[local_sas] = np.arange(len(local_sas))
    sa_idx = remap[sa_glob[local_pkts[:n]]].astype(np.uint16)
    rng = np.random.default_rng(0xF41)
    sas = [GcmSA(rng, 16, spi=int(spis[i])) for i in local_sas]
    _full_check(drv, sas, sa_idx, np.full(n, 1500), 16, 16, 0xF42)
